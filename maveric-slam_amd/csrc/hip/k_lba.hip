// k_lba.hip -- the local-BA Schur back-end (src/local_bundle_adjustment.c:128-250), batched:
// one 256-thread block per problem (a window of P poses and L landmarks), everything in LDS.
// Per chunk of LC landmarks, in the reference's order:
//   (1) zero A's diagonal blocks and B;
//   (2) wave 0 walks the chunk's factors (landmark-major, pose-minor as main's loops): lanes
//       recompute H = J^T J into the one LDS H buffer the way matmul2 does (0 * old H, then
//       the two products), then the lanes owning A/B/C target entries add it (matrix_add);
//   (3) invert A's 3x3 blocks (cofactor formulas, invert_3x3);
//   (4) BA = A B   (matmul2: 0 * old BA, then sequential k);
//   (5) C = C - B^T BA over the pose block (matmul2 with -1 scale, sequential k).
// Every value sees the reference's operations in its order, so C is bit-identical to the
// sequential loop (oracle/mv_oracle.c orc_lba_schur, itself pinned to the reference's own
// functions).  Latency-bound by the chunk sequence (the Schur accumulation is sequential);
// throughput comes from many problems per launch.
#include "maveric_hip.h"
#include "mv_internal.hpp"

namespace {

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void k_lba_schur(int P, int L, int LC, int as_built, const float *__restrict__ J_all,
                                                   float *__restrict__ C_all) {
    extern __shared__ float sm[];
    const int S = 6 * P + 1, TL = 3 * LC, t = threadIdx.x, lane = t & 63;
    const int nch = (L + LC - 1) / LC;
    float *H = sm, *A = H + 100, *B = A + TL * TL, *BA = B + S * TL, *C = BA + S * TL;
    const long b = blockIdx.x;
    const float *Jb = J_all + b * (long)nch * P * LC * 20;
    float *Cg = C_all + b * (long)S * S;
    for (int i = t; i < S * S; i += 256) C[i] = Cg[i];
    for (int i = t; i < 100; i += 256) H[i] = 0.f;
    for (int i = t; i < TL * TL; i += 256) A[i] = 0.f;
    for (int i = t; i < S * TL; i += 256) BA[i] = 0.f;
    __syncthreads();
    for (int ch = 0; ch < nch; ch++) {
        // (1)
        for (int i = t; i < TL * 3; i += 256) {  // diagonal blocks: row I + r, col I + c
            const int blk = i / 9, r = (i % 9) / 3, c = i % 3, I = 3 * blk;
            A[(I + r) * TL + I + c] = 0.f;
        }
        for (int i = t; i < S * TL; i += 256) B[i] = 0.f;
        __syncthreads();
        // (2)
        if (t < 64) {
            const float *Jc = Jb + (long)ch * P * LC * 20;
            for (int ci = 0; ci < LC; ci++)
                for (int p = 0; p < P; p++) {
                    const int pi = p * 6, li = ci * 3;
                    const float *Jf = Jc + 20 * (as_built ? p * ci : ci * P + p);
                    // matmul2(10, 10, 2, J, J, H, H, 2, 2, 10, 10, 1, 1, 0, false, true)
                    for (int e = lane; e < 100; e += 64) {
                        const int i = e / 10, j = e % 10;
                        float v = __fmul_rn(0.f, H[e]);
                        v = __fadd_rn(v, __fmul_rn(__fmul_rn(__fmul_rn(1.f, Jf[2 * i]), 1.f), Jf[2 * j]));
                        v = __fadd_rn(v, __fmul_rn(__fmul_rn(__fmul_rn(1.f, Jf[2 * i + 1]), 1.f), Jf[2 * j + 1]));
                        H[e] = v;
                    }
                    wsync();
                    // matrix_add targets (C[j * sC + i] = 1 * A[j * sA + i] + 1 * C[...]): 72 entries
                    int e = lane;
                    for (int rep = 0; rep < 2; rep++, e += 64) {
                        if (e < 9) {  // H_LL -> A block
                            const int i = e % 3, j = e / 3;
                            float &d = A[li * (TL + 1) + j * TL + i];
                            d = __fadd_rn(__fmul_rn(1.f, H[j * 10 + i]), __fmul_rn(1.f, d));
                        } else if (e < 27) {  // H_PL -> B
                            const int q = e - 9, i = q % 6, j = q / 6;
                            float &d = B[pi + li * S + j * S + i];
                            d = __fadd_rn(__fmul_rn(1.f, H[3 + j * 10 + i]), __fmul_rn(1.f, d));
                        } else if (e < 30) {  // landmark-residual -> B's last row
                            const int j = e - 27;
                            float &d = B[(li + 1) * S - 1 + j * S];
                            d = __fadd_rn(__fmul_rn(1.f, H[9 + j * 10]), __fmul_rn(1.f, d));
                        } else if (e < 66) {  // H_PP -> C
                            const int q = e - 30, i = q % 6, j = q / 6;
                            float &d = C[pi * (S + 1) + j * S + i];
                            d = __fadd_rn(__fmul_rn(1.f, H[33 + j * 10 + i]), __fmul_rn(1.f, d));
                        } else if (e < 72) {  // pose-residual -> C's last row
                            const int j = e - 66;
                            float &d = C[(pi + 1) * S - 1 + j * S];
                            d = __fadd_rn(__fmul_rn(1.f, H[39 + j * 10]), __fmul_rn(1.f, d));
                        }
                    }
                    wsync();
                }
        }
        __syncthreads();
        // (3) invert_3x3 of each diagonal block (column-major copy, cofactors / det)
        if (t < LC) {
            float *m = A + (3 * t) * TL + 3 * t;
            float a[9], v[9];
            for (int j = 0; j < 3; j++)
                for (int i = 0; i < 3; i++) a[j * 3 + i] = m[j * TL + i];
            const float det = __fadd_rn(
                __fsub_rn(__fmul_rn(a[0], __fsub_rn(__fmul_rn(a[4], a[8]), __fmul_rn(a[5], a[7]))),
                          __fmul_rn(a[1], __fsub_rn(__fmul_rn(a[3], a[8]), __fmul_rn(a[5], a[6])))),
                __fmul_rn(a[2], __fsub_rn(__fmul_rn(a[3], a[7]), __fmul_rn(a[4], a[6]))));
            v[0] = __fsub_rn(__fmul_rn(a[4], a[8]), __fmul_rn(a[5], a[7])) / det;
            v[1] = __fsub_rn(__fmul_rn(a[2], a[7]), __fmul_rn(a[1], a[8])) / det;
            v[2] = __fsub_rn(__fmul_rn(a[1], a[5]), __fmul_rn(a[2], a[4])) / det;
            v[3] = __fsub_rn(__fmul_rn(a[5], a[6]), __fmul_rn(a[3], a[8])) / det;
            v[4] = __fsub_rn(__fmul_rn(a[0], a[8]), __fmul_rn(a[2], a[6])) / det;
            v[5] = __fsub_rn(__fmul_rn(a[2], a[3]), __fmul_rn(a[0], a[5])) / det;
            v[6] = __fsub_rn(__fmul_rn(a[3], a[7]), __fmul_rn(a[4], a[6])) / det;
            v[7] = __fsub_rn(__fmul_rn(a[1], a[6]), __fmul_rn(a[0], a[7])) / det;
            v[8] = __fsub_rn(__fmul_rn(a[0], a[4]), __fmul_rn(a[1], a[3])) / det;
            for (int j = 0; j < 3; j++)
                for (int i = 0; i < 3; i++) m[j * TL + i] = v[j * 3 + i];
        }
        __syncthreads();
        // (4) BA[i][j] (stride S) = 0 * BA + sum_k A[i][k] B[k][j]   (i < TL, j < 6P)
        for (int e = t; e < TL * 6 * P; e += 256) {
            const int i = e / (6 * P), j = e % (6 * P);
            float v = __fmul_rn(0.f, BA[i * S + j]);
            for (int k = 0; k < TL; k++)
                v = __fadd_rn(v, __fmul_rn(__fmul_rn(__fmul_rn(1.f, A[i * TL + k]), 1.f), B[k * S + j]));
            BA[i * S + j] = v;
        }
        __syncthreads();
        // (5) C[i][j] (stride S) = 1 * C + sum_k (-1 * B[k][i]) * 1 * BA[k][j]   (i, j < 6P)
        for (int e = t; e < 36 * P * P; e += 256) {
            const int i = e / (6 * P), j = e % (6 * P);
            float v = __fmul_rn(1.f, C[i * S + j]);
            for (int k = 0; k < TL; k++)
                v = __fadd_rn(v, __fmul_rn(__fmul_rn(__fmul_rn(-1.f, B[k * S + i]), 1.f), BA[k * S + j]));
            C[i * S + j] = v;
        }
        __syncthreads();
    }
    for (int i = t; i < S * S; i += 256) Cg[i] = C[i];
}

}  // namespace

extern "C" int mv_lba_schur_dev(mv_context *ctx, int batch, int num_poses, int num_ldmks, int chunk, int semantics,
                                const float *J, float *C) {
    MV_REQUIRE(ctx && batch > 0 && num_poses > 0 && num_ldmks > 0 && chunk > 0 && J && C);
    MV_REQUIRE(semantics == MV_AS_BUILT || semantics == MV_AS_INTENDED);
    const long S = 6l * num_poses + 1, TL = 3l * chunk;
    const long lds = 4 * (100 + TL * TL + 2 * S * TL + S * S);
    MV_REQUIRE(lds <= 64 * 1024);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    MV_PROF_BEGIN(ctx->stream, "k_lba_schur");
    hipLaunchKernelGGL(k_lba_schur, dim3((unsigned)batch), dim3(256), (size_t)lds, ctx->stream, num_poses, num_ldmks,
                       chunk, semantics == MV_AS_BUILT ? 1 : 0, J, C);
    MV_PROF_END(ctx->stream);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}
