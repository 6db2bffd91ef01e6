// k_allpairs_i8.hip -- all-pairs int8 descriptor match (BASELINE config 5: quantized
// SuperPoint descriptors, 2048 kp/frame) on the int8 matrix cores.
//
// Score: the exact cosine of squared_dist/check_dist (src/tracking_main.c:18-57)
// over all 256 dims: a match needs dot > 0 and 100 dot^2 > 81 |a|^2 |b|^2
// (cos > MATCH_THRESHOLD 0.9); the kept j is the FIRST maximiser of
// dot^2 / |b|^2 (the cosine at fixed query).  Integer-exact.
//
//   k_i8_norms    |x|^2 of every row of both frames (v_dot4)
//   k_i8_screen   D = A . B^T with v_mfma_i32_32x32x32_i8 (exact int32), 128x128
//                 tile, the whole K = 256 panel staged once in LDS (2 x 32 KiB);
//                 epilogue f = dot * rsqrt|b|^2 for dot > 0, per-row (max1, idx1, max2)
//   k_i8_resolve  exact re-score of every candidate with f >= M (1 - 1e-5):
//                 integer dot, u128 cross-multiplied comparison, exact threshold.
// Per pair at 2048 kp: 2 * 2048^2 * 256 = 2.147 GOP on 2 x 512 KiB; MFMA-int8 bound.
#include <math.h>

#include "mv_internal.hpp"

namespace {

constexpr int BM = 128, BN = 128, KD = 256;
constexpr int LDR = KD + 16;      // bytes per staged row (272 B: conflict-free ds_read_b128)
constexpr int LDC = BM + 4;       // floats, transposed score tile
constexpr int STAGE_BYTES = 2 * BM * LDR;
constexpr int C_BYTES = BN * LDC * 4;
constexpr int LDS_BYTES = STAGE_BYTES > C_BYTES ? STAGE_BYTES : C_BYTES;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

struct Partial {
    float max1;
    int idx1;
    float max2;
    float pad;
};

__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total / 8, r = total % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__global__ __launch_bounds__(256) void k_i8_norms(long rows, const int8_t *__restrict__ d, int *__restrict__ nrm,
                                                  float *__restrict__ rnrm) {
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const int4 *p = reinterpret_cast<const int4 *>(d + r * KD);
    int s = 0;
#pragma unroll
    for (int v = 0; v < 16; v++) {
        int4 x = p[v];
        s = __builtin_amdgcn_sdot4(x.x, x.x, s, false);
        s = __builtin_amdgcn_sdot4(x.y, x.y, s, false);
        s = __builtin_amdgcn_sdot4(x.z, x.z, s, false);
        s = __builtin_amdgcn_sdot4(x.w, x.w, s, false);
    }
    nrm[r] = s;
    if (rnrm) rnrm[r] = s > 0 ? 1.0f / sqrtf((float)s) : 0.f;
}

__global__ __launch_bounds__(256, 2) void k_i8_screen(int tiles_r, int tiles_c, int cap, const int *__restrict__ n0v,
                                                      const int *__restrict__ n1v, const int8_t *__restrict__ desc0,
                                                      const int8_t *__restrict__ desc1,
                                                      const float *__restrict__ rnb, Partial *__restrict__ part) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    char *As = lds;
    char *Bs = lds + BM * LDR;
    const int per_pair = tiles_r * tiles_c;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int pair = L / per_pair, tile = L % per_pair;
    const int tr = tile / tiles_c, tc = tile % tiles_c;
    const int n0 = n0v[pair], n1 = n1v[pair];
    if (tr * BM >= n0 || tc * BN >= n1) return;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
    const int8_t *A = desc0 + (size_t)pair * cap * KD;
    const int8_t *B = desc1 + (size_t)pair * cap * KD;
    // stage the full K panels: 128 rows x 256 B each, 16 lanes per row
#pragma unroll
    for (int it = 0; it < 8; it++) {
        const int row = it * 16 + (t >> 4), ch = t & 15;
        const int ra = min(tr * BM + row, n0 - 1), rb = min(tc * BN + row, n1 - 1);
        int4 xa = *reinterpret_cast<const int4 *>(A + (size_t)ra * KD + ch * 16);
        int4 xb = *reinterpret_cast<const int4 *>(B + (size_t)rb * KD + ch * 16);
        *reinterpret_cast<int4 *>(As + row * LDR + ch * 16) = xa;
        *reinterpret_cast<int4 *>(Bs + row * LDR + ch * 16) = xb;
    }
    __syncthreads();
    i32x16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int g = 0; g < 16; g++) acc[m][n][g] = 0;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int kk = 0; kk < KD / 32; kk++) {
        i32x4 a[2], b[2];
#pragma unroll
        for (int m = 0; m < 2; m++) {
            a[m] = *reinterpret_cast<const i32x4 *>(As + (wr * 64 + m * 32 + fr) * LDR + kk * 32 + fh * 16);
            b[m] = *reinterpret_cast<const i32x4 *>(Bs + (wc * 64 + m * 32 + fr) * LDR + kk * 32 + fh * 16);
        }
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int n = 0; n < 2; n++) acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[m], b[n], acc[m][n], 0, 0, 0);
    }
    __syncthreads();
    float *Ct = reinterpret_cast<float *>(lds);
    const float *rb_pair = rnb + (size_t)pair * cap;
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int col = wc * 64 + n * 32 + fr;
        const int gcol = min(tc * BN + col, n1 - 1);
        const float rn = rb_pair[gcol];
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int row = wr * 64 + m * 32 + 8 * q + 4 * fh;
                float4 v;
                int d0 = acc[m][n][4 * q + 0], d1 = acc[m][n][4 * q + 1], d2 = acc[m][n][4 * q + 2],
                    d3 = acc[m][n][4 * q + 3];
                v.x = d0 > 0 ? (float)d0 * rn : -__builtin_inff();
                v.y = d1 > 0 ? (float)d1 * rn : -__builtin_inff();
                v.z = d2 > 0 ? (float)d2 * rn : -__builtin_inff();
                v.w = d3 > 0 ? (float)d3 * rn : -__builtin_inff();
                *reinterpret_cast<float4 *>(Ct + col * LDC + row) = v;
            }
    }
    __syncthreads();
    const int r = t & (BM - 1), half = t >> 7;
    const int cvalid = min(BN, n1 - tc * BN);
    float m1 = -__builtin_inff(), m2 = -__builtin_inff();
    int i1 = -1;
    const int cb = half * 64, ce = min(cb + 64, cvalid);
    for (int c = cb; c < ce; c++) {
        const float v = Ct[c * LDC + r];
        if (v > m1) {
            m2 = m1;
            m1 = v;
            i1 = tc * BN + c;
        } else if (v > m2) {
            m2 = v;
        }
    }
    __syncthreads();
    float *mx = Ct;
    if (half == 1) {
        mx[r] = m1;
        reinterpret_cast<int *>(mx)[BM + r] = i1;
        mx[2 * BM + r] = m2;
    }
    __syncthreads();
    if (half == 0) {
        const float u1 = mx[r], u2 = mx[2 * BM + r];
        const int ui = reinterpret_cast<int *>(mx)[BM + r];
        if (u1 > m1) {
            m2 = fmaxf(m1, u2);
            m1 = u1;
            i1 = ui;
        } else {
            m2 = fmaxf(m2, u1);
        }
        const int grow = tr * BM + r;
        if (grow < n0) part[((size_t)pair * cap + grow) * tiles_c + tc] = Partial{m1, i1, m2, 0.f};
    }
}

__device__ __forceinline__ int exact_dot_i8(const int8_t *a, const int8_t *b) {
    const int4 *p = reinterpret_cast<const int4 *>(a);
    const int4 *q = reinterpret_cast<const int4 *>(b);
    int s = 0;
#pragma unroll
    for (int v = 0; v < 16; v++) {
        int4 x = p[v], y = q[v];
        s = __builtin_amdgcn_sdot4(x.x, y.x, s, false);
        s = __builtin_amdgcn_sdot4(x.y, y.y, s, false);
        s = __builtin_amdgcn_sdot4(x.z, y.z, s, false);
        s = __builtin_amdgcn_sdot4(x.w, y.w, s, false);
    }
    return s;
}

// candidate (dot, nb, j) strictly better than current best?  max dot^2/nb, ties -> lower j
__device__ __forceinline__ bool better(long long d, long long nb, int j, long long bd, long long bn, int bj) {
    if (bj < 0) return true;
    unsigned __int128 l = (unsigned __int128)(unsigned long long)(d * d) * (unsigned long long)bn;
    unsigned __int128 r = (unsigned __int128)(unsigned long long)(bd * bd) * (unsigned long long)nb;
    return l > r || (l == r && j < bj);
}

__global__ __launch_bounds__(256) void k_i8_resolve(int tiles_c, int cap, const int *__restrict__ n0v,
                                                    const int *__restrict__ n1v, const int8_t *__restrict__ desc0,
                                                    const int8_t *__restrict__ desc1, const int *__restrict__ na_v,
                                                    const int *__restrict__ nb_v, const Partial *__restrict__ part,
                                                    int *__restrict__ match_idx, int *__restrict__ match_dot) {
    const int pair = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= cap) return;
    const int n0 = n0v[pair], n1 = n1v[pair];
    int best = -1;
    long long bd = 0, bn = 1;
    if (i < n0 && n1 > 0) {
        const long long na = na_v[(size_t)pair * cap + i];
        const int8_t *a = desc0 + ((size_t)pair * cap + i) * KD;
        const int8_t *B = desc1 + (size_t)pair * cap * KD;
        const int *nb = nb_v + (size_t)pair * cap;
        const Partial *p = part + ((size_t)pair * cap + i) * tiles_c;
        const int tiles = (n1 + BN - 1) / BN;
        float M = -__builtin_inff();
        for (int tt = 0; tt < tiles; tt++) M = fmaxf(M, p[tt].max1);
        if (na > 0 && M > 0.f) {
            const float win = M * (1.0f - 1e-5f);
            for (int tt = 0; tt < tiles; tt++) {
                const Partial q = p[tt];
                int jb = tt * BN, je = jb;
                if (q.max2 >= win)
                    je = min(jb + BN, n1);
                else if (q.max1 >= win) {
                    jb = q.idx1;
                    je = jb + 1;
                }
                for (int j = jb; j < je; j++) {
                    const long long d = exact_dot_i8(a, B + (size_t)j * KD);
                    const long long nbj = nb[j];
                    if (d <= 0 || nbj == 0) continue;
                    if (better(d, nbj, j, bd, bn, best)) {
                        best = j;
                        bd = d;
                        bn = nbj;
                    }
                }
            }
            if (best >= 0 && !((unsigned __int128)(100ll * bd * bd) >
                               (unsigned __int128)81 * (unsigned long long)(na * bn)))
                best = -1;
        }
    }
    match_idx[(size_t)pair * cap + i] = best;
    match_dot[(size_t)pair * cap + i] = best >= 0 ? (int)bd : 0;
}

}  // namespace

namespace mv {

size_t allpairs_i8_scratch_bytes(int batch, int cap) {
    const int tiles_c = (cap + BN - 1) / BN;
    const size_t rows = (size_t)batch * cap;
    return align_up(sizeof(Partial) * rows * tiles_c, 256) + 3 * align_up(4 * rows, 256);
}

int launch_allpairs_i8(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                       const int8_t *desc0, const int8_t *desc1, int *match_idx, int *match_dot) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx && match_dot && scratch);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    const int tiles_r = (cap + BM - 1) / BM, tiles_c = (cap + BN - 1) / BN;
    const size_t rows = (size_t)batch * cap;
    char *p = (char *)scratch;
    Partial *part = (Partial *)p;
    p += align_up(sizeof(Partial) * rows * tiles_c, 256);
    int *na = (int *)p;
    p += align_up(4 * rows, 256);
    int *nb = (int *)p;
    p += align_up(4 * rows, 256);
    float *rnb = (float *)p;
    const int nblk = (int)((rows + 255) / 256);
    MV_PROF_BEGIN(s, "k_i8_norms");
    hipLaunchKernelGGL(k_i8_norms, dim3(nblk), dim3(256), 0, s, (long)rows, desc0, na, (float *)nullptr);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    MV_PROF_BEGIN(s, "k_i8_norms");
    hipLaunchKernelGGL(k_i8_norms, dim3(nblk), dim3(256), 0, s, (long)rows, desc1, nb, rnb);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    const long blocks = (long)batch * tiles_r * tiles_c;
    MV_REQUIRE(blocks < (1l << 31));
    MV_PROF_BEGIN(s, "k_i8_screen");
    hipLaunchKernelGGL(k_i8_screen, dim3((unsigned)blocks), dim3(256), 0, s, tiles_r, tiles_c, cap, n0, n1, desc0,
                       desc1, rnb, part);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    MV_PROF_BEGIN(s, "k_i8_resolve");
    hipLaunchKernelGGL(k_i8_resolve, dim3((cap + 255) / 256, batch), dim3(256), 0, s, tiles_c, cap, n0, n1, desc0,
                       desc1, na, nb, part, match_idx, match_dot);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

extern "C" int mv_match_allpairs_i8_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                        const int8_t *desc0, const int8_t *desc1, int *match_idx, int *match_dot) {
    MV_REQUIRE(ctx != nullptr);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    void *scr = mv::scratch(ctx, mv::allpairs_i8_scratch_bytes(batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    return mv::launch_allpairs_i8(ctx->stream, scr, batch, cap, n0, n1, desc0, desc1, match_idx, match_dot);
}
