// k_trajectory.hip -- trajectory chaining (python/compute_trajectory.py:53-90), SURVEY §8(f)3.
//
// k_chain: one wave per sequence walks the relative transforms IN ORDER (the reference's
// sequential float64 rounding is the contract, so no tree scan).  Lane e < 12 owns entry
// (i, j) = (e / 4, e % 4) of [R | t]; per step it fetches column j of the current pose from
// lanes j, 4 + j, 8 + j (three 64-bit shuffles) and its own row i of the relative transform:
//   R'_ij = (Rr_i0 R_0j + Rr_i1 R_1j) + Rr_i2 R_2j                       (j < 3, both modes)
//   t'_i  = t_rel_i + t_i                          MV_CHAIN_AS_BUILT  (compute_trajectory.py:79)
//   t'_i  = ((Rr_i0 t_0 + Rr_i1 t_1) + Rr_i2 t_2) + t_rel_i   MV_CHAIN_COMPOSE (4x4 T_rel . pose)
// mul then add (no FMA), matching numpy on these shapes (the committed PLYs reproduce bit for
// bit).  The block stages 256 steps of relative transforms through LDS (24 KiB) with all 64
// lanes, so the walk itself only reads LDS: latency-bound, ~100-200 cycles per step.
// k_rebase: elementwise, one thread per pose.
#include "mv_internal.hpp"
#include "trajectory.h"

namespace {

constexpr int CHUNK = 256;  // steps staged per LDS round

__device__ __forceinline__ double shfl_d(double v, int src) {
    return __shfl(v, src, 64);
}

__global__ __launch_bounds__(64) void k_chain(int len, const double *__restrict__ rel, const int *__restrict__ present,
                                              const double *__restrict__ start, int mode,
                                              double *__restrict__ poses) {
    __shared__ double srel[CHUNK * 12];
    __shared__ int spres[CHUNK];
    const int b = blockIdx.x, lane = threadIdx.x;
    const int e = lane < 12 ? lane : 11, i = e >> 2, j = e & 3;
    const double *R = rel + (size_t)b * len * 12;
    const int *P = present ? present + (size_t)b * len : nullptr;
    double *O = poses + (size_t)b * (len + 1) * 12;
    double cur = start ? start[(size_t)b * 12 + e] : (j == i ? 1.0 : 0.0);
    if (lane < 12) O[e] = cur;
    for (int k0 = 0; k0 < len; k0 += CHUNK) {
        const int nk = min(CHUNK, len - k0);
        __syncthreads();  // (one wave: orders the previous round's reads before the refill)
        for (int x = lane; x < nk * 12; x += 64) srel[x] = R[(size_t)k0 * 12 + x];
        for (int x = lane; x < nk; x += 64) spres[x] = P ? P[k0 + x] : 1;
        __syncthreads();
        for (int k = 0; k < nk; k++) {
            const double c0 = shfl_d(cur, j), c1 = shfl_d(cur, 4 + j), c2 = shfl_d(cur, 8 + j);
            if (!spres[k]) {  // missing transform: the pose carries over (no output row is skipped here)
                if (lane < 12) O[(size_t)(k0 + k + 1) * 12 + e] = cur;
                continue;
            }
            const double *r = srel + k * 12 + 4 * i;
            double v;
            if (j < 3 || mode == MV_CHAIN_COMPOSE) {
                v = __dadd_rn(__dadd_rn(__dmul_rn(r[0], c0), __dmul_rn(r[1], c1)), __dmul_rn(r[2], c2));
                if (j == 3) v = __dadd_rn(v, r[3]);
            } else {
                v = __dadd_rn(r[3], cur);
            }
            cur = v;
            if (lane < 12) O[(size_t)(k0 + k + 1) * 12 + e] = cur;
        }
    }
}

__global__ __launch_bounds__(256) void k_rebase(long total, int len1, const double *__restrict__ base, int mode,
                                                double *__restrict__ poses) {
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= total) return;
    const long b = q / len1;
    const double *S = base + b * 12;
    double *p = poses + q * 12;
    double P[12], O[12];
#pragma unroll
    for (int x = 0; x < 12; x++) P[x] = p[x];
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            // pose_k applied after base: [R_k | t_k] . [R_s | t_s]
            double v = __dadd_rn(__dadd_rn(__dmul_rn(P[4 * r], S[c]), __dmul_rn(P[4 * r + 1], S[4 + c])),
                                 __dmul_rn(P[4 * r + 2], S[8 + c]));
            if (c == 3) v = mode == MV_CHAIN_COMPOSE ? __dadd_rn(v, P[4 * r + 3]) : __dadd_rn(P[4 * r + 3], S[4 * r + 3]);
            O[4 * r + c] = v;
        }
    }
#pragma unroll
    for (int x = 0; x < 12; x++) p[x] = O[x];
}

}  // namespace

extern "C" int mv_trajectory_chain_dev(mv_context *ctx, int batch, int len, const double *rel, const int *present,
                                       const double *start, int mode, double *poses) {
    MV_REQUIRE(ctx && batch > 0 && len >= 0 && (rel || len == 0) && poses);
    MV_REQUIRE(mode == MV_CHAIN_AS_BUILT || mode == MV_CHAIN_COMPOSE);
    MV_REQUIRE(batch < (1 << 30));
    MV_HIP_TRY(hipSetDevice(ctx->device));
    MV_PROF_BEGIN(ctx->stream, "k_chain");
    hipLaunchKernelGGL(k_chain, dim3((unsigned)batch), dim3(64), 0, ctx->stream, len, rel, present, start, mode, poses);
    MV_PROF_END(ctx->stream);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}

extern "C" int mv_trajectory_rebase_dev(mv_context *ctx, int batch, int len1, const double *base, int mode,
                                        double *poses) {
    MV_REQUIRE(ctx && batch > 0 && len1 > 0 && base && poses);
    MV_REQUIRE(mode == MV_CHAIN_AS_BUILT || mode == MV_CHAIN_COMPOSE);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const long total = (long)batch * len1;
    MV_REQUIRE(total < (1l << 40));
    hipLaunchKernelGGL(k_rebase, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, ctx->stream, total, len1, base,
                       mode, poses);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}

extern "C" int mv_trajectory_chain_host(mv_context *ctx, int len, const double *rel, const int *present,
                                        const double *start, int mode, double *poses) {
    MV_REQUIRE(ctx && len >= 0 && (rel || len == 0) && poses);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const size_t brel = mv::align_up((size_t)len * 96 + 8, 256), bpres = mv::align_up((size_t)len * 4 + 4, 256);
    const size_t bst = 256, bout = mv::align_up((size_t)(len + 1) * 96, 256);
    char *d = (char *)mv::stage(ctx, brel + bpres + bst + bout);
    if (!d) return MV_ERR_OUT_OF_MEMORY;
    double *d_rel = (double *)d;
    int *d_pres = (int *)(d + brel);
    double *d_start = (double *)(d + brel + bpres);
    double *d_out = (double *)(d + brel + bpres + bst);
    hipStream_t s = ctx->stream;
    if (len > 0) MV_HIP_TRY(hipMemcpyAsync(d_rel, rel, (size_t)len * 96, hipMemcpyHostToDevice, s));
    if (present && len > 0) MV_HIP_TRY(hipMemcpyAsync(d_pres, present, (size_t)len * 4, hipMemcpyHostToDevice, s));
    if (start) MV_HIP_TRY(hipMemcpyAsync(d_start, start, 96, hipMemcpyHostToDevice, s));
    const int st = mv_trajectory_chain_dev(ctx, 1, len, d_rel, present ? d_pres : nullptr, start ? d_start : nullptr,
                                           mode, d_out);
    if (st != MV_OK) return st;
    MV_HIP_TRY(hipMemcpyAsync(poses, d_out, (size_t)(len + 1) * 96, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    return mv::set_status(MV_OK);
}
