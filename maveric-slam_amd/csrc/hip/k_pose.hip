// k_pose.hip -- pose stage on gfx950.
//
// As-built (src/pnp_solver.c, bit-exact):
//   compute_essential_matrix is a stub returning E = I (:80-85); RANSAC counts
//   ||E [p1;1] - [p2;1]||^2 < thr in PIXELS (:89-105,143-149) and keeps the
//   first iteration's inlier list (equal counts never replace it, :152); the
//   pose is the McAdams SVD of E (R1 = U W, t = U[:,2], :168-194).
// As-intended (k_pose_ransac in k_pose_intended.hip): normalised 8-point
// hypotheses, Sampson scoring, cheirality, Gauss-Newton refinement.
#include "mv_internal.hpp"
#include "mv_svd3.hpp"

namespace {

using mv::Mat3;

// pnp_solver.c:89-105, evaluated exactly as the reference does
__device__ __forceinline__ float reproj_error(float x1, float y1, float x2, float y2, const Mat3 &E) {
    const float p1[3] = {x1, y1, 1.0f}, p2[3] = {x2, y2, 1.0f};
    float err = 0;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float t = E.m[i][0] * p1[0] + E.m[i][1] * p1[1] + E.m[i][2] * p1[2];
        const float d = t - p2[i];
        err += d * d;
    }
    return err;
}

__device__ __forceinline__ Mat3 identity3() {
    Mat3 E;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) E.m[i][j] = i == j ? 1.0f : 0.0f;
    return E;
}

__global__ void k_svd3(const float *A, float *U, float *S, float *V) {
    if (threadIdx.x != 0) return;
    Mat3 a, u, v;
    for (int i = 0; i < 9; i++) a.m[i / 3][i % 3] = A[i];
    float s[3];
    mv::svd3(a, u, s, v);
    for (int i = 0; i < 9; i++) {
        U[i] = u.m[i / 3][i % 3];
        V[i] = v.m[i / 3][i % 3];
    }
    for (int i = 0; i < 3; i++) S[i] = s[i];
}

__global__ void k_recover_pose(const float *E, float *R1, float *R2, float *t) {
    if (threadIdx.x != 0) return;
    Mat3 e, r1, r2;
    for (int i = 0; i < 9; i++) e.m[i / 3][i % 3] = E[i];
    float tt[3];
    mv::recover_pose_mcadams(e, r1, r2, tt);
    for (int i = 0; i < 9; i++) {
        R1[i] = r1.m[i / 3][i % 3];
        R2[i] = r2.m[i / 3][i % 3];
    }
    for (int i = 0; i < 3; i++) t[i] = tt[i];
}

// Block-ordered compaction of an inlier list (order = point index), cap 1000.
template <int NT>
__device__ __forceinline__ int block_scan_excl(int v, int *total, int *wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
        int s = lane < NT / 64 ? wsum[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < NT / 64) wsum[lane] = s;
    }
    __syncthreads();
    const int off = (w > 0 ? wsum[w - 1] : 0) + x - v;
    *total = wsum[NT / 64 - 1];
    __syncthreads();
    return off;
}

// single pair stub RANSAC (one 256-thread block), pts as [n][2]
__global__ __launch_bounds__(256) void k_ransac_stub(int n, const float *__restrict__ p1,
                                                     const float *__restrict__ p2, float thr,
                                                     float *__restrict__ E_out, int *__restrict__ inliers,
                                                     int *__restrict__ num_inliers) {
    __shared__ int wsum[4];
    const Mat3 E = identity3();
    const int per = (n + 255) / 256;
    const int i0 = threadIdx.x * per, i1 = min(i0 + per, n);
    int cnt = 0;
    for (int i = i0; i < i1; i++)
        if (reproj_error(p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1], E) < thr) cnt++;
    int total;
    int k = block_scan_excl<256>(cnt, &total, wsum);
    for (int i = i0; i < i1; i++)
        if (reproj_error(p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1], E) < thr) {
            if (k < 1000) inliers[k] = i;
            k++;
        }
    if (threadIdx.x == 0) {
        *num_inliers = min(total, 1000);
        for (int i = 0; i < 9; i++) E_out[i] = E.m[i / 3][i % 3];
    }
}

// ---------------------------------------------------------------------------
// Batched pose, as-built semantics.  One block per pair.  Correspondences are
// either explicit (pts0/pts1 [cap][2], n[b]) or an all-pairs match
// (kp0 [cap][2] with match_idx[cap] into kp1 [cap][2]), in query order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pose_as_built(int cap, const int *__restrict__ nv,
                                                       const float *__restrict__ pts0,
                                                       const float *__restrict__ pts1,
                                                       const int *__restrict__ match_idx,
                                                       const float *__restrict__ kp1, float thr,
                                                       float *__restrict__ T, int *__restrict__ num_matches,
                                                       int *__restrict__ num_inliers, int *__restrict__ status) {
    __shared__ int wsum[4];
    const int b = blockIdx.x;
    const int n = min(max(nv[b], 0), cap);  // as every batched kernel: never past the pair's slot
    const Mat3 E = identity3();
    const int per = (n + 255) / 256;
    const int i0 = threadIdx.x * per, i1 = min(i0 + per, n);
    int cnt = 0, nm = 0;
    for (int i = i0; i < i1; i++) {
        float x1 = pts0[((size_t)b * cap + i) * 2], y1 = pts0[((size_t)b * cap + i) * 2 + 1], x2, y2;
        if (match_idx) {
            const int j = match_idx[(size_t)b * cap + i];
            if ((unsigned)j >= (unsigned)cap) continue;  // -1 or out of range: no match
            x2 = kp1[((size_t)b * cap + j) * 2];
            y2 = kp1[((size_t)b * cap + j) * 2 + 1];
        } else {
            x2 = pts1[((size_t)b * cap + i) * 2];
            y2 = pts1[((size_t)b * cap + i) * 2 + 1];
        }
        nm++;
        if (reproj_error(x1, y1, x2, y2, E) < thr) cnt++;
    }
    int tot_in, tot_m;
    (void)block_scan_excl<256>(cnt, &tot_in, wsum);
    (void)block_scan_excl<256>(nm, &tot_m, wsum);
    if (threadIdx.x == 0) {
        Mat3 R1, R2;
        float t[3];
        mv::recover_pose_mcadams(E, R1, R2, t);
        float *o = T + (size_t)b * 12;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) o[i * 4 + j] = R1.m[i][j];
            o[i * 4 + 3] = t[i];
        }
        num_inliers[b] = min(tot_in, 1000);
        if (num_matches) num_matches[b] = tot_m;
        status[b] = tot_m > 0 ? (tot_in > 0 ? MV_OK : MV_ERR_DEGENERATE) : MV_ERR_NO_POINTS;
    }
}

}  // namespace

namespace mv {

int launch_intended_pose(hipStream_t s, void *scratch, const mv_pose_params *p, int batch, int cap, const int *n,
                         const float *pts0, const float *pts1, const int *match_idx, const float *kp1, float *T,
                         int *num_matches, int *num_inliers, int *status);
size_t intended_pose_scratch_bytes(int batch, int cap);

size_t pose_scratch_bytes(int batch, int cap) { return intended_pose_scratch_bytes(batch, cap); }

int launch_pose(hipStream_t s, void *scratch, const mv_pose_params *p, int batch, int cap, const int *n,
                const float *pts0, const float *pts1, const int *match_idx, const float *kp1, float *T,
                int *num_matches, int *num_inliers, int *status) {
    MV_REQUIRE(p && batch > 0 && cap > 0 && n && pts0 && T && num_inliers && status);
    MV_REQUIRE(match_idx ? kp1 != nullptr : pts1 != nullptr);
    if (p->semantics == MV_AS_BUILT) {
        hipLaunchKernelGGL(k_pose_as_built, dim3(batch), dim3(256), 0, s, cap, n, pts0, pts1, match_idx, kp1,
                           p->inlier_thresh, T, num_matches, num_inliers, status);
        MV_LAUNCH_CHECK();
        return MV_OK;
    }
    return launch_intended_pose(s, scratch, p, batch, cap, n, pts0, pts1, match_idx, kp1, T, num_matches,
                                num_inliers, status);
}

int launch_ransac_stub(hipStream_t s, int n, const float *pts1, const float *pts2, float thresh, float *E,
                       int *inliers, int *num_inliers) {
    hipLaunchKernelGGL(k_ransac_stub, dim3(1), dim3(256), 0, s, n, pts1, pts2, thresh, E, inliers, num_inliers);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

int launch_recover_pose(hipStream_t s, const float *E, float *R1, float *R2, float *t) {
    hipLaunchKernelGGL(k_recover_pose, dim3(1), dim3(64), 0, s, E, R1, R2, t);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

int launch_svd3(hipStream_t s, const float *A, float *U, float *S, float *V) {
    hipLaunchKernelGGL(k_svd3, dim3(1), dim3(64), 0, s, A, U, S, V);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv
