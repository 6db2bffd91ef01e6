// k_pose_intended.hip -- the pose the reference INTENDS (src/pnp_solver.c:36-86's
// 8-point design matrix, python/pairwise_pnp.py:667-694's findEssentialMat +
// recoverPose), as one 256-thread workgroup per frame-pair:
//
//   1. correspondences compacted into LDS in query order, normalised by K
//      (pnp_solver.c:28-34);
//   2. RANSAC: each lane draws 8 distinct samples (counter-based hash RNG),
//      builds the 8x9 design matrix in the reference's column order
//      (pnp_solver.c:42-50), and takes its null vector from a Householder QR
//      of A^T (backward stable, no pivoting, static register indexing);
//      hypotheses are MSAC-scored (sum of min(Sampson^2, (thr_px / f)^2)) on an evenly
//      strided subset of 128 correspondences (LDS broadcast reads);
//   3. preemption: the 2 best of each wave survive and are MSAC-scored on ALL
//      correspondences by the whole block; lowest (cost, hypothesis id) -> E;
//   4. E = U diag(s1,s2,s3) V^T (double Jacobi on E^T E), the four (R, t)
//      candidates R = U W V^T / U W^T V^T, t = +-u3, cheirality vote by
//      triangulated depth over the inliers (block reduction);
//   5. Gauss-Newton: residual r_i = (x2^T [t]x R x1) / s_i (Sampson), inliers
//      re-selected each iteration at min(thr, 3 rms) so outliers that fell inside
//      the RANSAC band drop out (exact data converges to machine precision),
//      per-correspondence Jacobian d r / d(omega, tangent(t)) (5 dof),
//      J^T J and J^T r assembled with wave64 shuffle reductions + LDS
//      (the [J|r]^T[J|r] pattern of src/local_bundle_adjustment.c:161-176),
//      5x5 LM-damped Cholesky solve in one lane, R <- exp(omega) R,
//      t <- normalise(t + B d).  The Gauss-Newton state, the per-correspondence terms, the
//      22 sums and the solve are float (the output is float).  Stops early once the step is below 1e-7 and the
//      inlier band is unchanged (refine_iters is the maximum).
// Output T = [R | t] with x1 ~ R x0 + t, |t| = 1 (the OpenCV recoverPose convention).
#include <math.h>

#include "mv_internal.hpp"

namespace {

constexpr int NT = 256;
// timing experiments only (wrong results): skip the GN per-point pass / reduction / solve
#ifndef PE_NOPOINTS
#define PE_NOPOINTS 0
#endif
#ifndef PE_NORED
#define PE_NORED 0
#endif
#ifndef PE_TRACE
#define PE_TRACE 0  // printf per-phase clock64() deltas of block 0 (timing experiments only)
#endif
#ifndef PE_NODECOMP
#define PE_NODECOMP 0
#endif
#ifndef PE_NOSCORE
#define PE_NOSCORE 0
#endif
#ifndef PE_NOHYP
#define PE_NOHYP 0
#endif
#ifndef PE_WAVES
#define PE_WAVES 3  // waves per SIMD (4: <= 128 VGPRs, 51 spilled, no faster -- the kernel is VALU-bound)
#endif
#ifndef PE_NOSOLVE
#define PE_NOSOLVE 0
#endif
constexpr int MAXP = 4096;  // correspondences per pair held in LDS (float4 each)

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// null vector of the 8x9 design matrix: Householder QR of A^T (9x8)
__device__ __forceinline__ bool eight_point(const float4 *P, const int idx[8], float e[9]) {
    float M[9][8];
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const float4 p = P[idx[c]];
        const float x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
        M[0][c] = x2 * x1;
        M[1][c] = x2 * y1;
        M[2][c] = x2;
        M[3][c] = y2 * x1;
        M[4][c] = y2 * y1;
        M[5][c] = y2;
        M[6][c] = x1;
        M[7][c] = y1;
        M[8][c] = 1.0f;
    }
    float beta[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float nrm2 = 0.f;
#pragma unroll
        for (int r = k; r < 9; r++) nrm2 += M[r][k] * M[r][k];
        const float nrm = sqrtf(nrm2);
        const float alpha = M[k][k] >= 0.f ? -nrm : nrm;
        M[k][k] -= alpha;  // v = x - alpha e1 stored in column k
        float vtv = 0.f;
#pragma unroll
        for (int r = k; r < 9; r++) vtv += M[r][k] * M[r][k];
        beta[k] = vtv > 0.f ? 2.0f / vtv : 0.f;
#pragma unroll
        for (int j = k + 1; j < 8; j++) {
            float s = 0.f;
#pragma unroll
            for (int r = k; r < 9; r++) s += M[r][k] * M[r][j];
            s *= beta[k];
#pragma unroll
            for (int r = k; r < 9; r++) M[r][j] -= s * M[r][k];
        }
    }
    float z[9];
#pragma unroll
    for (int r = 0; r < 9; r++) z[r] = r == 8 ? 1.f : 0.f;
#pragma unroll
    for (int k = 7; k >= 0; k--) {
        float s = 0.f;
#pragma unroll
        for (int r = k; r < 9; r++) s += M[r][k] * z[r];
        s *= beta[k];
#pragma unroll
        for (int r = k; r < 9; r++) z[r] -= s * M[r][k];
    }
    float n2 = 0.f;
#pragma unroll
    for (int r = 0; r < 9; r++) n2 += z[r] * z[r];
    if (!(n2 > 0.f)) return false;
#pragma unroll
    for (int r = 0; r < 9; r++) e[r] = z[r];
    return true;
}

__device__ __forceinline__ bool sampson_inlier(const float e[9], float4 p, float thr2) {
    const float x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
    const float ex0 = e[0] * x1 + e[1] * y1 + e[2];
    const float ex1 = e[3] * x1 + e[4] * y1 + e[5];
    const float ex2 = e[6] * x1 + e[7] * y1 + e[8];
    const float etx0 = e[0] * x2 + e[3] * y2 + e[6];
    const float etx1 = e[1] * x2 + e[4] * y2 + e[7];
    const float num = x2 * ex0 + y2 * ex1 + ex2;
    const float den = ex0 * ex0 + ex1 * ex1 + etx0 * etx0 + etx1 * etx1;
    return num * num < thr2 * den;
}

// MSAC cost of one correspondence: min(Sampson^2, thr^2) (fast reciprocal: the
// cost only has to be deterministic, not correctly rounded)
__device__ __forceinline__ float msac_cost(const float e[9], float4 p, float thr2, int &inl) {
    const float x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
    const float ex0 = e[0] * x1 + e[1] * y1 + e[2];
    const float ex1 = e[3] * x1 + e[4] * y1 + e[5];
    const float ex2 = e[6] * x1 + e[7] * y1 + e[8];
    const float etx0 = e[0] * x2 + e[3] * y2 + e[6];
    const float etx1 = e[1] * x2 + e[4] * y2 + e[7];
    const float num = x2 * ex0 + y2 * ex1 + ex2;
    const float den = ex0 * ex0 + ex1 * ex1 + etx0 * etx0 + etx1 * etx1;
    const bool in = num * num < thr2 * den;
    inl += in ? 1 : 0;
    return in ? num * num * __builtin_amdgcn_rcpf(den) : thr2;
}

// ---- small double linear algebra (one lane) ----
struct D3 {
    double v[3];
};
__device__ __forceinline__ D3 cross(const D3 &a, const D3 &b) {
    return {{a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2], a.v[0] * b.v[1] - a.v[1] * b.v[0]}};
}
__device__ __forceinline__ double dot3(const D3 &a, const D3 &b) {
    return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2];
}

// symmetric 3x3 eigen-decomposition by cyclic Jacobi (double); columns of V are eigenvectors
__device__ void jacobi_eig3(double A[3][3], double V[3][3], double w[3]) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) V[i][j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 16; sweep++) {
        const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
        if (off < 1e-60) break;
        for (int p = 0; p < 2; p++)
            for (int q = p + 1; q < 3; q++) {
                if (fabs(A[p][q]) < 1e-300) continue;
                const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; k++) {
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; k++) {
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; k++) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < 3; i++) w[i] = A[i][i];
}

// E (row-major double) -> U, V with E ~ U diag(1,1,0) V^T, det U = det V = +1
__device__ void essential_uv(const double E[9], double U[3][3], double V[3][3]) {
    double EtE[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            EtE[i][j] = E[0 * 3 + i] * E[0 * 3 + j] + E[1 * 3 + i] * E[1 * 3 + j] + E[2 * 3 + i] * E[2 * 3 + j];
    double Vr[3][3], w[3];
    jacobi_eig3(EtE, Vr, w);
    int o[3] = {0, 1, 2};  // sort descending
    for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++)
            if (w[o[b]] > w[o[a]]) {
                int t = o[a];
                o[a] = o[b];
                o[b] = t;
            }
    D3 v1 = {{Vr[0][o[0]], Vr[1][o[0]], Vr[2][o[0]]}};
    D3 v2 = {{Vr[0][o[1]], Vr[1][o[1]], Vr[2][o[1]]}};
    D3 v3 = cross(v1, v2);  // right-handed V
    D3 u1, u2;
    for (int i = 0; i < 3; i++) {
        u1.v[i] = E[i * 3 + 0] * v1.v[0] + E[i * 3 + 1] * v1.v[1] + E[i * 3 + 2] * v1.v[2];
        u2.v[i] = E[i * 3 + 0] * v2.v[0] + E[i * 3 + 1] * v2.v[1] + E[i * 3 + 2] * v2.v[2];
    }
    double n1 = sqrt(dot3(u1, u1));
    for (int i = 0; i < 3; i++) u1.v[i] /= n1;
    const double d12 = dot3(u1, u2);  // re-orthogonalise
    for (int i = 0; i < 3; i++) u2.v[i] -= d12 * u1.v[i];
    double n2 = sqrt(dot3(u2, u2));
    for (int i = 0; i < 3; i++) u2.v[i] /= n2;
    D3 u3 = cross(u1, u2);
    for (int i = 0; i < 3; i++) {
        U[i][0] = u1.v[i];
        U[i][1] = u2.v[i];
        U[i][2] = u3.v[i];
        V[i][0] = v1.v[i];
        V[i][1] = v2.v[i];
        V[i][2] = v3.v[i];
    }
}

// float forms for the Gauss-Newton update (one lane per iteration: latency, not throughput)
__device__ __forceinline__ void tangent_basis_f(const float *t, float *b) {
    const float ax[3] = {fabsf(t[0]) < 0.57f ? 1.f : 0.f,
                         fabsf(t[0]) < 0.57f ? 0.f : (fabsf(t[1]) < 0.57f ? 1.f : 0.f),
                         fabsf(t[0]) < 0.57f || fabsf(t[1]) < 0.57f ? 0.f : 1.f};
    float b1[3] = {t[1] * ax[2] - t[2] * ax[1], t[2] * ax[0] - t[0] * ax[2], t[0] * ax[1] - t[1] * ax[0]};
    const float r = 1.f / sqrtf(b1[0] * b1[0] + b1[1] * b1[1] + b1[2] * b1[2]);
    b1[0] *= r;
    b1[1] *= r;
    b1[2] *= r;
    b[0] = b1[0];
    b[1] = b1[1];
    b[2] = b1[2];
    b[3] = t[1] * b1[2] - t[2] * b1[1];
    b[4] = t[2] * b1[0] - t[0] * b1[2];
    b[5] = t[0] * b1[1] - t[1] * b1[0];
}
__device__ __forceinline__ void rodrigues_f(const float w[3], float R[3][3]) {
    const float th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    float a, b;
    if (th2 < 1e-2f) {  // |theta| < 0.1: Taylor to theta^6 (remainder < 3e-11)
        a = 1.f - th2 / 6.f * (1.f - th2 / 20.f * (1.f - th2 / 42.f));
        b = 0.5f * (1.f - th2 / 12.f * (1.f - th2 / 30.f * (1.f - th2 / 56.f)));
    } else {
        const float th = sqrtf(th2);
        a = sinf(th) / th;
        b = (1.f - cosf(th)) / th2;
    }
    const float K[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const float kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
            R[i][j] = (i == j ? 1.f : 0.f) + a * K[i][j] + b * kk;
        }
}

__device__ void rodrigues(const double w[3], double R[3][3]) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double a, b;
    if (th2 < 2.5e-3) {  // |theta| < 0.05: Taylor to theta^8 (remainder < 3e-21), no transcendentals
        a = 1.0 - th2 / 6.0 * (1.0 - th2 / 20.0 * (1.0 - th2 / 42.0 * (1.0 - th2 / 72.0)));
        b = 0.5 * (1.0 - th2 / 12.0 * (1.0 - th2 / 30.0 * (1.0 - th2 / 56.0 * (1.0 - th2 / 90.0))));
    } else {
        const double th = sqrt(th2);
        a = sin(th) / th;
        b = (1.0 - cos(th)) / th2;
    }
    const double K[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
            R[i][j] = (i == j ? 1.0 : 0.0) + a * K[i][j] + b * kk;
        }
}

__device__ __forceinline__ int block_sum_i(int v, int *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

struct PoseArgs {
    int cap;
    float fx, fy, cx, cy;
    int hypotheses;
    float thr2;  // (inlier_thresh / f)^2 in normalised units
    int refine_iters;
    unsigned long long seed;
};

__global__ __launch_bounds__(NT, PE_WAVES) void k_pose_ransac(PoseArgs a, const int *__restrict__ nv,
                                                    const float *__restrict__ pts0,
                                                    const float *__restrict__ pts1,
                                                    const int *__restrict__ match_idx,
                                                    const float *__restrict__ kp1, float *__restrict__ T,
                                                    int *__restrict__ num_matches, int *__restrict__ num_inliers,
                                                    int *__restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) float4 P[];  // [min(cap, MAXP)]
    __shared__ int wsum[4];
    __shared__ int s_best[2];
    __shared__ float s_E[9];
    __shared__ double s_pose[12];  // R (9) + t (3)
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int n_in = min(max(nv[b], 0), a.cap);
    const long long tk0 = PE_TRACE ? clock64() : 0;

    // ---- 1. compaction (query order) + normalisation ----
    const int per = (n_in + NT - 1) / NT;
    const int i0 = t * per, i1 = min(i0 + per, n_in);
    int cnt = 0;
    // a match index outside [0, cap) is "no match" (never dereferenced)
    for (int i = i0; i < i1; i++)
        cnt += (!match_idx || (unsigned)match_idx[(size_t)b * a.cap + i] < (unsigned)a.cap) ? 1 : 0;
    int x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int off = x - cnt;
    for (int k = 0; k < w; k++) off += wsum[k];
    const int n_all = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const int n = min(n_all, MAXP);
    for (int i = i0; i < i1; i++) {
        float x1 = pts0[((size_t)b * a.cap + i) * 2], y1 = pts0[((size_t)b * a.cap + i) * 2 + 1], x2, y2;
        if (match_idx) {
            const int j = match_idx[(size_t)b * a.cap + i];
            if ((unsigned)j >= (unsigned)a.cap) continue;
            x2 = kp1[((size_t)b * a.cap + j) * 2];
            y2 = kp1[((size_t)b * a.cap + j) * 2 + 1];
        } else {
            x2 = pts1[((size_t)b * a.cap + i) * 2];
            y2 = pts1[((size_t)b * a.cap + i) * 2 + 1];
        }
        if (off < MAXP)
            P[off] = make_float4((x1 - a.cx) / a.fx, (y1 - a.cy) / a.fy, (x2 - a.cx) / a.fx, (y2 - a.cy) / a.fy);
        off++;
    }
    __syncthreads();
    float *To = T + (size_t)b * 12;
    if (n < 8) {
        if (t < 12) To[t] = (t % 4 == t / 4) ? 1.f : 0.f;
        if (t == 0) {
            num_inliers[b] = 0;
            if (num_matches) num_matches[b] = n_all;
            status[b] = n_all == 0 ? MV_ERR_NO_POINTS : MV_ERR_DEGENERATE;
        }
        return;
    }

    const long long tk1 = PE_TRACE ? clock64() : 0;
    // ---- 2. hypotheses, preemptively MSAC-scored (sum of min(Sampson^2, thr^2); plain
    //         inlier counting cannot separate an outlier-contaminated 8-point solution that
    //         still explains every inlier within the band -- near-pure forward motion).
    //         Every hypothesis is scored on an evenly strided subset of PRE_M
    //         correspondences; the SURV best of each wave survive (preemptive RANSAC,
    //         Nister 2003) and are re-scored on all correspondences cooperatively. ----
    constexpr int PRE_M = 128, SURV = 2, NS = 4 * SURV;
    const int m = min(n, PRE_M);
    const unsigned step16 = ((unsigned)n << 16) / (unsigned)m;  // subset point k: (k * step16) >> 16 < n
    float best_cost = __builtin_inff();
    int best_h = 0x7fffffff;
    float best_e[9];
    for (int h = t; h < a.hypotheses; h += NT) {
        int idx[8];
        const unsigned long long base = a.seed ^ ((unsigned long long)b << 40) ^ ((unsigned long long)h << 8);
        int drawn = 0;
        for (int d = 0; d < 64 && drawn < 8; d++) {
            const unsigned long long r = splitmix64(base + d);
            const int c = (int)(((r >> 32) * (unsigned long long)n) >> 32);
            bool dup = false;
#pragma unroll
            for (int q = 0; q < 8; q++) dup |= (q < drawn) && idx[q] == c;
            if (!dup) {
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (q == drawn) idx[q] = c;
                drawn++;
            }
        }
        if (drawn < 8) continue;
        float e[9];
        if (PE_NOHYP) {
            for (int r = 0; r < 9; r++) e[r] = P[idx[r & 7]].x + r;
        } else if (!eight_point(P, idx, e)) {
            continue;
        }
        int c = 0;
        float cost = 0.f;
        int k = 0;
        for (; k + 4 <= (PE_NOSCORE ? 0 : m); k += 4) {  // 4 LDS broadcast reads in flight per step
            const float4 p0 = P[(k * step16) >> 16], p1 = P[((k + 1) * step16) >> 16];
            const float4 p2 = P[((k + 2) * step16) >> 16], p3 = P[((k + 3) * step16) >> 16];
            cost += msac_cost(e, p0, a.thr2, c);
            cost += msac_cost(e, p1, a.thr2, c);
            cost += msac_cost(e, p2, a.thr2, c);
            cost += msac_cost(e, p3, a.thr2, c);
        }
        for (; k < (PE_NOSCORE ? 0 : m); k++) cost += msac_cost(e, P[(k * step16) >> 16], a.thr2, c);
        if (cost < best_cost || (cost == best_cost && h < best_h)) {
            best_cost = cost;
            best_h = h;
#pragma unroll
            for (int r = 0; r < 9; r++) best_e[r] = e[r];
        }
    }
    const long long tk2 = PE_TRACE ? clock64() : 0;
    // ---- 3. survivors: the SURV lowest (partial cost, hypothesis id) keys of each wave (cost
    //         >= 0, so its bits order as uint), then full MSAC of the NS survivors ----
    __shared__ int s_sh[NS];
    __shared__ float s_sE[NS][9];
    {
        unsigned long long key = best_h == 0x7fffffff
                                     ? ~0ull
                                     : ((unsigned long long)__float_as_uint(best_cost) << 32) | (unsigned)best_h;
        for (int r = 0; r < SURV; r++) {
            unsigned long long k = key;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long k2 = __shfl_xor(k, o, 64);
                k = k2 < k ? k2 : k;
            }
            if (k == ~0ull) {
                if (lane == 0) s_sh[w * SURV + r] = -1;
            } else if (key == k) {  // the owner (keys are unique: hypothesis ids differ)
                s_sh[w * SURV + r] = best_h;
#pragma unroll
                for (int q = 0; q < 9; q++) s_sE[w * SURV + r][q] = best_e[q];
                key = ~0ull;
            }
        }
    }
    __syncthreads();
    float cs[NS];
    int cn[NS];
#pragma unroll
    for (int sv = 0; sv < NS; sv++) {
        cs[sv] = 0.f;
        cn[sv] = 0;
        if (s_sh[sv] < 0) continue;
        float e[9];
#pragma unroll
        for (int q = 0; q < 9; q++) e[q] = s_sE[sv][q];
        for (int i = t; i < n; i += NT) cs[sv] += msac_cost(e, P[i], a.thr2, cn[sv]);
    }
    __shared__ float s_red2[4][2 * NS];
    {
        float v[2 * NS];
#pragma unroll
        for (int sv = 0; sv < NS; sv++) {
            v[sv] = cs[sv];
            v[NS + sv] = (float)cn[sv];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int k = 0; k < 2 * NS; k++) v[k] += __shfl_xor(v[k], o, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 2 * NS; k++) s_red2[w][k] = v[k];
        }
    }
    __syncthreads();
    if (t == 0) {
        int bs = -1;
        float bc = 0.f;
        for (int sv = 0; sv < NS; sv++) {
            if (s_sh[sv] < 0) continue;
            const float c = s_red2[0][sv] + s_red2[1][sv] + s_red2[2][sv] + s_red2[3][sv];
            if (bs < 0 || c < bc || (c == bc && s_sh[sv] < s_sh[bs])) {
                bs = sv;
                bc = c;
            }
        }
        s_best[0] = bs < 0 ? -1
                           : (int)(s_red2[0][NS + bs] + s_red2[1][NS + bs] + s_red2[2][NS + bs] + s_red2[3][NS + bs]);
        if (bs >= 0)
            for (int r = 0; r < 9; r++) s_E[r] = s_sE[bs][r];
    }
    __syncthreads();
    if (s_best[0] < 0) {
        if (t < 12) To[t] = (t % 4 == t / 4) ? 1.f : 0.f;
        if (t == 0) {
            num_inliers[b] = 0;
            if (num_matches) num_matches[b] = n_all;
            status[b] = MV_ERR_DEGENERATE;
        }
        return;
    }
    float E[9];
    for (int r = 0; r < 9; r++) E[r] = s_E[r];
    const int ninl = s_best[0];

    const long long tk3 = PE_TRACE ? clock64() : 0;
    // ---- 4. decomposition + cheirality ----
    __shared__ double s_cand[4][12];
    if (t == 0) {
        double Ed[9], U[3][3], V[3][3];
        for (int r = 0; r < 9; r++) Ed[r] = E[r];
        if (PE_NODECOMP) {
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) U[i][j] = V[i][j] = i == j;
        } else {
            essential_uv(Ed, U, V);
        }
        const double W[3][3] = {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}};
        for (int c = 0; c < 4; c++) {
            double R[3][3];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    double s = 0;
                    for (int k = 0; k < 3; k++) {
                        double uw = 0;
                        for (int l = 0; l < 3; l++) uw += U[i][l] * (c < 2 ? W[l][k] : W[k][l]);
                        s += uw * V[j][k];
                    }
                    R[i][j] = s;
                }
            const double sg = (c & 1) ? -1.0 : 1.0;
            for (int i = 0; i < 9; i++) s_cand[c][i] = R[i / 3][i % 3];
            for (int i = 0; i < 3; i++) s_cand[c][9 + i] = sg * U[i][2];
        }
    }
    __syncthreads();
    int votes[4] = {0, 0, 0, 0};
    for (int i = t; i < n; i += NT) {
        const float4 p = P[i];
        if (!sampson_inlier(E, p, a.thr2)) continue;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const double *C = s_cand[c];
            D3 q = {{C[0] * p.x + C[1] * p.y + C[2], C[3] * p.x + C[4] * p.y + C[5], C[6] * p.x + C[7] * p.y + C[8]}};
            D3 m = {{-(double)p.z, -(double)p.w, -1.0}};
            D3 tt = {{C[9], C[10], C[11]}};
            const double aa = dot3(q, q), ab = dot3(q, m), bb = dot3(m, m);
            const double ra = -dot3(q, tt), rb = -dot3(m, tt);
            const double det = aa * bb - ab * ab;
            if (det <= 0) continue;
            const double z1 = (ra * bb - ab * rb) / det, z2 = (aa * rb - ab * ra) / det;
            votes[c] += (z1 > 0 && z2 > 0) ? 1 : 0;
        }
    }
    const long long tk4 = PE_TRACE ? clock64() : 0;
    __shared__ int s_votes[4];
    for (int c = 0; c < 4; c++) {
        int v = block_sum_i(votes[c], wsum);
        if (t == 0) s_votes[c] = v;
        __syncthreads();
    }
    if (t == 0) {
        int bc = 0;
        for (int c = 1; c < 4; c++)
            if (s_votes[c] > s_votes[bc]) bc = c;
        for (int i = 0; i < 12; i++) s_pose[i] = s_cand[bc][i];
    }
    __syncthreads();

    const long long tk5 = PE_TRACE ? clock64() : 0;
    // ---- 5. Gauss-Newton, inliers re-selected every iteration with the current
    //         model: |r_i| < th_k, th_0 = thr, th_{k+1} = min(thr, max(3 rms_k, 0.01 px))
    //         (removes outliers that fell inside the RANSAC band; noisy data keeps thr).
    //         Every thread holds the pose and solves the 5x5 normal equations itself from the
    //         22 block sums (identical float ops in every lane): one block barrier per
    //         iteration (the partial sums are double-buffered), no broadcast of the update. ----
    __shared__ float s_red[2][4][22];
    float R[9], tv[3], bs[6];  // the state: rotation, unit translation, tangent basis at t
#pragma unroll
    for (int i = 0; i < 9; i++) R[i] = (float)s_pose[i];
#pragma unroll
    for (int i = 0; i < 3; i++) tv[i] = (float)s_pose[9 + i];
    tangent_basis_f(tv, bs);
    const float th_max = sqrtf(a.thr2), th_min = 0.01f * th_max;
    float th = th_max;
    for (int it = 0; it < a.refine_iters; it++) {
        // the per-correspondence Jacobian and the 22 sums are float (the fixed point is set
        // by the float residual, ~1e-7 of a unit vector)
        float acc[22];  // J^T J (15, upper), J^T r (5), sum r^2, count
#pragma unroll
        for (int k = 0; k < 22; k++) acc[k] = 0.f;
        for (int i = t; i < (PE_NOPOINTS ? 0 : n); i += NT) {
            const float4 p = P[i];
            const float x1[3] = {p.x, p.y, 1.f}, x2[3] = {p.z, p.w, 1.f};
            const float q[3] = {R[0] * x1[0] + R[1] * x1[1] + R[2], R[3] * x1[0] + R[4] * x1[1] + R[5],
                                R[6] * x1[0] + R[7] * x1[1] + R[8]};
            // e = x2^T [t]x R x1 = (x2 x t) . (R x1)
            const float x2t[3] = {x2[1] * tv[2] - x2[2] * tv[1], x2[2] * tv[0] - x2[0] * tv[2],
                                  x2[0] * tv[1] - x2[1] * tv[0]};
            const float e = x2t[0] * q[0] + x2t[1] * q[1] + x2t[2] * q[2];
            const float Ex1[2] = {tv[1] * q[2] - tv[2] * q[1], tv[2] * q[0] - tv[0] * q[2]};  // (E x1)_{0,1}
            float Etx2[2];  // (E^T x2)_{0,1} = (R^T (x2 x t))_{0,1}
#pragma unroll
            for (int c = 0; c < 2; c++) Etx2[c] = R[c] * x2t[0] + R[3 + c] * x2t[1] + R[6 + c] * x2t[2];
            const float s2 = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Etx2[0] * Etx2[0] + Etx2[1] * Etx2[1];
            if (!(s2 > 0.f)) continue;
            const float inv = __builtin_amdgcn_rsqf(s2);  // native: a GN weight, not an output
            const float r = e * inv;  // Sampson distance (weight frozen at the current model)
            if (!(fabsf(r) < th)) continue;
            // d e / d omega = q x (x2 x t)  (R <- exp(omega) R);  d e / d t = q x x2
            const float dw[3] = {q[1] * x2t[2] - q[2] * x2t[1], q[2] * x2t[0] - q[0] * x2t[2],
                                 q[0] * x2t[1] - q[1] * x2t[0]};
            const float dt[3] = {q[1] * x2[2] - q[2] * x2[1], q[2] * x2[0] - q[0] * x2[2],
                                 q[0] * x2[1] - q[1] * x2[0]};
            const float J[5] = {dw[0] * inv, dw[1] * inv, dw[2] * inv,
                                (dt[0] * bs[0] + dt[1] * bs[1] + dt[2] * bs[2]) * inv,
                                (dt[0] * bs[3] + dt[1] * bs[4] + dt[2] * bs[5]) * inv};
            int k = 0;
#pragma unroll
            for (int u = 0; u < 5; u++) {
#pragma unroll
                for (int v = u; v < 5; v++) acc[k++] += J[u] * J[v];
            }
#pragma unroll
            for (int u = 0; u < 5; u++) acc[15 + u] += J[u] * r;
            acc[20] += r * r;
            acc[21] += 1.f;
        }
        // one block reduction of all 22 sums: wave shuffles, then 4 partials in LDS
        // (levels outer, sums inner: 22 independent shuffles in flight per level)
        if (!PE_NORED) {
#pragma unroll
            for (int k = 0; k < 22; k++) acc[k] += __shfl_xor(acc[k], 32, 64);
#define PE_SWZ(O)                                                                            \
    _Pragma("unroll") for (int k = 0; k < 22; k++) acc[k] += __int_as_float(                 \
        __builtin_amdgcn_ds_swizzle(__float_as_int(acc[k]), ((O) << 10) | 0x1F))
            PE_SWZ(16);
            PE_SWZ(8);
            PE_SWZ(4);
            PE_SWZ(2);
            PE_SWZ(1);
#undef PE_SWZ
        }
        float(*red)[22] = s_red[it & 1];
        if (lane < 22) {
            float v = acc[0];
#pragma unroll
            for (int k = 1; k < 22; k++) v = lane == k ? acc[k] : v;
            red[w][lane] = v;
        }
        __syncthreads();
        if (PE_NOSOLVE) continue;
        float H[15], g[5];
#pragma unroll
        for (int k = 0; k < 15; k++) H[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
#pragma unroll
        for (int k = 0; k < 5; k++) g[k] = red[0][15 + k] + red[1][15 + k] + red[2][15 + k] + red[3][15 + k];
        const float r2 = red[0][20] + red[1][20] + red[2][20] + red[3][20];
        const float cnt = red[0][21] + red[1][21] + red[2][21] + red[3][21];
        // (H + lambda diag H) d = -g: float Cholesky on the native reciprocal square root (the
        // step only has to be a descent direction); every loop fully unrolled: static register
        // indexing, no private (scratch) arrays
        float A[5][5];
#pragma unroll
        for (int u = 0, k = 0; u < 5; u++)
#pragma unroll
            for (int v = u; v < 5; v++, k++) {
                A[u][v] = H[k];
                A[v][u] = H[k];
            }
#pragma unroll
        for (int u = 0; u < 5; u++) A[u][u] = A[u][u] * (1.0f + 1e-6f) + 1e-30f;
        float L[5][5] = {}, rl[5] = {};
        bool ok = cnt >= 5.f;
#pragma unroll
        for (int i = 0; i < 5; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) {
                float sum = A[i][j];
#pragma unroll
                for (int m = 0; m < j; m++) sum -= L[i][m] * L[j][m];
                if (i == j) {
                    ok = ok && sum > 0.f;
                    rl[i] = __builtin_amdgcn_rsqf(fmaxf(sum, 1e-30f));  // 1 / L[i][i]
                    L[i][i] = fmaxf(sum, 1e-30f) * rl[i];
                } else {
                    L[i][j] = sum * rl[j];
                }
            }
        if (!ok) break;  // the same decision in every thread
        float y[5], d[5];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            float sum = -g[i];
#pragma unroll
            for (int m = 0; m < i; m++) sum -= L[i][m] * y[m];
            y[i] = sum * rl[i];
        }
#pragma unroll
        for (int i = 4; i >= 0; i--) {
            float sum = y[i];
#pragma unroll
            for (int m = i + 1; m < 5; m++) sum -= L[m][i] * d[m];
            d[i] = sum * rl[i];
        }
        float dR[3][3];
        rodrigues_f(d, dR);
        float Rn[9], tn[3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                Rn[i * 3 + j] = dR[i][0] * R[0 * 3 + j] + dR[i][1] * R[1 * 3 + j] + dR[i][2] * R[2 * 3 + j];
#pragma unroll
        for (int i = 0; i < 3; i++) tn[i] = tv[i] + d[3] * bs[i] + d[4] * bs[3 + i];
        const float rn = __builtin_amdgcn_rsqf(tn[0] * tn[0] + tn[1] * tn[1] + tn[2] * tn[2]);
#pragma unroll
        for (int i = 0; i < 9; i++) R[i] = Rn[i];
#pragma unroll
        for (int i = 0; i < 3; i++) tv[i] = tn[i] * rn;
        tangent_basis_f(tv, bs);
        const float th_new = fminf(th_max, fmaxf(3.f * sqrtf(r2 / cnt), th_min));
        float dmax = 0.f;
#pragma unroll
        for (int i = 0; i < 5; i++) dmax = fmaxf(dmax, fabsf(d[i]));
        // converged: a step below the float residual's resolution (1e-6 rad / unit-t, 100x
        // under the 1e-4 tolerance) and an inlier band that moved < 0.1 %
        const bool done = dmax < 1e-6f && fabsf(th_new - th) <= 1e-3f * th;
        th = th_new;
        if (done) break;
    }
    {  // [R | t] row-major, thread t < 12 writes entry t (static register indexing)
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 12; k++) v = t == k ? (k % 4 < 3 ? R[(k / 4) * 3 + k % 4] : tv[k / 4]) : v;
        if (t < 12) To[t] = v;
    }
    if (PE_TRACE && b == 0 && t == 0) {
        const long long tk6 = clock64();
        printf("pose phases (clk): compact %lld hyp+score %lld argmin %lld decomp %lld cheir %lld gn %lld\n",
               tk1 - tk0, tk2 - tk1, tk3 - tk2, tk4 - tk3, tk5 - tk4, tk6 - tk5);
    }
    if (t == 0) {
        num_inliers[b] = ninl;
        if (num_matches) num_matches[b] = n_all;
        status[b] = MV_OK;
    }
}

}  // namespace

namespace mv {

size_t intended_pose_scratch_bytes(int batch, int cap) {
    (void)batch;
    (void)cap;
    return 256;
}

int launch_intended_pose(hipStream_t s, void *scratch, const mv_pose_params *p, int batch, int cap, const int *n,
                         const float *pts0, const float *pts1, const int *match_idx, const float *kp1, float *T,
                         int *num_matches, int *num_inliers, int *status) {
    (void)scratch;
    MV_REQUIRE(p->hypotheses > 0 && p->fx > 0 && p->fy > 0 && p->refine_iters >= 0);
    PoseArgs a;
    a.cap = cap;
    a.fx = p->fx;
    a.fy = p->fy;
    a.cx = p->cx;
    a.cy = p->cy;
    a.hypotheses = p->hypotheses;
    const float f = 0.5f * (p->fx + p->fy);
    a.thr2 = (p->inlier_thresh / f) * (p->inlier_thresh / f);
    a.refine_iters = p->refine_iters;
    a.seed = p->seed;
    const size_t lds = sizeof(float4) * (size_t)(cap < MAXP ? cap : MAXP);
    MV_PROF_BEGIN(s, "k_pose_ransac");
    hipLaunchKernelGGL(k_pose_ransac, dim3(batch), dim3(NT), lds, s, a, n, pts0, pts1, match_idx, kp1, T,
                       num_matches, num_inliers, status);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv
