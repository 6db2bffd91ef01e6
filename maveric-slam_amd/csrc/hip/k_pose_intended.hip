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
//      hypotheses are MSAC-scored: sum of min(Sampson^2, (thr_px / f)^2) over all
//      correspondences (LDS broadcast reads);
//   3. block argmin (lowest cost, lowest hypothesis id) -> E;
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
//      t <- normalise(t + B d).
// Output T = [R | t] with x1 ~ R x0 + t, |t| = 1 (the OpenCV recoverPose convention).
#include <math.h>

#include "mv_internal.hpp"

namespace {

constexpr int NT = 256;
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

__device__ void rodrigues(const double w[3], double R[3][3]) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double th = sqrt(th2);
    double a, b;
    if (th < 1e-8) {
        a = 1.0 - th2 / 6.0;
        b = 0.5 - th2 / 24.0;
    } else {
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

__global__ __launch_bounds__(NT) void k_pose_ransac(PoseArgs a, const int *__restrict__ nv,
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
    const int n_in = min(nv[b], a.cap);

    // ---- 1. compaction (query order) + normalisation ----
    const int per = (n_in + NT - 1) / NT;
    const int i0 = t * per, i1 = min(i0 + per, n_in);
    int cnt = 0;
    for (int i = i0; i < i1; i++) cnt += (!match_idx || match_idx[(size_t)b * a.cap + i] >= 0) ? 1 : 0;
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
            if (j < 0) continue;
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

    // ---- 2. hypotheses, MSAC-scored (sum of min(Sampson^2, thr^2); plain inlier
    //         counting cannot separate an outlier-contaminated 8-point solution that
    //         still explains every inlier within the band -- near-pure forward motion) ----
    float best_cost = __builtin_inff();
    int best_cnt = -1, best_h = 0x7fffffff;
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
        if (!eight_point(P, idx, e)) continue;
        int c = 0;
        float cost = 0.f;
        for (int i = 0; i < n; i++) cost += msac_cost(e, P[i], a.thr2, c);
        if (cost < best_cost || (cost == best_cost && h < best_h)) {
            best_cost = cost;
            best_cnt = c;
            best_h = h;
#pragma unroll
            for (int r = 0; r < 9; r++) best_e[r] = e[r];
        }
    }
    // ---- 3. block argmin (cost asc, hypothesis id asc); cost >= 0 so its bits order as uint ----
    unsigned long long key = best_cnt < 0 ? ~0ull
                                          : ((unsigned long long)__float_as_uint(best_cost) << 32) | (unsigned)best_h;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long k2 = __shfl_xor(key, o, 64);
        key = k2 < key ? k2 : key;
    }
    __shared__ unsigned long long s_key[4];
    if (lane == 0) s_key[w] = key;
    __syncthreads();
    unsigned long long bk = s_key[0];
    for (int k = 1; k < 4; k++) bk = s_key[k] < bk ? s_key[k] : bk;
    if (bk == ~0ull) {
        if (t < 12) To[t] = (t % 4 == t / 4) ? 1.f : 0.f;
        if (t == 0) {
            num_inliers[b] = 0;
            if (num_matches) num_matches[b] = n_all;
            status[b] = MV_ERR_DEGENERATE;
        }
        return;
    }
    const int win_h = (int)(bk & 0xffffffff);
    if (best_cnt >= 0 && best_h == win_h) {
        for (int r = 0; r < 9; r++) s_E[r] = best_e[r];
        s_best[0] = best_cnt;
    }
    __syncthreads();
    float E[9];
    for (int r = 0; r < 9; r++) E[r] = s_E[r];
    const int ninl = s_best[0];

    // ---- 4. decomposition + cheirality ----
    __shared__ double s_cand[4][12];
    if (t == 0) {
        double Ed[9], U[3][3], V[3][3];
        for (int r = 0; r < 9; r++) Ed[r] = E[r];
        essential_uv(Ed, U, V);
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

    // ---- 5. Gauss-Newton, inliers re-selected every iteration with the current
    //         model: |r_i| < th_k, th_0 = thr, th_{k+1} = min(thr, max(3 rms_k, 0.01 px))
    //         (removes outliers that fell inside the RANSAC band; noisy data keeps thr) ----
    __shared__ double s_red[4][22];
    __shared__ double s_th;
    if (t == 0) s_th = sqrt((double)a.thr2);
    __syncthreads();
    const double th_max = sqrt((double)a.thr2);
    const double th_min = 0.01 * th_max;
    for (int it = 0; it < a.refine_iters; it++) {
        double R[9], tv[3];
        for (int i = 0; i < 9; i++) R[i] = s_pose[i];
        for (int i = 0; i < 3; i++) tv[i] = s_pose[9 + i];
        const double th = s_th;
        // tangent basis of the unit sphere at t
        D3 tt = {{tv[0], tv[1], tv[2]}};
        D3 ax = fabs(tv[0]) < 0.57 ? D3{{1, 0, 0}} : (fabs(tv[1]) < 0.57 ? D3{{0, 1, 0}} : D3{{0, 0, 1}});
        D3 b1 = cross(tt, ax);
        const double nb1 = sqrt(dot3(b1, b1));
        for (int i = 0; i < 3; i++) b1.v[i] /= nb1;
        D3 b2 = cross(tt, b1);
        double acc[22];  // J^T J (15, upper), J^T r (5), sum r^2, count
#pragma unroll
        for (int k = 0; k < 22; k++) acc[k] = 0;
        for (int i = t; i < n; i += NT) {
            const float4 p = P[i];
            D3 x1 = {{p.x, p.y, 1.0}}, x2 = {{p.z, p.w, 1.0}};
            D3 q = {{R[0] * x1.v[0] + R[1] * x1.v[1] + R[2], R[3] * x1.v[0] + R[4] * x1.v[1] + R[5],
                     R[6] * x1.v[0] + R[7] * x1.v[1] + R[8]}};
            D3 x2t = cross(x2, tt);  // e = x2^T [t]x R x1 = (x2 x t) . (R x1)
            const double e = dot3(x2t, q);
            D3 Ex1 = cross(tt, q);   // E x1
            double Etx2[3];          // E^T x2 = R^T (x2 x t)
            for (int c = 0; c < 3; c++)
                Etx2[c] = R[0 * 3 + c] * x2t.v[0] + R[1 * 3 + c] * x2t.v[1] + R[2 * 3 + c] * x2t.v[2];
            const double s2 = Ex1.v[0] * Ex1.v[0] + Ex1.v[1] * Ex1.v[1] + Etx2[0] * Etx2[0] + Etx2[1] * Etx2[1];
            if (!(s2 > 0)) continue;
            const double inv = 1.0 / sqrt(s2);
            const double r = e * inv;  // Sampson distance (weight frozen at the current model)
            if (!(fabs(r) < th)) continue;
            D3 dw = cross(q, x2t);   // d e / d omega   (R <- exp(omega) R)
            D3 dt = cross(q, x2);    // d e / d t
            const double J[5] = {dw.v[0] * inv, dw.v[1] * inv, dw.v[2] * inv, dot3(dt, b1) * inv,
                                 dot3(dt, b2) * inv};
            int k = 0;
#pragma unroll
            for (int u = 0; u < 5; u++) {
#pragma unroll
                for (int v = u; v < 5; v++) acc[k++] += J[u] * J[v];
            }
#pragma unroll
            for (int u = 0; u < 5; u++) acc[15 + u] += J[u] * r;
            acc[20] += r * r;
            acc[21] += 1.0;
        }
        // one block reduction of all 22 sums: wave shuffles, then 4 partials in LDS
#pragma unroll
        for (int k = 0; k < 22; k++) {
            double v = acc[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) s_red[w][k] = v;
        }
        __syncthreads();
        if (t == 0) {
            double H[15], g[5];
            for (int k = 0; k < 15; k++) H[k] = s_red[0][k] + s_red[1][k] + s_red[2][k] + s_red[3][k];
            for (int k = 0; k < 5; k++) g[k] = s_red[0][15 + k] + s_red[1][15 + k] + s_red[2][15 + k] + s_red[3][15 + k];
            const double r2 = s_red[0][20] + s_red[1][20] + s_red[2][20] + s_red[3][20];
            const double cnt = s_red[0][21] + s_red[1][21] + s_red[2][21] + s_red[3][21];
            // (H + lambda diag H) d = -g, Cholesky
            double A[5][5];
            int k = 0;
            for (int u = 0; u < 5; u++)
                for (int v = u; v < 5; v++) {
                    A[u][v] = H[k];
                    A[v][u] = H[k];
                    k++;
                }
            for (int u = 0; u < 5; u++) A[u][u] = A[u][u] * (1.0 + 1e-9) + 1e-300;
            double L[5][5] = {};
            bool ok = cnt >= 5;
            for (int i = 0; i < 5 && ok; i++)
                for (int j = 0; j <= i; j++) {
                    double sum = A[i][j];
                    for (int m = 0; m < j; m++) sum -= L[i][m] * L[j][m];
                    if (i == j) {
                        if (!(sum > 0)) {
                            ok = false;
                            break;
                        }
                        L[i][i] = sqrt(sum);
                    } else {
                        L[i][j] = sum / L[j][j];
                    }
                }
            if (ok) {
                double y[5], d[5];
                for (int i = 0; i < 5; i++) {
                    double sum = -g[i];
                    for (int m = 0; m < i; m++) sum -= L[i][m] * y[m];
                    y[i] = sum / L[i][i];
                }
                for (int i = 4; i >= 0; i--) {
                    double sum = y[i];
                    for (int m = i + 1; m < 5; m++) sum -= L[m][i] * d[m];
                    d[i] = sum / L[i][i];
                }
                double dR[3][3], Rn[3][3];
                rodrigues(d, dR);
                for (int i = 0; i < 3; i++)
                    for (int j = 0; j < 3; j++)
                        Rn[i][j] = dR[i][0] * R[0 * 3 + j] + dR[i][1] * R[1 * 3 + j] + dR[i][2] * R[2 * 3 + j];
                double tn[3];
                for (int i = 0; i < 3; i++) tn[i] = tv[i] + d[3] * b1.v[i] + d[4] * b2.v[i];
                const double nt = sqrt(tn[0] * tn[0] + tn[1] * tn[1] + tn[2] * tn[2]);
                for (int i = 0; i < 9; i++) s_pose[i] = Rn[i / 3][i % 3];
                for (int i = 0; i < 3; i++) s_pose[9 + i] = tn[i] / nt;
                s_th = fmin(th_max, fmax(3.0 * sqrt(r2 / cnt), th_min));
            }
        }
        __syncthreads();
    }
    if (t < 12) {
        const int r = t / 4, c = t % 4;
        To[t] = (float)(c < 3 ? s_pose[r * 3 + c] : s_pose[9 + r]);
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
