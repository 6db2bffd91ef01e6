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
//      correspondences by the whole block; the two lowest (cost, hypothesis id) are the
//      starts of the refinement;
//   4. per start: E = U diag(s1,s2,s3) V^T (closed-form eigenvectors of E^T E), the four
//      (R, t) candidates R = U W V^T / U W^T V^T, t = +-u3, cheirality vote by triangulated
//      depth over the inliers (block reduction);
//   5. per start: robust Gauss-Newton (IRLS) on the Sampson residuals r_i =
//      (x2^T [t]x R x1) / s_i with Cauchy weights whose scale shrinks from thr towards
//      2 rms (exact data converges to machine precision, noisy data keeps ~2 sigma),
//      per-correspondence Jacobian d r / d(omega, tangent(t)) (5 dof), J^T W J and
//      J^T W r assembled with wave64 reductions + LDS (the [J|r]^T[J|r] pattern of
//      src/local_bundle_adjustment.c:161-176), 5x5 Cholesky solve, R <- exp(omega) R,
//      t <- normalise(t + B d); float throughout (the output is float); stops once the
//      step is below 1e-6 and the scale settles (refine_iters is the maximum);
//   6. the refined pose with the lower robust cost (Cauchy at thr, capped at 3 thr) wins;
//      the second start is refined only when the first did not reach an exact fit.
// Output T = [R | t] with x1 ~ R x0 + t, |t| = 1 (the OpenCV recoverPose convention).
#include <math.h>

#include <type_traits>

#include "mv_internal.hpp"

// This kernel is the as-INTENDED pose, checked against ground truth within a tolerance,
// not bit-exact against the oracle: let every a * b + c contract to one FMA here (the
// library's -ffp-contract=off exists for the bit-exact as-built paths).  Sampson scoring
// drops from ~41 to ~26 VALU ops per (hypothesis, correspondence).
#pragma clang fp contract(fast)

namespace {

constexpr int NT = 256;
// correspondences in the preemptive scoring subset of the 256 hypotheses (the 8 survivors are then
// scored on all).  Same-box A/B (profiles/r05u_pose_prem_ab.log): 128 / 64 / 32 points -- exact
// data 0.498 / 0.442 / 0.415 ms, 0.5 px + 20 % outliers 0.996 / 0.939 / 0.905 ms per 8192 pairs,
// pose errors unchanged (realistic line p99: rotation 0.085 / 0.086 / 0.086 deg, translation
// direction 2.51 / 2.54 / 2.56 deg), every pose test green; 64 kept (the subset still ranks
// hypotheses under heavier contamination than the bench's)
constexpr int PE_PREM = 64;
// waves per SIMD, a lower bound.  Built without SLP packing (Makefile, profiles/r05al_pose_noslp_ab.log)
// the kernel takes 119 VGPRs and no scratch, i.e. 4 waves per SIMD either way; the history below is
// that of the SLP-packed build, whose cross-stream nondeterminism went with the packing.
// SLP-packed: 3: 155 VGPRs, no scratch.  4 (128 VGPRs, 38 VGPRs + 22 SGPRs spilled, 96 B of
// scratch per lane) was faster (0.523 vs 0.564 ms exact, 1.07 vs 1.17 ms noisy,
// profiles/r04y_pose_waves_ab.log) but NOT deterministic: with the image -> pose chain running on
// three streams at once, some poses of a 256-pair track came out different from the same track
// run alone (matches identical; tools/dbg_pipelines.py, profiles/r05m_pose_determinism.log), the
// spill-free build bit-identical in every round -- so no scratch in this kernel.  (Measured and
// not kept: every wave solving its group's normal equations itself, one barrier per Gauss-Newton
// iteration instead of two: 1.105 vs 1.097-1.113 ms noisy, profiles/r05p_pose_rsolve_ab.log; each
// start refined by ONE wave with wave reductions and no block barrier at all: 1.046-1.050 vs
// 0.995-0.996 ms noisy, 0.516-0.517 vs 0.494 exact -- the per-point passes, not the barriers, set
// the pace -- profiles/r05r_pose_wavegn_ab.log.)
constexpr int PE_WAVES = 3;
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

// msac_cost of two correspondences at once on packed FP32 (v_pk_fma_f32 with the
// hypothesis' coefficients splat): A = {x1 x1' y1 y1'}, B = {x2 x2' y2 y2'}, the
// scoring subset's point-pair layout, so the operands need no register shuffling
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v msac_cost2(const float e[9], float4 A, float4 B, float thr2) {
    const f2v x1 = {A.x, A.y}, y1 = {A.z, A.w}, x2 = {B.x, B.y}, y2 = {B.z, B.w};
    const f2v ex0 = e[0] * x1 + (e[1] * y1 + e[2]);
    const f2v ex1 = e[3] * x1 + (e[4] * y1 + e[5]);
    const f2v ex2 = e[6] * x1 + (e[7] * y1 + e[8]);
    const f2v etx0 = e[0] * x2 + (e[3] * y2 + e[6]);
    const f2v etx1 = e[1] * x2 + (e[4] * y2 + e[7]);
    const f2v num = x2 * ex0 + (y2 * ex1 + ex2);
    const f2v den = ex0 * ex0 + ex1 * ex1 + etx0 * etx0 + etx1 * etx1;
    const f2v nn = num * num, td = thr2 * den;
    f2v r;
    r.x = nn.x < td.x ? nn.x * __builtin_amdgcn_rcpf(den.x) : thr2;
    r.y = nn.y < td.y ? nn.y * __builtin_amdgcn_rcpf(den.y) : thr2;
    return r;
}

// msac_cost of one correspondence under two hypotheses at once (packed FP32, the point's
// coordinates splat): the survivors' full re-score
__device__ __forceinline__ f2v msac_cost2h(const f2v E[9], float4 p, float thr2, int &na, int &nb) {
    const float x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
    const f2v ex0 = E[0] * x1 + (E[1] * y1 + E[2]);
    const f2v ex1 = E[3] * x1 + (E[4] * y1 + E[5]);
    const f2v ex2 = E[6] * x1 + (E[7] * y1 + E[8]);
    const f2v etx0 = E[0] * x2 + (E[3] * y2 + E[6]);
    const f2v etx1 = E[1] * x2 + (E[4] * y2 + E[7]);
    const f2v num = x2 * ex0 + (y2 * ex1 + ex2);
    const f2v den = ex0 * ex0 + ex1 * ex1 + etx0 * etx0 + etx1 * etx1;
    const f2v nn = num * num, td = thr2 * den;
    const bool ia = nn.x < td.x, ib = nn.y < td.y;
    na += ia ? 1 : 0;
    nb += ib ? 1 : 0;
    f2v r;
    r.x = ia ? nn.x * __builtin_amdgcn_rcpf(den.x) : thr2;
    r.y = ib ? nn.y * __builtin_amdgcn_rcpf(den.y) : thr2;
    return r;
}

// ---- small 3-vector algebra ----
template <typename T>
struct V3 {
    T v[3];
};
using F3 = V3<float>;
template <typename T>
__device__ __forceinline__ V3<T> cross(const V3<T> &a, const V3<T> &b) {
    return {{a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2], a.v[0] * b.v[1] - a.v[1] * b.v[0]}};
}
template <typename T>
__device__ __forceinline__ T dot3(const V3<T> &a, const V3<T> &b) {
    return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2];
}
__device__ __forceinline__ F3 scale3(const F3 &a, float s) { return {{a.v[0] * s, a.v[1] * s, a.v[2] * s}}; }
__device__ __forceinline__ F3 mul_sym(const float A[3][3], const F3 &x) {
    return {{A[0][0] * x.v[0] + A[0][1] * x.v[1] + A[0][2] * x.v[2],
             A[1][0] * x.v[0] + A[1][1] * x.v[1] + A[1][2] * x.v[2],
             A[2][0] * x.v[0] + A[2][1] * x.v[1] + A[2][2] * x.v[2]}};
}

// The two leading eigenvectors (v1: largest eigenvalue) of the symmetric PSD 3x3 A, in
// closed form and float (E is a float estimate; the Gauss-Newton stage refines the pose
// in float from here).  Replaces a cyclic Jacobi in double, whose serial sweeps on one
// lane cost ~17k of the block's ~133k cycles (this: ~3k; per-phase clock64() stamps, round 3):
//   - the smallest eigenvalue from the trigonometric solution of the characteristic
//     cubic: for an essential matrix (l1 = l2, r = -1) l3 = q + 2p cos(pi - d) is flat
//     in d, so the angle's rounding enters squared;
//   - its eigenvector as the longest cross product of two rows of A - l3 I (rank 2: the
//     gap to l2 is the leading singular value squared);
//   - one exact Jacobi rotation of A restricted to the orthogonal complement.
// When l1 ~ l2 the split of the complement is arbitrary, in any method, and the
// candidate set {U W V^T, U W^T V^T} x {+-u3} does not depend on it (checked against
// numpy.linalg.eigh on essential, noisy and degenerate E).
__device__ void top2_eig3(const float A[3][3], F3 &v1, F3 &v2) {
    const float p1 = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    const float q = (A[0][0] + A[1][1] + A[2][2]) * (1.f / 3.f);
    const float d0 = A[0][0] - q, d1 = A[1][1] - q, d2 = A[2][2] - q;
    const float p2 = (d0 * d0 + d1 * d1 + d2 * d2 + 2.f * p1) * (1.f / 6.f);
    F3 v3 = {{0.f, 0.f, 1.f}};
    if (p2 > 1e-30f) {
        const float ip = __builtin_amdgcn_rsqf(p2), p = p2 * ip;
        const float b00 = d0 * ip, b11 = d1 * ip, b22 = d2 * ip;
        const float b01 = A[0][1] * ip, b02 = A[0][2] * ip, b12 = A[1][2] * ip;
        float r = 0.5f * (b00 * (b11 * b22 - b12 * b12) - b01 * (b01 * b22 - b12 * b02) + b02 * (b01 * b12 - b11 * b02));
        r = fminf(1.f, fmaxf(-1.f, r));
        const float l3 = q + 2.f * p * cosf(acosf(r) * (1.f / 3.f) + 2.09439510f);
        const F3 r0 = {{A[0][0] - l3, A[0][1], A[0][2]}};
        const F3 r1 = {{A[1][0], A[1][1] - l3, A[1][2]}};
        const F3 r2 = {{A[2][0], A[2][1], A[2][2] - l3}};
        const F3 c0 = cross(r0, r1), c1 = cross(r0, r2), c2 = cross(r1, r2);
        const float n0 = dot3(c0, c0), n1 = dot3(c1, c1), n2 = dot3(c2, c2);
        const F3 c = (n0 >= n1 && n0 >= n2) ? c0 : (n1 >= n2 ? c1 : c2);
        const float nc = fmaxf(fmaxf(n0, n1), n2);
        if (nc > 1e-37f) v3 = scale3(c, __builtin_amdgcn_rsqf(nc));
    }
    // orthonormal basis (a, b) of the complement of v3
    const float f0 = fabsf(v3.v[0]), f1 = fabsf(v3.v[1]), f2 = fabsf(v3.v[2]);
    const int ax = (f0 <= f1 && f0 <= f2) ? 0 : (f1 <= f2 ? 1 : 2);
    const F3 e = {{ax == 0 ? 1.f : 0.f, ax == 1 ? 1.f : 0.f, ax == 2 ? 1.f : 0.f}};
    F3 a = cross(v3, e);
    a = scale3(a, __builtin_amdgcn_rsqf(dot3(a, a)));
    const F3 b = cross(v3, a);
    const F3 Aa = mul_sym(A, a), Ab = mul_sym(A, b);
    const float m00 = dot3(a, Aa), m11 = dot3(b, Ab), m01 = dot3(a, Ab);
    float c = 1.f, s = 0.f;
    if (fabsf(m01) > 1e-30f * fmaxf(fabsf(m00), fabsf(m11))) {
        const float th = (m11 - m00) * __builtin_amdgcn_rcpf(2.f * m01);
        const float t = copysignf(1.f, th) * __builtin_amdgcn_rcpf(fabsf(th) + sqrtf(th * th + 1.f));
        c = __builtin_amdgcn_rsqf(t * t + 1.f);
        s = t * c;
    }
    const F3 x = {{c * a.v[0] - s * b.v[0], c * a.v[1] - s * b.v[1], c * a.v[2] - s * b.v[2]}};
    const F3 y = {{s * a.v[0] + c * b.v[0], s * a.v[1] + c * b.v[1], s * a.v[2] + c * b.v[2]}};
    const bool sw = dot3(y, mul_sym(A, y)) > dot3(x, mul_sym(A, x));
    v1 = sw ? y : x;
    v2 = sw ? x : y;
}

// E (row-major) -> U, V with E ~ U diag(1,1,0) V^T, det U = det V = +1
__device__ void essential_uv(const float E[9], float U[3][3], float V[3][3]) {
    float EtE[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            EtE[i][j] = E[0 * 3 + i] * E[0 * 3 + j] + E[1 * 3 + i] * E[1 * 3 + j] + E[2 * 3 + i] * E[2 * 3 + j];
    F3 v1, v2;
    top2_eig3(EtE, v1, v2);
    const F3 v3 = cross(v1, v2);  // right-handed V
    F3 u1, u2;
    for (int i = 0; i < 3; i++) {
        u1.v[i] = E[i * 3 + 0] * v1.v[0] + E[i * 3 + 1] * v1.v[1] + E[i * 3 + 2] * v1.v[2];
        u2.v[i] = E[i * 3 + 0] * v2.v[0] + E[i * 3 + 1] * v2.v[1] + E[i * 3 + 2] * v2.v[2];
    }
    u1 = scale3(u1, __builtin_amdgcn_rsqf(dot3(u1, u1)));
    const float d12 = dot3(u1, u2);  // re-orthogonalise
    for (int i = 0; i < 3; i++) u2.v[i] -= d12 * u1.v[i];
    u2 = scale3(u2, __builtin_amdgcn_rsqf(dot3(u2, u2)));
    const F3 u3 = cross(u1, u2);
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

// The 22 per-lane sums of one Gauss-Newton pass reduced over the wave by recursive
// halving: at each xor level the lane keeps half of its (padded) values, the upper half
// if its level bit is set, and adds its partner's partials of them.  Levels 32, 16, 8, 4,
// 2 take 22 -> 11 -> 6 (of 12) -> 3 -> 2 (of 4) -> 1 values, level 1 finishes the pair.
// Returns the full wave sum of value vi (vi = -1 for lanes left holding padding).
template <int NV, int NK, int LVL>
__device__ __forceinline__ void gn_halve(const float (&in)[NV], float (&out)[NK], bool hi) {
#pragma unroll
    for (int j = 0; j < NK; j++) {
        const float lo_v = j < NV ? in[j] : 0.f, hi_v = NK + j < NV ? in[NK + j] : 0.f;
        const float send = hi ? lo_v : hi_v, keep = hi ? hi_v : lo_v;
        float recv;
        if (LVL == 32)
            recv = __shfl_xor(send, 32, 64);
        else
            recv = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), (LVL << 10) | 0x1F));
        out[j] = keep + recv;
    }
}
__device__ __forceinline__ float gn_reduce_scatter22(const float (&acc)[22], int lane, int &vi) {
    float b11[11], c6[6], d3[3], e2[2], f1[1];
    const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8, h2 = lane & 4, h1 = lane & 2;
    gn_halve<22, 11, 32>(acc, b11, h5);
    gn_halve<11, 6, 16>(b11, c6, h4);
    gn_halve<6, 3, 8>(c6, d3, h3);
    gn_halve<3, 2, 4>(d3, e2, h2);
    gn_halve<2, 1, 2>(e2, f1, h1);
    const float f = f1[0] + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(f1[0]), (1 << 10) | 0x1F));
    // index held: within 22 by 11 h5; within 11 (as 12) by 6 h4; within 6 by 3 h3;
    // within 3 (as 4) by 2 h2; within 2 by h1
    const int i4 = (h2 ? 2 : 0) + (h1 ? 1 : 0);          // in the 3-group
    const int i16 = (h4 ? 6 : 0) + (h3 ? 3 : 0) + i4;   // in the 11-group
    vi = (i4 < 3 && i16 < 11) ? (h5 ? 11 : 0) + i16 : -1;
    return f;
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
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int n_in = min(max(nv[b], 0), a.cap);

    // ---- 1. compaction (query order) + normalisation ----
    const int per = (n_in + NT - 1) / NT;
    const int i0 = t * per, i1 = min(i0 + per, n_in);
    int cnt = 0;
    // a match index outside [0, cap) is "no match" (never dereferenced).  Up to PF_PER
    // entries per thread (cap <= 4 NT) are loaded, gathered and normalised here, before the
    // scan, so their load latency overlaps it instead of costing a second dependent pass.
    constexpr int PF_PER = 4;
    float4 pf[PF_PER];
    bool pok[PF_PER];
    if (per <= PF_PER) {
#pragma unroll
        for (int q = 0; q < PF_PER; q++) {
            const int i = i0 + q;
            pok[q] = false;
            pf[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i >= i1) continue;
            const size_t gi = (size_t)b * a.cap + i;
            float x2, y2;
            if (match_idx) {
                const int j = match_idx[gi];
                if ((unsigned)j >= (unsigned)a.cap) continue;
                x2 = kp1[((size_t)b * a.cap + j) * 2];
                y2 = kp1[((size_t)b * a.cap + j) * 2 + 1];
            } else {
                x2 = pts1[gi * 2];
                y2 = pts1[gi * 2 + 1];
            }
            const float x1 = pts0[gi * 2], y1 = pts0[gi * 2 + 1];
            pf[q] = make_float4((x1 - a.cx) / a.fx, (y1 - a.cy) / a.fy, (x2 - a.cx) / a.fx, (y2 - a.cy) / a.fy);
            pok[q] = true;
            cnt++;
        }
    } else {
        for (int i = i0; i < i1; i++)
            cnt += (!match_idx || (unsigned)match_idx[(size_t)b * a.cap + i] < (unsigned)a.cap) ? 1 : 0;
    }
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
    if (per <= PF_PER) {
#pragma unroll
        for (int q = 0; q < PF_PER; q++) {
            if (!pok[q]) continue;
            if (off < MAXP) P[off] = pf[q];
            off++;
        }
    } else {
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

    // ---- 2. hypotheses, preemptively MSAC-scored (sum of min(Sampson^2, thr^2); plain
    //         inlier counting cannot separate an outlier-contaminated 8-point solution that
    //         still explains every inlier within the band -- near-pure forward motion).
    //         Every hypothesis is scored on an evenly strided subset of PRE_M
    //         correspondences; the SURV best of each wave survive (preemptive RANSAC,
    //         Nister 2003) and are re-scored on all correspondences cooperatively. ----
    constexpr int PRE_M = PE_PREM, SURV = 2, NS = 4 * SURV;
    const int m = min(n, PRE_M);
    const unsigned step16 = ((unsigned)n << 16) / (unsigned)m;  // subset point k: (k * step16) >> 16 < n
    // the subset in point-pair layout (points 2k, 2k+1 of it in s_sub[k])
    __shared__ float4 s_sub[PRE_M / 2][2];
    if (t < m / 2) {
        const float4 pa = P[((2 * t) * step16) >> 16], pb = P[((2 * t + 1) * step16) >> 16];
        s_sub[t][0] = make_float4(pa.x, pb.x, pa.y, pb.y);
        s_sub[t][1] = make_float4(pa.z, pb.z, pa.w, pb.w);
    }
    __syncthreads();
    float best_cost = __builtin_inff();
    int best_h = 0x7fffffff;
    float best_e[9];
    for (int h = t; h < a.hypotheses; h += NT) {
        int idx[8];
        const unsigned long long base = a.seed ^ ((unsigned long long)b << 40) ^ ((unsigned long long)h << 8);
        int drawn = 0;
        unsigned long long r = 0;
        for (int d = 0; d < 64 && drawn < 8; d++) {  // two 32-bit draws per splitmix64 output
            if ((d & 1) == 0) r = splitmix64(base + (d >> 1));
            const unsigned u = (d & 1) ? (unsigned)r : (unsigned)(r >> 32);
            const int c = (int)(((unsigned long long)u * (unsigned)n) >> 32);
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
        f2v acc = {0.f, 0.f};
        const int m2 = m / 2;
        int k = 0;
        for (; k + 2 <= m2; k += 2) {  // 4 LDS broadcast reads in flight per step
            const float4 A0 = s_sub[k][0], B0 = s_sub[k][1], A1 = s_sub[k + 1][0], B1 = s_sub[k + 1][1];
            acc += msac_cost2(e, A0, B0, a.thr2);
            acc += msac_cost2(e, A1, B1, a.thr2);
        }
        if (k < m2) acc += msac_cost2(e, s_sub[k][0], s_sub[k][1], a.thr2);
        float cost = acc.x + acc.y;
        if (m & 1) {
            int c = 0;
            cost += msac_cost(e, P[((m - 1) * step16) >> 16], a.thr2, c);
        }
        if (cost < best_cost || (cost == best_cost && h < best_h)) {
            best_cost = cost;
            best_h = h;
#pragma unroll
            for (int r = 0; r < 9; r++) best_e[r] = e[r];
        }
    }
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
    for (int sv = 0; sv < NS; sv += 2) {  // two survivors per packed instruction
        f2v E2[9];
#pragma unroll
        for (int q = 0; q < 9; q++) E2[q] = f2v{s_sE[sv][q], s_sE[sv + 1][q]};
        f2v acc = {0.f, 0.f};
        int na = 0, nb = 0;
        if (s_sh[sv] >= 0 || s_sh[sv + 1] >= 0)
            for (int i = t; i < n; i += NT) acc += msac_cost2h(E2, P[i], a.thr2, na, nb);
        cs[sv] = s_sh[sv] >= 0 ? acc.x : 0.f;
        cs[sv + 1] = s_sh[sv + 1] >= 0 ? acc.y : 0.f;
        cn[sv] = s_sh[sv] >= 0 ? na : 0;
        cn[sv + 1] = s_sh[sv + 1] >= 0 ? nb : 0;
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
    // ---- 3b. the two lowest (full cost, hypothesis id) survivors are the starts of the
    //         refinement (below), and the refined pose with the lower robust cost wins.  Under pixel noise one start is not enough: the robust cost has local
    //         minima along the rotation / translation-direction ambiguity of forward motion and
    //         the best 8-point sample's pose can sit in one (the same algorithm on the CPU,
    //         0.5-1 px noise, 30 % outliers: single starts end 2-7 deg off in translation
    //         direction where the fit from the true pose is within 0.5; two starts: <= 1.6). ----
    __shared__ float s_E[2][9];
    __shared__ int s_nh;  // starts found (0, 1, 2)
    __shared__ bool s_exact;
    if (t == 0) {
        int b0 = -1, b1 = -1;
        float c0 = 0.f, c1 = 0.f;
        for (int sv = 0; sv < NS; sv++) {
            if (s_sh[sv] < 0) continue;
            const float c = s_red2[0][sv] + s_red2[1][sv] + s_red2[2][sv] + s_red2[3][sv];
            if (b0 < 0 || c < c0 || (c == c0 && s_sh[sv] < s_sh[b0])) {
                b1 = b0;
                c1 = c0;
                b0 = sv;
                c0 = c;
            } else if (b1 < 0 || c < c1 || (c == c1 && s_sh[sv] < s_sh[b1])) {
                b1 = sv;
                c1 = c;
            }
        }
        s_nh = b0 < 0 ? 0 : (b1 < 0 ? 1 : 2);
        // the best survivor's inliers fit (almost) exactly: sum of inlier r^2 = its MSAC cost
        // minus thr^2 per outlier, below 1e-3 thr^2 per inlier (exact projections: ~1e-12;
        // 0.5 px noise: ~0.2) -- the first start will likely be an exact fit
        if (b0 >= 0) {
            const float na0 = s_red2[0][NS + b0] + s_red2[1][NS + b0] + s_red2[2][NS + b0] + s_red2[3][NS + b0];
            s_exact = c0 - ((float)n - na0) * a.thr2 <= 1e-3f * na0 * a.thr2;
        }
        if (b0 >= 0)
            for (int r = 0; r < 9; r++) {
                s_E[0][r] = s_sE[b0][r];
                s_E[1][r] = s_sE[b1 >= 0 ? b1 : b0][r];
            }
    }
    __syncthreads();
    if (s_nh == 0) {
        if (t < 12) To[t] = (t % 4 == t / 4) ? 1.f : 0.f;
        if (t == 0) {
            num_inliers[b] = 0;
            if (num_matches) num_matches[b] = n_all;
            status[b] = MV_ERR_DEGENERATE;
        }
        return;
    }
    // ---- 4-6, per start: decomposition + cheirality, robust Gauss-Newton, the robust cost of
    //      the refined pose.  Two schedules over groups of waves, block-uniform:
    //      - sequential (one group = the block): the starts one after the other, the second only
    //        when the first did not reach an exact fit -- exact data costs one refinement;
    //      - concurrent (two groups = the block's halves, waves 0-1 and 2-3): when two starts
    //        exist and the best survivor's inliers are not an exact fit (noisy data, where both
    //        starts are refined anyway), each half refines one start, so the two Gauss-Newton
    //        chains share their barriers instead of running back to back.
    //      Every barrier is block-wide: a group that has converged keeps arriving at them. ----
    __shared__ float s_cand[2][4][12];
    __shared__ float s_uv[2][2][3][3];
    __shared__ int s_votes[4][4];  // [wave][candidate]
    __shared__ float s_red[2][4][22];
    __shared__ float s_state[2][2][16];  // [iteration parity][group]
    __shared__ float s_fin[4];
    __shared__ int s_fin_n[4];
    static_assert(MAXP <= 32 * (NT / 2), "the inlier mask holds 32 correspondences per thread of a half");
    const float th_max = sqrtf(a.thr2), th_min = 0.01f * th_max, r_cap = 3.f * th_max;
    float bR[9], bT[3], bcost = __builtin_inff();
    int bn = 0;
    // the schedule as a compile-time parameter: each gets its own code (constant strides)
    auto refine = [&](auto par_c) {
    constexpr bool par = decltype(par_c)::value;
    constexpr int G = par ? NT / 2 : NT;       // threads per group
    const int gid = par ? (w >> 1) : 0;        // this thread's group
    const int gt = par ? (t & (NT / 2 - 1)) : t;
    const int gw0 = par ? 2 * gid : 0;         // the group's first wave
    constexpr int gnw = par ? 2 : 4;           // its waves
    const int rounds = par ? 1 : s_nh;
    for (int rd = 0; rd < rounds; rd++) {
        const int sti = par ? gid : rd;
        float E[9];
        for (int r = 0; r < 9; r++) E[r] = s_E[sti][r];
        if (gt == 0) {
            float U[3][3], V[3][3];
            essential_uv(E, U, V);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    s_uv[gid][0][i][j] = U[i][j];
                    s_uv[gid][1][i][j] = V[i][j];
                }
        }
        __syncthreads();
        if (gt < 4) {  // candidate c = gt, one lane each
            const float W[3][3] = {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}};
            float U[3][3], V[3][3];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    U[i][j] = s_uv[gid][0][i][j];
                    V[i][j] = s_uv[gid][1][i][j];
                }
            const int c = gt;
            float R[3][3];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    float s = 0;
                    for (int k = 0; k < 3; k++) {
                        float uw = 0;
                        for (int l = 0; l < 3; l++) uw += U[i][l] * (c < 2 ? W[l][k] : W[k][l]);
                        s += uw * V[j][k];
                    }
                    R[i][j] = s;
                }
            const float sg = (c & 1) ? -1.f : 1.f;
            for (int i = 0; i < 9; i++) s_cand[gid][c][i] = R[i / 3][i % 3];
            for (int i = 0; i < 3; i++) s_cand[gid][c][9 + i] = sg * U[i][2];
        }
        __syncthreads();
        int votes[4] = {0, 0, 0, 0};
        unsigned inl_mask = 0;  // bit k: correspondence gt + k G is a Sampson inlier of E
        for (int i = gt, k = 0; i < n; i += G, k++)
            inl_mask |= sampson_inlier(E, P[i], a.thr2) ? 1u << k : 0u;
#pragma unroll
        for (int c = 0; c < 4; c++) {  // candidate-outer: 12 candidate floats live, not 48
            for (unsigned mk = inl_mask; mk; mk &= mk - 1) {
                const float4 p = P[gt + __builtin_ctz(mk) * G];
                // depths z1, z2 of the midpoint triangulation, q z1 + t = -m z2 in the least-
                // squares sense: z = num / det with det > 0, so only the numerators' signs count
                const float *C = s_cand[gid][c];
                const F3 q = {{C[0] * p.x + C[1] * p.y + C[2], C[3] * p.x + C[4] * p.y + C[5], C[6] * p.x + C[7] * p.y + C[8]}};
                const F3 m = {{-p.z, -p.w, -1.f}};
                const F3 tt = {{C[9], C[10], C[11]}};
                const float aa = dot3(q, q), ab = dot3(q, m), bb = dot3(m, m);
                const float ra = -dot3(q, tt), rb = -dot3(m, tt);
                const float det = aa * bb - ab * ab;
                const float n1 = ra * bb - ab * rb, n2 = aa * rb - ab * ra;
                votes[c] += (det > 0.f && n1 > 0.f && n2 > 0.f) ? 1 : 0;
            }
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
            int v = votes[c];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) s_votes[w][c] = v;
        }
        __syncthreads();
        auto gsum_votes = [&](int c) {
            int v = 0;
            for (int k = 0; k < gnw; k++) v += s_votes[gw0 + k][c];
            return v;
        };
        int bc = 0, bv = gsum_votes(0);
        for (int c = 1; c < 4; c++) {
            const int v = gsum_votes(c);
            if (v > bv) {
                bv = v;
                bc = c;
            }
        }

        // ---- robust Gauss-Newton: iteratively reweighted, Cauchy weights 1 / (1 + (r / c)^2)
        //      on the Sampson residuals below 3 thr (none above), the scale c_0 = thr,
        //      c_{k+1} = min(thr, max(2 rms_w, 0.01 thr)) (rms_w: the weighted rms of iteration
        //      k): on exact data c shrinks until the outliers that fell inside the band no
        //      longer pull (converges to machine precision), on noisy data it settles near
        //      2 sigma.  Weights and Sampson denominators are frozen within an iteration.  The
        //      group's first wave solves the 5x5 normal equations from the group's 22 sums; one
        //      block barrier per iteration after the sums, one after the state (both
        //      double-buffered). ----
        float R[9], tv[3], bs[6];
#pragma unroll
        for (int i = 0; i < 9; i++) R[i] = s_cand[gid][bc][i];
#pragma unroll
        for (int i = 0; i < 3; i++) tv[i] = s_cand[gid][bc][9 + i];
        tangent_basis_f(tv, bs);
        // with refine_iters = 0 no Gauss-Newton barrier separates these reads of the start from
        // thread 0's write of the refined pose into candidate slot 0 below (concurrent schedule)
        if (a.refine_iters == 0) __syncthreads();
        // the Cauchy scale.  An exact-fit start (s_exact: its inliers are exact projections)
        // starts at the floor: the annealing from thr only lets the outliers inside the band stop
        // pulling, and at the floor they pull with weight ~(c / r)^2 from the first iteration --
        // one Gauss-Newton iteration instead of two on the headline's pairs, 7 % of the pose
        // (profiles/r06p_pose_iters.log)
        float csc = (!par && rd == 0 && s_exact) ? th_min : th_max;
        bool act = true;     // this group still iterates (group-uniform)
        for (int it = 0; it < a.refine_iters; it++) {
            float acc[22];  // sum w J^T J (15, upper), sum w J^T r (5), sum w r^2, sum w
#pragma unroll
            for (int k = 0; k < 22; k++) acc[k] = 0.f;
            const float rcs = __builtin_amdgcn_rcpf(csc);
            for (int i = (!par || act) ? gt : n; i < n; i += G) {
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
                const float r = e * inv;                      // Sampson distance
                if (!(fabsf(r) < r_cap)) continue;
                const float u = r * rcs;
                const float wt = __builtin_amdgcn_rcpf(1.f + u * u);
                // d e / d omega = q x (x2 x t)  (R <- exp(omega) R);  d e / d t = q x x2
                const float dw[3] = {q[1] * x2t[2] - q[2] * x2t[1], q[2] * x2t[0] - q[0] * x2t[2],
                                     q[0] * x2t[1] - q[1] * x2t[0]};
                const float dt[3] = {q[1] * x2[2] - q[2] * x2[1], q[2] * x2[0] - q[0] * x2[2],
                                     q[0] * x2[1] - q[1] * x2[0]};
                const float J[5] = {dw[0] * inv, dw[1] * inv, dw[2] * inv,
                                    (dt[0] * bs[0] + dt[1] * bs[1] + dt[2] * bs[2]) * inv,
                                    (dt[0] * bs[3] + dt[1] * bs[4] + dt[2] * bs[5]) * inv};
                float Jw[5];
#pragma unroll
                for (int v = 0; v < 5; v++) Jw[v] = J[v] * wt;
                int k = 0;
#pragma unroll
                for (int v = 0; v < 5; v++) {
#pragma unroll
                    for (int x = v; x < 5; x++) acc[k++] += Jw[v] * J[x];
                }
#pragma unroll
                for (int v = 0; v < 5; v++) acc[15 + v] += Jw[v] * r;
                acc[20] += wt * r * r;
                acc[21] += wt;
            }
            // the 22 sums reduced over the wave by recursive halving (a reduce-scatter), then
            // the group's wave partials in LDS
            float(*red)[22] = s_red[it & 1];
            {
                int vi;  // the sum this lane holds after the halving
                const float f = gn_reduce_scatter22(acc, lane, vi);
                if (vi >= 0) red[w][vi] = f;
            }
            __syncthreads();
            float *st = s_state[it & 1][gid];
            if (w == gw0) {
                float H[15], g[5], r2 = 0.f, cnt = 0.f;
#pragma unroll
                for (int k = 0; k < 15; k++) H[k] = 0.f;
#pragma unroll
                for (int k = 0; k < 5; k++) g[k] = 0.f;
                for (int q = 0; q < gnw; q++) {
#pragma unroll
                    for (int k = 0; k < 15; k++) H[k] += red[gw0 + q][k];
#pragma unroll
                    for (int k = 0; k < 5; k++) g[k] += red[gw0 + q][15 + k];
                    r2 += red[gw0 + q][20];
                    cnt += red[gw0 + q][21];
                }
                // float Cholesky on the native reciprocal square root (the step only has to be
                // a descent direction); every loop fully unrolled: static register indexing
                float A[5][5];
#pragma unroll
                for (int v = 0, k = 0; v < 5; v++)
#pragma unroll
                    for (int x = v; x < 5; x++, k++) {
                        A[v][x] = H[k];
                        A[x][v] = H[k];
                    }
#pragma unroll
                for (int v = 0; v < 5; v++) A[v][v] = A[v][v] * (1.0f + 1e-6f) + 1e-30f;
                float L[5][5] = {}, rl[5] = {};
                bool ok = (!par || act) && cnt >= 5.f;
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
                const float cs_new = fminf(th_max, fmaxf(2.f * sqrtf(r2 / cnt), th_min));
                float dmax = 0.f;
#pragma unroll
                for (int i = 0; i < 5; i++) dmax = fmaxf(dmax, fabsf(d[i]));
                // converged: a step below 1e-4 rad / unit-t (Gauss-Newton converges quadratically
                // on exact data: the error left after such a step is ~1e-8) and a scale that moved
                // < 2 % (noisy data: the pose then moves far below its noise floor); 1e-6 / 0.1 %
                // measured the same on exact data and 9 % slower under 0.5 px noise
                const bool done = dmax < 1e-4f && fabsf(cs_new - csc) <= 2e-2f * csc;
                // lane k < 14 stores word k of the state (static register indexing):
                // R (9), t (3), scale, flags (bit 0: failed or stopped -- keep the old state;
                // bit 1: converged)
                if (lane < 14) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < 9; k++) v = lane == k ? Rn[k] : v;
#pragma unroll
                    for (int k = 0; k < 3; k++) v = lane == 9 + k ? tn[k] * rn : v;
                    v = lane == 12 ? cs_new : v;
                    v = lane == 13 ? __int_as_float((ok ? 0 : 1) | (done ? 2 : 0)) : v;
                    st[lane] = v;
                }
            }
            __syncthreads();
            const int flags = __float_as_int(st[13]);
            if ((!par || act) && !(flags & 1)) {
#pragma unroll
                for (int i = 0; i < 9; i++) R[i] = st[i];
#pragma unroll
                for (int i = 0; i < 3; i++) tv[i] = st[9 + i];
                tangent_basis_f(tv, bs);
                csc = st[12];
            }
            if constexpr (par) {
                act = act && !(flags & 3);
                // block-uniform exit: every group has stopped
                const bool other = !(__float_as_int(s_state[it & 1][gid ^ 1][13]) & 3);
                if (!act && !other) break;
            } else {
                if (flags & 3) break;  // the same decision in every thread
            }
        }

        // ---- the robust cost of the refined pose (Cauchy at the scale thr, capped at 3 thr) and
        //      its inliers (Sampson distance < thr): the lower cost over the starts wins ----
        float rcost = 0.f;
        int ninl = 0;
        for (int i = gt; i < n; i += G) {
            const float4 p = P[i];
            const float q[3] = {R[0] * p.x + R[1] * p.y + R[2], R[3] * p.x + R[4] * p.y + R[5],
                                R[6] * p.x + R[7] * p.y + R[8]};
            const float x2t[3] = {p.w * tv[2] - tv[1], tv[0] - p.z * tv[2], p.z * tv[1] - p.w * tv[0]};
            const float e = x2t[0] * q[0] + x2t[1] * q[1] + x2t[2] * q[2];
            const float Ex1[2] = {tv[1] * q[2] - tv[2] * q[1], tv[2] * q[0] - tv[0] * q[2]};
            float Etx2[2];
#pragma unroll
            for (int c = 0; c < 2; c++) Etx2[c] = R[c] * x2t[0] + R[3 + c] * x2t[1] + R[6 + c] * x2t[2];
            const float s2 = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Etx2[0] * Etx2[0] + Etx2[1] * Etx2[1];
            const float ar = s2 > 0.f ? fabsf(e) * __builtin_amdgcn_rsqf(s2) : r_cap;
            const float u = fminf(ar, r_cap) / th_max;
            rcost += __logf(1.f + u * u);
            ninl += ar < th_max ? 1 : 0;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            rcost += __shfl_xor(rcost, o, 64);
            ninl += __shfl_xor(ninl, o, 64);
        }
        if (lane == 0) {
            s_fin[w] = rcost;
            s_fin_n[w] = ninl;
        }
        if (par && gt == 0) {  // each half's refined pose, for the threads that write the output
#pragma unroll
            for (int i = 0; i < 9; i++) s_cand[gid][0][i] = R[i];
#pragma unroll
            for (int i = 0; i < 3; i++) s_cand[gid][0][9 + i] = tv[i];
        }
        __syncthreads();
        // the group costs; concurrent: start 0's group first, so a tie keeps start 0 as in the
        // sequential schedule
        for (int gg = 0; gg < (par ? 2 : 1); gg++) {
            const int w0 = par ? 2 * gg : 0, nw = par ? 2 : 4;
            float cost = 0.f;
            int cn_ = 0;
            for (int k = 0; k < nw; k++) {
                cost += s_fin[w0 + k];
                cn_ += s_fin_n[w0 + k];
            }
            if (cost < bcost) {  // the same decision in every thread (a tie keeps the earlier start)
                bcost = cost;
                bn = cn_;
#pragma unroll
                for (int i = 0; i < 9; i++) bR[i] = par ? s_cand[gg][0][i] : R[i];
#pragma unroll
                for (int i = 0; i < 3; i++) bT[i] = par ? s_cand[gg][0][9 + i] : tv[i];
            }
        }
        __syncthreads();  // s_uv, s_cand, s_votes, s_fin are the next start's
        if constexpr (!par)
            if (csc <= th_min * 1.0001f) break;  // an exact fit: no second start needed
    }
    };
    if (s_nh == 2 && !s_exact)
        refine(std::true_type{});
    else
        refine(std::false_type{});
    {  // [R | t] row-major, thread t < 12 writes entry t (static register indexing)
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 12; k++) v = t == k ? (k % 4 < 3 ? bR[(k / 4) * 3 + k % 4] : bT[k / 4]) : v;
        if (t < 12) To[t] = v;
    }
    if (t == 0) {
        num_inliers[b] = bn;
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
