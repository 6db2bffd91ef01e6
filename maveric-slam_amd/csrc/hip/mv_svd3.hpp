// mv_svd3.hpp -- branch-free 3x3 SVD of McAdams, Selle, Tamstorf, Teran,
// Sifakis (UW-Madison TR1690, 2011) as used by the reference (include/svd/svd.h:358-405),
// for one lane.  Every float operation is issued in the same order as the
// reference so the result is bit-identical (the TU must be built with
// -ffp-contract=off).  Outputs follow call_svd() (src/pnp_solver.c:8-25):
// U, the diagonal of R as S, and V (NOT transposed).
#pragma once
#include <hip/hip_runtime.h>

namespace mv {

struct Mat3 {
    float m[3][3];
};

// svd.h:37-48 / :54-62 -- approximate 1/sqrt with one or two Newton steps
__device__ __forceinline__ float rsqrt_nr1(float x) {
    const float h = 0.5f * x;
    const float y = __int_as_float(0x5f375a82 - (__float_as_int(x) >> 1));
    return y * (1.5f - h * y * y);
}
__device__ __forceinline__ float rsqrt_nr2(float x) {
    const float h = 0.5f * x;
    float y = __int_as_float(0x5f37599e - (__float_as_int(x) >> 1));
    y = y * (1.5f - h * y * y);
    return y * (1.5f - h * y * y);
}

// symmetric matrix (lower triangle) + accumulated quaternion (x, y, z, w)
struct SymQ {
    float s11, s21, s22, s31, s32, s33;
    float q[4];
};

// one Jacobi conjugation on the (p, q) = leading pair, then a cyclic relabel
__device__ __forceinline__ void jacobi_conj(SymQ &S, int x, int y, int z) {
    float ch = 2 * (S.s11 - S.s22);
    float sh = S.s21;
    const bool use = 5.828427124 * sh * sh < (double)(ch * ch);
    const float w = rsqrt_nr1(ch * ch + sh * sh);
    ch = use ? w * ch : (float)0.923879532;
    sh = use ? w * sh : (float)0.3826834323;
    const float sc = ch * ch + sh * sh;
    const float a = (ch * ch - sh * sh) / sc;
    const float b = (2 * sh * ch) / sc;
    const float o11 = S.s11, o21 = S.s21, o22 = S.s22, o31 = S.s31, o32 = S.s32, o33 = S.s33;
    const float r11 = a * (a * o11 + b * o21) + b * (a * o21 + b * o22);
    const float r21 = a * (-b * o11 + a * o21) + b * (-b * o21 + a * o22);
    const float r22 = -b * (-b * o11 + a * o21) + a * (-b * o21 + a * o22);
    const float r31 = a * o31 + b * o32;
    const float r32 = -b * o31 + a * o32;
    const float r33 = o33;
    float t0 = S.q[0] * sh, t1 = S.q[1] * sh, t2 = S.q[2] * sh;
    sh *= S.q[3];
    S.q[0] *= ch;
    S.q[1] *= ch;
    S.q[2] *= ch;
    S.q[3] *= ch;
    const float tv[3] = {t0, t1, t2};
    S.q[z] += sh;
    S.q[3] -= tv[z];
    S.q[x] += tv[y];
    S.q[y] -= tv[x];
    S.s11 = r22;
    S.s21 = r32;
    S.s22 = r33;
    S.s31 = r21;
    S.s32 = r31;
    S.s33 = r11;
}

__device__ __forceinline__ void qr_givens(float a1, float a2, float &ch, float &sh) {
    const float eps = (float)1e-6;
    const float r2 = a1 * a1 + a2 * a2;
    const float rho = r2 * rsqrt_nr2(r2);
    float s = rho > eps ? a2 : 0;
    float c = fabsf(a1) + fmaxf(rho, eps);
    if (a1 < 0) {
        const float tmp = s;
        s = c;
        c = tmp;
    }
    const float w = rsqrt_nr1(c * c + s * s);
    ch = c * w;
    sh = s * w;
}

__device__ __forceinline__ void neg_swap_cols(Mat3 &M, int c0, int c1) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const float z = -M.m[r][c0];
        M.m[r][c0] = M.m[r][c1];
        M.m[r][c1] = z;
    }
}

__device__ inline void svd3(const Mat3 &A, Mat3 &U, float S[3], Mat3 &V) {
    const float(*a)[3] = A.m;
    SymQ sq;
    sq.s11 = a[0][0] * a[0][0] + a[1][0] * a[1][0] + a[2][0] * a[2][0];
    sq.s21 = a[0][1] * a[0][0] + a[1][1] * a[1][0] + a[2][1] * a[2][0];
    sq.s22 = a[0][1] * a[0][1] + a[1][1] * a[1][1] + a[2][1] * a[2][1];
    sq.s31 = a[0][2] * a[0][0] + a[1][2] * a[1][0] + a[2][2] * a[2][0];
    sq.s32 = a[0][2] * a[0][1] + a[1][2] * a[1][1] + a[2][2] * a[2][1];
    sq.s33 = a[0][2] * a[0][2] + a[1][2] * a[1][2] + a[2][2] * a[2][2];
    sq.q[0] = 0;
    sq.q[1] = 0;
    sq.q[2] = 0;
    sq.q[3] = 1;
    for (int sweep = 0; sweep < 4; sweep++) {
        jacobi_conj(sq, 0, 1, 2);
        jacobi_conj(sq, 1, 2, 0);
        jacobi_conj(sq, 2, 0, 1);
    }
    const float x = sq.q[0], y = sq.q[1], z = sq.q[2], w = sq.q[3];
    const float xx = x * x, yy = y * y, zz = z * z, xz = x * z, xy = x * y, yz = y * z;
    const float wx = w * x, wy = w * y, wz = w * z;
    V.m[0][0] = 1 - 2 * (yy + zz);
    V.m[0][1] = 2 * (xy - wz);
    V.m[0][2] = 2 * (xz + wy);
    V.m[1][0] = 2 * (xy + wz);
    V.m[1][1] = 1 - 2 * (xx + zz);
    V.m[1][2] = 2 * (yz - wx);
    V.m[2][0] = 2 * (xz - wy);
    V.m[2][1] = 2 * (yz + wx);
    V.m[2][2] = 1 - 2 * (xx + yy);
    Mat3 Bm;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            Bm.m[i][j] = a[i][0] * V.m[0][j] + a[i][1] * V.m[1][j] + a[i][2] * V.m[2][j];
    float rho1 = Bm.m[0][0] * Bm.m[0][0] + Bm.m[1][0] * Bm.m[1][0] + Bm.m[2][0] * Bm.m[2][0];
    float rho2 = Bm.m[0][1] * Bm.m[0][1] + Bm.m[1][1] * Bm.m[1][1] + Bm.m[2][1] * Bm.m[2][1];
    float rho3 = Bm.m[0][2] * Bm.m[0][2] + Bm.m[1][2] * Bm.m[1][2] + Bm.m[2][2] * Bm.m[2][2];
    if (rho1 < rho2) {
        neg_swap_cols(Bm, 0, 1);
        neg_swap_cols(V, 0, 1);
        const float tmp = rho1;
        rho1 = rho2;
        rho2 = tmp;
    }
    if (rho1 < rho3) {
        neg_swap_cols(Bm, 0, 2);
        neg_swap_cols(V, 0, 2);
        const float tmp = rho1;
        rho1 = rho3;
        rho3 = tmp;
    }
    if (rho2 < rho3) {
        neg_swap_cols(Bm, 1, 2);
        neg_swap_cols(V, 1, 2);
    }
    // QR by three Givens rotations
    float ch1, sh1, ch2, sh2, ch3, sh3;
    Mat3 R;
    qr_givens(Bm.m[0][0], Bm.m[1][0], ch1, sh1);
    float ga = 1 - 2 * sh1 * sh1, gb = 2 * ch1 * sh1;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        R.m[0][j] = ga * Bm.m[0][j] + gb * Bm.m[1][j];
        R.m[1][j] = -gb * Bm.m[0][j] + ga * Bm.m[1][j];
        R.m[2][j] = Bm.m[2][j];
    }
    qr_givens(R.m[0][0], R.m[2][0], ch2, sh2);
    ga = 1 - 2 * sh2 * sh2;
    gb = 2 * ch2 * sh2;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const float r0 = R.m[0][j], r1 = R.m[1][j], r2 = R.m[2][j];
        Bm.m[0][j] = ga * r0 + gb * r2;
        Bm.m[1][j] = r1;
        Bm.m[2][j] = -gb * r0 + ga * r2;
    }
    qr_givens(Bm.m[1][1], Bm.m[2][1], ch3, sh3);
    ga = 1 - 2 * sh3 * sh3;
    gb = 2 * ch3 * sh3;
    S[0] = Bm.m[0][0];
    S[1] = ga * Bm.m[1][1] + gb * Bm.m[2][1];
    S[2] = -gb * Bm.m[1][2] + ga * Bm.m[2][2];
    const float p1 = sh1 * sh1, p2 = sh2 * sh2, p3 = sh3 * sh3;
    U.m[0][0] = (-1 + 2 * p1) * (-1 + 2 * p2);
    U.m[0][1] = 4 * ch2 * ch3 * (-1 + 2 * p1) * sh2 * sh3 + 2 * ch1 * sh1 * (-1 + 2 * p3);
    U.m[0][2] = 4 * ch1 * ch3 * sh1 * sh3 - 2 * ch2 * (-1 + 2 * p1) * sh2 * (-1 + 2 * p3);
    U.m[1][0] = 2 * ch1 * sh1 * (1 - 2 * p2);
    U.m[1][1] = -8 * ch1 * ch2 * ch3 * sh1 * sh2 * sh3 + (-1 + 2 * p1) * (-1 + 2 * p3);
    U.m[1][2] = -2 * ch3 * sh3 + 4 * sh1 * (ch3 * sh1 * sh3 + ch1 * ch2 * sh2 * (-1 + 2 * p3));
    U.m[2][0] = 2 * ch2 * sh2;
    U.m[2][1] = 2 * ch3 * (1 - 2 * p2) * sh3;
    U.m[2][2] = (-1 + 2 * p2) * (-1 + 2 * p3);
}

// src/pnp_solver.c:168-194: R1 = U W, R2 = U W^T, t = U[:,2]
__device__ inline void recover_pose_mcadams(const Mat3 &E, Mat3 &R1, Mat3 &R2, float t[3]) {
    Mat3 U, V;
    float S[3];
    svd3(E, U, S, V);
    const float W[3][3] = {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}};
    const float Wt[3][3] = {{0, 1, 0}, {-1, 0, 0}, {0, 0, 1}};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            R1.m[i][j] = U.m[i][0] * W[0][j] + U.m[i][1] * W[1][j] + U.m[i][2] * W[2][j];
            R2.m[i][j] = U.m[i][0] * Wt[0][j] + U.m[i][1] * Wt[1][j] + U.m[i][2] * Wt[2][j];
        }
#pragma unroll
    for (int i = 0; i < 3; i++) t[i] = U.m[i][2];
}

}  // namespace mv
