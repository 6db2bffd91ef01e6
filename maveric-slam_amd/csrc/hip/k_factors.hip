// k_factors.hip -- projection factors and pose normal equations (include/factors.h).
//   k_pf_linearize   thread per factor: the reference's error in its float order (quaternion
//                    sandwich, project, affine), the analytic 2 x 9 Jacobian, the residual
//                    column, and optionally H_factor = [J|r]^T [J|r] (two products per entry,
//                    matmul2's k order).  Bound: HBM (~60 B in, 88 B out per factor without H).
//   k_pose_ne        one wave per pose: lane e < 43 owns one entry of (HPP 36, g 6, r^T r 1)
//                    and adds the factors' contributions in factor order (the scatter order of
//                    local_bundle_adjustment.c), the J rows of 8 factors loaded ahead.
#include "factors.h"
#include "mv_internal.hpp"

namespace {

__device__ __forceinline__ void qmul(const float *a, const float *b, float *o) {  // types.c:19-26 order
    o[0] = __fsub_rn(__fsub_rn(__fsub_rn(__fmul_rn(a[0], b[0]), __fmul_rn(a[1], b[1])), __fmul_rn(a[2], b[2])),
                     __fmul_rn(a[3], b[3]));
    o[1] = __fsub_rn(__fadd_rn(__fadd_rn(__fmul_rn(a[0], b[1]), __fmul_rn(a[1], b[0])), __fmul_rn(a[2], b[3])),
                     __fmul_rn(a[3], b[2]));
    o[2] = __fadd_rn(__fadd_rn(__fsub_rn(__fmul_rn(a[0], b[2]), __fmul_rn(a[1], b[3])), __fmul_rn(a[2], b[0])),
                     __fmul_rn(a[3], b[1]));
    o[3] = __fadd_rn(__fsub_rn(__fadd_rn(__fmul_rn(a[0], b[3]), __fmul_rn(a[1], b[2])), __fmul_rn(a[2], b[1])),
                     __fmul_rn(a[3], b[0]));
}

__global__ __launch_bounds__(256) void k_pf_linearize(int F, const float *__restrict__ ldmk,
                                                      const float *__restrict__ pose, const float *__restrict__ cam,
                                                      const int *__restrict__ lid, const int *__restrict__ pid,
                                                      const float *__restrict__ meas, float *__restrict__ err,
                                                      float *__restrict__ Jout, float *__restrict__ Hout) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f >= F) return;
    const float *X = ldmk + 3l * lid[f], *T = pose + 7l * pid[f], *K = cam + 4l * pid[f];
    const float vq[4] = {0.f, X[0], X[1], X[2]}, qc[4] = {T[0], -T[1], -T[2], -T[3]};
    float qv[4], r[4];
    qmul(T, vq, qv);
    qmul(qv, qc, r);
    const float px = __fadd_rn(r[1], __fmul_rn(1.f, T[4])), py = __fadd_rn(r[2], __fmul_rn(1.f, T[5])),
                pz = __fadd_rn(r[3], __fmul_rn(1.f, T[6]));
    const float ux = px / pz, uy = py / pz;
    const float ex = __fadd_rn(__fadd_rn(__fmul_rn(ux, K[0]), K[2]), __fmul_rn(-1.f, meas[2l * f]));
    const float ey = __fadd_rn(__fadd_rn(__fmul_rn(uy, K[1]), K[3]), __fmul_rn(-1.f, meas[2l * f + 1]));
    err[2l * f] = ex;
    err[2l * f + 1] = ey;
    if (!Jout && !Hout) return;
    const float iz = 1.f / pz;
    const float d00 = __fmul_rn(K[0], iz), d02 = __fmul_rn(__fmul_rn(-__fmul_rn(K[0], px), iz), iz);
    const float d11 = __fmul_rn(K[1], iz), d12 = __fmul_rn(__fmul_rn(-__fmul_rn(K[1], py), iz), iz);
    const float w = T[0], x = T[1], y = T[2], z = T[3];
    const float ww = __fmul_rn(w, w), xx = __fmul_rn(x, x), yy = __fmul_rn(y, y), zz = __fmul_rn(z, z);
    const float R[9] = {__fsub_rn(__fsub_rn(__fadd_rn(ww, xx), yy), zz),
                        __fmul_rn(2.f, __fsub_rn(__fmul_rn(x, y), __fmul_rn(w, z))),
                        __fmul_rn(2.f, __fadd_rn(__fmul_rn(x, z), __fmul_rn(w, y))),
                        __fmul_rn(2.f, __fadd_rn(__fmul_rn(x, y), __fmul_rn(w, z))),
                        __fsub_rn(__fadd_rn(__fsub_rn(ww, xx), yy), zz),
                        __fmul_rn(2.f, __fsub_rn(__fmul_rn(y, z), __fmul_rn(w, x))),
                        __fmul_rn(2.f, __fsub_rn(__fmul_rn(x, z), __fmul_rn(w, y))),
                        __fmul_rn(2.f, __fadd_rn(__fmul_rn(y, z), __fmul_rn(w, x))),
                        __fadd_rn(__fsub_rn(__fsub_rn(ww, xx), yy), zz)};
    const float S[9] = {0.f, pz, -py, -pz, 0.f, px, py, -px, 0.f};
    float J[20];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        J[2 * c] = __fadd_rn(__fmul_rn(d00, R[c]), __fmul_rn(d02, R[6 + c]));
        J[2 * c + 1] = __fadd_rn(__fmul_rn(d11, R[3 + c]), __fmul_rn(d12, R[6 + c]));
        J[2 * (3 + c)] = __fadd_rn(__fmul_rn(d00, S[c]), __fmul_rn(d02, S[6 + c]));
        J[2 * (3 + c) + 1] = __fadd_rn(__fmul_rn(d11, S[3 + c]), __fmul_rn(d12, S[6 + c]));
    }
    J[12] = d00;
    J[13] = 0.f;
    J[14] = 0.f;
    J[15] = d11;
    J[16] = d02;
    J[17] = d12;
    J[18] = ex;
    J[19] = ey;
    if (Jout) {
        float4 *o = reinterpret_cast<float4 *>(Jout + 20l * f);
#pragma unroll
        for (int i = 0; i < 5; i++) o[i] = make_float4(J[4 * i], J[4 * i + 1], J[4 * i + 2], J[4 * i + 3]);
    }
    if (Hout) {
        float *h = Hout + 100l * f;
#pragma unroll
        for (int i = 0; i < 10; i++)
#pragma unroll
            for (int j = 0; j < 10; j++)
                h[10 * i + j] = __fadd_rn(__fadd_rn(0.f, __fmul_rn(J[2 * i], J[2 * j])), __fmul_rn(J[2 * i + 1], J[2 * j + 1]));
    }
}

__global__ __launch_bounds__(64) void k_pose_ne(const int *__restrict__ off, const float *__restrict__ J,
                                                float *__restrict__ HPP, float *__restrict__ g, float *__restrict__ ee) {
    const int p = blockIdx.x, e = threadIdx.x;
    // entry e: HPP (i, j) = rows 3+i, 3+j (e < 36); g i = (3+i, 9) (36 <= e < 42); r^T r = (9, 9)
    int ci, cj;
    if (e < 36) {
        ci = 3 + e / 6;
        cj = 3 + e % 6;
    } else if (e < 42) {
        ci = 3 + (e - 36);
        cj = 9;
    } else {
        ci = 9;
        cj = 9;
    }
    const int f0 = off[p], f1 = off[p + 1];
    float acc = 0.f;
    int f = f0;
    for (; f + 8 <= f1; f += 8) {
        float a0[8], a1[8], b0[8], b1[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const float *Jf = J + 20l * (f + u);
            a0[u] = Jf[2 * ci];
            a1[u] = Jf[2 * ci + 1];
            b0[u] = Jf[2 * cj];
            b1[u] = Jf[2 * cj + 1];
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            acc = __fadd_rn(__fadd_rn(__fadd_rn(0.f, __fmul_rn(a0[u], b0[u])), __fmul_rn(a1[u], b1[u])), acc);
    }
    for (; f < f1; f++) {
        const float *Jf = J + 20l * f;
        acc = __fadd_rn(__fadd_rn(__fadd_rn(0.f, __fmul_rn(Jf[2 * ci], Jf[2 * cj])), __fmul_rn(Jf[2 * ci + 1], Jf[2 * cj + 1])),
                        acc);
    }
    if (e < 36)
        HPP[36l * p + e] = acc;
    else if (e < 42)
        g[6l * p + e - 36] = acc;
    else if (e == 42)
        ee[p] = acc;
}

}  // namespace

extern "C" int mv_projection_factors_dev(mv_context *ctx, int num_factors, const float *landmarks,
                                         const float *poses, const float *cameras, const int *ldmk_id,
                                         const int *pose_id, const float *meas, float *err, float *J, float *H) {
    MV_REQUIRE(ctx && num_factors >= 0 && landmarks && poses && cameras && ldmk_id && pose_id && meas && err);
    MV_REQUIRE(!J || ((uintptr_t)J & 15) == 0);
    if (num_factors == 0) return mv::set_status(MV_OK);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    MV_PROF_BEGIN(ctx->stream, "k_pf_linearize");
    hipLaunchKernelGGL(k_pf_linearize, dim3((unsigned)((num_factors + 255) / 256)), dim3(256), 0, ctx->stream,
                       num_factors, landmarks, poses, cameras, ldmk_id, pose_id, meas, err, J, H);
    MV_PROF_END(ctx->stream);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}

extern "C" int mv_pose_normal_equations_dev(mv_context *ctx, int num_poses, const int *pose_offsets, const float *J,
                                            float *HPP, float *g, float *ee) {
    MV_REQUIRE(ctx && num_poses > 0 && pose_offsets && J && HPP && g && ee);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    MV_PROF_BEGIN(ctx->stream, "k_pose_ne");
    hipLaunchKernelGGL(k_pose_ne, dim3((unsigned)num_poses), dim3(64), 0, ctx->stream, pose_offsets, J, HPP, g, ee);
    MV_PROF_END(ctx->stream);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}
