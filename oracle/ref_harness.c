/*
 * ref_harness.c -- exports thin wrappers around the reference's header-only
 * code so tests can call it through ctypes.  Compiled by oracle/Makefile ONLY
 * where /root/reference exists; output goes to oracle/_ref/ (git-ignored).
 * The reference sources are used where they lie (include paths), never copied.
 */
#include <stdbool.h>
#include "gemmini_functions_cpu.h" /* include/gemmini_functions_cpu.h:14-124 */

/* C[I][J] += A[I][K] . B[J][K]^T  -- the all-pairs match shape */
void ref_matmul_nt(int I, int J, int K, const float *A, const float *B, float *C) {
    matmul((size_t)I, (size_t)J, (size_t)K, A, B, C, (size_t)K, (size_t)K, (size_t)J, 1.0f, 1.0f, false, true);
}

/* src/projection_factor.c + src/types.c: compute_error_ProjectionFactor on one factor.
 * pose [7] = (qw, qx, qy, qz, tx, ty, tz), cam [4] = (fx, fy, cx, cy). */
#include "projection_factor.h"
void ref_pf_error(const float *X, const float *pose, const float *meas, const float *cam, float *err) {
    Vector3f l = {X[0], X[1], X[2]};
    SE3 T;
    T.q.w = pose[0];
    T.q.x = pose[1];
    T.q.y = pose[2];
    T.q.z = pose[3];
    T.t.x = pose[4];
    T.t.y = pose[5];
    T.t.z = pose[6];
    ProjectionFactor f;
    f.landmark = &l;
    f.pose = &T;
    f.measurement.x = meas[0];
    f.measurement.y = meas[1];
    f.camera.fx = cam[0];
    f.camera.fy = cam[1];
    f.camera.cx = cam[2];
    f.camera.cy = cam[3];
    compute_error_ProjectionFactor(&f);
    err[0] = f.error.x;
    err[1] = f.error.y;
}

/* local_bundle_adjustment.c:161-169: H_factor = J_factor^T J_factor by gemmini matmul2 */
void ref_h_factor(const float *J20, float *H100) {
    matmul2(10, 10, 2, J20, J20, H100, H100, 2, 2, 10, 10, 1, 1, 0, false, true);
}
