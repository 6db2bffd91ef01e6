/*
 * factors.h -- projection factors and their normal equations (the
 * BASELINE north star's "projection_factor.c as per-correspondence Jacobian + J^T J / J^T r
 * assembly"), batched on the device.  Replaces, for many factors at once:
 *   compute_error_ProjectionFactor   src/projection_factor.c:28-33 (with src/types.c:3-73):
 *       e = K pi(q (x) X (x) q* + t) - z, float32 in the reference's order (bit-identical);
 *   the factor block [J | r] of src/local_bundle_adjustment.c:140-169 (a 2 x 10 column-major
 *       matrix, columns [landmark 3 | pose 6 | residual 1]; the reference fills it with
 *       placeholder numbers) -- here the analytic Jacobian: landmark columns D R(q), rotation
 *       columns -D [p]x (left perturbation p' = p + omega x p), translation columns D, with
 *       D = d(K pi)/dp at p = R X + t;
 *   H_factor = [J|r]^T [J|r] (:161-169, matmul2's k order) and its scatter into the pose block
 *       (:184-200), accumulated factor by factor in order.
 * Layouts: landmarks [L][3]; poses [P][7] = (qw, qx, qy, qz, tx, ty, tz); cameras [P][4] =
 * (fx, fy, cx, cy) per pose; factor f: (ldmk_id[f], pose_id[f], meas[f][2]).
 */
#ifndef MV_FACTORS_H
#define MV_FACTORS_H
#include "maveric_hip.h"
#ifdef __cplusplus
extern "C" {
#endif

/* err [F][2]; J [F][20] column-major 2 x 10 (may be NULL); H [F][100] row-major (may be NULL). */
int mv_projection_factors_dev(mv_context *ctx, int num_factors, const float *landmarks, const float *poses,
                              const float *cameras, const int *ldmk_id, const int *pose_id, const float *meas,
                              float *err, float *J, float *H);
/* Pose-only normal equations from the factors' J (pose refinement, one system per pose):
 * factors of pose p are [pose_offsets[p], pose_offsets[p+1]) and are summed in that order.
 * HPP [P][36] = sum J_pose^T J_pose, g [P][6] = sum J_pose^T r, ee [P] = sum r^T r. */
int mv_pose_normal_equations_dev(mv_context *ctx, int num_poses, const int *pose_offsets, const float *J,
                                 float *HPP, float *g, float *ee);

/* The local-BA Schur back-end (src/local_bundle_adjustment.c:128-250) for `batch`
 * independent windows of num_poses poses and num_ldmks landmarks (every landmark observed by
 * every pose, as in the reference), chunk landmarks at a time: J [batch][ceil(L/chunk)]
 * [num_poses * chunk][20] holds each chunk's factor blocks (2 x 10 column-major, [landmark |
 * pose | residual]); factor (landmark i of the chunk, pose p) is entry p * i with
 * MV_AS_BUILT (the reference's index, local_bundle_adjustment.c:158) and i * num_poses + p
 * with MV_AS_INTENDED.  C [batch][S][S] (S = 6 num_poses + 1, column-major) is accumulated
 * in place: the pose-pose Schur complement (plus the reference's residual row).  The
 * reference's order throughout (bit-identical to its own functions).  LDS: 4 (100 + 9 chunk^2
 * + 6 S chunk + S^2) bytes <= 64 KiB. */
int mv_lba_schur_dev(mv_context *ctx, int batch, int num_poses, int num_ldmks, int chunk, int semantics,
                     const float *J, float *C);

#ifdef __cplusplus
}
#endif
#endif
