/*
 * trajectory.h -- trajectory chaining + pose I/O, the step after the
 * per-pair poses: python/compute_trajectory.py:53-90 (chain, .pose.txt) and :6-43 (PLY).
 *
 * Poses are [3][4] float64, row-major [R | t] (the reference's np.eye(4)[:3, :] and the
 * dtype of outputs/transform_*.npy).  Relative transform k maps frame k to frame k+1.
 *
 * Two chain rules:
 *   MV_CHAIN_AS_BUILT  compute_trajectory.py:73-79 as it runs: R <- R_rel R, t <- t_rel + t
 *                      (t accumulates un-rotated).  Reproduces the committed
 *                      outputs/785/trajectory_000785_000789.ply bit for bit.
 *   MV_CHAIN_COMPOSE   pose <- T_rel . pose (4x4 left composition): R <- R_rel R,
 *                      t <- R_rel t + t_rel.  Reproduces the older outputs/785/trajectory.ply.
 * Every product is summed k = 0, 1, 2 (then + t_rel), mul then add, in float64 (numpy's
 * order for these shapes): the chain on the GPU equals the sequential host loop bit for bit.
 */
#ifndef MV_TRAJECTORY_H
#define MV_TRAJECTORY_H
#include "maveric_hip.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef enum { MV_CHAIN_AS_BUILT = 0, MV_CHAIN_COMPOSE = 1 } mv_chain_mode;

/* Batched chain on the device.  rel [batch][len][12], present [batch][len] (NULL = all
 * present; 0 = the transform file was missing: the reference skips it and the pose carries
 * over, compute_trajectory.py:86-87), start [batch][12] (NULL = identity).
 * poses [batch][len + 1][12]: poses[b][0] = start, poses[b][k + 1] = chain(rel[b][k], poses[b][k]).
 * One wave walks one sequence in order (the sequential rounding is the contract). */
int mv_trajectory_chain_dev(mv_context *ctx, int batch, int len, const double *rel, const int *present,
                            const double *start, int mode, double *poses);
/* Re-base chained poses onto a start pose (multi-GPU: a sequence sharded over ranks, each
 * rank chained from identity): poses[b][k] <- rule(poses[b][k], base[b]) for every k, i.e.
 * the pose the chain would reach from `base` instead of the identity.  AS_BUILT:
 * R <- R_k R_base, t <- t_k + t_base; COMPOSE: R <- R_k R_base, t <- R_k t_base + t_k.
 * Re-association: equal to the unsharded chain within float64 rounding, not bit for bit. */
int mv_trajectory_rebase_dev(mv_context *ctx, int batch, int len1, const double *base, int mode, double *poses);
/* One sequence, host pointers (synchronous). */
int mv_trajectory_chain_host(mv_context *ctx, int len, const double *rel, const int *present, const double *start,
                             int mode, double *poses);

/* Pose I/O (host code, no device).  np.savetxt(pose[:3, :], fmt='%.6f'): three lines of
 * four values (compute_trajectory.py:49-51). */
int mv_write_pose_txt(const char *path, const double *pose12);
/* write_ply (compute_trajectory.py:6-43): ASCII PLY, n vertices (x y z with Python's
 * shortest round-trip float repr, colour red / blue ... / black) and n - 1 edges i -> i+1. */
int mv_write_trajectory_ply(const char *path, int n, const double *xyz);
/* A (3, 4) float64 .npy (np.save of transform_*.npy, little-endian '<f8', C order).
 * MV_ERR_IO when the file is missing or not such an array. */
int mv_read_transform_npy(const char *path, double *T12);
/* compute_trajectory.py main(start, end, pose_dir, out_dir) with the chain on the GPU:
 * reads pose_dir/transform_%06d_%06d.npy for i in [start, end) (missing ones skipped),
 * writes out_dir/frame-%06d.pose.txt for start and every frame reached, and
 * out_dir/trajectory_%06d_%06d.ply.  *num_poses (may be NULL) = poses written. */
int mv_compute_trajectory(mv_context *ctx, int start_frame, int end_frame, const char *pose_dir,
                          const char *out_dir, int mode, int *num_poses);

#ifdef __cplusplus
}
#endif
#endif
