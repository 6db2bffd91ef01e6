/*
 * pnp_solver.h -- drop-in for the reference's include/pnp_solver.h:3-22
 * (src/pnp_solver.c).  Identical prototypes and results (bit-exact):
 *   - compute_essential_matrix is the reference's stub: E = I (pnp_solver.c:80-85);
 *   - ransac_essential_matrix draws its 8 samples per iteration with libc rand()
 *     exactly as the reference (the caller's rand() stream advances identically),
 *     and writes num_inliers indices into best_inliers (callers must size it;
 *     tracking_main.c:201 passes int[10], which the reference overruns);
 *   - recover_pose_from_essential_matrix uses the McAdams 3x3 SVD of svd.h on
 *     the GPU: R1 = U W, R2 = U W^T, t = U[:,2].
 * Differences: no printf from the SVD (pnp_solver.c:10-12); num_points <= 0
 * leaves the outputs untouched instead of dividing by zero (pnp_solver.c:123).
 * The real essential-matrix solver is in maveric_hip.h (mv_pose_batch_dev).
 */
#ifndef MV_PNP_SOLVER_H
#define MV_PNP_SOLVER_H
#ifdef __cplusplus
extern "C" {
#endif

void normalize_points(const int num_points, const float points[][2], const float K[3][3],
                      float normalized_points[][2]);

void compute_essential_matrix(const int num_points, const float pts1_norm[][2], const float pts2_norm[][2],
                              float E[3][3]);

float compute_reprojection_error(const float point1[2], const float point2[2], const float E[3][3]);

void ransac_essential_matrix(const int num_points, const float points1[][2], const float points2[][2],
                             const float K[3][3], const int num_iterations, const float inlier_threshold,
                             float best_E[3][3], int *best_inliers, int *num_inliers);

void recover_pose_from_essential_matrix(float E[3][3], float R1[3][3], float R2[3][3], float t[3]);

#ifdef __cplusplus
}
#endif
#endif
