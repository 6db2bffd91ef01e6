/*
 * pnp_solver.c -- drop-in for the reference's src/pnp_solver.c
 * (include/pnp_solver.h:3-22), bit-exact with it.
 *
 * normalize_points and compute_reprojection_error are O(1)-per-point helpers
 * with a scalar return; they are evaluated here in the reference's exact
 * float order (this file is built with -ffp-contract=off).  The O(n) RANSAC
 * inlier scan and the SVD-based pose recovery run as HIP kernels
 * (csrc/hip/k_pose.hip).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "maveric_hip.h"
#include "pnp_solver.h"

void normalize_points(const int num_points, const float points[][2], const float K[3][3],
                      float normalized_points[][2]) {
    for (int i = 0; i < num_points; ++i) { /* pnp_solver.c:28-34 */
        normalized_points[i][0] = (points[i][0] - K[0][2]) / K[0][0];
        normalized_points[i][1] = (points[i][1] - K[1][2]) / K[1][1];
    }
}

void compute_essential_matrix(const int num_points, const float pts1_norm[][2], const float pts2_norm[][2],
                              float E[3][3]) {
    /* The reference builds the 8x9 design matrix, never solves it and returns
     * E = I (pnp_solver.c:55-56,80-85).  The real solver is mv_pose_batch_dev. */
    (void)num_points;
    (void)pts1_norm;
    (void)pts2_norm;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) E[i][j] = i == j ? 1.0f : 0.0f;
}

float compute_reprojection_error(const float point1[2], const float point2[2], const float E[3][3]) {
    const float h1[3] = {point1[0], point1[1], 1.0f}; /* pnp_solver.c:89-105 */
    const float h2[3] = {point2[0], point2[1], 1.0f};
    float err = 0;
    for (int i = 0; i < 3; ++i) {
        float v = E[i][0] * h1[0] + E[i][1] * h1[1] + E[i][2] * h1[2];
        float d = v - h2[i];
        err += d * d;
    }
    return err;
}

void ransac_essential_matrix(const int num_points, const float points1[][2], const float points2[][2],
                             const float K[3][3], const int num_iterations, const float inlier_threshold,
                             float best_E[3][3], int *best_inliers, int *num_inliers) {
    (void)K;
    if (num_points <= 0) return; /* the reference evaluates rand() % 0 here (pnp_solver.c:123) */
    /* 8 samples per iteration from the caller's rand() stream (pnp_solver.c:121-124) */
    for (int it = 0; it < num_iterations; ++it)
        for (int s = 0; s < 8; ++s) (void)(rand() % num_points);
    if (num_iterations <= 0) return;
    mv_context *ctx = mv_default_context();
    if (!ctx) return;
    /* Every iteration evaluates the same E = I, so the first iteration's
     * inlier list is the one kept (pnp_solver.c:152-163). */
    float E[9];
    int cnt = 0;
    int st = mv_ransac_stub_host(ctx, num_points, &points1[0][0], &points2[0][0], inlier_threshold, E, best_inliers,
                                 &cnt);
    if (st != MV_OK) {
        fprintf(stderr, "ransac_essential_matrix: %s (%s)\n", mv_status_string(st), mv_last_error_message());
        return;
    }
    if (cnt > 0) {
        *num_inliers = cnt;
        memcpy(best_E, E, sizeof E);
    }
}

void recover_pose_from_essential_matrix(float E[3][3], float R1[3][3], float R2[3][3], float t[3]) {
    mv_context *ctx = mv_default_context();
    if (!ctx) return;
    int st = mv_recover_pose_host(ctx, &E[0][0], &R1[0][0], &R2[0][0], t);
    if (st != MV_OK)
        fprintf(stderr, "recover_pose_from_essential_matrix: %s (%s)\n", mv_status_string(st),
                mv_last_error_message());
}
