/*
 * ref_track_harness.c -- the reference's own tracking driver, src/tracking_main.c:68-228 (the
 * body of its main: softmax of frame 0, top-N of frame 1, the windowed match :103-194, the RANSAC
 * and the pose), run on frames the caller supplies.  TEST INFRASTRUCTURE (oracle-pinning tests,
 * the golden-fixture script and bench.py's cpu_c0 leg), built into oracle/_ref only where
 * /root/reference is present.
 *
 * tracking_main.c as a whole does not build: it includes quantized_pair0.h, which the reference
 * does not ship.  No stand-in header is written.  oracle/Makefile cuts main's helpers
 * (:9-66: MAX/MIN, MATCH_THRESHOLD, MAX_NUM_MATCH, N, squared_dist, check_dist, patch_to_grid,
 * grid_to_patch) and the body of main (:69-230) out of the reference text at build time into
 * oracle/_ref/ (git-ignored) and this file includes them; the names main reads from
 * quantized_pair0.h (image0_rows ... image1_desc) are the parameters of ref_tm_main.
 *
 * Linked beside it, from the reference's sources:
 *   src/top_N.c       compute_softmax / compute_top_N, reached WITHOUT a prototype as in the
 *                     reference binary (the float scale is promoted to double and the callee reads
 *                     its low 32 bits).  Built with -DMV_REF_TRUE_SCALE, this file
 *                     includes top_N.h before main's body, so the true scale arrives instead
 *                     (libmv_ref_track_ts.so).  Its exit(1) on >= 1000 valid cells (:91-94) is
 *                     renamed at compile time to ref_tm_exit, which returns to the caller.
 *   src/pnp_solver.c  + include/svd/svd.h, with ransac_essential_matrix and
 *                     recover_pose_from_essential_matrix renamed at compile time: main's calls
 *                     reach the capturing wrappers below, which call the reference's functions.
 *                     The wrapper gives the RANSAC a 1000-entry inlier buffer and copies the first
 *                     ten into main's best_inliers[10] (main passes int[10], the RANSAC writes one
 *                     entry per inlier: a stack overrun in the reference binary, undefined
 *                     behaviour that is not reproduced).  When no hypothesis has an inlier the
 *                     RANSAC writes neither E nor the count (main then reads uninitialised stack):
 *                     the wrapper pre-sets them to NaN / -1 so that case is visible.  n == 0 matches (the reference's
 *                     rand() % 0) returns to the caller with status 2 before the RANSAC runs.
 * main's printf lines and call_svd's are discarded.  -O0 like the reference's CMake default.
 */
#include <math.h>
#include <setjmp.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "frame.h"
#include "pnp_solver.h"
#ifdef MV_REF_TRUE_SCALE
#include "top_N.h"
#endif

int ref_tm_quiet_printf(const char *fmt, ...) {
    (void)fmt;
    return 0;
}
#define printf ref_tm_quiet_printf

static jmp_buf tm_env;

__attribute__((noreturn)) void ref_tm_exit(int code) {
    (void)code;
    longjmp(tm_env, 1);
}

/* the reference's functions under their compile-time names (pnp_solver.c built with -D renames) */
void ref_pnp_ransac_essential_matrix(const int num_points, const float points1[][2], const float points2[][2],
                                     const float K[3][3], const int num_iterations, const float inlier_threshold,
                                     float best_E[3][3], int *best_inliers, int *num_inliers);
void ref_pnp_recover_pose_from_essential_matrix(float E[3][3], float R1[3][3], float R2[3][3], float t[3]);

#define CAP_POINTS 1000
static struct {
    int n;
    float points1[CAP_POINTS][2], points2[CAP_POINTS][2];
    float K[9];
    int iterations;
    float thresh;
    float E[9];
    int inliers[CAP_POINTS], num_inliers;
    float R1[9], R2[9], t[3];
} cap;

void ransac_essential_matrix(const int num_points, const float points1[][2], const float points2[][2],
                             const float K[3][3], const int num_iterations, const float inlier_threshold,
                             float best_E[3][3], int *best_inliers, int *num_inliers) {
    cap.n = num_points;
    if (num_points > 0 && num_points <= CAP_POINTS) {
        memcpy(cap.points1, points1, sizeof(float) * 2 * (size_t)num_points);
        memcpy(cap.points2, points2, sizeof(float) * 2 * (size_t)num_points);
    }
    memcpy(cap.K, K, sizeof cap.K);
    cap.iterations = num_iterations;
    cap.thresh = inlier_threshold;
    if (num_points <= 0) longjmp(tm_env, 2); /* the reference divides by zero (pnp_solver.c:123) */
    static int all[CAP_POINTS];
    /* main's num_inliers and best_E are uninitialised stack, written only when a hypothesis has
     * more than zero inliers (pnp_solver.c:152-159): "never written" is made visible as -1 / NaN */
    *num_inliers = -1;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) best_E[i][j] = NAN;
    ref_pnp_ransac_essential_matrix(num_points, points1, points2, K, num_iterations, inlier_threshold, best_E, all,
                                    num_inliers);
    memcpy(cap.E, best_E, sizeof cap.E);
    cap.num_inliers = *num_inliers;
    memcpy(cap.inliers, all, sizeof all);
    for (int i = 0; i < 10 && i < *num_inliers; ++i) best_inliers[i] = all[i];
}

void recover_pose_from_essential_matrix(float E[3][3], float R1[3][3], float R2[3][3], float t[3]) {
    ref_pnp_recover_pose_from_essential_matrix(E, R1, R2, t);
    memcpy(cap.R1, R1, sizeof cap.R1);
    memcpy(cap.R2, R2, sizeof cap.R2);
    memcpy(cap.t, t, sizeof cap.t);
}

#include "tm_helpers.inc" /* tracking_main.c:9-66 */

static int ref_tm_main(const int image0_rows, const int image0_cols, const int image0_channels,
                       const int image0_feature_rows, const int image0_feature_cols, const float image0_semi_scale,
                       const int8_t *image0_semi, const float image0_desc_scale, const int8_t *image0_desc,
                       const int image1_rows, const int image1_cols, const int image1_channels,
                       const int image1_feature_rows, const int image1_feature_cols, const float image1_semi_scale,
                       const int8_t *image1_semi, const float image1_desc_scale, const int8_t *image1_desc) {
#include "tm_main_body.inc" /* tracking_main.c:69-230: main's body */
}

/* One run of main on the frame pair (24 x 80 cells: main's arrays are [1920]).  Returns 0, 1 (top_N.c
 * exit(1): >= 1000 valid cells) or 2 (no matches: the reference's rand() % 0).  Outputs: the match
 * list main hands to the RANSAC (n, points1 = frame-0 pixels, points2 = frame-1 pixels), the
 * RANSAC's E, inliers and count, and the pose. */
int ref_tracking_main(int rows, int cols, int feature_rows, int feature_cols, float semi_scale0, const int8_t *semi0,
                      const int8_t *desc0, float semi_scale1, const int8_t *semi1, const int8_t *desc1, int *n,
                      float *points1, float *points2, float *E, int *inliers, int *num_inliers, float *R1, float *R2,
                      float *t) {
    memset(&cap, 0, sizeof cap);
    int st = setjmp(tm_env);
    if (st == 0) ref_tm_main(rows, cols, 1, feature_rows, feature_cols, semi_scale0, semi0, 1.0f, desc0, rows, cols, 1,
                             feature_rows, feature_cols, semi_scale1, semi1, 1.0f, desc1);
    *n = cap.n;
    if (cap.n > 0 && cap.n <= CAP_POINTS) {
        memcpy(points1, cap.points1, sizeof(float) * 2 * (size_t)cap.n);
        memcpy(points2, cap.points2, sizeof(float) * 2 * (size_t)cap.n);
    }
    memcpy(E, cap.E, sizeof cap.E);
    *num_inliers = cap.num_inliers;
    memcpy(inliers, cap.inliers, sizeof(int) * (size_t)(cap.num_inliers > 0 ? cap.num_inliers : 0));
    memcpy(R1, cap.R1, sizeof cap.R1);
    memcpy(R2, cap.R2, sizeof cap.R2);
    memcpy(t, cap.t, sizeof cap.t);
    return st;
}
