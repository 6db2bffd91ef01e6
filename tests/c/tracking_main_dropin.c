/*
 * A C caller shaped like the reference's src/tracking_main.c:68-228, linked against
 * libmaveric_hip.so instead of src/top_N.c + src/pnp_solver.c (tests/test_dropin_c.py).
 *
 * Like tracking_main.c it does NOT include top_N.h: compute_softmax and compute_top_N are
 * implicitly declared (gcc: -Wimplicit-function-declaration), so the true float scale is
 * promoted to double at the call and the callee reads the low 32 bits of that double (SURVEY
 * F7: 0.0 for the committed frame's scale).  pnp_solver.h IS included, as in the reference.
 * The inline window loop of tracking_main.c:103-194 is replaced by the library's
 * mv_window_match_host (the batched seam; as-built semantics).
 *
 * Input (argv[1]): the frame written by the test -- int32 rows, cols, float semi_scale,
 * int8 semi[cells][65], int8 desc[cells][256]; the pair is (frame, frame), the reference's
 * self pair.  Output (argv[2]): every intermediate, for a bit-for-bit comparison.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "frame.h"
#include "maveric_hip.h"
#include "pnp_solver.h"

#define TOP_N 100
#define MAX_NUM_MATCH 150

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *in = fopen(argv[1], "rb");
    if (!in) return 2;
    int rows, cols;
    float scale;
    if (fread(&rows, 4, 1, in) != 1 || fread(&cols, 4, 1, in) != 1 || fread(&scale, 4, 1, in) != 1) return 2;
    const int cells = rows * cols;
    int8_t(*semi)[65] = malloc((size_t)cells * 65);
    int8_t(*desc)[256] = malloc((size_t)cells * 256);
    if (fread(semi, 65, cells, in) != (size_t)cells || fread(desc, 256, cells, in) != (size_t)cells) return 2;
    fclose(in);

    srand(0);  /* the rand() stream ransac_essential_matrix draws from (tracking_main.c:69) */
    Frame f0, f1;
    frame_create(rows * 8, cols * 8, 1, NULL, rows, cols, scale, (int8_t *)semi, 1.0f, (int8_t *)desc, &f0);
    frame_create(rows * 8, cols * 8, 1, NULL, rows, cols, scale, (int8_t *)semi, 1.0f, (int8_t *)desc, &f1);

    /* frame 0: softmax of every cell; frame 1: top-N -- no prototypes in scope (F7) */
    int num_valid0 = 0;
    int *max_indices0 = calloc(cells, sizeof(int));
    float *probs0 = calloc(cells, sizeof(float));
    compute_softmax(f0.semi_scale, f0.semi, &num_valid0, max_indices0, probs0);
    int num_selected1 = 0, patches1[TOP_N], indices1[TOP_N];
    float probs1[TOP_N];
    compute_top_N(f1.semi_scale, f1.semi, TOP_N, &num_selected1, patches1, indices1, probs1);
    if (num_selected1 < 0) return 3;

    /* the window match (the seam replacing tracking_main.c:103-194) */
    mv_window_params wp;
    mv_window_params_default(&wp);
    wp.semantics = MV_AS_BUILT;
    int num_matches = 0, query[MAX_NUM_MATCH];
    float points1[MAX_NUM_MATCH][2], points2[MAX_NUM_MATCH][2];
    if (mv_window_match_host(mv_default_context(), &wp, rows, cols, (const int8_t *)f0.desc, max_indices0, probs0,
                             (const int8_t *)f1.desc, num_selected1, patches1, indices1, &num_matches,
                             &points1[0][0], &points2[0][0], query) != MV_OK)
        return 4;

    /* RANSAC + pose (tracking_main.c:200-218); best_inliers sized for every point (the
     * reference passes int[10] and overruns it) */
    const float K[3][3] = {{517.306408f, 0.0f, 318.643040f}, {0.0f, 516.469215f, 255.313989f}, {0.0f, 0.0f, 1.0f}};
    float best_E[3][3], R1[3][3], R2[3][3], t[3];
    int best_inliers[1000], num_inliers = 0;
    ransac_essential_matrix(num_matches, (const float(*)[2])points1, (const float(*)[2])points2, K, 10, 1.1f,
                            best_E, best_inliers, &num_inliers);
    recover_pose_from_essential_matrix(best_E, R1, R2, t);

    FILE *out = fopen(argv[2], "wb");
    if (!out) return 2;
    fwrite(&num_valid0, 4, 1, out);
    fwrite(max_indices0, 4, cells, out);
    fwrite(probs0, 4, cells, out);
    fwrite(&num_selected1, 4, 1, out);
    fwrite(patches1, 4, TOP_N, out);
    fwrite(indices1, 4, TOP_N, out);
    fwrite(probs1, 4, TOP_N, out);
    fwrite(&num_matches, 4, 1, out);
    fwrite(points1, 8, MAX_NUM_MATCH, out);
    fwrite(points2, 8, MAX_NUM_MATCH, out);
    fwrite(R1, 4, 9, out);
    fwrite(R2, 4, 9, out);
    fwrite(t, 4, 3, out);
    fwrite(&num_inliers, 4, 1, out);
    fclose(out);
    printf("tracking_main_dropin: %d valid, %d selected, %d matches\n", num_valid0, num_selected1, num_matches);
    return 0;
}
