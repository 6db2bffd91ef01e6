/*
 * top_N.c -- drop-in for the reference's src/top_N.c (include/top_N.h:8-13).
 * Host C: marshals one frame to the GPU (k_softmax / k_top_n_select in
 * csrc/hip/k_frontend.hip) through the C ABI of maveric_hip.h.
 * No CPU compute path exists: without a gfx950 device the calls report the
 * failure on stderr, set the outputs to sentinels and mv_last_status().
 */
#include <stdio.h>

#include "maveric_hip.h"
#include "top_N.h"

#define MV_REF_CELLS 1920     /* 24 x 80, the loop bound of top_N.c:73,151 */
#define MV_REF_VALID_CAP 1000 /* MAX_VALID_FEATURES, top_N.c:51 */

void compute_top_N(float scale, int8_t semi[2400][65], int N, int *num_selected, int *N_patches, int *N_indices,
                   float *N_probs) {
    mv_context *ctx = mv_default_context();
    if (!ctx) {
        *num_selected = -1;
        return;
    }
    int st = mv_top_n_host(ctx, scale, &semi[0][0], MV_REF_CELLS, N, MV_REF_VALID_CAP, num_selected, N_patches,
                           N_indices, N_probs);
    if (st != MV_OK) {
        fprintf(stderr, "compute_top_N: %s (%s)\n", mv_status_string(st), mv_last_error_message());
        *num_selected = -1;
    }
}

void compute_softmax(float scale, int8_t semi[2400][65], int *num_valid, int *max_indices, float *probs) {
    mv_context *ctx = mv_default_context();
    if (!ctx) return;
    int nv = 0;
    int st = mv_softmax_host(ctx, scale, &semi[0][0], MV_REF_CELLS, &nv, max_indices, probs);
    if (st != MV_OK) {
        fprintf(stderr, "compute_softmax: %s (%s)\n", mv_status_string(st), mv_last_error_message());
        return;
    }
    *num_valid += nv; /* the reference increments the caller's counter (top_N.c:159) */
}
