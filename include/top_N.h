/*
 * top_N.h -- drop-in for the reference's include/top_N.h:8-13 (src/top_N.c).
 * Identical prototypes.  The work runs in HIP kernels (libmaveric_hip.so).
 *
 * As in the reference the grid is 1920 cells (24x80); the array bound in the
 * prototype is only a row-stride carrier (the reference header says 2400, the
 * implementation 1920).  Use mv_top_n_host()/mv_softmax_host() in
 * maveric_hip.h for other grid sizes.
 *
 * ABI note: a caller that calls these WITHOUT this prototype in
 * scope (as src/tracking_main.c does) passes `scale` as a double; the callee
 * then sees the low 32 bits of that double.  This library reproduces that
 * behaviour automatically because it is a property of the calling convention.
 *
 * Error behaviour: the reference calls exit(1) when 1000 cells pass the
 * validity filter (src/top_N.c:91-94).  This library never exits: it sets
 * *num_selected = -1 and mv_last_status() returns MV_ERR_CAPACITY.
 */
#ifndef MV_TOP_N_H
#define MV_TOP_N_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

void compute_top_N(float scale, int8_t semi[2400][65], int N, int *num_selected, int *N_patches, int *N_indices,
                   float *N_probs);

void compute_softmax(float scale, int8_t semi[2400][65], int *num_valid, int *max_indices, float *probs);

#ifdef __cplusplus
}
#endif
#endif
