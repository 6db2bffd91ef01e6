/*
 * tracking.c -- a compilable track() (include/tracking.h; the reference's
 * include/tracking.h:3-54 is pseudocode).  Runs the pipeline of
 * src/tracking_main.c:84-228 on the GPU through mv_track_pair_host().
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "maveric_hip.h"
#include "tracking.h"

/* shortest decimal that round-trips the float, read back as a double */
static double float_as_decimal(float f) {
    char buf[32];
    for (int prec = 1; prec <= 9; ++prec) {
        snprintf(buf, sizeof buf, "%.*g", prec, (double)f);
        if (strtof(buf, NULL) == f) return strtod(buf, NULL);
    }
    return (double)f;
}

static void identity(Transform *T) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) T->m[i][j] = (i == j) ? 1.0f : 0.0f;
}

int track(const Frame *last_frame, const Frame *current_frame, const int x_shift, const int y_shift,
          const int window_size, const float threshold, Transform *transform) {
    if (!transform) return MV_ERR_INVALID_ARG;
    identity(transform);
    if (!last_frame || !current_frame) return MV_OK;
    if (last_frame->feature_rows != current_frame->feature_rows ||
        last_frame->feature_cols != current_frame->feature_cols || window_size < 1)
        return MV_ERR_INVALID_ARG;
    mv_context *ctx = mv_default_context();
    if (!ctx) return MV_ERR_NO_DEVICE;
    mv_track_params p;
    mv_track_params_default(&p, MV_AS_BUILT);
    p.window.shift_x = x_shift;
    p.window.shift_y = y_shift;
    p.window.radius = (window_size - 1) / 2;
    const double thr = float_as_decimal(threshold);
    p.window.match_thresh_sq = thr * thr;
    /* tracking_main.c runs 10 RANSAC iterations of 8 rand() draws each */
    float p1[150][2], p2[150][2];
    int nm = 0;
    int st = mv_track_pair_host(ctx, &p, last_frame->feature_rows, last_frame->feature_cols,
                                last_frame->semi_scale, last_frame->semi, last_frame->desc,
                                current_frame->semi_scale, current_frame->semi, current_frame->desc,
                                &transform->m[0][0], &nm, &p1[0][0], &p2[0][0]);
    if (nm > 0)
        for (int i = 0; i < 10 * 8; ++i) (void)(rand() % nm);
    if (st != MV_OK && st != MV_ERR_DEGENERATE && st != MV_ERR_NO_POINTS) {
        identity(transform);
        return st;
    }
    return MV_OK;
}
