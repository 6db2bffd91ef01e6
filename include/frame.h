/*
 * frame.h -- drop-in for the reference's include/frame.h:7-47.
 *
 * Same struct layout and the same frame_create() signature.  Differences:
 *   - frame_create is `static inline` (the reference defines it non-static in
 *     the header, which breaks as soon as two translation units include it);
 *   - descriptor.h is not pulled in (its only symbol, descriptor_distance, is
 *     unused by the tracking path: include/descriptor.h:9-15).
 * Frames BORROW their semi/desc memory (host pointers, never freed here).
 */
#ifndef MV_FRAME_H
#define MV_FRAME_H
#include <stdint.h>

#define CELL_SIZE 8

typedef struct {
    int rows;     /* H (pixels) */
    int cols;     /* W (pixels) */
    int channels;
    const char *data;

    int num_features;
    int feature_rows; /* H / 8 : grid rows  (24 at 192x640) */
    int feature_cols; /* W / 8 : grid cols  (80 at 192x640) */
    const int *feature_xs;
    const int *feature_ys;

    float semi_scale;
    const int8_t *semi; /* [feature_rows*feature_cols][65], cell p = gx*rows + gy */
    float desc_scale;
    const int8_t *desc; /* [feature_rows*feature_cols][256] */
} Frame;

static inline void frame_create(const int rows, const int cols, const int channels, const char *data,
                                const int feature_rows, const int feature_cols, const float semi_scale,
                                const int8_t *semi, const float desc_scale, const int8_t *desc, Frame *frame) {
    frame->rows = rows;
    frame->cols = cols;
    frame->channels = channels;
    frame->data = data;
    frame->num_features = 0;
    frame->feature_rows = feature_rows;
    frame->feature_cols = feature_cols;
    frame->feature_xs = 0;
    frame->feature_ys = 0;
    frame->semi_scale = semi_scale;
    frame->semi = semi;
    frame->desc_scale = desc_scale;
    frame->desc = desc;
}
#endif
