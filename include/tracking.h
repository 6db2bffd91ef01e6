/*
 * tracking.h -- a compilable form of the reference's include/tracking.h:3-54.
 *
 * The reference header is pseudocode (nullptr, incomplete arrays, undefined
 * Transform).  Its intent -- match the features of `last_frame` inside a
 * shifted window of `current_frame`, then estimate the relative pose -- is
 * what src/tracking_main.c:84-228 actually does inline.  track() runs exactly
 * that pipeline on the GPU:
 *   softmax(last) -> top-N(current) -> windowed int8 match -> RANSAC(E) -> pose
 * with tracking_main.c's constants (N=100, 150 matches, K of :205-207,
 * 10 iterations, inlier threshold 1.1) and window
 *   x0 in [gx + x_shift - r, gx + x_shift + r],  r = (window_size - 1) / 2
 * (tracking_main.c:104-106,127-130 is x_shift = y_shift = 4, window_size = 9).
 * `threshold` is the cosine threshold (MATCH_THRESHOLD 0.9, tracking_main.c:12);
 * it is squared in double from the shortest decimal that round-trips the float
 * (0.9f -> 0.9 -> 0.81 exactly as the reference's double constant).
 * transform = [R1 | t] of recover_pose_from_essential_matrix.
 */
#ifndef MV_TRACKING_H
#define MV_TRACKING_H
#include "frame.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float m[3][4]; /* [R | t], row-major */
} Transform;

/* Returns 0 on success, a negative mv_status on failure (transform = identity). */
int track(const Frame *last_frame, const Frame *current_frame, const int x_shift, const int y_shift,
          const int window_size, const float threshold, Transform *transform);

#ifdef __cplusplus
}
#endif
#endif
