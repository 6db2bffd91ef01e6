/*
 * ref_window_harness.c -- the reference's own squared_dist (src/tracking_main.c:18-43) and its
 * window score expression (tracking_main.c:154, MATCH_THRESHOLD of :12), exported for the
 * oracle-pinning tests.  tracking_main.c as a whole does not build (it includes the unshipped
 * quantized_pair0.h), so oracle/Makefile extracts those self-contained pieces from
 * the reference text at build time into oracle/_ref/ (git-ignored; nothing is committed) and this
 * harness includes them.  No stand-in header is written.  Built at -O0 like the reference's
 * CMake default (no flags), so the int products wrap as the as-built binary's do.
 */
#include <stdint.h>

#include "tm_match_threshold.inc" /* tracking_main.c:12: #define MATCH_THRESHOLD 0.9 */
#include "tm_squared_dist.inc"    /* tracking_main.c:18-43: void squared_dist(...) { ... } */

void ref_squared_dist(const int8_t *desc1, const int8_t *desc2, int *sum, int *norm1_squared, int *norm2_squared) {
    squared_dist(desc1, desc2, sum, norm1_squared, norm2_squared);
}

float ref_window_score(int dot_product, int norm1_squared, int norm2_squared) {
#include "tm_score.inc" /* tracking_main.c:154: float dist_squared = ...; */
    return dist_squared;
}

int ref_window_pass(float dist_squared) { return dist_squared > (MATCH_THRESHOLD * MATCH_THRESHOLD); }
