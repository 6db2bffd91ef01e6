/*
 * ref_nms_harness.c -- the reference's own cell-level NMS (src/run_nms.c:43-175, the body of
 * its main) and grid helpers (:29-41), exported for the oracle-pinning tests.  run_nms.c as a
 * whole does not build (it includes the unshipped quantized_pair0.h), so
 * oracle/Makefile cuts the helpers and main's body out of the reference text at build time into
 * oracle/_ref/ (git-ignored; nothing is committed) and this harness includes them.  No stand-in
 * header is written: the names main reads from quantized_pair0.h (image1_rows ... image1_desc)
 * are the parameters of ref_run_nms, and the caller supplies the frame.  frame.h and
 * pnp_solver.h are the reference's own headers; top_N.c is linked from its source.
 *
 * As in the reference binary, compute_softmax is called WITHOUT a prototype (run_nms.c includes
 * neither top_N.h nor a declaration), so the float semi_scale is promoted to double and the
 * callee reads the low 32 bits of that double -- reproduced here by construction.
 * main's printf lines ("(x y) suppressing (x y)" and the surviving "x y" pixels) are collected
 * into the caller's buffer.
 */
#include <stdarg.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "frame.h"
#include "pnp_solver.h"

static char *nms_out;
static int nms_len, nms_cap, nms_overflow;

static int nms_printf(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int room = nms_cap - nms_len;
    const int n = vsnprintf(nms_out + nms_len, room > 0 ? (size_t)room : 0, fmt, ap);
    va_end(ap);
    if (n >= room) {
        nms_overflow = 1;
        nms_len = nms_cap;
    } else {
        nms_len += n;
    }
    return n;
}
#define printf nms_printf

#include "rn_helpers.inc" /* run_nms.c:29-41: patch_to_grid, grid_to_patch, patch_index_to_patch_coords */

static void ref_nms_main(const int image1_rows, const int image1_cols, const int image1_channels,
                         const int image1_feature_rows, const int image1_feature_cols,
                         const float image1_semi_scale, const int8_t image1_semi[1920][65],
                         const float image1_desc_scale, const int8_t image1_desc[1920][256]) {
#include "rn_main_body.inc" /* run_nms.c:44-174: main's body */
}

/* Returns the number of bytes written to out (NUL-terminated), or -1 if out was too small. */
int ref_run_nms(int rows, int cols, int feature_rows, int feature_cols, float semi_scale, const int8_t *semi,
                float desc_scale, const int8_t *desc, char *out, int out_cap) {
    nms_out = out;
    nms_len = 0;
    nms_cap = out_cap - 1;
    nms_overflow = 0;
    ref_nms_main(rows, cols, 1, feature_rows, feature_cols, semi_scale, (const int8_t(*)[65])semi, desc_scale,
                 (const int8_t(*)[256])desc);
    out[nms_len] = 0;
    return nms_overflow ? -1 : nms_len;
}
