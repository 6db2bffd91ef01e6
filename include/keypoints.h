/*
 * keypoints.h -- keypoint extraction + descriptor sampling: the step before
 * the fp32 all-pairs match, SuperPointFrontend.run after the network forward
 * (python/pairwise_pnp.py:197-257) with nms_fast (:116-179):
 *   softmax over the 65 cell channels -> 8x8 heatmap per cell -> pixels >= conf_thresh ->
 *   greedy NMS in descending confidence ((2 nms_dist + 1)^2 window) -> descending order ->
 *   border removal -> bilinear grid_sample of the coarse descriptors -> L2 normalise.
 * The outputs are laid out for mv_match_allpairs_f32_dev (kp [B][cap][2], desc [B][cap][256]).
 *
 * Numerics: float32 everywhere as in the reference; exp is the correctly rounded float32 exp
 * (numpy's SIMD expf is within a few ulp of it, so confidences may differ from a numpy run by
 * ulps; the keypoints and descriptors do not -- tests/test_keypoints.py).  Exact ties in
 * confidence: NMS visits them in row-major pixel order, the output lists them in reversed
 * row-major order (what the reference's two numpy argsorts produce; numpy does not promise it).
 */
#ifndef MV_KEYPOINTS_H
#define MV_KEYPOINTS_H
#include "maveric_hip.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float conf_thresh; /* 0.015 (pairwise_pnp.py:591) */
    int nms_dist;      /* 4 (:589) */
    int border;        /* 4 (border_remove, :99) */
} mv_kp_params;
void mv_kp_params_default(mv_kp_params *p);

/* batch frames of network outputs: semi [B][65][Hc][Wc], coarse_desc [B][256][Hc][Wc]
 * (NCHW float32), image size H x W (Hc = H / 8, Wc = W / 8 as in run()).
 * Outputs per frame b: num_kp[b] keypoints (at most cap: the cap most confident, a prefix of
 * the reference's list; status[b] = MV_ERR_CAPACITY when more survived), kp [B][cap][2]
 * (x, y pixels), conf [B][cap], desc [B][cap][256] unit rows.  heat (may be NULL):
 * [B][Hc*8][Wc*8] heatmap.  Rows past num_kp are not written.  Alignment: coarse_desc 4 B,
 * desc and heat 16 B (MV_ERR_INVALID_ARG otherwise). */
int mv_keypoints_dev(mv_context *ctx, const mv_kp_params *p, int batch, int Hc, int Wc, int H, int W,
                     const float *semi, const float *coarse_desc, int cap, int *num_kp, float *kp, float *conf,
                     float *desc, float *heat, int *status);
/* One frame, host pointers (synchronous); kp [cap][2], conf [cap], desc [cap][256]. */
int mv_keypoints_host(mv_context *ctx, const mv_kp_params *p, int Hc, int Wc, int H, int W, const float *semi,
                      const float *coarse_desc, int cap, int *num_kp, float *kp, float *conf, float *desc);

#ifdef __cplusplus
}
#endif
#endif
