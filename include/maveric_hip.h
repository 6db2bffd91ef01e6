/*
 * maveric_hip.h -- the C ABI of libmaveric_hip.so (MI355X / gfx950).
 *
 * Two layers:
 *   1. The reference's own API, unchanged (frame.h, top_N.h, pnp_solver.h,
 *      tracking.h).  Those entry points run on a lazily created default
 *      context (device 0) with host pointers, synchronously.
 *   2. This header: an explicit context, a stream, and BATCHED entry points
 *      over device pointers for throughput mode (many independent frame-pairs
 *      per launch).  All *_dev functions are stream-ordered and asynchronous.
 *      The all-pairs match (fp32, int8) and pose *_dev calls never allocate
 *      once mv_context_reserve() has covered (batch, cap), so they can be
 *      captured in a hipGraph; the window, keypoint and two-way calls size
 *      their scratch on first use: run each once at its largest shape before
 *      capturing it.
 *
 * Threading: a mv_context is NOT thread-safe -- give each host thread its own
 * (or serialise the calls).  The default context behind the reference's API
 * is per thread: every thread that calls compute_top_N, ransac_essential_matrix,
 * track(), ... gets its own context (device 0, own stream and buffers), created
 * on first use and destroyed when that thread exits.  mv_last_status() is
 * per thread as well.
 *
 * Conventions: plain C types only; every function returns an mv_status
 * (0 = success, negative = error) unless documented otherwise; nothing ever
 * calls exit().  Device arrays are row-major, batch-major:
 *   semi  [B][cells][65]  int8      desc  [B][cells][256] int8   (cell p = gx*rows + gy)
 *   fdesc [B][cap][256]   float     kp    [B][cap][2]     float (x, y pixels)
 *   T     [B][3][4]       float     ([R | t], x1 ~ R x0 + t, |t| = 1)
 */
#ifndef MV_MAVERIC_HIP_H
#define MV_MAVERIC_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MV_VERSION 100

typedef enum {
    MV_OK = 0,
    MV_ERR_INVALID_ARG = -1,
    MV_ERR_CAPACITY = -2,    /* a validity filter passed `cap` cells (reference: exit(1)) */
    MV_ERR_HIP = -3,         /* a HIP runtime call failed (mv_last_error_message()) */
    MV_ERR_NO_DEVICE = -4,   /* no usable gfx950 device: the library never falls back to the CPU */
    MV_ERR_NO_POINTS = -5,   /* pose requested on an empty correspondence set */
    MV_ERR_OUT_OF_MEMORY = -6,
    MV_ERR_DEGENERATE = -7,  /* pose: no hypothesis with enough support */
    MV_ERR_IO = -8           /* a file could not be read or written (trajectory.h) */
} mv_status;

typedef enum {
    MV_AS_BUILT = 0,   /* the reference exactly as it runs: F7 scale, stale-norm/64-dim/int32-wrap match, E = I */
    MV_AS_INTENDED = 1 /* true scale, exact cosine, real essential-matrix RANSAC + Gauss-Newton */
} mv_semantics;

typedef struct mv_context mv_context;

int mv_version(void);
const char *mv_status_string(int status);
int mv_last_status(void);               /* thread-local status of the last drop-in (void) call */
const char *mv_last_error_message(void);
int mv_device_count(void);              /* 0 when no HIP device is visible */

int mv_context_create(int device, mv_context **out);
int mv_context_destroy(mv_context *ctx);
/* Every later call runs on `hip_stream`; NULL is HIP's null (legacy default) stream, which is
 * what torch.cuda.current_stream() is until another stream is made current.  The new stream is
 * made to wait for the work already issued on the old one (the context's buffers -- scratch,
 * staged images -- are reused by the next launch).  Graph capture: switching onto a stream that
 * is being captured, or off one, issues no event record / wait (they would invalidate or leak
 * into the capture), so the caller orders the capture stream after the context's earlier work
 * (e.g. synchronise before capturing) and synchronises the graph's launches before the context
 * runs on another stream or grows its buffers (mv_context_reserve first: then nothing grows). */
int mv_context_set_stream(mv_context *ctx, void *hip_stream);
int mv_context_use_own_stream(mv_context *ctx); /* back to the context's own non-blocking stream */
void *mv_context_stream(mv_context *ctx);
int mv_context_synchronize(mv_context *ctx);
/* Pre-size scratch for up to `batch` pairs of `cap` keypoints / cells, for the context's CURRENT
 * all-pairs screen.  Under the default MV_SCREEN_I8 nothing is staged, so the staged int8 images
 * that sequence mode (mv_match_sequence_*) needs are NOT reserved: they are allocated by its first
 * call.  Before capturing sequence mode in a graph, either select MV_SCREEN_I8_STAGED, reserve,
 * and switch back, or run it once at its largest shape. */
int mv_context_reserve(mv_context *ctx, int batch, int cap);
mv_context *mv_default_context(void); /* the calling thread's; NULL (stderr once) without a device */

/* Kernel profiler: while enabled, every kernel launch is bracketed by two
 * hipEvents recorded on its own stream (no synchronisation is added).
 * mv_profile_query() synchronises the recorded events and returns the summed
 * device time and the launch count of one kernel (e.g. "k_ap_screen"). */
int mv_profile_enable(int on); /* on != 0 clears previous records */
int mv_profile_query(const char *kernel, double *total_ms, int *launches);

/* ------------------------------------------------------------------------ */
/* Windowed int8 front end  (src/top_N.c, src/tracking_main.c:84-194)        */
/* ------------------------------------------------------------------------ */
typedef struct {
    int shift_x, shift_y, radius; /* 4, 4, 4            (tracking_main.c:104-106) */
    int max_matches;              /* 150                (tracking_main.c:13)      */
    int semantics;                /* mv_semantics                                  */
    double match_thresh_sq;       /* 0.9 * 0.9          (tracking_main.c:12,155)  */
    double prob_thresh;           /* 0.2                (tracking_main.c:146)     */
} mv_window_params;
void mv_window_params_default(mv_window_params *p);

/* Per-frame / per-pair, host pointers, synchronous on the context's stream. */
int mv_softmax_host(mv_context *ctx, float scale, const int8_t *semi, int cells, int *num_valid,
                    int *max_indices, float *probs);
int mv_top_n_host(mv_context *ctx, float scale, const int8_t *semi, int cells, int N, int cap,
                  int *num_selected, int *patches, int *indices, float *probs);
int mv_window_match_host(mv_context *ctx, const mv_window_params *p, int rows, int cols, const int8_t *desc0,
                         const int *max_idx0, const float *probs0, const int8_t *desc1, int num_queries,
                         const int *patches1, const int *indices1, int *num_matches, float *points1,
                         float *points2, int *query_of_match);

/* Batched over B frames: softmax of every cell (compute_softmax, top_N.c:136-165).
 * scale[B] are the EFFECTIVE scales (apply mv_scale_as_built() for MV_AS_BUILT). */
int mv_softmax_batch_dev(mv_context *ctx, int batch, int cells, const float *scales, const int8_t *semi,
                         int *max_idx, float *probs, int *num_valid);
/* Cell-level NMS of the int8 path (src/run_nms.c:65-155) on softmax outputs, in place:
 * max_idx / probs [B][cells] (suppressed cells: index 64, prob 64 as in the reference);
 * kp [B][cells][2] = the surviving cells' pixels (x, y) in patch order, num_kp [B].
 * rows * cols <= 8192 (the walk holds a frame in LDS). */
int mv_run_nms_batch_dev(mv_context *ctx, int batch, int rows, int cols, int *max_idx, float *probs, int *num_kp,
                         float *kp);
/* Batched top-N selection from softmax outputs (compute_top_N, top_N.c:53-134).
 * status[B] = 0 or MV_ERR_CAPACITY.  Outputs [B][N]. */
int mv_top_n_select_batch_dev(mv_context *ctx, int batch, int cells, const int *max_idx, const float *probs,
                              int N, int cap, int *num_selected, int *patches, int *indices, float *sel_probs,
                              int *status);
/* Batched windowed match (tracking_main.c:103-194).  Queries are the top-N
 * lists ([B][N] + num_selected[B]); outputs points [B][max_matches][2]. */
int mv_window_match_batch_dev(mv_context *ctx, const mv_window_params *p, int batch, int rows, int cols,
                              const int8_t *desc0, const int *max_idx0, const float *probs0, const int8_t *desc1,
                              int N, const int *num_selected, const int *patches1, const int *indices1,
                              int *num_matches, float *points1, float *points2, int *query_of_match);
float mv_scale_as_built(float scale); /* low 32 bits of (double)scale, SURVEY F7 */

/* ------------------------------------------------------------------------ */
/* All-pairs descriptor match  (python/pairwise_pnp.py:635-659)              */
/* ------------------------------------------------------------------------ */
/* For every row i < n0[b] of desc0[b]: the FIRST j < n1[b] attaining the
 * maximum of the fp32 score s_ij = sum_k d0[i][k]*d1[j][k] (summed k = 0..255
 * sequentially, mul then add: the gemmini_functions_cpu.h:45-49 order), kept
 * when (double)s > thresh and s > 0.  match_idx = -1 otherwise.  Bit-exact: an
 * fp16 MFMA screen plus an exact re-score of every candidate within the
 * rounding bound (rows with |x| >= 2 or non-finite values take the exact path).
 * cap = row stride (keypoints per frame slot).
 * match_score may be NULL: the reference keeps only the matched pairs
 * (pairwise_pnp.py:649-657), so without a score output the exact re-score runs
 * only where the rounding window does not already decide the row; match_idx is
 * identical either way. */
/* How the all-pairs fp32 match screens its candidates before the exact fp32 re-score (the
 * outputs are bit-identical either way):
 *   MV_SCREEN_I8 (default)  ONE kernel reads both fp32 frames once, quantises them per row to
 *                           int8 inside the workgroup and screens on the int8 matrix cores with
 *                           a rigorous quantisation window (no staged image: prepare/run only
 *                           record the batch, and run_prepare stages nothing);
 *   MV_SCREEN_F16           screens on fp16 MFMAs against a staged fp16 image of frame 1
 *                           (2^14-scaled operands);
 *   MV_SCREEN_I8_STAGED     the int8 screen against a staged int8 image of frame 1 (the
 *                           image sequence mode reuses; run_prepare stages the next batch's
 *                           image inside the match launch).
 * Sequence mode always uses staged int8 images (under MV_SCREEN_I8 or MV_SCREEN_I8_STAGED).
 * The environment variable MV_AP_SCREEN=f16 / i8s selects the fp16 / staged-int8 screen for
 * contexts created afterwards. */
typedef enum { MV_SCREEN_I8 = 0, MV_SCREEN_F16 = 1, MV_SCREEN_I8_STAGED = 2 } mv_allpairs_screen;
int mv_context_set_allpairs_screen(mv_context *ctx, int screen);
int mv_context_allpairs_screen(mv_context *ctx);
int mv_match_allpairs_f32_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                              const float *desc0, const float *desc1, double thresh, int *match_idx,
                              float *match_score);
/* The same as two stages, for pipelining batches: prepare stages frame 1 (fp16 image,
 * norms) on the context's auxiliary stream, ordered after everything issued so far on the
 * context stream; run waits for it on the context stream and matches.  Issue
 * prepare(next batch) right after run(this batch) and before the pose of this batch: the
 * staging of the next batch then overlaps the pose.  run must be given exactly the
 * (batch, cap, n1, desc1) of the last prepare. */
int mv_match_allpairs_f32_prepare_dev(mv_context *ctx, int batch, int cap, const int *n1, const float *desc1);
int mv_match_allpairs_f32_run_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                  const float *desc0, const float *desc1, double thresh, int *match_idx,
                                  float *match_score);
/* run (this batch, prepared) + prepare (the next batch) in one call, both on the context
 * stream: with the int8 screen ONE kernel matches this batch and stages the next batch's
 * frame 1 into the context's second image (each workgroup takes a share of the next rows
 * after its tile), so the pipelined step has no separate staging kernel or stream hand-off.
 * Afterwards the next batch is the prepared one (call this again with it, or run_dev). */
int mv_match_allpairs_f32_run_prepare_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                          const float *desc0, const float *desc1, double thresh, int *match_idx,
                                          float *match_score, int next_batch, int next_cap, const int *next_n1,
                                          const float *next_desc1);
/* Sequence mode: the all-pairs match of CONSECUTIVE frames of one track (the reference's
 * driver, scripts/run_pairwise_pnp.sh:7-20, runs pairwise_pnp.py on frames i, i + 1).
 * desc[frames][cap][256] fp32, n[frames]; pair b = (frame b, frame b + 1) for
 * b < frames - 1, outputs match_idx / match_score [frames - 1][cap] exactly as
 * mv_match_allpairs_f32_dev on (desc[b], desc[b + 1]) would give them.  Every frame is
 * quantised once and its int8 image serves as frame 1 of one pair and frame 0 of the next.
 * Int8 screen only (MV_ERR_INVALID_ARG under MV_SCREEN_F16); frames >= 2; invalidates a
 * prepared batch (the scratch image is reused). */
int mv_match_sequence_f32_dev(mv_context *ctx, int frames, int cap, const int *n, const float *desc, double thresh,
                              int *match_idx, float *match_score);
/* Pipelined sequence mode: a track processed in chunks of frames.  Stage the first chunk with
 * mv_match_allpairs_f32_prepare_dev(ctx, frames, cap, n, desc) (the images of all its frames),
 * then call this per chunk: ONE kernel matches the chunk's frames - 1 pairs from the prepared
 * images and stages the next chunk's frames (next_*) into the context's second image, which
 * becomes the prepared one.  (frames, cap, n, desc) must be those of the last prepare. */
int mv_match_sequence_f32_run_prepare_dev(mv_context *ctx, int frames, int cap, const int *n, const float *desc,
                                          double thresh, int *match_idx, float *match_score, int next_frames,
                                          int next_cap, const int *next_n, const float *next_desc);
/* nn_match_two_way (pairwise_pnp.py:281-323): mutual nearest neighbours under the
 * float32 distance sqrt(2 - 2 clip(s, -1, 1)) of the score s above (np.argmin: the first
 * NaN, else the first minimum), kept when dist < (float)nn_thresh and the reverse nearest
 * neighbour of the match is the row itself.  match_idx[b][i] = j or -1 (i < n0[b]);
 * match_dist (may be NULL) = the kept distance.  nn_thresh < 0: MV_ERR_INVALID_ARG (the
 * reference raises).  Runs the all-pairs match both ways (frame 0 then frame 1 staged). */
int mv_match_two_way_f32_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                             const float *desc0, const float *desc1, double nn_thresh, int *match_idx,
                             float *match_dist);
/* int8 descriptors: exact cosine (dot > 0, 100 dot^2 > 81 |a|^2 |b|^2, first
 * maximum of dot^2/|b|^2); integer-exact (MFMA i8). */
int mv_match_allpairs_i8_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                             const int8_t *desc0, const int8_t *desc1, int *match_idx, int *match_dot);

/* ------------------------------------------------------------------------ */
/* Pose  (src/pnp_solver.c; python/pairwise_pnp.py:667-694)                  */
/* ------------------------------------------------------------------------ */
typedef struct {
    float fx, fy, cx, cy;  /* intrinsics */
    int semantics;         /* MV_AS_BUILT: stub RANSAC (E = I) + McAdams pose; MV_AS_INTENDED: below */
    int hypotheses;        /* RANSAC 8-point hypotheses per pair (as-built: iterations, 10) */
    float inlier_thresh;   /* as-built: ||E p1 - p2||^2 threshold (1.1); as-intended: Sampson, pixels */
    int refine_iters;      /* maximum Gauss-Newton iterations on the inliers (stops at convergence) */
    unsigned long long seed;
} mv_pose_params;
void mv_pose_params_default(mv_pose_params *p, int semantics);

/* Pose from matched points: pts0/pts1 [B][cap][2] pixels, n[b] points.
 * T[B][3][4], num_inliers[B], status[B]. */
int mv_pose_batch_dev(mv_context *ctx, const mv_pose_params *p, int batch, int cap, const int *n,
                      const float *pts0, const float *pts1, float *T, int *num_inliers, int *status);
/* Pose from an all-pairs match: correspondences (kp0[i], kp1[match_idx[i]]). */
int mv_pose_from_matches_dev(mv_context *ctx, const mv_pose_params *p, int batch, int cap, const int *n0,
                             const int *match_idx, const float *kp0, const float *kp1, float *T,
                             int *num_matches, int *num_inliers, int *status);

/* Single pair, host pointers (the pnp_solver.h drop-ins are built on these). */
int mv_ransac_stub_host(mv_context *ctx, int n, const float *pts1, const float *pts2, float thresh,
                        float *best_E, int *best_inliers, int *num_inliers);
int mv_recover_pose_host(mv_context *ctx, const float *E, float *R1, float *R2, float *t);
int mv_svd3_host(mv_context *ctx, const float *A, float *U, float *S, float *V);

/* tracking.h with explicit parameters and outputs. */
typedef struct {
    mv_window_params window;
    mv_pose_params pose;
    int top_n;       /* 100 */
    int valid_cap;   /* 1000 (MAX_VALID_FEATURES, top_N.c:51) */
} mv_track_params;
void mv_track_params_default(mv_track_params *p, int semantics);
int mv_track_pair_host(mv_context *ctx, const mv_track_params *p, int rows, int cols, float semi_scale0,
                       const int8_t *semi0, const int8_t *desc0, float semi_scale1, const int8_t *semi1,
                       const int8_t *desc1, float *T, int *num_matches, float *points1, float *points2);

#ifdef __cplusplus
}
#endif
#endif
