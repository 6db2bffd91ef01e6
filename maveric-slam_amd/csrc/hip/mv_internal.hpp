// mv_internal.hpp -- shared internals of libmaveric_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "maveric_hip.h"

struct mv_context {
    int device;
    hipStream_t own_stream;
    hipStream_t stream;  // where every *_dev launch goes
    void *scratch;       // device scratch, grown by mv_scratch()/mv_context_reserve()
    size_t scratch_bytes;
    // small host<->device staging for the single-pair host entry points
    void *stage_dev;
    size_t stage_bytes;
    // all-pairs fp32: its own scratch (frame-1 fp16 image, norms, range flags) so that a
    // prepare of the next batch on aux_stream never races the pose kernels on `stream`
    void *ap_scratch;
    size_t ap_scratch_bytes;
    void *ap_scratch2;  // the other image of run_prepare (swapped with ap_scratch per call)
    size_t ap_scratch2_bytes;
    hipStream_t aux_stream;  // created on first prepare
    hipEvent_t ev_in, ev_prep;
    int prep_batch, prep_cap;  // what the last prepare staged (run checks it)
    const int *prep_n1;
    const float *prep_desc1;
    int prep_screen;
    bool prep_staged;  // the prepared batch's frame 1 sits staged in ap_scratch (false: recorded only)
    int ap_screen;  // mv_allpairs_screen of the fp32 all-pairs match (0 = int8, the default)
    // set_stream / use_own_stream away from a stream record this event on it and make own_stream
    // wait on it: own_stream then orders after all work issued on every stream the context left
    // (no stream handle is kept, so a caller may destroy a stream once the context moved off it)
    hipEvent_t ev_retire;
    // int8 all-pairs adaptive dispatch (mv_match_allpairs_i8_dev): pinned count of the pairs the
    // last measuring call handed back, that call's batch, calls so far
    int *i8_count_host;
    int i8_meas_batch;
    unsigned i8_calls;
    bool i8_prefer_m;  // the last landed measurement: most pairs handed back
};

namespace mv {

void set_error(int status, const char *fmt, ...);
int set_status(int status);

// true while `s` is captured into a graph (or the query is refused: see mv_context.hip)
int capture_state(hipStream_t s, bool *cap);  // MV_OK + *cap, or MV_ERR_HIP (reported)
// Grow (never shrink) the context scratch; returns nullptr on failure.
void *scratch(mv_context *ctx, size_t bytes);
void *stage(mv_context *ctx, size_t bytes);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Wait for every stream this context has issued work on (its own stream -- which waits on every
// stream the context left, via ev_retire --, the current stream and the staging stream) -- before
// a context buffer is freed; other contexts and threads are not blocked (no device-wide
// synchronisation unless a synchronisation itself fails).
int quiesce(mv_context *ctx);
// bytes of one staged frame-1 image (ap_scratch / ap_scratch2) under `screen`
size_t ap_image_bytes(int screen, int batch, int cap);

// Kernel profiler (mv_profile_* in maveric_hip.h): when enabled, launchers
// bracket each kernel with hipEventRecord on the launch stream -- no sync.
bool prof_on();
void prof_begin(hipStream_t s, const char *kernel);
void prof_end(hipStream_t s);

}  // namespace mv

#define MV_PROF_BEGIN(s, name) \
    do {                       \
        if (mv::prof_on()) mv::prof_begin((s), (name)); \
    } while (0)
#define MV_PROF_END(s)         \
    do {                       \
        if (mv::prof_on()) mv::prof_end(s); \
    } while (0)

#define MV_HIP_TRY(expr)                                                                   \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) {                                                            \
            mv::set_error(MV_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr,           \
                          hipGetErrorString(_e));                                          \
            return MV_ERR_HIP;                                                             \
        }                                                                                  \
    } while (0)

#define MV_LAUNCH_CHECK() MV_HIP_TRY(hipGetLastError())

#define MV_REQUIRE(cond)                                                                   \
    do {                                                                                   \
        if (!(cond)) {                                                                     \
            mv::set_error(MV_ERR_INVALID_ARG, "%s:%d invalid argument: %s", __FILE__,      \
                          __LINE__, #cond);                                                \
            return MV_ERR_INVALID_ARG;                                                     \
        }                                                                                  \
    } while (0)

// ---------------------------------------------------------------------------
// Launchers implemented in the kernel translation units (stream-ordered).
// ---------------------------------------------------------------------------
namespace mv {
int launch_softmax(hipStream_t s, int batch, int cells, const float *scales, const int8_t *semi,
                   int *max_idx, float *probs, int *num_valid);
int launch_top_n_select(hipStream_t s, int batch, int cells, const int *max_idx, const float *probs, int N,
                        int cap, int *num_sel, int *patches, int *indices, float *sel_probs, int *status);
size_t allpairs_f32_scratch_bytes(int batch, int cap);
int launch_allpairs_f32_prepare(hipStream_t s, void *scratch, int batch, int cap, const int *n1,
                                const float *desc1);
int launch_allpairs_f32_match(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                              const float *desc0, const float *desc1, double thresh, int *match_idx,
                              float *match_score, int dmode = 0);
size_t allpairs_q8_scratch_bytes(int batch, int cap);
int launch_allpairs_q8_prepare(hipStream_t s, void *scratch, int batch, int cap, const int *n1,
                               const float *desc1);
int launch_allpairs_q8_match(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                             const float *desc0, const float *desc1, double thresh, int *match_idx,
                             float *match_score, int dmode = 0);
// sequence mode: frames 0 .. frames-1, pair b = (b, b + 1); every frame quantised once
int launch_allpairs_q8_sequence(hipStream_t s, void *scratch, int frames, int cap, const int *n, const float *desc,
                                double thresh, int *match_idx, float *match_score, bool prepared = false,
                                void *next_scratch = nullptr, int next_frames = 0, int next_cap = 0,
                                const int *next_n = nullptr, const float *next_desc = nullptr);
// the match plus the next batch's frame-1 staging into next_scratch, in one launch
int launch_allpairs_q8_match_prepare(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                                     const float *desc0, const float *desc1, double thresh, int *match_idx,
                                     float *match_score, int dmode, void *next_scratch, int next_batch,
                                     int next_cap, const int *next_n1, const float *next_desc1);
// the single-pass int8 screen (k_allpairs_direct.hip): no scratch, frame 1 quantised in-kernel
// only: per-pair flags -- the workgroups of pairs whose flag is 0 exit at once (k_q8t_match's
// hand-backs); null: every pair
int launch_allpairs_q8d_match(hipStream_t s, int batch, int cap, const int *n0, const int *n1, const float *desc0,
                              const float *desc1, double thresh, int *match_idx, float *match_score, int dmode = 0,
                              const int *only = nullptr);
// the one-workgroup-per-pair transposed kernel (k_allpairs_direct.hip), k_q8d_match for its
// hand-backs; scratch >= allpairs_q8t_scratch_bytes(batch)
bool allpairs_q8t_applies(int cap, int dmode);
size_t allpairs_q8t_scratch_bytes(int batch);
int launch_allpairs_q8t_match(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                              const float *desc0, const float *desc1, double thresh, int *match_idx,
                              float *match_score);
size_t allpairs_i8_scratch_bytes(int batch, int cap);
int launch_allpairs_i8(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                       const int8_t *desc0, const int8_t *desc1, int *match_idx, int *match_dot, bool direct = false,
                       int *count_host = nullptr);
size_t pose_scratch_bytes(int batch, int cap);
int launch_pose(hipStream_t s, void *scratch, const mv_pose_params *p, int batch, int cap, const int *n,
                const float *pts0, const float *pts1, const int *match_idx, const float *kp1, float *T,
                int *num_matches, int *num_inliers, int *status);
int launch_ransac_stub(hipStream_t s, int n, const float *pts1, const float *pts2, float thresh, float *E,
                       int *inliers, int *num_inliers);
int launch_recover_pose(hipStream_t s, const float *E, float *R1, float *R2, float *t);
int launch_svd3(hipStream_t s, const float *A, float *U, float *S, float *V);
}  // namespace mv
