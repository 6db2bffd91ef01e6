// mv_api.hip -- extern "C" entry points of libmaveric_hip.so that are not a
// single kernel launcher: parameter defaults, host-pointer (one frame / one
// pair) wrappers, batched pose, and the whole-pair tracking call.
#include <string.h>

#include "mv_internal.hpp"

namespace {

// bump allocator over the context staging buffer (host-pointer calls only)
struct Bump {
    char *base;
    size_t off;
    template <class T>
    T *take(size_t count) {
        off = mv::align_up(off, 256);
        T *p = reinterpret_cast<T *>(base + off);
        off += sizeof(T) * count;
        return p;
    }
};

size_t a256(size_t b) { return mv::align_up(b, 256); }

}  // namespace

extern "C" {

float mv_scale_as_built(float scale) {
    double d = (double)scale;
    uint64_t bits;
    memcpy(&bits, &d, sizeof bits);
    uint32_t lo = (uint32_t)bits;
    float f;
    memcpy(&f, &lo, sizeof f);
    return f;
}

void mv_window_params_default(mv_window_params *p) {
    p->shift_x = 4;
    p->shift_y = 4;
    p->radius = 4;
    p->max_matches = 150;
    p->semantics = MV_AS_BUILT;
    p->match_thresh_sq = 0.9 * 0.9;
    p->prob_thresh = 0.2;
}

void mv_pose_params_default(mv_pose_params *p, int semantics) {
    // tracking_main.c:205-207 intrinsics, :210-211 RANSAC constants
    p->fx = 517.306408f;
    p->fy = 516.469215f;
    p->cx = 318.643040f;
    p->cy = 255.313989f;
    p->semantics = semantics;
    if (semantics == MV_AS_BUILT) {
        p->hypotheses = 10;
        p->inlier_thresh = 1.1f;
        p->refine_iters = 0;
    } else {
        p->hypotheses = 256;
        p->inlier_thresh = 1.0f;  // px, cv2.findEssentialMat default
        p->refine_iters = 20;
    }
    p->seed = 0;
}

void mv_track_params_default(mv_track_params *p, int semantics) {
    mv_window_params_default(&p->window);
    p->window.semantics = semantics;
    mv_pose_params_default(&p->pose, semantics);
    p->top_n = 100;
    p->valid_cap = 1000;
}

int mv_softmax_batch_dev(mv_context *ctx, int batch, int cells, const float *scales, const int8_t *semi,
                         int *max_idx, float *probs, int *num_valid) {
    MV_REQUIRE(ctx != nullptr);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    return mv::launch_softmax(ctx->stream, batch, cells, scales, semi, max_idx, probs, num_valid);
}

int mv_top_n_select_batch_dev(mv_context *ctx, int batch, int cells, const int *max_idx, const float *probs, int N,
                              int cap, int *num_selected, int *patches, int *indices, float *sel_probs,
                              int *status) {
    MV_REQUIRE(ctx != nullptr);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    return mv::launch_top_n_select(ctx->stream, batch, cells, max_idx, probs, N, cap, num_selected, patches,
                                   indices, sel_probs, status);
}

int mv_softmax_host(mv_context *ctx, float scale, const int8_t *semi, int cells, int *num_valid, int *max_indices,
                    float *probs) {
    MV_REQUIRE(ctx && semi && cells > 0 && num_valid && max_indices && probs);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const size_t need = a256(4) + a256((size_t)cells * 65) + 2 * a256((size_t)cells * 4) + a256(4) + 4096;
    Bump bp{(char *)mv::stage(ctx, need), 0};
    if (!bp.base) return MV_ERR_OUT_OF_MEMORY;
    float *d_scale = bp.take<float>(1);
    int8_t *d_semi = bp.take<int8_t>((size_t)cells * 65);
    int *d_mi = bp.take<int>(cells);
    float *d_pr = bp.take<float>(cells);
    int *d_nv = bp.take<int>(1);
    hipStream_t s = ctx->stream;
    MV_HIP_TRY(hipMemcpyAsync(d_scale, &scale, 4, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_semi, semi, (size_t)cells * 65, hipMemcpyHostToDevice, s));
    int st = mv::launch_softmax(s, 1, cells, d_scale, d_semi, d_mi, d_pr, d_nv);
    if (st) return st;
    int nv = 0;
    MV_HIP_TRY(hipMemcpyAsync(max_indices, d_mi, (size_t)cells * 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(probs, d_pr, (size_t)cells * 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(&nv, d_nv, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    *num_valid = nv;
    return mv::set_status(MV_OK);
}

int mv_top_n_host(mv_context *ctx, float scale, const int8_t *semi, int cells, int N, int cap, int *num_selected,
                  int *patches, int *indices, float *probs) {
    MV_REQUIRE(ctx && semi && cells > 0 && N > 0 && cap > 0 && num_selected && patches && indices && probs);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const size_t need = a256(4) + a256((size_t)cells * 65) + 2 * a256((size_t)cells * 4) + 4 * a256(4) +
                        2 * a256((size_t)N * 4) + a256((size_t)N * 4) + 4096;
    Bump bp{(char *)mv::stage(ctx, need), 0};
    if (!bp.base) return MV_ERR_OUT_OF_MEMORY;
    float *d_scale = bp.take<float>(1);
    int8_t *d_semi = bp.take<int8_t>((size_t)cells * 65);
    int *d_mi = bp.take<int>(cells);
    float *d_pr = bp.take<float>(cells);
    int *d_nv = bp.take<int>(1);
    int *d_ns = bp.take<int>(1);
    int *d_st = bp.take<int>(1);
    int *d_pa = bp.take<int>(N);
    int *d_ix = bp.take<int>(N);
    float *d_sp = bp.take<float>(N);
    hipStream_t s = ctx->stream;
    MV_HIP_TRY(hipMemcpyAsync(d_scale, &scale, 4, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_semi, semi, (size_t)cells * 65, hipMemcpyHostToDevice, s));
    int st = mv::launch_softmax(s, 1, cells, d_scale, d_semi, d_mi, d_pr, d_nv);
    if (st) return st;
    st = mv::launch_top_n_select(s, 1, cells, d_mi, d_pr, N, cap, d_ns, d_pa, d_ix, d_sp, d_st);
    if (st) return st;
    int ns = 0, status = 0;
    MV_HIP_TRY(hipMemcpyAsync(&ns, d_ns, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(&status, d_st, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(patches, d_pa, (size_t)N * 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(indices, d_ix, (size_t)N * 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(probs, d_sp, (size_t)N * 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    if (status != MV_OK) {
        *num_selected = -1;
        mv::set_error(status, "top-N: %d or more cells passed the validity filter (cap %d)", cap, cap);
        return status;
    }
    *num_selected = ns;
    return mv::set_status(MV_OK);
}

int mv_window_match_host(mv_context *ctx, const mv_window_params *p, int rows, int cols, const int8_t *desc0,
                         const int *max_idx0, const float *probs0, const int8_t *desc1, int num_queries,
                         const int *patches1, const int *indices1, int *num_matches, float *points1,
                         float *points2, int *query_of_match) {
    MV_REQUIRE(ctx && p && rows > 0 && cols > 0 && desc0 && max_idx0 && probs0 && desc1 && num_matches &&
               points1 && points2 && num_queries >= 0);
    MV_REQUIRE(num_queries == 0 || (patches1 && indices1));
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const int cells = rows * cols, N = num_queries > 0 ? num_queries : 1, M = p->max_matches;
    const size_t need = 2 * a256((size_t)cells * 256) + 2 * a256((size_t)cells * 4) + 3 * a256((size_t)N * 4) +
                        2 * a256((size_t)M * 8) + a256((size_t)M * 4) + a256(4) + 4096;
    Bump bp{(char *)mv::stage(ctx, need), 0};
    if (!bp.base) return MV_ERR_OUT_OF_MEMORY;
    int8_t *d_d0 = bp.take<int8_t>((size_t)cells * 256);
    int8_t *d_d1 = bp.take<int8_t>((size_t)cells * 256);
    int *d_mi = bp.take<int>(cells);
    float *d_pr = bp.take<float>(cells);
    int *d_ns = bp.take<int>(1);
    int *d_pa = bp.take<int>(N);
    int *d_ix = bp.take<int>(N);
    int *d_nm = bp.take<int>(1);
    float *d_p1 = bp.take<float>((size_t)M * 2);
    float *d_p2 = bp.take<float>((size_t)M * 2);
    int *d_q = bp.take<int>(M);
    hipStream_t s = ctx->stream;
    MV_HIP_TRY(hipMemcpyAsync(d_d0, desc0, (size_t)cells * 256, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_d1, desc1, (size_t)cells * 256, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_mi, max_idx0, (size_t)cells * 4, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_pr, probs0, (size_t)cells * 4, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_ns, &num_queries, 4, hipMemcpyHostToDevice, s));
    if (num_queries > 0) {
        MV_HIP_TRY(hipMemcpyAsync(d_pa, patches1, (size_t)num_queries * 4, hipMemcpyHostToDevice, s));
        MV_HIP_TRY(hipMemcpyAsync(d_ix, indices1, (size_t)num_queries * 4, hipMemcpyHostToDevice, s));
    }
    int st = mv_window_match_batch_dev(ctx, p, 1, rows, cols, d_d0, d_mi, d_pr, d_d1, N, d_ns, d_pa, d_ix, d_nm,
                                       d_p1, d_p2, d_q);
    if (st) return st;
    int nm = 0;
    MV_HIP_TRY(hipMemcpyAsync(&nm, d_nm, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    if (nm > 0) {
        MV_HIP_TRY(hipMemcpyAsync(points1, d_p1, (size_t)nm * 8, hipMemcpyDeviceToHost, s));
        MV_HIP_TRY(hipMemcpyAsync(points2, d_p2, (size_t)nm * 8, hipMemcpyDeviceToHost, s));
        if (query_of_match) MV_HIP_TRY(hipMemcpyAsync(query_of_match, d_q, (size_t)nm * 4, hipMemcpyDeviceToHost, s));
        MV_HIP_TRY(hipStreamSynchronize(s));
    }
    *num_matches = nm;
    return mv::set_status(MV_OK);
}

int mv_pose_batch_dev(mv_context *ctx, const mv_pose_params *p, int batch, int cap, const int *n, const float *pts0,
                      const float *pts1, float *T, int *num_inliers, int *status) {
    MV_REQUIRE(ctx != nullptr);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    void *scr = mv::scratch(ctx, mv::pose_scratch_bytes(batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    return mv::launch_pose(ctx->stream, scr, p, batch, cap, n, pts0, pts1, nullptr, nullptr, T, nullptr,
                           num_inliers, status);
}

int mv_pose_from_matches_dev(mv_context *ctx, const mv_pose_params *p, int batch, int cap, const int *n0,
                             const int *match_idx, const float *kp0, const float *kp1, float *T, int *num_matches,
                             int *num_inliers, int *status) {
    MV_REQUIRE(ctx != nullptr && match_idx != nullptr);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    void *scr = mv::scratch(ctx, mv::pose_scratch_bytes(batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    return mv::launch_pose(ctx->stream, scr, p, batch, cap, n0, kp0, nullptr, match_idx, kp1, T, num_matches,
                           num_inliers, status);
}

int mv_ransac_stub_host(mv_context *ctx, int n, const float *pts1, const float *pts2, float thresh, float *best_E,
                        int *best_inliers, int *num_inliers) {
    MV_REQUIRE(ctx && n > 0 && pts1 && pts2 && best_E && best_inliers && num_inliers);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const size_t need = 2 * a256((size_t)n * 8) + a256(36) + a256(1000 * 4) + a256(4) + 4096;
    Bump bp{(char *)mv::stage(ctx, need), 0};
    if (!bp.base) return MV_ERR_OUT_OF_MEMORY;
    float *d_p1 = bp.take<float>((size_t)n * 2);
    float *d_p2 = bp.take<float>((size_t)n * 2);
    float *d_E = bp.take<float>(9);
    int *d_in = bp.take<int>(1000);
    int *d_n = bp.take<int>(1);
    hipStream_t s = ctx->stream;
    MV_HIP_TRY(hipMemcpyAsync(d_p1, pts1, (size_t)n * 8, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_p2, pts2, (size_t)n * 8, hipMemcpyHostToDevice, s));
    int st = mv::launch_ransac_stub(s, n, d_p1, d_p2, thresh, d_E, d_in, d_n);
    if (st) return st;
    int cnt = 0;
    MV_HIP_TRY(hipMemcpyAsync(&cnt, d_n, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(best_E, d_E, 36, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    if (cnt > 0) {
        MV_HIP_TRY(hipMemcpyAsync(best_inliers, d_in, (size_t)cnt * 4, hipMemcpyDeviceToHost, s));
        MV_HIP_TRY(hipStreamSynchronize(s));
    }
    *num_inliers = cnt;
    return mv::set_status(MV_OK);
}

static int small_call(mv_context *ctx, int which, const float *in, float *o1, float *o2, float *o3) {
    MV_REQUIRE(ctx && in && o1 && o2 && o3);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    Bump bp{(char *)mv::stage(ctx, 4096), 0};
    if (!bp.base) return MV_ERR_OUT_OF_MEMORY;
    float *d_in = bp.take<float>(9);
    float *d_1 = bp.take<float>(9);
    float *d_2 = bp.take<float>(9);
    float *d_3 = bp.take<float>(9);
    hipStream_t s = ctx->stream;
    MV_HIP_TRY(hipMemcpyAsync(d_in, in, 36, hipMemcpyHostToDevice, s));
    int st = which == 0 ? mv::launch_recover_pose(s, d_in, d_1, d_2, d_3) : mv::launch_svd3(s, d_in, d_1, d_2, d_3);
    if (st) return st;
    MV_HIP_TRY(hipMemcpyAsync(o1, d_1, 36, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(o2, d_2, which == 0 ? 36 : 12, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(o3, d_3, which == 0 ? 12 : 36, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    return mv::set_status(MV_OK);
}

int mv_recover_pose_host(mv_context *ctx, const float *E, float *R1, float *R2, float *t) {
    return small_call(ctx, 0, E, R1, R2, t);
}

int mv_svd3_host(mv_context *ctx, const float *A, float *U, float *S, float *V) {
    return small_call(ctx, 1, A, U, S, V);
}

int mv_track_pair_host(mv_context *ctx, const mv_track_params *p, int rows, int cols, float semi_scale0,
                       const int8_t *semi0, const int8_t *desc0, float semi_scale1, const int8_t *semi1,
                       const int8_t *desc1, float *T, int *num_matches, float *points1, float *points2) {
    MV_REQUIRE(ctx && p && rows > 0 && cols > 0 && semi0 && desc0 && semi1 && desc1 && T && num_matches);
    MV_REQUIRE(points1 && points2 && p->top_n > 0 && p->window.max_matches > 0);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const int cells = rows * cols, N = p->top_n, M = p->window.max_matches;
    const size_t need = 2 * a256(8) + 2 * a256((size_t)cells * 65) + 2 * a256((size_t)cells * 256) +
                        4 * a256((size_t)cells * 4) + 8 * a256(4) + 3 * a256((size_t)N * 4) +
                        2 * a256((size_t)M * 8) + a256(48) + 8192;
    Bump bp{(char *)mv::stage(ctx, need), 0};
    if (!bp.base) return MV_ERR_OUT_OF_MEMORY;
    float *d_sc = bp.take<float>(2);
    int8_t *d_s0 = bp.take<int8_t>((size_t)cells * 65);
    int8_t *d_s1 = bp.take<int8_t>((size_t)cells * 65);
    int8_t *d_d0 = bp.take<int8_t>((size_t)cells * 256);
    int8_t *d_d1 = bp.take<int8_t>((size_t)cells * 256);
    int *d_mi0 = bp.take<int>(cells);
    float *d_pr0 = bp.take<float>(cells);
    int *d_mi1 = bp.take<int>(cells);
    float *d_pr1 = bp.take<float>(cells);
    int *d_nv = bp.take<int>(2);
    int *d_ns = bp.take<int>(1);
    int *d_st = bp.take<int>(1);
    int *d_pa = bp.take<int>(N);
    int *d_ix = bp.take<int>(N);
    float *d_sp = bp.take<float>(N);
    int *d_nm = bp.take<int>(1);
    float *d_p1 = bp.take<float>((size_t)M * 2);
    float *d_p2 = bp.take<float>((size_t)M * 2);
    float *d_T = bp.take<float>(12);
    int *d_ni = bp.take<int>(1);
    int *d_ps = bp.take<int>(1);
    hipStream_t s = ctx->stream;
    const bool built = p->window.semantics == MV_AS_BUILT;
    float sc[2] = {built ? mv_scale_as_built(semi_scale0) : semi_scale0,
                   built ? mv_scale_as_built(semi_scale1) : semi_scale1};
    MV_HIP_TRY(hipMemcpyAsync(d_sc, sc, 8, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_s0, semi0, (size_t)cells * 65, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_s1, semi1, (size_t)cells * 65, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_d0, desc0, (size_t)cells * 256, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_d1, desc1, (size_t)cells * 256, hipMemcpyHostToDevice, s));
    int st = mv::launch_softmax(s, 1, cells, d_sc, d_s0, d_mi0, d_pr0, d_nv);
    if (!st) st = mv::launch_softmax(s, 1, cells, d_sc + 1, d_s1, d_mi1, d_pr1, d_nv + 1);
    if (!st)
        st = mv::launch_top_n_select(s, 1, cells, d_mi1, d_pr1, N, p->valid_cap, d_ns, d_pa, d_ix, d_sp, d_st);
    if (!st)
        st = mv_window_match_batch_dev(ctx, &p->window, 1, rows, cols, d_d0, d_mi0, d_pr0, d_d1, N, d_ns, d_pa,
                                       d_ix, d_nm, d_p1, d_p2, nullptr);
    if (!st) {
        void *scr = mv::scratch(ctx, mv::pose_scratch_bytes(1, M));
        if (!scr) return MV_ERR_OUT_OF_MEMORY;
        st = mv::launch_pose(s, scr, &p->pose, 1, M, d_nm, d_p1, d_p2, nullptr, nullptr, d_T, nullptr, d_ni, d_ps);
    }
    if (st) return st;
    int nm = 0, tst = 0, pst = 0;
    MV_HIP_TRY(hipMemcpyAsync(&nm, d_nm, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(&tst, d_st, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(&pst, d_ps, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(T, d_T, 48, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(points1, d_p1, (size_t)M * 8, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(points2, d_p2, (size_t)M * 8, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    if (tst != MV_OK) {
        mv::set_error(tst, "top-N capacity (%d) exceeded", p->valid_cap);
        return tst;
    }
    *num_matches = nm;
    return mv::set_status(pst);
}

}  // extern "C"
