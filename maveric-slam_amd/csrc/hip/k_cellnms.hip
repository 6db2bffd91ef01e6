// k_cellnms.hip -- the int8 path's cell-level NMS (src/run_nms.c:65-155), batched over frames.
//
// run_nms.c walks the grid corners (x outer, y inner) and, at each, suppresses cells of the
// 2x2 block around it in place; a corner's result depends on the corners before it that share
// a cell.  Corners (x, y) and (x', y') share a cell only if |x - x'| <= 1 and |y - y'| <= 1,
// and every earlier corner that shares a cell has a smaller t = 2x + y, while corners of equal
// t share none -- so the walk runs as a wavefront over t (2 cols + rows + 1 steps), the
// corners of one anti-diagonal in parallel on the lanes of one wave per frame.  The frame's
// max_idx (int8) and probs live in LDS during the walk (5 B per cell); one wave, so LDS
// writes of step t are visible to step t + 1 in program order (wave barrier + fences).
// Latency-bound by design (the sequential dependency is the reference's).
#include "mv_internal.hpp"

namespace {

constexpr int CNMS_MAX_CELLS = 8192;  // 40 KiB of LDS

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64) void k_run_nms(int rows, int cols, int *__restrict__ max_idx_all,
                                                float *__restrict__ probs_all, int *__restrict__ num_kp,
                                                float *__restrict__ kp_all) {
    __shared__ signed char smi[CNMS_MAX_CELLS];
    __shared__ float spr[CNMS_MAX_CELLS];
    const int b = blockIdx.x, lane = threadIdx.x;
    const int cells = rows * cols;
    int *mi = max_idx_all + (long)b * cells;
    float *pr = probs_all + (long)b * cells;
    for (int p = lane; p < cells; p += 64) {
        smi[p] = (signed char)mi[p];
        spr[p] = pr[p];
    }
    wave_sync();
    for (int t = 0; t <= 2 * cols + rows; t++) {
        // corners x with y = t - 2x in [0, rows]
        const int xlo = max(0, (t - rows + 1) / 2), xhi = min(cols, t / 2);
        for (int xi = xlo + lane; xi <= xhi; xi += 64) {
            const int yi = t - 2 * xi;
            int n = 0, pat[4], xs[4], ys[4];
            float pp[4];
#pragma unroll
            for (int xd = -1; xd <= 0; xd++) {
#pragma unroll
                for (int yd = -1; yd <= 0; yd++) {
                    const int xg = xi + xd, yg = yi + yd;
                    if (xg < 0 || xg >= cols || yg < 0 || yg >= rows) continue;
                    const int p = xg * rows + yg, idx = smi[p];
                    if (idx == 64) continue;
                    const int px = idx % 8, py = idx / 8;
                    if ((xd == -1 && px < 2) || (xd == 0 && px >= 6) || (yd == -1 && py < 2) || (yd == 0 && py >= 6))
                        continue;
                    pat[n] = p;
                    pp[n] = spr[p];
                    xs[n] = xg * 8 + px;
                    ys[n] = yg * 8 + py;
                    n++;
                }
            }
            for (int it = 0; it < 4; it++) {  // each round retires at least the maximum
                float mp = 0.f;
                int m = -1;
                for (int i = 0; i < n; i++)
                    if (pat[i] > 0 && pp[i] > mp) {  // (:110: patch 0 is not a candidate here)
                        mp = pp[i];
                        m = i;
                    }
                if (m == -1) break;
                for (int i = 0; i < n; i++)
                    if (pat[i] >= 0 && pp[i] > mp) {
                        mp = pp[i];
                        m = i;
                    }
                for (int i = 0; i < n; i++) {
                    if (i == m || pat[i] < 0) continue;
                    if (abs(xs[m] - xs[i]) < 4 && abs(ys[m] - ys[i]) < 4) {
                        smi[pat[i]] = 64;
                        spr[pat[i]] = 64.f;  // (:134)
                        pat[i] = -1;
                        pp[i] = -1.f;
                    }
                }
                pp[m] = -1.f;
                pat[m] = -1;
            }
        }
        wave_sync();
    }
    // write back in place, survivors in patch order
    int base = 0;
    float *kp = kp_all + (long)b * cells * 2;
    for (int p0 = 0; p0 < cells; p0 += 64) {
        const int p = p0 + lane;
        const int idx = p < cells ? smi[p] : 64;
        if (p < cells) {
            mi[p] = idx;
            pr[p] = spr[p];
        }
        const unsigned long long m = __ballot(idx != 64);
        if (idx != 64) {
            const int o = base + __popcll(m & ((1ull << lane) - 1ull));
            kp[2 * o] = (float)((p / rows) * 8 + idx % 8);
            kp[2 * o + 1] = (float)((p % rows) * 8 + idx / 8);
        }
        base += __popcll(m);
    }
    if (lane == 0) num_kp[b] = base;
}

}  // namespace

extern "C" int mv_run_nms_batch_dev(mv_context *ctx, int batch, int rows, int cols, int *max_idx, float *probs,
                                    int *num_kp, float *kp) {
    MV_REQUIRE(ctx && batch > 0 && rows > 0 && cols > 0 && max_idx && probs && num_kp && kp);
    MV_REQUIRE((long)rows * cols <= CNMS_MAX_CELLS);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    MV_PROF_BEGIN(ctx->stream, "k_run_nms");
    hipLaunchKernelGGL(k_run_nms, dim3((unsigned)batch), dim3(64), 0, ctx->stream, rows, cols, max_idx, probs, num_kp,
                       kp);
    MV_PROF_END(ctx->stream);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}
