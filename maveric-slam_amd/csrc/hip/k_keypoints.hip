// k_keypoints.hip -- keypoint extraction + descriptor sampling:
// SuperPointFrontend.run after the network forward (python/pairwise_pnp.py:197-257) and
// nms_fast (:116-179), batched over frames.  See include/keypoints.h.
//
//   k_kp_heat    thread per cell: 65 correctly rounded expf, the reference's sequential
//                float32 sum + 1e-5, 64 quotients -> the cell's 8x8 heatmap block
//   k_kp_nms     one 1024-thread block per frame:
//                (a) candidates (heat >= thresh) compacted in row-major order (a contiguous
//                    chunk of pixels per wave: ballot counts, one block scan, ballot writes);
//                (b) the greedy NMS as a fixed point: a candidate is KEPT when every
//                    higher-priority candidate in its (2d+1)^2 window is suppressed, and
//                    SUPPRESSED as soon as one of them is kept (priority: confidence, then
//                    row-major order -- the reference's visiting order).  Each round decides
//                    at least the highest-priority undecided candidate, and the result is the
//                    sequential greedy one (a candidate's fate depends only on higher ones);
//                (c) border filter, then the survivors in output order (confidence descending,
//                    ties in reversed row-major order): a bitonic sort of 64-bit keys in LDS
//                    (<= 4096 survivors) or, beyond, each one's rank counted through LDS tiles;
//   k_kp_nhwc    coarse descriptors [256][Hc*Wc] -> [Hc*Wc][256] (LDS tiles), so that each
//                bilinear corner is one contiguous 1 KiB row
//   k_kp_sample  one wave per keypoint: torch grid_sample's CPU arithmetic (fma unnormalise,
//                floor-distance weights, fma chain over the 4 corners), then the L2 norm with
//                the reference's sequential sum of squares (numpy axis-0 reduce) in one lane.
// Bound: k_kp_heat is FP64-exp / HBM bound (65 x 4 B in, 64 x 4 B out per cell); k_kp_nms is
// latency-bound (one block per frame); k_kp_sample reads 4 KiB per keypoint from L2.
#include <math.h>

#include "keypoints.h"
#include "mv_internal.hpp"

namespace {

constexpr int NMS_T = 1024;  // threads of the per-frame block
constexpr int KP_CH = 4;                 // channels per k_kp_sample_planes workgroup (144 KiB of LDS)
constexpr int KP_PLANE_CELLS = 9216;     // cells whose 4 channel planes fit LDS (144 KiB): KITTI 47x155 = 7285
constexpr int KP_PLANE_CELLS_S = 2048;   // the small-frame instantiation (32 KiB: several workgroups per CU)
constexpr int NC_LDS = 8192;  // candidates per frame held in LDS (more: the global per-pixel path)
constexpr int ROW_LDS = 2048; // heat rows indexed in LDS
// listed higher-priority neighbours per candidate.  16: the 192 x 640 network frames' dense
// candidates (2.2 % of pixels) rescanned their window every NMS round whenever more than 8 higher
// neighbours were listed (A/B in DESIGN 4.3)
constexpr int HN = 16;
static_assert(HN % 4 == 0, "16-B list pieces");
constexpr int SORT_N = 4096; // survivors sorted in LDS (more: ranked by counting)
__host__ __device__ inline long hn_cands(long P) { return (P + 7) / 8; }  // candidates with a list (more: rescanned)

struct KpScratch {
    float *heat;        // [B][P] (when the caller does not keep it)
    int *hn;            // [B][HNC][HN] higher-priority neighbour pixels of candidate k < HNC
    int *hc;            // [B][HNC] their count (HN + 1: more than HN, rescanned each round)
    int *cpix;          // [B][P] candidate pixel (row-major heat index)
    float *cconf;       // [B][P]
    unsigned char *st;  // [B][P] by PIXEL: 0 undecided, 1 kept, 2 suppressed (candidates only)
    int *kept;          // [B][P] surviving candidate ids (unordered)
    int *slot_pix;      // [B][cap] pixel of output slot
    float *nhwc;        // [B][Hc*Wc][256]
};

size_t a256(size_t x) { return mv::align_up(x, 256); }
bool kp_planes_path(int Hc, int Wc) { return (long)Hc * Wc <= KP_PLANE_CELLS; }

size_t kp_scratch_bytes(int B, int Hc, int Wc, int cap) {
    const size_t P = (size_t)Hc * Wc * 64;
    const size_t hnc = (size_t)hn_cands((long)P);
    return a256((size_t)B * P * 4) * 4 + a256((size_t)B * hnc * HN * 4) + a256((size_t)B * hnc * 4) +
           a256((size_t)B * P) + a256((size_t)B * cap * 4) +
           (kp_planes_path(Hc, Wc) ? 0 : a256((size_t)B * Hc * Wc * 256 * 4));  // the NHWC copy
}

KpScratch kp_scratch_map(char *base, int B, int Hc, int Wc, int cap) {
    const size_t P = (size_t)Hc * Wc * 64;
    KpScratch m;
    size_t o = 0;
    m.heat = (float *)(base + o);
    o += a256((size_t)B * P * 4);
    const size_t hnc = (size_t)hn_cands((long)P);
    m.hn = (int *)(base + o);
    o += a256((size_t)B * hnc * HN * 4);
    m.hc = (int *)(base + o);
    o += a256((size_t)B * hnc * 4);
    m.cpix = (int *)(base + o);
    o += a256((size_t)B * P * 4);
    m.cconf = (float *)(base + o);
    o += a256((size_t)B * P * 4);
    m.kept = (int *)(base + o);
    o += a256((size_t)B * P * 4);
    m.st = (unsigned char *)(base + o);
    o += a256((size_t)B * P);
    m.slot_pix = (int *)(base + o);
    o += a256((size_t)B * cap * 4);
    m.nhwc = (float *)(base + o);
    return m;
}

__global__ __launch_bounds__(256) void k_kp_heat(long cells, int Hc, int Wc, const float *__restrict__ semi,
                                                 float *__restrict__ heat) {
    const long q = (long)blockIdx.x * 256 + threadIdx.x;
    if (q >= cells) return;
    const long plane = (long)Hc * Wc;
    const long b = q / plane, cell = q % plane;
    const int hc = (int)(cell / Wc), wc = (int)(cell % Wc);
    const float *S = semi + b * 65 * plane + cell;
    float e[65];
    float den = 0.f;
#pragma unroll
    for (int c = 0; c < 65; c++) {
        e[c] = (float)exp((double)S[c * plane]);  // correctly rounded float32 exp (double, rounded once)
        den = __fadd_rn(den, e[c]);              // np.sum(dense, axis=0): channel by channel
    }
    den = __fadd_rn(den, 1e-5f);
    const int Wh = Wc * 8;
    float *H = heat + b * plane * 64 + (long)(hc * 8) * Wh + wc * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        float4 lo, hi;
        lo.x = __fdiv_rn(e[8 * i + 0], den);
        lo.y = __fdiv_rn(e[8 * i + 1], den);
        lo.z = __fdiv_rn(e[8 * i + 2], den);
        lo.w = __fdiv_rn(e[8 * i + 3], den);
        hi.x = __fdiv_rn(e[8 * i + 4], den);
        hi.y = __fdiv_rn(e[8 * i + 5], den);
        hi.z = __fdiv_rn(e[8 * i + 6], den);
        hi.w = __fdiv_rn(e[8 * i + 7], den);
        *reinterpret_cast<float4 *>(H + (long)i * Wh) = lo;
        *reinterpret_cast<float4 *>(H + (long)i * Wh + 4) = hi;
    }
}

// priority of candidate j over k: higher confidence, then earlier in row-major order
__device__ __forceinline__ bool before(float cj, int j, float ck, int k) { return cj > ck || (cj == ck && j < k); }

// the higher-priority candidates in the (2D+1)^2 window of pixel pk: all heat values loaded
// first (independent loads), then tested; the first HN pixels go to out (if out).  Returns
// the count.
template <int D>
__device__ int list_higher(const float *__restrict__ heat, int Hh, int Wh, float thresh, int pk, float ck,
                           int *__restrict__ out) {
    const int yk = pk / Wh, xk = pk % Wh;
    float v[2 * D + 1][2 * D + 1];
#pragma unroll
    for (int dy = -D; dy <= D; dy++)
#pragma unroll
        for (int dx = -D; dx <= D; dx++) {
            const int y = yk + dy, x = xk + dx;
            v[dy + D][dx + D] = (y >= 0 && y < Hh && x >= 0 && x < Wh) ? heat[y * Wh + x] : __builtin_nanf("");
        }
    int cnt = 0;
#pragma unroll
    for (int dy = -D; dy <= D; dy++)
#pragma unroll
        for (int dx = -D; dx <= D; dx++) {
            if (dy == 0 && dx == 0) continue;
            const int pj = pk + dy * Wh + dx;
            const float h = v[dy + D][dx + D];
            if (h >= thresh && before(h, pj, ck, pk)) {
                if (out && cnt < HN) out[cnt] = pj;
                cnt++;
            }
        }
    return cnt;
}

__device__ int list_higher_any(const float *__restrict__ heat, int Hh, int Wh, float thresh, int d, int pk, float ck,
                               int *__restrict__ out) {
    const int yk = pk / Wh, xk = pk % Wh;
    int cnt = 0;
    for (int y = max(yk - d, 0); y <= min(yk + d, Hh - 1); y++)
        for (int x = max(xk - d, 0); x <= min(xk + d, Wh - 1); x++) {
            const int pj = y * Wh + x;
            const float h = heat[pj];
            if (pj != pk && h >= thresh && before(h, pj, ck, pk)) {
                if (out && cnt < HN) out[cnt] = pj;
                cnt++;
            }
        }
    return cnt;
}

// The same window queries against the candidate list held in LDS (row-major pixel order,
// row r's candidates at ids [s_row[r], s_row[r + 1])): per window row a binary search for
// the first column >= xk - d, then a scan to xk + d -- LDS reads instead of the (2d+1)^2
// scattered heat loads per candidate (each a 64-line gather per wave instruction).
// list: the higher-priority candidates' ids (the first HN to out), their count returned.
__device__ int list_higher_lds(const int *s_cp, const float *s_cc, const int *s_row, int Hh, int Wh, int d, int k,
                               int pk, float ck, int *__restrict__ out) {
    const int yk = pk / Wh, xk = pk % Wh, xa = max(xk - d, 0), xb = min(xk + d, Wh - 1);
    int cnt = 0;
    for (int yy = max(yk - d, 0); yy <= min(yk + d, Hh - 1); yy++) {
        int lo = s_row[yy], hi = s_row[yy + 1];
        const int end = hi, pa = yy * Wh + xa, pb = yy * Wh + xb;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_cp[mid] < pa) lo = mid + 1;
            else hi = mid;
        }
        for (int j = lo; j < end; j++) {
            const int pj = s_cp[j];
            if (pj > pb) break;
            if (j != k && before(s_cc[j], pj, ck, pk)) {
                if (out && cnt < HN) out[cnt] = j;
                cnt++;
            }
        }
    }
    return cnt;
}

// rescan (more than HN higher-priority neighbours): any of them kept / still undecided
__device__ void rescan_higher_lds(const int *s_cp, const float *s_cc, const int *s_row, const unsigned char *s_st,
                                  int Hh, int Wh, int d, int k, int pk, float ck, bool &supp, bool &blocked) {
    const int yk = pk / Wh, xk = pk % Wh, xa = max(xk - d, 0), xb = min(xk + d, Wh - 1);
    for (int yy = max(yk - d, 0); yy <= min(yk + d, Hh - 1); yy++) {
        int lo = s_row[yy], hi = s_row[yy + 1];
        const int end = hi, pa = yy * Wh + xa, pb = yy * Wh + xb;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_cp[mid] < pa) lo = mid + 1;
            else hi = mid;
        }
        for (int j = lo; j < end; j++) {
            const int pj = s_cp[j];
            if (pj > pb) break;
            if (j != k && before(s_cc[j], pj, ck, pk)) {
                const unsigned char sj = __atomic_load_n(&s_st[j], __ATOMIC_RELAXED);
                supp |= sj == 1;
                blocked |= sj == 0;
            }
        }
    }
}

__global__ __launch_bounds__(NMS_T) void k_kp_nms(int Hh, int Wh, int H, int W, float thresh, int nms_dist,
                                                  int border, int cap, const float *__restrict__ heat_all,
                                                  int *__restrict__ hn_all, int *__restrict__ hc_all,
                                                  int *__restrict__ cpix_all,
                                                  float *__restrict__ cconf_all, unsigned char *__restrict__ st_all,
                                                  int *__restrict__ kept_all, int *__restrict__ slot_pix_all,
                                                  int *__restrict__ num_kp, float *__restrict__ kp_out,
                                                  float *__restrict__ conf_out, int *__restrict__ status) {
    __shared__ int wsum[NMS_T / 64];
    __shared__ int s_base, s_flag, s_nk;
    __shared__ unsigned long long skey[SORT_N];  // bitonic keys (or the rank tiles)
    __shared__ int s_cp[NC_LDS];                 // LDS path: candidate pixels (row-major order)
    __shared__ float s_cc[NC_LDS];               //           their confidences
    __shared__ int s_row[ROW_LDS + 1];           //           first candidate id of each heat row
    __shared__ unsigned char s_st[NC_LDS];       //           state per candidate id
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const long P = (long)Hh * Wh;
    const float *heat = heat_all + b * P;
    const long HNC = hn_cands(P);
    int *hn = hn_all + b * HNC * HN;
    int *hcnt = hc_all + b * HNC;
    int *cpix = cpix_all + b * P;
    float *cconf = cconf_all + b * P;
    unsigned char *st = st_all + b * P;
    int *kept = kept_all + b * P;
    int *slot_pix = slot_pix_all + (long)b * cap;

    // (a) row-major compaction of the candidates in ONE pass over the heatmap: wave w owns a
    //     contiguous chunk of pixels, reads it with 8 float4 loads per lane in flight (a
    //     heatmap is ~1.9 MB per KITTI frame and one 1024-thread block per frame per CU has
    //     to keep that many bytes in flight), and writes its candidates in pixel order to its
    //     own segment of two scratch arrays free at this point (kept: pixel, hn: confidence
    //     bits); after the block scan each wave moves its segment to its final ids
    constexpr int NWV = NMS_T / 64, CU_ = 8;
    const long cw = ((P + NWV * 256 * CU_ - 1) / (NWV * 256 * CU_)) * (256 * CU_);  // pixels per wave
    const long q0 = min(P, (long)w * cw), q1 = min(P, q0 + cw);  // multiples of 4 (P = 64 Hc Wc)
    int *spix = kept + q0;
    float *sconf = reinterpret_cast<float *>(hn) + q0;  // hn holds >= P ints
    const unsigned long long lt = (1ull << lane) - 1ull;
    int cntw = 0;
    for (long p0 = q0; p0 < q1; p0 += 256 * CU_) {
        float4 h[CU_];
#pragma unroll
        for (int u = 0; u < CU_; u++)  // clamped: branch-free, so all CU_ loads are in flight
            h[u] = *reinterpret_cast<const float4 *>(heat + min(p0 + 256 * u + 4 * lane, q1 - 4));
#pragma unroll
        for (int u = 0; u < CU_; u++) {
            const long p = p0 + 256 * u + 4 * lane;
            const bool v = p < q1;
            const float hv[4] = {h[u].x, h[u].y, h[u].z, h[u].w};
            unsigned long long m[4];
            int r = cntw;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                m[e] = __ballot(v && hv[e] >= thresh);
                r += __popcll(m[e] & lt);  // candidates of lower lanes (pixels p0 + 256 u + < 4 lane)
            }
#pragma unroll
            for (int e = 0; e < 4; e++) {
                if (v && hv[e] >= thresh) {
                    spix[r] = (int)(p + e);
                    sconf[r] = hv[e];
                    st[p + e] = 0;
                    r++;
                }
                cntw += __popcll(m[e]);
            }
        }
    }
    if (lane == 0) wsum[w] = cntw;
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int k = 0; k < NWV; k++) {
            const int c = wsum[k];
            wsum[k] = acc;
            acc += c;
        }
        s_base = acc;
    }
    __syncthreads();
    const bool lds_path = s_base <= NC_LDS && Hh <= ROW_LDS;  // block-uniform
    {
        const int off = wsum[w];
        for (int i = lane; i < cntw; i += 64) {
            const int pp = spix[i];
            const float cc = sconf[i];
            cpix[off + i] = pp;
            cconf[off + i] = cc;
            if (lds_path) {
                s_cp[off + i] = pp;
                s_cc[off + i] = cc;
                s_st[off + i] = 0;
            }
        }
    }
    if (lds_path) {  // row index: s_row[y] = first id whose row is >= y (candidates are row-major)
        __syncthreads();
        const int ncl = s_base;
        if (ncl == 0) {
            for (int y = t; y <= Hh; y += NMS_T) s_row[y] = 0;
        } else {
            for (int k = t; k < ncl; k += NMS_T) {
                const int r = s_cp[k] / Wh, rp = k > 0 ? s_cp[k - 1] / Wh : -1;
                for (int y = rp + 1; y <= r; y++) s_row[y] = k;
                if (k == ncl - 1)
                    for (int y = r + 1; y <= Hh; y++) s_row[y] = ncl;
            }
        }
    }
    const int nc = s_base;

    // (b) greedy NMS as a fixed point over rounds.  Candidates and their priority are read
    //     straight from the heatmap (a pixel is a candidate iff heat >= thresh; ids are
    //     row-major, so pixel order is id order); states are kept per pixel.  Round 0 lists each
    //     candidate's higher-priority neighbours (all (2d+1)^2 heat values loaded at once) and
    //     keeps those without any; later rounds only read the listed neighbours' states.
    const int d = nms_dist;
    __syncthreads();
    for (int k = t; k < nc; k += NMS_T) {
        const int pk = cpix[k];
        const float ck = cconf[k];
        int cnt = 0;
        int *out = k < HNC ? hn + (long)k * HN : nullptr;
        if (lds_path)
            cnt = list_higher_lds(s_cp, s_cc, s_row, Hh, Wh, d, k, pk, ck, out);  // ids, not pixels
        else if (d == 4)
            cnt = list_higher<4>(heat, Hh, Wh, thresh, pk, ck, out);
        else
            cnt = list_higher_any(heat, Hh, Wh, thresh, d, pk, ck, out);
        if (k < HNC) hcnt[k] = cnt;  // > HN: the list is partial, rescanned each round
        if (cnt == 0) {
            if (lds_path) s_st[k] = 1;
            else st[pk] = 1;
        }
    }
    __syncthreads();
    for (;;) {
        if (t == 0) s_flag = 0;
        __syncthreads();
        int undecided = 0;
        for (int k = t; k < nc; k += NMS_T) {
            const int pk = lds_path ? s_cp[k] : cpix[k];
            if ((lds_path ? s_st[k] : st[pk]) != 0) continue;
            bool supp = false, blocked = false;
            const int c = k < HNC ? hcnt[k] : HN + 1;
            if (c <= HN) {
                int q[HN];  // the list in 16-B pieces (HN * 4 B per candidate: 16-B aligned)
                const int4 *h4 = reinterpret_cast<const int4 *>(hn + (long)k * HN);
#pragma unroll
                for (int i4 = 0; i4 < HN / 4; i4++) {
                    const int4 v = 4 * i4 < c ? h4[i4] : make_int4(-1, -1, -1, -1);
                    q[4 * i4] = 4 * i4 < c ? v.x : -1;
                    q[4 * i4 + 1] = 4 * i4 + 1 < c ? v.y : -1;
                    q[4 * i4 + 2] = 4 * i4 + 2 < c ? v.z : -1;
                    q[4 * i4 + 3] = 4 * i4 + 3 < c ? v.w : -1;
                }
#pragma unroll
                for (int i = 0; i < HN; i++) {
                    if (q[i] < 0) continue;
                    const unsigned char sj = lds_path ? __atomic_load_n(&s_st[q[i]], __ATOMIC_RELAXED)
                                                      : __atomic_load_n(&st[q[i]], __ATOMIC_RELAXED);
                    supp |= sj == 1;
                    blocked |= sj == 0;
                }
            } else if (lds_path) {
                rescan_higher_lds(s_cp, s_cc, s_row, s_st, Hh, Wh, d, k, pk, s_cc[k], supp, blocked);
            } else {  // more than HN higher neighbours: rescan the window
                const float ck = cconf[k];
                const int yk = pk / Wh, xk = pk % Wh;
                for (int yy = max(yk - d, 0); yy <= min(yk + d, Hh - 1); yy++)
                    for (int xx = max(xk - d, 0); xx <= min(xk + d, Wh - 1); xx++) {
                        const int pj = yy * Wh + xx;
                        const float h = heat[pj];
                        if (pj == pk || !(h >= thresh) || !before(h, pj, ck, pk)) continue;
                        const unsigned char sj = __atomic_load_n(&st[pj], __ATOMIC_RELAXED);
                        supp |= sj == 1;
                        blocked |= sj == 0;
                    }
            }
            const unsigned char ns = supp ? 2 : (!blocked ? 1 : 0);
            if (ns == 0)
                undecided = 1;
            else if (lds_path)
                s_st[k] = ns;
            else
                st[pk] = ns;
        }
        if (undecided) s_flag = 1;
        __syncthreads();
        if (!s_flag) break;
    }

    // (c) survivors inside the border; slot = rank (confidence desc, ties reversed row-major)
    if (t == 0) s_nk = 0;
    __syncthreads();
    for (int k = t; k < nc; k += NMS_T) {
        const int p = cpix[k], y = p / Wh, x = p % Wh;
        if ((lds_path ? s_st[k] : st[p]) != 1) continue;
        if (x < border || x >= W - border || y < border || y >= H - border) continue;
        kept[atomicAdd(&s_nk, 1)] = k;
    }
    __syncthreads();
    const int nk = s_nk;
    if (nk <= SORT_N) {
        // bitonic sort (descending) of (confidence bits << 32 | pixel): confidence descending,
        // ties in reversed row-major order; heat >= 0, so the float bits order as integers
        int n2 = 1;
        while (n2 < nk) n2 <<= 1;
        for (int k = t; k < n2; k += NMS_T) {
            unsigned long long key = 0ull;
            if (k < nk) {
                const int j = kept[k];
                key = ((unsigned long long)__float_as_uint(cconf[j]) << 32) | (unsigned)cpix[j];
            }
            skey[k] = key;
        }
        __syncthreads();
        for (int size = 2; size <= n2; size <<= 1)
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int i = t; i < n2 / 2; i += NMS_T) {
                    const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                    const bool desc = (lo & size) == 0;
                    const unsigned long long x = skey[lo], y = skey[hi];
                    if ((x < y) == desc) {
                        skey[lo] = y;
                        skey[hi] = x;
                    }
                }
                __syncthreads();
            }
        for (int r = t; r < min(nk, cap); r += NMS_T) {
            const unsigned long long key = skey[r];
            const int pm = (int)(unsigned)(key & 0xffffffffu);
            const long o = (long)b * cap + r;
            kp_out[2 * o] = (float)(pm % Wh);
            kp_out[2 * o + 1] = (float)(pm / Wh);
            conf_out[o] = __uint_as_float((unsigned)(key >> 32));
            slot_pix[r] = pm;
        }
    } else {
        // many survivors: slot = number ranked before (LDS tiles of the survivor list)
        float *t_conf = reinterpret_cast<float *>(skey);
        int *t_pix = reinterpret_cast<int *>(skey) + NMS_T;
        for (int k0 = 0; k0 < nk; k0 += NMS_T) {
            const int k = k0 + t;
            const int my = k < nk ? kept[k] : 0;
            const float cm = k < nk ? cconf[my] : 0.f;
            const int pm = k < nk ? cpix[my] : 0;
            int rank = 0;
            for (int j0 = 0; j0 < nk; j0 += NMS_T) {
                __syncthreads();
                if (j0 + t < nk) {
                    const int j = kept[j0 + t];
                    t_conf[t] = cconf[j];
                    t_pix[t] = cpix[j];
                }
                __syncthreads();
                const int lim = min(NMS_T, nk - j0);
                for (int q = 0; q < lim; q++) {
                    const float cq = t_conf[q];
                    rank += (cq > cm || (cq == cm && t_pix[q] > pm)) ? 1 : 0;
                }
            }
            if (k < nk && rank < cap) {
                const long o = (long)b * cap + rank;
                kp_out[2 * o] = (float)(pm % Wh);
                kp_out[2 * o + 1] = (float)(pm / Wh);
                conf_out[o] = cm;
                slot_pix[rank] = pm;
            }
        }
    }
    if (t == 0) {
        num_kp[b] = min(nk, cap);
        status[b] = nk > cap ? MV_ERR_CAPACITY : MV_OK;
    }
}

// grid_sample's coordinate arithmetic for a keypoint at heatmap pixel pix (row-major, Wh
// wide): pairwise_pnp.py:245-246's normalisation to [-1, 1] (double, rounded to float),
// torch's unnormalise (align_corners = False: one fma), floor, and the 4 corner weights
__device__ __forceinline__ void kp_geometry(int pix, int Hc, int Wc, int H, int W, int Wh, int &x0, int &y0,
                                            float w[4]) {
    const double x = (double)(pix % Wh), y = (double)(pix / Wh);
    const float gx = (float)(x / ((double)W / 2.) - 1.), gy = (float)(y / ((double)H / 2.) - 1.);
    const float ix = fmaf(gx + 1.f, (float)Wc / 2.f, -0.5f), iy = fmaf(gy + 1.f, (float)Hc / 2.f, -0.5f);
    const float x0f = floorf(ix), y0f = floorf(iy);
    const float wx = ix - x0f, e = 1.f - wx, n = iy - y0f, s = 1.f - n;
    w[0] = s * e;
    w[1] = s * wx;
    w[2] = n * e;
    w[3] = n * wx;
    x0 = (int)x0f;
    y0 = (int)y0f;
}

// torch grid_sample's CPU arithmetic for 4 channels: a product, then an fma chain over the
// other three corners (nw, ne, sw, se)
__device__ __forceinline__ float4 kp_bilinear4(float4 a, float4 bq, float4 c, float4 dd, float wnw, float wne,
                                               float wsw, float wse) {
    float v[4];
    const float *A = &a.x, *Bv = &bq.x, *C = &c.x, *Dv = &dd.x;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float r = __fmul_rn(A[i], wnw);
        r = fmaf(Bv[i], wne, r);
        r = fmaf(C[i], wsw, r);
        v[i] = fmaf(Dv[i], wse, r);
    }
    return make_float4(v[0], v[1], v[2], v[3]);
}

// a wave's 256-channel row (lane holds channels 4 lane .. 4 lane + 3): L2 norm with the
// reference's sequential sum of squares (numpy axis-0 reduce) in one lane, IEEE sqrt and
// division, stored to out
__device__ __forceinline__ void kp_normalize_store(float4 v, float *sq, float &nrm, int lane, float *out) {
    sq[4 * lane + 0] = __fmul_rn(v.x, v.x);
    sq[4 * lane + 1] = __fmul_rn(v.y, v.y);
    sq[4 * lane + 2] = __fmul_rn(v.z, v.z);
    sq[4 * lane + 3] = __fmul_rn(v.w, v.w);
    // wave-local LDS hand-off (waves of the block retire independently: no block barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
        float ss = 0.f;
        for (int ch = 0; ch < 256; ch++) ss = __fadd_rn(ss, sq[ch]);  // numpy's sequential axis-0 sum
        nrm = sqrtf(ss);  // IEEE sqrt (-fhip-fp32-correctly-rounded-divide-sqrt; __fsqrt_rn is the native one here)
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float m = nrm;
    float4 o;
    o.x = __fdiv_rn(v.x, m);
    o.y = __fdiv_rn(v.y, m);
    o.z = __fdiv_rn(v.z, m);
    o.w = __fdiv_rn(v.w, m);
    *reinterpret_cast<float4 *>(out + 4 * lane) = o;
}

// [B][256][HW] -> [B][HW][256], 64 x 64 tiles
__global__ __launch_bounds__(256) void k_kp_nhwc(int HW, const float *__restrict__ in, float *__restrict__ out) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z, c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
    const float *I = in + (long)b * 256 * HW;
    float *O = out + (long)b * HW * 256;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int p = p0 + tx;
        tile[r][tx] = p < HW ? I[(long)(c0 + r) * HW + p] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int p = p0 + r;
        if (p < HW) O[(long)p * 256 + c0 + tx] = tile[tx][r];
    }
}

// one wave per keypoint on the transposed (NHWC) rows: 4 corners x 256 channels, 16 B per lane
// (gathering the corners straight from the NCHW planes measured 2.09 ms against 0.81 + 0.24 ms
// transposed per 256 KITTI frames: 64 channel planes per gather)
__global__ __launch_bounds__(256) void k_kp_sample(int B, int cap, int Hc, int Wc, int H, int W, int Wh,
                                                   const int *__restrict__ num_kp, const int *__restrict__ slot_pix,
                                                   const float *__restrict__ nhwc, float *__restrict__ desc) {
    __shared__ float sq[4][256];
    __shared__ float nrm[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long q = (long)blockIdx.x * 4 + wv;
    if (q >= (long)B * cap) return;
    const int b = (int)(q / cap), slot = (int)(q % cap);
    if (slot >= num_kp[b]) return;  // wave-uniform
    int x0, y0;
    float w[4];
    kp_geometry(slot_pix[q], Hc, Wc, H, W, Wh, x0, y0, w);
    const float wnw = w[0], wne = w[1], wsw = w[2], wse = w[3];
    const float *D = nhwc + (long)b * Hc * Wc * 256 + 4 * lane;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    auto at = [&](int yy, int xx) {
        if (!(xx >= 0 && xx < Wc && yy >= 0 && yy < Hc)) return z;
        return *reinterpret_cast<const float4 *>(D + ((long)yy * Wc + xx) * 256);
    };
    const float4 v = kp_bilinear4(at(y0, x0), at(y0, x0 + 1), at(y0 + 1, x0), at(y0 + 1, x0 + 1), wnw, wne, wsw, wse);
    kp_normalize_store(v, sq[wv], nrm[wv], lane, desc + q * 256);
}

// 4 channels per workgroup, all keypoints of its frame: the channels' planes -- 4 Hc Wc
// contiguous floats of the network's [256][Hc][Wc] output -- are copied once into LDS with
// 16-B loads (16 in flight per thread: one workgroup per CU fills the LDS, so the bytes in
// flight have to come from the loads themselves), and each keypoint's 4 raw bilinear values
// are written to its descriptor row (16 B); k_kp_normalize then finishes the rows in place.
// Replaces the NCHW->NHWC transpose (7.4 MB read + 7.4 MB written per KITTI frame) and the
// 4 KiB corner reads per keypoint by one 7.4 MB read.  XCD-aware: the 8 channel quads that
// share a 128-B line of every descriptor row run on one XCD (consecutively on it), so their
// 16-B pieces merge in that XCD's L2 instead of leaving 8 partial lines.
template <int CH>
struct KpCh {
    float v[CH];
};
// CELLS: the LDS capacity in cells -- KP_PLANE_CELLS (one 144 KiB workgroup per CU) or
// KP_PLANE_CELLS_S for frames of at most that many cells (the network at 192 x 640: 24 x 80 =
// 1920 cells, 32 KiB: several workgroups per CU, whose copies and samples overlap)
template <int CH, int CELLS>
__global__ __launch_bounds__(256) void k_kp_sample_planes(int B, int cap, int Hc, int Wc, int H, int W, int Wh,
                                                          const int *__restrict__ num_kp,
                                                          const int *__restrict__ slot_pix,
                                                          const float *__restrict__ coarse, float *__restrict__ desc) {
    __shared__ __attribute__((aligned(16))) float plf[CH * CELLS + 4];
    constexpr int LG = 32 / CH;  // workgroups whose pieces share a 128-B line of a row
    const int i = blockIdx.x, xcd = i & 7, k = i >> 3;
    const int G = xcd + 8 * (k / LG);  // (frame, line group)
    const int b = G >> 3, cb = (G & 7) * LG + k % LG;
    if (b >= B) return;
    const int nk = min(num_kp[b], cap);
    if (nk <= 0) return;  // block-uniform
    const int HW = Hc * Wc, c0 = cb * CH, nf = CH * HW;
    // the first KPF slots of every thread: pixel loads issued and the bilinear geometry
    // (grid_sample's unnormalise, floor, weights) computed before the plane copy, so that
    // their latency hides under it
    constexpr int KPF = 4;
    int gx0[KPF], gy0[KPF];
    float gw[KPF][4];  // nw, ne, sw, se
    int gpix[KPF];
#pragma unroll
    for (int u = 0; u < KPF; u++)  // branch-free (clamped) so the KPF loads are in flight together
        gpix[u] = slot_pix[(long)b * cap + min((int)threadIdx.x + 256 * u, nk - 1)];
#pragma unroll
    for (int u = 0; u < KPF; u++) {
        kp_geometry(gpix[u], Hc, Wc, H, W, Wh, gx0[u], gy0[u], gw[u]);
    }
    const float *I = coarse + ((long)b * 256 + c0) * HW;  // 4-B aligned
    // I[h] is the first 16-B aligned float; I[f] goes to plf[f + o] with h + o in {0, 4}, so
    // the aligned body lands on 16-B aligned LDS slots.  Head and tail (< 4 floats each) are
    // copied one float at a time: nothing outside [I, I + nf) is read.
    const int h = (int)(((16 - ((uintptr_t)I & 15)) & 15) >> 2), o = (4 - h) & 3;
    const int n4 = (nf - h) >> 2, tail = nf - h - 4 * n4;
    const float4 *G4 = reinterpret_cast<const float4 *>(I + h);
    float4 *L4 = reinterpret_cast<float4 *>(plf + h + o);
    // 16 loads in flight per thread to the end: past n4 the index is clamped, so a lane
    // re-copies float4 n4 - 1 onto itself -- branch-free, or the compiler sinks each load
    // into its store's branch and serialises them
    for (int j = threadIdx.x; j < n4; j += 16 * 256) {
        float4 t[16];
#pragma unroll
        for (int u = 0; u < 16; u++) t[u] = G4[min(j + u * 256, n4 - 1)];
#pragma unroll
        for (int u = 0; u < 16; u++) L4[min(j + u * 256, n4 - 1)] = t[u];
    }
    if (threadIdx.x < h) plf[threadIdx.x + o] = I[threadIdx.x];
    if (threadIdx.x < tail) plf[h + 4 * n4 + o + threadIdx.x] = I[h + 4 * n4 + threadIdx.x];
    __syncthreads();
    const float *L = plf + o;  // plane c of the group: L + c HW
    auto at = [&](int yy, int xx) {
        KpCh<CH> r;
        const bool in = xx >= 0 && xx < Wc && yy >= 0 && yy < Hc;
        const float *c = L + (in ? yy * Wc + xx : 0);
#pragma unroll
        for (int j = 0; j < CH; j++) r.v[j] = in ? c[j * HW] : 0.f;
        return r;
    };
    auto emit = [&](int slot, int x0, int y0, const float *w) {
        const KpCh<CH> a = at(y0, x0), bq = at(y0, x0 + 1), c = at(y0 + 1, x0), dd = at(y0 + 1, x0 + 1);
        KpCh<CH> v;
#pragma unroll
        for (int j = 0; j < CH; j++) {  // torch grid_sample's CPU arithmetic (as kp_bilinear4)
            float r = __fmul_rn(a.v[j], w[0]);
            r = fmaf(bq.v[j], w[1], r);
            r = fmaf(c.v[j], w[2], r);
            v.v[j] = fmaf(dd.v[j], w[3], r);
        }
        float *out = desc + ((long)b * cap + slot) * 256 + c0;
        if constexpr (CH == 4)
            *reinterpret_cast<float4 *>(out) = make_float4(v.v[0], v.v[1], v.v[2], v.v[3]);
        else
            *reinterpret_cast<float2 *>(out) = make_float2(v.v[0], v.v[1]);
    };
#pragma unroll
    for (int u = 0; u < KPF; u++) {
        const int slot = threadIdx.x + 256 * u;
        if (slot < nk) emit(slot, gx0[u], gy0[u], gw[u]);
    }
    for (int slot = threadIdx.x + 256 * KPF; slot < nk; slot += 256) {  // cap > 1024
        int x0, y0;
        float w[4];
        kp_geometry(slot_pix[(long)b * cap + slot], Hc, Wc, H, W, Wh, x0, y0, w);
        emit(slot, x0, y0, w);
    }
}

// one wave per keypoint: the raw row written by k_kp_sample_planes, normalised in place
__global__ __launch_bounds__(256) void k_kp_normalize(int B, int cap, const int *__restrict__ num_kp,
                                                      float *__restrict__ desc) {
    __shared__ float sq[4][256];
    __shared__ float nrm[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long q = (long)blockIdx.x * 4 + wv;
    if (q >= (long)B * cap) return;
    const int b = (int)(q / cap), slot = (int)(q % cap);
    if (slot >= num_kp[b]) return;  // wave-uniform
    const float4 v = *reinterpret_cast<const float4 *>(desc + q * 256 + 4 * lane);
    kp_normalize_store(v, sq[wv], nrm[wv], lane, desc + q * 256);
}

}  // namespace

extern "C" void mv_kp_params_default(mv_kp_params *p) {
    if (!p) return;
    p->conf_thresh = 0.015f;
    p->nms_dist = 4;
    p->border = 4;
}

extern "C" int mv_keypoints_dev(mv_context *ctx, const mv_kp_params *p, int batch, int Hc, int Wc, int H, int W,
                                const float *semi, const float *coarse_desc, int cap, int *num_kp, float *kp,
                                float *conf, float *desc, float *heat, int *status) {
    MV_REQUIRE(ctx && p && batch > 0 && Hc > 0 && Wc > 0 && cap > 0 && semi && coarse_desc && num_kp && kp && conf &&
               desc && status);
    MV_REQUIRE(Hc * 8 <= H && Wc * 8 <= W && p->nms_dist >= 0 && p->border >= 0);
    MV_REQUIRE((long)Hc * Wc * 64 < (1l << 30) && (long)batch * cap < (1l << 31));
    MV_REQUIRE(((uintptr_t)coarse_desc & 3) == 0 && ((uintptr_t)desc & 15) == 0 && ((uintptr_t)heat & 15) == 0);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    char *scr = (char *)mv::scratch(ctx, kp_scratch_bytes(batch, Hc, Wc, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    const KpScratch m = kp_scratch_map(scr, batch, Hc, Wc, cap);
    float *hm = heat ? heat : m.heat;
    hipStream_t s = ctx->stream;
    const long cells = (long)batch * Hc * Wc;
    MV_PROF_BEGIN(s, "k_kp_heat");
    hipLaunchKernelGGL(k_kp_heat, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, cells, Hc, Wc, semi, hm);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    MV_PROF_BEGIN(s, "k_kp_nms");
    hipLaunchKernelGGL(k_kp_nms, dim3((unsigned)batch), dim3(NMS_T), 0, s, Hc * 8, Wc * 8, H, W, p->conf_thresh,
                       p->nms_dist, p->border, cap, hm, m.hn, m.hc, m.cpix, m.cconf, m.st, m.kept, m.slot_pix, num_kp, kp,
                       conf, status);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    const int HW = Hc * Wc;
    const long waves = (long)batch * cap;
    if (kp_planes_path(Hc, Wc)) {
        MV_PROF_BEGIN(s, "k_kp_sample_planes");
        if (HW <= KP_PLANE_CELLS_S)
            hipLaunchKernelGGL((k_kp_sample_planes<KP_CH, KP_PLANE_CELLS_S>),
                               dim3((unsigned)batch * (256 / KP_CH)), dim3(256), 0, s, batch, cap, Hc, Wc, H, W, Wc * 8,
                               num_kp, m.slot_pix, coarse_desc, desc);
        else
            hipLaunchKernelGGL((k_kp_sample_planes<KP_CH, KP_PLANE_CELLS>), dim3((unsigned)batch * (256 / KP_CH)),
                               dim3(256), 0, s, batch, cap, Hc, Wc, H, W, Wc * 8, num_kp, m.slot_pix, coarse_desc, desc);
        MV_PROF_END(s);
        MV_LAUNCH_CHECK();
        MV_PROF_BEGIN(s, "k_kp_normalize");
        hipLaunchKernelGGL(k_kp_normalize, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, batch, cap, num_kp,
                           desc);
        MV_PROF_END(s);
        MV_LAUNCH_CHECK();
        return mv::set_status(MV_OK);
    }
    MV_PROF_BEGIN(s, "k_kp_nhwc");
    hipLaunchKernelGGL(k_kp_nhwc, dim3((unsigned)((HW + 63) / 64), 4, (unsigned)batch), dim3(256), 0, s, HW,
                       coarse_desc, m.nhwc);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    MV_PROF_BEGIN(s, "k_kp_sample");
    hipLaunchKernelGGL(k_kp_sample, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, batch, cap, Hc,
                       Wc, H, W, Wc * 8, num_kp, m.slot_pix, m.nhwc, desc);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}

extern "C" int mv_keypoints_host(mv_context *ctx, const mv_kp_params *p, int Hc, int Wc, int H, int W,
                                 const float *semi, const float *coarse_desc, int cap, int *num_kp, float *kp,
                                 float *conf, float *desc) {
    MV_REQUIRE(ctx && p && Hc > 0 && Wc > 0 && cap > 0 && semi && coarse_desc && num_kp && kp && conf && desc);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const size_t plane = (size_t)Hc * Wc;
    const size_t bs = a256(65 * plane * 4), bd = a256(256 * plane * 4), bk = a256((size_t)cap * 8),
                 bc = a256((size_t)cap * 4), bo = a256((size_t)cap * 1024);
    char *d = (char *)mv::stage(ctx, bs + bd + bk + bc + bo + 512);
    if (!d) return MV_ERR_OUT_OF_MEMORY;
    float *d_semi = (float *)d, *d_desc = (float *)(d + bs), *d_kp = (float *)(d + bs + bd),
          *d_conf = (float *)(d + bs + bd + bk), *d_out = (float *)(d + bs + bd + bk + bc);
    int *d_n = (int *)(d + bs + bd + bk + bc + bo), *d_st = d_n + 64;
    hipStream_t s = ctx->stream;
    MV_HIP_TRY(hipMemcpyAsync(d_semi, semi, 65 * plane * 4, hipMemcpyHostToDevice, s));
    MV_HIP_TRY(hipMemcpyAsync(d_desc, coarse_desc, 256 * plane * 4, hipMemcpyHostToDevice, s));
    int st = mv_keypoints_dev(ctx, p, 1, Hc, Wc, H, W, d_semi, d_desc, cap, d_n, d_kp, d_conf, d_out, nullptr, d_st);
    if (st != MV_OK) return st;
    int n = 0, fst = 0;
    MV_HIP_TRY(hipMemcpyAsync(&n, d_n, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipMemcpyAsync(&fst, d_st, 4, hipMemcpyDeviceToHost, s));
    MV_HIP_TRY(hipStreamSynchronize(s));
    if (n > 0) {
        MV_HIP_TRY(hipMemcpyAsync(kp, d_kp, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        MV_HIP_TRY(hipMemcpyAsync(conf, d_conf, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        MV_HIP_TRY(hipMemcpyAsync(desc, d_out, (size_t)n * 1024, hipMemcpyDeviceToHost, s));
        MV_HIP_TRY(hipStreamSynchronize(s));
    }
    *num_kp = n;
    return mv::set_status(fst);
}
