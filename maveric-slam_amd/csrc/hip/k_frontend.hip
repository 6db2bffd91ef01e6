// k_frontend.hip -- the windowed int8 front end of src/tracking_main.c on gfx950:
//   k_softmax         approx softmax of every cell        (src/top_N.c:12-49,136-165)
//   k_top_n_select    validity filter + interpolated threshold + ordered
//                     compaction to N                     (src/top_N.c:53-134)
//   k_window_eval     one wave per query, lanes = window candidates
//                                                         (src/tracking_main.c:18-43,114-165)
//   k_window_compact  query-ordered compaction, cap MAX_NUM_MATCH
//                                                         (src/tracking_main.c:167-192)
// All float arithmetic keeps the reference's evaluation order; the TU is built
// with -ffp-contract=off and IEEE division.  Data are int8 and HBM/L2 bound:
// no MFMA here (the window dot is 64..256 int8 MACs per candidate, v_dot4).
#include "mv_internal.hpp"


namespace {

constexpr int kSemiC = 65;
constexpr int kDescD = 256;

// top_N.c:59-63 ; :12-20
__device__ __forceinline__ void scale_poly(float scale, float sp[5]) {
    sp[0] = 1.0f;
#pragma unroll
    for (int i = 1; i < 5; i++) sp[i] = sp[i - 1] * scale / (float)i;
}

__device__ __forceinline__ float approx_exp(const float sp[5], int x) {
    float acc = 1.0f;
    int xp = x;
    acc += sp[1] * (float)xp;
    xp *= x;
    acc += sp[2] * (float)xp;
    xp *= x;
    acc += sp[3] * (float)xp;
    xp *= x;
    acc += sp[4] * (float)xp;
    return acc;
}

// ---------------------------------------------------------------------------
// k_softmax: block = 256 consecutive (frame, cell) rows of 65 int8, staged into LDS by
// LDS DMA (16,640 B per block, 16-B aligned).  The reference walks all 65 logits, skipping
// the negative ones (top_N.c:29-41); here each lane first builds its row's 64-bit mask of
// non-negative logits from 16 aligned dwords (sign bits, four logits per dword) and then
// visits only those, in ascending order -- so the float sum and the strict-max updates
// happen in exactly the reference's order -- computing approx_exp arithmetically (the same
// expression, the same bits).  Logit 64 (the dustbin) is added last and never wins the max.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_softmax(int total_rows, int cells, const float *__restrict__ scales,
                                                 const int8_t *__restrict__ semi, int *__restrict__ max_idx,
                                                 float *__restrict__ probs, int *__restrict__ num_valid) {
    __shared__ __attribute__((aligned(16))) int lds32[256 * kSemiC / 4 + 4];
    __shared__ float sp_s[2][5];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const long r0 = (long)blockIdx.x * 256;
    const int nrows = (int)min((long)256, (long)total_rows - r0);
    const int nbytes = nrows * kSemiC;
    const long base = r0 * kSemiC;  // multiple of 16 (256*65 = 16640)
    if (nrows == 256) {
        // 1040 16-B pieces: 4 per lane + 16 (wave 0, lanes 0..15); non-temporal (each logit is
        // read once): 0.913 -> 0.882 ms per 8192 frames, profiles/r06w_softmax_nt_ab.log
        const int8_t *src = semi + base;
        char *dst = reinterpret_cast<char *>(lds32);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int piece = i * 256 + w * 64;  // this wave's 64 pieces of pass i
            __builtin_amdgcn_global_load_lds(src + (long)(piece + lane) * 16, dst + piece * 16, 16, 0, 2);
        }
        if (w == 0 && lane < 16) __builtin_amdgcn_global_load_lds(src + (1024 + lane) * 16, dst + 1024 * 16, 16, 0, 2);
    } else {
        const int *g32 = reinterpret_cast<const int *>(semi + base);
        for (int i = t; i < nbytes / 4; i += 256) lds32[i] = g32[i];
        for (int i = (nbytes / 4) * 4 + t; i < nbytes; i += 256)
            reinterpret_cast<int8_t *>(lds32)[i] = semi[base + i];
    }
    const int f_first = (int)(r0 / cells);
    if (t < 2) {  // the polynomial of the (at most two) frames the block spans (top_N.c:59-63)
        const int f = f_first + t;
        if ((long)f * cells < (long)total_rows) {
            float sp[5];
            scale_poly(scales[f], sp);
#pragma unroll
            for (int i = 0; i < 5; i++) sp_s[t][i] = sp[i];
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t >= nrows) return;
    const long r = r0 + t;
    const int frame = (int)(r / cells);
    const int fl = frame - f_first;  // < 2 whenever cells >= 256
    float sp[5];
    if (fl < 2) {
#pragma unroll
        for (int i = 0; i < 5; i++) sp[i] = sp_s[fl][i];
    } else {
        scale_poly(scales[frame], sp);  // tiny frames
    }
    // the row's 65 bytes: dwords re-aligned to the row start.  First a 16-bit mask of the dwords
    // holding a non-negative logit (4 VALU per dword: alignbyte, bfi = ~u & 0x80808080, min, shift-or),
    // then those dwords' non-negative bytes in ascending order (most logits are negative: typically
    // 1-3 dwords per row)
    const int rb = t * kSemiC, o = rb & 3, d0 = rb >> 2;
    unsigned dm = 0;
    unsigned wv = (unsigned)lds32[d0];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const unsigned wn = (unsigned)lds32[d0 + j + 1];
        const unsigned u = __builtin_amdgcn_alignbyte(wn, wv, o);  // bytes 4j .. 4j+3 of the row
        wv = wn;
        const unsigned nn = ~u & 0x80808080u;
        dm |= min(nn, 1u) << j;
    }
    const int8_t *row = reinterpret_cast<const int8_t *>(lds32) + rb;
    int best = 64;
    float best_e = 0.0f;
    float den = 1.17549435e-38f;  // FLT_MIN (top_N.c:30)
    while (dm) {
        const int j = __builtin_ctz(dm);
        dm &= dm - 1;
        const unsigned u = __builtin_amdgcn_alignbyte((unsigned)lds32[d0 + j + 1], (unsigned)lds32[d0 + j], o);
        unsigned nn = ~u & 0x80808080u;  // bit 8 k + 7: byte k of the dword is >= 0
        while (nn) {
            const int i = 4 * j + (__builtin_ctz(nn) >> 3);
            nn &= nn - 1;
            const float e = approx_exp(sp, (int)row[i]);
            if (e > best_e) {
                best_e = e;
                best = i;
            }
            den += e;
        }
    }
    const int x64 = (int)row[64];
    if (x64 >= 0) den += approx_exp(sp, x64);
    max_idx[r] = best;
    probs[r] = best != 64 ? best_e / den : -1.0f;
    // (*num_valid)++ per valid cell (top_N.c:160): one atomic per wave and frame, not per
    // cell (per-cell atomics on one counter per frame serialise in L2)
    const bool v = best != 64;
    const int f0 = __shfl(frame, 0, 64);
    const unsigned long long vm = __ballot(v);
    if (__ballot(frame != f0) == 0) {  // the whole active wave is one frame (cells >= 64: common)
        if ((threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1 && vm)
            atomicAdd(&num_valid[f0], __popcll(vm));
    } else if (v) {
        atomicAdd(&num_valid[frame], 1);
    }
}

// ---------------------------------------------------------------------------
// Block-wide exclusive scan helper (1024 threads = 16 waves).
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ int block_exclusive_scan(int v, int *total, int *wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
        int s = lane < NT / 64 ? wsum[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < NT / 64) wsum[lane] = s;  // inclusive wave prefix
    }
    __syncthreads();
    int off = (w > 0 ? wsum[w - 1] : 0) + x - v;
    *total = wsum[NT / 64 - 1];
    __syncthreads();
    return off;
}

// k_top_n_select: ONE WAVE per frame (4 frames per 256-thread block, no block barrier): the frame's
// cells in chunks of 64 consecutive ones (coalesced loads), a ballot of the valid cells per chunk
// -- so the selection keeps patch order by construction: a selected cell's slot is the running
// count plus the popcount of the ballot below its lane (mbcnt).  Pass 1 counts the valid cells
// (top_N.c:71-73: index != 64 and prob > 0.01, double compare) and their min / max prob; pass 2
// (the frame's 58 KB again, from L2) writes every valid cell when they are at most N, otherwise
// those with prob >= the interpolated threshold (top_N.c:95-133) until N are written.
// (Round 5: one 1024-thread block per frame, two block-wide scans -- 0.348 ms per 8192 frames,
// latency-bound.)
__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__global__ __launch_bounds__(256) void k_top_n_select(int batch, int cells, const int *__restrict__ max_idx,
                                                      const float *__restrict__ probs, int N, int cap,
                                                      int *__restrict__ num_sel, int *__restrict__ patches,
                                                      int *__restrict__ indices, float *__restrict__ sel_probs,
                                                      int *__restrict__ status) {
    const int lane = threadIdx.x & 63;
    const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= batch) return;  // wave-uniform
    const int *mi = max_idx + (long)f * cells;
    const float *pr = probs + (long)f * cells;
    int nv = 0;
    float pmax = 0.0f, pmin = 3.40282347e+38f;  // FLT_MAX
    constexpr int U = 4;                        // chunks in flight
    for (int base = 0; base < cells; base += 64 * U) {
        int idx[U];
        float p[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int c = base + 64 * u + lane;
            idx[u] = c < cells ? mi[c] : 64;
            p[u] = c < cells ? pr[c] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool v = idx[u] != 64 && (double)p[u] > 0.01;
            nv += __popcll(__ballot(v));
            if (v) {
                pmax = fmaxf(pmax, p[u]);
                pmin = fminf(pmin, p[u]);
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // exact, order-independent
        pmax = fmaxf(pmax, __shfl_xor(pmax, o, 64));
        pmin = fminf(pmin, __shfl_xor(pmin, o, 64));
    }
    if (nv >= cap) {  // the reference exits here (top_N.c:91-94)
        if (lane == 0) {
            num_sel[f] = 0;
            status[f] = MV_ERR_CAPACITY;
        }
        return;
    }
    const bool all = nv <= N;
    const float split = (float)N / (float)nv;
    const float thr = all ? 0.0f : pmax * split + pmin * (1 - split);
    int *op = patches + (long)f * N;
    int *oi = indices + (long)f * N;
    float *opr = sel_probs + (long)f * N;
    int k = 0;  // cells selected so far (wave-uniform)
    for (int base = 0; base < cells && k < N; base += 64 * U) {
        int idx[U];
        float p[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int c = base + 64 * u + lane;
            idx[u] = c < cells ? mi[c] : 64;
            p[u] = c < cells ? pr[c] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool sel = idx[u] != 64 && (double)p[u] > 0.01 && (all || p[u] >= thr);
            const unsigned long long m = __ballot(sel);
            const int pos = k + lanes_below(m);
            if (sel && pos < N) {
                op[pos] = base + 64 * u + lane;
                oi[pos] = idx[u];
                opr[pos] = p[u];
            }
            k += __popcll(m);
        }
    }
    if (lane == 0) {
        num_sel[f] = all ? nv : min(k, N);
        status[f] = MV_OK;
    }
}

// ---------------------------------------------------------------------------
// Windowed match.
// ---------------------------------------------------------------------------
struct WinArgs {
    int rows, cols, N;
    int shift_x, shift_y, radius, as_built;
    double thr_sq, prob_thr;
};

struct QueryResult {  // one per (pair, query slot), consumed by k_window_compact
    int found, bx, by, best_patch;  // best_patch: frame-0 patch of the winner (compact reads its index)
    float score;
};

__device__ __forceinline__ int wrap_mul(int a, int b) { return (int)((unsigned)a * (unsigned)b); }

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// strict "a better than b" for as-intended (dot^2/na) with tie -> lower order
__device__ __forceinline__ bool exact_better(long long da, long long na, int ka, long long db, long long nb,
                                             int kb) {
    if (ka < 0) return false;
    if (kb < 0) return true;
    unsigned __int128 l = (unsigned __int128)(unsigned long long)(da * da) * (unsigned long long)nb;
    unsigned __int128 r = (unsigned __int128)(unsigned long long)(db * db) * (unsigned long long)na;
    if (l != r) return l > r;
    return ka < kb;
}

// Candidate source for the per-query evaluation: frame 0 straight from global memory (L2
// serves the overlap of neighbouring windows).  An LDS-tiled variant (union of an 8x8 query
// tile's windows DMA'd once) measured 2x slower at 14 % query density: see DESIGN.md.
struct GlobalCands {
    const int8_t *d0;  // this pair's frame-0 descriptors
    const int *mi0;
    const float *pr0;
    int rows;
    double prob_thr;
    __device__ __forceinline__ bool valid(int, int, int p) const {
        return mi0[p] != 64 && !((double)pr0[p] < prob_thr);
    }
    __device__ __forceinline__ int4 chunk(int x, int y, int j) const {
        return reinterpret_cast<const int4 *>(d0 + ((long)x * rows + y) * kDescD)[j];
    }
    __device__ __forceinline__ int dword(int x, int y, int i) const {
        return reinterpret_cast<const int *>(d0 + ((long)x * rows + y) * kDescD)[i];
    }
    __device__ __forceinline__ const int8_t *row(int x, int y) const { return d0 + ((long)x * rows + y) * kDescD; }
};
// dot and squared norm of the first 64 int8 (4 chunks) against q (16 dwords)
template <class CS>
__device__ __forceinline__ void dot64c(const CS &C, int x, int y, const int *q, int &dot, int &nrm) {
#pragma unroll
    for (int v = 0; v < 4; v++) {
        int4 c = C.chunk(x, y, v);
        dot = __builtin_amdgcn_sdot4(c.x, q[4 * v + 0], dot, false);
        dot = __builtin_amdgcn_sdot4(c.y, q[4 * v + 1], dot, false);
        dot = __builtin_amdgcn_sdot4(c.z, q[4 * v + 2], dot, false);
        dot = __builtin_amdgcn_sdot4(c.w, q[4 * v + 3], dot, false);
        nrm = __builtin_amdgcn_sdot4(c.x, c.x, nrm, false);
        nrm = __builtin_amdgcn_sdot4(c.y, c.y, nrm, false);
        nrm = __builtin_amdgcn_sdot4(c.z, c.z, nrm, false);
        nrm = __builtin_amdgcn_sdot4(c.w, c.w, nrm, false);
    }
}

// One query (a whole wave): tracking_main.c:114-165 on the window of frame-1 cell (x1, y1).
// Returns the result in every lane; best_patch is the frame-0 patch of the winner.
template <class CS>
__device__ __forceinline__ QueryResult eval_query(const WinArgs &a, const CS &C, const int8_t *qd, int x1, int y1,
                                                  int lane, int &best_patch_out) {
    QueryResult res = {0, 0, 0, -1, 0.0f};
    // query: lane holds dword `lane` (bytes 4*lane .. 4*lane+3) for cooperative 256-D work,
    // and every lane holds the first 64 bytes for the per-candidate 64-D dot.
    const int qv = reinterpret_cast<const int *>(qd)[lane];
    int q64[16];
#pragma unroll
    for (int v = 0; v < 16; v++) q64[v] = __shfl(qv, v, 64);
    const int n2_256 = wave_sum(__builtin_amdgcn_sdot4(qv, qv, 0, false));
    const int n2_64 = wave_sum(lane < 16 ? __builtin_amdgcn_sdot4(qv, qv, 0, false) : 0);
    int xlo = max(x1 + a.shift_x - a.radius, 0), xhi = min(x1 + a.shift_x + a.radius, a.cols - 1);
    int ylo = max(y1 + a.shift_y - a.radius, 0), yhi = min(y1 + a.shift_y + a.radius, a.rows - 1);
    const int ny = yhi - ylo + 1;
    const int ncand = (xhi >= xlo && yhi >= ylo) ? (xhi - xlo + 1) * ny : 0;

    // as-built latch state (carried across 64-candidate chunks)
    bool latched = false;
    int n1f = 0;
    // running best
    float best_d = 0.0f;
    int best_k = -1;
    long long best_dot = 0, best_na = 1;
    int best_patch = 0;

    for (int base = 0; base < ncand; base += 64) {
        const int k = base + lane;
        int patch0 = 0;
        bool valid = false;
        if (k < ncand) {
            const int x0 = xlo + k / ny, y0 = ylo + k % ny;
            patch0 = x0 * a.rows + y0;
            valid = C.valid(x0, y0, patch0);
        }
        const int cx0 = xlo + min(k, ncand - 1) / ny, cy0 = ylo + min(k, ncand - 1) % ny;
        float d = __builtin_nanf("");
        long long cdot = 0, cna = 0;
        if (a.as_built) {
            int dot_64 = 0, n1_64 = 0;
            if (valid) dot64c(C, cx0, cy0, q64, dot_64, n1_64);
            // resolve the latch: the first valid candidate (scan order) whose
            // full 256-D norm is non-zero computes the full dot; candidates
            // before it (all-zero descriptors) divide 0 by 0.
            unsigned long long vm = __ballot(valid);
            int f_lane = -1;   // lane of the latching candidate in this chunk
            int dot_f = 0;
            while (!latched && vm) {
                const int l = __ffsll((long long)vm) - 1;
                const int lx0 = __shfl(cx0, l, 64), ly0 = __shfl(cy0, l, 64);
                const int cv = C.dword(lx0, ly0, lane);
                const int full_n1 = wave_sum(__builtin_amdgcn_sdot4(cv, cv, 0, false));
                const int full_dot = wave_sum(__builtin_amdgcn_sdot4(cv, qv, 0, false));
                vm &= vm - 1;
                if (full_n1 != 0) {
                    latched = true;
                    n1f = full_n1;
                    f_lane = l;
                    dot_f = full_dot;
                } else if (lane == l) {
                    d = (float)wrap_mul(full_dot, full_dot) / (float)wrap_mul(full_n1, n2_256);
                }
            }
            if (valid) {
                if (lane == f_lane) {
                    d = (float)wrap_mul(dot_f, dot_f) / (float)wrap_mul(n1f, n2_256);
                } else if (latched && (f_lane < 0 || lane > f_lane)) {
                    d = (float)wrap_mul(dot_64, dot_64) / (float)wrap_mul(n1f, n2_64);
                }
            }
            bool pass = valid && (double)d > a.thr_sq;
            // first strict maximum in scan order: max d, ties -> smallest k
            float bd = pass ? d : -__builtin_inff();
            int bk = pass ? k : 0x7fffffff;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                float od = __shfl_xor(bd, o, 64);
                int ok = __shfl_xor(bk, o, 64);
                if (od > bd || (od == bd && ok < bk)) {
                    bd = od;
                    bk = ok;
                }
            }
            if (bk != 0x7fffffff && (best_k < 0 || bd > best_d)) {
                best_d = bd;
                best_k = bk;
                best_patch = __shfl(patch0, bk - base, 64);
            }
        } else {
            int dot = 0, na = 0;
            if (valid) {
                const int4 *q4 = reinterpret_cast<const int4 *>(qd);  // wave-uniform address
#pragma unroll
                for (int v = 0; v < 16; v++) {
                    int4 x = C.chunk(cx0, cy0, v), y = q4[v];
                    dot = __builtin_amdgcn_sdot4(x.x, y.x, dot, false);
                    dot = __builtin_amdgcn_sdot4(x.y, y.y, dot, false);
                    dot = __builtin_amdgcn_sdot4(x.z, y.z, dot, false);
                    dot = __builtin_amdgcn_sdot4(x.w, y.w, dot, false);
                    na = __builtin_amdgcn_sdot4(x.x, x.x, na, false);
                    na = __builtin_amdgcn_sdot4(x.y, x.y, na, false);
                    na = __builtin_amdgcn_sdot4(x.z, x.z, na, false);
                    na = __builtin_amdgcn_sdot4(x.w, x.w, na, false);
                }
            }
            cdot = dot;
            cna = na;
            bool pass = valid && dot > 0 && na != 0 && n2_256 != 0 &&
                        (unsigned __int128)(100ll * cdot * cdot) >
                            (unsigned __int128)81 * (unsigned long long)(cna * (long long)n2_256);
            long long bd = pass ? cdot : 0, bn = pass ? cna : 1;
            int bk = pass ? k : -1;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                long long od = __shfl_xor(bd, o, 64), on = __shfl_xor(bn, o, 64);
                int ok = __shfl_xor(bk, o, 64);
                if (exact_better(od, on, ok, bd, bn, bk)) {
                    bd = od;
                    bn = on;
                    bk = ok;
                }
            }
            if (bk >= 0 && exact_better(bd, bn, bk, best_dot, best_na, best_k)) {
                best_dot = bd;
                best_na = bn;
                best_k = bk;
                best_d = (float)((double)bd * (double)bd / ((double)bn * (double)n2_256));
                best_patch = __shfl(patch0, bk - base, 64);
            }
        }
    }
    if (best_k >= 0) {
        res.found = 1;
        res.bx = xlo + best_k / ny;
        res.by = ylo + best_k % ny;
        res.score = best_d;
    }
    best_patch_out = best_k >= 0 ? best_patch : -1;
    return res;
}

// As-intended query (tracking_main.c:114-165 with the exact cosine), latency-shaped: the
// validity of up to 128 window candidates is read at once (two per lane), the valid ones are
// compacted into a wave-local LDS list, and every valid candidate is scored by 4 lanes (64 B
// each, the query's matching 64 B held in registers): two dependent global round trips per
// query for up to 16 valid candidates, instead of validity -> descriptor per 64-candidate chunk.
template <class CS>
__device__ __forceinline__ QueryResult eval_query_intended(const WinArgs &a, const CS &C, const int8_t *qd, int x1,
                                                           int y1, int lane, int *lst, int &best_patch_out) {
    QueryResult res = {0, 0, 0, -1, 0.0f};
    const int q4 = lane & 3, cslot = lane >> 2;
    const int qv = reinterpret_cast<const int *>(qd)[lane];
    int4 qa[4];
#pragma unroll
    for (int v = 0; v < 4; v++) qa[v] = reinterpret_cast<const int4 *>(qd + 64 * q4)[v];
    const int n2_256 = wave_sum(__builtin_amdgcn_sdot4(qv, qv, 0, false));
    const int xlo = max(x1 + a.shift_x - a.radius, 0), xhi = min(x1 + a.shift_x + a.radius, a.cols - 1);
    const int ylo = max(y1 + a.shift_y - a.radius, 0), yhi = min(y1 + a.shift_y + a.radius, a.rows - 1);
    const int ny = yhi - ylo + 1;
    const int ncand = (xhi >= xlo && yhi >= ylo) ? (xhi - xlo + 1) * ny : 0;
    const unsigned long long lower = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    long long best_dot = 0, best_na = 1;
    int best_k = -1;
    for (int vb = 0; vb < ncand; vb += 128) {
        const int k0 = vb + lane, k1 = vb + 64 + lane;
        const int kk0 = min(k0, ncand - 1), kk1 = min(k1, ncand - 1);
        const int x0a = xlo + kk0 / ny, y0a = ylo + kk0 % ny, x0b = xlo + kk1 / ny, y0b = ylo + kk1 % ny;
        const bool va = C.valid(x0a, y0a, x0a * a.rows + y0a), vbb = C.valid(x0b, y0b, x0b * a.rows + y0b);
        const bool v0 = k0 < ncand && va, v1 = k1 < ncand && vbb;
        const unsigned long long b0 = __ballot(v0), b1 = __ballot(v1);
        const int n0c = __popcll(b0), nv = n0c + __popcll(b1);
        if (v0) lst[__popcll(b0 & lower)] = k0;  // scan order
        if (v1) lst[n0c + __popcll(b1 & lower)] = k1;
        for (int c0 = 0; c0 < nv; c0 += 16) {
            const int c = c0 + cslot;
            int dot = 0, na = 0, k = -1;
            if (c < nv) {
                k = lst[c];
                const int4 *cp = reinterpret_cast<const int4 *>(C.row(xlo + k / ny, ylo + k % ny) + 64 * q4);
                int4 x[4];
#pragma unroll
                for (int v = 0; v < 4; v++) x[v] = cp[v];
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    dot = __builtin_amdgcn_sdot4(x[v].x, qa[v].x, dot, false);
                    dot = __builtin_amdgcn_sdot4(x[v].y, qa[v].y, dot, false);
                    dot = __builtin_amdgcn_sdot4(x[v].z, qa[v].z, dot, false);
                    dot = __builtin_amdgcn_sdot4(x[v].w, qa[v].w, dot, false);
                    na = __builtin_amdgcn_sdot4(x[v].x, x[v].x, na, false);
                    na = __builtin_amdgcn_sdot4(x[v].y, x[v].y, na, false);
                    na = __builtin_amdgcn_sdot4(x[v].z, x[v].z, na, false);
                    na = __builtin_amdgcn_sdot4(x[v].w, x[v].w, na, false);
                }
            }
            dot += __shfl_xor(dot, 1, 64);
            dot += __shfl_xor(dot, 2, 64);
            na += __shfl_xor(na, 1, 64);
            na += __shfl_xor(na, 2, 64);
            const long long cdot = dot, cna = na;
            const bool pass = q4 == 0 && c < nv && dot > 0 && na != 0 && n2_256 != 0 &&
                              (unsigned __int128)(100ll * cdot * cdot) >
                                  (unsigned __int128)81 * (unsigned long long)(cna * (long long)n2_256);
            long long bd = pass ? cdot : 0, bn = pass ? cna : 1;
            int bk = pass ? k : -1;
#pragma unroll
            for (int o = 4; o < 64; o <<= 1) {  // the 16 scoring lanes (q4 == 0)
                const long long od = __shfl_xor(bd, o, 64), on = __shfl_xor(bn, o, 64);
                const int ok = __shfl_xor(bk, o, 64);
                if (exact_better(od, on, ok, bd, bn, bk)) {
                    bd = od;
                    bn = on;
                    bk = ok;
                }
            }
            if (bk >= 0 && exact_better(bd, bn, bk, best_dot, best_na, best_k)) {
                best_dot = bd;
                best_na = bn;
                best_k = bk;
            }
        }
    }
    if (best_k >= 0) {
        res.found = 1;
        res.bx = xlo + best_k / ny;
        res.by = ylo + best_k % ny;
        res.score = (float)((double)best_dot * (double)best_dot / ((double)best_na * (double)n2_256));
        best_patch_out = res.bx * a.rows + res.by;
    } else {
        best_patch_out = -1;
    }
    return res;
}

// one wave per query slot; 4 waves per block; candidates straight from global memory
__global__ __launch_bounds__(256) void k_window_eval(WinArgs a, const int8_t *__restrict__ desc0,
                                                     const int *__restrict__ max_idx0,
                                                     const float *__restrict__ probs0,
                                                     const int8_t *__restrict__ desc1,
                                                     const int *__restrict__ num_sel,
                                                     const int *__restrict__ patches1,
                                                     QueryResult *__restrict__ out) {
    __shared__ int lst_s[4][128];
    const int lane = threadIdx.x & 63;
    const int qslot = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int pair = blockIdx.y;
    if (qslot >= a.N) return;
    QueryResult res = {0, 0, 0, -1, 0.0f};
    const int nsel = num_sel[pair];
    const int cells = a.rows * a.cols;
    if (qslot < nsel) {
        const int patch1 = __builtin_amdgcn_readfirstlane(patches1[(long)pair * a.N + qslot]);
        const int x1 = patch1 / a.rows, y1 = patch1 % a.rows;
        const GlobalCands C = {desc0 + (long)pair * cells * kDescD, max_idx0 + (long)pair * cells,
                               probs0 + (long)pair * cells, a.rows, a.prob_thr};
        int bp;
        const int8_t *qd = desc1 + ((long)pair * cells + patch1) * kDescD;
        if (a.as_built)
            res = eval_query(a, C, qd, x1, y1, lane, bp);
        else
            res = eval_query_intended(a, C, qd, x1, y1, lane, lst_s[threadIdx.x >> 6], bp);
        res.best_patch = bp;
    }
    if (lane == 0) out[(long)pair * a.N + qslot] = res;
}

// ---------------------------------------------------------------------------
// Window match, fast path (rows <= 64, window <= kWinList cells): the default at both the
// reference's 24x80 grid and the 47x155 KITTI grid.
//
// k_window_mask: one 64-bit word per frame-0 grid column, bit y set when cell (x, y) is a
// candidate (tracking_main.c:121-125: index != 64 and !(prob < 0.2), double compare).  A
// column's cells are contiguous (p = x*rows + y), so a wave takes 64 columns = 64 * rows
// consecutive cells: one ballot per 64 cells (dense 256-B loads), the ballot words in the wave's
// LDS slice, then each lane cuts its column's rows bits out of (at most) two of them.  (Round 5:
// one wave per column, 47 of 64 lanes loading 188 B -- 2.1 TB/s, launch-bound.)
//
// k_window_query: one wave walks kQPW consecutive top-N queries (patch order, so the windows
// of a wave overlap in L1/L2).  Per query the wave reads the masks of the window's columns
// (one word per lane), builds the scan-ordered candidate list in LDS, and loads the
// descriptors of up to 32 candidates at once -- while the next query's masks and query row
// are already in flight.  Blocks are remapped so that all blocks of a pair run on one XCD
// (dispatch is round-robin over the 8 XCDs): the pair's frame-0 descriptors stream from one L2.
// ---------------------------------------------------------------------------
constexpr int kQPW = 8;        // queries per wave
constexpr int kWinList = 256;  // candidate-list capacity per wave (window cells)

__global__ __launch_bounds__(256) void k_window_mask(long total_cols, int rows, const int *__restrict__ mi0,
                                                     const float *__restrict__ pr0, double prob_thr,
                                                     unsigned long long *__restrict__ masks) {
    __shared__ unsigned long long wb[4][64];  // per wave: rows ballot words of 64 cells (rows <= 64)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long c0 = ((long)blockIdx.x * 4 + w) * 64;  // the wave's first column
    if (c0 >= total_cols) return;                      // wave-uniform; no block barrier below
    const int ncol = (int)min(64l, total_cols - c0);
    const long cell0 = c0 * rows, ncell = (long)ncol * rows;
    for (int k = 0; k < rows; k++) {
        const long i = (long)k * 64 + lane;
        bool v = false;
        if (i < ncell) {
            const long p = cell0 + i;
            v = mi0[p] != 64 && !((double)pr0[p] < prob_thr);
        }
        const unsigned long long bw = __ballot(v);
        if (lane == 0) wb[w][k] = bw;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes
    __builtin_amdgcn_wave_barrier();
    if (lane < ncol) {
        const int sb = lane * rows, k0 = sb >> 6, off = sb & 63;
        unsigned long long m = wb[w][k0] >> off;
        if (off + rows > 64) m |= wb[w][k0 + 1] << (64 - off);
        if (rows < 64) m &= (1ull << rows) - 1ull;
        masks[c0 + lane] = m;
    }
}

struct QueryPrefetch {
    int patch1, ncol, ny, origin;  // origin: frame-0 cell (xlo, ylo) of the window
    unsigned long long bits;       // lane j < ncol: candidate rows of window column j (bit = y - ylo)
    int4 q[4];                     // query bytes: as-intended 32*(lane&7) .. +31 (q[0..1]); as-built 0 .. 63
    int qv;                        // query dword `lane`
};

template <bool kBuilt>
__device__ __forceinline__ QueryPrefetch window_prefetch(const WinArgs &a, const unsigned long long *mk,
                                                         const int8_t *d1, int patch1, int lane) {
    QueryPrefetch f;
    f.patch1 = patch1;
    f.bits = 0;
    f.ncol = 0;
    f.ny = 1;
    f.origin = 0;
    if (patch1 < 0) return f;
    const int x1 = patch1 / a.rows, y1 = patch1 % a.rows;
    const int xlo = max(x1 + a.shift_x - a.radius, 0), xhi = min(x1 + a.shift_x + a.radius, a.cols - 1);
    const int ylo = max(y1 + a.shift_y - a.radius, 0), yhi = min(y1 + a.shift_y + a.radius, a.rows - 1);
    f.origin = xlo * a.rows + ylo;
    if (xhi >= xlo && yhi >= ylo) {
        f.ncol = xhi - xlo + 1;
        f.ny = yhi - ylo + 1;
        if (lane < f.ncol) {
            const unsigned long long keep = f.ny == 64 ? ~0ull : ((1ull << f.ny) - 1);
            f.bits = (mk[xlo + lane] >> ylo) & keep;
        }
    }
    const int8_t *qd = d1 + (long)patch1 * kDescD;
    if (kBuilt) {
        const int4 *qp = reinterpret_cast<const int4 *>(qd);
#pragma unroll
        for (int v = 0; v < 4; v++) f.q[v] = qp[v];
    } else {
        const int4 *qp = reinterpret_cast<const int4 *>(qd + 32 * (lane & 7));
        f.q[0] = qp[0];
        f.q[1] = qp[1];
    }
    f.qv = reinterpret_cast<const int *>(qd)[lane];
    return f;
}

// Scan-ordered candidate list of the prefetched window.  An entry is the candidate's cell
// offset from the window origin (column*rows + row offset): increasing in scan order (x outer,
// y inner), and origin + entry addresses the descriptor without a division.
__device__ __forceinline__ int window_list(const QueryPrefetch &f, int lane, int rows, int *lst) {
    const int cnt = __popcll(f.bits);
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int nv = __shfl(incl, 63, 64);
    int pos = incl - cnt;
    unsigned long long b = f.bits;
    const int colbase = lane * rows;
    while (b) {
        const int yb = __ffsll((long long)b) - 1;
        b &= b - 1;
        lst[pos++] = colbase + yb;
    }
    return nv;
}

__device__ __forceinline__ void dot_x4(const int4 *x, const int4 *q, int nv4, int &dot, int &na) {
#pragma unroll
    for (int v = 0; v < 4; v++) {
        if (v >= nv4) break;
        dot = __builtin_amdgcn_sdot4(x[v].x, q[v].x, dot, false);
        dot = __builtin_amdgcn_sdot4(x[v].y, q[v].y, dot, false);
        dot = __builtin_amdgcn_sdot4(x[v].z, q[v].z, dot, false);
        dot = __builtin_amdgcn_sdot4(x[v].w, q[v].w, dot, false);
        na = __builtin_amdgcn_sdot4(x[v].x, x[v].x, na, false);
        na = __builtin_amdgcn_sdot4(x[v].y, x[v].y, na, false);
        na = __builtin_amdgcn_sdot4(x[v].z, x[v].z, na, false);
        na = __builtin_amdgcn_sdot4(x[v].w, x[v].w, na, false);
    }
}

// a * b for a < 2^45, b < 2^32 as (hi, lo32): two v_mad_u64_u32, exact
__device__ __forceinline__ void mul45x32(unsigned long long a, unsigned b, unsigned long long &hi, unsigned &lo) {
    const unsigned long long p0 = (unsigned long long)(unsigned)a * b;
    hi = (unsigned long long)(unsigned)(a >> 32) * b + (p0 >> 32);
    lo = (unsigned)p0;
}

// exact "candidate a beats b" for the as-intended score dot^2/na (dot > 0, |dot|, na < 2^23:
// 256 products of int8), ties -> lower scan position; k < 0 = none
__device__ __forceinline__ bool better_i32(int da, int na, int ka, int db, int nb, int kb) {
    if (ka < 0) return false;
    if (kb < 0) return true;
    unsigned long long lh, rh;
    unsigned ll, rl;
    mul45x32((unsigned long long)((long long)da * da), (unsigned)nb, lh, ll);
    mul45x32((unsigned long long)((long long)db * db), (unsigned)na, rh, rl);
    if (lh != rh) return lh > rh;
    if (ll != rl) return ll > rl;
    return ka < kb;
}

// As-intended (exact cosine, tracking_main.c:114-165 as meant): 8 lanes per candidate (32 B
// each), four candidates per lane group per round: 32 candidate rows in flight.
__device__ __forceinline__ void query_intended(const int8_t *d0, const QueryPrefetch &f, int nv, const int *lst,
                                               int lane, int n2, int &best_dot, int &best_na, int &best_k) {
    const int q8 = lane & 7, cslot = lane >> 3;
    const int8_t *wbase = d0 + (long)f.origin * kDescD + 32 * q8;
    for (int c0 = 0; c0 < nv; c0 += 32) {
        int k[4];
        int4 x[4][2];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = c0 + 8 * u + cslot;
            k[u] = c < nv ? lst[c] : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (k[u] >= 0) {
                const int4 *p = reinterpret_cast<const int4 *>(wbase + (long)k[u] * kDescD);
                x[u][0] = p[0];
                x[u][1] = p[1];
            }
        }
        int bd = 0, bn = 1, bk = -1;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            int d = 0, n = 0;
            if (k[u] >= 0) dot_x4(x[u], f.q, 2, d, n);
            d += __shfl_xor(d, 1, 64);
            n += __shfl_xor(n, 1, 64);
            d += __shfl_xor(d, 2, 64);
            n += __shfl_xor(n, 2, 64);
            d += __shfl_xor(d, 4, 64);
            n += __shfl_xor(n, 4, 64);
            const bool pass = k[u] >= 0 && d > 0 && n != 0 && n2 != 0 &&
                              (unsigned long long)(100ll * d * d) > 81ull * (unsigned long long)((long long)n * n2);
            if (pass && better_i32(d, n, k[u], bd, bn, bk)) {
                bd = d;
                bn = n;
                bk = k[u];
            }
        }
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {  // the 8 lane groups (every lane of a group agrees)
            const int od = __shfl_xor(bd, o, 64), on = __shfl_xor(bn, o, 64), ok = __shfl_xor(bk, o, 64);
            if (better_i32(od, on, ok, bd, bn, bk)) {
                bd = od;
                bn = on;
                bk = ok;
            }
        }
        if (bk >= 0 && better_i32(bd, bn, bk, best_dot, best_na, best_k)) {
            best_dot = bd;
            best_na = bn;
            best_k = bk;
        }
    }
}

// As-built: the first candidate (scan order) with a non-zero 256-D norm latches
// norm1 and is scored in 256-D; every later candidate is scored in 64-D against the stale
// norm1 with int32-wrapped products, float division and a double compare; candidates before
// the latch are all-zero descriptors (0/0 = NaN: never pass).  One lane per candidate.
// Returns the winner's list position.
__device__ __forceinline__ void query_built(const WinArgs &a, const int8_t *d0, const QueryPrefetch &f, int nv,
                                            const int *lst, int lane, int &best_pos, float &best_d) {
    const int8_t *wbase = d0 + (long)f.origin * kDescD;
    const int n2_256 = wave_sum(__builtin_amdgcn_sdot4(f.qv, f.qv, 0, false));
    int n2_64 = 0, unused = 0;
    dot_x4(f.q, f.q, 4, n2_64, unused);
    // latch: the first listed candidate whose full norm is non-zero (almost always the first)
    int latch = -1, n1f = 0, dot_f = 0;
    for (int j = 0; j < nv; j++) {
        const int cv = reinterpret_cast<const int *>(wbase + (long)lst[j] * kDescD)[lane];
        const int full_n1 = wave_sum(__builtin_amdgcn_sdot4(cv, cv, 0, false));
        if (full_n1 != 0) {
            latch = j;
            n1f = full_n1;
            dot_f = wave_sum(__builtin_amdgcn_sdot4(cv, f.qv, 0, false));
            break;
        }
    }
    if (latch < 0) return;
    const int den64 = wrap_mul(n1f, n2_64);
    {  // the latching candidate itself (256-D)
        const float d = (float)wrap_mul(dot_f, dot_f) / (float)wrap_mul(n1f, n2_256);
        if ((double)d > a.thr_sq) {
            best_pos = latch;
            best_d = d;
        }
    }
    for (int c0 = latch + 1; c0 < nv; c0 += 64) {
        const int c = c0 + lane;
        float d = -__builtin_inff();
        int pc = 0x7fffffff;
        if (c < nv) {
            const int4 *p = reinterpret_cast<const int4 *>(wbase + (long)lst[c] * kDescD);
            int4 x[4];
#pragma unroll
            for (int v = 0; v < 4; v++) x[v] = p[v];
            int dot = 0, nn = 0;
            dot_x4(x, f.q, 4, dot, nn);
            const float dd = (float)wrap_mul(dot, dot) / (float)den64;
            if ((double)dd > a.thr_sq) {
                d = dd;
                pc = c;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {  // first strict maximum: max d, ties -> lowest position
            const float od = __shfl_xor(d, o, 64);
            const int oc = __shfl_xor(pc, o, 64);
            if (od > d || (od == d && oc < pc)) {
                d = od;
                pc = oc;
            }
        }
        if (pc != 0x7fffffff && (best_pos < 0 || d > best_d)) {
            best_d = d;
            best_pos = pc;
        }
    }
}

template <bool kBuilt>
__global__ __launch_bounds__(256) void k_window_query(WinArgs a, int blocks_per_pair, int nblocks,
                                                      const unsigned long long *__restrict__ masks,
                                                      const int8_t *__restrict__ desc0,
                                                      const int8_t *__restrict__ desc1,
                                                      const int *__restrict__ num_sel,
                                                      const int *__restrict__ patches1,
                                                      QueryResult *__restrict__ out) {
    __shared__ int lst_s[4][kWinList];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // XCD-aware remap: physical block b runs on XCD b % 8; give each XCD a contiguous run of
    // logical blocks (whole pairs).  gridDim.x is a multiple of 8.
    const int b = blockIdx.x, per_xcd = gridDim.x >> 3;
    const int logical = (b & 7) * per_xcd + (b >> 3);
    if (logical >= nblocks) return;
    const int pair = logical / blocks_per_pair;
    const int qbase = ((logical % blocks_per_pair) * 4 + w) * kQPW;
    if (qbase >= a.N) return;  // wave-uniform; the kernel has no block barrier
    const int nq = min(kQPW, a.N - qbase);
    const int nsel = num_sel[pair];
    const long cells = (long)a.rows * a.cols;
    const int8_t *d0 = desc0 + pair * cells * kDescD;
    const int8_t *d1 = desc1 + pair * cells * kDescD;
    const unsigned long long *mk = masks + (long)pair * a.cols;
    const int my_patch = (lane < nq && qbase + lane < nsel) ? patches1[(long)pair * a.N + qbase + lane] : -1;
    int *lst = lst_s[w];
    QueryResult mine = {0, 0, 0, -1, 0.0f};  // lane i: query qbase + i

    QueryPrefetch cur = window_prefetch<kBuilt>(a, mk, d1, __shfl(my_patch, 0, 64), lane);
    for (int i = 0; i < nq; i++) {
        if (cur.patch1 < 0) break;  // queries past num_selected (patch order: all later ones too)
        const QueryPrefetch nxt =
            window_prefetch<kBuilt>(a, mk, d1, i + 1 < nq ? __shfl(my_patch, i + 1, 64) : -1, lane);
        const int nv = window_list(cur, lane, a.rows, lst);
        QueryResult res = {0, 0, 0, -1, 0.0f};
        int entry = -1;
        if (!kBuilt) {
            int n2 = 0, unused = 0;
            dot_x4(cur.q, cur.q, 2, n2, unused);
            n2 += __shfl_xor(n2, 1, 64);
            n2 += __shfl_xor(n2, 2, 64);
            n2 += __shfl_xor(n2, 4, 64);
            int bd = 0, bn = 1, bk = -1;
            query_intended(d0, cur, nv, lst, lane, n2, bd, bn, bk);
            if (bk >= 0) {
                entry = bk;
                res.score = (float)((double)bd * (double)bd / ((double)bn * (double)n2));
            }
        } else {
            int bpos = -1;
            float bdv = 0.0f;
            query_built(a, d0, cur, nv, lst, lane, bpos, bdv);
            if (bpos >= 0) {
                entry = lst[bpos];
                res.score = bdv;
            }
        }
        if (entry >= 0) {
            res.found = 1;
            res.best_patch = cur.origin + entry;
            res.bx = res.best_patch / a.rows;
            res.by = res.best_patch % a.rows;
        }
        if (lane == i) mine = res;
        cur = nxt;
    }
    if (lane < nq) out[(long)pair * a.N + qbase + lane] = mine;
}

// ---------------------------------------------------------------------------
// Window-match constants and the per-tile fold shared by the as-intended kernel below.  The
// (pair, band of kBandW grid columns) eligibility test is kept from the band-tiled kernel this
// replaced (measured slower and removed; in history).
// ---------------------------------------------------------------------------
constexpr int kBandW = 5;
constexpr int kBandList = 960;  // candidate-list capacity the eligibility test checks ((kBandW + 2r) * rows)

typedef int i32x4_t __attribute__((ext_vector_type(4)));

// One 16x16 tile's elements (lane: candidate column; rows 4 h + j): window membership, the
// as-intended pass test 100 dot^2 > 81 |c|^2 |q|^2 and the exact running best.  The pass
// test is screened in fp32 (relative error < 2^-20 on both sides) and decided in 64-bit
// integers only within that margin.
// the fold of one tile into the lane's 4 queries' bests, branch-free but for the rare exact cases.
// The threshold is the INITIAL best: 100 d^2 > 81 |a|^2 |q|^2 is "beats (d^2, n) = (81 |q|^2, 100)",
// and whatever beats a best that passed the threshold passes it too -- so one test per candidate,
// d^2 n_best > d_best^2 n (ties to the lower scan position), screened in float with margins its
// rounding cannot cross (each side within 2e-7 of its exact value) and decided exactly (64-bit
// integers) only inside the margins; fbq / fbn carry the best's d^2 and n as floats for the screen
// (n < 2^24: the float is exact, and is the only copy kept; bk < 0: the threshold is the best).
// Round 5's form -- better_i32 in a branch taken by every passing candidate, the best updated
// inside it -- picked wrong winners on the GPU in windows full of exact ties
// (tests/test_gpu_frontend.py::test_window_match_exact_ties_and_threshold: 38 of 99 matches), while
// a CPU emulation of its algorithm agrees with the oracle and an -O1 build of it fails differently
// (87): the code generated for it, not the algorithm (tools/diag/dbg_window_tie.py,
// profiles/r06l_window_tie_bisect.log).
__device__ __forceinline__ void window_fold(const i32x4_t &acc, bool cv, int cx, int cy, int cp, int cna, int r,
                                            const int *rcx, const int *rcy, const float *frn2, int *bd, int *bk,
                                            float *fbq, float *fbn) {
    const float fna = (float)cna;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int d = acc[j];
        const bool in = cv && (unsigned)(cx - rcx[j] + r) <= (unsigned)(2 * r) &&
                        (unsigned)(cy - rcy[j] + r) <= (unsigned)(2 * r) && d > 0;
        const float fd = (float)d, fd2 = fd * fd;
        const float L = fd2 * fbn[j], Rr = fbq[j] * fna;
        bool win = in && L > Rr * 1.000002f;
        if (in && !win && L >= Rr * 0.999998f) {  // rare: exact
            if (bk[j] < 0)  // against the threshold; |a|^2 and |q|^2 < 2^24: exact as floats
                win = (unsigned long long)(100ll * d * d) > 81ull * (unsigned long long)((long long)cna * (int)frn2[j]);
            else
                win = better_i32(d, cna, cp, bd[j], (int)fbn[j], bk[j]);
        }
        bd[j] = win ? d : bd[j];
        bk[j] = win ? cp : bk[j];
        fbq[j] = win ? fd2 : fbq[j];
        fbn[j] = win ? fna : fbn[j];
    }
}

// ---------------------------------------------------------------------------
// Window match, per-wave MFMA (as-intended; the default): one wave owns 16 consecutive
// top-N queries of a pair -- patch order, so they span a few grid columns -- and sweeps the
// candidates of the union of their windows' columns (column masks -> scan-ordered list in the
// wave's LDS slice) with v_mfma_i32_16x16x64_i8, the candidates' rows gathered by LDS-DMA into
// the wave's own 2-tile ring two 16-candidate tiles ahead.  No block barrier and nothing shared
// between waves: the rest of the gather latency is hidden by occupancy (4 waves per SIMD).
// ---------------------------------------------------------------------------
constexpr int kWQ = 16;            // queries per wave

constexpr int kWaveList = 512;     // candidate-list capacity per wave (more: several passes)


constexpr int kWinTileB = 16 * kDescD;  // one staged tile: 16 candidates x 256 B
#pragma clang diagnostic ignored "-Winline-asm"  // m0 in the clobber list (as k_allpairs_i8.hip)
// 64 lanes x 16 B from global (SGPR base + per-lane 32-bit offset) into LDS at M0 (wave-uniform)
__device__ __forceinline__ void glds16_win(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_mov_b32 m0, %2\n\t"
        "global_load_lds_dwordx4 %0, %1"
        :
        : "v"(voff), "s"(sbase), "s"(lds_byte)
        : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void wait_vm_win() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

constexpr int WIN_WPE = 2;  // waves per EU the launch bound asks for (the kernel takes 126 VGPRs)
__global__ __launch_bounds__(256, WIN_WPE) void k_window_wave(WinArgs a, int blocks_per_pair, int nblocks,
                                                     const unsigned long long *__restrict__ masks,
                                                     const int8_t *__restrict__ desc0,
                                                     const int8_t *__restrict__ desc1,
                                                     const int *__restrict__ num_sel,
                                                     const int *__restrict__ patches1,
                                                     QueryResult *__restrict__ out) {
    __shared__ unsigned short lst_s[4][kWaveList];
    // per wave: 2 staged tiles (3: 52 KiB per block, 3 blocks -- waves per SIMD -- per CU instead of 4,
    // 2.56 against 2.12 ms, profiles/r06iv_window_ring3_ab.log)
    __shared__ __attribute__((aligned(16))) char bst_s[4][2][kWinTileB];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int b = blockIdx.x, per_xcd = gridDim.x >> 3;
    const int logical = (b & 7) * per_xcd + (b >> 3);
    if (logical >= nblocks) return;
    const int pair = logical / blocks_per_pair;
    const int q0 = ((logical % blocks_per_pair) * 4 + w) * kWQ;
    const int nsel = min(num_sel[pair], a.N);
    if (q0 >= nsel) return;  // wave-uniform; the kernel has no block barrier
    const int nq = min(kWQ, nsel - q0);
    const int R = a.rows, r = a.radius;
    const long cells = (long)R * a.cols;
    const int8_t *d0 = desc0 + pair * cells * kDescD;
    const int8_t *d1 = desc1 + pair * cells * kDescD;
    const int h = lane >> 4, col = lane & 15;
    unsigned short *lst = lst_s[w];

    // queries: row `col` = query q0 + col (A: bytes 64 s + 16 h .. +15)
    const bool rv = col < nq;
    const int qp = patches1[(long)pair * a.N + q0 + min(col, nq - 1)];
    const int xfirst = __shfl(qp, 0, 64) / R, xlast = __shfl(qp, nq - 1, 64) / R;
    const int cx0 = max(xfirst + a.shift_x - r, 0), cx1 = min(xlast + a.shift_x + r, a.cols - 1);
    i32x4_t A[4];
    {
        const i32x4_t *qrow = reinterpret_cast<const i32x4_t *>(d1 + (long)qp * kDescD + 16 * h);
#pragma unroll
        for (int s2 = 0; s2 < 4; s2++) A[s2] = rv ? qrow[4 * s2] : i32x4_t{0, 0, 0, 0};
    }
    unsigned long long bits = 0;
    if (cx0 + lane <= cx1 && lane < 64) bits = masks[(long)pair * a.cols + cx0 + lane];
    int n2 = 0;
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++)
#pragma unroll
        for (int u = 0; u < 4; u++) n2 = __builtin_amdgcn_sdot4(A[s2][u], A[s2][u], n2, false);
    n2 += __shfl_xor(n2, 16, 64);
    n2 += __shfl_xor(n2, 32, 64);
    const int qcx = rv ? qp / R + a.shift_x : -(1 << 20), qcy = rv ? qp % R + a.shift_y : -(1 << 20);
    int rcx[4], rcy[4], bd[4], bk[4];
    float frn2[4], fbq[4], fbn[4];  // |query|^2, the best's d^2 and |candidate|^2 (the norms exact)
#pragma unroll
    for (int j = 0; j < 4; j++) {
        frn2[j] = (float)__shfl(n2, 4 * h + j, 64);
        rcx[j] = __shfl(qcx, 4 * h + j, 64);
        rcy[j] = __shfl(qcy, 4 * h + j, 64);
        bd[j] = 0;
        bk[j] = -1;
        fbq[j] = 81.0f * frn2[j];  // the threshold as the initial best (81 |q|^2, 100)
        fbn[j] = 100.f;
    }
    // candidate list: columns cx0 .. cx1 (<= 64 when the 16 queries span <= 64 - 2r columns;
    // wider spans take the column groups in turn), scan order, in passes of kWaveList
    for (int cg = cx0; cg <= cx1; cg += 64) {
        if (cg > cx0) bits = (cg + lane <= cx1) ? masks[(long)pair * a.cols + cg + lane] : 0ull;
        const int cnt = __popcll(bits);
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const int total = __builtin_amdgcn_readfirstlane(__shfl(incl, 63, 64));  // uniform: scalar loops
        for (int lb = 0; lb < total; lb += kWaveList) {
            {
                int pos = incl - cnt - lb;
                unsigned long long bb = bits;
                const int xy = (cg + lane) << 6;
                while (bb && pos < kWaveList) {
                    const int yb = __ffsll((long long)bb) - 1;
                    bb &= bb - 1;
                    if (pos >= 0) lst[pos] = (unsigned short)(xy | yb);
                    pos++;
                }
            }
            const int nc = min(kWaveList, total - lb);
            const int ntiles = (nc + 15) >> 4;
            // B tiles by LDS-DMA into the wave's 2-slot ring, two tiles ahead of the MFMAs (no VGPRs
            // held for the prefetch): instruction k of a tile stages candidates 4 k .. 4 k + 3, lane l
            // -> candidate 4 k + (l >> 4), LDS chunk l & 15 <- source chunk (l & 15) ^ candidate
            // (16-B chunks XOR-swizzled by candidate: the fragment reads are conflict-free); lanes past
            // the list repeat its last cell and are not folded.  The sweep waits on these gathers, not
            // on its VALU (rocprof: VALU issue ~35 % of the SIMD cycles, profiles/r06it_window_pmc.txt):
            // one tile ahead in registers 2.226 ms, two ahead through LDS 2.13 (r06iu_window_dma_ab.log).
            // (Round 6 before this: the register prefetch unmasked and its last tile peeled, 2.315 ->
            // 2.226 ms, r06in / r06io; two register sets taking turns: 145 VGPRs, 2.65 ms, r06im.)
            const unsigned ring = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)&bst_s[w][0][0];
            auto stage = [&](int t) {
                const unsigned dst = __builtin_amdgcn_readfirstlane(ring + (unsigned)((t & 1) * kWinTileB));
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int c = 4 * k + (lane >> 4);
                    const int xy = lst[min(t * 16 + c, nc - 1)];
                    const unsigned voff =
                        (unsigned)(((xy >> 6) * R + (xy & 63)) * kDescD) + ((unsigned)((lane & 15) ^ c) << 4);
                    glds16_win(d0, voff, dst + 1024u * k);
                }
            };
            auto tile = [&](int nt) {
                const int cr = nt * 16 + col;
                const int xyc = lst[min(cr, nc - 1)];
                const i32x4_t *sb = reinterpret_cast<const i32x4_t *>(&bst_s[w][nt & 1][0]) + col * 16;
                i32x4_t bc[4];
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) bc[s2] = sb[(4 * s2 + h) ^ col];
                i32x4_t acc = {0, 0, 0, 0};
                int cna = 0;
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) {
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[s2], bc[s2], acc, 0, 0, 0);
#pragma unroll
                    for (int u = 0; u < 4; u++) cna = __builtin_amdgcn_sdot4(bc[s2][u], bc[s2][u], cna, false);
                }
                // the slot's reads are done (their values were consumed above): stage tile nt + 2 into it
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
                if (nt + 2 < ntiles) stage(nt + 2);
                cna += __shfl_xor(cna, 16, 64);
                cna += __shfl_xor(cna, 32, 64);
                const bool cv = cr < nc;
                const int cx = cv ? xyc >> 6 : (1 << 24), cy = xyc & 63;
                const int cp = cx * R + cy;
                window_fold(acc, cv, cx, cy, cp, cna, r, rcx, rcy, frn2, bd, bk, fbq, fbn);
            };
            stage(0);
            if (ntiles > 1) stage(1);
            for (int nt = 0; nt < ntiles; nt++) {  // wave-uniform
                if (nt + 1 < ntiles)
                    wait_vm_win<4>();  // tile nt landed (tile nt + 1's 4 pieces may be in flight)
                else
                    wait_vm_win<0>();
                tile(nt);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int bn = (int)fbn[j];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const int od = __shfl_xor(bd[j], o, 64), on = __shfl_xor(bn, o, 64), ok = __shfl_xor(bk[j], o, 64);
            if (better_i32(od, on, ok, bd[j], bn, bk[j])) {
                bd[j] = od;
                bn = on;
                bk[j] = ok;
            }
        }
        fbn[j] = (float)bn;
    }
    if (col == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int qi = 4 * h + j;
            if (qi >= nq) continue;
            QueryResult res = {0, 0, 0, -1, 0.0f};
            if (bk[j] >= 0) {
                res.found = 1;
                res.best_patch = bk[j];
                res.bx = bk[j] / R;
                res.by = bk[j] % R;
                res.score = (float)((double)bd[j] * (double)bd[j] / ((double)fbn[j] * (double)frn2[j]));
            }
            out[(long)pair * a.N + q0 + qi] = res;
        }
    }
}

__global__ __launch_bounds__(1024) void k_window_compact(int N, int rows, int max_matches,
                                                         const QueryResult *__restrict__ qr,
                                                         const int *__restrict__ num_sel,
                                                         const int *__restrict__ patches1,
                                                         const int *__restrict__ indices1,
                                                         const int *__restrict__ max_idx0, long cells,
                                                         int *__restrict__ num_matches, float *__restrict__ points1,
                                                         float *__restrict__ points2, int *__restrict__ qom) {
    __shared__ int wsum[16];
    const int pair = blockIdx.x, t = threadIdx.x;
    const int per = (N + 1023) / 1024;
    const int q0 = t * per, q1 = min(q0 + per, N);
    const int nsel = num_sel[pair];
    const QueryResult *r = qr + (long)pair * N;
    int cnt = 0;
    for (int q = q0; q < q1; q++) cnt += (q < nsel && r[q].found) ? 1 : 0;
    int total;
    int k = block_exclusive_scan<1024>(cnt, &total, wsum);
    for (int q = q0; q < q1; q++) {
        if (!(q < nsel && r[q].found)) continue;
        if (k < max_matches) {
            const int patch1 = patches1[(long)pair * N + q];
            const int x1 = patch1 / rows, y1 = patch1 % rows;
            const int idx1 = indices1[(long)pair * N + q];
            const QueryResult m = r[q];
            const int best_index = max_idx0[(long)pair * cells + m.best_patch];  // image0 index of the winner
            float *p1 = points1 + ((long)pair * max_matches + k) * 2;
            float *p2 = points2 + ((long)pair * max_matches + k) * 2;
            p1[0] = (float)(m.bx * 8 + best_index % 8);
            p1[1] = (float)(m.by * 8 + best_index / 8);
            p2[0] = (float)(x1 * 8 + idx1 % 8);
            p2[1] = (float)(y1 * 8 + idx1 / 8);
            if (qom) qom[(long)pair * max_matches + k] = q;
        }
        k++;
    }
    if (t == 0) num_matches[pair] = min(total, max_matches);
}

}  // namespace

namespace mv {

int launch_softmax(hipStream_t s, int batch, int cells, const float *scales, const int8_t *semi, int *max_idx,
                   float *probs, int *num_valid) {
    MV_REQUIRE(batch > 0 && cells > 0 && scales && semi && max_idx && probs && num_valid);
    MV_REQUIRE(((uintptr_t)semi & 3) == 0);
    const long rows = (long)batch * cells;
    MV_HIP_TRY(hipMemsetAsync(num_valid, 0, sizeof(int) * batch, s));
    const int blocks = (int)((rows + 255) / 256);
    MV_PROF_BEGIN(s, "k_softmax");
    hipLaunchKernelGGL(k_softmax, dim3(blocks), dim3(256), 0, s, (int)rows, cells, scales, semi, max_idx, probs,
                       num_valid);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

int launch_top_n_select(hipStream_t s, int batch, int cells, const int *max_idx, const float *probs, int N,
                        int cap, int *num_sel, int *patches, int *indices, float *sel_probs, int *status) {
    MV_REQUIRE(batch > 0 && cells > 0 && N > 0 && cap > 0);
    MV_PROF_BEGIN(s, "k_top_n_select");
    hipLaunchKernelGGL(k_top_n_select, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, s, batch, cells, max_idx,
                       probs, N, cap, num_sel, patches, indices, sel_probs, status);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

// The window match needs per-query scratch; it is taken from the context.
extern "C" int mv_window_match_batch_dev(mv_context *ctx, const mv_window_params *p, int batch, int rows, int cols,
                                         const int8_t *desc0, const int *max_idx0, const float *probs0,
                                         const int8_t *desc1, int N, const int *num_selected, const int *patches1,
                                         const int *indices1, int *num_matches, float *points1, float *points2,
                                         int *query_of_match) {
    MV_REQUIRE(ctx && p && batch > 0 && rows > 0 && cols > 0 && N > 0 && p->max_matches > 0);
    MV_REQUIRE(desc0 && max_idx0 && probs0 && desc1 && num_selected && patches1 && indices1);
    MV_REQUIRE(num_matches && points1 && points2);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    WinArgs a;
    a.rows = rows;
    a.cols = cols;
    a.N = N;
    a.shift_x = p->shift_x;
    a.shift_y = p->shift_y;
    a.radius = p->radius;
    a.as_built = p->semantics == MV_AS_BUILT;
    a.thr_sq = p->match_thresh_sq;
    a.prob_thr = p->prob_thresh;
    const long cells = (long)rows * cols;
    // fast path: one mask word per column and a window list that fits the wave's LDS slice
    const int wside = 2 * p->radius + 1;
    const bool fast = rows <= 64 && p->radius >= 0 && wside <= 64 && (long)wside * min(wside, rows) <= kWinList;
    const size_t qr_bytes = mv::align_up(sizeof(QueryResult) * (size_t)batch * N, 256);
    char *sc = (char *)mv::scratch(ctx, qr_bytes + (fast ? sizeof(unsigned long long) * (size_t)batch * cols : 0));
    if (!sc) return MV_ERR_OUT_OF_MEMORY;
    QueryResult *qr = (QueryResult *)sc;
    if (fast) {
        unsigned long long *masks = (unsigned long long *)(sc + qr_bytes);
        const long tcols = (long)batch * cols;
        MV_PROF_BEGIN(ctx->stream, "k_window_mask");
        hipLaunchKernelGGL(k_window_mask, dim3((unsigned)((tcols + 255) / 256)), dim3(256), 0, ctx->stream, tcols, rows,
                           max_idx0, probs0, a.prob_thr, masks);
        MV_PROF_END(ctx->stream);
        MV_LAUNCH_CHECK();
        const bool tiled = !a.as_built && kBandW + 2 * p->radius <= 64 && cells <= 65536 && cols <= 1024 &&
                           (long)(kBandW + 2 * p->radius) * rows <= kBandList;
        if (tiled) {
            const int bpp = (N + 4 * kWQ - 1) / (4 * kWQ);
            const long nblk = (long)bpp * batch;
            MV_REQUIRE(nblk < (1l << 30));
            const unsigned g = (unsigned)((nblk + 7) / 8 * 8);
            MV_PROF_BEGIN(ctx->stream, "k_window_eval");
            hipLaunchKernelGGL(k_window_wave, dim3(g), dim3(256), 0, ctx->stream, a, bpp, (int)nblk, masks, desc0,
                               desc1, num_selected, patches1, qr);
            MV_PROF_END(ctx->stream);
            MV_LAUNCH_CHECK();
        } else {
        const int bpp = (N + 4 * kQPW - 1) / (4 * kQPW);
        const long nblocks = (long)bpp * batch;
        MV_REQUIRE(nblocks < (1l << 30));
        const unsigned grid = (unsigned)((nblocks + 7) / 8 * 8);
        MV_PROF_BEGIN(ctx->stream, "k_window_eval");
        if (a.as_built)
            hipLaunchKernelGGL(k_window_query<true>, dim3(grid), dim3(256), 0, ctx->stream, a, bpp, (int)nblocks,
                               masks, desc0, desc1, num_selected, patches1, qr);
        else
            hipLaunchKernelGGL(k_window_query<false>, dim3(grid), dim3(256), 0, ctx->stream, a, bpp, (int)nblocks,
                               masks, desc0, desc1, num_selected, patches1, qr);
        MV_PROF_END(ctx->stream);
        MV_LAUNCH_CHECK();
        }
    } else {
        MV_PROF_BEGIN(ctx->stream, "k_window_eval");
        hipLaunchKernelGGL(k_window_eval, dim3((N + 3) / 4, batch), dim3(256), 0, ctx->stream, a, desc0, max_idx0,
                           probs0, desc1, num_selected, patches1, qr);
        MV_PROF_END(ctx->stream);
        MV_LAUNCH_CHECK();
    }
    MV_PROF_BEGIN(ctx->stream, "k_window_compact");
    hipLaunchKernelGGL(k_window_compact, dim3(batch), dim3(1024), 0, ctx->stream, N, rows, p->max_matches, qr,
                       num_selected, patches1, indices1, max_idx0, cells, num_matches, points1, points2,
                       query_of_match);
    MV_PROF_END(ctx->stream);
    MV_LAUNCH_CHECK();
    return MV_OK;
}
