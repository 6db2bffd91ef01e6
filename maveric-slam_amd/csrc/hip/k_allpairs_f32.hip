// k_allpairs_f32.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659)
// with the gemmini_functions_cpu.h:14-56 summation order as the exact score.
//
// k_ap_match: ONE kernel per batch.  A 512-thread block (8 waves: 4 row groups x 2 column
// groups) owns 128 query rows of one pair and sweeps ALL column tiles of the other frame:
//   * S = D0 . D1^T on v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, k permuted); each wave
//     computes 32 rows x 64 columns of a 128-column tile (2 accumulators of 32x32);
//   * K = 256 streamed in 32-wide slices into a DOUBLE-BUFFERED LDS image by
//     global_load_lds (HBM/L2 -> LDS DMA, no staging VGPRs, issued from inline asm with
//     immediate K offsets so the compiler does not drain it before unrelated ds_reads);
//     the image is XOR-swizzled by 16-B chunk (chunk ^ ((row >> 1) & 7)) on the SOURCE
//     address and on the read -> conflict-free ds_read_b128; one barrier per slice;
//   * after each column tile every lane folds its accumulators into a lane-local running
//     (max1, idx1, max2) per row (selects only) -- no per-tile LDS epilogue;
//   * |a_i|^2 and max_j |b_j|^2 from each thread's own DMA'd chunks (bound only);
//   * at the end: cross-lane / cross-wave merge of the triples, then the EXACT re-score in
//     the reference order (v_mul_f32 + v_add_f32, k = 0..255) of the screen maximiser.
//     Rounding bound: both the MFMA chain and the sequential sum are within
//     gamma_256 * sum|a_k b_k| <= gamma_256 |a| |b| of the real dot, so every possible
//     maximiser has a screen score >= M - 2 delta, delta = 2 gamma_256 |a| max|b|.  When
//     the runner-up is inside that window the row is AMBIGUOUS and one wave re-scores all
//     of its columns exactly (slow path: only near-duplicate descriptors trigger it).
//   Result = the reference's rule: the first j with the maximum exact score, kept when
//   (double)score > thresh and score > 0 (max_score starts at 0, pairwise_pnp.py:644).
// Bound: FP32 MFMA (157.3 TF/s); per pair 2 * n0 * n1 * 256 FLOP = 536.9 MFLOP at 1024^2
// on 2 x 1 MiB of descriptors.
#include <math.h>

#include <utility>

#include "mv_internal.hpp"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, KD = 256, KS = KD / BK, NT = 512;
constexpr int TILE_FLOATS = BM * BK;  // one A or B slice: 128 rows x 128 B, swizzled
// LDS map (ONE array -- a second __shared__ object can de-pipeline the DMA), byte offsets
constexpr int OFF_STAGE = 0;                          // [2 buf][A, B][128][32] f32
constexpr int STAGE_BYTES = 2 * 2 * TILE_FLOATS * 4;  // 65,536
constexpr int OFF_ANORM = STAGE_BYTES;                // [128] f32 |a_i|^2
constexpr int OFF_TRIP = OFF_ANORM + BM * 4;          // [2 wc][128] {m1, i1, m2}
constexpr int OFF_AMB = OFF_TRIP + 2 * BM * 12;       // [128] i32 ambiguous rows
constexpr int OFF_MISC = OFF_AMB + BM * 4;            // [8] f32 per-wave max|b|^2, [1] i32 #ambiguous
constexpr int LDS_BYTES = OFF_MISC + 48;

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <class F, int... I>
__device__ __forceinline__ void static_for(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// 16-B-per-lane HBM/L2 -> LDS DMA (global_load_lds_dwordx4, SADDR form): source = SGPR
// base + 32-bit VGPR byte offset; LDS destination = M0 (wave-uniform byte address) + lane *
// 16.  No instruction offset: it would displace the LDS destination as well.  The slice's
// K offset goes into the scalar base instead (one s_add per load, no VALU).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_byte)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// Fold one tile's two columns of a row (v0 at column j, v1 at j + 32; -inf past n1) into the
// running triple.  Earlier tiles hold smaller column indices, so a tie never replaces
// (strict >); within the pair the lower column wins a tie.  Selects only.
__device__ __forceinline__ void fold2(float v0, float v1, int j, float &m1, int &i1, float &m2) {
    const bool hi = v1 > v0;
    const float t1 = fmaxf(v0, v1), t2 = fminf(v0, v1);
    const int tj = hi ? j + 32 : j;
    const bool top = t1 > m1;
    m2 = top ? fmaxf(m1, t2) : fmaxf(m2, t1);
    m1 = top ? t1 : m1;
    i1 = top ? tj : i1;
}

// order-independent merge of two (max1, idx1, max2) triples
__device__ __forceinline__ void merge(float &m1, int &i1, float &m2, float o1, int oi, float o2) {
    if (o1 > m1 || (o1 == m1 && oi < i1)) {
        m2 = fmaxf(o2, m1);
        m1 = o1;
        i1 = oi;
    } else {
        m2 = fmaxf(m2, o1);
    }
}

// XCD-aware bijective remap: blocks b and b+8 share an XCD (round-robin dispatch); give
// each XCD a contiguous run of logical blocks so a pair's row tiles share one L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total / 8, r = total % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// the reference's score: s = 0; s = s + a[k]*b[k], k = 0..255 (no FMA: -ffp-contract=off)
__device__ __forceinline__ float exact_dot(const float *__restrict__ a, const float *__restrict__ b) {
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < KD; k += 4) {
        const float4 x = *reinterpret_cast<const float4 *>(a + k);
        const float4 y = *reinterpret_cast<const float4 *>(b + k);
        s = __fadd_rn(s, __fmul_rn(x.x, y.x));
        s = __fadd_rn(s, __fmul_rn(x.y, y.y));
        s = __fadd_rn(s, __fmul_rn(x.z, y.z));
        s = __fadd_rn(s, __fmul_rn(x.w, y.w));
    }
    return s;
}

__device__ __forceinline__ float sum8(float v) {  // over the 8 lanes (l & 7) of a DMA row
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    return v;
}

__device__ __forceinline__ float nrm4(float4 x, float acc) {
    return fmaf(x.x, x.x, fmaf(x.y, x.y, fmaf(x.z, x.z, fmaf(x.w, x.w, acc))));
}

__global__ __launch_bounds__(NT, 2) void k_ap_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                    const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                    const float *__restrict__ desc1, double thresh,
                                                    int *__restrict__ match_idx, float *__restrict__ match_score) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    const float *stage_lds = reinterpret_cast<const float *>(lds + OFF_STAGE);
    float *anorm2 = reinterpret_cast<float *>(lds + OFF_ANORM);
    float *trip = reinterpret_cast<float *>(lds + OFF_TRIP);
    int *amb = reinterpret_cast<int *>(lds + OFF_AMB);
    float *misc = reinterpret_cast<float *>(lds + OFF_MISC);
    int *namb_p = reinterpret_cast<int *>(lds + OFF_MISC) + 8;

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int pair = L / tiles_r, tr = L % tiles_r;
    const int n0 = n0v[pair], n1 = n1v[pair];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
    const int row0 = tr * BM;
    int *oidx = match_idx + (size_t)pair * cap + row0;
    float *oscore = match_score + (size_t)pair * cap + row0;
    // rows in [n0, cap) report "no match"
    if (t < BM && row0 + t < cap && (row0 + t >= n0 || n1 <= 0)) {
        oidx[t] = -1;
        oscore[t] = 0.f;
    }
    if (row0 >= n0 || n1 <= 0) return;
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;
    const int ntc = (n1 + BN - 1) / BN;

    // ---- DMA map: wave w fills rows w*16 .. w*16+15 of each slice (A and B), 8 rows
    //      (1 KiB) per instruction; lane l lands at row (l >> 3), chunk position l & 7 and
    //      fetches global chunk (l & 7) ^ ((row >> 1) & 7) of that row ----
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int dr0 = wu * 16 + (lane >> 3), dr1 = dr0 + 8;
    const int dc0 = ((lane & 7) ^ ((dr0 >> 1) & 7)) * 4, dc1 = ((lane & 7) ^ ((dr1 >> 1) & 7)) * 4;
    // per-lane source byte offsets (rows clamped into [0, n)); A's stay fixed, B's advance per tile
    const unsigned oA0 = (unsigned)(min(row0 + dr0, n0 - 1) * KD + dc0) * 4u;
    const unsigned oA1 = (unsigned)(min(row0 + dr1, n0 - 1) * KD + dc1) * 4u;
    unsigned oB0 = (unsigned)(min(dr0, n1 - 1) * KD + dc0) * 4u;
    unsigned oB1 = (unsigned)(min(dr1, n1 - 1) * KD + dc1) * 4u;
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)(lds + OFF_STAGE);
    const unsigned dst_w = lds_base + (unsigned)(wu * 16 * BK * 4);
#define AP_STAGE(BUF, KSI)                                                                   \
    do {                                                                                     \
        const unsigned d_ = dst_w + (unsigned)((BUF) * 2 * TILE_FLOATS * 4);                 \
        const float *sa_ = A + (KSI) * BK, *sb_ = B + (KSI) * BK;                            \
        glds16(sa_, oA0, d_);                                                                \
        glds16(sa_, oA1, d_ + 8 * BK * 4);                                                   \
        glds16(sb_, oB0, d_ + TILE_FLOATS * 4);                                              \
        glds16(sb_, oB1, d_ + TILE_FLOATS * 4 + 8 * BK * 4);                                 \
    } while (0)

    // ---- fragment read map: lane half h takes k = h*16 + s at MFMA step s (chunk h*4 + s/4)
    const int fr = lane & 31, fh = lane >> 5;
    const int ra = wr * 32 + fr, rb = wc * 64 + fr;  // rb + 32 has the same swizzle
    const int swa = (ra >> 1) & 7, swb = (rb >> 1) & 7;
    const int offa = ra * BK, offb = TILE_FLOATS + rb * BK;

    f32x16 acc0, acc1;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        acc0[q] = 0.f;
        acc1[q] = 0.f;
    }
    float m1[16], m2[16];
    int i1[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        m1[q] = -__builtin_inff();
        m2[q] = -__builtin_inff();
        i1[q] = 0x7fffffff;
    }
    float asq0 = 0.f, asq1 = 0.f, bsq0 = 0.f, bsq1 = 0.f, bmax = 0.f;
    const int nro0 = dr0 * BK + (lane & 7) * 4, nro1 = dr1 * BK + (lane & 7) * 4;  // own chunks

#define AP_SLICE(ks)                                                                          \
    do {                                                                                      \
        constexpr int cur = (ks) & 1; /* KS is even: slice ks of a tile lives in buffer ks & 1 */ \
 /* DMA of the next slice (the next tile's slice 0 after the last) overlaps the MFMAs */ \
            if constexpr ((ks) + 1 < KS) { \
                AP_STAGE(cur ^ 1, ks + 1); \
            } else { \
                if (!last_tile) { \
                    oB0 = (unsigned)(min((tc + 1) * BN + dr0, n1 - 1) * KD + dc0) * 4u; \
                    oB1 = (unsigned)(min((tc + 1) * BN + dr1, n1 - 1) * KD + dc1) * 4u; \
                    AP_STAGE(cur ^ 1, 0); \
                } \
            } \
            const float *base = stage_lds + cur * 2 * TILE_FLOATS; \
            { /* norms for the rounding bound, from this thread's own DMA'd chunks */ \
                const float4 nb0 = *reinterpret_cast<const float4 *>(base + TILE_FLOATS + nro0); \
                const float4 nb1 = *reinterpret_cast<const float4 *>(base + TILE_FLOATS + nro1); \
                bsq0 = nrm4(nb0, bsq0); \
                bsq1 = nrm4(nb1, bsq1); \
                if (tc == 0) { \
                    const float4 na0 = *reinterpret_cast<const float4 *>(base + nro0); \
                    const float4 na1 = *reinterpret_cast<const float4 *>(base + nro1); \
                    asq0 = nrm4(na0, asq0); \
                    asq1 = nrm4(na1, asq1); \
                } \
            } \
_Pragma("unroll") \
            for (int v = 0; v < 4; v++) { /* 3 float4 fragment reads feed 8 MFMAs (4 k-steps x 2 n) */ \
                const float4 a = *reinterpret_cast<const float4 *>(base + offa + (((fh * 4 + v) ^ swa) * 4)); \
                const float4 b0 = *reinterpret_cast<const float4 *>(base + offb + (((fh * 4 + v) ^ swb) * 4)); \
                const float4 b1 = \
                    *reinterpret_cast<const float4 *>(base + offb + 32 * BK + (((fh * 4 + v) ^ swb) * 4)); \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b0.x, acc0, 0, 0, 0); \
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b1.x, acc1, 0, 0, 0); \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b0.y, acc0, 0, 0, 0); \
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b1.y, acc1, 0, 0, 0); \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b0.z, acc0, 0, 0, 0); \
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b1.z, acc1, 0, 0, 0); \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b0.w, acc0, 0, 0, 0); \
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b1.w, acc1, 0, 0, 0); \
            } \
            if constexpr ((ks) == KS - 1) { \
 /* column tile done: fold the accumulators into the lane-local triples */ \
                const int col = tc * BN + wc * 64 + fr; \
                const float lo0 = col < n1 ? 0.f : -__builtin_inff(); /* + 0 keeps, + -inf drops */ \
                const float lo1 = col + 32 < n1 ? 0.f : -__builtin_inff(); \
_Pragma("unroll") \
                for (int q = 0; q < 16; q++) { \
                    fold2(acc0[q] + lo0, acc1[q] + lo1, col, m1[q], i1[q], m2[q]); \
                    acc0[q] = 0.f; \
                    acc1[q] = 0.f; \
                } \
                { /* row norms: the 8 lanes (l & 7) of a DMA row hold its 8 chunks */ \
                    const float c0 = sum8(bsq0), c1 = sum8(bsq1); \
                    bmax = fmaxf(bmax, fmaxf(tc * BN + dr0 < n1 ? c0 : 0.f, tc * BN + dr1 < n1 ? c1 : 0.f)); \
                    bsq0 = bsq1 = 0.f; \
                    if (tc == 0) { \
                        const float r0 = sum8(asq0), r1 = sum8(asq1); \
                        if ((lane & 7) == 0) { \
                            anorm2[dr0] = r0; \
                            anorm2[dr1] = r1; \
                        } \
                    } \
                } \
            } \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* the next slice has landed */ \
            __syncthreads(); \
    } while (0)

    AP_STAGE(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int tc = 0; tc < ntc; tc++) {
        const bool last_tile = tc + 1 == ntc;
        AP_SLICE(0);
        AP_SLICE(1);
        AP_SLICE(2);
        AP_SLICE(3);
        AP_SLICE(4);
        AP_SLICE(5);
        AP_SLICE(6);
        AP_SLICE(7);
    }
#undef AP_STAGE
#undef AP_SLICE

    // ---- merge the triples: across the 32 lanes of each half, then across the 2 column waves ----
#pragma unroll
    for (int q = 0; q < 16; q++) {
        float a1 = m1[q], a2 = m2[q];
        int ai = i1[q];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            const float b1 = __shfl_xor(a1, o, 64), b2 = __shfl_xor(a2, o, 64);
            const int bi = __shfl_xor(ai, o, 64);
            merge(a1, ai, a2, b1, bi, b2);
        }
        if (fr == 0) {
            const int row = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * fh;  // 32x32 C/D row map
            float *tp = trip + (wc * BM + row) * 3;
            tp[0] = a1;
            reinterpret_cast<int *>(tp)[1] = ai;
            tp[2] = a2;
        }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) bmax = fmaxf(bmax, __shfl_xor(bmax, o, 64));
    if (lane == 0) misc[w] = bmax;
    if (t == 0) *namb_p = 0;
    __syncthreads();
    float bmax2 = misc[0];
#pragma unroll
    for (int k = 1; k < 8; k++) bmax2 = fmaxf(bmax2, misc[k]);

    // ---- exact re-score, fast path: the screen maximiser is the only possible maximiser ----
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double gamma = KD * u / (1.0 - KD * u);
    const double nb = sqrt((double)bmax2);
    if (t < BM && row0 + t < n0) {
        const float *tp0 = trip + t * 3, *tp1 = trip + (BM + t) * 3;
        float M = tp0[0], M2 = tp0[2];
        int I = reinterpret_cast<const int *>(tp0)[1];
        merge(M, I, M2, tp1[0], reinterpret_cast<const int *>(tp1)[1], tp1[2]);
        const double delta = 2.0 * gamma * sqrt((double)anorm2[t]) * nb * 1.01 + 1e-30;
        int best = -1;
        float bs = 0.f;
        bool ambiguous = false;
        if ((double)M + delta > thresh) {
            if ((double)M2 >= (double)M - 2.0 * delta) {
                ambiguous = true;
                amb[atomicAdd(namb_p, 1)] = t;
            } else {
                const float e = exact_dot(A + (size_t)(row0 + t) * KD, B + (size_t)I * KD);
                if ((double)e > thresh && e > 0.f) {
                    bs = e;
                    best = I;
                }
            }
        }
        if (!ambiguous) {
            oidx[t] = best;
            oscore[t] = best >= 0 ? bs : 0.f;
        }
    }
    __syncthreads();
    // ---- slow path: one wave re-scores every column of an ambiguous row exactly ----
    const int namb = *namb_p;
    for (int k = w; k < namb; k += NT / 64) {
        const int r = amb[k];
        const float *a = A + (size_t)(row0 + r) * KD;
        int best = 0x7fffffff;
        float bs = -__builtin_inff();
        for (int j = lane; j < n1; j += 64) {
            const float e = exact_dot(a, B + (size_t)j * KD);
            if (e > bs) {  // j ascending per lane: strict > keeps the first
                bs = e;
                best = j;
            }
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const float ob = __shfl_xor(bs, o, 64);
            const int oj = __shfl_xor(best, o, 64);
            if (ob > bs || (ob == bs && oj < best)) {
                bs = ob;
                best = oj;
            }
        }
        if (lane == 0) {
            const bool keep = (double)bs > thresh && bs > 0.f;
            oidx[r] = keep ? best : -1;
            oscore[r] = keep ? bs : 0.f;
        }
    }
}

}  // namespace

namespace mv {

size_t allpairs_f32_scratch_bytes(int batch, int cap) {
    (void)batch;
    (void)cap;
    return 256;
}

int launch_allpairs_f32(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                        const float *desc0, const float *desc1, double thresh, int *match_idx,
                        float *match_score) {
    (void)scratch;
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx && match_score);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    const int tiles_r = (cap + BM - 1) / BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    MV_REQUIRE(cap <= (1 << 21));  // per-lane DMA source offsets are 32-bit byte offsets into a pair
    MV_PROF_BEGIN(s, "k_ap_match");
    hipLaunchKernelGGL(k_ap_match, dim3((unsigned)blocks), dim3(NT), 0, s, tiles_r, cap, n0, n1, desc0, desc1, thresh,
                       match_idx, match_score);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

extern "C" int mv_match_allpairs_f32_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                         const float *desc0, const float *desc1, double thresh, int *match_idx,
                                         float *match_score) {
    MV_REQUIRE(ctx != nullptr);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    return mv::launch_allpairs_f32(ctx->stream, nullptr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                   match_score);
}
