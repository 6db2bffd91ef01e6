// k_allpairs_f32.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659)
// with the gemmini_functions_cpu.h:14-56 summation order as the exact score.
//
// Two kernels per batch:
//   k_ap_split  one pass over both frames: every fp32 descriptor a becomes a bf16 pair
//               (a_hi = bf16(a), a_lo = bf16(a - a_hi)) stored SLICE-INTERLEAVED
//               ([hi k0..k0+31 | lo k0..k0+31] per 32-wide k slice, 1 KiB per row, the
//               same bytes as the fp32 row) and |a|^2.  HBM-bound: 4 B read + 4 B written
//               per element.
//   k_ap_match  a 512-thread block (8 waves: 4 row groups x 2 column groups) owns 128 query
//               rows of one pair and sweeps ALL column tiles of the other frame:
//     * screen S ~= D0 . D1^T as a_hi b_hi + a_hi b_lo + a_lo b_hi on
//       v_mfma_f32_32x32x16_bf16 (3 bf16 products per fp32 product: 3/16 of the fp32-MFMA
//       cycles), each wave 32 rows x 64 columns of a 128-column tile;
//     * k streamed in 32-wide slices through a NBUF-deep LDS ring filled by
//       global_load_lds (HBM/L2 -> LDS DMA, no staging VGPRs, issued NBUF-1 slices ahead),
//       XOR-swizzled by 16-B chunk (chunk ^ ((row >> 1) & 7)) on the SOURCE address and on
//       the read -> conflict-free ds_read_b128; one barrier per slice;
//     * after each column tile every lane folds its accumulators into a lane-local running
//       (max1, idx1, max2) per row (selects only);
//     * at the end: cross-lane / cross-wave merge of the triples, then the EXACT re-score in
//       the reference order (v_mul_f32 + v_add_f32, k = 0..255, fp32 inputs) of the screen
//       maximiser.
//   Why the result is exact (bit-identical to the reference): with d_j the real dot product,
//   s_j the screen and e_j the reference's sequential fp32 sum,
//     |s_j - d_j| <= ds = (3.1 * 2^-16 + 1.02 gamma_768(2^-23)) |a| max|b|
//       (split residuals and the dropped a_lo b_lo term; 768 fp32 accumulations inside the
//        MFMA bounded with unit roundoff 2^-23, i.e. even for truncating adders),
//     |e_j - d_j| <= de = gamma_256(2^-24) |a| |b|.
//   Any column whose exact score can reach the screen maximiser's has s_j >= M - 2(ds + de).
//   If the runner-up screen value is below that window, the screen maximiser IS the
//   reference's maximiser (ties included) and one exact dot decides the threshold; otherwise
//   the row is AMBIGUOUS and one wave re-scores all of its columns exactly (slow path:
//   only rows that can pass the threshold and have a near-equal runner-up reach it).
//   Result = the reference's rule: the first j with the maximum exact score, kept when
//   (double)score > thresh and score > 0 (max_score starts at 0, pairwise_pnp.py:644).
// Bound: BF16 MFMA.  Per pair 2 * n0 * n1 * 256 algorithmic FLOP (536.9 MFLOP at 1024^2),
// executed as 3x that on the bf16 pipe: peak 2.5 PF / 3 = 833 TF/s fp32-equivalent.
#include <math.h>

#include "mv_internal.hpp"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, KD = 256, KS = KD / BK, NT = 512, NBUF = 4;
constexpr int ROW_BYTES = 2 * KD * 2;            // split row: 256 hi + 256 lo bf16 = 1 KiB
constexpr int SL_ROW = BK * 2 * 2;               // one row of one slice: 32 hi + 32 lo = 128 B
constexpr int SL_BYTES = BM * SL_ROW;            // one operand slice (A or B): 16 KiB
constexpr int BUF_BYTES = 2 * SL_BYTES;          // A + B
static_assert(KS % NBUF == 0, "ring slots must be compile-time per slice");
// LDS map (ONE array -- a second __shared__ object can de-pipeline the DMA), byte offsets
constexpr int OFF_STAGE = 0;                     // [NBUF][A, B][128 rows][128 B]
constexpr int OFF_TRIP = NBUF * BUF_BYTES;       // [2 wc][128] {m1, i1, m2}
constexpr int OFF_AMB = OFF_TRIP + 2 * BM * 12;  // [128] i32 ambiguous rows
constexpr int OFF_MISC = OFF_AMB + BM * 4;       // [8] f32 per-wave max|b|^2, [1] i32 #ambiguous
constexpr int LDS_BYTES = OFF_MISC + 48;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

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

// s_waitcnt on vmcnt only (expcnt / lgkmcnt left at their no-wait maxima)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

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

__device__ __forceinline__ unsigned pack_bf16(float x, float y) {
    const bf16x2 v = {(__bf16)x, (__bf16)y};  // v_cvt_pk_bf16_f32 (round to nearest even)
    return __builtin_bit_cast(unsigned, v);
}

// ---- k_ap_split: one wave per descriptor row (rows >= n are never read downstream) ----
__global__ __launch_bounds__(256) void k_ap_split(int batch, int cap, const int *__restrict__ n0v,
                                                  const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                  const float *__restrict__ desc1, char *__restrict__ split0,
                                                  char *__restrict__ split1, float *__restrict__ nrm0,
                                                  float *__restrict__ nrm1) {
    const long R = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long per_frame = (long)batch * cap;
    if (R >= 2 * per_frame) return;
    const int frame = R >= per_frame;
    const long fr = frame ? R - per_frame : R;
    const int pair = (int)(fr / cap), r = (int)(fr % cap);
    if (r >= (frame ? n1v : n0v)[pair]) return;
    const int lane = threadIdx.x & 63;
    const float4 v = *reinterpret_cast<const float4 *>((frame ? desc1 : desc0) + fr * KD + lane * 4);
    const unsigned h01 = pack_bf16(v.x, v.y), h23 = pack_bf16(v.z, v.w);
    // a - a_hi is exact in f32 (a_hi is within 2^-8 of a); then rounded to bf16
    const float hx = __uint_as_float(h01 << 16), hy = __uint_as_float(h01 & 0xffff0000u);
    const float hz = __uint_as_float(h23 << 16), hw = __uint_as_float(h23 & 0xffff0000u);
    const unsigned l01 = pack_bf16(v.x - hx, v.y - hy), l23 = pack_bf16(v.z - hz, v.w - hw);
    // element k = 4 lane .. 4 lane + 3 sits in slice lane / 8 at position (lane & 7) * 4
    char *row = (frame ? split1 : split0) + fr * ROW_BYTES + (lane >> 3) * SL_ROW + (lane & 7) * 8;
    *reinterpret_cast<uint2 *>(row) = make_uint2(h01, h23);
    *reinterpret_cast<uint2 *>(row + BK * 2) = make_uint2(l01, l23);
    float q = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, v.w * v.w)));
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
    if (lane == 0) (frame ? nrm1 : nrm0)[fr] = q;
}

__global__ __launch_bounds__(NT, 1) void k_ap_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                    const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                    const float *__restrict__ desc1,
                                                    const char *__restrict__ split0,
                                                    const char *__restrict__ split1,
                                                    const float *__restrict__ nrm0,
                                                    const float *__restrict__ nrm1, double thresh,
                                                    int *__restrict__ match_idx, float *__restrict__ match_score) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
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
    const char *SA = split0 + (size_t)pair * cap * ROW_BYTES;
    const char *SB = split1 + (size_t)pair * cap * ROW_BYTES;
    const int ntc = (n1 + BN - 1) / BN;

    // ---- DMA map: wave w fills rows w*16 .. w*16+15 of each slice (A and B), 8 rows
    //      (1 KiB) per instruction; lane l lands at row (l >> 3), chunk position l & 7 and
    //      fetches source chunk (l & 7) ^ ((row >> 1) & 7) of that row ----
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int dr0 = wu * 16 + (lane >> 3), dr1 = dr0 + 8;
    const int dc0 = ((lane & 7) ^ ((dr0 >> 1) & 7)) * 16, dc1 = ((lane & 7) ^ ((dr1 >> 1) & 7)) * 16;
    // per-lane source byte offsets (rows clamped into [0, n)); A's stay fixed, B's advance per tile
    const unsigned oA0 = (unsigned)min(row0 + dr0, n0 - 1) * ROW_BYTES + dc0;
    const unsigned oA1 = (unsigned)min(row0 + dr1, n0 - 1) * ROW_BYTES + dc1;
    unsigned oB0 = (unsigned)min(dr0, n1 - 1) * ROW_BYTES + dc0;
    unsigned oB1 = (unsigned)min(dr1, n1 - 1) * ROW_BYTES + dc1;
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)(lds + OFF_STAGE);
    const unsigned dst_w = lds_base + (unsigned)(wu * 16 * SL_ROW);
#define AP_STAGE(BUF, KSI)                                                                   \
    do {                                                                                     \
        const unsigned d_ = dst_w + (unsigned)((BUF) * BUF_BYTES);                           \
        const char *sa_ = SA + (KSI) * SL_ROW, *sb_ = SB + (KSI) * SL_ROW;                   \
        glds16(sa_, oA0, d_);                                                                \
        glds16(sa_, oA1, d_ + 8 * SL_ROW);                                                   \
        glds16(sb_, oB0, d_ + SL_BYTES);                                                     \
        glds16(sb_, oB1, d_ + SL_BYTES + 8 * SL_ROW);                                        \
    } while (0)

    // ---- fragment read map: at k16 step s of a slice, lane half h holds k = s*16 + h*8 .. +7:
    //      hi chunk s*2 + h, lo chunk 4 + s*2 + h of the 128-B slice row ----
    const int fr = lane & 31, fh = lane >> 5;
    const int ra = wr * 32 + fr, rb = wc * 64 + fr;  // rb + 32 has the same swizzle
    const int swa = (ra >> 1) & 7, swb = (rb >> 1) & 7;
    const int offa = ra * SL_ROW, offb = SL_BYTES + rb * SL_ROW;

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

    // Ring schedule: global slice g = tc*KS + ks lives in slot g % NBUF = ks % NBUF.  At slice
    // g the block issues slice g + NBUF - 1 into the slot read at g - 1 (freed by that
    // slice's barrier), computes slice g, then waits until slice g + 1 has landed: the DMA
    // groups issued after it (4 instructions each) may stay in flight.
#define AP_SLICE(ks)                                                                          \
    do {                                                                                      \
        constexpr int nx = (ks) + NBUF - 1; /* slice issued now, counted from this tile */    \
        if constexpr (nx < KS) {                                                              \
            AP_STAGE(nx % NBUF, nx);                                                          \
        } else if (!last_tile) {                                                              \
            if constexpr (nx == KS) { /* first slice of the next column tile */               \
                oB0 = (unsigned)min((tc + 1) * BN + dr0, n1 - 1) * ROW_BYTES + dc0;           \
                oB1 = (unsigned)min((tc + 1) * BN + dr1, n1 - 1) * ROW_BYTES + dc1;           \
            }                                                                                 \
            AP_STAGE(nx % NBUF, nx - KS);                                                     \
        }                                                                                     \
        const char *base = lds + OFF_STAGE + ((ks) % NBUF) * BUF_BYTES;                       \
        _Pragma("unroll") for (int st = 0; st < 2; st++) {                                    \
            const int ch = st * 2 + fh;                                                       \
            const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(base + offa + ((ch ^ swa) * 16));       \
            const bf16x8 al = *reinterpret_cast<const bf16x8 *>(base + offa + (((ch + 4) ^ swa) * 16)); \
            const bf16x8 b0h = *reinterpret_cast<const bf16x8 *>(base + offb + ((ch ^ swb) * 16));      \
            const bf16x8 b0l = *reinterpret_cast<const bf16x8 *>(base + offb + (((ch + 4) ^ swb) * 16)); \
            const bf16x8 b1h = *reinterpret_cast<const bf16x8 *>(base + offb + 32 * SL_ROW + ((ch ^ swb) * 16)); \
            const bf16x8 b1l =                                                                \
                *reinterpret_cast<const bf16x8 *>(base + offb + 32 * SL_ROW + (((ch + 4) ^ swb) * 16)); \
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b0h, acc0, 0, 0, 0);           \
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b1h, acc1, 0, 0, 0);           \
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b0l, acc0, 0, 0, 0);           \
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b1l, acc1, 0, 0, 0);           \
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b0h, acc0, 0, 0, 0);           \
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b1h, acc1, 0, 0, 0);           \
        }                                                                                     \
        if constexpr ((ks) == KS - 1) { /* column tile done: fold into the lane triples */    \
            const int col = tc * BN + wc * 64 + fr;                                           \
            const float lo0 = col < n1 ? 0.f : -__builtin_inff(); /* + 0 keeps, + -inf drops */ \
            const float lo1 = col + 32 < n1 ? 0.f : -__builtin_inff();                        \
            _Pragma("unroll") for (int q = 0; q < 16; q++) {                                  \
                fold2(acc0[q] + lo0, acc1[q] + lo1, col, m1[q], i1[q], m2[q]);                \
                acc0[q] = 0.f;                                                                \
                acc1[q] = 0.f;                                                                \
            }                                                                                 \
        }                                                                                     \
        /* slice g + 1 must have landed: in flight after it are the groups of slices */       \
        /* g + 2 .. g + NBUF - 1, all issued unless past the block's last slice */           \
        if (!last_tile) {                                                                     \
            wait_vm<4 * (NBUF - 2)>();                                                        \
        } else {                                                                              \
            constexpr int fl = (KS - 2 - (ks)) < (NBUF - 2) ? (KS - 2 - (ks)) : (NBUF - 2);  \
            wait_vm<4 * (fl > 0 ? fl : 0)>();                                                 \
        }                                                                                     \
        __syncthreads();                                                                      \
    } while (0)

    // prologue: slices 0 .. NBUF-2 of tile 0, then wait for slice 0
    static_assert(NBUF == 4, "prologue issues NBUF - 1 = 3 slices");
    AP_STAGE(0, 0);
    AP_STAGE(1, 1);
    AP_STAGE(2, 2);
    wait_vm<4 * (NBUF - 2)>();
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
    // max_j |b_j|^2 over the pair's valid columns (from k_ap_split)
    const float *nb2 = nrm1 + (size_t)pair * cap;
    float bmax = 0.f;
    for (int j = t; j < n1; j += NT) bmax = fmaxf(bmax, nb2[j]);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) bmax = fmaxf(bmax, __shfl_xor(bmax, o, 64));
    if (lane == 0) misc[w] = bmax;
    if (t == 0) *namb_p = 0;
    __syncthreads();
    float bmax2 = misc[0];
#pragma unroll
    for (int k = 1; k < 8; k++) bmax2 = fmaxf(bmax2, misc[k]);

    // ---- exact re-score, fast path: the screen maximiser is the only possible maximiser ----
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;
    const double u24 = 5.9604644775390625e-08, u23 = 2 * u24;
    const double gam_e = KD * u24 / (1.0 - KD * u24);
    const double gam_s = 3 * KD * u23 / (1.0 - 3 * KD * u23);
    const double coef = 3.1 * 1.52587890625e-05 + 1.02 * gam_s + gam_e;  // ds + de per |a| max|b|
    const double nb = sqrt((double)bmax2);
    if (t < BM && row0 + t < n0) {
        const float *tp0 = trip + t * 3, *tp1 = trip + (BM + t) * 3;
        float M = tp0[0], M2 = tp0[2];
        int I = reinterpret_cast<const int *>(tp0)[1];
        merge(M, I, M2, tp1[0], reinterpret_cast<const int *>(tp1)[1], tp1[2]);
        const double delta = coef * sqrt((double)nrm0[(size_t)pair * cap + row0 + t]) * nb * 1.01 + 1e-30;
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

// scratch: split0 | split1 (batch * cap * 1 KiB each) | nrm0 | nrm1 (batch * cap f32 each)
size_t allpairs_f32_scratch_bytes(int batch, int cap) {
    const size_t rows = (size_t)batch * cap;
    return 2 * rows * ROW_BYTES + 2 * align_up(rows * 4, 256);
}

int launch_allpairs_f32(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                        const float *desc0, const float *desc1, double thresh, int *match_idx,
                        float *match_score) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx && match_score && scratch);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    const int tiles_r = (cap + BM - 1) / BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    MV_REQUIRE(cap <= (1 << 21));  // per-lane DMA source offsets are 32-bit byte offsets into a pair
    const size_t rows = (size_t)batch * cap;
    char *split0 = (char *)scratch, *split1 = split0 + rows * ROW_BYTES;
    float *nrm0 = (float *)(split1 + rows * ROW_BYTES);
    float *nrm1 = (float *)((char *)nrm0 + align_up(rows * 4, 256));
    const long split_blocks = (long)((2 * rows + 3) / 4);
    MV_REQUIRE(split_blocks < (1l << 31));
    MV_PROF_BEGIN(s, "k_ap_split");
    hipLaunchKernelGGL(k_ap_split, dim3((unsigned)split_blocks), dim3(256), 0, s, batch, cap, n0, n1, desc0, desc1,
                       split0, split1, nrm0, nrm1);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    MV_PROF_BEGIN(s, "k_ap_match");
    hipLaunchKernelGGL(k_ap_match, dim3((unsigned)blocks), dim3(NT), 0, s, tiles_r, cap, n0, n1, desc0, desc1,
                       split0, split1, nrm0, nrm1, thresh, match_idx, match_score);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

extern "C" int mv_match_allpairs_f32_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                         const float *desc0, const float *desc1, double thresh, int *match_idx,
                                         float *match_score) {
    MV_REQUIRE(ctx != nullptr && batch > 0 && cap > 0);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    void *scr = mv::scratch(ctx, mv::allpairs_f32_scratch_bytes(batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    return mv::launch_allpairs_f32(ctx->stream, scr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                   match_score);
}
