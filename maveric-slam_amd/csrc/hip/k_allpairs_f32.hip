// k_allpairs_f32.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659)
// with the gemmini_functions_cpu.h:14-56 summation order as the exact score.
//
// Two kernels per batch (plus a 4-byte-per-pair memset):
//   k_ap_split  one pass over both frames: every fp32 descriptor row becomes an fp16 row of
//               2^14 * a (round to nearest even; 512 B per row) and |a|^2.  A pair whose
//               values leave |a_k| < 2 (or are not finite) is flagged: all of its rows take the
//               exact slow path, so the fp16 range never has to be trusted.  HBM-bound: 4 B read
//               + 2 B written per element.
//   k_ap_match  a 256-thread block (4 waves, one per SIMD, 32 rows each; two blocks per CU run
//               out of phase, so one block's A load / fold overlaps the other's MFMAs) owns
//               128 query rows of one pair and sweeps ALL column tiles of the other frame:
//     * the wave's 32 rows x 256 k of A (fp16, 64 VGPRs) are loaded ONCE into registers;
//       only B streams (512 B per column per block);
//     * screen S ~= D0 . D1^T on v_mfma_f32_32x32x16_f16 (exact fp16 products, fp32
//       accumulation), each wave 32 rows x 128 columns of a tile (4 accumulators);
//     * k streamed in 64-wide slices (128 B per row) through a NBUF-deep LDS ring filled by
//       global_load_lds (HBM/L2 -> LDS DMA, no staging VGPRs, issued NBUF-1 slices ahead),
//       XOR-swizzled by 16-B chunk (chunk ^ ((row >> 1) & 7)) on the SOURCE address and on
//       the read -> conflict-free ds_read_b128; one barrier per slice;
//     * after each column tile every lane folds its accumulators into a lane-local running
//       (max1, idx1, max2) per row (selects only);
//     * at the end: cross-lane merge of the triples, then the EXACT re-score in the reference
//       order (v_mul_f32 + v_add_f32, k = 0..255, fp32 inputs) of the screen maximiser.
//   Why the result is exact (bit-identical to the reference): with d_j the real dot product,
//   s_j the screen (unscaled by 2^-28) and e_j the reference's sequential fp32 sum,
//     |s_j - d_j| <= ds = (2^-10 + 2^-22 + 1.01 gamma_256(2^-23)) |a| B
//                         + 1.001 * 2^-24 (|a| + B) + 2^-48,          B = max_j |b_j|
//       (fp16 rounding 2^-11 per operand; values below the fp16 normal range, 2^-28 in
//        original units, bounded as if flushed; sum |x_k| <= 16 |x|; 256 fp32 accumulations
//        inside the MFMA bounded with unit roundoff 2^-23, i.e. even for truncating adders),
//     |e_j - d_j| <= de = gamma_256(2^-24) |a| B.
//   Any column whose exact score can reach the screen maximiser's has s_j >= M - 2(ds + de).
//   If the runner-up screen value is below that window, the screen maximiser IS the
//   reference's maximiser (ties included) and one exact dot decides the threshold; otherwise
//   the row is AMBIGUOUS and one wave re-scores all of its columns exactly (slow path:
//   only rows that can pass the threshold and have a near-equal runner-up reach it).
//   Result = the reference's rule: the first j with the maximum exact score, kept when
//   (double)score > thresh and score > 0 (max_score starts at 0, pairwise_pnp.py:644).
// Bound: FP16 MFMA.  Per pair 2 * n0 * n1 * 256 algorithmic FLOP (536.9 MFLOP at 1024^2);
// dense fp16 MFMA peak 2.5 PF/s.
#include <math.h>

#include <algorithm>

#include "mv_internal.hpp"

namespace {

// NW: waves per block (32 rows each): 4 -> two blocks per CU, 8 -> one
constexpr int NW = 4, NT = 64 * NW, BM = 32 * NW, BN = 64, BK = 128, KD = 256, KS = KD / BK, RW = BM / NW;
constexpr int NBUF = 4;  // ring slots: two column tiles of KS = 2 slices
constexpr int ROW_BYTES = KD * 2;                // fp16 row: 512 B
constexpr int SL_ROW = BK * 2;                   // one row of one slice: 128 fp16 = 256 B = 16 chunks
constexpr int SL_BYTES = BN * SL_ROW;            // one B slice: 16 KiB
constexpr int DMA_PER_SLICE = SL_BYTES / 1024 / NW;  // 1-KiB DMA instructions per wave per slice
constexpr float SCALE = 16384.f;                 // 2^14: |a_k| < 2 -> |2^14 a_k| < 2^15 < 65504
static_assert(KS == 2 && NBUF == 2 * KS, "the loop body covers two column tiles = NBUF slices");
static_assert(RW == 32 && (NW == 4 || NW == 8), "one wave per 32 rows (32x32 MFMA), 4 or 8 waves");
// LDS map (ONE array -- a second __shared__ object can de-pipeline the DMA), byte offsets.
// The epilogue reuses the region of the (then free) ring.
constexpr int MT_STRIDE = 32 * 8 + 16;           // transpose row: 32 lanes' (m1, m2) + pad
constexpr int NCAND = 16;                        // listed candidates per row (more: wide row)
constexpr int OFF_CL = NW * 32 * MT_STRIDE;      // [BM][NCAND] candidate columns
constexpr int OFF_LM = OFF_CL + BM * NCAND * 4;  // [BM] wide rows' inside lanes
constexpr int EPI_BYTES = OFF_LM + BM * 4;
constexpr int OFF_STAGE = 0;                     // [NBUF][64 B rows][256 B]
constexpr int RING_BYTES = NBUF * SL_BYTES > EPI_BYTES ? NBUF * SL_BYTES : EPI_BYTES;
constexpr int OFF_ANRM = RING_BYTES;             // [BM] f32 |a|^2 (< 0: row outside the fp16 range)
constexpr int OFF_MISC = OFF_ANRM + BM * 4;      // [NW] f32 per-wave max|b|^2
constexpr int LDS_BYTES = OFF_MISC + 4 * NW;
static_assert(LDS_BYTES * (8 / NW) <= 160 * 1024, "LDS per CU");

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// 16-B-per-lane HBM/L2 -> LDS DMA (global_load_lds_dwordx4, SADDR form): source = SGPR
// base + 32-bit VGPR byte offset; LDS destination = M0 (wave-uniform byte address) + lane *
// 16.  No instruction offset: it would displace the LDS destination as well.  The constant
// K offset (KOFF) and LDS offset (DOFF) are added INSIDE the asm, so the compiler cannot
// hoist one address per slice into long-lived registers.
// (the m0 clobber warning fires at template instantiation: ignored for the whole file)
#pragma clang diagnostic ignored "-Winline-asm"
template <int KOFF, int DOFF>
__device__ __forceinline__ void glds16(const void *sbase, unsigned voff, unsigned lds_byte) {
    unsigned tmp;
    asm volatile(
        "v_add_u32 %0, %4, %1\n\t"
        "s_add_u32 m0, %3, %5\n\t"
        "global_load_lds_dwordx4 %0, %2"
        : "=&v"(tmp)
        : "v"(voff), "s"(sbase), "s"(lds_byte), "i"(KOFF), "i"(DOFF)
        : "memory", "m0", "scc");
}

// s_waitcnt on vmcnt only (expcnt / lgkmcnt left at their no-wait maxima)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// (f & keep) | tag in one instruction (keep in a VGPR: one SGPR operand only)
__device__ __forceinline__ float tagf(float f, unsigned keep, unsigned tag) {
    float r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(keep), "s"(tag));
    return r;
}
// top-2 of {m1, m2, a, b} given m1 >= m2: m1' = max3(m1, a, b), m2' = max(m2, med3(m1, a, b))
__device__ __forceinline__ void fold3(float a, float b, float &m1, float &m2) {
    float md;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(md) : "v"(m1), "v"(a), "v"(b));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m1) : "v"(m1), "v"(a), "v"(b));
    asm("v_max_f32 %0, %1, %2" : "=v"(m2) : "v"(m2), "v"(md));
}

// xor-shuffles within 32 lanes by ds_swizzle (immediate pattern: no lane-address VGPRs)
template <int M>
__device__ __forceinline__ float swz_xor(float v) {
    static_assert(M >= 0 && M < 32, "ds_swizzle bit mode stays within 32 lanes");
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (M << 10) | 0x1F));
}
template <int M>
__device__ __forceinline__ int swz_xor(int v) {
    static_assert(M >= 0 && M < 32, "ds_swizzle bit mode stays within 32 lanes");
    return __builtin_amdgcn_ds_swizzle(v, (M << 10) | 0x1F);
}

// XCD-aware bijective remap: blocks b and b+8 share an XCD (round-robin dispatch); give
// each XCD a contiguous run of logical blocks so a pair's row tiles share one L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total / 8, r = total % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}


// nn_match_two_way's distance (pairwise_pnp.py:303): sqrt(2 - 2 clip(dot, -1, 1)) in float32
// (np.clip keeps NaN); IEEE sqrt
__device__ __forceinline__ float dist_of(float e) {
    const float c = e != e ? e : fminf(fmaxf(e, -1.f), 1.f);
    return sqrtf(__fsub_rn(2.f, __fmul_rn(2.f, c)));
}
// is (v, j) a better candidate than (bv, bj)?  dmode 0: larger dot, ties to the smaller index
// (NaN never wins: `score > max_score`); dmode 1: np.argmin -- the first NaN, else the smaller
// distance, ties to the smaller index
__device__ __forceinline__ bool better(int dmode, float v, int j, float bv, int bj) {
    if (!dmode) return v > bv || (v == bv && j < bj);
    const bool nv = v != v, nb = bv != bv;
    if (nv || nb) return nv && (!nb || j < bj);
    return v < bv || (v == bv && j < bj);
}

// The reference's sequential fp32 dot (mul then add, k = 0..255).  Latency-bound: loads go
// out U = 16 float4 per operand at a time (four round trips per dot).
__device__ __forceinline__ float exact_dot(const float *__restrict__ a, const float *__restrict__ b) {
    constexpr int U = 16;
    float s = 0.f;
#pragma unroll
    for (int bt = 0; bt < KD / (4 * U); bt++) {
        float4 xa[U], xb[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            xa[u] = *reinterpret_cast<const float4 *>(a + 4 * U * bt + 4 * u);
            xb[u] = *reinterpret_cast<const float4 *>(b + 4 * U * bt + 4 * u);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const float4 x = xa[u], y = xb[u];
            s = __fadd_rn(s, __fmul_rn(x.x, y.x));
            s = __fadd_rn(s, __fmul_rn(x.y, y.y));
            s = __fadd_rn(s, __fmul_rn(x.z, y.z));
            s = __fadd_rn(s, __fmul_rn(x.w, y.w));
        }
    }
    return s;
}

// ---- k_ap_split: frame 1 only.  32 lanes per row: lane l converts floats 4l .. 4l+3 and
//      128 + 4l .. +3 (each load instruction reads 512 contiguous bytes of two rows; each
//      8-B store writes 256 contiguous bytes); SPLIT_RPG rows per lane group per iteration,
//      all loads issued first; a 256-thread block strides over the batch (rows >= n1 are
//      never read downstream) ----
constexpr int SPLIT_RPG = 4;
constexpr int SPLIT_ROWS = 8 * SPLIT_RPG;  // rows per block iteration: 8 row groups x SPLIT_RPG
typedef float f32x4v __attribute__((ext_vector_type(4)));
// waves per EU: 8 (with SPLIT_RPG 2: 46 VGPRs) lets split waves co-reside with two k_ap_match
// waves; measured: 0.34 -> 0.44 ms beside the pose, and the overlapped pipeline (bench
// --pipeline 2/3) only +2 %: 1 kept
constexpr int SPLIT_WPE = 1;
constexpr int SPLIT_GRID = 256 * 64;  // grid-stride blocks at most
__global__ __launch_bounds__(256, SPLIT_WPE) void k_ap_split(int batch, int cap, const int *__restrict__ n1v,
                                                  const float *__restrict__ desc1, char *__restrict__ h1,
                                                  float *__restrict__ nrm1, int *__restrict__ bad) {
    const long rows = (long)batch * cap;
    const int sub = threadIdx.x & 31, rg = threadIdx.x >> 5;
    for (long R0 = (long)blockIdx.x * SPLIT_ROWS; R0 < rows; R0 += (long)gridDim.x * SPLIT_ROWS) {
        f32x4v lo[SPLIT_RPG], hi[SPLIT_RPG];
        long c[SPLIT_RPG];
#pragma unroll
        for (int r = 0; r < SPLIT_RPG; r++) {  // rows past n1 lie inside the cap stride: read, never stored
            const long R = R0 + 8 * r + rg;
            c[r] = R < rows ? R : rows - 1;
            lo[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4v *>(desc1 + c[r] * KD + 4 * sub));
            hi[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4v *>(desc1 + c[r] * KD + 128 + 4 * sub));
        }
#pragma unroll
        for (int r = 0; r < SPLIT_RPG; r++) {
            const long R = R0 + 8 * r + rg;
            const f32x4v x = lo[r], y = hi[r];
            const int out = (int)!(fabsf(x[0]) < 2.f) | (int)!(fabsf(x[1]) < 2.f) | (int)!(fabsf(x[2]) < 2.f) |
                            (int)!(fabsf(x[3]) < 2.f) | (int)!(fabsf(y[0]) < 2.f) | (int)!(fabsf(y[1]) < 2.f) |
                            (int)!(fabsf(y[2]) < 2.f) | (int)!(fabsf(y[3]) < 2.f);  // NaN: out of range
            float q = fmaf(x[0], x[0], fmaf(x[1], x[1], fmaf(x[2], x[2], x[3] * x[3])));
            q = fmaf(y[0], y[0], fmaf(y[1], y[1], fmaf(y[2], y[2], fmaf(y[3], y[3], q))));
            q += swz_xor<1>(q);
            q += swz_xor<2>(q);
            q += swz_xor<4>(q);
            q += swz_xor<8>(q);
            q += swz_xor<16>(q);  // the row's 32 lanes
            const int pair = (int)(c[r] / cap);
            if (R < rows && (int)(c[r] - (long)pair * cap) < n1v[pair]) {
                const f16x4 hx = {(_Float16)(x[0] * SCALE), (_Float16)(x[1] * SCALE), (_Float16)(x[2] * SCALE),
                                  (_Float16)(x[3] * SCALE)};  // exact 2^14 scale, RNE
                const f16x4 hy = {(_Float16)(y[0] * SCALE), (_Float16)(y[1] * SCALE), (_Float16)(y[2] * SCALE),
                                  (_Float16)(y[3] * SCALE)};
                *reinterpret_cast<f16x4 *>(h1 + R * ROW_BYTES + 8 * sub) = hx;
                *reinterpret_cast<f16x4 *>(h1 + R * ROW_BYTES + 256 + 8 * sub) = hy;
                if (out) bad[pair] = 1;
                if (sub == 0) nrm1[R] = q;
            }
        }
    }
}

__global__ __launch_bounds__(NT, 8 / NW) void k_ap_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                    const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                    const float *__restrict__ desc1, const char *__restrict__ h1,
                                                    const float *__restrict__ nrm1, const int *__restrict__ bad,
                                                    double thresh, int dmode, int *__restrict__ match_idx,
                                                    float *__restrict__ match_score) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    float *anrm = reinterpret_cast<float *>(lds + OFF_ANRM);
    float *misc = reinterpret_cast<float *>(lds + OFF_MISC);

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int pair = L / tiles_r, tr = L % tiles_r;
    const int n0 = min(max(n0v[pair], 0), cap), n1 = min(max(n1v[pair], 0), cap);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int row0 = tr * BM;
    int *oidx = match_idx + (size_t)pair * cap + row0;
    float *oscore = match_score ? match_score + (size_t)pair * cap + row0 : nullptr;  // null: indices only
    // rows in [n0, cap) report "no match"
    if (t < BM && row0 + t < cap && (row0 + t >= n0 || n1 <= 0)) {
        oidx[t] = -1;
        if (oscore) oscore[t] = 0.f;
    }
    if (row0 >= n0 || n1 <= 0) return;
    const bool flagged = bad[pair] != 0;
    const char *SB = h1 + (size_t)pair * cap * ROW_BYTES;
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;
    const int ntc = flagged ? 0 : (n1 + BN - 1) / BN;  // a flagged pair skips the screen

    // max_j |b_j|^2 over the pair's valid columns (from k_ap_split), published by the
    // prologue barrier
    {
        const float *nb2 = nrm1 + (size_t)pair * cap;
        float bmax = 0.f;
        for (int j = t; j < n1; j += NT) bmax = fmaxf(bmax, nb2[j]);
        bmax = fmaxf(bmax, swz_xor<1>(bmax));
        bmax = fmaxf(bmax, swz_xor<2>(bmax));
        bmax = fmaxf(bmax, swz_xor<4>(bmax));
        bmax = fmaxf(bmax, swz_xor<8>(bmax));
        bmax = fmaxf(bmax, swz_xor<16>(bmax));
        bmax = fmaxf(__builtin_amdgcn_readlane(__float_as_int(bmax), 0) == 0 ? 0.f : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bmax), 0)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bmax), 32)));
        if (lane == 0) misc[w] = bmax;
    }

    // ---- B DMA map: wave w fills rows w*16 .. w*16+15 of each slice, 4 rows (1 KiB) per
    //      instruction; lane l lands at row (l >> 4), chunk position l & 15 and fetches
    //      source chunk (l & 15) ^ (row & 15) of that row (256-B rows: 16 chunks) ----
    const int wu = __builtin_amdgcn_readfirstlane(w);
    constexpr int RPW = BN / NW;  // slice rows each wave DMAs: 16 (4 waves) or 8 (8 waves)
    const int dr = wu * RPW + (lane >> 4);  // (dr & 4) == 0, so (dr + 4 g) & 15 = (dr & 15) ^ 4 g
    const unsigned dcb = (unsigned)((lane & 15) ^ (dr & 15)) * 16;
    unsigned oB[RPW / 4];
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)(lds + OFF_STAGE);
    const unsigned dst_w = lds_base + (unsigned)(wu * RPW * SL_ROW);
#define AP_STAGE(SLOT, KSI)                                                                  \
    do {                                                                                     \
        glds16<(KSI) * SL_ROW, (SLOT) * SL_BYTES>(SB, oB[0], dst_w);                         \
        glds16<(KSI) * SL_ROW, (SLOT) * SL_BYTES + 4 * SL_ROW>(SB, oB[1], dst_w);            \
        if constexpr (RPW == 16) {                                                           \
            glds16<(KSI) * SL_ROW, (SLOT) * SL_BYTES + 8 * SL_ROW>(SB, oB[RPW / 4 - 2], dst_w);  \
            glds16<(KSI) * SL_ROW, (SLOT) * SL_BYTES + 12 * SL_ROW>(SB, oB[RPW / 4 - 1], dst_w); \
        }                                                                                    \
    } while (0)
#define AP_TILE_OFFSETS(TC)                                                                  \
    do {                                                                                     \
        const int nb_ = (TC) * BN + dr;                                                      \
        _Pragma("unroll") for (int g_ = 0; g_ < RPW / 4; g_++)                               \
            oB[g_] = (unsigned)min(nb_ + 4 * g_, n1 - 1) * ROW_BYTES + (dcb ^ (64u * g_));   \
    } while (0)
    AP_TILE_OFFSETS(0);
    // prologue: slices 0, 1, 2 (tile 0 both k-slices, tile 1 k-slice 0), issued before the A
    // rows are read so that both latencies overlap
    if (ntc > 0) {
        AP_STAGE(0, 0);
        AP_STAGE(1, 1);
        if (ntc > 1) {
            AP_TILE_OFFSETS(1);
            AP_STAGE(2, 0);
        }
    }
    // ---- A: this wave's 32 rows x 256 k, fp32 -> 2^14-scaled fp16 straight into registers
    //      (v_mfma_f32_32x32x16_f16 A operand: lane l holds row l & 31, k = 16 s + 8 (l >> 5)
    //      .. +7 at k16 step s).  |a|^2 and the fp16 range check come along. ----
    const int fr = lane & 31, fh = lane >> 5;
    f16x8 aF[KD / 16];
    {
        const float *arow = A + (size_t)min(row0 + w * RW + fr, n0 - 1) * KD + fh * 8;
        float4 xs[KD / 8];  // all 32 loads in flight at once, then convert
#pragma unroll
        for (int s = 0; s < KD / 16; s++) {
            xs[2 * s] = *reinterpret_cast<const float4 *>(arow + s * 16);
            xs[2 * s + 1] = *reinterpret_cast<const float4 *>(arow + s * 16 + 4);
        }
        float q = 0.f;
        int out = 0;  // any |a_k| >= 2 or NaN (comparisons with NaN are false)
#pragma unroll
        for (int s = 0; s < KD / 16; s++) {
            const float4 x = xs[2 * s], y = xs[2 * s + 1];
            out |= (int)!(fabsf(x.x) < 2.f) | (int)!(fabsf(x.y) < 2.f) | (int)!(fabsf(x.z) < 2.f) | (int)!(fabsf(x.w) < 2.f) |
                   (int)!(fabsf(y.x) < 2.f) | (int)!(fabsf(y.y) < 2.f) | (int)!(fabsf(y.z) < 2.f) | (int)!(fabsf(y.w) < 2.f);
            q = fmaf(x.x, x.x, fmaf(x.y, x.y, fmaf(x.z, x.z, fmaf(x.w, x.w, q))));
            q = fmaf(y.x, y.x, fmaf(y.y, y.y, fmaf(y.z, y.z, fmaf(y.w, y.w, q))));
            aF[s] = f16x8{(_Float16)(x.x * SCALE), (_Float16)(x.y * SCALE), (_Float16)(x.z * SCALE),
                          (_Float16)(x.w * SCALE), (_Float16)(y.x * SCALE), (_Float16)(y.y * SCALE),
                          (_Float16)(y.z * SCALE), (_Float16)(y.w * SCALE)};
        }
        q += __shfl_xor(q, 32, 64);
        out |= __shfl_xor(out, 32, 64);
        if (fh == 0) anrm[w * RW + fr] = out ? -1.f : q;
    }


    // ---- B fragment map: column block c (0, 1) of a tile, lane l reads row 32 c + (l & 31)
    //      at chunk (2 s + (l >> 5)) ^ (row & 15) for k16 step s of the slice ----
    const int rdb = fr * SL_ROW;
    const int xsw = fh ^ (fr & 15);  // chunk(2 s + fh) ^ (fr & 15) = 2 s ^ xsw

    // ---- running per-row top-2 (m1, m2) of TAGGED screen values: the low tb bits of each
    //      value are replaced by its column's tag 2 tc + half (the lane's own index gives the
    //      column within the half), so the fold needs no index registers ----
    const f32x16 zero16 = {};
    float m1[16], m2[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        m1[q] = -__builtin_inff();
        m2[q] = -__builtin_inff();
    }
    const int tb = 2 * ntc <= 256 ? 8 : 32 - __builtin_clz(2 * ntc - 1);
    const unsigned tkeep = ~((1u << tb) - 1u);
    unsigned vkeep = tkeep;
    asm volatile("" : "+v"(vkeep));

    // Ring schedule: the loop body covers tiles T and T+1 = slices g = 2T .. 2T+3 in slots
    // J = 0..3.  At slot J the block issues slice g + 3 (tile T + (J+3)/2, k-slice (J+3)%2)
    // into slot (J+3)%4 -- the slot read at g - 1, freed by that slice's barrier -- computes
    // slot J, then waits until slice g + 1 has landed (the two later groups may stay in flight).
    // Tiles alternate between two accumulator pairs (A: even tiles, B: odd tiles); a tile is
    // folded during the FIRST slot of the next tile, so the fold's VALU work interleaves with
    // that slot's MFMAs.  The sweep's last tile (the only one that can reach past n1) is
    // folded after the loop, masked.
    f32x16 accA0 = zero16, accA1 = zero16, accB0 = zero16, accB1 = zero16;
    // fold rows [Q0, Q1) of tile TC's accumulators
#define AP_FOLD_ROWS(X0, X1, TC, Q0, Q1)                                                      \
    do {                                                                                      \
        const unsigned g0_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)(TC)), g1_ = g0_ + 1u; \
        _Pragma("unroll") for (int q = (Q0); q < (Q1); q++)                                   \
            fold3(tagf(X0[q], vkeep, g0_), tagf(X1[q], vkeep, g1_), m1[q], m2[q]);            \
    } while (0)
#define AP_FOLD(X0, X1, TC) AP_FOLD_ROWS(X0, X1, TC, 0, 16)
#define AP_SLOT(J, C0, C1, F0, F1, FOLD)                                                      \
    do {                                                                                      \
        constexpr int nx = (J) + NBUF - 1;                                                    \
        const int ntile = T + nx / KS; /* tile of the slice issued now */                     \
        if (ntile < ntc) {                                                                    \
            if constexpr (nx % KS == 0) AP_TILE_OFFSETS(ntile);                               \
            AP_STAGE(nx % NBUF, nx % KS);                                                     \
        }                                                                                     \
        const char *base = lds + OFF_STAGE + (J) * SL_BYTES + rdb;                            \
        {                                                                                     \
            /* fragment reads run PF k16 steps ahead of the MFMAs (counted lgkm waits) */      \
            constexpr int PF = 4;                                                             \
            f16x8 b0_[BK / 16], b1_[BK / 16];                                                 \
            _Pragma("unroll") for (int s_ = 0; s_ < BK / 16 + PF; s_++) {                     \
                if (s_ < BK / 16) {                                                           \
                    const int ch_ = ((2 * s_) ^ xsw) * 16;                                    \
                    b0_[s_] = *reinterpret_cast<const f16x8 *>(base + ch_);                   \
                    b1_[s_] = *reinterpret_cast<const f16x8 *>(base + 32 * SL_ROW + ch_);     \
                }                                                                             \
                if (s_ >= PF) {                                                               \
                    const int m_ = s_ - PF;                                                   \
                    const f16x8 a_ = aF[((J) % KS) * (BK / 16) + m_];                         \
                    const bool z_ = (J) % KS == 0 && m_ == 0; /* a tile's first MFMA: C = 0 */ \
                    C0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_, b0_[m_], z_ ? zero16 : C0, 0, 0, 0); \
                    C1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_, b1_[m_], z_ ? zero16 : C1, 0, 0, 0); \
                }                                                                             \
            }                                                                                 \
        }                                                                                     \
        /* the previous tile's fold, half of its rows beside each k-slice's MFMAs */          \
        if (FOLD) AP_FOLD_ROWS(F0, F1, T + (J) / KS - 1, 8 * ((J) % KS), 8 * ((J) % KS) + 8);  \
        if (ntile < ntc) {                                                                    \
            wait_vm<DMA_PER_SLICE * (NBUF - 2)>();                                            \
        } else {                                                                              \
            wait_vm<0>(); /* tail of the sweep: drain */                                      \
        }                                                                                     \
        __syncthreads();                                                                      \
    } while (0)

    wait_vm<0>();
    __syncthreads();
    float bmax2 = misc[0];
#pragma unroll
    for (int k = 1; k < NW; k++) bmax2 = fmaxf(bmax2, misc[k]);
    for (int T = 0; T < ntc; T += 2) {
        AP_SLOT(0, accA0, accA1, accB0, accB1, T > 0);
        AP_SLOT(1, accA0, accA1, accB0, accB1, T > 0);
        if (T + 1 < ntc) {
            AP_SLOT(2, accB0, accB1, accA0, accA1, true);
            AP_SLOT(3, accB0, accB1, accA0, accA1, true);
        }
    }
    if (ntc > 0) {  // the last tile: columns past n1 pushed to a finite -3e38 (a tag keeps it finite)
        const int tl = ntc - 1;
        f32x16 x0 = (tl & 1) ? accB0 : accA0, x1 = (tl & 1) ? accB1 : accA1;
        const int col = tl * BN + fr;
        const float lo0 = col < n1 ? 0.f : -3.0e38f;
        const float lo1 = col + 32 < n1 ? 0.f : -3.0e38f;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            x0[q] += lo0;
            x1[q] += lo1;
        }
        AP_FOLD(x0, x1, tl);
    }
#undef AP_STAGE
#undef AP_STAGE_PIECE
#undef AP_SLOT
#undef AP_FOLD
#undef AP_FOLD_ROWS
#undef AP_TILE_OFFSETS

    // ---- per row, merge the 32 lanes' (m1, m2): transposed through LDS (the ring is free;
    //      the wave reads back only what it wrote: the epilogue has no block barrier).  Row r
    //      gets its lanes' entries [r][e] (e = the lane = the column within the tag's half);
    //      lane (fr, fh) folds entries 16 fh .. +15 of row fr and the halves combine: lanes
    //      fr and fr + 32 end with row fr's (M, E, M2) ----
    char *mt = lds + w * 32 * MT_STRIDE;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int r = (q & 3) + 8 * (q >> 2) + 4 * fh;  // 32x32 C/D row map
        float2 v;
        v.x = m1[q];
        v.y = m2[q];
        *reinterpret_cast<float2 *>(mt + r * MT_STRIDE + fr * 8) = v;
    }
    float e1[16], e2[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float4 v = *reinterpret_cast<const float4 *>(mt + fr * MT_STRIDE + (fh * 16 + 2 * i) * 8);
        e1[2 * i] = v.x;
        e2[2 * i] = v.y;
        e1[2 * i + 1] = v.z;
        e2[2 * i + 1] = v.w;
    }
    float M = -__builtin_inff(), M2 = -__builtin_inff();
    int E = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {  // equal maxima land in M2: ambiguous
        M2 = fmaxf(fmaxf(M2, e2[i]), fminf(M, e1[i]));
        E = e1[i] > M ? fh * 16 + i : E;
        M = fmaxf(M, e1[i]);
    }
    {
        const float oM = __shfl_xor(M, 32, 64), oM2 = __shfl_xor(M2, 32, 64);
        const int oE = __shfl_xor(E, 32, 64);
        M2 = fmaxf(fmaxf(M2, oM2), fminf(M, oM));
        E = (oM > M || (oM == M && oE < E)) ? oE : E;
        M = fmaxf(M, oM);
    }

    // ---- decide row w*32 + fr in its two lanes.  Window (unscaled): delta bounds screen vs
    //      exact score per column; a tag moves a value by < rho |value|, rho = 2^(tb-23), so
    //      dp = delta + 2.2 rho (|M| + 2 delta) bounds |tagged screen - exact| for every column
    //      that can compete with the maximiser.  Ms + dp <= thresh: no column can pass; a
    //      runner-up below Ms - 2 dp: the screen maximiser I is the reference's maximiser (ties
    //      included) and one exact dot decides; otherwise the columns inside the window are
    //      listed (each lane's maximum) and scored exactly; a lane with TWO values inside (its
    //      m2 too), more than NCAND lanes inside, a row outside the fp16 range or a flagged
    //      pair takes the wave-wide exact scan ("wide" rows, below). ----
    int *clist = reinterpret_cast<int *>(lds + OFF_CL);
    unsigned *lmask = reinterpret_cast<unsigned *>(lds + OFF_LM);
    const double u24 = 5.9604644775390625e-08, u23 = 2 * u24;
    const double gam_e = KD * u24 / (1.0 - KD * u24);
    const double gam_s = KD * u23 / (1.0 - KD * u23);
    const double rel = 9.765625e-04 + 2.384185791015625e-07 + 1.01 * gam_s + gam_e;  // 2^-10 + 2^-22 + ...
    const double Bn = sqrt((double)bmax2);
    const double rho = ldexp(1.0, tb - 23);
    const int rl = w * RW + fr;
    const bool live = row0 + rl < n0;
    const float an2 = anrm[rl];
    const bool full = flagged || an2 < 0.f;  // outside the fp16 screen's range: exact scan
    const float *arow = A + (size_t)(row0 + rl) * KD;
    // dmode 0: maximum dot (first strict), kept above thresh and 0 (pairwise_pnp.py:639-651);
    // dmode 1: minimum distance sqrt(2 - 2 clip(dot)) (nn_match_two_way, :302-306), no threshold
    float bs = dmode ? __builtin_inff() : -__builtin_inff();
    int bj = 0x7fffffff;
    bool wide = live && full;
    // dmode 1: distinct dots can round to one distance; columns within TIE of the maximiser's
    // exact dot are treated as competitors (a distance tie needs |d1 - d2| of a few ulp)
    const double tie = dmode ? 1e-5 : 0.0;
    if (wide && fh == 0) lmask[rl] = 0xffffffffu;
    if (live && !full) {
        const double an = sqrt(fmax((double)an2, 0.0));
        const double delta =
            (rel * an * Bn + 1.001 * 5.9604644775390625e-08 * (an + Bn) + 3.552713678800501e-15) * 1.01 + 1e-30;
        const double Ms = (double)M * 3.725290298461914e-09;  // screen / 2^28
        const double M2s = (double)M2 * 3.725290298461914e-09;
        const double dp = delta + 2.2 * rho * (fabs(Ms) + 2.0 * delta);
        // competitors: columns whose exact score can reach the maximiser's; for the distance
        // (dmode 1) also every column that can clip to 1 with it (distance-0 ties), and a
        // maximiser that can clip to -1 ties every column (all distances 2)
        const double lo = dmode ? fmin(Ms - 2.0 * dp, 1.0 - dp) - tie : Ms - 2.0 * dp;
        if (dmode && Ms - dp <= -1.0 + tie) {
            wide = true;
            if (fh == 0) lmask[rl] = 0xffffffffu;
        } else if (Ms + dp > thresh) {
            if (M2s < lo) {
                const unsigned tg = __float_as_uint(M) & ~tkeep;
                const int I = (int)(tg >> 1) * BN + (int)(tg & 1) * 32 + E;
                if (I >= n1) {  // cannot happen for a tagged in-range maximum; never read past n1
                    wide = true;
                    if (fh == 0) lmask[rl] = 0xffffffffu;
                } else if (fh == 0) {
                    // decision-only (no score output): when every exact score within the window
                    // clears both tests, the maximiser's exact dot decides nothing -- skip it
                    const bool sure = !oscore && (dmode || Ms - dp > fmax(thresh, 0.0));
                    // (Ms = M 2^-28 is exact in float, and Ms > thresh, Ms > 0: the keep test passes)
                    bs = sure ? (float)Ms : exact_dot(arow, B + (size_t)I * KD);
                    if (dmode) bs = sure ? 0.f : dist_of(bs);
                    bj = I;
                }
            } else {  // both lanes of the row take this branch
                const double lim = lo * 268435456.0;
                // padding columns (past n1: the last tile's -3e38) are never candidates; a
                // padding entry's m2 can only be padding too
                const float pad_hi = -1.0e38f;
                unsigned in1 = 0, in2 = 0;
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    in1 |= ((double)e1[i] >= lim && e1[i] > pad_hi ? 1u : 0u) << i;
                    in2 |= ((double)e2[i] >= lim && e2[i] > pad_hi ? 1u : 0u) << i;
                }
                const unsigned o1 = __shfl_xor(in1, 32, 64), o2 = __shfl_xor(in2, 32, 64);
                const unsigned inside = fh ? (o1 | (in1 << 16)) : (in1 | (o1 << 16));
                if ((in2 | o2) || __popc(inside) > NCAND) {
                    wide = true;
                    if (fh == 0) lmask[rl] = inside;
                } else {
                    int k = fh ? __popc(o1) : 0;
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        if ((in1 >> i) & 1u) {
                            const unsigned tg = __float_as_uint(e1[i]) & ~tkeep;
                            clist[rl * NCAND + k++] = (int)(tg >> 1) * BN + (int)(tg & 1) * 32 + fh * 16 + i;
                        }
                    const int nc = __popc(inside);
                    for (int c = fh; c < nc; c += 2) {  // the row's two lanes split the list
                        const int j = clist[rl * NCAND + c];
                        if ((unsigned)j >= (unsigned)n1) continue;  // an LDS-held index: checked
                        const float *ap = arow;
                        asm volatile("" : "+v"(ap));  // keep the A row's loads inside the loop
                        const float e = exact_dot(ap, B + (size_t)j * KD);
                        const float v = dmode ? dist_of(e) : e;
                        if (better(dmode, v, j, bs, bj)) {
                            bs = v;
                            bj = j;
                        }
                    }
                }
            }
        }
    }
    {
        const float ob = __shfl_xor(bs, 32, 64);
        const int oj = __shfl_xor(bj, 32, 64);
        if (better(dmode, ob, oj, bs, bj)) {
            bs = ob;
            bj = oj;
        }
    }
    if (fh == 0 && live && !wide) {
        const bool keep = bj != 0x7fffffff && (dmode || ((double)bs > thresh && bs > 0.f));
        oidx[rl] = keep ? bj : -1;
        if (oscore) oscore[rl] = keep ? bs : 0.f;
    }

    // ---- wide rows (rare): the wave scores every column of every listed lane exactly, one
    //      column per lane at a time (lane l: columns f + 32 (l + 64 i) of inside lane f) ----
    for (unsigned dm = (unsigned)__ballot(fh == 0 && wide); dm; dm &= dm - 1) {
        const int r = w * RW + __builtin_ctz(dm);
        const float *a = A + (size_t)(row0 + r) * KD;
        float ws = dmode ? __builtin_inff() : -__builtin_inff();
        int wj = 0x7fffffff;
        for (unsigned Lm = lmask[r]; Lm; Lm &= Lm - 1) {
            const int f = __builtin_ctz(Lm);
            for (int j = f + 32 * lane; j < n1; j += 32 * 64) {
                const float *ap = a;
                asm volatile("" : "+v"(ap));  // keep the A row's loads inside the loop
                const float e = exact_dot(ap, B + (size_t)j * KD);
                const float v = dmode ? dist_of(e) : e;
                if (better(dmode, v, j, ws, wj)) {
                    ws = v;
                    wj = j;
                }
            }
        }
#define AP_WRED(O)                                                                           \
        do {                                                                                 \
            const float ob = O == 32 ? __shfl_xor(ws, 32, 64) : swz_xor<O & 31>(ws);         \
            const int oj = O == 32 ? __shfl_xor(wj, 32, 64) : swz_xor<O & 31>(wj);           \
            if (better(dmode, ob, oj, ws, wj)) {                                             \
                ws = ob;                                                                     \
                wj = oj;                                                                     \
            }                                                                                \
        } while (0)
        AP_WRED(1);
        AP_WRED(2);
        AP_WRED(4);
        AP_WRED(8);
        AP_WRED(16);
        AP_WRED(32);
#undef AP_WRED
        if (lane == 0) {
            const bool keep = wj != 0x7fffffff && (dmode || ((double)ws > thresh && ws > 0.f));
            oidx[r] = keep ? wj : -1;
            if (oscore) oscore[r] = keep ? ws : 0.f;
        }
    }
}

}  // namespace

namespace mv {

// scratch: h1 (batch * cap * 512 B) | nrm1 (batch * cap f32) | bad (batch i32); the int8
// screen's layout (k_allpairs_q8.hip) shares the buffer: the size covers both
size_t allpairs_f32_scratch_bytes(int batch, int cap) {
    const size_t rows = (size_t)batch * cap;
    const size_t f16 = rows * ROW_BYTES + align_up(rows * 4, 256) + align_up((size_t)batch * 4, 256);
    return std::max(f16, allpairs_q8_scratch_bytes(batch, cap));
}
// one staged image under `screen`: fp16 (516 B per row) or int8 (268 B per row)
size_t ap_image_bytes(int screen, int batch, int cap) {
    if (screen != MV_SCREEN_F16) return allpairs_q8_scratch_bytes(batch, cap);
    const size_t rows = (size_t)batch * cap;
    return rows * ROW_BYTES + align_up(rows * 4, 256) + align_up((size_t)batch * 4, 256);
}

namespace {
struct ApScratch {
    char *h1;
    float *nrm1;
    int *bad;
};
ApScratch ap_scratch_map(void *scratch, int batch, int cap) {
    const size_t rows = (size_t)batch * cap;
    ApScratch m;
    m.h1 = (char *)scratch;
    m.nrm1 = (float *)(m.h1 + rows * ROW_BYTES);
    m.bad = (int *)((char *)m.nrm1 + align_up(rows * 4, 256));
    return m;
}
}  // namespace

// frame 1 -> fp16 image + |b|^2 + per-pair range flag (k_ap_split)
int launch_allpairs_f32_prepare(hipStream_t s, void *scratch, int batch, int cap, const int *n1,
                                const float *desc1) {
    MV_REQUIRE(batch > 0 && cap > 0 && n1 && desc1 && scratch);
    MV_REQUIRE(((uintptr_t)desc1 & 15) == 0);
    MV_REQUIRE(cap <= (1 << 22));  // per-lane DMA source offsets are 32-bit byte offsets into a pair
    const size_t rows = (size_t)batch * cap;
    const ApScratch m = ap_scratch_map(scratch, batch, cap);
    const long split_blocks = std::min<long>((long)((rows + SPLIT_ROWS - 1) / SPLIT_ROWS), (long)SPLIT_GRID);
    MV_HIP_TRY(hipMemsetAsync(m.bad, 0, (size_t)batch * 4, s));
    MV_PROF_BEGIN(s, "k_ap_split");
    hipLaunchKernelGGL(k_ap_split, dim3((unsigned)split_blocks), dim3(256), 0, s, batch, cap, n1, desc1, m.h1, m.nrm1,
                       m.bad);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

// the sweep + exact re-score (k_ap_match) over a prepared frame 1
int launch_allpairs_f32_match(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                              const float *desc0, const float *desc1, double thresh, int *match_idx,
                              float *match_score, int dmode) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx && scratch);  // match_score optional
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    const int tiles_r = (cap + BM - 1) / BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    const ApScratch m = ap_scratch_map(scratch, batch, cap);
    MV_PROF_BEGIN(s, "k_ap_match");
    hipLaunchKernelGGL(k_ap_match, dim3((unsigned)blocks), dim3(NT), 0, s, tiles_r, cap, n0, n1, desc0, desc1, m.h1,
                       m.nrm1, m.bad, dmode ? -1e300 : thresh, dmode, match_idx, match_score);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

namespace {
void *ap_scratch(mv_context *ctx, size_t bytes) {
    if (bytes <= ctx->ap_scratch_bytes) return ctx->ap_scratch;
    if (ctx->ap_scratch) {
        (void)mv::quiesce(ctx);  // growing: nothing of this context may still use the old buffer
        (void)hipFree(ctx->ap_scratch);
        ctx->ap_scratch = nullptr;
        ctx->ap_scratch_bytes = 0;
        ctx->prep_desc1 = nullptr;  // a prepared frame 1 lived in the freed buffer
    }
    const size_t b = mv::align_up(bytes, 1 << 20);
    if (hipMalloc(&ctx->ap_scratch, b) != hipSuccess) {
        mv::set_error(MV_ERR_OUT_OF_MEMORY, "all-pairs scratch allocation of %zu bytes failed", b);
        ctx->ap_scratch = nullptr;
        return nullptr;
    }
    ctx->ap_scratch_bytes = b;
    return ctx->ap_scratch;
}
}  // namespace

namespace {
// staging of frame 1 for the screens that match against an image (fp16, staged int8; the
// default int8 screen stages only for sequence mode, which reuses the images)
int ap_prepare(int screen, hipStream_t s, void *scr, int batch, int cap, const int *n1, const float *desc1) {
    return screen == MV_SCREEN_F16 ? mv::launch_allpairs_f32_prepare(s, scr, batch, cap, n1, desc1)
                                   : mv::launch_allpairs_q8_prepare(s, scr, batch, cap, n1, desc1);
}
// the match; MV_SCREEN_I8 reads both fp32 frames directly (no image, scr unused)
int ap_match(mv_context *ctx, int screen, hipStream_t s, void *scr, int batch, int cap, const int *n0, const int *n1,
             const float *desc0, const float *desc1, double thresh, int *match_idx, float *match_score,
             int dmode = 0) {
    if (screen == MV_SCREEN_I8) {
        if (mv::allpairs_q8t_applies(cap, dmode)) {
            void *fl = mv::scratch(ctx, mv::allpairs_q8t_scratch_bytes(batch));
            if (!fl) return MV_ERR_OUT_OF_MEMORY;
            return mv::launch_allpairs_q8t_match(s, fl, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                                 match_score);
        }
        return mv::launch_allpairs_q8d_match(s, batch, cap, n0, n1, desc0, desc1, thresh, match_idx, match_score,
                                             dmode);
    }
    return screen == MV_SCREEN_F16
               ? mv::launch_allpairs_f32_match(s, scr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                               match_score, dmode)
               : mv::launch_allpairs_q8_match(s, scr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                              match_score, dmode);
}
}  // namespace

extern "C" int mv_match_allpairs_f32_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                         const float *desc0, const float *desc1, double thresh, int *match_idx,
                                         float *match_score) {
    MV_REQUIRE(ctx != nullptr && batch > 0 && cap > 0);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->ap_screen == MV_SCREEN_I8)  // one pass, no image
        return ap_match(ctx, ctx->ap_screen, ctx->stream, nullptr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                        match_score);
    void *scr = ap_scratch(ctx, mv::ap_image_bytes(ctx->ap_screen, batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    ctx->prep_desc1 = nullptr;  // the prepared image is overwritten
    if (ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));  // a staging in flight
    const int st = ap_prepare(ctx->ap_screen, ctx->stream, scr, batch, cap, n1, desc1);
    if (st != MV_OK) return st;
    return ap_match(ctx, ctx->ap_screen, ctx->stream, scr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                    match_score);
}

extern "C" int mv_match_allpairs_f32_prepare_dev(mv_context *ctx, int batch, int cap, const int *n1,
                                                 const float *desc1) {
    MV_REQUIRE(ctx != nullptr && batch > 0 && cap > 0 && n1 && desc1);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->ap_screen == MV_SCREEN_I8) {  // the one-pass match reads frame 1 itself: record only
        ctx->prep_screen = ctx->ap_screen;
        ctx->prep_staged = false;  // sequence mode stages these frames on first use
        ctx->prep_batch = batch;
        ctx->prep_cap = cap;
        ctx->prep_n1 = n1;
        ctx->prep_desc1 = desc1;
        return mv::set_status(MV_OK);
    }
    void *scr = ap_scratch(ctx, mv::ap_image_bytes(ctx->ap_screen, batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    if (!ctx->aux_stream) {
        MV_HIP_TRY(hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking));
        MV_HIP_TRY(hipEventCreateWithFlags(&ctx->ev_in, hipEventDisableTiming));
        MV_HIP_TRY(hipEventCreateWithFlags(&ctx->ev_prep, hipEventDisableTiming));
    }
    // inputs (and the previous run's use of the scratch) as of this call on the context stream
    MV_HIP_TRY(hipEventRecord(ctx->ev_in, ctx->stream));
    MV_HIP_TRY(hipStreamWaitEvent(ctx->aux_stream, ctx->ev_in, 0));
    const int st = ap_prepare(ctx->ap_screen, ctx->aux_stream, scr, batch, cap, n1, desc1);
    if (st != MV_OK) return st;
    MV_HIP_TRY(hipEventRecord(ctx->ev_prep, ctx->aux_stream));
    ctx->prep_screen = ctx->ap_screen;
    ctx->prep_staged = true;
    ctx->prep_batch = batch;
    ctx->prep_cap = cap;
    ctx->prep_n1 = n1;
    ctx->prep_desc1 = desc1;
    return MV_OK;
}

extern "C" int mv_match_allpairs_f32_run_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                             const float *desc0, const float *desc1, double thresh, int *match_idx,
                                             float *match_score) {
    MV_REQUIRE(ctx != nullptr);
    if (!ctx->prep_desc1 || ctx->prep_batch != batch || ctx->prep_cap != cap || ctx->prep_n1 != n1 ||
        ctx->prep_desc1 != desc1 || ctx->prep_screen != ctx->ap_screen) {
        mv::set_error(MV_ERR_INVALID_ARG, "mv_match_allpairs_f32_run_dev: no matching prepare for this batch");
        return MV_ERR_INVALID_ARG;
    }
    MV_HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->prep_staged && ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));
    return ap_match(ctx, ctx->ap_screen, ctx->stream, ctx->ap_scratch, batch, cap, n0, n1, desc0, desc1, thresh,
                    match_idx, match_score);
}

namespace {
// the context's second image, grown to `need` bytes (run_prepare's staging target)
int ap_scratch2(mv_context *ctx, size_t need) {
    if (ctx->ap_scratch2_bytes >= need) return MV_OK;
    if (ctx->ap_scratch2) {
        (void)mv::quiesce(ctx);  // growing: nothing of this context may still use the old buffer
        (void)hipFree(ctx->ap_scratch2);
        ctx->ap_scratch2 = nullptr;
        ctx->ap_scratch2_bytes = 0;
    }
    const size_t b = mv::align_up(need, 1 << 20);
    if (hipMalloc(&ctx->ap_scratch2, b) != hipSuccess) {
        mv::set_error(MV_ERR_OUT_OF_MEMORY, "all-pairs scratch allocation of %zu bytes failed", b);
        return MV_ERR_OUT_OF_MEMORY;
    }
    ctx->ap_scratch2_bytes = b;
    return MV_OK;
}
void ap_swap_prepared(mv_context *ctx, int batch, int cap, const int *n1, const float *desc1) {
    void *t = ctx->ap_scratch;
    size_t tb = ctx->ap_scratch_bytes;
    ctx->ap_scratch = ctx->ap_scratch2;
    ctx->ap_scratch_bytes = ctx->ap_scratch2_bytes;
    ctx->ap_scratch2 = t;
    ctx->ap_scratch2_bytes = tb;
    ctx->prep_batch = batch;
    ctx->prep_cap = cap;
    ctx->prep_n1 = n1;
    ctx->prep_desc1 = desc1;
    ctx->prep_staged = true;
}
}  // namespace

extern "C" int mv_match_allpairs_f32_run_prepare_dev(mv_context *ctx, int batch, int cap, const int *n0,
                                                     const int *n1, const float *desc0, const float *desc1,
                                                     double thresh, int *match_idx, float *match_score,
                                                     int next_batch, int next_cap, const int *next_n1,
                                                     const float *next_desc1) {
    MV_REQUIRE(ctx != nullptr && next_batch > 0 && next_cap > 0 && next_n1 && next_desc1);
    if (!ctx->prep_desc1 || ctx->prep_batch != batch || ctx->prep_cap != cap || ctx->prep_n1 != n1 ||
        ctx->prep_desc1 != desc1 || ctx->prep_screen != ctx->ap_screen) {
        mv::set_error(MV_ERR_INVALID_ARG, "mv_match_allpairs_f32_run_prepare_dev: no matching prepare for this batch");
        return MV_ERR_INVALID_ARG;
    }
    MV_HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->ap_screen == MV_SCREEN_I8) {  // one pass: nothing to stage for the next batch
        const int st = ap_match(ctx, ctx->ap_screen, ctx->stream, nullptr, batch, cap, n0, n1, desc0, desc1, thresh,
                                match_idx, match_score);
        if (st != MV_OK) return st;
        ctx->prep_batch = next_batch;
        ctx->prep_cap = next_cap;
        ctx->prep_n1 = next_n1;
        ctx->prep_desc1 = next_desc1;
        ctx->prep_staged = false;  // recorded, not staged (sequence mode needs a prepare)
        return mv::set_status(MV_OK);
    }
    const int sc = ap_scratch2(ctx, mv::ap_image_bytes(ctx->ap_screen, next_batch, next_cap));
    if (sc != MV_OK) return sc;
    if (ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));
    int st;
    if (ctx->ap_screen == MV_SCREEN_I8_STAGED) {
        st = mv::launch_allpairs_q8_match_prepare(ctx->stream, ctx->ap_scratch, batch, cap, n0, n1, desc0, desc1,
                                                  thresh, match_idx, match_score, 0, ctx->ap_scratch2, next_batch,
                                                  next_cap, next_n1, next_desc1);
    } else {  // the fp16 screen: the two kernels in stream order
        st = ap_match(ctx, ctx->ap_screen, ctx->stream, ctx->ap_scratch, batch, cap, n0, n1, desc0, desc1, thresh,
                      match_idx, match_score);
        if (st == MV_OK)
            st = ap_prepare(ctx->ap_screen, ctx->stream, ctx->ap_scratch2, next_batch, next_cap, next_n1, next_desc1);
    }
    if (st != MV_OK) return st;
    ap_swap_prepared(ctx, next_batch, next_cap, next_n1, next_desc1);  // the next batch is now the prepared one
    return mv::set_status(MV_OK);
}

namespace {
// nn_match_two_way's keep (pairwise_pnp.py:307-313): dist < nn_thresh (float32 compare) and
// the reverse argmin of the match is the row itself
__global__ __launch_bounds__(256) void k_two_way_keep(long total, int cap, const int *__restrict__ n0v,
                                                      const int *__restrict__ n1v, const int *__restrict__ ridx,
                                                      float nn_thresh, int *__restrict__ fidx,
                                                      float *__restrict__ fdist, int keep_dist) {
    const long q = (long)blockIdx.x * 256 + threadIdx.x;
    if (q >= total) return;
    const long b = q / cap;
    const int i = (int)(q % cap);
    const int n0 = min(max(n0v[b], 0), cap), n1 = min(max(n1v[b], 0), cap);
    const int j = fidx[q];
    const bool keep = i < n0 && j >= 0 && j < n1 && fdist[q] < nn_thresh && ridx[b * cap + j] == i;
    fidx[q] = keep ? j : -1;
    if (keep_dist && !keep) fdist[q] = 0.f;
}
}  // namespace

extern "C" int mv_match_two_way_f32_dev(mv_context *ctx, int batch, int cap, const int *n0, const int *n1,
                                        const float *desc0, const float *desc1, double nn_thresh, int *match_idx,
                                        float *match_dist) {
    MV_REQUIRE(ctx != nullptr && batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx);
    if (!(nn_thresh >= 0.0)) {
        mv::set_error(MV_ERR_INVALID_ARG, "nn_match_two_way: nn_thresh should be non-negative");
        return MV_ERR_INVALID_ARG;
    }
    MV_HIP_TRY(hipSetDevice(ctx->device));
    const int sc = ctx->ap_screen;
    void *scr = nullptr;
    if (sc != MV_SCREEN_I8) {  // the image screens stage each direction
        scr = ap_scratch(ctx, mv::ap_image_bytes(ctx->ap_screen, batch, cap));
        if (!scr) return MV_ERR_OUT_OF_MEMORY;
        ctx->prep_desc1 = nullptr;  // the prepared image is overwritten
        if (ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));  // a staging in flight
    }
    const size_t nb = mv::align_up((size_t)batch * cap * 4, 256);
    char *tmp = (char *)mv::scratch(ctx, 2 * nb);
    if (!tmp) return MV_ERR_OUT_OF_MEMORY;
    int *ridx = (int *)tmp;
    float *fdist = match_dist ? match_dist : (float *)(tmp + nb);
    hipStream_t s = ctx->stream;
    // forward: rows of frame 0 against frame 1 (argmin distance + its exact distance)
    int st = sc == MV_SCREEN_I8 ? MV_OK : ap_prepare(sc, s, scr, batch, cap, n1, desc1);
    if (st == MV_OK) st = ap_match(ctx, sc, s, scr, batch, cap, n0, n1, desc0, desc1, 0.0, match_idx, fdist, 1);
    // reverse: rows of frame 1 against frame 0 (indices only)
    if (st == MV_OK && sc != MV_SCREEN_I8) st = ap_prepare(sc, s, scr, batch, cap, n0, desc0);
    if (st == MV_OK) st = ap_match(ctx, sc, s, scr, batch, cap, n1, n0, desc1, desc0, 0.0, ridx, nullptr, 1);
    if (st != MV_OK) return st;
    const long total = (long)batch * cap;
    hipLaunchKernelGGL(k_two_way_keep, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, total, cap, n0, n1,
                       ridx, (float)nn_thresh, match_idx, fdist, match_dist ? 1 : 0);
    MV_LAUNCH_CHECK();
    return mv::set_status(MV_OK);
}


namespace {
// Sequence mode on the default screen (cap <= 1024): k_q8t_match over the F - 1 pairs (frame b,
// frame b + 1) addressed in place -- desc0 = desc, desc1 = desc + one frame, n0 = n, n1 = n + 1 -- a
// whole pair per workgroup, each frame read once as frame 1 and once as frame 0 (the staged int8
// images of k_q8_match<AI8> read 24 % fewer bytes but run the older, slower sweep: 4.0 ms per 8192
// pairs against the one-pass kernel's 3.5)
bool seq_one_pass(const mv_context *ctx, int cap) {
    return ctx->ap_screen == MV_SCREEN_I8 && mv::allpairs_q8t_applies(cap, 0);
}
int seq_one_pass_run(mv_context *ctx, int frames, int cap, const int *n, const float *desc, double thresh,
                     int *match_idx, float *match_score) {
    void *fl = mv::scratch(ctx, mv::allpairs_q8t_scratch_bytes(frames - 1));
    if (!fl) return MV_ERR_OUT_OF_MEMORY;
    return mv::launch_allpairs_q8t_match(ctx->stream, fl, frames - 1, cap, n, n + 1, desc, desc + (size_t)cap * 256,
                                         thresh, match_idx, match_score);
}
}  // namespace

extern "C" int mv_match_sequence_f32_dev(mv_context *ctx, int frames, int cap, const int *n, const float *desc,
                                         double thresh, int *match_idx, float *match_score) {
    MV_REQUIRE(ctx != nullptr && frames >= 2 && cap > 0 && n && desc && match_idx);
    if (ctx->ap_screen == MV_SCREEN_F16) {
        mv::set_error(MV_ERR_INVALID_ARG, "mv_match_sequence_f32_dev: the int8 screens only");
        return MV_ERR_INVALID_ARG;
    }
    MV_HIP_TRY(hipSetDevice(ctx->device));
    if (seq_one_pass(ctx, cap)) {
        const int st = seq_one_pass_run(ctx, frames, cap, n, desc, thresh, match_idx, match_score);
        return st != MV_OK ? st : mv::set_status(MV_OK);
    }
    void *scr = ap_scratch(ctx, mv::ap_image_bytes(ctx->ap_screen, frames, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    ctx->prep_desc1 = nullptr;  // the prepared image is overwritten
    if (ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));  // a staging in flight
    const int st = mv::launch_allpairs_q8_sequence(ctx->stream, scr, frames, cap, n, desc, thresh, match_idx,
                                                   match_score);
    return st != MV_OK ? st : mv::set_status(MV_OK);
}

extern "C" int mv_match_sequence_f32_run_prepare_dev(mv_context *ctx, int frames, int cap, const int *n,
                                                     const float *desc, double thresh, int *match_idx,
                                                     float *match_score, int next_frames, int next_cap,
                                                     const int *next_n, const float *next_desc) {
    MV_REQUIRE(ctx != nullptr && frames >= 2 && next_frames >= 2 && next_cap > 0 && next_n && next_desc);
    if (ctx->ap_screen == MV_SCREEN_F16 || !ctx->prep_desc1 || ctx->prep_batch != frames ||
        ctx->prep_cap != cap || ctx->prep_n1 != n || ctx->prep_desc1 != desc || ctx->prep_screen == MV_SCREEN_F16) {
        mv::set_error(MV_ERR_INVALID_ARG,
                      "mv_match_sequence_f32_run_prepare_dev: no matching prepare for these frames (int8 screen)");
        return MV_ERR_INVALID_ARG;
    }
    MV_HIP_TRY(hipSetDevice(ctx->device));
    if (seq_one_pass(ctx, cap)) {  // nothing staged: match this chunk in place, record the next one
        const int st = seq_one_pass_run(ctx, frames, cap, n, desc, thresh, match_idx, match_score);
        if (st != MV_OK) return st;
        ctx->prep_batch = next_frames;
        ctx->prep_cap = next_cap;
        ctx->prep_n1 = next_n;
        ctx->prep_desc1 = next_desc;
        ctx->prep_staged = false;
        return mv::set_status(MV_OK);
    }
    if (!ctx->prep_staged) {  // recorded by the one-pass screen's prepare: stage the images now
        void *scr = ap_scratch(ctx, mv::ap_image_bytes(ctx->ap_screen, frames, cap));
        if (!scr) return MV_ERR_OUT_OF_MEMORY;
        if (ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));
        const int ps = ap_prepare(ctx->ap_screen, ctx->stream, scr, frames, cap, n, desc);
        if (ps != MV_OK) return ps;
        ctx->prep_staged = true;
    }
    const int sc = ap_scratch2(ctx, mv::ap_image_bytes(ctx->ap_screen, next_frames, next_cap));
    if (sc != MV_OK) return sc;
    if (ctx->aux_stream) MV_HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_prep, 0));
    const int st = mv::launch_allpairs_q8_sequence(ctx->stream, ctx->ap_scratch, frames, cap, n, desc, thresh,
                                                   match_idx, match_score, true, ctx->ap_scratch2, next_frames,
                                                   next_cap, next_n, next_desc);
    if (st != MV_OK) return st;
    ap_swap_prepared(ctx, next_frames, next_cap, next_n, next_desc);
    return mv::set_status(MV_OK);
}
