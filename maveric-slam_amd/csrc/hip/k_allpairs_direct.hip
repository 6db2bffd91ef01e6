// k_allpairs_direct.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659,
// exact score in the gemmini_functions_cpu.h:45-49 order) in ONE pass over the fp32 inputs:
// the default screen (MV_SCREEN_I8).  SURVEY §8(d)'s algorithmic bytes per pair -- both frames
// read once (2 x n x 1 KiB), the match written once -- are the only HBM traffic: frame 1 is
// quantised to int8 INSIDE the workgroup, never staged through memory.
//
//   k_q8d_match  one 512-thread workgroup (8 waves x 64 rows, one per CU, 2 waves per SIMD)
//                owns 512 query rows of one pair; a pair's row blocks sit on one XCD, so
//                frame 1 comes from HBM once and from that XCD's L2 for the other block.
//     A phase    each wave reads its 64 frame-0 rows as fp32 once and quantises them into 64
//                VGPRs of int8 MFMA operands (per-row scale s_a; q8_common.hpp).
//     B stream   frame 1 streams as fp32 half-tiles (32 rows = 32 KiB) through a 3-slot LDS
//                staging ring by LDS-DMA (global_load_lds_dwordx4, one 1-KiB row per wave
//                instruction, issued one tile ahead).  Inside the sweep of tile t every thread
//                quantises 16 values of tile t + 1 from staging (16 lanes per frame-1 row; the
//                row's max |b| and |b|^2 by DPP reductions) into the int8 tile ring (2 slots of
//                16 KiB + 64 per-column words), one stage per MFMA step.
//     sweep      v_mfma_i32_32x32x32_i8 over 64-column tiles.  Integer keys (the fast path):
//                column j is quantised with the power-of-two multiple q_j = 127 * 2^e_j,
//                e_j in {0, 1, 2} (|b_jk| <= 1 required, as for unit-norm descriptors), so the
//                exact integer dot D_ij scaled by 2^(2 - e_j) is one exact integer in the units
//                of 1/508 for every column: the key (D_ij << (tb + 2 - e_j)) | tag -- ONE
//                v_lshl_or_b32 per value, the column's shift riding in a VGPR -- is folded into a
//                lane-local top-2 per row with v_max3_i32 / v_med3_i32 / v_max_i32.  A pair with
//                a column outside that range (or a non-finite value) is swept again on the
//                float path: per-column scale s_j = RN(m_j RN(1/127)), screen RN(D s_j) by one
//                FMA, tagged in the low mantissa bits (as k_q8_match).
//     epilogue   q8_common.hpp: the window decisions, exact re-scores where it does not decide.
// The window's B terms come from the sweep itself: every workgroup quantises the whole frame 1
// of its pair, so Bn = max_j |b_j| (from the fp32 |b_j|^2) and Eb = 8 max_j s_j (+ 2^-21 Bn on
// the float path; the integer path's scaling is exact: |b_jk - q_jk / q_j| <= 1 / (2 q_j)) and
// the pair's range flags are known to it after the sweep, before any decision.
// LDS (141.2 KiB): staging 3 x 32 KiB | int8 ring 2 x 17.25 KiB (+ 2.5 KiB: the exchange build's
// 4-slot ring) | (|a|^2, s_a) per row | per-wave statistics | each column's key shift (4 KiB);
// the A images (8 x 8 KiB) use staging slot 2 + the ring before the sweep, the epilogue (102 KiB)
// the staging + ring after it.
// Bound: HBM -- 2 KiB read + 4 B written per query row (2,105,344 B per 1024^2
// pair); int8 MFMA 2 n0 n1 256 ops per pair beside it.
#include "q8_common.hpp"

namespace {

using namespace q8;

constexpr int D_NW = 8, D_NT = 64 * D_NW, D_BM = 32 * RG * D_NW;  // 512 rows per workgroup
constexpr int D_HROWS = 32, D_HALF = D_HROWS * KD * 4;             // one staging slot: 32 fp32 rows
#ifndef D_PAD
#define D_PAD 1  // int8 ring rows padded to 272 B (conflict-free, immediate-offset fragment reads)
#endif
// the int8 tile ring: 64 rows (columns of frame 1) of 256 codes, row stride D_RS; D_PAD: 272 B
// (17 chunks: the 16-lane phases of a ds_read_b128 hit distinct banks, and every B-fragment address
// is a per-lane base + a compile-time offset); else 256 B with the 16-B chunks XOR-swizzled by row
constexpr int D_RS = D_PAD ? KD + 16 : KD;
constexpr int D_TILE = BN * D_RS, D_SLOT = D_TILE + BN * 4;        // + the tile's 64 per-column words
constexpr int D_OFF_RING = 3 * D_HALF;                              // 2 int8 tile slots
// [BM] float2 (|a|^2, s_a), past the int8 ring of either sweep (the pair exchange's: 4 slots of
// 64 padded rows after 2 staging slots)
constexpr int D_OFF_ROW = D_OFF_RING + 2 * D_SLOT > 2 * D_HALF + 4 * D_SLOT ? D_OFF_RING + 2 * D_SLOT
                                                                           : 2 * D_HALF + 4 * D_SLOT;
constexpr int D_OFF_MISC = D_OFF_ROW + D_BM * 8;                    // [NW][4] per-wave statistics
constexpr int D_OFF_X = D_OFF_MISC + D_NW * 16;                     // pair exchange: flags, SOLO, statistics
#ifndef D_COLWIN
#define D_COLWIN 1  // the epilogue's window per maximiser column (0: the pair's widest, for A/B)
#endif
constexpr int D_OFF_COL = D_OFF_X + 64;  // integer path: each frame-1 column's key shift (1 B)
constexpr int D_NCOL = 64 * BN;           // the integer path's column limit (2 ntc <= 128)
#ifndef D_EXACT_EA
#define D_EXACT_EA 0  // the A phase measures each row's quantisation residual (rowe) for the window
#endif
constexpr int D_OFF_ROWE = D_OFF_COL + D_NCOL;  // [BM] float |rho|^2 per row (D_EXACT_EA)
constexpr int D_LDS = D_OFF_ROWE + (D_EXACT_EA ? D_BM * 4 : 0);
constexpr int D_OFF_AIMG = 2 * D_HALF;  // A images: staging slot 2 + the ring (before the sweep)
static_assert(D_OFF_AIMG + D_NW * 32 * KD <= D_OFF_ROW, "A images fit staging slot 2 + the ring");
static_assert(epi_bytes<D_NW>() <= D_OFF_ROW, "the epilogue fits staging + ring");
static_assert(D_LDS <= 160 * 1024, "one workgroup per CU");
constexpr int D_PF = 1;       // k32 steps of B fragments read ahead of the MFMAs
constexpr int QS_LOAD = 1;    // the k32 step whose slot issues the quantisation's staging reads
#ifndef D_QB
#define D_QB 4  // A phase: frame-0 row quads in flight per wave (4 x 16-B loads per lane each)
#endif
constexpr float IK_MMAX = 1.003f;  // integer path: max |b_jk| allowed (RNE(x 127) stays <= 127)
#ifndef D_CC
// 1: integer path, |b_j| bounded from the codes (v_dot4) and NaN caught by v_maximum3 instead of
// summing the fp32 squares (12 VALU per tile and wave fewer) -- fails the out-of-range parity test
// (tests/test_gpu_allpairs.py::test_allpairs_f32_out_of_screen_range): experimental, off
#define D_CC 0
#endif

#ifdef MV_TRACE  // phase stamps (s_memtime) per (block, wave): tools/trace_direct.py
constexpr int D_TRACE_BLOCKS = 16384;
__device__ unsigned long long g_d_trace[D_TRACE_BLOCKS * D_NW * 10];
// pair-exchange event counts (per wave): flag waits entered, polls, foreign-XCD flags, spin
// timeouts, waves gone SOLO, final statistics taken / recomputed, imports
__device__ unsigned g_x_cnt[8];
#ifdef X_COUNT  // (global atomics: they slow the kernel down several-fold -- counts only)
#define X_CNT(K) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_x_cnt[K], 1u); } while (0)
#else
#define X_CNT(K) do { } while (0)
#endif
#define D_STAMP(K) do { __builtin_amdgcn_sched_barrier(0); ts_[K] = __builtin_amdgcn_s_memtime(); if ((K) < 2) ts_[4 + (K)] = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define D_SYNC() __syncthreads()
#else
#define D_STAMP(K) do { } while (0)
#define D_SYNC() __syncthreads()
#endif
#ifndef MV_TRACE
#define X_CNT(K) do { } while (0)
#endif

// max |b| and sum |b|^2 over a row's 16 lanes (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror), the two reductions interleaved so that every DPP read is two
// instructions behind the write it reads (no NaN canonicalisation in the max: NaN is caught by
// |b|^2); every lane of the 16 ends with the same values
__device__ __forceinline__ void row16_max_sum(float &m, float &q2) {
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_add_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_add_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_add_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(m), "+v"(q2));
}
// two values of one row folded into its lane-local top-2 on integer keys (held in float
// registers' bits): the keys (d << sh) | tag by v_lshl_or_b32 (shift per lane in a VGPR, tag in
// an SGPR), m1' = max3(m1, ka, kb), m2' = max(m2, med3(m1, ka, kb)) -- one asm block, so that
// no hazard padding is placed between its dependent instructions
__device__ __forceinline__ void fold_keys(int a, int b, int sha, int shb, unsigned ta, unsigned tb, float &m1f,
                                          float &m2f) {
    int ka, kb, md, m1 = __float_as_int(m1f), m2 = __float_as_int(m2f);
    asm("v_lshl_or_b32 %0, %5, %7, %9\n\t"
        "v_lshl_or_b32 %1, %6, %8, %10\n\t"
        "v_med3_i32 %2, %3, %0, %1\n\t"
        "v_max3_i32 %3, %3, %0, %1\n\t"
        "v_max_i32 %4, %4, %2"
        : "=&v"(ka), "=&v"(kb), "=&v"(md), "+v"(m1), "+v"(m2)
        : "v"(a), "v"(b), "v"(sha), "v"(shb), "s"(ta), "s"(tb));
    m1f = __int_as_float(m1);
    m2f = __int_as_float(m2);
}
// sum of an int over a row's 16 lanes (every lane of the 16 ends with it)
__device__ __forceinline__ void row16_sum_i(int &c) {
    asm("s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(c));
}
// max over a row's 16 lanes (NaN-propagating when the inputs came from v_maximum3)
__device__ __forceinline__ void row16_max(float &m) {
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(m));
}
// max(m, |a|, |b|) propagating NaN (IEEE maximum): the codes' norm bound needs no fp32 sum to see it
__device__ __forceinline__ float absmaximum3(float m, float a, float b) {
    float r;
    asm("v_maximum3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Half h of frame 1 (rows 32 h .. +31, clamped to n1 - 1) -> staging slot at LDS byte `slot`:
// wave w copies rows 4 w .. +3, one 1-KiB row per instruction.  Within a row, LDS position p
// (16-B unit) holds source chunk 4 (p & 15) + (p >> 4), so that the reader below -- lane sub
// taking positions sub + 16 i, i.e. the 16 consecutive floats 16 sub .. +15 -- is conflict-free.
// Timing experiments (wrong results; tools/gpu_ab.sh with --check 0): D_EXP_NODMA skips the
// sweep's LDS-DMA issue, D_EXP_NOQUANT the next tile's quantisation, D_EXP_NOFOLD the top-2 fold.
#ifndef D_EXP_NODMA
#define D_EXP_NODMA 0
#endif
#ifndef D_EXP_NOQUANT
#define D_EXP_NOQUANT 0
#endif
#ifndef D_EXP_NOFOLD
#define D_EXP_NOFOLD 0
#endif
#ifndef X_EXP_NOSTORE
#define X_EXP_NOSTORE 0  // timing experiments only (wrong results): no exchange-slot stores
#endif
#ifndef X_EXP_OWNIMPORT
#define X_EXP_OWNIMPORT 0  // timing experiments only (wrong results): import this block's own slot
#endif
#ifndef X_EXP_NOIMPORT
#define X_EXP_NOIMPORT 0  // timing experiments only (wrong results): imports re-read one 16-B chunk
#endif
__device__ __forceinline__ void dma_half(const float *B, int h, int n1, int wu, unsigned chunk16, unsigned slot) {
    if (D_EXP_NODMA && h >= 2) return;
    const unsigned dst = slot + (unsigned)(wu * 4 * KD * 4);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = min(32 * h + 4 * wu + i, n1 - 1);
        const unsigned voff = (unsigned)j * (KD * 4) + chunk16;
        if (i == 0) glds16<0>(B, voff, dst);
        if (i == 1) glds16<KD * 4>(B, voff, dst);
        if (i == 2) glds16<2 * KD * 4>(B, voff, dst);
        if (i == 3) glds16<3 * KD * 4>(B, voff, dst);
    }
}

// Quantise staging slot `stg` (frame-1 rows j0 .. j0 + 31) into rows 32 hh .. +31 of the int8
// tile slot `rq`: thread t takes floats 16 sub .. +15 of row t >> 4.  In stages, so that the
// sweep spreads them over its MFMA steps; branch-free, so that a segment stays one basic block.
//   IK: q_j = 127 * 2^e_j (e_j = 2, 1, 0 for m_j < 1/4, < 1/2, above), the per-column word
//       = the key shift tb + 2 - e_j; rows j >= n1 (padding) get q = 0 (zero codes: D = 0).
//   float: q_j = RN(127 RN(1/m_j)), the per-column word = s_j = RN(m_j RN(1/127)).
// Statistics over the rows below n1 of real halves (`live`: a half past the end holds stale
// bytes; clamped padding rows duplicate row n1 - 1): max s_j (the window's Eb), max |b_j|^2
// (Bn), and `bad`: IK -- a value outside [-IK_MMAX, IK_MMAX] or non-finite (the pair takes the
// float path); float -- non-finite or a row scale outside [2^-40, 2^40] (the exact path).
template <bool IK>
struct QHalf {
    f32x4v x0, x1, x2, x3;
    float m, qa, qb, q, s;
    int sh;
    i32x4 code;
    __device__ __forceinline__ void load(const char *stg, int t) {  // 4 ds_read_b128
        const char *src = stg + (t >> 4) * (KD * 4) + (t & 15) * 16;
        x0 = *reinterpret_cast<const f32x4v *>(src);
        x1 = *reinterpret_cast<const f32x4v *>(src + 256);
        x2 = *reinterpret_cast<const f32x4v *>(src + 512);
        x3 = *reinterpret_cast<const f32x4v *>(src + 768);
    }
    // the same 16 floats straight from frame 1 in memory (row j clamped to n1 - 1): the exchange
    // kernel's solo path
    __device__ __forceinline__ void load_global(const float *B, int j, int n1, int t) {
        const float *src = B + (size_t)min(j, n1 - 1) * KD + 16 * (t & 15);
        x0 = *reinterpret_cast<const f32x4v *>(src);
        x1 = *reinterpret_cast<const f32x4v *>(src + 4);
        x2 = *reinterpret_cast<const f32x4v *>(src + 8);
        x3 = *reinterpret_cast<const f32x4v *>(src + 12);
    }
    static constexpr bool CC = IK && D_CC;  // |b_j| from the codes
    __device__ __forceinline__ void absmax() {
        if constexpr (CC) {
            m = absmaximum3(0.f, x0[0], x0[1]);
            m = absmaximum3(m, x0[2], x0[3]);
            m = absmaximum3(m, x1[0], x1[1]);
            m = absmaximum3(m, x1[2], x1[3]);
            m = absmaximum3(m, x2[0], x2[1]);
            m = absmaximum3(m, x2[2], x2[3]);
            m = absmaximum3(m, x3[0], x3[1]);
            m = absmaximum3(m, x3[2], x3[3]);
            return;
        }
        m = absmax3(0.f, x0[0], x0[1]);
        m = absmax3(m, x0[2], x0[3]);
        m = absmax3(m, x1[0], x1[1]);
        m = absmax3(m, x1[2], x1[3]);
        m = absmax3(m, x2[0], x2[1]);
        m = absmax3(m, x2[2], x2[3]);
        m = absmax3(m, x3[0], x3[1]);
        m = absmax3(m, x3[2], x3[3]);
    }
    __device__ __forceinline__ void sumsq() {
        if constexpr (CC) return;
        qa = __builtin_fmaf(x0[0], x0[0], __builtin_fmaf(x0[1], x0[1], __builtin_fmaf(x0[2], x0[2], x0[3] * x0[3])));
        qb = __builtin_fmaf(x1[0], x1[0], __builtin_fmaf(x1[1], x1[1], __builtin_fmaf(x1[2], x1[2], x1[3] * x1[3])));
        qa = __builtin_fmaf(x2[0], x2[0], __builtin_fmaf(x2[1], x2[1], __builtin_fmaf(x2[2], x2[2], __builtin_fmaf(x2[3], x2[3], qa))));
        qb = __builtin_fmaf(x3[0], x3[0], __builtin_fmaf(x3[1], x3[1], __builtin_fmaf(x3[2], x3[2], __builtin_fmaf(x3[3], x3[3], qb))));
    }
    __device__ __forceinline__ void reduce(int j, int n1, int tb) {
        if constexpr (CC) {
            row16_max(m);
        } else {
            qa = qa + qb;
            row16_max_sum(m, qa);  // qa = |b|^2 from here on
        }
        if constexpr (IK) {
            // e from m's biased exponent: [1/2, 2) -> 0, [1/4, 1/2) -> 1, below -> 2 (m q_e < 128)
            const int e = min(max(126 - (int)((__float_as_uint(m) >> 23) & 0xffu), 0), 2);
            q = j < n1 ? __builtin_ldexpf(127.f, e) : 0.f;
            s = __builtin_ldexpf(1.f / 127.f, -e);  // = 1 / q rounded: the Eb bound
            sh = tb + 2 - e;
        } else {
            q = m > 0.f ? 127.f * __builtin_amdgcn_rcpf(m) : 0.f;
            s = m * (1.f / 127.f);
        }
    }
    __device__ __forceinline__ void pack01() {
        code[0] = pack4(x0[0], x0[1], x0[2], x0[3], q);
        code[1] = pack4(x1[0], x1[1], x1[2], x1[3], q);
    }
    __device__ __forceinline__ void pack23() {
        code[2] = pack4(x2[0], x2[1], x2[2], x2[3], q);
        code[3] = pack4(x3[0], x3[1], x3[2], x3[3], q);
        if constexpr (CC) {  // |c_j|^2 of the codes; |b_j| <= s_j (|c_j| + 8) (|b_jk - c_jk s_j| <= s_j / 2)
            int c2 = __builtin_amdgcn_sdot4(code[0], code[0], 0, false);
            c2 = __builtin_amdgcn_sdot4(code[1], code[1], c2, false);
            c2 = __builtin_amdgcn_sdot4(code[2], code[2], c2, false);
            c2 = __builtin_amdgcn_sdot4(code[3], code[3], c2, false);
            row16_sum_i(c2);
            const float bn = s * (__builtin_amdgcn_sqrtf((float)c2) + 8.0f) * 1.0001f;  // v_sqrt: 1 ulp
            qa = bn * bn;  // an upper bound of |b_j|^2 (the window's Bn)
        }
    }
    // cs: the tile's entries of the per-column key shifts kept for the epilogue (IK; live halves)
    __device__ __forceinline__ void store(char *rq, int hh, int t, bool live, float &smax, float &b2max, bool &bad,
                                          unsigned char *cs) {
        const int r = t >> 4, sub = t & 15, row = 32 * hh + r;
        *reinterpret_cast<i32x4 *>(rq + row * D_RS + (D_PAD ? sub << 4 : (sub ^ (row & 15)) << 4)) = code;
        if constexpr (IK) {
            if (sub == 0) {
                reinterpret_cast<int *>(rq + D_TILE)[row] = sh;
                if (live) cs[row] = (unsigned char)sh;
            }
            bad = bad | (live & !((qa <= 1e30f) & (m <= IK_MMAX)));  // CC: m carries any NaN
        } else {
            if (sub == 0) reinterpret_cast<float *>(rq + D_TILE)[row] = s;
            bad = bad | (live & !((qa <= FLT_MAX) & ((m == 0.f) | ((m >= SCALE_LO) & (m <= SCALE_HI)))));
        }
        smax = vmax(smax, live ? s : 0.f);
        b2max = vmax(b2max, live ? qa : 0.f);
    }
    // exchange mode (k_q8d_match's pair exchange): the IK store into ring rows that carry their key
    // shift in the row padding (bytes 256 .. 259 of a D_RS row) -- the same bytes also into this
    // block's exchange slot `xs` when `xon` (plain stores: the lines stay in the XCD's L2)
    __device__ __forceinline__ void store_x(char *rq, int hh, int t, bool live, float &smax, float &b2max, bool &bad,
                                            char *xs, bool xon) {
        const int r = t >> 4, sub = t & 15, row = 32 * hh + r;
        *reinterpret_cast<i32x4 *>(rq + row * D_RS + (sub << 4)) = code;
        if (sub == 0) reinterpret_cast<int *>(rq + D_TILE)[row] = sh;
        if (xon && !X_EXP_NOSTORE) {
            *reinterpret_cast<i32x4 *>(xs + r * KD + (sub << 4)) = code;
            // this wave's 4 rows' shifts (lanes 0, 16, 32, 48), one whole 128-B line per wave
            const i32x4 s4 = {__builtin_amdgcn_readlane(sh, 0), __builtin_amdgcn_readlane(sh, 16),
                              __builtin_amdgcn_readlane(sh, 32), __builtin_amdgcn_readlane(sh, 48)};
            if ((t & 63) < 8) *reinterpret_cast<i32x4 *>(xs + 32 * KD + (t >> 6) * 128 + (t & 7) * 16) = s4;
        }
        bad = bad | (live & !((qa <= 1e30f) & (m <= IK_MMAX)));
        smax = vmax(smax, live ? s : 0.f);
        b2max = vmax(b2max, live ? qa : 0.f);
    }
};

// The pair's frame-1 state after a sweep (every workgroup of the pair computes the same).
struct Sweep {
    float smax, b2max;
    bool bad;
};

// The sweep over all column tiles of frame 1 against the wave's A rows (aI): m1 / m2 get the
// lane-local tagged top-2 per row (IK: integer keys in the registers' bits).  first: halves 0, 1
// were issued before the A phase (else they are issued here).  Ends with every DMA drained and
// every wave past its last LDS read of staging / ring (the epilogue may reuse them).
template <bool IK>
__device__ __forceinline__ Sweep sweep(char *lds, const float *B, int n1, int t, int lane, int wu, unsigned chunk16,
                                       unsigned lds_base, const i32x4 (&aI)[RG][KD / 32], float (&m1)[RG][16],
                                       float (&m2)[RG][16], int tb, unsigned tkeep, bool first) {
    const int ntc = (n1 + BN - 1) / BN, nh = 2 * ntc;  // column tiles, staging halves (>= 2)
    const int fr = lane & 31, fh = lane >> 5;
    char *ring = lds + D_OFF_RING;
    unsigned char *colsh = reinterpret_cast<unsigned char *>(lds + D_OFF_COL);
    Sweep st = {0.f, 0.f, false};
    if (!first) {
        dma_half(B, 0, n1, wu, chunk16, lds_base);
        dma_half(B, 1, n1, wu, chunk16, lds_base + D_HALF);
    }
    if (nh > 2) {
        dma_half(B, 2, n1, wu, chunk16, lds_base + 2 * D_HALF);
        wait_vm<4>();
    } else {
        wait_vm<0>();
    }
    __syncthreads();  // halves 0, 1 landed
    {
        QHalf<IK> h;
#pragma unroll
        for (int hh = 0; hh < 2; hh++) {
            h.load(lds + hh * D_HALF, t);
            h.absmax();
            h.sumsq();
            h.reduce(32 * hh + (t >> 4), n1, tb);
            h.pack01();
            h.pack23();
            h.store(ring, hh, t, true, st.smax, st.b2max, st.bad, colsh);
        }
    }
    __syncthreads();  // tile 0 in ring slot 0; staging slots 0, 1 free
    if (nh > 3) dma_half(B, 3, n1, wu, chunk16, lds_base);

    // B fragment: column block c (0, 1), lane row 32 c + fr, k32 step s: chunk (2 s + fh)
    const int rdb = fr * D_RS + (D_PAD ? fh * 16 : 0);
    const int xsw = fh ^ (fr & 15);  // !D_PAD: chunk (2 s + fh) ^ (fr & 15) = 2 s ^ xsw

    i32x16 acc[RG][2];
    const float kinit = IK ? __int_as_float((int)0x80000000) : -__builtin_inff();
#pragma unroll
    for (int g = 0; g < RG; g++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            m1[g][q] = kinit;
            m2[g][q] = kinit;
        }
    // "tile -1" of group 1, folded beside tile 0, never a maximum: IK -2^22 (below every real
    // dot, |D| <= 127^2 256 < 2^22) at the widest shift; float 0 with the offset -3e38
#pragma unroll
    for (int q = 0; q < 16; q++) {
        acc[1][0][q] = IK ? -(1 << 22) : 0;
        acc[1][1][q] = IK ? -(1 << 22) : 0;
    }
    unsigned vkeep = tkeep;
    asm volatile("" : "+v"(vkeep));  // a VGPR operand: v_and_or_b32 may read one SGPR only
    // the tile before: float dequantisation (fma(t, 2^21 s, -2^23 s); -3e38 past n1) / key shifts
    float pr0 = 0.f, pr1 = 0.f, pc0 = -3.0e38f, pc1 = -3.0e38f;
    int sh0 = tb + 2, sh1 = tb + 2;

    // the fold of rows 2 S, 2 S + 1 of group FG (tile tags G0, G0 + 1)
#define D_FOLD2(FG, S, G0)                                                                   \
    do {                                                                                     \
        _Pragma("unroll") for (int q = 2 * (S); q < 2 * (S) + 2; q++) {                      \
            if constexpr (IK) {                                                              \
                /* v_lshl_or_b32 keys; v_max3_i32 / v_med3_i32 / v_max_i32 top-2 */          \
                fold_keys(acc[FG][0][q], acc[FG][1][q], sh0, sh1, (G0), (G0) + 1u, m1[FG][q], m2[FG][q]); \
            } else {                                                                         \
                const float a_ = __builtin_fmaf(__int_as_float(acc[FG][0][q]), pr0, pc0);    \
                const float b_ = __builtin_fmaf(__int_as_float(acc[FG][1][q]), pr1, pc1);    \
                fold3(tag(a_, vkeep, (G0)), tag(b_, vkeep, (G0) + 1u), m1[FG][q], m2[FG][q]); \
            }                                                                                \
        }                                                                                    \
    } while (0)
    // group G's MFMAs on the tile at `rs` (fragments read D_PF k32 steps ahead), folding group
    // FG meanwhile, and this thread's share of the next tile's quantisation from staging STG
    // into rows 32 HH .. of slot rq, one stage per k32 step; every step is fenced
    // (sched_barrier) so that the stages stay spread over the MFMAs
#define D_SEG(G, FG, G0, STG, HH, J0, LIVE)                                                  \
    do {                                                                                     \
        const char *base = rs + rdb;                                                         \
        int xs_ = xsw;                                                                       \
        if (!D_PAD) asm volatile("" : "+v"(xs_)); /* per-use offsets: not 8 loop-invariant VGPRs */ \
        i32x4 b0_[KD / 32], b1_[KD / 32];                                                    \
        QHalf<IK> qh_;                                                                       \
        _Pragma("unroll") for (int s_ = 0; s_ < KD / 32 + D_PF; s_++) {                      \
            if (D_EXP_NOQUANT) {                                                             \
            } else if (s_ == QS_LOAD) qh_.load((STG), t);                                    \
            else if (s_ == QS_LOAD + 1) qh_.absmax();                                        \
            else if (s_ == QS_LOAD + 2) qh_.sumsq();                                         \
            else if (s_ == QS_LOAD + 3) qh_.reduce((J0) + (t >> 4), n1, tb);                 \
            else if (s_ == QS_LOAD + 4) qh_.pack01();                                        \
            else if (s_ == QS_LOAD + 5) qh_.pack23();                                        \
            else if (s_ == QS_LOAD + 6) qh_.store(rq, (HH), t, (LIVE), st.smax, st.b2max, st.bad, colsh + (tc + 1) * BN); \
            if (s_ < KD / 32) {                                                              \
                const int ch_ = D_PAD ? 32 * s_ : ((2 * s_) ^ xs_) * 16;                     \
                b0_[s_] = *reinterpret_cast<const i32x4 *>(base + ch_);                      \
                b1_[s_] = *reinterpret_cast<const i32x4 *>(base + 32 * D_RS + ch_);          \
            }                                                                                \
            if (s_ >= D_PF) {                                                                \
                const int m_ = s_ - D_PF;                                                    \
                if (m_ == 0) {                                                               \
                    if constexpr (IK) {                                                      \
                        const i32x16 z_ = {};                                                \
                        acc[G][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][0], b0_[0], z_, 0, 0, 0); \
                        acc[G][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][0], b1_[0], z_, 0, 0, 0); \
                    } else {                                                                 \
                        acc[G][0] = mfma_i8_from4(aI[G][0], b0_[0]);                         \
                        acc[G][1] = mfma_i8_from4(aI[G][0], b1_[0]);                         \
                    }                                                                        \
                } else {                                                                     \
                    acc[G][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b0_[m_], acc[G][0], 0, 0, 0); \
                    acc[G][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b1_[m_], acc[G][1], 0, 0, 0); \
                }                                                                            \
                if (D_EXP_NOFOLD)                                                            \
                    asm volatile("" : : "v"(acc[FG][0][2 * m_]), "v"(acc[FG][1][2 * m_]));  \
                else                                                                         \
                    D_FOLD2(FG, m_, G0);                                                     \
            }                                                                                \
            __builtin_amdgcn_sched_barrier(0);                                               \
        }                                                                                    \
    } while (0)

    // Tile t sweeps from ring slot t & 1 while tile t + 1 is quantised into the other slot from
    // staging halves 2t + 2 (during group 0) and 2t + 3 (during group 1); half 2t + 4 is issued
    // at the top (into the slot half 2t + 1 left), 2t + 5 at the middle (into the slot half
    // 2t + 2 left).  Every half thus has one whole tile of latency cover.  In the last
    // iteration the quantisation runs on stale staging bytes into the unused slot (no DMA is in
    // flight then, `live` false): branch-free segments, nothing read afterwards.
    int sA = 2, sB = 0;  // staging slots of halves 2t + 2, 2t + 3
    for (int tc = 0; tc < ntc; tc++) {
        if (2 * tc + 3 < nh) {  // half 2t + 2 landed (2t + 3 may be in flight)
            wait_vm<4>();
        } else {
            wait_vm<0>();
        }
        D_SYNC();  // tile t complete in its slot; staging slot of half 2t + 1 free
        const int sN = 3 - sA - sB;  // the third staging slot
        if (2 * tc + 4 < nh) dma_half(B, 2 * tc + 4, n1, wu, chunk16, lds_base + (unsigned)(sN * D_HALF));
        const char *rs = ring + (tc & 1) * D_SLOT;
        char *rq = ring + ((tc + 1) & 1) * D_SLOT;
        const char *stA = lds + sA * D_HALF, *stB = lds + sB * D_HALF;
        const bool live = tc + 1 < ntc;
        const unsigned gp_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)max(tc - 1, 0));
        D_SEG(0, 1, gp_, stA, 0, 32 * (2 * tc + 2), live);
        if constexpr (IK) {  // the key shifts of tile tc's columns
            const int *rl_ = reinterpret_cast<const int *>(rs + D_TILE);
            sh0 = rl_[fr];
            sh1 = rl_[fr + 32];
        } else {  // the dequantisation operands of tile tc: fma(t, 2^21 s, -2^23 s)
            const float *rl_ = reinterpret_cast<const float *>(rs + D_TILE);
            const int col_ = tc * BN + fr;
            const float s0_ = rl_[fr], s1_ = rl_[fr + 32];
            pr0 = col_ < n1 ? 2097152.0f * s0_ : 0.f;
            pr1 = col_ + 32 < n1 ? 2097152.0f * s1_ : 0.f;
            pc0 = col_ < n1 ? -8388608.0f * s0_ : -3.0e38f;
            pc1 = col_ + 32 < n1 ? -8388608.0f * s1_ : -3.0e38f;
        }
        if (2 * tc + 4 < nh) {  // half 2t + 3 landed (2t + 4 may be in flight)
            wait_vm<4>();
        } else {
            wait_vm<0>();
        }
        // the staging slot of half 2t + 2 is free for half 2t + 5: a wave quantises exactly the
        // staging rows it copies itself (rows 4 w .. +3 of every half), so its own reads of them
        // (done in group 0) and its own vmcnt are the whole condition -- no block barrier
        if (2 * tc + 5 < nh) dma_half(B, 2 * tc + 5, n1, wu, chunk16, lds_base + (unsigned)(sA * D_HALF));
        const unsigned gc_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)tc);
        D_SEG(1, 0, gc_, stB, 1, 32 * (2 * tc + 3), live);
        // halves 2t + 4, 2t + 5 sit in slots sN, sA
        const int nA = sN, nB = sA;
        sA = nA;
        sB = nB;
    }
    {  // group 1 of the last tile
        const unsigned gl_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)(ntc - 1));
#pragma unroll
        for (int s = 0; s < 8; s++) D_FOLD2(1, s, gl_);
    }
#undef D_FOLD2
#undef D_SEG
    return st;
}

// The block-wide reduction of the sweep statistics (one barrier; every wave is then past its
// sweep, so staging + ring are free for the epilogue).
__device__ __forceinline__ Sweep block_stats(Sweep st, float *misc, int w, int lane) {
    float smax = fmaxf(st.smax, swz_xor<16>(st.smax));
    float b2max = fmaxf(st.b2max, swz_xor<16>(st.b2max));
    smax = fmaxf(smax, __shfl_xor(smax, 32, 64));
    b2max = fmaxf(b2max, __shfl_xor(b2max, 32, 64));
    const bool wbad = __ballot(st.bad) != 0;
    __syncthreads();  // misc may still be read by a previous call
    if (lane == 0) {
        misc[4 * w] = smax;
        misc[4 * w + 1] = b2max;
        misc[4 * w + 2] = wbad ? 1.f : 0.f;
    }
    __syncthreads();
    Sweep r = {0.f, 0.f, false};
#pragma unroll
    for (int k = 0; k < D_NW; k++) {
        r.smax = fmaxf(r.smax, misc[4 * k]);
        r.b2max = fmaxf(r.b2max, misc[4 * k + 1]);
        r.bad = r.bad || misc[4 * k + 2] != 0.f;
    }
    return r;
}

// ---------------------------------------------------------------------------------------------
// Pair exchange (k_q8d_match with both row blocks of a pair running: 512 < n0, cap <= 1024):
// frame 1 is quantised ONCE per pair instead of once per block.  Block w (0, 1) quantises rows
// 32 w .. 32 w + 31 of every 64-column tile ("its half") from its own fp32 staging and gets the
// other half from the partner block through their XCD's L2 (the in-sweep quantisation was ~1/4
// of the sweep's cycles: tools/gpu_trace_exp.sh, noquant).  Per block, in memory: XR exchange
// slots of 32 int8 ring rows (D_RS bytes: 256 codes + the key shift in the row padding) -- byte
// for byte the rows as they sit in the LDS ring, so that the import is a plain LDS-DMA copy --
// then the block's final statistics; per block a progress flag ((XCC id + 1) << 16 | tiles
// stored), zeroed before every launch.
//   tile t:  top     every wave's vmcnt(0) + the block barrier: this block's halves of tiles
//                    <= t + 1 are stored; thread 0 publishes t + 2 (agent-scope atomic store);
//                    each wave LDS-DMAs the partner's flag (sc1: device scope, past the L1).
//            seg 0   MFMAs of tile t (group 0); quantisation of own half of tile t + 2 (load ..
//                    reduce, from staging slot t & 1)
//            middle  flag >= t + 2: the partner's half of tile t + 1 is stored and the partner
//                    is past its top of tile t.  Each wave LDS-DMAs its 4 rows of that half (sc1)
//                    into ring slot (t + 1) % 3.
//            seg 1   MFMAs (group 1); pack + store own half of tile t + 2 into ring slot
//                    (t + 2) % 3 and exchange slot (t + 2) % XR, which held tile t - 1 (the
//                    partner copied it in its tile t - 2, complete at its top of tile t - 1).
// Wave w copies exactly the rows the partner's wave w stores (4 w .. 4 w + 3), so each wave checks
// the flag for itself.  The statistics (Bn, Eb, range flag) of the partner half arrive at the end
// as the partner block's own (flag X_FINAL).  A flag published on another XCD (the per-XCD L2s
// are not coherent with each other) or one that does not advance within X_SPIN polls puts the
// wave in SOLO mode: it quantises the partner rows itself from frame 1 in memory and stores
// nothing more, its block stops publishing from the next tile, and without the partner's final
// statistics the block recomputes them from frame 1.  Slower, never wrong, never waiting on a
// block that may not be resident.
#ifndef D_XCH
#define D_XCH 0  // 1: the pair exchange (allpairs_q8d_xch_bytes > 0); 0: every block quantises all of frame 1
#endif
#ifndef X_UNIQUE
// 1: one exchange slot per tile (never reused within a launch: the imports are plain LDS-DMA
// loads -- no line of a slot can be in this CU's L1 before the slot was written); 0: 4 slots
// reused in turn, imported with sc1 (L1-bypassing) LDS-DMA loads
#define X_UNIQUE 1
#endif
constexpr int XR = X_UNIQUE ? 16 : 4;       // exchange slots per block (16 = the tiles of cap 1024)
// an exchange slot: 32 rows of 256 codes (256-B aligned: every line written whole), then per wave
// one 128-B line holding its 4 rows' key shifts (replicated: the line is written whole)
constexpr int X_SLOT = 32 * KD + 8 * 128;
constexpr int X_BLOCK = XR * X_SLOT + 256;  // + the block's final statistics
constexpr int X_OFF_RING = 2 * D_HALF;      // exchange mode: 2 staging slots (own halves), 4 ring slots
constexpr int X_RSLOT = D_SLOT;             // an exchange-mode ring slot: 64 padded rows + 64 key shifts
constexpr unsigned X_FINAL = 0xffffu;
static_assert(X_OFF_RING + 4 * X_RSLOT <= D_OFF_ROW, "the exchange ring fits below the row data");
static_assert(D_PAD, "the exchange keeps the key shifts in the ring rows' padding");
#ifndef X_SPIN
#define X_SPIN 512  // flag polls (~0.4 us each) before SOLO
#endif
#ifndef X_FORCE_SOLO
// test builds (tools/build_variant.sh xsolo -DX_FORCE_SOLO=1): in pairs p % 3 == 1, block
// (p / 3) & 1 goes SOLO at tile (p / 6) % ntc -- the SOLO quantisation, the partner's spin-out and
// the statistics recompute then run under the parity tests
#define X_FORCE_SOLO 0
#endif

// LDS-DMA with sc1 (device scope: served by the XCD's L2, never a stale L1 line)
template <int DOFF>
__device__ __forceinline__ void glds16_sc1(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_add_u32 m0, %2, %3\n\t"
        "global_load_lds_dwordx4 %0, %1 sc1"
        :
        : "v"(voff), "s"(sbase), "s"(lds_byte), "i"(DOFF)
        : "memory", "m0", "scc");
}
__device__ __forceinline__ void glds4_sc1(const void *sbase, unsigned lds_byte) {
    asm volatile(
        "s_mov_b32 m0, %1\n\t"
        "global_load_lds_dword %0, %2 sc1"
        :
        : "v"(0u), "s"(lds_byte), "s"(sbase)
        : "memory", "m0");
}
__device__ __forceinline__ void glds4_x(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_mov_b32 m0, %1\n\t"
        "global_load_lds_dword %0, %2"
        :
        : "v"(voff), "s"(lds_byte), "s"(sbase)
        : "memory", "m0");
}
__device__ __forceinline__ void glds4_x_sc1(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_mov_b32 m0, %1\n\t"
        "global_load_lds_dword %0, %2 sc1"
        :
        : "v"(voff), "s"(lds_byte), "s"(sbase)
        : "memory", "m0");
}
// vmcnt wait that is also a compiler memory barrier (LDS written by DMA is read after it; stores
// before it are not sunk below it)
template <int N>
__device__ __forceinline__ void wait_vm_mem() {
    asm volatile("s_waitcnt vmcnt(%0)" : : "i"(N) : "memory");
}
__device__ __forceinline__ unsigned xcc_tag() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x + 1u;
}

struct XPair {
    char *own;             // this block's X_BLOCK
    const char *par;       // the partner's
    unsigned *fown;        // this block's flag
    const unsigned *fpar;  // the partner's
    int w;                 // this block's half
    unsigned tag;          // (XCC id + 1) of this block
    int solo_at;           // X_FORCE_SOLO: the tile this block goes SOLO at (-1: never)
};
__device__ __forceinline__ void x_publish(const XPair &xp, unsigned v) {
    __hip_atomic_store(xp.fown, (xp.tag << 16) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 1: the flag says >= need from this XCD; -1: from another XCD; 0: not yet
__device__ __forceinline__ int x_check(unsigned v, unsigned need, unsigned tag) {
    const unsigned ft = v >> 16;
    return ft == 0u ? 0 : ft != tag ? -1 : (v & 0xffffu) >= need ? 1 : 0;
}
// poll the partner's flag (this wave, flag word xw[wu]) until >= need: true, or SOLO: false
__device__ __forceinline__ bool x_wait(const XPair &xp, const unsigned *xw, unsigned fw_l, int wu, int lane,
                                       unsigned need) {
    X_CNT(0);
    for (int i = 0; i < X_SPIN; i++) {
        if (lane == 0) glds4_sc1(xp.fpar, fw_l);
        wait_vm_mem<0>();
        X_CNT(1);
        const int c = x_check(__builtin_amdgcn_readfirstlane(xw[wu]), need, xp.tag);
        if (c < 0) X_CNT(2);
        if (c != 0) return c > 0;
        __builtin_amdgcn_s_sleep(8);
    }
    X_CNT(3);
    return false;
}
// this wave's 4 rows of the partner's half (rows 4 wu .. + 3 of half pw), exchange slot `src` ->
// the ring slot at LDS byte `slot`: one LDS-DMA per 256-B row (16 lanes) + the rows' 4 key
// shifts (4 lanes) -- 5 instructions per wave
__device__ __forceinline__ void x_import(const char *src, unsigned slot, int pw, int wu, int lane) {
    if (X_EXP_NOIMPORT) {  // keep the instruction count: re-read one chunk
#pragma unroll
        for (int k = 0; k < 5; k++)
            if (lane < 4) glds16<0>(src, 0u, slot + (unsigned)((32 * pw + 4 * wu + k) * D_RS));
        return;
    }
    if (lane < 16) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int row = 4 * wu + k;
            if (X_UNIQUE)
                glds16<0>(src, (unsigned)(row * KD + 16 * lane), slot + (unsigned)((32 * pw + row) * D_RS));
            else
                glds16_sc1<0>(src, (unsigned)(row * KD + 16 * lane), slot + (unsigned)((32 * pw + row) * D_RS));
        }
    }
    if (lane < 4) {
        const unsigned so = (unsigned)(32 * KD + wu * 128 + 4 * lane), sd = slot + (unsigned)(D_TILE + (32 * pw + 4 * wu) * 4);
        if (X_UNIQUE)
            glds4_x(src, so, sd);
        else
            glds4_x_sc1(src, so, sd);
    }
}
// SOLO: this thread's 16 values of the partner half of `tile` quantised here (frame 1 in memory)
__device__ __forceinline__ void x_solo(char *rq, const float *B, int tile, int pw, int n1, int t, int tb) {
    QHalf<true> h;
    const int r = t >> 4, sub = t & 15, row = 32 * pw + r, j = tile * BN + row;
    h.load_global(B, j, n1, t);
    h.absmax();
    h.sumsq();
    h.reduce(j, n1, tb);
    h.pack01();
    h.pack23();
    *reinterpret_cast<i32x4 *>(rq + row * D_RS + (sub << 4)) = h.code;
    if (sub == 0) reinterpret_cast<int *>(rq + D_TILE)[row] = h.sh;
}
// the statistics of half pw of every tile, from frame 1 in memory (the partner's are missing)
__device__ __forceinline__ Sweep x_stats(const float *B, int pw, int n1, int t, int tb) {
    Sweep st = {0.f, 0.f, false};
    const int ntc = (n1 + BN - 1) / BN;
    for (int tile = 0; tile < ntc; tile++) {
        QHalf<true> h;
        const int j = tile * BN + 32 * pw + (t >> 4);
        h.load_global(B, j, n1, t);
        h.absmax();
        h.sumsq();
        h.reduce(j, n1, tb);
        const bool live = j < n1;  // rows past n1 repeat row n1 - 1: the same statistics either way
        st.bad = st.bad | (live & !((h.qa <= 1e30f) & (h.m <= IK_MMAX)));
        st.smax = vmax(st.smax, live ? h.s : 0.f);
        st.b2max = vmax(st.b2max, live ? h.qa : 0.f);
    }
    return st;
}

// The integer-key sweep with the pair exchange: the same m1 / m2 and (after x_final) the same
// statistics as sweep<true>.  Own halves of tiles 0, 1 were issued before the A phase into
// staging slots 0, 1.  Returns this block's statistics of its own halves.
// Schedule (tile T: own half staged at the top of T - 4 into staging slot T & 1, quantised
// during T - 3 into ring slot T % 4 and exchange slot T % XR, stored by the top of T - 2, where
// the flag then says "T + 1 tiles stored"; the partner half imported at the END of tile T - 2,
// landed by the top of T):
//   top of t    vmcnt(2) (everything but the newest import) + barrier; publish t + 3; stage t + 4
//   seg 0       MFMAs of tile t (group 0); own tile t + 3: load .. reduce
//   middle      LDS-DMA of the partner's flag
//   seg 1       MFMAs (group 1); own tile t + 3: pack, store
//   end of t    the flag >= t + 3 (the partner is past its top of t, a whole tile ago in step):
//               import the partner half of tile t + 2
// Exchange slot t + 3 (written in seg 1 of t) held tile t - 1, which the partner imported at the
// end of its tile t - 3 and had landed at its top of t - 1 -- before it published t + 2, which
// this wave saw at the end of tile t - 1.
__device__ __forceinline__ Sweep sweep_x(char *lds, const float *B, int n1, int t, int lane, int wu, unsigned chunk16,
                                         unsigned lds_base, const i32x4 (&aI)[RG][KD / 32], float (&m1)[RG][16],
                                         float (&m2)[RG][16], int tb, const XPair &xp) {
    const int ntc = (n1 + BN - 1) / BN;  // >= 3 (the kernel's condition)
    const int fr = lane & 31, fh = lane >> 5, w = xp.w, pw = 1 - w;
    char *ring = lds + X_OFF_RING;
    const unsigned ring_l = lds_base + X_OFF_RING;  // ring slot 0
    unsigned *xw = reinterpret_cast<unsigned *>(lds + D_OFF_X);  // [NW] flags, [NW] solo
    const unsigned fw_l = lds_base + D_OFF_X + 4u * (unsigned)wu;
    Sweep st = {0.f, 0.f, false};
    bool wsolo = false;
    if (t == 0) xw[D_NW] = 0u;
    auto go_solo = [&]() {
        X_CNT(4);
        wsolo = true;
        if (lane == 0) xw[D_NW] = 1u;
    };
    // ---- prologue: own halves of tiles 0, 1, 2 -> ring slots and exchange slots 0, 1, 2 ----
    wait_vm_mem<0>();
    __syncthreads();  // staging slots 0, 1 landed
    {
        QHalf<true> h;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int j = k * BN + 32 * w + (t >> 4);
            h.load(lds + k * D_HALF, t);
            h.absmax();
            h.sumsq();
            h.reduce(j, n1, tb);
            h.pack01();
            h.pack23();
            h.store_x(ring + k * X_RSLOT, w, t, true, st.smax, st.b2max, st.bad, xp.own + k * X_SLOT, true);
        }
    }
    wait_vm_mem<0>();
    __syncthreads();  // every wave's stores done; staging slots 0, 1 free
    if (t == 0) x_publish(xp, 2u);
    dma_half(B, 2 * 2 + w, n1, wu, chunk16, lds_base);  // own half of tile 2 -> staging slot 0
    if (ntc > 3) {
        dma_half(B, 2 * 3 + w, n1, wu, chunk16, lds_base + D_HALF);  // tile 3 -> staging slot 1
        wait_vm_mem<4>();
    } else {
        wait_vm_mem<0>();
    }
    __syncthreads();  // tile 2 staged
    {
        QHalf<true> h;
        const int j = 2 * BN + 32 * w + (t >> 4);
        h.load(lds, t);
        h.absmax();
        h.sumsq();
        h.reduce(j, n1, tb);
        h.pack01();
        h.pack23();
        h.store_x(ring + 2 * X_RSLOT, w, t, true, st.smax, st.b2max, st.bad, xp.own + 2 * X_SLOT, true);
    }
    wait_vm_mem<0>();
    __syncthreads();
    // (tile 2 is published at the top of tile 0, after the imports below have landed: a flag of 3
    // must also mean "past the import of tile 0", which exchange slot 0's reuse relies on)
    // the partner halves of tiles 0, 1
    if (x_wait(xp, xw, fw_l, wu, lane, 2u) && !(X_FORCE_SOLO && xp.solo_at == 0)) {
        x_import(xp.par, ring_l, pw, wu, lane);
        x_import(xp.par + X_SLOT, ring_l + (unsigned)X_RSLOT, pw, wu, lane);
    } else {
        go_solo();
        x_solo(ring, B, 0, pw, n1, t, tb);
        x_solo(ring + X_RSLOT, B, 1, pw, n1, t, tb);
    }
    bool pend = !wsolo;  // the newest VMEM instructions are an import (5 per wave)

    const int rdb = fr * D_RS + fh * 16;
    i32x16 acc[RG][2];
#pragma unroll
    for (int g = 0; g < RG; g++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            m1[g][q] = __int_as_float((int)0x80000000);
            m2[g][q] = __int_as_float((int)0x80000000);
        }
#pragma unroll
    for (int q = 0; q < 16; q++) {  // "tile -1" of group 1 (see sweep)
        acc[1][0][q] = -(1 << 22);
        acc[1][1][q] = -(1 << 22);
    }
    int sh0 = tb + 2, sh1 = tb + 2;

#define X_FOLD2(FG, S, G0)                                                                   \
    do {                                                                                     \
        _Pragma("unroll") for (int q = 2 * (S); q < 2 * (S) + 2; q++)                        \
            fold_keys(acc[FG][0][q], acc[FG][1][q], sh0, sh1, (G0), (G0) + 1u, m1[FG][q], m2[FG][q]); \
    } while (0)
    // group G's MFMAs on the tile at `rs`, folding group FG meanwhile; QS: the quantisation
    // stages of own half of tile t + 3 in this segment (0: load .. reduce; 1: pack, store)
#define X_SEG(G, FG, G0, QS)                                                                 \
    do {                                                                                     \
        const char *base = rs + rdb;                                                         \
        i32x4 b0_[KD / 32], b1_[KD / 32];                                                    \
        _Pragma("unroll") for (int s_ = 0; s_ < KD / 32 + D_PF; s_++) {                      \
            if ((QS) == 0) {                                                                 \
                if (s_ == 1) qh.load(stg, t);                                                \
                else if (s_ == 2) qh.absmax();                                               \
                else if (s_ == 3) qh.sumsq();                                                \
                else if (s_ == 4) qh.reduce(jq, n1, tb);                                     \
            } else {                                                                         \
                if (s_ == 1) qh.pack01();                                                    \
                else if (s_ == 2) qh.pack23();                                               \
                else if (s_ == 3) qh.store_x(rq, w, t, live, st.smax, st.b2max, st.bad, xq, xon); \
            }                                                                                \
            if (s_ < KD / 32) {                                                              \
                b0_[s_] = *reinterpret_cast<const i32x4 *>(base + 32 * s_);                  \
                b1_[s_] = *reinterpret_cast<const i32x4 *>(base + 32 * D_RS + 32 * s_);      \
            }                                                                                \
            if (s_ >= D_PF) {                                                                \
                const int m_ = s_ - D_PF;                                                    \
                if (m_ == 0) {                                                               \
                    const i32x16 z_ = {};                                                    \
                    acc[G][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][0], b0_[0], z_, 0, 0, 0); \
                    acc[G][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][0], b1_[0], z_, 0, 0, 0); \
                } else {                                                                     \
                    acc[G][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b0_[m_], acc[G][0], 0, 0, 0); \
                    acc[G][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b1_[m_], acc[G][1], 0, 0, 0); \
                }                                                                            \
                X_FOLD2(FG, m_, G0);                                                         \
            }                                                                                \
            __builtin_amdgcn_sched_barrier(0);                                               \
        }                                                                                    \
    } while (0)

    for (int tc = 0; tc < ntc; tc++) {
        if (pend)
            wait_vm_mem<5>();  // staging of tile tc + 3, own stores of tile tc + 2, the import of tile tc
        else
            wait_vm_mem<0>();
        __syncthreads();  // tile tc complete in its ring slot; every wave's stores done
        const bool bsolo = xw[D_NW] != 0u;
        wsolo = wsolo | bsolo;
        if (t == 0 && !bsolo) x_publish(xp, (unsigned)min(tc + 3, ntc));
        if (tc + 4 < ntc) dma_half(B, 2 * (tc + 4) + w, n1, wu, chunk16, lds_base + (unsigned)((tc & 1) * D_HALF));
        const char *rs = ring + (tc & 3) * X_RSLOT;
        char *rq = ring + ((tc + 3) & 3) * X_RSLOT;
        char *xq = xp.own + ((tc + 3) % XR) * X_SLOT;
        const char *stg = lds + ((tc + 1) & 1) * D_HALF;
        const bool live = tc + 3 < ntc;
        const bool imp = tc + 2 < ntc;
        const bool xon = live && !wsolo;
        const int jq = (tc + 3) * BN + 32 * w + (t >> 4);
        QHalf<true> qh;
        const unsigned gp_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)max(tc - 1, 0));
        X_SEG(0, 1, gp_, 0);
        sh0 = reinterpret_cast<const int *>(rs + D_TILE)[fr];  // the key shifts of tile tc's columns
        sh1 = reinterpret_cast<const int *>(rs + D_TILE)[fr + 32];
        const bool poll = imp && !wsolo;
        if (poll && lane == 0) glds4_sc1(xp.fpar, fw_l);
        const unsigned gc_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)tc);
        X_SEG(1, 0, gc_, 1);
        pend = false;
        if (imp) {  // the partner half of tile tc + 2
            if (poll) {
                if (xon)
                    wait_vm_mem<2>();  // the flag (this wave's 2 exchange stores after it may fly)
                else
                    wait_vm_mem<0>();
                int c = x_check(__builtin_amdgcn_readfirstlane(xw[wu]), (unsigned)(tc + 3), xp.tag);
                if (c < 0) X_CNT(2);
                if (c == 0) c = x_wait(xp, xw, fw_l, wu, lane, (unsigned)(tc + 3)) ? 1 : -1;
                if (X_FORCE_SOLO && xp.solo_at >= 0 && tc + 2 >= xp.solo_at) c = -1;
                if (c < 0) go_solo();
            }
            if (!wsolo) {
                x_import((X_EXP_OWNIMPORT ? (const char *)xp.own : xp.par) + ((tc + 2) % XR) * X_SLOT,
                         ring_l + (unsigned)(((tc + 2) & 3) * X_RSLOT), pw, wu, lane);
                X_CNT(7);
                pend = true;
            } else {
                x_solo(ring + ((tc + 2) & 3) * X_RSLOT, B, tc + 2, pw, n1, t, tb);
            }
        }
    }
    {  // group 1 of the last tile
        const unsigned gl_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)(ntc - 1));
#pragma unroll
        for (int s = 0; s < 8; s++) X_FOLD2(1, s, gl_);
    }
#undef X_FOLD2
#undef X_SEG
    wait_vm_mem<0>();
    return st;
}

// After block_stats of sweep_x: publish this block's statistics (unless SOLO: its exchange
// stores stopped, so the flag must not move), take the partner's, or recompute them.
__device__ __forceinline__ Sweep x_final(Sweep st, const XPair &xp, char *lds, const float *B, int n1, int t,
                                         int lane, int w, int tb, float *misc) {
    unsigned *xw = reinterpret_cast<unsigned *>(lds + D_OFF_X);
    float *pst = reinterpret_cast<float *>(lds + D_OFF_X + 4 * (D_NW + 1));  // partner smax, b2max, bad, ok
    if (t == 0) {
        const bool bsolo = xw[D_NW] != 0u;  // block_stats' barriers made every wave's word visible
        if (!bsolo) {
            float *o = reinterpret_cast<float *>(xp.own + XR * X_SLOT);
            o[0] = st.smax;
            o[1] = st.b2max;
            o[2] = st.bad ? 1.f : 0.f;
            wait_vm_mem<0>();
            x_publish(xp, X_FINAL);
        }
        int ok = 0;
        for (int i = 0; i < X_SPIN; i++) {
            const int c = x_check(__hip_atomic_load(xp.fpar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), X_FINAL,
                                  xp.tag);
            if (c != 0) {
                ok = c > 0;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        if (ok) {
            const float *p = reinterpret_cast<const float *>(xp.par + XR * X_SLOT);
            pst[0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pst[1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pst[2] = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        pst[3] = ok ? 1.f : 0.f;
    }
    __syncthreads();
    Sweep p;
    if (w == 0) X_CNT(pst[3] != 0.f ? 5 : 6);
    if (pst[3] != 0.f) {
        p.smax = pst[0];
        p.b2max = pst[1];
        p.bad = pst[2] != 0.f;
    } else {
        p = block_stats(x_stats(B, 1 - xp.w, n1, t, tb), misc, w, lane);
    }
    st.smax = fmaxf(st.smax, p.smax);
    st.b2max = fmaxf(st.b2max, p.b2max);
    st.bad = st.bad || p.bad;
    return st;
}

__global__ __launch_bounds__(D_NT, 2) void k_q8d_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                       const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                       const float *__restrict__ desc1, double thresh, int dmode,
                                                       int *__restrict__ match_idx, float *__restrict__ match_score,
                                                       char *__restrict__ xch, unsigned *__restrict__ xflag) {
    __shared__ __attribute__((aligned(16))) char lds[D_LDS];
#ifdef MV_TRACE
    unsigned long long ts_[10] = {};
    D_STAMP(0);
#endif
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int pair = L / tiles_r, tr = L % tiles_r;
    const int n0 = min(max(n0v[pair], 0), cap), n1 = min(max(n1v[pair], 0), cap);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int row0 = tr * D_BM;
    int *oidx = match_idx + (size_t)pair * cap + row0;
    float *oscore = match_score ? match_score + (size_t)pair * cap + row0 : nullptr;  // null: indices only
    if (row0 + t < cap && (row0 + t >= n0 || n1 <= 0)) {  // rows in [n0, cap): no match
        oidx[t] = -1;
        if (oscore) oscore[t] = 0.f;
    }
    if (row0 >= n0 || n1 <= 0) return;
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;
    const int ntc = (n1 + BN - 1) / BN;

    const int wu = __builtin_amdgcn_readfirstlane(w);
    const unsigned chunk16 = (unsigned)(4 * (lane & 15) + (lane >> 4)) * 16;
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    float2 *rowv = reinterpret_cast<float2 *>(lds + D_OFF_ROW);
    float *misc = reinterpret_cast<float *>(lds + D_OFF_MISC);

    // the pair exchange when both row blocks of the pair run (see sweep_x); both decide alike
    const bool xmode = xch != nullptr && tiles_r == 2 && n0 > D_BM && ntc >= 3;
    XPair xp = {};
    if (xmode) {
        char *xb = xch + (size_t)pair * 2 * X_BLOCK;
        xp.own = xb + tr * X_BLOCK;
        xp.par = xb + (1 - tr) * X_BLOCK;
        xp.fown = xflag + 2 * (size_t)pair + tr;
        xp.fpar = xflag + 2 * (size_t)pair + 1 - tr;
        xp.w = tr;
        xp.tag = xcc_tag();
        xp.solo_at = X_FORCE_SOLO && pair % 3 == 1 && ((pair / 3) & 1) == tr ? (pair / 6) % ntc : -1;
    }
    // ---- prologue: halves 0, 1 (exchange: own halves of tiles 0, 1) in flight beside the A phase ----
    dma_half(B, xmode ? tr : 0, n1, wu, chunk16, lds_base);
    dma_half(B, xmode ? 2 + tr : 1, n1, wu, chunk16, lds_base + D_HALF);
    i32x4 aI[RG][KD / 32];
    float *rowe = D_EXACT_EA ? reinterpret_cast<float *>(lds + D_OFF_ROWE) : nullptr;
    a_phase<false, D_QB, D_EXACT_EA>(lds + D_OFF_AIMG + w * 32 * KD, rowv, w * 64, row0, n0, lane, A, nullptr,
                                     nullptr, nullptr, false, aI, rowe);
    D_STAMP(1);
    __syncthreads();  // the A images (staging slot 2 + the ring) are consumed
    float m1[RG][16], m2[RG][16];

    // the integer-key sweep; tag width: keys (D << (tb + 2)) | tag must fit 31 bits
    const int tbi = 2 * ntc <= 2 ? 1 : 32 - __builtin_clz(2 * ntc - 1);
    if (tbi <= 7) {
        Sweep st;
        if (xmode)
            st = x_final(block_stats(sweep_x(lds, B, n1, t, lane, wu, chunk16, lds_base, aI, m1, m2, tbi, xp), misc, w,
                                     lane),
                         xp, lds, B, n1, t, lane, w, tbi, misc);
        else
            st = block_stats(sweep<true>(lds, B, n1, t, lane, wu, chunk16, lds_base, aI, m1, m2, tbi,
                                         ~((1u << tbi) - 1u), true),
                             misc, w, lane);
        D_STAMP(2);
        if (!st.bad) {
            const double Bn = sqrt((double)st.b2max) * 1.0001;
            const double Eb = 8.0001 * (double)st.smax + 1e-30;  // exact power-of-two scaling
            // the window per maximiser column (its own 1 / q_j) unless the exchange ran
            epilogue<D_NW, true>(lds, rowv, m1, m2, Bn, Eb, false, tbi, ~((1u << tbi) - 1u), w, lane, row0, n0,
                                 n1, A, B, oidx, oscore, thresh, dmode, 1.0 / 508.0,
                                 xmode || !D_COLWIN ? nullptr : reinterpret_cast<const unsigned char *>(lds + D_OFF_COL),
                                 rowe);
            D_STAMP(3);
#ifdef MV_TRACE
            if (lane == 0 && blockIdx.x < D_TRACE_BLOCKS) {
                unsigned long long *o = g_d_trace + ((size_t)blockIdx.x * D_NW + w) * 10;
                for (int k = 0; k < 6; k++) o[k] = ts_[k];  // memtime x 4, memrealtime at entry / after A
                o[6] = __smid();
                o[7] = __builtin_amdgcn_s_memrealtime();
                o[9] = ts_[9];
            }
#endif
            return;
        }
    }
    // the float path: a column outside the integer keys' range, a non-finite value, or too many
    // column tiles for the key width
    const int tb = 2 * ntc <= 256 ? 8 : 32 - __builtin_clz(2 * ntc - 1);
    const Sweep st = block_stats(sweep<false>(lds, B, n1, t, lane, wu, chunk16, lds_base, aI, m1, m2, tb,
                                              ~((1u << tb) - 1u), tbi > 7), misc, w, lane);
    const double Bn = sqrt((double)st.b2max) * 1.0001;
    const double Eb = (8.001 * (double)st.smax + 4.76837158203125e-07 * Bn) * 1.0001 + 1e-30;
    epilogue<D_NW, false>(lds, rowv, m1, m2, Bn, Eb, st.bad, tb, ~((1u << tb) - 1u), w, lane, row0, n0, n1, A, B,
                          oidx, oscore, thresh, dmode);
}

}  // namespace

namespace mv {

// the pair exchange's buffer: per pair 2 x X_BLOCK, then 2 flags per pair (0: no exchange)
size_t allpairs_q8d_xch_bytes(int batch, int cap) {
    if (!D_XCH || batch <= 0 || (cap + D_BM - 1) / D_BM != 2) return 0;
    return (size_t)batch * (2 * X_BLOCK + 8);
}

int launch_allpairs_q8d_match(hipStream_t s, int batch, int cap, const int *n0, const int *n1, const float *desc0,
                              const float *desc1, double thresh, int *match_idx, float *match_score, int dmode,
                              void *xch, size_t xch_bytes) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    MV_REQUIRE((long)cap * KD * 4 < (1l << 32));  // 32-bit DMA source offsets within a pair
    const int tiles_r = (cap + D_BM - 1) / D_BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    const size_t xb = allpairs_q8d_xch_bytes(batch, cap);
    char *x = xb && xch && xch_bytes >= xb ? static_cast<char *>(xch) : nullptr;
    unsigned *xf = x ? reinterpret_cast<unsigned *>(x + (size_t)batch * 2 * X_BLOCK) : nullptr;
    if (xf) MV_HIP_TRY(hipMemsetAsync(xf, 0, (size_t)batch * 8, s));
    MV_PROF_BEGIN(s, "k_q8d_match");
    hipLaunchKernelGGL(k_q8d_match, dim3((unsigned)blocks), dim3(D_NT), 0, s, tiles_r, cap, n0, n1, desc0, desc1,
                       dmode ? -1e300 : thresh, dmode, match_idx, match_score, x, xf);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

#ifdef MV_TRACE
extern "C" int mv_debug_direct_trace(void *host, long bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_d_trace), (size_t)bytes) == hipSuccess ? 0 : -3;
}
extern "C" int mv_debug_exchange_counts(unsigned *host8, int reset) {
    if (hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_x_cnt), 8 * sizeof(unsigned)) != hipSuccess) return -3;
    if (reset) {
        const unsigned z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_x_cnt), z, sizeof z) != hipSuccess) return -3;
    }
    return 0;
}
#endif
