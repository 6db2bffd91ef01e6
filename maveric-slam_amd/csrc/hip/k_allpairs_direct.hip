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
// LDS (~138.7 KiB): staging 3 x 32 KiB | int8 ring 2 x 17.25 KiB | (|a|^2, s_a) per row |
// per-wave statistics | each column's key shift (4 KiB);
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
// [BM] float2 (|a|^2, s_a), past the int8 ring
constexpr int D_OFF_ROW = D_OFF_RING + 2 * D_SLOT;
constexpr int D_OFF_MISC = D_OFF_ROW + D_BM * 8;                    // [NW][4] per-wave statistics
#ifndef D_COLWIN
#define D_COLWIN 1  // the epilogue's window per maximiser column (0: the pair's widest, for A/B)
#endif
constexpr int D_OFF_COL = D_OFF_MISC + D_NW * 16;  // integer path: each frame-1 column's key shift (1 B)
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
#define D_STAMP(K) do { __builtin_amdgcn_sched_barrier(0); ts_[K] = __builtin_amdgcn_s_memtime(); if ((K) < 2) ts_[4 + (K)] = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define D_SYNC() __syncthreads()
#else
#define D_STAMP(K) do { } while (0)
#define D_SYNC() __syncthreads()
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
__device__ __forceinline__ void dma_half(const float *B, int h, int n1, int wu, unsigned chunk16, unsigned slot) {
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
            if (s_ == QS_LOAD) qh_.load((STG), t);                                           \
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
                D_FOLD2(FG, m_, G0);                                                         \
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

__global__ __launch_bounds__(D_NT, 2) void k_q8d_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                       const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                       const float *__restrict__ desc1, double thresh, int dmode,
                                                       int *__restrict__ match_idx, float *__restrict__ match_score) {
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

    // ---- prologue: halves 0, 1 in flight beside the A phase ----
    dma_half(B, 0, n1, wu, chunk16, lds_base);
    dma_half(B, 1, n1, wu, chunk16, lds_base + D_HALF);
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
        const Sweep st = block_stats(sweep<true>(lds, B, n1, t, lane, wu, chunk16, lds_base, aI, m1, m2, tbi,
                                                 ~((1u << tbi) - 1u), true),
                                     misc, w, lane);
        D_STAMP(2);
        if (!st.bad) {
            const double Bn = sqrt((double)st.b2max) * 1.0001;
            const double Eb = 8.0001 * (double)st.smax + 1e-30;  // exact power-of-two scaling
            // the window per maximiser column (its own 1 / q_j)
            epilogue<D_NW, true>(lds, rowv, m1, m2, Bn, Eb, false, tbi, ~((1u << tbi) - 1u), w, lane, row0, n0,
                                 n1, A, B, oidx, oscore, thresh, dmode, 1.0 / 508.0,
                                 !D_COLWIN ? nullptr : reinterpret_cast<const unsigned char *>(lds + D_OFF_COL),
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

int launch_allpairs_q8d_match(hipStream_t s, int batch, int cap, const int *n0, const int *n1, const float *desc0,
                              const float *desc1, double thresh, int *match_idx, float *match_score, int dmode) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    MV_REQUIRE((long)cap * KD * 4 < (1l << 32));  // 32-bit DMA source offsets within a pair
    const int tiles_r = (cap + D_BM - 1) / D_BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    MV_PROF_BEGIN(s, "k_q8d_match");
    hipLaunchKernelGGL(k_q8d_match, dim3((unsigned)blocks), dim3(D_NT), 0, s, tiles_r, cap, n0, n1, desc0, desc1,
                       dmode ? -1e300 : thresh, dmode, match_idx, match_score);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv

#ifdef MV_TRACE
extern "C" int mv_debug_direct_trace(void *host, long bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_d_trace), (size_t)bytes) == hipSuccess ? 0 : -3;
}
#endif
