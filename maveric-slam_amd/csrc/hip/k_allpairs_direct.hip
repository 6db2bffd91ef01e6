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
// the int8 tile ring: 64 rows (columns of frame 1) of 256 codes, row stride D_RS = 272 B (17
// chunks: the 16-lane phases of a ds_read_b128 hit distinct banks, and every B-fragment address is
// a per-lane base + a compile-time offset; round 3's 256-B rows with XOR-swizzled chunks needed
// per-read address VALU, 20 per tile and wave)
constexpr int D_RS = KD + 16;
constexpr int D_TILE = BN * D_RS, D_SLOT = D_TILE + BN * 4;        // + the tile's 64 per-column words
constexpr int D_OFF_RING = 3 * D_HALF;                              // 2 int8 tile slots
// [BM] float2 (|a|^2, s_a), past the int8 ring
constexpr int D_OFF_ROW = D_OFF_RING + 2 * D_SLOT;
constexpr int D_OFF_MISC = D_OFF_ROW + D_BM * 8;                    // [NW][4] per-wave statistics
constexpr int D_OFF_COL = D_OFF_MISC + D_NW * 16;  // integer path: each frame-1 column's key shift (1 B)
constexpr int D_NCOL = 64 * BN;           // the integer path's column limit (2 ntc <= 128)
constexpr int D_LDS = D_OFF_COL + D_NCOL;
constexpr int D_OFF_AIMG = 2 * D_HALF;  // A images: staging slot 2 + the ring (before the sweep)
static_assert(D_OFF_AIMG + D_NW * 32 * KD <= D_OFF_ROW, "A images fit staging slot 2 + the ring");
static_assert(epi_bytes<D_NW>() <= D_OFF_ROW, "the epilogue fits staging + ring");
static_assert(D_LDS <= 160 * 1024, "one workgroup per CU");
constexpr int D_PF = 1;       // k32 steps of B fragments read ahead of the MFMAs
constexpr int QS_LOAD = 1;    // the k32 step whose slot issues the quantisation's staging reads
// A phase: frame-0 row quads in flight per wave (4 x 16-B loads per lane each); fewer bytes in
// flight measured faster in both kernels (k_q8t_match 2: 3.505, 4: 3.54, 8: 3.91 ms --
// profiles/r05h_flag_qb_ab.json; k_q8d_match round 4: 2: 4.153-4.161, 4: 4.176-4.195 ms)
constexpr int D_QB = 2;
constexpr float IK_MMAX = 1.003f;  // integer path: max |b_jk| allowed (RNE(x 127) stays <= 127)
// (Measured and not kept, round 5: |b_j| bounded from the codes by v_dot4 and NaN caught by
// v_maximum3 instead of summing the fp32 squares -- 12 VALU per tile and wave fewer, but it failed
// tests/test_gpu_allpairs.py::test_allpairs_f32_out_of_screen_range.)

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
// the same with the keys built by compiler-visible instructions, for the first values folded after
// an MFMA chain's last instruction: the compiler pads the MFMA-result -> VALU hazard before its own
// instructions, not before an asm block (k_i8t_match's first pair per unit read stale registers)
__device__ __forceinline__ void fold_keys_cv(int a, int b, int sha, int shb, unsigned ta, unsigned tb, float &m1f,
                                             float &m2f) {
    const int ka = (int)(((unsigned)a << (sha & 31)) | ta), kb = (int)(((unsigned)b << (shb & 31)) | tb);
    int md, m1 = __float_as_int(m1f), m2 = __float_as_int(m2f);
    asm("v_med3_i32 %0, %1, %3, %4\n\t"
        "v_max3_i32 %1, %1, %3, %4\n\t"
        "v_max_i32 %2, %2, %0"
        : "=&v"(md), "+v"(m1), "+v"(m2)
        : "v"(ka), "v"(kb));
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
// GRP (k_q8t_match): one exponent e for each group of 4 consecutive columns (a wave's 4 rows of
// the half: the max of their m_j by two lane swaps), so that the transposed fold needs one key
// shift per group; the group's shift byte goes to the slot's shift table (byte D_TILE + 4 (2 jb +
// h) + q for group 8 jb + 2 q + h) -- the per-column words are not written.
template <bool IK, bool GRP = false>
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
    __device__ __forceinline__ void absmax() {
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
        qa = __builtin_fmaf(x0[0], x0[0], __builtin_fmaf(x0[1], x0[1], __builtin_fmaf(x0[2], x0[2], x0[3] * x0[3])));
        qb = __builtin_fmaf(x1[0], x1[0], __builtin_fmaf(x1[1], x1[1], __builtin_fmaf(x1[2], x1[2], x1[3] * x1[3])));
        qa = __builtin_fmaf(x2[0], x2[0], __builtin_fmaf(x2[1], x2[1], __builtin_fmaf(x2[2], x2[2], __builtin_fmaf(x2[3], x2[3], qa))));
        qb = __builtin_fmaf(x3[0], x3[0], __builtin_fmaf(x3[1], x3[1], __builtin_fmaf(x3[2], x3[2], __builtin_fmaf(x3[3], x3[3], qb))));
    }
    __device__ __forceinline__ void reduce(int j, int n1, int tb) {
        qa = qa + qb;
        row16_max_sum(m, qa);  // qa = |b|^2 from here on
        if constexpr (IK) {
            // e from m's biased exponent: [1/2, 2) -> 0, [1/4, 1/2) -> 1, below -> 2 (m q_e < 128)
            float mg = m;
            if constexpr (GRP) {  // the group's max: lanes 16 apart (ds_swizzle), then 32 apart
                mg = fmaxf(mg, swz_xor<16>(mg));
                mg = fmaxf(mg, __shfl_xor(mg, 32, 64));
            }
            const int e = min(max(126 - (int)((__float_as_uint(mg) >> 23) & 0xffu), 0), 2);
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
    }
    // cs: the tile's entries of the per-column key shifts kept for the epilogue (IK; live halves)
    __device__ __forceinline__ void store(char *rq, int hh, int t, bool live, float &smax, float &b2max, bool &bad,
                                          unsigned char *cs) {
        const int r = t >> 4, sub = t & 15, row = 32 * hh + r;
        *reinterpret_cast<i32x4 *>(rq + row * D_RS + (sub << 4)) = code;
        if constexpr (IK && GRP) {
            if ((t & 63) == 0) {  // the wave's group: 8 hh + w -> jb = hh, q = (w >> 1) & 3, h = w & 1
                const int w = t >> 6;
                rq[D_TILE + 4 * (2 * hh + (w & 1)) + ((w >> 1) & 3)] = (char)sh;
            }
            if (sub == 0 && live) cs[row] = (unsigned char)sh;
            bad = bad | (live & !((qa <= 1e30f) & (m <= IK_MMAX)));
        } else if constexpr (IK) {
            if (sub == 0) {
                reinterpret_cast<int *>(rq + D_TILE)[row] = sh;
                if (live) cs[row] = (unsigned char)sh;
            }
            bad = bad | (live & !((qa <= 1e30f) & (m <= IK_MMAX)));
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
    const int rdb = fr * D_RS + fh * 16;

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
                const int ch_ = 32 * s_;                                                     \
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

// row block L of the launch (pair L / tiles_r, rows 512 (L % tiles_r) ..)
__device__ __forceinline__ void q8d_block(char *lds, int L, int tiles_r, int cap, const int *__restrict__ n0v,
                                          const int *__restrict__ n1v, const float *__restrict__ desc0,
                                          const float *__restrict__ desc1, double thresh, int dmode,
                                          int *__restrict__ match_idx, float *__restrict__ match_score) {
#ifdef MV_TRACE
    unsigned long long ts_[10] = {};
    D_STAMP(0);
#endif
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
    a_phase<false, D_QB>(lds + D_OFF_AIMG + w * 32 * KD, rowv, w * 64, row0, n0, lane, A, nullptr, nullptr,
                         nullptr, false, aI);
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
                                 reinterpret_cast<const unsigned char *>(lds + D_OFF_COL));
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


__global__ __launch_bounds__(D_NT, 2) void k_q8d_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                       const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                       const float *__restrict__ desc1, double thresh, int dmode,
                                                       int *__restrict__ match_idx, float *__restrict__ match_score) {
    __shared__ __attribute__((aligned(16))) char lds[D_LDS];
    q8d_block(lds, xcd_remap(blockIdx.x, gridDim.x), tiles_r, cap, n0v, n1v, desc0, desc1, thresh, dmode, match_idx,
              match_score);
}
// the pairs k_q8t_match handed back (flags `only`), a grid-stride loop over the row blocks: a
// few workgroups scan the flags instead of one exiting workgroup per row block
__global__ __launch_bounds__(D_NT, 2) void k_q8d_handback(int tiles_r, int cap, const int *__restrict__ n0v,
                                                          const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                          const float *__restrict__ desc1, double thresh,
                                                          int *__restrict__ match_idx, float *__restrict__ match_score,
                                                          const int *__restrict__ only, int nblocks) {
    __shared__ __attribute__((aligned(16))) char lds[D_LDS];
    // the flag scan first, in scalar registers: a workgroup with nothing handed back leaves before
    // any of the (spilling) float-path code runs
    int L = blockIdx.x;
    while (L < nblocks && !__builtin_amdgcn_readfirstlane(only[L / tiles_r])) L += gridDim.x;
    for (; L < nblocks; L += gridDim.x) {
        if (!__builtin_amdgcn_readfirstlane(only[L / tiles_r])) continue;  // uniform: one flag per block
        q8d_block(lds, L, tiles_r, cap, n0v, n1v, desc0, desc1, thresh, 0, match_idx, match_score);
        __syncthreads();  // the next row block reuses the LDS
    }
}

// =============================================================================================
// k_q8t_match -- ONE workgroup per pair (cap <= 1024): frame 1 quantised ONCE per pair.
// k_q8d_match's two 512-row workgroups each quantise the whole of frame 1 (~190 of its ~350 VALU
// per tile and wave).  Here 8 waves own 128 query rows each, which the 256-register budget holds
// only in the TRANSPOSED product: the frame-1 tile is the MFMA A operand (32 columns j x 32 k,
// read from the int8 ring) and the wave's frame-0 codes the B operand (aI, 4 groups x 8 k32 steps
// = 128 VGPRs), so D[j][i] leaves each lane ONE query row i = 32 g + (lane & 31) and 16 columns
// j = 8 (r >> 2) + (r & 3) + 4 (lane >> 5) -- the lane-local top-2 is 2 registers per group
// instead of 32.  Keys: (D << (tb + 2 - e)) | tag with the tag (2 tc + jb) 16 + r (the column up to
// the lane half, which the lane itself is) in an SGPR and the shift in a VGPR, one shift per group
// of 4 consecutive columns (QHalf<true, true>: e uniform over the group, so the 4 shifts of a lane
// and column block come from one LDS dword).  Per tile and wave: 8 units (jb, g) of 8 MFMAs,
// every unit folding the previous unit's 16 values (5 VALU per 2 values) beside its MFMAs and
// reading its fragments from LDS one k32 step ahead; the next tile's quantisation in 7 stages over
// units 0..3 (half A) and 4..7 (half B).
// Range: a pair whose frame 1 leaves the integer keys' range (a value outside +-1.003, a
// non-finite value, |b_j|^2 > 4 -- keys then need more than 31 bits at tb = 9) is marked in
// `fallback` and redone by k_q8d_match (its float path), launched after this kernel with the flags.
constexpr int T_RG = 4;                             // 32-row groups per wave: 128 query rows
constexpr int T_BM = 32 * T_RG * D_NW;              // 1024 rows: the whole pair
constexpr int T_OFF_ROW = D_OFF_RING + 2 * D_SLOT;  // [T_BM] float2 (|a|^2, s_a)
constexpr int T_OFF_MISC = T_OFF_ROW + T_BM * 8;    // [NW][4] per-wave statistics
constexpr int T_OFF_COL = T_OFF_MISC + D_NW * 16;   // each frame-1 column's key shift (1 B)
constexpr int T_LDS = T_OFF_COL + T_BM;
constexpr int T_EPI_MASK = D_NW * 8192;             // epilogue: [NW] 8-KiB re-score buffers, [T_BM] wide masks
static_assert(T_EPI_MASK + T_BM * 4 <= T_OFF_ROW, "the epilogue fits staging + ring");
constexpr unsigned T_RESCAN = 0x80000000u;  // wide-mask bit: the row is left to k_q8t_rescan
// a row left to k_q8t_rescan: its match index holds INT_MIN + lim + 2^28 (< -1, never an index),
// lim = the window's low end in key units, rounded up and clamped to +-2^28 (clamping only widens)
constexpr int T_LIM_BIAS = 1 << 28;
__device__ __forceinline__ int rs_encode(int lim) {
    return (int)(0x80000000u + (unsigned)(min(max(lim, -T_LIM_BIAS), T_LIM_BIAS) + T_LIM_BIAS));
}
__device__ __forceinline__ int rs_decode(int v) { return (int)((unsigned)v - 0x80000000u) - T_LIM_BIAS; }
static_assert(D_OFF_AIMG + D_NW * 32 * KD <= T_OFF_ROW, "A images fit staging slot 2 + the ring");
static_assert(T_LDS <= 160 * 1024, "one workgroup per CU");
constexpr float T_B2MAX = 4.f;  // |b_j|^2 bound of the keys' range at tb <= 9
constexpr int T_PFD = 2;  // k32 steps the frame-1 fragments are read ahead of their MFMA (1: 3.66 ms, 2: 3.53, 3: 3.52 -- profiles/r05g_pfd_ab.json)

__device__ __forceinline__ Sweep sweep_t(char *lds, const float *B, int n1, int t, int lane, int wu, unsigned chunk16,
                                         unsigned lds_base, const i32x4 (&aI)[T_RG][KD / 32], float (&m1)[T_RG],
                                         float (&m2)[T_RG], int tb) {
    const int ntc = (n1 + BN - 1) / BN, nh = 2 * ntc;
    const int fr = lane & 31, fh = lane >> 5;
    char *ring = lds + D_OFF_RING;
    unsigned char *colsh = reinterpret_cast<unsigned char *>(lds + T_OFF_COL);
    Sweep st = {0.f, 0.f, false};
    if (nh > 2) {
        dma_half(B, 2, n1, wu, chunk16, lds_base + 2 * D_HALF);
        wait_vm<4>();
    } else {
        wait_vm<0>();
    }
    __syncthreads();  // halves 0, 1 landed
    {
        QHalf<true, true> h;
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

    const int rdb = fr * D_RS + fh * 16;  // frame-1 fragment: ring row 32 jb + fr, k chunk 2 s + fh
    const float kinit = __int_as_float((int)0x80000000);
#pragma unroll
    for (int g = 0; g < T_RG; g++) {
        m1[g] = kinit;
        m2[g] = kinit;
    }
    i32x16 acc[2];
#pragma unroll
    for (int q = 0; q < 16; q++) {  // the unit before tile 0: folded, then discarded
        acc[0][q] = 0;
        acc[1][q] = 0;
    }
    int sv0[4] = {0, 0, 0, 0}, sv1[4] = {0, 0, 0, 0};  // key shifts of groups q of column block 0 / 1
    QHalf<true, true> qh;

    // unit U of the tile: column block jb = U >> 2, row group g = U & 3: 8 MFMAs into acc[U & 1],
    // each beside the fold of 2 of the previous unit's 16 values (acc[(U + 1) & 1], row group
    // (U + 3) & 3, shifts PSV, tags PT + r), and quantisation stages 2 (U & 3), 2 (U & 3) + 1 at
    // k32 steps 0 and 4; the fragments read T_PFD k32 steps ahead across the tile's units (fb_: the
    // tile's 64 k32 steps, constant indices: only the T_PFD + 1 live ones take registers)
#define T_UNIT(U, PSV, PT, STG, HH, J0, LIVE)                                                 \
    do {                                                                                     \
        _Pragma("unroll") for (int s_ = 0; s_ < KD / 32; s_++) {                             \
            if (s_ == 0 || s_ == 4) {                                                        \
                const int k_ = 2 * ((U) & 3) + (s_ != 0);                                    \
                if (k_ == 0) qh.load((STG), t);                                              \
                else if (k_ == 1) qh.absmax();                                               \
                else if (k_ == 2) qh.sumsq();                                                \
                else if (k_ == 3) qh.reduce((J0) + (t >> 4), n1, tb);                        \
                else if (k_ == 4) qh.pack01();                                               \
                else if (k_ == 5) qh.pack23();                                               \
                else if (k_ == 6) qh.store(rq, (HH), t, (LIVE), st.smax, st.b2max, st.bad, colsh + (tc + 1) * BN); \
            }                                                                                \
            const int gn_ = 8 * (U) + s_ + T_PFD;                                            \
            if (gn_ < 64) fb_[gn_] = *reinterpret_cast<const i32x4 *>(rs + rdb + (gn_ >> 5) * 32 * D_RS + 32 * (gn_ & 7)); \
            if (s_ == 0) {                                                                   \
                const i32x16 z_ = {};                                                        \
                acc[(U) & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb_[8 * (U)], aI[(U) & 3][0], z_, 0, 0, 0); \
            } else {                                                                         \
                acc[(U) & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb_[8 * (U) + s_], aI[(U) & 3][s_], acc[(U) & 1], 0, 0, 0); \
            }                                                                                \
            if (s_ == 0)                                                                     \
                fold_keys_cv(acc[((U) + 1) & 1][0], acc[((U) + 1) & 1][1], PSV[0], PSV[0], (PT), (PT) + 1u, \
                             m1[((U) + 3) & 3], m2[((U) + 3) & 3]);                          \
            else                                                                             \
                fold_keys(acc[((U) + 1) & 1][2 * s_], acc[((U) + 1) & 1][2 * s_ + 1], PSV[s_ >> 1], PSV[s_ >> 1], \
                          (PT) + 2u * s_, (PT) + 2u * s_ + 1u, m1[((U) + 3) & 3], m2[((U) + 3) & 3]); \
            __builtin_amdgcn_sched_barrier(0);                                               \
        }                                                                                    \
    } while (0)

    int sA = 2, sB = 0;  // staging slots of halves 2t + 2, 2t + 3
    for (int tc = 0; tc < ntc; tc++) {
        if (2 * tc + 3 < nh) {  // half 2t + 2 landed (2t + 3 may be in flight)
            wait_vm<4>();
        } else {
            wait_vm<0>();
        }
        D_SYNC();  // tile t complete in its slot; the slot of tile t - 1 and staging of half 2t + 1 free
        i32x4 fb_[64];
        _Pragma("unroll") for (int p_ = 0; p_ < T_PFD; p_++)
            fb_[p_] = *reinterpret_cast<const i32x4 *>(ring + (tc & 1) * D_SLOT + rdb + 32 * p_);
        const int sN = 3 - sA - sB;
        if (2 * tc + 4 < nh) dma_half(B, 2 * tc + 4, n1, wu, chunk16, lds_base + (unsigned)(sN * D_HALF));
        const char *rs = ring + (tc & 1) * D_SLOT;
        char *rq = ring + ((tc + 1) & 1) * D_SLOT;
        const char *stA = lds + sA * D_HALF, *stB = lds + sB * D_HALF;
        const bool live = tc + 1 < ntc;
        const unsigned tg0 = __builtin_amdgcn_readfirstlane(32u * (unsigned)tc);  // (2 tc + jb) 16
        const unsigned tgp = tg0 - 16u;                                           // tile tc - 1, jb 1
        const unsigned tg1 = tg0 + 16u;
        {
            const unsigned d_ = *reinterpret_cast<const unsigned *>(rs + D_TILE + 4 * fh);
            sv0[0] = (int)d_;
            sv0[1] = (int)(d_ >> 8);
            sv0[2] = (int)(d_ >> 16);
            sv0[3] = (int)(d_ >> 24);
        }
        T_UNIT(0, sv1, tgp, stA, 0, 32 * (2 * tc + 2), live);
        if (tc == 0) {  // unit 0 of tile 0 folded the zeros of "unit -1"
            m1[3] = kinit;
            m2[3] = kinit;
        }
        T_UNIT(1, sv0, tg0, stA, 0, 32 * (2 * tc + 2), live);
        T_UNIT(2, sv0, tg0, stA, 0, 32 * (2 * tc + 2), live);
        T_UNIT(3, sv0, tg0, stA, 0, 32 * (2 * tc + 2), live);
        if (2 * tc + 4 < nh) {  // half 2t + 3 landed (2t + 4 may be in flight)
            wait_vm<4>();
        } else {
            wait_vm<0>();
        }
        // half 2t + 2's staging rows were read by this wave's own load stage: free for 2t + 5
        if (2 * tc + 5 < nh) dma_half(B, 2 * tc + 5, n1, wu, chunk16, lds_base + (unsigned)(sA * D_HALF));
        {
            const unsigned d_ = *reinterpret_cast<const unsigned *>(rs + D_TILE + 4 * (2 + fh));
            sv1[0] = (int)d_;
            sv1[1] = (int)(d_ >> 8);
            sv1[2] = (int)(d_ >> 16);
            sv1[3] = (int)(d_ >> 24);
        }
        T_UNIT(4, sv0, tg0, stB, 1, 32 * (2 * tc + 3), live);
        T_UNIT(5, sv1, tg1, stB, 1, 32 * (2 * tc + 3), live);
        T_UNIT(6, sv1, tg1, stB, 1, 32 * (2 * tc + 3), live);
        T_UNIT(7, sv1, tg1, stB, 1, 32 * (2 * tc + 3), live);
        const int nA = sN, nB = sA;
        sA = nA;
        sB = nB;
    }
#undef T_UNIT
    {  // unit 7 of the last tile
        const unsigned tl = __builtin_amdgcn_readfirstlane(32u * (unsigned)(ntc - 1) + 16u);
        // the first pair by compiler-visible instructions: the MFMA-result hazard is padded before
        // them (an asm block right after the chain's last MFMA would read stale registers)
        fold_keys_cv(acc[1][0], acc[1][1], sv1[0], sv1[0], tl, tl + 1u, m1[3], m2[3]);
#pragma unroll
        for (int m_ = 1; m_ < KD / 32; m_++)
            fold_keys(acc[1][2 * m_], acc[1][2 * m_ + 1], sv1[m_ >> 1], sv1[m_ >> 1], tl + 2u * m_, tl + 2u * m_ + 1u,
                      m1[3], m2[3]);
    }
    return st;
}

// The transposed layout's decisions (the IK window of q8_common.hpp's epilogue, dmode 0): row
// i = 32 g + fr of the wave sits in lanes fr (columns with (j >> 2) & 1 = 0) and fr + 32 (= 1), each
// with its half's (m1, m2).  Runner-up outside the window: the maximiser, exactly scored only when
// the window straddles the threshold (or scores are asked for) -- deferred, cooperatively loaded
// (coop_exact_dots) two groups at a time; inside: each half's m1 is a candidate when inside, and a
// half whose m2 is inside may hide more -- the wave re-scores every column of such "wide" halves.
__device__ __forceinline__ unsigned epilogue_t(char *epi, const float2 *rowv, const float (&m1)[T_RG],
                                           const float (&m2)[T_RG], double Bn, double Eb, int tb, int w, int lane,
                                           int n0, int n1, const float *__restrict__ A, const float *__restrict__ B,
                                           int *__restrict__ oidx, float *__restrict__ oscore, double thresh,
                                           const unsigned char *colsh, int *rs_flag, unsigned char *rs_colsh) {
    const int fr = lane & 31, fh = lane >> 5;
    const double u24 = 5.9604644775390625e-08;
    const double gam_e = KD * u24 / (1.0 - KD * u24);
    const unsigned tmask = (1u << tb) - 1u;
    auto kv = [&](float a) { return (double)(__float_as_int(a) >> tb); };
    auto kcol = [&](float a, int h) {  // the column of key a held by lane half h
        const unsigned tg = __float_as_uint(a) & tmask;
        return (int)(tg >> 4) * 32 + 8 * (int)((tg >> 2) & 3u) + (int)(tg & 3u) + 4 * h;
    };
    unsigned *lmask = reinterpret_cast<unsigned *>(epi + T_EPI_MASK);
    char *cbuf = epi + w * 8192;
    float bs_g[T_RG];
    int bj_g[T_RG], need_g[T_RG];
    bool out_g[T_RG];
    unsigned wide_rows[T_RG];
#pragma unroll
    for (int g = 0; g < T_RG; g++) {
        const float e1 = m1[g], e2 = m2[g];
        const float o1 = __shfl_xor(e1, 32, 64), o2 = __shfl_xor(e2, 32, 64);
        const int i1 = __float_as_int(e1), j1 = __float_as_int(o1);
        const float M = i1 >= j1 ? e1 : o1;                 // equal keys: M2 = M, ambiguous
        const int Mh = i1 > j1 ? fh : (j1 > i1 ? 1 - fh : 0);
        const float lo1 = i1 >= j1 ? o1 : e1;
        const float M2 = __int_as_float(max(max(__float_as_int(e2), __float_as_int(o2)), __float_as_int(lo1)));
        const int rl = w * (32 * T_RG) + g * 32 + fr;
        const bool live = rl < n0;
        const float2 rv = rowv[rl];
        float bs = -__builtin_inff();
        int bj = 0x7fffffff, need = -1;
        bool wide = live && rv.y < 0.f;  // a row outside the int8 range: every column
        bool rescan = false;             // wide, re-screened (rescan_t) against limit lim_k
        int lim_k = 0;
        unsigned wm = 3u;
        if (live && !(rv.y < 0.f)) {
            const double s_a = (double)rv.y;
            const double an = sqrt(fmax((double)rv.x, 0.0)) * 1.0001;
            const double ea = 8.001 * s_a + 4.76837158203125e-07 * an;
            const double dq = (an * Eb + ea * Bn + ea * Eb) * 1.0001;
            const double delta = dq + u24 * (an * Bn + dq) * 1.01 + gam_e * an * Bn + 1e-30;
            const double sa_k = s_a * (1.0 / 508.0);
            const double Ms = kv(M) * sa_k;
            const double M2s = __float_as_int(M2) != (int)0x80000000 ? kv(M2) * sa_k : -__builtin_inf();
            const double dp = delta;
            double dpI = dp;  // the maximiser's own column window (its 1 / q_I)
            const int I = kcol(M, Mh);
            if (I < n1) {
                const int eI = tb + 2 - (int)colsh[I];
                const double EbI = 8.0001 * (double)__builtin_ldexpf(1.f / 127.f, -eI) + 1e-30;
                const double dqI = (an * EbI + ea * Bn + ea * EbI) * 1.0001;
                dpI = fmin(dp, dqI + u24 * (an * Bn + dqI) * 1.01 + gam_e * an * Bn + 1e-30);
            }
            const double lo = Ms - dpI - dp;
            if (Ms + dpI > thresh || M2s + dp > thresh) {
                if (M2s < lo) {
                    if (I >= n1) {  // a padding column (zero codes) on top: all real dots below 0
                        wide = true;
                    } else if (!oscore && Ms - dpI > fmax(thresh, 0.0)) {
                        bs = FLT_MAX;  // sure: the maximiser clears the threshold, no dot needed
                        bj = I;
                    } else {
                        need = I;
                    }
                } else {  // both lanes of the row take this branch
                    const double lim = lo / sa_k;
                    const bool in1 = kv(e1) >= lim, in2 = kv(e2) >= lim;
                    const bool oin1 = __shfl_xor(in1 ? 1 : 0, 32, 64) != 0;
                    const bool oin2 = __shfl_xor(in2 ? 1 : 0, 32, 64) != 0;
                    if (in2 || oin2) {  // a half holds two columns inside: re-screen the row
                        wide = true;
                        rescan = true;
                        lim_k = (int)fmin(fmax(ceil(lim), -2147483647.0), 2147483647.0);
                        wm = (in1 ? 1u << fh : 0u) | (oin1 ? 1u << (1 - fh) : 0u);
                    } else if (in1) {
                        const int j = kcol(e1, fh);
                        if ((unsigned)j < (unsigned)n1) {
                            const float *ap = A + (size_t)rl * KD;
                            asm volatile("" : "+v"(ap));
                            bs = exact_dot(ap, B + (size_t)j * KD);
                            bj = j;
                        }
                    }
                }
            }
        }
        {  // the row's two lanes: the better exact candidate (ambiguous rows)
            const float ob = __shfl_xor(bs, 32, 64);
            const int oj = __shfl_xor(bj, 32, 64);
            if (better(0, ob, oj, bs, bj)) {
                bs = ob;
                bj = oj;
            }
        }
        bs_g[g] = bs;
        bj_g[g] = bj;
        need_g[g] = need;
        out_g[g] = fh == 0 && live && !wide;
        if (fh == 0 && wide) lmask[rl] = rescan ? T_RESCAN : wm;
        if (fh == 0 && rescan) oidx[rl] = rs_encode(lim_k);  // k_q8t_rescan's work
        wide_rows[g] = (unsigned)__ballot(fh == 0 && wide);
    }
    unsigned nwide = 0, nneed = 0;  // (traced builds) the wave's wide rows and deferred dots
    bool rescan_any = false;
#pragma unroll
    for (int g = 0; g < T_RG; g++) {
        nwide += __popc(wide_rows[g]);
        nneed += __popcll(__ballot(need_g[g] >= 0));
    }
    // the deferred maximiser scores, two groups per call: lane (fr, fh) takes row fr of group 2 c + fh
#pragma unroll
    for (int c = 0; c < T_RG / 2; c++) {
        const int Ih = fh ? need_g[2 * c + 1] : need_g[2 * c];
        float e = 0.f;
        if (__ballot(Ih >= 0))
            e = coop_exact_dots(A, B, w * (32 * T_RG) + (2 * c + fh) * 32 + fr, Ih, lane, cbuf);
        const float eo = __shfl_xor(e, 32, 64);
        const float e0 = fh ? eo : e, e1 = fh ? e : eo;
        if (need_g[2 * c] >= 0) {
            bs_g[2 * c] = e0;
            bj_g[2 * c] = need_g[2 * c];
        }
        if (need_g[2 * c + 1] >= 0) {
            bs_g[2 * c + 1] = e1;
            bj_g[2 * c + 1] = need_g[2 * c + 1];
        }
    }
#pragma unroll
    for (int g = 0; g < T_RG; g++)
        if (out_g[g]) {
            const int rl = w * (32 * T_RG) + g * 32 + fr;
            const bool keep = bj_g[g] != 0x7fffffff && (double)bs_g[g] > thresh && bs_g[g] > 0.f;
            oidx[rl] = keep ? bj_g[g] : -1;
            if (oscore) oscore[rl] = keep ? bs_g[g] : 0.f;
        }
    // wide rows left here (rows outside the int8 range, a padding column on top; with
    // round 5's first form every wide row): every column of the listed halves, one column per lane
#pragma unroll
    for (int g = 0; g < T_RG; g++)
        for (unsigned dm = wide_rows[g]; dm; dm &= dm - 1) {
            const int r = w * (32 * T_RG) + g * 32 + __builtin_ctz(dm);
            const unsigned wm = lmask[r];
            if (wm & T_RESCAN) {  // k_q8t_rescan's: the pair's column shifts and tag width for it
                rescan_any = true;
                continue;
            }
            const float *a = A + (size_t)r * KD;
            float ws = -__builtin_inff();
            int wj = 0x7fffffff;
            for (int j = lane; j < n1; j += 64) {
                if (!((wm >> ((j >> 2) & 1)) & 1u)) continue;
                const float *ap = a;
                asm volatile("" : "+v"(ap));
                const float e = exact_dot(ap, B + (size_t)j * KD);
                if (better(0, e, j, ws, wj)) {
                    ws = e;
                    wj = j;
                }
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float ob = __shfl_xor(ws, o, 64);
                const int oj = __shfl_xor(wj, o, 64);
                if (better(0, ob, oj, ws, wj)) {
                    ws = ob;
                    wj = oj;
                }
            }
            if (lane == 0) {
                const bool keep = wj != 0x7fffffff && (double)ws > thresh && ws > 0.f;
                oidx[r] = keep ? wj : -1;
                if (oscore) oscore[r] = keep ? ws : 0.f;
            }
        }
    if (rescan_any) {  // wave-uniform; every such wave writes the same bytes
        const i32x4 v = *reinterpret_cast<const i32x4 *>(colsh + 16 * lane);
        *reinterpret_cast<i32x4 *>(rs_colsh + 16 * lane) = v;
        if (lane == 0) *rs_flag = tb + 1;
    }
    return nwide << 16 | nneed;
}

__global__ __launch_bounds__(D_NT, 2) void k_q8t_match(int cap, const int *__restrict__ n0v,
                                                       const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                       const float *__restrict__ desc1, double thresh,
                                                       int *__restrict__ match_idx, float *__restrict__ match_score,
                                                       int *__restrict__ fallback, int *__restrict__ rs_flags,
                                                       unsigned char *__restrict__ rs_colsh) {
    __shared__ __attribute__((aligned(16))) char lds[T_LDS];
#ifdef MV_TRACE
    unsigned long long ts_[10] = {};
    D_STAMP(0);
#endif
    const int pair = blockIdx.x;
    const int n0 = min(max(n0v[pair], 0), cap), n1 = min(max(n1v[pair], 0), cap);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int *oidx = match_idx + (size_t)pair * cap;
    float *oscore = match_score ? match_score + (size_t)pair * cap : nullptr;  // null: indices only
    for (int r = t; r < cap; r += D_NT)
        if (r >= n0 || n1 <= 0) {  // rows in [n0, cap): no match
            oidx[r] = -1;
            if (oscore) oscore[r] = 0.f;
        }
    if (n0 <= 0 || n1 <= 0) return;
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;
    const int ntc = (n1 + BN - 1) / BN;
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const unsigned chunk16 = (unsigned)(4 * (lane & 15) + (lane >> 4)) * 16;
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    float2 *rowv = reinterpret_cast<float2 *>(lds + T_OFF_ROW);
    float *misc = reinterpret_cast<float *>(lds + T_OFF_MISC);
    // ---- prologue: halves 0, 1 in flight beside the A phase (128 rows per wave) ----
    dma_half(B, 0, n1, wu, chunk16, lds_base);
    dma_half(B, 1, n1, wu, chunk16, lds_base + D_HALF);
    i32x4 aI[T_RG][KD / 32];
    // the A rows' loads software-pipelined (batch b + 1 issued before batch b is quantised): 3.504-3.514
    // against 3.527-3.541 ms per launch, same box, ABAB (profiles/r06d_apipe_ab.log)
    a_phase_pipe<D_QB, T_RG>(lds + D_OFF_AIMG + w * 32 * KD, rowv, w * (32 * T_RG), 0, n0, lane, A, aI);
    D_STAMP(1);
    __syncthreads();  // the A images (staging slot 2 + the ring) are consumed
    float m1[T_RG], m2[T_RG];
    const int tb = 32 - __builtin_clz(32 * ntc - 1);  // tags (2 tc + jb) 16 + r < 32 ntc
    const Sweep st = block_stats(sweep_t(lds, B, n1, t, lane, wu, chunk16, lds_base, aI, m1, m2, tb), misc, w, lane);
    D_STAMP(2);
    if (st.bad || !(st.b2max <= T_B2MAX)) {  // outside the keys' range: k_q8d_match redoes the pair
        if (t == 0) fallback[pair] = 1;
        return;
    }
    const double Bn = sqrt((double)st.b2max) * 1.0001;
    const double Eb = 8.0001 * (double)st.smax + 1e-30;
    const unsigned ecnt = epilogue_t(lds, rowv, m1, m2, Bn, Eb, tb, w, lane, n0, n1, A, B, oidx, oscore, thresh,
                                     reinterpret_cast<const unsigned char *>(lds + T_OFF_COL), rs_flags + pair,
                                     rs_colsh + (size_t)pair * T_BM);
    (void)ecnt;
#ifdef MV_TRACE
    D_STAMP(3);
    ts_[8] = ecnt;
    if (lane == 0 && blockIdx.x < D_TRACE_BLOCKS) {
        unsigned long long *o = g_d_trace + ((size_t)blockIdx.x * D_NW + w) * 10;
        for (int k = 0; k < 6; k++) o[k] = ts_[k];  // memtime x 4, memrealtime at entry / after A
        o[6] = __smid();
        o[7] = __builtin_amdgcn_s_memrealtime();
        o[8] = ts_[8];
        o[9] = ts_[9];
    }
#endif
}

// ---------------------------------------------------------------------------
// k_q8t_rescan: the wide rows k_q8t_match leaves (a lane half holding two columns inside the
// window: more may hide below its runner-up, and a row's two lanes keep only their halves' top 2).
// Scoring every column of such a half exactly -- n1 / 2 sequential 256-term dots per row -- was
// what SuperPoint's own descriptors made expensive: 15.8 wide rows per 394-keypoint pair (4 %),
// the epilogue's p90 at 487 k cycles per wave against a 55 k sweep (profiles/r05d_wide_rows.json).
// Instead each row is re-screened: a workgroup of 4 waves takes a flagged pair's pending rows 32 at
// a time (each wave every 4th 32-column block of frame 1; their bests merged in LDS), rebuilds their codes exactly as the A phase made them (same m, q, pack4: the same
// integers) as the MFMA B operand, and per 32-column block of frame 1 rebuilds the codes as the
// sweep made them (q_j = 127 * 2^e_j from the column's key shift, which k_q8t_match exported with
// the tag width) through an 8-KiB LDS buffer; 8 MFMAs give the block's exact screen D_ij, and
// every column whose key D << (2 - e_j) reaches the row's limit (the window's low end: the same
// test k_q8t_match applies to its candidates) is listed -- a superset of the columns that can beat
// the maximiser.  Listed columns are scored exactly (coop_exact_dots) whenever some lane's list
// could overflow in the next block, and at the end.  A separate kernel so that k_q8t_match keeps
// its registers (the in-kernel form pushed it from 240 VGPRs to 256 + 4 spilled: 0.6-3 % on the
// headline, profiles/r05e_rescreen_inkernel_ab.json).
// ---------------------------------------------------------------------------
constexpr int RS_CAP = 32;  // listed columns per (row, lane half) between exact-score rounds
constexpr int RS_CF = 8;    // frame-1 columns in flight per lane
constexpr int RS_NW = 4;    // waves per workgroup: column blocks w, w + 4, ... of the same rows

__global__ __launch_bounds__(64 * RS_NW) void k_q8t_rescan(int batch, int cap, const int *__restrict__ n1v,
                                                           const float *__restrict__ desc0,
                                                           const float *__restrict__ desc1, double thresh,
                                                           int *__restrict__ match_idx, float *__restrict__ match_score,
                                                           const int *__restrict__ rs_flags,
                                                           const unsigned char *__restrict__ rs_colsh) {
    __shared__ __attribute__((aligned(16))) char bufs[RS_NW][32 * KD];  // per wave: row image / column stage / dots
    __shared__ int cls[RS_NW][64 * RS_CAP];                              // per wave: [row fr][half fh] listed columns
    __shared__ int slotss[RS_NW][32], limss[RS_NW][32];                  // per wave: the batch (identical copies)
    __shared__ float red_s[RS_NW][32];
    __shared__ int red_j[RS_NW][32];
    __shared__ __attribute__((aligned(16))) unsigned char colsh[T_BM];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int fr = lane & 31, fh = lane >> 5, sub = lane & 15, rq = lane >> 4;
    char *buf = bufs[w];
    int *mycl = cls[w] + (fh * 32 + fr) * RS_CAP;
    int *slots = slotss[w], *lims = limss[w];
    for (int pair = blockIdx.x; pair < batch; pair += gridDim.x) {
        const int fl = __builtin_amdgcn_readfirstlane(rs_flags[pair]);
        if (!fl) continue;  // uniform over the workgroup
        const int tb = fl - 1;
        const int n1 = min(max(n1v[pair], 0), cap);
        const float *A = desc0 + (size_t)pair * cap * KD;
        const float *B = desc1 + (size_t)pair * cap * KD;
        int *oidx = match_idx + (size_t)pair * cap;
        float *oscore = match_score ? match_score + (size_t)pair * cap : nullptr;
        __syncthreads();  // the previous pair's colsh / red reads done
        if (w == 0)
            *reinterpret_cast<i32x4 *>(colsh + 16 * lane) =
                *reinterpret_cast<const i32x4 *>(rs_colsh + (size_t)pair * T_BM + 16 * lane);
        __syncthreads();
        const int nblk = (n1 + 31) / 32;
        // one batch of ns pending rows (slots / lims): every wave, its share of the column blocks
        auto run_batch = [&](int ns) {
            // the rows' codes as the A phase made them: 16 lanes per row, 4 rows per pass
#pragma unroll 2
            for (int qd = 0; qd < 8; qd++) {
                const int sl = 4 * qd + rq;
                const float *ar = A + (size_t)slots[min(sl, ns - 1)] * KD;
                f32x4v x[4];
#pragma unroll
                for (int u = 0; u < 4; u++) x[u] = *reinterpret_cast<const f32x4v *>(ar + 4 * (sub + 16 * u));
                float m = 0.f;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    m = absmax3(m, x[u][0], x[u][1]);
                    m = absmax3(m, x[u][2], x[u][3]);
                }
                m = fmaxf(m, swz_xor<1>(m));
                m = fmaxf(m, swz_xor<2>(m));
                m = fmaxf(m, swz_xor<4>(m));
                m = fmaxf(m, swz_xor<8>(m));
                const float q = m > 0.f ? 127.f * __builtin_amdgcn_rcpf(m) : 0.f;
                char *rowp = buf + sl * KD + 4 * (sub & 3);
#pragma unroll
                for (int u = 0; u < 4; u++)
                    *reinterpret_cast<int *>(rowp + ((((sub >> 2) + 4 * u) ^ (sl & 15)) << 4)) =
                        pack4(x[u][0], x[u][1], x[u][2], x[u][3], q);
            }
            i32x4 aF[KD / 32];
#pragma unroll
            for (int s2 = 0; s2 < KD / 32; s2++)
                aF[s2] = *reinterpret_cast<const i32x4 *>(buf + fr * KD + (((2 * s2 + fh) ^ (fr & 15)) << 4));
            const bool mine = fr < ns;
            const int myrow = slots[min(fr, ns - 1)];
            const int lim = lims[min(fr, ns - 1)];
            int cnt = 0;
            float bs = -__builtin_inff();
            int bj = 0x7fffffff;
            auto flush = [&]() {  // exact scores of the listed columns, one list position per round
                for (int k = 0; __ballot(k < cnt); k++) {
                    const int j = k < cnt ? mycl[k] : -1;
                    const float e = coop_exact_dots(A, B, myrow, j, lane, buf);
                    if (j >= 0 && better(0, e, j, bs, bj)) {
                        bs = e;
                        bj = j;
                    }
                }
                cnt = 0;
            };
            for (int blk = w; blk < nblk; blk += RS_NW) {
                // columns 32 blk + c as the sweep quantised them: one 1-KiB column per load
                // instruction (lane l: floats 4 l .. +3)
#pragma unroll
                for (int c0 = 0; c0 < 32; c0 += RS_CF) {
                    f32x4v x[RS_CF];
#pragma unroll
                    for (int i = 0; i < RS_CF; i++) {
                        const int j = min(32 * blk + c0 + i, n1 - 1);
                        x[i] = *reinterpret_cast<const f32x4v *>(B + (size_t)j * KD + 4 * lane);
                    }
#pragma unroll
                    for (int i = 0; i < RS_CF; i++) {
                        const int c = c0 + i, j = 32 * blk + c;
                        const float qc = j < n1 ? __builtin_ldexpf(127.f, tb + 2 - (int)colsh[j]) : 0.f;
                        *reinterpret_cast<int *>(buf + c * KD + (((lane >> 2) ^ (c & 15)) << 4) + 4 * (lane & 3)) =
                            pack4(x[i][0], x[i][1], x[i][2], x[i][3], qc);
                    }
                }
                i32x4 bF[KD / 32];
#pragma unroll
                for (int s2 = 0; s2 < KD / 32; s2++)
                    bF[s2] = *reinterpret_cast<const i32x4 *>(buf + fr * KD + (((2 * s2 + fh) ^ (fr & 15)) << 4));
                const i32x16 z = {};
                i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(bF[0], aF[0], z, 0, 0, 0);
#pragma unroll
                for (int s2 = 1; s2 < KD / 32; s2++)
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(bF[s2], aF[s2], acc, 0, 0, 0);
                if (mine) {
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) {
                        const int jq = 32 * blk + 8 * qq + 4 * fh;  // a 4-column group: one key shift
                        const int d = jq < n1 ? (int)colsh[jq] - tb : 0;
#pragma unroll
                        for (int e = 0; e < 4; e++) {
                            const int j = jq + e;
                            if (j < n1 && acc[4 * qq + e] * (1 << d) >= lim) mycl[cnt++] = j;
                        }
                    }
                }
                if (__ballot(cnt > RS_CAP - 16)) flush();  // the next block adds at most 16
            }
            flush();
            const float ob = __shfl_xor(bs, 32, 64);
            const int oj = __shfl_xor(bj, 32, 64);
            if (better(0, ob, oj, bs, bj)) {
                bs = ob;
                bj = oj;
            }
            if (fh == 0) {
                red_s[w][fr] = bs;
                red_j[w][fr] = bj;
            }
            __syncthreads();
            if (w == 0 && fh == 0 && mine) {  // the waves' bests: the same order-free maximum
#pragma unroll
                for (int v = 1; v < RS_NW; v++)
                    if (better(0, red_s[v][fr], red_j[v][fr], bs, bj)) {
                        bs = red_s[v][fr];
                        bj = red_j[v][fr];
                    }
                const bool keep = bj != 0x7fffffff && (double)bs > thresh && bs > 0.f;
                oidx[myrow] = keep ? bj : -1;
                if (oscore) oscore[myrow] = keep ? bs : 0.f;
            }
            __syncthreads();  // red reused by the next batch
        };
        // the pending rows (index < -1), gathered 32 at a time in row order -- every wave the
        // same list, into its own copy (the reads of oidx precede any write of this pair's rows:
        // a batch writes only rows already gathered)
        int ns = 0;
        for (int r0 = 0; r0 < cap; r0 += 64) {
            const int r = r0 + lane;
            const int v = r < cap ? oidx[r] : -1;
            bool pend = v < -1;
            for (unsigned long long mask = __ballot(pend); mask; mask = __ballot(pend)) {
                const int rank = __popcll(mask & ((1ull << lane) - 1ull)), room = 32 - ns;
                if (pend && rank < room) {
                    slots[ns + rank] = r;
                    lims[ns + rank] = rs_decode(v);
                    pend = false;
                }
                ns += min(__popcll(mask), room);
                if (ns == 32) {
                    run_batch(32);
                    ns = 0;
                }
            }
        }
        if (ns) run_batch(ns);
    }
}

}  // namespace

namespace mv {

int launch_allpairs_q8d_handback(hipStream_t s, int batch, int cap, const int *n0, const int *n1, const float *desc0,
                                 const float *desc1, double thresh, int *match_idx, float *match_score,
                                 const int *only);

int launch_allpairs_q8d_match(hipStream_t s, int batch, int cap, const int *n0, const int *n1, const float *desc0,
                              const float *desc1, double thresh, int *match_idx, float *match_score, int dmode,
                              const int *only) {
    if (only) return launch_allpairs_q8d_handback(s, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                                  match_score, only);
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


int launch_allpairs_q8d_handback(hipStream_t s, int batch, int cap, const int *n0, const int *n1, const float *desc0,
                                 const float *desc1, double thresh, int *match_idx, float *match_score,
                                 const int *only) {
    const int tiles_r = (cap + D_BM - 1) / D_BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31) && (long)cap * KD * 4 < (1l << 32));
    MV_PROF_BEGIN(s, "k_q8d_handback");
    hipLaunchKernelGGL(k_q8d_handback, dim3((unsigned)min(blocks, 256l)), dim3(D_NT), 0, s, tiles_r, cap, n0, n1,
                       desc0, desc1, thresh, match_idx, match_score, only, (int)blocks);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

// k_q8t_match (one workgroup per pair) where it applies -- cap <= 1024, the indices / scores
// match (dmode 0) -- with the pairs it hands back (outside the integer keys' range) redone by
// k_q8d_match in the same stream: flags[batch] in `scratch` (zeroed here)
bool allpairs_q8t_applies(int cap, int dmode) {
    static const int off = [] {
        const char *e = getenv("MV_Q8_KERNEL");  // "d": k_q8d_match only (A/B of the two layouts)
        return e && e[0] == 'd' ? 1 : 0;
    }();
    return !off && dmode == 0 && cap > 0 && cap <= T_BM;
}
// scratch: [batch] hand-back flags | [batch] re-screen flags (tag width + 1) | [batch][T_BM] the
// pairs' column key shifts (written only for pairs with re-screened rows)
size_t allpairs_q8t_scratch_bytes(int batch) {
    return 2 * align_up((size_t)batch * 4, 256) + (size_t)batch * T_BM;
}

int launch_allpairs_q8t_match(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                              const float *desc0, const float *desc1, double thresh, int *match_idx,
                              float *match_score) {
    MV_REQUIRE(batch > 0 && cap > 0 && cap <= T_BM && n0 && n1 && desc0 && desc1 && match_idx && scratch);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    const size_t fb = align_up((size_t)batch * 4, 256);
    int *flags = static_cast<int *>(scratch);
    int *rflags = reinterpret_cast<int *>(static_cast<char *>(scratch) + fb);
    unsigned char *rcolsh = static_cast<unsigned char *>(scratch) + 2 * fb;
    MV_HIP_TRY(hipMemsetAsync(flags, 0, 2 * fb, s));
    MV_PROF_BEGIN(s, "k_q8t_match");
    hipLaunchKernelGGL(k_q8t_match, dim3((unsigned)batch), dim3(D_NT), 0, s, cap, n0, n1, desc0, desc1, thresh,
                       match_idx, match_score, flags, rflags, rcolsh);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    // the wide rows it left: 4 waves per workgroup, a grid-stride loop over pairs
    MV_PROF_BEGIN(s, "k_q8t_rescan");
    hipLaunchKernelGGL(k_q8t_rescan, dim3((unsigned)min(batch, 1024)), dim3(64 * RS_NW), 0, s, batch, cap, n1, desc0,
                       desc1, thresh, match_idx, match_score, rflags, rcolsh);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return launch_allpairs_q8d_match(s, batch, cap, n0, n1, desc0, desc1, thresh, match_idx, match_score, 0, flags);
}

}  // namespace mv

#ifdef MV_TRACE
extern "C" int mv_debug_direct_trace(void *host, long bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_d_trace), (size_t)bytes) == hipSuccess ? 0 : -3;
}
#endif
