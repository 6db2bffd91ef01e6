// k_allpairs_q8.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659) with
// the gemmini_functions_cpu.h:14-56 summation order as the exact score, screened on the INT8
// matrix cores against a STAGED int8 image of frame 1 (MV_SCREEN_I8_STAGED, and sequence mode,
// where every frame's image serves two pairs).  The single-pass kernel that quantises frame 1
// inside the workgroup (the default screen) is k_allpairs_direct.hip; the window argument,
// the A phase and the epilogue are shared (q8_common.hpp).
//
//   k_q8_split  frame 1, one pass: every fp32 row b_j becomes int8 q_jk = RNE(b_jk * 127 / m_j)
//               (m_j = max_k |b_jk|) with its dequantisation scale s_j = RN(m_j / 127), |b_j|^2
//               and the residual energy |eps_j|^2, eps_jk = b_jk - q_jk s_j.  A pair with a
//               non-finite value or a row scale outside [2^-40, 2^40] is flagged: all of its
//               rows take the exact path.  HBM-bound: 1 KiB read, 268 B written per row.
//   k_q8_match  a 256-thread block (4 waves x 64 rows, two blocks per CU) owns 256 query rows of
//               one pair: each wave reads its rows as fp32 ONCE, quantises them in registers
//               (per-row scale s_a, 64 VGPRs of int8 A operands), then streams frame 1's int8
//               image in 64-column tiles (16 KiB + the tile's 64 scales) through a 4-slot LDS
//               ring (global_load_lds, 3 tiles in flight) into v_mfma_i32_32x32x32_i8.  The
//               exact integer dot D_ij becomes the screen f_ij = RN(D_ij s_j) in one FMA, tagged
//               with its column tile in the low mantissa bits and folded into a lane-local top-2
//               per row.  Fused form: each workgroup then stages a share of the NEXT batch's
//               frame 1 (the k_q8_split passes).
// Bound: HBM (A fp32 1 KiB per row) and int8 MFMA; per pair 2 n0 n1 256 algorithmic ops.
#include "q8_common.hpp"

namespace {

using namespace q8;

constexpr int Q_NW = 4, Q_NT = 64 * Q_NW, Q_BM = 32 * RG * Q_NW, Q_NBUF = 4;
constexpr int Q_PF = 2;                            // k32 steps of B fragments read ahead of the MFMAs
constexpr int Q_OFF_MISC = Q_NBUF * SLOT;          // [2][NW] f32 per-wave max |b|^2, |eps|^2
constexpr int Q_OFF_ROW = Q_OFF_MISC + 2 * Q_NW * 4;  // [BM] float2 per row (|a|^2, s_a; s_a < 0: exact path)
constexpr int Q_LDS = Q_OFF_ROW + Q_BM * 8;
static_assert(epi_bytes<Q_NW>() <= Q_NBUF * SLOT, "epilogue fits the ring");
static_assert(2 * Q_LDS <= 160 * 1024, "two blocks per CU");

// ---- k_q8_split: 16 lanes per row (lane sub holds floats 4 (sub + 16 u) .. +3, u < 4: every
//      load instruction reads 256 contiguous bytes of 4 rows), QS_RPG rows per lane group in
//      flight; a 256-thread block strides over the batch (rows >= n1 are never read
//      downstream and are not written) ----
constexpr int QS_RPG = 2, QS_GRID = 256 * 64, QS_ROWS = 16 * QS_RPG;
// one pass: rows R0 + 16 r + (thread >> 4), r < QS_RPG, below `rows` (= batch * cap)
__device__ __forceinline__ void q8_split_pass(long R0, long rows, int cap, const int *__restrict__ n1v,
                                              const float *__restrict__ desc1, char *__restrict__ q1,
                                              float *__restrict__ s1, float *__restrict__ nb2,
                                              float *__restrict__ eb2, int *__restrict__ bad) {
    const int sub = threadIdx.x & 15, rg = threadIdx.x >> 4;
    f32x4v x[QS_RPG][4];
    long c[QS_RPG];
#pragma unroll
    for (int r = 0; r < QS_RPG; r++) {
        const long R = R0 + 16 * r + rg;
        c[r] = R < rows ? R : rows - 1;
#pragma unroll
        for (int u = 0; u < 4; u++)
            x[r][u] = __builtin_nontemporal_load(
                reinterpret_cast<const f32x4v *>(desc1 + c[r] * KD + 4 * (sub + 16 * u)));
    }
#pragma unroll
    for (int r = 0; r < QS_RPG; r++) {
        const long R = R0 + 16 * r + rg;
        float m = 0.f, q2 = 0.f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            m = absmax3(m, x[r][u][0], x[r][u][1]);
            m = absmax3(m, x[r][u][2], x[r][u][3]);
#pragma unroll
            for (int e = 0; e < 4; e++) q2 = __builtin_fmaf(x[r][u][e], x[r][u][e], q2);
        }
        m = fmaxf(m, swz_xor<1>(m));
        m = fmaxf(m, swz_xor<2>(m));
        m = fmaxf(m, swz_xor<4>(m));
        m = fmaxf(m, swz_xor<8>(m));
        q2 += swz_xor<1>(q2);
        q2 += swz_xor<2>(q2);
        q2 += swz_xor<4>(q2);
        q2 += swz_xor<8>(q2);
        const float q = m > 0.f ? 127.f / m : 0.f;
        const float s = m / 127.f;
        int pk[4];
        float e2 = 0.f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            pk[u] = pack4(x[r][u][0], x[r][u][1], x[r][u][2], x[r][u][3], q);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float v = __builtin_fmaf(x[r][u][e], q, MAGIC_RNE) - MAGIC_RNE;  // exact
                const float ep = __builtin_fmaf(-v, s, x[r][u][e]);
                e2 = __builtin_fmaf(ep, ep, e2);
            }
        }
        e2 += swz_xor<1>(e2);
        e2 += swz_xor<2>(e2);
        e2 += swz_xor<4>(e2);
        e2 += swz_xor<8>(e2);
        // finite (|b|^2 propagates NaN / inf) and a representable scale (zero rows: s = 0,
        // q = 0, every screen value of the column 0 -- exact, no flag needed)
        const bool ok = q2 <= FLT_MAX && (m == 0.f || (m >= SCALE_LO && m <= SCALE_HI));
        const int pair = (int)(c[r] / cap);
        if (R < rows && (int)(c[r] - (long)pair * cap) < n1v[pair]) {
#pragma unroll
            for (int u = 0; u < 4; u++) *reinterpret_cast<int *>(q1 + R * KD + 4 * (sub + 16 * u)) = pk[u];
            if (!ok) bad[pair] = 1;
            if (sub == 0) {
                s1[R] = s;
                nb2[R] = q2;
                eb2[R] = e2;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_q8_split(int batch, int cap, const int *__restrict__ n1v,
                                                  const float *__restrict__ desc1, char *__restrict__ q1,
                                                  float *__restrict__ s1, float *__restrict__ nb2,
                                                  float *__restrict__ eb2, int *__restrict__ bad) {
    const long rows = (long)batch * cap;
    for (long R0 = (long)blockIdx.x * QS_ROWS; R0 < rows; R0 += (long)gridDim.x * QS_ROWS)
        q8_split_pass(R0, rows, cap, n1v, desc1, q1, s1, nb2, eb2, bad);
}

// ---- k_q8_match ----
// AI8 (sequence mode): frame 0 arrives already quantised by k_q8_split -- its int8 image q0,
// scales s0v, |a|^2 na2v and pair flags bad0 (the previous pair's frame-1 image) -- so the A
// phase copies 256 B per row instead of reading 1 KiB of fp32 and quantising it.  The window
// is unchanged: the split's codes RNE(a RN(127/m)) with s_a = RN(m/127) satisfy the same
// |1 - q s_a| < 2^-21 that the in-register quantisation guarantees.
template <bool AI8>
__device__ __forceinline__ void q8_match_block(int tiles_r, int cap, const int *__restrict__ n0v,
                                               const int *__restrict__ n1v, const float *__restrict__ desc0,
                                               const float *__restrict__ desc1, const char *__restrict__ q1,
                                               const float *__restrict__ s1v, const float *__restrict__ nb2v,
                                               const float *__restrict__ eb2v, const int *__restrict__ bad,
                                               double thresh, int dmode, int *__restrict__ match_idx,
                                               float *__restrict__ match_score, const char *__restrict__ q0,
                                               const float *__restrict__ s0v, const float *__restrict__ na2v,
                                               const int *__restrict__ bad0) {
    __shared__ __attribute__((aligned(16))) char lds[Q_LDS];
    float *misc = reinterpret_cast<float *>(lds + Q_OFF_MISC);
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int pair = L / tiles_r, tr = L % tiles_r;
    const int n0 = min(max(n0v[pair], 0), cap), n1 = min(max(n1v[pair], 0), cap);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int row0 = tr * Q_BM;
    int *oidx = match_idx + (size_t)pair * cap + row0;
    float *oscore = match_score ? match_score + (size_t)pair * cap + row0 : nullptr;  // null: indices only
    if (row0 + t < cap && (row0 + t >= n0 || n1 <= 0)) {  // rows in [n0, cap): no match
        oidx[t] = -1;
        if (oscore) oscore[t] = 0.f;
    }
    if (row0 >= n0 || n1 <= 0) return;
    const bool flagged = bad[pair] != 0;
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;
    const char *QB = q1 + (size_t)pair * cap * KD;
    const float *sb = s1v + (size_t)pair * cap;
    const int ntc = flagged ? 0 : (n1 + BN - 1) / BN;  // a flagged pair skips the screen

    // Bn^2 = max |b_j|^2, Eb^2 = max |eps_j|^2 over the pair's columns (published by the
    // prologue barrier)
    {
        const float *p2 = nb2v + (size_t)pair * cap, *e2 = eb2v + (size_t)pair * cap;
        float bm = 0.f, em = 0.f;
        for (int j = t; j < n1; j += Q_NT) {
            bm = fmaxf(bm, p2[j]);
            em = fmaxf(em, e2[j]);
        }
        bm = fmaxf(bm, swz_xor<1>(bm));
        bm = fmaxf(bm, swz_xor<2>(bm));
        bm = fmaxf(bm, swz_xor<4>(bm));
        bm = fmaxf(bm, swz_xor<8>(bm));
        bm = fmaxf(bm, swz_xor<16>(bm));
        em = fmaxf(em, swz_xor<1>(em));
        em = fmaxf(em, swz_xor<2>(em));
        em = fmaxf(em, swz_xor<4>(em));
        em = fmaxf(em, swz_xor<8>(em));
        em = fmaxf(em, swz_xor<16>(em));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        em = fmaxf(em, __shfl_xor(em, 32, 64));
        if (lane == 0) {
            misc[w] = bm;
            misc[Q_NW + w] = em;
        }
    }

    // ---- B DMA map: wave w fills rows w*16 .. +15 of a tile, 4 rows (1 KiB) per instruction;
    //      lane l -> row (l >> 4), chunk position l & 15, source chunk (l & 15) ^ (row & 15);
    //      plus the tile's 64 scales (every wave the same 256 B, so all waves count 5 loads per
    //      tile) ----
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int dr = wu * 16 + (lane >> 4);
    const unsigned dcb = (unsigned)((lane & 15) ^ (dr & 15)) * 16;
    unsigned oB[4], oR;
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    const unsigned dst_w = lds_base + (unsigned)(wu * 16 * KD);
#define Q8_STAGE(SLOT_)                                                                      \
    do {                                                                                     \
        glds16<(SLOT_) * SLOT>(QB, oB[0], dst_w);                                            \
        glds16<(SLOT_) * SLOT + 4 * KD>(QB, oB[1], dst_w);                                   \
        glds16<(SLOT_) * SLOT + 8 * KD>(QB, oB[2], dst_w);                                   \
        glds16<(SLOT_) * SLOT + 12 * KD>(QB, oB[3], dst_w);                                  \
        glds4<(SLOT_) * SLOT + TILE>(sb, oR, lds_base);                                      \
    } while (0)
#define Q8_OFFSETS(TC)                                                                       \
    do {                                                                                     \
        const int nb_ = (TC) * BN + dr;                                                      \
        _Pragma("unroll") for (int g_ = 0; g_ < 4; g_++)                                     \
            oB[g_] = (unsigned)min(nb_ + 4 * g_, n1 - 1) * KD + (dcb ^ (64u * g_));          \
        oR = (unsigned)min((TC) * BN + lane, n1 - 1) * 4;                                    \
    } while (0)
    // prologue DMA: tiles 0, 1 into slots 0, 1 -- issued before the A rows are read so both
    // latencies overlap (slots 2, 3 hold the A images meanwhile; tile 2 follows the A phase)
    for (int g = 0; g < 2 && g < ntc; g++) {
        Q8_OFFSETS(g);
        if (g == 0) Q8_STAGE(0);
        if (g == 1) Q8_STAGE(1);
    }

    // ---- A: the wave's 64 rows into registers (slots 2-3 hold the images meanwhile) ----
    const int fr = lane & 31, fh = lane >> 5;
    i32x4 aI[RG][KD / 32];
    float2 *rowv = reinterpret_cast<float2 *>(lds + Q_OFF_ROW);
    a_phase<AI8>(lds + 2 * SLOT + w * 32 * KD, rowv, w * 64, row0, n0, lane, A,
                 AI8 ? q0 + (size_t)pair * cap * KD : nullptr, AI8 ? s0v + (size_t)pair * cap : nullptr,
                 AI8 ? na2v + (size_t)pair * cap : nullptr, AI8 && bad0[pair] != 0, aI);
    __syncthreads();  // every wave's image is read: slot 2 takes tile 2
    if (ntc > 2) {
        Q8_OFFSETS(2);
        Q8_STAGE(2);
    }

    // B fragment: column block c (0, 1), lane row 32 c + fr, k32 step s: chunk (2 s + fh)
    const int rdb = fr * KD;
    const int xsw = fh ^ (fr & 15);  // chunk (2 s + fh) ^ (fr & 15) = 2 s ^ xsw

    // Accumulators start at the bits of 4.0 (0x40800000, an inline constant of the MFMA's C
    // operand: no registers): t = 4 + D 2^-21 as a float (|D| <= 127^2 * 256 < 2^22), so
    // f = fma(t, 2^21 s_j, -2^23 s_j) = RN(D s_j) (the product is exact inside the fma).
    // Columns past n1 (last tile only) get s = 0 and the offset -3e38.  The low tb bits of f
    // are then replaced by the column tag 2 tc + half.
    i32x16 acc[RG][2];
    float m1[RG][16], m2[RG][16];
#pragma unroll
    for (int g = 0; g < RG; g++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            m1[g][q] = -__builtin_inff();
            m2[g][q] = -__builtin_inff();
        }
#pragma unroll
    for (int q = 0; q < 16; q++) {  // "tile -1" of group 1, folded beside tile 0: never a maximum
        acc[1][0][q] = 0;
        acc[1][1][q] = 0;
    }
    const int tb = 2 * ntc <= 256 ? 8 : 32 - __builtin_clz(2 * ntc - 1);
    const unsigned tkeep = ~((1u << tb) - 1u);
    unsigned vkeep = tkeep;
    asm volatile("" : "+v"(vkeep));  // a VGPR operand: v_and_or_b32 may read one SGPR only

    // Software pipeline over the two 32-row groups: tile tc's MFMAs for group 0 issue beside
    // the fold of group 1 of tile tc - 1, then tile tc's MFMAs for group 1 beside the fold of
    // group 0 of tile tc.  Each wave thus always has independent VALU work between its MFMAs
    // (the fold of one group never waits on the MFMAs in flight), with one accumulator set.
    // The B fragments are read from LDS once per group (2 ds_read_b128 per MFMA pair).
    // fold rows 2 S, 2 S + 1 of group FG (tile tags G0, G0 + 1; scales R, offsets C)
#define Q8_FOLD2(FG, S, G0)                                                                  \
    do {                                                                                     \
        _Pragma("unroll") for (int q = 2 * (S); q < 2 * (S) + 2; q++) {                      \
            const float a_ = __builtin_fmaf(__int_as_float(acc[FG][0][q]), pr0, pc0);        \
            const float b_ = __builtin_fmaf(__int_as_float(acc[FG][1][q]), pr1, pc1);        \
            fold3(tag(a_, vkeep, (G0)), tag(b_, vkeep, (G0) + 1u), m1[FG][q], m2[FG][q]);    \
        }                                                                                    \
    } while (0)
    // group G's MFMAs on slot J (fragments read Q_PF k32 steps ahead), folding group FG meanwhile
#define Q8_SEG(J, G, FG, G0)                                                                 \
    do {                                                                                     \
        const char *base = lds + (J) * SLOT + rdb;                                           \
        int xs_ = xsw;                                                                       \
        asm volatile("" : "+v"(xs_)); /* per-use offsets: not 8 loop-invariant VGPRs */      \
        i32x4 b0_[KD / 32], b1_[KD / 32];                                                    \
        _Pragma("unroll") for (int s_ = 0; s_ < KD / 32 + Q_PF; s_++) {                      \
            if (s_ < KD / 32) {                                                              \
                const int ch_ = ((2 * s_) ^ xs_) * 16;                                       \
                b0_[s_] = *reinterpret_cast<const i32x4 *>(base + ch_);                      \
                b1_[s_] = *reinterpret_cast<const i32x4 *>(base + 32 * KD + ch_);            \
            }                                                                                \
            if (s_ >= Q_PF) {                                                                \
                const int m_ = s_ - Q_PF;                                                    \
                if (m_ == 0) {                                                               \
                    acc[G][0] = mfma_i8_from4(aI[G][0], b0_[0]);                             \
                    acc[G][1] = mfma_i8_from4(aI[G][0], b1_[0]);                             \
                } else {                                                                     \
                    acc[G][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b0_[m_], acc[G][0], 0, 0, 0); \
                    acc[G][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b1_[m_], acc[G][1], 0, 0, 0); \
                }                                                                            \
                Q8_FOLD2(FG, m_, G0);                                                        \
            }                                                                                \
        }                                                                                    \
    } while (0)
    // the dequantisation operands of tile TC (read from its slot J): fma(t, 2^21 s, -2^23 s)
#define Q8_SCALES(J, TC)                                                                     \
    do {                                                                                     \
        const float *rl_ = reinterpret_cast<const float *>(lds + (J) * SLOT + TILE);         \
        const int col_ = (TC) * BN + fr;                                                     \
        const float s0_ = rl_[fr], s1_ = rl_[fr + 32];                                       \
        pr0 = col_ < n1 ? 2097152.0f * s0_ : 0.f;                                            \
        pr1 = col_ + 32 < n1 ? 2097152.0f * s1_ : 0.f;                                       \
        pc0 = col_ < n1 ? -8388608.0f * s0_ : -3.0e38f;                                      \
        pc1 = col_ + 32 < n1 ? -8388608.0f * s1_ : -3.0e38f;                                 \
    } while (0)
    // ring: tile g lives in slot g % 4; at tile g issue tile g + 3 into the slot read at g - 1
    // (whose scales the previous tile left in pr*)
#define Q8_SLOT(J)                                                                           \
    do {                                                                                     \
        const int tc = T + (J);                                                              \
        const int ntile = tc + Q_NBUF - 1;                                                   \
        if (ntile < ntc) {                                                                   \
            Q8_OFFSETS(ntile);                                                               \
            Q8_STAGE((J + Q_NBUF - 1) % Q_NBUF);                                             \
        }                                                                                    \
        const unsigned gp_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)max(tc - 1, 0));  \
        Q8_SEG(J, 0, 1, gp_);                                                                \
        Q8_SCALES(J, tc);                                                                    \
        const unsigned gc_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)tc);              \
        Q8_SEG(J, 1, 0, gc_);                                                                \
        if (ntile < ntc) {                                                                   \
            wait_vm<5 * (Q_NBUF - 2)>();                                                     \
        } else {                                                                             \
            wait_vm<0>();                                                                    \
        }                                                                                    \
        __syncthreads();                                                                     \
    } while (0)

    // tile 0 landed (younger: tiles 1 and 2, 5 ops each)
    if (ntc > 2) {
        wait_vm<10>();
    } else {
        wait_vm<0>();
    }
    __syncthreads();
    // scales of the tile before (tile -1: a column that never wins)
    float pr0 = 0.f, pr1 = 0.f, pc0 = -3.0e38f, pc1 = -3.0e38f;
    for (int T = 0; T < ntc; T += 4) {
        Q8_SLOT(0);
        if (T + 1 < ntc) Q8_SLOT(1);
        if (T + 2 < ntc) Q8_SLOT(2);
        if (T + 3 < ntc) Q8_SLOT(3);
    }
    if (ntc > 0) {  // group 1 of the last tile
        const unsigned gl_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)(ntc - 1));
#pragma unroll
        for (int s = 0; s < 8; s++) Q8_FOLD2(1, s, gl_);
    }
#undef Q8_STAGE
#undef Q8_OFFSETS
#undef Q8_FOLD2
#undef Q8_SEG
#undef Q8_SCALES
#undef Q8_SLOT

    // ---- epilogue (the ring is free: the sweep's last barrier follows a full drain) ----
    float bmax2 = misc[0], emax2 = misc[Q_NW];
#pragma unroll
    for (int k = 1; k < Q_NW; k++) {
        bmax2 = fmaxf(bmax2, misc[k]);
        emax2 = fmaxf(emax2, misc[Q_NW + k]);
    }
    const double Bn = sqrt((double)bmax2) * 1.0001, Eb = sqrt((double)emax2) * 1.0001 + 1e-30;
    epilogue<Q_NW>(lds, rowv, m1, m2, Bn, Eb, flagged, tb, tkeep, w, lane, row0, n0, n1, A, B, oidx, oscore,
                   thresh, dmode);
}

// The match of one 256-row tile of one pair (q8_match_block), then -- when a next batch is
// given (nrows > 0) -- this block's share of the next batch's frame-1 staging (the k_q8_split
// passes, rows blockIdx * rpb .. +rpb): the separate staging kernel, its launch and its
// stream hand-off leave the pipelined step; its HBM reads overlap the co-resident block's sweep.
template <bool AI8>
__global__ __launch_bounds__(Q_NT, 2) void k_q8_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                      const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                      const float *__restrict__ desc1, const char *__restrict__ q1,
                                                      const float *__restrict__ s1v, const float *__restrict__ nb2v,
                                                      const float *__restrict__ eb2v, const int *__restrict__ bad,
                                                      double thresh, int dmode, int *__restrict__ match_idx,
                                                      float *__restrict__ match_score, long nrows, int ncap,
                                                      const int *__restrict__ nn1, const float *__restrict__ ndesc1,
                                                      char *__restrict__ nq1, float *__restrict__ ns1,
                                                      float *__restrict__ nnb2, float *__restrict__ neb2,
                                                      int *__restrict__ nbad, const char *__restrict__ q0,
                                                      const float *__restrict__ s0v, const float *__restrict__ na2v,
                                                      const int *__restrict__ bad0) {
    const long rpb = ((nrows + gridDim.x - 1) / gridDim.x + QS_ROWS - 1) / QS_ROWS * QS_ROWS;
    const long lo = (long)blockIdx.x * rpb, hi = min(lo + rpb, nrows);
    q8_match_block<AI8>(tiles_r, cap, n0v, n1v, desc0, desc1, q1, s1v, nb2v, eb2v, bad, thresh, dmode, match_idx,
                        match_score, q0, s0v, na2v, bad0);
    if (nrows > 0) {
        __syncthreads();  // every wave is past its sweep (the tail needs no LDS)
        for (long R0 = lo; R0 < hi; R0 += QS_ROWS) q8_split_pass(R0, hi, ncap, nn1, ndesc1, nq1, ns1, nnb2, neb2, nbad);
    }
}

}  // namespace

namespace mv {

// scratch: q1 (rows * 256 B) | s1 | nb2 | eb2 (rows f32 each) | bad (batch i32)
size_t allpairs_q8_scratch_bytes(int batch, int cap) {
    const size_t rows = (size_t)batch * cap;
    return rows * KD + 3 * align_up(rows * 4, 256) + align_up((size_t)batch * 4, 256);
}

namespace {
struct Q8Scratch {
    char *q1;
    float *s1, *nb2, *eb2;
    int *bad;
};
Q8Scratch q8_map(void *scratch, int batch, int cap) {
    const size_t rows = (size_t)batch * cap, fb = align_up(rows * 4, 256);
    Q8Scratch m;
    m.q1 = (char *)scratch;
    m.s1 = (float *)(m.q1 + rows * KD);
    m.nb2 = (float *)((char *)m.s1 + fb);
    m.eb2 = (float *)((char *)m.nb2 + fb);
    m.bad = (int *)((char *)m.eb2 + fb);
    return m;
}
}  // namespace

int launch_allpairs_q8_prepare(hipStream_t s, void *scratch, int batch, int cap, const int *n1, const float *desc1) {
    MV_REQUIRE(batch > 0 && cap > 0 && n1 && desc1 && scratch);
    MV_REQUIRE(((uintptr_t)desc1 & 15) == 0);
    MV_REQUIRE((long)cap * KD < (1l << 31));  // 32-bit DMA source offsets within a pair
    const size_t rows = (size_t)batch * cap;
    const Q8Scratch m = q8_map(scratch, batch, cap);
    const long blocks = std::min<long>((long)((rows + QS_ROWS - 1) / QS_ROWS), (long)QS_GRID);
    MV_HIP_TRY(hipMemsetAsync(m.bad, 0, (size_t)batch * 4, s));
    MV_PROF_BEGIN(s, "k_q8_split");
    hipLaunchKernelGGL(k_q8_split, dim3((unsigned)blocks), dim3(256), 0, s, batch, cap, n1, desc1, m.q1, m.s1, m.nb2,
                       m.eb2, m.bad);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

int launch_allpairs_q8_match_prepare(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                                     const float *desc0, const float *desc1, double thresh, int *match_idx,
                                     float *match_score, int dmode, void *next_scratch, int next_batch,
                                     int next_cap, const int *next_n1, const float *next_desc1) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx && scratch);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    MV_REQUIRE((long)cap * KD < (1l << 31));
    const int tiles_r = (cap + Q_BM - 1) / Q_BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    const Q8Scratch m = q8_map(scratch, batch, cap);
    Q8Scratch nm = {};
    long nrows = 0;
    if (next_scratch) {
        MV_REQUIRE(next_batch > 0 && next_cap > 0 && next_n1 && next_desc1 && next_scratch != scratch);
        MV_REQUIRE(((uintptr_t)next_desc1 & 15) == 0);
        MV_REQUIRE((long)next_cap * KD < (1l << 31));
        nm = q8_map(next_scratch, next_batch, next_cap);
        nrows = (long)next_batch * next_cap;
        MV_HIP_TRY(hipMemsetAsync(nm.bad, 0, (size_t)next_batch * 4, s));
    }
    MV_PROF_BEGIN(s, "k_q8_match");
    hipLaunchKernelGGL(k_q8_match<false>, dim3((unsigned)blocks), dim3(Q_NT), 0, s, tiles_r, cap, n0, n1, desc0,
                       desc1, m.q1, m.s1, m.nb2, m.eb2, m.bad, dmode ? -1e300 : thresh, dmode, match_idx, match_score,
                       nrows, next_cap, next_n1, next_desc1, nm.q1, nm.s1, nm.nb2, nm.eb2, nm.bad,
                       (const char *)nullptr, (const float *)nullptr, (const float *)nullptr, (const int *)nullptr);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

int launch_allpairs_q8_match(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                             const float *desc0, const float *desc1, double thresh, int *match_idx,
                             float *match_score, int dmode) {
    return launch_allpairs_q8_match_prepare(s, scratch, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                            match_score, dmode, nullptr, 0, 0, nullptr, nullptr);
}

// Sequence mode: frames 0 .. F-1 of one track, pair b = (frame b, frame b + 1).  Every frame
// is quantised ONCE (one k_q8_split over all F frames); pair b then reads frame b's image as
// its A operand and frame b + 1's as its B operand -- plain offsets into the one scratch.
// prepared = true: the frames' images are already in scratch (a prepare / the previous
// run_prepare staged them).  next_scratch: the launch also stages the next chunk's frames into
// it (k_q8_split passes after each workgroup's tile, as launch_allpairs_q8_match_prepare).
int launch_allpairs_q8_sequence(hipStream_t s, void *scratch, int frames, int cap, const int *n, const float *desc,
                                double thresh, int *match_idx, float *match_score, bool prepared,
                                void *next_scratch, int next_frames, int next_cap, const int *next_n,
                                const float *next_desc) {
    MV_REQUIRE(frames >= 2 && cap > 0 && n && desc && match_idx && scratch);
    MV_REQUIRE(((uintptr_t)desc & 15) == 0);
    MV_REQUIRE((long)cap * KD < (1l << 31));
    if (!prepared) {
        const int st = launch_allpairs_q8_prepare(s, scratch, frames, cap, n, desc);
        if (st != MV_OK) return st;
    }
    const int batch = frames - 1, tiles_r = (cap + Q_BM - 1) / Q_BM;
    const long blocks = (long)batch * tiles_r;
    MV_REQUIRE(blocks < (1l << 31));
    const Q8Scratch m = q8_map(scratch, frames, cap);
    Q8Scratch nm = {};
    long nrows = 0;
    if (next_scratch) {
        MV_REQUIRE(next_frames > 0 && next_cap > 0 && next_n && next_desc && next_scratch != scratch);
        MV_REQUIRE(((uintptr_t)next_desc & 15) == 0);
        MV_REQUIRE((long)next_cap * KD < (1l << 31));
        nm = q8_map(next_scratch, next_frames, next_cap);
        nrows = (long)next_frames * next_cap;
        MV_HIP_TRY(hipMemsetAsync(nm.bad, 0, (size_t)next_frames * 4, s));
    }
    const size_t fr = (size_t)cap;
    MV_PROF_BEGIN(s, "k_q8_match_seq");
    hipLaunchKernelGGL(k_q8_match<true>, dim3((unsigned)blocks), dim3(Q_NT), 0, s, tiles_r, cap, n, n + 1, desc,
                       desc + fr * KD, m.q1 + fr * KD, m.s1 + fr, m.nb2 + fr, m.eb2 + fr, m.bad + 1, thresh, 0,
                       match_idx, match_score, nrows, next_cap, next_n, next_desc, nm.q1, nm.s1, nm.nb2, nm.eb2,
                       nm.bad, (const char *)m.q1, (const float *)m.s1, (const float *)m.nb2, (const int *)m.bad);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

}  // namespace mv
