// q8_common.hpp -- the parts of the int8-screened all-pairs fp32 match (python/pairwise_pnp.py:
// 635-659, exact score in the gemmini_functions_cpu.h:45-49 order) shared by its two kernels:
//   k_q8_match  (k_allpairs_q8.hip)      frame 1 streamed as the int8 image k_q8_split staged
//   k_q8d_match (k_allpairs_direct.hip)  frame 1 streamed as fp32 and quantised in the workgroup
// Device helpers, the A phase (frame-0 rows fp32 -> int8 MFMA operands in registers) and the
// epilogue (per-row merge of the lanes' tagged top-2, the window decisions, exact re-scores).
//
// Window (both kernels).  With a = q_a s_a + eps_a, b = q_b s_b + eps_b (real arithmetic, s the
// float scales used), d = a.b and D = q_a.q_b (exact integer):
//   |d - s_a s_b D| <= |a| Eb + |eps_a| Bn + |eps_a| Eb =: dq        (Cauchy-Schwarz)
// with Bn >= max_j |b_j|, Eb >= max_j |eps_j| over the pair's columns and
// |eps_a| <= 8 s_a + 2^-21 |a| (|x - RNE(x q) s| <= s / 2 + |x| |1 - q s|, |1 - q s| < 2^-21).
// The screen in real units, s_a f = s_a RN(D s_b), adds 2^-24 (|a| Bn + dq); the reference's
// sequential fp32 sum e adds gamma_256(2^-24) |a| Bn.  So |s_a f_j - e_j| <= delta for every
// column: a runner-up below M - 2 delta' leaves the screen maximiser as the reference's maximiser
// (ties included) and one exact dot decides the threshold (none when the window lies entirely
// above it and no score is asked for); otherwise the columns inside the window are re-scored
// exactly.  Negative dots leave the accumulator below 2^23 (t = 2^23 + D/2): their screen is
// D s_b / 2 >= D s_b, never below the truth -- the window stays conservative.
#pragma once
#include <float.h>
#include <math.h>

#include "mv_internal.hpp"

namespace q8 {

constexpr int KD = 256;
constexpr int RG = 2;                      // 32-row groups per wave (64 rows)
constexpr int BN = 64;                     // columns per tile
constexpr int TILE = BN * KD;              // 16 KiB: one int8 column tile, whole K
constexpr int SLOT = TILE + BN * 4;        // + the tile's 64 scales s_j
constexpr int MT_STRIDE = 32 * 8 + 16;     // epilogue transpose row: 32 (m1, m2) + pad
constexpr int NCAND = 16;                  // listed candidates per row (more: wide row)
constexpr float MAGIC_RNE = 12582912.f;    // 1.5 * 2^23: fma(x, q, MAGIC) = MAGIC + RNE(x q), |x q| < 2^22
constexpr float SCALE_LO = 9.094947017729282e-13f, SCALE_HI = 1099511627776.f;  // 2^-40, 2^40
// epilogue LDS of a block of NW waves: transposes, candidate lists, wide-row lane masks
template <int NW>
constexpr int epi_bytes() { return NW * 32 * MT_STRIDE + NW * 64 * NCAND * 4 + NW * 64 * 4; }

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

// logical block -> a contiguous run of logical blocks per XCD (blocks b, b + 8 share one):
// a pair's row blocks land on one XCD and share frame 1 through its L2
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total / 8, r = total % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

#pragma clang diagnostic ignored "-Winline-asm"
// LDS-DMA, 16 B per lane: LDS[m0 + 16 lane] <- global[sbase + voff] (the ring stays inline asm
// with counted waits: the builtin makes the compiler drain vmcnt in front of every LDS read)
template <int DOFF>
__device__ __forceinline__ void glds16(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_add_u32 m0, %2, %3\n\t"
        "global_load_lds_dwordx4 %0, %1"
        :
        : "v"(voff), "s"(sbase), "s"(lds_byte), "i"(DOFF)
        : "memory", "m0", "scc");
}
template <int DOFF>
__device__ __forceinline__ void glds4(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_add_u32 m0, %2, %3\n\t"
        "global_load_lds_dword %0, %1"
        :
        : "v"(voff), "s"(sbase), "s"(lds_byte), "i"(DOFF)
        : "memory", "m0", "scc");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// the tagged top-2 fold: m1' = max3(m1, a, b), m2' = max(m2, med3(m1, a, b))
__device__ __forceinline__ void fold3(float a, float b, float &m1, float &m2) {
    float md;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(md) : "v"(m1), "v"(a), "v"(b));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m1) : "v"(m1), "v"(a), "v"(b));
    asm("v_max_f32 %0, %1, %2" : "=v"(m2) : "v"(m2), "v"(md));
}
__device__ __forceinline__ float tag(float f, unsigned keep, unsigned tg) {
    float r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(keep), "s"(tg));
    return r;
}
// max(m, |a|, |b|) in one instruction (maxNum: a NaN operand is dropped -- callers catch NaN
// through a sum of squares, which propagates it)
__device__ __forceinline__ float absmax3(float m, float a, float b) {
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
template <int M>
__device__ __forceinline__ float swz_xor(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (M << 10) | 0x1F));
}
template <int M>
__device__ __forceinline__ int swz_xor(int v) {
    return __builtin_amdgcn_ds_swizzle(v, (M << 10) | 0x1F);
}
// D = 0x40800000 (the bits of 4.0) + A.B: the first k32 step of a chain, C as the inline
// constant 4.0 (a builtin with a constant C operand gets it hoisted into 16 VGPRs).  The
// chain's next MFMA reads D as SrcC with exact overlap (hardware forwarding, no wait states).
__device__ __forceinline__ i32x16 mfma_i8_from4(i32x4 a, i32x4 b) {
    i32x16 d;
    asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, 4.0" : "=&v"(d) : "v"(a), "v"(b));
    return d;
}
// four int8 RNE(x q) packed into a dword (byte i = element i): the magic sum's low byte is
// the two's-complement integer
__device__ __forceinline__ int pack4(float x0, float x1, float x2, float x3, float q) {
    const unsigned f0 = __float_as_uint(__builtin_fmaf(x0, q, MAGIC_RNE));
    const unsigned f1 = __float_as_uint(__builtin_fmaf(x1, q, MAGIC_RNE));
    const unsigned f2 = __float_as_uint(__builtin_fmaf(x2, q, MAGIC_RNE));
    const unsigned f3 = __float_as_uint(__builtin_fmaf(x3, q, MAGIC_RNE));
    const unsigned p01 = __builtin_amdgcn_perm(f1, f0, 0x0c0c0400u);
    const unsigned p23 = __builtin_amdgcn_perm(f3, f2, 0x0c0c0400u);
    return (int)__builtin_amdgcn_perm(p23, p01, 0x05040100u);
}

// The reference's sequential fp32 dot (mul then add, k = 0..255), 4 load batches per operand.
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
// The deferred maximiser re-scores load their rows COOPERATIVELY (coop_exact_dots) with
// Q8_COOP_PD 16-float chunks in flight.  Why: exact_dot's per-lane loads put 64 different rows
// (64 cache lines) under every load instruction, so a wave's re-scores cost ~38 x 128 line
// lookups of the L1 -- the near-threshold epilogue ran ~40 k cycles per wave, line-rate bound;
// the cooperative loads touch 16 lines per instruction.  Round 4's first cooperative form (its
// chunk loop fully unrolled: ~890 VGPRs spilled) lost (47.5 k cycles against 43.0 k); with the
// rounds of PD chunks kept as a loop, PD = 2 (17 spills, fewer than exact_dot's build): one box
// (profiles/r04n_coop_depth_ab.log) with scores 5.63-5.66 vs 5.85-5.86 ms, near threshold
// 5.25-5.26 vs 5.30, headline 4.27-4.30 vs 4.34-4.35; PD = 4 spills 130 and loses 30 %.
constexpr int Q8_COOP_PD = 2;
// The reference's sequential fp32 dot for the wave's 64 (row, column) pairs at once -- lane L's
// pair: A row `arow`, B row `bcol` (< 0: none) -- with the rows' bytes loaded COOPERATIVELY: per
// 16-float chunk, each load instruction takes 16 pairs' 64-B segments (4 lanes per segment, 16
// segments per instruction instead of exact_dot's one 16-B piece of 64 different rows), PD chunks
// in flight in registers, each staged through the wave's own 8 KiB of LDS (`buf`: [pair][A | B]
// [4 x 16 B], the 16-B quarters XOR-swizzled by pair: at most 2-way bank conflicts), from where
// each lane reads its own pair's chunk and adds its 16 products in order.
template <int PD = Q8_COOP_PD>
__device__ __forceinline__ float coop_exact_dots(const float *__restrict__ A, const float *__restrict__ B, int arow,
                                                 int bcol, int lane, char *buf) {
    constexpr int NC = KD / 16;  // chunks
    static_assert(PD >= 1 && PD <= NC, "chunks in flight");
    const int q = lane & 3;
    const float *pa[4];
    const float *pb[4];
    int soff[4];
    unsigned amask = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int p = 16 * i + (lane >> 2);
        const int r = __shfl(arow, p, 64), c = __shfl(bcol, p, 64);
        amask |= c >= 0 ? 1u << i : 0u;
        pa[i] = A + (size_t)(c >= 0 ? r : 0) * KD + 4 * q;
        pb[i] = B + (size_t)(c >= 0 ? c : 0) * KD + 4 * q;
        soff[i] = p * 128 + ((q ^ ((p >> 2) & 3)) << 4);
    }
    const int roff = lane * 128;
    const int rsw = (lane >> 2) & 3;
    float4 qa[PD][4], qb[PD][4];  // chunks c .. c + PD - 1 in flight
#pragma unroll
    for (int d = 0; d < PD; d++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const bool on = (amask >> i) & 1u;
            qa[d][i] = on ? *reinterpret_cast<const float4 *>(pa[i] + 16 * d) : make_float4(0.f, 0.f, 0.f, 0.f);
            qb[d][i] = on ? *reinterpret_cast<const float4 *>(pb[i] + 16 * d) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    float s = 0.f;
    static_assert(NC % PD == 0, "whole rounds of PD chunks");
#pragma unroll 1
    for (int c0 = 0; c0 < NC; c0 += PD)  // not unrolled: the compiler would hoist every chunk's loads
#pragma unroll
    for (int d = 0; d < PD; d++) {
        const int c = c0 + d;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            *reinterpret_cast<float4 *>(buf + soff[i]) = qa[d][i];
            *reinterpret_cast<float4 *>(buf + soff[i] + 64) = qb[d][i];
        }
        if (c + PD < NC) {  // the freed slot takes chunk c + PD
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const bool on = (amask >> i) & 1u;
                qa[d][i] = on ? *reinterpret_cast<const float4 *>(pa[i] + 16 * (c + PD)) : make_float4(0.f, 0.f, 0.f, 0.f);
                qb[d][i] = on ? *reinterpret_cast<const float4 *>(pb[i] + 16 * (c + PD)) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        // a wave's LDS operations complete in order: its reads below see every lane's writes
        float4 a4[4], b4[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            a4[j] = *reinterpret_cast<const float4 *>(buf + roff + ((j ^ rsw) << 4));
            b4[j] = *reinterpret_cast<const float4 *>(buf + roff + 64 + ((j ^ rsw) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            s = __fadd_rn(s, __fmul_rn(a4[j].x, b4[j].x));
            s = __fadd_rn(s, __fmul_rn(a4[j].y, b4[j].y));
            s = __fadd_rn(s, __fmul_rn(a4[j].z, b4[j].z));
            s = __fadd_rn(s, __fmul_rn(a4[j].w, b4[j].w));
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this chunk's reads done before the next writes
    }
    return bcol >= 0 ? s : 0.f;
}
// nn_match_two_way's distance (pairwise_pnp.py:303): sqrt(2 - 2 clip(dot, -1, 1)) in float32
__device__ __forceinline__ float dist(float e) {
    const float c = e != e ? e : fminf(fmaxf(e, -1.f), 1.f);
    return sqrtf(__fsub_rn(2.f, __fmul_rn(2.f, c)));
}
// dmode 0: larger dot, ties to the smaller index (NaN never wins); dmode 1: np.argmin
__device__ __forceinline__ bool better(int dmode, float v, int j, float bv, int bj) {
    if (!dmode) return v > bv || (v == bv && j < bj);
    const bool nv = v != v, nb = bv != bv;
    if (nv || nb) return nv && (!nb || j < bj);
    return v < bv || (v == bv && j < bj);
}

// ---- the A phase: the wave's 2 x 32 frame-0 rows (rbase + 32 g + i of the block), fp32 ->
//      int8.  Loaded COALESCED: 16 lanes per row, lane sub = lane & 15 holds floats 4 (sub +
//      16 u) .. +3 (u < 4), so every load instruction reads 256 contiguous bytes of 4 rows.  Per
//      row (a 16-lane reduction): m = max |a_k|, q = RN(127 RN(1/m)), s_a = RN(m RN(1/127)) --
//      |1 - q s_a| < 2^-21, the window's A term -- |a|^2 and the range check; the codes go to
//      the wave's row-major int8 image in LDS (img: 8 KiB, 16-B chunks swizzled by row) and
//      come back in the i8 MFMA A layout (lane l: row l & 31, k = 32 s + 16 (l >> 5) .. +15).
//      rowv[r] = (|a|^2, s_a); s_a < 0 marks a row for the exact path (non-finite, zero or out
//      of range).  AI8 (sequence mode): the rows arrive already quantised by k_q8_split (q0,
//      s0, |a|^2, pair flag bad0) and are copied (256 B per row). ----
//      NG: 32-row groups (RG = 2 for the 64-row waves; k_q8t_match's 128-row waves take 4).
//      (Measured and not kept, round 4: the row's own quantisation residual |rho| measured here for
//      the epilogue's A term instead of the worst case 8 s_a -- 0.7 % faster near the threshold,
//      3 % slower on the headline.)
template <bool AI8, int QB = 4, int NG = RG>  // QB: row quads (4 loads per lane each) in flight
__device__ __forceinline__ void a_phase(char *img, float2 *rowv, int rbase, int row0, int n0, int lane,
                                        const float *__restrict__ A, const char *__restrict__ QA,
                                        const float *__restrict__ s0p, const float *__restrict__ na2p, bool bad0,
                                        i32x4 (&aI)[NG][KD / 32]) {
    const int fr = lane & 31, fh = lane >> 5;
    const int sub = lane & 15, rq = lane >> 4;
#pragma unroll
    for (int g = 0; g < NG; g++) {
        if constexpr (AI8) {
            // lane sub holds chunk sub (k = 16 sub .. +15) of row 4 qd + rq, stored at the
            // swizzled chunk the readback expects
            i32x4 v[8];
#pragma unroll
            for (int qd = 0; qd < 8; qd++) {
                const int ga = min(row0 + rbase + g * 32 + 4 * qd + rq, n0 - 1);
                v[qd] = *reinterpret_cast<const i32x4 *>(QA + (size_t)ga * KD + 16 * sub);
            }
            if (lane < 32) {
                const int ga = min(row0 + rbase + g * 32 + lane, n0 - 1);
                const float sa = s0p[ga], q2 = na2p[ga];
                // the in-register path's range rule on m = 127 s_a, conservatively; zero rows too
                const bool afull = bad0 || !(q2 <= FLT_MAX) || !(sa >= SCALE_LO) || !(sa <= SCALE_HI * (1.f / 128.f));
                rowv[rbase + g * 32 + lane] = make_float2(q2, afull ? -1.f : sa);
            }
#pragma unroll
            for (int qd = 0; qd < 8; qd++) {
                const int r = 4 * qd + rq;
                *reinterpret_cast<i32x4 *>(img + r * KD + ((sub ^ (r & 15)) << 4)) = v[qd];
            }
        } else {
#pragma unroll
            for (int qd0 = 0; qd0 < 8; qd0 += QB) {
                f32x4v x[QB][4];
#pragma unroll
                for (int qd = 0; qd < QB; qd++) {
                    const float *ar = A + (size_t)min(row0 + rbase + g * 32 + 4 * (qd0 + qd) + rq, n0 - 1) * KD;
#pragma unroll
                    for (int u = 0; u < 4; u++) x[qd][u] = *reinterpret_cast<const f32x4v *>(ar + 4 * (sub + 16 * u));
                }
#pragma unroll
                for (int qd = 0; qd < QB; qd++) {
                    const int r = 4 * (qd0 + qd) + rq;  // row within the group
                    float m = 0.f, qa = 0.f, qb = 0.f;
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        m = absmax3(m, x[qd][u][0], x[qd][u][1]);
                        m = absmax3(m, x[qd][u][2], x[qd][u][3]);
                        qa = __builtin_fmaf(x[qd][u][0], x[qd][u][0], qa);
                        qb = __builtin_fmaf(x[qd][u][1], x[qd][u][1], qb);
                        qa = __builtin_fmaf(x[qd][u][2], x[qd][u][2], qa);
                        qb = __builtin_fmaf(x[qd][u][3], x[qd][u][3], qb);
                    }
                    float q2 = qa + qb;
                    m = fmaxf(m, swz_xor<1>(m));
                    q2 += swz_xor<1>(q2);
                    m = fmaxf(m, swz_xor<2>(m));
                    q2 += swz_xor<2>(q2);
                    m = fmaxf(m, swz_xor<4>(m));
                    q2 += swz_xor<4>(q2);
                    m = fmaxf(m, swz_xor<8>(m));
                    q2 += swz_xor<8>(q2);
                    const float q = m > 0.f ? 127.f * __builtin_amdgcn_rcpf(m) : 0.f;
                    const bool afull = !(q2 <= FLT_MAX) || m < SCALE_LO || m > SCALE_HI;  // zero rows too
                    if (sub == 0) rowv[rbase + g * 32 + r] = make_float2(q2, afull ? -1.f : m * (1.f / 127.f));
                    char *rowp = img + r * KD + 4 * (sub & 3);
#pragma unroll
                    for (int u = 0; u < 4; u++)  // k = 4 sub + 64 u: chunk (sub >> 2) + 4 u
                        *reinterpret_cast<int *>(rowp + ((((sub >> 2) + 4 * u) ^ (r & 15)) << 4)) =
                            pack4(x[qd][u][0], x[qd][u][1], x[qd][u][2], x[qd][u][3], q);
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own image writes
#pragma unroll
        for (int s2 = 0; s2 < KD / 32; s2++)
            aI[g][s2] = *reinterpret_cast<const i32x4 *>(img + fr * KD + (((2 * s2 + fh) ^ (fr & 15)) << 4));
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the reads complete before the next group's writes
    }
}

// a_phase<false, QB, NG> with the loads software-pipelined: batch b + 1's QB row quads are issued
// before batch b is quantised (two register sets of QB x 4 f32x4), across the group boundaries, so
// a wave always has 2 QB quads in flight instead of alternating between loading and quantising.
template <int QB, int NG>
__device__ __forceinline__ void a_phase_pipe(char *img, float2 *rowv, int rbase, int row0, int n0, int lane,
                                             const float *__restrict__ A, i32x4 (&aI)[NG][KD / 32]) {
    const int fr = lane & 31, fh = lane >> 5;
    const int sub = lane & 15, rq = lane >> 4;
    constexpr int NB = NG * 8 / QB;  // batches of QB quads (8 quads = 32 rows per group)
    f32x4v xs[2][QB][4];
    auto load = [&](int bt, f32x4v (&x)[QB][4]) {
#pragma unroll
        for (int qd = 0; qd < QB; qd++) {
            const int rr = bt * QB * 4 + 4 * qd + rq;  // row within the wave's NG * 32
            const float *ar = A + (size_t)min(row0 + rbase + rr, n0 - 1) * KD;
#pragma unroll
            for (int u = 0; u < 4; u++) x[qd][u] = *reinterpret_cast<const f32x4v *>(ar + 4 * (sub + 16 * u));
        }
    };
    load(0, xs[0]);
#pragma unroll
    for (int bt = 0; bt < NB; bt++) {
        if (bt + 1 < NB) load(bt + 1, xs[(bt + 1) & 1]);
        const int g = bt * QB / 8;
#pragma unroll
        for (int qd = 0; qd < QB; qd++) {
            const f32x4v(&x)[4] = xs[bt & 1][qd];
            const int r = (bt * QB + qd) % 8 * 4 + rq;  // row within the group
            float m = 0.f, qa = 0.f, qb = 0.f;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                m = absmax3(m, x[u][0], x[u][1]);
                m = absmax3(m, x[u][2], x[u][3]);
                qa = __builtin_fmaf(x[u][0], x[u][0], qa);
                qb = __builtin_fmaf(x[u][1], x[u][1], qb);
                qa = __builtin_fmaf(x[u][2], x[u][2], qa);
                qb = __builtin_fmaf(x[u][3], x[u][3], qb);
            }
            float q2 = qa + qb;
            m = fmaxf(m, swz_xor<1>(m));
            q2 += swz_xor<1>(q2);
            m = fmaxf(m, swz_xor<2>(m));
            q2 += swz_xor<2>(q2);
            m = fmaxf(m, swz_xor<4>(m));
            q2 += swz_xor<4>(q2);
            m = fmaxf(m, swz_xor<8>(m));
            q2 += swz_xor<8>(q2);
            const float q = m > 0.f ? 127.f * __builtin_amdgcn_rcpf(m) : 0.f;
            const bool afull = !(q2 <= FLT_MAX) || m < SCALE_LO || m > SCALE_HI;  // zero rows too
            if (sub == 0) rowv[rbase + g * 32 + r] = make_float2(q2, afull ? -1.f : m * (1.f / 127.f));
            char *rowp = img + r * KD + 4 * (sub & 3);
#pragma unroll
            for (int u = 0; u < 4; u++)  // k = 4 sub + 64 u: chunk (sub >> 2) + 4 u
                *reinterpret_cast<int *>(rowp + ((((sub >> 2) + 4 * u) ^ (r & 15)) << 4)) =
                    pack4(x[u][0], x[u][1], x[u][2], x[u][3], q);
        }
        if ((bt + 1) * QB % 8 == 0) {  // group g complete in the image: back in the MFMA layout
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own image writes
#pragma unroll
            for (int s2 = 0; s2 < KD / 32; s2++)
                aI[g][s2] = *reinterpret_cast<const i32x4 *>(img + fr * KD + (((2 * s2 + fh) ^ (fr & 15)) << 4));
            __builtin_amdgcn_s_waitcnt(0xc07f);  // the reads complete before the next group's writes
        }
    }
}

// ---- the epilogue (wave-local): per row the 32 lanes' (m1, m2) are merged through LDS (lanes
//      fr and fr + 32 end with row fr's (M, E, M2)), then the row is decided in its two lanes;
//      rare wide rows are re-scored by the whole wave.  epi = the block's epilogue LDS
//      (epi_bytes<NW>()), free of every other use.  Bn, Eb: upper bounds of max |b_j| and
//      max |eps_j| over the pair's columns; flagged: every row of the pair takes the exact
//      path.  tb, tkeep: the tag width and mask of the sweep.
//      IK = false: m1/m2 hold tagged float screen values (the tag moves a value by < 2^(tb-23)
//      relative: the rho term), a column's real screen = value * s_a.  IK = true: they hold the
//      bits of exact integer keys (D_eff << tb) | tag, real screen = (key >> tb) * s_a * bscale;
//      padding columns (index >= n1, zero codes) are excluded by index. ----
template <int NW, bool IK = false>
__device__ __forceinline__ void epilogue(char *epi, const float2 *rowv, float (&m1)[RG][16], float (&m2)[RG][16],
                                         double Bn, double Eb, bool flagged, int tb, unsigned tkeep, int w, int lane,
                                         int row0, int n0, int n1, const float *__restrict__ A,
                                         const float *__restrict__ B, int *__restrict__ oidx,
                                         float *__restrict__ oscore, double thresh, int dmode, double bscale = 1.0,
                                         const unsigned char *colsh = nullptr) {
    const int fr = lane & 31, fh = lane >> 5;
    const double u24 = 5.9604644775390625e-08;
    const double gam_e = KD * u24 / (1.0 - KD * u24);
    const double rho = IK ? 0.0 : ldexp(1.0, tb - 23);
    // key order and value: float compares of the tagged screen values, or signed-int compares of
    // the key bits
    auto kgt = [](float a, float b) { return IK ? __float_as_int(a) > __float_as_int(b) : a > b; };
    auto kmax = [&](float a, float b) { return kgt(a, b) ? a : b; };
    auto kmin = [&](float a, float b) { return kgt(a, b) ? b : a; };
    auto kval = [&](float a) { return IK ? (double)(__float_as_int(a) >> tb) : (double)a; };
    const float kneg = IK ? __int_as_float((int)0x80000000) : -__builtin_inff();
    auto kcol = [&](float a, int lanecol) {  // the column of a tagged value held by lane column lanecol
        const unsigned tg = __float_as_uint(a) & ~tkeep;
        return (int)(tg >> 1) * BN + (int)(tg & 1) * 32 + lanecol;
    };
    // dmode 1: distinct dots can round to one distance: columns within TIE of the maximiser's
    // exact dot are competitors (a distance tie needs |d1 - d2| of a few ulp)
    const double tie = dmode ? 1e-5 : 0.0;
    char *mt = epi + w * 32 * MT_STRIDE;
    int *clist = reinterpret_cast<int *>(epi + NW * 32 * MT_STRIDE);
    unsigned *lmask = reinterpret_cast<unsigned *>(epi + NW * 32 * MT_STRIDE + NW * 64 * NCAND * 4);
    static_assert(RG == 2, "the deferred re-scores put group g on lane half g");
    unsigned wide_rows[RG];
    float bs_g[RG];
    int bj_g[RG], need_g[RG];  // need_g: the maximiser's column when its exact score is deferred, else -1
    bool out_g[RG];            // this lane writes the row (fh == 0, live, not wide)
#pragma unroll
    for (int g = 0; g < RG; g++) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int r = (q & 3) + 8 * (q >> 2) + 4 * fh;  // 32x32 C/D row map
            float2 v;
            v.x = m1[g][q];
            v.y = m2[g][q];
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
        float M = kneg, M2 = kneg;
        int E = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {  // equal maxima land in M2: ambiguous
            M2 = kmax(kmax(M2, e2[i]), kmin(M, e1[i]));
            E = kgt(e1[i], M) ? fh * 16 + i : E;
            M = kmax(M, e1[i]);
        }
        {
            const float oM = __shfl_xor(M, 32, 64), oM2 = __shfl_xor(M2, 32, 64);
            const int oE = __shfl_xor(E, 32, 64);
            M2 = kmax(kmax(M2, oM2), kmin(M, oM));
            E = (kgt(oM, M) || (!kgt(M, oM) && oE < E)) ? oE : E;
            M = kmax(M, oM);
        }
        // the mt region is rewritten by the next group: its reads must have completed
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)

        const int rl = w * 64 + g * 32 + fr;
        const bool live = row0 + rl < n0;
        const float2 rv = rowv[rl];
        const bool full = flagged || rv.y < 0.f;
        const float *arow = A + (size_t)(row0 + rl) * KD;
        float bs = dmode ? __builtin_inff() : -__builtin_inff();
        int bj = 0x7fffffff, need = -1;
        bool wide = live && full;
        if (wide && fh == 0) lmask[rl] = 0xffffffffu;
        if (live && !full) {
            const double s_a = (double)rv.y;
            const double an = sqrt(fmax((double)rv.x, 0.0)) * 1.0001;
            // |eps_a| <= s_a |rho| + |1 - q s_a| |a| (|1 - q s_a| < 2^-21), |rho| <= 8
            const double ea = 8.001 * s_a + 4.76837158203125e-07 * an;
            const double dq = (an * Eb + ea * Bn + ea * Eb) * 1.0001;
            const double delta = dq + u24 * (an * Bn + dq) * 1.01 + gam_e * an * Bn + 1e-30;
            const double sa_k = s_a * bscale;  // screen units -> units of a.b
            const double Ms = kval(M) * sa_k;
            const double M2s = kgt(M2, kneg) ? kval(M2) * sa_k : -__builtin_inf();
            const double dp = delta + 2.2 * rho * (fabs(Ms) + 2.0 * delta);
            // colsh (IK): the window of the maximiser's own column I -- its 1 / q_I instead of the
            // pair's max (Eb = 8 max_j 1 / q_j): |e_I - screen_I| <= dpI, every other column keeps
            // dp.  So: no match when M + dpI <= thresh and M2 + dp <= thresh (no other column can
            // clear it); competitors reach M - dpI - dp; sure when M - dpI > thresh
            double dpI = dp;
            if (IK && colsh && !dmode) {
                const int I0 = kcol(M, E);
                if (I0 < n1) {
                    const int eI = tb + 2 - (int)colsh[I0];
                    const double EbI = 8.0001 * (double)__builtin_ldexpf(1.f / 127.f, -eI) + 1e-30;
                    const double dqI = (an * EbI + ea * Bn + ea * EbI) * 1.0001;
                    dpI = fmin(dp, dqI + u24 * (an * Bn + dqI) * 1.01 + gam_e * an * Bn + 1e-30);
                }
            }
            // competitors: columns whose exact score can reach the maximiser's; for the distance
            // (dmode 1) also every column that can clip to 1 with it (distance-0 ties), and a
            // maximiser that can clip to -1 ties every column (all distances 2)
            const double lo = dmode ? fmin(Ms - 2.0 * dp, 1.0 - dp) - tie : Ms - dpI - dp;
            if (dmode && Ms - dp <= -1.0 + tie) {
                wide = true;
                if (fh == 0) lmask[rl] = 0xffffffffu;
            } else if (Ms + dpI > thresh || M2s + dp > thresh) {
                if (M2s < lo) {
                    const int I = kcol(M, E);
                    if (I >= n1) {  // a padding column on top (IK: all real dots below 0); never read past n1
                        wide = true;
                        if (fh == 0) lmask[rl] = 0xffffffffu;
                    } else {
                        // decision-only (no score output): every exact score inside the window
                        // clears both tests -- the maximiser's exact dot decides nothing
                        const bool sure = !oscore && (dmode || Ms - dpI > fmax(thresh, 0.0));
                        if (!sure) {
                            need = I;  // scored below, after both groups, by lane half g
                        } else if (fh == 0) {
                            bs = dmode ? 0.f : FLT_MAX;
                            bj = I;
                        }
                    }
                } else {  // both lanes of the row take this branch
                    const double lim = lo / sa_k;  // in screen units
                    const float pad_hi = -1.0e38f;  // float: padding columns (past n1) sit at -3e38
                    unsigned in1 = 0, in2 = 0;
#pragma unroll
                    for (int i = 0; i < 16; i++) {  // padding columns (past n1) are never candidates
                        in1 |= (kval(e1[i]) >= lim && (IK || e1[i] > pad_hi) && kcol(e1[i], fh * 16 + i) < n1 ? 1u : 0u)
                               << i;
                        in2 |= (kval(e2[i]) >= lim && (IK || e2[i] > pad_hi) && kcol(e2[i], fh * 16 + i) < n1 ? 1u : 0u)
                               << i;
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
                            if ((in1 >> i) & 1u) clist[rl * NCAND + k++] = kcol(e1[i], fh * 16 + i);
                        const int nc = __popc(inside);
                        for (int c = fh; c < nc; c += 2) {  // the row's two lanes split the list
                            const int j = clist[rl * NCAND + c];
                            if ((unsigned)j >= (unsigned)n1) continue;  // an LDS-held index: checked
                            const float *ap = arow;
                            asm volatile("" : "+v"(ap));  // keep the A row's loads inside the loop
                            const float e = exact_dot(ap, B + (size_t)j * KD);
                            const float v = dmode ? dist(e) : e;
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
        bs_g[g] = bs;
        bj_g[g] = bj;
        need_g[g] = need;
        out_g[g] = fh == 0 && live && !wide;
        wide_rows[g] = (unsigned)__ballot(fh == 0 && wide);
    }

    // ---- the maximisers' exact scores: lane (fr, fh) takes row fr of group fh, so the two
    //      groups' sequential 256-term dots (and their row loads) run side by side instead of one
    //      after the other on half the lanes ----
    {
        const int Ih = fh ? need_g[1] : need_g[0];
        float e = 0.f;
        if (__ballot(Ih >= 0))  // wave-uniform; the wave's own transpose slice is free by now
            e = coop_exact_dots(A, B, row0 + w * 64 + fh * 32 + fr, Ih, lane, mt);
        const float eo = __shfl_xor(e, 32, 64);
        const float e0 = fh ? eo : e, e1 = fh ? e : eo;
#pragma unroll
        for (int g = 0; g < RG; g++)
            if (need_g[g] >= 0) {
                const float eg = g ? e1 : e0;
                bs_g[g] = dmode ? dist(eg) : eg;
                bj_g[g] = need_g[g];
            }
    }
#pragma unroll
    for (int g = 0; g < RG; g++)
        if (out_g[g]) {
            const int rl = w * 64 + g * 32 + fr;
            const float bs = bs_g[g];
            const int bj = bj_g[g];
            const bool keep = bj != 0x7fffffff && (dmode || ((double)bs > thresh && bs > 0.f));
            oidx[rl] = keep ? bj : -1;
            if (oscore) oscore[rl] = keep ? bs : 0.f;
        }

    // ---- wide rows (rare): the wave scores every column of every listed lane exactly, one
    //      column per lane at a time (lane l: columns f + 32 (l + 64 i) of inside lane f) ----
#pragma unroll
    for (int g = 0; g < RG; g++)
        for (unsigned dm = wide_rows[g]; dm; dm &= dm - 1) {
            const int r = w * 64 + g * 32 + __builtin_ctz(dm);
            const float *a = A + (size_t)(row0 + r) * KD;
            float ws = dmode ? __builtin_inff() : -__builtin_inff();
            int wj = 0x7fffffff;
            for (unsigned Lm = lmask[r]; Lm; Lm &= Lm - 1) {
                const int f = __builtin_ctz(Lm);
                for (int j = f + 32 * lane; j < n1; j += 32 * 64) {
                    const float *ap = a;
                    asm volatile("" : "+v"(ap));
                    const float e = exact_dot(ap, B + (size_t)j * KD);
                    const float v = dmode ? dist(e) : e;
                    if (better(dmode, v, j, ws, wj)) {
                        ws = v;
                        wj = j;
                    }
                }
            }
#define Q8_WRED(O)                                                                           \
            do {                                                                             \
                const float ob = O == 32 ? __shfl_xor(ws, 32, 64) : swz_xor<O & 31>(ws);     \
                const int oj = O == 32 ? __shfl_xor(wj, 32, 64) : swz_xor<O & 31>(wj);       \
                if (better(dmode, ob, oj, ws, wj)) {                                         \
                    ws = ob;                                                                 \
                    wj = oj;                                                                 \
                }                                                                            \
            } while (0)
            Q8_WRED(1);
            Q8_WRED(2);
            Q8_WRED(4);
            Q8_WRED(8);
            Q8_WRED(16);
            Q8_WRED(32);
#undef Q8_WRED
            if (lane == 0) {
                const bool keep = wj != 0x7fffffff && (dmode || ((double)ws > thresh && ws > 0.f));
                oidx[r] = keep ? wj : -1;
                if (oscore) oscore[r] = keep ? ws : 0.f;
            }
        }
}

}  // namespace q8
