// k_allpairs_q8.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659) with
// the gemmini_functions_cpu.h:14-56 summation order as the exact score, screened on the INT8
// matrix cores (twice the fp16 rate, a quarter of the fp32 bytes per streamed column).
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
//               exact integer dot D_ij becomes the screen f_ij = RN(D_ij s_j) in one FMA
//               (accumulators start at the bits of 2^23), tagged with its column tile in the
//               low mantissa bits and folded into a lane-local top-2 per row.  Epilogue: as the
//               fp16 screen's (k_allpairs_f32.hip), with the quantisation window below.
//
// Why the result is exact.  With a = q_a s_a + eps_a, b = q_b s_b + eps_b (real arithmetic,
// s the float scales actually used), d = a.b (real) and D = q_a.q_b (exact integer):
//   d - s_a s_b D = a.eps_b + eps_a.b - eps_a.eps_b,
//   |d - s_a s_b D| <= |a| Eb + |eps_a| Bn + |eps_a| Eb =: dq     (Cauchy-Schwarz)
// with Bn = max_j |b_j|, Eb = max_j |eps_j| over the pair's columns (k_q8_split), and
// |eps_a| <= 8 s_a + 2^-22 |a| (RNE of x * RN(127/m): |x - q s_a| <= s_a / 2 + 2^-23 |x|; the
// fp32 norms carry a 1e-4 safety factor).  The screen in real units, s_a f = s_a RN(D s_b),
// adds 2^-24 (|a| Bn + dq); the reference's sequential fp32 sum e adds gamma_256(2^-24)|a| Bn.
// So |s_a f_j - e_j| <= delta for every column, and the fp16 kernel's argument carries over
// verbatim: a runner-up below M - 2 delta' leaves the screen maximiser as the reference's
// maximiser (ties included), one exact dot decides the threshold (none when the window lies
// entirely above it and no score is asked for); otherwise the columns inside the window are
// re-scored exactly.  Negative dots leave the accumulator below 2^23 (t = 2^23 + D/2): their
// screen is D s_b / 2 >= D s_b, i.e. never below the truth -- the window stays conservative.
// Bound: HBM (A fp32 1 KiB per row) and int8 MFMA; per pair 2 n0 n1 256 algorithmic ops.
#include <float.h>
#include <math.h>

#include "mv_internal.hpp"

namespace {

constexpr int KD = 256;
// timing experiments only (wrong results): Q8_EXP_NOFOLD (one of 16 rows folded)
#ifndef Q8_EXP_NOFOLD
#define Q8_EXP_NOFOLD 0
#endif
#ifndef Q8_QB
#define Q8_QB 4  // row quads of frame 0 in flight per wave in the A phase (4 loads per lane each)
#endif
#ifndef Q8_PF
#define Q8_PF 2  // k32 steps of B fragments read ahead of the MFMAs
#endif
#ifdef Q8_EXP_TRACE
constexpr int Q8_TRACE_BLOCKS = 8192;
__device__ unsigned long long g_q8_trace[Q8_TRACE_BLOCKS * 4 * 10];
#define Q8_STAMP(K) do { __builtin_amdgcn_sched_barrier(0); ts_[K] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define Q8_STAMP(K) do { } while (0)
#endif
#ifndef Q8_STAGGER
#define Q8_STAGGER 0  // > 0: first-generation second-slot blocks start this many 100-MHz ticks late
#endif
constexpr int Q_NW = 4, Q_NT = 64 * Q_NW, Q_RG = 2, Q_BM = 32 * Q_RG * Q_NW, Q_BN = 64, Q_NBUF = 4;
constexpr int Q_TILE = Q_BN * KD;                  // 16 KiB: one int8 column tile, whole K
constexpr int Q_SLOT = Q_TILE + Q_BN * 4;          // + the tile's 64 scales s_j
constexpr int Q_OFF_MISC = Q_NBUF * Q_SLOT;        // [2][NW] f32 per-wave max |b|^2, |eps|^2
constexpr int Q_OFF_ROW = Q_OFF_MISC + 2 * Q_NW * 4;  // [BM] float2 per row (|a|^2, s_a; s_a < 0: exact path)
constexpr int Q_OFF_TEXP = Q_OFF_ROW + 2 * 32 * Q_RG * Q_NW * 4;  // [16] i32 tile exponents (integer fold)
constexpr int Q_LDS = Q_OFF_TEXP + 16 * 4;
constexpr int QI_TB = 5, QI_SHR = 4;  // integer fold: tag bits (<= 16 tiles), exponent span (2^22 << 9 < 2^31)
constexpr int QI_NONE = -100000;      // exponent of an all-zero tile
constexpr int MT_STRIDE = 32 * 8 + 16;             // epilogue transpose row: 32 (m1, m2) + pad
constexpr int Q_NCAND = 16;                        // listed candidates per row (more: wide row)
constexpr int Q_OFF_CL = Q_NW * 32 * MT_STRIDE;    // epilogue, inside the ring: [BM][NCAND]
constexpr int Q_OFF_LM = Q_OFF_CL + Q_BM * Q_NCAND * 4;  // [BM] wide rows' inside lanes
static_assert(Q_OFF_LM + Q_BM * 4 <= Q_NBUF * Q_SLOT, "epilogue fits the ring");
static_assert(2 * Q_LDS <= 160 * 1024, "two blocks per CU");
constexpr float MAGIC_RNE = 12582912.f;  // 1.5 * 2^23: fma(x, q, MAGIC) = MAGIC + RNE(x q), |x q| < 2^22
constexpr float SCALE_LO = 9.094947017729282e-13f, SCALE_HI = 1099511627776.f;  // 2^-40, 2^40

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total / 8, r = total % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

#pragma clang diagnostic ignored "-Winline-asm"
template <int DOFF>
__device__ __forceinline__ void glds16_q8(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_add_u32 m0, %2, %3\n\t"
        "global_load_lds_dwordx4 %0, %1"
        :
        : "v"(voff), "s"(sbase), "s"(lds_byte), "i"(DOFF)
        : "memory", "m0", "scc");
}
template <int DOFF>
__device__ __forceinline__ void glds4_q8(const void *sbase, unsigned voff, unsigned lds_byte) {
    asm volatile(
        "s_add_u32 m0, %2, %3\n\t"
        "global_load_lds_dword %0, %1"
        :
        : "v"(voff), "s"(sbase), "s"(lds_byte), "i"(DOFF)
        : "memory", "m0", "scc");
}
template <int N>
__device__ __forceinline__ void wait_vm_q8() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
typedef float f2q __attribute__((ext_vector_type(2)));
#ifndef Q8_PKFMA
#define Q8_PKFMA 0  // 1: dequantise two rows per v_pk_fma_f32 (measured 2.47 vs 2.42 ms: not kept)
#endif
// d = a * r + c on both halves (one issue): v_pk_fma_f32, inline so it is never scalarised
__device__ __forceinline__ f2q pkfma_q8(f2q a, f2q r, f2q c) {
    f2q d;
    asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(r), "v"(c));
    return d;
}
// the tagged top-2 fold on integer keys held in the float registers' bits
__device__ __forceinline__ void fold3_i8k(int a, int b, float &m1f, float &m2f) {
    int md, m1 = __float_as_int(m1f), m2 = __float_as_int(m2f);
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(md) : "v"(m1), "v"(a), "v"(b));
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(m1) : "v"(m1), "v"(a), "v"(b));
    asm("v_max_i32 %0, %1, %2" : "=v"(m2) : "v"(m2), "v"(md));
    m1f = __int_as_float(m1);
    m2f = __int_as_float(m2);
}
__device__ __forceinline__ float tag_q8(float f, unsigned keep, unsigned tag) {
    float r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(keep), "s"(tag));
    return r;
}
// an integer-fold key -> the float path's tagged screen value: tag = column tag (2 tc + half),
// D = the integer dot, f = D 2^e_t exactly (|D| < 2^22), its low tb bits replaced by the tag
// as tag_q8 does; keys below every real one (tile -1, INT_MIN) -> -inf
__device__ __forceinline__ float q8_key_value(int key, const int *texp, int e_base, unsigned keep) {
    if (key < (int)0x82000000) return -__builtin_inff();  // |real keys| <= 127^2 256 2^9 < 2^31 - 2^25
    const unsigned tag = (unsigned)key & ((1u << QI_TB) - 1u);
    const int e = texp[tag >> 1];
    const int sh = e == QI_NONE ? 0 : e - e_base;
    const int d = (key >> QI_TB) >> sh;
    const float f = e == QI_NONE ? 0.f : ldexpf((float)d, e);
    return __uint_as_float((__float_as_uint(f) & keep) | tag);
}
__device__ __forceinline__ void fold3_q8(float a, float b, float &m1, float &m2) {
    float md;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(md) : "v"(m1), "v"(a), "v"(b));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m1) : "v"(m1), "v"(a), "v"(b));
    asm("v_max_f32 %0, %1, %2" : "=v"(m2) : "v"(m2), "v"(md));
}
// max(m, |a|, |b|) in one instruction (no NaN canonicalisation: NaN is caught by the norm)
__device__ __forceinline__ float absmax3(float m, float a, float b) {
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
template <int M>
__device__ __forceinline__ float swz_xor_q8(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (M << 10) | 0x1F));
}
template <int M>
__device__ __forceinline__ int swz_xor_q8(int v) {
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
// the integer fold's chain start: C = 0 (inline constant)
__device__ __forceinline__ i32x16 mfma_i8_from0(i32x4 a, i32x4 b) {
    i32x16 d;
    asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
    return d;
}
// key = (D << sh) | tag: the integer fold's dequantisation (tile scale 2^e_t relative to the
// pair's base exponent) and column tag in one instruction; sh in a VGPR, the tag in an SGPR
// (a VOP3 reads one SGPR)
__device__ __forceinline__ int lshl_or_v_q8(int d, int sh, unsigned tag) {
    int r;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(d), "v"(sh), "s"(tag));
    return r;
}
// four int8 RNE(x q) packed into a dword (byte i = element i): the magic sum's low byte is
// the two's-complement integer
__device__ __forceinline__ int pack4_q8(float x0, float x1, float x2, float x3, float q) {
    const unsigned f0 = __float_as_uint(__builtin_fmaf(x0, q, MAGIC_RNE));
    const unsigned f1 = __float_as_uint(__builtin_fmaf(x1, q, MAGIC_RNE));
    const unsigned f2 = __float_as_uint(__builtin_fmaf(x2, q, MAGIC_RNE));
    const unsigned f3 = __float_as_uint(__builtin_fmaf(x3, q, MAGIC_RNE));
    const unsigned p01 = __builtin_amdgcn_perm(f1, f0, 0x0c0c0400u);
    const unsigned p23 = __builtin_amdgcn_perm(f3, f2, 0x0c0c0400u);
    return (int)__builtin_amdgcn_perm(p23, p01, 0x05040100u);
}

// The reference's sequential fp32 dot (mul then add, k = 0..255), 4 load batches per operand.
__device__ __forceinline__ float exact_dot_q8(const float *__restrict__ a, const float *__restrict__ b) {
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
// nn_match_two_way's distance (pairwise_pnp.py:303): sqrt(2 - 2 clip(dot, -1, 1)) in float32
__device__ __forceinline__ float dist_q8(float e) {
    const float c = e != e ? e : fminf(fmaxf(e, -1.f), 1.f);
    return sqrtf(__fsub_rn(2.f, __fmul_rn(2.f, c)));
}
// dmode 0: larger dot, ties to the smaller index (NaN never wins); dmode 1: np.argmin
__device__ __forceinline__ bool better_q8(int dmode, float v, int j, float bv, int bj) {
    if (!dmode) return v > bv || (v == bv && j < bj);
    const bool nv = v != v, nb = bv != bv;
    if (nv || nb) return nv && (!nb || j < bj);
    return v < bv || (v == bv && j < bj);
}

// ---- k_q8_split: 16 lanes per row (lane sub holds floats 4 (sub + 16 u) .. +3, u < 4: every
//      load instruction reads 256 contiguous bytes of 4 rows), QS_RPG rows per lane group in
//      flight; a 256-thread block strides over the batch (rows >= n1 are never read
//      downstream and are not written) ----
#ifndef Q8_INTFOLD
#define Q8_INTFOLD 0  // 1: integer fold for pairs with whole 64-column tiles (bit-exact; measured no faster yet)
#endif
#ifndef QS_RPG
#define QS_RPG (Q8_INTFOLD ? 4 : 2)  // Q8_INTFOLD: one pass = one 64-row tile
#endif
static_assert(!Q8_INTFOLD || QS_RPG == 4, "tile mode stages whole 64-row tiles per pass");
#ifndef QS_GRID
#define QS_GRID (256 * 64)
#endif
constexpr int QS_ROWS = 16 * QS_RPG;
#ifndef Q8_FUSE_HEAD
#define Q8_FUSE_HEAD 0
#endif
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
    // tile mode (Q8_INTFOLD): the pass's 64 rows are one 64-column tile of one pair whose n1 is a
    // multiple of 64 -- their codes share one power-of-two scale (the integer fold's input)
    const int pair0 = (int)(min(R0, rows - 1) / cap);
    const bool tile_mode = Q8_INTFOLD && (cap & 63) == 0 && (min(max(n1v[pair0], 0), cap) & 63) == 0;
    float tile_max = 0.f;
    if (Q8_INTFOLD) {
        __shared__ float s_tmax[16];
        float mm = 0.f;
#pragma unroll
        for (int r = 0; r < QS_RPG; r++) {
            float m = 0.f;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                m = absmax3(m, x[r][u][0], x[r][u][1]);
                m = absmax3(m, x[r][u][2], x[r][u][3]);
            }
            const long R = R0 + 16 * r + rg;
            const bool live = R < rows && (int)(c[r] - (long)(c[r] / cap) * cap) < n1v[c[r] / cap];
            mm = fmaxf(mm, live ? m : 0.f);
        }
        mm = fmaxf(mm, swz_xor_q8<1>(mm));
        mm = fmaxf(mm, swz_xor_q8<2>(mm));
        mm = fmaxf(mm, swz_xor_q8<4>(mm));
        mm = fmaxf(mm, swz_xor_q8<8>(mm));
        if (sub == 0) s_tmax[rg] = mm;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; i++) tile_max = fmaxf(tile_max, s_tmax[i]);
        __syncthreads();  // s_tmax is rewritten by the next pass
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
        m = fmaxf(m, swz_xor_q8<1>(m));
        m = fmaxf(m, swz_xor_q8<2>(m));
        m = fmaxf(m, swz_xor_q8<4>(m));
        m = fmaxf(m, swz_xor_q8<8>(m));
        q2 += swz_xor_q8<1>(q2);
        q2 += swz_xor_q8<2>(q2);
        q2 += swz_xor_q8<4>(q2);
        q2 += swz_xor_q8<8>(q2);
        float q = m > 0.f ? 127.f / m : 0.f;
        float s = m / 127.f;
        float mr = m;  // the magnitude the range check sees
        if (tile_mode) {  // one power-of-two scale 2^e >= M / 127 for the tile's 64 rows
            const float M = tile_max;
            int ex;
            (void)frexpf(M, &ex);  // M < 2^ex
            const int e = ldexpf(127.f, ex - 7) >= M ? ex - 7 : ex - 6;
            s = M > 0.f ? ldexpf(1.f, e) : 0.f;
            q = M > 0.f ? ldexpf(1.f, -e) : 0.f;
            mr = M;
        }
        int pk[4];
        float e2 = 0.f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            pk[u] = pack4_q8(x[r][u][0], x[r][u][1], x[r][u][2], x[r][u][3], q);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float v = __builtin_fmaf(x[r][u][e], q, MAGIC_RNE) - MAGIC_RNE;  // exact
                const float ep = __builtin_fmaf(-v, s, x[r][u][e]);
                e2 = __builtin_fmaf(ep, ep, e2);
            }
        }
        e2 += swz_xor_q8<1>(e2);
        e2 += swz_xor_q8<2>(e2);
        e2 += swz_xor_q8<4>(e2);
        e2 += swz_xor_q8<8>(e2);
        // finite (|b|^2 propagates NaN / inf) and a representable scale (zero rows: s = 0,
        // q = 0, every screen value of the column 0 -- exact, no flag needed)
        const bool ok = q2 <= FLT_MAX && (mr == 0.f || (mr >= SCALE_LO && mr <= SCALE_HI));
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
#ifdef Q8_EXP_TRACE
    unsigned long long ts_[8] = {};
    Q8_STAMP(0);
#endif
#if Q8_STAGGER > 0
    if (blockIdx.x >= 256 && blockIdx.x < 512) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)Q8_STAGGER) __builtin_amdgcn_s_sleep(8);
    }
#endif
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
    const int ntc = flagged ? 0 : (n1 + Q_BN - 1) / Q_BN;  // a flagged pair skips the screen

    // Bn^2 = max |b_j|^2, Eb^2 = max |eps_j|^2 over the pair's columns (published by the
    // prologue barrier)
    {
        const float *p2 = nb2v + (size_t)pair * cap, *e2 = eb2v + (size_t)pair * cap;
        float bm = 0.f, em = 0.f;
        for (int j = t; j < n1; j += Q_NT) {
            bm = fmaxf(bm, p2[j]);
            em = fmaxf(em, e2[j]);
        }
        bm = fmaxf(bm, swz_xor_q8<1>(bm));
        bm = fmaxf(bm, swz_xor_q8<2>(bm));
        bm = fmaxf(bm, swz_xor_q8<4>(bm));
        bm = fmaxf(bm, swz_xor_q8<8>(bm));
        bm = fmaxf(bm, swz_xor_q8<16>(bm));
        em = fmaxf(em, swz_xor_q8<1>(em));
        em = fmaxf(em, swz_xor_q8<2>(em));
        em = fmaxf(em, swz_xor_q8<4>(em));
        em = fmaxf(em, swz_xor_q8<8>(em));
        em = fmaxf(em, swz_xor_q8<16>(em));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        em = fmaxf(em, __shfl_xor(em, 32, 64));
        if (lane == 0) {
            misc[w] = bm;
            misc[Q_NW + w] = em;
        }
        // integer fold: each tile's scale exponent (tile t's rows all hold 2^e_t), published by
        // the barrier after the A phase
        if (Q8_INTFOLD && t < 16) {
            int ex = QI_NONE;
            if (t < ntc) {
                const float st = sb[t * Q_BN];
                if (st > 0.f) {
                    (void)frexpf(st, &ex);
                    ex -= 1;  // st = 2^(ex - 1)
                }
            }
            reinterpret_cast<int *>(lds + Q_OFF_TEXP)[t] = ex;
        }
    }

    // ---- B DMA map (as k_i8_match): wave w fills rows w*16 .. +15 of a tile, 4 rows (1 KiB)
    //      per instruction; lane l -> row (l >> 4), chunk position l & 15, source chunk
    //      (l & 15) ^ (row & 15); plus the tile's 64 scales (every wave the same 256 B, so
    //      all waves count 5 loads per tile) ----
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int dr = wu * 16 + (lane >> 4);
    const unsigned dcb = (unsigned)((lane & 15) ^ (dr & 15)) * 16;
    unsigned oB[4], oR;
    const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)lds;
    const unsigned dst_w = lds_base + (unsigned)(wu * 16 * KD);
#define Q8_STAGE(SLOT)                                                                       \
    do {                                                                                     \
        glds16_q8<(SLOT) * Q_SLOT>(QB, oB[0], dst_w);                                        \
        glds16_q8<(SLOT) * Q_SLOT + 4 * KD>(QB, oB[1], dst_w);                               \
        glds16_q8<(SLOT) * Q_SLOT + 8 * KD>(QB, oB[2], dst_w);                               \
        glds16_q8<(SLOT) * Q_SLOT + 12 * KD>(QB, oB[3], dst_w);                              \
        glds4_q8<(SLOT) * Q_SLOT + Q_TILE>(sb, oR, lds_base);                                \
    } while (0)
#define Q8_OFFSETS(TC)                                                                       \
    do {                                                                                     \
        const int nb_ = (TC) * Q_BN + dr;                                                    \
        _Pragma("unroll") for (int g_ = 0; g_ < 4; g_++)                                     \
            oB[g_] = (unsigned)min(nb_ + 4 * g_, n1 - 1) * KD + (dcb ^ (64u * g_));          \
        oR = (unsigned)min((TC) * Q_BN + lane, n1 - 1) * 4;                                  \
    } while (0)
    // prologue DMA: tiles 0, 1 into slots 0, 1 -- issued before the A rows are read so both
    // latencies overlap (slots 2, 3 hold the A images meanwhile; tile 2 follows the A phase)
    for (int g = 0; g < 2 && g < ntc; g++) {
        Q8_OFFSETS(g);
        if (g == 0) Q8_STAGE(0);
        if (g == 1) Q8_STAGE(1);
    }

    // ---- A: the wave's 2 x 32 rows (w*64 + 32 g + i), fp32 -> int8.  Loaded COALESCED: 16
    //      lanes per row, lane sub = lane & 15 holds floats 4 (sub + 16 u) .. +3 (u < 4), so every
    //      load instruction reads 256 contiguous bytes of 4 rows.  Per row (a 16-lane
    //      reduction): m = max |a_k|, q = RN(127 RN(1/m)), s_a = RN(m RN(1/127)) -- |1 - q s_a|
    //      < 2^-21, the window's A term -- |a|^2 and the range check; the codes go to the wave's
    //      row-major int8 image in LDS (ring slots 2-3, 16-B chunks swizzled by row) and come back
    //      in the i8 MFMA A layout (lane l: row l & 31, k = 32 s + 16 (l >> 5) .. +15).  (Loading
    //      the MFMA layout directly -- each lane its own row in 16-B pieces at 128-B stride --
    //      asks the memory pipeline for every line four times.) ----
    const int fr = lane & 31, fh = lane >> 5;
    i32x4 aI[Q_RG][KD / 32];
    // per-row epilogue inputs go to LDS (not live in VGPRs across the sweep)
    float2 *rowv = reinterpret_cast<float2 *>(lds + Q_OFF_ROW);
    {
        char *img = lds + 2 * Q_SLOT + w * 32 * KD;  // 8 KiB per wave, one row group at a time
        const int sub = lane & 15, rq = lane >> 4;
        constexpr int QB = Q8_QB;  // row quads (4 QB loads per lane) in flight
#pragma unroll
        for (int g = 0; g < Q_RG; g++) {
            if constexpr (AI8) {
                // the group's 32 rows of the split image: lane sub holds chunk sub (k = 16 sub ..
                // +15) of row 4 qd + rq, stored at the swizzled chunk the readback expects
                const char *QA = q0 + (size_t)pair * cap * KD;
                i32x4 v[8];
#pragma unroll
                for (int qd = 0; qd < 8; qd++) {
                    const int ga = min(row0 + w * 64 + g * 32 + 4 * qd + rq, n0 - 1);
                    v[qd] = *reinterpret_cast<const i32x4 *>(QA + (size_t)ga * KD + 16 * sub);
                }
                if (lane < 32) {  // row lane of the group: |a|^2 and s_a (< 0: exact path)
                    const size_t ga = (size_t)pair * cap + min(row0 + w * 64 + g * 32 + lane, n0 - 1);
                    const float sa = s0v[ga], q2 = na2v[ga];
                    // the in-register path's range rule on m = 127 s_a, conservatively; zero rows too
                    const bool afull = bad0[pair] != 0 || !(q2 <= FLT_MAX) || !(sa >= SCALE_LO) ||
                                       !(sa <= SCALE_HI * (1.f / 128.f));
                    rowv[w * 64 + g * 32 + lane] = make_float2(q2, afull ? -1.f : sa);
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
                    const float *ar = A + (size_t)min(row0 + w * 64 + g * 32 + 4 * (qd0 + qd) + rq, n0 - 1) * KD;
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
                    m = fmaxf(m, swz_xor_q8<1>(m));
                    q2 += swz_xor_q8<1>(q2);
                    m = fmaxf(m, swz_xor_q8<2>(m));
                    q2 += swz_xor_q8<2>(q2);
                    m = fmaxf(m, swz_xor_q8<4>(m));
                    q2 += swz_xor_q8<4>(q2);
                    m = fmaxf(m, swz_xor_q8<8>(m));
                    q2 += swz_xor_q8<8>(q2);
                    const float q = m > 0.f ? 127.f * __builtin_amdgcn_rcpf(m) : 0.f;
                    const bool afull = !(q2 <= FLT_MAX) || m < SCALE_LO || m > SCALE_HI;  // zero rows too: exact path
                    if (sub == 0) rowv[w * 64 + g * 32 + r] = make_float2(q2, afull ? -1.f : m * (1.f / 127.f));
                    char *rowp = img + r * KD + 4 * (sub & 3);
#pragma unroll
                    for (int u = 0; u < 4; u++)  // k = 4 sub + 64 u: chunk (sub >> 2) + 4 u
                        *reinterpret_cast<int *>(rowp + ((((sub >> 2) + 4 * u) ^ (r & 15)) << 4)) =
                            pack4_q8(x[qd][u][0], x[qd][u][1], x[qd][u][2], x[qd][u][3], q);
                }
            }
            }  // !AI8
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own image writes
#pragma unroll
            for (int s2 = 0; s2 < KD / 32; s2++)
                aI[g][s2] = *reinterpret_cast<const i32x4 *>(img + fr * KD + (((2 * s2 + fh) ^ (fr & 15)) << 4));
            __builtin_amdgcn_s_waitcnt(0xc07f);  // the reads complete before the next group's writes
        }
    }
    __syncthreads();  // every wave's image is read: slot 2 takes tile 2
    if (ntc > 2) {
        Q8_OFFSETS(2);
        Q8_STAGE(2);
    }

    Q8_STAMP(1);
    // B fragment: column block c (0, 1), lane row 32 c + fr, k32 step s: chunk (2 s + fh)
    const int rdb = fr * KD;
    const int xsw = fh ^ (fr & 15);  // chunk (2 s + fh) ^ (fr & 15) = 2 s ^ xsw

    // Accumulators start at the bits of 4.0 (0x40800000, an inline constant of the MFMA's C
    // operand: no registers): t = 4 + D 2^-21 as a float (|D| <= 127^2 * 256 < 2^22), so
    // f = fma(t, 2^21 s_j, -2^23 s_j) = RN(D s_j) (the product is exact inside the fma).
    // Columns past n1 (last tile only) get s = 0 and the offset -3e38.  The low tb bits of f
    // are then replaced by the column tag 2 tc + half.
    // The integer fold (Q8_INTFOLD; pairs with whole 64-column tiles, at most 16 of them, whose
    // tile scales 2^e_t span <= 2^QI_SHR): the accumulators start at 0 and each value becomes
    // the key (D << (e_t - e_base + QI_TB)) | tag -- one v_lshl_or_b32 in place of the
    // dequantising FMA and the tag -- folded with v_max3_i32 / v_med3_i32 (|D| < 2^22: the key
    // fits 31 bits).  After the sweep the keys become the float path's tagged values exactly
    // (f = D 2^e_t is exact), so the merge and the decisions are shared.
    const int *texp = reinterpret_cast<const int *>(lds + Q_OFF_TEXP);
    bool int_ok = false;
    int e_base = 0;
    if (Q8_INTFOLD && ntc > 0 && ntc <= 16 && (n1 & (Q_BN - 1)) == 0 && (cap & (Q_BN - 1)) == 0) {
        int emx = QI_NONE, emn = 1 << 30;
        for (int i = 0; i < ntc; i++) {
            const int e = texp[i];
            if (e != QI_NONE) {
                emx = max(emx, e);
                emn = min(emn, e);
            }
        }
        int_ok = emx == QI_NONE || emx - emn <= QI_SHR;
        e_base = emx == QI_NONE ? 0 : emx - QI_SHR;
    }
    i32x16 acc[Q_RG][2];
    float m1[Q_RG][16], m2[Q_RG][16];
    {
        const float minit = int_ok ? __int_as_float((int)0x80000000) : -__builtin_inff();
        const int ainit = int_ok ? -(1 << 22) : 0;  // "tile -1": -3e38 (float) / INT_MIN keys
#pragma unroll
        for (int g = 0; g < Q_RG; g++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                m1[g][q] = minit;
                m2[g][q] = minit;
            }
#pragma unroll
        for (int q = 0; q < 16; q++) {  // "tile -1" of group 1, folded beside tile 0: never a maximum
            acc[1][0][q] = ainit;
            acc[1][1][q] = ainit;
        }
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
#if Q8_PKFMA
    // rows 2 S and 2 S + 1 of a half share the lane's column, hence its scale and offset: one
    // v_pk_fma_f32 (splat operands) dequantises both (adjacent accumulator registers)
#define Q8_FOLD2_F(FG, S, G0, R0, R1, C0, C1)                                                \
    do {                                                                                     \
        const f2q a2_ = pkfma_q8(                                                            \
            f2q{__int_as_float(acc[FG][0][2 * (S)]), __int_as_float(acc[FG][0][2 * (S) + 1])}, (R0), (C0)); \
        const f2q b2_ = pkfma_q8(                                                            \
            f2q{__int_as_float(acc[FG][1][2 * (S)]), __int_as_float(acc[FG][1][2 * (S) + 1])}, (R1), (C1)); \
        _Pragma("unroll") for (int u_ = 0; u_ < 2; u_++) {                                   \
            const int q = 2 * (S) + u_;                                                      \
            if (Q8_EXP_NOFOLD && q != 0) continue;                                           \
            fold3_q8(tag_q8(a2_[u_], vkeep, (G0)), tag_q8(b2_[u_], vkeep, (G0) + 1u), m1[FG][q], m2[FG][q]); \
        }                                                                                    \
    } while (0)
#else
#define Q8_FOLD2_F(FG, S, G0, R0, R1, C0, C1)                                                \
    do {                                                                                     \
        _Pragma("unroll") for (int q = 2 * (S); q < 2 * (S) + 2; q++) {                      \
            if (Q8_EXP_NOFOLD && q != 0) continue;                                           \
            const float a_ = __builtin_fmaf(__int_as_float(acc[FG][0][q]), (R0).x, (C0).x);  \
            const float b_ = __builtin_fmaf(__int_as_float(acc[FG][1][q]), (R1).x, (C1).x);  \
            fold3_q8(tag_q8(a_, vkeep, (G0)), tag_q8(b_, vkeep, (G0) + 1u), m1[FG][q], m2[FG][q]); \
        }                                                                                    \
    } while (0)
#endif
    // the integer fold of rows 2 S, 2 S + 1 of group FG (the tile's shift in shv)
#define Q8_FOLD2_I(FG, S, G0, R0, R1, C0, C1)                                                \
    do {                                                                                     \
        _Pragma("unroll") for (int q = 2 * (S); q < 2 * (S) + 2; q++) {                      \
            const int ka_ = lshl_or_v_q8(acc[FG][0][q], shv, (G0));                          \
            const int kb_ = lshl_or_v_q8(acc[FG][1][q], shv, (G0) + 1u);                     \
            fold3_i8k(ka_, kb_, m1[FG][q], m2[FG][q]);                                       \
        }                                                                                    \
    } while (0)
    // group G's MFMAs on slot J (fragments read PF k32 steps ahead), folding group FG meanwhile
#define Q8_SEG(J, G, FG, G0, R0, R1, C0, C1)                                                 \
    do {                                                                                     \
        constexpr int PF = Q8_PF;                                                            \
        const char *base = lds + (J) * Q_SLOT + rdb;                                         \
        int xs_ = xsw;                                                                       \
        asm volatile("" : "+v"(xs_)); /* per-use offsets: not 8 loop-invariant VGPRs */      \
        i32x4 b0_[KD / 32], b1_[KD / 32];                                                    \
        _Pragma("unroll") for (int s_ = 0; s_ < KD / 32 + PF; s_++) {                        \
            if (s_ < KD / 32) {                                                              \
                const int ch_ = ((2 * s_) ^ xs_) * 16;                                       \
                b0_[s_] = *reinterpret_cast<const i32x4 *>(base + ch_);                      \
                b1_[s_] = *reinterpret_cast<const i32x4 *>(base + 32 * KD + ch_);            \
            }                                                                                \
            if (s_ >= PF) {                                                                  \
                const int m_ = s_ - PF;                                                      \
                if (m_ == 0) {                                                               \
                    acc[G][0] = Q8_MFMA0(aI[G][0], b0_[0]);                                  \
                    acc[G][1] = Q8_MFMA0(aI[G][0], b1_[0]);                                  \
                } else {                                                                     \
                    acc[G][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b0_[m_], acc[G][0], 0, 0, 0); \
                    acc[G][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aI[G][m_], b1_[m_], acc[G][1], 0, 0, 0); \
                }                                                                            \
                Q8_FOLD2(FG, m_, G0, R0, R1, C0, C1);                                        \
            }                                                                                \
        }                                                                                    \
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
        Q8_SEG(J, 0, 1, gp_, pr0, pr1, pc0, pc1);                                            \
        Q8_SCALES(J, tc);                                                                    \
        const unsigned gc_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)tc);              \
        Q8_SEG(J, 1, 0, gc_, pr0, pr1, pc0, pc1);                                            \
        if (ntile < ntc) {                                                                   \
            wait_vm_q8<5 * (Q_NBUF - 2)>();                                                  \
        } else {                                                                             \
            wait_vm_q8<0>();                                                                 \
        }                                                                                    \
        __syncthreads();                                                                     \
    } while (0)

    // tile 0 landed (younger: tiles 1 and 2, 5 ops each)
    if (ntc > 2) {
        wait_vm_q8<10>();
    } else {
        wait_vm_q8<0>();
    }
    __syncthreads();
    Q8_STAMP(2);
    // scales of the tile before, as splat pairs (the packed dequantisation's operands); the
    // integer fold's shift of the tile before (tile -1: any)
    f2q pr0 = {0.f, 0.f}, pr1 = {0.f, 0.f}, pc0 = {-3.0e38f, -3.0e38f}, pc1 = {-3.0e38f, -3.0e38f};
    int shv = QI_SHR + QI_TB;
#define Q8_SWEEP()                                                                           \
    do {                                                                                     \
        for (int T = 0; T < ntc; T += 4) {                                                   \
            Q8_SLOT(0);                                                                      \
            if (T + 1 < ntc) Q8_SLOT(1);                                                     \
            if (T + 2 < ntc) Q8_SLOT(2);                                                     \
            if (T + 3 < ntc) Q8_SLOT(3);                                                     \
        }                                                                                    \
        if (ntc > 0) { /* group 1 of the last tile */                                        \
            const unsigned gl_ = __builtin_amdgcn_readfirstlane(2u * (unsigned)(ntc - 1));   \
            _Pragma("unroll") for (int s = 0; s < 8; s++) Q8_FOLD2(1, s, gl_, pr0, pr1, pc0, pc1); \
        }                                                                                    \
    } while (0)
    if (Q8_INTFOLD && int_ok) {
#define Q8_FOLD2 Q8_FOLD2_I
#define Q8_MFMA0 mfma_i8_from0
#define Q8_SCALES(J, TC)                                                                     \
    do {                                                                                     \
        const int e_ = texp[TC];                                                             \
        shv = (e_ == QI_NONE ? 0 : e_ - e_base) + QI_TB;                                     \
    } while (0)
        Q8_SWEEP();
#undef Q8_FOLD2
#undef Q8_MFMA0
#undef Q8_SCALES
        // keys -> the float path's tagged values (exact: f = D 2^e_t), for the shared merge
#pragma unroll
        for (int g = 0; g < Q_RG; g++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                m1[g][q] = q8_key_value(__float_as_int(m1[g][q]), texp, e_base, vkeep);
                m2[g][q] = q8_key_value(__float_as_int(m2[g][q]), texp, e_base, vkeep);
            }
    } else {
#define Q8_FOLD2 Q8_FOLD2_F
#define Q8_MFMA0 mfma_i8_from4
#define Q8_SCALES(J, TC)                                                                     \
    do {                                                                                     \
        const float *rl_ = reinterpret_cast<const float *>(lds + (J) * Q_SLOT + Q_TILE);     \
        const int col_ = (TC) * Q_BN + fr;                                                   \
        const float s0_ = rl_[fr], s1_ = rl_[fr + 32];                                       \
        const float r0_ = col_ < n1 ? 2097152.0f * s0_ : 0.f;                                \
        const float r1_ = col_ + 32 < n1 ? 2097152.0f * s1_ : 0.f;                           \
        const float c0_ = col_ < n1 ? -8388608.0f * s0_ : -3.0e38f;                          \
        const float c1_ = col_ + 32 < n1 ? -8388608.0f * s1_ : -3.0e38f;                     \
        pr0 = f2q{r0_, r0_};                                                                 \
        pr1 = f2q{r1_, r1_};                                                                 \
        pc0 = f2q{c0_, c0_};                                                                 \
        pc1 = f2q{c1_, c1_};                                                                 \
    } while (0)
        Q8_SWEEP();
#undef Q8_FOLD2
#undef Q8_MFMA0
#undef Q8_SCALES
    }
    Q8_STAMP(3);
#undef Q8_STAGE
#undef Q8_OFFSETS
#undef Q8_FOLD2_F
#undef Q8_FOLD2_I
#undef Q8_SWEEP
#undef Q8_SEG
#undef Q8_SLOT

    // ---- epilogue (wave-local; the ring is free: the sweep's last barrier follows a full drain) ----
    float bmax2 = misc[0], emax2 = misc[Q_NW];
#pragma unroll
    for (int k = 1; k < Q_NW; k++) {
        bmax2 = fmaxf(bmax2, misc[k]);
        emax2 = fmaxf(emax2, misc[Q_NW + k]);
    }
    const double u24 = 5.9604644775390625e-08;
    const double gam_e = KD * u24 / (1.0 - KD * u24);
    const double Bn = sqrt((double)bmax2) * 1.0001, Eb = sqrt((double)emax2) * 1.0001 + 1e-30;
    const double rho = ldexp(1.0, tb - 23);
    // dmode 1: distinct dots can round to one distance: columns within TIE of the maximiser's
    // exact dot are competitors (a distance tie needs |d1 - d2| of a few ulp)
    const double tie = dmode ? 1e-5 : 0.0;
    char *mt = lds + w * 32 * MT_STRIDE;
    int *clist = reinterpret_cast<int *>(lds + Q_OFF_CL);
    unsigned *lmask = reinterpret_cast<unsigned *>(lds + Q_OFF_LM);
    unsigned wide_rows[Q_RG];
#pragma unroll
    for (int g = 0; g < Q_RG; g++) {
        // per row, merge the 32 lanes' (m1, m2): transposed through LDS; lanes fr and fr + 32
        // end with row fr's (M, E, M2)
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
        // the mt region is rewritten by the next group: its reads must have completed
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)

        // ---- decide the row in its two lanes (the fp16 kernel's logic, quantisation window) ----
        const int rl = w * 64 + g * 32 + fr;
        const bool live = row0 + rl < n0;
        const float2 rv = rowv[rl];
        const bool full = flagged || rv.y < 0.f;
        const float *arow = A + (size_t)(row0 + rl) * KD;
        float bs = dmode ? __builtin_inff() : -__builtin_inff();
        int bj = 0x7fffffff;
        bool wide = live && full;
        if (wide && fh == 0) lmask[rl] = 0xffffffffu;
        if (live && !full) {
            const double s_a = (double)rv.y;
            const double an = sqrt(fmax((double)rv.x, 0.0)) * 1.0001;
            const double ea = 8.001 * s_a + 4.76837158203125e-07 * an;  // |1 - q s_a| < 2^-21
            const double dq = (an * Eb + ea * Bn + ea * Eb) * 1.0001;
            const double delta = dq + u24 * (an * Bn + dq) * 1.01 + gam_e * an * Bn + 1e-30;
            const double Ms = (double)M * s_a;
            const double M2s = M2 > -__builtin_inff() ? (double)M2 * s_a : -__builtin_inf();
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
                    const int I = (int)(tg >> 1) * Q_BN + (int)(tg & 1) * 32 + E;
                    if (I >= n1) {  // cannot happen for a tagged in-range maximum; never read past n1
                        wide = true;
                        if (fh == 0) lmask[rl] = 0xffffffffu;
                    } else if (fh == 0) {
                        // decision-only (no score output): every exact score inside the window
                        // clears both tests -- the maximiser's exact dot decides nothing
                        const bool sure = !oscore && (dmode || Ms - dp > fmax(thresh, 0.0));
                        if (sure) {
                            bs = dmode ? 0.f : FLT_MAX;
                        } else {
                            const float e = exact_dot_q8(arow, B + (size_t)I * KD);
                            bs = dmode ? dist_q8(e) : e;
                        }
                        bj = I;
                    }
                } else {  // both lanes of the row take this branch
                    const double lim = lo / s_a;  // in screen units
                    const float pad_hi = -1.0e38f;  // padding columns (past n1) are never candidates
                    unsigned in1 = 0, in2 = 0;
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        in1 |= ((double)e1[i] >= lim && e1[i] > pad_hi ? 1u : 0u) << i;
                        in2 |= ((double)e2[i] >= lim && e2[i] > pad_hi ? 1u : 0u) << i;
                    }
                    const unsigned o1 = __shfl_xor(in1, 32, 64), o2 = __shfl_xor(in2, 32, 64);
                    const unsigned inside = fh ? (o1 | (in1 << 16)) : (in1 | (o1 << 16));
                    if ((in2 | o2) || __popc(inside) > Q_NCAND) {
                        wide = true;
                        if (fh == 0) lmask[rl] = inside;
                    } else {
                        int k = fh ? __popc(o1) : 0;
#pragma unroll
                        for (int i = 0; i < 16; i++)
                            if ((in1 >> i) & 1u) {
                                const unsigned tg = __float_as_uint(e1[i]) & ~tkeep;
                                clist[rl * Q_NCAND + k++] = (int)(tg >> 1) * Q_BN + (int)(tg & 1) * 32 + fh * 16 + i;
                            }
                        const int nc = __popc(inside);
                        for (int c = fh; c < nc; c += 2) {  // the row's two lanes split the list
                            const int j = clist[rl * Q_NCAND + c];
                            const float *ap = arow;
                            asm volatile("" : "+v"(ap));  // keep the A row's loads inside the loop
                            const float e = exact_dot_q8(ap, B + (size_t)j * KD);
                            const float v = dmode ? dist_q8(e) : e;
                            if (better_q8(dmode, v, j, bs, bj)) {
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
            if (better_q8(dmode, ob, oj, bs, bj)) {
                bs = ob;
                bj = oj;
            }
        }
        if (fh == 0 && live && !wide) {
            const bool keep = bj != 0x7fffffff && (dmode || ((double)bs > thresh && bs > 0.f));
            oidx[rl] = keep ? bj : -1;
            if (oscore) oscore[rl] = keep ? bs : 0.f;
        }
        wide_rows[g] = (unsigned)__ballot(fh == 0 && wide);
    }

    Q8_STAMP(4);
    // ---- wide rows (rare): the wave scores every column of every listed lane exactly, one
    //      column per lane at a time (lane l: columns f + 32 (l + 64 i) of inside lane f) ----
#pragma unroll
    for (int g = 0; g < Q_RG; g++)
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
                    const float e = exact_dot_q8(ap, B + (size_t)j * KD);
                    const float v = dmode ? dist_q8(e) : e;
                    if (better_q8(dmode, v, j, ws, wj)) {
                        ws = v;
                        wj = j;
                    }
                }
            }
#define Q8_WRED(O)                                                                           \
            do {                                                                             \
                const float ob = O == 32 ? __shfl_xor(ws, 32, 64) : swz_xor_q8<O & 31>(ws);  \
                const int oj = O == 32 ? __shfl_xor(wj, 32, 64) : swz_xor_q8<O & 31>(wj);    \
                if (better_q8(dmode, ob, oj, ws, wj)) {                                      \
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
#ifdef Q8_EXP_TRACE
    Q8_STAMP(5);
    if (lane == 0 && blockIdx.x < Q8_TRACE_BLOCKS) {
        unsigned long long *o = g_q8_trace + ((size_t)blockIdx.x * Q_NW + w) * 10;
        for (int k = 0; k < 6; k++) o[k] = ts_[k];
        o[8] = __smid();
        o[9] = __builtin_amdgcn_s_memrealtime();
    }
#endif
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
    if (Q8_FUSE_HEAD)  // timing switch: the staging share before the tile instead of after it
        for (long R0 = lo; R0 < hi; R0 += QS_ROWS) q8_split_pass(R0, hi, ncap, nn1, ndesc1, nq1, ns1, nnb2, neb2, nbad);
    q8_match_block<AI8>(tiles_r, cap, n0v, n1v, desc0, desc1, q1, s1v, nb2v, eb2v, bad, thresh, dmode, match_idx,
                        match_score, q0, s0v, na2v, bad0);
    if (!Q8_FUSE_HEAD && nrows > 0) {
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

#ifdef Q8_EXP_TRACE
// timing experiment only: per-(block, wave) phase stamps of the last k_q8_match launch
extern "C" int mv_debug_q8_trace(void *host, long bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_q8_trace), (size_t)bytes) == hipSuccess ? 0 : -3;
}
#endif
