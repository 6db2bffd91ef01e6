// k_allpairs_f32.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659)
// with the gemmini_functions_cpu.h:14-56 summation order as the exact score.
//
// Two kernels per launch:
//   k_ap_screen   S = D0 . D1^T with v_mfma_f32_32x32x2_f32 (exact f32 FMA chain,
//                 k permuted), 128x128 tile per 256-thread block, K = 256 staged
//                 through LDS in BK = 32 slices; epilogue reduces every row of the
//                 tile to (max1, idx1, max2) and also publishes max_j |d1_j|^2.
//   k_ap_resolve  one lane per query row: M = max over tiles, rounding bound
//                 delta = 2 gamma_256 |a| max|b| (both the MFMA chain and the
//                 sequential sum are within gamma_256 sum|a_k b_k| of the real
//                 dot), then an EXACT sequential re-score (v_mul_f32 + v_add_f32,
//                 k = 0..255) of every column whose screen score is >= M - 2 delta
//                 -- that set provably contains every possible maximiser -- and
//                 the reference's rule: first j with the maximum, kept when > thresh.
// Bound: the screen is FP32-MFMA bound (2*256 FLOP per score, 157 TF/s chip);
// per pair 2*1024*1024*256 = 536.9 MFLOP on 2 x 1 MiB of descriptors.
#include <math.h>

#include "mv_internal.hpp"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, KD = 256;
constexpr int LDK = BK + 4;        // padded staging row: 144 B -> conflict-free ds_read_b128
constexpr int LDC = BM + 4;        // transposed score tile Ct[col][row]
constexpr int STAGE_FLOATS = 2 * BM * LDK;
constexpr int C_FLOATS = BN * LDC;
constexpr int LDS_FLOATS = STAGE_FLOATS > C_FLOATS ? STAGE_FLOATS : C_FLOATS;

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Partial {
    float max1;
    int idx1;
    float max2;
    float pad;
};

__device__ __forceinline__ void triple_push(float v, int j, float &m1, int &i1, float &m2) {
    if (v > m1) {
        m2 = m1;
        m1 = v;
        i1 = j;
    } else if (v > m2) {
        m2 = v;
    }
}

// XCD-aware bijective remap: blocks b and b+8 share an XCD (dispatch is
// round-robin); give each XCD a contiguous run of logical tiles so the 64
// tiles of one pair (2 MiB of descriptors) share one 4 MiB L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int q = total / 8, r = total % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__global__ __launch_bounds__(256, 2) void k_ap_screen(int tiles_r, int tiles_c, int cap,
                                                      const int *__restrict__ n0v, const int *__restrict__ n1v,
                                                      const float *__restrict__ desc0,
                                                      const float *__restrict__ desc1, Partial *__restrict__ part,
                                                      unsigned *__restrict__ bmax2) {
    __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
    float *As = lds;
    float *Bs = lds + BM * LDK;

    const int per_pair = tiles_r * tiles_c;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int pair = L / per_pair;
    const int tile = L % per_pair;
    const int tr = tile / tiles_c, tc = tile % tiles_c;
    const int n0 = n0v[pair], n1 = n1v[pair];
    if (tr * BM >= n0 || tc * BN >= n1) return;

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w >> 1, wc = w & 1;
    const float *A = desc0 + (size_t)pair * cap * KD;
    const float *B = desc1 + (size_t)pair * cap * KD;

    // staging map: element idx = it*256 + t -> row idx/8, float4 column idx%8
    const int srow = t >> 3, sc4 = t & 7;
    // one staged row per it = 0..3: rows it*32 + srow (named registers, no arrays)
    const int ao0 = min(tr * BM + 0 * 32 + srow, n0 - 1) * KD + sc4 * 4;
    const int ao1 = min(tr * BM + 1 * 32 + srow, n0 - 1) * KD + sc4 * 4;
    const int ao2 = min(tr * BM + 2 * 32 + srow, n0 - 1) * KD + sc4 * 4;
    const int ao3 = min(tr * BM + 3 * 32 + srow, n0 - 1) * KD + sc4 * 4;
    const int bo0 = min(tc * BN + 0 * 32 + srow, n1 - 1) * KD + sc4 * 4;
    const int bo1 = min(tc * BN + 1 * 32 + srow, n1 - 1) * KD + sc4 * 4;
    const int bo2 = min(tc * BN + 2 * 32 + srow, n1 - 1) * KD + sc4 * 4;
    const int bo3 = min(tc * BN + 3 * 32 + srow, n1 - 1) * KD + sc4 * 4;
    float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
    float bsq0 = 0.f, bsq1 = 0.f, bsq2 = 0.f, bsq3 = 0.f;
#define AP_GLOAD(kt)                                                                   \
    do {                                                                               \
        ra0 = *reinterpret_cast<const float4 *>(A + ao0 + (kt) * BK);                 \
        ra1 = *reinterpret_cast<const float4 *>(A + ao1 + (kt) * BK);                 \
        ra2 = *reinterpret_cast<const float4 *>(A + ao2 + (kt) * BK);                 \
        ra3 = *reinterpret_cast<const float4 *>(A + ao3 + (kt) * BK);                 \
        rb0 = *reinterpret_cast<const float4 *>(B + bo0 + (kt) * BK);                 \
        rb1 = *reinterpret_cast<const float4 *>(B + bo1 + (kt) * BK);                 \
        rb2 = *reinterpret_cast<const float4 *>(B + bo2 + (kt) * BK);                 \
        rb3 = *reinterpret_cast<const float4 *>(B + bo3 + (kt) * BK);                 \
    } while (0)
#define AP_ST1(it, ra, rb, bsq)                                                        \
    do {                                                                               \
        *reinterpret_cast<float4 *>(As + ((it) * 32 + srow) * LDK + sc4 * 4) = ra;    \
        *reinterpret_cast<float4 *>(Bs + ((it) * 32 + srow) * LDK + sc4 * 4) = rb;    \
        bsq += rb.x * rb.x + rb.y * rb.y + rb.z * rb.z + rb.w * rb.w;                 \
    } while (0)
#define AP_LSTORE()                                                                    \
    do {                                                                               \
        AP_ST1(0, ra0, rb0, bsq0);                                                     \
        AP_ST1(1, ra1, rb1, bsq1);                                                     \
        AP_ST1(2, ra2, rb2, bsq2);                                                     \
        AP_ST1(3, ra3, rb3, bsq3);                                                     \
    } while (0)

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int g = 0; g < 16; g++) acc[i][j][g] = 0.f;

    // fragment read map (k permuted: lane half h takes k = h*16 + s at MFMA step s)
    const int fr = lane & 31, fh = lane >> 5;
    const float *a_frag = As + (wr * 64 + fr) * LDK + fh * 16;
    const float *b_frag = Bs + (wc * 64 + fr) * LDK + fh * 16;

    AP_GLOAD(0);
    AP_LSTORE();
    __syncthreads();
    constexpr int KT = KD / BK;
    for (int kt = 0; kt < KT; kt++) {
        if (kt + 1 < KT) {
            AP_GLOAD(kt + 1);
        }
#pragma unroll
        for (int v = 0; v < 4; v++) {  // 4 k-steps of 2 per ds_read_b128
            const float4 a0 = *reinterpret_cast<const float4 *>(a_frag + v * 4);
            const float4 a1 = *reinterpret_cast<const float4 *>(a_frag + 32 * LDK + v * 4);
            const float4 b0 = *reinterpret_cast<const float4 *>(b_frag + v * 4);
            const float4 b1 = *reinterpret_cast<const float4 *>(b_frag + 32 * LDK + v * 4);
            const float av[2][4] = {{a0.x, a0.y, a0.z, a0.w}, {a1.x, a1.y, a1.z, a1.w}};
            const float bv[2][4] = {{b0.x, b0.y, b0.z, b0.w}, {b1.x, b1.y, b1.z, b1.w}};
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int n = 0; n < 2; n++)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][s], bv[n][s], acc[m][n], 0, 0, 0);
        }
        __syncthreads();
        if (kt + 1 < KT) {
            AP_LSTORE();
            __syncthreads();
        }
    }

#undef AP_GLOAD
#undef AP_ST1
#undef AP_LSTORE
    // ---- max |b_j|^2 over this tile's columns (8 lanes share a staged row) ----
    float bm = 0.f;
#pragma unroll
    for (int it = 0; it < 4; it++) {
        float v = it == 0 ? bsq0 : it == 1 ? bsq1 : it == 2 ? bsq2 : bsq3;
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        bm = fmaxf(bm, v);
    }
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) bm = fmaxf(bm, __shfl_xor(bm, o, 64));
    if (tr == 0 && lane == 0) atomicMax(&bmax2[pair], __float_as_uint(bm));

    // ---- scores -> LDS, transposed: Ct[col][row] (C/D map: col = lane&31,
    //      row = (g&3) + 8*(g>>2) + 4*(lane>>5)) ----
    float *Ct = lds;
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int col = wc * 64 + n * 32 + fr;
                const int row = wr * 64 + m * 32 + 8 * q + 4 * fh;
                float4 v = make_float4(acc[m][n][4 * q + 0], acc[m][n][4 * q + 1], acc[m][n][4 * q + 2],
                                       acc[m][n][4 * q + 3]);
                *reinterpret_cast<float4 *>(Ct + col * LDC + row) = v;
            }
    __syncthreads();

    // ---- per-row (max1, idx1, max2) over the tile's valid columns ----
    const int r = t & (BM - 1), half = t >> 7;
    const int cvalid = min(BN, n1 - tc * BN);
    float m1 = -__builtin_inff(), m2 = -__builtin_inff();
    int i1 = -1;
    const int cb = half * 64, ce = min(cb + 64, cvalid);
    for (int c = cb; c < ce; c++) triple_push(Ct[c * LDC + r], tc * BN + c, m1, i1, m2);
    __syncthreads();
    float *mx = lds;  // reuse: [128] m1, [128] i1, [128] m2 of the upper half
    if (half == 1) {
        mx[r] = m1;
        reinterpret_cast<int *>(mx)[BM + r] = i1;
        mx[2 * BM + r] = m2;
    }
    __syncthreads();
    if (half == 0) {
        const float u1 = mx[r], u2 = mx[2 * BM + r];
        const int ui = reinterpret_cast<int *>(mx)[BM + r];
        if (u1 > m1) {
            m2 = fmaxf(m1, u2);
            m1 = u1;
            i1 = ui;
        } else {
            m2 = fmaxf(m2, u1);
        }
        const int grow = tr * BM + r;
        if (grow < n0) {
            Partial p;
            p.max1 = m1;
            p.idx1 = i1;
            p.max2 = m2;
            p.pad = 0.f;
            part[((size_t)pair * cap + grow) * tiles_c + tc] = p;
        }
    }
}

// exact score in the reference order: s = 0; s = s + a[k]*b[k], k = 0..255
__device__ __forceinline__ float exact_dot(const float *__restrict__ a, const float *__restrict__ b) {
    float s = 0.f;
#pragma unroll 4
    for (int k = 0; k < KD; k += 4) {
        float4 x = *reinterpret_cast<const float4 *>(a + k);
        float4 y = *reinterpret_cast<const float4 *>(b + k);
        s = __fadd_rn(s, __fmul_rn(x.x, y.x));
        s = __fadd_rn(s, __fmul_rn(x.y, y.y));
        s = __fadd_rn(s, __fmul_rn(x.z, y.z));
        s = __fadd_rn(s, __fmul_rn(x.w, y.w));
    }
    return s;
}

__global__ __launch_bounds__(256) void k_ap_resolve(int tiles_c, int cap, const int *__restrict__ n0v,
                                                    const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                    const float *__restrict__ desc1,
                                                    const Partial *__restrict__ part,
                                                    const unsigned *__restrict__ bmax2, double thresh,
                                                    int *__restrict__ match_idx, float *__restrict__ match_score) {
    const int pair = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= cap) return;
    const int n0 = n0v[pair], n1 = n1v[pair];
    int best = -1;
    float bs = 0.f;
    if (i < n0 && n1 > 0) {
        const float *a = desc0 + ((size_t)pair * cap + i) * KD;
        const float *B = desc1 + (size_t)pair * cap * KD;
        const Partial *p = part + ((size_t)pair * cap + i) * tiles_c;
        const int tiles = (n1 + BN - 1) / BN;
        float M = -__builtin_inff();
        for (int tt = 0; tt < tiles; tt++) M = fmaxf(M, p[tt].max1);
        float na2 = 0.f;
        for (int k = 0; k < KD; k += 4) {
            float4 x = *reinterpret_cast<const float4 *>(a + k);
            na2 += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
        }
        const double u = 5.9604644775390625e-08;  // 2^-24
        const double gamma = KD * u / (1.0 - KD * u);
        const double nb = sqrt((double)__uint_as_float(bmax2[pair]));
        const double delta = 2.0 * gamma * sqrt((double)na2) * nb * 1.01 + 1e-30;
        if ((double)M + delta > thresh) {
            const double win = (double)M - 2.0 * delta;
            for (int tt = 0; tt < tiles; tt++) {
                const Partial q = p[tt];
                if ((double)q.max2 >= win) {  // ambiguous tile: re-score all of its columns
                    const int je = min(tt * BN + BN, n1);
                    for (int j = tt * BN; j < je; j++) {
                        float e = exact_dot(a, B + (size_t)j * KD);
                        if ((double)e > thresh && e > bs) {
                            bs = e;
                            best = j;
                        }
                    }
                } else if ((double)q.max1 >= win) {
                    const int j = q.idx1;
                    float e = exact_dot(a, B + (size_t)j * KD);
                    if ((double)e > thresh && e > bs) {
                        bs = e;
                        best = j;
                    }
                }
            }
        }
    }
    match_idx[(size_t)pair * cap + i] = best;
    match_score[(size_t)pair * cap + i] = best >= 0 ? bs : 0.f;
}

}  // namespace

namespace mv {

size_t allpairs_f32_scratch_bytes(int batch, int cap) {
    const int tiles_c = (cap + BN - 1) / BN;
    return align_up(sizeof(Partial) * (size_t)batch * cap * tiles_c, 256) + align_up(sizeof(unsigned) * batch, 256);
}

int launch_allpairs_f32(hipStream_t s, void *scratch, int batch, int cap, const int *n0, const int *n1,
                        const float *desc0, const float *desc1, double thresh, int *match_idx,
                        float *match_score) {
    MV_REQUIRE(batch > 0 && cap > 0 && n0 && n1 && desc0 && desc1 && match_idx && match_score && scratch);
    MV_REQUIRE(((uintptr_t)desc0 & 15) == 0 && ((uintptr_t)desc1 & 15) == 0);
    const int tiles_r = (cap + BM - 1) / BM, tiles_c = (cap + BN - 1) / BN;
    Partial *part = (Partial *)scratch;
    unsigned *bmax2 =
        (unsigned *)((char *)scratch + align_up(sizeof(Partial) * (size_t)batch * cap * tiles_c, 256));
    MV_HIP_TRY(hipMemsetAsync(bmax2, 0, sizeof(unsigned) * batch, s));
    const long blocks = (long)batch * tiles_r * tiles_c;
    MV_REQUIRE(blocks < (1l << 31));
    MV_PROF_BEGIN(s, "k_ap_screen");
    hipLaunchKernelGGL(k_ap_screen, dim3((unsigned)blocks), dim3(256), 0, s, tiles_r, tiles_c, cap, n0, n1, desc0,
                       desc1, part, bmax2);
    MV_PROF_END(s);
    MV_LAUNCH_CHECK();
    MV_PROF_BEGIN(s, "k_ap_resolve");
    hipLaunchKernelGGL(k_ap_resolve, dim3((cap + 255) / 256, batch), dim3(256), 0, s, tiles_c, cap, n0, n1, desc0,
                       desc1, part, bmax2, thresh, match_idx, match_score);
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
    void *scr = mv::scratch(ctx, mv::allpairs_f32_scratch_bytes(batch, cap));
    if (!scr) return MV_ERR_OUT_OF_MEMORY;
    return mv::launch_allpairs_f32(ctx->stream, scr, batch, cap, n0, n1, desc0, desc1, thresh, match_idx,
                                   match_score);
}
