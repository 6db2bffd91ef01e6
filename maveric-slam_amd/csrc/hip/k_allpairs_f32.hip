// k_allpairs_f32.hip -- all-pairs fp32 descriptor match (python/pairwise_pnp.py:635-659)
// with the gemmini_functions_cpu.h:14-56 summation order as the exact score.
//
// k_ap_match: ONE kernel per batch.  A 256-thread block owns 128 query rows of one pair and
// sweeps ALL column tiles of the other frame:
//   * S = D0 . D1^T on v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, k permuted), 4 waves
//     in 2x2, 64x64 per wave (4 accumulators of 32x32);
//   * K = 256 streamed in 32-wide slices into a DOUBLE-BUFFERED LDS image by
//     global_load_lds (HBM/L2 -> LDS DMA, no staging VGPRs); the image is XOR-swizzled by
//     16-B chunk (chunk ^ ((row >> 1) & 7)) on the SOURCE address and on the read, which
//     makes the 16-lane ds_read_b128 groups conflict-free; one barrier per slice;
//   * after each 128-column tile every lane folds its accumulators into a lane-local
//     running (max1, idx1, max2) per row -- no LDS epilogue per tile;
//   * |a_i|^2 and max_j |b_j|^2 are accumulated from the MFMA operand fragments;
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

#include "mv_internal.hpp"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, KD = 256, KS = KD / BK;
constexpr int TILE_FLOATS = BM * BK;  // one A or B slice: 128 rows x 128 B, swizzled
// LDS map (a single array -- a second __shared__ object can de-pipeline glds -- byte offsets)
constexpr int OFF_STAGE = 0;                          // [2 buf][A, B][128][32] f32
constexpr int STAGE_BYTES = 2 * 2 * TILE_FLOATS * 4;  // 65,536
constexpr int OFF_ANORM = STAGE_BYTES;                // [128] f32 |a_i|^2
constexpr int OFF_TRIP = OFF_ANORM + BM * 4;          // [2 wc][128] {m1, i1, m2}
constexpr int OFF_AMB = OFF_TRIP + 2 * BM * 12;       // [128] i32 ambiguous rows
constexpr int OFF_MISC = OFF_AMB + BM * 4;            // [4] f32 per-wave max|b|^2, [4] i32 #ambiguous
constexpr int LDS_BYTES = OFF_MISC + 32;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16-B-per-lane HBM/L2 -> LDS DMA (global_load_lds_dwordx4): LDS destination = M0 (wave-
// uniform byte address) + lane * 16.  Issued from inline asm on purpose: the compiler
// cannot tell the two LDS buffers apart and would otherwise drain the DMA (vmcnt(0))
// before the first ds_read of the OTHER buffer; the kernel counts vmcnt itself.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const void *gsrc, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_byte) : "memory", "m0");
}
#pragma clang diagnostic pop

// branch-free (selects only): push value v of column j into the triple when `ok`
__device__ __forceinline__ void push(bool ok, float v, int j, float &m1, int &i1, float &m2) {
    const bool top = ok && (v > m1 || (v == m1 && j < i1));
    const float lo = ok ? fmaxf(m2, v) : m2;
    m2 = top ? m1 : lo;
    m1 = top ? v : m1;
    i1 = top ? j : i1;
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

__device__ __forceinline__ float sum8(float v) {  // sum over the 8 lanes that share a staged row
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    return v;
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

__global__ __launch_bounds__(256, 2) void k_ap_match(int tiles_r, int cap, const int *__restrict__ n0v,
                                                     const int *__restrict__ n1v, const float *__restrict__ desc0,
                                                     const float *__restrict__ desc1, double thresh,
                                                     int *__restrict__ match_idx, float *__restrict__ match_score) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    float *stage_lds = reinterpret_cast<float *>(lds + OFF_STAGE);
    float *anorm2 = reinterpret_cast<float *>(lds + OFF_ANORM);
    float *trip = reinterpret_cast<float *>(lds + OFF_TRIP);
    int *amb = reinterpret_cast<int *>(lds + OFF_AMB);
    float *misc = reinterpret_cast<float *>(lds + OFF_MISC);
    int *namb_p = reinterpret_cast<int *>(lds + OFF_MISC) + 4;

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
    const int nsteps = ((n1 + BN - 1) / BN) * KS;

    // DMA map: wave w fills rows w*32 .. w*32+31 of a slice, 8 rows (1 KiB) per instruction;
    // lane l lands at LDS row (l >> 3), chunk position l & 7, and fetches the global chunk
    // (l & 7) ^ ((row >> 1) & 7) of that row (source-side swizzle, lane-linear LDS writes).
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int drow = lane >> 3;
    float asq0 = 0.f, asq1 = 0.f, bsq0 = 0.f, bsq1 = 0.f, bmax = 0.f;
    const unsigned lds_base =
        (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char *)(lds + OFF_STAGE);
    auto stage = [&](int buf, int gs) {
        const int ks = gs % KS, crow0 = (gs / KS) * BN;
        const unsigned bufa = lds_base + (unsigned)(buf * 2 * TILE_FLOATS) * 4u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = wu * 32 + i * 8 + drow;
            const int c = (lane & 7) ^ ((row >> 1) & 7);
            const float *sa = A + (size_t)min(row0 + row, n0 - 1) * KD + ks * BK + c * 4;
            const float *sb = B + (size_t)min(crow0 + row, n1 - 1) * KD + ks * BK + c * 4;
            const unsigned dst = bufa + (unsigned)((wu * 32 + i * 8) * BK) * 4u;
            glds16(sa, dst);
            glds16(sb, dst + TILE_FLOATS * 4u);
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[m][n][q] = 0.f;
    // running triples, one per row (m, q) of this lane's half, over this lane's columns
    float m1[2][16], m2[2][16];
    int i1[2][16];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            m1[m][q] = -__builtin_inff();
            m2[m][q] = -__builtin_inff();
            i1[m][q] = 0x7fffffff;
        }

    // fragment read map (k permuted: lane half h takes k = h*16 + s at MFMA step s, i.e.
    // chunk h*4 + s/4 of its row); rows +32 share the swizzle ((row >> 1) & 7 unchanged)
    const int fr = lane & 31, fh = lane >> 5;
    const int ra = wr * 64 + fr, rb = wc * 64 + fr;
    const int swa = (ra >> 1) & 7, swb = (rb >> 1) & 7;
    int offa[4], offb[4];
#pragma unroll
    for (int v = 0; v < 4; v++) {
        offa[v] = ra * BK + (((fh * 4 + v) ^ swa) * 4);
        offb[v] = TILE_FLOATS + rb * BK + (((fh * 4 + v) ^ swb) * 4);
    }
    const bool a_norms = wc == 0, b_norms = wr == 0;  // wave-uniform: one wave per row set

    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int g = 0; g < nsteps; g++) {
        const int cur = g & 1;
        if (g + 1 < nsteps) stage(cur ^ 1, g + 1);  // DMA of the next slice overlaps the MFMAs
        const float *base = stage_lds + cur * 2 * TILE_FLOATS;
#pragma unroll
        for (int v = 0; v < 4; v++) {  // 4 float4 fragment reads = 4 k-steps of 2
            const float4 a0 = *reinterpret_cast<const float4 *>(base + offa[v]);
            const float4 a1 = *reinterpret_cast<const float4 *>(base + offa[v] + 32 * BK);
            const float4 b0 = *reinterpret_cast<const float4 *>(base + offb[v]);
            const float4 b1 = *reinterpret_cast<const float4 *>(base + offb[v] + 32 * BK);
            const float av[2][4] = {{a0.x, a0.y, a0.z, a0.w}, {a1.x, a1.y, a1.z, a1.w}};
            const float bv[2][4] = {{b0.x, b0.y, b0.z, b0.w}, {b1.x, b1.y, b1.z, b1.w}};
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int n = 0; n < 2; n++)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][s], bv[n][s], acc[m][n], 0, 0, 0);
            // norms for the rounding bound only (any summation order is fine here)
            if (a_norms && g < KS) {
                asq0 = fmaf(a0.x, a0.x, fmaf(a0.y, a0.y, fmaf(a0.z, a0.z, fmaf(a0.w, a0.w, asq0))));
                asq1 = fmaf(a1.x, a1.x, fmaf(a1.y, a1.y, fmaf(a1.z, a1.z, fmaf(a1.w, a1.w, asq1))));
            }
            if (b_norms) {
                bsq0 = fmaf(b0.x, b0.x, fmaf(b0.y, b0.y, fmaf(b0.z, b0.z, fmaf(b0.w, b0.w, bsq0))));
                bsq1 = fmaf(b1.x, b1.x, fmaf(b1.y, b1.y, fmaf(b1.z, b1.z, fmaf(b1.w, b1.w, bsq1))));
            }
        }
        if ((g % KS) == KS - 1) {
            // column tile done: fold the accumulators into the lane-local triples
            const int tc = g / KS;
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const int col = tc * BN + wc * 64 + n * 32 + fr;
                const bool ok = col < n1;
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int q = 0; q < 16; q++) {
                        push(ok, acc[m][n][q], col, m1[m][q], i1[m][q], m2[m][q]);
                        acc[m][n][q] = 0.f;
                    }
            }
            if (b_norms) {  // |b_col|^2: the two lane halves hold the two k halves
                const float c0 = bsq0 + __shfl_xor(bsq0, 32, 64), c1 = bsq1 + __shfl_xor(bsq1, 32, 64);
                const int col0 = tc * BN + wc * 64 + fr;
                bmax = fmaxf(bmax, fmaxf(col0 < n1 ? c0 : 0.f, col0 + 32 < n1 ? c1 : 0.f));
                bsq0 = bsq1 = 0.f;
            }
            if (a_norms && tc == 0) {
                const float r0 = asq0 + __shfl_xor(asq0, 32, 64), r1 = asq1 + __shfl_xor(asq1, 32, 64);
                if (fh == 0) {
                    anorm2[ra] = r0;
                    anorm2[ra + 32] = r1;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next slice has landed
        __syncthreads();
    }

    // ---- merge the triples: across the 32 lanes of each half, then across the 2 column waves ----
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            float a1 = m1[m][q], a2 = m2[m][q];
            int ai = i1[m][q];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                const float b1 = __shfl_xor(a1, o, 64), b2 = __shfl_xor(a2, o, 64);
                const int bi = __shfl_xor(ai, o, 64);
                merge(a1, ai, a2, b1, bi, b2);
            }
            if (fr == 0) {
                const int row = wr * 64 + m * 32 + (q & 3) + 8 * (q >> 2) + 4 * fh;
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
    const float bmax2 = fmaxf(fmaxf(misc[0], misc[1]), fmaxf(misc[2], misc[3]));

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
    for (int k = w; k < namb; k += 4) {
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
    MV_PROF_BEGIN(s, "k_ap_match");
    hipLaunchKernelGGL(k_ap_match, dim3((unsigned)blocks), dim3(256), 0, s, tiles_r, cap, n0, n1, desc0, desc1,
                       thresh, match_idx, match_score);
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
