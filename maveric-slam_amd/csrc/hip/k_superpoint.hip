// k_superpoint.hip -- the quantized SuperPoint front-end (include/superpoint.h)
// on gfx950: grayscale frames -> int8 semi / desc + scales, bit-identical to the CPU oracle
// (oracle/sp_oracle.c, itself bit-identical to PyTorch's quantized kernels).
//
//   conv1a        fused into conv1b's workgroups: image -> (/ 255, bilinear resize, quantize) in
//                 LDS over the tile + 2 pixels -> conv1a (Cin = 1: 9 taps as three v_dot4_i32_i8
//                 per output channel) + relu over the tile + 1 pixel, written as conv1b's input
//                 tile -- conv1a's 64-channel full-resolution output never reaches HBM.
//   k_sp_conv     every other layer as an implicit GEMM on v_mfma_i32_32x32x32_i8: A = the
//                 layer's weights as MFMA fragments (64 couts per workgroup, prefetched from
//                 L2 four k32 steps ahead), B = 32 pixels x 32 channels of one tap read from the
//                 workgroup's NHWC input tile in LDS (16 x 32 output pixels + halo, 16-B chunks
//                 XOR-swizzled by pixel: conflict-free ds_read_b128).  Wave w owns tile rows
//                 4w .. 4w + 3, i.e. 8 MFMAs (4 pixel rows x 2 cout blocks) per k32 step.
//                 Epilogue: int32 + quantised bias -> fp32 x rs -> round to nearest even ->
//                 clamp (relu) -> the 2 x 2 max pool on the int32 accumulators (requantisation is
//                 monotonic: the max commutes with it) -> NHWC int8, or for the two heads the
//                 Frame layout [cells][C] (cell = gx * rows + gy).
//   k_sp_presence / k_sp_min_gap  run()'s output quantisation (superpoint_inference.py:199-206):
//                 the 256-code presence mask of each head of each frame (32 workgroups per head),
//                 the smallest float gap between its present dequantised values, then every value
//                 rounded to that step, in place.
// Bounds: MFMA i8 (2 x 10.4 GMAC per 192 x 640 frame) with HBM beside it (~16 MB of int8
// activations written and read per frame).
#include <math.h>

#include "mv_internal.hpp"
#include "superpoint.h"

struct mv_superpoint {
    int device;
    void *wdev;           // fragments + packed conv1a weights + quantised biases
    size_t wbytes;
    size_t frag_off[12];  // byte offsets into wdev (layer 0: packed dot4 weights [64][3])
    size_t bq_off[12];    // int32 quantised biases [cout_pad]
    float rs[12];         // requantisation scales
    int cout_pad[12], ns[12];
    float in_inv;         // 1 / (float) in_scale
    float dq_semi, dq_desc;  // the heads' dequantisation scales (float) out_scale
    void *act;            // activation ping-pong buffers
    size_t act_bytes;
    hipEvent_t done;      // recorded after each forward on its stream: the buffers' last use
    bool used;
};

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int SP_NT = 256;          // 4 waves

// Requantisation, bit-identical to clamp(rint((float) a * rs), lo, 127): the product rounded to
// float, + 1.5 * 2^23 rounds it to an integer (round to nearest even) held in the low mantissa
// bits, v_med3_i32 clamps on those bits (monotonic: out-of-range sums clamp to the right end),
// and the code is the low byte (the magic's low byte is 0).  lo_bits: MAGIC_BITS + lo.
constexpr float SP_MAGIC = 12582912.0f;
constexpr int SP_MAGIC_BITS = 0x4B400000;
__device__ __forceinline__ int requant_bits(int a, float rs, int lo_bits) {
    const float f = (float)a * rs;
    const int bits = __float_as_int(f + SP_MAGIC);
    return max(min(bits, SP_MAGIC_BITS + 127), lo_bits);
}
// the same from the exact integer already held as a float (conv1a on the f16 matrix cores)
__device__ __forceinline__ int requant_bitsf(float a, float rs, int lo_bits) {
    const float f = a * rs;
    const int bits = __float_as_int(f + SP_MAGIC);
    return max(min(bits, SP_MAGIC_BITS + 127), lo_bits);
}
// four at once (the packed v_pk_mul_f32 / v_pk_add_f32 form measured 1-3 % slower)
__device__ __forceinline__ void requant4(int (&v)[4], int a0, int a1, int a2, int a3, float rs, int lo_bits) {
    v[0] = requant_bits(a0, rs, lo_bits);
    v[1] = requant_bits(a1, rs, lo_bits);
    v[2] = requant_bits(a2, rs, lo_bits);
    v[3] = requant_bits(a3, rs, lo_bits);
}
// low bytes of four requantised words -> one dword
// The 4 packed dwords a lane holds of one 32-channel block (channels 8 qq + 4 fh .. +3, qq = 0..3:
// the MFMA's row layout) regrouped across the lane pair (l, l ^ 32) into 16 CONTIGUOUS channels
// 16 fh .. +15 by two v_permlane32_swap (lanes 32-63 of the first operand <-> lanes 0-31 of the
// second): one 16-B store per lane instead of four scattered 4-B ones.
__device__ __forceinline__ i32x4 regroup16(const int (&d)[4]) {
    const auto p02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
    const auto p13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
    return i32x4{(int)p02[0], (int)p02[1], (int)p13[0], (int)p13[1]};
}
__device__ __forceinline__ int pack4b(int a, int b, int c, int d) {
    const unsigned ab = __builtin_amdgcn_perm((unsigned)b, (unsigned)a, 0x0c0c0400u);
    const unsigned cd = __builtin_amdgcn_perm((unsigned)d, (unsigned)c, 0x0c0c0400u);
    return (int)__builtin_amdgcn_perm(cd, ab, 0x05040100u);
}

// torch's bilinear source index (align_corners=False): lambda1, i0, i1
__device__ __forceinline__ float sp_src(float scale, int d, int n_in, int &i0, int &i1) {
    float src = __builtin_fmaf(scale, (float)d + 0.5f, -0.5f);
    src = src < 0.f ? 0.f : src;
    int i = (int)floorf(src);
    i = i > n_in - 1 ? n_in - 1 : i;
    float lam = src - (float)i;
    lam = lam < 0.f ? 0.f : (lam > 1.f ? 1.f : lam);
    i0 = i;
    i1 = i + (i < n_in - 1 ? 1 : 0);
    return lam;
}

// OMODE 0: NHWC [B][Ho][Wo][cstride]; OMODE 1: the Frame layout [B][Ho * Wo][cstride] with
// cell = x * Ho + y, channels >= cstride not stored (cstride = 65 for semi)
// conv1a fused in front of conv1b (FUSE1A): the workgroup computes its own input tile -- the
// image resized and quantised over the tile + 2 pixels into LDS, conv1a + relu over the tile +
// 1 pixel (zero outside the image: conv1b's padding) -- instead of loading conv1a's output.
struct Conv1aArgs {
    const uint8_t *img;
    int H, W;  // source frame
    float in_inv, rs;
    const int *wpk, *bq;
};

// workgroups per CU for the 64-channel layers (LDS 50 KB; VGPRs <= 168; 2 per CU measured 4-6 %
// slower, profiles/r05f_sp_geo_ab.log).  Measured and left out (profiles/r05x, r05aa): B fragments a
// k32 step ahead, s_setprio 1 over the K loop, 10 tile loads in flight, free scheduling of the K loop
// (no sched_barrier per k32 step), the frames resized once per pixel by a separate pass
// (profiles/r04s_sp_preresize_ab.log) -- all within noise or slower.
constexpr int SP_OCC64 = 3;
// Tile geometry.  GEO 0: 16 x 32 output pixels, a wave's 4 MFMA pixel blocks are its 4 rows of
// 32.  GEO 1 (the 24 x 80 layers: conv4a/b, convPa/Da at 192 x 640): 24 x 16 pixels, a wave's 3
// blocks are 2 rows x 16 columns each (lane fr -> row fr >> 4, column fr & 15), so 24 x 80 is 5
// whole tiles -- GEO 0 covers it with 2 x 3 tiles of which 37.5 % lie outside the frame.
template <int GEO> struct SpGeo {
    static constexpr int TY = GEO ? 24 : 16, TX = GEO ? 16 : 32;
    static constexpr int JN = GEO ? 3 : 4, RB = GEO ? 2 : 1, WR = JN * RB;  // blocks, rows per block / wave
};
template <int CIN, int KS, bool POOL, bool RELU, int OMODE, bool FUSE1A = false, int GEO = 0>
__global__ __launch_bounds__(SP_NT, CIN == 64 ? SP_OCC64 : 2) void k_sp_conv(const int8_t *__restrict__ in, int H, int W,
                                                      const i32x4 *__restrict__ wf, const int *__restrict__ bq,
                                                      float rs, int ngroups, int tiles_x, int tiles_y,
                                                      int8_t *__restrict__ out, int cstride, Conv1aArgs c1) {
    using G = SpGeo<GEO>;
    static_assert(GEO == 0 || (CIN != 64 && !POOL && OMODE == 0 && !FUSE1A), "GEO 1: the 128-channel unpooled layers");
    constexpr int TY = G::TY, TX = G::TX, JN = G::JN, RB = G::RB, WR = G::WR;
    constexpr int P = KS / 2, IY = TY + 2 * P, IX = TX + 2 * P, NCH = CIN / 16, NS = KS * KS * CIN / 32;
    constexpr int PF = CIN == 64 ? 2 : 4;  // weight fragments in flight (k32 steps)
    static_assert(CIN % 32 == 0 && NCH <= 16, "channels in 32-k steps, at most 256");
    // LDS tile layout.  64 channels: each pixel's 4 chunks padded to 5 (an odd stride: 16 lanes
    // reading one chunk of 16 consecutive pixels hit 16 distinct bank groups), so a B fragment's
    // address is a per-lane base + a compile-time offset (ds_read_b128 immediate, no VALU).
    // 128 channels (the padding would cost the second workgroup per CU): chunk c of pixel x
    // stored at c ^ ((x / 2) & 7), the lane's XOR term precomputed per tap column.
    constexpr bool PADL = NCH <= 4;
    constexpr int PS = PADL ? NCH + 1 : NCH;  // chunks per pixel
    constexpr int SWS = NCH >= 16 ? 1 : 16 / NCH;
    __shared__ i32x4 tile[IY * IX * PS];
    int bid = blockIdx.x;
    const int tx = bid % tiles_x;
    bid /= tiles_x;
    const int ty = bid % tiles_y;
    bid /= tiles_y;
    const int g = bid % ngroups, b = bid / ngroups;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 31, fh = lane >> 5;
    const int y0 = ty * TY, x0 = tx * TX;
    // the first weight fragments and the bias, issued before the input tile is built so that
    // their latency hides under it.  The accumulators start at the layer's quantised bias (row q
    // of channel block cb = channel 64 g + 32 cb + 8 (q >> 2) + 4 fh + (q & 3)), the C operand of
    // each chain's first MFMA: no add in the epilogue, and the 2 x 2 max pool commutes with it
    const i32x4 *wa = wf + (size_t)(2 * g) * NS * 64 + lane, *wb = wa + NS * 64;
    i32x4 ra[PF], rb[PF];
#pragma unroll
    for (int u = 0; u < PF; u++) {
        ra[u] = u < NS ? wa[u * 64] : i32x4{0, 0, 0, 0};
        rb[u] = u < NS ? wb[u * 64] : i32x4{0, 0, 0, 0};
    }
    i32x16 b0, b1;
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
        const i32x4 u0 = *reinterpret_cast<const i32x4 *>(bq + 64 * g + 8 * qq + 4 * fh);
        const i32x4 u1 = *reinterpret_cast<const i32x4 *>(bq + 64 * g + 32 + 8 * qq + 4 * fh);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            b0[4 * qq + e] = u0[e];
            b1[4 * qq + e] = u1[e];
        }
    }
    auto chunk_at = [&](int px, int x, int c) { return px * PS + (PADL ? c : (c ^ ((x / SWS) & (NCH - 1)))); };

    constexpr int NCHUNK = IY * IX * NCH;
    if constexpr (FUSE1A) {
        static_assert(CIN == 64 && KS == 3 && PADL, "conv1a feeds conv1b");
        constexpr int QY = IY + 2, QX = IX + 2, QXS = QX + 2;
        __shared__ int8_t qim[QY * QXS];
        __shared__ float lut[256];  // k / 255 (IEEE division), the driver's astype(float32) / 255.
        // the bilinear source rows / columns of the tile's QY rows and QX columns, once per
        // workgroup: (weight of the far sample, its complement, near / far offsets)
        __shared__ float4 rowc[QY], colc[QX];
        lut[t] = (float)t / 255.0f;
        const float sy = (float)c1.H / (float)H, sx = (float)c1.W / (float)W;
        if (t < QY) {
            int ya, yb;
            const float h1 = sp_src(sy, min(max(y0 + t - 2, 0), H - 1), c1.H, ya, yb);
            rowc[t] = make_float4(h1, 1.f - h1, __int_as_float(ya * c1.W), __int_as_float(yb * c1.W));
        } else if (t >= 64 && t < 64 + QX) {
            int xa, xb;
            const float w1 = sp_src(sx, min(max(x0 + (t - 64) - 2, 0), W - 1), c1.W, xa, xb);
            colc[t - 64] = make_float4(w1, 1.f - w1, __int_as_float(xa), __int_as_float(xb));
        }
        __syncthreads();
        const uint8_t *im = c1.img + (size_t)b * c1.H * c1.W;
        // every pixel's four source bytes loaded before any is used (all gathers of the thread in
        // flight at once; out-of-frame pixels read a clamped in-frame byte and store 0)
        constexpr int NQ = (QY * QX + SP_NT - 1) / SP_NT;
        uint8_t src4[NQ][4];
#pragma unroll
        for (int u = 0; u < NQ; u++) {
            const int i = min(t + u * SP_NT, QY * QX - 1), r = i / QX, c = i % QX;
            const float4 rc = rowc[r], cc = colc[c];
            const int ra = __float_as_int(rc.z), rb = __float_as_int(rc.w);
            const int xa = __float_as_int(cc.z), xb = __float_as_int(cc.w);
            src4[u][0] = im[ra + xa];
            src4[u][1] = im[ra + xb];
            src4[u][2] = im[rb + xa];
            src4[u][3] = im[rb + xb];
        }
#pragma unroll
        for (int u = 0; u < NQ; u++) {
            const int i = t + u * SP_NT;
            if (i >= QY * QX) break;
            const int r = i / QX, c = i % QX;
            const int gy = y0 + r - 2, gx = x0 + c - 2;
            int v = 0;
            if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
                const float4 rc = rowc[r], cc = colc[c];
                const float h1 = rc.x, h0 = rc.y, w1 = cc.x, w0 = cc.y;
                const float a00 = lut[src4[u][0]], a01 = lut[src4[u][1]];
                const float a10 = lut[src4[u][2]], a11 = lut[src4[u][3]];
                const float t0 = __builtin_fmaf(a00, w0, a01 * w1);
                const float t1 = __builtin_fmaf(a10, w0, a11 * w1);
                const float x = __builtin_fmaf(t0, h0, t1 * h1);
                float qv = __builtin_rintf(x * c1.in_inv);
                qv = fminf(fmaxf(qv, -128.f), 127.f);
                v = (int)qv;
            }
            qim[r * QXS + c] = (int8_t)v;
        }
        __syncthreads();
        // conv1a + relu over the tile + halo on v_mfma_f32_32x32x16_f16: K = the 9 taps (+ 7 zero),
        // A = the weights (lanes < 32: taps 0-7, lanes >= 32: tap 8), B = 32 tile pixels' taps;
        // pixels outside the image are conv1b's zero padding, not conv1a evaluated there
        // on the f16 matrix cores: int8 taps and weights are exact in f16, every partial sum an
        // integer below 2^24 (exact in f32), the bias the C input -- the accumulator IS the
        // integer sum as a float, so the requantisation skips its int -> float conversion
        typedef _Float16 h8 __attribute__((ext_vector_type(8)));
        typedef float f32x16 __attribute__((ext_vector_type(16)));
        h8 a1[2];
        f32x16 bias[2];
#pragma unroll
        for (int cb = 0; cb < 2; cb++) {
            const int co = 32 * cb + fr;
            const unsigned lo = (unsigned)(fh ? c1.wpk[3 * co + 2] : c1.wpk[3 * co]);
            const unsigned hi = fh ? 0u : (unsigned)c1.wpk[3 * co + 1];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                a1[cb][k] = (_Float16)(float)(((int)(lo << (24 - 8 * k))) >> 24);
                a1[cb][4 + k] = (_Float16)(float)(((int)(hi << (24 - 8 * k))) >> 24);
            }
#pragma unroll
            for (int q = 0; q < 16; q++) bias[cb][q] = (float)c1.bq[32 * cb + (q & 3) + 8 * (q >> 2) + 4 * fh];
        }
        constexpr int NPX = IY * IX, NBLK = (NPX + 31) / 32;
#pragma unroll 1
        for (int blk = w; blk < NBLK; blk += SP_NT / 64) {
            const int px = blk * 32 + fr, pxc = min(px, NPX - 1);
            const int r = pxc / IX, x = pxc % IX;
            const int8_t *q0 = qim + r * QXS + x;
            const int gy = y0 + r - 1, gx = x0 + x - 1;
            const bool in_img = px < NPX && gy >= 0 && gy < H && gx >= 0 && gx < W;
            h8 bv;
            if (fh == 0) {
                bv[0] = (_Float16)(float)q0[0];
                bv[1] = (_Float16)(float)q0[1];
                bv[2] = (_Float16)(float)q0[2];
                bv[3] = (_Float16)(float)q0[QXS];
                bv[4] = (_Float16)(float)q0[QXS + 1];
                bv[5] = (_Float16)(float)q0[QXS + 2];
                bv[6] = (_Float16)(float)q0[2 * QXS];
                bv[7] = (_Float16)(float)q0[2 * QXS + 1];
            } else {
                bv = h8{};
                bv[0] = (_Float16)(float)q0[2 * QXS + 2];
            }
#pragma unroll
            for (int cb = 0; cb < 2; cb++) {
                const f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[cb], bv, bias[cb], 0, 0, 0);
                int dw[4];
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    int v[4];
#pragma unroll
                    for (int e = 0; e < 4; e++) v[e] = requant_bitsf(d[4 * qq + e], c1.rs, SP_MAGIC_BITS);
                    dw[qq] = pack4b(v[0], v[1], v[2], v[3]);
                }
                // the lane pair's 32 channels regrouped: this lane's chunk 2 cb + fh, one 16-B store
                // (4-B stores at the 80-B pixel stride hit 4-way bank conflicts)
                const i32x4 chunk = regroup16(dw);
                if (px < NPX) tile[chunk_at(px, x, 2 * cb + fh)] = in_img ? chunk : i32x4{0, 0, 0, 0};
            }
        }
    }
    // ---- the input tile (zero outside the image), 8 16-B loads in flight per thread ----
    // (4 consecutive lanes read one pixel's 64 contiguous bytes: giving an 8-lane group one chunk
    // of 8 pixels instead -- conflict-free LDS stores -- made the 64-channel layers 3-4x slower:
    // the loads must stay lane-contiguous)
    const int8_t *src = in + (size_t)b * H * W * CIN;
    constexpr int LIF = 8;  // 16-B loads in flight per thread (10 / 12 / 16 measured the same)
    for (int i0 = 0; i0 < (FUSE1A ? 0 : NCHUNK); i0 += LIF * SP_NT) {
        i32x4 v[LIF];
#pragma unroll
        for (int u = 0; u < LIF; u++) {
            const int i = i0 + u * SP_NT + t;
            const int c = i % NCH, px = i / NCH, x = px % IX, r = px / IX;
            const int gy = y0 + r - P, gx = x0 + x - P;
            v[u] = i32x4{0, 0, 0, 0};
            if (i < NCHUNK && gy >= 0 && gy < H && gx >= 0 && gx < W)
                v[u] = *reinterpret_cast<const i32x4 *>(src + ((size_t)gy * W + gx) * CIN + c * 16);
        }
#pragma unroll
        for (int u = 0; u < LIF; u++) {
            const int i = i0 + u * SP_NT + t;
            if (i >= NCHUNK) continue;
            const int c = i % NCH, px = i / NCH, x = px % IX;
            tile[chunk_at(px, x, c)] = v[u];
        }
    }
    __syncthreads();

    // a wave whose 4 rows all lie below the frame (the 24-row layers' second tile row: a quarter
    // of their waves) has nothing to compute; the 128-channel epilogue has no block barrier
    if constexpr (CIN != 64) {
        if (y0 + WR * w >= H) return;
    }
    // ---- K loop: 9 taps (or 1) x CIN / 32 steps, fully unrolled: every LDS offset a constant ----
    i32x16 acc[JN][2];
    // per-lane bases: the lane's pixel (row WR w + [fr >> 4], column fr or fr & 15), chunk half fh
    // (padded layout); XOR terms per kx
    const int prow = WR * w + (GEO ? fr >> 4 : 0), pcol = GEO ? fr & 15 : fr;
    const i32x4 *lb = tile + (prow * IX + pcol) * PS + (PADL ? fh : 0);
    int xs[KS];
#pragma unroll
    for (int kx = 0; kx < KS; kx++) xs[kx] = fh ^ (((pcol + kx) / SWS) & (NCH - 1));
    // the B fragments of k32 step s
    auto bfrag = [&](int s, int j) {
        const int tap = s * 32 / CIN, ky = tap / KS, kx = tap % KS, c0 = (s * 32 % CIN) / 16;
        const int off = ((RB * j + ky) * IX + kx) * PS;
        return PADL ? lb[off + c0] : lb[off + (c0 ^ xs[kx])];
    };
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const i32x4 a0 = ra[s % PF], a1 = rb[s % PF];
        if (s + PF < NS) {
            ra[s % PF] = wa[(s + PF) * 64];
            rb[s % PF] = wb[(s + PF) * 64];
        }
        i32x4 bc[JN];
#pragma unroll
        for (int j = 0; j < JN; j++) bc[j] = bfrag(s, j);
#pragma unroll
        for (int j = 0; j < JN; j++) {
            acc[j][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bc[j], s == 0 ? b0 : acc[j][0], 0, 0, 0);
            acc[j][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bc[j], s == 0 ? b1 : acc[j][1], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // one k32 step at a time
    }

    // ---- epilogue: lane = pixel fr of each row; 16 couts (4 groups of 4) per 32-cout block ----
    const int lo = SP_MAGIC_BITS + (RELU ? 0 : -128);
    if constexpr (CIN == 64) {
        // 64-channel layers (168 VGPRs: the lane-pair regroup below spilled the K loop): each wave writes its
        // requantised outputs into its own LDS rows (64 B per pixel), then reads them back 16 B per
        // lane and stores whole pixel runs -- 2 KiB contiguous per output row.  Chunk c of staged
        // pixel P sits at 16-B position (c + (P >> 1)) & 3: conflict-free for both the 8-lane
        // ds_write_b128 groups (pixels fr .. fr + 7, one chunk: 32-bank rows) and the 16-lane
        // ds_read_b128 groups (4 pixels x 4 chunks: 64-bank rows); the 80-B padded stride this
        // replaces left the reads 3-way conflicted (42 % of the non-pooled layers' LDS cycles)
        constexpr int PB = 64;
        // per-lane bases, computed where used (the row / pair offsets are compile-time
        // immediates; hoisted address registers spilled these 168-VGPR kernels): reads take chunk
        // k = lane & 3 of pixel lane >> 2 (+ 16 per read), whose 16-B position is (k + (lane >> 3)) & 3
        static_assert(4 * 4 * 32 * PB <= IY * IX * PS * 16, "staging fits the input tile");
        __syncthreads();  // every wave past its last read of the input tile
        char *stg = reinterpret_cast<char *>(tile) + w * (4 * 32 * PB);
        if constexpr (POOL) {
            const int Ho = H / 2, Wo = W / 2;
#pragma unroll
            for (int jp = 0; jp < 2; jp++) {
                // both lanes of a column pair hold the pair's 2 x 2 maxima of both channel blocks:
                // the even lane requantises block 0, the odd lane block 1
                const int cbx = fr & 1;
                int m[16];
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    int v0 = max(acc[2 * jp][0][q], acc[2 * jp + 1][0][q]);
                    int v1 = max(acc[2 * jp][1][q], acc[2 * jp + 1][1][q]);
                    v0 = max(v0, __builtin_amdgcn_update_dpp(0, v0, 0xB1, 0xF, 0xF, false));  // lane ^ 1
                    v1 = max(v1, __builtin_amdgcn_update_dpp(0, v1, 0xB1, 0xF, 0xF, false));
                    m[q] = cbx ? v1 : v0;
                }
                int dw[4];
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    int v[4];
                    requant4(v, m[4 * qq], m[4 * qq + 1], m[4 * qq + 2], m[4 * qq + 3], rs, lo);
                    dw[qq] = pack4b(v[0], v[1], v[2], v[3]);
                }
                // 16-B stores (4-B ones would be 4-way bank conflicted)
                // pixel jp * 16 + fr / 2, chunk 2 cbx + fh, position (chunk + (fr >> 2)) & 3 (the
                // non-fused pooled layer keeps the plain order: the swizzled one spilled it)
                const int pa = (fr >> 1) * PB + ((FUSE1A ? ((2 * cbx + fh + (fr >> 2)) & 3) : 2 * cbx + fh) << 4);
                *reinterpret_cast<i32x4 *>(stg + jp * 16 * PB + pa) = regroup16(dw);
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
            __builtin_amdgcn_wave_barrier();
            const int ra = (lane >> 2) * PB + ((FUSE1A ? (((lane & 3) + (lane >> 3)) & 3) : lane & 3) << 4);
#pragma unroll
            for (int jp = 0; jp < 2; jp++) {
                const int p = lane >> 2, k = lane & 3;  // 16 pooled pixels x 4 chunks
                const int gy = y0 + 4 * w + 2 * jp, gx = x0 + 2 * p;
                const i32x4 v = *reinterpret_cast<const i32x4 *>(stg + jp * 16 * PB + ra);
                if (gy < H && gx < W)
                    *reinterpret_cast<i32x4 *>(out + (((size_t)b * Ho + gy / 2) * Wo + gx / 2) * cstride + 64 * g + 16 * k) = v;
            }
        } else {
            const int wa = fr * PB + (((fh + (fr >> 1)) & 3) << 4);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int cb = 0; cb < 2; cb++) {
                    int dw[4];
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) {
                        int v[4];
                        requant4(v, acc[j][cb][4 * qq], acc[j][cb][4 * qq + 1], acc[j][cb][4 * qq + 2], acc[j][cb][4 * qq + 3], rs, lo);
                        dw[qq] = pack4b(v[0], v[1], v[2], v[3]);
                    }
                    // pixel j * 32 + fr, chunk 2 cb + fh, position (chunk + (fr >> 1)) & 3 = wa ^ 32 cb
                    *reinterpret_cast<i32x4 *>(stg + j * 32 * PB + (wa ^ (cb << 5))) = regroup16(dw);
                }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const int ra = (lane >> 2) * PB + ((((lane & 3) + (lane >> 3)) & 3) << 4);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int c = lane + 64 * i, p = c >> 2, k = c & 3;  // 32 pixels x 4 chunks
                    const int gy = y0 + 4 * w + j, gx = x0 + p;
                    const i32x4 v = *reinterpret_cast<const i32x4 *>(stg + j * 32 * PB + i * 16 * PB + ra);
                    if (gy < H && gx < W)
                        *reinterpret_cast<i32x4 *>(out + (((size_t)b * H + gy) * W + gx) * cstride + 64 * g + 16 * k) = v;
                }
        }
        return;
    }
    if constexpr (POOL) {
        const int Ho = H / 2, Wo = W / 2;
#pragma unroll
        for (int jp = 0; jp < 2; jp++) {
            // the even lane of a column pair requantises channel block 0, the odd lane block 1
            const int cbx = fr & 1, gy = y0 + 4 * w + 2 * jp, gx = x0 + fr - cbx;
            int m[16];
#pragma unroll
            for (int q = 0; q < 16; q++) {
                int v0 = max(acc[2 * jp][0][q], acc[2 * jp + 1][0][q]);
                int v1 = max(acc[2 * jp][1][q], acc[2 * jp + 1][1][q]);
                v0 = max(v0, __builtin_amdgcn_update_dpp(0, v0, 0xB1, 0xF, 0xF, false));  // lane ^ 1
                v1 = max(v1, __builtin_amdgcn_update_dpp(0, v1, 0xB1, 0xF, 0xF, false));
                m[q] = cbx ? v1 : v0;
            }
            if (gy < H && gx < W) {  // both lanes of a regroup pair (same fr) or neither
                int8_t *dst = out + (((size_t)b * Ho + gy / 2) * Wo + gx / 2) * cstride;
                int d[4];
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    int v[4];
                    requant4(v, m[4 * qq], m[4 * qq + 1], m[4 * qq + 2], m[4 * qq + 3], rs, lo);
                    d[qq] = pack4b(v[0], v[1], v[2], v[3]);
                }
                *reinterpret_cast<i32x4 *>(dst + 64 * g + 32 * cbx + 16 * fh) = regroup16(d);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < JN; j++) {
            const int gy = y0 + prow + RB * j, gx = x0 + pcol;
            if (gy >= H || gx >= W) continue;  // both lanes of a pair (same fr) or neither
            int8_t *dst = OMODE == 0 ? out + (((size_t)b * H + gy) * W + gx) * cstride
                                     : out + ((size_t)b * H * W + (size_t)gx * H + gy) * cstride;
#pragma unroll
            for (int cb = 0; cb < 2; cb++) {
                if constexpr (OMODE == 0) {  // NHWC activations: 64 / 128 / 256 channels (host-checked)
                    int d[4];
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) {
                        int v[4];
                        requant4(v, acc[j][cb][4 * qq], acc[j][cb][4 * qq + 1], acc[j][cb][4 * qq + 2], acc[j][cb][4 * qq + 3], rs, lo);
                        d[qq] = pack4b(v[0], v[1], v[2], v[3]);
                    }
                    *reinterpret_cast<i32x4 *>(dst + 64 * g + 32 * cb + 16 * fh) = regroup16(d);
                    __builtin_amdgcn_sched_barrier(0);  // one block at a time: the register budget
                    continue;
                }
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    const int co = 64 * g + 32 * cb + 8 * qq + 4 * fh;
                    int v[4];
                    requant4(v, acc[j][cb][4 * qq], acc[j][cb][4 * qq + 1], acc[j][cb][4 * qq + 2], acc[j][cb][4 * qq + 3], rs, lo);
                    if (OMODE == 0 || (cstride % 4 == 0 && co + 4 <= cstride)) {
                        *reinterpret_cast<int *>(dst + co) = pack4b(v[0], v[1], v[2], v[3]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; e++)
                            if (co + e < cstride) dst[co + e] = (int8_t)v[e];
                    }
                }
            }
        }
    }
}

// The 1 x 1 heads (convPb, convDb: 256 input channels, no halo) as a weight-stationary pass.  The
// heads are data movement: 256 B of input per pixel against 65 / 256 outputs, ~2 k MFMA cycles per
// 64 KiB tile -- round 4's tiled k_sp_conv1x1 (8 x 32 pixels x 128 channels per workgroup, in git
// history up to round 5) ran its 576 / 1152 tile workgroups (2 per CU) in 1.1 / 2.3 rounds of
// load-then-compute each (25 / 28 us per 64 frames, profiles/r05w_sp_layers.txt).  Here a workgroup keeps its share of the
// weights in registers (wave w: channel blocks CBW w .. CBW w + CBW - 1, 8 k32 fragments each)
// and streams HD_NB consecutive 32-pixel blocks through a double-buffered LDS tile, the loads of
// the next HD_D blocks in flight in registers while a block is multiplied -- straight-line code
// (no loop back-edge, across which the compiler would wait for every outstanding load).  Blocks
// follow the output order: Frame cells (x H + y) for OMODE 1, so a block's semi outputs are
// 32 x 65 contiguous bytes (staged in LDS, stored as whole words by the next block), row-major
// pixels for OMODE 2 (run()'s NCHW planes: 32 consecutive floats per channel).  The integer
// products, bias and requantisation are those of the 3 x 3 layers' epilogue: outputs in the Frame
// layout (OMODE 1) or, OMODE 2, already dequantised as run()'s NCHW float32 [B][C][H][W] (out is a
// float *, cstride = C, dq = the head's out_scale: PyTorch's dequantise dq * (float) code).
// HD_NB: 32-pixel blocks per workgroup (4 / 16 measured 1-2 % slower: profiles/r05ak_sp_head_nb_ab.log).
constexpr int HD_PS = 17, HD_D = 3, HD_NB = 8;
constexpr int SP_MG_CHUNKS = 32;  // presence-mask chunks per (frame, head): k_sp_presence's split
// FULL: every frame whole blocks (H W % 32 == 0), every workgroup HD_NB of them and out 4-B
// aligned -- no lane or block guards, so the loads stay in flight (a load under a branch is sunk
// to its use, a store under one makes the compiler wait for every outstanding load at the join);
// otherwise the guarded form.
// PRES (OMODE 1, FULL, frames of >= HD_NB blocks: a workgroup spans at most 2 frames): run()'s
// presence mask of the head's codes (k_sp_presence's work) from the epilogue -- each code marks
// a word of an LDS "seen" array per frame, ORed at the end into chunk 0 of pres[frame][head]
// (zeroed by the launcher) with vector atomics.
template <int OMODE, int NCB, bool FULL, bool PRES = false>
__global__ __launch_bounds__(SP_NT, 2) void k_sp_head(const int8_t *__restrict__ in, int H, int W, int nblk_f,
                                                      int nblk, const i32x4 *__restrict__ wf,
                                                      const int *__restrict__ bq, float rs,
                                                      int8_t *__restrict__ out, int cstride, float dq,
                                                      unsigned *__restrict__ pres) {
    constexpr int CBW = (NCB + 3) / 4, NS = 8;
    constexpr bool STAGE = OMODE == 1 && NCB * 32 < 128;  // the semi head: 65-byte cells
    static_assert(!PRES || (OMODE == 1 && FULL), "presence from the int8 heads' full form");
    __shared__ i32x4 tile[2][32 * HD_PS];
    __shared__ int stg[STAGE ? 2 : 1][STAGE ? 32 * 65 / 4 + 1 : 1];
    __shared__ int seen[PRES ? 2 : 1][PRES ? 256 : 1];  // per frame slot: code + 128 present
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 31, fh = lane >> 5;
    const int HW = H * W;
    const int kb = blockIdx.x * HD_NB, nmine = min(HD_NB, nblk - kb);
    // the wave's weights and bias first (the block loads after them: waiting for a block's loads
    // then implies the weights, in the in-order count).  A wave past the last channel block (the
    // semi head's wave 3) recomputes the last one and stores the same values again.
    i32x4 aw[CBW][NS];
    i32x16 bias[CBW];
    int cbs[CBW];
#pragma unroll
    for (int c = 0; c < CBW; c++) {
        const int cb = min(CBW * w + c, NCB - 1);
        cbs[c] = cb;
#pragma unroll
        for (int s = 0; s < NS; s++) aw[c][s] = wf[((size_t)cb * NS + s) * 64 + lane];
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const i32x4 x = *reinterpret_cast<const i32x4 *>(bq + 32 * cb + 8 * qq + 4 * fh);
#pragma unroll
            for (int e = 0; e < 4; e++) bias[c][4 * qq + e] = x[e];
        }
    }
    // block j of this workgroup (j >= nmine: the last one again, loaded but never used): frame
    // fb[j], first pixel 32 fi[j]
    int fb[HD_NB], fi[HD_NB];
    fb[0] = kb / nblk_f;
    fi[0] = kb - fb[0] * nblk_f;
#pragma unroll
    for (int j = 1; j < HD_NB; j++) {
        const bool wrap = fi[j - 1] + 1 == nblk_f, past = j >= nmine;
        fb[j] = past ? fb[j - 1] : fb[j - 1] + (wrap ? 1 : 0);
        fi[j] = past ? fi[j - 1] : (wrap ? 0 : fi[j - 1] + 1);
    }
    // thread t loads chunks t and t + 256 of a block: pixels (t >> 4) and (t >> 4) + 16, chunk t & 15
    auto load = [&](int j, i32x4 (&r)[2]) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
            int p = 32 * fi[j] + (t >> 4) + 16 * u;
            if (!FULL) p = min(p, HW - 1);  // clamped: never stored
            const int y = OMODE == 1 ? p % H : p / W, x = OMODE == 1 ? p / H : p % W;
            r[u] = *reinterpret_cast<const i32x4 *>(in + ((size_t)fb[j] * HW + (size_t)y * W + x) * 256 + (t & 15) * 16);
        }
    };
    i32x4 R[HD_D][2];
#pragma unroll
    for (int d = 0; d < HD_D; d++) load(d, R[d]);
    auto stage_out = [&](int j) {  // block j's staged semi bytes -> out
        int8_t *gd = out + ((size_t)fb[j] * HW + 32 * fi[j]) * 65;
        if (FULL) {  // 520 words: 4 B aligned (H W % 4 == 0, out 4-B aligned)
            int *gw = reinterpret_cast<int *>(gd);
            gw[t] = stg[j & 1][t];
            gw[t + SP_NT] = stg[j & 1][t + SP_NT];
            if (t < 32 * 65 / 4 - 2 * SP_NT) gw[t + 2 * SP_NT] = stg[j & 1][t + 2 * SP_NT];
            return;
        }
        const int nb = min(32, HW - 32 * fi[j]) * 65;
        const int8_t *ls = reinterpret_cast<const int8_t *>(stg[j & 1]);
        for (int o = t; o < nb; o += SP_NT) gd[o] = ls[o];
    };
    const int lo = SP_MAGIC_BITS - 128;  // the heads have no relu
    if (PRES) {
        seen[0][t] = 0;
        seen[1][t] = 0;  // ordered before the marks by the first block's barrier
    }
#pragma unroll
    for (int j = 0; j < HD_NB; j++) {
        if (!FULL && j >= nmine) break;  // workgroup-uniform
        i32x4 *tb = tile[j & 1];
#pragma unroll
        for (int u = 0; u < 2; u++) tb[((t >> 4) + 16 * u) * HD_PS + (t & 15)] = R[j % HD_D][u];
        __syncthreads();
        if (STAGE && j > 0) stage_out(j - 1);
        if (j + HD_D < HD_NB) load(j + HD_D, R[j % HD_D]);  // past nmine: a repeat, unused
        i32x16 acc[CBW];
        const i32x4 *lb = tb + fr * HD_PS + fh;
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const i32x4 bv = lb[2 * s];
#pragma unroll
            for (int c = 0; c < CBW; c++)
                acc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aw[c][s], bv, s == 0 ? bias[c] : acc[c], 0, 0, 0);
        }
        const int p = 32 * fi[j] + fr;
        const bool inside = FULL || p < HW;
#pragma unroll
        for (int c = 0; c < CBW; c++) {
            const int cb = cbs[c];
            int dw[4];  // OMODE 1, 256 channels: the packed codes, 4 per word
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const int co = 32 * cb + 8 * qq + 4 * fh;
                int v[4];
                requant4(v, acc[c][4 * qq], acc[c][4 * qq + 1], acc[c][4 * qq + 2], acc[c][4 * qq + 3], rs, lo);
                if constexpr (OMODE == 2) {
                    float *fo = reinterpret_cast<float *>(out) + ((size_t)fb[j] * cstride + co) * HW + p;
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if (inside && (NCB * 32 == 256 || co + e < cstride))
                            fo[(size_t)e * HW] = dq * (float)(v[e] - SP_MAGIC_BITS);
                } else if constexpr (STAGE) {
                    int8_t *cell = reinterpret_cast<int8_t *>(stg[j & 1]) + fr * 65;
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if (co + e < 65) cell[co + e] = (int8_t)v[e];
                } else {
                    dw[qq] = pack4b(v[0], v[1], v[2], v[3]);
                }
                if constexpr (PRES) {  // the code's low byte + 128 (the magic's low byte is 0)
                    int *sn = seen[fb[j] - fb[0]];
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if (NCB * 32 == 256 || co + e < cstride) sn[(v[e] + 128) & 255] = 1;
                }
            }
            if constexpr (OMODE == 1 && !STAGE) {  // channels 32 cb + 16 fh .. + 15 per lane
                if (inside)
                    *reinterpret_cast<i32x4 *>(out + ((size_t)fb[j] * HW + p) * cstride + 32 * cb + 16 * fh) =
                        regroup16(dw);
            }
        }
    }
    if (STAGE || PRES) __syncthreads();
    if (STAGE) stage_out(nmine - 1);
    if (PRES && w < 2) {  // wave w: frame slot w (slot 1 only when the workgroup reaches the next frame)
        const int b = fb[0] + w;
        if (b <= fb[HD_NB - 1]) {
            unsigned *pw = pres + (size_t)(b * 2 + (NCB == 8 ? 1 : 0)) * SP_MG_CHUNKS * 8;
#pragma unroll
            for (int k = 0; k < 4; k++) {  // codes 64 k .. 64 k + 63: words 2 k, 2 k + 1
                const unsigned long long bm = __ballot(seen[w][64 * k + lane] != 0);
                if (lane < 2 && (unsigned)(bm >> (32 * lane)) != 0u)
                    atomicOr(pw + 2 * k + lane, (unsigned)(bm >> (32 * lane)));
            }
        }
    }
}

// run()'s output quantisation (superpoint_inference.py:199-206), head h (0: semi, C = 65;
// 1: desc, C = 256) of frame b, split over SP_MG_CHUNKS workgroups per head: k_sp_presence ORs
// the 256-code presence mask of a chunk into pres[b][h][chunk][8] (its own slot: no atomics, no
// clearing -- 128 waves ORing into one (frame, head)'s 32 B serialised at the L2); k_sp_min_gap
// ORs a head's chunk masks, derives the smallest
// gap between present dequantised codes (every workgroup, from the same mask) and rounds its
// chunk to that step in place.

__device__ __forceinline__ void sp_head(int8_t *semi, int8_t *desc, long cells, int b, int h, int8_t *&base, long &lo,
                                        long &hi) {
    const int C = h ? 256 : 65;
    base = (h ? desc : semi) + (size_t)b * cells * C;
    const long n = cells * C, per = ((n + SP_MG_CHUNKS - 1) / SP_MG_CHUNKS + 15) / 16 * 16;
    lo = min(n, per * blockIdx.z);
    hi = min(n, lo + per);
}

__global__ __launch_bounds__(SP_NT) void k_sp_presence(const int8_t *__restrict__ semi, const int8_t *__restrict__ desc,
                                                       long cells, unsigned *__restrict__ pres) {
    // per wave 8 replicas of a 256-byte "seen" array in LDS (lane l stores into replica l & 7,
    // replicas 65 dwords apart: neighbouring lanes' equal codes land in different banks): one
    // byte store per code (lanes storing the same code store the same 1: no atomics), then the
    // replicas are ORed and 4 ballots turn them into the 256-bit mask
    constexpr int RS = 65 * 4;  // replica stride, bytes
    __shared__ unsigned seen_w[SP_NT / 64][8 * RS / 4];
    const int b = blockIdx.x, h = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
    unsigned char *seen_all = reinterpret_cast<unsigned char *>(seen_w[w]);
    unsigned char *seen = seen_all + (lane & 7) * RS;
    for (int i = lane; i < 8 * RS / 4; i += 64) seen_w[w][i] = 0u;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    int8_t *base;
    long lo, hi;
    sp_head(const_cast<int8_t *>(semi), const_cast<int8_t *>(desc), cells, b, h, base, lo, hi);
    const bool al = ((uintptr_t)(base + lo) & 15) == 0;
    constexpr int U = 4;  // 16-B loads in flight per thread
    for (long i0 = lo + 16 * t; i0 < hi; i0 += 16 * SP_NT * U) {
        i32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + 16 * SP_NT * u;
            if (al && i + 16 <= hi) v[u] = *reinterpret_cast<const i32x4 *>(base + i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + 16 * SP_NT * u;
            if (i >= hi) break;
            if (!(al && i + 16 <= hi)) {
                for (int k = 0; k < 4; k++) {
                    int x = 0;
                    for (int e = 0; e < 4; e++) {
                        const long j = i + 4 * k + e;
                        // past the chunk: repeat its first code (already present)
                        x |= ((j < hi ? base[j] : base[lo]) & 0xff) << (8 * e);
                    }
                    v[u][k] = x;
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++)
#pragma unroll
                for (int e = 0; e < 4; e++) seen[((v[u][k] << (24 - 8 * e)) >> 24) + 128] = 1;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    __shared__ unsigned wm[SP_NT / 64][8];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // codes 64 k .. 64 k + 63: words 2 k, 2 k + 1
        unsigned any = 0;
#pragma unroll
        for (int r = 0; r < 8; r++) any |= seen_all[r * RS + 64 * k + lane];
        const unsigned long long bm = __ballot(any != 0);
        if (lane == 0) {
            wm[w][2 * k] = (unsigned)bm;
            wm[w][2 * k + 1] = (unsigned)(bm >> 32);
        }
    }
    __syncthreads();
    if (t < 8) {
        unsigned x = 0;
#pragma unroll
        for (int k = 0; k < SP_NT / 64; k++) x |= wm[k][t];
        pres[((size_t)(b * 2 + h) * SP_MG_CHUNKS + blockIdx.z) * 8 + t] = x;
    }
}

__global__ __launch_bounds__(SP_NT) void k_sp_min_gap(int8_t *__restrict__ semi, int8_t *__restrict__ desc, long cells,
                                                      float s_semi, float s_desc, const unsigned *__restrict__ pres,
                                                      float *__restrict__ semi_scale, float *__restrict__ desc_scale) {
    __shared__ float gmin[SP_NT / 64];
    __shared__ int cnts[SP_NT / 64];
    __shared__ unsigned char lut[256];  // code + 128 -> its rounded value (one division per code)
    const int b = blockIdx.x, h = blockIdx.y, t = threadIdx.x, lane = t & 63;
    const float s = h ? s_desc : s_semi;
    __shared__ unsigned pm[8];  // the head's mask: its chunks' masks ORed
    if (t < 8) {
        const unsigned *pc = pres + (size_t)(b * 2 + h) * SP_MG_CHUNKS * 8 + t;
        unsigned x = 0;
#pragma unroll
        for (int c = 0; c < SP_MG_CHUNKS; c++) x |= pc[8 * c];
        pm[t] = x;
    }
    __syncthreads();
    // thread v: the gap from code v (present) to the next present code, in dequantised floats
    float gap = INFINITY;
    int cnt;
    {
        const int v = t;
        const bool here = (pm[v >> 5] >> (v & 31)) & 1u;
        // the next present code above v: the rest of v's word, then the following words
        int nx = -1;
        const unsigned rest = (v & 31) == 31 ? 0u : pm[v >> 5] & ~((2u << (v & 31)) - 1u);
        if (rest) nx = (v & ~31) + __builtin_ctz(rest);
        for (int k = (v >> 5) + 1; k < 8 && nx < 0; k++)
            if (pm[k]) nx = 32 * k + __builtin_ctz(pm[k]);
        if (here && nx >= 0) {
            const float d = (float)(nx - 128) * s - (float)(v - 128) * s;
            gap = d > 0.f ? d : INFINITY;
        }
        cnt = here ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        gap = fminf(gap, __shfl_xor(gap, o, 64));
        cnt += __shfl_xor(cnt, o, 64);
    }
    if (lane == 0) {
        gmin[t >> 6] = gap;
        cnts[t >> 6] = cnt;
    }
    __syncthreads();
    float g = gmin[0];
    int distinct = cnts[0];
#pragma unroll
    for (int k = 1; k < SP_NT / 64; k++) {
        g = fminf(g, gmin[k]);
        distinct += cnts[k];
    }
    if (distinct < 2) g = 0.f;
    if (t == 0 && blockIdx.z == 0) (h ? desc_scale : semi_scale)[b] = g;
    if (g == 0.f) return;  // fewer than two distinct values: the raw codes stay
    int8_t *base;
    long lo, hi;
    sp_head(semi, desc, cells, b, h, base, lo, hi);
    auto requant = [&](int q) {  // round(outs / scale0) of one code, clamped to int8
        const float f = (float)q * s;
        float r = __builtin_rintf(f / g);
        return (int)fminf(fmaxf(r, -128.f), 127.f);
    };
    lut[t] = (unsigned char)requant(t - 128);  // SP_NT = 256 threads: one code each
    __syncthreads();
    const bool al = ((uintptr_t)(base + lo) & 15) == 0;
    if (al) {
        constexpr int U = 4;  // 16 codes per load, 4 loads in flight per thread
        long i0 = lo + 16 * t;
        for (; i0 + 16 * SP_NT * (U - 1) + 16 <= hi; i0 += 16 * SP_NT * U) {
            i32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = *reinterpret_cast<const i32x4 *>(base + i0 + 16 * SP_NT * u);
#pragma unroll
            for (int u = 0; u < U; u++) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const unsigned x = (unsigned)v[u][k] ^ 0x80808080u;  // bytes = code + 128
                    v[u][k] = (int)(lut[x & 0xff] | (lut[(x >> 8) & 0xff] << 8) | (lut[(x >> 16) & 0xff] << 16) |
                                    ((unsigned)lut[x >> 24] << 24));
                }
                *reinterpret_cast<i32x4 *>(base + i0 + 16 * SP_NT * u) = v[u];
            }
        }
        for (; i0 < hi; i0 += 16 * SP_NT) {  // the rest: whole 16-B pieces, then the partial one
            if (i0 + 16 <= hi) {
                i32x4 v = *reinterpret_cast<const i32x4 *>(base + i0);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const unsigned x = (unsigned)v[k] ^ 0x80808080u;
                    v[k] = (int)(lut[x & 0xff] | (lut[(x >> 8) & 0xff] << 8) | (lut[(x >> 16) & 0xff] << 16) |
                                 ((unsigned)lut[x >> 24] << 24));
                }
                *reinterpret_cast<i32x4 *>(base + i0) = v;
            } else {
                for (long j = i0; j < hi; j++) base[j] = (int8_t)lut[(int)base[j] + 128];
            }
        }
    } else {
        for (long j = lo + t; j < hi; j += SP_NT) base[j] = (int8_t)lut[(int)base[j] + 128];
    }
}

template <int CIN, int KS, bool POOL, bool RELU, int OMODE, bool FUSE1A = false, int GEO = 0>
int launch_conv(hipStream_t st, const mv_superpoint *net, int li, int B, int H, int W, const int8_t *in,
                int8_t *out, int cstride, Conv1aArgs c1 = Conv1aArgs{}) {
    using G = SpGeo<GEO>;
    const int tiles_x = (W + G::TX - 1) / G::TX, tiles_y = (H + G::TY - 1) / G::TY, ngroups = net->cout_pad[li] / 64;
    const long blocks = (long)B * ngroups * tiles_y * tiles_x;
    MV_REQUIRE(blocks < (1l << 31));
    // the epilogue stores 16 B per lane: NHWC outputs with 16-B aligned pixels
    MV_REQUIRE((OMODE != 0 && !POOL) || (cstride % 16 == 0 && cstride >= 64 * ngroups && ((uintptr_t)out & 15) == 0));
    const char *wd = static_cast<const char *>(net->wdev);
    hipLaunchKernelGGL((k_sp_conv<CIN, KS, POOL, RELU, OMODE, FUSE1A, GEO>), dim3((unsigned)blocks), dim3(SP_NT), 0, st, in,
                       H, W, reinterpret_cast<const i32x4 *>(wd + net->frag_off[li]),
                       reinterpret_cast<const int *>(wd + net->bq_off[li]), net->rs[li], ngroups, tiles_x, tiles_y,
                       out, cstride, c1);
    MV_LAUNCH_CHECK();
    return MV_OK;
}

// the heads through k_sp_head
template <int OMODE>
int launch_head(hipStream_t st, const mv_superpoint *net, int li, int B, int H, int W, const int8_t *in, int8_t *out,
                int cstride, float dq = 0.f, unsigned *pres = nullptr, bool *pres_done = nullptr) {
    if (pres_done) *pres_done = false;
    const int HW = H * W, nblk_f = (HW + 31) / 32;
    const long nblk = (long)B * nblk_f;
    MV_REQUIRE((long)B * HW * 256 < (1l << 40) && nblk > 0 && nblk < (1l << 31) - HD_NB);
    MV_REQUIRE((cstride == 65 || cstride == 256) && (OMODE == 2 || cstride == 65 || ((uintptr_t)out & 15) == 0));
    const unsigned grid = (unsigned)((nblk + HD_NB - 1) / HD_NB);
    const char *wd = static_cast<const char *>(net->wdev);
    const i32x4 *wf = reinterpret_cast<const i32x4 *>(wd + net->frag_off[li]);
    const int *bq = reinterpret_cast<const int *>(wd + net->bq_off[li]);
    const bool full = HW % 32 == 0 && nblk % HD_NB == 0 && ((uintptr_t)out & 3) == 0;
    const bool fuse = OMODE == 1 && pres && full && nblk_f >= HD_NB;
#define MV_HEAD(NCB, FULL, PRES)                                                                                   \
    hipLaunchKernelGGL((k_sp_head<OMODE, NCB, FULL, PRES>), dim3(grid), dim3(SP_NT), 0, st, in, H, W, nblk_f,         \
                       (int)nblk, wf, bq, net->rs[li], out, cstride, dq, pres)
    if (cstride == 65) {
        if (fuse)
            MV_HEAD(3, true, OMODE == 1);
        else if (full)
            MV_HEAD(3, true, false);
        else
            MV_HEAD(3, false, false);
    } else {
        if (fuse)
            MV_HEAD(8, true, OMODE == 1);
        else if (full)
            MV_HEAD(8, true, false);
        else
            MV_HEAD(8, false, false);
    }
#undef MV_HEAD
    MV_LAUNCH_CHECK();
    if (pres_done) *pres_done = fuse;
    return MV_OK;
}

// the 128-channel unpooled layers: the tile geometry covering H x W with fewer padded pixels
// (GEO 1 wins at 24 x 80: 1920 against 3072)
template <int CIN, int KS, bool POOL, bool RELU, int OMODE>
int launch_conv_geo(hipStream_t st, const mv_superpoint *net, int li, int B, int H, int W, const int8_t *in,
                    int8_t *out, int cstride) {
    auto area = [&](int ty, int tx) { return (long)((H + ty - 1) / ty) * ty * ((W + tx - 1) / tx) * tx; };
    if (area(SpGeo<1>::TY, SpGeo<1>::TX) < area(SpGeo<0>::TY, SpGeo<0>::TX))
        return launch_conv<CIN, KS, POOL, RELU, OMODE, false, 1>(st, net, li, B, H, W, in, out, cstride);
    return launch_conv<CIN, KS, POOL, RELU, OMODE, false, 0>(st, net, li, B, H, W, in, out, cstride);
}

constexpr int SP_CIN[12] = {1, 64, 64, 64, 64, 128, 128, 128, 128, 256, 128, 256};
constexpr int SP_COUT[12] = {64, 64, 64, 64, 128, 128, 128, 128, 256, 65, 256, 256};
constexpr int SP_K[12] = {3, 3, 3, 3, 3, 3, 3, 3, 3, 1, 3, 1};

}  // namespace

extern "C" int mv_superpoint_create(mv_context *ctx, const mv_sp_weights *wt, mv_superpoint **out) {
    MV_REQUIRE(ctx && wt && out && wt->in_scale > 0.0);
    *out = nullptr;
    for (int l = 0; l < 12; l++) {
        const mv_sp_layer &L = wt->layer[l];
        MV_REQUIRE(L.w && L.bias && L.cin == SP_CIN[l] && L.cout == SP_COUT[l] && L.k == SP_K[l]);
        MV_REQUIRE(L.w_scale > 0.0 && L.out_scale > 0.0);
    }
    MV_HIP_TRY(hipSetDevice(ctx->device));
    mv_superpoint *net = new mv_superpoint();
    net->device = ctx->device;
    net->in_inv = 1.0f / (float)wt->in_scale;
    net->dq_semi = (float)wt->layer[9].out_scale;
    net->dq_desc = (float)wt->layer[11].out_scale;
    // host image of the device weights
    size_t off = 0;
    for (int l = 0; l < 12; l++) {
        const mv_sp_layer &L = wt->layer[l];
        net->cout_pad[l] = (L.cout + 63) / 64 * 64;
        net->ns[l] = L.k * L.k * L.cin / 32;
        net->frag_off[l] = off;
        off += l == 0 ? 64 * 3 * 4 : (size_t)net->cout_pad[l] / 32 * net->ns[l] * 64 * 16;
        off = mv::align_up(off, 256);
        net->bq_off[l] = off;
        off += (size_t)net->cout_pad[l] * 4;
        off = mv::align_up(off, 256);
    }
    char *hbuf = static_cast<char *>(calloc(off, 1));
    if (!hbuf) {
        delete net;
        return MV_ERR_OUT_OF_MEMORY;
    }
    double in_scale = wt->in_scale;
    for (int l = 0; l < 12; l++) {
        const mv_sp_layer &L = wt->layer[l];
        const int K = L.k, CIN = L.cin, COUT = L.cout;
        if (l == 10) in_scale = wt->layer[7].out_scale;  // convDa reads conv4b, like convPa
        // PyTorch's QuantizeBias (qint32 at w_scale * in_scale, float reciprocal) and XNNPACK's
        // fp32 requantisation scale
        const float binv = 1.0f / (float)(L.w_scale * in_scale);
        net->rs[l] = (float)in_scale * (float)L.w_scale / (float)L.out_scale;
        int *bq = reinterpret_cast<int *>(hbuf + net->bq_off[l]);
        for (int co = 0; co < COUT; co++) {
            float v = nearbyintf(L.bias[co] * binv);
            v = v < -2147483648.f ? -2147483648.f : (v > 2147483520.f ? 2147483520.f : v);
            bq[co] = (int)v;
        }
        if (l == 0) {
            int *pk = reinterpret_cast<int *>(hbuf + net->frag_off[0]);
            for (int co = 0; co < 64; co++) {
                unsigned wv[12] = {0};
                for (int tp = 0; tp < 9; tp++) wv[tp] = (uint8_t)L.w[co * 9 + tp];
                for (int d = 0; d < 3; d++)
                    pk[3 * co + d] = (int)(wv[4 * d] | (wv[4 * d + 1] << 8) | (wv[4 * d + 2] << 16) | (wv[4 * d + 3] << 24));
            }
        } else {
            // fragment (cb, s): lane -> cout cb * 32 + lane % 32, k = 32 s + 16 (lane / 32) + i,
            // k = tap * CIN + cin, tap = ky * K + kx
            int8_t *fr = reinterpret_cast<int8_t *>(hbuf + net->frag_off[l]);
            const int NS = net->ns[l];
            for (int cb = 0; cb < net->cout_pad[l] / 32; cb++)
                for (int s = 0; s < NS; s++)
                    for (int ln = 0; ln < 64; ln++)
                        for (int i = 0; i < 16; i++) {
                            const int co = cb * 32 + ln % 32, k = 32 * s + 16 * (ln / 32) + i;
                            const int tap = k / CIN, ci = k % CIN, ky = tap / K, kx = tap % K;
                            fr[(((size_t)cb * NS + s) * 64 + ln) * 16 + i] =
                                co < COUT ? L.w[(((size_t)co * CIN + ci) * K + ky) * K + kx] : 0;
                        }
        }
        in_scale = L.out_scale;
    }
    if (hipMalloc(&net->wdev, off) != hipSuccess) {
        free(hbuf);
        delete net;
        return MV_ERR_OUT_OF_MEMORY;
    }
    net->wbytes = off;
    const hipError_t e = hipMemcpy(net->wdev, hbuf, off, hipMemcpyHostToDevice);
    free(hbuf);
    if (e != hipSuccess) {
        (void)hipFree(net->wdev);
        delete net;
        mv::set_error(MV_ERR_HIP, "hipMemcpy of the SuperPoint weights: %s", hipGetErrorString(e));
        return MV_ERR_HIP;
    }
    if (hipEventCreateWithFlags(&net->done, hipEventDisableTiming) != hipSuccess) {
        (void)hipFree(net->wdev);
        delete net;
        mv::set_error(MV_ERR_HIP, "hipEventCreate for the SuperPoint net");
        return MV_ERR_HIP;
    }
    *out = net;
    return MV_OK;
}

extern "C" int mv_superpoint_destroy(mv_superpoint *net) {
    if (!net) return MV_OK;
    (void)hipSetDevice(net->device);
    if (net->used) (void)hipEventSynchronize(net->done);  // the last forward, on whatever stream it ran
    if (net->done) (void)hipEventDestroy(net->done);
    if (net->act) (void)hipFree(net->act);
    if (net->wdev) (void)hipFree(net->wdev);
    delete net;
    return MV_OK;
}

namespace {
// the network on `batch` frames into the heads' int8 codes semi [B][cells][65], desc [B][cells][256]
// (Frame layout, before run()'s min-gap step) or, semi_f / desc_f given, into the heads'
// dequantised NCHW float32 outputs (run()'s net.forward); act: the two activation buffers of
// a_bytes each
int sp_network(hipStream_t st, mv_superpoint *net, int batch, int H, int W, int oh, int ow, const uint8_t *images,
               int8_t *A, int8_t *Bf, int8_t *semi, int8_t *desc, float *semi_f = nullptr, float *desc_f = nullptr,
               unsigned *pres = nullptr, bool *pres_done = nullptr) {
    if (pres_done) *pres_done = false;
    const char *wd = static_cast<const char *>(net->wdev);
    int r;
    int h = oh, w = ow;
    MV_PROF_BEGIN(st, "k_sp_conv");
    {
        const Conv1aArgs c1{images, H, W, net->in_inv, net->rs[0], reinterpret_cast<const int *>(wd + net->frag_off[0]),
                            reinterpret_cast<const int *>(wd + net->bq_off[0])};
        if ((r = launch_conv<64, 3, true, true, 0, true>(st, net, 1, batch, h, w, nullptr, Bf, 64, c1)) != MV_OK)
            return r;
    }
    h /= 2, w /= 2;
    if ((r = launch_conv<64, 3, false, true, 0>(st, net, 2, batch, h, w, Bf, A, 64)) != MV_OK) return r;
    if ((r = launch_conv<64, 3, true, true, 0>(st, net, 3, batch, h, w, A, Bf, 64)) != MV_OK) return r;
    h /= 2, w /= 2;
    if ((r = launch_conv<64, 3, false, true, 0>(st, net, 4, batch, h, w, Bf, A, 128)) != MV_OK) return r;
    if ((r = launch_conv<128, 3, true, true, 0>(st, net, 5, batch, h, w, A, Bf, 128)) != MV_OK) return r;
    h /= 2, w /= 2;
    if ((r = launch_conv_geo<128, 3, false, true, 0>(st, net, 6, batch, h, w, Bf, A, 128)) != MV_OK) return r;
    if ((r = launch_conv_geo<128, 3, false, true, 0>(st, net, 7, batch, h, w, A, Bf, 128)) != MV_OK) return r;
    // heads: Bf holds the shared encoder output
    if ((r = launch_conv_geo<128, 3, false, true, 0>(st, net, 8, batch, h, w, Bf, A, 256)) != MV_OK) return r;
    bool pd0 = false, pd1 = false;
    if (pres && !semi_f) {  // the heads OR into chunk 0 of each (frame, head): the rest stays zero
        MV_HIP_TRY(hipMemsetAsync(pres, 0, (size_t)batch * 2 * SP_MG_CHUNKS * 8 * sizeof(unsigned), st));
    }
    if (semi_f)
        r = launch_head<2>(st, net, 9, batch, h, w, A, reinterpret_cast<int8_t *>(semi_f), 65, net->dq_semi);
    else
        r = launch_head<1>(st, net, 9, batch, h, w, A, semi, 65, 0.f, pres, &pd0);
    if (r != MV_OK) return r;
    if ((r = launch_conv_geo<128, 3, false, true, 0>(st, net, 10, batch, h, w, Bf, A, 256)) != MV_OK) return r;
    if (desc_f)
        r = launch_head<2>(st, net, 11, batch, h, w, A, reinterpret_cast<int8_t *>(desc_f), 256, net->dq_desc);
    else
        r = launch_head<1>(st, net, 11, batch, h, w, A, desc, 256, 0.f, pres, &pd1);
    if (r != MV_OK) return r;
    if (pres_done) *pres_done = pd0 && pd1;  // the same geometry: both or neither
    MV_PROF_END(st);
    return MV_OK;
}

// the net's activation buffers (grown to `need` bytes; the previous forward on any stream may
// still read the old ones)
int sp_act(mv_superpoint *net, size_t need) {
    if (net->act_bytes >= need) return MV_OK;
    if (net->act) {
        if (net->used) MV_HIP_TRY(hipEventSynchronize(net->done));
        MV_HIP_TRY(hipFree(net->act));
        net->act = nullptr;
        net->act_bytes = 0;
    }
    if (hipMalloc(&net->act, need) != hipSuccess) return MV_ERR_OUT_OF_MEMORY;
    net->act_bytes = need;
    return MV_OK;
}
}  // namespace

extern "C" int mv_superpoint_forward_dev(mv_context *ctx, mv_superpoint *net, int batch, int H, int W, int oh,
                                         int ow, const uint8_t *images, int8_t *semi, int8_t *desc,
                                         float *semi_scale, float *desc_scale) {
    MV_REQUIRE(ctx && net && batch > 0 && H > 0 && W > 0 && oh >= 8 && ow >= 8 && oh % 8 == 0 && ow % 8 == 0);
    MV_REQUIRE(images && semi && desc && semi_scale && desc_scale && net->device == ctx->device);
    MV_REQUIRE((long)oh * ow * 64 < (1l << 31) && (long)batch * H * W < (1l << 40));
    MV_HIP_TRY(hipSetDevice(ctx->device));
    // activation ping-pong buffers, oh * ow * 16 bytes per frame each (conv1b's pooled output, the
    // largest after the fused conv1a) + the presence masks
    const size_t a_bytes = mv::align_up((size_t)batch * oh * ow * 16, 256);
    const size_t need = 2 * a_bytes + (size_t)batch * 2 * SP_MG_CHUNKS * 8 * sizeof(unsigned);
    int r = sp_act(net, need);
    if (r != MV_OK) return r;
    int8_t *A = static_cast<int8_t *>(net->act), *Bf = A + a_bytes;
    hipStream_t st = ctx->stream;
    // the activations belong to the net, not the context: order this forward after the previous
    // one on whatever stream (context) it ran (free on the same stream)
    if (net->used) MV_HIP_TRY(hipStreamWaitEvent(st, net->done, 0));
    unsigned *pres = reinterpret_cast<unsigned *>(Bf + a_bytes);
    bool pres_done = false;
    if ((r = sp_network(st, net, batch, H, W, oh, ow, images, A, Bf, semi, desc, nullptr, nullptr, pres, &pres_done)) !=
        MV_OK)
        return r;
    const int h = oh / 8, w = ow / 8;
    MV_PROF_BEGIN(st, "k_sp_min_gap");
    if (!pres_done) {
        hipLaunchKernelGGL(k_sp_presence, dim3((unsigned)batch, 2, SP_MG_CHUNKS), dim3(SP_NT), 0, st, semi, desc,
                           (long)h * w, pres);
        MV_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_sp_min_gap, dim3((unsigned)batch, 2, SP_MG_CHUNKS), dim3(SP_NT), 0, st, semi, desc,
                       (long)h * w, net->dq_semi, net->dq_desc, pres, semi_scale, desc_scale);
    MV_LAUNCH_CHECK();
    MV_PROF_END(st);
    MV_HIP_TRY(hipEventRecord(net->done, st));
    net->used = true;
    return MV_OK;
}

extern "C" int mv_superpoint_forward_raw_dev(mv_context *ctx, mv_superpoint *net, int batch, int H, int W, int oh,
                                             int ow, const uint8_t *images, float *semi, float *coarse_desc) {
    MV_REQUIRE(ctx && net && batch > 0 && H > 0 && W > 0 && oh >= 8 && ow >= 8 && oh % 8 == 0 && ow % 8 == 0);
    MV_REQUIRE(images && semi && coarse_desc && net->device == ctx->device);
    MV_REQUIRE((long)oh * ow * 64 < (1l << 31) && (long)batch * H * W < (1l << 40));
    MV_REQUIRE(((uintptr_t)semi & 15) == 0 && ((uintptr_t)coarse_desc & 15) == 0);
    MV_HIP_TRY(hipSetDevice(ctx->device));
    // run()'s network outputs as pairwise_pnp.py receives them (outs = net.forward(inp), :197-199:
    // the quantized model's DeQuantStub): the heads' epilogue writes code * (float) out_scale as
    // NCHW float32 [B][C][oh / 8][ow / 8] directly (no int8 intermediate)
    const size_t a_bytes = mv::align_up((size_t)batch * oh * ow * 16, 256);
    int r = sp_act(net, 2 * a_bytes);
    if (r != MV_OK) return r;
    int8_t *A = static_cast<int8_t *>(net->act), *Bf = A + a_bytes;
    hipStream_t st = ctx->stream;
    if (net->used) MV_HIP_TRY(hipStreamWaitEvent(st, net->done, 0));
    if ((r = sp_network(st, net, batch, H, W, oh, ow, images, A, Bf, nullptr, nullptr, semi, coarse_desc)) != MV_OK)
        return r;
    MV_HIP_TRY(hipEventRecord(net->done, st));
    net->used = true;
    return MV_OK;
}
