/*
 * sp_oracle.c -- CPU ORACLE (test infrastructure only) of the quantized SuperPoint front-end
 * (SURVEY 8(f)1): python/superpoint_inference.py:29-83 (the net), :181-208 (run: forward, then
 * the per-output min-gap quantisation), :613-628 (image / 255, resize to 192 x 640), with the
 * int8 arithmetic of the library the reference runs it on: PyTorch's quantized engine
 * (torch.backends.quantized.engine = 'qnnpack', superpoint_inference.py:110; qint8 activations
 * take PyTorch's XNNPACK qs8 path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Restated arithmetic (pinned bit for bit against torch 2.10's own kernels in
 * tests/test_superpoint.py; the reference's golden quantized_image0.h agrees on 92-94 % of its
 * int8 values, the platform difference SURVEY 8(c) measured):
 *   resize   torch.nn.functional.interpolate(bilinear, align_corners=False, antialias=False) on
 *            the CPU: source index fma(in/out, dst + 0.5, -0.5) clamped at 0, lambda = src - i0,
 *            t_r = fma(a_r0, w0, a_r1 w1), out = fma(t_0, h0, t_1 h1);
 *   quantise q = clamp(nearbyint(x * (1 / (float) scale)), -128, 127)  (quantize_per_tensor, qint8);
 *   conv     int32 accumulation of int8 x int8 (zero points 0), bias quantised once as
 *            nearbyint(b * (1 / (float)(w_scale * in_scale)))  (PyTorch QuantizeBias, qint32),
 *            requantised as nearbyint((float) acc * rs) clamped to int8 with
 *            rs = (float) in_scale * (float) w_scale / (float) out_scale  (XNNPACK fp32 params);
 *   relu     max(q, 0) (zero point 0);  pool: 2 x 2 max of int8;
 *   min gap  f = (float) q * (float) scale (dequantize), scale0 = min of the gaps between the
 *            sorted distinct f, out = nearbyint(f / scale0)  (torch.unique / min / round).
 * Layouts: activations CHW int8; outputs [cells][C] with cell p = gx * rows + gy (the
 * header writer's loop order, superpoint_inference.py:649-655).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

typedef struct {
    const int8_t *w;   /* [cout][cin][k][k] */
    const float *bias; /* [cout] */
    int cin, cout, k;
    double w_scale, out_scale;
} orc_sp_layer;

typedef struct {
    double in_scale;
    orc_sp_layer layer[12]; /* conv1a 1b 2a 2b 3a 3b 4a 4b Pa Pb Da Db */
} orc_sp_net;

static void sp_weights(int n_in, int n_out, int *i0, int *i1, float *l0, float *l1) {
    const float scale = (float)n_in / (float)n_out;
    for (int d = 0; d < n_out; d++) {
        float src = fmaf(scale, (float)d + 0.5f, -0.5f);
        if (src < 0.f) src = 0.f;
        int i = (int)floorf(src);
        if (i > n_in - 1) i = n_in - 1;
        float lam = src - (float)i;
        lam = lam < 0.f ? 0.f : (lam > 1.f ? 1.f : lam);
        i0[d] = i;
        i1[d] = i + (i < n_in - 1 ? 1 : 0);
        l1[d] = lam;
        l0[d] = 1.f - lam;
    }
}

/* img [H][W] uint8 -> out [oh][ow] float: (img / 255) resized bilinearly */
ORC_EXPORT void orc_sp_resize(const uint8_t *img, int H, int W, int oh, int ow, float *out) {
    int *y0 = malloc(sizeof(int) * oh), *y1 = malloc(sizeof(int) * oh);
    int *x0 = malloc(sizeof(int) * ow), *x1 = malloc(sizeof(int) * ow);
    float *h0 = malloc(sizeof(float) * oh), *h1 = malloc(sizeof(float) * oh);
    float *w0 = malloc(sizeof(float) * ow), *w1 = malloc(sizeof(float) * ow);
    sp_weights(H, oh, y0, y1, h0, h1);
    sp_weights(W, ow, x0, x1, w0, w1);
    for (int y = 0; y < oh; y++)
        for (int x = 0; x < ow; x++) {
            const float a00 = (float)img[(size_t)y0[y] * W + x0[x]] / 255.0f;
            const float a01 = (float)img[(size_t)y0[y] * W + x1[x]] / 255.0f;
            const float a10 = (float)img[(size_t)y1[y] * W + x0[x]] / 255.0f;
            const float a11 = (float)img[(size_t)y1[y] * W + x1[x]] / 255.0f;
            const float t0 = fmaf(a00, w0[x], a01 * w1[x]);
            const float t1 = fmaf(a10, w0[x], a11 * w1[x]);
            out[(size_t)y * ow + x] = fmaf(t0, h0[y], t1 * h1[y]);
        }
    free(y0), free(y1), free(x0), free(x1), free(h0), free(h1), free(w0), free(w1);
}

ORC_EXPORT void orc_sp_quantize(const float *x, long n, double scale, int8_t *q) {
    const float inv = 1.0f / (float)scale;
    for (long i = 0; i < n; i++) {
        float v = nearbyintf(x[i] * inv);
        v = v < -128.f ? -128.f : (v > 127.f ? 127.f : v);
        q[i] = (int8_t)v;
    }
}

/* one quantized conv (stride 1, padding k / 2, zero points 0) on CHW int8, optional relu and
 * 2 x 2 max pool (h, w even) */
ORC_EXPORT void orc_sp_conv(const int8_t *in, int h, int w, const orc_sp_layer *L, double in_scale, int relu,
                            int pool, int8_t *out) {
    const int cin = L->cin, cout = L->cout, k = L->k, p = k / 2;
    const float rs = (float)in_scale * (float)L->w_scale / (float)L->out_scale;
    const float binv = 1.0f / (float)(L->w_scale * in_scale);
    int32_t *acc = malloc(sizeof(int32_t) * (size_t)h * w);
    int8_t *full = pool ? malloc((size_t)h * w) : NULL;
    for (int co = 0; co < cout; co++) {
        memset(acc, 0, sizeof(int32_t) * (size_t)h * w);
        for (int ci = 0; ci < cin; ci++) {
            const int8_t *src = in + (size_t)ci * h * w;
            for (int ky = 0; ky < k; ky++)
                for (int kx = 0; kx < k; kx++) {
                    const int32_t wv = L->w[(((size_t)co * cin + ci) * k + ky) * k + kx];
                    if (wv == 0) continue;
                    const int dy = ky - p, dx = kx - p;
                    const int ya = dy < 0 ? -dy : 0, yb = dy > 0 ? h - dy : h;
                    const int xa = dx < 0 ? -dx : 0, xb = dx > 0 ? w - dx : w;
                    for (int y = ya; y < yb; y++) {
                        int32_t *a = acc + (size_t)y * w;
                        const int8_t *s = src + (size_t)(y + dy) * w + dx;
                        for (int x = xa; x < xb; x++) a[x] += wv * (int32_t)s[x];
                    }
                }
        }
        float bqf = nearbyintf(L->bias[co] * binv);
        bqf = bqf < -2147483648.f ? -2147483648.f : (bqf > 2147483520.f ? 2147483520.f : bqf);
        const int32_t bq = (int32_t)bqf;
        int8_t *dst = pool ? full : out + (size_t)co * h * w;
        for (long i = 0; i < (long)h * w; i++) {
            float v = nearbyintf((float)(acc[i] + bq) * rs);
            v = v < -128.f ? -128.f : (v > 127.f ? 127.f : v);
            if (relu && v < 0.f) v = 0.f;
            dst[i] = (int8_t)v;
        }
        if (pool) {
            int8_t *o = out + (size_t)co * (h / 2) * (w / 2);
            for (int y = 0; y < h / 2; y++)
                for (int x = 0; x < w / 2; x++) {
                    int8_t m = full[(size_t)(2 * y) * w + 2 * x];
                    const int8_t c1 = full[(size_t)(2 * y) * w + 2 * x + 1], c2 = full[(size_t)(2 * y + 1) * w + 2 * x],
                                 c3 = full[(size_t)(2 * y + 1) * w + 2 * x + 1];
                    m = c1 > m ? c1 : m;
                    m = c2 > m ? c2 : m;
                    m = c3 > m ? c3 : m;
                    o[(size_t)y * (w / 2) + x] = m;
                }
        }
    }
    free(acc);
    free(full);
}

static int cmp_float(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

/* run()'s per-output quantisation (superpoint_inference.py:199-206) of the int8 network output
 * q [C][hc][wc] (its dequantised values (float) q * (float) scale) into out [cells][C]
 * (cell p = gx * hc + gy); returns scale0 (0 if fewer than two distinct values -- torch.min of
 * an empty tensor raises there -- and then the raw codes are written) */
ORC_EXPORT float orc_sp_min_gap(const int8_t *q, int C, int hc, int wc, double scale, int8_t *out) {
    const float s = (float)scale;
    int present[256] = {0};
    const long n = (long)C * hc * wc;
    for (long i = 0; i < n; i++) present[q[i] + 128] = 1;
    float vals[256];
    int nv = 0;
    for (int v = 0; v < 256; v++)
        if (present[v]) vals[nv++] = (float)(v - 128) * s;
    qsort(vals, nv, sizeof(float), cmp_float);
    float g = INFINITY;
    for (int i = 1; i < nv; i++) {
        const float d = vals[i] - vals[i - 1];
        if (d > 0.f && d < g) g = d;
    }
    if (nv < 2) g = 0.f; /* the raw codes are written */
    for (int c = 0; c < C; c++)
        for (int gy = 0; gy < hc; gy++)
            for (int gx = 0; gx < wc; gx++) {
                const int8_t qv = q[((size_t)c * hc + gy) * wc + gx];
                if (g == 0.f) {
                    out[((size_t)gx * hc + gy) * C + c] = qv;
                    continue;
                }
                const float f = (float)qv * s;
                float r = nearbyintf(f / g);
                r = r < -128.f ? -128.f : (r > 127.f ? 127.f : r);
                out[((size_t)gx * hc + gy) * C + c] = (int8_t)r;
            }
    return g;
}

/* the whole front-end: img [H][W] uint8 -> semi [cells][65], desc [cells][256] (int8 after the
 * min-gap quantisation) and their scales; the raw network outputs (int8, [65|256][hc][wc]) too
 * when semi_raw / desc_raw are given.  oh, ow: the resized image (multiples of 8). */
ORC_EXPORT int orc_sp_forward(const uint8_t *img, int H, int W, int oh, int ow, const orc_sp_net *net, int8_t *semi,
                              int8_t *desc, float *semi_scale, float *desc_scale, int8_t *semi_raw, int8_t *desc_raw) {
    if (oh % 8 || ow % 8) return -1;
    const size_t npx = (size_t)oh * ow;
    float *x = malloc(sizeof(float) * npx);
    int8_t *a = malloc(64 * npx), *b = malloc(64 * npx);
    orc_sp_resize(img, H, W, oh, ow, x);
    orc_sp_quantize(x, (long)npx, net->in_scale, b);
    const orc_sp_layer *L = net->layer;
    int h = oh, w = ow;
    orc_sp_conv(b, h, w, &L[0], net->in_scale, 1, 0, a);
    orc_sp_conv(a, h, w, &L[1], L[0].out_scale, 1, 1, b);
    h /= 2, w /= 2;
    orc_sp_conv(b, h, w, &L[2], L[1].out_scale, 1, 0, a);
    orc_sp_conv(a, h, w, &L[3], L[2].out_scale, 1, 1, b);
    h /= 2, w /= 2;
    orc_sp_conv(b, h, w, &L[4], L[3].out_scale, 1, 0, a);
    orc_sp_conv(a, h, w, &L[5], L[4].out_scale, 1, 1, b);
    h /= 2, w /= 2;
    orc_sp_conv(b, h, w, &L[6], L[5].out_scale, 1, 0, a);
    orc_sp_conv(a, h, w, &L[7], L[6].out_scale, 1, 0, b); /* b: the shared encoder output */
    const size_t cells = (size_t)h * w;
    int8_t *t = malloc(256 * cells), *sr = malloc(65 * cells), *dr = malloc(256 * cells);
    orc_sp_conv(b, h, w, &L[8], L[7].out_scale, 1, 0, t);
    orc_sp_conv(t, h, w, &L[9], L[8].out_scale, 0, 0, sr);
    orc_sp_conv(b, h, w, &L[10], L[7].out_scale, 1, 0, t);
    orc_sp_conv(t, h, w, &L[11], L[10].out_scale, 0, 0, dr);
    *semi_scale = orc_sp_min_gap(sr, 65, h, w, L[9].out_scale, semi);
    *desc_scale = orc_sp_min_gap(dr, 256, h, w, L[11].out_scale, desc);
    if (semi_raw) memcpy(semi_raw, sr, 65 * cells);
    if (desc_raw) memcpy(desc_raw, dr, 256 * cells);
    free(x), free(a), free(b), free(t), free(sr), free(dr);
    return 0;
}
