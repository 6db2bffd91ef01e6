/*
 * mv_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * A clean-room C restatement of the reference's tracking hot path
 * (rogerhh/maveric-slam @ 2025-01-17).  It is the CHECKER for the HIP product
 * path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  Nothing in maveric-slam_amd/ links or calls it.
 *
 * Pinning (see tests/test_oracle_pinning.py):
 *   - softmax / top-N / ransac / recover_pose / svd are checked bit-for-bit
 *     against the reference's own top_N.c + pnp_solver.c + svd.h compiled from
 *     /root/reference by oracle/Makefile into oracle/_ref/libmv_ref.so;
 *   - the gemmini matmul restatement against include/gemmini_functions_cpu.h
 *     compiled the same way;
 *   - the exact-softmax argmax against include/data/quantized/pair0_gt.h;
 *   - the windowed match loop (src/tracking_main.c:103-194) cannot be built:
 *     tracking_main.c includes quantized_pair0.h, which the reference does not
 *     ship.  Its restatement is pinned through the pinned softmax/top-N stages
 *     plus committed golden match lists (tests/golden/window_*.npz), i.e.
 *     "partially pinned" -- see DESIGN.md section Oracle.
 *
 * Every arithmetic expression keeps the reference's evaluation order
 * (float/double promotions included); compile with -ffp-contract=off.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* Approximate softmax and top-N                 (src/top_N.c:7-165)        */
/* ------------------------------------------------------------------------ */
#define ORC_TAYLOR_TERMS 5 /* top_N.c:7  (P) */

/* F7 of SURVEY.md: tracking_main.c calls compute_softmax/compute_top_N without
 * a prototype, so the float scale is promoted to double and the callee reads
 * the low 32 bits of that double as its float argument (x86-64 SysV ABI). */
ORC_EXPORT float orc_scale_as_built(float scale) {
    double d = (double)scale;
    uint64_t bits;
    memcpy(&bits, &d, sizeof bits);
    uint32_t lo = (uint32_t)(bits & 0xffffffffu);
    float f;
    memcpy(&f, &lo, sizeof f);
    return f;
}

/* top_N.c:59-63 (and again :141-145): sp[i] = sp[i-1] * scale / i */
static void orc_scale_poly(float scale, float sp[ORC_TAYLOR_TERMS]) {
    sp[0] = 1.0f;
    for (int i = 1; i < ORC_TAYLOR_TERMS; i++) sp[i] = sp[i - 1] * scale / (float)i;
}

/* top_N.c:12-20: 1 + sum_{i=1..4} sp[i] * x^i, x^i as an int */
ORC_EXPORT float orc_approx_exp(const float *sp, int8_t x) {
    float acc = 1.0f;
    int32_t xp = x;
    for (int i = 1; i < ORC_TAYLOR_TERMS; i++) {
        acc += sp[i] * (float)xp;
        if (i + 1 < ORC_TAYLOR_TERMS) xp *= x; /* the reference also forms x^5 (unused) */
    }
    return acc;
}

/* top_N.c:22-49 */
static void orc_approx_softmax(const float *sp, const int8_t *row, int *max_index, float *max_prob) {
    int best = 64;
    float best_e = 0.0f;
    float den = FLT_MIN;
    for (int i = 0; i < 65; i++) {
        if (row[i] < 0) continue;
        float e = orc_approx_exp(sp, row[i]);
        if (i != 64 && e > best_e) {
            best_e = e;
            best = i;
        }
        den += e;
    }
    *max_index = best;
    *max_prob = best_e / den;
}

/* top_N.c:136-165.  `cells` generalises the hard-coded 1920. */
ORC_EXPORT void orc_compute_softmax(float scale, const int8_t *semi, int cells, int *num_valid,
                                    int *max_indices, float *probs) {
    float sp[ORC_TAYLOR_TERMS];
    orc_scale_poly(scale, sp);
    for (int c = 0; c < cells; c++) {
        int mi;
        float pr;
        orc_approx_softmax(sp, semi + (size_t)c * 65, &mi, &pr);
        max_indices[c] = mi;
        if (mi != 64) {
            probs[c] = pr;
            (*num_valid)++;
        } else {
            probs[c] = -1.0f;
        }
    }
}

/* top_N.c:53-134.  Returns 0, or -1 where the reference calls exit(1)
 * (num_valid reaching `cap`, MAX_VALID_FEATURES=1000 at :51,91-94). */
ORC_EXPORT int orc_compute_top_N(float scale, const int8_t *semi, int cells, int N, int cap,
                                 int *num_selected, int *N_patches, int *N_indices, float *N_probs) {
    float sp[ORC_TAYLOR_TERMS];
    orc_scale_poly(scale, sp);
    *num_selected = 0;
    int *vp = (int *)malloc(sizeof(int) * (size_t)cap);
    int *vi = (int *)malloc(sizeof(int) * (size_t)cap);
    float *vpr = (float *)malloc(sizeof(float) * (size_t)cap);
    float pmax = 0.0f, pmin = FLT_MAX;
    int nv = 0, status = 0;
    for (int c = 0; c < cells; c++) {
        int mi = 64;
        float pr = -1.0f;
        orc_approx_softmax(sp, semi + (size_t)c * 65, &mi, &pr);
        if (mi != 64 && (double)pr > 0.01) {
            vp[nv] = c;
            vi[nv] = mi;
            vpr[nv] = pr;
            if (pr > pmax) pmax = pr;
            if (pr < pmin) pmin = pr;
            nv++;
            if (nv >= cap) {
                status = -1;
                goto done;
            }
        }
    }
    if (nv <= N) {
        *num_selected = nv;
        for (int k = 0; k < nv; k++) {
            N_patches[k] = vp[k];
            N_indices[k] = vi[k];
            N_probs[k] = vpr[k];
        }
        goto done;
    }
    {
        float split = (float)N / (float)nv;
        float thr = pmax * split + pmin * (1 - split);
        for (int k = 0; k < nv; k++) {
            if (vpr[k] >= thr) {
                N_patches[*num_selected] = vp[k];
                N_indices[*num_selected] = vi[k];
                N_probs[*num_selected] = vpr[k];
                (*num_selected)++;
                if (*num_selected >= N) break;
            }
        }
    }
done:
    free(vp);
    free(vi);
    free(vpr);
    return status;
}

/* ------------------------------------------------------------------------ */
/* Windowed int8 descriptor match              (src/tracking_main.c:18-194) */
/* ------------------------------------------------------------------------ */
typedef struct {
    int shift_x, shift_y, radius; /* tracking_main.c:104-106 (4,4,4) */
    int max_matches;              /* MAX_NUM_MATCH 150, :13 */
    int as_built;                 /* 1: stale-norm / 64-dim / int32-wrap (F8); 0: exact cosine */
} orc_window_params;

static int32_t wrap_mul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* squared_dist, tracking_main.c:18-43: the full 256-D dot and both squared norms when
 * *norm1_squared is 0 (the first valid candidate of a query), else the 64-D dot and query norm
 * with *norm1_squared left as it was (stale).  Pinned against the reference's own function
 * (tests/test_oracle_pinning.py::test_squared_dist_pinned). */
ORC_EXPORT void orc_squared_dist(const int8_t *desc1, const int8_t *desc2, int32_t *sum, int32_t *norm1_squared,
                                 int32_t *norm2_squared) {
    int32_t s = 0, n2 = 0;
    if (*norm1_squared == 0) {
        int32_t n1 = 0;
        for (int k = 0; k < 256; k++) {
            s += desc1[k] * desc2[k];
            n1 += desc1[k] * desc1[k];
            n2 += desc2[k] * desc2[k];
        }
        *norm1_squared = n1;
    } else {
        for (int k = 0; k < 64; k++) {
            s += desc1[k] * desc2[k];
            n2 += desc2[k] * desc2[k];
        }
    }
    *sum = s;
    *norm2_squared = n2;
}
/* tracking_main.c:154: (int)dot*dot / (float)(int)(n1*n2), both int products wrapping */
ORC_EXPORT float orc_window_score(int32_t dot, int32_t n1, int32_t n2) {
    return (float)wrap_mul(dot, dot) / (float)wrap_mul(n1, n2);
}
/* tracking_main.c:155: the float score against MATCH_THRESHOLD^2 in double */
ORC_EXPORT int orc_window_pass(float d) { return (double)d > 0.9 * 0.9; }

/* Returns the number of matches; points are [max_matches][2] (x, y) pixels.
 * q_of_match (optional) receives the query slot i of each match. */
ORC_EXPORT int orc_window_match(int rows, int cols, const int8_t *desc0, const int *max_idx0,
                                const float *probs0, const int8_t *desc1, int nq, const int *patches1,
                                const int *indices1, const orc_window_params *p, float *points1,
                                float *points2, int *q_of_match, float *score_of_match) {
    int nm = 0;
    for (int i = 0; i < nq; i++) {
        int patch1 = patches1[i];
        int x1 = patch1 / rows, y1 = patch1 % rows; /* patch_to_grid, :59-62 */
        const int8_t *q = desc1 + (size_t)patch1 * 256;
        int found = 0, best_index = -1, bx = 0, by = 0;
        float best = 0.0f;
        int64_t bdot = 0, bn1 = 0; /* as-intended running best (exact rational) */
        int xlo = x1 + p->shift_x - p->radius, xhi = x1 + p->shift_x + p->radius;
        int ylo = y1 + p->shift_y - p->radius, yhi = y1 + p->shift_y + p->radius;
        if (xlo < 0) xlo = 0;
        if (xhi > cols - 1) xhi = cols - 1;
        if (ylo < 0) ylo = 0;
        if (yhi > rows - 1) yhi = rows - 1;
        int32_t n1 = 0; /* :133, reset per query, latched by the first candidate */
        for (int x0 = xlo; x0 <= xhi; x0++) {
            for (int y0 = ylo; y0 <= yhi; y0++) {
                int patch0 = x0 * rows + y0; /* grid_to_patch, :64-66 */
                int idx0 = max_idx0[patch0];
                if (idx0 == 64) continue;
                if ((double)probs0[patch0] < 0.2) continue; /* :146 */
                const int8_t *c = desc0 + (size_t)patch0 * 256;
                if (p->as_built) {
                    /* squared_dist(desc0, desc1, ...) :18-43 -- note the argument order:
                     * its "desc1/norm1" is the CANDIDATE, "desc2/norm2" the query. */
                    int32_t dot = 0, n2 = 0;
                    orc_squared_dist(c, q, &dot, &n1, &n2);
                    const float d = orc_window_score(dot, n1, n2);
                    if (orc_window_pass(d)) {
                        if (!found || d > best) {
                            found = 1;
                            best_index = idx0;
                            best = d;
                            bx = x0;
                            by = y0;
                        }
                    }
                } else {
                    int64_t dot = 0, na = 0, nb = 0;
                    for (int k = 0; k < 256; k++) {
                        dot += c[k] * q[k];
                        na += c[k] * c[k];
                        nb += q[k] * q[k];
                    }
                    if (dot <= 0 || na == 0 || nb == 0) continue;
                    /* cos > 0.9  <=>  100 dot^2 > 81 na nb   (exact) */
                    if ((unsigned __int128)(100 * dot * dot) <= (unsigned __int128)81 * (uint64_t)(na * nb))
                        continue;
                    /* strictly better: dot^2/na > bdot^2/bn1 */
                    int better = !found ||
                                 (unsigned __int128)(dot * dot) * (uint64_t)bn1 >
                                     (unsigned __int128)(bdot * bdot) * (uint64_t)na;
                    if (better) {
                        found = 1;
                        best_index = idx0;
                        bdot = dot;
                        bn1 = na;
                        best = (float)((double)dot * (double)dot / ((double)na * (double)nb));
                        bx = x0;
                        by = y0;
                    }
                }
            }
        }
        if (found && nm < p->max_matches) { /* :167-188 */
            int idx1 = indices1[i];
            points1[nm * 2 + 0] = (float)(bx * 8 + best_index % 8);
            points1[nm * 2 + 1] = (float)(by * 8 + best_index / 8);
            points2[nm * 2 + 0] = (float)(x1 * 8 + idx1 % 8);
            points2[nm * 2 + 1] = (float)(y1 * 8 + idx1 / 8);
            if (q_of_match) q_of_match[nm] = i;
            if (score_of_match) score_of_match[nm] = best;
            nm++;
        }
        if (nm >= p->max_matches) break; /* :190-192 */
    }
    return nm;
}

/* ------------------------------------------------------------------------ */
/* McAdams et al. 3x3 SVD (TR1690, 2011)            (include/svd/svd.h)     */
/* Restated with the same float/double evaluation order.                     */
/* ------------------------------------------------------------------------ */
static float orc_rsqrt(float x) { /* svd.h:37-48, one Newton step */
    float h = 0.5f * x;
    int32_t i;
    memcpy(&i, &x, 4);
    i = 0x5f375a82 - (i >> 1);
    float y;
    memcpy(&y, &i, 4);
    return y * (1.5f - h * y * y);
}

static float orc_rsqrt2(float x) { /* svd.h:54-62, two Newton steps */
    float h = 0.5f * x;
    int32_t i;
    memcpy(&i, &x, 4);
    i = 0x5f37599e - (i >> 1);
    float y;
    memcpy(&y, &i, 4);
    y = y * (1.5f - h * y * y);
    return y * (1.5f - h * y * y);
}

/* Symmetric 3x3 stored as s[0]=s11 s[1]=s21 s[2]=s22 s[3]=s31 s[4]=s32 s[5]=s33;
 * quaternion q = (x, y, z, w).  One Jacobi conjugation (svd.h:148-216). */
static void orc_jacobi_step(int x, int y, int z, float s[6], float q[4]) {
    float ch = 2 * (s[0] - s[2]), sh = s[1];
    int take = 5.828427124 * sh * sh < (double)(ch * ch); /* gamma test in double */
    float w = orc_rsqrt(ch * ch + sh * sh);
    ch = take ? w * ch : (float)0.923879532;
    sh = take ? w * sh : (float)0.3826834323;

    float sc = ch * ch + sh * sh;
    float a = (ch * ch - sh * sh) / sc;
    float b = (2 * sh * ch) / sc;
    float t11 = s[0], t21 = s[1], t22 = s[2], t31 = s[3], t32 = s[4], t33 = s[5];
    float n11 = a * (a * t11 + b * t21) + b * (a * t21 + b * t22);
    float n21 = a * (-b * t11 + a * t21) + b * (-b * t21 + a * t22);
    float n22 = -b * (-b * t11 + a * t21) + a * (-b * t21 + a * t22);
    float n31 = a * t31 + b * t32;
    float n32 = -b * t31 + a * t32;
    float n33 = t33;

    float tq[3] = {q[0] * sh, q[1] * sh, q[2] * sh};
    sh *= q[3];
    q[0] *= ch;
    q[1] *= ch;
    q[2] *= ch;
    q[3] *= ch;
    q[z] += sh;
    q[3] -= tq[z];
    q[x] += tq[y];
    q[y] -= tq[x];

    /* cyclic relabel for the next pair */
    s[0] = n22;
    s[1] = n32;
    s[2] = n33;
    s[3] = n21;
    s[4] = n31;
    s[5] = n11;
}

static void orc_qr_givens(float a1, float a2, float *ch, float *sh) { /* svd.h:277-291 */
    float eps = (float)1e-6;
    float r2 = a1 * a1 + a2 * a2;
    float rho = r2 * orc_rsqrt2(r2);
    float s = rho > eps ? a2 : 0;
    float c = fabsf(a1) + fmaxf(rho, eps);
    if (a1 < 0) {
        float t = s;
        s = c;
        c = t;
    }
    float w = orc_rsqrt(c * c + s * s);
    *ch = c * w;
    *sh = s * w;
}

/* A, U, V row-major 3x3; S the diagonal of R.  Mirrors svd() (svd.h:358-405)
 * and call_svd()'s outputs (pnp_solver.c:8-25): the third output is V, not V^T. */
ORC_EXPORT void orc_svd3(const float *A, float *U, float *S, float *V) {
    float a[3][3];
    for (int i = 0; i < 9; i++) a[i / 3][i % 3] = A[i];
    /* A^T A, each entry summed k = 0,1,2 left to right (multAtB, :105-120) */
    float m[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m[i][j] = a[0][i] * a[0][j] + a[1][i] * a[1][j] + a[2][i] * a[2][j];
    float s[6] = {m[0][0], m[1][0], m[1][1], m[2][0], m[2][1], m[2][2]};
    float q[4] = {0, 0, 0, 1};
    for (int sweep = 0; sweep < 4; sweep++) { /* jacobiEigenanlysis, :226-244 */
        orc_jacobi_step(0, 1, 2, s, q);
        orc_jacobi_step(1, 2, 0, s, q);
        orc_jacobi_step(2, 0, 1, s, q);
    }
    /* quaternion -> V (quatToMat3, :122-146) */
    float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    float xx = qx * qx, yy = qy * qy, zz = qz * qz, xz = qx * qz, xy = qx * qy, yz = qy * qz;
    float wx = qw * qx, wy = qw * qy, wz = qw * qz;
    float v[3][3] = {{1 - 2 * (yy + zz), 2 * (xy - wz), 2 * (xz + wy)},
                     {2 * (xy + wz), 1 - 2 * (xx + zz), 2 * (yz - wx)},
                     {2 * (xz - wy), 2 * (yz + wx), 1 - 2 * (xx + yy)}};
    /* B = A V (multAB, :86-102) */
    float bm[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) bm[i][j] = a[i][0] * v[0][j] + a[i][1] * v[1][j] + a[i][2] * v[2][j];
    /* sort columns by descending norm with sign-flipping swaps (:247-274) */
    float rho[3];
    for (int j = 0; j < 3; j++) rho[j] = bm[0][j] * bm[0][j] + bm[1][j] * bm[1][j] + bm[2][j] * bm[2][j];
    static const int pairs[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int pidx = 0; pidx < 3; pidx++) {
        int c0 = pairs[pidx][0], c1 = pairs[pidx][1];
        if (rho[c0] < rho[c1]) {
            for (int r = 0; r < 3; r++) {
                float t = -bm[r][c0];
                bm[r][c0] = bm[r][c1];
                bm[r][c1] = t;
                t = -v[r][c0];
                v[r][c0] = v[r][c1];
                v[r][c1] = t;
            }
            if (pidx < 2) {
                float t = rho[c0];
                rho[c0] = rho[c1];
                rho[c1] = t;
            }
        }
    }
    /* QR by three Givens rotations (QRDecomposition, :294-356) */
    float ch1, sh1, ch2, sh2, ch3, sh3, ga, gb;
    float r[3][3];
    orc_qr_givens(bm[0][0], bm[1][0], &ch1, &sh1);
    ga = 1 - 2 * sh1 * sh1;
    gb = 2 * ch1 * sh1;
    for (int j = 0; j < 3; j++) {
        r[0][j] = ga * bm[0][j] + gb * bm[1][j];
        r[1][j] = -gb * bm[0][j] + ga * bm[1][j];
        r[2][j] = bm[2][j];
    }
    orc_qr_givens(r[0][0], r[2][0], &ch2, &sh2);
    ga = 1 - 2 * sh2 * sh2;
    gb = 2 * ch2 * sh2;
    for (int j = 0; j < 3; j++) {
        float top = ga * r[0][j] + gb * r[2][j];
        float bot = -gb * r[0][j] + ga * r[2][j];
        bm[0][j] = top;
        bm[1][j] = r[1][j];
        bm[2][j] = bot;
    }
    orc_qr_givens(bm[1][1], bm[2][1], &ch3, &sh3);
    ga = 1 - 2 * sh3 * sh3;
    gb = 2 * ch3 * sh3;
    for (int j = 0; j < 3; j++) {
        r[0][j] = bm[0][j];
        r[1][j] = ga * bm[1][j] + gb * bm[2][j];
        r[2][j] = -gb * bm[1][j] + ga * bm[2][j];
    }
    float p1 = sh1 * sh1, p2 = sh2 * sh2, p3 = sh3 * sh3;
    U[0] = (-1 + 2 * p1) * (-1 + 2 * p2);
    U[1] = 4 * ch2 * ch3 * (-1 + 2 * p1) * sh2 * sh3 + 2 * ch1 * sh1 * (-1 + 2 * p3);
    U[2] = 4 * ch1 * ch3 * sh1 * sh3 - 2 * ch2 * (-1 + 2 * p1) * sh2 * (-1 + 2 * p3);
    U[3] = 2 * ch1 * sh1 * (1 - 2 * p2);
    U[4] = -8 * ch1 * ch2 * ch3 * sh1 * sh2 * sh3 + (-1 + 2 * p1) * (-1 + 2 * p3);
    U[5] = -2 * ch3 * sh3 + 4 * sh1 * (ch3 * sh1 * sh3 + ch1 * ch2 * sh2 * (-1 + 2 * p3));
    U[6] = 2 * ch2 * sh2;
    U[7] = 2 * ch3 * (1 - 2 * p2) * sh3;
    U[8] = (-1 + 2 * p2) * (-1 + 2 * p3);
    S[0] = r[0][0];
    S[1] = r[1][1];
    S[2] = r[2][2];
    for (int i = 0; i < 9; i++) V[i] = v[i / 3][i % 3];
}

/* ------------------------------------------------------------------------ */
/* Pose: stub essential-matrix RANSAC + pose recovery (src/pnp_solver.c)    */
/* ------------------------------------------------------------------------ */
ORC_EXPORT void orc_normalize_points(int n, const float *pts, const float *K, float *out) { /* :28-34 */
    for (int i = 0; i < n; i++) {
        out[2 * i + 0] = (pts[2 * i + 0] - K[2]) / K[0];
        out[2 * i + 1] = (pts[2 * i + 1] - K[5]) / K[4];
    }
}

ORC_EXPORT float orc_reprojection_error(const float *p1, const float *p2, const float *E) { /* :89-105 */
    float h1[3] = {p1[0], p1[1], 1.0f}, h2[3] = {p2[0], p2[1], 1.0f};
    float err = 0;
    for (int i = 0; i < 3; i++) {
        float t = E[3 * i + 0] * h1[0] + E[3 * i + 1] * h1[1] + E[3 * i + 2] * h1[2];
        float d = t - h2[i];
        err += d * d;
    }
    return err;
}

/* :110-165 with the stubbed solve of :36-86 (E == I whatever the sample).
 * The 8 sample indices per iteration are drawn with libc rand() exactly as
 * the reference does, so the caller's rand() stream advances identically.
 * Returns -1 for n <= 0 (the reference divides by zero, :123). */
ORC_EXPORT int orc_ransac_essential_matrix(int n, const float *pts1, const float *pts2, const float *K,
                                           int iters, float thr, float *best_E, int *best_inliers,
                                           int *num_inliers) {
    (void)K;
    if (n <= 0) return -1;
    int best = 0;
    int *inl = (int *)malloc(sizeof(int) * 1000);
    for (int it = 0; it < iters; it++) {
        for (int s = 0; s < 8; s++) (void)(rand() % n);
        float E[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        int cnt = 0;
        for (int i = 0; i < n; i++) {
            float e = orc_reprojection_error(pts1 + 2 * i, pts2 + 2 * i, E);
            if (e < thr && cnt < 1000) inl[cnt++] = i;
        }
        if (cnt > best || cnt == 1000) {
            best = cnt;
            *num_inliers = cnt;
            memcpy(best_E, E, sizeof E);
            memcpy(best_inliers, inl, sizeof(int) * (size_t)cnt);
        }
    }
    free(inl);
    return 0;
}

/* :168-194: R1 = U W, R2 = U W^T, t = U[:,2] */
ORC_EXPORT void orc_recover_pose(const float *E, float *R1, float *R2, float *t) {
    float U[9], S[3], V[9];
    orc_svd3(E, U, S, V);
    static const float W[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    static const float Wt[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            R1[3 * i + j] = U[3 * i + 0] * W[j] + U[3 * i + 1] * W[3 + j] + U[3 * i + 2] * W[6 + j];
            R2[3 * i + j] = U[3 * i + 0] * Wt[j] + U[3 * i + 1] * Wt[3 + j] + U[3 * i + 2] * Wt[6 + j];
        }
    for (int i = 0; i < 3; i++) t[i] = U[3 * i + 2];
}

/* ------------------------------------------------------------------------ */
/* All-pairs fp32 match (python/pairwise_pnp.py:635-659) on the             */
/* gemmini_functions_cpu.h:14-56 summation order (k = 0..K-1, mul then add) */
/* ------------------------------------------------------------------------ */
ORC_EXPORT void orc_matmul_nt(int I, int J, int Kd, const float *A, const float *B, float *C) {
    for (int i = 0; i < I; i++)
        for (int j = 0; j < J; j++) {
            float acc = C[(size_t)i * J + j];
            const float *a = A + (size_t)i * Kd, *b = B + (size_t)j * Kd;
            for (int k = 0; k < Kd; k++) acc += a[k] * b[k];
            C[(size_t)i * J + j] = acc;
        }
}

/* First strict maximum over j of the exact score, kept only if > thresh
 * (double compare).  idx = -1 where no j qualifies. */
ORC_EXPORT void orc_allpairs_f32(const float *d0, int n0, const float *d1, int n1, int dim, double thresh,
                                 int *idx, float *score) {
    for (int i = 0; i < n0; i++) {
        const float *a = d0 + (size_t)i * dim;
        int best = -1;
        float bs = 0.0f;
        for (int j = 0; j < n1; j++) {
            const float *b = d1 + (size_t)j * dim;
            float s = 0.0f;
            for (int k = 0; k < dim; k++) s += a[k] * b[k];
            if ((double)s > thresh && s > bs) {
                bs = s;
                best = j;
            }
        }
        idx[i] = best;
        score[i] = best >= 0 ? bs : 0.0f;
    }
}

/* Row-argmax over a precomputed score matrix (the gemmini baseline's epilogue). */
ORC_EXPORT void orc_row_argmax(const float *S, int n0, int n1, double thresh, int *idx, float *score) {
    for (int i = 0; i < n0; i++) {
        int best = -1;
        float bs = 0.0f;
        for (int j = 0; j < n1; j++) {
            float s = S[(size_t)i * n1 + j];
            if ((double)s > thresh && s > bs) {
                bs = s;
                best = j;
            }
        }
        idx[i] = best;
        score[i] = best >= 0 ? bs : 0.0f;
    }
}

/* ------------------------------------------------------------------------ */
/* All-pairs int8 match (exact cosine, as-intended squared_dist semantics)  */
/* ------------------------------------------------------------------------ */
ORC_EXPORT void orc_allpairs_i8(const int8_t *d0, int n0, const int8_t *d1, int n1, int *idx, int *dot_out) {
    int64_t *nb = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n1 > 0 ? n1 : 1));
    for (int j = 0; j < n1; j++) {
        int64_t s = 0;
        for (int k = 0; k < 256; k++) s += d1[(size_t)j * 256 + k] * d1[(size_t)j * 256 + k];
        nb[j] = s;
    }
    for (int i = 0; i < n0; i++) {
        const int8_t *a = d0 + (size_t)i * 256;
        int64_t na = 0;
        for (int k = 0; k < 256; k++) na += a[k] * a[k];
        int best = -1;
        int64_t bd = 0, bn = 1;
        for (int j = 0; j < n1; j++) {
            const int8_t *b = d1 + (size_t)j * 256;
            int64_t dot = 0;
            for (int k = 0; k < 256; k++) dot += a[k] * b[k];
            if (dot <= 0 || na == 0 || nb[j] == 0) continue;
            if ((unsigned __int128)(100 * dot * dot) <= (unsigned __int128)81 * (uint64_t)(na * nb[j])) continue;
            if (best < 0 || (unsigned __int128)(dot * dot) * (uint64_t)bn >
                                (unsigned __int128)(bd * bd) * (uint64_t)nb[j]) {
                best = j;
                bd = dot;
                bn = nb[j];
            }
        }
        idx[i] = best;
        dot_out[i] = best >= 0 ? (int)bd : 0;
    }
    free(nb);
}

/* ---- trajectory chaining: python/compute_trajectory.py:53-90 (the loop body :73-79) ----
 * poses [len + 1][12] float64, row-major [R | t].  mode 0 (as built, :76-77):
 *   R <- transform[:3, :3] @ current_pose[:3, :3];  t <- transform[:3, 3] + current_pose[:3, 3]
 * mode 1 (the commented-out composition that produced outputs/785/trajectory.ply, here the
 * left product T_rel @ current_pose of the 4x4 matrices):  t <- R_rel t + t_rel.
 * numpy's order on these shapes: sum over k = 0, 1, 2 left to right, mul then add (pinned by
 * the committed PLY points, which this reproduces bit for bit).  present[k] == 0: the file was
 * missing (:86-87), the pose carries over. */
ORC_EXPORT void orc_trajectory_chain(int len, const double *rel, const int *present, const double *start, int mode,
                                     double *poses) {
    double cur[12];
    for (int e = 0; e < 12; e++) cur[e] = start ? start[e] : ((e >> 2) == (e & 3) ? 1.0 : 0.0);
    memcpy(poses, cur, sizeof cur);
    for (int k = 0; k < len; k++) {
        const double *T = rel + 12 * (size_t)k;
        double nx[12];
        if (present && !present[k]) {
            memcpy(poses + 12 * (size_t)(k + 1), cur, sizeof cur);
            continue;
        }
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) {
                double s = T[4 * i] * cur[j];
                s = s + T[4 * i + 1] * cur[4 + j];
                s = s + T[4 * i + 2] * cur[8 + j];
                nx[4 * i + j] = s;
            }
            if (mode == 1) {
                double s = T[4 * i] * cur[3];
                s = s + T[4 * i + 1] * cur[7];
                s = s + T[4 * i + 2] * cur[11];
                nx[4 * i + 3] = s + T[4 * i + 3];
            } else {
                nx[4 * i + 3] = T[4 * i + 3] + cur[4 * i + 3];
            }
        }
        memcpy(cur, nx, sizeof cur);
        memcpy(poses + 12 * (size_t)(k + 1), cur, sizeof cur);
    }
}

/* ---- keypoint extraction: SuperPointFrontend.run after the network (python/pairwise_pnp.py:
 * 197-257) and nms_fast (:116-179).  SURVEY §8(f)2.
 * Heatmap (:204-220): dense = exp(semi) (float32; here the correctly rounded exp, numpy's
 * SIMD expf is within ~1 ulp of it), den = sum_c dense[c] sequentially (numpy's axis-0
 * reduction) + float32(1e-5), heat[hc*8 + i][wc*8 + j] = dense[i*8 + j] / den. */
ORC_EXPORT void orc_kp_heatmap(const float *semi, int Hc, int Wc, float *heat) {
    const size_t plane = (size_t)Hc * Wc;
    const int Wh = Wc * 8;
    for (int hc = 0; hc < Hc; hc++)
        for (int wc = 0; wc < Wc; wc++) {
            float e[65], den = 0.f;
            for (int c = 0; c < 65; c++) {
                e[c] = (float)exp((double)semi[c * plane + (size_t)hc * Wc + wc]);
                den = den + e[c];
            }
            den = den + 1e-5f;
            for (int c = 0; c < 64; c++) heat[(size_t)(hc * 8 + c / 8) * Wh + wc * 8 + c % 8] = e[c] / den;
        }
}

typedef struct {
    float conf;
    int idx;  /* np.where order (row-major) */
} orc_cand;
static int cand_desc(const void *a, const void *b) { /* conf descending, then np.where order */
    const orc_cand *x = (const orc_cand *)a, *y = (const orc_cand *)b;
    if (x->conf != y->conf) return x->conf > y->conf ? -1 : 1;
    return x->idx - y->idx;
}
static int cand_desc_rev(const void *a, const void *b) { /* conf descending, ties reversed */
    const orc_cand *x = (const orc_cand *)a, *y = (const orc_cand *)b;
    if (x->conf != y->conf) return x->conf > y->conf ? -1 : 1;
    return y->idx - x->idx;
}

/* threshold (:222, float32 compare), nms_fast (greedy in descending confidence, ties in
 * np.where order, (2d+1)^2 window on an HxW grid), survivors sorted by descending confidence
 * (:229-231: argsort(-conf) then argsort(conf) reversed, so ties come out in REVERSED
 * np.where order -- what numpy's sorts do on these sizes; they do not promise it), border
 * removal (:233-237).  pts [cap][3] = (x, y, conf).  Returns the count, or -1 when more than `cap`
 * candidates pass the threshold (nothing written). */
ORC_EXPORT int orc_kp_select(const float *heat, int Hh, int Wh, int H, int W, float conf_thresh, int nms_dist,
                             int border, int cap, float *pts) {
    int nc = 0;
    for (int i = 0; i < Hh * Wh; i++)
        if (heat[i] >= conf_thresh) nc++;
    if (nc > cap) return -1;
    if (nc == 0) return 0;
    orc_cand *c = (orc_cand *)malloc(sizeof(orc_cand) * (size_t)nc);
    nc = 0;
    for (int i = 0; i < Hh * Wh; i++)
        if (heat[i] >= conf_thresh) {
            c[nc].conf = heat[i];
            c[nc].idx = i;
            nc++;
        }
    qsort(c, (size_t)nc, sizeof(orc_cand), cand_desc);
    const int pad = nms_dist, GW = W + 2 * pad, GH = H + 2 * pad;
    signed char *grid = (signed char *)calloc((size_t)GW * GH, 1);
    for (int k = 0; k < nc; k++) grid[(size_t)(c[k].idx / Wh + pad) * GW + c[k].idx % Wh + pad] = 1;
    int nk = 0;
    for (int k = 0; k < nc; k++) {
        const int y = c[k].idx / Wh + pad, x = c[k].idx % Wh + pad;
        if (grid[(size_t)y * GW + x] != 1) continue;
        for (int yy = y - pad; yy <= y + pad; yy++)
            for (int xx = x - pad; xx <= x + pad; xx++) grid[(size_t)yy * GW + xx] = 0;
        grid[(size_t)y * GW + x] = -1;
        c[nk++] = c[k]; /* kept, in descending order (ties: np.where order) */
    }
    qsort(c, (size_t)nk, sizeof(orc_cand), cand_desc_rev);
    int n = 0;
    for (int k = 0; k < nk; k++) {
        const int y = c[k].idx / Wh, x = c[k].idx % Wh;
        if (x < border || x >= W - border || y < border || y >= H - border) continue;
        pts[3 * n] = (float)x;
        pts[3 * n + 1] = (float)y;
        pts[3 * n + 2] = c[k].conf;
        n++;
    }
    free(grid);
    free(c);
    return n;
}

/* descriptor sampling (:240-254): torch grid_sample (bilinear, zeros padding,
 * align_corners=False) as its CPU kernel evaluates it -- ix = fma(gx + 1, Wc/2, -0.5),
 * weights from the floor distances, corners accumulated by an fma chain -- then L2
 * normalisation over the 256 channels (numpy: sequential sum of squares, sqrt, divide).
 * desc [256][Hc][Wc]; pts [n][3]; out [n][256]. */
ORC_EXPORT void orc_kp_sample(const float *desc, int Hc, int Wc, int H, int W, int n, const float *pts, float *out) {
    const size_t plane = (size_t)Hc * Wc;
    for (int p = 0; p < n; p++) {
        const float gx = (float)((double)pts[3 * p] / ((double)W / 2.) - 1.);
        const float gy = (float)((double)pts[3 * p + 1] / ((double)H / 2.) - 1.);
        const float ix = fmaf(gx + 1.f, (float)Wc / 2.f, -0.5f), iy = fmaf(gy + 1.f, (float)Hc / 2.f, -0.5f);
        const float x0f = floorf(ix), y0f = floorf(iy);
        const float w = ix - x0f, e = 1.f - w, nn = iy - y0f, s = 1.f - nn;
        const float wnw = s * e, wne = s * w, wsw = nn * e, wse = nn * w;
        const int x0 = (int)x0f, y0 = (int)y0f;
        float *o = out + (size_t)p * 256;
        for (int ch = 0; ch < 256; ch++) {
            const float *D = desc + ch * plane;
#define ORC_AT(yy, xx) (((xx) >= 0 && (xx) < Wc && (yy) >= 0 && (yy) < Hc) ? D[(size_t)(yy) * Wc + (xx)] : 0.f)
            float v = ORC_AT(y0, x0) * wnw;
            v = fmaf(ORC_AT(y0, x0 + 1), wne, v);
            v = fmaf(ORC_AT(y0 + 1, x0), wsw, v);
            v = fmaf(ORC_AT(y0 + 1, x0 + 1), wse, v);
#undef ORC_AT
            o[ch] = v;
        }
        float ss = 0.f;
        for (int ch = 0; ch < 256; ch++) {
            const float q = o[ch] * o[ch];
            ss = ss + q;
        }
        const float nrm = sqrtf(ss);
        for (int ch = 0; ch < 256; ch++) o[ch] = o[ch] / nrm;
    }
}

/* ---- nn_match_two_way: python/pairwise_pnp.py:281-323 ----
 * dmat = desc1^T desc2 (here the sequential fp32 dot of orc_allpairs_f32 -- the reference's
 * np.dot is BLAS, whose order differs by ulps), dist = sqrt(2 - 2 clip(dmat, -1, 1)) in
 * float32, idx = argmin over columns (np.argmin: first NaN, else first minimum), kept when
 * dist < (float)nn_thresh and argmin over rows of column idx is the row.  idx [n0] = j or -1,
 * dist [n0] = the kept distance or 0.  Returns the number kept (-1: nn_thresh < 0). */
static float orc_dist(float s) {
    const float c = s != s ? s : (s < -1.f ? -1.f : (s > 1.f ? 1.f : s));
    return sqrtf(2.f - 2.f * c);
}
static int orc_argmin_better(float v, int j, float bv, int bj) {
    const int nv = v != v, nb = bv != bv;
    if (nv || nb) return nv && (!nb || j < bj);
    return v < bv || (v == bv && j < bj);
}
ORC_EXPORT int orc_two_way_f32(const float *d0, int n0, const float *d1, int n1, int dim, double nn_thresh, int *idx,
                               float *dist) {
    if (nn_thresh < 0.0) return -1;
    for (int i = 0; i < n0; i++) {
        idx[i] = -1;
        dist[i] = 0.f;
    }
    if (n0 == 0 || n1 == 0) return 0;
    float *D = (float *)malloc(sizeof(float) * (size_t)n0 * n1);
    for (int i = 0; i < n0; i++)
        for (int j = 0; j < n1; j++) {
            const float *a = d0 + (size_t)i * dim, *b = d1 + (size_t)j * dim;
            float s = 0.0f;
            for (int k = 0; k < dim; k++) s += a[k] * b[k];
            D[(size_t)i * n1 + j] = orc_dist(s);
        }
    int *rev = (int *)malloc(sizeof(int) * (size_t)n1);
    for (int j = 0; j < n1; j++) {
        int bi = -1;
        float bv = INFINITY;
        for (int i = 0; i < n0; i++)
            if (bi < 0 || orc_argmin_better(D[(size_t)i * n1 + j], i, bv, bi)) {
                bv = D[(size_t)i * n1 + j];
                bi = i;
            }
        rev[j] = bi;
    }
    const float th = (float)nn_thresh;
    int kept = 0;
    for (int i = 0; i < n0; i++) {
        int bj = -1;
        float bv = INFINITY;
        for (int j = 0; j < n1; j++)
            if (bj < 0 || orc_argmin_better(D[(size_t)i * n1 + j], j, bv, bj)) {
                bv = D[(size_t)i * n1 + j];
                bj = j;
            }
        if (bv < th && rev[bj] == i) {
            idx[i] = bj;
            dist[i] = bv;
            kept++;
        }
    }
    free(rev);
    free(D);
    return kept;
}

/* ---- cell-level NMS of the int8 path: src/run_nms.c:65-155 (main after compute_softmax) ----
 * For every grid corner (x_grid_i, y_grid_i), x in [0, cols], y in [0, rows] (x outer, :68-69),
 * gather the (at most 4) cells around it whose keypoint lies in the quadrant next to the
 * corner (:75-104: x_delta -1 needs patch_x >= 2, 0 needs patch_x < 6, likewise y), then
 * repeatedly take the most probable (the first loop only over patches > 0, :108-114, then a
 * second pass over patches >= 0 from that maximum, :118-123) and suppress the others within
 * 4 px in x and y (< 4, :131) by setting their max_indices to 64 and probs to 64 (:133-134).
 * max_idx / probs [cells] are modified in place (cell p = gx * rows + gy); kp [cells][2]
 * receives the survivors' pixels in patch order (:147-155).  Returns their count. */
ORC_EXPORT int orc_run_nms(int rows, int cols, int *max_idx, float *probs, float *kp) {
    for (int xi = 0; xi <= cols; xi++)
        for (int yi = 0; yi <= rows; yi++) {
            int n = 0, pat[4], xs[4], ys[4];
            float pr[4];
            for (int xd = -1; xd <= 0; xd++) {
                const int xg = xi + xd;
                if (xg < 0 || xg >= cols) continue;
                for (int yd = -1; yd <= 0; yd++) {
                    const int yg = yi + yd;
                    if (yg < 0 || yg >= rows) continue;
                    const int p = xg * rows + yg, idx = max_idx[p];
                    if (idx == 64) continue;
                    const int px = idx % 8, py = idx / 8;
                    if (xd == -1 && px < 2) continue;
                    if (xd == 0 && px >= 6) continue;
                    if (yd == -1 && py < 2) continue;
                    if (yd == 0 && py >= 6) continue;
                    pat[n] = p;
                    pr[n] = probs[p];
                    xs[n] = xg * 8 + px;
                    ys[n] = yg * 8 + py;
                    n++;
                }
            }
            for (;;) {
                float mp = 0;
                int mi = -1;
                for (int i = 0; i < n; i++)
                    if (pat[i] > 0 && pr[i] > mp) {
                        mp = pr[i];
                        mi = i;
                    }
                if (mi == -1) break;
                for (int i = 0; i < n; i++)
                    if (pat[i] >= 0 && pr[i] > mp) {
                        mp = pr[i];
                        mi = i;
                    }
                for (int i = 0; i < n; i++) {
                    if (i == mi || pat[i] < 0) continue;
                    if (abs(xs[mi] - xs[i]) < 4 && abs(ys[mi] - ys[i]) < 4) {
                        max_idx[pat[i]] = 64;
                        probs[pat[i]] = 64;
                        pat[i] = -1;
                        pr[i] = -1;
                    }
                }
                pr[mi] = -1;
                pat[mi] = -1;
            }
        }
    int nk = 0;
    for (int p = 0; p < rows * cols; p++) {
        const int idx = max_idx[p];
        if (idx == 64) continue;
        kp[2 * nk] = (float)((p / rows) * 8 + idx % 8);
        kp[2 * nk + 1] = (float)((p % rows) * 8 + idx / 8);
        nk++;
    }
    return nk;
}

/* ---- projection factors: src/projection_factor.c:12-33 with src/types.c:3-73 (error), an
 * analytic Jacobian (the reference has none), and the factor's [J|r]^T [J|r] in the
 * local-BA layout of src/local_bundle_adjustment.c:161-169 (columns [landmark 3 | pose 6 |
 * residual 1], matmul2's k order).  pose [7] = (qw, qx, qy, qz, tx, ty, tz); cam [4] =
 * (fx, fy, cx, cy).  J [20] column-major 2 x 10: landmark, rotation (left perturbation
 * omega: p' = p + omega x p), translation, residual; H [100] row-major 10 x 10. ---- */
static void orc_qmul(const float *a, const float *b, float *o) { /* types.c:19-26 order */
    o[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    o[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    o[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    o[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}
ORC_EXPORT void orc_pf_linearize(int F, const float *ldmk, const float *pose, const int *lid, const int *pid,
                                 const float *meas, const float *cam, float *err, float *J, float *H) {
    for (int f = 0; f < F; f++) {
        const float *X = ldmk + 3 * (size_t)lid[f], *T = pose + 7 * (size_t)pid[f], *K = cam + 4 * (size_t)pid[f];
        const float vq[4] = {0.f, X[0], X[1], X[2]}, qc[4] = {T[0], -T[1], -T[2], -T[3]};
        float qv[4], r[4];
        orc_qmul(T, vq, qv);
        orc_qmul(qv, qc, r); /* apply_rotation, types.c:63-68 */
        const float px = r[1] + 1.f * T[4], py = r[2] + 1.f * T[5], pz = r[3] + 1.f * T[6];
        const float ux = px / pz, uy = py / pz; /* project2d, projection_factor.c:12-17 */
        const float ex = (ux * K[0] + K[2]) + -1.f * meas[2 * f], ey = (uy * K[1] + K[3]) + -1.f * meas[2 * f + 1];
        err[2 * f] = ex;
        err[2 * f + 1] = ey;
        /* d e / d p_c */
        const float iz = 1.f / pz;
        const float d00 = K[0] * iz, d02 = -(K[0] * px) * iz * iz, d11 = K[1] * iz, d12 = -(K[1] * py) * iz * iz;
        /* the linear map v -> q v q* (unnormalised q) */
        const float w = T[0], x = T[1], y = T[2], z = T[3];
        const float R[9] = {w * w + x * x - y * y - z * z, 2.f * (x * y - w * z), 2.f * (x * z + w * y),
                            2.f * (x * y + w * z), w * w - x * x + y * y - z * z, 2.f * (y * z - w * x),
                            2.f * (x * z - w * y), 2.f * (y * z + w * x), w * w - x * x - y * y + z * z};
        /* -[p]x */
        const float S[9] = {0.f, pz, -py, -pz, 0.f, px, py, -px, 0.f};
        float *Jf = J + 20 * (size_t)f;
        for (int c = 0; c < 3; c++) {
            Jf[2 * c] = d00 * R[c] + d02 * R[6 + c];
            Jf[2 * c + 1] = d11 * R[3 + c] + d12 * R[6 + c];
            Jf[2 * (3 + c)] = d00 * S[c] + d02 * S[6 + c];
            Jf[2 * (3 + c) + 1] = d11 * S[3 + c] + d12 * S[6 + c];
        }
        Jf[12] = d00;
        Jf[13] = 0.f;
        Jf[14] = 0.f;
        Jf[15] = d11;
        Jf[16] = d02;
        Jf[17] = d12;
        Jf[18] = ex;
        Jf[19] = ey;
        float *Hf = H + 100 * (size_t)f;
        for (int i = 0; i < 10; i++)
            for (int j = 0; j < 10; j++) {
                float s = 0.f;
                s += Jf[2 * i] * Jf[2 * j];
                s += Jf[2 * i + 1] * Jf[2 * j + 1];
                Hf[10 * i + j] = s;
            }
    }
}

/* Normal equations of each pose from its factors (pose-only refinement): the factors of pose
 * p are [off[p], off[p+1]) and are accumulated in that order, as the local-BA scatter adds
 * H_factor into the pose block one factor at a time (local_bundle_adjustment.c:184-200):
 * HPP [P][36] (rows 3..8 x cols 3..8 of H), g [P][6] (rows 3..8, col 9), ee [P] (9, 9). */
ORC_EXPORT void orc_pose_normal_equations(int P, const int *off, const float *H, float *HPP, float *g, float *ee) {
    for (int p = 0; p < P; p++) {
        float a[36] = {0}, b[6] = {0}, c = 0.f;
        for (int f = off[p]; f < off[p + 1]; f++) {
            const float *Hf = H + 100 * (size_t)f;
            for (int i = 0; i < 6; i++) {
                for (int j = 0; j < 6; j++) a[6 * i + j] = Hf[10 * (3 + i) + 3 + j] + a[6 * i + j];
                b[i] = Hf[10 * (3 + i) + 9] + b[i];
            }
            c = Hf[99] + c;
        }
        memcpy(HPP + 36 * (size_t)p, a, sizeof a);
        memcpy(g + 6 * (size_t)p, b, sizeof b);
        ee[p] = c;
    }
}

/* ---- local BA Schur back-end: src/local_bundle_adjustment.c:128-250 (main), with its
 * matrix_add (:35-44), invert_3x3 (:46-75), invert_block_diagonal_matrix (:77-83), the
 * zeroing helpers and matmul2 (gemmini_functions_cpu.h:60-124).  For every chunk of LC
 * landmarks: assemble A (block-diagonal 3x3 landmark blocks), B (pose x landmark, residual
 * row) and C (pose x pose, residual row) from the factors' H = J^T J, invert A's blocks, and
 * C -= B^T-side product (B A^-1) -- the Schur complement of the landmarks, accumulated in C
 * chunk after chunk.  J [L / LC][P * LC][20]: each chunk's factor buffer (2 x 10 column-major,
 * [landmark 3 | pose 6 | residual 1]); factor (landmark chunk_i, pose p) is buffer entry
 * p * chunk_i as built (:158, the reference's index), chunk_i * P + p as intended.
 * C [(6P+1)^2], column-major stride 6P+1, in/out (the reference starts from zeros). ---- */
static void orc_madd(const float *A, float *C, int rows, int cols, int sA, int sC) { /* :35-44, alpha = beta = 1 */
    for (int j = 0; j < cols; j++)
        for (int i = 0; i < rows; i++) C[j * sC + i] = 1.f * A[j * sA + i] + 1.f * C[j * sC + i];
}
static void orc_inv3(float *m, int stride) { /* :46-75 */
    float a[9], v[9];
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) a[j * 3 + i] = m[j * stride + i];
    const float det = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) +
                      a[2] * (a[3] * a[7] - a[4] * a[6]);
    v[0] = (a[4] * a[8] - a[5] * a[7]) / det;
    v[1] = (a[2] * a[7] - a[1] * a[8]) / det;
    v[2] = (a[1] * a[5] - a[2] * a[4]) / det;
    v[3] = (a[5] * a[6] - a[3] * a[8]) / det;
    v[4] = (a[0] * a[8] - a[2] * a[6]) / det;
    v[5] = (a[2] * a[3] - a[0] * a[5]) / det;
    v[6] = (a[3] * a[7] - a[4] * a[6]) / det;
    v[7] = (a[1] * a[6] - a[0] * a[7]) / det;
    v[8] = (a[0] * a[4] - a[1] * a[3]) / det;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) m[j * stride + i] = v[j * 3 + i];
}
/* matmul2 with D == C (C = sD * C first), row-major strides as in gemmini_functions_cpu.h */
static void orc_mm2(int I, int Jn, int K, const float *A, const float *B, float *C, int sA, int sB, int sC, float aS,
                    float bS, float dS, int tA, int tB) {
    const int sAi = tA ? 1 : sA, sAk = tA ? sA : 1, sBk = tB ? 1 : sB, sBj = tB ? sB : 1;
    for (int i = 0; i < I; i++)
        for (int j = 0; j < Jn; j++) C[i * sC + j] = dS * C[i * sC + j];
    for (int i = 0; i < I; i++)
        for (int j = 0; j < Jn; j++)
            for (int k = 0; k < K; k++) C[i * sC + j] += aS * A[i * sAi + k * sAk] * bS * B[k * sBk + j * sBj];
}
ORC_EXPORT void orc_lba_schur(int P, int L, int LC, int as_built, const float *J, float *C) {
    const int S = 6 * P + 1, TL = 3 * LC;
    float *A = (float *)calloc((size_t)TL * TL, sizeof(float));
    float *Bc = (float *)calloc((size_t)S * TL, sizeof(float));
    float *BA = (float *)calloc((size_t)S * TL, sizeof(float));
    float H[100] = {0}; /* (main's H_factor is uninitialised stack memory; +0 here) */
    for (int c0 = 0, ch = 0; c0 < L; c0 += LC, ch++) {
        for (int I = 0; I < TL; I += 3) /* zero_block_diagonal_matrix */
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) A[(I + i) * TL + I + j] = 0;
        memset(Bc, 0, sizeof(float) * (size_t)S * TL);
        const float *Jc = J + (size_t)ch * P * LC * 20;
        for (int ci = 0; ci < LC; ci++)
            for (int p = 0; p < P; p++) {
                const int pi = p * 6, li = ci * 3;
                const float *Jf = Jc + 20 * (size_t)(as_built ? p * ci : ci * P + p);
                orc_mm2(10, 10, 2, Jf, Jf, H, 2, 2, 10, 1.f, 1.f, 0.f, 0, 1);
                orc_madd(H, A + li * (TL + 1), 3, 3, 10, TL);
                orc_madd(H + 3, Bc + pi + li * S, 6, 3, 10, S);
                orc_madd(H + 9, Bc + (li + 1) * S - 1, 1, 3, 10, S);
                orc_madd(H + 33, C + pi * (S + 1), 6, 6, 10, S);
                orc_madd(H + 39, C + (pi + 1) * S - 1, 1, 6, 10, S);
            }
        for (int I = 0; I < TL; I += 3) orc_inv3(A + I * TL + I, TL);
        orc_mm2(TL, 6 * P, TL, A, Bc, BA, TL, S, S, 1.f, 1.f, 0.f, 0, 0);
        orc_mm2(6 * P, 6 * P, TL, Bc, BA, C, S, S, S, -1.f, 1.f, 1.f, 1, 0);
    }
    free(A);
    free(Bc);
    free(BA);
}
