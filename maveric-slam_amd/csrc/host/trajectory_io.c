/* trajectory_io.c -- pose I/O and the compute_trajectory driver (python/compute_trajectory.py),
 * host C around the chain kernel (k_trajectory.hip).  See include/trajectory.h. */
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "trajectory.h"

/* Python's repr(float) (shortest round-trip digits; fixed notation for decimal exponents
 * -4..15, else d.ddde+XX; '.0' on integral fixed values) -- what f"{point[0]}" writes for a
 * numpy float64 in write_ply (compute_trajectory.py:38). */
static void py_repr(double x, char *out, size_t cap) {
    if (isnan(x)) {
        snprintf(out, cap, "nan");
        return;
    }
    if (isinf(x)) {
        snprintf(out, cap, x > 0 ? "inf" : "-inf");
        return;
    }
    char e[64];
    for (int p = 0; p <= 16; p++) { /* shortest %.pe that reads back as x */
        snprintf(e, sizeof e, "%.*e", p, x);
        if (strtod(e, NULL) == x) break;
    }
    /* e = [-]d[.ddd]e(+|-)XX */
    const char *s = e;
    int neg = 0;
    if (*s == '-') {
        neg = 1;
        s++;
    }
    char dig[32];
    int nd = 0;
    for (; *s && *s != 'e'; s++)
        if (*s != '.') dig[nd++] = *s;
    while (nd > 1 && dig[nd - 1] == '0') nd--; /* (a minimal p has no trailing zero but 0e+00) */
    dig[nd] = 0;
    const int ex = atoi(s + 1);
    char buf[64];
    size_t o = 0;
    if (neg) buf[o++] = '-';
    if (ex >= -4 && ex < 16) {
        if (ex >= 0) {
            for (int k = 0; k <= ex; k++) buf[o++] = k < nd ? dig[k] : '0';
            buf[o++] = '.';
            if (nd > ex + 1)
                for (int k = ex + 1; k < nd; k++) buf[o++] = dig[k];
            else
                buf[o++] = '0';
        } else {
            buf[o++] = '0';
            buf[o++] = '.';
            for (int k = 0; k < -ex - 1; k++) buf[o++] = '0';
            for (int k = 0; k < nd; k++) buf[o++] = dig[k];
        }
        buf[o] = 0;
    } else {
        buf[o++] = dig[0];
        if (nd > 1) {
            buf[o++] = '.';
            for (int k = 1; k < nd; k++) buf[o++] = dig[k];
        }
        snprintf(buf + o, sizeof buf - o, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    }
    snprintf(out, cap, "%s", buf);
}

int mv_write_pose_txt(const char *path, const double *pose12) {
    if (!path || !pose12) return MV_ERR_INVALID_ARG;
    FILE *f = fopen(path, "w");
    if (!f) return MV_ERR_IO;
    for (int r = 0; r < 3; r++) /* np.savetxt(fmt='%.6f'): ' '-joined, '\n' per row */
        fprintf(f, "%.6f %.6f %.6f %.6f\n", pose12[4 * r], pose12[4 * r + 1], pose12[4 * r + 2], pose12[4 * r + 3]);
    return fclose(f) == 0 ? MV_OK : MV_ERR_IO;
}

int mv_write_trajectory_ply(const char *path, int n, const double *xyz) {
    if (!path || n < 0 || (n > 0 && !xyz)) return MV_ERR_INVALID_ARG;
    FILE *f = fopen(path, "w");
    if (!f) return MV_ERR_IO;
    const int ne = n > 0 ? n - 1 : 0;
    fprintf(f, "ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\nproperty float z\n"
               "property uchar red\nproperty uchar green\nproperty uchar blue\nelement edge %d\n"
               "property int vertex1\nproperty int vertex2\nend_header\n",
            n, ne);
    for (int i = 0; i < n; i++) {
        /* colours: [red] + [blue] * (n - 2) + [black], zipped with the points (n = 1: red) */
        int c0 = 0, c2 = 0;
        if (i == 0)
            c0 = 255;
        else if (i < n - 1)
            c2 = 255;
        char a[40], b[40], c[40];
        py_repr(xyz[3 * i], a, sizeof a);
        py_repr(xyz[3 * i + 1], b, sizeof b);
        py_repr(xyz[3 * i + 2], c, sizeof c);
        fprintf(f, "%s %s %s %d %d %d\n", a, b, c, c0, 0, c2);
    }
    for (int i = 0; i < ne; i++) fprintf(f, "%d %d\n", i, i + 1);
    return fclose(f) == 0 ? MV_OK : MV_ERR_IO;
}

int mv_read_transform_npy(const char *path, double *T12) {
    if (!path || !T12) return MV_ERR_INVALID_ARG;
    FILE *f = fopen(path, "rb");
    if (!f) return MV_ERR_IO;
    unsigned char pre[10];
    int st = MV_ERR_IO;
    if (fread(pre, 1, 8, f) != 8 || memcmp(pre, "\x93NUMPY", 6) != 0) goto done;
    unsigned hl;
    if (pre[6] == 1) {
        unsigned char h[2];
        if (fread(h, 1, 2, f) != 2) goto done;
        hl = h[0] | (h[1] << 8);
    } else {
        unsigned char h[4];
        if (fread(h, 1, 4, f) != 4) goto done;
        hl = h[0] | (h[1] << 8) | ((unsigned)h[2] << 16) | ((unsigned)h[3] << 24);
    }
    if (hl > 65536) goto done;
    {
        char *hd = (char *)malloc(hl + 1);
        if (!hd) goto done;
        const int ok = fread(hd, 1, hl, f) == hl;
        hd[hl] = 0;
        /* {'descr': '<f8', 'fortran_order': False, 'shape': (3, 4), } */
        const int good = ok && strstr(hd, "'descr': '<f8'") && strstr(hd, "'fortran_order': False") &&
                         strstr(hd, "'shape': (3, 4)");
        free(hd);
        if (!good) goto done;
    }
    if (fread(T12, sizeof(double), 12, f) != 12) goto done;
    st = MV_OK;
done:
    fclose(f);
    return st;
}

int mv_compute_trajectory(mv_context *ctx, int start_frame, int end_frame, const char *pose_dir,
                          const char *out_dir, int mode, int *num_poses) {
    if (!ctx || !pose_dir || !out_dir) return MV_ERR_INVALID_ARG;
    const int n = end_frame > start_frame ? end_frame - start_frame : 0;
    double *rel = (double *)calloc((size_t)n * 12 + 12, sizeof(double));
    int *present = (int *)calloc((size_t)n + 1, sizeof(int));
    double *poses = (double *)calloc((size_t)(n + 1) * 12, sizeof(double));
    double *pts = (double *)calloc((size_t)(n + 1) * 3, sizeof(double));
    int st = MV_ERR_OUT_OF_MEMORY, np_ = 0;
    char path[4096];
    if (!rel || !present || !poses || !pts) goto done;
    for (int k = 0; k < n; k++) { /* compute_trajectory.py:66-70: a missing file is skipped */
        const int i = start_frame + k;
        snprintf(path, sizeof path, "%s/transform_%06d_%06d.npy", pose_dir, i, i + 1);
        present[k] = mv_read_transform_npy(path, rel + 12 * (size_t)k) == MV_OK;
    }
    st = mv_trajectory_chain_host(ctx, n, rel, present, NULL, mode, poses);
    if (st != MV_OK) goto done;
    snprintf(path, sizeof path, "%s/frame-%06d.pose.txt", out_dir, start_frame);
    if ((st = mv_write_pose_txt(path, poses)) != MV_OK) goto done;
    for (int c = 0; c < 3; c++) pts[c] = poses[4 * c + 3];
    np_ = 1;
    for (int k = 0; k < n; k++) {
        if (!present[k]) continue;
        const double *P = poses + 12 * (size_t)(k + 1);
        snprintf(path, sizeof path, "%s/frame-%06d.pose.txt", out_dir, start_frame + k + 1);
        if ((st = mv_write_pose_txt(path, P)) != MV_OK) goto done;
        for (int c = 0; c < 3; c++) pts[3 * np_ + c] = P[4 * c + 3];
        np_++;
    }
    snprintf(path, sizeof path, "%s/trajectory_%06d_%06d.ply", out_dir, start_frame, end_frame);
    st = mv_write_trajectory_ply(path, np_, pts);
done:
    if (num_poses) *num_poses = st == MV_OK ? np_ : 0;
    free(rel);
    free(present);
    free(poses);
    free(pts);
    return st;
}
