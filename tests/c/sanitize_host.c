/* sanitize_host.c -- TEST DRIVER: the host C of maveric-slam_amd/csrc/host/ built with gcc
 * -fsanitize=address,undefined (tests/test_sanitize.py), linked with tests/c/no_device_stubs.c in
 * place of the HIP library.  Exercises the code that does real work on the host -- the local
 * feature pool (feature_pool.c: probing, chain-replacement deletion, pruning), the pose / .ply /
 * .npy file I/O and mv_compute_trajectory's file handling (trajectory_io.c), the drop-in's host
 * arithmetic (normalize_points, compute_reprojection_error in pnp_solver.c) -- and every drop-in
 * entry point's no-device error path (top_N.c, pnp_solver.c, tracking.c).  Exit status 0 = every
 * check held; a sanitizer report aborts the run (-fno-sanitize-recover).
 * usage: sanitize_host <scratch directory> */
#include <stdint.h>
#include <stdio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include "feature_pool.h"
#include "frame.h"
#include "maveric_hip.h"
#include "pnp_solver.h"
#include "top_N.h"
#include "tracking.h"
#include "trajectory.h"

static int g_fail = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c); \
            g_fail = 1;                                                \
        }                                                              \
    } while (0)

static unsigned g_rng = 12345u;
static unsigned rnd(void) {  /* xorshift32: the driver's own stream, independent of rand() */
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 17;
    g_rng ^= g_rng << 5;
    return g_rng;
}

static mv_local_feature_pool g_pool;  /* 3000 slots: static, not on the stack */

static void feature_pool_workloads(void) {
    /* (1) the reference's kind of workload: frames of 200 distinct ids (the invariant's strictly
     *     increasing frames need each id once per frame); then ids repeated within frames, and
     *     frames tracked on after an error (the reference exits there; the library must stay
     *     memory-safe) */
    mv_local_feature_pool_init(&g_pool);
    int ids[400];
    int errors = 0;
    for (int frame = 0; frame < 120; frame++) {
        for (int i = 0; i < 200; i++) ids[i] = (int)(30u * (unsigned)i + rnd() % 30u);
        const int st = mv_local_feature_pool_track_frame(&g_pool, frame, 200, ids);
        CHECK(st == MV_OK || st == MV_ERR_CAPACITY || st == MV_ERR_INVALID_ARG);
        if (st == MV_OK && !errors) CHECK(mv_local_feature_pool_check_invariant(&g_pool, frame) == MV_OK);
        errors += st != MV_OK;
    }
    mv_local_feature_pool_init(&g_pool);
    for (int frame = 0; frame < 120; frame++) {
        for (int i = 0; i < 200; i++) ids[i] = (int)(rnd() % 6000u);
        const int st = mv_local_feature_pool_track_frame(&g_pool, frame, 200, ids);
        CHECK(st == MV_OK || st == MV_ERR_CAPACITY || st == MV_ERR_INVALID_ARG);
    }
    /* (2) ids crowded onto homes around the table end (wrap-around probing and deletion) */
    mv_local_feature_pool_init(&g_pool);
    for (int frame = 0; frame < 60; frame++) {
        for (int i = 0; i < 64; i++) ids[i] = (int)(3000u * (rnd() % 40u) + 2990u + rnd() % 20u);
        (void)mv_local_feature_pool_track_frame(&g_pool, frame, 64, ids);
    }
    /* (3) the table API directly: inserts up to full, duplicate inserts, deletes of present and
     *     absent keys, pruning, key listing into an exactly sized buffer */
    mv_local_feature_pool_init(&g_pool);
    mv_local_feature v;
    mv_local_feature_init(&v);
    int full = 0;
    for (int k = 0; k < MV_LOCAL_FEATURE_POOL_CAPACITY + 10; k++) {
        mv_local_feature *slot = NULL;
        bool ins = false;
        mv_local_feature_init_with_id(&v, k * 7, k % 50);
        const int st = mv_local_feature_pool_insert(&g_pool, k * 7, &v, &slot, &ins);
        if (st != MV_OK) {
            full++;
            continue;
        }
        if (slot) mv_local_feature_update(slot, k % 50 + 1);
    }
    CHECK(full >= 10);
    CHECK(mv_local_feature_pool_load_factor(&g_pool) <= 1.0f);
    for (int k = 0; k < 2000; k++) (void)mv_local_feature_pool_delete(&g_pool, (int)(rnd() % 30000u));
    CHECK(mv_local_feature_pool_delete(&g_pool, -5) != MV_OK);
    (void)mv_local_feature_pool_remove_old(&g_pool, 60);
    static int keys[MV_LOCAL_FEATURE_POOL_CAPACITY];
    int nk = 0;
    mv_local_feature_pool_valid_keys(&g_pool, &nk, keys);
    CHECK(nk >= 0 && nk <= MV_LOCAL_FEATURE_POOL_CAPACITY && nk == g_pool.size);
    mv_local_feature f;
    mv_local_feature_init_with_id(&f, 3, 0);
    for (int fr = 1; fr < 3 * MV_MAX_LOCAL_FRAMES; fr++) mv_local_feature_update(&f, fr);
    (void)mv_local_feature_remove_old_frame(&f, 2 * MV_MAX_LOCAL_FRAMES);
}

static void write_npy(const char *path, const char *descr, const char *shape, const double *T, int n, int cut) {
    FILE *f = fopen(path, "wb");
    if (!f) return;
    char hd[128];
    int hl = snprintf(hd, sizeof hd, "{'descr': '%s', 'fortran_order': False, 'shape': %s, }", descr, shape);
    while ((10 + hl + 1) % 64) hd[hl++] = ' ';
    hd[hl++] = '\n';
    const unsigned char pre[10] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0, (unsigned char)(hl & 255),
                                   (unsigned char)(hl >> 8)};
    fwrite(pre, 1, 10, f);
    fwrite(hd, 1, (size_t)hl, f);
    fwrite(T, sizeof(double), (size_t)n, f);
    fclose(f);
    if (cut) {  /* a truncated copy */
        f = fopen(path, "r+b");
        if (f) {
            fseek(f, 0, SEEK_END);
            const long len = ftell(f);
            fclose(f);
            (void)!truncate(path, len - cut);
        }
    }
}

static void trajectory_io(const char *dir) {
    char p[512];
    double T[12], R[12];
    for (int i = 0; i < 12; i++) T[i] = (i % 5 == 0) ? 1.0 : 1e-3 * (i + 1) * ((i & 1) ? -1 : 1);
    T[3] = 1.0 / 3.0;
    T[7] = -123456.789e-9;
    T[11] = 7e300;
    snprintf(p, sizeof p, "%s/pose.txt", dir);
    CHECK(mv_write_pose_txt(p, T) == MV_OK);
    double xyz[3 * 40];
    for (int i = 0; i < 120; i++) xyz[i] = (double)(int)(rnd() % 2000u) / 7.0 - 100.0;
    snprintf(p, sizeof p, "%s/traj.ply", dir);
    CHECK(mv_write_trajectory_ply(p, 40, xyz) == MV_OK);
    CHECK(mv_write_trajectory_ply(p, 1, xyz) == MV_OK);
    snprintf(p, sizeof p, "%s/nodir/x.txt", dir);
    CHECK(mv_write_pose_txt(p, T) != MV_OK);
    /* .npy: good, wrong dtype, wrong shape, truncated data, missing */
    snprintf(p, sizeof p, "%s/good.npy", dir);
    write_npy(p, "<f8", "(3, 4)", T, 12, 0);
    CHECK(mv_read_transform_npy(p, R) == MV_OK && memcmp(R, T, sizeof T) == 0);
    snprintf(p, sizeof p, "%s/f4.npy", dir);
    write_npy(p, "<f4", "(3, 4)", T, 6, 0);
    CHECK(mv_read_transform_npy(p, R) != MV_OK);
    snprintf(p, sizeof p, "%s/shape.npy", dir);
    write_npy(p, "<f8", "(4, 4)", T, 12, 0);
    CHECK(mv_read_transform_npy(p, R) != MV_OK);
    snprintf(p, sizeof p, "%s/cut.npy", dir);
    write_npy(p, "<f8", "(3, 4)", T, 12, 13);
    CHECK(mv_read_transform_npy(p, R) != MV_OK);
    snprintf(p, sizeof p, "%s/none.npy", dir);
    CHECK(mv_read_transform_npy(p, R) != MV_OK);
    CHECK(mv_read_transform_npy(NULL, R) != MV_OK);
    /* mv_compute_trajectory: reads the transforms it finds, then the chain needs the device */
    for (int fr = 785; fr < 789; fr++) {
        snprintf(p, sizeof p, "%s/transform_%06d_%06d.npy", dir, fr, fr + 1);
        if (fr != 787) write_npy(p, "<f8", "(3, 4)", T, 12, 0);
    }
    int np_ = -1;
    CHECK(mv_compute_trajectory(NULL, 785, 789, dir, dir, MV_CHAIN_AS_BUILT, &np_) != MV_OK);
}

static int8_t g_semi[2400][65], g_desc[2400][256];

static void dropin_no_device(void) {
    for (int c = 0; c < 2400; c++) {
        for (int k = 0; k < 65; k++) g_semi[c][k] = (int8_t)(rnd() & 255u);
        for (int k = 0; k < 256; k++) g_desc[c][k] = (int8_t)(rnd() & 255u);
    }
    int nv = -7, mi[2400];
    float pr[2400];
    compute_softmax(0.05f, g_semi, &nv, mi, pr);
    int ns = -7, pa[100], ix[100];
    float pp[100];
    compute_top_N(0.05f, g_semi, 100, &ns, pa, ix, pp);
    CHECK(ns == -1);  /* no device: the status path, never exit() */
    /* host arithmetic of the drop-in */
    const float K[3][3] = {{718.856f, 0.f, 607.1928f}, {0.f, 718.856f, 185.2157f}, {0.f, 0.f, 1.f}};
    float pts1[64][2], pts2[64][2], n1[64][2];
    for (int i = 0; i < 64; i++) {
        pts1[i][0] = (float)(rnd() % 1241u);
        pts1[i][1] = (float)(rnd() % 376u);
        pts2[i][0] = pts1[i][0] + 0.5f;
        pts2[i][1] = pts1[i][1] - 0.25f;
    }
    normalize_points(64, (const float(*)[2])pts1, K, n1);
    float E[3][3] = {{0.f, -1.f, 0.f}, {1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    const float err = compute_reprojection_error(pts1[0], pts2[0], (const float(*)[3])E);
    CHECK(err == err);
    int inl[64], ni = -7;
    ransac_essential_matrix(64, (const float(*)[2])pts1, (const float(*)[2])pts2, K, 10, 1.1f, E, inl, &ni);
    ransac_essential_matrix(0, (const float(*)[2])pts1, (const float(*)[2])pts2, K, 10, 1.1f, E, inl, &ni);
    float R1[3][3], R2[3][3], t[3];
    recover_pose_from_essential_matrix(E, R1, R2, t);
    Frame f0, f1;
    frame_create(192, 640, 1, NULL, 24, 80, 0.05f, &g_semi[0][0], 0.01f, &g_desc[0][0], &f0);
    frame_create(192, 640, 1, NULL, 24, 80, 0.05f, &g_semi[0][0], 0.01f, &g_desc[0][0], &f1);
    Transform T;
    CHECK(track(&f0, &f1, 4, 4, 9, 0.9f, &T) == MV_ERR_NO_DEVICE);
    CHECK(T.m[0][0] == 1.0f && T.m[1][2] == 0.0f);  /* identity on failure */
    CHECK(track(NULL, &f1, 4, 4, 9, 0.9f, &T) == MV_OK);
    CHECK(track(&f0, &f1, 4, 4, 9, 0.9f, NULL) != MV_OK);
    f1.feature_rows = 23;
    CHECK(track(&f0, &f1, 4, 4, 9, 0.9f, &T) != MV_OK);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <scratch directory>\n", argv[0]);
        return 2;
    }
    feature_pool_workloads();
    trajectory_io(argv[1]);
    dropin_no_device();
    if (g_fail) return 1;
    printf("sanitize_host ok\n");
    return 0;
}
