"""BASELINE configs[2] end to end on the reference's own KITTI fixtures: the fp32 keypoints and
descriptors of KITTI 00 pairs 0 -> 1 and 10 -> 11 (include/data/tracking/pair0.h, pair10.h:
395 / 401 and 440 / 437 keypoints at 192 x 640) through the all-pairs match (oracle-exact) and
then the pose from those matched keypoints (the path of python/pairwise_pnp.py:635-694), against
the KITTI ground truth relative pose (outputs/00.txt frames 0, 1, 10, 11).

Tolerances (stated, loose by construction -- SURVEY F4):
- with the reference's own K (pairwise_pnp.py:667-669: the full-resolution KITTI K applied to
  the 192 x 640 keypoints, as the reference does) the principal point sits ~290 px right of and
  ~90 px below the resized image's centre, so the recovered translation direction is biased by
  ~20-25 degrees (the survey measured t . t_GT ~ 0.91 for the reference's own transform_*.npy);
  required: rotation within 1 degree of the ground truth, translation direction within 30.
- with K rescaled to the 192 x 640 image (fx, cx by 640/1241, fy, cy by 192/376): rotation within
  0.5 degree, translation direction within 8 (keypoints quantised to whole pixels of the
  resized image, real matches with their outliers).

Plus the as-intended pose under pixel noise: sigma 0.5 and 1 px on synthetic projections of
every reference transform (outputs/transform_*.npy) with 30 % outliers, stated tolerances."""
import numpy as np
import pytest

import synth
from conftest import load_golden

pytestmark = pytest.mark.gpu


def rel_gt(a, b):
    g = load_golden("poses.npz")
    frames = list(g["kitti00_frames"])
    gt = g["kitti00_gt"]
    Ta, Tb = np.eye(4), np.eye(4)
    Ta[:3] = gt[frames.index(a)]
    Tb[:3] = gt[frames.index(b)]
    return (np.linalg.inv(Tb) @ Ta)[:3]  # camera a coordinates -> camera b coordinates


def angles(T, Tg):
    """rotation angle of R Rg^T and the angle between the translation directions (degrees), by
    atan2 of sine and cosine (arccos of a float32 trace alone floors at ~0.03 degree)"""
    R, t = T[:, :3].astype(np.float64), T[:, 3].astype(np.float64)
    Rg, tg = Tg[:, :3], Tg[:, 3]
    M = R @ Rg.T
    s = np.linalg.norm([M[2, 1] - M[1, 2], M[0, 2] - M[2, 0], M[1, 0] - M[0, 1]]) / 2
    return (np.degrees(np.arctan2(s, (np.trace(M) - 1) / 2)),
            np.degrees(np.arctan2(np.linalg.norm(np.cross(t, tg)), t @ tg)))


def _run_pair(ctx, torch, orc, name, K):
    import mvtrack

    d = load_golden(name)
    dev = torch.device("cuda:0")
    cap = 512
    n0, n1 = d["image0_desc"].shape[0], d["image1_desc"].shape[0]
    D0 = np.zeros((1, cap, 256), np.float32)
    D1 = np.zeros((1, cap, 256), np.float32)
    D0[0, :n0], D1[0, :n1] = d["image0_desc"], d["image1_desc"]
    K0 = np.zeros((1, cap, 2), np.float32)
    K1 = np.zeros((1, cap, 2), np.float32)
    K0[0, :n0] = np.stack([d["image0_xs"], d["image0_ys"]], 1)
    K1[0, :n1] = np.stack([d["image1_xs"], d["image1_ys"]], 1)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    N0, N1 = t(np.array([n0], np.int32)), t(np.array([n1], np.int32))
    idx = torch.empty((1, cap), dtype=torch.int32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        ctx.match_allpairs_f32(t(D0), t(D1), N0, N1, idx, None, 0.8)
        prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                                  hypotheses=512, inlier_thresh=1.0, refine_iters=10, seed=5)
        T = torch.empty((1, 3, 4), dtype=torch.float32, device=dev)
        nm = torch.empty(1, dtype=torch.int32, device=dev)
        ni = torch.empty(1, dtype=torch.int32, device=dev)
        st = torch.empty(1, dtype=torch.int32, device=dev)
        ctx.pose_from_matches(prm, N0, idx, t(K0), t(K1), T, nm, ni, st)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    i2, _ = orc.allpairs_f32(d["image0_desc"], d["image1_desc"], 0.8)
    assert (idx[0, :n0].cpu().numpy() == i2).all()  # the match feeding the pose is the reference's
    return T[0].cpu().numpy(), int(nm[0]), int(ni[0]), int(st[0])


K_REF = synth.KITTI_K  # pairwise_pnp.py:667-669
K_192 = K_REF * np.array([[640 / 1241], [192 / 376], [1.0]])  # rows 0 and 1 rescaled to the resized image


@pytest.mark.parametrize("name,fa,fb", [("tracking_pair0.npz", 0, 1), ("tracking_pair10.npz", 10, 11)])
@pytest.mark.parametrize("kname,K,tol_r,tol_t", [("reference_K", K_REF, 1.0, 30.0), ("rescaled_K", K_192, 0.5, 8.0)])
def test_kitti_match_then_pose(ctx, orc, torch_cuda, name, fa, fb, kname, K, tol_r, tol_t):
    T, nm, ni, st = _run_pair(ctx, torch_cuda, orc, name, K)
    er, et = angles(T, rel_gt(fa, fb))
    print("%s %s: %d matches, %d inliers, rotation %.3f deg, translation direction %.2f deg"
          % (name, kname, nm, ni, er, et))
    assert st == 0 and nm >= 250 and ni >= 0.5 * nm
    assert er < tol_r and et < tol_t, (er, et)


@pytest.mark.parametrize("sigma,tol_r,tol_t", [(0.5, 0.15, 3.0), (1.0, 0.25, 6.0)])
def test_pose_pixel_noise_and_outliers(ctx, torch_cuda, sigma, tol_r, tol_t):
    """Synthetic projections of each reference transform (outputs/transform_000785_*.npy) with
    Gaussian pixel noise sigma in both views and 30 % outliers (400 correspondences): the
    as-intended pose within tol_r degrees (rotation) and tol_t degrees (translation direction).
    For scale: the Sampson least-squares fit started from the TRUE pose on the true inliers
    (scipy, float64) lands 0.01-0.04 deg / 0.1-0.7 deg from the truth on these instances; the
    RANSAC starts (8-point minimal samples under this noise) are 2-12 deg off in translation
    direction, and the two refined starts close most, not all, of that gap (measured 0.02-0.17
    deg / 0.1-5 deg at sigma 1)."""
    import mvtrack

    torch = torch_cuda
    Ts = load_golden("poses.npz")["transforms_785_790"]
    B, n = len(Ts), 400
    rng = np.random.default_rng(int(sigma * 10))
    P0 = np.zeros((B, n, 2), np.float32)
    P1 = np.zeros((B, n, 2), np.float32)
    for b, T in enumerate(Ts):
        _, x0, x1 = synth.synth_scene(rng, n, T[:, :3], T[:, 3])
        x0 = x0 + rng.normal(0, sigma, x0.shape)
        x1 = x1 + rng.normal(0, sigma, x1.shape)
        out = rng.random(n) < 0.3
        x1[out] = np.stack([rng.uniform(0, 1241, out.sum()), rng.uniform(0, 376, out.sum())], 1)
        P0[b], P1[b] = x0, x1
    K = synth.KITTI_K
    dev = torch.device("cuda:0")
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                              hypotheses=512, inlier_thresh=max(1.0, 2 * sigma), refine_iters=20, seed=9)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    Tt = torch.empty((B, 3, 4), dtype=torch.float32, device=dev)
    ni = torch.empty(B, dtype=torch.int32, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        ctx.pose_batch(prm, t(np.full(B, n, np.int32)), t(P0), t(P1), Tt, ni, st)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    Tn, st = Tt.cpu().numpy(), st.cpu().numpy()
    for b, Tg in enumerate(Ts):
        er, et = angles(Tn[b], Tg)
        print("sigma %.1f pair %d: rotation %.4f deg, translation direction %.3f deg" % (sigma, b, er, et))
        assert st[b] == 0 and er < tol_r and et < tol_t, (b, er, et)
