"""As-intended pose under pixel noise: error against the truth per refine_iters / inlier_thresh
(synthetic projections of outputs/transform_*.npy, 30 % outliers)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "maveric-slam_amd")]
import mvtrack  # noqa: E402
import synth  # noqa: E402


def angles(T, Tg):
    """rotation angle of R Rg^T and the angle between the translation directions (degrees), by
    atan2 of sine and cosine (arccos of a float32 trace alone floors at ~0.03 degree)"""
    R, t = T[:, :3].astype(np.float64), T[:, 3].astype(np.float64)
    Rg, tg = Tg[:, :3], Tg[:, 3]
    M = R @ Rg.T
    s = np.linalg.norm([M[2, 1] - M[1, 2], M[0, 2] - M[2, 0], M[1, 0] - M[0, 1]]) / 2
    return (np.degrees(np.arctan2(s, (np.trace(M) - 1) / 2)),
            np.degrees(np.arctan2(np.linalg.norm(np.cross(t, tg)), t @ tg)))


ctx = mvtrack.Context(0)
dev = torch.device("cuda:0")
Ts = np.load(os.path.join(ROOT, "tests/golden/poses.npz"))["transforms_785_790"]
K = synth.KITTI_K
for sigma in (0.0, 0.5, 1.0):
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
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    for thr in (1.0, 2.0):
        for iters in (0, 1, 3, 10, 50):
            prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                                      hypotheses=512, inlier_thresh=thr, refine_iters=iters, seed=9)
            Tt = torch.empty((B, 3, 4), dtype=torch.float32, device=dev)
            ni = torch.empty(B, dtype=torch.int32, device=dev)
            st = torch.empty(B, dtype=torch.int32, device=dev)
            ctx.set_stream(torch.cuda.current_stream())
            ctx.pose_batch(prm, t(np.full(B, n, np.int32)), t(P0), t(P1), Tt, ni, st)
            torch.cuda.synchronize()
            Tn = Tt.cpu().numpy()
            errs = [angles(Tn[b], Ts[b]) for b in range(B)]
            print("sigma %.1f thr %.1f iters %2d: " % (sigma, thr, iters)
                  + " ".join("%.4f/%.3f" % e for e in errs) + "  inl %s" % ni.cpu().numpy().tolist(), flush=True)
