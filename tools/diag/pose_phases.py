#!/usr/bin/env python3
"""Diagnosis (GPU; MV_LIB = a build of k_pose_intended.hip with per-phase s_memtime stamps, thread 0 of
each block -- tools/diag/r06aa_pose_phases.sh): median cycles per phase of k_pose_ransac on bench.py's
headline batch (exact projections + outliers), noisy keypoints with POSE_NOISE=1."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402
import mvtrack  # noqa: E402
import synth  # noqa: E402

dev = torch.device("cuda", 0)
n, B = 1024, 2048
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
K = synth.KITTI_K
d0, d1, kp0, kp1 = bench.gen_batch(torch, dev, B, n, seed=1)
if os.environ.get("POSE_NOISE"):
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    k1 = kp1 + 0.5 * torch.randn(kp1.shape, generator=g, device=dev)
    om = torch.rand((B, n), generator=g, device=dev) < 0.2
    rnd = torch.rand((B, n, 2), generator=g, device=dev) * torch.tensor([synth.KITTI_W, synth.KITTI_H], device=dev)
    kp1 = torch.where(om[:, :, None], rnd, k1).contiguous()
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
T = torch.empty((B, 3, 4), dtype=torch.float32, device=dev)
nm, ni, st = (torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3))
ctx.reserve(B, n)
ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None, 0.8)
p = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2], hypotheses=256,
                        inlier_thresh=1.0, refine_iters=10, seed=7)
for _ in range(3):
    ctx.pose_from_matches(p, nn_, idx, kp0, kp1, T, nm, ni, st)
torch.cuda.synchronize()
L = ctypes.CDLL(mvtrack.LIB_PATH)
buf = np.zeros((B, 10), np.uint64)
assert L.mv_dbg_pose_stamps(buf.ctypes.data_as(ctypes.c_void_p), B) == 0
d = np.diff(buf[:, :8].astype(np.int64), axis=1)
names = ["compact", "hyp+score", "survivors", "starts", "decomp+cheir", "gauss-newton", "final cost"]
tot = buf[:, 7].astype(np.int64) - buf[:, 0].astype(np.int64)
print("matches/pair %.0f, inliers/pair %.0f" % (float(nm.float().mean()), float(ni.float().mean())))
print("phase cycles per block (median / p90), thread 0's s_memtime:")
for k, nmn in enumerate(names):
    print("  %-14s %8.0f %8.0f" % (nmn, np.median(d[:, k]), np.percentile(d[:, k], 90)))
print("  %-14s %8.0f %8.0f" % ("total", np.median(tot), np.percentile(tot, 90)))
ctx.close()
