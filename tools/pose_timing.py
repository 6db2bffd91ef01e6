#!/usr/bin/env python3
"""Time k_pose_ransac alone on bench.py's synthetic batch for a grid of (hypotheses,
refine_iters, batch) -- where does the pose time go?  GPU box only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402
import mvtrack  # noqa: E402
import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = 1024
    ctx = mvtrack.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    K = synth.KITTI_K
    for B in [int(x) for x in os.environ.get("POSE_BATCHES", "256").split(",")]:
        d0, d1, kp0, kp1 = bench.gen_batch(torch, dev, B, n, seed=1)
        if os.environ.get("POSE_NOISE"):  # bench.py's noisy_pose keypoints: 0.5 px noise, 20 % outliers
            g = torch.Generator(device=dev)
            g.manual_seed(1234)
            k1 = kp1 + 0.5 * torch.randn(kp1.shape, generator=g, device=dev)
            om = torch.rand((B, n), generator=g, device=dev) < 0.2
            rnd = torch.rand((B, n, 2), generator=g, device=dev) * torch.tensor([synth.KITTI_W, synth.KITTI_H], device=dev)
            kp1 = torch.where(om[:, :, None], rnd, k1).contiguous()
        nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
        idx = torch.empty((B, n), dtype=torch.int32, device=dev)
        score = torch.empty((B, n), dtype=torch.float32, device=dev)
        T = torch.empty((B, 3, 4), dtype=torch.float32, device=dev)
        nm, ni, st = (torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3))
        ctx.reserve(B, n)
        ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, score, 0.8)
        for hyp in [int(x) for x in os.environ.get("POSE_HYPS", "64,128,256,512").split(",")]:
            for it in [int(x) for x in os.environ.get("POSE_ITERS", "0,3,10").split(",")]:
                p = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                                        hypotheses=hyp, inlier_thresh=1.0, refine_iters=it, seed=7)
                for _ in range(2):
                    ctx.pose_from_matches(p, nn_, idx, kp0, kp1, T, nm, ni, st)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    ctx.pose_from_matches(p, nn_, idx, kp0, kp1, T, nm, ni, st)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 10 * 1e3
                print("B=%d hyp=%d iters=%d: %.4f ms  ok=%d" % (B, hyp, it, ms, int((st == 0).sum())), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
