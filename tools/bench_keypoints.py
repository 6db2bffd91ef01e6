#!/usr/bin/env python3
"""Keypoint extraction + descriptor sampling (SuperPointFrontend.run after the
network, python/pairwise_pnp.py:197-257) on KITTI-size network outputs: Hc x Wc = 47 x 155
cells (376 x 1241 image), B frames per launch, cap 1024 keypoints per frame (the fp32 match
config).  Prints one JSON line: frames/s, per-kernel averages (HIP events), the HBM fraction
of the heatmap kernel against its algorithmic bytes, and the oracle's C restatement timed on
host threads beside it.  GPU only."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mvtrack  # noqa: E402
import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0


def cpu_baseline(frames, H, W, seconds):
    import concurrent.futures as cf

    import oracle

    threads = max(1, min(16, os.cpu_count() or 1))
    deadline = time.perf_counter() + seconds

    def worker(k):
        s, d = frames[k % len(frames)]
        done = 0
        while time.perf_counter() < deadline:
            oracle.keypoints(s, d, H, W)
            done += 1
        return done

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(worker, range(threads)))
    dt = time.perf_counter() - t0
    return {"value": round(total / dt, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": "%d KITTI-size frames through the oracle's C restatement in %.1f s on %d host threads"
                      % (total, dt, threads)}


def run(batch=1024, steps=10, warmup=2, distinct=8, check=1, cpu_seconds=0.0, cap=1024):
    dev = torch.device("cuda", 0)
    Hc, Wc, H, W = 47, 155, 376, 1241
    frames = [synth.synth_superpoint_outputs(100 + k, Hc, Wc) for k in range(distinct)]
    semi = torch.from_numpy(np.stack([frames[b % distinct][0] for b in range(batch)])).to(dev)
    cd = torch.from_numpy(np.stack([frames[b % distinct][1] for b in range(batch)])).to(dev)
    n = torch.zeros(batch, dtype=torch.int32, device=dev)
    kp = torch.zeros((batch, cap, 2), dtype=torch.float32, device=dev)
    conf = torch.zeros((batch, cap), dtype=torch.float32, device=dev)
    desc = torch.zeros((batch, cap, 256), dtype=torch.float32, device=dev)
    st = torch.zeros(batch, dtype=torch.int32, device=dev)
    ctx = mvtrack.Context(0)
    ctx.set_stream(torch.cuda.current_stream())

    def step():
        ctx.keypoints(semi, cd, H, W, n, kp, conf, desc, st)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    mvtrack.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    mvtrack.profile_enable(False)
    stages = {}
    for k in ("k_kp_heat", "k_kp_nms", "k_kp_sample_planes", "k_kp_normalize", "k_kp_nhwc", "k_kp_sample"):
        ms, c = mvtrack.profile_query(k)
        if c:  # the planes path (frames up to 9216 cells) or the transpose path
            stages[k] = round(ms / c, 4)
    checked = 0
    if check:
        import oracle

        for b in range(min(check, batch)):
            s_, d_ = frames[b % distinct]
            pts, d, _ = oracle.keypoints(s_, d_, H, W)
            k = int(n[b])
            assert k == min(cap, pts.shape[0])
            assert (kp[b, :k].cpu().numpy() == pts[:k, :2]).all()
            assert (desc[b, :k].cpu().numpy().view(np.int32) == d[:k].view(np.int32)).all()
            checked += 1
    cells = Hc * Wc
    heat_bytes = cells * (65 * 4 + 64 * 4)  # logits in, heatmap out (per frame)
    step_s = el / steps
    out = {
        "metric": "keypoint extraction frames/sec (heatmap + NMS + grid_sample), KITTI 376x1241, cap %d" % cap,
        "value": round(batch / step_s, 1), "unit": "frames/s", "batch": batch, "steps": steps,
        "ms_per_step": round(step_s * 1e3, 4), "stages_ms": stages,
        "keypoints_avg": float(n.float().mean()),
        "hbm_roofline": {"kernel": "k_kp_heat", "bytes_per_frame": heat_bytes,
                         "GBs": round(heat_bytes * batch / (stages["k_kp_heat"] * 1e-3) / 1e9, 1),
                         "frac": round(heat_bytes * batch / (stages["k_kp_heat"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "peak_GBs": HBM_PEAK_GBS},
        "checked_frames": checked,
    }
    if cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(frames, H, W, cpu_seconds)
    ctx.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024,
                    help="frames per launch (256 / 512 / 1024 measured 227 k / 241 k / 247 k frames/s)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    a = ap.parse_args()
    print(json.dumps(run(a.batch, a.steps, a.warmup, check=a.check, cpu_seconds=a.cpu_seconds)), flush=True)


if __name__ == "__main__":
    main()
