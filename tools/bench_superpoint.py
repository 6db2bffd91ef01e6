#!/usr/bin/env python3
"""The quantized SuperPoint front-end (include/superpoint.h) on KITTI frames:
B grayscale 376 x 1241 frames per launch -> the network at 192 x 640 -> int8 semi / desc +
scales.  Prints one JSON line: frames/s, the int8 MFMA fraction of the network's algorithmic
ops (2 x 10.4 GMAC per frame, counted from the layer shapes), per-stage times (HIP events),
and the oracle's C restatement on host threads beside it.  GPU only."""
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

I8_PEAK_TOPS = 5000.0  # dense int8 MFMA, MI355X_MICROARCH.md


def network_ops(oh, ow):
    """2 x MACs of one frame (every conv, zero-padding taps included as the GPU computes them)"""
    layers = [(1, 64, 3, 1), (64, 64, 3, 1), (64, 64, 3, 2), (64, 64, 3, 2), (64, 128, 3, 4), (128, 128, 3, 4),
              (128, 128, 3, 8), (128, 128, 3, 8), (128, 256, 3, 8), (256, 65, 1, 8), (128, 256, 3, 8), (256, 256, 1, 8)]
    macs = sum(ci * co * k * k * (oh // s) * (ow // s) for ci, co, k, s in layers)
    return 2 * macs


def cpu_baseline(imgs, weights, seconds):
    import concurrent.futures as cf

    import oracle

    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1))
    net = oracle.sp_net(weights)
    deadline = time.perf_counter() + seconds

    def worker(k):
        done = 0
        while time.perf_counter() < deadline:
            oracle.sp_forward(imgs[k % len(imgs)], net)
            done += 1
        return done

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(worker, range(threads)))
    dt = time.perf_counter() - t0
    return {"value": round(total / dt, 2), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": "%d KITTI frames through the oracle's C restatement in %.1f s on %d host threads"
                      % (total, dt, threads)}


def run(batch=512, steps=10, warmup=2, check=1, cpu_seconds=0.0, oh=192, ow=640):
    dev = torch.device("cuda", 0)
    W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
    ims = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_images.npz"))
    base = [ims["img_000000"], ims["img_000001"]]
    rng = np.random.default_rng(0)
    # distinct frames: the two KITTI frames shifted / brightness-jittered
    frames = []
    for b in range(batch):
        im = np.roll(base[b % 2], shift=(b // 2) % 17, axis=1).astype(np.int16) + rng.integers(-3, 4)
        frames.append(np.clip(im, 0, 255).astype(np.uint8))
    x = torch.from_numpy(np.stack(frames)).to(dev)
    ctx = mvtrack.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    sp = mvtrack.SuperPoint(ctx, W)
    out = sp.forward(x, oh, ow)
    for _ in range(warmup):
        sp.forward(x, oh, ow, out=out)
    torch.cuda.synchronize()
    mvtrack.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        sp.forward(x, oh, ow, out=out)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    mvtrack.profile_enable(False)
    stages = {}
    for k in ("k_sp_conv", "k_sp_min_gap"):
        ms, c = mvtrack.profile_query(k)
        if c:
            stages[k] = round(ms / c, 4)
    ms_step = el / steps * 1e3
    net_ms = sum(stages.values())
    ops = network_ops(oh, ow) * batch
    res = {"metric": "superpoint_frames_per_s", "value": round(batch * steps / el, 1), "unit": "frames/s",
           "batch": batch, "steps": steps, "ms_per_step": round(ms_step, 4), "stages_ms": stages,
           "config": {"workload": "quantized SuperPoint, KITTI 376x1241 uint8 frames -> %dx%d net" % (oh, ow)},
           "mfma_roofline": {"bound": "mfma", "achieved": round(ops / (net_ms * 1e-3) / 1e12, 1),
                             "peak": I8_PEAK_TOPS, "unit": "TOP/s",
                             "frac": round(ops / (net_ms * 1e-3) / 1e12 / I8_PEAK_TOPS, 4),
                             "ops_per_frame": network_ops(oh, ow)}}
    if check:
        import oracle

        semi, desc, ss, ds = (t.cpu().numpy() for t in out)
        net = oracle.sp_net(W)
        ok = True
        for b in (0, batch - 1):
            s2, d2, ss2, ds2, _, _ = oracle.sp_forward(frames[b], net, oh, ow)
            ok &= bool((semi[b] == s2).all() and (desc[b] == d2).all() and ss[b] == ss2 and ds[b] == ds2)
        res["oracle_exact"] = ok
    if cpu_seconds > 0:
        res["cpu_baseline"] = cpu_baseline(frames[:4], W, cpu_seconds)
    sp.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=0.0)
    a = ap.parse_args()
    print(json.dumps(run(a.batch, a.steps, a.warmup, a.check, a.cpu_seconds)))


if __name__ == "__main__":
    main()
