#!/usr/bin/env python3
"""int8 all-pairs match: 2048 kp x 256-D int8 per frame, drawn as
round(clip(N(0, 24))) like quantized_image0.h, exact cosine semantics (k_i8_*).  Prints one
JSON line: pairs/s, per-kernel averages (HIP events), and the int8 MFMA fraction of the
screen kernel against the dense int8 peak.  GPU only."""
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

I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: v_mfma_i32_32x32x32_i8 = 2x the BF16 rate (~5 POPS dense)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192,
                    help="pairs per launch (256 / 1024 / 2048 measured 0.67 / 0.76 / 0.80 M pairs/s)")
    ap.add_argument("--kp", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    print(json.dumps(run(args.batch, args.kp, args.steps, args.warmup, args.check, args.cpu_seconds)), flush=True)


def run(batch=8192, kp=2048, steps=20, warmup=3, check=1, cpu_seconds=0.0):
    args = argparse.Namespace(batch=batch, kp=kp, steps=steps, warmup=warmup, check=check, cpu_seconds=cpu_seconds)
    B, n, D = args.batch, args.kp, 256
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    d0 = torch.clamp(torch.round(torch.randn((B, n, D), generator=g, device=dev) * 24), -128, 127).to(torch.int8)
    noise = torch.round(torch.randn((B, n, D), generator=g, device=dev) * 6)
    perm = torch.argsort(torch.rand((B, n), generator=g, device=dev), dim=1)
    d1 = torch.gather(d0.float(), 1, perm[:, :, None].expand(B, n, D)) + noise
    fresh = torch.rand((B, n, 1), generator=g, device=dev) < 0.4
    d1 = torch.where(fresh, torch.round(torch.randn((B, n, D), generator=g, device=dev) * 24), d1)
    d1 = torch.clamp(d1, -128, 127).to(torch.int8).contiguous()
    nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
    idx = torch.empty((B, n), dtype=torch.int32, device=dev)
    dot = torch.empty((B, n), dtype=torch.int32, device=dev)
    ctx = mvtrack.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.reserve(B, n)
    for _ in range(args.warmup):
        ctx.match_allpairs_i8(d0, d1, nn_, nn_, idx, dot)
    torch.cuda.synchronize()
    mvtrack.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.match_allpairs_i8(d0, d1, nn_, nn_, idx, dot)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    mvtrack.profile_enable(False)
    stages = {}
    for k in ("k_i8_norms", "k_i8_prep", "k_i8_match", "k_i8t_match"):
        ms, c = mvtrack.profile_query(k)
        if c:
            stages[k] = round(ms / c, 4)
    checked = 0
    if args.check:
        import oracle

        for b in range(min(args.check, B)):
            i2, _ = oracle.allpairs_i8(d0[b].cpu().numpy(), d1[b].cpu().numpy())
            assert (idx[b].cpu().numpy() == i2).all(), "int8 match differs from the oracle"
            checked += 1
    ops = 2.0 * n * n * D * B
    km = "k_i8t_match" if "k_i8t_match" in stages else "k_i8_match"  # the transposed kernel (default)
    scr = stages[km] * 1e-3
    out = {"metric": "int8 all-pairs frame-pairs/sec (%d kp x 256-D, exact cosine)" % n,
           "value": round(B / (el / args.steps), 1), "unit": "pairs/s", "batch": B,
           "ms_per_step": round(el / args.steps * 1e3, 4), "stages_ms": stages,
           "matches_avg": float((idx >= 0).float().sum(1).mean()),
           "mfma_roofline": {"kernel": km, "achieved_TOPS": round(ops / scr / 1e12, 1) if scr else None,
                             "peak_TOPS": I8_PEAK_TOPS,
                             "frac": round(ops / scr / 1e12 / I8_PEAK_TOPS, 4) if scr else None},
           "checked_pairs": checked}
    if args.cpu_seconds > 0:  # the oracle's C restatement (exact cosine, sequential int MACs) on host threads
        import concurrent.futures as cf

        import oracle

        a0, a1 = d0[0].cpu().numpy(), d1[0].cpu().numpy()
        threads = max(1, min(16, os.cpu_count() or 1))
        deadline = time.perf_counter() + args.cpu_seconds

        def worker(_):
            c = 0
            while time.perf_counter() < deadline:
                oracle.allpairs_i8(a0, a1)
                c += 1
            return c

        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            total = sum(ex.map(worker, range(threads)))
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(total / dt, 2), "unit": "pairs/s", "cores": threads, "kind": "port",
                               "sample": "%d pairs of %dx%dx256 int8 in %.1f s on %d host threads"
                                         % (total, n, n, dt, threads)}
    ctx.close()
    return out


if __name__ == "__main__":
    main()
