#!/usr/bin/env python3
"""Projection-factor linearisation + pose normal equations (include/factors.h) at tracking
scale: P poses (frames) x M factors each (one per tracked landmark), e.g. 1024 x 1024.
Prints one JSON line: factors/s, per-kernel averages and the HBM fraction of k_pf_linearize
against its algorithmic bytes (landmark 12 B + pose/camera 44 B + ids 8 B + measurement 8 B
read, error 8 B + J 80 B written per factor).  GPU only."""
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

HBM_PEAK_GBS = 8000.0


def run(P=1024, M=1024, steps=20, warmup=3, check=1):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    F, L = P * M, P * M // 2
    ldmk = torch.stack([torch.rand(L, generator=g, device=dev) * 20 - 10, torch.rand(L, generator=g, device=dev) * 6 - 3,
                        torch.rand(L, generator=g, device=dev) * 55 + 5], 1).contiguous()
    q = torch.randn((P, 4), generator=g, device=dev) * torch.tensor([0.0, 0.05, 0.05, 0.05], device=dev)
    q[:, 0] += 1.0
    q = q / q.norm(dim=1, keepdim=True)
    pose = torch.cat([q, torch.randn((P, 3), generator=g, device=dev) * 0.5], 1).contiguous()
    cam = torch.tensor([718.856, 718.856, 607.1928, 185.2157], device=dev).repeat(P, 1).contiguous()
    pid = torch.arange(P, device=dev, dtype=torch.int32).repeat_interleave(M).contiguous()
    lid = torch.randint(0, L, (F,), generator=g, device=dev, dtype=torch.int32)
    meas = (torch.rand((F, 2), generator=g, device=dev) * torch.tensor([1241.0, 376.0], device=dev)).contiguous()
    off = (torch.arange(P + 1, device=dev, dtype=torch.int32) * M).contiguous()
    err = torch.empty((F, 2), device=dev)
    J = torch.empty((F, 20), device=dev)
    HPP = torch.empty((P, 36), device=dev)
    gr = torch.empty((P, 6), device=dev)
    ee = torch.empty(P, device=dev)
    ctx = mvtrack.Context(0)
    ctx.set_stream(torch.cuda.current_stream())

    def step():
        ctx.projection_factors(ldmk, pose, cam, lid, pid, meas, err, J)
        ctx.pose_normal_equations(off, J, HPP, gr, ee)

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
    for k in ("k_pf_linearize", "k_pose_ne"):
        ms, c = mvtrack.profile_query(k)
        stages[k] = round(ms / max(c, 1), 4)
    checked = 0
    if check:
        import oracle

        sel = slice(0, M * check)  # the first `check` poses
        e2, J2, H2 = oracle.pf_linearize(ldmk.cpu().numpy(), pose.cpu().numpy(), lid[sel].cpu().numpy(),
                                         pid[sel].cpu().numpy(), meas[sel].cpu().numpy(), cam.cpu().numpy())
        assert (err[sel].cpu().numpy().view(np.int32) == e2.view(np.int32)).all()
        assert (J[sel].cpu().numpy().view(np.int32) == J2.view(np.int32)).all()
        HPP2, g2, _ = oracle.pose_normal_equations(off[:check + 1].cpu().numpy(), H2)
        assert (HPP[:check].cpu().numpy() == HPP2).all() and (gr[:check].cpu().numpy() == g2).all()
        checked = check
    byt = 12 + 44 + 8 + 8 + 8 + 80
    lin = stages["k_pf_linearize"] * 1e-3
    out = {"metric": "projection factors linearised + pose normal equations, factors/sec (%d poses x %d)" % (P, M),
           "value": round(F / (el / steps), 1), "unit": "factors/s", "ms_per_step": round(el / steps * 1e3, 4),
           "stages_ms": stages,
           "hbm_roofline": {"kernel": "k_pf_linearize", "bytes_per_factor": byt,
                            "GBs": round(byt * F / lin / 1e9, 1), "frac": round(byt * F / lin / 1e9 / HBM_PEAK_GBS, 4),
                            "peak_GBs": HBM_PEAK_GBS},
           "checked_poses": checked}
    ctx.close()
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=1024)
    ap.add_argument("--per-pose", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps(run(a.poses, a.per_pose, a.steps)), flush=True)
