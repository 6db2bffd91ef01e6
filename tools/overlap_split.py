"""Feasibility timing: k_ap_split of batch k+1 (context 2) running concurrently with
k_ap_match of batch k (context 1), against the two run back to back.  Timing only."""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
sys.path.insert(0, ROOT)
import mvtrack  # noqa: E402
import bench  # noqa: E402

B, n = 1024, 1024
dev = torch.device("cuda", 0)
d0, d1, _, _ = bench.gen_batch(torch, dev, B, n, seed=1)
e0, e1, _, _ = bench.gen_batch(torch, dev, B, n, seed=2)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
c1, c2 = mvtrack.Context(0), mvtrack.Context(0)
c1.set_stream(s1)
c2.set_stream(s2)
c1.reserve(B, n)
c2.reserve(B, n)
c1.match_allpairs_f32_prepare(d1, nn_)
c2.match_allpairs_f32_prepare(e1, nn_)
torch.cuda.synchronize()


def t(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def match():
    c1.match_allpairs_f32_run(d0, d1, nn_, nn_, idx, None, 0.8)
    torch.cuda.synchronize()


def split():
    c2.match_allpairs_f32_prepare(e1, nn_)
    torch.cuda.synchronize()


def both():
    c2.match_allpairs_f32_prepare(e1, nn_)
    c1.match_allpairs_f32_run(d0, d1, nn_, nn_, idx, None, 0.8)
    torch.cuda.synchronize()


def seq():
    c1.match_allpairs_f32_run(d0, d1, nn_, nn_, idx, None, 0.8)
    c2.match_allpairs_f32_prepare(e1, nn_)
    torch.cuda.synchronize()


print("match %.3f ms  split %.3f ms  sequential %.3f ms  concurrent %.3f ms" % (t(match), t(split), t(seq), t(both)))
