#!/usr/bin/env python3
"""SURVEY 8(d) C0 on the CPU: the reference's tracking_main driver on the real KITTI pair
(quantized_image0 -> frame 000001, 24 x 80 cells, 51 matches as built), per pair on one core and
on P worker processes (one pair per process at a time: main's rand() and the capture are
process-global, so the driver is not thread-safe).  Kind 'reference': the body of
src/tracking_main.c's main cut out of the reference text and built at -O2 with src/top_N.c and
src/pnp_solver.c (oracle/_ref/libmv_ref_track_o2.so, oracle/ref_track_harness.c); 'port' when
oracle/_ref is absent: the oracle's restatement of the same driver.  Prints one JSON line.

Run by bench.py as a child process (never forked from a process that has touched the GPU).
TEST / BASELINE INFRASTRUCTURE: it executes the oracle, never the product."""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

K = np.array([[517.306408, 0.0, 318.643040], [0.0, 516.469215, 255.313989], [0.0, 0.0, 1.0]], np.float32)


def _pair():
    from make_tracking_main_fixtures import tracking_main_cases

    return tracking_main_cases()["kitti01"]


def _one_pair_fn():
    import oracle

    f0, f1 = _pair()
    if oracle.ref_track_available():
        return (lambda: len(oracle.ref_tracking_main(f0, f1, o2=True)["points1"])), "reference"

    def port():
        r = oracle.track_window(f0, f1, as_built=True)
        n = r["points1"].shape[0]
        if n > 0:
            _, E, _, ni = oracle.ransac_essential_matrix(r["points1"], r["points2"], K, 10, 1.1)
            if ni > 0:
                oracle.recover_pose(E)
        return n

    return port, "port"


def _worker(deadline):
    fn, _ = _one_pair_fn()
    c = 0
    while time.time() < deadline:
        fn()
        c += 1
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--procs", type=int, default=1)
    a = ap.parse_args()
    fn, kind = _one_pair_fn()
    matches = fn()
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < min(2.0, a.seconds / 4):
        fn()
        k += 1
    us1 = (time.perf_counter() - t0) / k * 1e6
    deadline = time.time() + a.seconds
    t1 = time.perf_counter()
    with cf.ProcessPoolExecutor(a.procs) as ex:
        tot = sum(ex.map(_worker, [deadline] * a.procs))
    dt = time.perf_counter() - t1
    print(json.dumps({"kind": kind, "us_per_pair_1core": round(us1, 1), "pairs": tot, "seconds": round(dt, 2),
                      "procs": a.procs, "value": round(tot / dt, 1), "matches": matches}), flush=True)


if __name__ == "__main__":
    main()
