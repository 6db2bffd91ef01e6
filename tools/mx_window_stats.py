#!/usr/bin/env python3
"""How wide the MX-fp8 screen's exactness window is on the reference's own descriptors
(tests/golden/tracking_pair*.npz) and on the bench's synthetic pairs: per row, whether the
window decides it (no match / one exact re-score) or leaves it ambiguous (candidate list).
Simulates E8M0 (32-k blocks) + e4m3 round-to-nearest-even in float64; CPU only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
import synth  # noqa: E402


def q8(x):
    r = x.reshape(x.shape[0], -1, 32)
    m = np.abs(r).max(-1, keepdims=True)
    e = np.floor(np.log2(np.maximum(m, 1e-30))) - 7
    s = r / 2.0 ** e
    ex = np.floor(np.log2(np.maximum(np.abs(s), 2.0 ** -6)))
    ulp = 2.0 ** (ex - 3)
    return (np.round(s / ulp) * ulp * 2.0 ** e).reshape(x.shape)


def q16(x):
    return (x * 16384).astype(np.float16).astype(np.float64) / 16384


def stat(label, a, b, thresh=0.8):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    an = np.linalg.norm(a, axis=1)
    B = np.linalg.norm(b, axis=1).max()
    r = np.arange(a.shape[0])
    for screen, q, rel in (("fp16", q16, 9.77e-4), ("mx", q8, 0.1295)):
        qa, qb = q(a), q(b)
        s = qa @ qb.T
        o = np.argsort(-s, axis=1)
        M, M2 = s[r, o[:, 0]], s[r, o[:, 1]]
        for bound, dp in (("worst", rel * an * B),
                          ("measured", np.linalg.norm(qa, axis=1) * np.linalg.norm(qb - b, axis=1).max()
                           + np.linalg.norm(qa - a, axis=1) * B)):
            live = M + dp > thresh
            amb = live & ~(M2 < M - 2 * dp)
            nc = (s >= (M - 2 * dp)[:, None]).sum(1)
            print("%-8s %-5s %-8s rows %5d decided-by-one-dot %5d ambiguous %5d (mean cand %.1f, >16: %d) dp %.4f"
                  % (label, screen, bound, a.shape[0], (live & ~amb).sum(), amb.sum(),
                     nc[amb].mean() if amb.any() else 0.0, (amb & (nc > 16)).sum(), dp.mean()))


def main():
    for name in ("pair0", "pair10"):
        d = np.load(os.path.join(ROOT, "tests", "golden", "tracking_%s.npz" % name))
        stat(name, d["image0_desc"], d["image1_desc"])
    p = synth.synth_pair_f32(0)
    stat("synth", p["desc0"], p["desc1"])


if __name__ == "__main__":
    main()
