#!/usr/bin/env python3
"""Diagnosis (GPU): tests/test_gpu_frontend.py::test_window_match_exact_ties_and_threshold's 24 x 80
case -- for every query whose matched frame-0 cell differs from the oracle's, both cells' exact
scores (dot, |a|^2 -> dot^2 / |a|^2) and scan positions."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import mvtrack  # noqa: E402
import oracle  # noqa: E402
import synth  # noqa: E402

rows, cols = 24, 80
f0, f1 = synth.synth_window_pair(77, rows=rows, cols=cols)
cells = rows * cols
rng = np.random.default_rng(5)
dirs = np.array([[-3, 4, 5], [-3, 5, 5], [-1, 2, 2]], np.int64)
pick = rng.integers(0, 3, cells)
mult = rng.integers(1, 5, cells)
d0 = np.zeros((cells, 256), np.int8)
d0[:, :3] = (dirs[pick] * mult[:, None]).astype(np.int8)
d1 = np.zeros((cells, 256), np.int8)
d1[:, 1] = d1[:, 2] = rng.integers(1, 9, cells).astype(np.int8)
g0, g1 = dict(f0), dict(f1)
g0["desc"], g1["desc"] = d0, d1
N = 100
r = oracle.track_window(g0, g1, as_built=False, N=N, cap=100000, max_matches=150)
ctx = mvtrack.Context(0)
p = mvtrack.window_params(mvtrack.AS_INTENDED, max_matches=150)
p1, p2, q = ctx.window_match_host(p, rows, cols, d0, r["max_idx0"], r["probs0"], d1, r["patches1"], r["indices1"])
print("matches gpu %d oracle %d" % (len(q), len(r["query"])))
bad = np.nonzero((p1 != r["points1"]).any(axis=1))[0]
print("differing matches:", len(bad))
for k in bad[:12]:
    qi = int(q[k])
    patch1 = int(r["patches1"][qi])
    x1, y1 = patch1 // rows, patch1 % rows
    a = d1[patch1].astype(np.int64)

    def cell_of(pt):  # the frame-0 cell a point came from (x = bx * 8 + idx % 8)
        return int(pt[0]) // 8, int(pt[1]) // 8

    out = []
    for name, pt in (("gpu", p1[k]), ("oracle", r["points1"][k])):
        bx, by = cell_of(pt)
        c = d0[bx * rows + by].astype(np.int64)
        dot, na = int(a @ c), int(c @ c)
        out.append("%s cell (%d,%d) cp %d dot %d |b|^2 %d d2n %.6f dir %s" % (
            name, bx, by, bx * rows + by, dot, na, dot * dot / na if na else -1, d0[bx * rows + by][:3]))
    print("query %d at (%d,%d) |a|^2 %d:\n   %s" % (qi, x1, y1, int(a @ a), "\n   ".join(out)))
ctx.close()
