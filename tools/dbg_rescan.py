"""Mismatches of the default all-pairs screen against the oracle on the quantisation-stress pairs
(tests/test_gpu_allpairs.py::test_allpairs_f32_quantisation_stress) -- per differing row: GPU and
oracle index, the oracle's exact dots of both columns.  Env THR (0.0), MV_LIB for a variant."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import mvtrack  # noqa: E402
import oracle  # noqa: E402
from test_gpu_allpairs import run_f32  # noqa: E402

rng = np.random.default_rng(31)
n = 160


def unit(k):
    x = rng.standard_normal((k, 256)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


a = unit(n)
b = a[rng.permutation(n)] + 0.03 * rng.standard_normal((n, 256)).astype(np.float32)
b /= np.linalg.norm(b, axis=1, keepdims=True)
scales = np.float32(2.0) ** rng.integers(-45, 46, n).astype(np.float32)
a_s = (a * scales[:, None]).astype(np.float32)
b_s = (b * np.float32(2.0) ** rng.integers(-39, 40, n).astype(np.float32)[:, None]).astype(np.float32)
spiky = a.copy()
spiky[:40] *= np.float32(1e-4)
spiky[:40, 3] = 1.0
sparse = a.copy()
sparse[40:80, 16:] = 0.0
sparse[80:84] = 0.0
bz = b.copy()
bz[10:14] = 0.0
near = a.copy()
near2 = np.concatenate([a, a + np.float32(1e-4) * unit(n)]).astype(np.float32)
pairs = [(a_s, b), (a, b_s), (spiky, b), (sparse, bz), (-a, b), (near, near2), (a, np.concatenate([b, -b]))]
thr = float(os.environ.get("THR", "0.0"))
ctx = mvtrack.Context(0)
for scores in (True, False):
    idx, sc = run_f32(ctx, torch, pairs, thresh=thr, scores=scores)
    for k, (x, y) in enumerate(pairs):
        i2, s2 = oracle.allpairs_f32(x, y, thr)
        bad = np.nonzero(idx[k, :x.shape[0]] != i2)[0]
        if len(bad):
            print("scores", scores, "pair", k, "rows differing", len(bad))
            dots = x.astype(np.float64) @ y.astype(np.float64).T
            for r in bad[:8]:
                g, o = idx[k, r], i2[r]
                top = np.argsort(-dots[r])[:5]
                print("  row %d gpu %d oracle %d  dot(gpu) %s dot(oracle) %s top5 %s %s" % (
                    r, g, o, dots[r, g] if g >= 0 else None, dots[r, o] if o >= 0 else None, top,
                    np.round(dots[r, top], 5)))
print("done")
