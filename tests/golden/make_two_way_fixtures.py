#!/usr/bin/env python3
"""Golden outputs of the reference's OWN PointTracker.nn_match_two_way
(python/pairwise_pnp.py:281-323) on the reference's committed fp32 descriptor fixtures
(tracking/pair0.h, pair10.h -> tests/golden/tracking_pair*.npz) and on synthetic pairs.

Runs ONLY in the build container where /root/reference exists.  pairwise_pnp.py cannot be
imported (cv2 / torchvision / matplotlib are absent), so the PointTracker class definition
alone is parsed out of the file and executed with numpy bound -- the reference's own code.
Only its outputs (3 x L match arrays) are stored; inputs are the committed fixtures or are
regenerated from seeds (synth.synth_pair_f32)."""
import ast
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
import synth  # noqa: E402

REF = os.environ.get("MV_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "python", "pairwise_pnp.py")


def inputs():
    """name -> (desc0 [n0, 256], desc1 [n1, 256]) float32 (also used by the tests)"""
    out = {}
    for name in ("pair0", "pair10"):
        d = np.load(os.path.join(HERE, "tracking_%s.npz" % name))
        out[name] = (d["image0_desc"], d["image1_desc"])
    for s in (0, 1):
        p = synth.synth_pair_f32(60 + s, n=300, noise=0.3)
        out["synth%d" % s] = (p["desc0"], p["desc1"])
    return out


THRESHOLDS = (0.7, 1.2)


def main():
    if not os.path.exists(SRC):
        print("reference not present; fixtures are already committed", file=sys.stderr)
        return 1
    tree = ast.parse(open(SRC).read())
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "PointTracker"][0]
    ns = {"np": np}
    exec(compile(ast.Module(body=[cls], type_ignores=[]), SRC, "exec"), ns)
    pt = object.__new__(ns["PointTracker"])
    res = {}
    for name, (a, b) in inputs().items():
        for th in THRESHOLDS:
            m = pt.nn_match_two_way(a.T.copy(), b.T.copy(), th)  # the reference takes D x N
            res["%s_%g" % (name, th)] = np.asarray(m, np.float64)
            print(name, th, m.shape[1], file=sys.stderr)
    np.savez_compressed(os.path.join(HERE, "two_way.npz"), **res)
    return 0


if __name__ == "__main__":
    sys.exit(main())
