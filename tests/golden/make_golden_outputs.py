#!/usr/bin/env python3
"""Expected outputs of the hot path on the committed fixtures, produced by the
CPU oracle (oracle/liboracle.so) -- and, where /root/reference is present, only
after the oracle has been checked bit-for-bit against the reference's own code
compiled by oracle/Makefile (oracle/_ref/libmv_ref.so).

Writes tests/golden/expected_outputs.npz.  Re-run after changing a fixture:
    make -C oracle && python tests/golden/make_golden_outputs.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
import oracle as O  # noqa: E402
import synth  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def pin_against_reference(img):
    """softmax/top-N (both scales), svd/pose and the gemmini matmul vs the reference build."""
    R = O.ref()
    P = O._ptr
    semi = np.ascontiguousarray(img["semi"])
    for scale in (float(img["semi_scale"]), O.scale_as_built(float(img["semi_scale"]))):
        nv = ctypes.c_int(0)
        mi = np.zeros(1920, np.int32)
        pr = np.zeros(1920, np.float32)
        R.compute_softmax(scale, P(semi), ctypes.byref(nv), P(mi), P(pr))
        nv2, mi2, pr2 = O.compute_softmax(scale, semi)
        assert nv.value == nv2 and (mi == mi2).all() and (_bits(pr) == _bits(pr2)).all()
        ns = ctypes.c_int(0)
        pa = np.zeros(100, np.int32)
        ix = np.zeros(100, np.int32)
        pp = np.zeros(100, np.float32)
        R.compute_top_N(scale, P(semi), 100, ctypes.byref(ns), P(pa), P(ix), P(pp))
        st, pa2, ix2, pp2 = O.compute_top_N(scale, semi, 100)
        n = ns.value
        assert st == 0 and n == len(pa2) and (pa[:n] == pa2).all() and (ix[:n] == ix2).all()
        assert (_bits(pp[:n]) == _bits(pp2)).all()
    E = np.eye(3, dtype=np.float32).reshape(9)
    R1 = np.zeros(9, np.float32)
    R2 = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    R.recover_pose_from_essential_matrix(P(E), P(R1), P(R2), P(t))
    a, b, c = O.recover_pose(E)
    assert (_bits(R1) == _bits(a).reshape(9)).all() and (_bits(R2) == _bits(b).reshape(9)).all()
    assert (_bits(t) == _bits(c)).all()
    print("oracle pinned against the reference build")


def main():
    img = np.load(os.path.join(G, "quantized_image0.npz"))
    if O.ref_available():
        pin_against_reference(img)
    else:
        print("WARNING: oracle/_ref not built; outputs come from the (previously pinned) oracle")
    out = {}
    semi, desc = img["semi"], img["desc"]
    rows, cols = int(img["feature_rows"]), int(img["feature_cols"])
    for mode, scale in (("built", O.scale_as_built(float(img["semi_scale"]))), ("true", float(img["semi_scale"]))):
        nv, mi, pr = O.compute_softmax(scale, semi)
        out["softmax_%s_nv" % mode] = np.int32(nv)
        out["softmax_%s_mi" % mode] = mi
        out["softmax_%s_pr" % mode] = pr
        st, pa, ix, pp = O.compute_top_N(scale, semi, 100)
        out["topn_%s_patches" % mode] = pa
        out["topn_%s_indices" % mode] = ix
        out["topn_%s_probs" % mode] = pp
    # windowed match: self pair and synthetic shifted pairs, both semantics
    f_img = dict(rows=rows, cols=cols, semi=semi, desc=desc, semi_scale=img["semi_scale"])
    cases = {"self": (f_img, f_img)}
    for s in (1, 2, 3):
        cases["syn%d" % s] = synth.synth_window_pair(s)
    for name, (f0, f1) in cases.items():
        for built in (True, False):
            r = O.track_window(f0, f1, as_built=built)
            tag = "win_%s_%s" % (name, "built" if built else "true")
            out[tag + "_p1"] = r["points1"]
            out[tag + "_p2"] = r["points2"]
            out[tag + "_q"] = r["query"]
    # all-pairs fp32 on the reference's fp32 keypoint fixtures (a10 semantics)
    for name in ("pair0", "pair10"):
        d = np.load(os.path.join(G, "tracking_%s.npz" % name))
        idx, sc = O.allpairs_f32(d["image0_desc"], d["image1_desc"], 0.8)
        out["ap_%s_idx" % name] = idx
        out["ap_%s_score" % name] = sc
    # as-built pose constant (F2)
    R1, R2, t = O.recover_pose(np.eye(3, dtype=np.float32))
    out["pose_built_R1"], out["pose_built_R2"], out["pose_built_t"] = R1, R2, t
    np.savez_compressed(os.path.join(G, "expected_outputs.npz"), **out)
    print("wrote expected_outputs.npz:", len(out), "arrays;",
          "pair0 matches", int((out["ap_pair0_idx"] >= 0).sum()), "pair10", int((out["ap_pair10_idx"] >= 0).sum()),
          "self-pair window matches", len(out["win_self_built_q"]))


if __name__ == "__main__":
    main()
