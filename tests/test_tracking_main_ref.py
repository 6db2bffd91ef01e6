"""The windowed match loop (src/tracking_main.c:103-194) pinned to the reference ITSELF: the body of
tracking_main.c's main, cut out of the reference text by oracle/Makefile and compiled with
src/top_N.c and src/pnp_solver.c (oracle/ref_track_harness.c), against the oracle's restatement
of the same driver (softmax -> top-N -> window match -> stub RANSAC -> pose), on the cases of
tests/golden/make_tracking_main_fixtures.py: the self pair (100 matches), the real KITTI pair
quantized_image0 -> frame 000001 through the SuperPoint oracle (51 matches as built),
synthetic pairs, scales whose as-built effective scale is 2 / -2, top_N.c's exit(1) and the empty
match list -- each in the as-built build (no prototype: SURVEY F7) and with top_N.h in scope (the
true scale).  The committed golden (tracking_main_ref.npz) is what the GPU test compares with."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

sys.path.insert(0, GOLDEN)
from make_tracking_main_fixtures import FIELDS, tracking_main_cases  # noqa: E402

K_TRACKING_MAIN = np.array([[517.306408, 0.0, 318.643040], [0.0, 516.469215, 255.313989], [0.0, 0.0, 1.0]],
                           np.float32)  # tracking_main.c:205-207


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def oracle_tracking_main(orc, f0, f1, true_scale):
    """the oracle's restatement of main (:84-228) with the scale the callee receives"""
    s0, s1 = float(f0["semi_scale"]), float(f1["semi_scale"])
    if not true_scale:  # F7: the callee reads the low 32 bits of the promoted double
        s0, s1 = orc.scale_as_built(s0), orc.scale_as_built(s1)
    _, mi0, pr0 = orc.compute_softmax(s0, f0["semi"])
    st, pa, ix, _ = orc.compute_top_N(s1, f1["semi"], 100)
    out = dict(status=0, points1=np.zeros((0, 2), np.float32), points2=np.zeros((0, 2), np.float32),
               num_inliers=-1, inliers=np.zeros(0, np.int32), E=None)
    if st != 0:
        out["status"] = 1  # top_N.c:91-94 exit(1)
        return out
    p1, p2, _, _ = orc.window_match(24, 80, f0["desc"], mi0, pr0, f1["desc"], pa, ix, as_built=True)
    out.update(points1=p1, points2=p2)
    if len(p1) == 0:
        out["status"] = 2  # pnp_solver.c:123 rand() % 0
        return out
    _, E, inl, ni = orc.ransac_essential_matrix(p1, p2, K_TRACKING_MAIN, 10, 1.1)
    out.update(num_inliers=ni, inliers=inl)
    if ni >= 0:
        out["E"] = E
        out["R1"], out["R2"], out["t"] = orc.recover_pose(E)
    return out


def assert_same(o, r, tag):
    assert int(o["status"]) == int(r["status"]), tag
    assert o["points1"].shape == r["points1"].shape and (o["points1"] == r["points1"]).all(), tag
    assert (o["points2"] == r["points2"]).all(), tag
    if int(r["status"]) != 0:
        return
    assert int(o["num_inliers"]) == int(r["num_inliers"]), tag
    assert (o["inliers"] == r["inliers"]).all(), tag
    if int(r["num_inliers"]) >= 0:
        assert (bits(o["E"]) == bits(r["E"])).all(), tag
        for k in ("R1", "R2", "t"):
            assert (bits(o[k]) == bits(r[k])).all(), (tag, k)
    else:
        assert np.isnan(np.asarray(r["E"])).all(), tag  # the RANSAC never wrote E


def golden_case(g, name, mode):
    return {k: g["%s_%s_%s" % (name, mode, k)] for k in FIELDS}


@pytest.mark.skipif("not __import__('oracle').ref_track_available()", reason="oracle/_ref not built here")
def test_oracle_equals_reference_tracking_main(orc):
    """the oracle's driver == the reference's own main, every case, both builds, bit for bit"""
    g = load_golden("tracking_main_ref.npz")
    counts = {}
    for name, (f0, f1) in tracking_main_cases().items():
        for mode, ts in (("built", False), ("true", True)):
            r = orc.ref_tracking_main(f0, f1, true_scale=ts)
            o = oracle_tracking_main(orc, f0, f1, ts)
            assert_same(o, r, (name, mode))
            assert_same(golden_case(g, name, mode), r, (name, mode, "golden"))  # the committed golden is current
            counts[(name, mode)] = len(r["points1"])
    assert counts[("self", "built")] == 100 and counts[("kitti01", "built")] == 51
    assert counts[("kitti01", "true")] != 51  # the true scale changes top-N, hence the matches


@pytest.mark.skipif("not __import__('oracle').ref_track_available()", reason="oracle/_ref not built here")
def test_reference_driver_o2_build_equals_o0(orc):
    """the -O2 build bench.py's cpu_c0 times gives the -O0 (CMake default) build's outputs"""
    for name, (f0, f1) in tracking_main_cases().items():
        assert_same(orc.ref_tracking_main(f0, f1, o2=True), orc.ref_tracking_main(f0, f1), name)


def test_oracle_equals_committed_tracking_main_golden(orc):
    """the same against the committed outputs of the reference (what the GPU box checks)"""
    g = load_golden("tracking_main_ref.npz")
    for name, (f0, f1) in tracking_main_cases().items():
        for mode, ts in (("built", False), ("true", True)):
            assert_same(oracle_tracking_main(orc, f0, f1, ts), golden_case(g, name, mode), (name, mode))


def test_kitti01_frame_is_the_superpoint_oracle_output(orc):
    """the stored frame 000001 is the C SuperPoint oracle's output on the committed KITTI image"""
    g = load_golden("tracking_main_ref.npz")
    w = dict(load_golden("superpoint_qnonorm.npz"))
    semi1, desc1, ss, _, _, _ = orc.sp_forward(load_golden("kitti00_images.npz")["img_000001"], orc.sp_net(w))
    assert (semi1 == g["kitti01_semi1"]).all() and (desc1 == g["kitti01_desc1"]).all()
    # python/superpoint_inference.py:648,657 writes frame 0's scale into frame 1's header; the
    # network's own scale for frame 1 happens to be the same value here
    assert np.float32(ss) == load_golden("quantized_image0.npz")["semi_scale"]
