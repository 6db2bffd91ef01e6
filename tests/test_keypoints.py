"""Keypoint extraction + descriptor sampling: SuperPointFrontend.run after the
network -- softmax -> heatmap -> threshold -> nms_fast -> sort -> border removal ->
grid_sample -> L2 normalise (python/pairwise_pnp.py:116-257).

CPU: the oracle is pinned against the reference's OWN code executed on synthetic network
outputs (tests/golden/make_keypoint_fixtures.py): bit for bit when the reference runs with
the correctly rounded float32 exp (every other operation its own numpy/torch code), and, with
numpy's SIMD expf, the same keypoints with confidences within 4 ulp and identical descriptors.
GPU (marked): the HIP pipeline equals the oracle bit for bit (points, confidences, descriptors)."""
import numpy as np
import pytest

import synth
from conftest import load_golden

CASES = ["small", "quantized_shape", "kitti", "kitti_b", "odd"]


def case(name):
    g = load_golden("keypoints.npz")
    seed, H, W, Hc, Wc = (int(v) for v in g[name + "_params"])
    semi, desc = synth.synth_superpoint_outputs(seed, Hc, Wc)
    return g, semi, desc, H, W


@pytest.mark.parametrize("name", CASES)
def test_oracle_bit_exact_vs_reference_with_correctly_rounded_exp(orc, name):
    g, semi, desc, H, W = case(name)
    pts, d, heat = orc.keypoints(semi, desc, H, W)
    ref = g[name + "_cr_pts"]
    assert pts.shape[0] == ref.shape[1]
    assert (pts.T.astype(np.float64) == ref).all()  # x, y, confidence, order
    cols = g[name + "_cr_desc_cols"]
    assert (d[cols].T.view(np.int32) == g[name + "_cr_desc"].view(np.int32)).all()
    if name == "small":
        assert (heat.view(np.int32) == g["small_cr_heatmap"].view(np.int32)).all()


@pytest.mark.parametrize("name", CASES)
def test_oracle_vs_reference_with_numpy_exp(orc, name):
    """numpy's float32 exp is not correctly rounded (~40 % of values differ by an ulp): the
    heatmap moves by a few ulp; the keypoints, their descriptors and (up to exact ties) their
    order do not."""
    g, semi, desc, H, W = case(name)
    pts, d, heat = orc.keypoints(semi, desc, H, W)
    ref = g[name + "_pts"]
    assert pts.shape[0] == ref.shape[1]
    got = {(int(x), int(y)): (c, k) for k, (x, y, c) in enumerate(pts)}
    exp = {(int(x), int(y)): (np.float32(c), k) for k, (x, y, c) in enumerate(ref.T)}
    assert got.keys() == exp.keys()
    ulp = max(abs(int(np.float32(got[p][0]).view(np.int32)) - int(exp[p][0].view(np.int32))) for p in got)
    assert ulp <= 4
    cols = g[name + "_desc_cols"]
    for j, c in enumerate(cols):  # the reference's c-th point, wherever the oracle ranks it
        x, y = int(ref[0, c]), int(ref[1, c])
        assert (d[got[(x, y)][1]] == g[name + "_desc"][:, j]).all()
    if name == "small":
        h = g["small_heatmap"]
        assert np.abs(heat.view(np.int32) - h.view(np.int32)).max() <= 4


def test_oracle_edge_cases(orc):
    # no candidate at all (every cell's dustbin dominates): run() returns no points
    semi = np.zeros((65, 6, 9), np.float32)
    semi[64] = 40.0
    pts, d, _ = orc.keypoints(semi, np.ones((256, 6, 9), np.float32), 48, 72)
    assert pts.shape == (0, 3) and d.shape == (0, 256)
    # a single candidate, and one inside the border band (removed)
    semi[64] = 40.0
    semi[9, 2, 3] = 60.0  # cell (2, 3), i = 1, j = 1 -> pixel (x, y) = (25, 17)
    semi[0, 0, 0] = 60.0  # pixel (0, 0): in the 4-pixel border band
    pts, d, _ = orc.keypoints(semi, np.ones((256, 6, 9), np.float32), 48, 72)
    assert pts.shape[0] == 1 and tuple(pts[0, :2]) == (25.0, 17.0)
    assert np.allclose(np.linalg.norm(d, axis=1), 1.0, atol=1e-6)
    # two candidates 3 px apart: the weaker is suppressed; 5 px apart: both kept
    semi = np.zeros((65, 6, 9), np.float32)
    semi[64] = 40.0
    semi[0, 2, 2] = 61.0  # (16, 16)
    semi[3, 2, 2] = 60.0  # (19, 16): within 4 px of (16, 16)
    semi[0, 2, 4] = 60.0  # (32, 16)
    pts, _, _ = orc.keypoints(semi, np.ones((256, 6, 9), np.float32), 48, 72)
    assert sorted(map(tuple, pts[:, :2].tolist())) == [(16.0, 16.0), (32.0, 16.0)]
