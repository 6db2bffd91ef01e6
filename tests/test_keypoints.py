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


# ------------------------------------------------------------------ GPU
def _gpu_batch(ctx, torch, frames, H, W, cap, heat=False):
    dev = torch.device("cuda:0")
    semi = torch.from_numpy(np.stack([f[0] for f in frames])).to(dev)
    cd = torch.from_numpy(np.stack([f[1] for f in frames])).to(dev)
    B, Hc, Wc = semi.shape[0], semi.shape[2], semi.shape[3]
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    kp = torch.zeros((B, cap, 2), dtype=torch.float32, device=dev)
    conf = torch.zeros((B, cap), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, cap, 256), dtype=torch.float32, device=dev)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    hm = torch.zeros((B, Hc * 8, Wc * 8), dtype=torch.float32, device=dev) if heat else None
    ctx.set_stream(torch.cuda.current_stream())
    ctx.keypoints(semi, cd, H, W, n, kp, conf, desc, st, heat=hm)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    out = (n.cpu().numpy(), kp.cpu().numpy(), conf.cpu().numpy(), desc.cpu().numpy(), st.cpu().numpy())
    return out + ((hm.cpu().numpy(),) if heat else ())


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_keypoints_bit_exact(ctx, orc, torch_cuda, name):
    g, semi, desc, H, W = case(name)
    pts, d, heat = orc.keypoints(semi, desc, H, W)
    n, kp, conf, dd, st, hm = _gpu_batch(ctx, torch_cuda, [(semi, desc)], H, W, cap=4096, heat=True)
    assert (hm[0].view(np.int32) == heat.view(np.int32)).all()
    assert st[0] == 0 and n[0] == pts.shape[0]
    k = n[0]
    assert (kp[0, :k] == pts[:, :2]).all() and (conf[0, :k].view(np.int32) == pts[:, 2].view(np.int32)).all()
    assert (dd[0, :k].view(np.int32) == d.view(np.int32)).all()
    # and the reference's own code (correctly rounded exp) on the fixture columns
    assert (kp[0, :k].T.astype(np.float64) == g[name + "_cr_pts"][:2]).all()


@pytest.mark.gpu
def test_gpu_keypoints_batch_cap_and_edges(ctx, orc, torch_cuda):
    """a batch of KITTI-size frames with a cap below the survivor count (prefix + status), a
    frame without candidates and a frame with one candidate."""
    frames = [synth.synth_superpoint_outputs(30 + i, 47, 155) for i in range(3)]
    empty = np.zeros((65, 47, 155), np.float32)
    empty[64] = 40.0
    one = empty.copy()
    one[9, 20, 30] = 60.0
    frames += [(empty, frames[0][1]), (one, frames[1][1])]
    cap = 1024
    n, kp, conf, dd, st = _gpu_batch(ctx, torch_cuda, frames, 376, 1241, cap)
    for b, (s_, d_) in enumerate(frames):
        pts, d, _ = orc.keypoints(s_, d_, 376, 1241)
        k = min(cap, pts.shape[0])
        assert n[b] == k and st[b] == (-2 if pts.shape[0] > cap else 0), b
        assert (kp[b, :k] == pts[:k, :2]).all() and (conf[b, :k] == pts[:k, 2]).all(), b
        assert (dd[b, :k].view(np.int32) == d[:k].view(np.int32)).all(), b
    assert n[3] == 0 and n[4] == 1 and tuple(kp[4, 0]) == (30 * 8 + 1.0, 20 * 8 + 1.0)


@pytest.mark.gpu
def test_gpu_keypoints_large_frame_transpose_path(ctx, orc, torch_cuda):
    """frames above the 9216 cells whose 4-channel planes fit LDS take the NCHW->NHWC
    transpose + per-keypoint sampling path: the same bits."""
    frames = [synth.synth_superpoint_outputs(50 + i, 60, 160) for i in range(2)]
    n, kp, conf, dd, st = _gpu_batch(ctx, torch_cuda, frames, 480, 1280, 1024)
    for b, (s_, d_) in enumerate(frames):
        pts, d, _ = orc.keypoints(s_, d_, 480, 1280)
        k = min(1024, pts.shape[0])
        assert n[b] == k and k > 100, b
        assert (kp[b, :k] == pts[:k, :2]).all() and (dd[b, :k].view(np.int32) == d[:k].view(np.int32)).all(), b


@pytest.mark.gpu
@pytest.mark.parametrize("Hc,Wc,p_corner,dustbin,nc_lo,nc_hi", [(12, 16, 0.0, -5.0, 3000, 8192),
                                                               (47, 155, 1.0, 2.0, 8193, 10 ** 6)])
def test_gpu_keypoints_dense_candidates(ctx, orc, torch_cuda, Hc, Wc, p_corner, dustbin, nc_lo, nc_hi):
    """dense candidate fields: a third of the pixels above threshold (most candidates have
    more than 8 higher-priority neighbours: the window rescans, many rounds) within the 8192
    candidates the NMS keeps in LDS, and more than 8192 (the global per-pixel path)."""
    s_, d_ = synth.synth_superpoint_outputs(7, Hc, Wc, p_corner=p_corner, dustbin=dustbin)
    H, W = Hc * 8, Wc * 8
    pts, d, heat = orc.keypoints(s_, d_, H, W)
    assert nc_lo <= int((heat >= 0.015).sum()) <= nc_hi  # the path this case is for
    n, kp, conf, dd, st = _gpu_batch(ctx, torch_cuda, [(s_, d_)], H, W, 8192)
    k = pts.shape[0]
    assert n[0] == k and st[0] == 0
    assert (kp[0, :k] == pts[:, :2]).all() and (conf[0, :k].view(np.int32) == pts[:, 2].view(np.int32)).all()
    assert (dd[0, :k].view(np.int32) == d.view(np.int32)).all()


@pytest.mark.gpu
def test_gpu_keypoints_feed_allpairs(ctx, orc, torch_cuda):
    """image pair -> keypoints -> all-pairs match on the device, end to end against the oracle."""
    torch = torch_cuda
    s0, d0 = synth.synth_superpoint_outputs(41, 47, 155)
    s1, d1 = s0.copy(), d0.copy()
    s1[:, :, 1:], d1[:, :, 1:] = s0[:, :, :-1], d0[:, :, :-1]  # frame 1: shifted one cell right
    n, kp, conf, dd, st = _gpu_batch(ctx, torch, [(s0, d0), (s1, d1)], 376, 1241, 1024)
    dev = torch.device("cuda:0")
    D0 = torch.from_numpy(dd[0:1].copy()).to(dev)
    D1 = torch.from_numpy(dd[1:2].copy()).to(dev)
    n0 = torch.tensor(n[0:1], dtype=torch.int32, device=dev)
    n1 = torch.tensor(n[1:2], dtype=torch.int32, device=dev)
    idx = torch.zeros((1, 1024), dtype=torch.int32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.match_allpairs_f32(D0, D1, n0, n1, idx, None, 0.8)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    i2, _ = orc.allpairs_f32(dd[0, :n[0]], dd[1, :n[1]], 0.8)
    assert (idx.cpu().numpy()[0, :n[0]] == i2).all() and (i2 >= 0).sum() > 100
