"""nn_match_two_way (python/pairwise_pnp.py:281-323): mutual nearest
neighbours under sqrt(2 - 2 clip(dot)).

CPU: the oracle equals the reference's OWN nn_match_two_way (executed on the committed
pair0/pair10 descriptor fixtures and synthetic pairs, tests/golden/make_two_way_fixtures.py):
the same matches; the reference's dot is BLAS-ordered and the oracle's sequential (the
gemmini order of the all-pairs path), so the distances agree through their dots (<= 5e-7).
GPU (marked): mv_match_two_way_f32_dev equals the oracle bit for bit (indices and distances),
including ties, clipped dots (> 1), NaN columns and ragged / empty pairs."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

sys.path.insert(0, GOLDEN)
import make_two_way_fixtures as fx  # noqa: E402  (inputs() only: no reference access)


def ref_matches(name, th):
    return load_golden("two_way.npz")["%s_%g" % (name, th)]


@pytest.mark.parametrize("th", fx.THRESHOLDS)
@pytest.mark.parametrize("name", ["pair0", "pair10", "synth0", "synth1"])
def test_oracle_vs_reference_two_way(orc, name, th):
    a, b = fx.inputs()[name]
    idx, dist = orc.two_way_f32(a, b, th)
    m = ref_matches(name, th)
    rows = np.nonzero(idx >= 0)[0]
    assert (rows == m[0].astype(int)).all() and (idx[rows] == m[1].astype(int)).all()
    # the distance amplifies the dot's BLAS-vs-sequential ulps near dot = 1: compare the dots
    # behind them, 1 - dist^2 / 2 (the two orders differ by <= 1.8e-7)
    dot_o = 1.0 - dist[rows].astype(np.float64) ** 2 / 2
    dot_r = 1.0 - m[2] ** 2 / 2
    assert rows.size == 0 or np.abs(dot_o - dot_r).max() <= 5e-7


def test_oracle_two_way_edges(orc):
    rng = np.random.default_rng(0)
    a = rng.standard_normal((20, 256)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    assert orc.two_way_f32(a, a[:0], 0.7)[0].tolist() == [-1] * 20
    idx, dist = orc.two_way_f32(a, a, 0.7)  # self match: every row its own neighbour
    assert (idx == np.arange(20)).all()
    with pytest.raises(AssertionError):
        orc.two_way_f32(a, a, -0.1)


def _gpu(ctx, torch, pairs, th, cap=None, dist=True):
    B = len(pairs)
    cap = cap or max(max(x.shape[0], y.shape[0]) for x, y in pairs)
    D0 = np.zeros((B, cap, 256), np.float32)
    D1 = np.zeros((B, cap, 256), np.float32)
    n0 = np.array([x.shape[0] for x, _ in pairs], np.int32)
    n1 = np.array([y.shape[0] for _, y in pairs], np.int32)
    for k, (x, y) in enumerate(pairs):
        D0[k, :x.shape[0]] = x
        D1[k, :y.shape[0]] = y
    dev = torch.device("cuda:0")
    t = lambda v: torch.from_numpy(v).to(dev)  # noqa: E731
    idx = torch.full((B, cap), -7, dtype=torch.int32, device=dev)
    dd = torch.zeros((B, cap), dtype=torch.float32, device=dev) if dist else None
    ctx.set_stream(torch.cuda.current_stream())
    ctx.match_two_way_f32(t(D0), t(D1), t(n0), t(n1), idx, dd, th)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    return idx.cpu().numpy(), (dd.cpu().numpy() if dist else None)


@pytest.mark.gpu
@pytest.mark.parametrize("th", fx.THRESHOLDS)
def test_gpu_two_way_fixtures(ctx, screen, orc, torch_cuda, th):
    inp = fx.inputs()
    names = ["pair0", "pair10", "synth0", "synth1"]
    for dist in (True, False):
        idx, dd = _gpu(ctx, torch_cuda, [inp[n] for n in names], th, dist=dist)
        for k, n in enumerate(names):
            a, b = inp[n]
            i2, d2 = orc.two_way_f32(a, b, th)
            assert (idx[k, :a.shape[0]] == i2).all(), (n, dist)
            if dist:
                assert (dd[k, :a.shape[0]].view(np.int32) == d2.view(np.int32)).all(), n
            m = ref_matches(n, th)  # and the reference's own output
            assert (np.nonzero(i2 >= 0)[0] == m[0].astype(int)).all()


@pytest.mark.gpu
def test_gpu_two_way_hard_cases(ctx, screen, orc, torch_cuda):
    """duplicated columns and rows (distance ties: first index wins both ways), dots above 1
    (clipped: distance 0 ties), a NaN column (flagged pair: np.argmin picks the first NaN),
    ragged and empty pairs, a 1024 x 1024 full-size pair."""
    import synth

    rng = np.random.default_rng(9)
    a = rng.standard_normal((200, 256)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = a[rng.permutation(200)] + 0.02 * rng.standard_normal((200, 256)).astype(np.float32)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    dup = np.concatenate([b, b[:30], (b[30:40] * np.float32(1 + 2 ** -22)).astype(np.float32)])
    adup = np.concatenate([a, a[:20]])
    nanb = dup.copy()
    nanb[5, 7] = np.nan
    big = synth.synth_pair_f32(77)
    pairs = [(adup, dup), (a, nanb), (a[:1], b[:3]), (a[:0], b), (a, b[:0]), (a[:37], b[:301]),
             (big["desc0"], big["desc1"])]
    for th in (0.7, 2.0, 0.0):
        idx, dd = _gpu(ctx, torch_cuda, pairs, th, cap=1024)
        for k, (x, y) in enumerate(pairs):
            if x.shape[0] == 0:
                continue
            i2, d2 = orc.two_way_f32(x, y, th)
            assert (idx[k, :x.shape[0]] == i2).all(), (th, k)
            assert (dd[k, :x.shape[0]].view(np.int32) == d2.view(np.int32)).all(), (th, k)
            assert (idx[k, x.shape[0]:] == -1).all()


@pytest.mark.gpu
def test_gpu_two_way_clipped_far_above_one(ctx, screen, orc, torch_cuda):
    """Unnormalised descriptors whose dots exceed 1 by far more than the screen window: every
    such column clips to distance 0, so np.argmin takes the FIRST of them, not the largest dot."""
    rng = np.random.default_rng(12)
    a = rng.standard_normal((120, 256)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = np.concatenate([a[rng.permutation(120)] * np.float32(1.3), a[:60] * np.float32(1.7),
                        a[60:] * np.float32(0.999)]).astype(np.float32)
    b = b[rng.permutation(b.shape[0])]
    for th in (0.7, 2.0):
        idx, dd = _gpu(ctx, torch_cuda, [(a, b), (b[:100], a)], th, cap=256)
        for k, (x, y) in enumerate([(a, b), (b[:100], a)]):
            i2, d2 = orc.two_way_f32(x, y, th)
            assert (idx[k, :x.shape[0]] == i2).all(), (th, k)
            assert (dd[k, :x.shape[0]].view(np.int32) == d2.view(np.int32)).all(), (th, k)
