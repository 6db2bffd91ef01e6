"""GPU parity: all-pairs descriptor match (python/pairwise_pnp.py:635-659 semantics on the
gemmini_functions_cpu.h summation order) -- fp16 MFMA screen + exact fp32 re-score must give
the oracle's indices AND scores bit-for-bit; int8 MFMA path integer-exact."""
import numpy as np
import pytest

import synth
from conftest import load_golden

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def run_f32(ctx, torch, pairs, cap=None, thresh=0.8, scores=True):
    """pairs: list of (d0 [n0,256], d1 [n1,256]) float32; scores=False: indices only (the
    score output pointer is NULL -- the decision-only mode)"""
    B = len(pairs)
    cap = cap or max(max(a.shape[0], b.shape[0]) for a, b in pairs)
    D0 = np.zeros((B, cap, 256), np.float32)
    D1 = np.zeros((B, cap, 256), np.float32)
    n0 = np.zeros(B, np.int32)
    n1 = np.zeros(B, np.int32)
    rng = np.random.default_rng(0)
    for b, (a, c) in enumerate(pairs):
        D0[b] = rng.standard_normal((cap, 256)).astype(np.float32) * 7  # garbage beyond n must not matter
        D1[b] = rng.standard_normal((cap, 256)).astype(np.float32) * 7
        D0[b, :a.shape[0]] = a
        D1[b, :c.shape[0]] = c
        n0[b], n1[b] = a.shape[0], c.shape[0]
    dev = torch.device("cuda:0")
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    idx = torch.full((B, cap), -7, dtype=torch.int32, device=dev)
    sc = torch.zeros((B, cap), dtype=torch.float32, device=dev) if scores else None
    ctx.set_stream(torch.cuda.current_stream())
    ctx.match_allpairs_f32(t(D0), t(D1), t(n0), t(n1), idx, sc, thresh)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    return idx.cpu().numpy(), (sc.cpu().numpy() if scores else None)


@pytest.mark.parametrize("name", ["pair0", "pair10"])
def test_allpairs_f32_reference_fixtures(ctx, screen, orc, torch_cuda, name):
    d = load_golden("tracking_%s.npz" % name)
    exp = load_golden("expected_outputs.npz")
    idx, sc = run_f32(ctx, torch_cuda, [(d["image0_desc"], d["image1_desc"])])
    n0 = d["image0_desc"].shape[0]
    assert (idx[0, :n0] == exp["ap_%s_idx" % name]).all()
    assert (bits(sc[0, :n0]) == bits(exp["ap_%s_score" % name])).all()
    assert (idx[0, n0:] == -1).all()


def test_allpairs_f32_full_size_synthetic(ctx, screen, orc, torch_cuda):
    """BASELINE config 2: 1024 x 1024 x 256 fp32, checked against the oracle on 2 pairs."""
    pairs = []
    for s in range(2):
        p = synth.synth_pair_f32(s)
        pairs.append((p["desc0"], p["desc1"]))
    idx, sc = run_f32(ctx, torch_cuda, pairs)
    for b, (a, c) in enumerate(pairs):
        i2, s2 = orc.allpairs_f32(a, c, 0.8)
        assert (idx[b] == i2).all() and (bits(sc[b]) == bits(s2)).all()
        assert (i2 >= 0).sum() > 500


def test_allpairs_f32_ragged_batch(ctx, screen, orc, torch_cuda):
    rng = np.random.default_rng(4)
    shapes = [(1, 1), (1, 300), (129, 1), (127, 129), (300, 257), (0, 40), (40, 0), (511, 513), (128, 128)]
    pairs = []
    for k, (a, b) in enumerate(shapes):
        p = synth.synth_pair_f32(50 + k, n=max(a, 1), n1=max(b, 1), noise=0.25)
        pairs.append((p["desc0"][:a], p["desc1"][:b]))
    idx, sc = run_f32(ctx, torch_cuda, pairs, cap=640)
    for b, (a, c) in enumerate(pairs):
        if a.shape[0] == 0:
            continue
        if c.shape[0] == 0:
            assert (idx[b, :a.shape[0]] == -1).all()
            continue
        i2, s2 = orc.allpairs_f32(a, c, 0.8)
        assert (idx[b, :a.shape[0]] == i2).all() and (bits(sc[b, :a.shape[0]]) == bits(s2)).all()


def test_allpairs_f32_ties_and_near_ties(ctx, screen, orc, torch_cuda):
    """duplicate and rounding-level-perturbed columns force the exact re-score / ambiguous-tile path."""
    rng = np.random.default_rng(8)
    a = rng.standard_normal((300, 256)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = a[rng.permutation(300)].copy()
    b += 0.01 * rng.standard_normal(b.shape).astype(np.float32)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    b = np.concatenate([b, b[:40], b[:40] * np.float32(1 + 2 ** -23), b[50:60] * np.float32(1 - 2 ** -24)])
    b[400:410] = b[5]  # many identical columns in one tile and across tiles
    b = b[rng.permutation(b.shape[0])]
    idx, sc = run_f32(ctx, torch_cuda, [(a, b)])
    i2, s2 = orc.allpairs_f32(a, b, 0.8)
    assert (idx[0, :300] == i2).all() and (bits(sc[0, :300]) == bits(s2)).all()


def test_allpairs_f32_threshold_edges(ctx, screen, orc, torch_cuda):
    rng = np.random.default_rng(2)
    a = rng.standard_normal((64, 256)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = a.copy()
    for thr in (0.8, 0.999999, 1.0, -1.0, 0.0):
        idx, sc = run_f32(ctx, torch_cuda, [(a, b)], thresh=thr)
        i2, s2 = orc.allpairs_f32(a, b, thr)
        assert (idx[0, :64] == i2).all() and (bits(sc[0, :64]) == bits(s2)).all()


def test_allpairs_f32_out_of_screen_range(ctx, screen, orc, torch_cuda):
    """The fp16 screen only takes |x| < 2: unnormalised, huge, tiny, NaN and mixed-scale
    descriptors must still give the reference's answer (flagged pairs / wide windows route
    rows through the exact re-score)."""
    rng = np.random.default_rng(11)
    pairs = []
    for scale0, scale1 in ((5.0, 1.0), (1.0, 3e4), (1e-6, 1.0), (1e-20, 1e-20), (1.0, 1.0)):
        a = rng.standard_normal((96, 256)).astype(np.float32)
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        b = a[rng.permutation(96)][:80] + 0.05 * rng.standard_normal((80, 256)).astype(np.float32)
        b /= np.linalg.norm(b, axis=1, keepdims=True)
        pairs.append(((a * np.float32(scale0)).astype(np.float32), (b * np.float32(scale1)).astype(np.float32)))
    a, b = pairs[-1]
    b = b.copy()
    b[7, 3] = np.nan  # a NaN column: never the maximiser in the reference's comparisons
    b[9, :] *= np.float32(2.5)  # one column outside the fp16 range flags the whole pair
    pairs[-1] = (a, b)
    for thr in (0.8, 0.0):
        idx, sc = run_f32(ctx, torch_cuda, pairs, thresh=thr)
        for k, (a, b) in enumerate(pairs):
            i2, s2 = orc.allpairs_f32(a, b, thr)
            assert (idx[k, :a.shape[0]] == i2).all(), k
            assert (bits(sc[k, :a.shape[0]]) == bits(s2)).all(), k


def test_allpairs_f32_indices_only(ctx, screen, orc, torch_cuda):
    """match_score = NULL (what pairwise_pnp.py:639-659 keeps: the matched pairs, not the
    score): the exact re-score is skipped where the window already decides, and the indices
    must still equal the oracle's on every hard case -- full size, ties and near-ties,
    threshold edges, out-of-range and ragged inputs."""
    rng = np.random.default_rng(21)
    cases = []
    cases.append(([(p["desc0"], p["desc1"]) for p in (synth.synth_pair_f32(s) for s in range(2))], 0.8))
    a = rng.standard_normal((300, 256)).astype(np.float32)
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = a[rng.permutation(300)] + 0.01 * rng.standard_normal((300, 256)).astype(np.float32)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    b = np.concatenate([b, b[:40], b[:40] * np.float32(1 + 2 ** -23), b[50:60] * np.float32(1 - 2 ** -24)])
    b = b[rng.permutation(b.shape[0])]
    for thr in (0.8, 0.999999, 1.0, -1.0, 0.0):
        cases.append(([(a, b), (a[:64], a[:64].copy())], thr))
    odd = []
    for scale0, scale1 in ((5.0, 1.0), (1.0, 3e4), (1e-6, 1.0), (1e-20, 1e-20)):
        odd.append(((a[:96] * np.float32(scale0)).astype(np.float32), (b[:80] * np.float32(scale1)).astype(np.float32)))
    for k, (x, y) in enumerate([(1, 300), (129, 1), (127, 129), (511, 513)]):
        p = synth.synth_pair_f32(70 + k, n=x, n1=y, noise=0.25)
        odd.append((p["desc0"], p["desc1"]))
    cases.append((odd, 0.8))
    for pairs, thr in cases:
        idx, _ = run_f32(ctx, torch_cuda, pairs, thresh=thr, scores=False)
        idx_s, _ = run_f32(ctx, torch_cuda, pairs, thresh=thr, scores=True)
        for k, (x, y) in enumerate(pairs):
            i2, _ = orc.allpairs_f32(x, y, thr)
            assert (idx[k, :x.shape[0]] == i2).all(), (thr, k)
            assert (idx[k, :x.shape[0]] == idx_s[k, :x.shape[0]]).all(), (thr, k)
            assert (idx[k, x.shape[0]:] == -1).all()


def test_allpairs_f32_prepare_run_pipeline(ctx, screen, orc, torch_cuda):
    """prepare(next) issued between run(this) and the next run: identical to the one-call API;
    run without its prepare is refused."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    batches = []
    for s in range(3):
        p = synth.synth_pair_f32(70 + s, n=300, n1=280)
        batches.append((torch.from_numpy(p["desc0"][None].copy()).to(dev),
                        torch.from_numpy(np.ascontiguousarray(np.pad(p["desc1"], ((0, 20), (0, 0))))[None]).to(dev)))
    n0 = torch.tensor([300], dtype=torch.int32, device=dev)
    n1 = torch.tensor([280], dtype=torch.int32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    outs = []
    ctx.match_allpairs_f32_prepare(batches[0][1], n1)
    for k, (a, b) in enumerate(batches):
        idx = torch.full((1, 300), -7, dtype=torch.int32, device=dev)
        sc = torch.zeros((1, 300), dtype=torch.float32, device=dev)
        ctx.match_allpairs_f32_run(a, b, n0, n1, idx, sc, 0.8)
        if k + 1 < len(batches):
            ctx.match_allpairs_f32_prepare(batches[k + 1][1], n1)
        outs.append((idx, sc))
    torch.cuda.synchronize()
    for (a, b), (idx, sc) in zip(batches, outs):
        i2, s2 = orc.allpairs_f32(a[0].cpu().numpy(), b[0, :280].cpu().numpy(), 0.8)
        assert (idx[0].cpu().numpy() == i2).all()
        assert (bits(sc[0].cpu().numpy()) == bits(s2)).all()
    import mvtrack
    with pytest.raises(RuntimeError):  # batches[0] is not the staged batch any more
        ctx.match_allpairs_f32_run(batches[0][0], batches[0][1], n0, n1, outs[0][0], outs[0][1], 0.8)
    assert mvtrack.lib().mv_last_status() == mvtrack.MV_ERR_INVALID_ARG
    ctx.set_stream(None)


def run_i8(ctx, torch, pairs, cap=None, decoys=False):
    B = len(pairs)
    cap = cap or max(max(a.shape[0], b.shape[0]) for a, b in pairs)
    D0 = np.zeros((B, cap, 256), np.int8)
    D1 = np.zeros((B, cap, 256), np.int8)
    n0 = np.zeros(B, np.int32)
    n1 = np.zeros(B, np.int32)
    for b, (a, c) in enumerate(pairs):
        D0[b, :a.shape[0]] = a
        D1[b, :c.shape[0]] = c
        if decoys:  # slots past n1 repeat the queries: they must never be matched
            D1[b, c.shape[0]:] = np.resize(a, (cap - c.shape[0], 256))
        n0[b], n1[b] = a.shape[0], c.shape[0]
    dev = torch.device("cuda:0")
    t = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    idx = torch.full((B, cap), -7, dtype=torch.int32, device=dev)
    dot = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.match_allpairs_i8(t(D0), t(D1), t(n0), t(n1), idx, dot)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    return idx.cpu().numpy(), dot.cpu().numpy()


def test_allpairs_i8_full_size(ctx, orc, torch_cuda):
    """BASELINE config 5: 2048 kp x 256 int8 per frame."""
    a, b = synth.synth_pair_i8(0)
    idx, dot = run_i8(ctx, torch_cuda, [(a, b)])
    i2, d2 = orc.allpairs_i8(a, b)
    assert (idx[0] == i2).all() and (dot[0] == d2).all()
    assert (i2 >= 0).sum() > 1000


def test_allpairs_i8_ragged_and_degenerate(ctx, orc, torch_cuda):
    rng = np.random.default_rng(6)
    pairs = []
    for k, (na, nb) in enumerate([(1, 1), (130, 257), (300, 129), (7, 1000)]):
        a, b = synth.synth_pair_i8(10 + k, n=max(na, nb))
        a, b = a[:na].copy(), b[:nb].copy()
        if k == 1:
            a[3] = 0  # zero query
            b[:20] = b[20]  # duplicated columns: first index must win
        if k == 3:
            b[5] = a[2] * 2 // 2
        pairs.append((a, b))
    idx, dot = run_i8(ctx, torch_cuda, pairs, cap=1024)
    for b, (a, c) in enumerate(pairs):
        i2, d2 = orc.allpairs_i8(a, c)
        assert (idx[b, :a.shape[0]] == i2).all() and (dot[b, :a.shape[0]] == d2).all()


def test_allpairs_i8_ties_and_near_ties(ctx, orc, torch_cuda):
    """Columns with equal or nearly equal dot^2/|b|^2 take the exact re-score:
    b and b/2 tie exactly (first index wins), b and b + e_k differ in the 5th digit;
    rows whose every dot is <= 0 never match; slots past n1 hold strong decoys."""
    pairs = []
    for k, (na, nb) in enumerate([(200, 300), (129, 65), (64, 1000)]):
        a, b = synth.synth_pair_i8(40 + k, n=max(na, nb))
        a, b = a[:na].copy(), b[:nb].copy()
        m = nb // 4
        b[:m] = (b[:m] // 2) * 2
        b[nb // 2: nb // 2 + m] = b[:m] // 2          # exact ties with earlier columns
        for j in range(m, min(m + 40, nb // 2 - 1), 2):  # near ties
            b[j + 1] = b[j]
            b[j + 1, j % 256] = np.clip(int(b[j, j % 256]) + 1, -127, 127)
        if nb > 3 * 64:  # exact duplicates one tile apart: two candidates in one lane
            b[m + 64: m + 80] = b[m: m + 16]
        a[5] = 0
        a[5, 0] = -1
        b[:, 0] = np.abs(b[:, 0]) + 1                 # row 5: every dot < 0
        pairs.append((a, b))
    idx, dot = run_i8(ctx, torch_cuda, pairs, cap=1000, decoys=True)
    for q, (a, c) in enumerate(pairs):
        i2, d2 = orc.allpairs_i8(a, c)
        assert (idx[q, :a.shape[0]] == i2).all() and (dot[q, :a.shape[0]] == d2).all()
        assert i2[5] == -1 and (i2 >= 0).sum() > a.shape[0] // 8


def test_allpairs_i8_key_window(ctx, orc, torch_cuda):
    """k_i8_match's integer keys (unit-norm re-quantised frame 1, window (8 + 1.3e-4) |a| in
    127-units): queries re-observed with noise that puts their cosines around the 0.9
    threshold, spiky columns (one component carries the norm: codes +-127), columns that are
    scaled copies of others (equal cosines, first index wins), and frame-1 lengths that leave a
    partial last tile (zero-code padding columns)."""
    rng = np.random.default_rng(77)
    pairs = []
    for na, nb in ((700, 650), (333, 1027)):
        b = np.clip(np.round(rng.standard_normal((nb, 256)) * 24), -128, 127)
        sp = rng.choice(nb, nb // 8, replace=False)
        b[sp] = np.round(b[sp] * 0.1)
        b[sp, rng.integers(0, 256, sp.size)] = rng.choice([-127, 127], sp.size)
        half = rng.choice(nb, nb // 10, replace=False)
        b[half[1:]] = np.round(b[half[:-1]] / 2) * 1  # near copies at half scale
        src = rng.integers(0, nb, na)
        sig = rng.uniform(8.0, 15.0, na)[:, None]
        a = np.clip(np.round(b[src] + rng.standard_normal((na, 256)) * sig), -128, 127)
        pairs.append((a.astype(np.int8), b.astype(np.int8)))
    idx, dot = run_i8(ctx, torch_cuda, pairs, cap=1100, decoys=True)
    for q, (a, c) in enumerate(pairs):
        i2, d2 = orc.allpairs_i8(a, c)
        assert (idx[q, :a.shape[0]] == i2).all() and (dot[q, :a.shape[0]] == d2).all(), q
        assert 0 < (i2 >= 0).sum() < a.shape[0]


@pytest.mark.parametrize("n1,cap", [(8000, 8192), (8300, 8300)])
def test_allpairs_i8_long_frame1(ctx, orc, torch_cuda, n1, cap):
    """8192 columns: the widest integer-key tags (2 ntc = 256, tb = 8); past that the float
    screen (k_i8_match<false>, wider tags)."""
    a, b = synth.synth_pair_i8(90, n=n1)
    a = a[:96].copy()
    idx, dot = run_i8(ctx, torch_cuda, [(a, b)], cap=cap)
    i2, d2 = orc.allpairs_i8(a, b)
    assert (idx[0, :96] == i2).all() and (dot[0, :96] == d2).all()


def test_allpairs_f32_quantisation_stress(ctx, screen, orc, torch_cuda):
    """Inputs aimed at the int8 screen's window (k_allpairs_q8.hip): rows of every scale up to
    the 2^+-40 range limits and past them (exact path), spiky rows (one component carries the
    norm: the rest quantise to 0), sparse and zero rows on both sides, anti-correlated rows
    (every dot negative), and near-ties closer than one quantisation step."""
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
    sparse[80:84] = 0.0  # zero query rows
    bz = b.copy()
    bz[10:14] = 0.0  # zero columns
    near = a.copy()
    near2 = np.concatenate([a, a + np.float32(1e-4) * unit(n)]).astype(np.float32)  # near-ties per row
    pairs = [(a_s, b), (a, b_s), (spiky, b), (sparse, bz), (-a, b), (near, near2),
             (a, np.concatenate([b, -b]))]
    for thr in (0.8, 0.0, -1.0):
        for scores in (True, False):
            idx, sc = run_f32(ctx, torch_cuda, pairs, thresh=thr, scores=scores)
            for k, (x, y) in enumerate(pairs):
                i2, s2 = orc.allpairs_f32(x, y, thr)
                assert (idx[k, :x.shape[0]] == i2).all(), (thr, k)
                if scores:
                    assert (bits(sc[k, :x.shape[0]]) == bits(s2)).all(), (thr, k)


def test_allpairs_f32_column_windows(ctx, screen, orc, torch_cuda):
    """The one-pass screen decides each row on the window of its maximiser's own column (1 / q_j
    of that column, k_allpairs_direct.hip D_COLWIN) instead of the pair's widest: frame-1 columns
    of all three integer-key exponents (plain unit rows: e = 2; one component at 0.35 / 0.7 of
    the norm: e = 1 / 0), queries re-observing them with cosines that straddle the threshold, so
    that both sides of every window and the competitor bound (M - dp_I - dp) are exercised."""
    rng = np.random.default_rng(47)

    def frame1(n1):
        b = rng.standard_normal((n1, 256)).astype(np.float32)
        for j, v in zip(rng.choice(n1, 2 * n1 // 5, replace=False), [0.35, 0.7] * n1):
            c = rng.integers(256)
            b[j, c] = 0.0
            b[j] *= np.float32(np.sqrt(1.0 - v * v)) / np.linalg.norm(b[j])
            b[j, c] = np.float32(v) * rng.choice([-1.0, 1.0])
        b[:, :] /= np.linalg.norm(b, axis=1, keepdims=True)
        return b.astype(np.float32)

    pairs = []
    for n0, n1 in ((700, 600), (300, 1000)):
        b = frame1(n1)
        src = rng.integers(0, n1, n0)
        sig = rng.uniform(0.03, 0.065, n0).astype(np.float32)[:, None]
        a = b[src] + sig * rng.standard_normal((n0, 256)).astype(np.float32)
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        pairs.append((a.astype(np.float32), b))
    for thr in (0.8, 0.76, 0.83):
        for scores in (False, True):
            idx, sc = run_f32(ctx, torch_cuda, pairs, thresh=thr, scores=scores)
            for k, (x, y) in enumerate(pairs):
                i2, s2 = orc.allpairs_f32(x, y, thr)
                assert (idx[k, :x.shape[0]] == i2).all(), (thr, k, int((idx[k, :x.shape[0]] != i2).sum()))
                if scores:
                    assert (bits(sc[k, :x.shape[0]]) == bits(s2)).all(), (thr, k)


def _batch_f32(torch, pairs, cap):
    B = len(pairs)
    D0 = np.zeros((B, cap, 256), np.float32)
    D1 = np.zeros((B, cap, 256), np.float32)
    n0 = np.zeros(B, np.int32)
    n1 = np.zeros(B, np.int32)
    rng = np.random.default_rng(B)
    for b, (a, c) in enumerate(pairs):
        D0[b] = rng.standard_normal((cap, 256)).astype(np.float32) * 7
        D1[b] = rng.standard_normal((cap, 256)).astype(np.float32) * 7
        D0[b, :a.shape[0]] = a
        D1[b, :c.shape[0]] = c
        n0[b], n1[b] = a.shape[0], c.shape[0]
    dev = torch.device("cuda:0")
    return [torch.from_numpy(x).to(dev) for x in (D0, D1, n0, n1)]


def test_allpairs_f32_run_prepare_chain(ctx, screen, orc, torch_cuda):
    """mv_match_allpairs_f32_run_prepare_dev: batch k is matched while batch k+1's frame 1 is
    staged in the same launch (int8 screen) or right after (fp16); a chain of batches with
    different sizes, ragged / empty / flagged pairs, scores and indices-only, must equal the
    oracle batch by batch."""
    torch = torch_cuda
    rng = np.random.default_rng(91)
    batches = []
    for k, (B, cap) in enumerate(((3, 640), (5, 300), (2, 1024), (4, 512))):
        pairs = []
        for q in range(B):
            a = int(rng.integers(0, cap + 1))
            b = int(rng.integers(0, cap + 1))
            p = synth.synth_pair_f32(700 + 10 * k + q, n=max(a, 1), n1=max(b, 1), noise=0.25)
            pairs.append((p["desc0"][:a], p["desc1"][:b]))
        if k == 1:
            x, y = pairs[2]
            if y.shape[0] > 3:
                y = y.copy()
                y[3, 0] = np.inf  # a flagged pair
                pairs[2] = (x, y)
        batches.append((pairs, cap, _batch_f32(torch, pairs, cap)))
    ctx.set_stream(torch.cuda.current_stream())
    try:
        _, _, (D0, D1, N0, N1) = batches[0]
        ctx.match_allpairs_f32_prepare(D1, N1)
        for k, (pairs, cap, (D0, D1, N0, N1)) in enumerate(batches):
            scores = k % 2 == 0
            idx = torch.full((len(pairs), cap), -7, dtype=torch.int32, device=D0.device)
            sc = torch.zeros((len(pairs), cap), dtype=torch.float32, device=D0.device) if scores else None
            if k + 1 < len(batches):
                _, _, (_, nD1, _, nN1) = batches[k + 1]
                ctx.match_allpairs_f32_run_prepare(D0, D1, N0, N1, idx, sc, nD1, nN1)
            else:
                ctx.match_allpairs_f32_run(D0, D1, N0, N1, idx, sc, 0.8)
            torch.cuda.synchronize()
            idx = idx.cpu().numpy()
            sc = sc.cpu().numpy() if scores else None
            for q, (a, c) in enumerate(pairs):
                n0 = a.shape[0]
                assert (idx[q, n0:] == -1).all(), (k, q)
                if n0 == 0:
                    continue
                if c.shape[0] == 0:
                    assert (idx[q, :n0] == -1).all(), (k, q)
                    continue
                i2, s2 = orc.allpairs_f32(a, c, 0.8)
                assert (idx[q, :n0] == i2).all(), (k, q)
                if scores:
                    assert (bits(sc[q, :n0]) == bits(s2)).all(), (k, q)
        # the chain leaves the last batch prepared; a mismatched run is refused
        with pytest.raises(RuntimeError):
            _, cap, (D0, D1, N0, N1) = batches[0]
            ctx.match_allpairs_f32_run(D0, D1, N0, N1, torch.empty((3, cap), dtype=torch.int32, device=D0.device),
                                       None, 0.8)
    finally:
        ctx.set_stream(None)


def test_allpairs_screen_selection(ctx):
    import mvtrack

    c = mvtrack.Context(0)
    assert c.allpairs_screen() == "i8"  # the default
    c.set_allpairs_screen("f16")
    assert c.allpairs_screen() == "f16"
    c.set_allpairs_screen("i8s")
    assert c.allpairs_screen() == "i8s"
    with pytest.raises(RuntimeError):
        mvtrack.check(mvtrack.lib().mv_context_set_allpairs_screen(c.h, 7), "bad screen")
    c.close()


def test_prepare_then_one_shot_calls(ctx, screen, orc, torch_cuda):
    """a prepare of batch A still staging on the auxiliary stream must not race the
    one-shot match / two-way of batch B that follow on the context stream (they wait for it)."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    B, n = 64, 512
    pa = [synth.synth_pair_f32(900 + k, n=n) for k in range(B)]
    pb = [synth.synth_pair_f32(950 + k, n=n) for k in range(2)]
    A1 = t(np.stack([p["desc1"] for p in pa]))
    NA = t(np.full(B, n, np.int32))
    D0 = t(np.stack([p["desc0"] for p in pb]))
    D1 = t(np.stack([p["desc1"] for p in pb]))
    N2 = t(np.full(2, n, np.int32))
    idx = torch.full((2, n), -7, dtype=torch.int32, device=dev)
    dist = torch.zeros((2, n), dtype=torch.float32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        for _ in range(3):
            ctx.match_allpairs_f32_prepare(A1, NA)  # a large staging in flight ...
            ctx.match_allpairs_f32(D0, D1, N2, N2, idx, None, 0.8)  # ... then a one-shot batch
            torch.cuda.synchronize()
            for k, p in enumerate(pb):
                i2, _ = orc.allpairs_f32(p["desc0"], p["desc1"], 0.8)
                assert (idx[k].cpu().numpy() == i2).all(), k
            ctx.match_allpairs_f32_prepare(A1, NA)
            ctx.match_two_way_f32(D0, D1, N2, N2, idx, dist, 0.7)
            torch.cuda.synchronize()
            for k, p in enumerate(pb):
                i2, _ = orc.two_way_f32(p["desc0"], p["desc1"], 0.7)
                assert (idx[k].cpu().numpy() == i2).all(), k
    finally:
        ctx.set_stream(None)


@pytest.mark.parametrize("n1", [4096, 4097, 8192, 8193])
def test_allpairs_f32_long_frame1(ctx, screen, orc, torch_cuda, n1):
    """frame 1 beyond 4096 keypoints: the one-pass kernel leaves the integer keys (7-bit tags hold
    64 column tiles, n1 <= 4096) for the float sweep with 8-bit tags, and above 8192 (128 tiles)
    widens the tags to 9 bits (k_allpairs_direct.hip:464-495); the staged screens' tag widths
    change at the same tile counts.  Indices and exact scores against the oracle, with a
    re-observed subset spread over the whole of frame 1 (so late tiles hold maximisers) plus
    duplicated columns in the first and last tiles (ties across tag groups)."""
    rng = np.random.default_rng(n1)
    n0 = 320
    p = synth.synth_pair_f32(n1, n=n0, n1=n1, noise=0.3)
    a, b = p["desc0"], p["desc1"].copy()
    b[n1 - 5:n1] = b[0:5]  # exact duplicates: the first maximum (lowest index) must win
    b[n1 - 70] = a[3]  # an exact match deep in the last tiles
    for scores in (True, False):
        idx, sc = run_f32(ctx, torch_cuda, [(a, b)], cap=n1, scores=scores)
        i2, s2 = orc.allpairs_f32(a, b, 0.8)
        assert (idx[0, :n0] == i2).all()
        if scores:
            assert (bits(sc[0, :n0]) == bits(s2)).all()
    assert (i2 >= 0).sum() > 150 and i2[3] == n1 - 70 and (i2 > n1 // 2).any()


@pytest.mark.parametrize("scores", [True, False])
def test_allpairs_f32_full_size_survey_c1_noise(ctx, screen, orc, torch_cuda, scores):
    """SURVEY 8(d) C1 at full size: 1024 x 1024, the re-observed 60 % with sigma = 0.05 PER
    COMPONENT (noise norm ~0.8, renormalised): re-observed cosines ~0.78 straddle the 0.8
    threshold, so most rows take the exact re-score path -- indices (and scores) vs the oracle."""
    pairs = []
    for s in range(2):
        p = synth.synth_pair_f32(900 + s, noise=0.05 * 16.0)
        pairs.append((p["desc0"], p["desc1"]))
    idx, sc = run_f32(ctx, torch_cuda, pairs, scores=scores)
    for b, (a, c) in enumerate(pairs):
        i2, s2 = orc.allpairs_f32(a, c, 0.8)
        assert (idx[b] == i2).all()
        if scores:
            assert (bits(sc[b]) == bits(s2)).all()
        assert 30 < (i2 >= 0).sum() < 500  # near the threshold: a minority of the re-observed rows pass


def test_allpairs_f32_two_block_pairs(ctx, screen, orc, torch_cuda):
    """Pairs whose query rows span both 512-row workgroups of the one-pass kernel (cap 1024:
    each workgroup quantises all of frame 1 itself), mixed in one batch: 3-tile frames, partial
    last tiles, n0 just past one workgroup, pairs with only one live workgroup (n0 <= 512) or one
    column tile (n1 <= 128), a pair whose frame 1 leaves the integer keys' range (both workgroups
    must take the float sweep) and one with a NaN in rows 32 .. 63 of a late tile.  Indices and
    exact scores against the oracle, with and without scores."""
    rng = np.random.default_rng(77)
    shapes = [(513, 129), (1024, 1024), (700, 191), (600, 1000), (1000, 193), (512, 1024), (900, 128),
              (1024, 257), (777, 1024), (1024, 1023)]
    pairs = []
    for k, (x, y) in enumerate(shapes):
        p = synth.synth_pair_f32(300 + k, n=x, n1=y, noise=0.2)
        pairs.append((p["desc0"], p["desc1"].copy()))
    pairs[7][1][200, 17] = np.float32(1.5)  # outside +-1.003: the whole pair on the float sweep
    pairs[8][1][64 * 9 + 40, 5] = np.nan  # rows 32 .. 63 of tile 9: the second block's half
    for scores in (True, False):
        idx, sc = run_f32(ctx, torch_cuda, pairs, cap=1024, scores=scores)
        for k, (a, c) in enumerate(pairs):
            i2, s2 = orc.allpairs_f32(a, c, 0.8)
            n0 = a.shape[0]
            assert (idx[k, :n0] == i2).all(), (k, scores)
            assert (idx[k, n0:] == -1).all(), k
            if scores:
                assert (bits(sc[k, :n0]) == bits(s2)).all(), k
            assert (i2 >= 0).sum() > min(n0, c.shape[0]) // 4, k


@pytest.mark.parametrize("scores", [True, False])
def test_allpairs_f32_handbacks_across_the_grid(ctx, orc, torch_cuda, scores):
    """The default screen at cap <= 1024 runs k_q8t_match (one workgroup per pair); a pair outside
    its integer keys' range -- a component beyond +-1.003, |b_j|^2 > 4 with every component inside,
    a NaN -- is handed back to k_q8d_match's float path (k_q8d_handback: a grid-stride loop of at
    most 256 workgroups over the flagged row blocks).  520 pairs at cap 1024 = 1040 row blocks,
    so the loop takes more than one trip; every pair against the oracle (indices, exact scores)."""
    rng = np.random.default_rng(1234)
    B, n = 520, 64
    pairs = []
    for b in range(B):
        p = synth.synth_pair_f32(5000 + b, n=n, n1=n, noise=0.2)
        a, c = p["desc0"], p["desc1"].copy()
        if b % 7 == 3:
            c[rng.integers(n), rng.integers(256)] = np.float32(1.5)
        elif b % 11 == 5:
            c[rng.integers(n), :16] = np.float32(0.7)  # |b_j|^2 = 7.84 + ..., every component < 1.003
        elif b == 100:
            c[7, 200] = np.nan
        pairs.append((a, c))
    idx, sc = run_f32(ctx, torch_cuda, pairs, cap=1024, scores=scores)
    for b, (a, c) in enumerate(pairs):
        i2, s2 = orc.allpairs_f32(a, c, 0.8)
        assert (idx[b, :n] == i2).all(), b
        assert (idx[b, n:] == -1).all(), b
        if scores:
            assert (bits(sc[b, :n]) == bits(s2)).all(), b


@pytest.mark.parametrize("scores", [True, False])
def test_allpairs_f32_wide_rows_rescreened(ctx, screen, orc, torch_cuda, scores):
    """Clustered frame-1 columns (near-duplicates within the int8 window, as SuperPoint's own
    descriptors of repeated texture give): a query row then holds two or more in-window columns
    in one lane half of k_q8t_match -- a wide row, re-screened on the matrix cores (rescan_t) and
    its listed columns scored exactly; clusters of 40-80 members overflow the 16-column lists and
    take the full re-score.  Mixed cluster sizes, thresholds around the cluster scores, ragged
    pairs; indices (and exact scores) against the oracle."""
    rng = np.random.default_rng(4242)
    pairs = []
    for k, (n0, nc, spread) in enumerate([(400, 120, 0.02), (1024, 200, 0.01), (300, 40, 0.05), (700, 90, 0.003)]):
        cen = rng.standard_normal((nc, 256)).astype(np.float32)
        cen /= np.linalg.norm(cen, axis=1, keepdims=True)
        sizes = rng.integers(1, 12, nc)
        sizes[:3] = [40, 64, 80]  # overflowing lists
        cols = []
        for c in range(nc):
            m = cen[c] + spread * rng.standard_normal((sizes[c], 256)).astype(np.float32)
            cols.append(m / np.linalg.norm(m, axis=1, keepdims=True))
        b = np.concatenate(cols)[:1024]
        b = b[rng.permutation(b.shape[0])].astype(np.float32)
        q = cen[rng.integers(0, nc, n0)] + 0.15 * rng.standard_normal((n0, 256)).astype(np.float32) / 16
        a = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
        pairs.append((a, b))
    for thr in (0.8, 0.97):
        idx, sc = run_f32(ctx, torch_cuda, pairs, cap=1024, thresh=thr, scores=scores)
        for k, (a, c) in enumerate(pairs):
            i2, s2 = orc.allpairs_f32(a, c, thr)
            n0 = a.shape[0]
            assert (idx[k, :n0] == i2).all(), (k, thr)
            assert (idx[k, n0:] == -1).all(), k
            if scores:
                assert (bits(sc[k, :n0]) == bits(s2)).all(), (k, thr)
            if thr == 0.8:
                assert (i2 >= 0).sum() > n0 // 4, k
