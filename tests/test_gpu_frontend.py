"""GPU parity: softmax / top-N / windowed match (src/top_N.c, src/tracking_main.c:18-194)
against the oracle and the committed golden outputs.  Bit-exact (integer and float)."""
import ctypes

import numpy as np
import pytest

import synth
from conftest import load_golden

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def scales_for(orc, s):
    return {"built": orc.scale_as_built(s), "true": float(s)}


@pytest.mark.parametrize("mode", ["built", "true"])
def test_softmax_topn_image0_vs_golden(ctx, orc, image0, mode):
    exp = load_golden("expected_outputs.npz")
    s = scales_for(orc, image0["semi_scale"])[mode]
    nv, mi, pr = ctx.softmax_host(s, image0["semi"])
    assert nv == int(exp["softmax_%s_nv" % mode])
    assert (mi == exp["softmax_%s_mi" % mode]).all() and (bits(pr) == bits(exp["softmax_%s_pr" % mode])).all()
    st, pa, ix, pp = ctx.top_n_host(s, image0["semi"], 100)
    assert st == 0
    assert (pa == exp["topn_%s_patches" % mode]).all() and (ix == exp["topn_%s_indices" % mode]).all()
    assert (bits(pp) == bits(exp["topn_%s_probs" % mode])).all()


@pytest.mark.parametrize("seed", range(6))
def test_softmax_topn_random_vs_oracle(ctx, orc, seed):
    rng = np.random.default_rng(100 + seed)
    cells = [1920, 7285, 517, 64][seed % 4]
    semi = synth.synth_semi(rng, cells, p_key=[0.05, 0.2, 0.6, 0.9][seed % 4])
    for s in (0.0, 0.35622025, rng.uniform(0.01, 1.5)):
        nv, mi, pr = ctx.softmax_host(s, semi)
        nv2, mi2, pr2 = orc.compute_softmax(s, semi)
        assert nv == nv2 and (mi == mi2).all() and (bits(pr) == bits(pr2)).all()
        for N, cap in ((100, 1000), (1024, 8000), (7, 1000), (1, 100000)):
            st, pa, ix, pp = ctx.top_n_host(s, semi, N, cap)
            st2, pa2, ix2, pp2 = orc.compute_top_N(s, semi, N, cap)
            assert (st == 0) == (st2 == 0)
            if st == 0:
                assert (pa == pa2).all() and (ix == ix2).all() and (bits(pp) == bits(pp2)).all()


def test_top_n_capacity_error_matches_reference_exit(ctx, orc):
    rng = np.random.default_rng(9)
    semi = synth.synth_semi(rng, 7285, p_key=0.9)
    st2, *_ = orc.compute_top_N(0.0, semi, 100, 1000)
    st, *_ = ctx.top_n_host(0.0, semi, 100, 1000)
    assert st2 == -1 and st == -2  # MV_ERR_CAPACITY where the reference exit(1)s


def test_softmax_edge_rows(ctx, orc):
    semi = np.full((256 * 3 + 5, 65), -1, np.int8)
    semi[1, :] = 0  # all zero logits: first index wins
    semi[2, :] = 127
    semi[3, 64] = 127  # only dustbin
    semi[4, 63] = 5
    semi[5, :64] = -128
    semi[6, ::2] = 3
    for s in (0.0, 1.0, 4.0):
        nv, mi, pr = ctx.softmax_host(s, semi)
        nv2, mi2, pr2 = orc.compute_softmax(s, semi)
        assert nv == nv2 and (mi == mi2).all() and (bits(pr) == bits(pr2)).all()


def _window_case(ctx, orc, f0, f1, built, N=100, cap=1000, shift=(4, 4), radius=4, max_matches=150):
    import mvtrack

    r = orc.track_window(f0, f1, as_built=built, N=N, shift=shift, radius=radius, max_matches=max_matches, cap=cap)
    p = mvtrack.window_params(mvtrack.AS_BUILT if built else mvtrack.AS_INTENDED, shift_x=shift[0], shift_y=shift[1],
                              radius=radius, max_matches=max_matches)
    p1, p2, q = ctx.window_match_host(p, f0["rows"], f0["cols"], f0["desc"], r["max_idx0"], r["probs0"], f1["desc"],
                                      r["patches1"], r["indices1"])
    assert len(q) == len(r["query"])
    assert (q == r["query"]).all() and (p1 == r["points1"]).all() and (p2 == r["points2"]).all()
    return len(q)


@pytest.mark.parametrize("built", [True, False])
def test_window_match_golden_cases(ctx, orc, image0, built):
    exp = load_golden("expected_outputs.npz")
    cases = {"self": (image0, image0)}
    for s in (1, 2, 3):
        cases["syn%d" % s] = synth.synth_window_pair(s)
    for name, (f0, f1) in cases.items():
        n = _window_case(ctx, orc, f0, f1, built)
        tag = "win_%s_%s" % (name, "built" if built else "true")
        assert n == len(exp[tag + "_q"])


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("built", [True, False])
def test_window_match_random_windows(ctx, orc, seed, built):
    rows, cols = [(24, 80), (47, 155), (9, 13), (24, 80)][seed]
    f0, f1 = synth.synth_window_pair(200 + seed, rows=rows, cols=cols, shift=(2, 3) if seed == 3 else (4, 4))
    shift, radius = ((2, 3), 2) if seed == 3 else ((4, 4), 4)
    N = 1024 if rows * cols > 2000 else 100
    _window_case(ctx, orc, f0, f1, built, N=N, cap=100000, shift=shift, radius=radius,
                 max_matches=1024 if N == 1024 else 150)


def test_window_match_as_built_quirks(ctx, orc, image0):
    """zero descriptors before the latch (0/0 = NaN), int32 wrap, 64-dim later candidates."""
    f0 = dict(image0)
    d = image0["desc"].copy()
    d[0:40] = 0  # all-zero candidates: the latch moves past them
    d[100:140] = 127  # huge norms: n1*n2 wraps
    d[300:310] = -128
    f0["desc"] = d
    f1 = dict(image0)
    d1 = image0["desc"].copy()
    d1[200:260] = 127
    f1["desc"] = d1
    for built in (True, False):
        _window_case(ctx, orc, f0, f1, built)
        _window_case(ctx, orc, f0, f1, built, shift=(0, 0), radius=6)


def test_window_match_empty_and_cap(ctx, orc, image0):
    import mvtrack

    p = mvtrack.window_params(mvtrack.AS_BUILT)
    _, mi, pr = orc.compute_softmax(0.0, image0["semi"])
    p1, p2, q = ctx.window_match_host(p, 24, 80, image0["desc"], mi, pr, image0["desc"], np.zeros(0, np.int32),
                                      np.zeros(0, np.int32))
    assert len(q) == 0
    # cap: max_matches smaller than the number of found matches
    _window_case(ctx, orc, image0, image0, True, max_matches=17)
    _window_case(ctx, orc, image0, image0, False, max_matches=1)


def test_batched_frontend_vs_oracle(ctx, orc, torch_cuda):
    """softmax + top-N + window match for B pairs in one launch each (device pointers)."""
    import mvtrack

    torch = torch_cuda
    B, rows, cols, N = 6, 47, 155, 1024
    cells = rows * cols
    pairs = [synth.synth_window_pair(300 + b, rows=rows, cols=cols) for b in range(B)]
    dev = torch.device("cuda:0")
    semi0 = torch.from_numpy(np.stack([p[0]["semi"] for p in pairs])).to(dev)
    semi1 = torch.from_numpy(np.stack([p[1]["semi"] for p in pairs])).to(dev)
    desc0 = torch.from_numpy(np.stack([p[0]["desc"] for p in pairs])).to(dev)
    desc1 = torch.from_numpy(np.stack([p[1]["desc"] for p in pairs])).to(dev)
    for built in (True, False):
        s = [orc.scale_as_built(p[0]["semi_scale"]) if built else float(p[0]["semi_scale"]) for p in pairs]
        sc = torch.tensor(s, dtype=torch.float32, device=dev)
        mi0 = torch.empty((B, cells), dtype=torch.int32, device=dev)
        pr0 = torch.empty((B, cells), dtype=torch.float32, device=dev)
        mi1 = torch.empty_like(mi0)
        pr1 = torch.empty_like(pr0)
        nv = torch.empty(B, dtype=torch.int32, device=dev)
        ctx.set_stream(torch.cuda.current_stream())
        ctx.softmax_batch(sc, semi0, mi0, pr0, nv)
        ctx.softmax_batch(sc, semi1, mi1, pr1, nv)
        ns = torch.empty(B, dtype=torch.int32, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        pa = torch.empty((B, N), dtype=torch.int32, device=dev)
        ix = torch.empty((B, N), dtype=torch.int32, device=dev)
        sp = torch.empty((B, N), dtype=torch.float32, device=dev)
        ctx.top_n_select_batch(mi1, pr1, N, 100000, ns, pa, ix, sp, st)
        M = 1024
        nm = torch.empty(B, dtype=torch.int32, device=dev)
        p1 = torch.empty((B, M, 2), dtype=torch.float32, device=dev)
        p2 = torch.empty((B, M, 2), dtype=torch.float32, device=dev)
        qm = torch.empty((B, M), dtype=torch.int32, device=dev)
        prm = mvtrack.window_params(mvtrack.AS_BUILT if built else mvtrack.AS_INTENDED, max_matches=M)
        ctx.window_match_batch(prm, rows, cols, desc0, mi0, pr0, desc1, ns, pa, ix, nm, p1, p2, qm)
        torch.cuda.synchronize()
        ctx.set_stream(None)
        for b, (f0, f1) in enumerate(pairs):
            r = orc.track_window(f0, f1, as_built=built, N=N, cap=100000, max_matches=M)
            assert (mi0[b].cpu().numpy() == r["max_idx0"]).all()
            assert (bits(pr0[b].cpu().numpy()) == bits(r["probs0"])).all()
            n_sel = int(ns[b])
            assert n_sel == len(r["patches1"]) and (pa[b, :n_sel].cpu().numpy() == r["patches1"]).all()
            n = int(nm[b])
            assert n == len(r["query"]) and n > 0
            assert (p1[b, :n].cpu().numpy() == r["points1"]).all() and (p2[b, :n].cpu().numpy() == r["points2"]).all()


def test_dropin_symbols_match_oracle(orc, image0, ctx):
    """compute_softmax / compute_top_N with the reference signatures (default context)."""
    import mvtrack

    L = mvtrack.lib()
    semi = np.ascontiguousarray(image0["semi"])
    for s in (orc.scale_as_built(image0["semi_scale"]), float(image0["semi_scale"])):
        nv = ctypes.c_int(5)  # the reference adds to the caller's counter
        mi = np.zeros(1920, np.int32)
        pr = np.zeros(1920, np.float32)
        L.compute_softmax(s, semi.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nv),
                          mi.ctypes.data_as(ctypes.c_void_p), pr.ctypes.data_as(ctypes.c_void_p))
        nv2, mi2, pr2 = orc.compute_softmax(s, semi)
        assert nv.value == nv2 + 5 and (mi == mi2).all() and (bits(pr) == bits(pr2)).all()
        ns = ctypes.c_int(0)
        pa = np.zeros(100, np.int32)
        ix = np.zeros(100, np.int32)
        pp = np.zeros(100, np.float32)
        L.compute_top_N(s, semi.ctypes.data_as(ctypes.c_void_p), 100, ctypes.byref(ns),
                        pa.ctypes.data_as(ctypes.c_void_p), ix.ctypes.data_as(ctypes.c_void_p),
                        pp.ctypes.data_as(ctypes.c_void_p))
        st, pa2, ix2, pp2 = orc.compute_top_N(s, semi, 100)
        assert ns.value == len(pa2) and (pa[:ns.value] == pa2).all() and (bits(pp[:ns.value]) == bits(pp2)).all()


@pytest.mark.parametrize("grid,radius", [((24, 80), 4), ((47, 155), 4), ((60, 20), 7), ((24, 80), 8)])
def test_window_match_exact_ties_and_threshold(ctx, orc, grid, radius):
    """The as-intended window's float screens at their exact edges: every frame-0 cell holds an
    integer multiple of one of three directions -- v = (-3, 4, 5), whose cosine with every frame-1
    descriptor (multiples of u = (0, 1, 1)) is EXACTLY 0.9 (100 dot^2 == 81 |a|^2 |b|^2: no match,
    the test is strict), and w1 = (-3, 5, 5), w2 = (-1, 2, 2) above it -- so a window holds many
    candidates with exactly equal scores dot^2 / |b|^2 (m w and m' w tie for every m, m'), decided
    by the scan position, and threshold-equal ones (tracking_main.c:18-57; oracle/mv_oracle.c).
    Radius 4: the per-wave MFMA kernel (k_window_wave); 60 rows at radius 7: the per-query kernel
    with the column masks (k_window_query); radius 8 (17 x 17 windows): the general one (k_window_eval).  Round 5's k_window_wave failed this (38 of 99 matches on 24 x 80)."""
    rows, cols = grid
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
    N = 1024 if cells > 2000 else 100
    M = 1024 if N == 1024 else 150
    n = _window_case(ctx, orc, g0, g1, False, N=N, cap=100000, radius=radius, max_matches=M)
    assert n > 0
    _window_case(ctx, orc, g0, g1, True, N=N, cap=100000, radius=radius, max_matches=M)


@pytest.mark.parametrize("grid", [(64, 12), (1, 300), (63, 7)])
def test_window_match_grid_edges(ctx, orc, grid):
    """grids at the column-mask edges: 64 rows (a column is exactly one mask word), one row (64
    columns per ballot word), 63 rows (columns straddling ballot words) -- k_window_mask's 64
    columns per wave and the per-wave window kernel, both semantics"""
    rows, cols = grid
    f0, f1 = synth.synth_window_pair(91, rows=rows, cols=cols)
    for built in (False, True):
        _window_case(ctx, orc, f0, f1, built, N=100, cap=100000)


def test_window_match_multipass_lists(ctx, orc):
    """every frame-0 cell a candidate (one dominant logit) and frame 1's queries spread over the
    47 x 155 grid (valid cells only on every 12th column, every 8th row): a wave's 16 queries span
    ~36 columns, whose union (~44 columns x 47 rows) holds several times the 512-entry candidate
    list, so the per-wave kernel sweeps it in passes (its LDS staging ring restarting per pass);
    both semantics"""
    rows, cols = 47, 155
    f0, f1 = synth.synth_window_pair(93, rows=rows, cols=cols)
    g0, g1 = dict(f0), dict(f1)
    semi = np.full((rows * cols, 65), -128, np.int8)
    semi[:, 7] = 100
    g0["semi"] = semi
    semi1 = np.full((rows * cols, 65), -128, np.int8)
    semi1[:, 64] = 100  # the dustbin wins: not a query
    p = np.arange(rows * cols)
    on = ((p // rows) % 12 == 0) & ((p % rows) % 8 == 0)
    semi1[on, 64] = -128
    semi1[on, 9] = 100
    g1["semi"] = semi1
    r = orc.track_window(g0, g1, as_built=False, N=100, cap=100000, max_matches=150)
    assert (r["max_idx0"] != 64).all() and len(r["patches1"]) == on.sum()
    x = np.asarray(r["patches1"]) // rows
    spans = [(min(x[i + 15] + 8, cols - 1) - max(x[i], 0) + 1) * rows for i in range(0, len(x) - 15, 16)]
    assert max(spans) > 1024  # some wave's list takes three or more passes
    for built in (False, True):
        assert _window_case(ctx, orc, g0, g1, built, N=100, cap=100000, max_matches=150) > 0
