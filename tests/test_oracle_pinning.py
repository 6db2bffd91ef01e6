"""CPU: pin the oracle (oracle/mv_oracle.c) before it is trusted as the checker.

- against the reference's own code compiled from /root/reference by oracle/Makefile
  (skipped where oracle/_ref is absent, e.g. on the GPU box);
- against the reference's golden data (pair0_gt.h exact softmax; the survey's
  match counts on tracking/pair0.h and pair10.h);
- against the committed expected outputs (tests/golden/expected_outputs.npz).
"""
import ctypes

import numpy as np
import pytest

from conftest import load_golden


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


needs_ref = pytest.mark.skipif("not __import__('oracle').ref_available()", reason="oracle/_ref not built here")


def test_as_built_scale_is_zero(orc, image0):
    # the implicitly declared call passes a double; the callee reads 0.0f
    assert orc.scale_as_built(image0["semi_scale"]) == 0.0
    assert orc.scale_as_built(image0["desc_scale"]) == 0.0
    # a scale whose low 3 mantissa bits are set does not read as zero
    s = np.frombuffer(np.uint32(0x3F800007).tobytes(), np.float32)[0]
    assert orc.scale_as_built(float(s)) != 0.0


@needs_ref
@pytest.mark.parametrize("scale", ["built", "true", 0.05, 1.3, 0.0])
def test_softmax_topn_vs_reference(orc, image0, scale):
    R, P = orc.ref(), orc._ptr
    s = {"built": orc.scale_as_built(image0["semi_scale"]), "true": float(image0["semi_scale"])}.get(scale, scale)
    semi = np.ascontiguousarray(image0["semi"])
    nv = ctypes.c_int(0)
    mi = np.zeros(1920, np.int32)
    pr = np.zeros(1920, np.float32)
    R.compute_softmax(s, P(semi), ctypes.byref(nv), P(mi), P(pr))
    nv2, mi2, pr2 = orc.compute_softmax(s, semi)
    assert nv.value == nv2
    assert (mi == mi2).all() and (bits(pr) == bits(pr2)).all()
    for N in (1, 37, 100, 400):
        ns = ctypes.c_int(0)
        pa = np.zeros(N, np.int32)
        ix = np.zeros(N, np.int32)
        pp = np.zeros(N, np.float32)
        R.compute_top_N(s, P(semi), N, ctypes.byref(ns), P(pa), P(ix), P(pp))
        st, pa2, ix2, pp2 = orc.compute_top_N(s, semi, N)
        n = ns.value
        assert st == 0 and n == len(pa2)
        assert (pa[:n] == pa2).all() and (ix[:n] == ix2).all() and (bits(pp[:n]) == bits(pp2)).all()


@needs_ref
def test_softmax_topn_vs_reference_random_frames(orc):
    import synth

    R, P = orc.ref(), orc._ptr
    rng = np.random.default_rng(5)
    for seed in range(4):
        semi = np.ascontiguousarray(synth.synth_semi(rng, 1920, p_key=0.2 + 0.1 * seed))
        for s in (0.0, 0.2, 0.35622025, 0.9):
            nv = ctypes.c_int(0)
            mi = np.zeros(1920, np.int32)
            pr = np.zeros(1920, np.float32)
            R.compute_softmax(s, P(semi), ctypes.byref(nv), P(mi), P(pr))
            nv2, mi2, pr2 = orc.compute_softmax(s, semi)
            assert nv.value == nv2 and (mi == mi2).all() and (bits(pr) == bits(pr2)).all()
            ns = ctypes.c_int(0)
            pa = np.zeros(100, np.int32)
            ix = np.zeros(100, np.int32)
            pp = np.zeros(100, np.float32)
            R.compute_top_N(s, P(semi), 100, ctypes.byref(ns), P(pa), P(ix), P(pp))
            st, pa2, ix2, pp2 = orc.compute_top_N(s, semi, 100)
            assert st == 0 and ns.value == len(pa2) and (pa[:ns.value] == pa2).all()


@needs_ref
def test_svd_and_pose_vs_reference(orc):
    R, P = orc.ref(), orc._ptr
    rng = np.random.default_rng(1)
    mats = [np.eye(3), np.zeros((3, 3)), np.diag([3.0, 2.0, 1.0]), np.diag([1.0, 1.0, 0.0])]
    mats += [rng.standard_normal((3, 3)) for _ in range(500)]
    mats += [np.outer(rng.standard_normal(3), rng.standard_normal(3)) for _ in range(50)]  # rank 1
    for A in mats:
        A = np.ascontiguousarray(A, np.float32).reshape(9)
        U = np.zeros(9, np.float32)
        S = np.zeros(3, np.float32)
        V = np.zeros(9, np.float32)
        R.call_svd(P(A), P(U), P(S), P(V))
        U2, S2, V2 = orc.svd3(A)
        assert (bits(U) == bits(U2).reshape(9)).all() and (bits(S) == bits(S2)).all()
        assert (bits(V) == bits(V2).reshape(9)).all()
        R1 = np.zeros(9, np.float32)
        R2 = np.zeros(9, np.float32)
        t = np.zeros(3, np.float32)
        R.recover_pose_from_essential_matrix(P(A), P(R1), P(R2), P(t))
        a, b, c = orc.recover_pose(A)
        assert (bits(R1) == bits(a).reshape(9)).all() and (bits(R2) == bits(b).reshape(9)).all()
        assert (bits(t) == bits(c)).all()


@needs_ref
@pytest.mark.parametrize("n", [1, 8, 51, 150, 1200])
def test_ransac_vs_reference_including_rand_stream(orc, n):
    R, P = orc.ref(), orc._ptr
    libc = ctypes.CDLL("libc.so.6")
    rng = np.random.default_rng(n)
    p1 = (rng.uniform(0, 640, (n, 2))).astype(np.float32)
    p2 = (p1 + rng.normal(0, 0.8, (n, 2))).astype(np.float32)
    K = np.array([[517.306408, 0, 318.643040], [0, 516.469215, 255.313989], [0, 0, 1]], np.float32)
    for seed in (0, 7):
        libc.srand(seed)
        E = np.full(9, -5, np.float32)
        inl = np.full(max(n, 1000), -1, np.int32)
        ni = ctypes.c_int(-1)
        R.ransac_essential_matrix(n, P(p1), P(p2), P(K), 10, ctypes.c_float(1.1), P(E), P(inl), ctypes.byref(ni))
        nxt_ref = libc.rand()
        libc.srand(seed)
        st, E2, inl2, ni2 = orc.ransac_essential_matrix(p1, p2, K, 10, 1.1)
        nxt = libc.rand()
        assert st == 0 and nxt == nxt_ref
        assert ni.value == ni2  # -1: untouched when no point is an inlier
        if ni2 > 0:
            assert (inl[:ni2] == inl2).all()
            assert (bits(E) == bits(E2).reshape(9)).all()


@needs_ref
def test_gemmini_matmul_vs_reference(orc):
    R, P = orc.ref(), orc._ptr
    rng = np.random.default_rng(3)
    A = rng.standard_normal((67, 256)).astype(np.float32)
    B = rng.standard_normal((53, 256)).astype(np.float32)
    C = np.zeros((67, 53), np.float32)
    R.ref_matmul_nt(67, 53, 256, P(A), P(B), P(C))
    assert (bits(C) == bits(orc.matmul_nt(A, B))).all()


def test_softmax_argmax_vs_pair0_gt(orc, image0):
    """pair0_gt.h (superpoint_inference.py:666-711): exact softmax of frame 0."""
    g = load_golden("pair0_gt.npz")
    gi = g["image0_indices_gt"].reshape(-1)  # [80][24] -> cell gx*24 + gy
    gp = g["image0_probs_gt"].reshape(-1).astype(np.float64)
    semi = image0["semi"].astype(np.float64) * float(image0["semi_scale"])
    ex = np.exp(semi - semi.max(1, keepdims=True))
    ex /= ex.sum(1, keepdims=True)
    assert (ex[:, :64].argmax(1) == gi).all()
    assert np.abs(ex[np.arange(1920), gi] - gp).max() < 1e-5  # fixture parse is faithful
    _, mi, _ = orc.compute_softmax(float(image0["semi_scale"]), image0["semi"])
    valid = mi != 64
    assert valid.sum() == 410
    assert (mi[valid] == gi[valid]).all()  # the Taylor softmax keeps the exact argmax


def test_allpairs_oracle_is_sequential_fp32(orc):
    rng = np.random.default_rng(0)
    a = rng.standard_normal((40, 256)).astype(np.float32)
    b = rng.standard_normal((70, 256)).astype(np.float32)
    b[7] = a[3] * 1.0001
    b[9] = b[7]  # exact tie: the first j must win
    idx, sc = orc.allpairs_f32(a, b, -1e30)
    S = np.cumsum(a[:, None, :] * b[None, :, :], axis=2, dtype=np.float32)[:, :, -1]  # sequential order
    for i in range(40):
        j = int(np.argmax(S[i]))
        assert idx[i] == j and sc[i] == S[i, j]
    assert idx[3] == 7


def test_allpairs_fixture_match_counts(orc):
    exp = load_golden("expected_outputs.npz")
    for name, count in (("pair0", 319), ("pair10", 343)):
        d = load_golden("tracking_%s.npz" % name)
        idx, sc = orc.allpairs_f32(d["image0_desc"], d["image1_desc"], 0.8)
        assert int((idx >= 0).sum()) == count
        assert (idx == exp["ap_%s_idx" % name]).all() and (bits(sc) == bits(exp["ap_%s_score" % name])).all()
        # the BLAS (np.dot) order of the Python reference gives the same indices on these fixtures
        S = d["image0_desc"] @ d["image1_desc"].T
        blas = np.where(S.max(1) > 0.8, S.argmax(1), -1)
        assert (blas == idx).all()


def test_oracle_reproduces_committed_outputs(orc, image0):
    import synth

    exp = load_golden("expected_outputs.npz")
    for mode, scale in (("built", orc.scale_as_built(image0["semi_scale"])), ("true", float(image0["semi_scale"]))):
        nv, mi, pr = orc.compute_softmax(scale, image0["semi"])
        assert nv == int(exp["softmax_%s_nv" % mode]) and (mi == exp["softmax_%s_mi" % mode]).all()
        assert (bits(pr) == bits(exp["softmax_%s_pr" % mode])).all()
    cases = {"self": (image0, image0)}
    for s in (1, 2, 3):
        cases["syn%d" % s] = synth.synth_window_pair(s)
    for name, (f0, f1) in cases.items():
        for built in (True, False):
            r = orc.track_window(f0, f1, as_built=built)
            tag = "win_%s_%s" % (name, "built" if built else "true")
            assert (r["points1"] == exp[tag + "_p1"]).all() and (r["points2"] == exp[tag + "_p2"]).all()
    R1, R2, t = orc.recover_pose(np.eye(3, dtype=np.float32))
    assert (bits(R1) == bits(exp["pose_built_R1"])).all() and (bits(t) == bits(exp["pose_built_t"])).all()


def test_window_as_intended_matches_bruteforce(orc):
    import synth

    f0, f1 = synth.synth_window_pair(11, rows=12, cols=20)
    r = orc.track_window(f0, f1, as_built=False, N=40)
    d0 = f0["desc"].astype(np.int64)
    d1 = f1["desc"].astype(np.int64)
    for k, q in enumerate(r["query"]):
        patch1 = r["patches1"][q]
        x1, y1 = divmod(int(patch1), 12)
        best, bj = -1.0, None
        for x0 in range(max(x1, 0), min(x1 + 8, 19) + 1):
            for y0 in range(max(y1, 0), min(y1 + 8, 11) + 1):
                p0 = x0 * 12 + y0
                if r["max_idx0"][p0] == 64 or r["probs0"][p0] < 0.2:
                    continue
                dot = int(d0[p0] @ d1[patch1])
                na, nb = int(d0[p0] @ d0[p0]), int(d1[patch1] @ d1[patch1])
                if dot <= 0 or 100 * dot * dot <= 81 * na * nb:
                    continue
                c = dot * dot / na
                if c > best:
                    best, bj = c, (x0, y0, p0)
        x0, y0, p0 = bj
        idx = r["max_idx0"][p0]
        assert r["points1"][k, 0] == x0 * 8 + idx % 8 and r["points1"][k, 1] == y0 * 8 + idx // 8


@pytest.mark.skipif("not __import__('oracle').ref_window_available()", reason="oracle/_ref not built here")
def test_squared_dist_pinned(orc):
    """The oracle's squared_dist and window score (the arithmetic of tracking_main.c's windowed
    match) bit for bit against the reference's OWN squared_dist (:18-43) and score
    line (:154-155), extracted from its text at build time: random int8 descriptors incl. the
    extremes, per query a sequence of candidates through the latched (stale) norm1 and the 64-D
    branch, the int32 wrap of dot^2 and n1 n2 (most pairs overflow), and the threshold test."""
    R, L, P = orc.ref_window(), orc.lib(), orc._ptr
    rng = np.random.default_rng(18)
    wraps = calls = 0
    for q in range(300):
        if q % 3 == 0:
            query = rng.integers(-128, 128, 256).astype(np.int8)
        else:
            query = np.clip(np.round(rng.normal(0, 24 + q % 40, 256)), -128, 127).astype(np.int8)
        n1r = np.zeros(1, np.int32)
        n1o = np.zeros(1, np.int32)
        for c in range(int(rng.integers(1, 12))):  # the window's candidates, first one latches norm1
            cand = np.clip(np.round(query * rng.uniform(-1, 1.2) + rng.normal(0, 20, 256)), -128, 127).astype(np.int8)
            if c == 5:
                cand = np.full(256, -128, np.int8)  # extremes: 256 x 128^2 products
            sr, n2r = np.zeros(1, np.int32), np.zeros(1, np.int32)
            so, n2o = np.zeros(1, np.int32), np.zeros(1, np.int32)
            R.ref_squared_dist(P(cand), P(query), P(sr), P(n1r), P(n2r))
            L.orc_squared_dist(P(cand), P(query), P(so), P(n1o), P(n2o))
            assert (sr[0], n1r[0], n2r[0]) == (so[0], n1o[0], n2o[0]), (q, c)
            dr = R.ref_window_score(int(sr[0]), int(n1r[0]), int(n2r[0]))
            do = L.orc_window_score(int(so[0]), int(n1o[0]), int(n2o[0]))
            assert np.float32(dr).view(np.int32) == np.float32(do).view(np.int32) or (dr != dr and do != do), (q, c)
            assert R.ref_window_pass(dr) == L.orc_window_pass(do)
            calls += 1
            wraps += int(int(n1r[0]) * int(n2r[0]) > 2**31 - 1)
    assert calls > 1000 and wraps > calls // 2  # the overflowing products are exercised
    # threshold edges of the score test
    for d in (np.float32(0.81), np.nextafter(np.float32(0.81), np.float32(1)), np.nextafter(np.float32(0.81), np.float32(0))):
        assert R.ref_window_pass(float(d)) == L.orc_window_pass(float(d))


@pytest.mark.skipif("not __import__('oracle').ref_nms_available()", reason="oracle/_ref not built here")
def test_run_nms_pinned(orc):
    """The oracle's cell-level NMS (orc_run_nms) against the reference's OWN run_nms.c main
    (:44-174, extracted from its text at build time with its grid helpers, compute_softmax from
    top_N.c reached without a prototype as in the reference binary, F7): the same survivors in
    the same order, and as many suppressions as the oracle removes cells.  Frames: the committed
    quantized_image0 and random 24 x 80 ones; semi scales chosen so that the as-built effective
    scale (the low 32 bits of the promoted double) is 0, 2^-63, 2, 2^65 and -2."""
    import synth

    g = load_golden("quantized_image0.npz")
    rng = np.random.default_rng(29)
    frames = [g["semi"]] + [synth.synth_semi(rng, 1920, p_key=p) for p in (0.3, 0.5, 0.7, 0.9)]
    scales = [float(g["semi_scale"])]
    for low in (1, 2, 3, 6):  # float mantissa low bits -> effective 2^-63, 2, 2^65, -2
        scales.append(float((np.array([0.35], np.float32).view(np.uint32) & ~np.uint32(7) | np.uint32(low))
                            .view(np.float32)[0]))
    checked = nonempty = 0
    for semi in frames:
        for s in scales:
            sup, kp_ref = orc.ref_run_nms(semi, s)
            eff = orc.scale_as_built(s)
            _, mi, pr = orc.compute_softmax(eff, semi)
            before = int((mi != 64).sum())
            m2, _, kp = orc.run_nms(24, 80, mi, pr)
            assert [tuple(int(v) for v in p) for p in kp] == kp_ref, (s, eff)
            assert len(sup) == before - kp.shape[0], (s, eff)
            checked += 1
            nonempty += int(len(sup) > 0)
    assert checked == len(frames) * len(scales) and nonempty >= len(frames)  # suppressions exercised
