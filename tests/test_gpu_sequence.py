"""Sequence mode (mv_match_sequence_f32_dev): consecutive frames of one track, pair b =
(frame b, frame b + 1) as the reference's driver runs pairwise_pnp.py
(scripts/run_pairwise_pnp.sh:7-20; the match itself python/pairwise_pnp.py:635-659).  Every
frame is quantised once and serves as frame 1 of one pair and frame 0 of the next; the
outputs must be bit-identical to the oracle's per-pair match (gemmini_functions_cpu.h:14-56
order) and to the independent-pair entry point."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["i8", "i8s"])
def seq_screen(request, ctx):
    """the default screen runs sequence mode as k_q8t_match over the pairs in place (cap <= 1024);
    the staged int8 screen through each frame's image once (k_q8_match<AI8>): both must equal the
    oracle"""
    ctx.set_allpairs_screen(request.param)
    yield request.param
    ctx.set_allpairs_screen("i8")


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _track(rng, F, cap, ns, reobs=0.6, noise=0.3):
    """F frames of unit 256-D descriptors; frame b + 1 re-observes 60 % of frame b (+ noise)."""
    D = np.zeros((F, cap, 256), np.float32)
    prev = None
    for b in range(F):
        d = rng.standard_normal((cap, 256)).astype(np.float32)
        if prev is not None:
            m = int(reobs * cap)
            src = rng.permutation(cap)[:m]
            d[:m] = prev[src] + rng.standard_normal((m, 256)).astype(np.float32) * (noise / 16)
            d = d[rng.permutation(cap)]
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        D[b] = d
        prev = d
    for b, n in enumerate(ns):
        D[b, n:] = rng.standard_normal((cap - n, 256)).astype(np.float32) * 5  # junk past n
    return D


def _run_seq(ctx, torch, D, ns, scores=True):
    dev = torch.device("cuda:0")
    F, cap = D.shape[0], D.shape[1]
    d = torch.from_numpy(D).to(dev)
    n = torch.from_numpy(np.asarray(ns, np.int32)).to(dev)
    idx = torch.full((F - 1, cap), -7, dtype=torch.int32, device=dev)
    sc = torch.full((F - 1, cap), 7.0, dtype=torch.float32, device=dev) if scores else None
    ctx.set_stream(torch.cuda.current_stream())
    try:
        ctx.match_sequence_f32(d, n, idx, sc, 0.8)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    return idx.cpu().numpy(), (sc.cpu().numpy() if scores else None)


def test_sequence_vs_oracle_ragged(ctx, orc, torch_cuda, seq_screen):
    rng = np.random.default_rng(17)
    cap = 640
    ns = [640, 513, 0, 300, 640, 1, 257, 640]
    D = _track(rng, len(ns), cap, ns)
    D[3, 5] = 0.0          # a zero row in frame 3 (frame 0 of pair 3, frame 1 of pair 2)
    D[4, 7, 9] = np.inf    # frame 4 flagged: pairs 3 and 4 take the exact path
    D[6, 2] *= 3e-13       # a tiny row (scale below the screen's range)
    idx, sc = _run_seq(ctx, torch_cuda, D, ns)
    for b in range(len(ns) - 1):
        n0, n1 = ns[b], ns[b + 1]
        assert (idx[b, n0:] == -1).all(), b
        if n0 == 0:
            continue
        if n1 == 0:
            assert (idx[b, :n0] == -1).all(), b
            continue
        i2, s2 = orc.allpairs_f32(D[b, :n0], D[b + 1, :n1], 0.8)
        assert (idx[b, :n0] == i2).all(), b
        assert (_bits(sc[b, :n0]) == _bits(s2)).all(), b


@pytest.mark.parametrize("scores", [True, False])
def test_sequence_full_size_equals_pairs(ctx, orc, torch_cuda, scores, seq_screen):
    """65 frames x 1024 keypoints: equal to the independent-pair match of (frame b, frame b + 1),
    bit for bit, and to the oracle on the first and last pair."""
    torch = torch_cuda
    rng = np.random.default_rng(23)
    F, cap = 65, 1024
    ns = [cap] * F
    D = _track(rng, F, cap, ns)
    idx, sc = _run_seq(ctx, torch, D, ns, scores)
    dev = torch.device("cuda:0")
    d0 = torch.from_numpy(D[:-1].copy()).to(dev)
    d1 = torch.from_numpy(D[1:].copy()).to(dev)
    n = torch.full((F - 1,), cap, dtype=torch.int32, device=dev)
    ri = torch.full((F - 1, cap), -7, dtype=torch.int32, device=dev)
    rs = torch.zeros((F - 1, cap), dtype=torch.float32, device=dev) if scores else None
    ctx.set_stream(torch.cuda.current_stream())
    try:
        ctx.match_allpairs_f32(d0, d1, n, n, ri, rs, 0.8)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    assert (idx == ri.cpu().numpy()).all()
    if scores:
        assert (_bits(sc) == _bits(rs.cpu().numpy())).all()
    assert (idx >= 0).sum() > 0.4 * idx.size  # the track re-observes 60 %
    for b in (0, F - 2):
        i2, s2 = orc.allpairs_f32(D[b], D[b + 1], 0.8)
        assert (idx[b] == i2).all(), b
        if scores:
            assert (_bits(sc[b]) == _bits(s2)).all(), b


def test_sequence_refuses_f16_screen_and_short_tracks(ctx, torch_cuda):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    D = torch.zeros((2, 64, 256), dtype=torch.float32, device=dev)
    n = torch.full((2,), 64, dtype=torch.int32, device=dev)
    idx = torch.empty((1, 64), dtype=torch.int32, device=dev)
    ctx.set_allpairs_screen("f16")
    try:
        with pytest.raises(RuntimeError):
            ctx.match_sequence_f32(D, n, idx, None)
    finally:
        ctx.set_allpairs_screen("i8")
    with pytest.raises(RuntimeError):
        ctx.match_sequence_f32(D[:1], n[:1], idx, None)


def test_sequence_run_prepare_chain(ctx, orc, torch_cuda, seq_screen):
    """A track processed in chunks: the first chunk prepared, then each chunk matched while the next one's frames are staged in the
    same launch; chunks of different lengths and caps, ragged counts, scores and indices-only,
    each equal to the oracle pair by pair; a run without its prepare is refused."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(29)
    chunks = []
    for k, (F, cap) in enumerate(((4, 512), (6, 384), (3, 640), (5, 512))):
        ns = [int(rng.integers(1, cap + 1)) for _ in range(F)]
        if k == 1:
            ns[2] = 0
        D = _track(rng, F, cap, ns)
        chunks.append((D, ns, torch.from_numpy(D).to(dev), torch.from_numpy(np.asarray(ns, np.int32)).to(dev)))
    ctx.set_stream(torch.cuda.current_stream())
    try:
        D, ns, d, n = chunks[0]
        ctx.match_allpairs_f32_prepare(d, n)
        for k, (D, ns, d, n) in enumerate(chunks):
            F, cap = D.shape[0], D.shape[1]
            scores = k % 2 == 0
            idx = torch.full((F - 1, cap), -7, dtype=torch.int32, device=dev)
            sc = torch.zeros((F - 1, cap), dtype=torch.float32, device=dev) if scores else None
            if k + 1 < len(chunks):
                ctx.match_sequence_f32_run_prepare(d, n, idx, sc, chunks[k + 1][2], chunks[k + 1][3])
            else:
                ctx.match_sequence_f32(d, n, idx, sc)
            torch.cuda.synchronize()
            idx = idx.cpu().numpy()
            sc = sc.cpu().numpy() if scores else None
            for b in range(F - 1):
                n0, n1 = ns[b], ns[b + 1]
                assert (idx[b, n0:] == -1).all(), (k, b)
                if n0 == 0:
                    continue
                if n1 == 0:
                    assert (idx[b, :n0] == -1).all(), (k, b)
                    continue
                i2, s2 = orc.allpairs_f32(D[b, :n0], D[b + 1, :n1], 0.8)
                assert (idx[b, :n0] == i2).all(), (k, b)
                if scores:
                    assert (_bits(sc[b, :n0]) == _bits(s2)).all(), (k, b)
        # the one-shot call invalidated the prepared image: run_prepare is refused
        D, ns, d, n = chunks[0]
        with pytest.raises(RuntimeError):
            ctx.match_sequence_f32_run_prepare(d, n, torch.empty((D.shape[0] - 1, D.shape[1]), dtype=torch.int32,
                                                                 device=dev), None, d, n)
    finally:
        ctx.set_stream(None)


def test_sequence_track_end_to_end(ctx, orc, torch_cuda):
    """A camera moving by the 785 -> 786 transform per frame through a 3-D scene: each frame
    re-observes the previous frame's points still in view (60 % of its rows) and adds fresh
    ones; per-frame keypoints are exact projections.  Sequence-mode match + pose over the
    per-frame keypoints as two offset views (kp[:-1], kp[1:]) recovers every pair's rotation."""
    import mvtrack
    import synth

    torch = torch_cuda
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(41)
    F, n = 6, 512
    m = int(0.6 * n)
    R, t = synth.T_785_786[:, :3], synth.T_785_786[:, 3]
    K = synth.KITTI_K

    def project(P):
        q = P @ K.T
        return q[:, :2] / q[:, 2:3]

    P, _, _ = synth.synth_scene(rng, n, R, t)  # frame 0 points, visible in frame 1
    desc = [rng.standard_normal((n, 256))]
    pts = [P]
    for k in range(1, F):
        Q = pts[-1] @ R.T + t  # the previous frame's points in frame k
        q = project(Q)
        vis = np.nonzero((Q[:, 2] > 0.5) & (q[:, 0] >= 0) & (q[:, 0] < synth.KITTI_W) & (q[:, 1] >= 0) &
                         (q[:, 1] < synth.KITTI_H))[0]
        src = rng.permutation(vis)[:m]
        fresh, _, _ = synth.synth_scene(rng, n - len(src), R, t)
        order = rng.permutation(n)
        Pk = np.concatenate([Q[src], fresh])[order]
        dk = np.concatenate([desc[-1][src] / np.linalg.norm(desc[-1][src], axis=1, keepdims=True) +
                             rng.standard_normal((len(src), 256)) * (0.3 / 16),
                             rng.standard_normal((n - len(src), 256))])[order]
        pts.append(Pk)
        desc.append(dk)
    D = np.stack([d / np.linalg.norm(d, axis=1, keepdims=True) for d in desc]).astype(np.float32)
    KP = np.stack([project(p) for p in pts]).astype(np.float32)
    d = torch.from_numpy(D).to(dev)
    kp = torch.from_numpy(KP).to(dev)
    nf = torch.full((F,), n, dtype=torch.int32, device=dev)
    idx = torch.empty((F - 1, n), dtype=torch.int32, device=dev)
    T = torch.empty((F - 1, 3, 4), dtype=torch.float32, device=dev)
    nm = torch.empty(F - 1, dtype=torch.int32, device=dev)
    ni = torch.empty(F - 1, dtype=torch.int32, device=dev)
    st = torch.full((F - 1,), 99, dtype=torch.int32, device=dev)
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                              hypotheses=256, inlier_thresh=1.0, refine_iters=10, seed=7)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        ctx.match_sequence_f32(d, nf, idx, None, 0.8)
        ctx.pose_from_matches(prm, nf[:-1], idx, kp[:-1], kp[1:], T, nm, ni, st)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    idx = idx.cpu().numpy()
    for b in range(F - 1):
        i2, _ = orc.allpairs_f32(D[b], D[b + 1], 0.8)
        assert (idx[b] == i2).all(), b
    assert (st.cpu().numpy() == 0).all(), st
    assert (nm.cpu().numpy() >= 0.5 * n).all(), nm
    Rg = T[:, :, :3].double().cpu().numpy()
    assert np.abs(Rg - R[None]).max() < 1e-3
