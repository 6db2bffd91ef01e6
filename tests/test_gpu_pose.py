"""GPU parity: pose stage.
- as-built (src/pnp_solver.c): stub RANSAC + McAdams SVD pose, bit-exact vs the oracle;
- as-intended: 8-point RANSAC + cheirality + Gauss-Newton recovers the reference's own
  transforms (outputs/transform_*.npy, via synthetic projections with the K of
  pairwise_pnp.py:667-669) within the north-star tolerance 1e-4."""
import ctypes

import numpy as np
import pytest

import synth
from conftest import load_golden

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north_star: transforms within 1e-4 of reference


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def test_svd3_and_recover_pose_vs_oracle(ctx, orc):
    rng = np.random.default_rng(3)
    mats = [np.eye(3), np.zeros((3, 3)), np.diag([3.0, 2.0, 1.0])]
    mats += [rng.standard_normal((3, 3)) for _ in range(200)]
    for A in mats:
        A = A.astype(np.float32)
        U, S, V = ctx.svd3_host(A)
        U2, S2, V2 = orc.svd3(A)
        assert (bits(U) == bits(U2)).all() and (bits(S) == bits(S2)).all() and (bits(V) == bits(V2)).all()
        R1, R2, t = ctx.recover_pose_host(A)
        a, b, c = orc.recover_pose(A)
        assert (bits(R1) == bits(a)).all() and (bits(R2) == bits(b)).all() and (bits(t) == bits(c)).all()


def test_as_built_pose_constant(ctx):
    exp = load_golden("expected_outputs.npz")
    R1, R2, t = ctx.recover_pose_host(np.eye(3, dtype=np.float32))
    assert (bits(R1) == bits(exp["pose_built_R1"])).all() and (bits(t) == bits(exp["pose_built_t"])).all()


@pytest.mark.parametrize("n", [1, 9, 150, 1000, 2500])
def test_ransac_stub_vs_oracle(ctx, orc, n):
    rng = np.random.default_rng(n)
    p1 = rng.uniform(0, 640, (n, 2)).astype(np.float32)
    p2 = (p1 + rng.normal(0, 0.8, (n, 2))).astype(np.float32)
    E, inl, ni = ctx.ransac_stub_host(p1, p2, 1.1)
    K = np.eye(3, dtype=np.float32)
    st, E2, inl2, ni2 = orc.ransac_essential_matrix(p1, p2, K, 10, 1.1)
    if ni2 > 0:
        assert ni == ni2 and (inl == inl2).all() and (bits(E) == bits(E2)).all()
    else:
        assert ni == 0


def test_dropin_ransac_keeps_rand_stream(ctx, orc):
    import mvtrack

    L = mvtrack.lib()
    libc = ctypes.CDLL("libc.so.6")
    rng = np.random.default_rng(1)
    n = 51
    p1 = rng.uniform(0, 640, (n, 2)).astype(np.float32)
    p2 = (p1 + rng.normal(0, 0.8, (n, 2))).astype(np.float32)
    K = np.array([[517.306408, 0, 318.643040], [0, 516.469215, 255.313989], [0, 0, 1]], np.float32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    libc.srand(0)
    E = np.zeros(9, np.float32)
    inl = np.zeros(1000, np.int32)
    ni = ctypes.c_int(-1)
    L.ransac_essential_matrix(n, P(p1), P(p2), P(K), 10, ctypes.c_float(1.1), P(E), P(inl), ctypes.byref(ni))
    r1 = libc.rand()
    libc.srand(0)
    st, E2, inl2, ni2 = orc.ransac_essential_matrix(p1, p2, K, 10, 1.1)
    r2 = libc.rand()
    assert r1 == r2 and ni.value == ni2 and (inl[:ni2] == inl2).all()
    R1 = np.zeros(9, np.float32)
    R2 = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    L.recover_pose_from_essential_matrix(P(E), P(R1), P(R2), P(t))
    a, b, c = orc.recover_pose(E2)
    assert (bits(R1) == bits(a).reshape(9)).all() and (bits(t) == bits(c)).all()


def _pose_batch(ctx, torch, params, P0, P1, n):
    dev = torch.device("cuda:0")
    B, cap = P0.shape[0], P0.shape[1]
    T = torch.zeros((B, 3, 4), dtype=torch.float32, device=dev)
    ni = torch.zeros(B, dtype=torch.int32, device=dev)
    st = torch.full((B,), 99, dtype=torch.int32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.pose_batch(params, torch.from_numpy(n).to(dev), torch.from_numpy(P0).to(dev), torch.from_numpy(P1).to(dev),
                   T, ni, st)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    return T.cpu().numpy(), ni.cpu().numpy(), st.cpu().numpy()


def pose_error(T, Rg, tg):
    R, t = T[:, :3].astype(np.float64), T[:, 3].astype(np.float64)
    return np.abs(R - Rg).max(), np.abs(t - tg / np.linalg.norm(tg)).max()


def test_intended_pose_recovers_reference_transforms(ctx, torch_cuda):
    """outputs/transform_00078{5..9}_*.npy: noise-free projections of a synthetic scene, 30% outliers."""
    import mvtrack

    Ts = load_golden("poses.npz")["transforms_785_790"]
    B, n = len(Ts), 600
    P0 = np.zeros((B, n, 2), np.float32)
    P1 = np.zeros((B, n, 2), np.float32)
    rng = np.random.default_rng(0)
    for b, T in enumerate(Ts):
        _, x0, x1 = synth.synth_scene(rng, n, T[:, :3], T[:, 3])
        out = rng.random(n) < 0.3
        x1[out] = np.stack([rng.uniform(0, 1241, out.sum()), rng.uniform(0, 376, out.sum())], 1)
        P0[b], P1[b] = x0, x1
    K = synth.KITTI_K
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                              hypotheses=512, inlier_thresh=1.0, refine_iters=10, seed=1)
    T, ni, st = _pose_batch(ctx, torch_cuda, prm, P0, P1, np.full(B, n, np.int32))
    for b, Tg in enumerate(Ts):
        assert st[b] == 0
        eR, et = pose_error(T[b], Tg[:, :3], Tg[:, 3])
        assert eR < TOL and et < TOL, (b, eR, et)
        assert ni[b] >= 0.65 * n


def test_intended_pose_kitti_gt_pairs(ctx, torch_cuda):
    """KITTI 00 ground truth (outputs/00.txt) relative poses 0->1 and 10->11, and a pure
    translation / pure forward motion (degenerate E[2][2] = 0 for the naive 8-point)."""
    import mvtrack

    g = load_golden("poses.npz")
    frames = list(g["kitti00_frames"])
    gt = g["kitti00_gt"]

    def rel(a, b):
        Ta, Tb = np.eye(4), np.eye(4)
        Ta[:3] = gt[frames.index(a)]
        Tb[:3] = gt[frames.index(b)]
        Trel = np.linalg.inv(Tb) @ Ta  # camera a coords -> camera b coords
        return Trel[:3]

    cases = [rel(0, 1), rel(10, 11), np.hstack([np.eye(3), [[0.0], [0.0], [1.0]]]),
             np.hstack([np.eye(3), [[0.3], [0.0], [-0.95]]])]
    B, n = len(cases), 400
    P0 = np.zeros((B, n, 2), np.float32)
    P1 = np.zeros((B, n, 2), np.float32)
    rng = np.random.default_rng(1)
    for b, T in enumerate(cases):
        t = T[:, 3] / np.linalg.norm(T[:, 3])
        _, x0, x1 = synth.synth_scene(rng, n, T[:, :3], t)
        P0[b], P1[b] = x0, x1
    K = synth.KITTI_K
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2], seed=3)
    T, ni, st = _pose_batch(ctx, torch_cuda, prm, P0, P1, np.full(B, n, np.int32))
    for b, Tg in enumerate(cases):
        eR, et = pose_error(T[b], Tg[:, :3], Tg[:, 3])
        assert st[b] == 0 and eR < TOL and et < TOL, (b, eR, et)


def test_intended_pose_degenerate_inputs(ctx, torch_cuda):
    import mvtrack

    B, cap = 3, 16
    P0 = np.zeros((B, cap, 2), np.float32)
    P1 = np.zeros((B, cap, 2), np.float32)
    n = np.array([0, 5, 16], np.int32)
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED)
    T, ni, st = _pose_batch(ctx, torch_cuda, prm, P0, P1, n)
    assert st[0] == mvtrack.MV_ERR_NO_POINTS and st[1] == mvtrack.MV_ERR_DEGENERATE
    assert np.allclose(T[0], np.hstack([np.eye(3), np.zeros((3, 1))]))
    assert np.isfinite(T[2]).all()


def test_as_built_batched_pose_matches_stub(ctx, orc, torch_cuda):
    import mvtrack

    rng = np.random.default_rng(5)
    B, cap = 4, 200
    P0 = rng.uniform(0, 640, (B, cap, 2)).astype(np.float32)
    P1 = (P0 + rng.normal(0, 0.8, (B, cap, 2))).astype(np.float32)
    n = np.array([200, 150, 1, 0], np.int32)
    prm = mvtrack.pose_params(mvtrack.AS_BUILT)
    T, ni, st = _pose_batch(ctx, torch_cuda, prm, P0, P1, n)
    exp = load_golden("expected_outputs.npz")
    for b in range(B):
        if n[b] == 0:
            assert st[b] == mvtrack.MV_ERR_NO_POINTS
            continue
        st2, _, inl2, ni2 = orc.ransac_essential_matrix(P0[b, :n[b]], P1[b, :n[b]], np.eye(3, dtype=np.float32))
        assert ni[b] == max(ni2, 0)
        assert (bits(T[b, :, :3]) == bits(exp["pose_built_R1"])).all()
        assert (bits(T[b, :, 3]) == bits(exp["pose_built_t"])).all()


@pytest.mark.parametrize("semantics", ["built", "intended"])
def test_pose_clamps_counts_and_match_indices(ctx, torch_cuda, semantics):
    """n[b] > cap behaves as n[b] = cap (the pair's slot is never overrun, the last pair's
    included) and match indices outside [0, cap) count as "no match" in both pose kernels."""
    import mvtrack

    torch = torch_cuda
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(11)
    B, cap = 3, 64
    sem = mvtrack.AS_BUILT if semantics == "built" else mvtrack.AS_INTENDED
    prm = mvtrack.pose_params(sem)
    P0 = rng.uniform(0, 640, (B, cap, 2)).astype(np.float32)
    P1 = (P0 + rng.normal(0, 0.8, (B, cap, 2))).astype(np.float32)
    T1, ni1, st1 = _pose_batch(ctx, torch, prm, P0, P1, np.array([cap + 50, cap, 1 << 20], np.int32))
    T2, ni2, st2 = _pose_batch(ctx, torch, prm, P0, P1, np.full(B, cap, np.int32))
    assert (bits(T1) == bits(T2)).all() and (ni1 == ni2).all() and (st1 == st2).all()

    # pose from matches: out-of-range indices are dropped exactly like -1
    idx = np.tile(np.arange(cap, dtype=np.int32), (B, 1))
    bad = idx.copy()
    bad[:, ::5] = cap + 7
    bad[:, 1::7] = -9
    good = idx.copy()
    good[bad != idx] = -1

    def run(mi):
        T = torch.zeros((B, 3, 4), dtype=torch.float32, device=dev)
        nm = torch.zeros(B, dtype=torch.int32, device=dev)
        ni = torch.zeros(B, dtype=torch.int32, device=dev)
        st = torch.full((B,), 99, dtype=torch.int32, device=dev)
        ctx.set_stream(torch.cuda.current_stream())
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        ctx.pose_from_matches(prm, t(np.full(B, cap, np.int32)), t(mi), t(P0), t(P1), T, nm, ni, st)
        torch.cuda.synchronize()
        ctx.set_stream(None)
        return T.cpu().numpy(), nm.cpu().numpy(), ni.cpu().numpy(), st.cpu().numpy()

    a, b = run(bad), run(good)
    assert (a[1] == (good >= 0).sum(1)).all()
    for x, y in zip(a, b):
        assert (np.ascontiguousarray(x).view(np.int32) == np.ascontiguousarray(y).view(np.int32)).all()
