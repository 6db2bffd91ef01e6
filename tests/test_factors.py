"""Projection factors (BASELINE north star: projection_factor.c as
per-correspondence Jacobian + J^T J / J^T r assembly): error of src/projection_factor.c:12-33
(with src/types.c:3-73), an analytic Jacobian, the factor's [J|r]^T [J|r] in the local-BA
layout (src/local_bundle_adjustment.c:161-169) and each pose's normal equations.

CPU: the oracle's error equals the reference's own compute_error_ProjectionFactor and its
H_factor the reference's matmul2 on the same J (both compiled from /root/reference into
oracle/_ref; skipped where the reference is absent), bit for bit; the Jacobian matches central
differences of the error (float64).  GPU (marked): kernels equal the oracle bit for bit."""
import numpy as np
import pytest


def scene(seed, F=600, L=200, P=5):
    rng = np.random.default_rng(seed)
    ldmk = np.stack([rng.uniform(-10, 10, L), rng.uniform(-3, 3, L), rng.uniform(5, 60, L)], 1).astype(np.float32)
    q = rng.standard_normal((P, 4)) * np.array([1, 0.05, 0.05, 0.05]) + np.array([3.0, 0, 0, 0])
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    t = rng.standard_normal((P, 3)) * 0.5
    pose = np.concatenate([q, t], 1).astype(np.float32)
    cam = np.tile(np.array([718.856, 718.856, 607.1928, 185.2157], np.float32), (P, 1))
    pid = np.sort(rng.integers(0, P, F)).astype(np.int32)  # grouped by pose
    lid = rng.integers(0, L, F).astype(np.int32)
    meas = (rng.uniform(0, 1241, (F, 2)) * np.array([1, 376 / 1241])).astype(np.float32)
    off = np.searchsorted(pid, np.arange(P + 1)).astype(np.int32)
    return ldmk, pose, lid, pid, meas, cam, off


def test_error_and_hfactor_bit_exact_vs_reference(orc):
    if not orc.ref_available():
        pytest.skip("reference build absent (GPU box): pinned in the build container")
    R = orc.ref()
    ldmk, pose, lid, pid, meas, cam, _ = scene(1)
    err, J, H = orc.pf_linearize(ldmk, pose, lid, pid, meas, cam)
    P = orc._ptr
    for f in range(len(lid)):
        e = np.zeros(2, np.float32)
        R.ref_pf_error(P(ldmk[lid[f]].copy()), P(pose[pid[f]].copy()), P(meas[f].copy()), P(cam[pid[f]].copy()), P(e))
        assert (e.view(np.int32) == err[f].view(np.int32)).all(), f
        h = np.zeros(100, np.float32)
        R.ref_h_factor(P(J[f].copy()), P(h))
        assert (h == H[f]).all(), f  # values (the sign of an exact zero follows the old buffer there)


def test_jacobian_matches_central_differences(orc):
    ldmk, pose, lid, pid, meas, cam, _ = scene(2, F=80)
    _, J, _ = orc.pf_linearize(ldmk, pose, lid, pid, meas, cam)

    def err64(X, q, t, K, m):
        w, x, y, z = q
        Rm = np.array([[w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
                       [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
                       [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])
        p = Rm @ X + t
        return np.array([p[0] / p[2] * K[0] + K[2] - m[0], p[1] / p[2] * K[1] + K[3] - m[1]]), p

    h = 1e-6
    for f in range(len(lid)):
        X, q, t = ldmk[lid[f]].astype(np.float64), pose[pid[f], :4].astype(np.float64), pose[pid[f], 4:].astype(np.float64)
        K, m = cam[pid[f]].astype(np.float64), meas[f].astype(np.float64)
        e0, p = err64(X, q, t, K, m)
        Jf = J[f].reshape(10, 2).T  # column-major 2 x 10
        num = np.zeros((2, 9))
        for c in range(3):
            d = np.zeros(3)
            d[c] = h
            num[:, c] = (err64(X + d, q, t, K, m)[0] - err64(X - d, q, t, K, m)[0]) / (2 * h)
            # rotation: p -> p + omega x p, i.e. the landmark moved by R^T (omega x p) in the frame
            num[:, 3 + c] = (err64(X, q, t + np.cross(d, p), K, m)[0] - err64(X, q, t - np.cross(d, p), K, m)[0]) / (2 * h)
            num[:, 6 + c] = (err64(X, q, t + d, K, m)[0] - err64(X, q, t - d, K, m)[0]) / (2 * h)
        scale = max(1.0, np.abs(num).max())
        assert np.abs(Jf[:, :9] - num).max() < 2e-3 * scale, f
        assert (Jf[:, 9] == orc.pf_linearize(ldmk, pose, lid[f:f + 1], pid[f:f + 1], meas[f:f + 1], cam)[0][0]).all()


def test_pose_normal_equations_oracle(orc):
    ldmk, pose, lid, pid, meas, cam, off = scene(3)
    err, J, H = orc.pf_linearize(ldmk, pose, lid, pid, meas, cam)
    HPP, g, ee = orc.pose_normal_equations(off, H)
    for p in range(len(off) - 1):
        Jp = J[off[p]:off[p + 1]].reshape(-1, 10, 2).transpose(0, 2, 1).reshape(-1, 10).astype(np.float64)
        A = Jp[:, 3:9].T @ Jp[:, 3:9]
        assert np.allclose(HPP[p].reshape(6, 6), A, rtol=1e-4, atol=1e-3 * np.abs(A).max())
        assert np.allclose(g[p], Jp[:, 3:9].T @ Jp[:, 9], rtol=1e-4, atol=1e-3 * np.abs(Jp[:, 3:9].T @ Jp[:, 9]).max())


@pytest.mark.gpu
def test_gpu_factors_bit_exact(ctx, orc, torch_cuda):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    for seed, F in ((4, 1), (5, 777), (6, 20000)):
        ldmk, pose, lid, pid, meas, cam, off = scene(seed, F=F, L=max(50, F // 3), P=7)
        err, J, H = orc.pf_linearize(ldmk, pose, lid, pid, meas, cam)
        HPP, g, ee = orc.pose_normal_equations(off, H)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
        e_d = torch.zeros((F, 2), dtype=torch.float32, device=dev)
        J_d = torch.zeros((F, 20), dtype=torch.float32, device=dev)
        H_d = torch.zeros((F, 100), dtype=torch.float32, device=dev)
        P = off.shape[0] - 1
        HPP_d = torch.zeros((P, 36), dtype=torch.float32, device=dev)
        g_d = torch.zeros((P, 6), dtype=torch.float32, device=dev)
        ee_d = torch.zeros(P, dtype=torch.float32, device=dev)
        ctx.set_stream(torch.cuda.current_stream())
        ctx.projection_factors(t(ldmk), t(pose), t(cam), t(lid), t(pid), t(meas), e_d, J_d, H_d)
        ctx.pose_normal_equations(t(off), J_d, HPP_d, g_d, ee_d)
        e2 = torch.zeros((F, 2), dtype=torch.float32, device=dev)
        ctx.projection_factors(t(ldmk), t(pose), t(cam), t(lid), t(pid), t(meas), e2)  # error only
        torch.cuda.synchronize()
        ctx.set_stream(None)
        bits = lambda x: x.cpu().numpy().view(np.int32)  # noqa: E731
        assert (bits(e_d) == err.view(np.int32)).all() and (bits(e2) == err.view(np.int32)).all()
        assert (bits(J_d) == J.view(np.int32)).all()
        assert (H_d.cpu().numpy() == H).all()
        assert (HPP_d.cpu().numpy() == HPP).all() and (g_d.cpu().numpy() == g).all() and (ee_d.cpu().numpy() == ee).all()
