"""Local-BA Schur back-end (src/local_bundle_adjustment.c:128-250).

CPU: the oracle's chunk loop equals the reference's OWN functions (matrix_add,
invert_block_diagonal_matrix, zero_*, initialize_random_matrix, matmul2 -- compiled from
local_bundle_adjustment.c into oracle/_ref, driven through main's loop by
oracle/ref_lba_harness.c) bit for bit, NaN pattern included (the reference's placeholder
factors make the landmark blocks singular); with real projection factors (as intended) the
pose block equals the dense float64 Schur complement H_PP - H_PL H_LL^-1 H_LP.
GPU (marked): k_lba_schur equals the oracle bit for bit in both modes."""
import numpy as np
import pytest

from test_factors import scene


def real_window(seed, P=6, L=40, LC=4):
    """every landmark seen by every pose: factor blocks from the oracle's linearisation"""
    ldmk, pose, _, _, _, cam, _ = scene(seed, F=1, L=L, P=P)
    rng = np.random.default_rng(seed + 100)
    lid = np.repeat(np.arange(L), P).astype(np.int32)
    pid = np.tile(np.arange(P), L).astype(np.int32)
    meas = rng.uniform(0, 376, (L * P, 2)).astype(np.float32)
    return ldmk, pose, cam, lid, pid, meas


def chunked(J, P, L, LC):
    """[L*P, 20] landmark-major factors -> [chunks, P*LC, 20] with entry ci * P + p"""
    nch = -(-L // LC)
    out = np.zeros((nch, P * LC, 20), np.float32)
    for l in range(L):
        for p in range(P):
            out[l // LC, (l % LC) * P + p] = J[l * P + p]
    return out


@pytest.mark.parametrize("P,L,LC", [(8, 1000, 4), (3, 20, 2), (5, 36, 3)])
def test_oracle_vs_reference_functions(orc, P, L, LC):
    if not orc.ref_available():
        pytest.skip("reference build absent (GPU box): pinned in the build container")
    C = np.zeros((6 * P + 1) ** 2, np.float32)
    orc.ref_lba().ref_lba_schur_main(P, L, LC, orc._ptr(C))
    C2 = orc.lba_schur(P, L, LC, orc.lba_reference_J(P, L, LC), as_built=True)
    assert (C.view(np.int32) == C2.view(np.int32)).all()


def test_oracle_as_intended_is_the_schur_complement(orc):
    P, L, LC = 6, 40, 4
    ldmk, pose, cam, lid, pid, meas = real_window(7, P, L, LC)
    _, J, _ = orc.pf_linearize(ldmk, pose, lid, pid, meas, cam)
    C = orc.lba_schur(P, L, LC, chunked(J, P, L, LC), as_built=False)
    S = 6 * P + 1
    Cm = C.reshape(S, S).T  # column-major
    Jd = J.reshape(-1, 10, 2).transpose(0, 2, 1).astype(np.float64)  # [F, 2, 10]
    HPP = np.zeros((6 * P, 6 * P))
    Schur = np.zeros((6 * P, 6 * P))
    for l in range(L):
        HLL = np.zeros((3, 3))
        HPL = np.zeros((6 * P, 3))
        for p in range(P):
            Jf = Jd[l * P + p]
            HLL += Jf[:, :3].T @ Jf[:, :3]
            HPL[6 * p:6 * p + 6] += Jf[:, 3:9].T @ Jf[:, :3]
            HPP[6 * p:6 * p + 6, 6 * p:6 * p + 6] += Jf[:, 3:9].T @ Jf[:, 3:9]
        Schur += HPL @ np.linalg.inv(HLL) @ HPL.T
    ref = HPP - Schur
    assert np.abs(Cm[:6 * P, :6 * P] - ref).max() <= 2e-3 * np.abs(HPP).max()


def same_bits(a, b):
    """bit for bit, except that a NaN is any NaN (x86 makes the negative quiet NaN for 0/0 and
    inf - inf, the GPU the positive one)"""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return (na == nb).all() and (a[~na].view(np.int32) == b[~nb].view(np.int32)).all()


@pytest.mark.gpu
def test_gpu_lba_schur_bit_exact(ctx, orc, torch_cuda):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    ctx.set_stream(torch.cuda.current_stream())
    # as built: the reference's placeholder factors, two windows in one launch
    P, L, LC = 8, 1000, 4
    Jr = orc.lba_reference_J(P, L, LC)
    C = torch.zeros((2, (6 * P + 1) ** 2), dtype=torch.float32, device=dev)
    ctx.lba_schur(P, L, LC, torch.from_numpy(np.stack([Jr, Jr])).to(dev), C, semantics=0)
    # as intended: real factor blocks, 3 windows
    P2, L2, LC2 = 6, 40, 4
    Js = []
    for s in range(3):
        ldmk, pose, cam, lid, pid, meas = real_window(20 + s, P2, L2, LC2)
        Js.append(chunked(orc.pf_linearize(ldmk, pose, lid, pid, meas, cam)[1], P2, L2, LC2))
    C2 = torch.zeros((3, (6 * P2 + 1) ** 2), dtype=torch.float32, device=dev)
    ctx.lba_schur(P2, L2, LC2, torch.from_numpy(np.stack(Js)).to(dev), C2, semantics=1)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    exp = orc.lba_schur(P, L, LC, Jr, as_built=True)
    for b in range(2):
        assert same_bits(C[b].cpu().numpy(), exp)
    for s in range(3):
        e2 = orc.lba_schur(P2, L2, LC2, Js[s], as_built=False)
        assert same_bits(C2[s].cpu().numpy(), e2) and not np.isnan(e2).any()
