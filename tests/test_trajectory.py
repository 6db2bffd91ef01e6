"""Trajectory chaining + pose I/O (python/compute_trajectory.py).

CPU: the oracle's chain is pinned bit for bit by the reference's committed outputs
(outputs/785/trajectory_000785_000789.ply as built, the older outputs/785/trajectory.ply by
the 4x4 composition), the .pose.txt files to their printed 6 decimals, and the library's C
writers reproduce the committed files byte for byte (host code: no device needed).
GPU (marked): the chain kernel equals the oracle bit for bit, the rebase path (multi-GPU
sharding) within float64 rounding, and mv_compute_trajectory writes the reference's files.
A world-size-2 gloo test of the sharded chain lives in tests/test_dist.py."""
import os

import numpy as np
import pytest

import mvtrack
from conftest import load_golden


def traj_fixture():
    return load_golden("trajectory_785.npz")


def ply_points(text):
    lines = text.splitlines()
    nv = int([x for x in lines if x.startswith("element vertex")][0].split()[-1])
    body = lines[lines.index("end_header") + 1:]
    return np.array([[float(v) for v in body[i].split()[:3]] for i in range(nv)])


def transforms():
    return load_golden("poses.npz")["transforms_785_790"]


@pytest.mark.parametrize("mode,key", [(0, "trajectory_000785_000789_ply"), (1, "trajectory_ply")])
def test_oracle_chain_reproduces_reference_ply_points(orc, mode, key):
    exp = ply_points(traj_fixture()[key].tobytes().decode())
    poses = orc.trajectory_chain(transforms()[:4], mode=mode)  # main(785, 789): 4 transforms
    pts = poses[:, :, 3]
    assert pts.shape == exp.shape
    assert (pts.view(np.int64) == exp.view(np.int64)).all()  # bit for bit


def test_oracle_chain_matches_reference_pose_txt(orc):
    g = traj_fixture()
    poses = orc.trajectory_chain(transforms()[:4], mode=0)
    for k in range(5):
        txt = g["frame_%06d_pose_txt" % (785 + k)].tobytes().decode()
        ref = np.array([[float(v) for v in line.split()] for line in txt.splitlines()])
        assert np.abs(ref - poses[k]).max() <= 5.0001e-7


def test_c_writers_reproduce_reference_files_byte_for_byte(orc, tmp_path):
    g = traj_fixture()
    poses = orc.trajectory_chain(transforms()[:4], mode=0)
    for k in range(5):
        p = tmp_path / ("frame-%06d.pose.txt" % (785 + k))
        mvtrack.write_pose_txt(str(p), poses[k])
        assert p.read_bytes() == g["frame_%06d_pose_txt" % (785 + k)].tobytes()
    p = tmp_path / "t.ply"
    mvtrack.write_trajectory_ply(str(p), poses[:, :, 3])
    assert p.read_bytes() == g["trajectory_000785_000789_ply"].tobytes()


def _py_ply(points):
    """write_ply's text for `points` (compute_trajectory.py:6-43 restated with numpy float64
    formatting) -- the expectation for values the committed files do not cover."""
    n = len(points)
    colors = [[255, 0, 0]] + [[0, 0, 255]] * max(n - 2, 0) + [[0, 0, 0]]
    s = ("ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\nproperty float z\n"
         "property uchar red\nproperty uchar green\nproperty uchar blue\nelement edge %d\n"
         "property int vertex1\nproperty int vertex2\nend_header\n") % (n, max(n - 1, 0))
    for p, c in zip(points, colors):
        s += f"{np.float64(p[0])} {np.float64(p[1])} {np.float64(p[2])} {c[0]} {c[1]} {c[2]}\n"
    for i in range(n - 1):
        s += f"{i} {i + 1}\n"
    return s


@pytest.mark.parametrize("n", [0, 1, 2, 7])
def test_ply_writer_float_repr_and_shapes(tmp_path, n):
    rng = np.random.default_rng(n)
    special = [0.0, -0.0, 1e16, 9999999999999998.0, 1e-5, 1.5e-7, 0.0001, 123456789.0, 1 / 3, -2.5e300, 5e-324,
               1e22, 0.1, 100.0, -7.0, 1234567890123456.7]
    vals = np.array(special + list(rng.standard_normal(3 * 8) * 10.0 ** rng.integers(-8, 9, 3 * 8)))
    pts = vals[:3 * n].reshape(n, 3) if n else np.zeros((0, 3))
    p = tmp_path / "x.ply"
    mvtrack.write_trajectory_ply(str(p), pts)
    assert p.read_text() == _py_ply(pts)
    # every value at least once (7 points = 21 values per file)
    for off in range(0, len(vals) - 21, 21):
        q = vals[off:off + 21].reshape(7, 3)
        mvtrack.write_trajectory_ply(str(p), q)
        assert p.read_text() == _py_ply(q)


def test_npy_reader(tmp_path):
    T = transforms()[2]
    p = tmp_path / "t.npy"
    np.save(p, T)
    st, R = mvtrack.read_transform_npy(str(p))
    assert st == 0 and (R == T).all()
    np.save(p, T.astype(np.float32))
    assert mvtrack.read_transform_npy(str(p))[0] == mvtrack.MV_ERR_IO
    np.save(p, np.zeros((4, 4)))
    assert mvtrack.read_transform_npy(str(p))[0] == mvtrack.MV_ERR_IO
    assert mvtrack.read_transform_npy(str(tmp_path / "missing.npy"))[0] == mvtrack.MV_ERR_IO


def test_oracle_missing_transform_carries_pose(orc):
    T = transforms()
    pres = np.array([1, 0, 1, 1, 1], np.int32)
    full = orc.trajectory_chain(T, present=pres)
    assert (full[2] == full[1]).all()
    skip = orc.trajectory_chain(T[[0, 2, 3, 4]])
    assert (full[[0, 1, 3, 4, 5]] == skip).all()


# ------------------------------------------------------------------ GPU
def _rand_rel(rng, n):
    rel = np.zeros((n, 3, 4))
    for k in range(n):
        q = rng.standard_normal(4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        rel[k, :, :3] = [[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                         [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                         [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]]
        rel[k, :, 3] = rng.standard_normal(3)
    return rel


@pytest.mark.gpu
def test_gpu_chain_bit_exact(ctx, orc, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(3)
    B, n = 5, 700  # crosses the kernel's 256-step LDS rounds
    rel = np.stack([_rand_rel(rng, n) for _ in range(B)])
    pres = (rng.random((B, n)) > 0.1).astype(np.int32)
    start = np.stack([_rand_rel(rng, 1)[0] for _ in range(B)])
    dev = torch.device("cuda:0")
    ctx.set_stream(torch.cuda.current_stream())
    for mode in (0, 1):
        out = torch.zeros((B, n + 1, 3, 4), dtype=torch.float64, device=dev)
        ctx.trajectory_chain(torch.from_numpy(rel).to(dev), out, torch.from_numpy(pres).to(dev),
                             torch.from_numpy(start).to(dev), mode)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for b in range(B):
            exp = orc.trajectory_chain(rel[b], present=pres[b], start=start[b], mode=mode)
            assert (got[b].view(np.int64) == exp.view(np.int64)).all(), (mode, b)
    # reference transforms, identity start, no presence mask
    out = torch.zeros((1, 5, 3, 4), dtype=torch.float64, device=dev)
    ctx.trajectory_chain(torch.from_numpy(transforms()[None, :4].copy()).to(dev), out)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    assert (out[0].cpu().numpy().view(np.int64) == orc.trajectory_chain(transforms()[:4]).view(np.int64)).all()


@pytest.mark.gpu
def test_gpu_rebase_equals_sequential_chain(ctx, orc, torch_cuda):
    """a sequence split in two: the second half chained from identity and re-based on the first
    half's end equals the unsplit chain within float64 rounding (re-association)."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    rel = _rand_rel(rng, 300)
    dev = torch.device("cuda:0")
    ctx.set_stream(torch.cuda.current_stream())
    for mode in (0, 1):
        full = orc.trajectory_chain(rel, mode=mode)
        second = torch.from_numpy(orc.trajectory_chain(rel[150:], mode=mode)[None].copy()).to(dev)
        base = torch.from_numpy(full[150][None].copy()).to(dev)
        ctx.trajectory_rebase(base, second, mode)
        torch.cuda.synchronize()
        err = np.abs(second[0].cpu().numpy() - full[150:]).max()
        assert err < 1e-9 * max(1.0, np.abs(full).max()), (mode, err)
    ctx.set_stream(None)


@pytest.mark.gpu
def test_gpu_compute_trajectory_writes_reference_files(ctx, tmp_path):
    g = traj_fixture()
    T = transforms()
    for k in range(5):
        np.save(tmp_path / ("transform_%06d_%06d.npy" % (785 + k, 786 + k)), T[k])
    out = tmp_path / "out"
    out.mkdir()
    assert ctx.compute_trajectory(785, 789, str(tmp_path), str(out)) == 5
    for k in range(5):
        assert (out / ("frame-%06d.pose.txt" % (785 + k))).read_bytes() == g["frame_%06d_pose_txt" % (785 + k)].tobytes()
    assert (out / "trajectory_000785_000789.ply").read_bytes() == g["trajectory_000785_000789_ply"].tobytes()
    # a missing transform is skipped, as in the reference (no pose file, no vertex)
    os.remove(tmp_path / "transform_000786_000787.npy")
    out2 = tmp_path / "out2"
    out2.mkdir()
    assert ctx.compute_trajectory(785, 789, str(tmp_path), str(out2)) == 4
    assert not (out2 / "frame-000787.pose.txt").exists()
