"""CPU, world_size 2 over gloo: the multi-GPU harness of bench.py (one process per rank,
disjoint pair shards, barrier-bracketed timing, max-over-ranks, result all-gather).  The
per-rank step is the CPU oracle on small pairs -- the HIP path itself is covered by -m gpu."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    import time

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "maveric-slam_amd")):
        sys.path.insert(0, p)
    import bench
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 3
    seeds = [bench.pair_seed(rank, b) for b in range(B)]
    pairs = []
    for s in seeds:
        rng = np.random.default_rng(s)
        a = rng.standard_normal((48, 256)).astype(np.float32)
        b = a[rng.permutation(48)] + 0.05 * rng.standard_normal((48, 256)).astype(np.float32)
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        b /= np.linalg.norm(b, axis=1, keepdims=True)
        pairs.append((a, b))
    results = []

    def step():
        results.clear()
        for a, b in pairs:
            results.append(oracle.allpairs_f32(a, b, 0.8)[0])
        if rank == 1:
            time.sleep(0.05)  # the slow rank must set the reported time

    el = bench.timed_loop(step, 3, 1, lambda: None, dist.barrier)
    el_max = bench.max_over_ranks(torch, dist, el, "cpu")
    matches = float(sum(int((r >= 0).sum()) for r in results))
    sums = bench.gather_checksums(torch, dist, [matches, float(rank)], "cpu")
    q.put((rank, el, el_max, seeds, [s.tolist() for s in sums]))
    dist.destroy_process_group()


def test_two_rank_harness_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    (_, el0, max0, seeds0, sums0), (_, el1, max1, seeds1, sums1) = out
    assert max0 == max1 == max(el0, el1)
    assert el1 >= 3 * 0.05  # the slow rank dominates
    assert not set(seeds0) & set(seeds1)  # disjoint shards
    assert sums0 == sums1 and [s[1] for s in sums0] == [0.0, 1.0]
    assert all(s[0] > 100 for s in sums0)  # every rank matched its pairs


def _traj_worker(rank, world, port, q):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "maveric-slam_amd")):
        sys.path.insert(0, p)
    import mvtrack
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = np.load(os.path.join(root, "tests", "golden", "poses.npz"))["transforms_785_790"]
    rel = np.concatenate([g, g[::-1], g])  # 15 transforms, sharded 8 / 7 in order
    cut = [0, 8, 15]
    mine = rel[cut[rank]:cut[rank + 1]]

    def gather(x):  # the RCCL all-gather of the shard end poses (gloo here)
        t = torch.from_numpy(np.ascontiguousarray(x, np.float64))
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [o.numpy() for o in out]

    def rebase(poses, start):  # k_rebase's rule (host stand-in for the device kernel)
        out = poses.copy()
        for k in range(poses.shape[0]):
            P = poses[k]
            for i in range(3):
                for c in range(4):
                    v = P[i, 0] * start[0, c] + P[i, 1] * start[1, c] + P[i, 2] * start[2, c]
                    if c == 3:
                        v = v + P[i, 3] if mode == mvtrack.CHAIN_COMPOSE else P[i, 3] + start[i, 3]
                    out[k, i, c] = v
        return out

    res = {}
    for mode in (mvtrack.CHAIN_AS_BUILT, mvtrack.CHAIN_COMPOSE):
        res[mode] = mvtrack.chain_sharded(lambda r: oracle.trajectory_chain(r, mode=mode), rebase, gather, rank,
                                          mine, mode)
    q.put((rank, res))
    dist.destroy_process_group()


def test_two_rank_sharded_trajectory_gloo():
    """a sequence sharded over 2 ranks: local chains + all-gather of shard ends + re-base equal
    the unsharded chain (within float64 rounding: re-association)."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_traj_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.load(os.path.join(root, "tests", "golden", "poses.npz"))["transforms_785_790"]
    rel = np.concatenate([g, g[::-1], g])
    for mode in (0, 1):
        full = oracle.trajectory_chain(rel, mode=mode)
        got = np.concatenate([out[0][mode], out[1][mode][1:]])
        assert got.shape == full.shape
        assert np.abs(got - full).max() < 1e-12
        assert np.abs(out[1][mode][0] - out[0][mode][-1]).max() < 1e-12  # rank 1 starts where rank 0 ends


def test_sequence_shard_covers_every_pair_once():
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "maveric-slam_amd"))
    import mvtrack

    for F in (2, 3, 5, 17, 8193):
        for W in (1, 2, 3, 4, 8, 16):
            seen = []
            prev_hi = None
            for r in range(W):
                lo, hi = mvtrack.sequence_shard(F, W, r)
                if hi > lo:
                    assert hi - lo >= 2
                    if prev_hi is not None:
                        assert lo == prev_hi - 1  # one shared boundary frame
                    prev_hi = hi
                    seen += list(range(lo, hi - 1))
            assert seen == list(range(F - 1)), (F, W)
    with pytest.raises(ValueError):
        mvtrack.sequence_shard(1, 2, 0)


def test_bench_spawns_ranks_and_gathers_results():
    """bench.py --gpus 2 without a launcher starts its own 2 rank processes; --harness-cpu runs
    the same harness (barrier-bracketed timing, max over ranks, the per-step all-gather of every
    pair's T + match count) with the CPU oracle as the step over gloo: n_gpus 2, the gathered
    buffer holds N x B pairs from both ranks, one all-gather per step (warmup included)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--harness-cpu", "--batch", "3",
                        "--kp", "32", "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["steps"] == 2
    assert d["gathered_pairs"] == 2 * 3 and d["gathered_ranks"] == [0, 1]
    assert d["all_gathers"] == 3
    assert d["gathered_matches"] > 0 and d["value"] > 0


def _seq_worker(rank, world, port, q):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "maveric-slam_amd")):
        sys.path.insert(0, p)
    import mvtrack
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F, n = 6, 40
    rng = np.random.default_rng(5)  # every rank sees the same track (its frames only are used)
    D = rng.standard_normal((F, n, 256)).astype(np.float32)
    for b in range(1, F):
        D[b, :24] = D[b - 1, rng.permutation(n)[:24]] + 0.02 * rng.standard_normal((24, 256)).astype(np.float32)
    D /= np.linalg.norm(D, axis=2, keepdims=True)
    lo, hi = mvtrack.sequence_shard(F, world, rank)
    mine = [(b, oracle.allpairs_f32(D[b], D[b + 1], 0.8)[0].tolist()) for b in range(lo, hi - 1)]
    out = [None] * world
    dist.all_gather_object(out, mine)  # validation only
    q.put((rank, out))
    dist.destroy_process_group()


def test_two_rank_sequence_shards_gloo():
    """The sequence partition over 2 ranks (mvtrack.sequence_shard, one shared boundary frame,
    no exchange): each rank's contiguous pair range, matched by the CPU oracle and gathered,
    covers the track pair for pair.  The GPU sequence kernel on the same shards is
    test_two_rank_sequence_shards_gpu."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seq_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    F, n = 6, 40
    rng = np.random.default_rng(5)
    D = rng.standard_normal((F, n, 256)).astype(np.float32)
    for b in range(1, F):
        D[b, :24] = D[b - 1, rng.permutation(n)[:24]] + 0.02 * rng.standard_normal((24, 256)).astype(np.float32)
    D /= np.linalg.norm(D, axis=2, keepdims=True)
    got = sorted(x for shard in res[0] for x in shard)
    assert [b for b, _ in got] == list(range(F - 1))
    for b, idx in got:
        assert idx == oracle.allpairs_f32(D[b], D[b + 1], 0.8)[0].tolist(), b
    assert res[0] == res[1]


def _seq_gpu_worker(rank, world, port, q):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "maveric-slam_amd")):
        sys.path.insert(0, p)
    import mvtrack

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = _seq_track()
    F, n = D.shape[0], D.shape[1]
    lo, hi = mvtrack.sequence_shard(F, world, rank)
    dev = torch.device("cuda:0")
    ctx = mvtrack.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    d = torch.from_numpy(np.ascontiguousarray(D[lo:hi])).to(dev)
    ns = torch.full((hi - lo,), n, dtype=torch.int32, device=dev)
    idx = torch.empty((hi - lo - 1, n), dtype=torch.int32, device=dev)
    ctx.match_sequence_f32(d, ns, idx, None, 0.8)
    torch.cuda.synchronize()
    mine = [(lo + b, idx[b].cpu().numpy().tolist()) for b in range(hi - lo - 1)]
    ctx.close()
    out = [None] * world
    dist.all_gather_object(out, mine)
    q.put((rank, out))
    dist.destroy_process_group()


def _seq_track():
    F, n = 9, 96
    rng = np.random.default_rng(8)
    D = rng.standard_normal((F, n, 256)).astype(np.float32)
    for b in range(1, F):
        D[b, :60] = D[b - 1, rng.permutation(n)[:60]] + 0.02 * rng.standard_normal((60, 256)).astype(np.float32)
    D /= np.linalg.norm(D, axis=2, keepdims=True)
    return D


@pytest.mark.gpu
def test_two_rank_sequence_shards_gpu():
    """Sequence mode sharded over 2 ranks (two processes on the GPU, gloo for the gather): each
    rank runs mv_match_sequence_f32_dev on its contiguous frame range (one shared boundary
    frame); the gathered per-pair indices equal a single-process sequence match of the whole
    track and the oracle, pair for pair."""
    import sys

    import torch

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "oracle"), os.path.join(root, "maveric-slam_amd")):
        sys.path.insert(0, p)
    import mvtrack
    import oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seq_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    D = _seq_track()
    F, n = D.shape[0], D.shape[1]
    got = sorted(x for shard in res[0] for x in shard)
    assert [b for b, _ in got] == list(range(F - 1))
    dev = torch.device("cuda:0")
    c = mvtrack.Context(0)
    c.set_stream(torch.cuda.current_stream())
    d = torch.from_numpy(D).to(dev)
    idx = torch.empty((F - 1, n), dtype=torch.int32, device=dev)
    c.match_sequence_f32(d, torch.full((F,), n, dtype=torch.int32, device=dev), idx, None, 0.8)
    torch.cuda.synchronize()
    full = idx.cpu().numpy()
    c.close()
    for b, ix in got:
        assert ix == full[b].tolist(), b
        assert ix == oracle.allpairs_f32(D[b], D[b + 1], 0.8)[0].tolist(), b
    assert res[0] == res[1]


def test_bench_dead_rank_fails_fast_and_drops_its_pairs():
    """SURVEY §5 ("per-GPU worker failure = drop that GPU's pairs"), world size 3 over gloo: rank 1
    dies abruptly in the middle of the timed steps (the MV_BENCH_KILL_RANK test hook, exit 17) while
    the others wait in the per-step all-gather.  The spawning harness must notice within its grace
    period -- not the 10-minute collective default -- stop the blocked survivors, exit non-zero, and
    print a JSON line naming the dead rank, with the value computed from the surviving ranks' pairs."""
    import json
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MV_BENCH_KILL_RANK="1", MV_BENCH_KILL_STEP="2")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--harness-cpu", "--batch", "3",
                        "--kp", "32", "--steps", "6", "--warmup", "1", "--dist-timeout", "60", "--rank-grace", "2"],
                       capture_output=True, text=True, timeout=240, env=env)
    took = time.time() - t0
    assert r.returncode == 17, (r.returncode, r.stderr[-2000:])
    assert took < 120, took
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["partial"] is True and d["n_gpus"] == 3
    assert d["ranks_failed"][0]["rank"] == 1 and d["ranks_failed"][0]["exit"] == 17
    assert "rank 1" in d["error"]
    surv = {s["rank"]: s for s in d["ranks_surviving"]}
    assert sorted(surv) == [0, 2]
    # rank 1 died at its timed step 2: the survivors issued steps 0, 1 and were blocked in step 2's gather
    assert all(s["steps_issued"] == 2 and s["pairs_per_step"] == 3 for s in surv.values())
    assert d["value"] > 0
    assert "MV_BENCH_KILL_RANK" in r.stderr


def test_bench_names_every_rank_device_and_backend():
    """the gathered per-rank record (rank, device, backend) that shows which ranks the collective saw"""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--harness-cpu", "--batch", "2",
                        "--kp", "32", "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert [x["rank"] for x in d["ranks"]] == [0, 1, 2]
    assert all(x["backend"] == "gloo" for x in d["ranks"])
    assert len({x["pid"] for x in d["ranks"]}) == 3


def test_roofline_traffic_cites_the_newest_profile():
    """bench.py's roofline.traffic comes from the newest matching profiles/r*_summary.json, newest by
    round and tag (r05al after r05v, r06aa after r06z), not by a plain reverse name sort."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench

    names = ["r05v_summary.json", "r05al_summary.json", "r06z_summary.json", "r06aa_summary.json", "r06_summary.json",
             "r04zz_summary.json", "r06b_summary.json"]
    got = sorted(names, key=bench.profile_order_key)
    assert got == ["r04zz_summary.json", "r05v_summary.json", "r05al_summary.json", "r06_summary.json",
                   "r06b_summary.json", "r06z_summary.json", "r06aa_summary.json"]
    tr, src = bench.pmc_traffic("k_q8t_match", 8192, 1024, "i8", True)
    assert src is None or (tr > 0 and src.startswith("profiles/r"))
