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
