"""Pipelined contexts (bench.py --pipeline P): P contexts, each on its own HIP stream, take the
batches in turn -- match with the next batch's frame 1 staged in the same launch
(mv_match_allpairs_f32_run_prepare_dev) and the pose of the matches -- with no host
synchronisation between batches, so one context's pose runs beside another's match.  Every
batch's match indices, inlier counts, status and pose must be bit-identical to one context
running the same batches one after the other (and the indices equal the oracle's)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("P", [2, 3])
def test_pipelined_contexts_equal_sequential(ctx, orc, torch_cuda, P):
    import bench
    import mvtrack
    import synth

    torch = torch_cuda
    dev = torch.device("cuda:0")
    B, n, K = 4, 512, 7
    batches = [bench.gen_batch(torch, dev, B, n, seed=300 + k) for k in range(K)]
    nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
    Km = synth.KITTI_K
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=Km[0, 0], fy=Km[1, 1], cx=Km[0, 2], cy=Km[1, 2],
                              hypotheses=256, inlier_thresh=1.0, refine_iters=10, seed=7)

    def outputs():
        return dict(idx=torch.full((B, n), -7, dtype=torch.int32, device=dev),
                    T=torch.zeros((B, 3, 4), dtype=torch.float32, device=dev),
                    nm=torch.zeros(B, dtype=torch.int32, device=dev),
                    ni=torch.zeros(B, dtype=torch.int32, device=dev),
                    st=torch.full((B,), 99, dtype=torch.int32, device=dev))

    def host(o):
        return {k: v.cpu().numpy() for k, v in o.items()}

    # one context, one batch after the other
    ref = []
    ctx.set_stream(torch.cuda.current_stream())
    try:
        for d0, d1, kp0, kp1 in batches:
            o = outputs()
            ctx.match_allpairs_f32_prepare(d1, nn_)
            ctx.match_allpairs_f32_run(d0, d1, nn_, nn_, o["idx"], None, 0.8)
            ctx.pose_from_matches(prm, nn_, o["idx"], kp0, kp1, o["T"], o["nm"], o["ni"], o["st"])
            torch.cuda.synchronize()
            ref.append(host(o))
    finally:
        ctx.set_stream(None)

    # P contexts on P streams, batches in turn, no host sync until the end
    ctxs, streams = [], []
    try:
        for _ in range(P):
            c = mvtrack.Context(0)
            s = torch.cuda.Stream(device=dev)
            c.set_stream(s)
            c.reserve(B, n)
            ctxs.append(c)
            streams.append(s)
        torch.cuda.synchronize()  # the batches were drawn on the default stream
        for c in range(P):
            ctxs[c].match_allpairs_f32_prepare(batches[c][1], nn_)
        outs = []
        for k, (d0, d1, kp0, kp1) in enumerate(batches):
            cx = ctxs[k % P]
            o = outputs()
            streams[k % P].wait_stream(torch.cuda.current_stream())  # the output buffers' fills
            if k + P < K:
                cx.match_allpairs_f32_run_prepare(d0, d1, nn_, nn_, o["idx"], None, batches[k + P][1], nn_, 0.8)
            else:
                cx.match_allpairs_f32_run(d0, d1, nn_, nn_, o["idx"], None, 0.8)
            cx.pose_from_matches(prm, nn_, o["idx"], kp0, kp1, o["T"], o["nm"], o["ni"], o["st"])
            outs.append(o)
        torch.cuda.synchronize()
        got = [host(o) for o in outs]
    finally:
        for c in ctxs:
            c.close()

    for k in range(K):
        for key in ("idx", "nm", "ni", "st"):
            assert (got[k][key] == ref[k][key]).all(), (P, k, key)
        assert (_bits(got[k]["T"]) == _bits(ref[k]["T"])).all(), (P, k)
        assert (ref[k]["st"] == 0).all(), (k, ref[k]["st"])
    # the sequential reference itself against the oracle (first and last batch, one pair each)
    for k in (0, K - 1):
        d0, d1 = batches[k][0][0].cpu().numpy(), batches[k][1][0].cpu().numpy()
        i2, _ = orc.allpairs_f32(d0, d1, 0.8)
        assert (ref[k]["idx"][0] == i2).all(), k


@pytest.mark.gpu
def test_bench_two_ranks_on_the_hip_path():
    """bench.py's N-rank GPU path (not the --harness-cpu rehearsal): --gpus 2 spawns two rank
    processes that run the HIP match + pose on their own disjoint pair shards and all-gather every
    pair's result (one gather per pipeline cycle of 3 steps).  On a one-GPU box both ranks map to cuda:0 (LOCAL_RANK modulo the
    visible devices) and the gather goes through gloo (RCCL refuses two ranks on one device); the
    nccl branch is the same code with the device-resident gather.  Checks: n_gpus 2, the gathered
    buffer holds 2 x B pairs, each rank's slice equals its own results (asserted inside bench.py),
    both ranks' matches verified against the oracle (--check)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    B = 256
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--batch", str(B), "--steps", "3", "--warmup", "1", "--extra-steps", "0", "--score-steps", "2",
                        "--window-steps", "0", "--no-cpu-baseline", "--check", "2"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["steps"] == 3
    g = d["result_gather"]
    # the 3 pipelined contexts' results share one all-gather per cycle (4 steps: one full cycle)
    assert g["steps_per_gather"] == 3 and g["pairs_per_gather"] == 2 * 3 * B and g["backend"] == "gloo"
    assert g["gathers_in_timed_steps"] >= 1
    assert d["pose_ok"] == 2 * B and d["checked_pairs"] == 2 and d["value"] > 0
    assert d["with_scores"] is not None


def test_graph_capture_through_set_stream(ctx, orc, torch_cuda):
    """A match + pose captured into a hipGraph with the context moved ONTO the capture stream inside
    torch.cuda.graph (mv_context_set_stream issues no event record / wait across a capture: one
    would invalidate the capture or pull the context's own stream into it) and moved back after
    the capture ended.  Two replays equal the eager run bit for bit (indices, counts, status, T),
    and the indices equal the oracle's."""
    import bench
    import mvtrack
    import synth

    torch = torch_cuda
    dev = torch.device("cuda:0")
    B, n = 4, 512
    d0, d1, kp0, kp1 = bench.gen_batch(torch, dev, B, n, seed=910)
    nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
    Km = synth.KITTI_K
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=Km[0, 0], fy=Km[1, 1], cx=Km[0, 2], cy=Km[1, 2],
                              hypotheses=256, inlier_thresh=1.0, refine_iters=10, seed=7)

    def outputs():
        return dict(idx=torch.full((B, n), -7, dtype=torch.int32, device=dev),
                    T=torch.zeros((B, 3, 4), dtype=torch.float32, device=dev),
                    nm=torch.zeros(B, dtype=torch.int32, device=dev),
                    ni=torch.zeros(B, dtype=torch.int32, device=dev),
                    st=torch.full((B,), 99, dtype=torch.int32, device=dev))

    def run(o):
        ctx.match_allpairs_f32(d0, d1, nn_, nn_, o["idx"], None, 0.8)
        ctx.pose_from_matches(prm, nn_, o["idx"], kp0, kp1, o["T"], o["nm"], o["ni"], o["st"])

    ctx.reserve(B, n)  # nothing allocates inside the capture
    try:
        ctx.set_stream(torch.cuda.current_stream())
        ref = outputs()
        run(ref)
        torch.cuda.synchronize()
        ref = {k: v.cpu().numpy() for k, v in ref.items()}

        got = outputs()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            ctx.set_stream(torch.cuda.current_stream())  # the capture stream
            run(got)
        ctx.set_stream(torch.cuda.current_stream())  # off the (finished) capture stream
        for _ in range(2):
            for k, v in outputs().items():
                got[k].copy_(v)
            g.replay()
        torch.cuda.synchronize()
        gh = {k: v.cpu().numpy() for k, v in got.items()}
    finally:
        ctx.set_stream(None)
    for key in ("idx", "nm", "ni", "st"):
        assert (gh[key] == ref[key]).all(), key
    assert (_bits(gh["T"]) == _bits(ref["T"])).all()
    assert (ref["st"] == 0).all()
    i2, _ = orc.allpairs_f32(d0[0].cpu().numpy(), d1[0].cpu().numpy(), 0.8)
    assert (ref["idx"][0] == i2).all()


@pytest.mark.gpu
def test_bench_rccl_result_gather_one_rank():
    """bench.py's per-step result all-gather through RCCL (scripts/run_pairwise_pnp.sh:
    7-20 shards the pairs): --force-gather builds an nccl process group at world size 1, so each
    pipeline cycle's all_gather_into_tensor runs device-resident on the stream of the cycle's last
    step, after waiting for the other two contexts' copies.  bench.py asserts every step's gathered
    rows equal that context's T and match counts bit for bit; here: the backend is nccl, the gathers ran inside the timed steps, and
    the matches equal the oracle's (--check)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    B = 256
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--force-gather",
                        "--dist-backend", "nccl", "--batch", str(B), "--steps", "4", "--warmup", "1",
                        "--extra-steps", "0", "--score-steps", "2", "--window-steps", "0", "--no-cpu-baseline",
                        "--check", "2"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    g = d["result_gather"]
    assert g is not None and g["backend"] == "nccl" and g["pairs_per_gather"] == 3 * B
    assert g["steps_per_gather"] == 3 and g["streams"] == "pipelined"
    assert g["gathers_in_timed_steps"] >= 1  # one per pipeline cycle of the 5 warmup + timed steps
    assert d["n_gpus"] == 1 and d["pose_ok"] == B and d["checked_pairs"] == 2
