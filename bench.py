#!/usr/bin/env python3
"""bench.py -- tracked frame-pairs/s (match + pose), 1024 kp x 256-D fp32, KITTI shape.

One STEP = the hot path over one batch of B synthetic frame-pairs already resident in HBM:
    mv_match_allpairs_f32_*_dev  all-pairs fp32 match (python/pairwise_pnp.py:635-659 semantics,
                                 bit-exact to the gemmini_functions_cpu.h summation order)
    mv_pose_from_matches_dev     8-point RANSAC + cheirality + Gauss-Newton pose (the intent of
                                 src/pnp_solver.c / pairwise_pnp.py:667-694)
  and, with N > 1 ranks, the per-batch all-gather of every pair's result (T 3x4 + match count,
  52 B per pair) over RCCL -- inside the step.
Workload = BASELINE.json configs[1] (1024 x 1024 keypoints x 256-D fp32 synthetic descriptors)
with the pose of the metric's "match+PnP".  Pairs are independent (scripts/run_pairwise_pnp.sh:
7-20 runs them as separate processes): one process per GPU, each rank its own B pairs -- weak
scaling.  value = pairs processed by all ranks / max-over-ranks wall time.

--gpus N without a launcher: the script starts N rank processes itself (before any GPU call),
each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, and exits with their status; under
torch.distributed.run it is one rank.  --harness-cpu runs the same multi-rank harness with the
CPU oracle as the step over gloo (a test of the harness, never a measurement).

Extra fields: roofline of the dominant kernel, its algorithmic bytes per launch from SURVEY
§8(d) (2 x n x 1 KiB + n x 8 B per pair) and its average launch duration measured with HIP events
on the launch stream over a second, profiled run of the same steps (the headline loop itself runs
unprofiled); traffic = HBM bytes per launch from the committed rocprofv3 PMC summary of this
same command; cpu_baseline = the reference's gemmini matmul + row argmax on the host's cores
(rank 0, N = 1 only); secondary lines (N = 1): near-threshold workload (SURVEY C1 sigma), the
CPU C0 path, windowed front-end, int8 all-pairs, sequence mode, keypoints.
"""
import argparse
import ctypes  # noqa: F401  (ctypes-backed oracle calls release the GIL)
import datetime
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))

FP16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense FP16/BF16 MFMA peak (~2.5 PF, no sparsity)
I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: int8 MFMA = 2x the BF16 rate (~5 POPS dense)
HBM_PEAK_GBS = 8000.0
KD = 256
METRIC = "tracked frame-pairs/sec (match+PnP), 1024kp x 256-D KITTI shape"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192,
                    help="frame-pairs per GPU per step (one launch each; SURVEY §8d: >= 1000 pairs per launch)")
    ap.add_argument("--kp", type=int, default=1024, help="keypoints per frame")
    ap.add_argument("--hypotheses", type=int, default=256)
    ap.add_argument("--noise", type=float, default=0.3 / 16.0,
                    help="per-component noise of the re-observed descriptors (renormalised; |noise| ~ 16 x this)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="contexts (each with its own stream) taking the batches in turn: one batch's pose "
                         "overlaps the next batch's match.  The per-kernel durations (roofline, stages) "
                         "come from a second loop on ONE context, where kernels do not overlap")
    ap.add_argument("--score-steps", type=int, default=10,
                    help="secondary: steps timed with the exact score materialised (0 = skip)")
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="secondary lines at N = 1: near-threshold, int8 all-pairs, sequence, keypoints; 0 = skip")
    ap.add_argument("--screen", choices=("i8", "i8s", "f16"), default="i8",
                    help="all-pairs screen (outputs identical): int8 one-pass (default), int8 against a staged "
                         "image, or fp16 against a staged image")
    ap.add_argument("--check", type=int, default=2, help="pairs verified against the oracle after timing")
    ap.add_argument("--unfused", action="store_true",
                    help="staged screens: stage the next batch with the separate split kernel on the auxiliary "
                         "stream instead of inside the match launch")
    ap.add_argument("--window-steps", type=int, default=10,
                    help="secondary line (N = 1 only): the windowed int8 front-end of tracking_main.c "
                         "(tools/bench_window.py, 7285-cell KITTI grid, 8192 pairs); 0 = skip")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1: the collective backend (nccl = RCCL over xGMI, the product path; gloo stages the "
                         "per-step result gather through host memory -- how the N-rank GPU path is exercised on a "
                         "one-GPU box, where RCCL refuses two ranks on one device)")
    ap.add_argument("--force-gather", action="store_true",
                    help="initialise the process group (--dist-backend) and issue the per-step result all-gather "
                         "even at world size 1 -- how the RCCL gather on the pipelined streams is exercised on a "
                         "one-GPU box (a one-rank all_gather_into_tensor is a device-side copy through RCCL)")
    ap.add_argument("--gather-every", type=int, default=0,
                    help="steps whose per-pair results share one all-gather (0: the pipeline depth)")
    ap.add_argument("--harness-cpu", action="store_true",
                    help="test only: the multi-rank harness with the CPU oracle as the step (gloo)")
    ap.add_argument("--dist-timeout", type=float, default=180.0,
                    help="N > 1: seconds a collective may wait for a peer before the process group fails (a dead "
                         "or hung rank ends the run instead of blocking the survivors for the 10-minute default)")
    ap.add_argument("--rank-grace", type=float, default=5.0,
                    help="spawned ranks: seconds the surviving ranks get after one rank fails before they are "
                         "terminated (they are blocked in the step's all-gather by then)")
    return ap.parse_args(argv)


def pair_seed(rank, b):
    """Seed of pair b on `rank`: ranks draw disjoint pairs (pair id = rank * 2^20 + b)."""
    return 1000 + rank * (1 << 20) + b


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# Per-rank progress of the timed loop in a small shared file (spawned ranks only): slot r holds
# (steps issued, first-step start, last-step end, pairs per step) as float64, written by rank r after
# each timed step (two stores into a memory map, no syscall), read by the spawning parent when a rank
# fails -- SURVEY §5's "per-GPU worker failure = drop that GPU's pairs".
_PROGRESS = {"map": None, "rank": 0, "pairs": 0}


def progress_open(path, world, rank, pairs_per_step):
    if not path:
        return
    _PROGRESS["map"] = np.memmap(path, dtype=np.float64, mode="r+", shape=(world, 4))
    _PROGRESS["rank"], _PROGRESS["pairs"] = rank, pairs_per_step
    _PROGRESS["map"][rank] = (0.0, 0.0, 0.0, float(pairs_per_step))


def _fail_hook(step_i):
    """test hook (tests/test_dist.py): MV_BENCH_KILL_RANK=r with MV_BENCH_KILL_STEP=k makes rank r die
    abruptly (exit 17, no cleanup) at its k-th timed step -- a lost GPU / worker in the middle of the
    per-step all-gathers."""
    kr = os.environ.get("MV_BENCH_KILL_RANK")
    if kr is not None and int(kr) == int(os.environ.get("RANK", "0")) and \
            step_i == int(os.environ.get("MV_BENCH_KILL_STEP", "0")):
        sys.stderr.write("rank %s: MV_BENCH_KILL_RANK test hook, exiting at timed step %d\n" % (kr, step_i))
        sys.stderr.flush()
        os._exit(17)


def spawn_ranks(n, argv, grace=5.0):
    """--gpus N without a launcher: N child processes, one rank per GPU, started before this
    process touches the GPU.  All children are polled: when one exits non-zero, the others get
    `grace` seconds and are then terminated (they would otherwise block in the next all-gather
    until the process-group timeout), and this process prints rank 0's JSON line itself, from the
    surviving ranks' progress: their pairs only, the failed ranks named in `ranks_failed`, exit
    status non-zero.  All children successful: their status (0) is ours, rank 0 printed the line."""
    import tempfile

    env = dict(os.environ)
    env.update(WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               LOCAL_WORLD_SIZE=str(n))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    fd, prog_path = tempfile.mkstemp(prefix="mv_bench_progress_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    os.write(fd, bytes(n * 4 * 8))
    os.close(fd)
    env["MV_BENCH_PROGRESS"] = prog_path
    procs = []
    t_start = time.time()
    try:
        for r in range(n):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e))
        failed, t_fail = [], None
        while True:
            rcs = [p.poll() for p in procs]
            for r, rc in enumerate(rcs):
                if rc not in (None, 0, PEER_LOST) and not any(f["rank"] == r for f in failed):
                    failed.append({"rank": r, "exit": rc, "after_s": round(time.time() - t_start, 2)})
                    t_fail = t_fail or time.time()
            if all(rc is not None for rc in rcs):
                break
            if t_fail is not None and time.time() - t_fail > grace:
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                for p in procs:
                    try:
                        p.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        p.wait()
                break
            time.sleep(0.05)
        if not failed:
            # every non-zero exit was a survivor's lost collective: no rank names itself the cause
            if any(p.returncode == PEER_LOST for p in procs):
                failed = [{"rank": r, "exit": p.returncode, "after_s": None} for r, p in enumerate(procs)
                          if p.returncode == PEER_LOST]
                print(json.dumps({"metric": METRIC, "value": None, "n_gpus": n, "partial": True,
                                  "error": "collectives failed on ranks %s with no rank failing first" %
                                           [f["rank"] for f in failed], "ranks_failed": failed}), flush=True)
                return PEER_LOST
            return 0
        first = failed[0]["rank"]  # the first rank seen failing (polled in order)
        prog = np.fromfile(prog_path, dtype=np.float64).reshape(n, 4)
        dead = {f["rank"] for f in failed}
        alive = [r for r in range(n) if r not in dead]
        pairs = sum(int(prog[r, 0]) * int(prog[r, 3]) for r in alive)
        span = max([prog[r, 2] - prog[r, 1] for r in alive if prog[r, 0] > 0] or [0.0])
        out = {"metric": METRIC, "value": round(pairs / span, 2) if span > 0 else None, "unit": "pairs/s",
               "n_gpus": n, "higher_is_better": True, "scaling": "weak", "partial": True,
               "error": "rank %d exited with status %d; the other ranks were stopped" % (
                   first, [f["exit"] for f in failed if f["rank"] == first][0]),
               "ranks_failed": sorted(failed, key=lambda f: f["after_s"]),
               "ranks_surviving": [{"rank": r, "steps_issued": int(prog[r, 0]), "pairs_per_step": int(prog[r, 3]),
                                    "seconds": round(float(prog[r, 2] - prog[r, 1]), 4)} for r in alive],
               "note": "value = pairs of the surviving ranks' timed steps (host-issued; the failed ranks' pairs "
                       "dropped) / their longest span -- SURVEY 5: per-GPU worker failure drops that GPU's pairs"}
        print(json.dumps(out), flush=True)
        return max(1, max(f["exit"] if f["exit"] > 0 else 1 for f in failed))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        try:
            os.unlink(prog_path)
        except OSError:
            pass


def timed_loop(step, steps, warmup, sync, barrier):
    """warmup untimed steps, then EXACTLY `steps` steps bracketed by barrier + device sync."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    pm, pr = _PROGRESS["map"], _PROGRESS["rank"]
    if pm is not None:
        pm[pr, 0], pm[pr, 1] = 0.0, time.time()
    for i in range(steps):
        _fail_hook(i)
        step()
        if pm is not None:
            pm[pr, 0], pm[pr, 2] = float(i + 1), time.time()
    sync()
    barrier()
    return time.perf_counter() - t0


def max_over_ranks(torch, dist, x, device):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    e = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(e.item())


def gather_checksums(torch, dist, values, device):
    """All-gather a small per-rank result vector (validation only, outside the timed region)."""
    t = torch.as_tensor(values, dtype=torch.float64, device=device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [t.cpu()]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu() for o in out]


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ResultGather:
    """an all-gather of every pair's result -- T (3x4 fp32) and the match count, 13
    words = 52 B per pair -- into a [world * rows, 13] buffer on every rank (rank 0 keeps it for
    the report / trajectory chain).  The results of `every` consecutive steps (one per pipelined
    context, `every` = the pipeline depth by default) share ONE all-gather, issued on the last
    step's stream after it has waited for the others' copies: one collective launch per pipeline
    cycle instead of one per step (one GPU with a forced RCCL group: 1.6 % of the step against
    2.6 % per step, profiles/r06bb_gather_ab.log).  A no-op without a process group (world size 1
    unless --force-gather)."""

    def __init__(self, torch, dist, world, B, device, slots, coll_device=None, every=1):
        self.torch, self.dist, self.world = torch, dist, world
        self.active = dist.is_available() and dist.is_initialized()
        self.coll_device = device if coll_device is None else coll_device  # gloo + GPU results: via the host
        self.every, self.B = max(1, every), B
        self.res = [torch.empty((self.every * B, 13), dtype=torch.float32, device=device) for _ in range(2)]
        self.out = [torch.empty((world * self.every * B, 13), dtype=torch.float32, device=self.coll_device)
                    for _ in range(2)]
        self.count = 0  # collectives issued
        self.steps = 0
        self.events = []

    def __call__(self, slot, T, nmatch, stream=None):
        if not self.active:
            return
        torch = self.torch
        k = self.steps % self.every  # this step's rows in the current group
        g = (self.steps // self.every) & 1  # double-buffered groups
        self.steps += 1
        with (torch.cuda.stream(stream) if stream is not None else _NullCtx()):
            r = self.res[g][k * self.B:(k + 1) * self.B]
            r[:, :12].copy_(T.reshape(T.shape[0], 12))
            r[:, 12].copy_(nmatch.view(torch.float32))
            if k + 1 < self.every:
                ev = torch.cuda.Event()
                ev.record()
                self.events.append(ev)
                return
            if self.events:  # the group's other copies, made on the other contexts' streams
                cur = torch.cuda.current_stream()
                for ev in self.events:
                    cur.wait_event(ev)
                self.events = []
            full = self.res[g]
            if str(full.device) != str(self.coll_device):
                full = full.to(self.coll_device)  # ordered on `stream` (a blocking copy for the host)
            self.dist.all_gather_into_tensor(self.out[g], full)
        self.count += 1


def gen_batch(torch, dev, B, n, seed, noise=0.3 / 16.0):
    """B synthetic KITTI-shape pairs (synth.synth_pair_f32 semantics; descriptors drawn on the GPU):
    frame 0 = n unit-norm N(0, 1) rows; frame 1 = a random 60 % of them re-observed (+ per-component
    noise `noise`, renormalised) and 40 % fresh rows, shuffled; keypoints = exact projections of a
    3-D scene under the 785 -> 786 relative pose (outputs/transform_000785_000786.npy)."""
    import synth

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    d0 = torch.randn((B, n, KD), generator=g, device=dev)
    d0 = d0 / d0.norm(dim=2, keepdim=True)
    m = int(round(0.6 * n))
    src = torch.argsort(torch.rand((B, n), generator=g, device=dev), dim=1)[:, :m]
    d1 = torch.randn((B, n, KD), generator=g, device=dev)
    d1 = d1 / d1.norm(dim=2, keepdim=True)
    nz = torch.randn((B, m, KD), generator=g, device=dev) * noise
    reobs = torch.gather(d0, 1, src[:, :, None].expand(B, m, KD)) + nz
    d1[:, :m] = reobs / reobs.norm(dim=2, keepdim=True)
    order = torch.argsort(torch.rand((B, n), generator=g, device=dev), dim=1)
    d1 = torch.gather(d1, 1, order[:, :, None].expand(B, n, KD)).contiguous()
    rng = np.random.default_rng(seed)
    kp0 = np.empty((B, n, 2), np.float32)
    kp1 = np.empty((B, n, 2), np.float32)
    src_h = src.cpu().numpy()
    order_h = order.cpu().numpy()
    R, t = synth.T_785_786[:, :3], synth.T_785_786[:, 3]
    for b in range(B):
        _, x0, x1 = synth.synth_scene(rng, n, R, t)
        k1 = np.stack([rng.uniform(0, synth.KITTI_W, n), rng.uniform(0, synth.KITTI_H, n)], 1)
        k1[:m] = x1[src_h[b]]
        kp0[b] = x0
        kp1[b] = k1[order_h[b]]
    return d0.contiguous(), d1, torch.from_numpy(kp0).to(dev), torch.from_numpy(kp1).to(dev)


def pose_angles(T, Tg):
    """per pair: the rotation angle of R Rg^T and the angle between the translation directions
    (degrees; atan2 of sine and cosine, as tests/test_gpu_kitti_e2e.py)"""
    R, t = T[:, :, :3].astype(np.float64), T[:, :, 3].astype(np.float64)
    Rg, tg = Tg[:, :3], Tg[:, 3]
    M = R @ Rg.T
    s = np.linalg.norm(np.stack([M[:, 2, 1] - M[:, 1, 2], M[:, 0, 2] - M[:, 2, 0], M[:, 1, 0] - M[:, 0, 1]], 1), axis=1)
    rot = np.degrees(np.arctan2(s / 2, (np.trace(M, axis1=1, axis2=2) - 1) / 2))
    tra = np.degrees(np.arctan2(np.linalg.norm(np.cross(t, tg), axis=1), t @ tg))
    return rot, tra


def noisy_keypoints(torch, dev, kp1, seed=1234):
    """frame 1's keypoints moved by 0.5 px Gaussian noise and 20 % of them replaced by uniform
    pixels (outlier correspondences)"""
    import synth

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    B, n = kp1.shape[0], kp1.shape[1]
    k1 = kp1 + 0.5 * torch.randn(kp1.shape, generator=g, device=dev)
    out_m = torch.rand((B, n), generator=g, device=dev) < 0.2
    rnd = torch.rand((B, n, 2), generator=g, device=dev) * torch.tensor([synth.KITTI_W, synth.KITTI_H], device=dev)
    return torch.where(out_m[:, :, None], rnd, k1).contiguous()


def noisy_pose_line(torch, dev, cx, stream, pose_p, d0, d1, kp0, kp1, nn_, idx, T, nm, ni, st, fused, kmatch,
                    steps, sync, barrier, label="frame 1: +0.5 px Gaussian noise, 20% replaced by uniform pixels "
                                                "(outliers)"):
    """The headline step with the pose on realistic keypoints (noisy_keypoints), so the RANSAC sees
    contamination and the Gauss-Newton iterates (the headline's exact projections let it exit
    early).  Reports the rate, the kernels' times and the pose accuracy vs the truth."""
    import mvtrack
    import synth

    B = kp1.shape[0]
    k1 = noisy_keypoints(torch, dev, kp1)
    cx.set_stream(torch.cuda.current_stream())

    def np_step():
        if fused:
            cx.match_allpairs_f32_run_prepare(d0, d1, nn_, nn_, idx, None, d1, nn_, 0.8)
        else:
            cx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None, 0.8)
        cx.pose_from_matches(pose_p, nn_, idx, kp0, k1, T, nm, ni, st)

    cx.match_allpairs_f32_prepare(d1, nn_)
    el = timed_loop(np_step, steps, 2, sync, barrier)
    mvtrack.profile_enable(True)
    timed_loop(np_step, steps, 0, sync, barrier)
    mvtrack.profile_enable(False)
    k_ms, k_n = mvtrack.profile_query(kmatch)
    p_ms, p_n = mvtrack.profile_query("k_pose_ransac")
    rs_ms, rs_n = mvtrack.profile_query("k_q8t_rescan")
    rot, tra = pose_angles(T.double().cpu().numpy(), synth.T_785_786)
    cx.set_stream(stream)
    return {"value": round(B * steps / el, 2), "unit": "pairs/s", "ms_per_step": round(el / steps * 1e3, 4),
            "keypoints": label, "match_kernel_avg_ms": k_ms / max(k_n, 1),
            "matches_per_pair": round(float(nm.sum().item()) / B, 1),
            "stages_ms": dict({kmatch: round(k_ms / max(k_n, 1), 4), "k_pose_ransac": round(p_ms / max(p_n, 1), 4)},
                              **({"k_q8t_rescan": round(rs_ms / rs_n, 4)} if rs_n else {})),
            "pose_ok": int((st == 0).sum().item()), "inliers_per_pair": round(float(ni.sum().item()) / B, 1),
            "rot_err_deg": {"median": round(float(np.median(rot)), 4), "p99": round(float(np.percentile(rot, 99)), 4)},
            "tdir_err_deg": {"median": round(float(np.median(tra)), 4), "p99": round(float(np.percentile(tra, 99)), 4)}}


def algorithmic_bytes_per_pair(n):
    """both fp32 frames read once (2 x n x 256 x 4 B) + idx and score per query
    row (n x 8 B) = 2,105,344 B for a 1024^2 pair -- the figure every roofline here divides by."""
    return 2 * n * KD * 4 + n * 8


def design_bytes_per_pair(screen, n, fused):
    """What the screen's match launch itself moves per pair (indices only, 4 B per row):
    i8  -- both fp32 frames once + idx;  i8s -- frame 0 fp32, the staged int8 image of frame 1
    (256 B + scale per row) + idx, and fused the NEXT batch's frame 1 (1 KiB read, 268 B written);
    f16 -- frame 0 fp32 + the staged fp16 image (512 B per row + norm) + idx."""
    if screen == "i8":
        return 2 * n * KD * 4 + n * 4
    if screen == "i8s":
        return n * (KD * 4 + KD + 4 + 4) + (n * (KD * 4 + KD + 12) if fused else 0)
    return n * (KD * 4 + KD * 2 + 4 + 4)


def profile_order_key(path):
    """profiles/rNN<tag>_summary.json in the order they were made: round NN, then the tag as the
    profiles name it (a < ... < z < aa < ab ...: shorter tags first -- a plain name sort would put
    r06z above r06aa and r05v above r05al)"""
    import re

    m = re.match(r"r(\d+)([a-z]*)", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def pmc_traffic(kernel, B, n, screen, fused, noise=None):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of THIS
    command: profiles/*_summary.json written by tools/profile.sh over bench.py itself (bench_args
    without a tool script), the same batch / kp / screen / staging mode and descriptor noise
    (None: the default noise, i.e. no --noise in the profiled arguments).  None when absent."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")), key=profile_order_key,
                    reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        a = d.get("bench_args", "")
        if ".py" in a:  # a tool's profile (tools/prof_cmd.sh), not bench.py's
            continue
        toks = a.split()
        sc = toks[toks.index("--screen") + 1] if "--screen" in toks else "i8"
        nz = float(toks[toks.index("--noise") + 1]) if "--noise" in toks else None
        if sc != screen or ("--unfused" in toks) == fused or nz != noise:
            continue
        k = d.get("kernels", {}).get(kernel, {})
        if d.get("batch") == B and d.get("kp") == n and "hbm_bytes_per_launch" in k:
            return k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def cpu_info():
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    # the GPU box grants one GPU's share of its host (OMP_NUM_THREADS there); nproc shows the
    # whole machine
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return {"nproc": nproc, "affinity": aff, "threads": max(1, min(share, aff)), "cpu_model": model}


def cpu_baseline(seconds, n):
    """gemmini_functions_cpu.h matmul (C += A.B^T, sequential k) + row argmax, on all the host
    threads this process may use (ctypes releases the GIL).  'reference' when the reference's
    own header was compiled into oracle/_ref, else the oracle's restatement ('port')."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import concurrent.futures as cf

    import oracle

    kind = "port"
    mm = oracle.lib().orc_matmul_nt
    if oracle.ref_available():
        try:
            mm = oracle.ref().ref_matmul_nt
            kind = "reference"
        except Exception:
            pass
    L = oracle.lib()
    ci = cpu_info()
    threads = ci["threads"]
    rng = np.random.default_rng(0)
    A = rng.standard_normal((n, KD)).astype(np.float32)
    A /= np.linalg.norm(A, axis=1, keepdims=True)
    Bm = rng.standard_normal((n, KD)).astype(np.float32)
    Bm /= np.linalg.norm(Bm, axis=1, keepdims=True)
    P = oracle._ptr
    deadline = time.perf_counter() + seconds

    def worker(_):
        C = np.zeros((n, n), np.float32)
        idx = np.zeros(n, np.int32)
        sc = np.zeros(n, np.float32)
        pairs = 0
        while time.perf_counter() < deadline:
            C.fill(0)
            mm(n, n, KD, P(A), P(Bm), P(C))
            L.orc_row_argmax(P(C), n, n, 0.8, P(idx), P(sc))
            pairs += 1
        return pairs

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(worker, range(threads)))
    dt = time.perf_counter() - t0
    C = np.zeros((n, n), np.float32)
    t1 = time.perf_counter()
    mm(n, n, KD, P(A), P(Bm), P(C))
    one = time.perf_counter() - t1
    return dict(ci, value=total / dt, unit="pairs/s", cores=threads, kind=kind,
                all_cores_extrapolated={"value": round(total / dt / threads * ci["nproc"], 1), "cores": ci["nproc"],
                                        "note": "per-thread rate x nproc (not run: the box grants %d of its %d "
                                                "cores to one GPU)" % (threads, ci["nproc"])},
                sample="%d pairs of %dx%dx%d fp32 matmul + row argmax over %.1f s on %d host threads "
                       "(gemmini_functions_cpu.h:14-56 order, gcc -O2); 1 core: %.1f ms/pair"
                       % (total, n, n, KD, dt, threads, one * 1e3))


def cpu_c0(seconds):
    """the as-built tracking_main path (softmax + top-N + windowed match + stub
    RANSAC + pose, src/tracking_main.c:68-228) on the real KITTI pair (quantized_image0 -> frame
    000001, 24 x 80 cells), CPU only: the reference's OWN main body extracted from its text and built
    at -O2 with top_N.c / pnp_solver.c ('reference', oracle/_ref), or the oracle's restatement
    ('port') where oracle/_ref is absent.  tools/cpu_c0.py runs as a child process (main's rand()
    is process-global: one pair per worker PROCESS), per pair on one core and on the box's share of
    worker processes; the all-core figure for the whole host is the per-process rate x nproc
    (extrapolated: the box grants one GPU's share of its cores)."""
    ci = cpu_info()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "cpu_c0.py"), "--seconds", str(seconds),
                        "--procs", str(ci["threads"])], capture_output=True, text=True, timeout=seconds + 120)
    if r.returncode != 0:
        return dict(ci, error="tools/cpu_c0.py failed: %s" % r.stderr[-400:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    per_proc = d["value"] / max(d["procs"], 1)
    return dict(ci, metric="C0 as-built tracking_main pairs/s (KITTI 00 000000 -> 000001, 24x80-cell int8, CPU)",
                kind=d["kind"], us_per_pair_1core=d["us_per_pair_1core"], value=d["value"], unit="pairs/s",
                cores=d["procs"], matches=d["matches"],
                all_cores_extrapolated={"value": round(per_proc * ci["nproc"], 1), "cores": ci["nproc"],
                                        "note": "per-process rate x nproc (not run: the box grants %d of its %d "
                                                "cores to one GPU)" % (d["procs"], ci["nproc"])},
                sample="%d pairs over %.1f s on %d worker processes (%s; ctypes call included)" % (
                    d["pairs"], d["seconds"], d["procs"],
                    "src/tracking_main.c main body + top_N.c + pnp_solver.c, gcc -O2" if d["kind"] == "reference"
                    else "oracle restatement"))


def roofline(kernel, screen, B, n, avg_s, fused):
    """The dominant kernel against the HBM roofline on SURVEY §8(d)'s algorithmic bytes (and
    against the int8 / fp16 MFMA peak on its algorithmic ops, under `other`)."""
    algo = algorithmic_bytes_per_pair(n) * B
    design = design_bytes_per_pair(screen, n, fused) * B
    ops = 2.0 * n * n * KD * B
    gbs = algo / avg_s / 1e9
    peak_c = FP16_PEAK_TFLOPS if screen == "f16" else I8_PEAK_TOPS
    unit_c = "TFLOP/s" if screen == "f16" else "TOP/s"
    achieved_c = ops / avg_s / 1e12
    traffic, src = pmc_traffic(kernel, B, n, screen, fused)
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
            "traffic_ratio": round(traffic / algo, 4) if traffic else None,
            "kernel": kernel, "avg_launch_ms": round(avg_s * 1e3, 4),
            "algorithmic_bytes_per_launch": algo,
            "algorithmic_bytes_note": "SURVEY 8(d): 2 x %d x 256 x 4 B (both fp32 frames once) + %d x 8 B per pair "
                                      "x %d pairs" % (n, n, B),
            "design_bytes_per_launch": design,
            "traffic_overhead_bytes_per_launch": design - algo,
            "other": {"bound": "mfma", "achieved": round(achieved_c, 2), "peak": peak_c, "unit": unit_c,
                      "frac": round(achieved_c / peak_c, 4),
                      "note": "algorithmic 2*n0*n1*256 ops per pair on the %s MFMA screen" % (
                          "fp16" if screen == "f16" else "int8")}}


def main_cpu_harness(args, world, rank):
    """--harness-cpu: the multi-rank harness (spawn, barrier-bracketed timing, max over ranks,
    per-step result all-gather, JSON) with the CPU oracle as the step -- over gloo."""
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    if world > 1:
        dist.init_process_group(backend="gloo", timeout=datetime.timedelta(seconds=args.dist_timeout))
    B, n = args.batch, args.kp
    progress_open(os.environ.get("MV_BENCH_PROGRESS"), world, rank, B)
    pairs = []
    for b in range(B):
        r = np.random.default_rng(pair_seed(rank, b))
        a = r.standard_normal((n, KD)).astype(np.float32)
        c = a[r.permutation(n)] + 0.05 * r.standard_normal((n, KD)).astype(np.float32)
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        c /= np.linalg.norm(c, axis=1, keepdims=True)
        pairs.append((a, c))
    T = torch.zeros((B, 3, 4), dtype=torch.float32)
    nm = torch.zeros(B, dtype=torch.int32)
    gather = ResultGather(torch, dist, world, B, "cpu", 1)

    def step():
        for b, (a, c) in enumerate(pairs):
            idx, _ = oracle.allpairs_f32(a, c, 0.8)
            nm[b] = int((idx >= 0).sum())
            T[b, :, :3] = torch.eye(3)
            T[b, 0, 3] = float(rank)
        gather(0, T, nm)

    barrier = dist.barrier if world > 1 else (lambda: None)
    el = max_over_ranks(torch, dist, timed_loop(step, args.steps, args.warmup, lambda: None, barrier), "cpu")
    gathered = gather.out[0] if world > 1 else torch.cat([T.reshape(B, 12), nm.view(torch.float32)[:, None]], 1)
    out = {"metric": METRIC, "value": round(B * args.steps * world / el, 2), "unit": "pairs/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
           "harness": "cpu-oracle (test of the multi-rank harness, not a measurement)",
           "gathered_pairs": int(gathered.shape[0]),
           "gathered_matches": int(gathered[:, 12].contiguous().view(torch.int32).sum()),
           "gathered_ranks": sorted(set(int(x) for x in gathered[:, 3].tolist())),
           "all_gathers": gather.count}
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, {"rank": rank, "device": "cpu", "backend": dist.get_backend(), "pid": os.getpid()})
        out["ranks"] = ranks
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], args.rank_grace))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.harness_cpu:
        return main_cpu_harness(args, world, rank)

    import torch
    import torch.distributed as dist

    import mvtrack
    import synth

    # LOCAL_RANK -> device modulo the visible devices: N ranks may share a box with fewer GPUs
    # (a rehearsal of the N-rank path; with nccl, RCCL needs one device per rank)
    local = local % max(torch.cuda.device_count(), 1)
    if world > 1 or args.force_gather:
        if world == 1:  # a one-rank group (--force-gather): the rendezvous on this host
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        to = datetime.timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local), timeout=to)
        else:
            dist.init_process_group(backend="gloo", timeout=to)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    B, n = args.batch, args.kp
    progress_open(os.environ.get("MV_BENCH_PROGRESS"), world, rank, B)

    d0, d1, kp0, kp1 = gen_batch(torch, dev, B, n, seed=pair_seed(rank, 0), noise=args.noise)
    nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
    P = max(1, args.pipeline)
    idxs = [torch.empty((B, n), dtype=torch.int32, device=dev) for _ in range(P)]
    score = torch.empty((B, n), dtype=torch.float32, device=dev)
    Ts = [torch.empty((B, 3, 4), dtype=torch.float32, device=dev) for _ in range(P)]
    nmatches = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P)]
    ninls = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P)]
    statuses = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P)]

    # --pipeline P: P contexts, each with its own stream, take the batches in turn: one batch's
    # pose overlaps the next batch's match -- the host pipelining a user would do with P streams
    ctxs, streams = [], []
    for _ in range(P):
        c = mvtrack.Context(local)
        st_ = torch.cuda.Stream(device=dev) if P > 1 else torch.cuda.current_stream()
        c.set_stream(st_)
        c.set_allpairs_screen(args.screen)
        c.reserve(B, n)
        ctxs.append(c)
        streams.append(st_)
    K = synth.KITTI_K
    pose_p = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                                 hypotheses=args.hypotheses, inlier_thresh=1.0, refine_iters=10, seed=7)
    gather = ResultGather(torch, dist, world, B, dev, P, coll_dev, every=args.gather_every or P)

    # the reference keeps only the matched pairs (pairwise_pnp.py:649-657): no score output, so
    # the exact re-score runs only where the rounding window does not decide the row (indices
    # bit-identical to the with-score mode; tests/test_gpu_allpairs.py)
    out_score = [None]
    turn = [0]
    fused = args.screen in ("i8", "i8s") and not args.unfused

    def step():
        c = turn[0] % P
        turn[0] += 1
        cx = ctxs[c]
        if fused:  # i8: the one-pass match; i8s: this batch's match + the next batch staged, one launch
            cx.match_allpairs_f32_run_prepare(d0, d1, nn_, nn_, idxs[c], out_score[0], d1, nn_, 0.8)
        else:
            cx.match_allpairs_f32_run(d0, d1, nn_, nn_, idxs[c], out_score[0], 0.8)
            cx.match_allpairs_f32_prepare(d1, nn_)  # this context's next batch
        cx.pose_from_matches(pose_p, nn_, idxs[c], kp0, kp1, Ts[c], nmatches[c], ninls[c], statuses[c])
        gather(c, Ts[c], nmatches[c], streams[c] if P > 1 else None)

    for cx in ctxs:
        cx.match_allpairs_f32_prepare(d1, nn_)

    mvtrack.profile_enable(False)
    sync = torch.cuda.synchronize
    barrier = dist.barrier if gather.active else (lambda: None)

    # the headline: an unprofiled loop (no per-kernel events inside the measured wall time)
    elapsed = timed_loop(step, args.steps, args.warmup, sync, barrier)
    elapsed = max_over_ranks(torch, dist, elapsed, coll_dev)
    gathers_timed = gather.count

    # per-kernel durations for the roofline and the stage split: a second, profiled loop of the
    # same steps on ONE context (hipEvents on each kernel's own launch stream; with P > 1 the
    # kernels of different contexts overlap and their event times would include each other)
    def prof_step():
        turn[0] = 0
        step()

    sync()
    mvtrack.profile_enable(True)
    timed_loop(prof_step, args.steps, 0, sync, barrier)
    mvtrack.profile_enable(False)
    screen = ctxs[0].allpairs_screen()
    kmatch, ksplit = {"i8": ("k_q8d_match", None), "i8s": ("k_q8_match", "k_q8_split"),
                      "f16": ("k_ap_match", "k_ap_split")}[screen]
    kfb = None
    if screen == "i8" and mvtrack.profile_query("k_q8t_match")[1] > 0:
        # one workgroup per pair (cap <= 1024); k_q8d_handback then redoes only the pairs it hands back
        # (outside the integer keys' range: none in this data -- its launch is the workgroups' exit)
        kmatch, kfb = "k_q8t_match", "k_q8d_handback"
    k_ms, k_n = mvtrack.profile_query(kmatch)
    fb_ms, fb_n = mvtrack.profile_query(kfb) if kfb else (0.0, 0)
    rs_ms, rs_n = mvtrack.profile_query("k_q8t_rescan") if kfb else (0.0, 0)
    s_ms, s_n = mvtrack.profile_query(ksplit) if ksplit else (0.0, 0)
    p_ms, p_n = mvtrack.profile_query("k_pose_ransac")
    with_scores = None
    if args.score_steps > 0:
        out_score[0] = score
        for _ in range(2):
            step()
        sync()
        el_s = max_over_ranks(torch, dist, timed_loop(step, args.score_steps, 0, sync, barrier), coll_dev)
        mvtrack.profile_enable(True)
        timed_loop(prof_step, args.score_steps, 0, sync, barrier)
        mvtrack.profile_enable(False)
        ks_ms, ks_n = mvtrack.profile_query(kmatch)
        with_scores = {"value": round(B * args.score_steps * world / el_s, 2),
                       "ms_per_step": round(el_s / args.score_steps * 1e3, 4),
                       kmatch + "_ms": round(ks_ms / max(ks_n, 1), 4)}
        out_score[0] = None
        for c in range(P):  # leave idx from the headline mode
            if fused:
                ctxs[c].match_allpairs_f32_run_prepare(d0, d1, nn_, nn_, idxs[c], None, d1, nn_, 0.8)
            else:
                ctxs[c].match_allpairs_f32_run(d0, d1, nn_, nn_, idxs[c], None, 0.8)
                ctxs[c].match_allpairs_f32_prepare(d1, nn_)
        sync()

    idx, T, nmatch, status = idxs[0], Ts[0], nmatches[0], statuses[0]
    ok = int((status == 0).sum().item())
    checked = 0
    if args.check > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle

        for b in range(min(args.check, B)):
            i2, s2 = oracle.allpairs_f32(d0[b].cpu().numpy(), d1[b].cpu().numpy(), 0.8)
            assert (idx[b].cpu().numpy() == i2).all(), "timed match output differs from the oracle"
            if with_scores is not None:  # the with-score loop's exact scores, bit for bit
                assert (score[b].cpu().numpy().view(np.int32) == s2.view(np.int32)).all(), "score differs"
            checked += 1
        R = T[:, :, :3].double().cpu().numpy()
        err = np.abs(R - synth.T_785_786[None, :, :3]).max(axis=(1, 2))
        assert ok == B and float(err.max()) < 1e-3, "pose failed: ok=%d max|dR|=%g" % (ok, err.max())
    gathered = None
    if gather.active:  # the last all-gather's buffer: every rank's results, this rank's own slice
        sync()         # equal to its T and match count bit for bit, for every step of the group
        E = gather.every
        g = gather.out[((gather.steps // E) - 1) & 1].view(world, E, B, 13)
        for k in range(E):
            c = k % P
            assert torch.equal(g[rank, k, :, :12].to(dev).view(torch.int32), Ts[c].reshape(B, 12).view(torch.int32)), \
                "gathered T differs from this rank's (step %d of the group)" % k
            assert torch.equal(g[rank, k, :, 12].contiguous().to(dev).view(torch.int32), nmatches[c]), \
                "gathered match count differs from this rank's (step %d of the group)" % k
        g = g.reshape(world, E * B, 13)
        props = torch.cuda.get_device_properties(local)
        me = {"rank": rank, "device": local, "backend": dist.get_backend(),
              "pci_bus": "%s:%s" % (getattr(props, "pci_domain_id", "?"), getattr(props, "pci_bus_id", "?")),
              "pid": os.getpid()}
        ranks = [None] * world
        dist.all_gather_object(ranks, me)  # validation only: which device / backend every rank ran on
        gathered = {"ranks": ranks, "pairs_per_gather": int(g.shape[0] * g.shape[1]), "gathers_in_timed_steps": gathers_timed,
                    "bytes_per_gather": int(g.numel() * 4), "backend": args.dist_backend,
                    "steps_per_gather": gather.every, "streams": "pipelined" if P > 1 else "current",
                    "ranks_per_device": "%d ranks on %d device(s)" % (world, torch.cuda.device_count())}
    sums = gather_checksums(torch, dist, [float(nmatch.sum().item()), float(ok)], coll_dev)
    pairs_total = B * args.steps * world
    value = pairs_total / elapsed
    k_avg_s = (k_ms / max(k_n, 1)) * 1e-3
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: unit-norm N(0,1) 256-D descriptors, 60%% re-observed (+ per-component noise %.4g, "
                "renormalised), exact projections of a 3-D scene under outputs/transform_000785_000786.npy, "
                "KITTI K, 1241x376" % args.noise,
        "config": {"workload": "configs[1]: all-pairs match %dx%d kp x 256-D fp32 + RANSAC/GN pose per pair"
                               % (n, n), "pairs_per_gpu_per_step": B, "kp": n, "dim": KD,
                   "pose": "8-point RANSAC %d hyp + cheirality + 10 GN iters" % args.hypotheses,
                   "scores": "not materialised (pairwise_pnp.py keeps only the matched pairs); "
                             "indices bit-exact; see with_scores",
                   "parallelism": "pairs sharded one process per GPU (dp%d); per step one all-gather of the "
                                  "per-pair results (T + count, 52 B per pair)" % world},
        "roofline": roofline(kmatch, screen, B, n, k_avg_s, fused),
        "screen": screen,
        "staging": {"i8": "none (frame 1 quantised inside the match workgroup)",
                    "i8s": "fused into k_q8_match (next batch)" if fused else "k_q8_split on the auxiliary stream",
                    "f16": "k_ap_split"}[screen],
        "stages_ms_per_step": dict({kmatch: round(k_avg_s * 1e3, 4),
                                    "k_pose_ransac": round(p_ms / max(p_n, 1), 4)},
                                   **({ksplit: round(s_ms / max(s_n, 1), 4)} if ksplit else {}),
                                   **({kfb + " (hand-backs only)": round(fb_ms / max(fb_n, 1), 4)} if kfb else {}),
                                   **({"k_q8t_rescan (wide rows only)": round(rs_ms / rs_n, 4)} if rs_n else {})),
        "with_scores": with_scores,
        "result_gather": gathered,
        "checked_pairs": checked, "pose_ok": int(sum(float(x[1]) for x in sums)),
        "matches_per_pair": round(sum(float(x[0]) for x in sums) / (B * world), 1),
    }
    if rank == 0 and world == 1 and args.extra_steps > 0:
        # SURVEY §8(d) C1's noise (sigma 0.05 per component: re-observed cosines ~0.78, at the
        # 0.8 threshold), so that the near-threshold exact re-scores are timed
        cx = ctxs[0]
        e0, e1, ek0, ek1 = gen_batch(torch, dev, B, n, seed=pair_seed(rank, 7), noise=0.05)
        cx.set_stream(torch.cuda.current_stream())

        def nt_step():
            if fused:
                cx.match_allpairs_f32_run_prepare(e0, e1, nn_, nn_, idxs[0], None, e1, nn_, 0.8)
            else:
                cx.match_allpairs_f32(e0, e1, nn_, nn_, idxs[0], None, 0.8)
            cx.pose_from_matches(pose_p, nn_, idxs[0], ek0, ek1, Ts[0], nmatches[0], ninls[0], statuses[0])

        cx.match_allpairs_f32_prepare(e1, nn_)
        el = timed_loop(nt_step, args.extra_steps, 2, sync, barrier)
        mvtrack.profile_enable(True)
        timed_loop(nt_step, args.extra_steps, 0, sync, barrier)
        mvtrack.profile_enable(False)
        kn_ms, kn_n = mvtrack.profile_query(kmatch)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle

        i2, _ = oracle.allpairs_f32(e0[0].cpu().numpy(), e1[0].cpu().numpy(), 0.8)
        assert (idxs[0][0].cpu().numpy() == i2).all(), "near-threshold match differs from the oracle"
        kn_s = kn_ms / max(kn_n, 1) * 1e-3
        tr_nt, tr_src = pmc_traffic(kmatch, B, n, screen, fused, noise=0.05)
        out["near_threshold"] = {
            "value": round(B * args.extra_steps / el, 2), "unit": "pairs/s",
            "ms_per_step": round(el / args.extra_steps * 1e3, 4), "noise": 0.05,
            kmatch + "_ms": round(kn_s * 1e3, 4),
            "hbm_frac_8d": round(algorithmic_bytes_per_pair(n) * B / kn_s / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": tr_nt, "traffic_source": tr_src,
            "traffic_ratio": round(tr_nt / (algorithmic_bytes_per_pair(n) * B), 4) if tr_nt else None,
            "matches_per_pair": round(float(nmatches[0].sum().item()) / B, 1), "checked_pairs": 1}
        cx.set_stream(streams[0])
    if rank == 0 and world == 1 and args.extra_steps > 0:
        # the realistic step: SURVEY C1 descriptors (sigma 0.05: re-observed cosines at the 0.8
        # threshold, the exact re-scores timed) AND noisy / contaminated keypoints, with the match
        # kernel's own roofline (traffic: the sigma-0.05 PMC summary -- the same kernel on the same
        # descriptors as near_threshold)
        r = noisy_pose_line(torch, dev, ctxs[0], streams[0], pose_p, e0, e1, ek0, ek1, nn_, idxs[0], Ts[0],
                            nmatches[0], ninls[0], statuses[0], fused, kmatch, args.extra_steps, sync, barrier,
                            label="SURVEY C1 descriptors (sigma 0.05) + frame 1 keypoints +0.5 px Gaussian noise, "
                                  "20% replaced by uniform pixels (outliers)")
        ks = r.pop("match_kernel_avg_ms") * 1e-3
        algo = algorithmic_bytes_per_pair(n) * B
        tr_r, tr_rs = pmc_traffic(kmatch, B, n, screen, fused, noise=0.05)
        r["roofline"] = {"bound": "hbm", "kernel": kmatch, "avg_launch_ms": round(ks * 1e3, 4),
                         "achieved": round(algo / ks / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / ks / 1e9 / HBM_PEAK_GBS, 4), "traffic": tr_r, "traffic_source": tr_rs,
                         "traffic_ratio": round(tr_r / algo, 4) if tr_r else None}
        r["noise"] = 0.05
        out["realistic"] = r
        out["noisy_pose"] = noisy_pose_line(torch, dev, ctxs[0], streams[0], pose_p, d0, d1, kp0, kp1, nn_,
                                            idxs[0], Ts[0], nmatches[0], ninls[0], statuses[0], fused, kmatch,
                                            args.extra_steps, sync, barrier)
        out["noisy_pose"].pop("match_kernel_avg_ms")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, n)
        out["cpu_c0"] = cpu_c0(min(args.cpu_seconds, 8.0))
    if rank == 0 and world == 1 and args.window_steps > 0:
        # north-star secondary: the windowed match kernel, timed after (and outside)
        # the headline measurement
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_window

        w, _ = bench_window.run(batch=8192, steps=args.window_steps, warmup=2, check=1)
        out["window_frontend"] = {k: w[k] for k in ("metric", "value", "unit", "ms_per_step", "semantics",
                                                     "stages_ms", "hbm_roofline", "checked_pairs")}
    if rank == 0 and world == 1 and args.extra_steps > 0:
        # the other single-GPU configs beside the headline (not its value): BASELINE config 5
        # (int8 all-pairs, 2048 kp), sequence mode and SURVEY §8(f)2 keypoint extraction
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_i8
        import bench_keypoints
        import bench_sequence

        r = bench_i8.run(batch=8192, kp=2048, steps=args.extra_steps, warmup=2, check=1)
        out["i8_allpairs"] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "stages_ms",
                                                  "mfma_roofline", "checked_pairs")}
        r = bench_sequence.run(frames=B + 1, kp=n, steps=args.extra_steps, warmup=2, check=1, pipeline=P)
        out["sequence"] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "pairs_per_step", "stages_ms",
                                              "staging", "hbm_roofline", "checked_pairs", "pose_ok")}
        r = bench_keypoints.run(batch=1024, steps=args.extra_steps, warmup=2, check=1)
        out["keypoints"] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "stages_ms",
                                               "hbm_roofline", "checked_frames")}
        # the quantized SuperPoint network (KITTI frames -> int8 semi / desc)
        import bench_superpoint

        r = bench_superpoint.run(batch=512, steps=args.extra_steps, warmup=2, check=1)
        out["superpoint"] = {k: r[k] for k in ("metric", "value", "unit", "batch", "ms_per_step", "stages_ms",
                                                "mfma_roofline", "oracle_exact")}
        # the fp32 path of pairwise_pnp.py:577-694 from 8-bit frames to poses (SURVEY 8(f)1 + 2), in
        # a child process of its own: run inside this one, after the lines above, the same
        # two-stream chain measured 69-74 k pairs/s against 77-79 k alone (same stage times; no
        # single earlier line reproduced it: tools/dbg_ip_queues.py), so it is timed as a user runs it
        cp = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_image_pose.py"), "--frames", "257",
                             "--steps", str(args.extra_steps), "--warmup", "2", "--check", "1"],
                            capture_output=True, text=True, timeout=300)
        if cp.returncode != 0:  # recorded, not raised: a secondary line must not take the headline with it
            out["image_to_pose"] = {"error": "bench_image_pose.py exit %d: %s" % (cp.returncode, cp.stderr[-600:])}
            out.setdefault("secondary_errors", []).append("image_to_pose")  # visible at the top level
        else:
            r = json.loads([ln for ln in cp.stdout.splitlines() if ln.startswith("{")][-1])
            out["image_to_pose"] = {k: r.get(k) for k in ("metric", "value", "unit", "frames_per_step", "pipelines",
                                                           "ms_per_step", "stages_ms_per_step", "keypoints_per_frame",
                                                           "matches_per_pair", "pose_ok", "checked_pairs",
                                                           "pose_diff_pairs")}
    if rank == 0:
        print(json.dumps(out), flush=True)
    for cx in ctxs:
        cx.close()
    if gather.active:
        dist.destroy_process_group()


PEER_LOST = 75  # a rank's collective failed because a peer died or hung (it is a survivor, not the cause)


def _collective_error(e):
    """the exception was raised inside torch.distributed (a collective or the rendezvous store)"""
    import traceback

    return any("torch/distributed" in fr.filename.replace(os.sep, "/") for fr in traceback.extract_tb(e.__traceback__))


if __name__ == "__main__":
    try:
        main()
    except Exception as exc:  # noqa: BLE001
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 and _collective_error(exc):
            sys.stderr.write("rank %s: a collective failed (%s: %s) -- a peer rank died or hung; exiting %d\n" % (
                os.environ.get("RANK", "?"), type(exc).__name__, str(exc)[:300], PEER_LOST))
            sys.stderr.flush()
            os._exit(PEER_LOST)
        raise
