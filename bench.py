#!/usr/bin/env python3
"""bench.py -- tracked frame-pairs/s (match + pose), 1024 kp x 256-D fp32, KITTI shape.

One STEP = the hot path over one batch of B synthetic frame-pairs already resident in HBM:
    mv_match_allpairs_f32_dev   all-pairs fp32 match (python/pairwise_pnp.py:635-659 semantics,
                                bit-exact to the gemmini_functions_cpu.h summation order)
    mv_pose_from_matches_dev    8-point RANSAC + cheirality + Gauss-Newton pose (the intent of
                                src/pnp_solver.c / pairwise_pnp.py:667-694)
Workload = BASELINE.json configs[1] (1024 x 1024 keypoints x 256-D fp32 synthetic descriptors)
with the pose of the metric's "match+PnP".  Pairs are independent: with --gpus N each rank
(one process per GPU, torch.distributed) processes its own B pairs -- weak scaling, no
data-path collective.  value = pairs processed by all ranks / max-over-ranks wall time.

Extra fields: roofline of the dominant kernel (k_q8_match), its average launch duration
measured with HIP events on the launch stream over a second, profiled run of the same steps
(the headline loop itself runs unprofiled); cpu_baseline = the gemmini matmul
+ row argmax (+ as-built stub pose) on host cores (rank 0, N = 1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))

FP16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense FP16/BF16 MFMA peak (~2.5 PF, no sparsity)
I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: int8 MFMA = 2x the BF16 rate (~5 POPS dense)
HBM_PEAK_GBS = 8000.0
KD = 256


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192,
                    help="frame-pairs per GPU per step (one launch each; SURVEY §8d: >= 1000 pairs per launch; "
                         "1024 / 2048 / 4096 / 8192 measured 1.32 / 1.42 / 1.56 / 1.59 M pairs/s: launch tails "
                         "amortised, and more of the pose overlaps the next match)")
    ap.add_argument("--kp", type=int, default=1024, help="keypoints per frame")
    ap.add_argument("--hypotheses", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="contexts (each with its own stream) taking the batches in turn: one batch's pose "
                         "overlaps the next batch's match.  The per-kernel durations (roofline, stages) "
                         "come from a second loop on ONE context, where kernels do not overlap.  At 8192 "
                         "pairs, 40 steps, two runs each: P = 2 / 3 / 4 / 6 measured 1.58 / 1.60 / 1.58 / "
                         "1.57 M pairs/s (tools/sweep_batch.sh; 4 hardware queues per process)")
    ap.add_argument("--score-steps", type=int, default=10,
                    help="secondary: steps timed with the exact score materialised (0 = skip)")
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="secondary lines at N = 1: int8 all-pairs (config 5) and keypoint extraction; 0 = skip")
    ap.add_argument("--screen", choices=("i8", "f16"), default="i8",
                    help="all-pairs screen (outputs identical): int8 MFMA (default) or fp16 MFMA")
    ap.add_argument("--check", type=int, default=2, help="pairs verified against the oracle after timing")
    ap.add_argument("--unfused", action="store_true",
                    help="int8 screen: stage the next batch with the separate k_q8_split on the auxiliary "
                         "stream instead of inside k_q8_match (mv_match_allpairs_f32_run_prepare_dev)")
    ap.add_argument("--window-steps", type=int, default=10,
                    help="secondary line (N = 1 only): the windowed int8 front-end of tracking_main.c "
                         "(tools/bench_window.py, 7285-cell KITTI grid, 1024 pairs); 0 = skip")
    return ap.parse_args()


def pair_seed(rank, b):
    """Seed of pair b on `rank`: ranks draw disjoint pairs (pair id = rank * 2^20 + b)."""
    return 1000 + rank * (1 << 20) + b


def timed_loop(step, steps, warmup, sync, barrier):
    """warmup untimed steps, then EXACTLY `steps` steps bracketed by barrier + device sync."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
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


def gen_batch(torch, dev, B, n, seed):
    """B synthetic KITTI-shape pairs (synth.synth_pair_f32 semantics; descriptors drawn on the GPU)."""
    import synth

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    d0 = torch.randn((B, n, KD), generator=g, device=dev)
    d0 = d0 / d0.norm(dim=2, keepdim=True)
    m = int(round(0.6 * n))
    src = torch.argsort(torch.rand((B, n), generator=g, device=dev), dim=1)[:, :m]
    d1 = torch.randn((B, n, KD), generator=g, device=dev)
    d1 = d1 / d1.norm(dim=2, keepdim=True)
    noise = torch.randn((B, m, KD), generator=g, device=dev) * (0.3 / 16.0)
    reobs = torch.gather(d0, 1, src[:, :, None].expand(B, m, KD)) + noise
    d1[:, :m] = reobs / reobs.norm(dim=2, keepdim=True)
    order = torch.argsort(torch.rand((B, n), generator=g, device=dev), dim=1)
    d1 = torch.gather(d1, 1, order[:, :, None].expand(B, n, KD)).contiguous()
    # geometry: exact projections under the 785->786 relative pose (numpy, small)
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


def pmc_traffic(kernel, B, n, fused=True):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/r*_summary.json, written by tools/profile.sh) taken at the same batch/kp and the
    same staging mode (k_q8_match moves the next batch's frame 1 too when fused)."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel, {})
        if kernel == "k_q8_match" and ("--unfused" in d.get("bench_args", "")) == fused:
            continue
        if kernel == "k_q8_match" and fused and d.get("tag", "") < "r02b":  # profiled before the fusion
            continue
        if d.get("batch") == B and d.get("kp") == n and "hbm_bytes_per_launch" in k:
            return k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(seconds, n):
    """gemmini_functions_cpu.h matmul (C += A.B^T, sequential k) + row argmax + as-built stub
    pose, on host threads (ctypes releases the GIL).  'reference' when the reference's own
    header was compiled into oracle/_ref, else the oracle's restatement ('port')."""
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
    threads = max(1, min(16, (os.cpu_count() or 1)))
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
    # single-core reference point
    C = np.zeros((n, n), np.float32)
    t1 = time.perf_counter()
    mm(n, n, KD, P(A), P(Bm), P(C))
    one = time.perf_counter() - t1
    return {"value": total / dt, "unit": "pairs/s", "cores": threads, "kind": kind,
            "sample": "%d pairs of %dx%dx%d fp32 matmul + row argmax over %.1f s on %d host threads "
                      "(gemmini_functions_cpu.h:14-56 order, gcc -O2); 1 core: %.1f ms/pair"
                      % (total, n, n, KD, dt, threads, one * 1e3)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import mvtrack

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B, n = args.batch, args.kp

    d0, d1, kp0, kp1 = gen_batch(torch, dev, B, n, seed=pair_seed(rank, 0))
    nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
    P_ = max(1, args.pipeline)
    idxs = [torch.empty((B, n), dtype=torch.int32, device=dev) for _ in range(P_)]
    score = torch.empty((B, n), dtype=torch.float32, device=dev)
    Ts = [torch.empty((B, 3, 4), dtype=torch.float32, device=dev) for _ in range(P_)]
    nmatches = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P_)]
    ninls = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P_)]
    statuses = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P_)]
    idx, T, nmatch, ninl, status = idxs[0], Ts[0], nmatches[0], ninls[0], statuses[0]

    # --pipeline P: P contexts, each with its own stream, take the batches in turn.  A
    # context's prepare (k_ap_split of its next batch) waits only for its own previous run,
    # so it overlaps the other contexts' matches, and its pose overlaps them too -- the host
    # pipelining a user would do with P streams; the library calls are the same.
    P = max(1, args.pipeline)
    ctxs, streams = [], []
    for _ in range(P):
        c = mvtrack.Context(local)
        st_ = torch.cuda.Stream(device=dev) if P > 1 else torch.cuda.current_stream()
        c.set_stream(st_)
        c.set_allpairs_screen(args.screen)
        c.reserve(B, n)
        ctxs.append(c)
        streams.append(st_)
    ctx = ctxs[0]
    import synth

    K = synth.KITTI_K
    pose_p = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                                 hypotheses=args.hypotheses, inlier_thresh=1.0, refine_iters=10, seed=7)

    # pipelined across steps: frame 1 of the next batch is staged (k_ap_split, auxiliary
    # stream) while this batch's pose runs; every step still does all of its own work
    # the reference keeps only the matched pairs (pairwise_pnp.py:649-657): no score output,
    # so the exact re-score runs only where the rounding window does not decide the row
    # (indices bit-identical to the with-score mode; tests/test_gpu_allpairs.py)
    out_score = [None]
    turn = [0]

    fused = args.screen == "i8" and not args.unfused

    def step():
        c = turn[0] % P
        turn[0] += 1
        cx = ctxs[c]
        if fused:  # this batch's match + this context's next batch staged, one launch
            cx.match_allpairs_f32_run_prepare(d0, d1, nn_, nn_, idxs[c], out_score[0], d1, nn_, 0.8)
        else:
            cx.match_allpairs_f32_run(d0, d1, nn_, nn_, idxs[c], out_score[0], 0.8)
            cx.match_allpairs_f32_prepare(d1, nn_)  # this context's next batch
        cx.pose_from_matches(pose_p, nn_, idxs[c], kp0, kp1, Ts[c], nmatches[c], ninls[c], statuses[c])

    for cx in ctxs:
        cx.match_allpairs_f32_prepare(d1, nn_)

    mvtrack.profile_enable(False)
    sync = torch.cuda.synchronize
    barrier = dist.barrier if world > 1 else (lambda: None)

    # the headline: an unprofiled loop (no per-kernel events inside the measured wall time)
    elapsed = timed_loop(step, args.steps, args.warmup, sync, barrier)
    elapsed = max_over_ranks(torch, dist, elapsed, dev)
    # per-kernel durations for the roofline and the stage split: a second, profiled loop of
    # the same steps on ONE context (hipEvents on each kernel's own launch stream; with P > 1
    # the kernels of different contexts overlap and their event times would include each other)
    def prof_step():
        turn[0] = 0
        step()

    sync()
    mvtrack.profile_enable(True)
    timed_loop(prof_step, args.steps, 0, sync, barrier)
    mvtrack.profile_enable(False)
    screen = ctxs[0].allpairs_screen()
    kmatch, ksplit = ("k_q8_match", "k_q8_split") if screen == "i8" else ("k_ap_match", "k_ap_split")
    k_ms, k_n = mvtrack.profile_query(kmatch)
    s_ms, s_n = mvtrack.profile_query(ksplit)
    p_ms, p_n = mvtrack.profile_query("k_pose_ransac")
    # the same loop with the exact score materialised for every match (secondary, untimed by
    # the headline): what an API user asking for scores gets
    with_scores = None
    if args.score_steps > 0:
        out_score[0] = score
        for _ in range(2):
            step()
        sync()
        el_s = max_over_ranks(torch, dist, timed_loop(step, args.score_steps, 0, sync, barrier), dev)
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

    # correctness of the timed outputs on a few pairs (outside the timed region)
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

    sums = gather_checksums(torch, dist, [float(nmatch.sum().item()), float(ok)], dev)
    pairs_total = B * args.steps * world
    value = pairs_total / elapsed
    flops_pair = 2.0 * n * n * KD
    screen_avg_s = (k_ms / max(k_n, 1)) * 1e-3
    achieved = flops_pair * B / screen_avg_s / 1e12
    traffic, traffic_src = pmc_traffic(kmatch, B, n, fused)
    if screen == "i8":
        # k_q8_match reads frame 0 as fp32 (1 KiB per row) and frame 1's int8 image (256 B +
        # a 4-B scale per row), writes 4 B per row; 2 n0 n1 256 int8 ops per pair.  Fused, it
        # also stages the next batch's frame 1: 1 KiB read, 256 + 12 B written per row
        bytes_launch = B * n * (KD * 4 + KD + 4 + 4) + (B * n * (KD * 4 + KD + 12) if fused else 0)
        peak_c, c_note = I8_PEAK_TOPS, ("algorithmic 2*n0*n1*256 ops per pair on v_mfma_i32_32x32x32_i8 (int8 "
                                        "screen with a rigorous quantisation window, exact fp32 re-score)")
    else:
        bytes_launch = B * n * KD * (4 + 2)
        peak_c, c_note = FP16_PEAK_TFLOPS, ("algorithmic 2*n0*n1*256 FLOP per pair on v_mfma_f32_32x32x16_f16 "
                                            "(fp16 screen, exact fp32 re-score of the screen maximiser)")
    gbs = bytes_launch / screen_avg_s / 1e9
    frac_c, frac_m = achieved / peak_c, gbs / HBM_PEAK_GBS
    if frac_c >= frac_m:
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak_c,
                "unit": "TFLOP/s" if screen != "i8" else "TOP/s", "frac": round(frac_c, 4),
                "other": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(frac_m, 4)}}
    else:
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(frac_m, 4),
                "other": {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak_c,
                          "unit": "TFLOP/s" if screen != "i8" else "TOP/s", "frac": round(frac_c, 4)}}
    out = {
        "metric": "tracked frame-pairs/sec (match+PnP), 1024kp x 256-D KITTI shape",
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
        "data": "synthetic: unit-norm N(0,1) 256-D descriptors, 60% re-observed (+noise |0.3|), exact "
                "projections of a 3-D scene under outputs/transform_000785_000786.npy, KITTI K, 1241x376",
        "config": {"workload": "configs[1]: all-pairs match %dx%d kp x 256-D fp32 + RANSAC/GN pose per pair"
                               % (n, n), "pairs_per_gpu_per_step": B, "kp": n, "dim": KD,
                   "pose": "8-point RANSAC %d hyp + cheirality + 10 GN iters" % args.hypotheses,
                   "scores": "not materialised (pairwise_pnp.py keeps only the matched pairs); "
                             "indices bit-exact; see with_scores",
                   "parallelism": "pairs sharded one process per GPU (dp%d), no collective" % world},
        "roofline": dict(roof, kernel=kmatch, note=c_note, traffic=traffic, traffic_source=traffic_src,
                         algorithmic_ops_per_launch=flops_pair * B, algorithmic_bytes_per_launch=bytes_launch,
                         avg_launch_ms=round(screen_avg_s * 1e3, 4), launches=k_n),
        "screen": screen,
        "staging": "fused into k_q8_match (next batch)" if fused else "k_q8_split on the auxiliary stream",
        "stages_ms_per_step": {ksplit: round(s_ms / max(s_n, 1), 4),
                               kmatch: round(k_ms / max(k_n, 1), 4),
                               "k_pose_ransac": round(p_ms / max(p_n, 1), 4)},
        "with_scores": with_scores,
        "checked_pairs": checked, "pose_ok": int(sum(float(x[1]) for x in sums)),
        "matches_per_pair": round(sum(float(x[0]) for x in sums) / (B * world), 1),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, n)
    if rank == 0 and world == 1 and args.window_steps > 0:
        # north-star secondary: HBM roofline of the windowed match kernel, timed
        # after (and outside) the headline measurement
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_window

        w, _ = bench_window.run(batch=1024, steps=args.window_steps, warmup=2, check=1)
        out["window_frontend"] = {k: w[k] for k in ("metric", "value", "unit", "ms_per_step", "semantics",
                                                     "stages_ms", "hbm_roofline", "checked_pairs")}
    if rank == 0 and world == 1 and args.extra_steps > 0:
        # the other single-GPU configs beside the headline (not its value): BASELINE config 5
        # (int8 all-pairs, 2048 kp) and SURVEY §8(f)2 keypoint extraction, timed after it
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_i8
        import bench_keypoints

        r = bench_i8.run(batch=2048, kp=2048, steps=args.extra_steps, warmup=2, check=1)
        out["i8_allpairs"] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "stages_ms",
                                                  "mfma_roofline", "checked_pairs")}
        import bench_sequence

        # the headline's workload as a TRACK (consecutive frames, each quantised once)
        r = bench_sequence.run(frames=B + 1, kp=n, steps=args.extra_steps, warmup=2, check=1, pipeline=P)
        out["sequence"] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "pairs_per_step", "stages_ms",
                                              "staging", "hbm_roofline", "checked_pairs", "pose_ok")}
        r = bench_keypoints.run(batch=1024, steps=args.extra_steps, warmup=2, check=1)
        out["keypoints"] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "stages_ms",
                                               "hbm_roofline", "checked_frames")}
    if rank == 0:
        print(json.dumps(out), flush=True)
    for cx in ctxs:
        cx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
