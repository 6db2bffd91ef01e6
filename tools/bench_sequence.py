#!/usr/bin/env python3
"""Sequence mode of the headline (mv_match_sequence_f32_dev + pose): a track of consecutive
frames as the reference's driver runs them (scripts/run_pairwise_pnp.sh:7-20, pair = frames
i, i + 1), 1024 kp x 256-D fp32, every frame quantised once (k_q8_split over the chunk's
frames) and matched as frame 1 of one pair and frame 0 of the next (k_q8_match<AI8>), then
the headline's pose per pair.  One step = one chunk of FRAMES frames = FRAMES - 1 pairs; P
contexts on P streams take the chunks in turn.  Synthetic track: frame b + 1 re-observes 60 %
of frame b (+ noise |0.3|); each pair's keypoints are exact projections under the 785 -> 786
pose for its re-observed rows (as bench.gen_batch); see gen_track.  Prints one JSON line.  GPU only."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mvtrack  # noqa: E402

KD = 256
HBM_PEAK_GBS = 8000.0


def gen_track(dev, F, n, seed):
    """F consecutive frames [F][n][256] and per-pair keypoints [F-1][n][2] x 2, in a few
    launches: landmarks along the track, frame b observes landmarks b s .. b s + n - 1 (s = 0.4 n,
    so 60 % of frame b is re-observed by frame b + 1) in a random row order, each observation
    the landmark's unit descriptor + noise |0.3| / sqrt 2 per frame (|0.3| between frames)."""
    import synth

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    m = int(round(0.6 * n))
    sh = n - m
    base = torch.randn(((F - 1) * sh + n, KD), generator=g, device=dev)
    base = base / base.norm(dim=1, keepdim=True)
    perm = torch.argsort(torch.rand((F, n), generator=g, device=dev), dim=1)  # row -> local landmark
    lid = perm + torch.arange(F, device=dev)[:, None] * sh
    d = base[lid] + torch.randn((F, n, KD), generator=g, device=dev) * (0.3 / 16.0 / np.sqrt(2.0))
    d = d / d.norm(dim=2, keepdim=True)
    del base
    rng = np.random.default_rng(seed)
    perm_h = perm.cpu().numpy()
    inv = np.argsort(perm_h, axis=1)  # local landmark -> row
    kp0 = np.empty((F - 1, n, 2), np.float32)
    kp1 = np.empty((F - 1, n, 2), np.float32)
    R, t = synth.T_785_786[:, :3], synth.T_785_786[:, 3]
    for b in range(F - 1):
        _, x0, x1 = synth.synth_scene(rng, n, R, t)
        k1 = np.stack([rng.uniform(0, synth.KITTI_W, n), rng.uniform(0, synth.KITTI_H, n)], 1)
        loc = perm_h[b + 1]  # frame b + 1's rows: local landmark; re-observed when loc < m
        re = loc < m
        k1[re] = x1[inv[b][loc[re] + sh]]  # the frame-b row of the same landmark
        kp0[b] = x0
        kp1[b] = k1
    return d.contiguous(), torch.from_numpy(kp0).to(dev), torch.from_numpy(kp1).to(dev)


def run(frames=8193, kp=1024, steps=20, warmup=3, check=1, pipeline=3, fused=True):
    import synth

    dev = torch.device("cuda", 0)
    F, n, P = frames, kp, max(1, pipeline)
    B = F - 1
    d, kp0, kp1 = gen_track(dev, F, n, seed=4242)
    nf = torch.full((F,), n, dtype=torch.int32, device=dev)
    nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
    K = synth.KITTI_K
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                              hypotheses=256, inlier_thresh=1.0, refine_iters=10, seed=7)
    ctxs, outs = [], []
    for _ in range(P):
        c = mvtrack.Context(0)
        c.set_stream(torch.cuda.Stream(device=dev) if P > 1 else torch.cuda.current_stream())
        c.reserve(F, n)
        ctxs.append(c)
        outs.append(dict(idx=torch.empty((B, n), dtype=torch.int32, device=dev),
                         T=torch.empty((B, 3, 4), dtype=torch.float32, device=dev),
                         nm=torch.empty(B, dtype=torch.int32, device=dev),
                         ni=torch.empty(B, dtype=torch.int32, device=dev),
                         st=torch.empty(B, dtype=torch.int32, device=dev)))
    turn = [0]

    def step():
        c = turn[0] % P
        turn[0] += 1
        o = outs[c]
        if fused:  # this chunk's match + this context's next chunk staged, one launch
            ctxs[c].match_sequence_f32_run_prepare(d, nf, o["idx"], None, d, nf, 0.8)
        else:
            ctxs[c].match_sequence_f32(d, nf, o["idx"], None, 0.8)
        ctxs[c].pose_from_matches(prm, nn_, o["idx"], kp0, kp1, o["T"], o["nm"], o["ni"], o["st"])

    torch.cuda.synchronize()
    if fused:
        for c in ctxs:
            c.match_allpairs_f32_prepare(d, nf)  # the first chunk's frame images
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # per-kernel averages: a second loop on ONE context (no overlap inside the events)
    mvtrack.profile_enable(True)
    for _ in range(steps):
        turn[0] = 0
        step()
    torch.cuda.synchronize()
    mvtrack.profile_enable(False)
    st = {k: mvtrack.profile_query(k) for k in ("k_q8_split", "k_q8_match_seq", "k_q8t_match", "k_q8t_rescan", "k_q8d_handback",
                                                 "k_pose_ransac")}
    stages = {k: round(ms / max(c, 1), 4) for k, (ms, c) in st.items() if c > 0}
    o = outs[0]
    checked = 0
    if check > 0:
        import oracle

        for b in sorted({0, B - 1}):
            i2, _ = oracle.allpairs_f32(d[b].cpu().numpy(), d[b + 1].cpu().numpy(), 0.8)
            assert (o["idx"][b].cpu().numpy() == i2).all(), "sequence match differs from the oracle"
            checked += 1
    ok = int((o["st"] == 0).sum().item())
    R = o["T"][:, :, :3].double().cpu().numpy()
    err = np.abs(R - synth.T_785_786[None, :, :3]).max(axis=(1, 2))
    assert ok == B and float(err.max()) < 1e-3, "pose failed: ok=%d max|dR|=%g" % (ok, err.max())
    for c in ctxs:
        c.close()
    # algorithmic bytes of k_q8_match_seq: every frame's image read ONCE (int8 row + s + |b|^2 +
    # |eps|^2 = 268 B per row; pair b's frame 1 is pair b + 1's frame 0 -- the same bytes, and
    # rocprof counts them once: profiles/r02i_seq_summary.json, 1.003x this figure), the
    # index (4 B per row); fused: the next chunk's staging (per row 1 KiB read + 268 B written)
    split_bytes = F * n * (KD * 4 + 268)
    seq_bytes = F * n * 268 + B * n * 4 + (split_bytes if fused else 0)
    kseq = "k_q8_match_seq"
    if "k_q8t_match" in stages:  # the default screen: the one-pass kernel over the pairs in place --
        kseq = "k_q8t_match"     # both fp32 frames of every pair read (2 x 1 KiB per row) + the index
        seq_bytes = B * n * (2 * KD * 4 + 4)
        fused = False
    mseq = stages[kseq] * 1e-3
    return {
        "metric": "tracked frame-pairs/sec, sequence mode (consecutive frames), "
                  "1024kp x 256-D KITTI shape",
        "value": round(B * steps / el, 2), "unit": "pairs/s", "ms_per_step": round(el / steps * 1e3, 4),
        "frames_per_step": F, "pairs_per_step": B, "pipeline": P, "stages_ms": stages,
        "staging": ("none: k_q8t_match reads the fp32 frames in place (pair b = frames b, b + 1)"
                    if kseq == "k_q8t_match" else
                    "fused into k_q8_match_seq (next chunk)" if fused else "k_q8_split per chunk"),
        "hbm_roofline": {"kernel": kseq, "bytes_per_launch": seq_bytes,
                         "GBs": round(seq_bytes / mseq / 1e9, 1) if mseq > 0 else None,
                         "frac": round(seq_bytes / mseq / 1e9 / HBM_PEAK_GBS, 4) if mseq > 0 else None,
                         "includes_next_chunk_staging": fused, "peak_GBs": HBM_PEAK_GBS},
        "checked_pairs": checked, "pose_ok": ok,
        "data": "synthetic track: frame b+1 re-observes 60% of frame b (+noise |0.3|), exact projections "
                "under outputs/transform_000785_000786.npy per pair",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8193, help="frames per step (pairs = frames - 1)")
    ap.add_argument("--kp", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--pipeline", type=int, default=3)
    ap.add_argument("--unfused", action="store_true", help="split each chunk with k_q8_split instead")
    args = ap.parse_args()
    r = run(args.frames, args.kp, args.steps, args.warmup, args.check, args.pipeline, not args.unfused)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
