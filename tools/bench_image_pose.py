#!/usr/bin/env python3
"""The fp32 path of python/pairwise_pnp.py:577-694 end to end on the GPU: a track of F KITTI-shape
8-bit frames (376 x 1241, the two committed KITTI 00 frames shifted / brightness-jittered) ->
the quantized SuperPoint network's float outputs (mv_superpoint_forward_raw_dev) -> keypoints +
descriptors (mv_keypoints_dev, cap 1024) -> the all-pairs match of consecutive frames
(mv_match_allpairs_f32_dev on the views desc[0:F-1], desc[1:F]) -> the pose per pair
(mv_pose_from_matches_dev).  One step = one track of F frames; prints one JSON line: frame-pairs/s
(image -> pose), per-stage times (HIP events) and the checked stages.  GPU only."""
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
import synth  # noqa: E402

CAP = 1024


def frames_kitti(F, seed=0):
    ims = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_images.npz"))
    base = [ims["img_000000"], ims["img_000001"]]
    rng = np.random.default_rng(seed)
    out = []
    for b in range(F):
        im = np.roll(base[b % 2], shift=(b // 2) % 17, axis=1).astype(np.int16) + rng.integers(-3, 4)
        out.append(np.clip(im, 0, 255).astype(np.uint8))
    return out


def run(frames=257, steps=10, warmup=2, check=1, pipelines=2):
    """pipelines: independent (context, SuperPoint net, buffers, HIP stream) sets taking the steps
    in turn, so that one track's latency-bound stages (keypoint NMS: one block per frame; the
    match and pose launches of 256 pairs) overlap the next track's network on the other stream,
    as the headline's pipelined contexts do.  Stage times are measured on one pipeline alone."""
    dev = torch.device("cuda", 0)
    W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
    imgs = frames_kitti(frames)
    x = torch.from_numpy(np.stack(imgs)).to(dev)
    F, P = frames, frames - 1
    K = synth.KITTI_K  # pairwise_pnp.py:667-669
    prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2], hypotheses=256,
                              inlier_thresh=1.0, refine_iters=10, seed=7)

    class Pipe:
        def __init__(self):
            self.stream = torch.cuda.Stream(device=dev)
            self.ctx = mvtrack.Context(0)
            self.ctx.set_stream(self.stream)
            self.sp = mvtrack.SuperPoint(self.ctx, W)
            e = lambda *shape, dt=torch.float32: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
            self.semi, self.cdesc = e(F, 65, 24, 80), e(F, 256, 24, 80)
            self.nkp, self.kp, self.conf = e(F, dt=torch.int32), e(F, CAP, 2), e(F, CAP)
            self.desc, self.kst = e(F, CAP, 256), e(F, dt=torch.int32)
            self.idx = e(P, CAP, dt=torch.int32)
            self.T, self.nm, self.ni, self.st = e(P, 3, 4), e(P, dt=torch.int32), e(P, dt=torch.int32), e(P, dt=torch.int32)

        def step(self):
            with torch.cuda.stream(self.stream):
                self.sp.forward_raw(x, 192, 640, out=(self.semi, self.cdesc))
                self.ctx.keypoints(self.semi, self.cdesc, 192, 640, self.nkp, self.kp, self.conf, self.desc, self.kst)
                self.ctx.match_allpairs_f32(self.desc[:P], self.desc[1:], self.nkp[:P], self.nkp[1:], self.idx, None,
                                            0.8)
                self.ctx.pose_from_matches(prm, self.nkp[:P], self.idx, self.kp[:P], self.kp[1:], self.T, self.nm,
                                           self.ni, self.st)

    torch.cuda.synchronize()  # the inputs uploaded on the default stream
    pipes = [Pipe() for _ in range(max(1, pipelines))]
    for k in range(warmup * len(pipes)):
        pipes[k % len(pipes)].step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        pipes[k % len(pipes)].step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    p0 = pipes[0]
    mvtrack.profile_enable(True)
    for _ in range(steps):
        p0.step()
        torch.cuda.synchronize()
    mvtrack.profile_enable(False)
    stages = {}
    for k in ("k_sp_conv", "k_kp_heat", "k_kp_nms", "k_kp_sample_planes", "k_kp_normalize",
              "k_q8t_match", "k_q8t_rescan", "k_q8d_handback", "k_q8d_match", "k_pose_ransac"):
        ms, c = mvtrack.profile_query(k)
        if c:
            stages[k] = round(ms / steps, 4)
    nkp, idx, nm, st, kp = p0.nkp, p0.idx, p0.nm, p0.st, p0.kp
    res = {"metric": "image -> pose frame-pairs/sec (quantized SuperPoint + keypoints + fp32 all-pairs + pose), "
                     "KITTI 376x1241 frames, consecutive pairs",
           "value": round(P * steps / el, 1), "unit": "pairs/s", "frames_per_step": F, "steps": steps,
           "pipelines": len(pipes), "ms_per_step": round(el / steps * 1e3, 4), "stages_ms_per_step": stages,
           "keypoints_per_frame": round(float(nkp.float().mean()), 1),
           "matches_per_pair": round(float(nm.float().mean()), 1), "pose_ok": int((st == 0).sum())}
    if check:
        import oracle

        net = oracle.sp_net(W)
        s_sc, d_sc = np.float32(W["convPb_meta"][2]), np.float32(W["convDb_meta"][2])
        chain = []
        for b in (0, 1):
            _, _, _, _, sr, dr = oracle.sp_forward(imgs[b], net)
            pts, dsc, _ = oracle.keypoints(s_sc * sr.astype(np.float32), d_sc * dr.astype(np.float32), 192, 640)
            n = int(nkp[b])
            assert n == pts.shape[0] and (kp[b, :n].cpu().numpy() == pts[:, :2]).all(), "keypoints differ"
            chain.append(dsc)
        i2, _ = oracle.allpairs_f32(chain[0], chain[1], 0.8)
        assert (idx[0, :i2.shape[0]].cpu().numpy() == i2).all(), "match differs from the oracle chain"
        res["checked_pairs"] = 1
        # the same track on every pipeline: every stage identical bit for bit, the pose included
        # (pose_diff_pairs must be 0: DESIGN 4.3 -- the pose runs beside the other pipeline's network)
        res["pose_diff_pairs"] = 0
        for i, pp in enumerate(pipes[1:], 1):
            bad = [k for k in ("semi", "cdesc", "nkp", "kp", "desc", "idx") if not torch.equal(getattr(pp, k),
                                                                                            getattr(p0, k))]
            assert not bad, "pipeline %d differs from pipeline 0 in %s" % (i, bad)
            d = (pp.T - p0.T).abs().amax(dim=(1, 2))
            res["pose_diff_pairs"] += int((d > 0).sum())
        assert res["pose_diff_pairs"] == 0, "poses differ across pipelines in %d pairs" % res["pose_diff_pairs"]
    for pp in pipes:
        pp.sp.close()
        pp.ctx.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=257)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--pipelines", type=int, default=2)
    a = ap.parse_args()
    print(json.dumps(run(a.frames, a.steps, a.warmup, a.check, a.pipelines)))


if __name__ == "__main__":
    main()
