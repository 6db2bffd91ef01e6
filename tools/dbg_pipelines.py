"""Which stage differs between image -> pose pipelines run concurrently (tools/bench_image_pose.py
--pipelines N)?  Every pipeline takes the same track; after a reference run of pipeline 0 alone,
N pipelines run K rounds concurrently; each pipeline's stage outputs (network heads, keypoints,
descriptors, matches, poses) are compared with the reference, bit for bit."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import mvtrack  # noqa: E402
import synth  # noqa: E402
from bench_image_pose import CAP, frames_kitti  # noqa: E402

N = int(os.environ.get("NP", "3"))
ROUNDS = int(os.environ.get("ROUNDS", "4"))
F = 257
P = F - 1
dev = torch.device("cuda", 0)
W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
x = torch.from_numpy(np.stack(frames_kitti(F))).to(dev)
K = synth.KITTI_K
prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2], hypotheses=256,
                          inlier_thresh=1.0, refine_iters=10, seed=7)
NAMES = ("semi", "cdesc", "nkp", "kp", "desc", "idx", "T", "st")


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
            self.ctx.match_allpairs_f32(self.desc[:P], self.desc[1:], self.nkp[:P], self.nkp[1:], self.idx, None, 0.8)
            self.ctx.pose_from_matches(prm, self.nkp[:P], self.idx, self.kp[:P], self.kp[1:], self.T, self.nm, self.ni,
                                       self.st)

    def snap(self):
        return {k: getattr(self, k).clone() for k in NAMES}


torch.cuda.synchronize()
pipes = [Pipe() for _ in range(N)]
pipes[0].step()
torch.cuda.synchronize()
ref = pipes[0].snap()
pipes[0].step()
torch.cuda.synchronize()
print("pipeline 0 alone, twice:", {k: bool(torch.equal(v, ref[k])) for k, v in pipes[0].snap().items()})
SYNC = int(os.environ.get("SYNC", "1"))  # 0: rounds back to back (as the bench), compared at the end
for rd in range(ROUNDS):
    for p in pipes:
        p.step()
    if not SYNC and rd < ROUNDS - 1:
        continue
    torch.cuda.synchronize()
    for i, p in enumerate(pipes):
        s = p.snap()
        bad = [k for k in NAMES if not torch.equal(s[k], ref[k])]
        if bad:
            k = bad[0]
            d = (s[k] != ref[k])
            print("round %d pipeline %d differs in %s (first stage), %d elements; also %s" % (rd, i, k, int(d.sum()),
                                                                                           bad[1:]))
            if k in ("idx", "T", "st"):
                rows = torch.nonzero(d.reshape(d.shape[0], -1).any(1)).flatten()[:8].tolist()
                print("   pairs", rows)
if int(os.environ.get("PROF", "0")):  # pipeline 0 again with the stage timers on (the bench's profile pass)
    mvtrack.profile_enable(True)
    for _ in range(3):
        pipes[0].step()
        torch.cuda.synchronize()
    mvtrack.profile_enable(False)
    s = pipes[0].snap()
    print("pipeline 0 with stage timers:", {k: bool(torch.equal(v, ref[k])) for k, v in s.items()})
print("done")
