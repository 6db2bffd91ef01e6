"""Bit-determinism of the headline step (all-pairs match + pose) under concurrent streams: NP
contexts on their own streams run the same batch (bench.gen_batch, noisy keypoints so that the
pose refines) ROUNDS times back to back; every context's matches and poses are compared with a
solo run.  MV_LIB selects a build variant."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import mvtrack  # noqa: E402
import synth  # noqa: E402

NP, ROUNDS, B, n = int(os.environ.get("NP", "3")), int(os.environ.get("ROUNDS", "6")), int(os.environ.get("B", "4096")), 1024
dev = torch.device("cuda", 0)
d0, d1, kp0, kp1 = bench.gen_batch(torch, dev, B, n, seed=1)
kp1 = bench.noisy_keypoints(torch, dev, kp1)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
K = synth.KITTI_K
prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2], hypotheses=256,
                          inlier_thresh=1.0, refine_iters=10, seed=7)
torch.cuda.synchronize()


class C:
    def __init__(self):
        self.s = torch.cuda.Stream(device=dev)
        self.ctx = mvtrack.Context(0)
        self.ctx.set_stream(self.s)
        z = lambda *sh, dt=torch.int32: torch.zeros(sh, dtype=dt, device=dev)  # noqa: E731
        self.idx, self.T = z(B, n), z(B, 3, 4, dt=torch.float32)
        self.nm, self.ni, self.st = z(B), z(B), z(B)

    def step(self):
        with torch.cuda.stream(self.s):
            self.ctx.match_allpairs_f32(d0, d1, nn_, nn_, self.idx, None, 0.8)
            self.ctx.pose_from_matches(prm, nn_, self.idx, kp0, kp1, self.T, self.nm, self.ni, self.st)


cs = [C() for _ in range(NP)]
cs[0].step()
torch.cuda.synchronize()
ref_idx, ref_T = cs[0].idx.clone(), cs[0].T.clone()
for _ in range(ROUNDS):
    for c in cs:
        c.step()
torch.cuda.synchronize()
for i, c in enumerate(cs):
    di = int((c.idx != ref_idx).sum())
    dT = (c.T != ref_T).reshape(B, -1).any(1)
    print("context %d: idx elements differing %d, poses differing %d" % (i, di, int(dT.sum())))
print("done")
