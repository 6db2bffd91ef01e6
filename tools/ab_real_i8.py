"""configs[4]'s int8 all-pairs on the NETWORK's own int8 descriptors: the SuperPoint forward of a
257-frame KITTI track (tools/bench_image_pose.py's frames), each frame's 1920 cells x 256 codes,
consecutive frames matched (256 pairs, cap 2048).  Times k_i8t_match (default) or k_i8_match
(MV_I8_KERNEL=m, set by the caller) and reports the matches per pair."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import mvtrack  # noqa: E402
from bench_image_pose import frames_kitti  # noqa: E402

F, cap = 257, 2048
P = F - 1
dev = torch.device("cuda", 0)
W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
x = torch.from_numpy(np.stack(frames_kitti(F))).to(dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
sp = mvtrack.SuperPoint(ctx, W)
_, desc, _, _ = sp.forward(x, 192, 640)
cells = desc.shape[1]
D = torch.zeros((F, cap, 256), dtype=torch.int8, device=dev)
D[:, :cells] = desc
nn_ = torch.full((P,), cells, dtype=torch.int32, device=dev)
idx = torch.empty((P, cap), dtype=torch.int32, device=dev)
dot = torch.empty((P, cap), dtype=torch.int32, device=dev)


def call():
    ctx.match_allpairs_i8(D[:P], D[1:], nn_, nn_, idx, dot)


for _ in range(3):
    call()
torch.cuda.synchronize()
steps = 20
t0 = time.perf_counter()
for _ in range(steps):
    call()
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / steps
mvtrack.profile_enable(True)
for _ in range(steps):
    call()
torch.cuda.synchronize()
mvtrack.profile_enable(False)
st = {}
for k in ("k_i8_prep", "k_i8t_match", "k_i8t_rescan", "k_i8m_handback", "k_i8_norms", "k_i8_match"):
    ms, c = mvtrack.profile_query(k)
    if c:
        st[k] = round(ms / steps, 4)
print(json.dumps({"kernel": "m" if os.environ.get("MV_I8_KERNEL", "")[:1] == "m" else "t", "pairs": P, "cells": cells,
                  "matches_per_pair": round(float((idx[:, :cells] >= 0).sum()) / P, 1),
                  "call_ms": round(el * 1e3, 4), "stages_ms": st}))
sp.close()
ctx.close()
