"""Mismatch report: the reference's KITTI fixtures through match_allpairs_f32 under each screen,
padding (zero / garbage), cap and score-output mode, against the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "oracle")]
import mvtrack  # noqa: E402
import oracle as orc  # noqa: E402

dev = torch.device("cuda:0")
ctx = mvtrack.Context(0)
for name in ("pair0", "pair10"):
    d = np.load(os.path.join(ROOT, "tests/golden/tracking_%s.npz" % name))
    a, c = d["image0_desc"], d["image1_desc"]
    n0, n1 = a.shape[0], c.shape[0]
    i2, s2 = orc.allpairs_f32(a, c, 0.8)
    for scr in ("i8", "i8s", "f16"):
        ctx.set_allpairs_screen(scr)
        for pad in ("zero", "garbage"):
            for cap in (max(n0, n1), 512, 1024):
                for scores in (True, False):
                    rng = np.random.default_rng(0)
                    D0 = np.zeros((1, cap, 256), np.float32)
                    D1 = np.zeros((1, cap, 256), np.float32)
                    if pad == "garbage":
                        D0[:] = rng.standard_normal((1, cap, 256)) * 7
                        D1[:] = rng.standard_normal((1, cap, 256)) * 7
                    D0[0, :n0], D1[0, :n1] = a, c
                    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
                    idx = torch.full((1, cap), -7, dtype=torch.int32, device=dev)
                    sc = torch.zeros((1, cap), dtype=torch.float32, device=dev) if scores else None
                    ctx.set_stream(torch.cuda.current_stream())
                    ctx.match_allpairs_f32(t(D0), t(D1), t(np.array([n0], np.int32)), t(np.array([n1], np.int32)),
                                           idx, sc, 0.8)
                    torch.cuda.synchronize()
                    ctx.set_stream(None)
                    g = idx.cpu().numpy()[0, :n0]
                    bad = np.nonzero(g != i2)[0]
                    msg = "%s %s pad=%s cap=%d scores=%d: %d mismatches" % (name, scr, pad, cap, scores, len(bad))
                    if len(bad):
                        msg += " rows %s gpu %s oracle %s" % (bad[:6].tolist(), g[bad[:6]].tolist(), i2[bad[:6]].tolist())
                    print(msg, flush=True)
