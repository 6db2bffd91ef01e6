"""k_q8t_match (one workgroup per pair) against k_q8d_match (MV_Q8_KERNEL=d, set by the caller:
the choice is read once per process) over batch sizes and keypoint counts: where the one-pass
kernel stops paying (small batches leave CUs idle; its 1024-row workgroup is the latency).
Env: BS batch sizes (comma list), NS keypoints per frame (comma list), cap 1024.  One JSON line per
(batch, n): the match kernels' per-launch ms (HIP events) and the whole call."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "maveric-slam_amd"))
import bench  # noqa: E402
import mvtrack  # noqa: E402

cap = 1024
dev = torch.device("cuda", 0)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
kern = "d" if os.environ.get("MV_Q8_KERNEL", "")[:1] == "d" else "t"
for B in [int(x) for x in os.environ.get("BS", "128,256,512,1024,2048,4096").split(",")]:
    d0, d1, _, _ = bench.gen_batch(torch, dev, B, cap, seed=3, noise=0.3 / 16)
    for n in [int(x) for x in os.environ.get("NS", "400,1024").split(",")]:
        nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
        idx = torch.empty((B, cap), dtype=torch.int32, device=dev)
        for _ in range(3):
            ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None)
        torch.cuda.synchronize()
        steps = 20
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        mvtrack.profile_enable(True)
        for _ in range(steps):
            ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None)
        torch.cuda.synchronize()
        mvtrack.profile_enable(False)
        st = {}
        for k in ("k_q8t_match", "k_q8t_rescan", "k_q8d_handback", "k_q8d_match"):
            ms, c = mvtrack.profile_query(k)
            if c:
                st[k] = round(ms / steps, 4)
        print(json.dumps({"kernel": kern, "batch": B, "n": n, "call_ms": round(el * 1e3, 4), "stages_ms": st}),
              flush=True)
        del idx, nn_
    del d0, d1
ctx.close()
