"""Standalone k_ap_split (frame-1 fp32 -> 2^14-scaled fp16 image + |b|^2): HBM rate."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "maveric-slam_amd"))
import mvtrack  # noqa: E402

B, n, D = int(os.environ.get("B", 1024)), 1024, 256
dev = torch.device("cuda", 0)
d1 = torch.randn((B, n, D), device=dev) * 0.06
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
ctx.reserve(B, n)
for _ in range(3):
    ctx.match_allpairs_f32_prepare(d1, nn_)
torch.cuda.synchronize()
mvtrack.profile_enable(True)
t0 = time.perf_counter()
steps = 20
for _ in range(steps):
    ctx.match_allpairs_f32_prepare(d1, nn_)
torch.cuda.synchronize()
el = time.perf_counter() - t0
mvtrack.profile_enable(False)
ms, c = mvtrack.profile_query("k_ap_split")
kms = ms / max(c, 1)
byts = B * n * D * (4 + 2)
print(json.dumps({"k_ap_split_ms": round(kms, 4), "GBps": round(byts / (kms * 1e-3) / 1e9, 1),
                  "wall_ms": round(el / steps * 1e3, 4)}))
