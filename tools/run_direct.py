"""A short workload for counter passes: k_q8d_match on the headline batch (bench.gen_batch),
3 launches (the profiler averages per launch)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "maveric-slam_amd"))
import bench  # noqa: E402
import mvtrack  # noqa: E402

B, n = int(os.environ.get("TB", "8192")), 1024
dev = torch.device("cuda", 0)
d0, d1, _, _ = bench.gen_batch(torch, dev, B, n, seed=3)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
ctx.set_allpairs_screen(os.environ.get("SCREEN", "i8"))
for _ in range(3):
    ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None)
torch.cuda.synchronize()
print("ok", int((idx >= 0).sum()))
