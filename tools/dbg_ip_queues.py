#!/usr/bin/env python3
"""image -> pose line under bench.py-like process state: the line alone, then after EXTRA idle
HIP streams were created (bench.py's earlier lines leave their contexts' streams alive), then
after a 1-rank nccl process group.  GPU only (timing experiment)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
import torch  # noqa: E402

import bench_image_pose  # noqa: E402
import mvtrack  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "alone"
keep = []
if mode.startswith("streams"):
    for _ in range(int(mode[7:] or 1)):
        keep.append(torch.cuda.Stream(device=0))
elif mode.startswith("ctx"):
    for _ in range(int(mode[3:] or 1)):
        keep.append(mvtrack.Context(0))
elif mode in ("sp", "kp", "seq", "i8"):
    import bench_i8
    import bench_keypoints
    import bench_sequence
    import bench_superpoint
    if mode == "sp":
        bench_superpoint.run(batch=64, steps=10, warmup=2, check=0)
    elif mode == "kp":
        bench_keypoints.run(batch=1024, steps=10, warmup=2, check=0)
    elif mode == "seq":
        bench_sequence.run(frames=8193, kp=1024, steps=10, warmup=2, check=0, pipeline=3)
    else:
        bench_i8.run(batch=2048, kp=2048, steps=10, warmup=2, check=0)
elif mode == "nccl":
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.distributed.init_process_group("nccl", rank=0, world_size=1)
    t = torch.ones(4, device="cuda")
    torch.distributed.all_reduce(t)
    torch.cuda.synchronize()
r = bench_image_pose.run(frames=257, steps=10, warmup=2, check=0)
print(mode, r["value"], r["ms_per_step"])
