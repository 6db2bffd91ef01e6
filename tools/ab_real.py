"""The all-pairs match on SuperPoint's own descriptors (the image -> pose chain's consecutive pairs:
tools/bench_image_pose.py's KITTI track through mv_superpoint_forward_raw_dev + mv_keypoints_dev),
timed alone: k_q8t_match (default) or k_q8d_match (MV_Q8_KERNEL=d).  With a tracing build
(MV_LIB=build_variants/libmaveric_trace.so, tools/build_variant.sh trace -DMV_TRACE) also the
per-wave phase cycles of k_q8t_match (A phase, sweep, epilogue).  Env: F frames (257), THR (0.8)."""
import ctypes
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
from bench_image_pose import CAP, frames_kitti  # noqa: E402

F = int(os.environ.get("F", "257"))
THR = float(os.environ.get("THR", "0.8"))
P = F - 1
dev = torch.device("cuda", 0)
W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
x = torch.from_numpy(np.stack(frames_kitti(F))).to(dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
sp = mvtrack.SuperPoint(ctx, W)
semi = torch.empty((F, 65, 24, 80), dtype=torch.float32, device=dev)
cdesc = torch.empty((F, 256, 24, 80), dtype=torch.float32, device=dev)
nkp = torch.empty(F, dtype=torch.int32, device=dev)
kp = torch.zeros((F, CAP, 2), dtype=torch.float32, device=dev)
conf = torch.zeros((F, CAP), dtype=torch.float32, device=dev)
desc = torch.zeros((F, CAP, 256), dtype=torch.float32, device=dev)
kst = torch.empty(F, dtype=torch.int32, device=dev)
sp.forward_raw(x, 192, 640, out=(semi, cdesc))
ctx.keypoints(semi, cdesc, 192, 640, nkp, kp, conf, desc, kst)
idx = torch.empty((P, CAP), dtype=torch.int32, device=dev)


def call():
    ctx.match_allpairs_f32(desc[:P], desc[1:], nkp[:P], nkp[1:], idx, None, THR)


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
for k in ("k_q8t_match", "k_q8t_rescan", "k_q8d_handback", "k_q8d_match"):
    ms, c = mvtrack.profile_query(k)
    if c:
        st[k] = round(ms / steps, 4)
res = {"kernel": "d" if os.environ.get("MV_Q8_KERNEL", "")[:1] == "d" else "t", "pairs": P, "thresh": THR,
       "keypoints_mean": round(float(nkp.float().mean()), 1), "matches_mean": round(float((idx >= 0).sum()) / P, 1),
       "call_ms": round(el * 1e3, 4), "stages_ms": st}
lib = mvtrack.lib()
if hasattr(lib, "mv_debug_direct_trace") and res["kernel"] == "t":
    call()
    torch.cuda.synchronize()
    buf = np.zeros(P * 8 * 10, np.uint64)
    lib.mv_debug_direct_trace.argtypes = [ctypes.c_void_p, ctypes.c_long]
    assert lib.mv_debug_direct_trace(buf.ctypes.data, buf.nbytes) == 0
    tr = buf.reshape(P, 8, 10).astype(np.int64)
    d = np.diff(tr[:, :, :4], axis=2)
    res["phase_cycles_median_p90_max"] = {
        nm: [float(np.median(d[:, :, k])), float(np.percentile(d[:, :, k], 90)), float(d[:, :, k].max())]
        for k, nm in enumerate(["A", "sweep", "epilogue"])}
    c = tr[:, :, 8]
    wide, need = (c >> 16).sum(1), (c & 0xffff).sum(1)  # per pair (workgroup)
    res["wide_rows_per_pair_mean_p90_max"] = [float(wide.mean()), float(np.percentile(wide, 90)), int(wide.max())]
    res["deferred_dots_per_pair_mean"] = float(need.mean())
print(json.dumps(res))
sp.close()
ctx.close()
