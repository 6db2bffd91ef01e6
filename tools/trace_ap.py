"""Phase timing of k_ap_match (library built with EXTRA=-DAP_EXP_TRACE): per (block, wave)
s_memtime stamps at entry, A converted, ring primed, sweep done, last fold + merge done,
row decisions done, wide rows done."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
sys.path.insert(0, ROOT)
import mvtrack  # noqa: E402
import bench  # noqa: E402

B, n = int(os.environ.get("B", 1024)), 1024
dev = torch.device("cuda", 0)
d0, d1, kp0, kp1 = bench.gen_batch(torch, dev, B, n, seed=1000)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
sc = torch.empty((B, n), dtype=torch.float32, device=dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
ctx.reserve(B, n)
scores = os.environ.get("SCORES", "0") == "1"  # default: the bench's indices-only mode
for _ in range(3):
    ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, sc if scores else None, 0.8)
torch.cuda.synchronize()
nblk = B * (n // int(os.environ.get("BM", 128)))
NWV = int(os.environ.get("NW", 4))
buf = np.zeros(nblk * NWV * 10, np.uint64)
lib = mvtrack.lib()
lib.mv_debug_ap_trace.argtypes = [ctypes.c_void_p, ctypes.c_long]
assert lib.mv_debug_ap_trace(buf.ctypes.data, buf.nbytes) == 0
tr = buf.reshape(nblk, NWV, 10).astype(np.int64)
st = tr[:, :, :8]
d = np.diff(st, axis=2)
names = ["A-load", "prime", "sweep", "fold+merge", "decide", "wide", "-"]
print("per-wave phase cycles (median / p10 / p90 / max):")
for k, nm in enumerate(names[:6]):
    v = d[:, :, k].ravel()
    print("  %-10s %9.0f %9.0f %9.0f %9.0f" % (nm, np.median(v), np.percentile(v, 10), np.percentile(v, 90), v.max()))
tot = st[:, :, 7] - st[:, :, 0]
print("  wave total median %.0f  (sweep per 64-col tile %.0f)" % (np.median(tot), np.median(d[:, :, 2]) / (n / 64)))
sm = tr[:, 0, 8]
start, end = st[:, :, 0].min(1), st[:, :, 7].max(1)
cu = np.unique(sm)[0]
sel = np.where(sm == cu)[0]
o = sel[np.argsort(start[sel])]
rt = tr[:, 0, 9]
if rt[o[-1]] != rt[o[0]]:
    print("SCLK over the CU's run: %.3f GHz" % ((end[o[-1]] - end[o[0]]) / ((rt[o[-1]] - rt[o[0]]) / 100e6) / 1e9))

# timeline of the first CU: per block (wave 0) start / A converted / sweep done / end, in
# thousands of cycles from the CU's first start -- co-resident blocks in or out of phase?
t0 = start[o[0]]
print("CU %d timeline (kcycles): start  A-done  sweep-done  end" % cu)
for b in o[:12]:
    print("  blk %6d  %7.1f %7.1f %7.1f %7.1f" % (b, (st[b, 0, 0] - t0) / 1e3, (st[b, 0, 1] - t0) / 1e3,
                                                (st[b, 0, 3] - t0) / 1e3, (end[b] - t0) / 1e3))
# chip-wide: fraction of wave-time spent in A-load
print("A-load share of wave time: %.3f" % (d[:, :, 0].sum() / tot.sum()))
