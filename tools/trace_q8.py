"""Phase timing of k_q8_match (library built with EXTRA=-DQ8_EXP_TRACE): per (block, wave)
s_memtime stamps at entry, A quantised, ring primed, sweep done, decisions done, wide rows
done; plus one CU's block timeline (do co-resident blocks overlap their A loads?)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "maveric-slam_amd"))
sys.path.insert(0, ROOT)
import mvtrack  # noqa: E402
from bench import gen_batch  # noqa: E402

B, n = int(os.environ.get("B", 1024)), 1024
dev = torch.device("cuda", 0)
d0, d1, _, _ = gen_batch(torch, dev, B, n, seed=1000)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
ctx.reserve(B, n)
for _ in range(3):
    ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, None, 0.8)
torch.cuda.synchronize()
nblk = min(B * ((n + 255) // 256), 8192)
buf = np.zeros(nblk * 4 * 10, np.uint64)
lib = mvtrack.lib()
lib.mv_debug_q8_trace.argtypes = [ctypes.c_void_p, ctypes.c_long]
assert lib.mv_debug_q8_trace(buf.ctypes.data, buf.nbytes) == 0
tr = buf.reshape(nblk, 4, 10).astype(np.int64)
st = tr[:, :, :6]
d = np.diff(st, axis=2)
names = ["A-load+quant", "prime", "sweep", "decide", "wide"]
print("per-wave phase cycles (median / p10 / p90 / max):")
for k, nm in enumerate(names):
    v = d[:, :, k].ravel()
    print("  %-13s %9.0f %9.0f %9.0f %9.0f" % (nm, np.median(v), np.percentile(v, 10), np.percentile(v, 90), v.max()))
tot = st[:, :, 5] - st[:, :, 0]
print("  wave total median %.0f  (sweep per tile %.0f)" % (np.median(tot), np.median(d[:, :, 2]) / (n / 64)))
sm = tr[:, 0, 8]
start, end = st[:, :, 0].min(1), st[:, :, 5].max(1)
t0 = start.min()
print("distinct CUs", len(np.unique(sm)), "blocks", nblk, "kernel span (cycles) %d" % (end.max() - t0))
for cu in np.unique(sm)[:2]:
    sel = np.where(sm == cu)[0]
    o = sel[np.argsort(start[sel])]
    print("CU", cu, "timeline: start, A-done, primed, sweep-done, end (cycles from kernel start)")
    for b in o[:12]:
        print("  blk %5d  %8d %8d %8d %8d %8d" % (b, start[b] - t0, st[b, :, 1].max() - t0, st[b, :, 2].max() - t0,
                                                 st[b, :, 3].max() - t0, end[b] - t0))
rt = tr[:, 0, 9]
e5 = st[:, 0, 5]
a, b = np.argmin(rt), np.argmax(rt)
if rt[b] != rt[a]:
    print("SCLK: %.3f GHz" % ((e5[b] - e5[a]) / ((rt[b] - rt[a]) / 100e6) / 1e9))
