"""Phase timing of k_i8_match (library built with EXTRA=-DI8_EXP_TRACE): per (block, wave)
s_memtime stamps at kernel entry, A loaded, ring primed, main loop done, last fold done,
merge/candidate lists done, row decisions done, deep rows done."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "maveric-slam_amd"))
import mvtrack  # noqa: E402

B, n, D = 256, 2048, 256
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(5)
d0 = torch.clamp(torch.round(torch.randn((B, n, D), generator=g, device=dev) * 24), -128, 127).to(torch.int8)
d1 = torch.clamp(torch.round(torch.randn((B, n, D), generator=g, device=dev) * 24), -128, 127).to(torch.int8)
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
dot = torch.empty((B, n), dtype=torch.int32, device=dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
ctx.reserve(B, n)
for _ in range(3):
    ctx.match_allpairs_i8(d0, d1, nn_, nn_, idx, dot)
torch.cuda.synchronize()
nblk = B * ((n + 255) // 256)  # k_i8_match: 256 rows per block
buf = np.zeros(nblk * 4 * 10, np.uint64)
lib = mvtrack.lib()
lib.mv_debug_i8_trace.argtypes = [ctypes.c_void_p, ctypes.c_long]
assert lib.mv_debug_i8_trace(buf.ctypes.data, buf.nbytes) == 0
tr = buf.reshape(nblk, 4, 10).astype(np.int64)
st = tr[:, :, :8]
d = np.diff(st, axis=2)
names = ["A-load", "prime", "loop", "lastfold", "merge", "decide", "deep"]
np.set_printoptions(linewidth=160, suppress=True)
print("per-wave phase cycles (median / p10 / p90 / max):")
for k, nm in enumerate(names):
    v = d[:, :, k].ravel()
    print("  %-9s %9.0f %9.0f %9.0f %9.0f" % (nm, np.median(v), np.percentile(v, 10), np.percentile(v, 90), v.max()))
tot = st[:, :, 7] - st[:, :, 0]
print("  wave total median %.0f  (loop per tile %.0f)" % (np.median(tot), np.median(d[:, :, 2]) / (n / 64)))
# per-CU: blocks sharing a CU (same smid) and overlapping in time
sm = tr[:, 0, 8]
start, end = st[:, :, 0].min(1), st[:, :, 7].max(1)
print("distinct CUs", len(np.unique(sm)), "blocks", nblk)
cu = np.unique(sm)[0]
sel = np.where(sm == cu)[0]
o = sel[np.argsort(start[sel])]
print("CU", cu, "timeline (start, end, dur) rel. to first start:")
for b in o[:16]:
    print("  blk %5d  %9d %9d %9d" % (b, start[b] - start[o[0]], end[b] - start[o[0]], end[b] - start[b]))
# shader clock: s_memtime (SCLK) against s_memrealtime (100 MHz) at block ends on this CU
rt = tr[:, 0, 9]
e7 = st[:, 0, 7]
a, b = o[0], o[-1]
if rt[b] != rt[a]:
    print("SCLK over the CU's run: %.3f GHz" % ((e7[b] - e7[a]) / ((rt[b] - rt[a]) / 100e6) / 1e9))
