"""Phase timing of k_q8t_match (one workgroup per pair; MV_Q8_KERNEL=d: k_q8d_match, two) (library built with EXTRA=-DMV_TRACE, e.g. MV_LIB=
build_variants/libmaveric_trace.so from tools/build_variant.sh trace -DMV_TRACE): per (block, wave)
s_memtime stamps at entry, A phase done, sweep + statistics done, epilogue done.
Env: TB pairs (8192), TN per-component noise of the re-observed rows (bench default 0.3/16;
SURVEY C1: 0.05), TS=1 materialise the exact scores."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "maveric-slam_amd"))
import bench  # noqa: E402
import mvtrack  # noqa: E402

B, n = int(os.environ.get("TB", "8192")), 1024
dev = torch.device("cuda", 0)
d0, d1, _, _ = bench.gen_batch(torch, dev, B, n, seed=3, noise=float(os.environ.get("TN", 0.3 / 16)))
sc = torch.empty((B, n), dtype=torch.float32, device=dev) if os.environ.get("TS") == "1" else None
nn_ = torch.full((B,), n, dtype=torch.int32, device=dev)
idx = torch.empty((B, n), dtype=torch.int32, device=dev)
ctx = mvtrack.Context(0)
ctx.set_stream(torch.cuda.current_stream())
for _ in range(3):
    ctx.match_allpairs_f32(d0, d1, nn_, nn_, idx, sc)
torch.cuda.synchronize()
NW = 8
nblk = min(B * (2 if os.environ.get("MV_Q8_KERNEL", "")[:1] == "d" else 1), 16384)
buf = np.zeros(nblk * NW * 10, np.uint64)
lib = mvtrack.lib()
lib.mv_debug_direct_trace.argtypes = [ctypes.c_void_p, ctypes.c_long]
assert lib.mv_debug_direct_trace(buf.ctypes.data, buf.nbytes) == 0
tr = buf.reshape(nblk, NW, 10).astype(np.int64)
st = tr[:, :, :4]
d = np.diff(st, axis=2)
names = ["A-phase", "sweep+stats", "epilogue"]
print("per-wave phase cycles (median / p10 / p90 / max):")
for k, nm in enumerate(names):
    v = d[:, :, k].ravel()
    print("  %-12s %9.0f %9.0f %9.0f %9.0f" % (nm, np.median(v), np.percentile(v, 10), np.percentile(v, 90), v.max()))
c = tr[:, :, 8]
print("wide rows per pair: mean %.2f p90 %.0f max %d; deferred dots per pair mean %.1f" % (
    (c >> 16).sum(1).mean(), np.percentile((c >> 16).sum(1), 90), (c >> 16).sum(1).max(), (c & 0xffff).sum(1).mean()))
tot = st[:, :, 3] - st[:, :, 0]
print("wave total median %.0f; sweep per tile %.0f" % (np.median(tot), np.median(d[:, :, 1]) / 16))
sm = tr[:, 0, 6]
start, end = st[:, :, 0].min(1), st[:, :, 3].max(1)
cu = np.unique(sm)[0]
sel = np.where(sm == cu)[0]
o = sel[np.argsort(start[sel])]
print("distinct CU ids", len(np.unique(sm)), "; CU", cu, "timeline (start, end, dur):")
for b in o[:12]:
    print("  blk %5d  %9d %9d %9d" % (b, start[b] - start[o[0]], end[b] - start[o[0]], end[b] - start[b]))
rt = tr[:, 0, 7]
a, b = o[0], o[-1]
if rt[b] != rt[a]:
    print("SCLK over the CU's run: %.3f GHz" % ((st[b, 0, 3] - st[a, 0, 3]) / ((rt[b] - rt[a]) / 100e6) / 1e9))
# chip-wide phase concurrency over real time (s_memrealtime, 100 MHz, one clock for the chip):
# per 1-us bin, how many blocks are in their A phase and how many in sweep + epilogue -- a
# convoy (every CU loading frame 0 at once, HBM-bound, then every CU sweeping) shows as A-phase
# counts near the CU count alternating with near zero
r0, rA, rE = tr[:, 0, 4], tr[:, 0, 5], tr[:, 0, 7]
if (r0 > 0).all():
    t0 = r0.min()
    nb = int((rE.max() - t0) // 100) + 1
    a_cnt = np.zeros(nb)
    s_cnt = np.zeros(nb)
    for b in range(nblk):
        i0, i1, i2 = (r0[b] - t0) // 100, (rA[b] - t0) // 100, (rE[b] - t0) // 100
        a_cnt[i0:i1 + 1] += 1
        s_cnt[i1 + 1:i2 + 1] += 1
    mid = slice(nb // 5, 4 * nb // 5)
    av = a_cnt[mid]
    print("A-phase blocks in flight per us (middle 60%% of the launch): mean %.1f, p10 %.0f, p50 %.0f, p90 %.0f, "
          "max %.0f; sweep+epilogue mean %.1f" % (av.mean(), np.percentile(av, 10), np.percentile(av, 50),
                                                  np.percentile(av, 90), av.max(), s_cnt[mid].mean()))
    print("A-phase real time per block: median %.2f us, sweep+epilogue %.2f us; launch %.1f us" % (
        np.median(rA - r0) / 100, np.median(rE - rA) / 100, (rE.max() - t0) / 100))
    print("A-phase counts, first 120 us:", " ".join("%d" % x for x in a_cnt[:120]))
