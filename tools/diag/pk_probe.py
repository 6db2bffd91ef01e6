#!/usr/bin/env python3
"""Diagnosis only: tools/diag/pk_probe.hip's packed-FP32 forms checked bit for bit
against the scalar VALU, alone and while other work runs on another stream (the SuperPoint network,
whose head kernels perturbed the SLP-packed pose; a hipBLASLt GEMM; a memory-bound copy).  The first
mismatches are printed with the value each plausible misreading of the instruction would give.
GPU only."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import mvtrack  # noqa: E402
from bench_image_pose import frames_kitti  # noqa: E402

FORMS = {0: "pk_fma", 1: "pk_fma op_sel_hi:[0,1,1]", 2: "pk_fma op_sel:[1,0,0]",
         3: "pk_fma op_sel_hi:[1,0,1] neg_lo/hi:[1,0,0]", 4: "pk_fma op_sel:[0,1,0] neg_lo/hi:[1,0,0]",
         5: "pk_mul", 6: "pk_mov op_sel:[1,0]", 7: "pk_add neg_lo/hi:[0,1]", 8: "pk_fma op_sel:[0,1,0]",
         9: "pk_fma op_sel:[0,0,1]", 10: "pk_mul op_sel:[0,1]", 11: "pk_add op_sel:[0,1]",
         12: "pk_fma op_sel:[0,1,0] op_sel_hi:[1,0,1]", 13: "pk_fma neg_lo/hi:[1,0,0]",
         14: "pk_fma op_sel_hi:[1,0,1]", 15: "pk_mul op_sel:[1,0]"}
dev = torch.device("cuda", 0)
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "diag", "libpk_probe.so"))
W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
F = 257
x = torch.from_numpy(np.stack(frames_kitti(F))).to(dev)
ctx = mvtrack.Context(0)
sB = torch.cuda.Stream(device=dev)
ctx.set_stream(sB)
sp = mvtrack.SuperPoint(ctx, W)
semi, cdesc = torch.zeros(F, 65, 24, 80, device=dev), torch.zeros(F, 256, 24, 80, device=dev)
g = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
big = torch.zeros(64 << 20, device=dev)
sA = torch.cuda.Stream(device=dev)
bad = torch.zeros(16, dtype=torch.int32, device=dev)
samples = torch.zeros(1 + 10 * 32, dtype=torch.int32, device=dev)
nb = 8 * torch.cuda.get_device_properties(0).multi_processor_count
iters = int(os.environ.get("ITERS", "4096"))
reps = int(os.environ.get("REPS", "4"))
with torch.cuda.stream(sB):
    sp.forward_raw(x, 192, 640, out=(semi, cdesc))
torch.cuda.synchronize()


def partner(kind):
    with torch.cuda.stream(sB):
        for _ in range(2):
            if kind == "network":
                sp.forward_raw(x, 192, 640, out=(semi, cdesc))
            elif kind == "gemm":
                for _ in range(4):
                    g @ g
            elif kind == "copy":
                big.mul_(1.0)


f32 = np.float32


def fma(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


forms = [int(v) for v in os.environ.get("FORMS", ",".join(str(k) for k in FORMS)).split(",")]
conds = os.environ.get("PARTNERS", "solo,network,gemm,copy").split(",")
for f in forms:
    res = {}
    for cond in conds:
        bad.zero_()
        samples.zero_()
        torch.cuda.synchronize()
        for rep in range(reps):
            with torch.cuda.stream(sA):
                rc = lib.mv_dbg_pk_probe(f, nb, iters, 12345 + rep, ctypes.c_void_p(bad.data_ptr()),
                                         ctypes.c_void_p(samples.data_ptr()), ctypes.c_void_p(sA.cuda_stream))
                assert rc == 0, rc
            if cond != "solo":
                partner(cond)
            torch.cuda.synchronize()
        res[cond] = int(bad[f].item())
        smp = samples.cpu().numpy()
        if res[cond] and os.environ.get("SAMPLES", "1") != "0":
            rec = smp[1:].reshape(32, 10)[:min(4, int(smp[0]))]
            for r in rec:
                v = r[1:9].view(np.float32)
                ax, ay, bx, by, cx, cy, gx, gy = [f32(t) for t in v]
                alts = {"src1.lo for lo": fma(-ax, bx, cx), "no neg": fma(ax, by, cx), "src0.hi": fma(-ay, by, cx),
                        "src2.hi": fma(-ax, by, cy), "mul only": f32(-ax * by)} if f in (4, 8, 12) else {}
                print("   form %d %s: lane %s got (%r, %r)  in a=(%r,%r) b=(%r,%r) c=(%r,%r)  alt %s" % (
                    f, cond, ("lo" if r[0] & 0x100 else "") + ("hi" if r[0] & 0x200 else ""), gx, gy, ax, ay, bx,
                    by, cx, cy, {k: (float(a_), bool(a_ == gx)) for k, a_ in alts.items()}), flush=True)
    words = nb * 256 * iters * 4 * 2 * reps
    print("form %2d %-42s words %.3g per condition: mismatches %s" % (
        f, FORMS[f], words, ", ".join("%s %d" % (k, v) for k, v in res.items())), flush=True)
