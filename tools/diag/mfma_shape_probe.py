#!/usr/bin/env python3
"""Diagnosis (GPU): sustained int8 MFMA TOPS of the 32x32x32 and 16x16x64 shapes on random operands,
every CU busy, after >= 2 s of warm-up; alternating A/B launches (tools/diag/mfma_shape_probe.hip)."""
import ctypes
import os
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmfma_shape_probe.so"))
dev = torch.device("cuda", 0)
seed = torch.randint(-2**31, 2**31 - 1, (4096,), dtype=torch.int32, device=dev)
blocks, iters = 1024, 40
sink = torch.zeros(blocks * 512, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream()
# ops per launch: 32x32x32: 16 MFMAs of 65536 ops per iteration; 16x16x64: 64 of 32768
ops = {32: blocks * 8 * iters * 16 * 65536.0, 16: blocks * 8 * iters * 64 * 32768.0}


def launch(shape):
    rc = lib.mv_dbg_mfma_probe(shape, blocks, iters, ctypes.c_void_p(seed.data_ptr()), ctypes.c_void_p(sink.data_ptr()),
                               ctypes.c_void_p(st.cuda_stream))
    assert rc == 0, rc


t0 = time.time()
while time.time() - t0 < 3.0:
    launch(32)
    launch(16)
    torch.cuda.synchronize()
res = {32: [], 16: []}
for r in range(6):
    for shape in (32, 16):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            launch(shape)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        res[shape].append(ops[shape] / (ms * 1e-3) / 1e12)
for shape in (32, 16):
    v = sorted(res[shape])
    print("shape %dx%d: TOPS median %.0f (min %.0f max %.0f) = %.3f of 5000" % (
        shape, shape, v[len(v) // 2], v[0], v[-1], v[len(v) // 2] / 5000), flush=True)
