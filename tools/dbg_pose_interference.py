#!/usr/bin/env python3
"""Which kernel, running concurrently on another stream, changes k_pose_ransac's results?
Stream A repeats the pose on one fixed track's matches; stream B repeats one other stage
(SuperPoint network, keypoints, the all-pairs match) on its own buffers.  Every pose result is
compared with a solo run, bit for bit.  GPU only (diagnosis)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "maveric-slam_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import mvtrack  # noqa: E402
import synth  # noqa: E402
from bench_image_pose import CAP, frames_kitti  # noqa: E402

dev = torch.device("cuda", 0)
F, P = 257, 256
W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
x = torch.from_numpy(np.stack(frames_kitti(F))).to(dev)
K = synth.KITTI_K
prm = mvtrack.pose_params(mvtrack.AS_BUILT if os.environ.get("MODE") == "built" else mvtrack.AS_INTENDED,
                          fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                          hypotheses=int(os.environ.get("HYPS", "256")), inlier_thresh=1.0,
                          refine_iters=int(os.environ.get("REFINE", "10")), seed=7)
e = lambda *shape, dt=torch.float32: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731


def cu_stream(half):
    """a HIP stream restricted to one half of the CUs (hipExtStreamCreateWithCUMask), as a torch stream"""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(n):
        sel = ((c // 2) % 2) if os.environ.get("CUPAIRS") else (c % 2)  # CUPAIRS: whole CU pairs per half
        if sel == half:  # interleaved halves: every shader engine keeps CUs in both
            mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(st.value, device=dev)


class Pipe:
    def __init__(self, half=None):
        self.stream = torch.cuda.Stream(device=dev) if half is None else cu_stream(half)
        self.ctx = mvtrack.Context(0)
        self.ctx.set_stream(self.stream)
        self.sp = mvtrack.SuperPoint(self.ctx, W)
        self.semi, self.cdesc = e(F, 65, 24, 80), e(F, 256, 24, 80)
        self.nkp, self.kp, self.conf = e(F, dt=torch.int32), e(F, CAP, 2), e(F, CAP)
        self.desc, self.kst = e(F, CAP, 256), e(F, dt=torch.int32)
        self.idx = e(P, CAP, dt=torch.int32)
        self.T, self.nm, self.ni, self.st = e(P, 3, 4), e(P, dt=torch.int32), e(P, dt=torch.int32), e(P, dt=torch.int32)

    def net(self):
        self.sp.forward_raw(x, 192, 640, out=(self.semi, self.cdesc))

    def kps(self):
        self.ctx.keypoints(self.semi, self.cdesc, 192, 640, self.nkp, self.kp, self.conf, self.desc, self.kst)

    def match(self):
        self.ctx.match_allpairs_f32(self.desc[:P], self.desc[1:], self.nkp[:P], self.nkp[1:], self.idx, None, 0.8)

    def pose(self):
        self.ctx.pose_from_matches(prm, self.nkp[:P], self.idx, self.kp[:P], self.kp[1:], self.T, self.nm, self.ni,
                                   self.st)

    def net8(self):  # the int8 forward: the same layers, heads written as int8 cells (+ run()'s min gap)
        if not hasattr(self, "o8"):
            cells = 24 * 80
            self.o8 = (torch.empty((F, cells, 65), dtype=torch.int8, device=dev),
                       torch.empty((F, cells, 256), dtype=torch.int8, device=dev),
                       torch.empty(F, dtype=torch.float32, device=dev), torch.empty(F, dtype=torch.float32, device=dev))
        self.sp.forward(x, 192, 640, out=self.o8)

    def scat(self):  # fp32 stores scattered over 256 channel planes, as the raw heads write them
        self.cdesc.view(F, 256, -1).transpose(1, 2).copy_(self.desc.new_ones(F, 1920, 256) * 0.5)

    def gemm(self):  # a library MFMA GEMM (hipBLASLt bf16), no kernel of ours
        if not hasattr(self, "g"):
            self.g = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
        for _ in range(4):
            self.g2 = self.g @ self.g

    def copy(self):  # a memory-bound torch kernel of the heads' size (126 MB written as fp32)
        self.cdesc.copy_(self.cdesc * 1.0)

    def all(self):
        with torch.cuda.stream(self.stream):
            self.net(), self.kps(), self.match(), self.pose()


torch.cuda.synchronize()
cm = os.environ.get("CUMASK")  # "split": A and B on disjoint CU halves; "same": both on half 0
a, b = (Pipe(0), Pipe(1)) if cm == "split" else ((Pipe(0), Pipe(0)) if cm == "same" else (Pipe(), Pipe()))
a.all(), b.all()
torch.cuda.synchronize()
ref = a.T.clone()
ref_nm = a.nm.clone()
if os.environ.get("OOB"):  # does stream B's stage alone change a's buffers (no pose running on A)?
    snap = {k: getattr(a, k).clone() for k in ("semi", "cdesc", "nkp", "kp", "desc", "idx", "T", "nm", "ni", "st")}
    for stage in os.environ.get("STAGES", "net,kps,match,pose").split(","):
        with torch.cuda.stream(b.stream):
            for _ in range(3):
                getattr(b, stage)()
        torch.cuda.synchronize()
        changed = [k for k, v in snap.items() if not torch.equal(getattr(a, k), v)]
        print("stage %-5s alone on B: a's buffers changed: %s" % (stage, changed), flush=True)
    sys.exit(0)
if os.environ.get("FILLTEST"):  # solo runs, each after every CU's registers + LDS were filled with a pattern
    import ctypes
    fl = ctypes.CDLL(os.path.join(ROOT, "tools", "diag", "libstate_fill.so"))
    sink = torch.zeros(4096, dtype=torch.int32, device=dev)
    nb = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    for r in range(int(os.environ.get("ROUNDS", "8"))):
        pat = (0x7FC00000, 0x3F800000, 0xFFFFFFFF, 0x00000000)[r % 4]
        with torch.cuda.stream(a.stream):
            rc = fl.mv_dbg_state_fill(ctypes.c_uint32(pat), ctypes.c_void_p(sink.data_ptr()), nb,
                                      ctypes.c_void_p(a.stream.cuda_stream))
            assert rc == 0, rc
            a.pose()
        torch.cuda.synchronize()
        d = (a.T - ref).abs().amax(dim=(1, 2))
        print("fill 0x%08x then pose solo: pairs differing from the first solo run: %d" % (pat, int((d > 0).sum())),
              flush=True)
    sys.exit(0)
for stage in os.environ.get("STAGES", "none,net,kps,match,pose,all").split(","):
    bad = 0
    for r in range(int(os.environ.get("ROUNDS", "6"))):
        with torch.cuda.stream(a.stream):
            a.pose()
        with torch.cuda.stream(b.stream):
            for _ in range(2):
                if stage == "all":
                    b.net(), b.kps(), b.match(), b.pose()
                elif stage != "none":
                    getattr(b, stage)()
        with torch.cuda.stream(a.stream):
            a.pose()
        torch.cuda.synchronize()
        d = (a.T - ref).abs().amax(dim=(1, 2))
        bad += int((d > 0).sum())
        badnm = int((a.nm != ref_nm).sum())
        if os.environ.get("NM") and badnm:
            idx_ = torch.nonzero(a.nm != ref_nm).flatten()[:6]
            got, exp = a.nm[idx_], ref_nm[idx_]
            if os.environ.get("NM") == "f":
                got, exp = got.view(torch.float32), exp.view(torch.float32)
            print("   round %d: num_matches (phase checksum) differs in %d pairs: pairs %s got %s solo %s" % (
                r, badnm, idx_.tolist(), got.tolist(), exp.tolist()), flush=True)
    print("concurrent %-5s: pose pairs differing from the solo run: %d" % (stage, bad), flush=True)
    if bad and os.environ.get("RERUN"):
        with torch.cuda.stream(a.stream):
            a.pose()
        torch.cuda.synchronize()
        print("   a.pose() again alone: %d pairs differ" % int(((a.T - ref).abs().amax(dim=(1, 2)) > 0).sum()), flush=True)
