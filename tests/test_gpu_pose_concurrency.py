"""GPU: the pose kernels give bit-identical results whether they run alone or while the SuperPoint
network runs on another stream.  Round 5's SLP-vectorised as-intended pose differed in
5-40 % of a track's pairs beside the network: on MI355X a packed-FP32 instruction whose low lane
reads the HIGH half of src1 (v_pk_{fma,mul,add}_f32 op_sel:[x,1,...]) read that operand as zero in
~1.3e-4 of executions while the network ran (tools/diag/pk_probe.py, profiles/r06c_pk_probe.log).
The library holds no such instruction (tests/test_isa_guard.py); this test runs the consequence:
the image -> match chain on stream A (as the image -> pose bench does), then the pose on A while
stream B runs the network (tools/dbg_pose_interference.py's schedule: the round-5 SLP build of the
pose gave hundreds of differing pairs under it), every result checked bit for bit against the solo run --
for the as-intended pose (k_pose_ransac) and the as-built one (k_pose_as_built: the reference's stub
RANSAC + McAdams SVD, which held 62 of those instructions before round 6)."""
import os
import sys

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAP = 1024


def test_pose_bit_identical_beside_superpoint_network(torch_cuda):
    import mvtrack
    import synth

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_image_pose import frames_kitti

    torch = torch_cuda
    dev = torch.device("cuda:0")
    F, P = 257, 256  # tools/dbg_pose_interference.py's track: 256 pairs of 257 network frames
    W = dict(load_golden("superpoint_qnonorm.npz"))
    x = torch.from_numpy(np.stack(frames_kitti(F))).to(dev)
    K = synth.KITTI_K
    e = lambda *shape, dt=torch.float32: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731

    sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    ca, cb = mvtrack.Context(0), mvtrack.Context(0)
    ca.set_stream(sa)
    cb.set_stream(sb)
    spa, spb = mvtrack.SuperPoint(ca, W), mvtrack.SuperPoint(cb, W)
    try:
        semi, cdesc = e(F, 65, 24, 80), e(F, 256, 24, 80)
        semi_b, cdesc_b = e(F, 65, 24, 80), e(F, 256, 24, 80)
        nkp, kp, conf, desc, kst = e(F, dt=torch.int32), e(F, CAP, 2), e(F, CAP), e(F, CAP, 256), e(F, dt=torch.int32)
        idx = e(P, CAP, dt=torch.int32)
        with torch.cuda.stream(sa):
            spa.forward_raw(x, 192, 640, out=(semi, cdesc))
            ca.keypoints(semi, cdesc, 192, 640, nkp, kp, conf, desc, kst)
            ca.match_allpairs_f32(desc[:P], desc[1:], nkp[:P], nkp[1:], idx, None, 0.8)
        torch.cuda.synchronize()
        assert int((kst == 0).sum()) == F and int(nkp.min()) > 100
        for sem in (mvtrack.AS_INTENDED, mvtrack.AS_BUILT):
            prm = mvtrack.pose_params(sem, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2], hypotheses=256,
                                      inlier_thresh=1.0, refine_iters=10, seed=7)
            T, nm, ni, st = e(P, 3, 4), e(P, dt=torch.int32), e(P, dt=torch.int32), e(P, dt=torch.int32)

            def pose():
                ca.pose_from_matches(prm, nkp[:P], idx, kp[:P], kp[1:], T, nm, ni, st)

            with torch.cuda.stream(sa):
                pose()
            torch.cuda.synchronize()
            ref = (T.clone(), ni.clone(), st.clone())
            assert int((ref[2] == 0).sum()) > P // 2
            differing = 0
            for _ in range(4):  # tools/dbg_pose_interference.py's schedule, which made round 5's build differ
                with torch.cuda.stream(sa):
                    pose()
                with torch.cuda.stream(sb):
                    for _ in range(2):
                        spb.forward_raw(x, 192, 640, out=(semi_b, cdesc_b))
                with torch.cuda.stream(sa):
                    pose()  # beside the network on stream B
                torch.cuda.synchronize()
                d = (T.view(torch.int32) != ref[0].view(torch.int32)).reshape(P, 12).any(dim=1)
                d |= (ni != ref[1]) | (st != ref[2])
                differing += int(d.sum())
            assert differing == 0, "%s pose: %d pair results differ from the solo run beside the network" % (
                "as-intended" if sem == mvtrack.AS_INTENDED else "as-built", differing)
    finally:
        spa.close()
        spb.close()
        ca.close()
        cb.close()
