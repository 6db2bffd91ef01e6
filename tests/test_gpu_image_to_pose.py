"""The fp32 path of python/pairwise_pnp.py:577-694 on the GPU, image to pose: KITTI 00 frames
000000 / 000001 (8-bit, 376 x 1241) -> the quantized SuperPoint network's float outputs
(mv_superpoint_forward_raw_dev: what run() receives from net.forward, :197-199) -> keypoints +
descriptors (run() after the forward: softmax heatmap, NMS, border, grid_sample, L2;
mv_keypoints_dev) -> the all-pairs match (:639-659) -> the pose (:667-694's intent).  Each stage
bit-exact against the oracle chain (oracle/sp_oracle.c -> the keypoint oracle -> the all-pairs
oracle), the pose against the KITTI ground truth with tests/test_gpu_kitti_e2e.py's stated
tolerances (the reference's full-resolution K on the resized image)."""
import numpy as np
import pytest

import synth
from conftest import load_golden
from test_gpu_kitti_e2e import angles, rel_gt

pytestmark = pytest.mark.gpu

CAP = 1024


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def oracle_chain(orc, weights, imgs):
    net = orc.sp_net(weights)
    s_sc, d_sc = np.float32(weights["convPb_meta"][2]), np.float32(weights["convDb_meta"][2])
    out = []
    for img in imgs:
        _, _, _, _, sr, dr = orc.sp_forward(img, net)
        semi, cdesc = s_sc * sr.astype(np.float32), d_sc * dr.astype(np.float32)
        pts, desc, _ = orc.keypoints(semi, cdesc, 192, 640)
        out.append((semi, cdesc, pts, desc))
    return out


def test_image_to_pose_kitti_pair(ctx, orc, torch_cuda):
    import mvtrack

    torch = torch_cuda
    dev = torch.device("cuda:0")
    weights = dict(load_golden("superpoint_qnonorm.npz"))
    ims = load_golden("kitti00_images.npz")
    imgs = [ims["img_000000"], ims["img_000001"]]
    sp = mvtrack.SuperPoint(ctx, weights)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        x = torch.from_numpy(np.ascontiguousarray(np.stack(imgs), np.uint8)).to(dev)
        semi, cdesc = sp.forward_raw(x, 192, 640)
        nkp = torch.empty(2, dtype=torch.int32, device=dev)
        kp = torch.zeros((2, CAP, 2), dtype=torch.float32, device=dev)
        conf = torch.zeros((2, CAP), dtype=torch.float32, device=dev)
        desc = torch.zeros((2, CAP, 256), dtype=torch.float32, device=dev)
        kst = torch.empty(2, dtype=torch.int32, device=dev)
        ctx.keypoints(semi, cdesc, 192, 640, nkp, kp, conf, desc, kst)
        # pair (frame 0, frame 1): the keypoint outputs are the match's inputs as laid out
        n0, n1 = nkp[0:1].clone(), nkp[1:2].clone()
        idx = torch.empty((1, CAP), dtype=torch.int32, device=dev)
        sc = torch.empty((1, CAP), dtype=torch.float32, device=dev)
        ctx.match_allpairs_f32(desc[0:1], desc[1:2], n0, n1, idx, sc, 0.8)
        K = synth.KITTI_K  # pairwise_pnp.py:667-669
        prm = mvtrack.pose_params(mvtrack.AS_INTENDED, fx=K[0, 0], fy=K[1, 1], cx=K[0, 2], cy=K[1, 2],
                                  hypotheses=512, inlier_thresh=1.0, refine_iters=10, seed=5)
        T = torch.empty((1, 3, 4), dtype=torch.float32, device=dev)
        nm = torch.empty(1, dtype=torch.int32, device=dev)
        ni = torch.empty(1, dtype=torch.int32, device=dev)
        st = torch.empty(1, dtype=torch.int32, device=dev)
        ctx.pose_from_matches(prm, n0, idx, kp[0:1], kp[1:2], T, nm, ni, st)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
        sp.close()
    ref = oracle_chain(orc, weights, imgs)
    for b in range(2):
        o_semi, o_cdesc, o_pts, o_desc = ref[b]
        assert (bits(semi[b].cpu().numpy()) == bits(o_semi)).all(), ("semi", b)
        assert (bits(cdesc[b].cpu().numpy()) == bits(o_cdesc)).all(), ("coarse_desc", b)
        n = int(nkp[b])
        assert int(kst[b]) == 0 and n == o_pts.shape[0] and 300 < n < CAP, (b, n)
        assert (kp[b, :n].cpu().numpy() == o_pts[:, :2]).all(), ("keypoints", b)
        assert (bits(conf[b, :n].cpu().numpy()) == bits(o_pts[:, 2])).all(), ("confidences", b)
        assert (bits(desc[b, :n].cpu().numpy()) == bits(o_desc)).all(), ("descriptors", b)
    i2, s2 = orc.allpairs_f32(ref[0][3], ref[1][3], 0.8)
    n0 = ref[0][2].shape[0]
    assert (idx[0, :n0].cpu().numpy() == i2).all() and (bits(sc[0, :n0].cpu().numpy()) == bits(s2)).all()
    assert (idx[0, n0:].cpu().numpy() == -1).all()
    er, et = angles(T[0].cpu().numpy(), rel_gt(0, 1))
    print("image -> pose: %d / %d keypoints, %d matches, %d inliers, rotation %.3f deg, translation direction %.2f deg"
          % (int(nkp[0]), int(nkp[1]), int(nm[0]), int(ni[0]), er, et))
    assert int(st[0]) == 0 and int(nm[0]) == int((i2 >= 0).sum()) >= 250
    assert er < 1.0 and et < 30.0, (er, et)  # test_gpu_kitti_e2e.py's reference-K tolerances


def test_forward_raw_batch_and_partial_tiles(ctx, orc, torch_cuda):
    """the raw outputs on random frames at a small network size (partial tiles, Wc not a multiple
    of 4) and a batch of three, bit-exact against the oracle's dequantised heads"""
    import mvtrack

    torch = torch_cuda
    dev = torch.device("cuda:0")
    weights = dict(load_golden("superpoint_qnonorm.npz"))
    rng = np.random.default_rng(12)
    imgs = [rng.integers(0, 256, (100, 150), dtype=np.uint8) for _ in range(3)]
    oh, ow = 48, 72  # Wc = 9
    sp = mvtrack.SuperPoint(ctx, weights)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        semi, cdesc = sp.forward_raw(torch.from_numpy(np.stack(imgs)).to(dev), oh, ow)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
        sp.close()
    net = orc.sp_net(weights)
    s_sc, d_sc = np.float32(weights["convPb_meta"][2]), np.float32(weights["convDb_meta"][2])
    for b, img in enumerate(imgs):
        _, _, _, _, sr, dr = orc.sp_forward(img, net, oh, ow)
        assert (bits(semi[b].cpu().numpy()) == bits(s_sc * sr.astype(np.float32))).all(), b
        assert (bits(cdesc[b].cpu().numpy()) == bits(d_sc * dr.astype(np.float32))).all(), b
