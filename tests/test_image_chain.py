"""The oracle's fp32 image chain (python/pairwise_pnp.py:577-659: image -> quantized network ->
run()'s keypoints and descriptors -> all-pairs match) against the reference's own fp32 fixture of
the same KITTI pair (include/data/tracking/pair0.h: 395 / 401 keypoints of frames 000000 / 000001
at 192 x 640, written by superpoint_inference.py's fp32 writer).  The network's int8 codes carry
SURVEY 8(c)'s platform gap (93.6 / 92.3 % of quantized_image0.h's values equal), so keypoints are
compared as sets: most of the reference's keypoints come out at the same pixels, the strongest
ones among the reference's strongest, and the matched pairs agree.  (The GPU chain is bit-exact against this
oracle chain: tests/test_gpu_image_to_pose.py.)"""
import numpy as np

from conftest import load_golden


def test_oracle_image_chain_agrees_with_reference_pair0(orc):
    w = dict(load_golden("superpoint_qnonorm.npz"))
    net = orc.sp_net(w)
    ims = load_golden("kitti00_images.npz")
    ref = load_golden("tracking_pair0.npz")
    s_sc, d_sc = np.float32(w["convPb_meta"][2]), np.float32(w["convDb_meta"][2])
    chain = []
    for f, k in ((0, "img_000000"), (1, "img_000001")):
        _, _, _, _, sr, dr = orc.sp_forward(ims[k], net)
        pts, desc, _ = orc.keypoints(s_sc * sr.astype(np.float32), d_sc * dr.astype(np.float32), 192, 640)
        rx, ry = ref["image%d_xs" % f].astype(int), ref["image%d_ys" % f].astype(int)
        mine = set(zip(pts[:, 0].astype(int), pts[:, 1].astype(int)))
        theirs = set(zip(rx, ry))
        common = len(mine & theirs)
        print("frame %d: %d keypoints (reference %d), %d at the same pixels" % (f, len(mine), len(theirs), common))
        assert abs(len(mine) - len(theirs)) <= 0.05 * len(theirs) and common >= 0.8 * len(theirs)
        top = set(zip(rx[:20], ry[:20]))  # the strongest keypoints are the reference's strongest
        assert sum((int(x), int(y)) in top for x, y in pts[:10, :2]) >= 8
        chain.append((pts, desc))
    i2, _ = orc.allpairs_f32(chain[0][1], chain[1][1], 0.8)
    ir, _ = orc.allpairs_f32(ref["image0_desc"], ref["image1_desc"], 0.8)
    # matched pixel pairs common to both chains
    mp = {(tuple(chain[0][0][i, :2].astype(int)), tuple(chain[1][0][j, :2].astype(int))) for i, j in enumerate(i2) if j >= 0}
    rp = {((int(ref["image0_xs"][i]), int(ref["image0_ys"][i])), (int(ref["image1_xs"][j]), int(ref["image1_ys"][j])))
          for i, j in enumerate(ir) if j >= 0}
    print("matches: %d (reference fixture %d), %d identical pixel pairs" % (len(mp), len(rp), len(mp & rp)))
    assert len(mp) >= 250 and len(mp & rp) >= 0.7 * len(rp)
