#!/usr/bin/env python3
"""Golden outputs of the reference's OWN tracking driver (src/tracking_main.c:68-228) -- DATA only,
written in the build container where /root/reference exists; the GPU box uses the committed
tracking_main_ref.npz.

The driver is the body of tracking_main.c's main cut out of the reference text by
oracle/Makefile and compiled with src/top_N.c and src/pnp_solver.c (oracle/ref_track_harness.c,
oracle.ref_tracking_main): its match list (the points main hands to ransac_essential_matrix), the
RANSAC's E and inliers and the pose, for every case of tracking_main_cases() in two builds --
as built (compute_softmax / compute_top_N without a prototype: SURVEY F7) and with top_N.h in scope
(the true scale reaches top_N.c).

Cases (24 x 80 cells; main's arrays hold 1920):
  self        quantized_image0 with itself (100 matches)
  kitti01     quantized_image0 -> KITTI 00 frame 000001 run through the quantized SuperPoint
              network by the C oracle (oracle/sp_oracle.c, bit-exact with PyTorch's quantized
              kernels, tests/test_superpoint.py); frame 1's header scale is frame 0's, as
              python/superpoint_inference.py:648,657 writes semi_scale[0] for both images
              (51 matches as built).  Frame 1's int8 semi / desc are stored here.
  syn1..syn3  synth.synth_window_pair(seed) (frame 1 = frame 0 displaced by whole cells + noise)
  syn1_e2, syn1_em2  syn1 at semi scales whose as-built effective scale is 2 and -2 (float
              mantissa low bits 010 / 110: the promoted double's low word)
  cap         a frame 1 with > 1000 valid cells: top_N.c exit(1)s (status 1)
  none        all-zero descriptors in frame 1 (every score 0/0 = NaN): no match, the RANSAC's
              rand() % 0 (status 2)
"""
import os
import sys

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(OUT, "..", "..")
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "maveric-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

FIELDS = ("status", "points1", "points2", "E", "inliers", "num_inliers", "R1", "R2", "t")


def _scale_with_low_bits(low):
    return np.float32((np.array([0.35], np.float32).view(np.uint32) & ~np.uint32(7) | np.uint32(low))
                      .view(np.float32)[0])


def tracking_main_cases(golden_dir=OUT, frame1_kitti=None):
    """name -> (frame0, frame1).  frame1_kitti: (semi, desc) of frame 000001 (the stored copy when
    None)."""
    import synth

    g = np.load(os.path.join(golden_dir, "quantized_image0.npz"), allow_pickle=False)
    img0 = dict(rows=24, cols=80, semi=g["semi"], desc=g["desc"], semi_scale=np.float32(g["semi_scale"]))
    if frame1_kitti is None:
        t = np.load(os.path.join(golden_dir, "tracking_main_ref.npz"), allow_pickle=False)
        frame1_kitti = (t["kitti01_semi1"], t["kitti01_desc1"])
    cases = {"self": (img0, img0),
             "kitti01": (img0, dict(img0, semi=frame1_kitti[0], desc=frame1_kitti[1]))}
    for s in (1, 2, 3):
        cases["syn%d" % s] = synth.synth_window_pair(s)
    f0, f1 = cases["syn1"]
    for tag, low in (("e2", 2), ("em2", 6)):
        sc = _scale_with_low_bits(low)
        cases["syn1_" + tag] = (dict(f0, semi_scale=sc), dict(f1, semi_scale=sc))
    rng = np.random.default_rng(77)
    f0, f1 = synth.synth_window_pair(4)
    cases["cap"] = (f0, dict(f1, semi=synth.synth_semi(rng, 1920, p_key=0.9)))
    f0, f1 = synth.synth_window_pair(5)
    cases["none"] = (f0, dict(f1, desc=np.zeros((1920, 256), np.int8)))
    return cases


def main():
    import oracle

    oracle.build()
    assert oracle.ref_track_available(), "oracle/_ref/libmv_ref_track*.so not built (reference absent?)"
    w = dict(np.load(os.path.join(OUT, "superpoint_qnonorm.npz"), allow_pickle=False))
    ims = np.load(os.path.join(OUT, "kitti00_images.npz"), allow_pickle=False)
    semi1, desc1, _, _, _, _ = oracle.sp_forward(ims["img_000001"], oracle.sp_net(w))
    out = {"kitti01_semi1": semi1, "kitti01_desc1": desc1}
    for name, (f0, f1) in tracking_main_cases(frame1_kitti=(semi1, desc1)).items():
        for mode, ts in (("built", False), ("true", True)):
            r = oracle.ref_tracking_main(f0, f1, true_scale=ts)
            for k in FIELDS:
                out["%s_%s_%s" % (name, mode, k)] = np.asarray(r[k])
            print(name, mode, "status", r["status"], "matches", len(r["points1"]), "inliers", r["num_inliers"])
    assert len(out["self_built_points1"]) == 100 and len(out["kitti01_built_points1"]) == 51
    assert out["cap_built_status"] == 1 and out["none_built_status"] == 2
    np.savez_compressed(os.path.join(OUT, "tracking_main_ref.npz"), **out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
