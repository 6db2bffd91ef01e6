#!/usr/bin/env python3
"""SuperPoint front-end fixtures -- DATA only, written in the build container
where /root/reference exists; the GPU box uses the committed .npz files.

- superpoint_qnonorm.npz: the int8 weights, float biases and the per-tensor scales / zero
  points of python/superpoint_quantized_nonorm.pt (the archive python/superpoint_inference.py:571
  loads by default), read by maveric-slam_amd/sp_weights.py -- the no-code opcode walk: the
  archive is never unpickled and no TorchScript runs.
- kitti00_images.npz: datasets/kitti/sequences/00/image_0/000000.png and 000001.png decoded
  with PIL (8-bit grayscale, 376 x 1241) -- the image quantized_image0.h was made from
  (superpoint_inference.py:613-628) and its successor.
"""
import os
import sys

import numpy as np

REF = os.environ.get("MV_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(OUT, "..", "..", "maveric-slam_amd"))

import sp_weights  # noqa: E402


def main():
    L = sp_weights.load_superpoint(os.path.join(REF, "python", "superpoint_quantized_nonorm.pt"))
    out = {"input_scale": np.float64(L["input"]["scale"]), "input_zp": np.int64(L["input"]["zero_point"])}
    for n in sp_weights.LAYERS:
        d = L[n]
        out[n + "_w"] = d["w"]
        out[n + "_bias"] = d["bias"]
        out[n + "_meta"] = np.array([d["w_scale"], d["w_zp"], d["out_scale"], d["out_zp"]], np.float64)
    np.savez_compressed(os.path.join(OUT, "superpoint_qnonorm.npz"), **out)

    from PIL import Image

    imgs = {}
    for f in ("000000", "000001"):
        im = Image.open(os.path.join(REF, "datasets/kitti/sequences/00/image_0/%s.png" % f))
        a = np.asarray(im)
        if a.dtype != np.uint8 or a.ndim != 2:
            raise ValueError("%s: expected 8-bit grayscale" % f)
        imgs["img_" + f] = a
    np.savez_compressed(os.path.join(OUT, "kitti00_images.npz"), **imgs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
