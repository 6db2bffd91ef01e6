#!/usr/bin/env python3
"""Extract the reference's data fixtures into compact binary files (tests/golden/*.npz).

Runs ONLY in the survey/build container where /root/reference exists; the GPU box
uses the committed .npz files.  Everything written here is DATA the reference
holds (int8 SuperPoint outputs, fp32 keypoints/descriptors, exact-softmax ground
truth, the OpenCV pose outputs and KITTI GT poses) -- no reference source text.

Sources (paths relative to /root/reference):
  include/data/quantized/quantized_image0.h   int8 semi[1920][65], desc[1920][256] + scales
  include/data/quantized/pair0_gt.h           exact softmax probs_gt/indices_gt [80][24] x 2 frames
  include/data/tracking/pair0.h, pair10.h     fp32 keypoints + unit descriptors (2 frames each)
  include/data/tracking/pair0/image0.h        full-res (376x1241) frame 0, 1002 keypoints
  outputs/transform_00078{5..9}_*.npy         3x4 float64 [R|t] from cv2.findEssentialMat+recoverPose
  outputs/00.txt                              KITTI seq 00 GT poses (3x4 per line)
  outputs/785/*.pose.txt, *.ply               compute_trajectory.py outputs (file bytes)

Float literals are parsed with libc strtof (direct decimal->binary32 rounding,
exactly what the C compiler does for a `const float` initialiser).
"""
import ctypes
import os
import re
import sys

import numpy as np

REF = os.environ.get("MV_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

_libc = ctypes.CDLL("libc.so.6")
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]


def _read(rel):
    with open(os.path.join(REF, rel), "r") as f:
        return f.read()


def _scalar(text, name, kind):
    m = re.search(r"const\s+\w+\s+%s\s*=\s*([^;]+);" % re.escape(name), text)
    if not m:
        raise KeyError(name)
    s = m.group(1).strip()
    if kind == "f32":
        return np.float32(_libc.strtof(s.encode(), None))
    return int(s)


def _array(text, name, dtype, shape):
    m = re.search(r"const\s+\w+\s+%s\s*(\[[^=]*\])\s*=\s*\{" % re.escape(name), text)
    if not m:
        raise KeyError(name)
    start = m.end()
    end = text.index("};", start)
    body = text[start:end].replace("{", " ").replace("}", " ")
    toks = [t for t in re.split(r"[\s,]+", body) if t]
    n = int(np.prod(shape))
    if len(toks) != n:
        raise ValueError("%s: %d values, expected %d" % (name, len(toks), n))
    if dtype == np.float32:
        vals = np.array([_libc.strtof(t.encode(), None) for t in toks], dtype=np.float32)
    else:
        vals = np.array([int(t) for t in toks], dtype=np.int64).astype(dtype)
    return vals.reshape(shape)


def quantized_image0():
    t = _read("include/data/quantized/quantized_image0.h")
    d = dict(
        rows=_scalar(t, "image0_rows", "i"), cols=_scalar(t, "image0_cols", "i"),
        feature_rows=_scalar(t, "image0_feature_rows", "i"),
        feature_cols=_scalar(t, "image0_feature_cols", "i"),
        semi_scale=_scalar(t, "image0_semi_scale", "f32"),
        desc_scale=_scalar(t, "image0_desc_scale", "f32"),
    )
    cells = d["feature_rows"] * d["feature_cols"]
    d["semi"] = _array(t, "image0_semi", np.int8, (cells, 65))
    d["desc"] = _array(t, "image0_desc", np.int8, (cells, 256))
    np.savez_compressed(os.path.join(OUT, "quantized_image0.npz"),
                        **{k: np.asarray(v) for k, v in d.items()})
    return d


def pair0_gt():
    t = _read("include/data/quantized/pair0_gt.h")
    out = {}
    for f in ("image0", "image1"):
        out[f + "_probs_gt"] = _array(t, f + "_probs_gt", np.float32, (80, 24))
        out[f + "_indices_gt"] = _array(t, f + "_indices_gt", np.int32, (80, 24))
    np.savez_compressed(os.path.join(OUT, "pair0_gt.npz"), **out)


def tracking_pair(rel, outname, frames=("image0", "image1")):
    t = _read(rel)
    out = {}
    for f in frames:
        n = _scalar(t, f + "_num_features", "i")
        out[f + "_rows"] = np.int32(_scalar(t, f + "_rows", "i"))
        out[f + "_cols"] = np.int32(_scalar(t, f + "_cols", "i"))
        out[f + "_xs"] = _array(t, f + "_feature_xs", np.int32, (n,))
        out[f + "_ys"] = _array(t, f + "_feature_ys", np.int32, (n,))
        out[f + "_scores"] = _array(t, f + "_feature_scores", np.float32, (n,))
        out[f + "_desc"] = _array(t, f + "_feature_descriptors", np.float32, (n, 256))
        try:
            fr = _scalar(t, f + "_feature_rows", "i")
            fc = _scalar(t, f + "_feature_cols", "i")
            out[f + "_coord_to_index"] = _array(t, f + "_coord_to_index", np.int32, (fr * fc,))
        except KeyError:
            pass
    np.savez_compressed(os.path.join(OUT, outname), **out)


def poses():
    ts = []
    for a in range(785, 790):
        p = os.path.join(REF, "outputs", "transform_%06d_%06d.npy" % (a, a + 1))
        ts.append(np.load(p, allow_pickle=False))
    gt = np.loadtxt(os.path.join(REF, "outputs", "00.txt"))
    keep = [0, 1, 10, 11] + list(range(785, 791))
    np.savez_compressed(os.path.join(OUT, "poses.npz"),
                        transforms_785_790=np.stack(ts).astype(np.float64),
                        kitti00_frames=np.array(keep, dtype=np.int32),
                        kitti00_gt=gt[keep].reshape(-1, 3, 4))


def trajectory():
    """The reference's committed compute_trajectory.py outputs for frames 785..789 (output
    files, stored as bytes): five .pose.txt, the current script's PLY and the older one."""
    d = os.path.join(REF, "outputs", "785")
    out = {}
    for f in sorted(os.listdir(d)):
        key = f.replace("-", "_").replace(".", "_")
        out[key] = np.frombuffer(open(os.path.join(d, f), "rb").read(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "trajectory_785.npz"), **out)


def main():
    if not os.path.isdir(REF):
        print("reference not present; fixtures are already committed", file=sys.stderr)
        return 1
    quantized_image0()
    pair0_gt()
    tracking_pair("include/data/tracking/pair0.h", "tracking_pair0.npz")
    tracking_pair("include/data/tracking/pair10.h", "tracking_pair10.npz")
    tracking_pair("include/data/tracking/pair0/image0.h", "tracking_fullres_image0.npz",
                  frames=("image0",))
    poses()
    trajectory()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
