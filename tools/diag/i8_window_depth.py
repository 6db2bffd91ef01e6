"""Why k_i8t_match cannot serve the network's own int8 descriptors with a per-lane list (CPU only).

k_i8t_match screens a row against frame 1's UNIT-NORM codes q = RNE(b * 127 / |b|) and keeps a
lane-local top-2 per lane half (columns with (j >> 2) & 1 = h).  Its window is the rigorous
Cauchy-Schwarz bound on the codes' rounding, 2 * (8 + 1.3e-4) |a| in 127-units -- about 14 % of
the 0.9-cosine threshold score (114.3 |a|).  A row whose half holds K or more in-window columns is
"deep" for a K-slot list (a (K+1)-th may hide below), and ONE deep row hands the whole pair to
k_i8m_handback.  This counts, on the SuperPoint forward of KITTI 00 frames 000000 / 000001 (the
C oracle, 1920 cells x 256), the deep rows per pair for K = 2 .. 16, with the shipped window and
with the tightest per-frame rigorous one (the largest residual norm |q - b 127/|b|| of the frame
instead of 8).  Reference: python/superpoint_inference.py:197-208 (the int8 descriptors),
python/pairwise_pnp.py:639-659 (the match rule restated with integer dots)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402


def depth_table(a, b, bound, ks):
    a = a.astype(np.int64)
    b = b.astype(np.int64)
    nb = (b * b).sum(1)
    sc = np.zeros(len(b))
    sc[nb > 0] = 127.0 / np.sqrt(nb[nb > 0])
    qf = b * sc[:, None]
    q = np.rint(qf)
    res = np.sqrt(((q - qf) ** 2).sum(1))
    w = res.max() if bound == "residual" else 8.0 + 1.3e-4
    d = a @ q.astype(np.int64).T
    na = (a * a).sum(1)
    an = np.sqrt(na)
    da = an * w * 1.0001 + 1e-6
    m = d.max(1)
    cand = (na > 0) & (m + da > 114.3 * an * (1 - 1e-9))
    inw = d >= (m - 2 * da)[:, None]
    h = (np.arange(len(b)) >> 2) & 1
    per_half = np.maximum((inw & (h == 0)[None]).sum(1), (inw & (h == 1)[None]).sum(1))[cand]
    return w, int(cand.sum()), {k: int((per_half >= k).sum()) for k in ks}, int(per_half.max())


def main():
    W = dict(np.load(os.path.join(ROOT, "tests", "golden", "superpoint_qnonorm.npz")))
    ims = np.load(os.path.join(ROOT, "tests", "golden", "kitti00_images.npz"))
    net = orc.sp_net(W)
    d = [orc.sp_forward(ims[k], net)[1] for k in ("img_000000", "img_000001")]
    ks = (2, 3, 4, 6, 8, 12, 16)
    print("K-slot lane-half lists: deep rows per pair (any deep row hands the pair back)")
    for name, (a, b) in (("000000->000001", (d[0], d[1])), ("000001->000000", (d[1], d[0]))):
        for bound in ("shipped", "residual"):
            w, nc, tab, mx = depth_table(a, b, bound, ks)
            print("%s window %-8s (%.2f |a|): rows above the cosine bound %d, max in-window per half %d, deep rows %s"
                  % (name, bound, w, nc, mx, " ".join("K=%d:%d" % kv for kv in tab.items())))


if __name__ == "__main__":
    main()
