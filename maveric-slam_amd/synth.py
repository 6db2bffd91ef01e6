"""Synthetic frame-pairs of KITTI shape, numpy only.

Used by bench.py (workload generation, outside the timed region) and by the
tests.  Nothing here is on the hot path.

  synth_pair_f32     C1/C2: n keypoints x 256-D unit fp32 descriptors per frame;
                     a fraction `frac` of frame-0 points re-observed in frame 1
                     (descriptor + noise of norm `noise`, renormalised), the rest
                     fresh; keypoints are exact projections of a 3-D scene under
                     a known relative pose (default: outputs/transform_000785_000786.npy).
  synth_pair_i8      C4: int8 descriptors round(clip(N(0, 24))) (quantized_image0.h statistics).
  synth_window_pair  C0-shaped int8 frames (semi [cells][65] + desc [cells][256]) where frame 1
                     is frame 0 displaced by a whole number of cells plus int8 noise, so the
                     shifted-window match of tracking_main.c finds real correspondences.
"""
import numpy as np

# pairwise_pnp.py:667-669 (KITTI seq 00 intrinsics) and the full-resolution image size
KITTI_K = np.array([[718.856, 0.0, 607.1928], [0.0, 718.856, 185.2157], [0.0, 0.0, 1.0]])
KITTI_W, KITTI_H = 1241, 376
# outputs/transform_000785_000786.npy
T_785_786 = np.array([[9.99999363e-01, -7.87639940e-04, 8.08682728e-04, 3.92025607e-01],
                      [7.87321300e-04, 9.99999612e-01, 3.94265381e-04, 1.19524738e-01],
                      [-8.08992954e-04, -3.93628436e-04, 9.99999595e-01, -9.12156653e-01]])


def _normalize(x):
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def synth_scene(rng, n, R, t, K=KITTI_K, W=KITTI_W, H=KITTI_H, zmin=4.0, zmax=60.0, baseline=1.0):
    """n 3-D points visible in both views; x1 = R x0 + baseline * t."""
    Kinv = np.linalg.inv(K)
    X = np.zeros((0, 3))
    while X.shape[0] < n:
        m = 2 * (n - X.shape[0]) + 16
        uv = np.stack([rng.uniform(0, W, m), rng.uniform(0, H, m), np.ones(m)], 1)
        z = rng.uniform(zmin, zmax, m)
        P = (uv @ Kinv.T) * z[:, None]
        Q = P @ R.T + baseline * t
        ok = Q[:, 2] > 0.5
        q = Q[ok] @ K.T
        q = q[:, :2] / q[:, 2:3]
        inb = (q[:, 0] >= 0) & (q[:, 0] < W) & (q[:, 1] >= 0) & (q[:, 1] < H)
        X = np.concatenate([X, P[ok][inb]], 0)
    X = X[:n]
    p0 = X @ K.T
    p1 = (X @ R.T + baseline * t) @ K.T
    return X, p0[:, :2] / p0[:, 2:3], p1[:, :2] / p1[:, 2:3]


def synth_pair_f32(seed, n=1024, dim=256, frac=0.6, noise=0.3, T=T_785_786, K=KITTI_K, W=KITTI_W, H=KITTI_H,
                   n1=None):
    rng = np.random.default_rng(seed)
    n1 = n if n1 is None else n1
    R, t = T[:, :3], T[:, 3]
    _, kp0, kp1_true = synth_scene(rng, n, R, t, K, W, H)
    desc0 = _normalize(rng.standard_normal((n, dim)))
    m = min(int(round(frac * min(n, n1))), n1)
    src = rng.permutation(n)[:m]
    desc1 = np.empty((n1, dim))
    kp1 = np.empty((n1, 2))
    desc1[:m] = _normalize(desc0[src] + (noise / np.sqrt(dim)) * rng.standard_normal((m, dim)))
    kp1[:m] = kp1_true[src]
    desc1[m:] = _normalize(rng.standard_normal((n1 - m, dim)))
    kp1[m:] = np.stack([rng.uniform(0, W, n1 - m), rng.uniform(0, H, n1 - m)], 1)
    order = rng.permutation(n1)
    inv = np.empty(n1, np.int64)
    inv[order] = np.arange(n1)
    truth = np.full(n, -1, np.int64)
    truth[src] = inv[np.arange(m)]
    return dict(desc0=desc0.astype(np.float32), desc1=desc1[order].astype(np.float32),
                kp0=kp0.astype(np.float32), kp1=kp1[order].astype(np.float32), truth=truth, R=R, t=t)


def synth_pair_i8(seed, n=2048, frac=0.6, noise=6.0):
    rng = np.random.default_rng(seed)
    d0 = np.clip(np.round(rng.normal(0, 24, (n, 256))), -128, 127)
    m = int(round(frac * n))
    src = rng.permutation(n)[:m]
    d1 = np.empty((n, 256))
    d1[:m] = np.clip(np.round(d0[src] + rng.normal(0, noise, (m, 256))), -128, 127)
    d1[m:] = np.clip(np.round(rng.normal(0, 24, (n - m, 256))), -128, 127)
    order = rng.permutation(n)
    return d0.astype(np.int8), d1[order].astype(np.int8)


def synth_semi(rng, cells, p_key=0.25):
    """int8 [cells][65] logits: ~p_key of cells carry a keypoint (a positive peak),
    the rest are dustbin cells; negative background like quantized_image0.h."""
    semi = rng.integers(-110, -30, (cells, 65))
    semi[:, 64] = rng.integers(10, 40, cells)
    key = rng.random(cells) < p_key
    k = np.nonzero(key)[0]
    peak = rng.integers(0, 64, k.size)
    semi[k, peak] = rng.integers(20, 100, k.size)
    # a few weak positives elsewhere in some keypoint cells
    extra = k[rng.random(k.size) < 0.3]
    semi[extra, rng.integers(0, 64, extra.size)] = rng.integers(0, 15, extra.size)
    dust_off = k[rng.random(k.size) < 0.5]
    semi[dust_off, 64] = rng.integers(-20, 0, dust_off.size)
    return semi.astype(np.int8)


def synth_window_pair(seed, rows=24, cols=80, shift=(4, 4), jitter=1, noise=4.0):
    """frame1 cell (x, y) shows frame0 cell (x + shift_x + dx, y + shift_y + dy)."""
    rng = np.random.default_rng(seed)
    cells = rows * cols
    semi0 = synth_semi(rng, cells)
    desc0 = np.clip(np.round(rng.normal(0, 24, (cells, 256))), -128, 127).astype(np.int8)
    semi1 = synth_semi(rng, cells)
    desc1 = np.clip(np.round(rng.normal(0, 24, (cells, 256))), -128, 127)
    for x in range(cols):
        for y in range(rows):
            xs = x + shift[0] + rng.integers(-jitter, jitter + 1)
            ys = y + shift[1] + rng.integers(-jitter, jitter + 1)
            if 0 <= xs < cols and 0 <= ys < rows and rng.random() < 0.7:
                s, d = xs * rows + ys, x * rows + y
                desc1[d] = np.clip(np.round(desc0[s] + rng.normal(0, noise, 256)), -128, 127)
                semi1[d] = semi0[s]
    scale = np.float32(0.3562202453613281)
    f0 = dict(rows=rows, cols=cols, semi=semi0, desc=desc0, semi_scale=scale)
    f1 = dict(rows=rows, cols=cols, semi=semi1, desc=desc1.astype(np.int8), semi_scale=scale)
    return f0, f1


def synth_superpoint_outputs(seed, Hc, Wc, p_corner=0.3, dustbin=7.0):
    """Synthetic SuperPoint network outputs (what SuperPointNet.forward returns,
    pairwise_pnp.py:197-199): semi [65, Hc, Wc] and coarse_desc [256, Hc, Wc] float32.
    Logits ~ N(0, 1) with a dominant dustbin (channel 64, ~dustbin + N(0, 0.5)); a fraction
    p_corner of cells carries one spiked channel (a corner, +U(6, 11)), so that at
    conf_thresh 0.015 a few thousand pixels of a KITTI-size frame pass (as with real images).
    Descriptors: N(0, 1) per channel, smooth enough across cells to make bilinear sampling
    meaningful (a 2x2 box blur of white noise)."""
    rng = np.random.default_rng(seed)
    semi = rng.standard_normal((65, Hc, Wc)).astype(np.float32)
    semi[64] = (dustbin + 0.5 * rng.standard_normal((Hc, Wc))).astype(np.float32)
    spike = rng.random((Hc, Wc)) < p_corner
    ch = rng.integers(0, 64, (Hc, Wc))
    amp = rng.uniform(6.0, 11.0, (Hc, Wc)).astype(np.float32)
    hh, ww = np.nonzero(spike)
    semi[ch[hh, ww], hh, ww] += amp[hh, ww]
    w = rng.standard_normal((256, Hc + 1, Wc + 1)).astype(np.float32)
    desc = ((w[:, :-1, :-1] + w[:, 1:, :-1] + w[:, :-1, 1:] + w[:, 1:, 1:]) * np.float32(0.5)).astype(np.float32)
    return semi, desc
