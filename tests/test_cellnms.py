"""The int8 path's cell-level NMS (src/run_nms.c:65-155).

run_nms.c is a standalone main that includes quantized_pair0.h, which the reference does not
ship: it cannot be built whole, so the oracle is a restatement, pinned to the body of
that main cut out of the reference text and compiled by oracle/Makefile
(tests/test_oracle_pinning.py::test_run_nms_pinned), plus the hand-checked cases below.  GPU (marked): the wavefront kernel equals
the sequential oracle bit for bit on the committed quantized frame (both softmax scales),
random frames, and the full-resolution 47 x 155 grid."""
import numpy as np
import pytest

import synth
from conftest import load_golden


def frame_softmax(orc, semi, scale):
    return orc.compute_softmax(scale, semi)[1:]  # (max_idx, probs)


def test_oracle_hand_cases(orc):
    rows, cols = 3, 4
    mi = np.full(rows * cols, 64, np.int32)
    pr = np.full(rows * cols, -1.0, np.float32)

    def put(gx, gy, px, py, p):
        mi[gx * rows + gy] = py * 8 + px
        pr[gx * rows + gy] = p

    put(1, 1, 7, 7, 0.5)  # pixel (15, 15)
    put(2, 1, 1, 6, 0.9)  # pixel (17, 14): within 4 px -> suppresses (15, 15)
    put(2, 2, 7, 7, 0.3)  # pixel (23, 23): far from both
    m2, p2, kp = orc.run_nms(rows, cols, mi, pr)
    assert m2[1 * rows + 1] == 64 and p2[1 * rows + 1] == 64.0
    assert sorted(map(tuple, kp.tolist())) == [(17.0, 14.0), (23.0, 23.0)]
    # patch 0 alone is never a maximum in the first pass (run_nms.c:110): cell 0 survives
    # even with a close weaker neighbour only when that neighbour is the one taken
    mi[:] = 64
    put(0, 0, 7, 7, 0.9)  # (7, 7), patch 0
    put(1, 0, 1, 7, 0.5)  # (9, 7)
    m2, _, kp = orc.run_nms(rows, cols, mi, pr)
    assert sorted(map(tuple, kp.tolist())) == [(7.0, 7.0)]  # second pass takes patch 0, suppresses (9, 7)


def _gpu(ctx, torch, rows, cols, frames):
    dev = torch.device("cuda:0")
    mi = torch.from_numpy(np.stack([f[0] for f in frames]).astype(np.int32)).to(dev)
    pr = torch.from_numpy(np.stack([f[1] for f in frames]).astype(np.float32)).to(dev)
    n = torch.zeros(len(frames), dtype=torch.int32, device=dev)
    kp = torch.zeros((len(frames), rows * cols, 2), dtype=torch.float32, device=dev)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.run_nms_batch(rows, cols, mi, pr, n, kp)
    torch.cuda.synchronize()
    ctx.set_stream(None)
    return mi.cpu().numpy(), pr.cpu().numpy(), n.cpu().numpy(), kp.cpu().numpy()


@pytest.mark.gpu
def test_gpu_run_nms_bit_exact(ctx, orc, torch_cuda):
    g = load_golden("quantized_image0.npz")
    rows, cols = int(g["feature_rows"]), int(g["feature_cols"])
    frames = [frame_softmax(orc, g["semi"], s) for s in (float(g["semi_scale"]), 0.0, 0.05)]
    rng = np.random.default_rng(3)
    for k in range(5):
        frames.append(frame_softmax(orc, synth.synth_semi(rng, rows * cols, p_key=0.5), float(g["semi_scale"])))
    mi, pr, n, kp = _gpu(ctx, torch_cuda, rows, cols, frames)
    for b, (m0, p0) in enumerate(frames):
        m2, p2, k2 = orc.run_nms(rows, cols, m0, p0)
        assert (mi[b] == m2).all() and (pr[b].view(np.int32) == p2.view(np.int32)).all(), b
        assert n[b] == k2.shape[0] and (kp[b, :n[b]] == k2).all(), b
    # the full-resolution KITTI grid
    rows, cols = 47, 155
    frames = [frame_softmax(orc, synth.synth_semi(rng, rows * cols, p_key=0.6), 0.04) for _ in range(3)]
    mi, pr, n, kp = _gpu(ctx, torch_cuda, rows, cols, frames)
    for b, (m0, p0) in enumerate(frames):
        m2, p2, k2 = orc.run_nms(rows, cols, m0, p0)
        assert (mi[b] == m2).all() and n[b] == k2.shape[0] and (kp[b, :n[b]] == k2).all(), b
