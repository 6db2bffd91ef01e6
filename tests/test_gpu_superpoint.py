"""GPU parity: the quantized SuperPoint front-end (include/superpoint.h) --
uint8 frames -> int8 semi / desc + run()'s scales, bit-identical to the CPU oracle
(oracle/sp_oracle.c, pinned bit for bit to PyTorch's quantized kernels in test_superpoint.py)
on the reference's KITTI frames, random frames, partial tiles at a small network size and a
flat frame; and at the reference's own golden (quantized_image0.h, 93.6 / 92.3 % int8-exact,
SURVEY 8(c)'s platform gap)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def weights():
    return dict(load_golden("superpoint_qnonorm.npz"))


@pytest.fixture(scope="module")
def sp(ctx, weights):
    import mvtrack

    net = mvtrack.SuperPoint(ctx, weights)
    yield net
    net.close()


def _run(ctx, torch, sp, imgs, oh, ow):
    dev = torch.device("cuda:0")
    x = torch.from_numpy(np.ascontiguousarray(np.stack(imgs), np.uint8)).to(dev)
    ctx.set_stream(torch.cuda.current_stream())
    try:
        semi, desc, ss, ds = sp.forward(x, oh, ow)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
    return semi.cpu().numpy(), desc.cpu().numpy(), ss.cpu().numpy(), ds.cpu().numpy()


def _check(orc, weights, imgs, got, oh, ow):
    net = orc.sp_net(weights)
    semi, desc, ss, ds = got
    for b, img in enumerate(imgs):
        s2, d2, ss2, ds2, _, _ = orc.sp_forward(img, net, oh, ow)
        assert (semi[b] == s2).all(), ("semi", b, (semi[b] != s2).sum())
        assert (desc[b] == d2).all(), ("desc", b, (desc[b] != d2).sum())
        assert ss[b] == ss2 and ds[b] == ds2, (b, ss[b], ss2, ds[b], ds2)


def test_superpoint_kitti_frames_vs_oracle_and_golden(ctx, orc, torch_cuda, sp, weights):
    ims = load_golden("kitti00_images.npz")
    imgs = [ims["img_000000"], ims["img_000001"]]
    got = _run(ctx, torch_cuda, sp, imgs, 192, 640)
    _check(orc, weights, imgs, got, 192, 640)
    g = load_golden("quantized_image0.npz")
    assert (got[0][0] == g["semi"]).mean() >= 0.93 and (got[1][0] == g["desc"]).mean() >= 0.92
    assert got[2][0] == g["semi_scale"]


@pytest.mark.parametrize("shape,oh,ow", [((376, 1241), 192, 640), ((120, 200), 64, 96), ((30, 50), 24, 40)])
def test_superpoint_random_frames_vs_oracle(ctx, orc, torch_cuda, sp, weights, shape, oh, ow):
    rng = np.random.default_rng(oh + ow)
    imgs = [rng.integers(0, 256, shape, dtype=np.uint8) for _ in range(3)]
    # smooth structure (a random image is mostly noise for the net): blurred blobs
    yy, xx = np.mgrid[0:shape[0], 0:shape[1]]
    imgs.append((127 + 120 * np.sin(xx / 7.0) * np.cos(yy / 5.0)).astype(np.uint8))
    got = _run(ctx, torch_cuda, sp, imgs, oh, ow)
    _check(orc, weights, imgs, got, oh, ow)


@pytest.mark.parametrize("nf,shape,oh,ow", [(4, (64, 64), 64, 64), (8, (96, 128), 64, 128), (3, (200, 300), 192, 224)])
def test_superpoint_head_block_forms(ctx, orc, torch_cuda, sp, weights, nf, shape, oh, ow):
    """k_sp_head's forms: whole 32-cell blocks and whole 8-block workgroups (4 x 64 cells: the
    unguarded form, frames under 8 blocks so the presence pass stays separate; 8 x 128 cells:
    4 blocks per frame, 2 frames per workgroup) and the guarded form (3 x 672 cells: 21 blocks per
    frame, 63 blocks, not a whole number of workgroups)"""
    rng = np.random.default_rng(nf * 1000 + oh)
    yy, xx = np.mgrid[0:shape[0], 0:shape[1]]
    imgs = [(127 + 120 * np.sin(xx / (5.0 + k)) * np.cos(yy / (4.0 + k)) + rng.integers(-20, 21, shape)).clip(0, 255)
            .astype(np.uint8) for k in range(nf)]
    got = _run(ctx, torch_cuda, sp, imgs, oh, ow)
    _check(orc, weights, imgs, got, oh, ow)


def test_superpoint_flat_frame(ctx, orc, torch_cuda, sp, weights):
    imgs = [np.zeros((64, 64), np.uint8), np.full((64, 64), 255, np.uint8)]
    got = _run(ctx, torch_cuda, sp, imgs, 64, 64)
    _check(orc, weights, imgs, got, 64, 64)


def test_superpoint_frontend_mirror(ctx, torch_cuda, weights):
    """SuperPointFrontend.run's return shapes and values (superpoint_inference.py:178-208)"""
    import mvtrack

    fe = mvtrack.SuperPointFrontend(weights, ctx=ctx)
    img = load_golden("kitti00_images.npz")["img_000000"]
    s0, q0, s1, q1, outs = fe.run(img)
    assert tuple(q0.shape) == (1, 65, 24, 80) and tuple(q1.shape) == (1, 256, 24, 80) and outs is None
    g = load_golden("quantized_image0.npz")
    semi = q0[0].permute(2, 1, 0).reshape(-1, 65).cpu().numpy()
    assert (semi == g["semi"]).mean() >= 0.93 and np.float32(s0) == g["semi_scale"]
    fe.net.close()


def test_superpoint_into_window_track(ctx, orc, torch_cuda, sp, weights):
    """image -> network -> the windowed int8 track (tracking_main.c's path, both semantics): the
    GPU front-end's frames give the same matched points as the oracle's front-end + track"""
    import mvtrack

    ims = load_golden("kitti00_images.npz")
    imgs = [ims["img_000000"], ims["img_000001"]]
    semi, desc, ss, ds = _run(ctx, torch_cuda, sp, imgs, 192, 640)
    net = orc.sp_net(weights)
    ref = [orc.sp_forward(im, net) for im in imgs]
    frames = [dict(rows=24, cols=80, semi=semi[b], desc=desc[b], semi_scale=np.float32(ss[b])) for b in range(2)]
    oframes = [dict(rows=24, cols=80, semi=r[0], desc=r[1], semi_scale=np.float32(r[2])) for r in ref]
    for sem, as_built in ((mvtrack.AS_BUILT, True), (mvtrack.AS_INTENDED, False)):
        prm = mvtrack.track_params(sem)
        st, T, p1, p2 = ctx.track_pair_host(prm, 24, 80, frames[0], frames[1])
        r = orc.track_window(oframes[0], oframes[1], as_built=as_built)
        assert (p1 == r["points1"]).all() and (p2 == r["points2"]).all()
        assert len(p1) > 0


def test_superpoint_one_net_two_streams(ctx, orc, torch_cuda, sp, weights):
    """the net's activation buffers are shared by every context; two forwards issued on
    two contexts with their own streams and no host synchronisation between them must both equal
    the oracle (the second forward waits on the first one's completion event)."""
    import mvtrack

    torch = torch_cuda
    dev = torch.device("cuda:0")
    ims = load_golden("kitti00_images.npz")
    rng = np.random.default_rng(5)
    sets = [[ims["img_000000"], ims["img_000001"]] * 4, [rng.integers(0, 256, (376, 1241), dtype=np.uint8)
                                                          for _ in range(8)]]
    ctx2 = mvtrack.Context(0)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    try:
        xs = [torch.from_numpy(np.ascontiguousarray(np.stack(s), np.uint8)).to(dev) for s in sets]
        torch.cuda.synchronize()
        ctx.set_stream(s1)
        ctx2.set_stream(s2)
        outs = []
        for rep in range(3):
            outs.append(sp.forward(xs[0], 192, 640, ctx=ctx))
            outs.append(sp.forward(xs[1], 192, 640, ctx=ctx2))
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(None)
        ctx2.close()
    for k, o in enumerate(outs):
        imgs = sets[k % 2][:2]
        got = tuple(t.cpu().numpy()[:2] for t in o)
        _check(orc, weights, imgs, got, 192, 640)


def test_network_int8_descriptors_through_int8_allpairs(ctx, orc, torch_cuda, sp):
    """configs[4] on descriptors the NETWORK produced (not synthetic draws): the int8 desc of KITTI
    00 frames 000000 / 000001 from mv_superpoint_forward_dev (1920 cells x 256 each, bit-exact to
    the oracle above) matched all-pairs on the int8 matrix cores (k_i8t_match, both 1024-row
    workgroups of the pair live), indices and exact dots equal to the oracle's; both directions."""
    ims = load_golden("kitti00_images.npz")
    imgs = [ims["img_000000"], ims["img_000001"]]
    _, desc, _, _ = _run(ctx, torch_cuda, sp, imgs, 192, 640)
    dev = torch_cuda.device("cuda:0")
    for a, c in ((desc[0], desc[1]), (desc[1], desc[0])):
        n = a.shape[0]
        cap = 2048
        D0 = np.zeros((1, cap, 256), np.int8)
        D1 = np.zeros((1, cap, 256), np.int8)
        D0[0, :n], D1[0, :n] = a, c
        nn_ = torch_cuda.full((1,), n, dtype=torch_cuda.int32, device=dev)
        idx = torch_cuda.full((1, cap), -7, dtype=torch_cuda.int32, device=dev)
        dot = torch_cuda.zeros((1, cap), dtype=torch_cuda.int32, device=dev)
        ctx.set_stream(torch_cuda.cuda.current_stream())
        try:
            ctx.match_allpairs_i8(torch_cuda.from_numpy(D0).to(dev), torch_cuda.from_numpy(D1).to(dev), nn_, nn_, idx,
                                  dot)
            torch_cuda.cuda.synchronize()
        finally:
            ctx.set_stream(None)
        i2, d2 = orc.allpairs_i8(a, c)
        got_i, got_d = idx.cpu().numpy()[0], dot.cpu().numpy()[0]
        assert (got_i[:n] == i2).all() and (got_d[:n] == d2).all()
        assert (got_i[n:] == -1).all()
        assert (i2 >= 0).sum() > 100  # consecutive frames: many cells re-observed above cos 0.9


def test_int8_allpairs_adaptive_dispatch(ctx, orc, torch_cuda, sp):
    """mv_match_allpairs_i8_dev's adaptive dispatch: after a call whose pairs k_i8t_match mostly
    handed back (the network's own descriptors), the next calls run k_i8_match directly; then a
    batch of well-separated synthetic descriptors -- every call's indices and dots equal to the
    oracle's, whichever kernel ran (the pinned count is read without waiting, so the switch may
    come a call later: both paths are checked over the sequence)."""
    ims = load_golden("kitti00_images.npz")
    imgs = [ims["img_000000"], ims["img_000001"]]
    _, desc, _, _ = _run(ctx, torch_cuda, sp, imgs, 192, 640)
    dev = torch_cuda.device("cuda:0")
    cap, n = 2048, desc[0].shape[0]
    rng = np.random.default_rng(5)
    syn = rng.integers(-60, 61, (2, n, 256)).astype(np.int8)
    syn[1, :n // 2] = syn[0, :n // 2]  # half the rows re-observed exactly
    cases = [(desc[0], desc[1])] * 4 + [(syn[0], syn[1])] * 2 + [(desc[1], desc[0])] * 2
    exp = {}
    ctx.set_stream(torch_cuda.cuda.current_stream())
    try:
        for k, (a, c) in enumerate(cases):
            D0 = np.zeros((2, cap, 256), np.int8)
            D1 = np.zeros((2, cap, 256), np.int8)
            D0[:, :n], D1[:, :n] = a, c
            nn_ = torch_cuda.full((2,), n, dtype=torch_cuda.int32, device=dev)
            idx = torch_cuda.full((2, cap), -7, dtype=torch_cuda.int32, device=dev)
            dot = torch_cuda.zeros((2, cap), dtype=torch_cuda.int32, device=dev)
            ctx.match_allpairs_i8(torch_cuda.from_numpy(D0).to(dev), torch_cuda.from_numpy(D1).to(dev), nn_, nn_, idx,
                                  dot)
            torch_cuda.cuda.synchronize()
            key = (a.tobytes()[:64], c.tobytes()[:64])
            if key not in exp:
                exp[key] = orc.allpairs_i8(a, c)
            i2, d2 = exp[key]
            for b in range(2):
                got_i, got_d = idx.cpu().numpy()[b], dot.cpu().numpy()[b]
                assert (got_i[:n] == i2).all() and (got_d[:n] == d2).all(), (k, b)
                assert (got_i[n:] == -1).all(), (k, b)
    finally:
        ctx.set_stream(None)
