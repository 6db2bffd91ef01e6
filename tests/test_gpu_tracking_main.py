"""GPU parity against the reference's OWN tracking driver (src/tracking_main.c:68-228, extracted
and run in the build container: tests/golden/make_tracking_main_fixtures.py): the HIP softmax,
top-N, windowed match, stub RANSAC and pose give the reference's match list, inliers, E and pose
bit for bit -- on the real KITTI pair quantized_image0 -> frame 000001 (51 matches as built), the
self pair, synthetic pairs, F7 effective scales 2 / -2, top_N.c's exit(1) (MV_ERR_CAPACITY) and
the empty match list; in the as-built build and with the true scale."""
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

sys.path.insert(0, GOLDEN)
from make_tracking_main_fixtures import FIELDS, tracking_main_cases  # noqa: E402

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


@pytest.mark.parametrize("mode", ["built", "true"])
def test_gpu_window_track_equals_reference_main(ctx, mode):
    import mvtrack

    g = load_golden("tracking_main_ref.npz")
    wp = mvtrack.window_params(mvtrack.AS_BUILT)
    seen = 0
    for name, (f0, f1) in tracking_main_cases().items():
        ref = {k: g["%s_%s_%s" % (name, mode, k)] for k in FIELDS}
        s0, s1 = float(f0["semi_scale"]), float(f1["semi_scale"])
        if mode == "built":
            s0, s1 = mvtrack.scale_as_built(s0), mvtrack.scale_as_built(s1)
        _, mi0, pr0 = ctx.softmax_host(s0, f0["semi"])
        st, pa, ix, _ = ctx.top_n_host(s1, f1["semi"], 100)
        if int(ref["status"]) == 1:  # top_N.c exit(1)
            assert st == mvtrack.MV_ERR_CAPACITY, name
            continue
        assert st == 0, name
        p1, p2, _ = ctx.window_match_host(wp, 24, 80, f0["desc"], mi0, pr0, f1["desc"], pa, ix)
        assert p1.shape == ref["points1"].shape and (p1 == ref["points1"]).all(), (name, mode)
        assert (p2 == ref["points2"]).all(), (name, mode)
        if int(ref["status"]) == 2:  # no match: the reference's rand() % 0
            assert len(p1) == 0
            continue
        E, inl, ni = ctx.ransac_stub_host(p1, p2, 1.1)
        if int(ref["num_inliers"]) < 0:  # no hypothesis had an inlier: E and the count unwritten
            assert ni == 0, name
        else:
            assert ni == int(ref["num_inliers"]) and (inl == ref["inliers"]).all(), name
            assert (bits(E) == bits(ref["E"])).all(), name
            R1, R2, t = ctx.recover_pose_host(E)
            assert (bits(R1) == bits(ref["R1"])).all() and (bits(R2) == bits(ref["R2"])).all(), name
            assert (bits(t) == bits(ref["t"])).all(), name
        seen += 1
    assert seen >= 7


def test_gpu_track_pair_on_the_real_kitti_pair(ctx):
    """mv_track_pair_host (the batched seam's single-pair form) on quantized_image0 -> 000001: the
    reference main's 51 matches as built"""
    import mvtrack

    g = load_golden("tracking_main_ref.npz")
    f0, f1 = tracking_main_cases()["kitti01"]
    st, T, p1, p2 = ctx.track_pair_host(mvtrack.track_params(mvtrack.AS_BUILT), 24, 80, f0, f1)
    assert st in (0, mvtrack.MV_ERR_DEGENERATE)
    assert len(p1) == 51 and (p1 == g["kitti01_built_points1"]).all() and (p2 == g["kitti01_built_points2"]).all()
    assert (bits(T[:, :3]) == bits(g["kitti01_built_R1"])).all() and (bits(T[:, 3]) == bits(g["kitti01_built_t"])).all()
