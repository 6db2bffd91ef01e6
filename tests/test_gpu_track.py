"""GPU parity: the whole tracking_main.c pipeline through the drop-in track()
(include/tracking.h) and mv_track_pair_host(), against the oracle."""
import ctypes

import numpy as np
import pytest

import synth
from conftest import load_golden

pytestmark = pytest.mark.gpu


class Frame(ctypes.Structure):  # include/frame.h (same layout as the reference's frame.h:7-30)
    _fields_ = [("rows", ctypes.c_int), ("cols", ctypes.c_int), ("channels", ctypes.c_int),
                ("data", ctypes.c_void_p), ("num_features", ctypes.c_int), ("feature_rows", ctypes.c_int),
                ("feature_cols", ctypes.c_int), ("feature_xs", ctypes.c_void_p), ("feature_ys", ctypes.c_void_p),
                ("semi_scale", ctypes.c_float), ("semi", ctypes.c_void_p), ("desc_scale", ctypes.c_float),
                ("desc", ctypes.c_void_p)]


def make_frame(f, keep):
    semi = np.ascontiguousarray(f["semi"], np.int8)
    desc = np.ascontiguousarray(f["desc"], np.int8)
    keep += [semi, desc]
    fr = Frame()
    fr.rows, fr.cols = f["rows"] * 8, f["cols"] * 8
    fr.feature_rows, fr.feature_cols = f["rows"], f["cols"]
    fr.semi_scale = float(f["semi_scale"])
    fr.desc_scale = 1.0
    fr.semi = semi.ctypes.data
    fr.desc = desc.ctypes.data
    return fr


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


@pytest.mark.parametrize("case", ["self", "syn1", "syn2"])
def test_track_dropin_matches_tracking_main(ctx, orc, image0, case):
    import mvtrack

    L = mvtrack.lib()
    f0, f1 = (image0, image0) if case == "self" else synth.synth_window_pair(int(case[-1]))
    keep = []
    F0, F1 = make_frame(f0, keep), make_frame(f1, keep)
    T = (ctypes.c_float * 12)()
    # tracking_main.c calls compute_softmax/compute_top_N without prototypes (F7): AS_BUILT
    st = L.track(ctypes.byref(F0), ctypes.byref(F1), 4, 4, 9, ctypes.c_float(0.9), T)
    assert st == 0
    exp = load_golden("expected_outputs.npz")
    T = np.array(T, np.float32).reshape(3, 4)
    assert (bits(T[:, :3]) == bits(exp["pose_built_R1"])).all() and (bits(T[:, 3]) == bits(exp["pose_built_t"])).all()
    # the matches behind it
    prm = mvtrack.track_params(mvtrack.AS_BUILT)
    st, T2, p1, p2 = ctx.track_pair_host(prm, f0["rows"], f0["cols"], f0, f1)
    r = orc.track_window(f0, f1, as_built=True)
    assert st in (0, mvtrack.MV_ERR_DEGENERATE)
    assert (p1 == r["points1"]).all() and (p2 == r["points2"]).all()


def test_track_pair_intended_matches_oracle(ctx, orc):
    import mvtrack

    f0, f1 = synth.synth_window_pair(3)
    prm = mvtrack.track_params(mvtrack.AS_INTENDED)
    st, T, p1, p2 = ctx.track_pair_host(prm, f0["rows"], f0["cols"], f0, f1)
    r = orc.track_window(f0, f1, as_built=False)
    assert (p1 == r["points1"]).all() and (p2 == r["points2"]).all()
    assert np.isfinite(T).all()


def test_track_null_last_frame_is_identity(ctx):
    import mvtrack

    L = mvtrack.lib()
    T = (ctypes.c_float * 12)()
    assert L.track(None, None, 4, 4, 9, ctypes.c_float(0.9), T) == 0
    assert np.allclose(np.array(T).reshape(3, 4), np.hstack([np.eye(3), np.zeros((3, 1))]))


def test_dropin_threads_get_their_own_default_context(ctx, orc, image0):
    """The reference's API runs on an implicit context; it is per thread, so concurrent
    callers never share staging or scratch.  Four threads run track() and the
    host window match on different pairs at once; every result equals the serial one."""
    import threading

    import mvtrack

    L = mvtrack.lib()
    L.mv_default_context.restype = ctypes.c_void_p
    pairs = [(image0, image0)] + [synth.synth_window_pair(k) for k in (1, 2, 3)]
    keep = []
    frames = [(make_frame(a, keep), make_frame(b, keep)) for a, b in pairs]

    def run_track(k):
        T = (ctypes.c_float * 12)()
        st = L.track(ctypes.byref(frames[k][0]), ctypes.byref(frames[k][1]), 4, 4, 9, ctypes.c_float(0.9), T)
        return st, bits(np.array(T, np.float32))

    serial = [run_track(k) for k in range(4)]
    out, ctxs, errs = {}, {}, []
    alive = threading.Barrier(4, timeout=120)  # all four contexts exist at once

    def worker(k):
        try:
            ctxs[k] = L.mv_default_context()
            for rep in range(5):
                out[(k, rep)] = run_track(k)
            alive.wait()
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    assert len(set(ctxs.values())) == 4 and L.mv_default_context() not in ctxs.values()
    for (k, rep), (st, T) in out.items():
        assert st == serial[k][0] and (T == serial[k][1]).all(), (k, rep)
