"""ctypes front-end to the CPU ORACLE (oracle/liboracle.so) and, when built,
to the reference's own code compiled by oracle/Makefile (oracle/_ref/libmv_ref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (maveric-slam_amd/).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MV_ORACLE_SO: another build of the same sources (tests/test_sanitize.py: the ASan/UBSan one)
ORACLE_SO = os.environ.get("MV_ORACLE_SO") or os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libmv_ref.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_D = ctypes.c_double


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_scale_as_built.restype = _F
        L.orc_scale_as_built.argtypes = [_F]
        L.orc_approx_exp.restype = _F
        L.orc_compute_softmax.argtypes = [_F, _P, _I, _P, _P, _P]
        L.orc_compute_top_N.restype = _I
        L.orc_compute_top_N.argtypes = [_F, _P, _I, _I, _I, _P, _P, _P, _P]
        L.orc_window_match.restype = _I
        L.orc_window_match.argtypes = [_I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P]
        L.orc_svd3.argtypes = [_P, _P, _P, _P]
        L.orc_normalize_points.argtypes = [_I, _P, _P, _P]
        L.orc_reprojection_error.restype = _F
        L.orc_reprojection_error.argtypes = [_P, _P, _P]
        L.orc_ransac_essential_matrix.restype = _I
        L.orc_ransac_essential_matrix.argtypes = [_I, _P, _P, _P, _I, _F, _P, _P, _P]
        L.orc_recover_pose.argtypes = [_P, _P, _P, _P]
        L.orc_matmul_nt.argtypes = [_I, _I, _I, _P, _P, _P]
        L.orc_allpairs_f32.argtypes = [_P, _I, _P, _I, _I, _D, _P, _P]
        L.orc_row_argmax.argtypes = [_P, _I, _I, _D, _P, _P]
        L.orc_allpairs_i8.argtypes = [_P, _I, _P, _I, _P, _P]
        L.orc_trajectory_chain.argtypes = [_I, _P, _P, _P, _I, _P]
        L.orc_kp_heatmap.argtypes = [_P, _I, _I, _P]
        L.orc_pf_linearize.argtypes = [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P]
        L.orc_pose_normal_equations.argtypes = [_I, _P, _P, _P, _P, _P]
        L.orc_lba_schur.argtypes = [_I, _I, _I, _I, _P, _P]
        L.orc_run_nms.restype = _I
        L.orc_run_nms.argtypes = [_I, _I, _P, _P, _P]
        L.orc_two_way_f32.restype = _I
        L.orc_two_way_f32.argtypes = [_P, _I, _P, _I, _I, _D, _P, _P]
        L.orc_kp_select.restype = _I
        L.orc_kp_select.argtypes = [_P, _I, _I, _I, _I, _F, _I, _I, _I, _P]
        L.orc_kp_sample.argtypes = [_P, _I, _I, _I, _I, _I, _P, _P]
        L.orc_squared_dist.argtypes = [_P, _P, _P, _P, _P]
        L.orc_window_score.restype = _F
        L.orc_window_score.argtypes = [_I, _I, _I]
        L.orc_window_pass.restype = _I
        L.orc_window_pass.argtypes = [_F]
        L.orc_sp_resize.argtypes = [_P, _I, _I, _I, _I, _P]
        L.orc_sp_quantize.argtypes = [_P, ctypes.c_long, _D, _P]
        L.orc_sp_conv.argtypes = [_P, _I, _I, _P, _D, _I, _I, _P]
        L.orc_sp_min_gap.restype = _F
        L.orc_sp_min_gap.argtypes = [_P, _I, _I, _I, _D, _P]
        L.orc_sp_forward.argtypes = [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]
        _lib = L
    return _lib


REF_WINDOW_SO = os.path.join(HERE, "_ref", "libmv_ref_window.so")
_ref_window = None


def ref_window_available():
    return os.path.exists(REF_WINDOW_SO)


def ref_window():
    """The reference's own squared_dist (tracking_main.c:18-43) and window score line (:154,
    MATCH_THRESHOLD :12), extracted from its text and compiled by oracle/Makefile; build-container
    only."""
    global _ref_window
    if _ref_window is None:
        R = ctypes.CDLL(REF_WINDOW_SO)
        R.ref_squared_dist.argtypes = [_P, _P, _P, _P, _P]
        R.ref_window_score.restype = _F
        R.ref_window_score.argtypes = [_I, _I, _I]
        R.ref_window_pass.restype = _I
        R.ref_window_pass.argtypes = [_F]
        _ref_window = R
    return _ref_window


REF_NMS_SO = os.path.join(HERE, "_ref", "libmv_ref_nms.so")
_ref_nms = None


def ref_nms_available():
    return os.path.exists(REF_NMS_SO)


def ref_run_nms(semi, semi_scale, rows=192, cols=640, feature_rows=24, feature_cols=80):
    """The reference's own cell-level NMS: the body of src/run_nms.c's main (:44-174) with its
    grid helpers (:29-41), extracted from its text and compiled by oracle/Makefile with
    src/top_N.c (compute_softmax reached without a prototype, as in the reference binary: F7).
    Its grid is fixed at 24 x 80 cells (:62-63, 1920-entry arrays).  Returns (suppressions
    [(x, y, x', y')], survivors [(x, y)]) parsed from main's printf lines.  Build container only."""
    global _ref_nms
    if _ref_nms is None:
        R = ctypes.CDLL(REF_NMS_SO)
        R.ref_run_nms.restype = _I
        R.ref_run_nms.argtypes = [_I, _I, _I, _I, _F, _P, _F, _P, ctypes.c_char_p, _I]
        _ref_nms = R
    semi = np.ascontiguousarray(semi, dtype=np.int8)
    assert semi.shape == (1920, 65)
    desc = np.zeros((1920, 256), np.int8)  # main never reads the descriptors
    buf = ctypes.create_string_buffer(1 << 20)
    n = _ref_nms.ref_run_nms(rows, cols, feature_rows, feature_cols, float(semi_scale), _ptr(semi), 1.0, _ptr(desc),
                             buf, len(buf))
    assert n >= 0, "output buffer too small"
    sup, kp = [], []
    for line in buf.value.decode().splitlines():
        if "suppressing" in line:
            a, b = line.split(" suppressing ")
            sup.append(tuple(int(v) for v in a.strip("()").split()) + tuple(int(v) for v in b.strip("()").split()))
        else:
            kp.append(tuple(int(v) for v in line.split()))
    return sup, kp


REF_TRACK_SO = os.path.join(HERE, "_ref", "libmv_ref_track.so")
REF_TRACK_TS_SO = os.path.join(HERE, "_ref", "libmv_ref_track_ts.so")
REF_TRACK_O2_SO = os.path.join(HERE, "_ref", "libmv_ref_track_o2.so")
_ref_track = {}


def ref_track_available():
    return os.path.exists(REF_TRACK_SO) and os.path.exists(REF_TRACK_TS_SO)


def _ref_track_lib(true_scale, o2=False):
    key = (true_scale, o2)
    if key not in _ref_track:
        R = ctypes.CDLL(REF_TRACK_O2_SO if o2 else REF_TRACK_TS_SO if true_scale else REF_TRACK_SO)
        R.ref_tracking_main.restype = _I
        R.ref_tracking_main.argtypes = [_I, _I, _I, _I, _F, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]
        _ref_track[key] = R
    return _ref_track[key]


def ref_tracking_main(frame0, frame1, true_scale=False, o2=False):
    """The reference's OWN tracking driver: the body of src/tracking_main.c's main (:69-230 --
    softmax, top-N, the windowed match :103-194, RANSAC, pose) cut out of its text by
    oracle/Makefile, with src/top_N.c and src/pnp_solver.c compiled from source
    (oracle/ref_track_harness.c).  The frames take the place of quantized_pair0.h's image0_* /
    image1_* (24 x 80 cells: main's arrays hold 1920).  true_scale=False: compute_softmax /
    compute_top_N reached without a prototype as in the reference binary;
    true_scale=True: top_N.h in scope, the float scale arrives.  Returns dict(status (0, 1: top_N.c
    exit(1), 2: no matches), points1 (frame-0 pixels), points2 (frame-1 pixels), E, inliers, R1,
    R2, t, num_inliers).  num_inliers = -1 and E = NaN when no RANSAC hypothesis had an inlier (the
    reference then leaves both unwritten: main reads uninitialised stack).  o2: the as-built driver
    compiled at -O2 (the C0 timing build) instead of -O0 (the reference's CMake default).  Not
    thread-safe (main's rand() and the capture are process-global)."""
    if o2 and true_scale:
        raise ValueError("the -O2 build is the as-built driver only")
    R = _ref_track_lib(bool(true_scale), bool(o2))
    rows, cols = int(frame0["rows"]), int(frame0["cols"])
    assert rows * cols == 1920 and int(frame1["rows"]) == rows and int(frame1["cols"]) == cols
    s0 = np.ascontiguousarray(frame0["semi"], np.int8)
    d0 = np.ascontiguousarray(frame0["desc"], np.int8)
    s1 = np.ascontiguousarray(frame1["semi"], np.int8)
    d1 = np.ascontiguousarray(frame1["desc"], np.int8)
    n = ctypes.c_int(0)
    p1 = np.zeros((1000, 2), np.float32)
    p2 = np.zeros((1000, 2), np.float32)
    E = np.zeros(9, np.float32)
    inl = np.zeros(1000, np.int32)
    ni = ctypes.c_int(0)
    R1 = np.zeros(9, np.float32)
    R2 = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    st = R.ref_tracking_main(rows * 8, cols * 8, rows, cols, float(frame0["semi_scale"]), _ptr(s0), _ptr(d0),
                             float(frame1["semi_scale"]), _ptr(s1), _ptr(d1), ctypes.byref(n), _ptr(p1), _ptr(p2),
                             _ptr(E), _ptr(inl), ctypes.byref(ni), _ptr(R1), _ptr(R2), _ptr(t))
    k = n.value
    return dict(status=st, points1=p1[:k].copy(), points2=p2[:k].copy(), E=E.reshape(3, 3),
                inliers=inl[:max(ni.value, 0)].copy(), R1=R1.reshape(3, 3), R2=R2.reshape(3, 3), t=t,
                num_inliers=ni.value)


def ref_available():
    return os.path.exists(REF_SO)


_ref = None


def ref():
    """The reference's own top_N.c / pnp_solver.c / svd.h / gemmini matmul."""
    global _ref
    if _ref is None:
        R = ctypes.CDLL(REF_SO)
        R.compute_softmax.argtypes = [_F, _P, _P, _P, _P]
        R.compute_top_N.argtypes = [_F, _P, _I, _P, _P, _P, _P]
        R.normalize_points.argtypes = [_I, _P, _P, _P]
        R.compute_reprojection_error.restype = _F
        R.compute_reprojection_error.argtypes = [_P, _P, _P]
        R.ransac_essential_matrix.argtypes = [_I, _P, _P, _P, _I, _F, _P, _P, _P]
        R.recover_pose_from_essential_matrix.argtypes = [_P, _P, _P, _P]
        R.call_svd.argtypes = [_P, _P, _P, _P]
        R.ref_matmul_nt.argtypes = [_I, _I, _I, _P, _P, _P]
        R.ref_pf_error.argtypes = [_P, _P, _P, _P, _P]
        R.ref_h_factor.argtypes = [_P, _P]
        _ref = R
    return _ref


# --------------------------------------------------------------------------
# numpy-level helpers
# --------------------------------------------------------------------------
def scale_as_built(scale):
    return float(lib().orc_scale_as_built(float(scale)))


def compute_softmax(scale, semi):
    semi = np.ascontiguousarray(semi, dtype=np.int8)
    cells = semi.shape[0]
    nv = ctypes.c_int(0)
    mi = np.zeros(cells, np.int32)
    pr = np.zeros(cells, np.float32)
    lib().orc_compute_softmax(float(scale), _ptr(semi), cells, ctypes.byref(nv), _ptr(mi), _ptr(pr))
    return nv.value, mi, pr


def compute_top_N(scale, semi, N, cap=1000):
    semi = np.ascontiguousarray(semi, dtype=np.int8)
    ns = ctypes.c_int(0)
    pa = np.zeros(max(N, 1), np.int32)
    ix = np.zeros(max(N, 1), np.int32)
    pr = np.zeros(max(N, 1), np.float32)
    st = lib().orc_compute_top_N(float(scale), _ptr(semi), semi.shape[0], N, cap, ctypes.byref(ns),
                                 _ptr(pa), _ptr(ix), _ptr(pr))
    n = ns.value
    return st, pa[:n].copy(), ix[:n].copy(), pr[:n].copy()


class WindowParams(ctypes.Structure):
    _fields_ = [("shift_x", _I), ("shift_y", _I), ("radius", _I), ("max_matches", _I), ("as_built", _I)]


def window_match(rows, cols, desc0, max_idx0, probs0, desc1, patches1, indices1, as_built=True,
                 shift=(4, 4), radius=4, max_matches=150):
    desc0 = np.ascontiguousarray(desc0, np.int8)
    desc1 = np.ascontiguousarray(desc1, np.int8)
    max_idx0 = np.ascontiguousarray(max_idx0, np.int32)
    probs0 = np.ascontiguousarray(probs0, np.float32)
    patches1 = np.ascontiguousarray(patches1, np.int32)
    indices1 = np.ascontiguousarray(indices1, np.int32)
    p = WindowParams(shift[0], shift[1], radius, max_matches, 1 if as_built else 0)
    cap = max(max_matches, 1)
    p1 = np.zeros((cap, 2), np.float32)
    p2 = np.zeros((cap, 2), np.float32)
    q = np.zeros(cap, np.int32)
    sc = np.zeros(cap, np.float32)
    n = lib().orc_window_match(rows, cols, _ptr(desc0), _ptr(max_idx0), _ptr(probs0), _ptr(desc1),
                               len(patches1), _ptr(patches1), _ptr(indices1), ctypes.byref(p), _ptr(p1),
                               _ptr(p2), _ptr(q), _ptr(sc))
    return p1[:n].copy(), p2[:n].copy(), q[:n].copy(), sc[:n].copy()


def track_window(frame0, frame1, as_built=True, N=100, shift=(4, 4), radius=4, max_matches=150, cap=1000):
    """The whole tracking_main.c:84-194 front half on one pair.
    frame = dict(rows, cols (grid), semi[cells,65] i8, desc[cells,256] i8, semi_scale)."""
    s0, s1 = float(frame0["semi_scale"]), float(frame1["semi_scale"])
    if as_built:
        s0, s1 = scale_as_built(s0), scale_as_built(s1)
    _, mi0, pr0 = compute_softmax(s0, frame0["semi"])
    st, pa, ix, pr = compute_top_N(s1, frame1["semi"], N, cap)
    if st != 0:
        raise RuntimeError("top-N capacity exceeded")
    p1, p2, q, sc = window_match(frame0["rows"], frame0["cols"], frame0["desc"], mi0, pr0, frame1["desc"],
                                 pa, ix, as_built, shift, radius, max_matches)
    return dict(max_idx0=mi0, probs0=pr0, patches1=pa, indices1=ix, probs1=pr, points1=p1, points2=p2,
                query=q, score=sc)


def svd3(A):
    A = np.ascontiguousarray(A, np.float32).reshape(9)
    U = np.zeros(9, np.float32)
    S = np.zeros(3, np.float32)
    V = np.zeros(9, np.float32)
    lib().orc_svd3(_ptr(A), _ptr(U), _ptr(S), _ptr(V))
    return U.reshape(3, 3), S, V.reshape(3, 3)


def recover_pose(E):
    E = np.ascontiguousarray(E, np.float32).reshape(9)
    R1 = np.zeros(9, np.float32)
    R2 = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    lib().orc_recover_pose(_ptr(E), _ptr(R1), _ptr(R2), _ptr(t))
    return R1.reshape(3, 3), R2.reshape(3, 3), t


def ransac_essential_matrix(pts1, pts2, K, iters=10, thr=1.1):
    pts1 = np.ascontiguousarray(pts1, np.float32)
    pts2 = np.ascontiguousarray(pts2, np.float32)
    K = np.ascontiguousarray(K, np.float32)
    n = pts1.shape[0]
    E = np.zeros(9, np.float32)
    inl = np.zeros(max(n, 1000), np.int32)
    ni = ctypes.c_int(-1)
    st = lib().orc_ransac_essential_matrix(n, _ptr(pts1), _ptr(pts2), _ptr(K), iters, thr, _ptr(E), _ptr(inl),
                                           ctypes.byref(ni))
    return st, E.reshape(3, 3), inl[:max(ni.value, 0)].copy(), ni.value


def allpairs_f32(d0, d1, thresh=0.8):
    d0 = np.ascontiguousarray(d0, np.float32)
    d1 = np.ascontiguousarray(d1, np.float32)
    idx = np.zeros(d0.shape[0], np.int32)
    sc = np.zeros(d0.shape[0], np.float32)
    lib().orc_allpairs_f32(_ptr(d0), d0.shape[0], _ptr(d1), d1.shape[0], d0.shape[1], float(thresh), _ptr(idx),
                           _ptr(sc))
    return idx, sc


def matmul_nt(A, B):
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    C = np.zeros((A.shape[0], B.shape[0]), np.float32)
    lib().orc_matmul_nt(A.shape[0], B.shape[0], A.shape[1], _ptr(A), _ptr(B), _ptr(C))
    return C


def row_argmax(S, thresh=0.8):
    S = np.ascontiguousarray(S, np.float32)
    idx = np.zeros(S.shape[0], np.int32)
    sc = np.zeros(S.shape[0], np.float32)
    lib().orc_row_argmax(_ptr(S), S.shape[0], S.shape[1], float(thresh), _ptr(idx), _ptr(sc))
    return idx, sc


def allpairs_i8(d0, d1):
    d0 = np.ascontiguousarray(d0, np.int8)
    d1 = np.ascontiguousarray(d1, np.int8)
    idx = np.zeros(d0.shape[0], np.int32)
    dot = np.zeros(d0.shape[0], np.int32)
    lib().orc_allpairs_i8(_ptr(d0), d0.shape[0], _ptr(d1), d1.shape[0], _ptr(idx), _ptr(dot))
    return idx, dot


def trajectory_chain(rel, present=None, start=None, mode=0):
    """compute_trajectory.py:73-79 chain (mode 0 as built, 1 = T_rel @ pose): rel [len, 3, 4]
    float64 -> poses [len + 1, 3, 4]."""
    rel = np.ascontiguousarray(rel, np.float64).reshape(-1, 12)
    n = rel.shape[0]
    out = np.zeros((n + 1, 12), np.float64)
    pr = None if present is None else np.ascontiguousarray(present, np.int32)
    st = None if start is None else np.ascontiguousarray(start, np.float64).reshape(12)
    lib().orc_trajectory_chain(n, _ptr(rel), None if pr is None else _ptr(pr), None if st is None else _ptr(st),
                               int(mode), _ptr(out))
    return out.reshape(n + 1, 3, 4)


def kp_heatmap(semi):
    """SuperPointFrontend.run softmax -> heatmap (pairwise_pnp.py:204-220): semi [65, Hc, Wc]."""
    semi = np.ascontiguousarray(semi, np.float32)
    Hc, Wc = semi.shape[1], semi.shape[2]
    heat = np.zeros((Hc * 8, Wc * 8), np.float32)
    lib().orc_kp_heatmap(_ptr(semi), Hc, Wc, _ptr(heat))
    return heat


def kp_select(heat, H, W, conf=0.015, nms_dist=4, border=4, cap=1 << 20):
    """threshold + nms_fast + sort + border removal -> pts [n, 3] (x, y, conf) float32."""
    heat = np.ascontiguousarray(heat, np.float32)
    pts = np.zeros((min(cap, heat.size), 3), np.float32)
    n = lib().orc_kp_select(_ptr(heat), heat.shape[0], heat.shape[1], H, W, conf, nms_dist, border,
                            pts.shape[0], _ptr(pts))
    assert n >= 0, "more than cap candidates"
    return pts[:n].copy()


def kp_sample(desc, H, W, pts):
    """grid_sample + L2 normalise (pairwise_pnp.py:240-254): desc [256, Hc, Wc] -> [n, 256]."""
    desc = np.ascontiguousarray(desc, np.float32)
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
    out = np.zeros((pts.shape[0], 256), np.float32)
    if pts.shape[0]:
        lib().orc_kp_sample(_ptr(desc), desc.shape[1], desc.shape[2], H, W, pts.shape[0], _ptr(pts), _ptr(out))
    return out


def keypoints(semi, desc, H, W, conf=0.015, nms_dist=4, border=4):
    heat = kp_heatmap(semi)
    pts = kp_select(heat, H, W, conf, nms_dist, border)
    return pts, kp_sample(desc, H, W, pts), heat


def two_way_f32(d0, d1, nn_thresh=0.7):
    """nn_match_two_way (pairwise_pnp.py:281-323) on row-major descriptors [n, 256] ->
    (idx [n0] (-1: no match), dist [n0])."""
    d0 = np.ascontiguousarray(d0, np.float32)
    d1 = np.ascontiguousarray(d1, np.float32)
    idx = np.zeros(d0.shape[0], np.int32)
    dist = np.zeros(d0.shape[0], np.float32)
    k = lib().orc_two_way_f32(_ptr(d0), d0.shape[0], _ptr(d1), d1.shape[0], d0.shape[1], float(nn_thresh), _ptr(idx),
                              _ptr(dist))
    assert k >= 0, "nn_thresh < 0"
    return idx, dist


def run_nms(rows, cols, max_idx, probs):
    """src/run_nms.c:65-155 on compute_softmax outputs -> (max_idx', probs', kp [n, 2])."""
    mi = np.ascontiguousarray(max_idx, np.int32).copy()
    pr = np.ascontiguousarray(probs, np.float32).copy()
    kp = np.zeros((rows * cols, 2), np.float32)
    n = lib().orc_run_nms(rows, cols, _ptr(mi), _ptr(pr), _ptr(kp))
    return mi, pr, kp[:n].copy()


def pf_linearize(ldmk, pose, lid, pid, meas, cam):
    """projection factors -> (err [F, 2], J [F, 20] col-major 2x10, H [F, 100])."""
    ldmk = np.ascontiguousarray(ldmk, np.float32)
    pose = np.ascontiguousarray(pose, np.float32)
    lid = np.ascontiguousarray(lid, np.int32)
    pid = np.ascontiguousarray(pid, np.int32)
    meas = np.ascontiguousarray(meas, np.float32)
    cam = np.ascontiguousarray(cam, np.float32)
    F = lid.shape[0]
    err = np.zeros((F, 2), np.float32)
    J = np.zeros((F, 20), np.float32)
    H = np.zeros((F, 100), np.float32)
    lib().orc_pf_linearize(F, _ptr(ldmk), _ptr(pose), _ptr(lid), _ptr(pid), _ptr(meas), _ptr(cam), _ptr(err),
                           _ptr(J), _ptr(H))
    return err, J, H


def pose_normal_equations(off, H):
    off = np.ascontiguousarray(off, np.int32)
    H = np.ascontiguousarray(H, np.float32)
    P = off.shape[0] - 1
    HPP = np.zeros((P, 36), np.float32)
    g = np.zeros((P, 6), np.float32)
    ee = np.zeros(P, np.float32)
    lib().orc_pose_normal_equations(P, _ptr(off), _ptr(H), _ptr(HPP), _ptr(g), _ptr(ee))
    return HPP, g, ee


def lba_schur(P, L, LC, J, as_built=True, C=None):
    """local_bundle_adjustment.c main's Schur loop: J [L/LC, P*LC, 20] -> C [(6P+1)^2] col-major."""
    J = np.ascontiguousarray(J, np.float32)
    S = 6 * P + 1
    C = np.zeros(S * S, np.float32) if C is None else np.ascontiguousarray(C, np.float32).copy()
    lib().orc_lba_schur(P, L, LC, 1 if as_built else 0, _ptr(J), _ptr(C))
    return C


def lba_reference_J(P, L, LC):
    """the factor buffers main() uses: initialize_random_matrix(J, 2 P LC, 10) every chunk
    (local_bundle_adjustment.c:89-95, :149-151): element (i, j) of the column-major
    (2 P LC) x 10 matrix is i * 10 + j."""
    rows = 2 * P * LC
    m = np.zeros(rows * 10, np.float32)
    for j in range(10):
        for i in range(rows):
            m[j * rows + i] = i * 10 + j
    return np.tile(m.reshape(P * LC, 20)[None], (-(-L // LC), 1, 1))


_ref_lba = None


def ref_lba():
    """the reference's local_bundle_adjustment.c functions driven through main's loop
    (oracle/ref_lba_harness.c); build-container only."""
    global _ref_lba
    if _ref_lba is None:
        R = ctypes.CDLL(os.path.join(HERE, "_ref", "libmv_ref_lba.so"))
        R.ref_lba_schur_main.argtypes = [_I, _I, _I, _P]
        _ref_lba = R
    return _ref_lba


# ---------------- local feature pool: the reference's own code (oracle/ref_pool_harness.c) ----------------
REF_POOL_SO = os.path.join(HERE, "_ref", "libmv_ref_pool.so")
_ref_pool = None


def ref_pool_available():
    return os.path.exists(REF_POOL_SO)


def ref_pool():
    """include/local_feature_pool.h + src/local_feature_matching.c's generator, compiled from
    the reference's sources (oracle/Makefile); build-container only."""
    global _ref_pool
    if _ref_pool is None:
        R = ctypes.CDLL(REF_POOL_SO)
        R.ref_pool_run.argtypes = [_I, _I, _P, _P, _P]
        R.ref_pool_run.restype = _I
        R.ref_pool_replay.argtypes = [_I, _P, _P, _P, _P]
        R.ref_pool_replay.restype = _I
        _ref_pool = R
    return _ref_pool


def ref_pool_run(num_frames, nfeat=200):
    """the reference workload (srand(0), generate_word_ids): ids [F, nfeat], the table after
    each frame [F, capacity, 13] (key, occupied, word_id, frame_ptr, num_frames, frames[8]),
    sizes [F]"""
    R = ref_pool()
    cap = R.ref_pool_capacity()
    ids = np.zeros((num_frames, nfeat), np.int32)
    tab = np.zeros((num_frames, cap, 13), np.int32)
    sz = np.zeros(num_frames, np.int32)
    done = R.ref_pool_run(num_frames, nfeat, _ptr(ids), _ptr(tab), _ptr(sz))
    assert done == num_frames, "the reference pool gave up in frame %d" % done
    return ids, tab, sz


def ref_pool_replay(id_lists):
    """the same frame loop on the given per-frame id lists -> (tables, sizes, frames completed:
    len(id_lists), or the frame in which the reference exit()ed)"""
    R = ref_pool()
    cap = R.ref_pool_capacity()
    n = np.array([len(x) for x in id_lists], np.int32)
    flat = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int32) for x in id_lists]) if len(id_lists) else
                                np.zeros(0, np.int32))
    tab = np.zeros((len(id_lists), cap, 13), np.int32)
    sz = np.zeros(len(id_lists), np.int32)
    done = R.ref_pool_replay(len(id_lists), _ptr(n), _ptr(flat), _ptr(tab), _ptr(sz))
    return tab, sz, done


# ---------------- quantized SuperPoint front-end (sp_oracle.c) ----------------
SP_LAYERS = ("conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b",
             "convPa", "convPb", "convDa", "convDb")


class SpLayer(ctypes.Structure):
    _fields_ = [("w", _P), ("bias", _P), ("cin", _I), ("cout", _I), ("k", _I), ("w_scale", _D), ("out_scale", _D)]


class SpNet(ctypes.Structure):
    _fields_ = [("in_scale", _D), ("layer", SpLayer * 12)]


def sp_net(weights):
    """ctypes net from a weights dict (tests/golden/superpoint_qnonorm.npz layout: <layer>_w,
    <layer>_bias, <layer>_meta = [w_scale, w_zp, out_scale, out_zp], input_scale); the arrays
    are kept alive on the returned object"""
    net = SpNet()
    net.in_scale = float(weights["input_scale"])
    keep = []
    for i, n in enumerate(SP_LAYERS):
        w = np.ascontiguousarray(weights[n + "_w"], np.int8)
        b = np.ascontiguousarray(weights[n + "_bias"], np.float32)
        meta = weights[n + "_meta"]
        if meta[1] != 0 or meta[3] != 0:
            raise ValueError("zero points other than 0 are not restated")
        keep += [w, b]
        L = net.layer[i]
        L.w, L.bias = w.ctypes.data, b.ctypes.data
        L.cout, L.cin, L.k = w.shape[0], w.shape[1], w.shape[2]
        L.w_scale, L.out_scale = float(meta[0]), float(meta[2])
    net._keep = keep
    return net


def sp_resize(img, oh=192, ow=640):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros((oh, ow), np.float32)
    lib().orc_sp_resize(_ptr(img), img.shape[0], img.shape[1], oh, ow, _ptr(out))
    return out


def sp_quantize(x, scale):
    x = np.ascontiguousarray(x, np.float32)
    q = np.zeros(x.shape, np.int8)
    lib().orc_sp_quantize(_ptr(x), x.size, float(scale), _ptr(q))
    return q


def sp_conv(x, net, i, in_scale, relu, pool):
    """layer i of the net on CHW int8 x"""
    x = np.ascontiguousarray(x, np.int8)
    c, h, w = x.shape
    L = net.layer[i]
    out = np.zeros((L.cout, h // 2, w // 2) if pool else (L.cout, h, w), np.int8)
    lib().orc_sp_conv(_ptr(x), h, w, ctypes.byref(L), float(in_scale), int(relu), int(pool), _ptr(out))
    return out


def sp_forward(img, net, oh=192, ow=640):
    """(semi [cells][65], desc [cells][256], semi_scale, desc_scale, semi_raw, desc_raw)"""
    img = np.ascontiguousarray(img, np.uint8)
    cells = (oh // 8) * (ow // 8)
    semi = np.zeros((cells, 65), np.int8)
    desc = np.zeros((cells, 256), np.int8)
    sr = np.zeros((65, oh // 8, ow // 8), np.int8)
    dr = np.zeros((256, oh // 8, ow // 8), np.int8)
    ss, ds = ctypes.c_float(), ctypes.c_float()
    r = lib().orc_sp_forward(_ptr(img), img.shape[0], img.shape[1], oh, ow, ctypes.byref(net), _ptr(semi), _ptr(desc),
                             ctypes.byref(ss), ctypes.byref(ds), _ptr(sr), _ptr(dr))
    if r != 0:
        raise ValueError("orc_sp_forward: %d" % r)
    return semi, desc, np.float32(ss.value), np.float32(ds.value), sr, dr
