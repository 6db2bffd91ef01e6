"""mvtrack -- Python front-end over libmaveric_hip.so (the C ABI of include/*.h).

The product is the C/HIP library; this module only marshals numpy arrays and
torch device tensors into it (ctypes), for tests, smoke() and bench.py.
It never computes anything itself and never falls back to the CPU: if the
library or a gfx950 device is missing, every call raises.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MV_LIB: an alternate in-tree build of the same library (a tracing or A/B variant built on the
# CPU by tools/build_variant.sh); the default is the shipping build
LIB_PATH = os.environ.get("MV_LIB") or os.path.join(HERE, "libmaveric_hip.so")
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

MV_OK = 0
MV_ERR_INVALID_ARG = -1
MV_ERR_CAPACITY = -2
MV_ERR_HIP = -3
MV_ERR_NO_DEVICE = -4
MV_ERR_NO_POINTS = -5
MV_ERR_OUT_OF_MEMORY = -6
MV_ERR_DEGENERATE = -7
MV_ERR_IO = -8
AS_BUILT = 0
AS_INTENDED = 1

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_D = ctypes.c_double


SCREENS = {"i8": 0, "f16": 1, "i8s": 2}  # mv_allpairs_screen (i8s: int8 against a staged image)


class MVError(RuntimeError):
    pass


class WindowParams(ctypes.Structure):
    _fields_ = [("shift_x", _I), ("shift_y", _I), ("radius", _I), ("max_matches", _I), ("semantics", _I),
                ("match_thresh_sq", _D), ("prob_thresh", _D)]


class PoseParams(ctypes.Structure):
    _fields_ = [("fx", _F), ("fy", _F), ("cx", _F), ("cy", _F), ("semantics", _I), ("hypotheses", _I),
                ("inlier_thresh", _F), ("refine_iters", _I), ("seed", ctypes.c_ulonglong)]


class KpParams(ctypes.Structure):
    _fields_ = [("conf_thresh", _F), ("nms_dist", _I), ("border", _I)]


class SpLayer(ctypes.Structure):
    _fields_ = [("w", _P), ("bias", _P), ("cin", _I), ("cout", _I), ("k", _I), ("w_scale", _D), ("out_scale", _D)]


class SpWeights(ctypes.Structure):
    _fields_ = [("in_scale", _D), ("layer", SpLayer * 12)]


class TrackParams(ctypes.Structure):
    _fields_ = [("window", WindowParams), ("pose", PoseParams), ("top_n", _I), ("valid_cap", _I)]


def build(force=False):
    """Compile the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-s", "-C", CSRC, "-j8"]
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    subprocess.run(cmd, check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        # PyTorch-ROCm bundles its own libamdhip64 (same SONAME, different file name in
        # its NEEDED entries).  Load it first so this library binds to the SAME HIP
        # runtime; loading ours first would make torch pull in a second runtime copy.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "mv_version": (_I, []),
            "mv_status_string": (ctypes.c_char_p, [_I]),
            "mv_last_status": (_I, []),
            "mv_last_error_message": (ctypes.c_char_p, []),
            "mv_device_count": (_I, []),
            "mv_context_create": (_I, [_I, ctypes.POINTER(_P)]),
            "mv_context_destroy": (_I, [_P]),
            "mv_context_set_stream": (_I, [_P, _P]),
            "mv_context_use_own_stream": (_I, [_P]),
            "mv_context_set_allpairs_screen": (_I, [_P, _I]),
            "mv_context_allpairs_screen": (_I, [_P]),
            "mv_context_stream": (_P, [_P]),
            "mv_context_synchronize": (_I, [_P]),
            "mv_context_reserve": (_I, [_P, _I, _I]),
            "mv_default_context": (_P, []),
            "mv_profile_enable": (_I, [_I]),
            "mv_profile_query": (_I, [ctypes.c_char_p, ctypes.POINTER(_D), ctypes.POINTER(_I)]),
            "mv_window_params_default": (None, [_P]),
            "mv_pose_params_default": (None, [_P, _I]),
            "mv_track_params_default": (None, [_P, _I]),
            "mv_scale_as_built": (_F, [_F]),
            "mv_softmax_host": (_I, [_P, _F, _P, _I, _P, _P, _P]),
            "mv_top_n_host": (_I, [_P, _F, _P, _I, _I, _I, _P, _P, _P, _P]),
            "mv_window_match_host": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P]),
            "mv_softmax_batch_dev": (_I, [_P, _I, _I, _P, _P, _P, _P, _P]),
            "mv_top_n_select_batch_dev": (_I, [_P, _I, _I, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
            "mv_window_match_batch_dev": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P,
                                               _P]),
            "mv_match_allpairs_f32_dev": (_I, [_P, _I, _I, _P, _P, _P, _P, _D, _P, _P]),
            "mv_match_allpairs_f32_prepare_dev": (_I, [_P, _I, _I, _P, _P]),
            "mv_match_allpairs_f32_run_dev": (_I, [_P, _I, _I, _P, _P, _P, _P, _D, _P, _P]),
            "mv_match_allpairs_f32_run_prepare_dev": (_I, [_P, _I, _I, _P, _P, _P, _P, _D, _P, _P, _I, _I, _P, _P]),
            "mv_match_sequence_f32_dev": (_I, [_P, _I, _I, _P, _P, _D, _P, _P]),
            "mv_match_sequence_f32_run_prepare_dev": (_I, [_P, _I, _I, _P, _P, _D, _P, _P, _I, _I, _P, _P]),
            "mv_match_allpairs_i8_dev": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P]),
            "mv_match_two_way_f32_dev": (_I, [_P, _I, _I, _P, _P, _P, _P, _D, _P, _P]),
            "mv_run_nms_batch_dev": (_I, [_P, _I, _I, _I, _P, _P, _P, _P]),
            "mv_projection_factors_dev": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
            "mv_pose_normal_equations_dev": (_I, [_P, _I, _P, _P, _P, _P, _P]),
            "mv_lba_schur_dev": (_I, [_P, _I, _I, _I, _I, _I, _P, _P]),
            "mv_pose_batch_dev": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P]),
            "mv_superpoint_create": (_I, [_P, _P, ctypes.POINTER(_P)]),
            "mv_superpoint_destroy": (_I, [_P]),
            "mv_superpoint_forward_dev": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
            "mv_superpoint_forward_raw_dev": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
            "mv_pose_from_matches_dev": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
            "mv_ransac_stub_host": (_I, [_P, _I, _P, _P, _F, _P, _P, _P]),
            "mv_recover_pose_host": (_I, [_P, _P, _P, _P, _P]),
            "mv_svd3_host": (_I, [_P, _P, _P, _P, _P]),
            "mv_track_pair_host": (_I, [_P, _P, _I, _I, _F, _P, _P, _F, _P, _P, _P, _P, _P, _P]),
            "compute_top_N": (None, [_F, _P, _I, _P, _P, _P, _P]),
            "compute_softmax": (None, [_F, _P, _P, _P, _P]),
            "normalize_points": (None, [_I, _P, _P, _P]),
            "compute_essential_matrix": (None, [_I, _P, _P, _P]),
            "compute_reprojection_error": (_F, [_P, _P, _P]),
            "ransac_essential_matrix": (None, [_I, _P, _P, _P, _I, _F, _P, _P, _P]),
            "recover_pose_from_essential_matrix": (None, [_P, _P, _P, _P]),
            "track": (_I, [_P, _P, _I, _I, _I, _F, _P]),
            "mv_kp_params_default": (None, [_P]),
            "mv_keypoints_dev": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P]),
            "mv_keypoints_host": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P]),
            "mv_trajectory_chain_dev": (_I, [_P, _I, _I, _P, _P, _P, _I, _P]),
            "mv_trajectory_rebase_dev": (_I, [_P, _I, _I, _P, _I, _P]),
            "mv_trajectory_chain_host": (_I, [_P, _I, _P, _P, _P, _I, _P]),
            "mv_write_pose_txt": (_I, [ctypes.c_char_p, _P]),
            "mv_write_trajectory_ply": (_I, [ctypes.c_char_p, _I, _P]),
            "mv_read_transform_npy": (_I, [ctypes.c_char_p, _P]),
            "mv_compute_trajectory": (_I, [_P, _I, _I, ctypes.c_char_p, ctypes.c_char_p, _I, ctypes.POINTER(_I)]),
            "mv_local_feature_init": (None, [_P]),
            "mv_local_feature_init_with_id": (None, [_P, _I, _I]),
            "mv_local_feature_update": (None, [_P, _I]),
            "mv_local_feature_remove_old_frame": (ctypes.c_bool, [_P, _I]),
            "mv_local_feature_pool_init": (None, [_P]),
            "mv_local_feature_pool_insert": (_I, [_P, _I, _P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_bool)]),
            "mv_local_feature_pool_delete": (_I, [_P, _I]),
            "mv_local_feature_pool_remove_old": (_I, [_P, _I]),
            "mv_local_feature_pool_valid_keys": (None, [_P, ctypes.POINTER(_I), _P]),
            "mv_local_feature_pool_load_factor": (_F, [_P]),
            "mv_local_feature_pool_check_invariant": (_I, [_P, _I]),
            "mv_local_feature_pool_track_frame": (_I, [_P, _I, _I, _P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _np(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def kp_params(**kw):
    """mv_kp_params (conf_thresh 0.015, nms_dist 4, border 4 -- pairwise_pnp.py:589-591, :99)."""
    p = KpParams()
    lib().mv_kp_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


# ---------------- trajectory (include/trajectory.h; python/compute_trajectory.py) ----------------
CHAIN_AS_BUILT, CHAIN_COMPOSE = 0, 1


def write_pose_txt(path, pose):
    """np.savetxt(pose[:3, :], fmt='%.6f') (compute_trajectory.py:49-51), in C."""
    p = np.ascontiguousarray(pose, np.float64).reshape(-1)[:12].copy()
    check(lib().mv_write_pose_txt(os.fsencode(path), _np(p)), "write_pose_txt")


def write_trajectory_ply(path, xyz):
    """write_ply (compute_trajectory.py:6-43), in C."""
    x = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
    check(lib().mv_write_trajectory_ply(os.fsencode(path), x.shape[0], _np(x)), "write_trajectory_ply")


def read_transform_npy(path):
    """A (3, 4) float64 .npy read by the library's C reader -> (status, [3, 4])."""
    T = np.zeros(12, np.float64)
    st = lib().mv_read_transform_npy(os.fsencode(path), _np(T))
    return st, T.reshape(3, 4)


def sequence_shard(frames, world, rank):
    """Frames [lo, hi) of a track of `frames` frames that `rank` of `world` matches in sequence
    mode: the frames - 1 pairs (b, b + 1) are split into contiguous, near-equal ranges, and a
    rank's frames run one past its last pair, so neighbouring ranks share one boundary frame
    and every pair is matched by exactly one rank -- no data-path collective.  A rank with no
    pair gets lo == hi."""
    if frames < 2 or world < 1 or not 0 <= rank < world:
        raise ValueError("sequence_shard: frames >= 2, 0 <= rank < world")
    pairs = frames - 1
    p_lo = rank * pairs // world
    p_hi = (rank + 1) * pairs // world
    return (p_lo, p_hi + 1) if p_hi > p_lo else (p_lo, p_lo)


def chain_sharded(chain_local, rebase, gather, rank, rel_local, mode):
    """A sequence sharded over ranks in order (rank r holds transforms [k_r, k_{r+1})):
    each rank chains its shard from the identity (chain_local(rel) -> poses [len+1, 3, 4]),
    the ranks exchange their shard's end pose (gather(last) -> [world] list, rank order:
    the RCCL all-gather on GPUs), every rank folds the ends of the ranks before it into its
    start pose (host, world x 3x4) and re-bases its poses on it (rebase(poses, start)).
    Returns this rank's poses [len+1, 3, 4]; its pose 0 is the previous rank's last pose."""
    import numpy as _n

    poses = chain_local(rel_local)
    ends = gather(_n.asarray(poses[-1], _n.float64))
    start = _n.eye(4)[:3].copy()
    for r in range(rank):  # start <- end_r applied after start (the chain rule, k_rebase order)
        E = _n.asarray(ends[r], _n.float64)
        nxt = _n.zeros((3, 4))
        for i in range(3):
            for c in range(4):
                v = E[i, 0] * start[0, c]
                v = v + E[i, 1] * start[1, c]
                v = v + E[i, 2] * start[2, c]
                if c == 3:
                    v = v + E[i, 3] if mode == CHAIN_COMPOSE else E[i, 3] + start[i, 3]
                nxt[i, c] = v
        start = nxt
    if rank == 0:
        return poses
    return rebase(poses, start)


# ---------------- local feature pool (include/feature_pool.h; include/local_feature_pool.h) ----------------
MAX_LOCAL_FRAMES, LOCAL_FEATURE_POOL_CAPACITY = 8, 3000


class LocalFeature(ctypes.Structure):
    """mv_local_feature = the reference's LocalFeature (local_feature_pool.h:16-22)."""
    _fields_ = [("word_id", _I), ("frame_ptr", _I), ("num_frames", _I), ("frames", _I * MAX_LOCAL_FRAMES),
                ("coords_3D", _F * 3)]


class _LfpEntry(ctypes.Structure):
    _fields_ = [("key", _I), ("value", LocalFeature), ("is_occupied", ctypes.c_bool)]


class _LfpPool(ctypes.Structure):
    _fields_ = [("entries", _LfpEntry * LOCAL_FEATURE_POOL_CAPACITY), ("size", _I), ("capacity", _I)]


class LocalFeaturePool:
    """The local feature pool (host, C): the reference's LocalFeaturePool API with error codes
    in place of its exit() calls.  table() -> int32 [capacity, 13] (key, occupied, word_id,
    frame_ptr, num_frames, frames[8]), the layout the parity tests compare slot by slot."""

    def __init__(self):
        self._p = _LfpPool()
        ctypes.memset(ctypes.byref(self._p), 0, ctypes.sizeof(self._p))
        lib().mv_local_feature_pool_init(ctypes.byref(self._p))

    @property
    def size(self):
        return self._p.size

    @property
    def capacity(self):
        return self._p.capacity

    def insert(self, key, frame_num):
        """local_feature_pool_insert of a feature first seen at frame_num -> (status,
        inserted, the entry's LocalFeature or None)"""
        f = LocalFeature()
        lib().mv_local_feature_init_with_id(ctypes.byref(f), key, frame_num)
        out = _P()
        ins = ctypes.c_bool(False)
        st = lib().mv_local_feature_pool_insert(ctypes.byref(self._p), key, ctypes.byref(f), ctypes.byref(out),
                                                ctypes.byref(ins))
        feat = ctypes.cast(out, ctypes.POINTER(LocalFeature)).contents if out.value else None
        return st, ins.value, feat

    def delete(self, key):
        return lib().mv_local_feature_pool_delete(ctypes.byref(self._p), key)

    def remove_old(self, current_frame_num):
        return lib().mv_local_feature_pool_remove_old(ctypes.byref(self._p), current_frame_num)

    def valid_keys(self):
        keys = np.zeros(LOCAL_FEATURE_POOL_CAPACITY, np.int32)
        n = _I(0)
        lib().mv_local_feature_pool_valid_keys(ctypes.byref(self._p), ctypes.byref(n), _np(keys))
        return keys[:n.value].copy()

    def load_factor(self):
        return float(lib().mv_local_feature_pool_load_factor(ctypes.byref(self._p)))

    def check_invariant(self, cur_frame):
        return lib().mv_local_feature_pool_check_invariant(ctypes.byref(self._p), cur_frame)

    def track_frame(self, frame_num, word_ids):
        ids = np.ascontiguousarray(word_ids, np.int32)
        return lib().mv_local_feature_pool_track_frame(ctypes.byref(self._p), frame_num, ids.size, _np(ids))

    def table(self):
        # an entry is 16 words: key, word_id, frame_ptr, num_frames, frames[8], coords[3],
        # is_occupied (byte 0 of word 15)
        assert ctypes.sizeof(_LfpEntry) == 64
        raw = np.frombuffer(self._p, dtype=np.int32, count=LOCAL_FEATURE_POOL_CAPACITY * 16).reshape(-1, 16)
        t = np.empty((self._p.capacity, 13), np.int32)
        t[:, 0] = raw[:, 0]
        t[:, 1] = raw[:, 15] & 0xFF
        t[:, 2:13] = raw[:, 1:12]
        return t


def _t(x):
    """device pointer of a torch tensor (or None)"""
    return None if x is None else ctypes.c_void_p(x.data_ptr())


def check(st, what=""):
    if st != MV_OK:
        L = lib()
        raise MVError("%s: %s (%s)" % (what, L.mv_status_string(st).decode(), L.mv_last_error_message().decode()))


def device_count():
    return lib().mv_device_count()


def profile_enable(on=True):
    check(lib().mv_profile_enable(1 if on else 0), "profile_enable")


def profile_query(kernel):
    """(total device ms, launches) of `kernel` since profile_enable(True)."""
    ms = ctypes.c_double(0)
    n = ctypes.c_int(0)
    check(lib().mv_profile_query(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)), "profile_query")
    return ms.value, n.value


def window_params(semantics=AS_BUILT, **kw):
    p = WindowParams()
    lib().mv_window_params_default(ctypes.byref(p))
    p.semantics = semantics
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def pose_params(semantics=AS_INTENDED, **kw):
    p = PoseParams()
    lib().mv_pose_params_default(ctypes.byref(p), semantics)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def track_params(semantics=AS_BUILT):
    p = TrackParams()
    lib().mv_track_params_default(ctypes.byref(p), semantics)
    return p


def scale_as_built(scale):
    return float(lib().mv_scale_as_built(float(scale)))


class Context:
    """An mv_context on one device.  `stream` may be a torch.cuda.Stream."""

    def __init__(self, device=0):
        L = lib()
        h = ctypes.c_void_p()
        check(L.mv_context_create(device, ctypes.byref(h)), "mv_context_create")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().mv_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream):
        """Run later calls on `stream` (a torch.cuda.Stream -- torch's default stream is HIP's null
        stream, handle 0, and is used as such); None: back to the context's own stream."""
        if stream is None:
            check(lib().mv_context_use_own_stream(self.h), "use_own_stream")
        else:
            check(lib().mv_context_set_stream(self.h, ctypes.c_void_p(stream.cuda_stream)), "set_stream")

    def set_allpairs_screen(self, screen):
        """'i8' (default: one pass, frame 1 quantised in-kernel), 'f16' or 'i8s' (int8 against a
        staged image): how the fp32 all-pairs match screens before its exact re-score."""
        check(lib().mv_context_set_allpairs_screen(self.h, SCREENS[screen]), "set_allpairs_screen")

    def allpairs_screen(self):
        r = lib().mv_context_allpairs_screen(self.h)
        if r < 0:
            check(r, "allpairs_screen")
        return {v: k for k, v in SCREENS.items()}[r]

    def synchronize(self):
        check(lib().mv_context_synchronize(self.h), "synchronize")

    def reserve(self, batch, cap):
        check(lib().mv_context_reserve(self.h, batch, cap), "reserve")

    # ---------------- host-pointer calls (numpy) ----------------
    def softmax_host(self, scale, semi):
        semi = np.ascontiguousarray(semi, np.int8)
        cells = semi.shape[0]
        nv = ctypes.c_int(0)
        mi = np.zeros(cells, np.int32)
        pr = np.zeros(cells, np.float32)
        check(lib().mv_softmax_host(self.h, float(scale), _np(semi), cells, ctypes.byref(nv), _np(mi), _np(pr)),
              "softmax_host")
        return nv.value, mi, pr

    def top_n_host(self, scale, semi, N, cap=1000):
        semi = np.ascontiguousarray(semi, np.int8)
        ns = ctypes.c_int(0)
        pa = np.zeros(N, np.int32)
        ix = np.zeros(N, np.int32)
        pr = np.zeros(N, np.float32)
        st = lib().mv_top_n_host(self.h, float(scale), _np(semi), semi.shape[0], N, cap, ctypes.byref(ns), _np(pa),
                                 _np(ix), _np(pr))
        n = max(ns.value, 0)
        return st, pa[:n].copy(), ix[:n].copy(), pr[:n].copy()

    def window_match_host(self, params, rows, cols, desc0, max_idx0, probs0, desc1, patches1, indices1):
        desc0 = np.ascontiguousarray(desc0, np.int8)
        desc1 = np.ascontiguousarray(desc1, np.int8)
        max_idx0 = np.ascontiguousarray(max_idx0, np.int32)
        probs0 = np.ascontiguousarray(probs0, np.float32)
        patches1 = np.ascontiguousarray(patches1, np.int32)
        indices1 = np.ascontiguousarray(indices1, np.int32)
        M = params.max_matches
        p1 = np.zeros((M, 2), np.float32)
        p2 = np.zeros((M, 2), np.float32)
        q = np.zeros(M, np.int32)
        nm = ctypes.c_int(0)
        check(lib().mv_window_match_host(self.h, ctypes.byref(params), rows, cols, _np(desc0), _np(max_idx0),
                                         _np(probs0), _np(desc1), len(patches1), _np(patches1), _np(indices1),
                                         ctypes.byref(nm), _np(p1), _np(p2), _np(q)), "window_match_host")
        n = nm.value
        return p1[:n].copy(), p2[:n].copy(), q[:n].copy()

    def ransac_stub_host(self, pts1, pts2, thresh=1.1):
        pts1 = np.ascontiguousarray(pts1, np.float32)
        pts2 = np.ascontiguousarray(pts2, np.float32)
        n = pts1.shape[0]
        E = np.zeros(9, np.float32)
        inl = np.zeros(max(n, 1000), np.int32)
        ni = ctypes.c_int(0)
        check(lib().mv_ransac_stub_host(self.h, n, _np(pts1), _np(pts2), float(thresh), _np(E), _np(inl),
                                        ctypes.byref(ni)), "ransac_stub_host")
        return E.reshape(3, 3), inl[:ni.value].copy(), ni.value

    def recover_pose_host(self, E):
        E = np.ascontiguousarray(E, np.float32).reshape(9)
        R1 = np.zeros(9, np.float32)
        R2 = np.zeros(9, np.float32)
        t = np.zeros(3, np.float32)
        check(lib().mv_recover_pose_host(self.h, _np(E), _np(R1), _np(R2), _np(t)), "recover_pose_host")
        return R1.reshape(3, 3), R2.reshape(3, 3), t

    def svd3_host(self, A):
        A = np.ascontiguousarray(A, np.float32).reshape(9)
        U = np.zeros(9, np.float32)
        S = np.zeros(3, np.float32)
        V = np.zeros(9, np.float32)
        check(lib().mv_svd3_host(self.h, _np(A), _np(U), _np(S), _np(V)), "svd3_host")
        return U.reshape(3, 3), S, V.reshape(3, 3)

    def track_pair_host(self, params, rows, cols, f0, f1):
        """f = dict(semi_scale, semi [cells,65] i8, desc [cells,256] i8)"""
        s0 = np.ascontiguousarray(f0["semi"], np.int8)
        d0 = np.ascontiguousarray(f0["desc"], np.int8)
        s1 = np.ascontiguousarray(f1["semi"], np.int8)
        d1 = np.ascontiguousarray(f1["desc"], np.int8)
        M = params.window.max_matches
        T = np.zeros((3, 4), np.float32)
        p1 = np.zeros((M, 2), np.float32)
        p2 = np.zeros((M, 2), np.float32)
        nm = ctypes.c_int(0)
        st = lib().mv_track_pair_host(self.h, ctypes.byref(params), rows, cols, float(f0["semi_scale"]), _np(s0),
                                      _np(d0), float(f1["semi_scale"]), _np(s1), _np(d1), _np(T), ctypes.byref(nm),
                                      _np(p1), _np(p2))
        n = nm.value
        return st, T, p1[:n].copy(), p2[:n].copy()

    # ---------------- batched device calls (torch tensors on this device) ----------------
    def softmax_batch(self, scales, semi, max_idx, probs, num_valid):
        B, cells = semi.shape[0], semi.shape[1]
        check(lib().mv_softmax_batch_dev(self.h, B, cells, _t(scales), _t(semi), _t(max_idx), _t(probs),
                                         _t(num_valid)), "softmax_batch")

    def projection_factors(self, landmarks, poses, cameras, ldmk_id, pose_id, meas, err, J=None, H=None):
        """Device tensors (include/factors.h): err [F, 2], J [F, 20], H [F, 100]."""
        check(lib().mv_projection_factors_dev(self.h, ldmk_id.shape[0], _t(landmarks), _t(poses), _t(cameras),
                                              _t(ldmk_id), _t(pose_id), _t(meas), _t(err), _t(J), _t(H)),
              "projection_factors")

    def pose_normal_equations(self, pose_offsets, J, HPP, g, ee):
        check(lib().mv_pose_normal_equations_dev(self.h, pose_offsets.shape[0] - 1, _t(pose_offsets), _t(J), _t(HPP),
                                                 _t(g), _t(ee)), "pose_normal_equations")

    def lba_schur(self, num_poses, num_ldmks, chunk, J, C, semantics=AS_INTENDED):
        """local-BA Schur back-end on device tensors J [B, chunks, P*chunk, 20], C [B, S*S]."""
        check(lib().mv_lba_schur_dev(self.h, J.shape[0], num_poses, num_ldmks, chunk, int(semantics), _t(J), _t(C)),
              "lba_schur")

    def run_nms_batch(self, rows, cols, max_idx, probs, num_kp, kp):
        """src/run_nms.c cell NMS on device tensors max_idx/probs [B, cells] (in place)."""
        check(lib().mv_run_nms_batch_dev(self.h, max_idx.shape[0], rows, cols, _t(max_idx), _t(probs), _t(num_kp),
                                         _t(kp)), "run_nms_batch")

    def top_n_select_batch(self, max_idx, probs, N, cap, num_sel, patches, indices, sel_probs, status):
        B, cells = max_idx.shape[0], max_idx.shape[1]
        check(lib().mv_top_n_select_batch_dev(self.h, B, cells, _t(max_idx), _t(probs), N, cap, _t(num_sel),
                                              _t(patches), _t(indices), _t(sel_probs), _t(status)),
              "top_n_select_batch")

    def window_match_batch(self, params, rows, cols, desc0, max_idx0, probs0, desc1, num_sel, patches1, indices1,
                           num_matches, points1, points2, query_of_match=None):
        B, N = patches1.shape[0], patches1.shape[1]
        check(lib().mv_window_match_batch_dev(self.h, ctypes.byref(params), B, rows, cols, _t(desc0), _t(max_idx0),
                                              _t(probs0), _t(desc1), N, _t(num_sel), _t(patches1), _t(indices1),
                                              _t(num_matches), _t(points1), _t(points2), _t(query_of_match)),
              "window_match_batch")

    def match_allpairs_f32(self, desc0, desc1, n0, n1, match_idx, match_score, thresh=0.8):
        B, cap = desc0.shape[0], desc0.shape[1]
        check(lib().mv_match_allpairs_f32_dev(self.h, B, cap, _t(n0), _t(n1), _t(desc0), _t(desc1), float(thresh),
                                              _t(match_idx), _t(match_score)), "match_allpairs_f32")

    def match_allpairs_f32_prepare(self, desc1, n1):
        """Stage frame 1 of a batch on the auxiliary stream (see mv_match_allpairs_f32_prepare_dev)."""
        B, cap = desc1.shape[0], desc1.shape[1]
        check(lib().mv_match_allpairs_f32_prepare_dev(self.h, B, cap, _t(n1), _t(desc1)), "match_allpairs_f32_prepare")

    def match_allpairs_f32_run(self, desc0, desc1, n0, n1, match_idx, match_score, thresh=0.8):
        """Match a batch staged by match_allpairs_f32_prepare(desc1, n1)."""
        B, cap = desc0.shape[0], desc0.shape[1]
        check(lib().mv_match_allpairs_f32_run_dev(self.h, B, cap, _t(n0), _t(n1), _t(desc0), _t(desc1), float(thresh),
                                                  _t(match_idx), _t(match_score)), "match_allpairs_f32_run")

    def match_allpairs_f32_run_prepare(self, desc0, desc1, n0, n1, match_idx, match_score, next_desc1, next_n1,
                                       thresh=0.8):
        """Match the prepared batch (desc1, n1) and stage the next batch's frame 1 in the same
        launch (mv_match_allpairs_f32_run_prepare_dev); the next batch is then the prepared one."""
        B, cap = desc0.shape[0], desc0.shape[1]
        nB, ncap = next_desc1.shape[0], next_desc1.shape[1]
        check(lib().mv_match_allpairs_f32_run_prepare_dev(self.h, B, cap, _t(n0), _t(n1), _t(desc0), _t(desc1),
                                                          float(thresh), _t(match_idx), _t(match_score), nB, ncap,
                                                          _t(next_n1), _t(next_desc1)), "match_allpairs_f32_run_prepare")

    def keypoints(self, semi, coarse_desc, H, W, num_kp, kp, conf, desc, status, heat=None, params=None):
        """Device tensors: semi [B, 65, Hc, Wc], coarse_desc [B, 256, Hc, Wc] (network outputs)
        -> num_kp [B], kp [B, cap, 2], conf [B, cap], desc [B, cap, 256], status [B]
        (SuperPointFrontend.run after the forward; include/keypoints.h)."""
        B, Hc, Wc = semi.shape[0], semi.shape[2], semi.shape[3]
        p = params or kp_params()
        check(lib().mv_keypoints_dev(self.h, ctypes.byref(p), B, Hc, Wc, int(H), int(W), _t(semi), _t(coarse_desc),
                                     kp.shape[1], _t(num_kp), _t(kp), _t(conf), _t(desc), _t(heat), _t(status)),
              "keypoints")

    def keypoints_host(self, semi, coarse_desc, H, W, cap=4096, params=None):
        """numpy, one frame: semi [65, Hc, Wc], coarse_desc [256, Hc, Wc] -> (pts [n, 3] (x, y,
        conf), desc [n, 256], status)."""
        semi = np.ascontiguousarray(semi, np.float32)
        cd = np.ascontiguousarray(coarse_desc, np.float32)
        Hc, Wc = semi.shape[1], semi.shape[2]
        kp = np.zeros((cap, 2), np.float32)
        conf = np.zeros(cap, np.float32)
        desc = np.zeros((cap, 256), np.float32)
        n = ctypes.c_int(0)
        p = params or kp_params()
        st = lib().mv_keypoints_host(self.h, ctypes.byref(p), Hc, Wc, int(H), int(W), _np(semi), _np(cd), cap,
                                     ctypes.byref(n), _np(kp), _np(conf), _np(desc))
        if st not in (MV_OK, MV_ERR_CAPACITY):
            check(st, "keypoints_host")
        k = n.value
        return np.concatenate([kp[:k], conf[:k, None]], axis=1), desc[:k].copy(), st

    def trajectory_chain(self, rel, poses, present=None, start=None, mode=CHAIN_AS_BUILT):
        """Device tensors: rel [B, len, 3, 4] float64 -> poses [B, len + 1, 3, 4] (k_chain)."""
        B, n = rel.shape[0], rel.shape[1]
        check(lib().mv_trajectory_chain_dev(self.h, B, n, _t(rel), _t(present), _t(start), int(mode), _t(poses)),
              "trajectory_chain")

    def trajectory_rebase(self, base, poses, mode=CHAIN_AS_BUILT):
        """Device tensors: poses [B, len1, 3, 4] re-based on base [B, 3, 4] in place (k_rebase)."""
        check(lib().mv_trajectory_rebase_dev(self.h, poses.shape[0], poses.shape[1], _t(base), int(mode), _t(poses)),
              "trajectory_rebase")

    def trajectory_chain_host(self, rel, present=None, start=None, mode=CHAIN_AS_BUILT):
        """numpy: one sequence rel [len, 3, 4] float64 -> poses [len + 1, 3, 4] (on the GPU)."""
        r = np.ascontiguousarray(rel, np.float64).reshape(-1, 12)
        out = np.zeros((r.shape[0] + 1, 12), np.float64)
        pr = None if present is None else np.ascontiguousarray(present, np.int32)
        st = None if start is None else np.ascontiguousarray(start, np.float64).reshape(12)
        check(lib().mv_trajectory_chain_host(self.h, r.shape[0], _np(r), None if pr is None else _np(pr),
                                             None if st is None else _np(st), int(mode), _np(out)),
              "trajectory_chain_host")
        return out.reshape(-1, 3, 4)

    def compute_trajectory(self, start_frame, end_frame, pose_dir, out_dir, mode=CHAIN_AS_BUILT):
        """compute_trajectory.py main() with the chain on the GPU; returns poses written."""
        n = ctypes.c_int(0)
        check(lib().mv_compute_trajectory(self.h, int(start_frame), int(end_frame), os.fsencode(pose_dir),
                                          os.fsencode(out_dir), int(mode), ctypes.byref(n)), "compute_trajectory")
        return n.value

    def match_two_way_f32(self, desc0, desc1, n0, n1, match_idx, match_dist=None, nn_thresh=0.7):
        """nn_match_two_way (pairwise_pnp.py:281-323) on device tensors: match_idx [B, cap]."""
        B, cap = desc0.shape[0], desc0.shape[1]
        check(lib().mv_match_two_way_f32_dev(self.h, B, cap, _t(n0), _t(n1), _t(desc0), _t(desc1), float(nn_thresh),
                                             _t(match_idx), _t(match_dist)), "match_two_way_f32")

    def match_allpairs_i8(self, desc0, desc1, n0, n1, match_idx, match_dot):
        B, cap = desc0.shape[0], desc0.shape[1]
        check(lib().mv_match_allpairs_i8_dev(self.h, B, cap, _t(n0), _t(n1), _t(desc0), _t(desc1), _t(match_idx),
                                             _t(match_dot)), "match_allpairs_i8")

    def pose_batch(self, params, n, pts0, pts1, T, num_inliers, status):
        B, cap = pts0.shape[0], pts0.shape[1]
        check(lib().mv_pose_batch_dev(self.h, ctypes.byref(params), B, cap, _t(n), _t(pts0), _t(pts1), _t(T),
                                      _t(num_inliers), _t(status)), "pose_batch")

    def match_sequence_f32(self, desc, n, match_idx, match_score, thresh=0.8):
        """Consecutive frames desc[F][cap][256] -> pairs (b, b + 1): match_idx[F-1][cap]
        (mv_match_sequence_f32_dev; every frame quantised once)."""
        F, cap = desc.shape[0], desc.shape[1]
        check(lib().mv_match_sequence_f32_dev(self.h, F, cap, _t(n), _t(desc), float(thresh), _t(match_idx),
                                              _t(match_score)), "match_sequence_f32")

    def match_sequence_f32_run_prepare(self, desc, n, match_idx, match_score, next_desc, next_n, thresh=0.8):
        """Match the prepared chunk desc[F] (pairs b, b + 1) and stage the next chunk's frames in the
        same launch (mv_match_sequence_f32_run_prepare_dev); prepare the first chunk with
        match_allpairs_f32_prepare(desc, n)."""
        F, cap = desc.shape[0], desc.shape[1]
        nF, ncap = next_desc.shape[0], next_desc.shape[1]
        check(lib().mv_match_sequence_f32_run_prepare_dev(self.h, F, cap, _t(n), _t(desc), float(thresh),
                                                          _t(match_idx), _t(match_score), nF, ncap, _t(next_n),
                                                          _t(next_desc)), "match_sequence_f32_run_prepare")

    def pose_from_matches(self, params, n0, match_idx, kp0, kp1, T, num_matches, num_inliers, status):
        B, cap = kp0.shape[0], kp0.shape[1]
        check(lib().mv_pose_from_matches_dev(self.h, ctypes.byref(params), B, cap, _t(n0), _t(match_idx), _t(kp0),
                                             _t(kp1), _t(T), _t(num_matches), _t(num_inliers), _t(status)),
              "pose_from_matches")


# ---------------- quantized SuperPoint front-end (include/superpoint.h) ----------------
SP_LAYERS = ("conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b",
             "convPa", "convPb", "convDa", "convDb")


def superpoint_weights(src):
    """Weights dict (<layer>_w, <layer>_bias, <layer>_meta = [w_scale, w_zp, out_scale, out_zp],
    input_scale) from the reference's TorchScript archive (read without unpickling or running it:
    sp_weights.load_superpoint), from an .npz of that layout, or from such a dict."""
    if isinstance(src, dict):
        return src
    if str(src).endswith(".npz"):
        return dict(np.load(src, allow_pickle=False))
    import sp_weights

    L = sp_weights.load_superpoint(src)
    out = {"input_scale": np.float64(L["input"]["scale"])}
    for n in SP_LAYERS:
        d = L[n]
        if d["w_zp"] != 0 or d["out_zp"] != 0:
            raise MVError("%s: non-zero zero points are not supported" % n)
        out[n + "_w"], out[n + "_bias"] = d["w"], d["bias"]
        out[n + "_meta"] = np.array([d["w_scale"], d["w_zp"], d["out_scale"], d["out_zp"]], np.float64)
    return out


class SuperPoint:
    """The quantized SuperPoint network on the GPU (mv_superpoint_*): uint8 frames [B][H][W] ->
    Frame-layout int8 semi [B][cells][65], desc [B][cells][256] and their run() scales."""

    def __init__(self, ctx, weights):
        W = superpoint_weights(weights)
        sw = SpWeights()
        sw.in_scale = float(W["input_scale"])
        keep = []
        for i, n in enumerate(SP_LAYERS):
            w = np.ascontiguousarray(W[n + "_w"], np.int8)
            b = np.ascontiguousarray(W[n + "_bias"], np.float32)
            meta = W[n + "_meta"]
            keep += [w, b]
            L = sw.layer[i]
            L.w, L.bias = w.ctypes.data, b.ctypes.data
            L.cout, L.cin, L.k = w.shape[0], w.shape[1], w.shape[2]
            L.w_scale, L.out_scale = float(meta[0]), float(meta[2])
        h = _P()
        check(lib().mv_superpoint_create(ctx.h, ctypes.byref(sw), ctypes.byref(h)), "superpoint_create")
        self.h, self.ctx = h, ctx

    def close(self):
        if self.h:
            lib().mv_superpoint_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self, images, oh=192, ow=640, out=None, ctx=None):
        """images: torch uint8 [B][H][W] on the context's device; returns (semi, desc,
        semi_scale, desc_scale) torch tensors (or fills `out`, the same four).  ctx: run on another
        context's stream (default: the one the net was created with)"""
        import torch

        B, H, W = images.shape
        cells = (oh // 8) * (ow // 8)
        if out is None:
            dev = images.device
            out = (torch.empty((B, cells, 65), dtype=torch.int8, device=dev),
                   torch.empty((B, cells, 256), dtype=torch.int8, device=dev),
                   torch.empty(B, dtype=torch.float32, device=dev), torch.empty(B, dtype=torch.float32, device=dev))
        semi, desc, ss, ds = out
        check(lib().mv_superpoint_forward_dev((ctx or self.ctx).h, self.h, B, H, W, oh, ow, _t(images), _t(semi), _t(desc),
                                              _t(ss), _t(ds)), "superpoint_forward")
        return semi, desc, ss, ds

    def forward_raw(self, images, oh=192, ow=640, out=None, ctx=None):
        """images: torch uint8 [B][H][W] -> the network's float outputs as pairwise_pnp.py's
        run() receives them (semi [B, 65, oh/8, ow/8], coarse_desc [B, 256, oh/8, ow/8] float32
        NCHW: code x the head's output scale), the input of Context.keypoints"""
        import torch

        B, H, W = images.shape
        hc, wc = oh // 8, ow // 8
        if out is None:
            dev = images.device
            out = (torch.empty((B, 65, hc, wc), dtype=torch.float32, device=dev),
                   torch.empty((B, 256, hc, wc), dtype=torch.float32, device=dev))
        semi, cdesc = out
        check(lib().mv_superpoint_forward_raw_dev((ctx or self.ctx).h, self.h, B, H, W, oh, ow, _t(images),
                                                  _t(semi), _t(cdesc)), "superpoint_forward_raw")
        return semi, cdesc


class SuperPointFrontend:
    """Mirror of SuperPointFrontend (python/superpoint_inference.py:86-208) on the GPU: the
    network from the same archive (read without unpickling), run() on one frame.  run() takes the
    8-bit grayscale frame as decoded (the driver's / 255 and resize to 192 x 640,
    superpoint_inference.py:613-628, happen on the GPU) and returns run()'s
    (scale0, q_outs0 [1, 65, Hc, Wc], scale1, q_outs1 [1, 256, Hc, Wc], None): the int8 codes as
    torch int32 tensors like the reference's .int(); the float network outputs are not kept."""

    def __init__(self, weights_path, nms_dist=4, conf_thresh=0.015, nn_thresh=0.7, cuda=True, ctx=None, size=(192, 640)):
        self.name = "SuperPoint"
        self.nms_dist, self.conf_thresh, self.nn_thresh = nms_dist, conf_thresh, nn_thresh
        self.cell, self.border_remove = 8, 4
        self.ctx = ctx or Context(0)
        self.net = SuperPoint(self.ctx, weights_path)
        self.size = size

    def run(self, img):
        import torch

        img = torch.as_tensor(np.ascontiguousarray(img, np.uint8)).cuda()
        oh, ow = self.size
        stream = torch.cuda.current_stream()
        self.ctx.set_stream(stream)
        semi, desc, ss, ds = self.net.forward(img[None], oh, ow)
        torch.cuda.synchronize()
        hc, wc = oh // 8, ow // 8
        q0 = semi[0].view(wc, hc, 65).permute(2, 1, 0)[None].int()
        q1 = desc[0].view(wc, hc, 256).permute(2, 1, 0)[None].int()
        return float(ss[0].item()), q0, float(ds[0].item()), q1, None
