"""CPU: the local feature pool (include/feature_pool.h, csrc/host/feature_pool.c) against the
reference's OWN include/local_feature_pool.h, compiled from its source with the workload
generator of src/local_feature_matching.c (oracle/ref_pool_harness.c -> oracle/_ref), slot
by slot after every frame; where that build is absent, against the golden vectors it made
(tests/golden/feature_pool_ref.npz, tools/make_pool_golden.py)."""
import ctypes
import os
import sys
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import mvtrack  # noqa: E402
import oracle  # noqa: E402

needs_ref = pytest.mark.skipif(not oracle.ref_pool_available(), reason="oracle/_ref not built (no /root/reference)")


def test_pool_struct_is_the_reference_layout():
    assert ctypes.sizeof(mvtrack._LfpEntry) == 64 and ctypes.sizeof(mvtrack.LocalFeature) == 56
    assert ctypes.sizeof(mvtrack._LfpPool) == 3000 * 64 + 8
    if oracle.ref_pool_available():
        assert oracle.ref_pool().ref_pool_sizeof() == ctypes.sizeof(mvtrack._LfpPool)


def test_pool_golden_reference_workload():
    """src/local_feature_matching.c's 100 frames x 200 ids (srand(0)): sizes and every table."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "feature_pool_ref.npz"))
    P = mvtrack.LocalFeaturePool()
    for f in range(g["ids"].shape[0]):
        assert P.track_frame(f, g["ids"][f].astype(np.int32)) == mvtrack.MV_OK
        assert P.size == g["sizes"][f]
        assert zlib.crc32(np.ascontiguousarray(P.table()).tobytes()) == g["table_crc32"][f], f
        assert P.check_invariant(f) == mvtrack.MV_OK
    assert (P.table() == g["final_table"]).all()


@needs_ref
def test_pool_reference_workload_slot_by_slot():
    ids, tab, sz = oracle.ref_pool_run(100, 200)
    P = mvtrack.LocalFeaturePool()
    for f in range(100):
        assert P.track_frame(f, ids[f]) == mvtrack.MV_OK
        assert (P.table() == tab[f]).all(), f
        assert P.size == sz[f]


def _collision_frames(seed, n_frames=40):
    """distinct ids per frame, most homed on 24 slots around the wrap (2988..2999, 0..11) so
    clusters run past slot 2999 and deletions shift entries across it; frame sizes vary,
    including empty frames (everything ages out) and bursts; at most 2400 live keys."""
    rng = np.random.default_rng(seed)
    homes = np.r_[np.arange(2988, 3000), np.arange(0, 12)]
    frames = []
    for f in range(n_frames):
        n = [0, 300, 5, 150, 299][f % 5] if f % 7 else 0
        crowded = homes[rng.integers(0, homes.size, 4 * n)] + 3000 * rng.integers(0, 40, 4 * n)
        spread = rng.integers(0, 120000, 4 * n)
        pool = np.where(rng.random(4 * n) < 0.7, crowded, spread)
        frames.append(np.unique(pool)[:n][rng.permutation(min(n, np.unique(pool).size))].astype(np.int32))
    return frames


def _spread_frames(seed, n_frames=40):
    """distinct ids per frame over a wide range (homes spread over the table), frame sizes
    0..300: clusters, chain refills and mass ageing without wrap-around clusters."""
    rng = np.random.default_rng(seed)
    return [rng.choice(200000, [0, 300, 5, 150, 299][f % 5] if f % 7 else 0, replace=False).astype(np.int32)
            for f in range(n_frames)]


def _vs_reference(frames):
    """the same layouts as the reference frame by frame, and -- where its refill rule leaves a
    key unreachable and it exits ("Key not found") -- an error from the same frame here
    (feature_pool.h).  Returns (frames the reference completed, its largest size)."""
    tab, sz, done = oracle.ref_pool_replay(frames)
    P = mvtrack.LocalFeaturePool()
    for f in range(done):
        assert P.track_frame(f, frames[f]) == mvtrack.MV_OK
        assert (P.table() == tab[f]).all(), f
        assert P.size == sz[f] and P.check_invariant(f) == mvtrack.MV_OK
    if done < len(frames):
        assert P.track_frame(done, frames[done]) == mvtrack.MV_ERR_INVALID_ARG
    return done, int(sz[:done].max()) if done else 0


@needs_ref
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_pool_spread_ids_vs_reference(seed):
    done, top = _vs_reference(_spread_frames(seed))
    assert top > 1000  # a high load was reached


@needs_ref
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_pool_wrap_clusters_vs_reference(seed):
    """ids crowded on the homes around the table end"""
    _vs_reference(_collision_frames(seed))


@needs_ref
def test_pool_reference_gives_up_and_so_do_we():
    """at least one stress case reaches the reference's unreachable-key exit (the error path
    is exercised, not only the agreeing prefix)"""
    assert any(_vs_reference(_collision_frames(s))[0] < 40 for s in (1, 2, 3, 4))


def test_pool_api_and_error_codes():
    P = mvtrack.LocalFeaturePool()
    st, ins, feat = P.insert(5, 0)
    assert st == mvtrack.MV_OK and ins and feat.word_id == 5 and feat.num_frames == 1
    st, ins, feat = P.insert(3005, 0)  # same home slot: probes to slot 6
    assert st == mvtrack.MV_OK and ins and P.table()[6, 0] == 3005
    st, ins, feat = P.insert(5, 1)
    assert st == mvtrack.MV_OK and not ins and feat.word_id == 5
    assert P.delete(5) == mvtrack.MV_OK and P.table()[5, 0] == 3005  # shifted back to its home
    assert P.delete(5) == mvtrack.MV_ERR_INVALID_ARG  # absent (the reference exits)
    assert P.insert(-1, 0)[0] == mvtrack.MV_ERR_INVALID_ARG
    assert list(P.valid_keys()) == [3005] and abs(P.load_factor() - 1 / 3000) < 1e-9
    # the frame ring: 8 frames kept, the 9th overwrites the oldest
    f = mvtrack.LocalFeature()
    L = mvtrack.lib()
    L.mv_local_feature_init_with_id(ctypes.byref(f), 7, 0)
    for fr in range(1, 10):
        L.mv_local_feature_update(ctypes.byref(f), fr)
    assert f.num_frames == 8 and f.frame_ptr == 2 and f.frames[f.frame_ptr] == 2
    assert not L.mv_local_feature_remove_old_frame(ctypes.byref(f), 3) and f.num_frames == 7
    # aging out: a feature seen once at frame 0 is gone after frame 8
    Q = mvtrack.LocalFeaturePool()
    Q.track_frame(0, [1, 2, 3])
    for fr in range(1, 8):
        Q.track_frame(fr, [])
        assert Q.size == 3
    Q.track_frame(8, [])
    assert Q.size == 0 and Q.check_invariant(8) == mvtrack.MV_OK
    # a full pool refuses inserts
    R = mvtrack.LocalFeaturePool()
    assert R.track_frame(0, np.arange(3000)) == mvtrack.MV_OK and R.size == 3000
    assert R.insert(5000, 0)[0] == mvtrack.MV_ERR_CAPACITY
