"""The pair-exchange protocol of k_q8d_match (maveric-slam_amd/csrc/hip/k_allpairs_direct.hip,
sweep_x) as a state machine, run under random interleavings on the CPU: two blocks of W waves,
per block XR = 3 exchange slots, one progress flag, a SOLO word.  Every wave reads exactly the
steps the kernel's waves take -- block barrier (after every wave's stores completed), thread 0's
publish, the per-wave flag poll with a spin budget, the partner-half import (a read that lasts
until the next barrier), the own-half store into slot (t + 2) % 3 -- and the checker asserts that
every import sees the tile it expects, unchanged for its whole duration (no slot is overwritten
while the partner may still read it), and that both blocks always finish (no deadlock) for any
relative speed, spin budget and forced SOLO point.  Pure host logic: no GPU."""
import random

import pytest

XR = 3


class Slot:
    def __init__(self):
        self.tile = None
        self.writing = False
        self.version = 0


class Block:
    """slots[s][w]: the rows of exchange slot s that wave w stores (4 w .. 4 w + 3) -- and that the
    partner's wave w imports"""
    def __init__(self, w, W):
        self.w = w
        self.flag = 0
        self.solo = False
        self.slots = [[Slot() for _ in range(W)] for _ in range(XR)]
        self.arrived = {}


def run(ntc, W, seed, spin, force=None, max_steps=200000):
    """force: (block, tile) -- that block's wave 0 goes SOLO at that tile (X_FORCE_SOLO)"""
    rng = random.Random(seed)
    blocks = [Block(0, W), Block(1, W)]
    stats = {"imports": 0, "solo_waves": 0}

    def barrier(b, key):
        b.arrived[key] = b.arrived.get(key, 0) + 1
        while b.arrived[key] < W:
            yield

    def write(b, w, slot, tile):
        s = b.slots[slot][w]
        assert not s.writing
        s.writing = True
        s.version += 1
        yield
        s.tile = tile
        s.writing = False

    def wait_flag(p, need):
        for _ in range(spin):
            if p.flag >= need:
                return True
            yield
        return False

    def wave(b, w):
        p = blocks[1 - b.w]
        wsolo = False
        pending = None  # (slot, tile, version at the read's start)

        def end_read():
            if pending is not None:
                s = p.slots[pending[0]][w]
                assert s.tile == pending[1] and not s.writing and s.version == pending[2], \
                    "slot %d overwritten during the import of tile %d" % (pending[0], pending[1])

        def start_read(slot, tile):
            s = p.slots[slot][w]
            assert s.tile == tile and not s.writing, "import of tile %d found %s" % (tile, s.tile)
            stats["imports"] += 1
            return (slot, tile, s.version)

        for k in range(2):
            yield from write(b, w, k, k)
        yield from barrier(b, "pro")
        if w == 0:
            b.flag = max(b.flag, 2)
        ok = yield from wait_flag(p, 1)
        if force == (b.w, 0) and w == 0:
            ok = False
        if ok:
            pending = start_read(0, 0)
        else:
            wsolo = True
            b.solo = True
        for tc in range(ntc):
            yield
            end_read()
            pending = None
            yield from barrier(b, tc)
            bsolo = b.solo
            wsolo = wsolo or bsolo
            if w == 0 and not bsolo:
                b.flag = max(b.flag, min(tc + 2, ntc))
            yield
            if tc + 1 < ntc:
                if not wsolo:
                    ok = yield from wait_flag(p, tc + 2)
                    if force is not None and force[0] == b.w and w == 0 and tc + 1 >= force[1]:
                        ok = False
                    if not ok:
                        wsolo = True
                        b.solo = True
                if not wsolo:
                    pending = start_read((tc + 1) % XR, tc + 1)
            yield
            if tc + 2 < ntc and not wsolo:
                yield from write(b, w, (tc + 2) % XR, tc + 2)
        yield
        end_read()
        stats["solo_waves"] += wsolo

    live = [wave(b, w) for b in blocks for w in range(W)]
    steps = 0
    while live:
        steps += 1
        assert steps < max_steps, "no progress: deadlock"
        g = rng.choice(live)
        try:
            next(g)
        except StopIteration:
            live.remove(g)
    return stats


@pytest.mark.parametrize("ntc", [3, 4, 7, 16])
def test_exchange_protocol_random_interleavings(ntc):
    """generous spin budget: no SOLO, every partner half imported, every import intact"""
    for seed in range(40):
        st = run(ntc, W=3, seed=seed, spin=10 ** 6)
        assert st["solo_waves"] == 0
        assert st["imports"] == 2 * 3 * ntc  # both blocks, every wave, tiles 0 .. ntc - 1


@pytest.mark.parametrize("ntc", [3, 5, 16])
def test_exchange_protocol_short_spins_and_forced_solo(ntc):
    """spin budgets down to one poll (spurious SOLO at any point, either block) and forced SOLO
    at every tile: still no import ever sees a stale or half-written slot, and both finish"""
    solos = 0
    for seed in range(60):
        for spin in (1, 2, 5, 50):
            st = run(ntc, W=3, seed=seed * 7 + spin, spin=spin)
            solos += st["solo_waves"]
        for blk in (0, 1):
            for t in range(ntc):
                run(ntc, W=2, seed=seed, spin=300, force=(blk, t))
    assert solos > 0
