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

XR = 4  # X_UNIQUE=0; X_UNIQUE=1 gives every tile its own slot (xr = ntc)


class Slot:
    def __init__(self):
        self.tile = None
        self.writing = False
        self.version = 0


class Block:
    """slots[s][w]: the rows of exchange slot s that wave w stores (4 w .. 4 w + 3) -- and that the
    partner's wave w imports"""
    def __init__(self, w, W, xr):
        self.w = w
        self.flag = 0
        self.solo = False
        self.slots = [[Slot() for _ in range(W)] for _ in range(xr)]
        self.arrived = {}


def run(ntc, W, seed, spin, force=None, xr=XR, max_steps=400000):
    """force: (block, tile) -- that block's wave 0 goes SOLO from that tile's import on
    (X_FORCE_SOLO); xr: exchange slots per block (ntc: one per tile, never reused)"""
    rng = random.Random(seed)
    blocks = [Block(0, W, xr), Block(1, W, xr)]
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
        pending = []  # imports in flight: (slot, tile, version at the read's start)

        def land(keep):  # the imports older than the newest `keep` have landed (vmcnt)
            while len(pending) > keep:
                slot, tile, ver = pending.pop(0)
                s = p.slots[slot][w]
                assert s.tile == tile and not s.writing and s.version == ver, \
                    "slot %d overwritten during the import of tile %d" % (slot, tile)

        def start_read(tile):
            slot = tile % xr
            s = p.slots[slot][w]
            assert s.tile == tile and not s.writing, "import of tile %d found %s" % (tile, s.tile)
            stats["imports"] += 1
            pending.append((slot, tile, s.version))

        def forced(tile):
            return force is not None and force[0] == b.w and w == 0 and tile >= force[1]

        # prologue: own halves of tiles 0, 1 (publish 2), tile 2, import tiles 0, 1
        for k in range(2):
            yield from write(b, w, k % xr, k)
        yield from barrier(b, "p0")
        if w == 0:
            b.flag = max(b.flag, 2)
        yield from write(b, w, 2 % xr, 2)
        yield from barrier(b, "p1")  # tile 2 is published at the top of tile 0 (after the imports below land)
        ok = yield from wait_flag(p, 2)
        if ok and not forced(0):
            start_read(0)
            start_read(1)
        else:
            wsolo = True
            b.solo = True
        for tc in range(ntc):
            yield
            land(1)  # top: everything but the newest import
            yield from barrier(b, tc)
            bsolo = b.solo
            wsolo = wsolo or bsolo
            if w == 0 and not bsolo:
                b.flag = max(b.flag, min(tc + 3, ntc))
            yield
            if tc + 3 < ntc and not wsolo:  # seg 1: own half of tile tc + 3
                yield from write(b, w, (tc + 3) % xr, tc + 3)
            yield
            if tc + 2 < ntc:  # end of the tile: the partner half of tile tc + 2
                if not wsolo:
                    ok = yield from wait_flag(p, tc + 3)
                    if not ok or forced(tc + 2):
                        wsolo = True
                        b.solo = True
                if not wsolo:
                    start_read(tc + 2)
        yield
        land(0)
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
@pytest.mark.parametrize("unique", [False, True])
def test_exchange_protocol_random_interleavings(ntc, unique):
    """generous spin budget: no SOLO, every partner half imported, every import intact"""
    for seed in range(40):
        st = run(ntc, W=3, seed=seed, spin=10 ** 6, xr=ntc if unique else XR)
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
