"""CPU model of the work partition in csrc/comm/oneshot.hip: for every (n, world, blocks) the one-shot
chunks and the two-shot (slice, sub-chunk) ranges tile [0, n) exactly once, stay 16-B aligned, and
each workgroup's ranges are the same on every rank (the flag protocol pairs workgroup b with b)."""
import itertools

import pytest


def oneshot_ranges(n, G):
    per = -(-n // G)
    per = (per + 3) & ~3
    return [(b * per, min(b * per + per, n)) for b in range(G)]


def twoshot_ranges(n, world, G):
    L = -(-n // world)
    L = (L + 3) & ~3
    per = -(-L // G)
    per = (per + 3) & ~3
    out = {}
    for b in range(G):
        for sl in range(world):
            lo = sl * L + b * per
            hi = min(lo + per, sl * L + L, n)
            lo = min(lo, hi)
            out[(b, sl)] = (lo, hi)
    return out


@pytest.mark.parametrize("n,world,G", list(itertools.product([1, 3, 4, 5, 257, 1000, 18866, 65543, 1394282],
                                                             [2, 3, 4, 8], [1, 7, 64, 128])))
def test_partition_tiles_exactly_once(n, world, G):
    cover = bytearray(n)
    for lo, hi in oneshot_ranges(n, G):
        assert lo % 4 == 0
        for i in range(max(lo, 0), max(lo, hi)):
            cover[i] += 1
    assert all(c == 1 for c in cover)
    cover = bytearray(n)
    for (b, sl), (lo, hi) in twoshot_ranges(n, world, G).items():
        assert lo % 4 == 0 or lo == hi
        for i in range(lo, hi):
            cover[i] += 1
    assert all(c == 1 for c in cover)


@pytest.mark.parametrize("n,world", list(itertools.product([64, 1000, 18880, 1394304], [2, 3, 4, 8])))
def test_dp_owner_slices_match_kernel_geometry(n, world):
    """DataParallel.owner_slices (checkpoint gather of owner-only optimizer moments) must be exactly
    the union of the kernel's per-workgroup ranges of each slice."""
    from hops_examples_amd.parallel.dp import DataParallel

    class _A:
        numel = n

    dp = DataParallel.__new__(DataParallel)
    dp.arena, dp.world, dp._fused_opt = _A(), world, object()
    sl = dp.owner_slices()
    rng = twoshot_ranges(n, world, 64)
    for r in range(world):
        idx = set()
        for b in range(64):
            lo, hi = rng[(b, r)]
            idx.update(range(lo, hi))
        assert idx == set(range(sl[r].start, sl[r].stop)), r
