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
        assert idx == set().union(*[set(range(s.start, s.stop)) for s in sl[r]]), r


def piece_ranges(cuts, world, G):
    """csrc/comm/oneshot.hip PieceSlices: workgroup b's range of slice s of piece k."""
    out = {}
    for k, (p0, p1) in enumerate(zip(cuts[:-1], cuts[1:])):
        L = ((p1 - p0 + world - 1) // world + 3) & ~3
        per = ((L + G - 1) // G + 3) & ~3
        for s in range(world):
            for b in range(G):
                lo = p0 + s * L + b * per
                hi = min(lo + per, p0 + s * L + L, p1)
                out[(k, s, b)] = (min(lo, hi), hi)
    return out


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("cuts", [[0, 1024, 4096, 4160, 100000], [0, 64, 128], [0, 25_600_000, 51_200_000, 76_800_000,
                                                                              102_400_064]])
def test_per_bucket_owner_pieces(world, cuts):
    """Per-bucket ownership (DataParallel rs-mode): the kernel's piece ranges tile the arena exactly once,
    every rank owns part of every bucket large enough to split, and ``owner_pieces`` is exactly rank r's
    ranges — the dp_rs_k bucket slice and the step tail's pieces agree."""
    from hops_examples_amd.parallel.oneshot import owner_pieces

    n = cuts[-1]
    G = 16
    rng = piece_ranges(cuts, world, G)
    own = owner_pieces(n, world, cuts)
    cover = {}
    for (k, s, b), (lo, hi) in rng.items():
        assert lo % 4 == 0 or lo == hi
        cover[(k, s)] = cover.get((k, s), 0) + (hi - lo)
    assert sum(cover.values()) == n
    for r in range(world):
        total = sum(x.stop - x.start for x in own[r])
        assert total == sum(v for (k, s), v in cover.items() if s == r)
        for k, (p0, p1) in enumerate(zip(cuts[:-1], cuts[1:])):
            if p1 - p0 >= 4 * world * 2:
                assert any(p0 <= x.start < p1 for x in own[r]), (r, k)  # a share of every bucket
        # dp_rs_k's slice of bucket k: [p0 + r L, p0 + (r + 1) L) clipped
        for k, (p0, p1) in enumerate(zip(cuts[:-1], cuts[1:])):
            L = ((p1 - p0 + world - 1) // world + 3) & ~3
            lo, hi = min(p1, p0 + r * L), min(p1, p0 + (r + 1) * L)
            if hi > lo:
                assert slice(lo, hi) in own[r]
