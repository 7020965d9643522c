"""Lane-level model of the three-points-per-wave group sums (klt.hip wave_scan /
gsum3), CPU only.

The 21-lane point groups (lanes 0-20, 21-41, 42-62) are summed by an inclusive
wave scan -- DPP row_shr 1, 2, 4, 8, then row_bcast:15 into rows 1 and 3 and
row_bcast:31 into rows 2 and 3 -- and the difference of the scan at the group's
last lane and the exclusive scan at its first.  Groups whose point has left
the iteration loop are disabled lanes while the others keep summing; a DPP read
of a disabled lane skips the write, so the add takes its `old` operand (0).
The model applies exactly those rules and checks that every active group gets
its exact total modulo 2^32, whatever the stale registers of the disabled
lanes hold.  The device path itself is checked bit-exact against the oracle by
tests/test_klt_gpu.py (test_batch_three_points_per_wave*)."""
import random

G3 = 21
M32 = 0xFFFFFFFF


def _wave_scan(v, active, stale):
    r = [v[L] if active[L] else stale[L] for L in range(64)]

    def step(src, rowmask):
        out = list(r)
        for L in range(64):
            if not active[L] or not (rowmask >> (L // 16)) & 1:
                continue
            s = src(L)
            add = r[s] if s is not None and active[s] else 0  # invalid / disabled source: old = 0
            out[L] = (r[L] + add) & M32
        return out

    for sh in (1, 2, 4, 8):
        r = step(lambda L, sh=sh: L - sh if L % 16 >= sh else None, 0xF)
    r = step(lambda L: (L // 16) * 16 - 1, 0xA)  # row_bcast:15
    r = step(lambda L: 31, 0xC)                  # row_bcast:31
    return r


def _group(lane):
    return min(lane // G3, 2)  # lane 63 shadows group 2


def test_group_totals_exact_under_any_activity():
    rng = random.Random(20261018)
    checks = 0
    for _ in range(3000):
        big = rng.random() < 0.3
        lim = (1 << 31) // G3 if big else 1 << 12
        v = [rng.randrange(-lim + 1, lim) & M32 for _ in range(64)]
        stale = [rng.getrandbits(32) for _ in range(64)]
        grp_on = [rng.random() < 0.6 for _ in range(3)]
        if not any(grp_on):
            continue
        active = [grp_on[_group(L)] for L in range(64)]
        s = _wave_scan(v, active, stale)
        for g in range(3):
            if not grp_on[g]:
                continue
            first, last = G3 * g, G3 * g + G3 - 1
            got = (s[last] - ((s[first] - v[first]) & M32)) & M32
            want = sum(v[first:last + 1]) & M32
            assert got == want, (g, grp_on)
            if big:  # the fast path's bound: the signed total fits int32
                tot = sum((x - (1 << 32)) if x >> 31 else x for x in v[first:last + 1])
                assert -(1 << 31) <= tot < (1 << 31)
            checks += 1
    assert checks > 3000
