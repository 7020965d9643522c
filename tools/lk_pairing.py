"""How much LK iteration work the two-points-per-wave layout wastes (diagnostic).

A wave of klt_kernel<2> iterates each level until BOTH of its points are done,
so a level costs max(n_a, n_b) iterations of the wave.  This runs the oracle's
diagnostic build (-DORC_ITER_STATS: per-point iteration log) on configs[1] pairs
and reports sum(max) against sum(mean) per level and direction.
    gcc -O2 -fPIC -std=c11 -D_GNU_SOURCE -ffp-contract=off -DORC_ITER_STATS -shared \\
        -o /tmp/liboracle_iter.so oracle/{klt,detect,preint,factors,clahe,camera,ins,aux_factors,marg,fmat,orc_pool}.c -lm -lpthread
    python3 tools/lk_pairing.py /tmp/liboracle_iter.so [pairs]"""
import ctypes as C
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "oracle"), os.path.join(R, "ic-gvins_amd")]
import oracle as orc  # noqa: E402
from gvx import synth  # noqa: E402

orc.LIB_PATH = sys.argv[1]
npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = orc.lib()
n_log = C.c_int.in_dll(L, "orc_iter_log_n")
log = (C.c_int * (3 << 20)).in_dll(L, "orc_iter_log")
I, J, P, Q = synth.make_batch(npairs, 1280, 560, 150, distinct=npairs)
tot = {}
for i in range(npairs):
    n_log.value = 0
    orc.klt_fb(I[i], J[i], P[i], Q[i], reuse_pyramids=True, nthreads=1)
    a = np.frombuffer(log, np.int32, 3 * n_log.value).reshape(-1, 3)
    # call order: forward levels 3..0 then backward levels 3..0 (one job per level)
    seg, d, prev = [], 0, None
    for lv, pt, j in a:
        if prev is not None and lv > prev:
            d += 1
        prev = lv
        seg.append((d, lv, pt, j))
    for d, lv in {(s[0], s[1]) for s in seg}:
        it = np.zeros(150, np.int64)
        for s in seg:
            if s[0] == d and s[1] == lv:
                it[s[2]] = s[3]
        pairs = it.reshape(-1, 2)
        t = tot.setdefault((d, lv), [0, 0.0, 0])
        t[0] += int(pairs.max(1).sum())
        t[1] += float(pairs.mean(1).sum())
        t[2] += int(it.sum())
print("dir level  sum(max)  sum(mean)  waste")
W = M = 0
for (d, lv), (mx, mean, s) in sorted(tot.items()):
    print(f"{'fb'[d]}   L{lv}   {mx:8d}  {mean:9.1f}  {mx / mean - 1:6.1%}")
    W += mx
    M += mean
print(f"all        {W:8d}  {M:9.1f}  {W / M - 1:6.1%}   (iterations per point {2 * M / (150 * npairs):.2f})")
