#!/usr/bin/env python3
"""How far can LK's accumulation order move the result?  (VERDICT r01 item 2,
DESIGN.md section 2.)  The restatement and the GPU sum the 21x21 window products
exactly (int64); OpenCV 4.x sums them in fp32, in its scalar-loop order or in
its 4-lane CV_SIMD128 order.  This runs the oracle's klt_fb (fwd + bwd LK + FB +
border) in all three orders on the configs[1] and configs[2] synthetic inputs
and reports status / keep flips, the max |dnext| over points whose status
and keep agree and how many of them move by more than the north_star's 1e-4 px
-- each fp32 order against the exact one, and the two fp32 orders (two OpenCV
builds) against each other.  CPU only.

    python tools/accum_flips.py [--pairs1 64] [--pairs2 8] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))
import oracle as orc  # noqa: E402
from gvx import synth  # noqa: E402


TOL_PX = 1e-4


def compare(w, h, n, level, pairs, seed0, threads):
    p = orc.KltParams.default(max_level=level)
    res = {}
    tot = 0
    runs = {m: [] for m in (orc.ACC_EXACT, orc.ACC_F32, orc.ACC_F32X4)}
    for i in range(pairs):
        I, J, P, Q, _ = synth.make_pair(w, h, n, seed0 + i)
        tot += len(P)
        for m in runs:
            with orc.lk_accum(m):
                runs[m].append(orc.klt_fb(I, J, P, Q, params=p, nthreads=threads))
    pairs_cmp = ((orc.ACC_EXACT, orc.ACC_F32, "f32_scalar"), (orc.ACC_EXACT, orc.ACC_F32X4, "f32_simd4"),
                 (orc.ACC_F32, orc.ACC_F32X4, "f32_scalar_vs_f32_simd4"))
    for m0, m, name in pairs_cmp:
        st_flips = keep_flips = 0
        dmax_f = dmax_b = 0.0
        n_diff = n_over_f = n_over_b = 0
        for e, f in zip(runs[m0], runs[m]):
            st_flips += int(np.sum(e["st_f"] != f["st_f"])) + int(np.sum(e["st_b"] != f["st_b"]))
            keep_flips += int(np.sum(e["keep"] != f["keep"]))
            same = (e["st_f"] == f["st_f"]) & (e["st_b"] == f["st_b"]) & (e["keep"] == f["keep"]) & (e["st_f"] > 0)
            df = np.abs(e["next"][same] - f["next"][same]).max(initial=0.0)
            sb = same & (e["st_b"] > 0)
            db = np.abs(e["back"][sb] - f["back"][sb]).max(initial=0.0)
            n_diff += int(np.sum(np.any(e["next"][same] != f["next"][same], axis=1)))
            # points past the north_star's 1e-4 px (per coordinate)
            n_over_f += int(np.sum(np.abs(e["next"][same] - f["next"][same]).max(axis=1, initial=0.0) > TOL_PX))
            n_over_b += int(np.sum(np.abs(e["back"][sb] - f["back"][sb]).max(axis=1, initial=0.0) > TOL_PX))
            dmax_f, dmax_b = max(dmax_f, float(df)), max(dmax_b, float(db))
        res[name] = {"status_flips": st_flips, "keep_flips": keep_flips, "points": tot,
                     "max_abs_dnext_px": dmax_f, "max_abs_dback_px": dmax_b,
                     "points_with_any_dnext": n_diff, "points_dnext_over_1e-4px": n_over_f,
                     "points_dback_over_1e-4px": n_over_b}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs1", type=int, default=64)
    ap.add_argument("--pairs2", type=int, default=8)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--json")
    a = ap.parse_args()
    out = {"configs[1] 1280x560 N150 L3": compare(1280, 560, 150, 3, a.pairs1, synth.SEED, a.threads),
           "configs[2] 1920x1200 N500 L4": compare(1920, 1200, 500, 4, a.pairs2, synth.SEED, a.threads)}
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
