#!/usr/bin/env python3
"""Write the stamp-probe variant of csrc/preint.hip (s_memtime at the step's
start, after the G stores, after the K reads landed and at the step's end,
kept in the pn row of the step instead of (dt, p)) to argv[1]; build it with
tools/variant.sh stamp <file> preint.hip and read it with tools/preint_stamps.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(ROOT, "ic-gvins_amd/csrc/preint.hip")).read()


def rep(a, b):
    global s
    assert s.count(a) == 1, a[:70]
    s = s.replace(a, b)


rep("""            if (pns && k - kc == c) {
                prow[0] = dt;
                prow[1] = p[0];
                prow[2] = p[1];
                prow[3] = p[2];
            }
""", """            double st0 = (double)__builtin_amdgcn_s_memtime();  // STAMP PROBE
""")
rep("""            const double qdg = a * wdc;""", """            double st1 = (double)__builtin_amdgcn_s_memtime();  // STAMP PROBE
            const double qdg = a * wdc;""")
rep("""            __builtin_amdgcn_sched_barrier(0);
            phi_mv(f, Jc, y);""", """            __builtin_amdgcn_sched_barrier(0);
            double st2 = (double)__builtin_amdgcn_s_memtime() + K[0] * 0.0;  // STAMP PROBE (after K landed)
            phi_mv(f, Jc, y);""")
rep("""            wave_lds_sync();  // the next step's stores after this step's reads
        }""", """            if (pns && k - kc == c) {  // STAMP PROBE
                prow[0] = st0;
                prow[1] = st1;
                prow[2] = st2;
                prow[3] = (double)__builtin_amdgcn_s_memtime() + Pc[14] * 0.0;
            }
            wave_lds_sync();  // the next step's stores after this step's reads
        }""")
open(sys.argv[1], "w").write(s)
