#!/usr/bin/env python3
"""Write the record-phase stamp variant of csrc/preint.hip to argv[1]: per
chunk, s_memtime at the chunk's top, after the staged records' wait, after the
record build (LDS drained) and after the next chunk's DMA issue, kept in the pn
row of the chunk's first step (tools/preint_rstamps.py reads them)."""
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
""", "")
rep("""        __builtin_amdgcn_s_waitcnt(VMCNT0);
        wave_lds_sync();""", """        const double r0 = (double)__builtin_amdgcn_s_memtime();  // STAMP PROBE
        __builtin_amdgcn_s_waitcnt(VMCNT0);
        wave_lds_sync();
        const double r1 = (double)__builtin_amdgcn_s_memtime();  // STAMP PROBE""")
rep("""        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage_and_store(kc);
        prk = kc + c;""", """        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const double r2 = (double)__builtin_amdgcn_s_memtime();  // STAMP PROBE
        stage_and_store(kc);
        prk = kc + c;
        prow[0] = r0;
        prow[1] = r1;
        prow[2] = r2;
        prow[3] = (double)__builtin_amdgcn_s_memtime();  // STAMP PROBE""")
open(sys.argv[1], "w").write(s)
