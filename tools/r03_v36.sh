#!/bin/bash
# factor kernels timed by dispatch-attached events (hipExtLaunchKernel): factor tests,
# pf_scale, configs[3] line, and a rocprofv3 kernel trace of the same line to compare
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v36
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_factor_parity_gpu.py tests/test_ba_gpu.py tests/test_factorset_gpu.py tests/test_aux_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u tools/pf_scale.py > $O/pf_scale.txt 2> $O/pf_scale.err || { tail -20 $O/pf_scale.err; exit 1; }
tail -3 $O/pf_scale.txt
timeout -k 10 300 python -u bench.py --config 4 --no-cpu > $O/c4.json 2> $O/c4.err
python3 -c "import json;d=json.load(open('$O/c4.json'));print('c4', d['value'], d['roofline']['frac'], d['roofline']['device_ms_per_step'], d['preint_factor_roofline']['frac'], d['window_factors']['gnss_roofline'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --config 4 --no-cpu > $O/prof.log 2>&1
cd $R
python3 - $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/prof/*/*kernel_trace.csv")[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    for k in ("preint_factor_kernel", "reproj_kernel", "small_kernel"):
        if k in n:
            d[(k, r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    print(k, len(v), "avg_us", round(sum(v) / len(v), 2), "min_us", round(min(v), 2))
PY
