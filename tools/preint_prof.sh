#!/bin/bash
# Per-kernel device time of the preintegration launches (configs[3] bench leg) for
# libgvx variants, one rocprofv3 kernel-trace pass each:
#   bash tools/preint_prof.sh <tag> <variant>...   (base = the in-tree libgvx.so)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && GVX_LIB="$lib" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/$v -- python3 $R/bench.py --config 4 --no-cpu --steps 10 --warmup 3 > $O/$v.json 2> $O/$v.err)
  python3 - "$O/$v" "$O/$v.json" "$v" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    n = r['Name']
    if 'preint' in n and 'factor' not in n:
        out.append('%s %.1f' % (n.split('::')[-1].split('(')[0].split('<')[0][7:], float(r['AverageNs']) / 1000))
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], 'steps/s %.3g' % d['preint_steps_per_s'], d['preint_device_ms_per_launch'], ' | '.join(out))
PY
done
