# per-kernel device time of the preintegration family over preint_loop.py's warm
# launches (rocprofv3 kernel trace), for the in-tree library and variants
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out/${1:?tag}; mkdir -p $O; shift
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$R/ic-gvins_amd/gvx/variants/libgvx_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && GVX_LIB="$lib" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -- python3 $R/tools/preint_loop.py > $O/tr_$v.json 2> $O/tr_$v.err)
  python3 - "$O/tr_$v" "$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'preint' in n and 'factor' not in n:
        d[n.split('(')[0].split('::')[-1]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
out = []
for n, v in d.items():
    v = sorted(v)
    out.append('%s med %.1f us (n %d)' % (n, v[len(v) // 2], len(v)))
print(sys.argv[2], ' | '.join(out))
PY
done
# the chain / pre / cov launches at a tenth of the segments (latency- vs throughput-bound)
(cd /tmp && export TMPDIR=/tmp && PREINT_REPS=58 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_small -- python3 $R/tools/preint_loop.py > $O/tr_small.json 2> $O/tr_small.err)
