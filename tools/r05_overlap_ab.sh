# r05: the headline step with and without the next batch's pyramid pass beside
# the LK (bench.py --overlap), side legs off, interleaved twice
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/${1:?tag}; mkdir -p $O
for r in 1 2; do
for ov in "" "--overlap"; do
  n=plain; [ -n "$ov" ] && n=overlap
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-pre --no-factors --no-sequence $ov > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { tail -20 $O/bench_${n}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['device_ms_per_step'])"
done
done
