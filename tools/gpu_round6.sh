# Round 6 validation: the whole GPU suite + smoke, the default bench (all legs), a rocprofv3 kernel-stats
# profile of the headline bench, under gpurun_out/TAG (copy the records to keep into profiles/r06_*).
set -o pipefail
TAG=${1:-r6final}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head -20; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }

python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['kernels_ms']); print('roofline', d['roofline']['frac'], d['roofline']['kernel'])
for k in ('room0_slam_loop','optimize_map','scene0000_ba'): print(k, json.dumps(d.get(k))[:600])
print('stress', d.get('grid_query_stress',{}).get('frac'), d.get('stress_iteration',{}).get('ms_per_iteration'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -14 $OUT/kernels.md
