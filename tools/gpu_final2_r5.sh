# Round-5 final build (prefetch on the lean stream, merged Adam): GPU suite + smoke, bench (all legs), rocprof stats
set -o pipefail
TAG=r5final2; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['kernels_ms']); print('roofline frac', d['roofline']['frac']); print('room0', d.get('room0',{}).get('frames_per_s')); print('stress iter', d.get('stress_iteration',{}).get('value'), d.get('stress_iteration',{}).get('ms_per_iteration'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -14 $OUT/kernels.md
