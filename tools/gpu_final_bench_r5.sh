# Round-5 final bench (all legs; roofline from the r05 counter files) + rocprofv3 kernel stats + tracking stats
set -o pipefail
TAG=r5final; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['kernels_ms']); print('roofline', d['roofline']); print('room0', d.get('room0',{}).get('frames_per_s')); print('stress', d.get('grid_query_stress',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -16 $OUT/kernels.md
