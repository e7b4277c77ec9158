# Round-5 final measurements: GPU suite + smoke, PMC counters and HBM traffic (room0 + stress) -> profiles/r05_*,
# the default bench (all legs; its roofline reads the r05 counter files), rocprofv3 kernel stats.
set -o pipefail
TAG=r5final; OUT=gpurun_out/$TAG; mkdir -p $OUT profiles; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log; cp $OUT/tests.log profiles/r05_gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_counters.sh $TAG || exit 1
C=$OUT/counters
cp $C/room0_sq.txt profiles/r05_room0_pmc.txt && cp $C/stress_sq.txt profiles/r05_stress_pmc.txt && cp $C/traffic.json profiles/r05_traffic.json && cp $C/traffic_stress.json profiles/r05_traffic_stress.json && cp $C/stress_kernels.md profiles/r05_stress_kernels.md || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cp $OUT/bench.json profiles/r05_bench.json
python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['kernels_ms']); print('roofline', d['roofline']); print('room0', d.get('room0',{}).get('frames_per_s')); print('stress', d.get('grid_query_stress',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && cp $OUT/kernels.md profiles/r05_room0_kernels.md && head -16 $OUT/kernels.md
