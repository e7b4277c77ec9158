# round 5 (re-entry) baseline: full GPU suite, default bench, units-mode wave timeline, rocprof stats
set -o pipefail
D=gpurun_out/r5d; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d.get('kernels_ms'))" $D/bench.json
timeout -k 10 240 python -u tools/probes/wave_timeline.py > $D/tl_default.log 2>&1 || { tail -30 $D/tl_default.log; exit 1; }
cat $D/tl_default.log
timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/tl_serial.log 2>&1 || { tail -30 $D/tl_serial.log; exit 1; }
cat $D/tl_serial.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
python tools/prof_summary.py $D/prof > $D/prof_summary.md 2>&1; head -30 $D/prof_summary.md
