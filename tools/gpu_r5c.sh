# forward variants A/B (NSLAM_FWD_MODE parts | units) + forward parity tests on the default
set -o pipefail
D=gpurun_out/r5c; mkdir -p $D; export TMPDIR=/tmp
for r in 1 2 3; do for m in parts units; do
NSLAM_FWD_MODE=$m timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/ab_${m}_$r.json 2> $D/ab_$m.err || { tail -20 $D/ab_$m.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', 'fwd', d['kernels_ms'].get('query_fwd'))" $D/ab_${m}_$r.json "$m round $r"
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_scenes.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
