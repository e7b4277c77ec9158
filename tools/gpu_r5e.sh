# producer/consumer forward: variant bit-exactness, GPU tests in pc mode, bench A/B units vs pc, timeline
set -o pipefail
D=gpurun_out/r5e; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "forward_variants" > $D/tests_variants.log 2>&1 || { tail -40 $D/tests_variants.log; exit 1; }
tail -2 $D/tests_variants.log
NSLAM_FWD_MODE=pc timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused.py > $D/tests_pc_a.log 2>&1 || { tail -40 $D/tests_pc_a.log; exit 1; }
tail -2 $D/tests_pc_a.log
for r in 1 2; do for m in units pc; do
NSLAM_FWD_MODE=$m timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/ab_${m}_$r.json 2> $D/ab_$m.err || { tail -20 $D/ab_$m.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', 'fwd', d['kernels_ms'].get('query_fwd'))" $D/ab_${m}_$r.json "$m round $r"
done; done
NSLAM_FWD_MODE=pc timeout -k 10 240 python -u tools/probes/wave_timeline.py > $D/tl_pc.log 2>&1 || { tail -30 $D/tl_pc.log; exit 1; }
cat $D/tl_pc.log
NSLAM_FWD_MODE=pc timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/tests_pc_all.log 2>&1 || { tail -40 $D/tests_pc_all.log; exit 1; }
tail -2 $D/tests_pc_all.log
