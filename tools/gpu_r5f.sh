# pc forward iteration: bit-exactness, A/B units vs pc, timeline with wait accounting
set -o pipefail
D=gpurun_out/r5f; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "forward_variants" > $D/tests_variants.log 2>&1 || { tail -40 $D/tests_variants.log; exit 1; }
tail -1 $D/tests_variants.log
for r in 1 2; do for m in units pc; do
NSLAM_FWD_MODE=$m timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/ab_${m}_$r.json 2> $D/ab_$m.err || { tail -20 $D/ab_$m.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', 'fwd', d['kernels_ms'].get('query_fwd'))" $D/ab_${m}_$r.json "$m round $r"
done; done
NSLAM_FWD_MODE=pc timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/tl_pc.log 2>&1 || { tail -30 $D/tl_pc.log; exit 1; }
head -12 $D/tl_pc.log
