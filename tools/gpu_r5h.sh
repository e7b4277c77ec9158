# relu / mask on float bits (no SGPR lane masks): parity subset, A/B units vs pc, pc timelines
set -o pipefail
D=gpurun_out/r5h; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_parity.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for r in 1 2; do for m in units pc; do
NSLAM_FWD_MODE=$m timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/ab_${m}_$r.json 2> $D/ab_$m.err || { tail -20 $D/ab_$m.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', 'fwd', d['kernels_ms'].get('query_fwd'))" $D/ab_${m}_$r.json "$m round $r"
done; done
for v in tl tl_d2; do
NSLAM_LIB=$PWD/nice-slam_amd/libnslam_$v.so NSLAM_FWD_MODE=pc timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/$v.log 2>&1 || { tail -30 $D/$v.log; exit 1; }
echo "== $v"; sed -n 2,8p $D/$v.log
done
NSLAM_FWD_MODE=units timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/units.log 2>&1 || { tail -30 $D/units.log; exit 1; }
echo "== units"; sed -n 2,9p $D/units.log
