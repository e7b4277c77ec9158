# apply_mask on bit fields (backward) + pc producer breakdown
set -o pipefail
D=gpurun_out/r5j; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
run() {  # name lib mode
  NSLAM_LIB=$PWD/nice-slam_amd/$2 NSLAM_FWD_MODE=$3 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/$1.json 2> $D/$1.err || { tail -20 $D/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],4), 'ms', d['kernels_ms'])" $D/$1.json "$1"
}
for r in 1 2; do
run units_$r libnslam.so units
run d1_$r libnslam_d1.so pc
run d3_$r libnslam_d3.so pc
run d4_$r libnslam_d4.so pc
run d2_$r libnslam_d2.so pc
done
for v in tl tl_d1; do
NSLAM_LIB=$PWD/nice-slam_amd/libnslam_$v.so NSLAM_FWD_MODE=pc timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/$v.log 2>&1 || { tail -30 $D/$v.log; exit 1; }
echo "== $v"; sed -n 2,8p $D/$v.log
done
NSLAM_FWD_MODE=units timeout -k 10 240 python -u tools/probes/wave_timeline.py > $D/units.log 2>&1 || { tail -30 $D/units.log; exit 1; }
echo "== units"; cat $D/units.log
