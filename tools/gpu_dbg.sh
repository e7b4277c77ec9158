# late tape stores (NSLAM_LATE_TAPE): GPU parity tests, then A/B timing + kernel stats
set -o pipefail
mkdir -p gpurun_out/r3lt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3lt/tests.log 2>&1 || { tail -30 gpurun_out/r3lt/tests.log; exit 1; }
tail -1 gpurun_out/r3lt/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > gpurun_out/r3lt/$n.json 2> gpurun_out/r3lt/$n.err || { tail -5 gpurun_out/r3lt/$n.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), {k: v for k, v in d['kernels_ms'].items() if 'query' in k})" gpurun_out/r3lt/$n.json $n
}
for r in 1 2; do
run late$r
run early$r NSLAM_LIB=$PWD/nice-slam_amd/libnslam_earlytape.so
done
for L in libnslam libnslam_earlytape; do
NSLAM_LIB=$PWD/nice-slam_amd/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3lt/prof_$L -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > gpurun_out/r3lt/prof_$L.log 2>&1 || exit 1
python tools/prof_summary.py gpurun_out/r3lt/prof_$L > gpurun_out/r3lt/k_$L.md 2>&1 && echo "== $L" && sed -n 5,8p gpurun_out/r3lt/k_$L.md | cut -c1-160
done
