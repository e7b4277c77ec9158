# walk step codes (NSLAM_WALK_CODES) vs the scalar-unit walk: GPU parity tests, then A/B timing
set -o pipefail
mkdir -p gpurun_out/r3w
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w/tests.log 2>&1 || { tail -30 gpurun_out/r3w/tests.log; exit 1; }
tail -1 gpurun_out/r3w/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > gpurun_out/r3w/$n.json 2> gpurun_out/r3w/$n.err || { tail -5 gpurun_out/r3w/$n.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), {k: v for k, v in d['kernels_ms'].items() if 'bwd' in k})" gpurun_out/r3w/$n.json $n
}
for r in 1 2; do
run codes$r
run oldwalk$r NSLAM_LIB=$PWD/nice-slam_amd/libnslam_oldwalk.so
done
timeout -k 10 300 python bench.py --leg frames > gpurun_out/r3w/frames.json 2> gpurun_out/r3w/frames.err || { tail -5 gpurun_out/r3w/frames.err; exit 1; }
tail -1 gpurun_out/r3w/frames.json | cut -c1-300
