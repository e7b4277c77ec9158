# quick GPU check: gpu tests + hipGraph bench (no baselines/stress).  usage: bash tools/gpu_quick2.sh TAG [--skip-tests]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "--skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
  tail -3 $OUT/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" $OUT/gpu_tests.log | head -30; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('graph', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['kernels_ms'])"
