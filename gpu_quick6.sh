set -o pipefail
mkdir -p gpurun_out/q6
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q6/tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/q6/tests.log
[ $rc -eq 0 ] || { grep -n "^E " gpurun_out/q6/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk > gpurun_out/q6/bench.json 2> gpurun_out/q6/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/q6/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q6/bench.json')); print(d['value'], d['ms_per_step'], d['room0'])"
