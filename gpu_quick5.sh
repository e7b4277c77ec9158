set -o pipefail
mkdir -p gpurun_out/q5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q5/tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/q5/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk > gpurun_out/q5/bench.json 2> gpurun_out/q5/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/q5/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q5/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q5/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > gpurun_out/q5/prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/q5/prof.log; exit 1; }
find gpurun_out/q5/prof -name "*kernel_stats.csv" -exec head -8 {} \;
