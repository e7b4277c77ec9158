set -o pipefail
mkdir -p gpurun_out/prof_r1f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_r1f.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests_r1f.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r1f.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke_r1f.log; exit 1; }
tail -1 gpurun_out/smoke_r1f.log
timeout -k 10 600 python -X faulthandler bench.py --steps 50 --warmup 10 > gpurun_out/bench_r1f.json 2> gpurun_out/bench_r1f.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_r1f.err; exit 1; }
cat gpurun_out/bench_r1f.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1f -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > gpurun_out/prof_r1f.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_r1f.log; exit 1; }
head -12 gpurun_out/prof_r1f/run_kernel_stats.csv | cut -c1-160
exit $rc
