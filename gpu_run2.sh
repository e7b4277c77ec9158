set -o pipefail
mkdir -p gpurun_out/prof_r1b
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests_r1c.log 2>&1 && echo TESTS_OK
tail -3 gpurun_out/gpu_tests_r1c.log
timeout -k 10 600 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r1b.json 2> gpurun_out/bench_r1b.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_r1b.err; exit 1; }
cat gpurun_out/bench_r1b.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1b -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1b/bench.json 2> gpurun_out/prof_r1b/bench.err || { echo PROF_FAIL; tail -20 gpurun_out/prof_r1b/bench.err; exit 1; }
find gpurun_out/prof_r1b -name "*stats*" | head
