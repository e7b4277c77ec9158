set -o pipefail
mkdir -p gpurun_out/prof_r1c
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests_r1d.log 2>&1 && echo TESTS_OK
tail -3 gpurun_out/gpu_tests_r1d.log
timeout -k 10 600 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r1c.json 2> gpurun_out/bench_r1c.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_r1c.err; exit 1; }
cat gpurun_out/bench_r1c.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1c -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1c/bench.json 2> gpurun_out/prof_r1c/bench.err || { echo PROF_FAIL; tail -20 gpurun_out/prof_r1c/bench.err; exit 1; }
find gpurun_out/prof_r1c -name "*stats*" | head
