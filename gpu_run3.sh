set -o pipefail
mkdir -p gpurun_out/prof_r1d
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests_r1e.log 2>&1 && echo TESTS_OK
tail -3 gpurun_out/gpu_tests_r1e.log
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_r1d.json 2> gpurun_out/bench_r1d.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_r1d.err; exit 1; }
cat gpurun_out/bench_r1d.json; tail -3 gpurun_out/bench_r1d.err
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --eager --no-cpu-baseline > gpurun_out/bench_r1d_eager.json 2> gpurun_out/bench_r1d_eager.err || { echo EAGER_FAIL; tail -30 gpurun_out/bench_r1d_eager.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r1d_eager.json')); print('eager', d['value'], d['ms_per_step'])"
