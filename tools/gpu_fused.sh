set -o pipefail
mkdir -p gpurun_out/r1g
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py -q -x > gpurun_out/r1g/fused_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r1g/fused_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r1g/bench.json 2> gpurun_out/r1g/bench.err || { tail -30 gpurun_out/r1g/bench.err; exit 1; }
cat gpurun_out/r1g/bench.json
