# Round 6: fused frustum rows kernel (ABI v20): tests + drop-in legs
set -o pipefail
OUT=gpurun_out/${1:-r6g}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_loop.py tests/test_gpu_mapper.py tests/test_gpu_dropins.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "not stress" > $OUT/tests.log 2>&1 || { grep -E "PASSED|FAILED" $OUT/tests.log | tail; tail -60 $OUT/tests.log; exit 1; }
grep -cE "PASSED" $OUT/tests.log; tail -1 $OUT/tests.log
for leg in optimize_map slam_loop; do
  timeout -k 10 400 python -u bench.py --leg $leg > $OUT/$leg.json 2> $OUT/$leg.err || { tail -30 $OUT/$leg.err; exit 1; }
  echo "== $leg"; tail -c 3000 $OUT/$leg.json; echo
done
