# Round 6: mapper tests (prefetch inside the stage graphs), the drop-in legs with BA baselines, and a
# kernel-stats profile of the optimize_map leg
set -o pipefail
OUT=gpurun_out/${1:-r6e}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mapper.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "PASSED|FAILED" $OUT/tests.log; tail -60 $OUT/tests.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/tests.log | cut -c1-120
for leg in optimize_map scene0000 slam_loop; do
  timeout -k 10 400 python -u bench.py --leg $leg > $OUT/$leg.json 2> $OUT/$leg.err || { tail -30 $OUT/$leg.err; exit 1; }
  echo "== $leg"; tail -c 3000 $OUT/$leg.json; echo
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --leg slam_loop > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1; head -30 $OUT/kernels.md
