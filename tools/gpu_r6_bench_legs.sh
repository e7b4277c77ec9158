# Round 6: the drop-in legs of bench.py (optimize_map, scene0000 BA, measured SLAM loop) + the tracker graph test
set -o pipefail
OUT=gpurun_out/${1:-r6b}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mapper.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -8
for leg in optimize_map scene0000 slam_loop; do
  timeout -k 10 400 python -u bench.py --leg $leg > $OUT/$leg.json 2> $OUT/$leg.err || { tail -30 $OUT/$leg.err; exit 1; }
  echo "== $leg"; tail -c 3000 $OUT/$leg.json; echo
done
timeout -k 10 400 python -u tools/probes/touched_rows.py --split coherent --iters 6 --configs apartment,stress > $OUT/touched_coherent.json 2> $OUT/touched.err || { tail -30 $OUT/touched.err; exit 1; }
cat $OUT/touched_coherent.json
