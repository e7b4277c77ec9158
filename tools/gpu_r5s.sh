# the prefetch / Adam topology test, then the whole GPU suite on the final tree
set -o pipefail
D=gpurun_out/r5s; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "prefetch_matches_serial" > $D/t1.log 2>&1 || { tail -40 $D/t1.log; exit 1; }
tail -2 $D/t1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
