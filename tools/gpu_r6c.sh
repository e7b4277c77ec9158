# Round 6: the engine tests (lean_main topology), the capture probe, then the topology A/B
set -o pipefail
OUT=gpurun_out/${1:-r6c}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 240 --timeout-method thread -k "branch_order or prefetch_matches" > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python -u tools/probes/capture_ops.py > $OUT/capture.log 2>&1 || { tail -30 $OUT/capture.log; exit 1; }
cat $OUT/capture.log
ROUNDS=3 bash tools/gpu_ab_env.sh ${1:-r6c}/ab NSLAM_BWD_TOPOLOGY=wgrad_main NSLAM_BWD_TOPOLOGY=lean_main
