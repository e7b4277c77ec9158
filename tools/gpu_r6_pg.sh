# Round 6: the d/dpts mask-only backward at 3 waves per SIMD — its parity tests (tracker, bundle
# adjustment, camera gradients, mapper loop), then the reference-API legs against the previous build.
set -o pipefail
OUT=gpurun_out/r6pg2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_mapper.py tests/test_gpu_dropins.py "tests/test_gpu_configs.py::test_scene0000_bundle_adjustment_window5" tests/test_gpu_fused.py > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ROUNDS=2 bash tools/gpu_ab_legs.sh r6pg2/legs ab/libnslam_base.so nice-slam_amd/libnslam.so
