# Round 6: the d/dpts backward with dc in the scatter image (no stash) — d/dpts bit-identity against the
# round-start build, its parity tests, then the reference-API legs of the three builds.
set -o pipefail
OUT=gpurun_out/r6pg3; mkdir -p $OUT; export TMPDIR=/tmp
NSLAM_LIB=ab/libnslam_base.so timeout -k 10 120 python tools/probes/pg_equal.py $OUT/base.npz > /dev/null &&
timeout -k 10 120 python tools/probes/pg_equal.py $OUT/new.npz > /dev/null &&
python -c "
import numpy as np
a, b = np.load('$OUT/base.npz'), np.load('$OUT/new.npz')
print({k: bool(np.array_equal(a[k], b[k])) for k in a.files if k.startswith('gp')})" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_mapper.py tests/test_gpu_dropins.py "tests/test_gpu_configs.py::test_scene0000_bundle_adjustment_window5" tests/test_gpu_fused.py > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ROUNDS=2 bash tools/gpu_ab_legs.sh r6pg3/legs ab/libnslam_base.so ab/libnslam_stash.so nice-slam_amd/libnslam.so
