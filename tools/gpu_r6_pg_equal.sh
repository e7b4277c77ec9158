# Round 6: the d/dpts backward of the previous build and this one on the same inputs, compared.
set -o pipefail
OUT=gpurun_out/r6pgeq; mkdir -p $OUT
NSLAM_LIB=ab/libnslam_base.so timeout -k 10 120 python tools/probes/pg_equal.py $OUT/base.npz &&
timeout -k 10 120 python tools/probes/pg_equal.py $OUT/new.npz &&
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/r6pgeq/base.npz"), np.load("gpurun_out/r6pgeq/new.npz")
for k in a.files:
    x, y = a[k], b[k]
    d = np.abs(x - y).max()
    print(k, x.shape, "bit-identical" if np.array_equal(x, y) else f"max diff {d:.3e} rel {np.linalg.norm(x - y) / max(np.linalg.norm(x), 1e-30):.3e}")
PY
