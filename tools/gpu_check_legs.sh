# The whole GPU suite, then chosen bench legs (each a child of bench.py --leg), printed one JSON line each.
# usage: bash tools/gpu_check_legs.sh TAG LEG [LEG ...]
set -o pipefail
OUT=gpurun_out/${1:?tag}; shift; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head -20; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for L in "$@"; do
  timeout -k 10 300 python bench.py --leg $L > $OUT/leg_$L.json 2> $OUT/leg_$L.err || { tail -20 $OUT/leg_$L.err; exit 1; }
  echo "$L: $(grep '^{' $OUT/leg_$L.json | tail -1 | cut -c1-900)"
done
