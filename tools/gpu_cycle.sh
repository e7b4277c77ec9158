# One GPU measurement cycle: gpu tests -> hipGraph bench -> eager bench -> rocprofv3 kernel stats.
# usage (via gpurun): bash tools/gpu_cycle.sh TAG [--skip-tests]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
if [ "$2" != "--skip-tests" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q > $OUT/gpu_tests.log 2>&1; rc=$?
  tail -3 $OUT/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; stop tests $rc; }
fi
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; stop bench 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --eager --no-cpu-baseline > $OUT/bench_eager.json 2> $OUT/bench_eager.err || { tail -30 $OUT/bench_eager.err; stop eager 1; }
python -c "import json; d=json.load(open('$OUT/bench_eager.json')); print('eager', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; stop prof 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -30 $OUT/kernels.md
