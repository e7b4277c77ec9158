# GPU cycle: gpu tests -> bench (room0 + stress + baselines) -> 2-rank gloo rehearsal of the
# sharded path on one GPU -> rocprofv3 kernel stats.  usage: bash tools/gpu_cycle2.sh TAG [--skip-tests]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
if [ "$2" != "--skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
  tail -3 $OUT/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; stop tests $rc; }
fi
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; stop bench 1; }
cat $OUT/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { tail -30 $OUT/bench_gloo2.err; stop gloo2 1; }
cat $OUT/bench_gloo2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; stop prof 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -24 $OUT/kernels.md
