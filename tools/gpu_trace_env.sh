# Round 6: a kernel trace of the captured room0 iteration under the given environment settings.
# usage: bash tools/gpu_trace_env.sh TAG "VAR=a VAR2=b" ["VAR=c" ...]
set -o pipefail
OUT=gpurun_out/${1:?tag}; shift; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$i -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk $BENCH_ARGS > $OUT/t$i.json 2> $OUT/t$i.err || { tail -20 $OUT/t$i.err; exit 1; }
  grep '^{' $OUT/t$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$E', d['ms_per_step'])"
done
