# Round measurement: default bench (room0 + frames/s + stress + baselines) -> PMC traffic passes ->
# rocprofv3 kernel stats of the hipGraph bench.  usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_traffic.sh $TAG || exit 1
cp $OUT/traffic.json profiles/r01_traffic.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; echo "STOP bench"; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; echo "STOP prof"; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -16 $OUT/kernels.md
