# Kernel timeline of one hipGraph-replayed mapping iteration (7th gather from the end: the eager
# timer steps are the last 5).  usage: bash tools/gpu_trace.sh TAG
set -o pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python tools/timeline.py $OUT/trace/run_kernel_trace.csv 7 > $OUT/timeline.txt && cat $OUT/timeline.txt
