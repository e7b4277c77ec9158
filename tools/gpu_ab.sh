# A/B of two libnslam builds (same ABI) on one box: knob-probe timing, then a one-iteration kernel
# timeline of each.  usage: bash tools/gpu_ab.sh TAG LIB_A LIB_B   (paths relative to the repo)
set -o pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
export TMPDIR=/tmp
for L in ${2:?lib a} ${3:?lib b}; do
  n=$(basename $L .so)
  NSLAM_LIB=$PWD/$L timeout -k 10 200 python -u tools/probes/knobs.py default > $OUT/knobs_$n.log 2>&1 || { tail -20 $OUT/knobs_$n.log; exit 1; }
  echo "$n: $(tail -1 $OUT/knobs_$n.log)"
done
for L in $2 $3; do
  n=$(basename $L .so)
  export NSLAM_LIB=$PWD/$L
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/trace_$n.log 2>&1 || { tail -20 $OUT/trace_$n.log; exit 1; }
  python tools/timeline.py $OUT/trace_$n/run_kernel_trace.csv 7 > $OUT/timeline_$n.txt && echo "== $n" && cat $OUT/timeline_$n.txt
done
