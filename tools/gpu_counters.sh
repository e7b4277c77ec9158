# Counter evidence of a round: per-kernel SQ counters (MFMA busy, VALU, waves,
# waits, LDS) and HBM bytes at room0 and at the stress shape (configs[4]), plus rocprofv3 kernel
# durations of the stress iteration.  Every rocprofv3 --pmc pass is its own run (one counter group
# each, within the per-block limits), eager launches (per-dispatch counters).
# usage: bash tools/gpu_counters.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG/counters
mkdir -p $OUT
export TMPDIR=/tmp
# eager launches, branches serialised, no ray prefetch: each kernel runs alone, so its counter window
# (GRBM_GUI_ACTIVE) holds no other kernel's work
ROOM0="python bench.py --steps 6 --warmup 3 --no-cpu-baseline --eager --serial-branches --no-prefetch --no-stress --no-frames --no-bulk"
STRESS="python bench.py --leg stress_iter"
GRIDQ="python bench.py --leg stress"   # the standalone grid query (k_grid_fwd) at the stress shape
pass() {  # name, command, counters...
  local name=$1 cmd=$2; shift 2
  mkdir -p $(dirname $OUT/$name)
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- $cmd > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY"
G2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LEVEL_WAVES"
pass room0_g1 "$ROOM0" $G1
pass room0_g2 "$ROOM0" $G2
pass room0_fetch "$ROOM0" FETCH_SIZE
pass room0_write "$ROOM0" WRITE_SIZE
pass room0_grbm "$ROOM0" GRBM_GUI_ACTIVE GRBM_COUNT
export NSLAM_BENCH_EAGER=1
pass stress_g1 "$STRESS" $G1
pass stress_fetch "$STRESS" FETCH_SIZE
pass stress_write "$STRESS" WRITE_SIZE
pass stress_grbm "$STRESS" GRBM_GUI_ACTIVE GRBM_COUNT
unset NSLAM_BENCH_EAGER
# k_grid_fwd's bytes join the stress traffic summary (its passes are subdirectories of the same dirs)
pass stress_fetch/gridq "$GRIDQ" FETCH_SIZE
pass stress_write/gridq "$GRIDQ" WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stress_prof -o run -- $STRESS > $OUT/stress_prof.log 2>&1 || { tail -20 $OUT/stress_prof.log; echo "STOP stress prof"; exit 1; }
python tools/pmc_summary.py $OUT/room0_g1 $OUT/room0_g2 $OUT/room0_grbm > $OUT/room0_sq.txt
python tools/pmc_summary.py $OUT/stress_g1 $OUT/stress_grbm > $OUT/stress_sq.txt
python tools/traffic.py $OUT/room0_fetch $OUT/room0_write "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- $ROOM0" > $OUT/traffic.json
python tools/traffic.py $OUT/stress_fetch $OUT/stress_write "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- $STRESS (NSLAM_BENCH_EAGER=1); -- $GRIDQ" > $OUT/traffic_stress.json
python tools/prof_summary.py $OUT/stress_prof > $OUT/stress_kernels.md
head -12 $OUT/stress_kernels.md; grep -A3 "== k_" $OUT/room0_sq.txt | head -60
