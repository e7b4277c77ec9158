set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline --eager > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
run p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
run p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run p3 FETCH_SIZE
run p4 WRITE_SIZE
run p5 TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum
ls gpurun_out/pmc
