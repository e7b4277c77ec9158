set -o pipefail
OUT=gpurun_out/r2ic
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/ic -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline --eager --no-stress --no-frames --no-bulk > $OUT/ic.log 2>&1 || { tail -8 $OUT/ic.log; exit 1; }
python tools/pmc_summary.py $OUT/ic > $OUT/summary.txt; cat $OUT/summary.txt
