# HBM traffic per launch at the stress shape (configs[4]): separate rocprofv3 --pmc FETCH_SIZE and
# WRITE_SIZE passes over the standalone 512^3 grid query and over the stress mapping iteration
# (eager launches), summarised to $OUT/traffic_stress.json.  usage: bash tools/gpu_traffic_stress.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export NSLAM_BENCH_EAGER=1
for C in FETCH_SIZE WRITE_SIZE; do
  for L in stress stress_iter; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$C/$L -o run -- python bench.py --leg $L > $OUT/pmc_${C}_$L.log 2>&1 || { tail -5 $OUT/pmc_${C}_$L.log; echo "STOP $C $L"; exit 1; }
  done
done
python tools/traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python bench.py --leg stress|stress_iter (NSLAM_BENCH_EAGER=1)" > $OUT/traffic_stress.json && python -c "
import json; d=json.load(open('$OUT/traffic_stress.json'))['kernels']
for k,v in d.items(): print(k, v['dispatches'], v['hbm_bytes_per_launch'])"
