# HBM traffic per kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over the bench's
# eager launches, summarised to $OUT/traffic.json.  usage: bash tools/gpu_traffic.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --steps 8 --warmup 3 --eager --no-cpu-baseline --no-stress --no-frames --no-bulk"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; echo "STOP fetch"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; echo "STOP write"; exit 1; }
python tools/traffic.py $OUT/fetch $OUT/write "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- $CMD" > $OUT/traffic.json && python -c "
import json; d=json.load(open('$OUT/traffic.json'))['kernels']
for k,v in d.items(): print(k, v['dispatches'], v['hbm_bytes_per_launch'])"
