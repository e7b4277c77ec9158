# Round measurement: PMC traffic passes -> default bench (room0 + frames/s + stress + bulk + baselines)
# -> rocprofv3 kernel stats of the hipGraph bench -> tracking-iteration kernel stats; summaries are
# copied to profiles/<ROUND>_*.  usage: bash tools/gpu_round.sh TAG ROUND   (e.g. r2final r02)
set -o pipefail
TAG=${1:?tag}
ROUND=${2:?round prefix, e.g. r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_traffic.sh $TAG || exit 1
cp $OUT/traffic.json profiles/${ROUND}_traffic.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; echo "STOP bench"; exit 1; }
cp $OUT/bench.json profiles/${ROUND}_bench.json
python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][-1])
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms'); print('roofline', d['roofline']['kernel'], round(d['roofline']['frac'],3), d['roofline']['traffic']); print('room0', d.get('room0',{}).get('frames_per_s')); print('stress', d.get('grid_query_stress',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; echo "STOP prof"; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && cp $OUT/kernels.md profiles/${ROUND}_room0_kernels.md && head -16 $OUT/kernels.md
