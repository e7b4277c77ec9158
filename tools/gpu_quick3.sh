# tests -> bench (no CPU baseline / stress).  usage: bash tools/gpu_quick3.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; echo "STOP tests"; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python -X faulthandler bench.py --no-cpu-baseline --no-stress > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; echo "STOP bench"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['kernels_ms']); print(d['room0']['ms_per_iteration'], d['room0']['frames_per_s'])
b=d['bulk_forward']; print({k: (round(v.get('ms', v.get('ms_per_image')),2)) for k,v in b.items()})"
