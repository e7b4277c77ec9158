# tests -> default bench -> 2-rank gloo rehearsal of the sharded bench.  usage: bash tools/gpu_v10.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; echo "STOP tests"; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python -X faulthandler bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; echo "STOP bench"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { tail -30 $OUT/bench_gloo2.err; echo "STOP gloo2"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_gloo2.json')); print('gloo2', d['value'], d['ms_per_step'], d.get('exchange_bytes_per_step'))"
