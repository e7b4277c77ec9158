# fused GPU tests + graph bench + eager bench (no profiler)
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -q -x > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('graph', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['kernels_ms'])"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --eager > $OUT/bench_eager.json 2> $OUT/bench_eager.err || { tail -30 $OUT/bench_eager.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_eager.json')); print('eager', round(d['value']/1e6,2), round(d['ms_per_step'],4))"
