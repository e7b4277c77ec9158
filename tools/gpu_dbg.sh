# late prefetch (gather + sampler beside the colour weight gradients): tests + A/B timing + timeline
set -o pipefail
mkdir -p gpurun_out/r3l
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3l/tests.log 2>&1 || { tail -30 gpurun_out/r3l/tests.log; exit 1; }
tail -1 gpurun_out/r3l/tests.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > gpurun_out/r3l/$n.json 2> gpurun_out/r3l/$n.err || { tail -5 gpurun_out/r3l/$n.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4))" gpurun_out/r3l/$n.json $n
}
for r in 1 2; do
run late$r NSLAM_PREFETCH_LATE=1
run early$r NSLAM_PREFETCH_LATE=0
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3l/trace -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk > gpurun_out/r3l/trace.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/r3l/trace/run_kernel_trace.csv 7 > gpurun_out/r3l/timeline.txt && cat gpurun_out/r3l/timeline.txt
