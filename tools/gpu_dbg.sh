# fused colour Adam (ABI v14) vs separate Adam, pipelined vs not: quick bench per variant + timelines
set -o pipefail
mkdir -p gpurun_out/r3h
run() {  # name, env..., (BARGS: bench args)
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames $BARGS > gpurun_out/r3h/$n.json 2> gpurun_out/r3h/$n.err || { tail -5 gpurun_out/r3h/$n.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4))" gpurun_out/r3h/$n.json $n
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h/fused_tests.log 2>&1 || { tail -30 gpurun_out/r3h/fused_tests.log; exit 1; }
tail -1 gpurun_out/r3h/fused_tests.log
BARGS= run fused NSLAM_FUSE_ADAM=1
BARGS= run unfused NSLAM_FUSE_ADAM=0
BARGS=--pipeline run pipe NSLAM_FUSE_ADAM=1
BARGS= run fused2 NSLAM_FUSE_ADAM=1
BARGS= run unfused2 NSLAM_FUSE_ADAM=0
for V in fused pipe; do
  if [ $V = pipe ]; then A=--pipeline; else A=; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3h/trace_$V -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk $A > gpurun_out/r3h/trace_$V.log 2>&1 || exit 1
  python tools/timeline.py gpurun_out/r3h/trace_$V/run_kernel_trace.csv 7 > gpurun_out/r3h/timeline_$V.txt && echo "== $V" && cat gpurun_out/r3h/timeline_$V.txt
done
