# capture-order experiment of the pipelined mapping iteration (quick bench per variant + one timeline)
set -o pipefail
mkdir -p gpurun_out/r3f
for V in 0 1 2; do
  NSLAM_PIPE_ORDER=$V timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames --pipeline > gpurun_out/r3f/o$V.json 2> gpurun_out/r3f/o$V.err || { tail -5 gpurun_out/r3f/o$V.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4))" gpurun_out/r3f/o$V.json order$V
done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames --no-pipeline > gpurun_out/r3f/nopipe.json 2> gpurun_out/r3f/nopipe.err || exit 1
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('nopipe', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4))" gpurun_out/r3f/nopipe.json
for V in 1 2; do
NSLAM_PIPE_ORDER=$V timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3f/trace$V -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk --pipeline > gpurun_out/r3f/trace$V.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/r3f/trace$V/run_kernel_trace.csv 7 > gpurun_out/r3f/timeline$V.txt && cat gpurun_out/r3f/timeline$V.txt
done
