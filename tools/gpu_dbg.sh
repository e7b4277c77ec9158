# ABI v15 camera gradient: GPU tests (fused + loop), then frames/s
set -o pipefail
mkdir -p gpurun_out/r3t2
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_loop.py tests/test_gpu_dropins.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3t2/tests.log 2>&1 || { tail -30 gpurun_out/r3t2/tests.log; exit 1; }
tail -1 gpurun_out/r3t2/tests.log
timeout -k 10 300 python bench.py --leg frames > gpurun_out/r3t2/frames.json 2> gpurun_out/r3t2/frames.err || { tail -5 gpurun_out/r3t2/frames.err; exit 1; }
tail -1 gpurun_out/r3t2/frames.json | cut -c1-400
timeout -k 10 300 python bench.py --leg frames > gpurun_out/r3t2/frames2.json 2> gpurun_out/r3t2/frames2.err || { tail -5 gpurun_out/r3t2/frames2.err; exit 1; }
tail -1 gpurun_out/r3t2/frames2.json | cut -c1-400
