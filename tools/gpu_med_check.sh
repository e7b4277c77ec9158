set -o pipefail
mkdir -p gpurun_out/r6med
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -q --timeout 240 --timeout-method thread -k "median or render_loss or cam_grad_step or tracker" > gpurun_out/r6med/tests.log 2>&1 || { tail -30 gpurun_out/r6med/tests.log; exit 1; }
tail -1 gpurun_out/r6med/tests.log
bash tools/gpu_track_prof.sh r6medtp
