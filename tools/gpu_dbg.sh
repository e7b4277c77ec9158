# robustness: smoke(), 2-rank gloo rehearsal of the sharded bench on one GPU
set -o pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s/smoke.log 2>&1 || { tail -20 gpurun_out/r3s/smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3s/smoke.log | tail -2
bash tools/gpu_cycle.sh r3s gloo2
