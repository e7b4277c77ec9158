set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > gpurun_out/gpu_tests_r1a.log 2>&1; rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/gpu_tests_r1a.log
exit $rc
