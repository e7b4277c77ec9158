# GPU test run: bash tools/gpu_tests.sh TAG [pytest selection...]   (default: the whole -m gpu suite)
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -60
[ $rc -ne 0 ] && tail -80 $OUT/tests.log
exit $rc
