# quick perf check: cw phases, knob timings, one-iteration timeline.  usage: bash tools/gpu_quick.sh TAG [pytest]
set -o pipefail
D=gpurun_out/${1:?tag}
mkdir -p $D
export TMPDIR=/tmp
if [ "$2" = pytest ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
  tail -1 $D/pytest.log
fi
timeout -k 10 200 python -u tools/probes/cw_phases.py > $D/cw_phases.log 2>&1 || { tail -20 $D/cw_phases.log; exit 1; }
cat $D/cw_phases.log
timeout -k 10 300 python -u tools/probes/knobs.py default merged merged_all > $D/knobs.log 2>&1 || { tail -20 $D/knobs.log; exit 1; }
cat $D/knobs.log
bash tools/gpu_trace.sh $1
