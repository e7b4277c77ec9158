# One GPU measurement cycle.  usage (via gpurun): bash tools/gpu_cycle.sh TAG [steps...]
# steps (default: tests bench prof): tests | tests-fast (fused+parity only) | bench | bench-quick
# (no baselines / stress / side legs) | eager | gloo2 (2-rank gloo rehearsal of the sharded bench)
# | gloo2ar (the same with --exchange allreduce) | prof (rocprofv3 kernel stats) | trace (timeline of one replayed iteration) | phases
# (s_memtime phase breakdown of the backward waves; needs `make -C nice-slam_amd/csrc phases`).
# Every GPU step runs under its own timeout; the first failure ends the script.
set -o pipefail
TAG=${1:?tag}; shift
STEPS=${*:-tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
summ() { python -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d.get('kernels_ms'))
r=d.get('room0'); print('  room0', r) if r else None" "$1" "$2"; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; stop tests 1; }
      tail -2 $OUT/gpu_tests.log ;;
    tests-fast)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_fast.log 2>&1 || { tail -30 $OUT/gpu_tests_fast.log; stop tests-fast 1; }
      tail -2 $OUT/gpu_tests_fast.log ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; stop bench 1; }
      summ $OUT/bench.json bench ;;
    bench-quick)
      timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk > $OUT/bench_quick.json 2> $OUT/bench_quick.err || { tail -30 $OUT/bench_quick.err; stop bench-quick 1; }
      summ $OUT/bench_quick.json quick ;;
    eager)
      timeout -k 10 300 python bench.py --steps 30 --warmup 5 --eager --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/bench_eager.json 2> $OUT/bench_eager.err || { tail -30 $OUT/bench_eager.err; stop eager 1; }
      summ $OUT/bench_eager.json eager ;;
    gloo2)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { tail -30 $OUT/bench_gloo2.err; stop gloo2 1; }
      summ $OUT/bench_gloo2.json gloo2 ;;
    gloo2ar)  # the same rehearsal with the all-reduce exchange (replicated Adam)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --exchange allreduce > $OUT/bench_gloo2_allreduce.json 2> $OUT/bench_gloo2_allreduce.err || { tail -30 $OUT/bench_gloo2_allreduce.err; stop gloo2ar 1; }
      summ $OUT/bench_gloo2_allreduce.json gloo2ar ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-bulk > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; stop prof 1; }
      python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -30 $OUT/kernels.md ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; stop trace 1; }
      python tools/timeline.py $OUT/trace/run_kernel_trace.csv 7 > $OUT/timeline.txt && cat $OUT/timeline.txt ;;
    phases)
      NSLAM_LIB=nice-slam_amd/libnslam_phases.so timeout -k 10 200 python tools/probes/phases.py > $OUT/phases.txt 2>&1 || { tail -20 $OUT/phases.txt; stop phases 1; }
      cat $OUT/phases.txt ;;
    variant:*)  # timing of an experiment build (make -C nice-slam_amd/csrc variant V=name X=...)
      v=${s#variant:}
      NSLAM_LIB=nice-slam_amd/libnslam_$v.so timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -30 $OUT/bench_$v.err; stop $s 1; }
      summ $OUT/bench_$v.json $v ;;
    probe:*)  # python tools/probes/<name>.py
      v=${s#probe:}
      timeout -k 10 300 python tools/probes/$v.py > $OUT/probe_$v.txt 2>&1 || { tail -30 $OUT/probe_$v.txt; stop $s 1; }
      cat $OUT/probe_$v.txt ;;
    *) stop "unknown step $s" 2 ;;
  esac
done
