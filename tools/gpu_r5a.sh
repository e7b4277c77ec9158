# round 5 first GPU call: wave timelines, the new tests, the forced world-1 RCCL bench
set -o pipefail
D=gpurun_out/r5a; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/probes/wave_timeline.py > $D/tl_default.log 2>&1 || { tail -30 $D/tl_default.log; exit 1; }
cat $D/tl_default.log
timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/tl_serial.log 2>&1 || { tail -30 $D/tl_serial.log; exit 1; }
cat $D/tl_serial.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_decoders.py tests/test_gpu_sharded.py tests/test_datasets_cpu.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -3 $D/tests.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
tail -c 600 $D/bench_default.json
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames --force-exchange > $D/bench_rccl1_allreduce.json 2> $D/bench_rccl1_allreduce.err || { tail -20 $D/bench_rccl1_allreduce.err; exit 1; }
tail -c 900 $D/bench_rccl1_allreduce.json
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames --force-exchange --exchange sharded > $D/bench_rccl1_sharded.json 2> $D/bench_rccl1_sharded.err || { tail -20 $D/bench_rccl1_sharded.err; exit 1; }
tail -c 900 $D/bench_rccl1_sharded.json
timeout -k 10 200 python -u bench.py --leg frame_io > $D/frame_io.json 2> $D/frame_io.err || { tail -20 $D/frame_io.err; exit 1; }
cat $D/frame_io.json
timeout -k 10 300 python -u tools/probes/touched_rows.py > $D/touched_rows.json 2> $D/touched_rows.err || { tail -20 $D/touched_rows.err; exit 1; }
cat $D/touched_rows.json
NSLAM_PREFETCH_AT=after_fwd timeout -k 10 240 python -u tools/probes/wave_timeline.py > $D/tl_after_fwd.log 2>&1 || { tail -30 $D/tl_after_fwd.log; exit 1; }
cat $D/tl_after_fwd.log
for r in 1 2; do for at in start after_fwd; do
NSLAM_PREFETCH_AT=$at timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/ab_${at}_$r.json 2> $D/ab_$at.err || { tail -20 $D/ab_$at.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms')" $D/ab_${at}_$r.json "$at round $r"
done; done
