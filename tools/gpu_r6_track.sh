# Round 6: tracker-iteration launches folded (nslam_loss_sum_best; the pose formed in the gather) — the
# tests, then the SLAM loop's track_frame and the room0 headline bench against the previous commit (a
# worktree in ab/head, built beside this tree).
set -o pipefail
OUT=gpurun_out/r6track; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_mapper.py tests/test_gpu_dropins.py tests/test_gpu_fused.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for V in head new; do
    if [ $V = head ]; then D=ab/head; else D=.; fi
    (cd $D && timeout -k 10 300 python bench.py --leg slam_loop) > $OUT/loop_${V}_$r.json 2> $OUT/loop_$V.err || { tail -20 $OUT/loop_$V.err; exit 1; }
    (cd $D && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames) > $OUT/bench_${V}_$r.json 2> $OUT/bench_$V.err || { tail -20 $OUT/bench_$V.err; exit 1; }
    python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); b=json.loads([l for l in open(sys.argv[4]) if l.startswith('{')][-1])
print(f'{sys.argv[2]:5s} round {sys.argv[3]}: track_frame {d[\"track_frame_ms\"]:.3f} ms, loop {d[\"frames_per_s\"]:.1f} fps, room0 {b[\"ms_per_step\"]:.4f} ms')" $OUT/loop_${V}_$r.json $V $r $OUT/bench_${V}_$r.json
  done
done
