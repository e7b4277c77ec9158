# A/B of environment settings on the tracker: the measured SLAM loop leg's track_frame (ms per frame, 10
# camera iterations) and loop rate.  usage: ROUNDS=2 bash tools/gpu_ab_track.sh TAG "VAR=a" "VAR=b" ...
set -o pipefail
OUT=gpurun_out/${1:?tag}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python bench.py --leg slam_loop > $OUT/loop_${i}_$r.json 2> $OUT/loop_$i.err || { tail -20 $OUT/loop_$i.err; exit 1; }
    python -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(f'{sys.argv[2]:28s} round {sys.argv[3]}: track_frame {d[\"track_frame_ms\"]:.3f} ms, loop {d[\"frames_per_s\"]:.1f} fps')" $OUT/loop_${i}_$r.json "$E" $r
  done
done
