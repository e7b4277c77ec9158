# A/B of libraries (NSLAM_LIB) on the bench's reference-API legs: optimize_map (room0, with and without
# BA), scene0000 (BA window 5) and the measured SLAM loop.  usage: ROUNDS=2 bash tools/gpu_ab_legs.sh TAG lib1 lib2 ...
set -o pipefail
OUT=gpurun_out/${1:?tag}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for L in "$@"; do
    i=$((i+1))
    for leg in optimize_map scene0000 slam_loop; do
      NSLAM_LIB=$L timeout -k 10 300 python bench.py --leg $leg > $OUT/${leg}_${i}_$r.json 2> $OUT/${leg}_$i.err || { tail -20 $OUT/${leg}_$i.err; exit 1; }
    done
    python - "$OUT" $i $r "$L" <<'PY'
import json, sys
out, i, r, lib = sys.argv[1:]
def last(f): return json.loads([l for l in open(f) if l.startswith("{")][-1])
om, sc, lp = (last(f"{out}/{k}_{i}_{r}.json") for k in ("optimize_map", "scene0000", "slam_loop"))
print(f"{lib:42s} round {r}: optimize_map {om['optimize_map']['ms_per_iteration']:.4f} BA {om['optimize_map_ba']['ms_per_iteration']:.4f} "
      f"(engine BA colour {om['engine_ba_ms_per_iteration']['color']:.4f}) scene0000 BA {sc['optimize_map_ba']['ms_per_iteration']:.4f} "
      f"loop {lp['frames_per_s']:.1f} fps track {lp['track_frame_ms']:.3f} ms")
PY
  done
done
