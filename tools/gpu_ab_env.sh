# A/B of engine environment knobs on one box: the room0 colour-stage bench under each setting, ROUNDS
# alternating rounds, then each setting's median.  usage: ROUNDS=3 bash tools/gpu_ab_env.sh TAG "VAR=a" "VAR=b" ...
set -o pipefail
OUT=gpurun_out/${1:?tag}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $OUT/ab_${i}_$r.json 2> $OUT/ab_$i.err || { tail -20 $OUT/ab_$i.err; exit 1; }
    python -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], 'round', sys.argv[3], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms')" $OUT/ab_${i}_$r.json "$E" $r
  done
done
python - "$OUT" "$@" <<'PY'
import json, statistics, sys, glob
out = sys.argv[1]
for i, e in enumerate(sys.argv[2:], 1):
    v = [json.loads([l for l in open(f) if l.startswith("{")][-1])["ms_per_step"] for f in sorted(glob.glob(f"{out}/ab_{i}_[0-9]*.json"))]
    print(f"{e:40s} median {statistics.median(v):.4f} ms over {len(v)}: {[round(x, 4) for x in v]}")
PY
