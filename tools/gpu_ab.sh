# A/B of libnslam builds (same ABI) on one box: the room0 colour-stage bench of each, then a
# one-iteration kernel timeline of each.  usage: bash tools/gpu_ab.sh TAG LIB...   (paths relative
# to the repo; build variants with make -C nice-slam_amd/csrc variant V=name X="-D...")
set -o pipefail
OUT=gpurun_out/${1:?tag}; shift
mkdir -p $OUT
export TMPDIR=/tmp
[ $# -ge 1 ] || { echo "no libraries"; exit 2; }
summ() { python -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d.get('kernels_ms'))" "$1" "$2"; }
# ROUNDS=k: k alternating rounds of the benches (A B C A B C ...), then each library's median
for r in $(seq 1 ${ROUNDS:-1}); do
  for L in "$@"; do
    n=$(basename $L .so)
    NSLAM_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $OUT/bench_${n}_$r.json 2> $OUT/bench_$n.err || { tail -20 $OUT/bench_$n.err; exit 1; }
    summ $OUT/bench_${n}_$r.json "$n round $r"
  done
done
python - "$OUT" "$@" <<'PY'
import json, statistics, sys, glob, os
out = sys.argv[1]
for L in sys.argv[2:]:
    n = os.path.basename(L)[:-3]
    v = []
    for f in sorted(glob.glob(f"{out}/bench_{n}_[0-9]*.json")):
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        v.append(d["ms_per_step"])
    print(f"{n:24s} median {statistics.median(v):.4f} ms over {len(v)}: {[round(x, 4) for x in v]}")
PY
[ -n "$NO_TRACE" ] && exit 0
for L in "$@"; do
  n=$(basename $L .so)
  NSLAM_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-stress --no-frames --no-bulk > $OUT/trace_$n.log 2>&1 || { tail -20 $OUT/trace_$n.log; exit 1; }
  python tools/timeline.py $OUT/trace_$n/run_kernel_trace.csv 7 > $OUT/timeline_$n.txt && echo "== $n" && cat $OUT/timeline_$n.txt
done
