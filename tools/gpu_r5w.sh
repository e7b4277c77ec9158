# forward variants in the round-5 topology: units (default) / parts / pc
set -o pipefail
D=gpurun_out/r5w; mkdir -p $D; export TMPDIR=/tmp
run() {  # name mode
  NSLAM_FWD_MODE=$2 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/$1.json 2> $D/$1.err || { tail -20 $D/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); k=d['kernels_ms']; print(sys.argv[2], round(d['ms_per_step'],4), 'ms', {x: k.get(x) for x in ('query_fwd','query_bwd.color_wgrad','query_bwd.middle+fine+color','adam')})" $D/$1.json "$1"
}
for r in 1 2; do
run units_$r units
run parts_$r parts
run pc_$r pc
done
