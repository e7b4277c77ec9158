# A/B: colour weight-gradient chunk count 256 (default) / 224 / 192 — fewer CUs for k_color_wgrad, more for the mask-only launch
set -o pipefail
D=gpurun_out/r5r; mkdir -p $D; export TMPDIR=/tmp
run() {  # name lib
  NSLAM_LIB=$PWD/nice-slam_amd/$2 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/$1.json 2> $D/$1.err || { tail -20 $D/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); k=d['kernels_ms']; print(sys.argv[2], round(d['ms_per_step'],4), 'ms', {x: k.get(x) for x in ('query_fwd','query_bwd.color_wgrad','query_bwd.middle+fine+color','adam')})" $D/$1.json "$1"
}
for r in 1 2 3; do
run base_$r libnslam.so
run cw224_$r libnslam_cw224.so
run cw192_$r libnslam_cw192.so
done
