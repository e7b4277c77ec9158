# knob sweep at the round-3 state: forward parts, lean-kernel occupancy (variant builds), quick bench each
set -o pipefail
mkdir -p gpurun_out/r3k
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > gpurun_out/r3k/$n.json 2> gpurun_out/r3k/$n.err || { tail -5 gpurun_out/r3k/$n.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['frac'],3))" gpurun_out/r3k/$n.json $n
}
for r in 1 2; do
run default$r NSLAM_FWD_PARTS=0
run parts3_$r NSLAM_FWD_PARTS=3
run fwdlb3_$r NSLAM_LIB=$PWD/nice-slam_amd/libnslam_fwdlb3.so
done
