# pc forward experiments: query_fwd time of variant builds (NSLAM_LIB) in pc mode; units for reference
set -o pipefail
D=gpurun_out/r5i; mkdir -p $D; export TMPDIR=/tmp
run() {  # name lib mode
  NSLAM_LIB=$PWD/nice-slam_amd/$2 NSLAM_FWD_MODE=$3 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/$1.json 2> $D/$1.err || { tail -20 $D/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],4), 'ms', 'fwd', d['kernels_ms'].get('query_fwd'))" $D/$1.json "$1"
}
for r in 1 2; do
run units_$r libnslam.so units
run pc_$r libnslam.so pc
run fd2_$r libnslam_fd2.so pc
run c4_$r libnslam_c4.so pc
run d2_$r libnslam_d2.so pc
run d2fd2_$r libnslam_d2fd2.so pc
run d1_$r libnslam_d1.so pc
done
