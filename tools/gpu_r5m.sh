# A/B of candidate defaults (ReLU/mask formulation vs before, branch order, wgrad chunk count, unit order,
# 4-wave units), then the round's final measurements (tools/gpu_final_r5.sh) on the current default
set -o pipefail
D=gpurun_out/r5m; mkdir -p $D; export TMPDIR=/tmp
run() {  # name lib [env]
  env NSLAM_LIB=$PWD/nice-slam_amd/$2 $3 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/$1.json 2> $D/$1.err || { tail -20 $D/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); k=d['kernels_ms']; print(sys.argv[2], round(d['ms_per_step'],4), 'ms', {x: k[x] for x in ('query_fwd','query_bwd.color_wgrad','query_bwd.middle+fine+color','query_bwd')})" $D/$1.json "$1"
}
for r in 1 2; do
run base_$r libnslam.so
run pre_$r libnslam_pre.so
run lean1st_$r libnslam.so NSLAM_WGRAD_FIRST=0
run cw128_$r libnslam_cw128.so
run ord1_$r libnslam_ord1.so
run u4_$r libnslam_u4.so
done
bash tools/gpu_final_r5.sh
