# A/B: the mask-only launch at a 6-wave register bound (77 VGPRs, no spills) vs the default 4 (92 VGPRs, 5 waves)
set -o pipefail
D=gpurun_out/r5v; mkdir -p $D; export TMPDIR=/tmp
NSLAM_LIB=$PWD/nice-slam_amd/libnslam_lb6.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "engine or merged" > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
run() {  # name lib
  NSLAM_LIB=$PWD/nice-slam_amd/$2 timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/$1.json 2> $D/$1.err || { tail -20 $D/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); k=d['kernels_ms']; print(sys.argv[2], round(d['ms_per_step'],4), 'ms', {x: k.get(x) for x in ('query_fwd','query_bwd.color_wgrad','query_bwd.middle+fine+color','adam')})" $D/$1.json "$1"
}
for r in 1 2 3; do
run base_$r libnslam.so
run lb6_$r libnslam_lb6.so
done
