# pc forward diagnosis: timelines of the full pc kernel, consumers-skip (d1), producers-skip (d2), units
set -o pipefail
D=gpurun_out/r5g; mkdir -p $D; export TMPDIR=/tmp
for v in tl tl_d1 tl_d2; do
NSLAM_LIB=$PWD/nice-slam_amd/libnslam_$v.so NSLAM_FWD_MODE=pc timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/$v.log 2>&1 || { tail -30 $D/$v.log; exit 1; }
echo "== $v"; sed -n 2,8p $D/$v.log
done
NSLAM_FWD_MODE=units timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/units.log 2>&1 || { tail -30 $D/units.log; exit 1; }
echo "== units"; sed -n 2,20p $D/units.log
