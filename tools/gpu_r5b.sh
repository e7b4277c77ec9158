# production-register timelines of the room0 iteration; dynamic-forward A/B
set -o pipefail
D=gpurun_out/r5b; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/probes/wave_timeline.py > $D/tl_default.log 2>&1 || { tail -30 $D/tl_default.log; exit 1; }
cat $D/tl_default.log
timeout -k 10 240 python -u tools/probes/wave_timeline.py --no-prefetch --serial > $D/tl_serial.log 2>&1 || { tail -30 $D/tl_serial.log; exit 1; }
cat $D/tl_serial.log
for r in 1 2; do for dyn in 0 1; do
NSLAM_FWD_DYN=$dyn timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/ab_dyn${dyn}_$r.json 2> $D/ab_dyn$dyn.err || { tail -20 $D/ab_dyn$dyn.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', 'fwd', d['kernels_ms'].get('query_fwd'))" $D/ab_dyn${dyn}_$r.json "dyn=$dyn round $r"
done; done
