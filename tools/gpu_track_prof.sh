# The tracker probe alone, then under rocprofv3 --kernel-trace --stats; one frame's dispatch timeline.
set -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/probes/track_frames.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/probes/track_frames.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernels.md 2>&1 && head -30 $OUT/kernels.md
python tools/probes/frame_timeline.py $OUT/prof > $OUT/timeline.txt && head -80 $OUT/timeline.txt
