# Round 6: kernel trace of the measured SLAM loop leg (track_frame every frame, optimize_map every 5th).
set -o pipefail
OUT=gpurun_out/r6loop; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --leg slam_loop > $OUT/loop.json 2> $OUT/loop.err || { tail -20 $OUT/loop.err; exit 1; }
tail -1 $OUT/loop.json; python tools/prof_summary.py $OUT/prof > $OUT/kernels.md && head -30 $OUT/kernels.md
