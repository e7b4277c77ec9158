set -o pipefail
mkdir -p gpurun_out/trk
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trk -o run -- python tools/probes/track_prof.py > gpurun_out/trk/log.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/trk/log.txt; exit 1; }
head -40 gpurun_out/trk/run_kernel_stats.csv | cut -c1-220
