# Round 6: kernel traces of the captured room0 iteration in three topologies (default; branches
# serialised; serialised without the ray prefetch: one queue) to measure the graph's inter-node gaps.
set -o pipefail
OUT=gpurun_out/r6gaps; mkdir -p $OUT; export TMPDIR=/tmp
for V in default serial serial_nopf; do
  case $V in default) A="";; serial) A="--serial-branches";; serial_nopf) A="--serial-branches --no-prefetch";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$V -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stress --no-frames --no-bulk $A > $OUT/$V.json 2> $OUT/$V.err || { tail -20 $OUT/$V.err; exit 1; }
  grep '^{' $OUT/$V.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', d['ms_per_step'])"
done
