set -o pipefail
mkdir -p gpurun_out/sweep
for px in 1000 2000 4000 8000 16000; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --pixels $px > gpurun_out/sweep/b$px.json 2> gpurun_out/sweep/b$px.err || { tail -5 gpurun_out/sweep/b$px.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/b$px.json')); print($px, round(d['value']/1e6,1), round(d['ms_per_step'],3), d['kernels_ms'])"
done
