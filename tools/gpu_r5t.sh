# N>1 rehearsal on the one-GPU box with the round-5 engine defaults: 2 gloo ranks (all-reduce exchange, the
# N>1 default) and 2 forced-world-1... (the driver's 8-GPU SCALE run uses RCCL; gloo exercises the code path)
set -o pipefail
D=gpurun_out/r5t; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline --no-stress --no-bulk --no-frames > $D/gloo2.json 2> $D/gloo2.err || { tail -30 $D/gloo2.err; exit 1; }
tail -c 700 $D/gloo2.json
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-stress --no-bulk --no-frames --force-exchange > $D/rccl1.json 2> $D/rccl1.err || { tail -20 $D/rccl1.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['ms_per_step'],4), 'ms', d.get('launch_mode'), d.get('exchange'), d.get('exchange_backend'), d.get('collective_ms_per_step'))" $D/rccl1.json
