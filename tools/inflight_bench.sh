export TMPDIR=/tmp
mkdir -p gpurun_out/bfl
B="timeout -k 10 200 python bench.py --secondary '' --cpu-baseline off --steps 100"
for F in 1 2 3; do
  eval $B --tiles --inflight $F > gpurun_out/bfl/tiles_f$F.json || exit 1
  eval $B --shard 0/8 --inflight $F > gpurun_out/bfl/shard8_f$F.json || exit 1
done
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --backend gloo --same-device --steps 20 --warmup 4 --inflight 2 --cpu-baseline off > gpurun_out/bfl/gloo_n$n.json 2> gpurun_out/bfl/gloo_n$n.err || { tail -20 gpurun_out/bfl/gloo_n$n.err; exit 1; }
done
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/bfl/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); c=d['config']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], c.get('kernel_ms'), c.get('frames_in_flight'), c.get('tiles_frame_check'))
P
