#!/bin/bash
# Same-box comparison of the single-process bench and the multi-rank path at one rank
# (--force-dist: gloo rendezvous, RCCL reward all-gather every --metrics-every steps).
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > gpurun_out/bench_plain_$i.log 2>/dev/null || exit 1
  echo "plain: $(tail -1 gpurun_out/bench_plain_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us/step")')"
  for me in 8 1000; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 100 --warmup 10 --force-dist --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line --metrics-every $me > gpurun_out/bench_dist_$me.log 2>/dev/null || exit 1
    echo "dist metrics_every=$me: $(tail -1 gpurun_out/bench_dist_$me.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), "us/step", d.get("gathered_rewards_ok"))')"
  done
done
