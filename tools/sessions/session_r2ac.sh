#!/bin/bash
# Round 2 (r2ac): rehearse bench.py's two-rank path on the one-GPU box (gloo,
# both ranks on cuda:0), weak and strong scaling.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
tools/gpu_session.sh \
  "two_rank_weak:300:$R --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --share-device --no-cpu --chains 16384 > gpurun_out/two_rank_weak.json" \
  "two_rank_strong:300:$R --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --share-device --no-cpu --scaling strong --chains 32768 > gpurun_out/two_rank_strong.json"
