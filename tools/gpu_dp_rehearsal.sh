#!/bin/bash
# N>1 rehearsal on a one-GPU box: bench.py with 2 ranks on cuda:0 over gloo through torch DDP (the
# driver's real N>1 runs use RCCL, one rank per GPU), then the N=1 bench line.
set -o pipefail
O=gpurun_out/${TAG:-dp}
mkdir -p $O
UNET_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 \
  > $O/dp2.json 2> $O/dp2.err || { echo "dp2 failed"; tail -30 $O/dp2.err; exit 1; }
cat $O/dp2.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
