#!/bin/bash
# Round-2 session R: two-rank gloo rehearsal of bench.py's multi-rank path on one GPU (the RCCL path
# needs one GPU per rank; its one-rank job is in tests/test_gpu_multi.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > gpurun_out/n2_gloo.log 2>&1 || { tail -20 gpurun_out/n2_gloo.log; exit 1; }
grep '"metric"' gpurun_out/n2_gloo.log | cut -c1-400
