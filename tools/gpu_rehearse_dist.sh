#!/bin/bash
# Rehearse the multi-rank bench (barrier, sharding, max-over-ranks, the training all-reduce) with
# 2 ranks sharing one GPU over gloo. The real N-GPU run uses RCCL, one GPU per rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1 NONODE_DIST_BACKEND=gloo
for wl in ${WLS:-egno egno_train segno segno_train}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --workload $wl --steps 5 --warmup 2 > gpurun_out/dist2_$wl.json 2> gpurun_out/dist2_$wl.err
  rc=$?; echo "dist2 $wl rc=$rc"; cat gpurun_out/dist2_$wl.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/dist2_$wl.err; exit $rc; }
done
exit 0
