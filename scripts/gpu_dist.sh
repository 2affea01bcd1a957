#!/bin/bash
# multi-rank rehearsal on one GPU: 2 ranks over gloo (test + bench launch path)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dist
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || exit $?
MAS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 16 --warmup 16 --horizon 16 --envs 4096 > $O/bench2.log 2>&1 || exit $?
echo ok
