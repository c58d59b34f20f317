# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks sharing cuda:0 over
# gloo (RCCL cannot put two ranks on one GPU), then the real 1-rank line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > gpurun_out/bench_dist2.log 2>&1
rc=$?; echo "dist2 rc=$rc"; tail -2 gpurun_out/bench_dist2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config e2e --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/bench_dist2_e2e.log 2>&1
rc=$?; echo "dist2 e2e rc=$rc"; tail -1 gpurun_out/bench_dist2_e2e.log
exit $rc
