# The driver's multi-GPU launch form rehearsed on one GPU: torch.distributed.run
# with one rank over RCCL (the default backend), then two ranks over gloo
# sharing the box's GPU (labelled a rehearsal in the line).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6_dist1_rccl.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > gpurun_out/r6_dist2_gloo.log 2>&1 || exit 1
exit 0
