# Round 4: N>1 rehearsal on one MI355X (2 ranks over gloo) on the final tree (after ABI 7).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --records 4194304 > gpurun_out/r04w2_gloo2.log 2>&1 || exit 1
