# Round 4, first box run: server overflow e2e tests, bench (pipelined PCIe legs), N=2 gloo rehearsal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_e2e_square.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04a_e2e.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r04a_bench.log 2>&1 || exit 2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > gpurun_out/r04a_bench_gloo2.log 2>&1 || exit 3
