# Round 6, first GPU check: parity suite, the self-spawning N>1 bench (gloo
# rehearsal on one GPU), the NCCL refusal on a one-GPU box, the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/probe_register.py > gpurun_out/probe_register.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r06a.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --records 4194304 > gpurun_out/bench_spawn_gloo2.log 2>&1 || exit 2
timeout -k 10 120 python3 bench.py --gpus 2 --steps 5 > gpurun_out/bench_nccl2_refused.log 2>&1; echo "nccl2 rc=$?" >> gpurun_out/bench_nccl2_refused.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default_r06a.log 2>&1 || exit 3
