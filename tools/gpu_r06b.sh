# Round 6: repair pass (sdx exit slots) -- stream parity in every mode, then
# the straddle rows, then the rest of the GPU suite, the launcher checks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/probe_register.py > gpurun_out/probe_register.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stream_r06b.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/stream_bench.py --reps 5 --only straddle > gpurun_out/stream_straddle_r06b.log 2>&1 || exit 2
timeout -k 10 300 python3 -u tools/stream_bench.py --reps 5 --only 256K >> gpurun_out/stream_straddle_r06b.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --ignore=tests/test_gpu_stream.py > gpurun_out/pytest_gpu_r06b.log 2>&1 || exit 4
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --records 4194304 > gpurun_out/bench_spawn_gloo2.log 2>&1 || exit 5
timeout -k 10 120 python3 bench.py --gpus 2 --steps 5 > gpurun_out/bench_nccl2_refused.log 2>&1; echo "nccl2 rc=$?" >> gpurun_out/bench_nccl2_refused.log

# interleaved A/B: landing slots kept (cur) / dropped (noland, the repair pass covers them) / round 5
bash tools/ab_variants.sh "r05 cur zm zmnl" "string_0-16_8M multiple_primitives_str0-64 zh4_random_4M multiple_primitives_zeros_4M zh4_straddle_heavy_4M zh4_straddle_heavy_long_256K zh4_random_256K" 1 5 > gpurun_out/ab_noland_r06b.log 2>&1 || exit 6
exit 0
