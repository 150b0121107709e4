# Round 6: the repair pass (exit slots), the zero map, the fused scan --
# straddle rows (diagnostics), stream parity in every mode, the rest of the
# GPU suite, the launcher, then an interleaved A/B against round 5's library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/stream_bench.py --reps 5 --only straddle > gpurun_out/stream_straddle_r06d.log 2>&1 || exit 2
timeout -k 10 300 python3 -u tools/stream_bench.py --reps 5 --only 256K >> gpurun_out/stream_straddle_r06d.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stream_r06d.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_stream_r06d.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --ignore=tests/test_gpu_stream.py > gpurun_out/pytest_gpu_r06d.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu_r06d.log
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --records 4194304 > gpurun_out/bench_spawn_gloo2.log 2>&1
echo "rc=$?" >> gpurun_out/bench_spawn_gloo2.log
timeout -k 10 120 python3 bench.py --gpus 2 --steps 5 > gpurun_out/bench_nccl2_refused.log 2>&1; echo "nccl2 rc=$?" >> gpurun_out/bench_nccl2_refused.log
bash tools/ab_variants.sh "r05 now nownl" "string_0-16_8M multiple_primitives_str0-64 zh4_random_4M multiple_primitives_zeros_4M zh4_straddle_heavy_4M" 1 5 > gpurun_out/ab_r06d.log 2>&1
exit 0
