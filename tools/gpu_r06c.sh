# Round 6: the repair pass with bitmap-deduplicated exit slots: the straddle
# rows first (diagnostics), then stream parity in every mode.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/stream_bench.py --reps 5 --only straddle > gpurun_out/stream_straddle_r06c.log 2>&1 || exit 2
timeout -k 10 300 python3 -u tools/stream_bench.py --reps 5 --only 256K >> gpurun_out/stream_straddle_r06c.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -q --timeout 200 --timeout-method thread > gpurun_out/pytest_stream_r06c.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_stream_r06c.log
exit 0
