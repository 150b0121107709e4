# Round 4: the table-scan stream decoder (sdx.hip): its parity tests, then the whole-call bench against the old decoders.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04b_stream_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04b_stream_new.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 --single 7 > gpurun_out/r04b_stream_legacy.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/pcie_sweep.py > gpurun_out/r04b_pcie_sweep.log 2>&1 || exit 4
