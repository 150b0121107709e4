# Round 4: short strings compacted in the decode's stage, aligned stores out.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04v_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04v_phases.log 2>&1 || exit 3
