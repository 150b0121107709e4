# Round 4: stream decoder after the scan fixes: tests, whole-call bench, kernel
# split (0-64 B with the zero-byte / exact filter), per-phase clocks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04d_stream.log 2>&1 || exit 2
for T in 0 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04d_sprof_t$T -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only multiple_primitives_str0-64 --tables $T > gpurun_out/r04d_sprof_t$T.log 2>&1 || exit 3
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04d_sprof_two -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only two_str_request > gpurun_out/r04d_sprof_two.log 2>&1 || exit 4
SRPC_GPU_LIB=build_ab/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04d_phases.log 2>&1 || exit 5
