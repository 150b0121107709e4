# Round 4: stream decoder after the cluster test, run composition, extra slot,
# decode fast path: tests, whole call, per-phase clocks, kernel split.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04g_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04g_phases.log 2>&1 || exit 3
for F in multiple_primitives_str0-64 two_str_request string_0-16_8M; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_sprof_$F -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only $F > gpurun_out/r04g_sprof_$F.log 2>&1 || exit 4
done
