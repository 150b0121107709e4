# Round 4: decode chars gather by segments; K1 table cost (tables modes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04k_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04k_phases.log 2>&1 || exit 3
for T in 0 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_sprof_t$T -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only str0-64 --tables $T > gpurun_out/r04k_sprof_t$T.log 2>&1 || exit 4
done
