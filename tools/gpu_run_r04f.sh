# Round 4: stream decoder (staging fix, gap-program parse): tests, whole call,
# per-phase clocks, stream PMC; TILE unpack and AoS counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04f_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_ab/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04f_phases.log 2>&1 || exit 3
PMC_TOOL=stream_bench.py timeout -k 10 900 bash tools/pmc_paths.sh r04f_stream multiple_primitives_str0-64 two_str_request || exit 4
timeout -k 10 900 bash tools/pmc_paths.sh r04_tile add_request_58B two_numbers_response || exit 5
timeout -k 10 900 bash tools/pmc_paths.sh r04_aos aos || exit 6
