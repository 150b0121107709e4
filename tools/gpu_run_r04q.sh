# Round 4: two-string parity in bench_paths (tiled vs look-back, stream index),
# quad TILE unpack and all-kinds AoS rows on this box, phases with the
# decode's fast-path share, the STALLED test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_paths.py --only two_str --reps 10 > gpurun_out/r04q_two_str.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_paths.py --only quad_tile --reps 10 > gpurun_out/r04q_quad_tile.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04q_aos.log 2>&1 || exit 4
timeout -k 10 300 python3 tools/bench_paths.py --only aos --reps 10 > gpurun_out/r04q_aos_all.log 2>&1 || exit 5
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04q_phases.log 2>&1 || exit 6
