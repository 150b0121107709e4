# Round 4: which box is this (partition modes, clocks) and the rows that moved
# between boxes (quad TILE unpack, all-kinds AoS).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showcomputepartition --showmemorypartition --showclocks --showproductname; rocminfo | grep -E "Marketing|Compute Unit|Max Clock") > gpurun_out/r04r_box.log 2>&1
timeout -k 10 300 python3 tools/bench_paths.py --only quad_tile --reps 10 > gpurun_out/r04r_quad_tile.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04r_aos.log 2>&1 || exit 4
timeout -k 10 300 python3 tools/bench_paths.py --only quad_dword --reps 10 > gpurun_out/r04r_quad.log 2>&1 || exit 5
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1 || exit 6
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04r_stream.log 2>&1 || exit 7
