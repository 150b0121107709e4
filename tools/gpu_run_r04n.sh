# Round 4: sdx only (legacy decoders deleted), first string's lengths from the
# fixed pass; AoS layout kernels with plain loads, staged tile sizes; tiled
# two-string unpack row; kernel trace of the adversarial-stream test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py tests/test_gpu_aos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04n_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04n_phases.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/bench_paths.py --only aos --reps 10 > gpurun_out/r04n_aos.log 2>&1 || exit 4
for T in 12288 16384; do
  SRPC_AOS_NOLAY=1 SRPC_AOS_TILE_BYTES=$T timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04n_aos_nolay_$T.log 2>&1 || exit 5
done
SRPC_AOS_NOLAY=1 timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04n_aos_nolay.log 2>&1 || exit 6
timeout -k 10 300 python3 tools/bench_paths.py --only two_str --reps 10 > gpurun_out/r04n_two_str.log 2>&1 || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04n_adv -o run --output-format csv -- python3 -u -m pytest tests/test_gpu_stream.py -k adversarial -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_adv.log 2>&1 || exit 8
