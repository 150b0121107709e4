# Round 4: decode copies chars lane per record (no spills, 8 blocks per CU),
# cluster pick inside the candidate test; AoS layout kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py tests/test_gpu_aos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04m_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04m_phases.log 2>&1 || exit 3
for F in str0-64 0-1024; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04m_sprof_$F -o run --output-format csv -- python3 tools/stream_bench.py --reps 5 --only $F > gpurun_out/r04m_sprof_$F.log 2>&1 || exit 4
done
timeout -k 10 300 python3 tools/bench_paths.py --only aos --reps 10 > gpurun_out/r04m_aos.log 2>&1 || exit 5
SRPC_AOS_NOLAY=1 timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04m_aos_nolay.log 2>&1 || exit 6
