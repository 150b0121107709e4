# Round 4: decode gathers chars from the stage (no image; 8 blocks per CU),
# record kernels at their measured tile depths: tests, whole call, phases.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py tests/test_gpu_rec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stream_bench.py --reps 10 > gpurun_out/r04j_stream.log 2>&1 || exit 2
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04j_phases.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/bench_paths.py --only _request_ --reps 10 > gpurun_out/r04j_paths_req.log 2>&1 || exit 4
timeout -k 10 300 python3 tools/bench_paths.py --only _response_ --reps 10 > gpurun_out/r04j_paths_resp.log 2>&1 || exit 5
