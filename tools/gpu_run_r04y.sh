# Round 4: the speculation's chunk repair -- stream parity, phases, A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/r04y_stream_tests.log 2>&1 || exit 2
SRPC_GPU_LIB=build_ab/sx_rep.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04y_phases.log 2>&1 || exit 3
SRPC_GPU_LIB=build_ab/base.so timeout -k 10 300 python -u tools/stream_bench.py > gpurun_out/r04y_stream_base.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/stream_bench.py > gpurun_out/r04y_stream_new.log 2>&1 || exit 5
timeout -k 10 300 python -u tools/stream_bench.py --tables 8 > gpurun_out/r04y_stream_norep.log 2>&1 || exit 6
SRPC_GPU_LIB=build_ab/base.so timeout -k 10 300 python -u tools/stream_bench.py > gpurun_out/r04y_stream_base2.log 2>&1 || exit 7
