# Round 4 final: C++ API test (host-terminated calls added) + host tests, then the bench line reading the final kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cpp_api.py tests/test_gpu_host.py > gpurun_out/r04f2_tests.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py > gpurun_out/r04f2_bench.log 2>&1 || exit 3
