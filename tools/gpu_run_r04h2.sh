# Round 4: host-terminated batches (ABI 7) -- parity, then the bench line with the native pipeline legs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_host.py > gpurun_out/r04h2_host_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/r04h2_bench.log 2>&1 || exit 3
