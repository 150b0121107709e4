# Round 4: TILE gather reverted, AoS unpack back on the staged kernels by
# default (layout unpack behind a hook): AoS + parity tests, rows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aos.py tests/test_gpu_parity.py tests/test_gpu_rec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04u_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_paths.py --only quad --reps 10 > gpurun_out/r04u_quad.log 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_paths.py --only aos --reps 10 > gpurun_out/r04u_aos.log 2>&1 || exit 3
