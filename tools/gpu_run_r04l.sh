# Round 4: AoS layout kernels (all-kinds struct, plain and behind a vtable
# slot): tests, rows vs the staged kernels (SRPC_AOS_NOLAY=1), PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_paths.py --only aos --reps 10 > gpurun_out/r04l_aos.log 2>&1 || exit 2
SRPC_AOS_NOLAY=1 timeout -k 10 300 python3 tools/bench_paths.py --only all_kinds_aos --reps 10 > gpurun_out/r04l_aos_nolay.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/bench_paths.py --only aos --reps 10 > gpurun_out/r04l_aos2.log 2>&1 || exit 4
bash tools/pmc_paths.sh r04l aos || exit 5
