# Round 4: AoS run-layout unpack with whole-line piece stores -- parity, then old / new interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_aos.py > gpurun_out/r04z2_aos_tests.log 2>&1 || exit 2
for r in 1 2; do
  for m in 0 1; do
    echo "## SRPC_AOS_RUN_PIECE=$m round $r" >> gpurun_out/r04z2_aos_ab.log
    SRPC_AOS_RUN_PIECE=$m timeout -k 10 200 python -u tools/bench_paths.py --only aos >> gpurun_out/r04z2_aos_ab.log 2>&1 || exit 3
  done
done
