# Round 4: the tile table loaded with the index (record-tile unpack) -- parity, phases, A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiled.py > gpurun_out/r04v3_tests.log 2>&1 || exit 2
SRPC_GPU_LIB=build_ab/ph.so timeout -k 10 200 python -u tools/var_phases.py --case two_str --tiled > gpurun_out/r04v3_phases.log 2>&1 || exit 3
for r in 1 2; do
  echo "## base round $r" >> gpurun_out/r04v3_ab.log
  SRPC_GPU_LIB=build_ab/base.so timeout -k 10 200 python -u tools/bench_paths.py --only two_str --no-stream >> gpurun_out/r04v3_ab.log 2>&1 || exit 4
  echo "## new round $r" >> gpurun_out/r04v3_ab.log
  timeout -k 10 200 python -u tools/bench_paths.py --only two_str --no-stream >> gpurun_out/r04v3_ab.log 2>&1 || exit 5
done
