# Round 4: gated scans on a capped grid -- full -m gpu, then string rows A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g2_pytest.log 2>&1 || exit 2
for r in 1 2; do
  echo "## base round $r" >> gpurun_out/r04g2_ab.log
  SRPC_GPU_LIB=build_ab/base.so timeout -k 10 200 python -u tools/bench_paths.py --only str --no-stream >> gpurun_out/r04g2_ab.log 2>&1 || exit 3
  echo "## new round $r" >> gpurun_out/r04g2_ab.log
  timeout -k 10 200 python -u tools/bench_paths.py --only str --no-stream >> gpurun_out/r04g2_ab.log 2>&1 || exit 4
done
