# Round-end evidence on one MI355X: GPU tests, smoke, the driver's bench
# command, rocprofv3 kernel stats + PMC traffic of the bench (16M launches),
# and the all-path and stream tables.
# usage (through gpurun): bash tools/gpu_final.sh rNN [1|2]
# (part 1: smoke, bench, tests, profile; part 2: the two tables; default both)
set -o pipefail
R=${1:-r02}
P=${2:-all}
mkdir -p gpurun_out
if [ "$P" != 2 ]; then
  timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${R}.log 2>&1 || exit 1
  timeout -k 10 300 python3 bench.py > gpurun_out/bench_default_${R}.log 2>&1 || exit 2
  bash tools/gpu_profile.sh "$R" || exit 3
fi
if [ "$P" != 1 ]; then
  timeout -k 10 400 python3 tools/bench_paths.py --reps 10 --out gpurun_out/paths_${R}.json > gpurun_out/paths_${R}.log 2>&1 || exit 4
  timeout -k 10 400 python3 -u tools/stream_bench.py --reps 10 --out gpurun_out/stream_${R}.json > gpurun_out/stream_${R}.log 2>&1 || exit 5
fi
