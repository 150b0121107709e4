# Round profile on one MI355X: parity tests, variant sweep, bench, rocprofv3
# kernel stats and the two PMC passes, summarised into gpurun_out/.
# usage (from the repo root, through gpurun): bash tools/gpu_profile.sh rNN
set -o pipefail
R=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
# the strong-scaling line (64M records) is left out so every launch is a 16M one
BENCH="python3 bench.py --cpu-seconds 0 --no-pcie --no-verify --strong-records 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${R}.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- $BENCH --steps 20 --warmup 3 > gpurun_out/prof_stats.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- $BENCH --steps 5 --warmup 1 > gpurun_out/prof_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- $BENCH --steps 5 --warmup 1 > gpurun_out/prof_write.log 2>&1 || exit 5
python tools/pmc_summary.py --stats gpurun_out/prof_stats --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write --records 16777216 --out gpurun_out/pmc_traffic_${R}.json > /dev/null || exit 6
