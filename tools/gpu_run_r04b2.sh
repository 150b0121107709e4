# Round 4: the final bench.py once more (native legs failure-tolerant).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/r04b2_bench.log 2>&1 || exit 2
