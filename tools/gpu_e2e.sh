#!/bin/bash
# Calculator e2e over loopback (BASELINE configs[4]) on the GPU box: the pure
# square stream at three batch sizes, the scalar CPU server, and mixed traffic
# (a poisoned frame at index 0, 1 % and 10 % divide requests the GPU server
# does not have, four methods on the GPU).  Usage: tools/gpu_e2e.sh [log]
set -o pipefail
mkdir -p gpurun_out
log=${1:-gpurun_out/e2e.log}
: > "$log"
E=./tools/e2e_square
N=1048576
for b in 65536 262144 1048576; do
  timeout -k 10 120 $E --mode gpu --n $N --batch $b --port 18400 >> "$log" 2>&1 || exit 2
done
timeout -k 10 120 $E --mode cpu --n $N --port 18401 >> "$log" 2>&1 || exit 3
timeout -k 10 120 $E --mode gpu --n $N --batch 262144 --port 18402 --poison 0 >> "$log" 2>&1 || exit 4
timeout -k 10 120 $E --mode gpu --n $N --batch 262144 --port 18403 --foreign 0.01 >> "$log" 2>&1 || exit 5
timeout -k 10 120 $E --mode gpu --n $N --batch 262144 --port 18404 --foreign 0.10 >> "$log" 2>&1 || exit 6
timeout -k 10 120 $E --mode gpu --n $N --batch 262144 --port 18405 --mix 0.5 --gpu-methods all >> "$log" 2>&1 || exit 7
timeout -k 10 120 $E --mode cpu --n $N --port 18406 --mix 0.5 >> "$log" 2>&1 || exit 8
