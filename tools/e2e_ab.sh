#!/bin/bash
# Config-5 server A/B on one box: the pure-square 1M stream at 64K and 256K
# frames per batch, two batches in flight (default) vs one (SRPC_SERVER_SLOTS=1),
# interleaved, ROUNDS rounds.  Usage: tools/e2e_ab.sh LOG [ROUNDS]
log=$1; rounds=${2:-3}
: > "$log"
port=18500
for r in $(seq 1 "$rounds"); do
  for slots in 2 1; do
    for b in 65536 262144; do
      port=$((port + 1))
      echo "## slots=$slots batch=$b round=$r" >> "$log"
      SRPC_SERVER_SLOTS=$slots timeout -k 10 120 ./tools/e2e_square --mode gpu --n 1048576 --batch $b --port $port >> "$log" 2>&1 || exit 2
    done
  done
done
