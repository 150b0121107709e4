#!/bin/bash
# Interleaved A/B of library builds (build_ab/<name>.so, tools/ab_build.py) on
# stream_bench rows: ROUNDS rounds, each running every variant on every row.
#   bash tools/ab_variants.sh "v1 v2 ..." "row1 row2 ..." [ROUNDS] [REPS]
variants=$1; rows=$2; rounds=${3:-2}; reps=${4:-5}
for r in $(seq 1 "$rounds"); do
  for v in $variants; do
    for row in $rows; do
      echo "## $v round $r"
      SRPC_GPU_LIB=build_ab/$v.so timeout -k 10 120 python -u tools/stream_bench.py --reps "$reps" --only "$row" || exit 1
    done
  done
done
