# Counters for the kernels of tools/bench_paths.py cases (one MI355X): kernel
# durations, HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes), and SQ
# issue / stall / LDS counters, one --pmc pass per group (each within the
# per-block limits: <= 8 SQ, <= 4 TCC counters).  Summarised per kernel into
# gpurun_out/pmc_paths_<tag>.txt by tools/pmc_paths_table.py.
# usage (through gpurun): bash tools/pmc_paths.sh <tag> <filter> [<filter> ...]
# (PMC_TOOL=stream_bench.py PMC_ARGS='--single 2': the stream decode cases)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
for F in "$@"; do
  D=gpurun_out/pmc_${TAG}_$F
  RUN="python3 tools/${PMC_TOOL:-bench_paths.py} --only $F --reps 3 $PMC_ARGS"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/stats -o run --output-format csv -- $RUN > $D.stats.log 2>&1 || exit 1
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $D/p$i -o run --output-format csv -- $RUN > $D.p$i.log 2>&1 || exit $((10+i))
  done
  python3 tools/pmc_paths_table.py $D > gpurun_out/pmc_paths_${TAG}_$F.txt || exit 9
done
