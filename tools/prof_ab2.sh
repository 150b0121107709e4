# rocprofv3 kernel tables of build_ab/{base,new}.so on one bench_paths filter.
# usage: bash tools/prof_ab2.sh FILTER  -> gpurun_out/table_{base,new}.txt
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F=${1:-str}
for v in base new; do
  SRPC_GPU_LIB=build_ab/$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_$v -o run --output-format csv -- python3 tools/bench_paths.py --only "$F" --reps 10 > gpurun_out/prof_$v.log 2>&1 || exit 1
  python3 tools/kernel_table.py $(ls gpurun_out/prof_$v/*kernel_trace.csv | head -1) > gpurun_out/table_$v.txt || exit 2
done
