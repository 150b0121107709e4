# SQ counters for the VAR-path kernels (one MI355X), one --pmc pass per group.
# usage (through gpurun): bash tools/pmc_var.sh [bench_paths filter]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F=${1:-multiple}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_var$i -o run --output-format csv -- python3 tools/bench_paths.py --only "$F" --reps 3 > gpurun_out/pmc_var$i.log 2>&1 || exit $i
done
python3 tools/pmc_table.py gpurun_out/pmc_var1 gpurun_out/pmc_var2 gpurun_out/pmc_var3 > gpurun_out/pmc_var_table.txt || exit 9
