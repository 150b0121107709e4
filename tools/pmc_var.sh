set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d gpurun_out/pmc_var1 -o run --output-format csv -- python3 tools/bench_paths.py --only str --reps 3 > gpurun_out/pmc_var1.log 2>&1 || exit 2
