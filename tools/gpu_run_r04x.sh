# Round 4: decode phases with the speculation's segments per block.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SRPC_GPU_LIB=build_sx/sx_phases.so timeout -k 10 300 python -u tools/sx_phases.py > gpurun_out/r04x_phases.log 2>&1 || exit 2
