# Round 4: phase clock of the multi-string record-tile unpack, look-back vs tile table.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SRPC_GPU_LIB=build_ab/ph.so timeout -k 10 200 python -u tools/var_phases.py --case two_str --tiled > gpurun_out/r04v2_phases.log 2>&1 || exit 2
SRPC_GPU_LIB=build_ab/ph.so timeout -k 10 200 python -u tools/var_phases.py --case two_str >> gpurun_out/r04v2_phases.log 2>&1 || exit 3
