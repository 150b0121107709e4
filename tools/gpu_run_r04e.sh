# Round 4: counters of the TILE unpack on the enveloped rows and of the AoS
# kernels (HBM bytes: the in-place unpack's read-for-ownership), one MI355X.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 bash tools/pmc_paths.sh r04_tile add_request_58B two_numbers_response || exit 1
timeout -k 10 900 bash tools/pmc_paths.sh r04_aos aos || exit 2
