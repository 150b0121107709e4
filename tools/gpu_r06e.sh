bash tools/gpu_prof_rows.sh "r05 now" "string_0-16_8M multiple_primitives_zeros_4M zh4_straddle_heavy_long_256K zh4_straddle_heavy_4M" r06e
