# Round 4 final evidence on the final tree (tools/gpu_final.sh: full -m gpu, smoke, bench, rocprof, PMC, paths, streams).
bash tools/gpu_final.sh r04
