#!/usr/bin/env bash
# C2 (4/6, 32 x 64 MiB) as the main batch in fresh processes: its own 3 GiB buffer
# from 2 MiB chunks (the default) vs 1 GiB chunks, alternating, legs off.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L="--preset c2 --steps 20 --warmup 5 --cpu-baseline 0 --host-path 0 --alloc-probe 0 --c5-leg 0 --c5-bytes 0 --bytes-path 0 --pooled 0 --ceilings 0 --shape-legs="
for rep in 1 2 3; do
  for mib in 2 1024; do
    echo "=== rep $rep chunk $mib MiB" | tee -a gpurun_out/c2place.log
    SLIME_RS_VMM_CHUNK_MIB=$mib timeout -k 10 200 python bench.py $L > gpurun_out/c2place_${rep}_${mib}.log 2>&1 || exit 1
  done
done
