#!/usr/bin/env bash
# A/B of the placement threshold: default 6100 vs 6260, alternating, main leg + shapes only
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L="--steps 10 --warmup 3 --cpu-baseline 0 --host-path 0 --alloc-probe 0 --c5-leg 0 --c5-bytes 0 --bytes-path 0 --pooled 0 --ceilings 0"
for rep in 1 2 3; do
  for thr in 6100 6260; do
    echo "=== rep $rep thr $thr" | tee -a gpurun_out/placeab.log
    SLIME_RS_PLACEMENT_MIN_GBS=$thr timeout -k 10 300 python bench.py $L > gpurun_out/placeab_${rep}_${thr}.log 2>&1 || exit 1
  done
done
