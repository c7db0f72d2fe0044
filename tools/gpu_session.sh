#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, microbenchmarks, bench, rocprofv3.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_session.sh [steps...]
#   steps: tests smoke micro bench prof pmc   (default: all but pmc)
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124 or
# a signal) ends the session immediately.  A plain test failure (exit 1) is
# recorded and the session continues.
# NOTE (round 6): the A/B environment variables some steps set -- SLIME_RS_QUEUE, SLIME_RS_PIPE,
# SLIME_RS_GRID_TARGET, SLIME_RS_SEGMENTS -- were removed from the library in round 5 and now do
# nothing: re-running such a step does not reproduce its A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=("$@")
[ ${#STEPS[@]} -eq 0 ] && STEPS=(tests smoke micro bench prof)

run() {  # run <name> <limit-seconds> <command...>
  local name=$1 lim=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/session.log"
  tail -n 25 "$OUT/$name.log"
  # A failed parity run (a wrong or faulting kernel) ends the session too:
  # nothing after it should run on a kernel that is not known to be right.
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ "$name" = pytest_gpu ] || grep -q "illegal memory access" "$OUT/$name.log"; }; then
    echo "!!! $name ended with rc=$rc: stopping the session" | tee -a "$OUT/session.log"
    exit $rc
  fi
  return 0
}

has() { for s in "${STEPS[@]}"; do [ "$s" = "$1" ] && return 0; done; return 1; }

rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > "$OUT/device.txt" || true
timeout 30 amd-smi static -g 0 2>/dev/null | grep -E "MODEL_NUMBER|PRODUCT_NAME|VENDOR: |OAM_ID" >> "$OUT/device.txt" || true
nproc > "$OUT/host.txt"; grep -m1 "model name" /proc/cpuinfo >> "$OUT/host.txt" || true

has tests && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has micro && run micro 600 python tools/microbench.py
has bench && run bench 600 python bench.py
if has bench3; then
  for i in 1 2 3; do run bench_rep$i 300 python bench.py --cpu-baseline 0; done
fi
has prof && run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --cpu-baseline 0
has ubench && run ubench 600 python tools/ubench.py
has variants && run variants 600 python tools/apply_variants.py
if has placement; then
  for d in 0 1; do for sep in 0 1; do
    run var_d${d}_s${sep} 300 python tools/apply_variants.py --decode $d --separate $sep --variants 8,6 --blocks 256,512,1024
  done; done
fi
if has rot; then
  for pad in 0 4160; do
    run rot_enc_inpl_p$pad 300 python tools/apply_variants.py --separate 0 --pad $pad --variants 8,11,6,12 --blocks 256,512,1024
    run rot_enc_sep_p$pad 300 python tools/apply_variants.py --separate 1 --pad $pad --variants 8,11,6,12 --blocks 256,512,1024
    run rot_dec_sep_p$pad 300 python tools/apply_variants.py --decode 1 --separate 1 --pad $pad --variants 8,11,6,12 --blocks 256,512,1024
  done
  run rot_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --variants 8,11 --blocks 256,512,1024
  run rot_c5dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --decode 1 --variants 8,11 --blocks 256,512,1024
fi
if has sep; then
  for r in 1 2; do
  for sep in 0 1 2; do
    run sep_enc_${sep}_r$r 300 python tools/apply_variants.py --separate $sep --variants 8 --blocks 256,512
    run sep_dec_${sep}_r$r 300 python tools/apply_variants.py --decode 1 --separate $sep --variants 8 --blocks 256,512
  done; done
fi
if has variants2; then
  run var_enc 300 python tools/apply_variants.py
  run var_dec 300 python tools/apply_variants.py --decode 1
  run var_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16
  run var_c5dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --decode 1
  run var_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --blocks 256,512,1024,2048
fi
if has grid; then
  for g in 1024 4096 8192; do
    run bench_grid$g 300 env SLIME_RS_GRID_TARGET=$g python bench.py --steps 5 --cpu-baseline 0
  done
fi
has placeprobe && run placeprobe 600 python tools/placement_probe.py
has placemap && run placemap 600 python tools/placement_map.py
if has placepmc; then  # counters on fast vs slow buffers (kernel-trace durations classify each dispatch)
  i=0
  for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
             "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum" \
             "TCC_EA0_WRREQ" \
             "TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum TCC_WRITEBACK_sum" \
             "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum"; do
    i=$((i+1))
    run ppmc$i 240 rocprofv3 --pmc $set --kernel-trace -d "$OUT/ppmc$i" -o run --output-format csv -- \
      python3 tools/placement_probe.py --reps 2
  done
fi
if has gridk; then  # block budget per k (SLIME_RS_GRID_TARGET), device-resident encode+decode
  for kn in "8 12 256 128 0,1,2,3" "10 14 1024 16 0,1,2,3" "12 16 1024 16 0,1,2,3" "16 20 1024 16 0,1,2,3" "4 6 64 32 0,1"; do
    set -- $kn
    for g in 256 512 1024; do
      run gridk_${1}_${2}_g$g 300 env SLIME_RS_GRID_TARGET=$g python bench.py --need $1 --total $2 --object-mib $3 \
        --objects $4 --erase $5 --steps 5 --warmup 1 --cpu-baseline 0 --bytes-path 0 --host-path 0
    done
  done
fi
if has shapes; then  # BASELINE shapes through bench.py (device-resident, encode + repair)
  run shape_c3_64mib_shards 300 python bench.py --object-mib 512 --objects 64 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run shape_c2 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run shape_c5_all64 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 64 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run shape_c4_mixed 300 python bench.py --erase 0,3,8,11 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
fi
if has segs; then  # column segments per object (more independent stripe streams for small batches)
  run segs_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 8 --blocks 512,1024 --nseg 1,2,4,8
  run segs_c2dec 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --decode 1 --variants 8 --blocks 512,1024 --nseg 1,2,4,8
  run segs_c3 300 python tools/apply_variants.py --variants 8 --blocks 512,1024 --nseg 1,2,4
  run segs_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --variants 8 --blocks 256,512 --nseg 1,2,4,8
  run segs_c5dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --decode 1 --variants 8 --blocks 256,512 --nseg 1,2,4,8
fi
if has shapes2; then  # product defaults vs forced segment counts on the small-batch shapes
  for sg in 0 1 4 16; do
    run sh2_c2_s$sg 300 env SLIME_RS_SEGMENTS=$sg python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
    run sh2_c5_s$sg 300 env SLIME_RS_SEGMENTS=$sg python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  done
  run sh2_c3 300 python bench.py --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run sh2_c5_all64 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 64 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
fi
if has slowsegs; then  # on a slow allocation (if the box has one): do more independent streams help?
  run slowsegs_enc 400 python tools/apply_variants.py --hunt slow --variants 8,11 --blocks 512,1024 --nseg 1,2,4,8,16
  run slowsegs_dec 400 python tools/apply_variants.py --hunt slow --decode 1 --separate 0 --variants 8 --blocks 512,1024 --nseg 1,2,4,8,16
fi
has mall && run mall 300 bash -c "make ubench >/dev/null && python tools/mall_probe.py"
if has offsets; then  # batch base offset inside one allocation; once plain, once under the profiler
  run offsets_plain 300 python tools/offset_probe.py
  run offsets_prof 300 rocprofv3 --kernel-trace -d "$OUT/offsets_prof" -o run --output-format csv -- python3 tools/offset_probe.py
fi
if has widek; then  # k > 16: the generic one-column kernel
  run widek_16_20 300 python bench.py --need 16 --total 20 --object-mib 256 --objects 32 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run widek_20_24 300 python bench.py --need 20 --total 24 --object-mib 256 --objects 32 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run widek_32_40 300 python bench.py --need 32 --total 40 --object-mib 256 --objects 32 --erase 0,1,2,3,4,5,6,7 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run widek_64_80 300 python bench.py --need 64 --total 80 --object-mib 256 --objects 16 --erase 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
fi
if has ranks2; then  # the N > 1 path end to end: 2 ranks sharing this box's one GPU
  run ranks2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --objects 64
fi
if has widebytes; then  # fused byte path at need > 16
  run widebytes_20_24 300 python bench.py --need 20 --total 24 --object-mib 256 --objects 32 --steps 3 --cpu-baseline 0 --host-path 0
  run widebytes_40_56 300 python bench.py --need 40 --total 56 --object-mib 256 --objects 16 --erase 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 --steps 3 --cpu-baseline 0 --host-path 0
fi
if has sizes; then  # object size vs k: is 10/14 slower because of k or because of 1 GiB objects?
  run sizes_10_14_256m 300 python bench.py --need 10 --total 14 --object-mib 256 --objects 128 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run sizes_8_12_1g 300 python bench.py --need 8 --total 12 --object-mib 1024 --objects 32 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run sizes_10_14_1g 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 32 --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
  run sizes_8_12_256m 300 python bench.py --steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0
fi
if has clocks; then  # box state under sustained load: which clocks/limits differ on slow-placement boxes?
  ( timeout -k 5 40 python tools/sustained.py --seconds 12 --idle 1 > "$OUT/clocks_load.log" 2>&1 ) &
  LOADPID=$!
  sleep 8
  timeout -k 5 30 rocm-smi --showclocks --showperflevel --showpower --showmaxpower --showtemp --showmemuse > "$OUT/clocks_smi_load.log" 2>&1
  timeout -k 5 40 amd-smi metric -g 0 > "$OUT/clocks_amdsmi_load.log" 2>&1
  wait $LOADPID
  timeout -k 5 40 amd-smi static -g 0 > "$OUT/clocks_amdsmi_static.log" 2>&1
  timeout -k 5 40 amd-smi partition > "$OUT/clocks_partition.log" 2>&1 || true
  echo "=== clocks done" | tee -a "$OUT/session.log"
fi
if has slowsweep; then  # kernel knobs on whatever box this is (the log names its placement mode)
  run sweep_enc 400 python tools/apply_variants.py --variants 8,2,6,11 --blocks 256,512,1024,2048 --nseg 1,4,16
  run sweep_dec 400 python tools/apply_variants.py --decode 1 --separate 0 --variants 8,2,6,11 --blocks 256,512,1024,2048 --nseg 1,4,16
fi
if has bytesshapes; then  # fused byte path on small and large batches
  run bshape_c2 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --steps 5 --cpu-baseline 0 --host-path 0
  run bshape_c5 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 --steps 3 --cpu-baseline 0 --host-path 0
fi
if has c5segs; then  # C5 (10/14, 64 x 1 GiB) with forced segment counts
  for sg in 0 2 8 16; do
    run c5segs_s$sg 300 env SLIME_RS_SEGMENTS=$sg python bench.py --need 10 --total 14 --object-mib 1024 --objects 64 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0
  done
fi
if has k10; then  # why is 10/14 slower than 8/12?  unroll x blocks x segments at C5 shape (64 x 1 GiB -> 32 here)
  run k10_enc 400 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 8,10,6 --blocks 256,384,512,768 --nseg 1,4
  run k8_1g_enc 400 python tools/apply_variants.py --need 8 --total 12 --mib 1024 --nobj 32 --variants 8,10,6 --blocks 256,512 --nseg 1,4
fi
has allocvar && run allocvar 600 python tools/alloc_variance.py --rounds 8
has contig && run contig 600 python tools/alloc_contig.py --rounds 6
has hbmmap && run hbmmap 600 python tools/hbm_map.py
has bytesvar && run bytesvar 600 python tools/bytes_variants.py
if has bvs; then
  for i in 1 2 3; do run bvs$i 300 python tools/bytes_vs_symbols.py; done
fi
if has bvspmc; then
  run bvs_pmc1 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d "$OUT/bvs_pmc1" -o p --output-format csv -- python3 tools/bytes_vs_symbols.py
  run bvs_pmc2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/bvs_pmc2" -o p --output-format csv -- python3 tools/bytes_vs_symbols.py
fi
if has hunt3; then
  P="0,65536,262144,524288,1048576,2097152,4194304"
  run hunt3_slow 600 python tools/apply_variants.py --hunt slow --variants 8 --blocks 512 --inflight 0 --pad $P
  run hunt3_fast 600 python tools/apply_variants.py --hunt fast --variants 8 --blocks 512 --inflight 0 --pad $P
fi
if has hunt2; then
  run hunt2_slow 600 python tools/apply_variants.py --hunt slow --variants 8 --blocks 256,512,1024 --inflight 1,2,4,8,128 --pad 0
  run hunt2_fast 600 python tools/apply_variants.py --hunt fast --variants 8 --blocks 256,512,1024 --inflight 1,2,4,8,128 --pad 0
fi
if has hunt; then
  run hunt_slow 600 python tools/apply_variants.py --hunt slow --variants 0,1,2,4,8,11 --blocks 256,512,1024 --inflight 0,16 --pad 0,64,4160
  run hunt_fast 600 python tools/apply_variants.py --hunt fast --variants 0,1,2,4,8,11 --blocks 256,512,1024 --inflight 0,16 --pad 0,64,4160
fi
if has sustained; then
  run sustained1 300 python tools/sustained.py --seconds 8 --idle 2
  run smi 60 rocm-smi --showclocks --showperflevel --showpower
  run sustained2 300 python tools/sustained.py --seconds 8 --idle 0
fi
has hostpipe && run hostpipe 900 python tools/host_pipe.py
has counters && run counters 120 rocprofv3 -L
has hashprobe && run hashprobe 600 bash -c "make hashprobe >/dev/null && python tools/hash_probe.py"
if has pmcplace; then  # counters that may separate the fast/slow placement modes
  run place_plain 300 python tools/placement_pmc.py
  i=0
  for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" \
             "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
             "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" \
             "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum" \
             "TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum" \
             "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum" \
             "TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum"; do
    i=$((i+1))
    run place_pmc$i 300 rocprofv3 --pmc $set --kernel-trace -d "$OUT/place_pmc$i" -o run --output-format csv -- \
      python3 tools/placement_pmc.py
  done
fi
if has pmc; then
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o bench --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o bench --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0
fi
if has pipe; then  # software-pipelined apply kernel (variants 13-15) against the product forms
  V=8,10,6,13,14,15
  run pipe_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants $V --blocks 256,512,768,1024 --nseg 8
  run pipe_c5dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --decode 1 --separate 0 --variants $V --blocks 256,512,768,1024 --nseg 8
  run pipe_c3 300 python tools/apply_variants.py --variants $V --blocks 256,512,768,1024 --nseg 2
  run pipe_c3dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants $V --blocks 256,512,768,1024 --nseg 2
  run pipe_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants $V --blocks 256,512,768,1024 --nseg 8
fi
if has pipek; then  # the pipelined kernel at the other k <= 16 (product: U4 <= 10, U2 above)
  V=8,6,13,14,15
  run pipek_4_6 300 python tools/apply_variants.py --need 4 --total 6 --mib 256 --nobj 128 --variants $V --blocks 256,512,1024 --nseg 2
  run pipek_6_9 300 python tools/apply_variants.py --need 6 --total 9 --mib 256 --nobj 128 --variants $V --blocks 256,512,1024 --nseg 2
  run pipek_8_12 300 python tools/apply_variants.py --need 8 --total 12 --mib 256 --nobj 128 --variants $V --blocks 256,512,1024 --nseg 2
  run pipek_12_16 300 python tools/apply_variants.py --need 12 --total 16 --mib 1024 --nobj 16 --variants $V --blocks 256,512,1024 --nseg 16
  run pipek_16_20 300 python tools/apply_variants.py --need 16 --total 20 --mib 1024 --nobj 16 --variants $V --blocks 256,512,1024 --nseg 16
fi
if has pipeab; then  # product dispatch with and without the pipelined kernel, BASELINE shapes, same box
  B="--steps 5 --cpu-baseline 0 --bytes-path 0 --host-path 0"
  for pp in 1 0; do
    run ab_c3_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py $B
    run ab_c2_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 $B
    run ab_c5_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --need 10 --total 14 --object-mib 1024 --objects 32 $B
    run ab_64mib_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --object-mib 512 --objects 64 $B
  done
fi
if has bytesab; then  # byte kernels with and without the pipeline (both legs of bench.py switch)
  B="--steps 5 --cpu-baseline 0 --host-path 0"
  for pp in 1 0; do
    run bab_c3_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py $B
    run bab_c2_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 $B
    run bab_c5_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 $B
  done
fi
if has c5geo; then  # 10/14 geometry with the pipelined kernel: segments x segments-in-flight x blocks
  run c5geo_enc 400 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 14,15 --blocks 256,384,512 --nseg 2,4,8 --inflight 0,64,128 --rounds 2
  run c5geo_c3 400 python tools/apply_variants.py --variants 14,15 --blocks 256,384,512 --nseg 1,2,4 --inflight 0,64,128 --rounds 2
fi
if has wideab; then  # k > 16: pipelined wide kernel vs the chunked one, and its block budget
  B="--object-mib 256 --steps 3 --cpu-baseline 0 --bytes-path 0 --host-path 0"
  for cfg in "20 24 32 0,1,2,3" "32 40 32 0,1,2,3,4,5,6,7" "64 80 16 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15"; do
    set -- $cfg
    run wab_$1_$2_p1 300 env SLIME_RS_PIPE=1 python bench.py --need $1 --total $2 --objects $3 --erase $4 $B
    run wab_$1_$2_p0 300 env SLIME_RS_PIPE=0 python bench.py --need $1 --total $2 --objects $3 --erase $4 $B
    run wab_$1_$2_p1_g256 300 env SLIME_RS_PIPE=1 SLIME_RS_GRID_TARGET=256 python bench.py --need $1 --total $2 --objects $3 --erase $4 $B
    run wab_$1_$2_p1_g1024 300 env SLIME_RS_PIPE=1 SLIME_RS_GRID_TARGET=1024 python bench.py --need $1 --total $2 --objects $3 --erase $4 $B
  done
fi
if has widebytesab; then  # need > 16 byte path: pipelined wide decode vs the chunked one
  B="--object-mib 256 --steps 3 --cpu-baseline 0 --host-path 0"
  for pp in 1 0; do
    run wbab_20_24_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --need 20 --total 24 --objects 32 $B
    run wbab_40_56_p$pp 300 env SLIME_RS_PIPE=$pp python bench.py --need 40 --total 56 --objects 16 --erase 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 $B
  done
fi
if has mathcost; then  # pipelined kernel with XOR stand-in math: is the field math on the critical path?
  run mc_c3 300 python tools/apply_variants.py --variants 15,16,14,17 --blocks 256,512 --nseg 2
  run mc_c3dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15,16 --blocks 256,512 --nseg 2
  run mc_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,16,14,17 --blocks 256,512 --nseg 8
fi
if has rwsplit; then  # the product walk split into its read-only and write-only halves
  run rw_c3 300 python tools/apply_variants.py --variants 15,16,18,19 --blocks 256,512 --nseg 2
  run rw_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,16,18,19 --blocks 256,512 --nseg 8
fi
if has linealign; then  # 10/14 (L = 26843546: shard bases 8 B off 16 B) with shard strides padded to 16/64/128/256 B
  run la_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,18,19 --blocks 256 --nseg 8 --pad 0,2,6,22,38
  run la_c5dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 8 --pad 0,2,38
fi
if has pow2; then  # is 10/14 slow because of k, or because its shards are not power-of-two sized?
  run p2_c3 300 python tools/apply_variants.py --variants 15,18,19 --blocks 256 --nseg 2
  run p2_k8_25m 300 python tools/apply_variants.py --need 8 --total 12 --mib 800 --nobj 128 --variants 15,18,19 --blocks 256 --nseg 2
  run p2_k10_128m 300 python tools/apply_variants.py --need 10 --total 14 --mib 1280 --nobj 32 --variants 15,18,19 --blocks 256 --nseg 8
  run p2_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,18,19 --blocks 256 --nseg 8
fi
if has segalign; then  # column segments rounded to whole 1 KiB: 10/14 (odd splits) before/after, padded strides
  run sa_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,18,19 --blocks 256 --nseg 1,2,4,8 --pad 0,2,38
  run sa_c5dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 8 --pad 0,38
  run sa_c3 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 2
  B="--cpu-baseline 0 --host-path 0"
  run sa_bench_c5_64 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 64 --steps 3 $B
  run sa_bench_c5_32 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 32 --steps 5 $B
  run sa_bench_c10_256 300 python bench.py --need 10 --total 14 --object-mib 256 --objects 128 --steps 5 $B
  run sa_bench_c2 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --steps 5 $B
  run sa_bench_c3 300 python bench.py --steps 5 $B
fi
if has shardalign; then  # bench with line-aligned shard strides (default) vs packed (--shard-align 1)
  B="--cpu-baseline 0 --host-path 0 --bytes-path 0"
  for al in 64 1; do
    run al${al}_c5_64 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 64 --steps 3 --shard-align $al $B
    run al${al}_c10_256 300 python bench.py --need 10 --total 14 --object-mib 256 --objects 128 --steps 5 --shard-align $al $B
  done
  run al64_c3 300 python bench.py --steps 5 $B
  run al64_c2 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --steps 5 $B
  run al64_c4mixed 300 python bench.py --erase 0,3,8,11 --steps 5 $B
  run al64_c3_sep 300 python bench.py --decode-dst separate --steps 5 $B
fi
if has pipe4; then  # 4 KiB tiles per wave per stream (pipe U4) against the product U3, C3 and C5
  run p4_c3 300 python tools/apply_variants.py --variants 15,20 --blocks 256,512 --nseg 2 --rounds 4
  run p4_c3dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15,20 --blocks 256 --nseg 2 --rounds 4
  run p4_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,20 --blocks 256 --nseg 8 --pad 38 --rounds 4
fi
if has xcd; then  # XCD-grouped work order against the product's round-robin one
  run xcd_c3 300 python tools/apply_variants.py --variants 15,21 --blocks 256 --nseg 2 --rounds 5
  run xcd_c3dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15,21 --blocks 256 --nseg 2 --rounds 5
  run xcd_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 32 --variants 15,21 --blocks 256 --nseg 8 --pad 38 --rounds 5
fi
if has slowtile; then  # tile size per wave on a slow-placement allocation (if the box gives one)
  run st_slow 400 python tools/apply_variants.py --hunt slow --variants 15,20,14,13 --blocks 256,512 --nseg 2,8 --rounds 3
fi
if has slowrw; then  # read-only / write-only halves of the walk on slow vs fast allocations of one box
  run srw_slow 400 python tools/apply_variants.py --hunt slow --variants 15,18,19 --blocks 256 --nseg 2 --rounds 3
  run srw_fast 400 python tools/apply_variants.py --hunt fast --variants 15,18,19 --blocks 256 --nseg 2 --rounds 3
fi
if has slowpad; then  # shard-stride skew (256 B-aligned pads) on slow vs fast allocations, pipelined product kernel
  P="0,64,1024,16384,262208,1048640,4194368"
  run spad_slow 500 python tools/apply_variants.py --hunt slow --variants 15 --blocks 256 --nseg 2 --rounds 2 --pad $P
  run spad_fast 500 python tools/apply_variants.py --hunt fast --variants 15 --blocks 256 --nseg 2 --rounds 2 --pad $P
fi
echo "=== session done" | tee -a "$OUT/session.log"
