#!/usr/bin/env bash
# Round-4 GPU-box session: every GPU step under its own time limit; the first
# crash/abort/timeout ends the session (nothing more runs on the GPU).
# Usage (repo root, on the box):  bash tools/gpu_r04.sh <step> [<step>...]
# NOTE (round 6): the A/B environment variables these steps set -- SLIME_RS_MFMA*, SLIME_RS_QUEUE,
# SLIME_RS_PIPE, SLIME_RS_GRID_TARGET, SLIME_RS_SEGMENTS, SLIME_RS_HOST_PIPE -- were removed from the
# library in round 5 and now do nothing: re-running a step does not reproduce its A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
NOLEGS="--cpu-baseline 0 --host-path 0 --alloc-probe 0 --c5-leg 0"

run() {  # run <name> <limit-seconds> <command...>
  local name=$1 lim=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/session.log"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then
    echo "!!! $name ended with rc=$rc: stopping the session" | tee -a "$OUT/session.log"
    exit $rc
  fi
}

nproc > "$OUT/host.txt"; grep -m1 "model name" /proc/cpuinfo >> "$OUT/host.txt" || true
for step in "$@"; do
  case "$step" in
    tests_alloc) run pytest_alloc 400 python -u -m pytest tests/test_gpu_device_alloc.py -x -q --timeout 200 --timeout-method thread ;;
    tests_host) run pytest_host 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "map or recover or host or unchanged or RecoverData or reconstruct" ;;
    kfd) run kfd 120 python -c "import sys; sys.argv=['bench.py']; sys.path.insert(0, '.'); import bench, torch; print('kfd_gpus', bench.kfd_gpus(), 'torch', torch.cuda.device_count())" ;;
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    tests_sched) run pytest_sched 400 python -u -m pytest tests/test_gpu_schedule.py -x -v --timeout 120 --timeout-method thread ;;
    tests_full) run pytest_full 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench20) run bench20 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    profdrv) run profdrv 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
          run prof_summary 120 sh -c "python3 tools/prof_summary.py \$(dirname \$(find $OUT/prof -name bench_kernel_trace.csv | head -1)) > $OUT/prof_summary.json" ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
            python3 bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-path 0 --bytes-path 0 --alloc-probe 0 ;;
    pmc_fetch) run pmc_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    pmc_write) run pmc_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    # byte-path kernels (object_bytes_path leg) at C3 and C5: kernel stats + traffic passes
    bprof_c3) run bprof_c3 600 rocprofv3 --kernel-trace --stats -d "$OUT/bprof_c3" -o bench --output-format csv -- \
            python3 bench.py --steps 5 --warmup 1 $NOLEGS ;;
    bprof_c5) run bprof_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/bprof_c5" -o bench --output-format csv -- \
            python3 bench.py --preset c5 --global-objects 16 --steps 5 --warmup 1 $NOLEGS ;;
    bpmc_c3) run bpmc_c3_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/bpmc_c3_fetch" -o pmc \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 $NOLEGS &&
          run bpmc_c3_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/bpmc_c3_write" -o pmc \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 $NOLEGS ;;
    bpmc_c5) run bpmc_c5_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/bpmc_c5_fetch" -o pmc \
            --output-format csv -- python3 bench.py --preset c5 --global-objects 16 --steps 3 --warmup 1 $NOLEGS &&
          run bpmc_c5_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/bpmc_c5_write" -o pmc \
            --output-format csv -- python3 bench.py --preset c5 --global-objects 16 --steps 3 --warmup 1 $NOLEGS ;;
    tests_switch) run pytest_switch 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mid_object_switch or encode_objects or write_chunks" ;;
    tests_mfma_bytes) run pytest_mfma_bytes 400 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 200 --timeout-method thread -k "byte or bytes or encode_objects or decode_objects" ;;
    mfma_tests) run pytest_mfma 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread ;;
    # wide codes: matrix-core kernel (default), its non-pipelined form, the VALU kernels
    # wide codes: matrix-core kernel forms (SLIME_RS_MFMA_MODE 2 = K-step refill, default; 1 two tile
    # buffers; 0 no prefetch) against the VALU kernels (SLIME_RS_MFMA=0), same box
    wide) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          E20=$E16,16,17,18,19
          WIDE="--bytes-path 0 --steps 5 --warmup 2 $NOLEGS"
          for shp in "64 80 $E16" "48 64 $E16" "80 100 $E20" "40 48 0,1,2,3,4,5,6,7"; do
            set -- $shp
            for v in "queue:SLIME_RS_MFMA_MODE=2" "static:SLIME_RS_MFMA_QUEUE=0" "m0:SLIME_RS_MFMA_MODE=0" "valu:SLIME_RS_MFMA=0"; do
              run wide_$1_$2_${v%%:*} 300 env ${v#*:} python bench.py --need $1 --total $2 --objects 32 --erase $3 $WIDE || exit 1
            done
          done ;;
    # wide codes on the fused byte path (object_bytes_path leg), matrix cores vs VALU
    widebytes) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          WB="--steps 3 --warmup 1 $NOLEGS"
          for shp in "64 80 $E16" "80 100 $E16,16,17,18,19" "40 56 $E16"; do
            set -- $shp
            for v in "mfma:SLIME_RS_MFMA=1" "enc0:SLIME_RS_MFMA_ENC_FORM=0"; do
              run wbytes_$1_$2_${v%%:*} 300 env ${v#*:} python bench.py --need $1 --total $2 --objects 32 --erase $3 $WB || exit 1
            done
          done ;;
    # the matrix-core kernel on the BASELINE shapes (SLIME_RS_MFMA_MINK=1), symbol path only
    mink1) run mink1_c3 300 env SLIME_RS_MFMA_MINK=1 python bench.py --bytes-path 0 --steps 5 $NOLEGS &&
           run mink1_c5 300 env SLIME_RS_MFMA_MINK=1 python bench.py --preset c5 --global-objects 16 --bytes-path 0 --steps 5 $NOLEGS &&
           run mink1_c2 300 env SLIME_RS_MFMA_MINK=1 python bench.py --preset c2 --bytes-path 0 --steps 5 $NOLEGS ;;
    # kernel times of the wide byte path (64/80, 32 x 256 MiB): rocprofv3 stats
    wprof80) E20=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19
          for v in "f2:SLIME_RS_MFMA_ENC_FORM=2" "f0:SLIME_RS_MFMA_ENC_FORM=0"; do
            run wprof80_${v%%:*} 300 env ${v#*:} rocprofv3 --kernel-trace --stats -d "$OUT/wprof80_${v%%:*}" -o bench --output-format csv -- \
              python3 bench.py --need 80 --total 100 --objects 32 --erase $E20 --steps 3 --warmup 1 $NOLEGS || exit 1
            run wprof96_${v%%:*} 300 env ${v#*:} rocprofv3 --kernel-trace --stats -d "$OUT/wprof96_${v%%:*}" -o bench --output-format csv -- \
              python3 bench.py --need 96 --total 100 --objects 32 --erase 0,1,2,3 --steps 3 --warmup 1 $NOLEGS || exit 1
            run wprof48_${v%%:*} 300 env ${v#*:} rocprofv3 --kernel-trace --stats -d "$OUT/wprof48_${v%%:*}" -o bench --output-format csv -- \
              python3 bench.py --need 48 --total 64 --objects 32 --erase 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 --steps 3 --warmup 1 $NOLEGS || exit 1
          done ;;
    wprof) run wprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/wprof" -o bench --output-format csv -- \
             python3 bench.py --need 64 --total 80 --objects 32 --erase 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 --steps 3 --warmup 1 $NOLEGS ;;
    # C2 and buffer placement: the default (2 MiB chunks, unprobed below 16 GiB), probed, hipMalloc
    c2place) run c2p_default 300 python bench.py --preset c2 --bytes-path 0 --steps 10 $NOLEGS &&
             run c2p_probe1 300 env SLIME_RS_PLACEMENT_PROBE_GIB=1 python bench.py --preset c2 --bytes-path 0 --steps 10 $NOLEGS &&
             run c2p_torch 300 python bench.py --preset c2 --allocator torch --bytes-path 0 --steps 10 $NOLEGS &&
             run c2p_default2 300 python bench.py --preset c2 --bytes-path 0 --steps 10 $NOLEGS ;;
    # matrix-core kernel geometry: column segments per object (window per shard) x grid
    mfmageo) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          G="--bytes-path 0 --steps 5 --warmup 2 $NOLEGS"
          for sg in 1 2 4 8 16; do
            run mgeo_6480_s$sg 300 env SLIME_RS_SEGMENTS=$sg python bench.py --need 64 --total 80 --objects 32 --erase $E16 $G || exit 1
          done
          run mgeo_80100_g768 300 env SLIME_RS_GRID_TARGET=768 python bench.py --need 80 --total 100 --objects 32 --erase $E16,16,17,18,19 $G || exit 1
          for sg in 1 2 4; do
            run mgeo_6480_s${sg}_g1024 300 env SLIME_RS_SEGMENTS=$sg SLIME_RS_GRID_TARGET=1024 python bench.py --need 64 --total 80 --objects 32 --erase $E16 $G || exit 1
            run mgeo_80100_s$sg 300 env SLIME_RS_SEGMENTS=$sg python bench.py --need 80 --total 100 --objects 32 --erase $E16,16,17,18,19 $G || exit 1
          done ;;
    # 17 <= k <= 32: matrix cores (SLIME_RS_MFMA_MINK=17) vs the VALU k-template kernels
    mfmak32) G="--bytes-path 0 --steps 5 --warmup 2 $NOLEGS"
          for shp in "32 40 0,1,2,3,4,5,6,7" "24 32 0,1,2,3,4,5,6,7" "20 24 0,1,2,3" "17 20 0,1,2"; do
            set -- $shp
            run mk32_$1_$2_mfma 300 env SLIME_RS_MFMA_MINK=17 python bench.py --need $1 --total $2 --objects 32 --erase $3 $G || exit 1
            run mk32_$1_$2_valu 300 python bench.py --need $1 --total $2 --objects 32 --erase $3 $G || exit 1
          done ;;
    # HBM traffic of the matrix-core kernels (FETCH_SIZE / WRITE_SIZE passes): 64/80 with the byte leg, 40/48 symbol only
    wpmc) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          W6480="python3 bench.py --need 64 --total 80 --objects 32 --erase $E16 --steps 2 --warmup 1 $NOLEGS"
          W4048="python3 bench.py --need 40 --total 48 --objects 32 --erase 0,1,2,3,4,5,6,7 --steps 2 --warmup 1 --bytes-path 0 $NOLEGS"
          run wpmc_6480_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/wpmc_6480_fetch" -o pmc --output-format csv -- $W6480 &&
          run wpmc_6480_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/wpmc_6480_write" -o pmc --output-format csv -- $W6480 &&
          run wpmc_4048_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/wpmc_4048_fetch" -o pmc --output-format csv -- $W4048 &&
          run wpmc_4048_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/wpmc_4048_write" -o pmc --output-format csv -- $W4048 ;;
    # 17 <= need <= 32 byte path: matrix cores (product rule) vs VALU
    widebytes32) WB="--steps 3 --warmup 1 $NOLEGS"
          for shp in "32 40 0,1,2,3,4,5,6,7" "28 36 0,1,2,3,4,5,6,7" "24 32 0,1,2,3,4,5,6,7"; do
            set -- $shp
            for v in "mfma:SLIME_RS_MFMA=1" "valu:SLIME_RS_MFMA=0"; do
              run wb32_$1_$2_${v%%:*} 300 env ${v#*:} python bench.py --need $1 --total $2 --objects 32 --erase $3 $WB || exit 1
            done
          done ;;
    g768) E20=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19
          run g768_80100 300 env SLIME_RS_GRID_TARGET=768 python bench.py --need 80 --total 100 --objects 32 --erase $E20 --bytes-path 0 --steps 5 --warmup 2 $NOLEGS &&
          run g512_80100 300 python bench.py --need 80 --total 100 --objects 32 --erase $E20 --bytes-path 0 --steps 5 --warmup 2 $NOLEGS ;;
    # shard strides off the power-of-two grid (--shard-align 192: C3 2^23 -> 2^23 + 128 symbols)
    sstride) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          S="--bytes-path 0 --steps 5 --warmup 2 $NOLEGS"
          run ss_c3_64 300 python bench.py $S &&
          run ss_c3_192 300 python bench.py --shard-align 192 $S &&
          run ss_c3_320 300 python bench.py --shard-align 320 $S &&
          run ss_c2_64 300 python bench.py --preset c2 $S &&
          run ss_c2_192 300 python bench.py --preset c2 --shard-align 192 $S &&
          run ss_6480_64 300 python bench.py --need 64 --total 80 --objects 32 --erase $E16 $S &&
          run ss_6480_192 300 python bench.py --need 64 --total 80 --objects 32 --erase $E16 --shard-align 192 $S &&
          run ss_c3_64b 300 python bench.py $S ;;
    # cache policy of the matrix-core kernel (SLIME_RS_MFMA_NT=<loads><stores>, 1 = non-temporal)
    mfmant) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          G="--bytes-path 0 --steps 5 --warmup 2 $NOLEGS"
          for nt in 11 01 10 00 11; do
            run mnt_6480_$nt 300 env SLIME_RS_MFMA_NT=$nt python bench.py --need 64 --total 80 --objects 32 --erase $E16 $G || exit 1
          done
          for nt in 11 01; do
            run mnt_4048_$nt 300 env SLIME_RS_MFMA_NT=$nt python bench.py --need 40 --total 48 --objects 32 --erase 0,1,2,3,4,5,6,7 $G || exit 1
          done ;;
    # SQ counters (where wave-cycles go) for the matrix-core kernel at 64/80 and the C3 VALU kernel
    sqpass) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
          SQC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"
          run sq_6480 120 timeout -s KILL 90 rocprofv3 --pmc $SQC -d "$OUT/sq_6480" -o pmc --output-format csv -- \
            python3 bench.py --need 64 --total 80 --objects 32 --erase $E16 --steps 2 --warmup 1 --bytes-path 0 $NOLEGS &&
          run sq_c3 120 timeout -s KILL 90 rocprofv3 --pmc $SQC -d "$OUT/sq_c3" -o pmc --output-format csv -- \
            python3 bench.py --steps 2 --warmup 1 --bytes-path 0 $NOLEGS ;;
    shapes) run shape_c2 300 python bench.py --preset c2 $NOLEGS &&
            run shape_c5 400 python bench.py --preset c5 --global-objects 16 $NOLEGS &&
            run shape_ns64 300 python bench.py --preset ns64 $NOLEGS --bytes-path 0 ;;
    c5_64) run c5_64 600 python bench.py --preset c5 $NOLEGS ;;
    c2tail) run c2tail 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 256 --nseg 2 --rounds 5 --queue 400802 --timed 3 ;;
    c2u) run c2u_enc 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 256,512 --nseg 2 --rounds 5 --queue 400802,400801,500801,600801,600802,800801 &&
         run c2u_dec 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --decode 1 --separate 0 --variants 13 --blocks 256,512 --nseg 2 --rounds 5 --queue 400802,400801,500801,600801,600802,800801 ;;
    hosttrace) run hosttrace 300 python tools/host_trace.py &&
               run hosttrace_2d 300 env SLIME_RS_DMA_2D=1 python tools/host_trace.py &&
               run hosttrace_b 300 python tools/host_trace.py ;;
    rehearse2) run rehearse2 400 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --objects 32 --steps 5 --warmup 1 --bytes-path 0 &&
               run rehearse2_c5 400 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --preset c5 --global-objects 8 --steps 3 --warmup 1 &&
               run rehearse2_torchrun 400 env SLIME_BENCH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --objects 32 --steps 5 --warmup 1 ;;
    placeforce) run placeforce 300 env SLIME_RS_PLACEMENT_MIN_GBS=99999 python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 --steps 20 &&
                run placeforce2 300 env SLIME_RS_PLACEMENT_MIN_GBS=99999 python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 --steps 20 ;;
    tests_cstride) run pytest_cstride 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "chunk_stride or encode_objects or decode_objects" --timeout 120 --timeout-method thread ;;
    cstride) run cstride_c3_1 400 python bench.py --chunk-align 1 $NOLEGS &&
             run cstride_c3_256 400 python bench.py --chunk-align 256 $NOLEGS &&
             run cstride_c5_1 400 python bench.py --preset c5 --global-objects 16 --chunk-align 1 $NOLEGS &&
             run cstride_c5_256 400 python bench.py --preset c5 --global-objects 16 --chunk-align 256 $NOLEGS &&
             run cstride_c2_256 400 python bench.py --preset c2 --chunk-align 256 $NOLEGS ;;
    bqv) run bqv 400 python tools/bytes_queue_variants.py --rounds 5 --blocks 256,512 ;;
    q512) run q512_enc 300 python tools/apply_variants.py --variants 13 --blocks 256,512 --nseg 1 --rounds 5 --queue 802 &&
          run q512_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 13 --blocks 256,512 --nseg 1 --rounds 5 --queue 802 ;;
    redob) run redob 400 python tools/bytes_queue_variants.py --rounds 5 --redo-blocks 256,512,1024 ;;
    c4mixed) run c4mixed 400 python bench.py --erase 0,3,8,11 $NOLEGS ;;
    c2trace) run c2trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/c2trace" -o bench --output-format csv -- \
            python3 bench.py --preset c2 --steps 20 --warmup 2 $NOLEGS --bytes-path 0 ;;
    bqv_c2) run bqv_c2 300 python tools/bytes_queue_variants.py --shapes c2 --rounds 8 --blocks 256,512 ;;
    hostsweep) for W in 16 8 4 32; do for S in 3 4 6; do
                 run hs_w${W}_s${S} 120 env SLIME_RS_OBJ_WINDOW_MIB=$W SLIME_RS_HOST_STAGES=$S python tools/host_trace.py --reps 10 || exit $?
               done; done ;;
    c5u) run c5u_enc 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --pad 38 --variants 13 --blocks 256,512 --nseg 4 --rounds 5 --queue 802,200803,200802,100806 &&
         run c5u_dec 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --pad 38 --decode 1 --separate 0 --variants 13 --blocks 256,512 --nseg 4 --rounds 5 --queue 802,200803,200802,100806 ;;
    proffull) run proffull 600 rocprofv3 --kernel-trace --stats -d "$OUT/proffull" -o bench --output-format csv -- python3 bench.py ;;
    rehearse4) run rehearse4 400 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --objects 16 --steps 5 --warmup 1 &&
               run rehearse4_c5 400 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --preset c5 --global-objects 8 --steps 3 --warmup 1 ;;
    c2blk) run c2blk_enc 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 128,192,256,320 --nseg 2 --rounds 6 --queue 400802 &&
           run c2blk_dec 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --decode 1 --separate 0 --variants 13 --blocks 128,192,256,320 --nseg 2 --rounds 6 --queue 400802 ;;
    torchrun1) run torchrun1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 ;;
    gpus2) python bench.py --gpus 2 --steps 1 --warmup 0 > "$OUT/gpus2.log" 2>&1; echo "gpus2 rc=$? (2 expected on a 1-GPU box)" | tee -a "$OUT/session.log"; tail -n 3 "$OUT/gpus2.log" ;;
    # host leg only (unchanged caller, write_chunks/reconstruct): RecoverData overlap and copy-pool size, alternated twice
    hostab) HA="--objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0"
            for rep in 1 2; do
              for v in "base:SLIME_RS_RECOVER_OVERLAP=1" "noov:SLIME_RS_RECOVER_OVERLAP=0" "t8:SLIME_RS_COPY_THREADS=8" "t8noov:SLIME_RS_COPY_THREADS=8 SLIME_RS_RECOVER_OVERLAP=0"; do
                run hostab_${v%%:*}_$rep 300 env ${v#*:} python bench.py $HA || exit 1
              done
            done ;;
    latprobe) run latprobe 200 python tools/latency_probe.py ;;
    latc) run latc 200 tools/latency_c 300 ;;
    tinyab) for rep in 1 2; do for v in 4 0; do run tiny_lat_${v}_$rep 200 env SLIME_RS_TINY_UNITS=$v tools/latency_c 200 || exit 1; done; done ;;
    directab2) for rep in 1 2; do for v in 16384 256; do run direct2_lat_${v}_$rep 200 env SLIME_RS_DIRECT_KIB=$v tools/latency_c 200 || exit 1; done; done ;;
    bigdirect) for rep in 1 2; do run bd_host_def_$rep 300 python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 && run bd_host_64_$rep 300 env SLIME_RS_OBJ_WINDOW_MIB=64 SLIME_RS_DIRECT_KIB=131072 python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 || exit 1; done ;;
    tests_knobsoff) run pytest_knobsoff 1100 env SLIME_RS_DIRECT_KIB=0 SLIME_RS_ONE_OBJECT_UNITS=0 SLIME_RS_TINY_UNITS=0 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    ssab) for rep in 1 2 3; do for v in 0 1; do run ss_lat_${v}_$rep 200 env SLIME_RS_DIRECT_STREAM_SYNC=$v tools/latency_c 300 || exit 1; done; done ;;
    winab) for rep in 1 2; do for v in 16 4 2; do run win_lat_${v}_$rep 200 env SLIME_RS_OBJ_WINDOW_MIB=$v tools/latency_c 200 || exit 1; done; done ;;
    cohab) for rep in 1 2; do for v in d 1 0; do run coh_lat_${v}_$rep 200 env SLIME_RS_PIN_COHERENT=$v tools/latency_c 200 || exit 1; done; done &&
           for v in d 1; do run coh_host_$v 300 env SLIME_RS_PIN_COHERENT=$v python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 || exit 1; done ;;
    tinyab3) for rep in 1 2 3; do for v in 1024 0; do run tiny3_lat_${v}_$rep 200 env SLIME_RS_ONE_OBJECT_UNITS=$v tools/latency_c 200 || exit 1; done; done &&
             for rep in 1 2; do for v in 1024 0; do run tiny3_host_${v}_$rep 300 env SLIME_RS_ONE_OBJECT_UNITS=$v python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 || exit 1; done; done ;;
    tinyab2) for rep in 1 2 3; do for v in 4 64 1024; do run tiny2_lat_${v}_$rep 200 env SLIME_RS_TINY_UNITS=$v tools/latency_c 200 || exit 1; done; done &&
             for rep in 1 2; do for v in 4 1024; do run tiny2_host_${v}_$rep 300 env SLIME_RS_TINY_UNITS=$v python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 || exit 1; done; done ;;
    directab) for rep in 1 2; do for v in 256 1024 4096 0; do run direct_lat_${v}_$rep 200 env SLIME_RS_DIRECT_KIB=$v tools/latency_c 200 || exit 1; done; done ;;
    tests_direct0) run pytest_host_direct0 400 env SLIME_RS_DIRECT_KIB=0 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "map or recover or host or unchanged or RecoverData or reconstruct" ;;
    tests_small) run pytest_small 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 280 --timeout-method thread -k small_calls_same ;;
    altpaths) run alt_copyengines 400 env SLIME_RS_BLIT_KIB=0 SLIME_RS_BLIT_D2H_KIB=0 SLIME_RS_DMA_2D=0 SLIME_RS_D2H_PARTS=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "map or recover or host or unchanged or RecoverData or reconstruct or write_chunks or copy_kernel_threshold" &&
              run alt_allblit 400 env SLIME_RS_BLIT_KIB=65536 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "host or reconstruct or write_chunks or copy_kernel_threshold" ;;
    spinab) for rep in 1 2; do for v in 200 0; do run spin_lat_${v}_$rep 200 env SLIME_RS_SPIN_US=$v tools/latency_c 200 &&
              run spin_conc_${v}_$rep 200 env SLIME_RS_SPIN_US=$v tools/latency_c 300 8 || exit 1; done; done ;;
    upgab) HA="--objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0"
           for rep in 1 2; do for v in 1 0; do run upg_lat_${v}_$rep 200 env SLIME_RS_UP_GROUPS=$v tools/latency_c 200 &&
             run upg_host_${v}_$rep 200 env SLIME_RS_UP_GROUPS=$v python bench.py $HA || exit 1; done; done ;;
    partsab) HA="--objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0"
             for rep in 1 2; do for v in 4 1; do run parts_lat_${v}_$rep 200 env SLIME_RS_D2H_PARTS=$v tools/latency_c 200 &&
               run parts_host_${v}_$rep 200 env SLIME_RS_D2H_PARTS=$v python bench.py $HA || exit 1; done; done ;;
    latc2) for rep in 1 2; do run latc2_$rep 200 tools/latency_c 200 || exit 1; done ;;
    c2seg) for rep in 1 2; do for sg in 0 4 8 16; do
             if [ $sg = 0 ]; then run c2seg_${sg}_$rep 200 python bench.py --preset c2 --steps 20 --warmup 3 --bytes-path 0 $NOLEGS || exit 1;
             else run c2seg_${sg}_$rep 200 env SLIME_RS_SEGMENTS=$sg python bench.py --preset c2 --steps 20 --warmup 3 --bytes-path 0 $NOLEGS || exit 1; fi; done; done ;;
    thrab) sleep 20; HA="--objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0"
           for rep in 1 2; do for t in 8 12 15; do run thr_${t}_$rep 200 env SLIME_RS_COPY_THREADS=$t python bench.py $HA || exit 1; done; done ;;
    dma2dab) sleep 20; HA="--objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0"
             for rep in 1 2; do run rc2d_off_$rep 120 python tools/rc_trace.py && run rc2d_on_$rep 120 env SLIME_RS_DMA_2D=1 python tools/rc_trace.py &&
               run host2d_off_$rep 200 python bench.py $HA && run host2d_on_$rep 200 env SLIME_RS_DMA_2D=1 python bench.py $HA || exit 1; done ;;
    rctrace) run rctrace 200 env SLIME_RS_PIPE_TRACE=1 python tools/rc_trace.py &&
             run rcprof 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/rcprof" -o rc --output-format csv -- python3 tools/rc_trace.py ;;
    hugeab) HA="--objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0"
            for rep in 1 2; do run hugeab_on_$rep 200 python bench.py $HA && run hugeab_off_$rep 200 env SLIME_RS_CODEC_HUGEPAGE=0 python bench.py $HA || exit 1; done ;;
    blitbig) for rep in 1 2; do for v in 4096 65536; do run blitbig_${v}_$rep 200 env SLIME_RS_BLIT_D2H_KIB=$v python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 &&
               run blitcp_${v}_$rep 200 env SLIME_RS_BLIT_D2H_KIB=$v python tools/cp_trace.py || exit 1; done; done ;;
    serialab) for rep in 1 2; do for v in 512 2048; do run serialab_${v}_$rep 200 env SLIME_RS_COPY_SERIAL_KIB=$v tools/latency_c 200 &&
                run cp_serial_${v}_$rep 200 env SLIME_RS_COPY_SERIAL_KIB=$v python tools/cp_trace.py || exit 1; done; done ;;
    cptrace) run cptrace 200 env SLIME_RS_PIPE_TRACE=1 python tools/cp_trace.py &&
             run cptrace_st4 200 env SLIME_RS_HOST_STAGES=4 python tools/cp_trace.py &&
             run cptrace_t0 200 env SLIME_RS_COPY_THREADS=0 python tools/cp_trace.py ;;
    tests_blit) run pytest_blit 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "copy_kernel_threshold or write_chunks_and_reconstruct" ;;
    concc) for t in 1 2 4 8 16; do run concc_$t 120 tools/latency_c 400 $t || exit 1; done ;;
    concsmall) run conc4k 200 python tools/host_concurrency.py --kib 4 --reps 300 --delay 0 --threads 1,2,4,8,16 &&
               run conc64k 200 python tools/host_concurrency.py --kib 64 --reps 200 --delay 0 --threads 1,2,4,8,16 ;;
    latwin) for rep in 1 2; do for w in 16 4 2; do run latwin_${w}_$rep 120 env SLIME_RS_OBJ_WINDOW_MIB=$w tools/latency_c 100 || exit 1; done; done ;;
    latab) for rep in 1 2; do run latab_blit_$rep 120 tools/latency_c 200 && run latab_sdma_$rep 120 env SLIME_RS_BLIT_KIB=0 tools/latency_c 200 &&
             run latab_rocblit_$rep 120 env SLIME_RS_BLIT_KIB=0 GPU_FORCE_BLIT_COPY_SIZE=4096 tools/latency_c 200 || exit 1; done ;;
    latenv) run latenv_base 120 tools/latency_c 200 && run latenv_blit 120 env GPU_FORCE_BLIT_COPY_SIZE=4096 tools/latency_c 200 &&
            run latenv_nosdma 120 env HSA_ENABLE_SDMA=0 tools/latency_c 200 && run latenv_base2 120 tools/latency_c 200 ;;
    latcprof) run latcprof 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/latcprof" -o lat --output-format csv -- tools/latency_c 50 ;;
    lattrace) run lattrace 200 env SLIME_RS_PIPE_TRACE=1 python tools/latency_probe.py ;;
    latprof) run latprof 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/latprof" -o lat --output-format csv -- \
            python3 tools/latency_probe.py ;;
    hostonly) run hostonly 300 python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 ;;
    hostprof) run hostprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/hostprof" -o host --output-format csv -- \
            python3 bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== session done" | tee -a "$OUT/session.log"
