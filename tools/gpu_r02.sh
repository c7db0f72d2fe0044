#!/usr/bin/env bash
# Round-2 GPU-box session: every GPU step under its own time limit; the first
# crash/abort/timeout ends the session (nothing more runs on the GPU).
# Usage (repo root, on the box):  bash tools/gpu_r02.sh <step> [<step>...]
# NOTE (round 6): the A/B environment variables these steps set -- SLIME_RS_MFMA*, SLIME_RS_QUEUE,
# SLIME_RS_PIPE, SLIME_RS_GRID_TARGET, SLIME_RS_SEGMENTS, SLIME_RS_HOST_PIPE -- were removed from the
# library in round 5 and now do nothing: re-running a step does not reproduce its A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

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
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_nocpu) run bench_nocpu 300 python bench.py --cpu-baseline 0 --host-path 0 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
            python3 bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-path 0 --bytes-path 0 --alloc-probe 0 ;;
    pmc_fetch) run pmc_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-path 0 --bytes-path 0 --alloc-probe 0 ;;
    pmc_write) run pmc_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-path 0 --bytes-path 0 --alloc-probe 0 ;;
    phased_enc) run phased_enc 400 python tools/apply_variants.py --variants 15 --blocks 256 --rounds 3 \
            --phased 3:700:460,3:800:530,3:900:600,6:1300:860,6:1500:1000 ;;
    phased_dec) run phased_dec 400 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 \
            --rounds 3 --phased 3:800:530,6:1400:930 ;;
    phased_slow) run phased_slow 600 python tools/apply_variants.py --hunt slow --variants 15,18,19 --blocks 256 \
            --rounds 3 --phased 3:700:460,3:800:530,3:900:600,6:1300:860,6:1500:1000 ;;
    burst) run burst 400 python tools/apply_variants.py --variants 15 --blocks 256 --rounds 3 --burst 1,2,3 ;;
    burst_dec) run burst_dec 400 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 \
            --rounds 3 --burst 1,2,3 ;;
    burst_slow) run burst_slow 600 python tools/apply_variants.py --hunt slow --variants 15 --blocks 256 --rounds 3 \
            --burst 1,2,3 ;;
    stage) run stage 400 python tools/apply_variants.py --variants 14,15 --blocks 256,512 --rounds 3 --burst 1 --batched 2,3 ;;
    stage_dec) run stage_dec 400 python tools/apply_variants.py --decode 1 --separate 0 --variants 14,15 --blocks 256,512 \
            --rounds 3 --burst 1 --batched 2,3 ;;
    stage_fast) run stage_fast 600 python tools/apply_variants.py --hunt fast --variants 15 --blocks 256,512 --rounds 3 \
            --burst 1 --batched 2,3 ;;
    hostbd) run hostbd 300 python tools/host_breakdown.py ;;
    hostbd16) run hostbd16 300 python tools/host_breakdown.py --mib 16 ;;
    shapes) run shape_64mib 300 python bench.py --object-mib 512 --objects 64 --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
            run shape_c2 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --cpu-baseline 0 --host-path 0 &&
            run shape_c5 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 --cpu-baseline 0 --host-path 0 &&
            run shape_c3_again 300 python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 ;;
    hostdiag) run hostdiag 600 python tools/host_diag.py ;;
    hostdiag4) run hostdiag4 600 python tools/host_diag.py --threads 4,8 --pre bench &&
               run hostdiag5 600 python tools/host_diag.py --threads 0,2,4 --pre none &&
               run bench_host 300 python bench.py --cpu-baseline 0 --bytes-path 0 ;;
    hosttrace) run trace_bytes 300 env SLIME_RS_PIPE_TRACE=1 python bench.py --cpu-baseline 0 &&
               run trace_nobytes 300 env SLIME_RS_PIPE_TRACE=1 python bench.py --cpu-baseline 0 --bytes-path 0 &&
               run trace_bytes2 300 env SLIME_RS_PIPE_TRACE=1 python bench.py --cpu-baseline 0 ;;
    hostorder) run order_before 300 python bench.py --cpu-baseline 0 &&
               run order_after 300 python bench.py --cpu-baseline 0 --host-order after-free &&
               run order_after_10s 300 python bench.py --cpu-baseline 0 --host-order after-free --host-delay 10 ;;
    sdma) run order_after_nosdma 300 env HSA_ENABLE_SDMA=0 python bench.py --cpu-baseline 0 --host-order after-free &&
          run order_before_nosdma 300 env HSA_ENABLE_SDMA=0 python bench.py --cpu-baseline 0 ;;
    c2sweep) for g in 256 512 1024 2048; do for sg in 8 16 32; do
               run c2_g${g}_s${sg} 120 env SLIME_RS_GRID_TARGET=$g SLIME_RS_SEGMENTS=$sg python bench.py --need 4 --total 6 \
                 --object-mib 64 --objects 32 --erase 0,1 --cpu-baseline 0 --host-path 0 --bytes-path 0 --steps 20 || exit $?
             done; done ;;
    widemath) run wide_20_24 300 python tools/apply_variants.py --need 20 --total 24 --nobj 32 --wide 1 --blocks 256,1024 &&
              run wide_32_40 300 python tools/apply_variants.py --need 32 --total 40 --nobj 32 --wide 1 --blocks 256,1024 &&
              run wide_64_80 300 python tools/apply_variants.py --need 64 --total 80 --nobj 16 --wide 1 --blocks 256,1024 ;;
    pipek) run pipek_20_24 300 python tools/apply_variants.py --need 20 --total 24 --nobj 32 --wide 1 --pipek 1,2 --blocks 256,512,1024 &&
           run pipek_24_28 300 python tools/apply_variants.py --need 24 --total 28 --nobj 32 --wide 1 --pipek 1,2 --blocks 256,512,1024 &&
           run pipek_32_40 300 python tools/apply_variants.py --need 32 --total 40 --nobj 32 --wide 1 --pipek 1 --blocks 256,512,1024 &&
           run pipek_20_24_dec 300 python tools/apply_variants.py --need 20 --total 24 --nobj 32 --wide 1 --pipek 1,2 --blocks 256,512,1024 --decode 1 ;;
    pipekcheck) run pipek_check 300 python tools/pipek_check.py ;;
    k32ab) for kn in "20 24 32" "24 28 32" "32 40 32" "17 20 32"; do set -- $kn
             run k32_${1}_${2} 200 python bench.py --need $1 --total $2 --objects $3 --erase 0,1,2,3 --cpu-baseline 0 --host-path 0 &&
             run k32off_${1}_${2} 200 env SLIME_RS_K32=0 python bench.py --need $1 --total $2 --objects $3 --erase 0,1,2,3 --cpu-baseline 0 --host-path 0 || exit $?
           done ;;
    pipek48) run pipek_40_48 300 python tools/apply_variants.py --need 40 --total 48 --nobj 16 --wide 1 --pipek 1 --blocks 256,512,1024 &&
             run pipek_48_56 300 python tools/apply_variants.py --need 48 --total 56 --nobj 16 --wide 1 --pipek 1 --blocks 256,512,1024 ;;
    hostconc) run hostconc 400 python tools/host_concurrency.py ;;
    hostconc_q16) run hostconc_q16 400 env GPU_MAX_HW_QUEUES=16 python tools/host_concurrency.py ;;
    ns64) run ns64_harness 300 python tools/apply_variants.py --mib 512 --nobj 64 --variants 13,14,15,20 \
            --blocks 256,512,1024 --nseg 1,2,4,8 &&
          run ns64_bench 300 python bench.py --object-mib 512 --objects 64 --cpu-baseline 0 --host-path 0 --bytes-path 0 ;;
    c5sweep) for g in 256 512; do for sg in 16 32 64; do
               run c5_g${g}_s${sg} 200 env SLIME_RS_GRID_TARGET=$g SLIME_RS_SEGMENTS=$sg python bench.py --need 10 --total 14 \
                 --object-mib 1024 --objects 8 --cpu-baseline 0 --host-path 0 --bytes-path 0 --steps 10 || exit $?
             done; done ;;
    slowcheck) (timeout 20 amd-smi metric --usage --mem-usage > "$OUT/smi_before.txt" 2>&1 || true)
               run sc_bench1 300 python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 --steps 20 &&
               (timeout 20 amd-smi metric --usage --mem-usage > "$OUT/smi_mid.txt" 2>&1 || true) &&
               for i in 1 2 3 4 5 6; do echo "sleep $i/6" | tee -a "$OUT/session.log"; sleep 20; done &&
               run sc_bench2 300 python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 --steps 20 &&
               run sc_c5 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 8 --cpu-baseline 0 --host-path 0 ;;
    hostdiag2) run hostdiag2 600 python tools/host_diag.py --threads 4 --pre bench &&
               run hostdiag3 600 python tools/host_diag.py --threads 4 --pre none &&
               run bench_hostonly 300 python bench.py --cpu-baseline 0 --bytes-path 0 ;;
    tail) run tail_enc 300 python tools/apply_variants.py --variants 15 --blocks 256,512 --nseg 1,2,4 --rounds 3 --timed 3 &&
          run tail_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 2 --rounds 3 --timed 3 ;;
    queue) run queue_enc 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 4,8,16 &&
           run queue_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 4,8,16 &&
           run queue_blocks 300 python tools/apply_variants.py --variants 15 --blocks 256,512,1024 --nseg 2 --rounds 3 --queue 8,16 ;;
    queue2) run queue2_enc 300 python tools/apply_variants.py --variants 15 --blocks 256,512 --nseg 2 --rounds 5 --queue 1,2,4,104,108 &&
            run queue2_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 1,2,4,104 ;;
    queue3) run queue3_enc 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 104,801,802,804,808,1602,1604 &&
            run queue3_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 104,801,802,804,1602 ;;
    qab) for q in 0 1; do
           run qab_c3_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
           run qab_ns64_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --object-mib 512 --objects 64 --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
           run qab_c5_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 --cpu-baseline 0 --host-path 0 --bytes-path 0 || exit $?
         done
         for q in 0 2; do
           run qab_c2_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
           run qab_k16_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need 16 --total 20 --objects 64 --erase 0,1,2,3 --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
           run qab_k3_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need 3 --total 5 --objects 64 --erase 0,1 --cpu-baseline 0 --host-path 0 --bytes-path 0 || exit $?
         done ;;
    queue4) run queue4_enc 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 802,808,20802,40802,40801,80801 --timed 2 &&
            run queue4_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 802,20802,40802,40801 ;;
    queuek) run queuek_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13,14,15 --blocks 256,512 --nseg 8 --rounds 5 --queue 802,804,200803,100806,100812,400802 &&
            run queuek_16 300 python tools/apply_variants.py --need 16 --total 20 --nobj 64 --variants 13,14 --blocks 256,1024 --nseg 4 --rounds 5 --queue 100806,100812,200803 ;;
    qab2) for kn in "1 2 0" "2 3 0" "3 5 0,1" "4 6 0,1" "6 9 0,1,2" "8 12 0,1,2,3" "12 16 0,1,2,3" "13 17 0,1,2,3" "16 20 0,1,2,3"; do
            set -- $kn
            for q in 0 1; do
              run qab2_${1}_${2}_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need $1 --total $2 --objects 64 --erase $3 --cpu-baseline 0 --host-path 0 --bytes-path 0 || exit $?
            done
          done
          for q in 0 1; do run qab2_c2_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --cpu-baseline 0 --host-path 0 --bytes-path 0 || exit $?; done ;;
    qab3) for kn in "20 24 0,1,2,3" "24 28 0,1,2,3" "28 32 0,1,2,3" "32 40 0,1,2,3"; do
            set -- $kn
            for q in 0 1; do
              run qab3_${1}_${2}_q$q 200 env SLIME_RS_QUEUE=$q python bench.py --need $1 --total $2 --objects 32 --erase $3 --cpu-baseline 0 --host-path 0 --bytes-path 0 || exit $?
            done
          done ;;
    queue5) run queue5_enc 300 python tools/apply_variants.py --variants 15 --blocks 256,512 --nseg 2 --rounds 5 --queue 802,803,801,400802,400801,200803,200802 &&
            run queue5_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256,512 --nseg 2 --rounds 5 --queue 802,803,400802,200803 ;;
    bytesab) for q in 1 0; do run bytesab_c3_q$q 300 env SLIME_RS_QUEUE=$q python bench.py --cpu-baseline 0 --host-path 0 || exit $?; done
             for q in 1 0; do run bytesab_c5_q$q 300 env SLIME_RS_QUEUE=$q python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 --cpu-baseline 0 --host-path 0 || exit $?; done ;;
    bytesab2) run bab_c3 300 python tools/bytes_ab.py &&
              run bab_c5 300 python tools/bytes_ab.py --need 10 --total 14 --object-mib 1024 --objects 16 &&
              run bab_c2 300 python tools/bytes_ab.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 &&
              run bab_k16 300 python tools/bytes_ab.py --need 16 --total 20 --objects 32 ;;
    c2tail) run c2tail 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 256 --nseg 8 --rounds 5 --queue 400802 --timed 3 &&
            run c2big 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 256 --erase 0,1 --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
            run c2std 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --cpu-baseline 0 --host-path 0 --bytes-path 0 ;;
    ns64b) run ns64_final 300 python bench.py --object-mib 512 --objects 64 --cpu-baseline 0 --host-path 0 --bytes-path 0 ;;
    vmm) run vmm_256 300 tools/vmm_probe malloc,vmm-id:256,vmm-rnd:256,malloc 2 &&
         run vmm_2 400 tools/vmm_probe malloc,vmm-id:2,vmm-rnd:2,malloc 2 &&
         run vmm_1024 300 tools/vmm_probe malloc,vmm-id:1024,vmm-rnd:1024,malloc 2 ;;
    vmm1g) run vmm1g 400 tools/vmm_probe malloc,vmm-id:1024,vmm-rnd:1024,malloc 5 ;;
    vmmid) run vmmid 500 tools/vmm_probe malloc,vmm-id:2,vmm-id:64,vmm-id:256,malloc 4 ;;
    vmmsz) run vmmsz 600 tools/vmm_probe malloc,vmm-id:16,vmm-id:128,vmm-id:512,vmm-id:2 3 ;;
    vmmorder) run vmmorder 600 tools/vmm_probe vmm-id:2,malloc,malloc,vmm-id:2,malloc 3 ;;
    vmmmix) run vmmmix 500 tools/vmm_probe malloc,vmm-rnd:2,vmm-id:2,vmm-rnd:64,malloc 4 ;;
    allocab) run bench_torch 300 python bench.py --allocator torch --cpu-baseline 0 --host-path 0 &&
             run bench_vmm 300 python bench.py --cpu-baseline 0 --host-path 0 &&
             run bench_torch2 300 python bench.py --allocator torch --cpu-baseline 0 --host-path 0 &&
             run bench_vmm2 300 python bench.py --cpu-baseline 0 --host-path 0 ;;
    vmm2) run vmm2 500 tools/vmm_probe malloc,vmm-id:2,vmm-id:2,malloc,vmm-id:2 3 &&
          run bench_vmm_2m 300 python bench.py --cpu-baseline 0 --host-path 0 ;;
    ondemand) run od_enc 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 802,1010802,1020802,1040802,1080802,1020804 &&
              run od_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 2 --rounds 5 --queue 802,1020802,1040802,1080802 &&
              run od_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 256 --nseg 8 --rounds 7 --queue 400802,1420802,1440802,1480802 ;;
    spread) run spread_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --variants 15 --blocks 256 --nseg 1,4,16,32 --rounds 5 --queue 802 &&
            run spread_c3 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 1,2,4 --rounds 5 --queue 802 &&
            run spread_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 256 --nseg 1,8 --rounds 7 --queue 400802 ;;
    spread2) run spread2_c5 300 python tools/apply_variants.py --need 10 --total 14 --mib 1024 --nobj 16 --variants 15 --blocks 256 --nseg 1,2,4,8 --rounds 5 --queue 802 &&
             run spread2_c2 300 python tools/apply_variants.py --need 4 --total 6 --mib 64 --nobj 32 --variants 13 --blocks 256 --nseg 2,4,8,16 --rounds 7 --queue 400802 &&
             run spread2_ns 300 python tools/apply_variants.py --mib 512 --nobj 64 --variants 15 --blocks 256 --nseg 1,2,4 --rounds 5 --queue 802 ;;
    shapes2) run shape2_ns64 300 python bench.py --object-mib 512 --objects 64 --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
             run shape2_c2 300 python bench.py --need 4 --total 6 --object-mib 64 --objects 32 --erase 0,1 --cpu-baseline 0 --host-path 0 &&
             run shape2_c5 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 16 --cpu-baseline 0 --host-path 0 &&
             run shape2_c5x8 300 python bench.py --need 10 --total 14 --object-mib 1024 --objects 8 --cpu-baseline 0 --host-path 0 --bytes-path 0 ;;
    torchrun1) run torchrun1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 ;;
    ntpol) run ntpol_enc 300 python tools/apply_variants.py --variants 15 --blocks 256 --nseg 1 --rounds 5 --queue 802,20010802,30010802,40010802 &&
           run ntpol_dec 300 python tools/apply_variants.py --decode 1 --separate 0 --variants 15 --blocks 256 --nseg 1 --rounds 5 --queue 802,20010802,30010802,40010802 ;;
    bytesk32) run bab_20_24 300 python tools/bytes_ab.py --need 20 --total 24 --objects 32 &&
              run bab_32_40 300 python tools/bytes_ab.py --need 32 --total 40 --objects 32 ;;
    orderab) run order_torch 300 python bench.py --allocator torch --cpu-baseline 0 --host-path 0 --bytes-path 0 &&
             run order_vmm 300 python bench.py --cpu-baseline 0 --host-path 0 --bytes-path 0 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== session done" | tee -a "$OUT/session.log"
