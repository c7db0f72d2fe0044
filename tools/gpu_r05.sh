#!/usr/bin/env bash
# Round-5 GPU-box session: every GPU step under its own time limit; the first
# crash/abort/timeout ends the session (nothing more runs on the GPU).
# Usage (repo root, on the box):  bash tools/gpu_r05.sh <step> [<step>...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
NOLEGS="--cpu-baseline 0 --host-path 0 --alloc-probe 0 --c5-leg 0 --shape-legs= --pooled 0"

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

# pmc <name> <counter> <bench args...>: one counter pass of bench.py
pmc() {
  local name=$1 counter=$2; shift 2
  run "$name" 300 timeout -s KILL 240 rocprofv3 --pmc "$counter" -d "$OUT/$name" -o pmc --output-format csv -- \
    python3 bench.py "$@"
}

nproc > "$OUT/host.txt"; grep -m1 "model name" /proc/cpuinfo >> "$OUT/host.txt" || true
for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    tests_switch) run pytest_switch 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mid_object_switch or encode_objects or write_chunks or redo" ;;
    tests_mfma) run pytest_mfma 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread ;;
    tests_host) run pytest_host 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "map or recover or host or unchanged or RecoverData or reconstruct or pool" ;;
    tests_sched) run pytest_sched 400 python -u -m pytest tests/test_gpu_schedule.py -x -v --timeout 200 --timeout-method thread ;;
    tests_fuzz) run pytest_fuzz 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fuzz" ;;
    tests_bench) run pytest_bench 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 200 --timeout-method thread ;;
    hostrep) for i in 1 2 3; do run hostrep_$i 400 python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 --shape-legs= --pooled 0 || exit 1; done ;;
    proxysweep) run proxy_sweep 300 python tools/proxy_sweep.py --threads 1,4,8,16,25 --mib 64,1 --seconds 1.5 &&
                run proxy_sweep_c0 300 env SLIME_RS_COPY_THREADS=0 python tools/proxy_sweep.py --threads 8,16,25 --mib 64,1 --seconds 1.5 &&
                run proxy_sweep_c4 300 env SLIME_RS_COPY_THREADS=4 python tools/proxy_sweep.py --threads 8,16,25 --mib 64,1 --seconds 1.5 ;;
    # C2 gap: the same 4/6 kernel on 32 (C2), 64 and 128 objects of 64 MiB, and a rocprof trace of C2
    c2size) for n in 32 64 128 32; do run c2size_$n 300 python bench.py --preset c2 --objects $n --bytes-path 0 --steps 20 --warmup 5 $NOLEGS || exit 1; done &&
            run c2prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/c2prof" -o c2 --output-format csv -- \
              python3 bench.py --preset c2 --bytes-path 0 --steps 20 --warmup 5 $NOLEGS ;;
    proxyq) run proxy_q8 300 env GPU_MAX_HW_QUEUES=8 python tools/proxy_sweep.py --threads 8,16,25 --mib 64,1 --seconds 1.5 &&
            run proxy_q16 300 env GPU_MAX_HW_QUEUES=16 python tools/proxy_sweep.py --threads 8,16,25 --mib 64,1 --seconds 1.5 ;;
    proxysched) for sc in auto yield blocking spin; do
                  run proxy_sched_$sc 300 python tools/proxy_sweep.py --threads 8,16,25 --mib 64,1 --seconds 1.5 --sched $sc || exit 1
                done ;;
    latc) run latc 200 tools/latency_c 300 ;;
    # wide codes, this tree's library against ab/base (the previous build), alternating in one box
    wideab) E16=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15
            WB="--steps 5 --warmup 2 $NOLEGS"
            cp slime_amd/lib/libslime_rs.so /tmp/ab_new.so
            for rep in 1 2; do
              for v in new $(ls ab); do
                if [ "$v" = new ]; then cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so; else cp ab/$v/libslime_rs.so slime_amd/lib/libslime_rs.so; fi
                for shp in "80 100 $E16,16,17,18,19" "64 80 $E16" "72 90 $E16,16,17"; do
                  set -- $shp
                  run wab_$1_$2_${v}_$rep 300 python bench.py --need $1 --total $2 --objects 32 --erase $3 $WB || exit 1
                done
              done
            done
            cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so ;;
    # which part of the wide kernel costs: rows 16 vs 20 at K steps 4 and 5 (symbol path)
    wshape) for shp in "64 80" "64 84" "80 96" "80 100" "72 88" "72 90" "48 64" "48 68"; do
              set -- $shp
              E=$(python -c "print(','.join(map(str,range($2-$1))))")
              run wsh_$1_$2 300 python bench.py --need $1 --total $2 --objects 32 --erase $E --bytes-path 0 --steps 5 --warmup 2 $NOLEGS || exit 1
            done ;;
    wpmc80) E20=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19
            pmc wpmc80_fetch FETCH_SIZE --need 80 --total 100 --objects 32 --erase $E20 --steps 3 --warmup 1 $NOLEGS &&
            pmc wpmc80_write WRITE_SIZE --need 80 --total 100 --objects 32 --erase $E20 --steps 3 --warmup 1 $NOLEGS &&
            pmc wpmc80_sq "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM" \
              --need 80 --total 100 --objects 32 --erase $E20 --steps 3 --warmup 1 $NOLEGS ;;
    wshape2) for shp in "64 96" "80 96" "48 80" "64 80" "32 64" "80 100"; do
              set -- $shp
              E=$(python -c "print(','.join(map(str,range($2-$1))))")
              run wsh2_$1_$2 300 python bench.py --need $1 --total $2 --objects 32 --erase $E --bytes-path 0 --steps 5 --warmup 2 $NOLEGS || exit 1
            done ;;
    # k > 80: this tree vs ab/* on 96/100, 90/100 (six K steps) and 100/116 (seven)
    wideab2) WB="--steps 5 --warmup 2 $NOLEGS"
             cp slime_amd/lib/libslime_rs.so /tmp/ab_new.so
             for rep in 1 2; do
               for v in new $(ls ab); do
                 if [ "$v" = new ]; then cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so; else cp ab/$v/libslime_rs.so slime_amd/lib/libslime_rs.so; fi
                 for shp in "96 100" "90 100" "100 116"; do
                   set -- $shp
                   E=$(python -c "print(','.join(map(str,range($2-$1))))")
                   run wab_$1_$2_${v}_$rep 300 python bench.py --need $1 --total $2 --objects 32 --erase $E $WB || exit 1
                 done
               done
             done
             cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so ;;
    widevar) for rep in 1 2; do
               run wv_80_100_$rep 300 python tools/wide_variants.py --need 80 --total 100 --variants 0,2,5,6,7 &&
               run wv_76_96_$rep 300 python tools/wide_variants.py --need 76 --total 96 --variants 0,2,5,6,7 || exit 1
             done ;;
    # do many input shards per wave cost through the address translation? the same bytes in
    # objects whose shards share 2 MiB pages (32 MiB and 8 MiB objects) against 256 MiB objects
    wtlb) for shp in "80 100" "64 80" "8 12"; do
            set -- $shp
            E=$(python -c "print(','.join(map(str,range(min(4, $2-$1)))))")
            for om in "256 32" "32 256" "8 1024"; do
              set -- $1 $2 $om
              run wtlb_$1_$2_$3 300 python bench.py --need $1 --total $2 --object-mib $3 --objects $4 --erase $E --bytes-path 0 --steps 5 --warmup 2 $NOLEGS || exit 1
            done
          done ;;
    wilv) for rep in 1 2; do
            run wilv_80_100_$rep 300 python tools/wide_variants.py --need 80 --total 100 --variants 0,2,8 &&
            run wilv_72_90_$rep 300 python tools/wide_variants.py --need 72 --total 90 --variants 0,2,8 || exit 1
          done ;;
    # many short objects at wide codes (the flat walk), this tree vs ab/*, alternating
    wshort) cp slime_amd/lib/libslime_rs.so /tmp/ab_new.so
            for rep in 1 2; do
              for v in new $(ls ab); do
                if [ "$v" = new ]; then cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so; else cp ab/$v/libslime_rs.so slime_amd/lib/libslime_rs.so; fi
                run wshort_${v}_$rep 300 python tools/short_objects.py --shapes 80/100,40/56,64/80 --L 64,512,2048 --nobj 4096 || exit 1
              done
            done
            cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so ;;
    wshortb) cp slime_amd/lib/libslime_rs.so /tmp/ab_new.so
            for rep in 1 2; do
              for v in new $(ls ab); do
                if [ "$v" = new ]; then cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so; else cp ab/$v/libslime_rs.so slime_amd/lib/libslime_rs.so; fi
                run wshortb_${v}_$rep 300 python tools/short_objects.py --shapes 80/100,40/56,64/80 --bytes 16384,65536,262144 --nobj 1024 || exit 1
              done
            done
            cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so ;;
    wshortt) cp slime_amd/lib/libslime_rs.so /tmp/ab_new.so
            for rep in 1 2; do
              for v in new $(ls ab); do
                if [ "$v" = new ]; then cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so; else cp ab/$v/libslime_rs.so slime_amd/lib/libslime_rs.so; fi
                run wshortt_${v}_$rep 300 python tools/short_objects.py --shapes 80/100,40/56 --L 67,515,2051 --nobj 4096 || exit 1
              done
            done
            cp /tmp/ab_new.so slime_amd/lib/libslime_rs.so ;;
    wilvapi) for rep in 1 2; do
               run wilvapi_contig_$rep 300 python tools/short_objects.py --shapes 80/100,72/90,96/100,40/56 --L 4194304 --nobj 1 &&
               run wilvapi_blocks_$rep 300 python tools/short_objects.py --shapes 80/100,72/90,96/100,40/56 --L 64 --nobj 65536 || exit 1
             done ;;
    profshort) for cfg in "80/100 16384" "80/100 262144" "40/56 16384" "64/80 16384" "64/80 262144"; do
                 read -r shp sz <<< "$cfg"; tag=$(echo "${shp}_$sz" | tr / _)
                 run profshort_$tag 300 rocprofv3 --kernel-trace --stats -d "$OUT/profshort_$tag" -o short --output-format csv -- \
                   python3 tools/short_objects.py --shapes $shp --bytes $sz --nobj 1024 --rounds 3 || exit 1
               done ;;
    wprof80) E20=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19
             run wprof80 300 rocprofv3 --kernel-trace --stats -d "$OUT/wprof80" -o bench --output-format csv -- \
               python3 bench.py --need 80 --total 100 --objects 32 --erase $E20 --steps 3 --warmup 1 $NOLEGS ;;
    tests_full) run pytest_full 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread ;;
    bench20) run bench20 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchq) run benchq 400 python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-path 0 --alloc-probe 0 --bytes-path 0 ;;
    hostonly) run hostonly 400 python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 --shape-legs= ;;
    rehearse2) run rehearse2 400 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --objects 32 --steps 5 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 &&
               run rehearse2_torchrun 400 env SLIME_BENCH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --objects 32 --steps 5 --warmup 1 --bytes-path 0 \
                 --cpu-baseline 0 --alloc-probe 0 ;;
    # the driver's command under the profiler, without the pooled leg (rocprofv3 segfaulted
    # inside the runtime under its 25 concurrent host threads, profiles/r05/s4_pmc_c2/c2prof.log)
    profdrv) run profdrv 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 --pooled 0 ;;
    # PMC traffic passes per BASELINE shape (symbol path), each its own run
    pmc_c3) pmc pmc_c3_fetch FETCH_SIZE --steps 3 --warmup 1 $NOLEGS --bytes-path 0 &&
            pmc pmc_c3_write WRITE_SIZE --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    pmc_c2) pmc pmc_c2_fetch FETCH_SIZE --preset c2 --steps 3 --warmup 1 $NOLEGS --bytes-path 0 &&
            pmc pmc_c2_write WRITE_SIZE --preset c2 --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    pmc_ns64) pmc pmc_ns64_fetch FETCH_SIZE --preset ns64 --steps 3 --warmup 1 $NOLEGS --bytes-path 0 &&
              pmc pmc_ns64_write WRITE_SIZE --preset ns64 --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    bpmc_c3) pmc bpmc_c3_fetch FETCH_SIZE --steps 3 --warmup 1 $NOLEGS &&
             pmc bpmc_c3_write WRITE_SIZE --steps 3 --warmup 1 $NOLEGS ;;
    bpmc_c5) pmc bpmc_c5_fetch FETCH_SIZE --preset c5 --global-objects 16 --steps 3 --warmup 1 $NOLEGS &&
             pmc bpmc_c5_write WRITE_SIZE --preset c5 --global-objects 16 --steps 3 --warmup 1 $NOLEGS ;;
    *) echo "unknown step $step" | tee -a "$OUT/session.log"; exit 2 ;;
  esac
done
echo "=== session done" | tee -a "$OUT/session.log"
