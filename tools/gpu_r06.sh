#!/usr/bin/env bash
# Round-6 GPU-box session: every GPU step under its own time limit; the first
# crash/abort/timeout ends the session (nothing more runs on the GPU).
# Usage (repo root, on the box):  bash tools/gpu_r06.sh <step> [<step>...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
NOLEGS="--cpu-baseline 0 --host-path 0 --alloc-probe 0 --c5-leg 0 --c5-bytes 0 --shape-legs= --pooled 0"

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
    tests_host) run pytest_host 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_host.py -x -q --timeout 120 --timeout-method thread -m gpu -k "map or recover or host or unchanged or RecoverData or reconstruct or pool or create or parity or write_chunks" ;;
    tests_switch) run pytest_switch 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mid_object_switch or encode_objects or write_chunks or redo" ;;
    tests_mfma) run pytest_mfma 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread ;;
    tests_bench) run pytest_bench 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 200 --timeout-method thread ;;
    tests_full) run pytest_full 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread ;;
    bench20) run bench20 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    # the driver's command under the profiler WITH the pooled leg
    profpool) run profpool 700 rocprofv3 --kernel-trace --stats -d "$OUT/profpool" -o bench --output-format csv -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
            python tools/prof_summary.py "$OUT/profpool" > "$OUT/profpool_summary.json" &&
            rm -f "$OUT/profpool/bench_kernel_trace.csv" ;;
    # only the pooled leg under the profiler (short), to reproduce the r05 fault quickly
    profpoolonly) run profpoolonly 400 rocprofv3 --kernel-trace --stats -d "$OUT/profpoolonly" -o pool --output-format csv -- \
            python3 bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --host-path 0 --alloc-probe 0 --c5-leg 0 --shape-legs= ;;
    hostonly) run hostonly 400 python bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --cpu-baseline 0 --alloc-probe 0 --c5-leg 0 --shape-legs= ;;
    pmc_c3) pmc pmc_c3_fetch FETCH_SIZE --steps 3 --warmup 1 $NOLEGS --bytes-path 0 &&
            pmc pmc_c3_write WRITE_SIZE --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    pmc_c2) pmc pmc_c2_fetch FETCH_SIZE --preset c2 --steps 3 --warmup 1 $NOLEGS --bytes-path 0 &&
            pmc pmc_c2_write WRITE_SIZE --preset c2 --steps 3 --warmup 1 $NOLEGS --bytes-path 0 ;;
    # second-pass walk variants (s19): the harness at commit b1d0ca6 only, its variants were not kept
    # the byte encode's second pass: re-encode vs top-bit correction (tools/topbits_fix.*)
    topbits) run topbits 500 python tools/topbits_fix.py --shapes c5,c3 --rounds 6 --fix-blocks 512,256 ;;
    # the same through the product API (slime_rs_switch_bits 2 vs 1) on the bench's data
    topbits_ab) run topbits_ab 500 python tools/topbits_ab.py --shapes c5,c3,c5_512 --rounds 8 ;;
    # 4/6 (C2) unroll / unit variants of the queue apply on the stamped twin, twice
    c2var) C="python tools/c2_stamps.py --need 4 --total 6 --mib 64"
      G="0:0,0:0:104,0:0:204,0:0:304,0:0:404,0:0:504,0:0:604,0:512:104,0:512:304,0:1024:304,0:512:204"
      run c2var_1 300 $C --nobj 32 --reps 16 --geometry $G &&
      run c2var_2 300 $C --nobj 32 --reps 16 --geometry $G &&
      run c2var_64 300 $C --nobj 64 --reps 12 --geometry $G ;;
    # the product's three-tile units at k <= 4 against the old two-tile form (twin), 4/6 and 3/5
    c2unit_check) C="python tools/c2_stamps.py --mib 64"
      run c2chk_46 300 $C --need 4 --total 6 --nobj 32,64 --reps 16 --geometry 0:0,0:0:1104 &&
      run c2chk_35 300 $C --need 3 --total 5 --nobj 32,64 --reps 16 --geometry 0:0,0:0:1203 ;;
    # unit size at 8/12 (C3, 64 MiB shards) and 10/14 on the twin, twice
    c3unit) C="python tools/c2_stamps.py"
      for rep in 1 2; do
        run c3unit_$rep 300 $C --need 8 --total 12 --mib 256 --nobj 128 --reps 6 --geometry 0:0,0:0:1308,0:0:1408,0:0:1508 &&
        run c3unit_ns64_$rep 300 $C --need 8 --total 12 --mib 512 --nobj 64 --reps 6 --geometry 0:0,0:0:1308,0:0:1408 &&
        run c5unit_$rep 300 $C --need 10 --total 14 --mib 1024 --nobj 16 --reps 6 --geometry 0:0,0:0:1310 || exit 1
      done ;;
    # units of 3 / 4 / 6 tiles at 4/6 and 3/5 (the C of the queue walk), twice, and 8/12 for reference
    c2unit) C="python tools/c2_stamps.py --mib 64"
      for rep in 1 2; do
        run c2unit_46_$rep 300 $C --need 4 --total 6 --nobj 32,64 --reps 16 --geometry 0:0,0:0:604,0:0:704,0:0:804 &&
        run c2unit_35_$rep 300 $C --need 3 --total 5 --nobj 32,64 --reps 16 --geometry 0:0,0:0:903,0:0:1003 || exit 1
      done ;;
    tests_phased) run pytest_phased 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "phased" ;;
    bpmc_c3) pmc bpmc_c3_fetch FETCH_SIZE --steps 3 --warmup 1 $NOLEGS &&
             pmc bpmc_c3_write WRITE_SIZE --steps 3 --warmup 1 $NOLEGS ;;
    bpmc_c5) pmc bpmc_c5_fetch FETCH_SIZE --preset c5 --global-objects 16 --steps 3 --warmup 1 $NOLEGS &&
             pmc bpmc_c5_write WRITE_SIZE --preset c5 --global-objects 16 --steps 3 --warmup 1 $NOLEGS ;;
    # C2's fixed cost per launch split by per-wave stamps, and the same under a kernel trace
    stamps) run stamps_c2 300 python tools/c2_stamps.py --need 4 --total 6 --mib 64 --nobj 32,64,128 &&
            run stamps_c3 300 python tools/c2_stamps.py --need 8 --total 12 --mib 256 --nobj 32,64,128 --reps 6 &&
            run stamps_c2_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/stamps_c2_prof" -o st --output-format csv -- \
              python3 tools/c2_stamps.py --need 4 --total 6 --mib 64 --nobj 32,64,128 ;;
    # C2 geometry A/B on the stamped twin: segments per object x blocks
    c2geo) run c2geo 300 python tools/c2_stamps.py --need 4 --total 6 --mib 64 --nobj 32 --reps 16 \
             --geometry 0:0,1:256,2:256,4:256,8:256,2:512,4:512,1:512 &&
           run c2geo_c3 300 python tools/c2_stamps.py --need 8 --total 12 --mib 256 --nobj 128 --reps 6 \
             --geometry 0:0,2:256,1:512 ;;
    # segments per object (TicketWalk spread) across the BASELINE shapes, on the stamped twin
    spreadsweep) C="python tools/c2_stamps.py"
      run ss_c2_32 300 $C --need 4 --total 6 --mib 64 --nobj 32 --reps 16 --geometry 0:0,4:0,8:0,16:0,32:0 &&
      run ss_c2_64 300 $C --need 4 --total 6 --mib 64 --nobj 64 --reps 12 --geometry 0:0,2:0,4:0,8:0 &&
      run ss_c2_128 300 $C --need 4 --total 6 --mib 64 --nobj 128 --reps 8 --geometry 0:0,2:0,4:0 &&
      run ss_c3_128 300 $C --need 8 --total 12 --mib 256 --nobj 128 --reps 6 --geometry 0:0,2:0,4:0 &&
      run ss_c3_32 300 $C --need 8 --total 12 --mib 256 --nobj 32 --reps 8 --geometry 0:0,4:0,8:0,16:0 &&
      run ss_ns64 300 $C --need 8 --total 12 --mib 512 --nobj 64 --reps 6 --geometry 0:0,2:0,4:0,8:0 &&
      run ss_c5_64 300 $C --need 10 --total 14 --mib 1024 --nobj 64 --reps 4 --geometry 0:0,2:0,4:0 &&
      run ss_c5_16 300 $C --need 10 --total 14 --mib 1024 --nobj 16 --reps 6 --geometry 0:0,8:0,16:0,32:0 ;;
    spreadsweep2) C="python tools/c2_stamps.py"
      for rep in 1 2; do
        run ss2_c2_32_$rep 300 $C --need 4 --total 6 --mib 64 --nobj 32 --reps 20 --geometry 0:0,8:0,16:0,2:0,4:0 &&
        run ss2_c2_64_$rep 300 $C --need 4 --total 6 --mib 64 --nobj 64 --reps 12 --geometry 0:0,4:0,2:0 &&
        run ss2_c3_32_$rep 300 $C --need 8 --total 12 --mib 256 --nobj 32 --reps 10 --geometry 0:0,8:0,4:0 &&
        run ss2_c3_128_$rep 300 $C --need 8 --total 12 --mib 256 --nobj 128 --reps 6 --geometry 0:0,2:0 &&
        run ss2_c5_64_$rep 300 $C --need 10 --total 14 --mib 1024 --nobj 64 --reps 4 --geometry 0:0,2:0 &&
        run ss2_c5_8_$rep 300 $C --need 10 --total 14 --mib 1024 --nobj 8 --reps 8 --geometry 0:0,16:0,4:0,32:0 || exit 1
      done ;;
    # the driver's command under the profiler, without the pooled leg (the profiler's own fault, s1_segv)
    profdrv) run profdrv 700 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 --pooled 0 &&
            python tools/prof_summary.py "$OUT/prof" > "$OUT/prof_summary.json" ;;
    rehearse2) run rehearse2 500 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --objects 32 --steps 5 --warmup 1 --cpu-baseline 0 --alloc-probe 0 &&
               run rehearse2_torchrun 500 env SLIME_BENCH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --objects 32 --steps 5 --warmup 1 --cpu-baseline 0 --alloc-probe 0 ;;
    # what one fused byte encode call enqueues, and the gaps between (C5 and C3 shapes)
    etl) run etl_c5_plain 300 python tools/encode_timeline.py run &&
         run etl_c5 300 rocprofv3 --kernel-trace -d "$OUT/etl_c5" -o etl --output-format csv -- python3 tools/encode_timeline.py run &&
         python3 tools/encode_timeline.py show "$OUT/etl_c5" > "$OUT/etl_c5_show.txt" &&
         run etl_c3 300 rocprofv3 --kernel-trace -d "$OUT/etl_c3" -o etl --output-format csv -- python3 tools/encode_timeline.py run --need 8 --total 12 --mib 256 --nobj 128 &&
         python3 tools/encode_timeline.py show "$OUT/etl_c3" > "$OUT/etl_c3_show.txt" ;;
    # C5's per-GPU share at N = 8 / 4 / 2 (8 / 16 / 32 objects of 1 GiB, 10/14) on the stamped twin
    c5share) C="python tools/c2_stamps.py --need 10 --total 14 --mib 1024"
      run c5s_8 300 $C --nobj 8 --reps 10 --geometry 0:0,4:0,2:0,8:512,4:512 &&
      run c5s_16 300 $C --nobj 16 --reps 8 --geometry 0:0,2:0,8:0,4:512 &&
      run c5s_32 300 $C --nobj 32 --reps 6 --geometry 0:0,1:0,4:0,2:512 &&
      run c5s_8b 300 $C --nobj 8 --reps 10 --geometry 0:0,4:0,2:0 ;;
    # four ranks on one GPU: the N = 4 code paths (shape legs limited to C2 so four ranks fit in one HBM)
    rehearse4) run rehearse4 500 env SLIME_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --objects 32 --steps 3 --warmup 1 --cpu-baseline 0 --alloc-probe 0 --shape-legs=c2 ;;
    # slime's default redundancy 3/5 (multi_config.go:139,152) as a device batch: the narrow-code spread rule
    spread35) C="python tools/c2_stamps.py --need 3 --total 5 --mib 64"
      run ss35_32 300 $C --nobj 32 --reps 16 --geometry 0:0,2:0,4:0,16:0 &&
      run ss35_64 300 $C --nobj 64 --reps 12 --geometry 0:0,1:0,2:0 &&
      run ss35_32b 300 $C --nobj 32 --reps 16 --geometry 0:0,2:0 ;;
    spread35b) for rep in 1 2 3; do
        run ss35b_$rep 300 python tools/c2_stamps.py --need 3 --total 5 --mib 64 --nobj 32 --reps 16 --geometry 0:0,2:0,4:0 &&
        run ss46b_$rep 300 python tools/c2_stamps.py --need 4 --total 6 --mib 64 --nobj 32 --reps 16 --geometry 0:0,2:0,4:0 || exit 1
      done ;;
    # the profiler's fault against the number of concurrent callers (first crash ends the session)
    profthreads) for t in ${PROF_THREADS:-2 4 8 16}; do
        run profpool_t$t 400 rocprofv3 --kernel-trace --stats -d "$OUT/profpool_t$t" -o pool --output-format csv -- \
          python3 bench.py --objects 8 --steps 2 --warmup 1 --bytes-path 0 --c5-bytes 0 --cpu-baseline 0 --host-path 0 \
          --alloc-probe 0 --c5-leg 0 --shape-legs= --pool-threads $t || exit 1
        rm -f "$OUT/profpool_t$t/pool_kernel_trace.csv"  # tens of MB a run; the stats CSV stays
      done ;;
    # two segments an object for wide codes at 64 objects? 10/14, 12/16, 16/20 (k + rows 14, 16, 20)
    spreadwide) C="python tools/c2_stamps.py"
      for rep in 1 2; do
        run sw_c5_64_$rep 300 $C --need 10 --total 14 --mib 1024 --nobj 64 --reps 4 --geometry 0:0,2:0 &&
        run sw_12_64_$rep 300 $C --need 12 --total 16 --mib 1024 --nobj 64 --reps 4 --geometry 0:0,2:0 &&
        run sw_16_64_$rep 300 $C --need 16 --total 20 --mib 1024 --nobj 64 --reps 4 --geometry 0:0,2:0 &&
        run sw_16_128_$rep 300 $C --need 16 --total 20 --mib 256 --nobj 128 --reps 6 --geometry 0:0,2:0 || exit 1
      done ;;
    *) echo "unknown step $step" | tee -a "$OUT/session.log"; exit 2 ;;
  esac
done
echo "=== session done" | tee -a "$OUT/session.log"
