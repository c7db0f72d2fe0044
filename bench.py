#!/usr/bin/env python3
"""RS encode+decode throughput, device-resident, need=8/total=12 (BASELINE.json).

One step = one pass of the hot path over one batch of synthetic objects
resident in HBM:
  encode     all total-need parity shards of every object   (CreateParity x r, one launch)
  decode     rebuild data shards {0,1,2,3} of every object   (RecoverData, erased rows only, one launch)
from the symbol-domain shards (MapToGF already applied; the codec is timed
separately by tools/).  Objects are partitioned across ranks (one process per
GPU, no data-path collective: "weak" scaling, each rank owns its own batch).

value = (sum of object bytes encoded + decoded over all ranks) / (max over
ranks of the timed K steps), in GiB/s.  roofline: algorithmic HBM bytes per
launch of the dominant kernel (rs_apply_queue_kernel<8>) / its average duration,
from HIP events recorded on the launch stream.  cpu_baseline: the oracle's
faithful scalar C restatement of the reference's Go path, on a bounded sample.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--objects B] [--object-mib S]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (must precede slime_amd: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from slime_amd import batch  # noqa: E402
from slime_amd import device as D  # noqa: E402
from slime_amd.codeobj import kernel_code_id  # noqa: E402

GIB = 1 << 30
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# The same guide's measured achievable HBM rate (float4 copy, 79% of spec): the
# north star's "HBM roofline" read as what the chip streams, reported beside
# `frac` (which stays against the spec).
HBM_ACHIEVABLE_GBS = 6290.0


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


PRESETS = {
    # BASELINE.json configs: (need, total, object MiB, objects per GPU, global objects, erased)
    "c2": (4, 6, 64, 32, 0, "0,1"),
    "c3": (8, 12, 256, 128, 0, "0,1,2,3"),
    "c5": (10, 14, 1024, 0, 64, "0,1,2,3"),  # 64 objects partitioned over the ranks (strong)
    "ns64": (8, 12, 512, 64, 0, "0,1,2,3"),  # north star's "64 MiB shards"
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node, one rank each.  Without a torchrun environment (WORLD_SIZE unset) "
                         "and N > 1, bench.py starts the N ranks itself before anything touches a GPU")
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None,
                    help="a BASELINE config: c2 (4/6, 32 x 64 MiB), c3 (8/12, 128 x 256 MiB, the default shape), "
                         "c5 (10/14, 64 x 1 GiB partitioned over the ranks), ns64 (8/12, 64 x 512 MiB)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rendezvous only: every rank reports its object partition, no GPU work "
                         "(tests the N-rank launch on a machine without GPUs)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--total", type=int, default=12)
    ap.add_argument("--objects", type=int, default=128, help="objects per GPU (C3/C4: 128; weak scaling)")
    ap.add_argument("--global-objects", type=int, default=0,
                    help="partition this many objects across ranks instead (strong scaling, e.g. C5: 64)")
    ap.add_argument("--object-mib", type=int, default=256, help="object size in MiB (C3/C4: 256)")
    ap.add_argument("--erase", type=str, default="0,1,2,3", help="erased shards for the decode leg")
    ap.add_argument("--decode-dst", choices=["inplace", "separate"], default="inplace",
                    help="rebuild into the erased slots of each object (repair) or into a separate buffer")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle CPU path on rank 0 at N=1")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="wall time budget of the CPU sample")
    ap.add_argument("--c5-leg", type=int, default=1,
                    help="also run BASELINE config 5 (10/14, 64 x 1 GiB partitioned over the ranks, encode + "
                         "decode {0,1,2,3}) and report it as c5_partitioned")
    ap.add_argument("--bytes-path", type=int, default=1,
                    help="also time the fused object-bytes pipeline (MapToGF+encode+MapFromGF, repair)")
    ap.add_argument("--c5-bytes", type=int, default=1,
                    help="also time the fused object-bytes pipeline at BASELINE config 5's shape per GPU: 10/14, "
                         "16 x 1 GiB objects on 256 B-aligned chunk strides (object_bytes_path_c5)")
    ap.add_argument("--ceilings", type=int, default=1,
                    help="measure torch copy/fill HBM rates after the timed region (roofline.measured_streams)")
    ap.add_argument("--host-path", type=int, default=1,
                    help="rank 0 at N=1: PCIe-inclusive writeChunks/reconstruct from host memory (never `value`)")
    ap.add_argument("--host-order", choices=["before-free", "after-free"], default="before-free",
                    help="run the host leg before the device buffers are freed (default) or after the bytes leg "
                         "freed them: the driver then wipes the freed VRAM with the same DMA engines the host "
                         "path uses, which slows its transfers for seconds (DESIGN.md, End-to-end)")
    ap.add_argument("--host-delay", type=float, default=0.0, help="seconds to wait before the host leg")
    ap.add_argument("--pooled", type=int, default=1,
                    help="at every N: rank 0 drives the host entry points as one proxy does (--pool-threads "
                         "concurrent PUT + GET requests, SLIME_RS_ANY_DEVICE) over the GPUs of all N ranks, the "
                         "other ranks parked at a barrier; reported as host_path.pooled (never `value`)")
    ap.add_argument("--pool-threads", type=int, default=25,
                    help="concurrent requests of the pooled leg (slime's --parallel-requests default, main.go:107-109)")
    ap.add_argument("--pool-seconds", type=float, default=2.0, help="timed seconds per pooled workload")
    ap.add_argument("--allocator", choices=["vmm", "torch"], default="vmm",
                    help="batch buffers from slime_rs_device_alloc (physical chunks mapped into one range: the "
                         "placement the kernels stream well from, DESIGN.md 'Placement modes') or torch.empty "
                         "(hipMalloc through the caching allocator)")
    ap.add_argument("--alloc-probe", type=int, default=1,
                    help="with --allocator vmm: also time 3 encodes and decodes of the same batch in a torch.empty "
                         "(hipMalloc) buffer, reported as allocator_probe (not value)")
    ap.add_argument("--chunk-align", type=int, default=256,
                    help="byte path: chunk stride alignment in bytes (256: every chunk on a line boundary, the "
                         "device slot layout; 1: the wire layout, chunks 4L apart)")
    ap.add_argument("--shard-align", type=int, default=64,
                    help="device shard stride rounded up to this many symbols (64 = 256 B: every shard "
                         "starts on a cache-line boundary; 1 = packed, stride L)")
    ap.add_argument("--traffic", type=str,
                    default=",".join(os.path.join(ROOT, "profiles", r, "pmc_traffic.json") for r in ("r06", "r05", "r04")),
                    help="PMC-derived HBM bytes per launch, comma-separated files (tools/pmc_traffic.py over "
                         "rocprofv3 --pmc passes; an entry is used only when its config and the kernel's machine "
                         "code match this build)")
    ap.add_argument("--shape-legs", type=str, default="c2,ns64",
                    help="after the timed region, also time these BASELINE shapes per GPU (weak), each in the "
                         "main batch's buffer re-laid (no allocation): c2 (4/6, 32 x 64 MiB), ns64 (8/12, "
                         "64 x 512 MiB, the north star's 64 MiB shards); '' for none")
    args = ap.parse_args(argv)
    if args.preset:
        given = {a.split("=")[0] for a in (argv if argv is not None else sys.argv[1:]) if a.startswith("--")}
        need, total, mib, per_gpu, glob, erase = PRESETS[args.preset]
        for key, val in (("need", need), ("total", total), ("object_mib", mib), ("objects", per_gpu or 128),
                         ("global_objects", glob), ("erase", erase)):
            if "--" + key.replace("_", "-") not in given:  # explicit flags win over the preset
                setattr(args, key, val)
    return args


# ---- N-rank launch without torchrun ---------------------------------------------

def kfd_gpus(base: str = "/sys/class/kfd/kfd/topology/nodes", dri: str = "/dev/dri") -> int:
    """GPUs this process may open, counted from the KFD topology in sysfs
    (nodes with SIMDs whose DRM render node is accessible), narrowed by
    ROCR/HIP/CUDA_VISIBLE_DEVICES.  Reads files only: it never starts the HIP
    runtime, so the launcher below can count devices before spawning ranks."""
    try:
        nodes = sorted((d for d in os.listdir(base) if d.isdigit()), key=int)
    except OSError:
        return 0
    n = 0
    for nd in nodes:
        props = {}
        try:
            for line in open(os.path.join(base, nd, "properties")):
                kv = line.split()
                if len(kv) == 2:
                    props[kv[0]] = kv[1]
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        minor = props.get("drm_render_minor")
        if minor is not None and not os.access(f"{dri}/renderD{minor}", os.R_OK | os.W_OK):
            continue  # a GPU of this node that this container may not open
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def visible_gpus() -> int:
    """GPUs this process may use (kfd_gpus).  SLIME_BENCH_DEVICE_COUNT stands
    in for it under --dry-run only (tests)."""
    fake = os.environ.get("SLIME_BENCH_DEVICE_COUNT")
    if fake is not None and "--dry-run" in sys.argv[1:]:
        return int(fake)
    return kfd_gpus()


def shared_gpu_rehearsal() -> bool:
    """SLIME_BENCH_SHARE_GPU=1: let more ranks than GPUs share them (rank r on
    GPU r % n) -- a rehearsal of the multi-rank path on a 1-GPU box, never a
    scaling number: the line then says "rehearsal" and n_gpus counts the
    distinct GPUs actually used."""
    return os.environ.get("SLIME_BENCH_SHARE_GPU") == "1"


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) outside torchrun: start N copies of this script, one
    per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1),
    as child processes -- this parent never touches a GPU and never execs.
    Rank 0's JSON line is the output; the exit status is the first failing
    rank's (the other ranks are then stopped: they would wait at a barrier)."""
    import subprocess
    ndev = visible_gpus()
    if args.gpus > ndev and not shared_gpu_rehearsal():
        print(f"bench.py: --gpus {args.gpus} but {ndev} visible GPU(s); one rank per GPU", file=sys.stderr, flush=True)
        return 2
    env = dict(os.environ, WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = []
    for r in range(args.gpus):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(args.gpus))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    import signal

    def stop(signum, _frame):  # the launcher is being stopped: stop the ranks it started, then exit
        for q in procs:
            if q.poll() is None:
                q.terminate()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # the exact children this launcher started
                    q.terminate()
        time.sleep(0.05)
    return rc


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cgroup_cpus() -> float | None:
    """CPU quota of this process's cgroup (cpu.max), in CPUs; None if unlimited/unknown."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        return None


def _mem_available() -> int:
    """MemAvailable of this host in bytes (16 GiB if unreadable)."""
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) << 10
    except (OSError, ValueError, IndexError):
        pass
    return 16 << 30


def _cpu_leg(OC, sample, need: int, total: int, have: list[int], threads: int, seconds: float) -> dict:
    """`threads` host threads, each on its own copy of the sample object, each
    running the reference's per-object path until ~`seconds` of wall time: r
    CreateParity passes (multi_store.go:528-531 -> vector.go:18-41) and one
    RecoverData recomputing all need rows (vector.go:50-88, multi_store.go:237)
    on the oracle's C restatement (uint64 products, `%`p twice per term,
    vector.go:97).  Returns the rate and thread 0's first outputs."""
    import threading

    import numpy as np

    L = sample.shape[1]
    objs = []
    for _ in range(threads):
        o = np.zeros((total, L), dtype=np.uint32)
        o[:need] = sample[:need]  # the data shards; parity rows are recomputed
        objs.append(o)
    reps = [0] * threads
    first = {}
    deadline = time.perf_counter() + seconds

    def work(t, o):
        while True:
            OC.encode_object(o, need, total)
            rc, rec = OC.recover_data([o[i] for i in have], have)
            assert rc == 0
            if t == 0 and not first:
                first["parity"] = o[need:].copy()
                first["data"] = rec
            reps[t] += 1
            if time.perf_counter() >= deadline:
                return

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work, args=(i, o)) for i, o in enumerate(objs)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    nbytes = 2 * sum(reps) * need * L * 4  # encode + decode of each object pass (L columns)
    return {"value": round(nbytes / GIB / dt, 4), "unit": "GiB/s", "cores": threads,
            "object_passes": sum(reps), "seconds": round(dt, 2), "_first": first}


def _matrix_cores(k: int, rows: int) -> bool:
    """Whether the library runs this shape on its matrix-core kernels (the rule
    in rs_apply_mfma.hip mfma_wanted: k >= 33, or 17 <= k <= 32 with k x rows
    >= 128; at most 32 output rows and k <= 112) -- for the line's labels."""
    from slime_amd import _native as N
    if N.lib.slime_rs_kernel_matrix_cores(-1) != 1 or rows > 32 or k > 112 or rows < 1:
        return False
    return k >= 33 or (k >= 17 and k * rows >= 128)


def cpu_baseline(sample, sample_name: str, need: int, total: int, erase: list[int], seconds: float,
                 samples: dict | None = None) -> dict:
    """The reference's algorithm on host cores, on the
    bench's own input: `sample` is one object of the timed batch copied out of
    HBM after the timed steps (total x L symbols: its data shards and the
    parity the GPU wrote).  The oracle's faithful C restatement runs one object
    per thread, as the reference does (the RS math is single-threaded per
    object, multi_store.go:528-531), on 1 thread and on every core this
    process may run on.  `value` is the all-core figure; `verified`: the CPU's
    parity equals the GPU's for that object and its RecoverData gives back
    the data shards."""
    import numpy as np

    from oracle import oracle_c as OC

    have = [i for i in range(total) if i not in erase][:need]
    t_pin = time.perf_counter()
    pin = oracle_pin(samples or {})
    pin_s = time.perf_counter() - t_pin
    # Every core this process may run on: its affinity set, capped by its
    # cgroup's CPU quota when there is one (a 1-GPU share of the GPU box sees
    # 256 CPUs but may use 16; more threads than that only time-slice).
    affinity = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    ncores = max(1, min(affinity, int(quota))) if quota else affinity
    one = _cpu_leg(OC, sample, need, total, have, 1, seconds * 0.4)
    first = one.pop("_first")
    ok = bool(np.array_equal(first["parity"], sample[need:])) and \
        all(np.array_equal(first["data"][t], sample[t]) for t in range(need))
    # The all-core leg gives every thread its own copy of the object and of
    # RecoverData's outputs ((total + need) x 4 bytes per column): on a host
    # with many cores and no quota that is far more memory than the sample.
    # Threads take a column slice of the sample instead (the rate is per byte),
    # sized so that all copies fit in min(8 GiB, a quarter of MemAvailable).
    L = sample.shape[1]
    budget = min(8 << 30, _mem_available() // 4)
    cols = max(4096, min(L, budget // (ncores * (total + need) * 4))) & ~63
    cols = min(cols, L)
    allc = _cpu_leg(OC, np.ascontiguousarray(sample[:, :cols]), need, total, have, ncores, seconds * 0.6)
    allc.pop("_first")
    allc["columns_per_thread"] = int(cols)
    mib = sample.shape[1] * need * 4 / (1 << 20)
    # Small objects (a proxy's small requests): the same per-object path on one
    # thread, per call, on the first columns of the sample (the shards of an
    # S-byte object), beside host_path.latency's GPU calls.
    small = []
    for kib in (4, 64, 1024):
        Ls = -(-(kib << 10) // 4 // need)
        o = np.ascontiguousarray(sample[:, :Ls])
        OC.object_reps(o, need, total, have, 1)  # warm
        reps = max(1, int(0.2 / max(1e-6, Ls * need * (total - need + need) * 2e-9)))
        t0 = time.perf_counter()
        rec = OC.object_reps(o, need, total, have, reps)
        dt = time.perf_counter() - t0
        ok = ok and all(np.array_equal(rec[t], sample[t, :Ls]) for t in range(need))
        small.append({"object_kib": kib, "encode_plus_recover_us": round(dt / reps * 1e6, 2), "calls": reps})
    return {"value": allc["value"], "unit": "GiB/s", "cores": ncores, "kind": "port",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cores": affinity,
            "cgroup_cpu_quota": quota, "verified": ok,
            "oracle_pin": pin, "oracle_pin_seconds": round(pin_s, 2),
            "single_thread": one, "all_cores": allc,
            "small_objects_one_thread": {"sizes": small,
                                         "what": "per object, in C with the reference's matrix cache: r "
                                                 "one-row CreateParity calls + RecoverData (inverse per call), "
                                                 "1 thread -- the RS math only (the reference also runs MapToGF / "
                                                 "MapFromGF byte passes); compare host_path.latency (GPU, bytes "
                                                 "in and out)"},
            "sample": f"{sample_name} ({mib:.0f} MiB of data shards, copied from HBM after the timed steps), "
                      f"need={need} total={total}: per object, r CreateParity passes (multi_store.go:528-531) + "
                      f"RecoverData(erase {erase}) recomputing all need rows (vector.go:80-85); 1 thread "
                      f"({one['object_passes']} passes in {one['seconds']} s) and {ncores} threads on copies of it "
                      f"({allc['object_passes']} passes over the first {allc['columns_per_thread']} columns in "
                      f"{allc['seconds']} s); oracle/rs_oracle.c, gcc -O2; "
                      "verified = the CPU's parity equals the GPU's for this object and RecoverData returns its data"}


def batch_empty(args, numel: int, dtype: torch.dtype, dev: int) -> torch.Tensor:
    """A device batch buffer: slime_rs_device_alloc (default) or torch.empty."""
    if args.allocator == "vmm":
        return D.device_empty(numel, dtype, dev)
    return torch.empty(numel, dtype=dtype, device=f"cuda:{dev}")


ORACLE_COLS = 4096  # columns per object pinned to the oracle (plus the last column)


def column_sample(v3: torch.Tensor, L: int, seed: int, ncols: int = ORACLE_COLS) -> dict:
    """Columns of every object of a batch for the oracle pin (oracle_pin, run
    inside the cpu_baseline leg): a window of `ncols` consecutive columns at a
    per-object seeded offset, plus the last column L-1, gathered on the
    device from v3 = [object][row][column] int32 words and copied to the host.
    A copy only: nothing here computes."""
    import numpy as np

    nobj, rows, _ = v3.shape
    w = min(ncols, L)
    g = torch.Generator().manual_seed(seed)
    off = torch.randint(0, L - w + 1, (nobj,), generator=g)
    idx = torch.cat([off[:, None] + torch.arange(w)[None, :], torch.full((nobj, 1), L - 1)], dim=1)
    cols = torch.gather(v3, 2, idx.to(v3.device)[:, None, :].expand(nobj, rows, w + 1))
    return {"cols": cols.cpu().numpy().view(np.uint32), "offsets": off.tolist(), "window": w, "L": L}


def oracle_pin(samples: dict) -> dict:
    """Every object of every timed batch against the reference's arithmetic
    (oracle/rs_oracle.c: vector.go:90-102 applyMatrix, :50-88 RecoverData), on
    the sampled columns: the parity rows equal the oracle's encode of the data
    rows, and the oracle's RecoverData from the survivors (the first `need`
    available rows, multi_store.go:218-235) returns the data rows -- the
    erased ones as the timed decode rebuilt them.  Byte batches are taken
    back to symbols with the object's mapping first (MapToGFWith, map.go:74-98:
    big-endian words XOR the mapping); the mapping choice itself is pinned by
    tests/test_gpu_fullsize.py.  Runs only inside the cpu_baseline leg."""
    import numpy as np

    from oracle import oracle_c as OC

    out = {}
    for name, smp in samples.items():
        need, total, have = smp["need"], smp["total"], smp["have"]
        cols = smp["cols"]
        good = 0
        for o in range(cols.shape[0]):
            sym = cols[o]
            if smp.get("mapping") is not None:
                sym = sym.byteswap() ^ np.uint32(smp["mapping"][o])
            sym = np.ascontiguousarray(sym, dtype=np.uint32)
            enc = np.zeros_like(sym)
            enc[:need] = sym[:need]
            OC.encode_object(enc, need, total)
            rc, rec = OC.recover_data([sym[i] for i in have], have)
            if rc == 0 and np.array_equal(enc[need:], sym[need:]) and \
                    all(np.array_equal(rec[t], sym[t]) for t in range(need)):
                good += 1
        out[name] = {"objects": int(cols.shape[0]), "verified_objects": good,
                     "columns_per_object": int(cols.shape[2]), "window": smp["window"],
                     "includes_last_column": True, "domain": "bytes" if smp.get("mapping") is not None else "symbols"}
    return out


ALLOCATOR_NOTE = {"vmm": "slime_rs_device_alloc: HIP virtual memory, physical chunks mapped in order",
                  "torch": "torch.empty (hipMalloc via the caching allocator)"}


def bytes_leg(args, dev: int, rank: int, need: int, total: int, erase: list[int], nobj: int, mib: int | None = None,
              samples: dict | None = None, tag: str = "bytes") -> dict:
    """writeChunks / reconstruct on device from object bytes (rs_bytes.hip): one
    speculative encode pass that also picks gf.MapToGF's mapping (switching an
    object to 1<<31 once one of its words >= p has been seen), a redo pass over
    the units encoded before that, and an in-place repair of the erased chunks
    from chunk bytes.  Objects that would need MapToGF's random
    fallback are re-drawn before timing and counted.  A HIP
    event recorded by the library between the two encode passes
    (slime_rs_encode_objects_phased) splits the encode time into the
    speculative pass and the 1<<31 re-encode.  `samples`: where to leave the
    column sample of every object for the oracle pin (cpu_baseline leg)."""
    import numpy as np

    S = (mib or args.object_mib) << 20
    L, cs, slot = D.slot_geometry(S, need, total, chunk_align=args.chunk_align)
    chunk_stride = cs if args.chunk_align > 1 else 0
    slots = batch_empty(args, nobj * slot, torch.uint8, dev)
    placement = D.placement(slots) if args.allocator == "vmm" else None
    words = slots.view(torch.int32)
    D.fill_symbols(words, 0xB17E5 + 7919 * rank)
    enc = D.Plan.encode(need, total, dev)
    have = [i for i in range(total) if i not in erase][:need]
    dec = D.Plan.reconstruct(need, total, have, erase, dev).set_outputs(erase)
    mapping = torch.empty(nobj, dtype=torch.int32, device=f"cuda:{dev}")
    status = torch.empty(nobj, dtype=torch.int32, device=f"cuda:{dev}")
    stream = torch.cuda.current_stream(dev)
    redraws = 0
    for attempt in range(64):
        D.encode_objects(enc, slots, slot, S, nobj, mapping, status, stream, chunk_stride)
        bad = status.nonzero().flatten().tolist()
        if not bad:
            break
        for o in bad:  # re-draw the object from another seed
            D.fill_symbols(words[o * slot // 4:(o * slot + need * cs) // 4], 0xB17E5 + (attempt + 1) * 2**32 + o)
        redraws += len(bad)

    def erased():
        return slots.view(nobj, slot)[:, : total * cs].view(nobj, total, cs)[:, erase, : 4 * L]

    truth = erased().clone()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        D.encode_objects(enc, slots, slot, S, nobj, mapping, status, stream, chunk_stride,
                         phase_event=None if ev is None else ev[3])
        if ev is not None:
            ev[1].record(stream)
        D.decode_objects(dec, slots, slot, L, nobj, mapping, stream, chunk_stride)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    for e in events:  # torch creates an event at its first record; the library records e[3] again mid-encode
        e[3].record(stream)
    batch.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    batch.barrier()
    elapsed = time.perf_counter() - t0
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    pass0_ms = sum(e[0].elapsed_time(e[3]) for e in events) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps
    ok = bool(torch.equal(erased(), truth)) and int(status.sum().item()) == 0
    ms = mapping.cpu().numpy().view("uint32")
    if samples is not None:
        smp = column_sample(words.view(nobj, slot // 4)[:, : total * cs // 4].view(nobj, total, cs // 4), L,
                            0x5A3D + need)
        smp.update(need=need, total=total, have=have, mapping=ms.copy())
        samples[tag] = smp
    elapsed, bad_ranks = batch.max_over_ranks([elapsed, 0.0 if ok else 1.0])
    world = dist.get_world_size() if dist.is_initialized() else 1
    del slots, words, truth
    torch.cuda.empty_cache()
    # Roofline of each leg (SURVEY.md §8(d) algorithmic bytes: encode 4L(k+r),
    # decode 4L(k+e) per object) over its kernel time, and the PMC traffic of
    # the same kernels' machine code when a committed summary has it.
    alg_enc = nobj * 4 * L * total
    alg_dec = nobj * 4 * L * (need + len(erase))
    kernels = {"encode": ["encode_bytes_queue_kernel", "encode_bytes_redo_kernel"], "decode": ["decode_bytes_queue_kernel"]}
    if _top_bits(need, S):  # the second pass corrects from top bits (rs_bytes_launch.hpp)
        kernels["encode"] = ["encode_bytes_queue_bits_kernel", "encode_bytes_fix_kernel", "encode_bytes_redo_kernel"]
    if _matrix_cores(need, total - need) and need >= 25:
        kernels["encode"] = ["encode_bytes_mfma_kernel"]
    if _matrix_cores(need, len(erase)):
        kernels["decode"] = ["decode_bytes_mfma_kernel"]
    replay = _bytes_traffic(args, f"{need}/{total} S={S} nobj={nobj} cs={cs}", need, kernels)

    def leg(what, alg, ms):
        ach = alg / (ms * 1e-3) / 1e9
        t = replay.get(what)
        return {"kernels": [f"{k}<{need},...>" for k in kernels[what]], "alg_bytes": alg,
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": t, "traffic_over_alg": round(t / alg, 4) if t else None}
    # value: every rank's objects (weak: nobj per GPU) over the slowest rank's time.
    return {"value": round(2 * nobj * world * S * args.steps / GIB / elapsed, 2), "unit": "GiB/s",
            "scaling": "weak", "n_ranks": world,
            "config": f"need={need} total={total}, {S >> 20} MiB objects x {nobj} per GPU, chunk stride {cs} B; "
                      f"encode (both passes) + repair erased {erase}",
            "encode_gibs": round(nobj * S / GIB / (enc_ms * 1e-3), 2),
            "decode_gibs": round(nobj * S / GIB / (dec_ms * 1e-3), 2),
            "kernel_ms": {"encode_both_passes": round(enc_ms, 4), "encode_pass0": round(pass0_ms, 4),
                          "encode_redo": round(enc_ms - pass0_ms, 4), "decode": round(dec_ms, 4)},
            "redo_share": round((enc_ms - pass0_ms) / enc_ms, 4) if enc_ms else None,
            "roofline": {"encode": leg("encode", alg_enc, enc_ms), "decode": leg("decode", alg_dec, dec_ms),
                         "traffic_source": replay.get("source")},
            "mappings": {"0": int((ms == 0).sum()), "1<<31": int((ms == 0x80000000).sum()),
                         "other": int(((ms != 0) & (ms != 0x80000000)).sum())},
            "fallback_redraws": redraws, "verified": bad_ranks == 0.0, "placement": placement,
            "chunk_stride": cs, "chunk_bytes": 4 * L,
            "second_pass": "top-bit correction" if _top_bits(need, S) else "re-encode",
            "what": "object bytes in HBM -> MapToGF + encode + MapFromGF (speculative pass that switches an object "
                    "to 1<<31 once a word >= p is seen, then a redo of the units encoded before: re-encoded, or "
                    "corrected from the top bits the first pass stored, second_pass) and repair of "
                    "erased chunks from chunk bytes; encode_pass0 / encode_redo split at a HIP event the library "
                    "records between the passes (the redo includes its list build and the 1<<31 edge columns)"}


def _top_bits(need: int, S: int) -> bool:
    """Whether the fused encode's second pass corrects the switched units from
    top bits (slime_rs_switch_bits: mode 0 = objects >= 1 GiB at need <= 10)."""
    mode = D.N.lib.slime_rs_switch_bits(-1)
    return need <= 10 and (mode == 1 or (mode == 0 and S >= 1 << 30))


def _bytes_traffic(args, config: str, need: int, kernels: dict) -> dict:
    """PMC bytes per step of the byte path's kernels at `config`, replayed from
    profiles/r06/pmc_bytes.json (then r04's) only where every kernel's machine
    code matches this build (slime_amd/codeobj.py); {} otherwise."""
    for rnd in ("r06", "r04"):
        path = os.path.join(ROOT, "profiles", rnd, "pmc_bytes.json")
        try:
            entries = json.load(open(path))
        except (OSError, ValueError):
            continue
        for e in (x for x in entries if x.get("config") == config):
            ks = e.get("kernels", {})
            out = {}
            for what, names in kernels.items():
                if not all(n in ks and ks[n].get("kernel_code") == kernel_code_id(D.N.LIB_PATH, (f"{n}ILi{need}E",))
                           for n in names):
                    break
                out[what] = sum(ks[n]["hbm_bytes"] for n in names)
            else:
                out["source"] = (f"replayed: profiles/{rnd}/pmc_bytes.json (session {e.get('session', '?')}, "
                                 "matching machine code)")
                return out
    return {}


def host_leg(need, total, erase, obj_mib=64, reps=5):
    """PCIe-inclusive object rate from host memory (HTTP bodies <= 64 MiB), on
    caller-reused buffers, median of `reps`.  Reported beside the
    device-resident `value`, never as it.

    Two callers are timed.  The fused object entry points (write_chunks /
    reconstruct: one device pass each) need writeChunks/reconstruct to call
    them.  The UNCHANGED caller (multi_store.go as it is) issues the Go API
    call by call: MapToGF, splitVector, r CreateParity calls (each uploads all
    need data shards again, :528-531) and a MapFromGF per chunk (:554) on
    write; MapToGFWith per survivor (:224), RecoverData (:237) and MapFromGF
    per data row (:239) on read."""
    import numpy as np
    from slime_amd import _native as N
    from slime_amd import gf, objects, rs
    rng = np.random.default_rng(0x5113E)
    data = rng.integers(0, 256, size=obj_mib << 20, dtype=np.uint8)
    cb = objects.chunk_size(data.size, need)
    chunks = [np.zeros(cb, dtype=np.uint8) for _ in range(total)]
    out = np.zeros(data.size, dtype=np.uint8)
    have = [i for i in range(total) if i not in erase][:need]
    r = total - need

    last_split = {}

    def med(fn):
        """Median wall time of `reps` calls after a warm one; last_split gets the
        pipeline split (slime_rs_host_stats) of the median call itself."""
        fn()
        N.host_stats(reset=True)  # the pipeline split covers the timed calls only
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0, N.host_stats(reset=True)))
        t, st = sorted(ts, key=lambda x: x[0])[len(ts) // 2]
        last_split.clear()
        last_split.update(st)
        return t

    def split(st):  # ms per call of the windowed pipeline, from slime_rs_host_stats
        c = max(1, st["calls"])
        return {k[:-3] + "_ms": round(st[k] / 1e3 / c, 3) for k in ("copy_in_us", "enqueue_us", "wait_us",
                                                                      "copy_out_us", "total_us")}

    box = {}
    t_w = med(lambda: box.update(m=objects.write_chunks(data, need, total, out=chunks)[0]))
    split_w = split(last_split)
    t_wz = med(lambda: objects.write_chunks(data, need, total, out=chunks, alias=True))
    surv = [chunks[i] for i in have]
    t_r = med(lambda: objects.reconstruct(surv, have, box["m"], data.size, out=out))
    split_r = split(last_split)
    ok = bool(np.array_equal(out, data))

    # The unchanged caller, call by call (Go API mirrors, slime_amd.rs / .gf).
    m, words = gf.MapToGF(data)
    parts = objects.split_vector(words, need)
    par = [np.zeros(parts[0].size, dtype=np.uint32) for _ in range(r)]
    t_cp = med(lambda: [rs.CreateParity(parts, need + i, par[i]) for i in range(r)])
    sym = [gf.MapToGFWith(chunks[i], m) for i in have]
    rec = [np.zeros(sym[0].size, dtype=np.uint32) for _ in range(need)]
    t_rd = med(lambda: rs.RecoverData(sym, have, rec))
    unchanged = unchanged_caller(data, need, total, have, chunks, m, box["m"], max(7, reps))
    with_device_codec = None
    prev = gf.codec_placement(1)
    try:  # the same caller with the codec through the GPU (round 3's form), for comparison
        u = unchanged_caller(data, need, total, have, chunks, m, box["m"], 3)
        with_device_codec = {"write_gibs": u["write_gibs"], "read_gibs": u["read_gibs"],
                             "split_ms": {"write": u["write"]["split_ms"], "read": u["read"]["split_ms"]},
                             "verified": u["verified"]}
    finally:
        gf.codec_placement(prev)
    par2 = [np.zeros(parts[0].size, dtype=np.uint32) for _ in range(r)]
    t_cps = med(lambda: rs.CreateParities(parts, total, par2))
    g = lambda t: round(data.size / GIB / t, 2)  # noqa: E731
    digests = digest_leg(data, need, total, chunks, have, out, med, g)
    latency = latency_leg(need, total, erase)
    return {"write_chunks_gibs": g(t_w), "reconstruct_gibs": g(t_r), "write_chunks_zero_copy_gibs": g(t_wz),
            "link": link_probe(obj_mib),
            "pipeline_split": {"write_chunks": split_w, "reconstruct": split_r,
                               "what": "the median call's split: host copies in/out, launches, waits on the device/link side "
                                       "(a large wait with normal copies = DMA contention, DESIGN.md End-to-end)"},
            "unchanged_caller": dict(unchanged, create_parity_x_r_gibs=g(t_cp),
                                     create_parities_batched_gibs=g(t_cps), recover_data_reused_out_gibs=g(t_rd),
                                     with_device_codec=with_device_codec),
            "digests": digests,
            "latency": latency,
            "object_mib": obj_mib, "erased": erase, "verified": ok,
            "what": "host bytes -> pinned 3-stage ring -> fused byte kernels -> host chunk bytes (and back), "
                    "PCIe-inclusive; not `value`"}


def latency_leg(need, total, erase, sizes_kib=(4, 64, 1024, 8192), reps=25) -> dict:
    """Per-call latency from host memory at request-body sizes (a proxy serves
    objects of every size, main.go:107-109): median and p90 microseconds of the
    fused write_chunks / reconstruct and of the unchanged Go API's
    CreateParity (one row) / RecoverData, caller-reused outputs.  `c_abi`
    calls the C entry points with their argument arrays built once, as the cgo
    shim holds them (what a Go caller waits); `python` goes through the Python
    mirror (slime_amd.objects / rs), whose argument marshalling adds ~15 us."""
    import ctypes
    import numpy as np
    from slime_amd import _native as N
    from slime_amd import gf, objects, rs
    lib = N.lib
    have = [i for i in range(total) if i not in erase][:need]
    pc = time.perf_counter

    def stats(fn):
        fn()
        ts = []
        for _ in range(reps):
            t0 = pc()
            fn()
            ts.append(pc() - t0)
        ts.sort()
        return {"p50_us": round(ts[len(ts) // 2] * 1e6, 1), "p90_us": round(ts[(9 * len(ts)) // 10] * 1e6, 1)}

    def ptrs(arrs):
        return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])

    def checked(rc):
        if rc:
            raise RuntimeError(f"latency leg: status {rc}")

    rows, ok = [], True
    rng = np.random.default_rng(0x1A7)
    for kib in sizes_kib:
        data = rng.integers(0, 256, size=kib << 10, dtype=np.uint8)
        S = data.size
        cb = objects.chunk_size(S, need)
        chunks = [np.zeros(cb, dtype=np.uint8) for _ in range(total)]
        out = np.zeros(S, dtype=np.uint8)
        m_box = ctypes.c_uint32(0)
        # C-ABI, arguments prepared once (a cgo caller's marshalled slices)
        p_data, p_chunks, p_out = data.ctypes.data, ptrs(chunks), out.ctypes.data
        surv = [chunks[i] for i in have]
        p_surv, p_have = ptrs(surv), (ctypes.c_int * need)(*have)
        c_w = stats(lambda: checked(lib.slime_rs_write_chunks(p_data, S, need, total, p_chunks, ctypes.byref(m_box))))
        m = int(m_box.value)
        c_r = stats(lambda: checked(lib.slime_rs_reconstruct(p_surv, p_have, need, cb, m, S, p_out)))
        ok = ok and bool(np.array_equal(out, data))
        mm, words = gf.MapToGF(data)
        parts = objects.split_vector(words, need)
        L = parts[0].size
        par = np.zeros(L, dtype=np.uint32)
        p_parts, lens = ptrs(parts), (ctypes.c_uint64 * need)(*([L] * need))
        c_cp = stats(lambda: checked(lib.slime_rs_create_parity(p_parts, lens, need, need, par.ctypes.data)))
        sym = [gf.MapToGFWith(chunks[i], m) for i in have]
        rec = [np.zeros(L, dtype=np.uint32) for _ in range(need)]
        p_sym, p_rec = ptrs(sym), ptrs(rec)
        c_rd = stats(lambda: checked(lib.slime_rs_recover_data(p_sym, lens, need, p_have, need, p_rec)))
        ok = ok and all(np.array_equal(rec[i], parts[i]) for i in range(need))
        # the Python mirror, call by call
        box = {}
        w = stats(lambda: box.update(m=objects.write_chunks(data, need, total, out=chunks)[0]))
        rc = stats(lambda: objects.reconstruct(surv, have, box["m"], S, out=out))
        ok = ok and bool(np.array_equal(out, data)) and mm == m == box["m"]
        cp = stats(lambda: rs.CreateParity(parts, need, par))
        rd = stats(lambda: rs.RecoverData(sym, have, rec))
        ok = ok and all(np.array_equal(rec[i], parts[i]) for i in range(need))
        rows.append({"object_kib": kib,
                     "c_abi": {"write_chunks": c_w, "reconstruct": c_r, "create_parity_one_row": c_cp,
                               "recover_data": c_rd},
                     "python": {"write_chunks": w, "reconstruct": rc, "create_parity_one_row": cp,
                                "recover_data": rd}})
    return {"sizes": rows, "reps": reps, "erased": erase, "verified": ok,
            "what": "wall time per host call (host bytes in, host bytes out, PCIe and launch included), "
                    "median and 90th percentile; c_abi: the C entry points with argument arrays built once "
                    "(the cgo shim's view); python: the Python mirror"}


def unchanged_caller(data, need, total, have, chunks, m, m_fused, reps) -> dict:
    """multi_store.go as it is, call by call through the Go-API mirrors, on
    fresh outputs (Go's make).  writeChunks = MapToGF (:526) + splitVector
    (:527) + r CreateParity (:528-531) + a MapFromGF per chunk, each on its
    own goroutine (:552-554: here one thread per part, all concurrent).
    reconstruct's slow path = make([]byte, 0, Size+16) (:204) + MapToGFWith
    per survivor (:224) + RecoverData (:237) + MapFromGF per data row
    appended in order (:238-241).  `reps` timed calls of each after a warm
    one: total min / median / max, every phase of every rep, and the median
    call's split with `other` = total - the phases (Python between the
    calls).  fresh_alloc_alone_ms: the same fresh outputs allocated and first
    touched by one thread, timed on their own -- NOT part of the total; it
    says how much of the phases is Go's make() (page faults).  Each rep also
    records the process's page faults during the call and the time to drop
    its intermediate buffers afterwards (deferred_free_ms, off the clock)."""
    import concurrent.futures as cf
    import resource

    import numpy as np
    from slime_amd import _native as N
    from slime_amd import gf, objects, rs
    r = total - need
    pc = time.perf_counter
    goroutines = cf.ThreadPoolExecutor(max_workers=total)  # one per part, as writeChunks' go statements

    # Every phase's intermediate buffers are handed back in `garbage` and
    # dropped after the call's clock stops: Go's collector frees them off the
    # request path, while CPython would munmap them (several ms per 64 MiB)
    # inside the call.  The drop is timed on its own (deferred_free_ms).
    def write(garbage):
        t0 = pc()
        mm, w = gf.MapToGF(data)
        t1 = pc()
        ps = objects.split_vector(w, need)
        t2 = pc()
        pv = [rs.CreateParity(ps, need + i) for i in range(r)]
        t3 = pc()
        out = list(goroutines.map(lambda p: gf.MapFromGF(mm, p), ps + pv))
        t4 = pc()
        garbage.extend([w, ps, pv])
        return (mm, out), [("map_to_gf", t1 - t0), ("split_vector", t2 - t1), (f"create_parity_x{r}", t3 - t2),
                           (f"map_from_gf_x{total}_concurrent", t4 - t3)]

    def read(garbage):
        t0 = pc()
        buf = np.empty(data.size + 16, dtype=np.uint8)  # make([]byte, 0, Size+16) (:204)
        t1 = pc()
        cs = [gf.MapToGFWith(chunks[i], m) for i in have]
        t2 = pc()
        vs = rs.RecoverData(cs, have)
        t3 = pc()
        o = 0
        for v in vs:
            b = gf.MapFromGF(m, v)
            n = min(len(b), buf.size - o)
            buf[o:o + n] = np.frombuffer(b, dtype=np.uint8, count=n)
            o += n
            garbage.append(b)
        t4 = pc()
        garbage.extend([cs, vs])
        return buf[:data.size], [("make_output", t1 - t0), (f"map_to_gf_with_x{need}", t2 - t1),
                                 ("recover_data", t3 - t2), (f"map_from_gf_append_x{need}", t4 - t3)]

    def faults():
        ru = resource.getrusage(resource.RUSAGE_SELF)
        return ru.ru_minflt + ru.ru_majflt

    def runs_of(fn):
        fn([])
        runs = []
        for _ in range(reps):
            garbage = []
            f0 = faults()
            t0 = pc()
            res, split = fn(garbage)
            t = pc() - t0
            f1 = faults()
            del garbage[:]
            t_free = pc() - t0 - t
            runs.append((t, dict(split), res, f1 - f0, t_free))
        return runs

    ms = lambda x: round(x * 1e3, 3)  # noqa: E731

    def summary(runs):
        ts = sorted(r_[0] for r_ in runs)
        med = sorted(runs, key=lambda x: x[0])[len(runs) // 2]
        split = {k: ms(v) for k, v in med[1].items()}
        split["other"] = round(ms(med[0]) - sum(split.values()), 3)
        split["total"] = ms(med[0])
        return {"total_ms": {"min": ms(ts[0]), "median": ms(med[0]), "max": ms(ts[-1])},
                "split_ms": split,
                "reps_ms": [dict({k: ms(v) for k, v in r_[1].items()}, total=ms(r_[0]), page_faults=r_[3],
                                 deferred_free_ms=ms(r_[4])) for r_ in runs]}, med
    try:
        wruns = runs_of(write)
        rruns = runs_of(read)
    finally:
        goroutines.shutdown()
    wsum, wmed = summary(wruns)
    rsum, rmed = summary(rruns)
    mm, wc = wmed[2]
    ok_w = mm == m_fused and all(bytes(c) == bytes(x) for c, x in zip(wc, chunks))
    ok_r = all(bytes(x[2]) == data.tobytes() for x in rruns[:1] + [rmed])
    L = chunks[0].size // 4

    def alloc_write(garbage):
        bufs = [np.empty((data.size + 3) // 4, dtype=np.uint32)] + \
               [np.zeros(L, dtype=np.uint32) for _ in range(r)] + [gf._new_bytearray(None, 4 * L) for _ in range(total)]
        for b in bufs:
            np.frombuffer(b, dtype=np.uint8)[::4096] = 1
        garbage.extend(bufs)
        return None, []

    def alloc_read(garbage):
        bufs = [np.empty(L, dtype=np.uint32) for _ in range(2 * need)] + [gf._new_bytearray(None, 4 * L) for _ in range(need)] + \
               [np.empty(data.size + 16, dtype=np.uint8)]
        for b in bufs:
            np.frombuffer(b, dtype=np.uint8)[::4096] = 1
        garbage.extend(bufs)
        return None, []

    a_w = sorted(x[0] for x in runs_of(alloc_write))[reps // 2]
    a_r = sorted(x[0] for x in runs_of(alloc_read))[reps // 2]
    return {"write_gibs": round(data.size / GIB / wmed[0], 2), "read_gibs": round(data.size / GIB / rmed[0], 2),
            "write": wsum, "read": rsum, "reps": reps,
            "fresh_alloc_alone_ms": {"write": ms(a_w), "read": ms(a_r),
                                     "what": "the phases' fresh outputs allocated and first touched by one thread, "
                                             "timed alone (median); not part of total"},
            "codec": dict(N.codec_info(), placement="device" if gf.codec_placement() else "host"),
            "verified": bool(ok_w and ok_r),
            "what": f"multi_store.go unchanged: MapToGF + splitVector + {r} x CreateParity + {total} x MapFromGF on "
                    f"{total} concurrent threads (write); make + {need} x MapToGFWith + RecoverData + {need} x "
                    "MapFromGF appended (read); fresh outputs per call as Go's make(); CreateParity/RecoverData "
                    "host->GPU->host; the codec on the host cores (placement host) or through the GPU "
                    "(with_device_codec); split = the median call's phases, other = total - phases"}


def digest_leg(data, need, total, chunks, have, out, med, g) -> dict:
    """Chunk digests on the write path (store.DataV per chunk, multi_store.go:554-556)
    and the object verify on the read path (:244-249), host threads."""
    import hashlib
    from slime_amd import _native as N
    from slime_amd import objects
    sha_ext, threads = N.digest_info()
    box = {}
    t_fused = med(lambda: box.update(r=objects.write_chunks_digest(data, need, total, out=chunks)))
    m, _, shas, _ = box["r"]
    t_fz = med(lambda: objects.write_chunks_digest(data, need, total, out=chunks, alias=True))
    t_seq = med(lambda: (objects.write_chunks(data, need, total, out=chunks), objects.chunk_digests(chunks)))
    t_dig = med(lambda: objects.chunk_digests(chunks))
    t_hdr = med(lambda: objects.chunk_digests(chunks, headers=True))
    one = chunks[0]
    t_one = med(lambda: objects.sha256(one))
    want = hashlib.sha256(data.tobytes()).digest()
    surv = [chunks[i] for i in have]
    t_rv = med(lambda: objects.reconstruct(surv, have, m, data.size, out=out, sha=want))
    t_obj = med(lambda: objects.sha256(out))
    ok = shas == [hashlib.sha256(c.tobytes()).digest() for c in chunks] and bytes(out) == data.tobytes()
    chunk_bytes = sum(c.size for c in chunks)
    return {"write_chunks_digest_gibs": g(t_fused), "write_chunks_digest_zero_copy_gibs": g(t_fz),
            "write_chunks_then_digests_gibs": g(t_seq),
            "chunk_sha256_gbs": round(chunk_bytes / t_dig / 1e9, 2),
            "chunk_sha256_fnv_header_gbs": round(chunk_bytes / t_hdr / 1e9, 2),
            "sha256_one_thread_gbs": round(one.size / t_one / 1e9, 2),
            "reconstruct_verify_gibs": g(t_rv), "object_sha256_gbs": round(data.size / t_obj / 1e9, 2),
            "sha_extensions": sha_ext, "digest_threads": threads + 1, "verified": bool(ok),
            "what": f"write_chunks_digest hashes the {total} chunks while the device pipeline runs (object GiB/s); "
                    "the sequential form is write_chunks then chunk_digests; verify = reconstruct + the object's "
                    "SHA-256 (one message, one thread)"}


def link_probe(mib: int) -> dict:
    """The host side's own ceilings in this process, beside the host-path rates
    (their run-to-run spread, DESIGN.md "End-to-end"): pinned DMA each way and
    a single-thread host memcpy, median of 5, GB/s."""
    import numpy as np
    n = mib << 20
    pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    src = np.ones(n, dtype=np.uint8)
    dst = np.empty(n, dtype=np.uint8)
    dst[:] = 0

    def dma(h2d: bool) -> float:
        ts = []
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            if h2d:
                dev.copy_(pin, non_blocking=True)
            else:
                pin.copy_(dev, non_blocking=True)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e-3)
        return sorted(ts[1:])[2]

    def memcpy() -> float:
        ts = []
        for _ in range(6):
            t0 = time.perf_counter()
            np.copyto(dst, src)
            ts.append(time.perf_counter() - t0)
        return sorted(ts[1:])[2]

    out = {"h2d_pinned_gbs": round(n / dma(True) / 1e9, 1), "d2h_pinned_gbs": round(n / dma(False) / 1e9, 1),
           "host_memcpy_1thread_gbs": round(n / memcpy() / 1e9, 1), "bytes": n}
    del pin, dev
    return out


def board_info(dev: int) -> dict:
    """Board identity of `dev` read in-process from sysfs (amdgpu exposes
    product_name / product_number / VRAM vendor under the PCI device), so a
    bench line can be matched with the board it ran on.  Nothing is spawned:
    this process has initialised the GPU (no exec after GPU init)."""
    p = torch.cuda.get_device_properties(dev)
    bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}.0"
    info = {"bdf": bdf, "name": p.name, "arch": getattr(p, "gcnArchName", None),
            "hbm_gib": round(p.total_memory / GIB, 1), "cus": p.multi_processor_count}
    for key, fname in (("product_name", "product_name"), ("model_number", "product_number"),
                       ("vram_vendor", "mem_info_vram_vendor"), ("vbios", "vbios_version")):
        try:
            val = open(f"/sys/bus/pci/devices/{bdf}/{fname}").read().strip()
        except OSError:
            continue
        if val:
            info[key] = val
    return info


def shape_label(need: int, total: int, mib: int) -> str:
    """BASELINE.json's config name for a shape, if it is one of them."""
    return {(8, 12, 256): "C3+C4: ", (4, 6, 64): "C2: ", (10, 14, 1024): "C5: ",
            (8, 12, 512): "north-star 64 MiB shards: "}.get((need, total, mib), "")


def stream_ceilings(dev: int, stream, gib: int = 4, reps: int = 5) -> dict:
    """the achieved rate beside measured stream rates on this
    GPU in this process, after the timed region: torch's device copy (1:1
    read:write) and fill (write-only) over `gib` GiB, median of `reps`, in
    GB/s of HBM traffic.  Reference points from library kernels, not ceilings
    of the apply kernel (its 2:1 mix runs above the copy)."""
    import torch
    n = (gib << 30) // 4
    a = torch.empty(n, dtype=torch.int32, device=f"cuda:{dev}")
    b = torch.empty_like(a)
    a.fill_(1)

    def timed(fn, nbytes):
        fn()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return round(nbytes / (sorted(ts)[len(ts) // 2] * 1e-3) / 1e9, 1)

    with torch.cuda.stream(stream):
        copy = timed(lambda: b.copy_(a), 2 * a.numel() * 4)
        fill = timed(lambda: b.fill_(7), a.numel() * 4)
    del a, b
    torch.cuda.empty_cache()
    return {"torch_copy_gbs": copy, "torch_fill_gbs": fill, "bytes": f"{gib} GiB per pass, median of {reps}"}


class SymbolBatch:
    """One rank's batch in HBM: nobj objects of S bytes as symbol-domain shards
    ([object][shard][SS] uint32, SS = L rounded up to --shard-align), the need
    data shards filled with seeded symbols; the encode plan (all total-need
    parity rows) and the decode plan (the erased rows only, rebuilt into
    their slots in place, or into a separate buffer with --decode-dst
    separate).  One step = one encode launch + one decode launch."""

    def __init__(self, args, dev: int, seed: int, need: int, total: int, S: int, nobj: int, erase: list[int],
                 decode_dst: str = "inplace", reuse: torch.Tensor | None = None):
        self.need, self.total, self.S, self.nobj, self.erase = need, total, S, nobj, erase
        self.have = [i for i in range(total) if i not in erase][:need]
        self.L = L = ceil_div(ceil_div(S, 4), need)  # perVector = ceil(ceil(S/4)/need) (multi_store.go:272)
        # Shard stride SS >= L, rounded to --shard-align so every shard base is
        # line-aligned (L = 26843546 at C5 would put every shard 8 B off a 16 B
        # boundary; DESIGN.md "Line-aligned segments").  The pad columns are
        # never read or written; the algorithmic bytes are L's.
        self.SS = SS = ceil_div(L, max(1, args.shard_align)) * max(1, args.shard_align)
        self.lay = D.layout_of(total, L, SS)
        numel = max(1, nobj) * total * SS
        # `reuse`: re-lay another batch's buffer (its placement is that batch's)
        # instead of allocating -- the legs after the timed C3 region.
        self.owned = reuse is None or reuse.numel() < numel
        self.buf = batch_empty(args, numel, torch.int32, dev) if self.owned else reuse[:numel]
        self.placement = (D.placement(self.buf) if self.owned else dict(D.placement(reuse), relaid=True)) \
            if args.allocator == "vmm" else None
        D.fill_symbols(self.buf, seed)
        self.enc = D.Plan.encode(need, total, dev)
        self.dec = D.Plan.reconstruct(need, total, self.have, erase, dev)
        self.decode_dst = decode_dst
        if decode_dst == "inplace":
            # Repair: rebuilt shards go back into their erased slots (the faster
            # placement: output streams next to the input streams).
            self.dec.set_outputs(erase)
            self.rec, self.rec_lay = self.buf, self.lay
        else:
            self.rec = batch_empty(args, max(1, nobj) * len(erase) * SS, torch.int32, dev)
            self.rec_lay = D.layout_of(len(erase), L, SS)
        self.stream = torch.cuda.current_stream(dev)

    def encode(self, buf=None):
        b = self.buf if buf is None else buf
        self.enc(b, self.lay, b, self.lay, self.L, self.nobj, stream=self.stream, dst_offset=self.need * self.SS)

    def decode(self, buf=None):
        b = self.buf if buf is None else buf
        rec, rlay = (b, self.lay) if self.decode_dst == "inplace" else (self.rec, self.rec_lay)
        self.dec(b, self.lay, rec, rlay, self.L, self.nobj, stream=self.stream)

    def rebuilt(self):
        """The erased rows as the decode wrote them (nobj x e x L)."""
        if self.decode_dst == "inplace":
            return self.buf.view(self.nobj, self.total, self.SS)[:, self.erase, :self.L]
        return self.rec.view(self.nobj, len(self.erase), self.SS)[:, :, :self.L]

    def run(self, steps: int, warmup: int) -> dict:
        """The timed region: warmup untimed steps, then exactly `steps`, bracketed
        by a barrier and a device synchronize on both sides; HIP events on the
        launch stream around every launch.  Checks afterwards that every rebuilt
        shard equals the true one (the data as filled and the parity of one
        encode: encode is idempotent on fixed data)."""
        if self.nobj == 0:
            batch.barrier()
            batch.barrier()
            return {"elapsed": 0.0, "enc_all": [0.0], "dec_all": [0.0], "ok": True}
        self.encode()
        truth = self.buf.view(self.nobj, self.total, self.SS)[:, self.erase, :self.L].clone()
        for _ in range(warmup):
            self.encode()
            self.decode()
        torch.cuda.synchronize()
        events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        batch.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for ev in events:
            ev[0].record(self.stream)
            self.encode()
            ev[1].record(self.stream)
            self.decode()
            ev[2].record(self.stream)
        torch.cuda.synchronize()
        batch.barrier()
        elapsed = time.perf_counter() - t0
        ok = bool(torch.equal(self.rebuilt(), truth))
        del truth
        return {"elapsed": elapsed, "enc_all": [e[0].elapsed_time(e[1]) for e in events],
                "dec_all": [e[1].elapsed_time(e[2]) for e in events], "ok": ok}

    def sample(self, seed: int) -> dict:
        """column_sample of every object as the timed steps left it: the data
        rows (erased ones rebuilt by the last decode) and the parity rows of
        the last encode."""
        smp = column_sample(self.buf.view(self.nobj, self.total, self.SS), self.L, seed)
        if self.decode_dst != "inplace":  # the rebuilt rows live in self.rec (same seed: same columns)
            rec = column_sample(self.rec.view(self.nobj, len(self.erase), self.SS), self.L, seed)
            smp["cols"][:, self.erase] = rec["cols"]
        smp.update(need=self.need, total=self.total, have=self.have)
        return smp

    def alg_bytes(self) -> tuple[int, int]:
        """Algorithmic HBM bytes per launch: encode 4L(k + r),
        decode 4L(k + e) per object."""
        return (self.nobj * 4 * self.L * self.total, self.nobj * 4 * self.L * (self.need + len(self.erase)))

    def free(self):
        del self.buf, self.rec
        torch.cuda.empty_cache()
        D.release_deferred()


def symbol_traffic(args, need: int, total: int, L: int, nobj: int, kname: str) -> tuple:
    """HBM bytes per launch of the symbol path's apply kernel at this shape.
    PMC counters cannot be read inside this process (they need rocprofv3 --pmc
    passes of their own), so the bytes are replayed from the committed
    summaries of such passes (--traffic: tools/pmc_traffic.py output, one
    entry or a list) only when one was taken on this config AND this kernel's
    machine code; the second value says where they came from."""
    code_id = kernel_code_id(D.N.LIB_PATH, (f"{kname}ILi{need}E",))
    config = f"{need}/{total} L={L} nobj={nobj}"
    for path in (p for p in args.traffic.split(",") if p):
        try:
            tj = json.load(open(path))
        except (OSError, ValueError):
            continue
        for e in tj if isinstance(tj, list) else [tj]:
            if code_id and e.get("config") == config and e.get("kernel") == kname and e.get("kernel_code") == code_id:
                return e.get("hbm_bytes_per_launch"), (
                    f"replayed: {os.path.relpath(path, ROOT)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, "
                    f"session {e.get('session', '?')}, kernel code {code_id})")
    return None, "not measured for this kernel's machine code/config"


def apply_kernel_name(need: int, rows: int, L: int, shard_bytes_span: int) -> str:
    """The kernel the library dispatches a launch of this shape to
    (rs_apply.hip: the pipelined kernels for shards under 4 GiB unless the
    kernel form was switched, with the dynamic (ticket) schedule for k <= 32
    unless switched off; wide codes on the matrix cores, rs_apply_mfma.hip)."""
    kname = "rs_apply_kernel"
    if L < (1 << 30) and D.lib.slime_rs_kernel_pipeline(-1) == 1:
        queue = need <= 32 and D.lib.slime_rs_kernel_schedule(-1) == 1
        kname = "rs_apply_queue_kernel" if queue else "rs_apply_pipe_kernel"
    if _matrix_cores(need, rows) and shard_bytes_span < (1 << 32):
        kname = "rs_apply_mfma_kernel"  # wide codes (rs_apply_mfma.hip)
    return kname


def c5_leg(args, dev: int, rank: int, world: int, samples: dict | None = None) -> dict:
    """BASELINE config 5 inside every `bench.py --gpus N` run: need=10/total=14,
    64 x 1 GiB objects partitioned over the N ranks (batch.partition: 64 at
    N=1, 8 each at N=8), encode all parity + decode erased {0,1,2,3}.  Objects
    are independent (multi_store.go:528-531), so there is no exchange: each
    rank times its share and the leg's value is all 64 objects' bytes over the
    max-over-ranks time ("strong": total work fixed as N grows)."""
    need, total, mib, _, glob, erase_s = PRESETS["c5"]
    erase = [int(x) for x in erase_s.split(",")]
    first, nobj = batch.partition(glob, world, rank)
    S = mib << 20
    sb = SymbolBatch(args, dev, 0xC5C5 + 7919 * rank, need, total, S, nobj, erase)
    res = sb.run(args.steps, args.warmup)
    if samples is not None and nobj:
        samples["c5_partitioned"] = sb.sample(0xC5C5)
    enc_ms = sum(res["enc_all"]) / len(res["enc_all"])
    dec_ms = sum(res["dec_all"]) / len(res["dec_all"])
    enc_alg, dec_alg = sb.alg_bytes()
    kname = apply_kernel_name(need, total - need, sb.L, total * sb.SS * 4)
    frac = (enc_alg + dec_alg) / 2 / ((enc_ms + dec_ms) / 2 * 1e-3) / 1e9 / HBM_PEAK_GBS if nobj else None
    mine = {"rank": rank, "objects": [first, nobj], "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
            "frac": round(frac, 4) if frac else None, "verified": res["ok"], "placement": sb.placement}
    sb.free()
    per_rank = [json.loads(x) for x in batch.gather_strings(json.dumps(mine))]
    elapsed, = batch.max_over_ranks([res["elapsed"]])
    return {"value": round(2 * glob * S * args.steps / GIB / elapsed, 2), "unit": "GiB/s", "scaling": "strong",
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "n_ranks": world,
            "config": f"C5: need={need} total={total}, {glob} x {mib} MiB objects partitioned over {world} rank(s); "
                      f"encode all parity + decode erased {erase}",
            "kernel": f"{kname}<{need},vec>", "per_rank": per_rank,
            "frac_min": min((p["frac"] for p in per_rank if p["frac"]), default=None),
            "verified": all(p["verified"] for p in per_rank)}


POOL_WORKLOADS = (  # (label, object MiB, pattern: 0 fused entry points, 1 the unchanged Go caller)
    ("fused_64mib", 64, 0), ("fused_1mib", 1, 0), ("unchanged_caller_64mib", 64, 1))


def pool_devices(world: int, ndev: int) -> list[int]:
    """The GPUs of this job's ranks (one per rank, rank r on GPU r % ndev):
    the device pool of the pooled leg may use exactly these."""
    return sorted({r % max(1, ndev) for r in range(world)})


def pooled_leg(args, rank: int, world: int, devices: list[int]) -> dict | None:
    """The deployment shape of the Go library on a node: ONE proxy process
    serving --pool-threads concurrent requests (main.go:107-109: 25), each a
    PUT (Multi.writeChunks, multi_store.go:516-557) then a GET of the same
    object (Multi.reconstruct's slow path, :185-252), every call through the
    *_ex forms with SLIME_RS_ANY_DEVICE, so the library's device pool spreads
    them over the GPUs of all N ranks (SLIME_RS_DEVICES = those GPUs).  Rank 0
    drives it from C++ threads (tools/proxy_load.cpp: no GIL between calls, as
    goroutines); the other ranks wait at a barrier.  Workloads: the fused
    entry points at 64 MiB (the proxy's request-body bound) and 1 MiB, and
    the unchanged caller (MapToGF + 4 x CreateParity + 12 x MapFromGF; 8 x
    MapToGFWith + RecoverData + 8 x MapFromGF) at 64 MiB.  Per-device call
    counts come from slime_rs_pool_calls.  PCIe-inclusive host memory in and
    out: never `value`."""
    batch.barrier()
    out = None
    if rank == 0:
        import ctypes

        from slime_amd import _native as N
        path = os.path.join(ROOT, "tools", "libproxy_load.so")
        lib = ctypes.CDLL(path)
        lib.proxy_load.restype = ctypes.c_int
        lib.proxy_load.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_double, ctypes.c_uint64,
                                   ctypes.POINTER(ctypes.c_double)]
        need, total, erase = 8, 12, [0, 1, 2, 3]
        have = [i for i in range(total) if i not in erase][:need]
        c_have = (ctypes.c_int * need)(*have)
        legs, ok = {}, True
        for label, mib, pattern in POOL_WORKLOADS:
            before = [N.pool_calls(d)[0] for d in devices]
            res = (ctypes.c_double * 10)()
            rc = lib.proxy_load(args.pool_threads, mib << 20, need, total, c_have, pattern, args.pool_seconds,
                                0x9001 + mib, res)
            after = [N.pool_calls(d)[0] for d in devices]
            reqs, wall = res[0], res[1]
            good = rc == 0 and res[2] == 1.0
            ok = ok and good
            legs[label] = {
                "object_mib": mib, "requests": int(reqs), "seconds": round(wall, 3),
                "gibs": round(2 * reqs * (mib << 20) / GIB / wall, 2) if wall else None,
                "requests_per_s": round(reqs / wall, 1) if wall else None,
                "calls_per_s": round(res[3] / wall, 1) if wall else None,
                "put_ms": {"p50": round(res[4], 3), "p99": round(res[5], 3)},
                "get_ms": {"p50": round(res[6], 3), "p99": round(res[7], 3)},
                "per_device_calls": {str(d): a - b for d, a, b in zip(devices, after, before)},
                "failed_calls": int(res[8]), "status": rc, "setup_s": round(res[9], 2), "verified": good}
        out = {"threads": args.pool_threads, "devices": devices, "host_call_slots": N.lib.slime_rs_host_call_slots(),
               "need": need, "total": total, "erased": erase,
               "workloads": legs, "verified": ok,
               "what": "one process, --pool-threads concurrent PUT (writeChunks) + GET (reconstruct) requests per "
                       "thread loop (fused: the shim's WriteChunks, whole data chunks aliasing the object), every call "
                       "through the cgo shim's *_ex forms with SLIME_RS_ANY_DEVICE over the "
                       "GPUs of all N ranks (tools/proxy_load.cpp); gibs = object bytes written + read per second; "
                       "per-request p50/p99 ms; verified = each thread's first and last GET returned its object, "
                       "its chunks were stable, and the unchanged caller's chunks equal the fused path's"}
    batch.barrier()
    return out


def shape_leg(args, name: str, dev: int, rank: int, world: int, reuse: torch.Tensor | None,
              samples: dict | None = None) -> dict:
    """A BASELINE shape beside the headline C3+C4 (PRESETS[name]: c2 = config
    2, 4/6 x 32 x 64 MiB; ns64 = the north star's "8/12 on 64 MiB shards", 64 x
    512 MiB), timed like the main region (W untimed steps, K timed ones of one
    encode + one decode launch, barrier + synchronize on both sides, HIP
    events on the launch stream) in `reuse` -- the main batch's buffer re-laid,
    so the leg allocates nothing.  Per GPU ("weak"): every rank runs its own
    batch of this shape.  The reference's loop is the same per-object
    multi_store.go:528-531 at that shape."""
    need, total, mib, per_gpu, _, erase_s = PRESETS[name]
    erase = [int(x) for x in erase_s.split(",")]
    S = mib << 20
    sb = SymbolBatch(args, dev, 0x5113E + 0x1000 * (1 + sorted(PRESETS).index(name)) + 7919 * rank,
                     need, total, S, per_gpu, erase, reuse=reuse)
    res = sb.run(args.steps, args.warmup)
    if samples is not None and per_gpu:
        samples[name] = sb.sample(0x5A30 + need)
    enc_ms = sum(res["enc_all"]) / len(res["enc_all"])
    dec_ms = sum(res["dec_all"]) / len(res["dec_all"])
    enc_alg, dec_alg = sb.alg_bytes()
    r = total - need
    kname = apply_kernel_name(need, r, sb.L, total * sb.SS * 4)
    traffic, source = symbol_traffic(args, need, total, sb.L, per_gpu, kname)
    ach = (enc_alg + dec_alg) / 2 / ((enc_ms + dec_ms) / 2 * 1e-3) / 1e9
    placement, L, SS = sb.placement, sb.L, sb.SS
    if sb.owned:
        sb.free()
    del sb
    elapsed, bad = batch.max_over_ranks([res["elapsed"], 0.0 if res["ok"] else 1.0])
    return {"value": round(2 * per_gpu * world * S * args.steps / GIB / elapsed, 2), "unit": "GiB/s",
            "scaling": "weak", "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "config": f"{shape_label(need, total, mib)}need={need} total={total}, {mib} MiB objects x {per_gpu} per "
                      f"GPU; encode all parity + decode erased {erase}",
            "symbols_per_shard": L, "shard_stride_symbols": SS,
            "encode_gibs": round(per_gpu * S / GIB / (enc_ms * 1e-3), 2),
            "decode_gibs": round(per_gpu * S / GIB / (dec_ms * 1e-3), 2),
            "kernel_ms": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4),
                          "encode_min_max": [round(min(res["enc_all"]), 4), round(max(res["enc_all"]), 4)],
                          "decode_min_max": [round(min(res["dec_all"]), 4), round(max(res["dec_all"]), 4)]},
            "roofline": {"bound": "hbm", "kernel": f"{kname}<{need},vec>", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "encode_frac": round(enc_alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "decode_frac": round(dec_alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_over_alg":
                             round(traffic / ((enc_alg + dec_alg) / 2), 4) if traffic else None,
                         "traffic_source": source, "alg_bytes_per_launch": {"encode": enc_alg, "decode": dec_alg}},
            "placement": placement, "verified": bad == 0.0}


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # Start the N ranks here, before anything initialises a GPU.
        sys.exit(launch_ranks(args))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus not in (1, world):
        print(f"bench.py: --gpus {args.gpus} under a launcher with WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)
    if world > 1:
        # Control plane only (barrier + max-over-ranks timing): objects are
        # independent, the data path exchanges nothing between GPUs.
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # One rank per GPU.  More ranks than visible GPUs would put two ranks on
    # one device and overstate the scaling curve: refuse.
    ndev = visible_gpus()
    if (world > ndev or local >= ndev) and not (shared_gpu_rehearsal() and ndev > 0):
        print(f"bench.py: {world} ranks (local rank {local}) but {ndev} visible GPU(s); one rank per GPU",
              file=sys.stderr, flush=True)
        sys.exit(2)
    devices = pool_devices(world, ndev)
    if args.pooled and "SLIME_RS_DEVICES" not in os.environ:
        # The library reads it once, at its first host call (none yet).
        os.environ["SLIME_RS_DEVICES"] = ",".join(map(str, devices))
    if args.dry_run:
        first, count = batch.partition(args.global_objects, world, rank) if args.global_objects else \
            (rank * args.objects, args.objects)
        c5 = batch.partition(PRESETS["c5"][4], world, rank)
        parts = batch.gather_strings(json.dumps([rank, local, first, count]))
        c5parts = batch.gather_strings(json.dumps([rank, local, c5[0], c5[1]]))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_ranks": world, "need": args.need, "total": args.total,
                              "object_mib": args.object_mib, "scaling": "strong" if args.global_objects else "weak",
                              "partitions": [json.loads(p) for p in parts],
                              "c5_partitioned": None if not args.c5_leg else
                              {"need": 10, "total": 14, "object_mib": 1024, "objects": PRESETS["c5"][4],
                               "partitions": [json.loads(p) for p in c5parts]},
                              "shapes": {n: {"need": PRESETS[n][0], "total": PRESETS[n][1], "object_mib": PRESETS[n][2],
                                             "objects_per_rank": PRESETS[n][3], "scaling": "weak"}
                                         for n in args.shape_legs.split(",") if n and
                                         PRESETS[n][:3] != (args.need, args.total, args.object_mib)},
                              "object_bytes_paths": [name for name, on in (
                                  ("object_bytes_path", args.bytes_path),
                                  ("object_bytes_path_c5", args.c5_bytes and
                                   (args.need, args.total, args.object_mib) != PRESETS["c5"][:3])) if on],
                              "host_path.pooled": None if not args.pooled else
                              {"driver_rank": 0, "threads": args.pool_threads, "devices": devices,
                               "pool_env": os.environ.get("SLIME_RS_DEVICES"),
                               "workloads": [w[0] for w in POOL_WORKLOADS]}}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    dev = local % max(1, ndev)
    torch.cuda.set_device(dev)

    need, total = args.need, args.total
    r = total - need
    erase = [int(x) for x in args.erase.split(",") if x != ""]
    if not erase or len(erase) > r or len(set(erase)) != len(erase) or not all(0 <= e < total for e in erase):
        print(f"bench.py: --erase needs 1..{r} distinct shard indices below total={total}", file=sys.stderr)
        sys.exit(2)
    S = args.object_mib << 20
    if args.global_objects:
        _, nobj = batch.partition(args.global_objects, world, rank)
        total_objs, scaling = args.global_objects, "strong"
    else:
        nobj, total_objs, scaling = args.objects, args.objects * world, "weak"

    sb = SymbolBatch(args, dev, 0x5113E + 7919 * rank, need, total, S, nobj, erase, args.decode_dst)
    L, SS, lay, placement = sb.L, sb.SS, sb.lay, sb.placement
    res = sb.run(args.steps, args.warmup)
    elapsed, enc_all, dec_all, ok = res["elapsed"], res["enc_all"], res["dec_all"], res["ok"]
    enc_ms = sum(enc_all) / args.steps
    dec_ms = sum(dec_all) / args.steps
    elapsed, enc_ms_max, dec_ms_max, bad = batch.max_over_ranks([elapsed, enc_ms, dec_ms, 0.0 if ok else 1.0])

    obj_bytes = nobj * S
    total_bytes = 2 * total_objs * S * args.steps
    value = total_bytes / GIB / elapsed
    enc_alg, dec_alg = sb.alg_bytes()
    launch_ms = (enc_ms + dec_ms) / 2
    achieved = (enc_alg + dec_alg) / 2 / (launch_ms * 1e-3) / 1e9
    kname = apply_kernel_name(need, r, L, total * SS * 4)
    traffic, traffic_source = symbol_traffic(args, need, total, L, nobj, kname)
    # Distinct devices across ranks (n_gpus), by PCI address.
    bdfs = batch.gather_strings(board_info(dev)["bdf"])
    # The CPU baseline's input: object 0 of this batch as the GPU left it
    # (data shards + the parity of the timed encodes), copied out before the
    # buffer is freed.
    cpu_sample = None
    # Column samples of every object of every timed batch, for the oracle pin
    # inside the cpu_baseline leg (rank 0 at N = 1, as that leg).
    samples = {} if rank == 0 and world == 1 and args.cpu_baseline else None
    if samples is not None and nobj:
        cpu_sample = sb.buf.view(nobj, total, SS)[0, :, :L].cpu().numpy().view("uint32").copy()
        samples["main"] = sb.sample(0x5A17)

    host = None
    want_host = rank == 0 and world == 1 and args.host_path

    def run_host_leg():
        if args.host_delay > 0:
            time.sleep(args.host_delay)
        # This rank's GPU only: the library's device pool would otherwise spread
        # the host calls over every visible GPU (include/slime_rs.h).
        from slime_amd import _native as N
        with N.on_device(dev):
            return dict(host_leg(need, total, erase), order=args.host_order, delay_s=args.host_delay, device=dev)

    if want_host and args.host_order == "before-free":
        host = run_host_leg()
    # The proxy's shape, at every N, while the batch buffers are still held
    # (freed VRAM is wiped by the same DMA engines the host path uses).
    pooled = pooled_leg(args, rank, world, devices) if args.pooled else None
    # After the host leg: the probe's buffers go back to the driver, whose
    # wipe of freed VRAM would slow the host leg's DMA (DESIGN.md End-to-end).
    ceilings = stream_ceilings(dev, sb.stream) if args.ceilings else None
    # The same batch in a hipMalloc'd (torch.empty) buffer, a few launches: what
    # the allocator choice is worth in this process (DESIGN.md "the allocator
    # changes the odds").  Not part of `value`.
    alloc_probe = None
    if args.allocator == "vmm" and args.alloc_probe and nobj:
        alt = torch.empty(nobj * total * SS, dtype=torch.int32, device=f"cuda:{dev}")
        alt_probe = D.probe_placement(alt)  # fresh: the probe overwrites it
        D.fill_symbols(alt, 0x5113E + 7919 * rank)
        pe, pd = [], []
        for k in range(4):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(sb.stream)
            sb.encode(alt)
            ev[1].record(sb.stream)
            sb.decode(alt)
            ev[2].record(sb.stream)
            torch.cuda.synchronize()
            if k:
                pe.append(ev[0].elapsed_time(ev[1]))
                pd.append(ev[1].elapsed_time(ev[2]))
        del alt
        pem, pdm = sorted(pe)[1], sorted(pd)[1]
        kept = (placement or {}).get("probes") or [{}]
        alloc_probe = {"buffer": "torch.empty (hipMalloc)", "encode_ms": round(pem, 4), "decode_ms": round(pdm, 4),
                       "frac": round((enc_alg + dec_alg) / 2 / ((pem + pdm) / 2 * 1e-3) / 1e9 / 8000.0, 4),
                       "launches": 3, "probe_gbs": round(alt_probe, 1),
                       "library_buffer_probe_gbs": kept[(placement or {}).get("chosen") or 0].get("probe_gbs"),
                       "threshold_gbs": float(D.lib.slime_rs_placement_threshold()),
                       "what": "slime_rs_probe_placement over the fresh hipMalloc buffer before it was filled, "
                               "beside the probe of the library buffer that was kept"}
    # The other BASELINE shapes, in the main buffer re-laid (after the
    # allocator probe, which reads the main batch's contents no more).
    shapes = {}
    for name in (x for x in args.shape_legs.split(",") if x):
        pn, pt, pm, ppg, _, _ = PRESETS[name]
        if (pn, pt, pm) != (need, total, args.object_mib):
            shapes[name] = shape_leg(args, name, dev, rank, world, sb.buf, samples)
    sb.free()
    bytes_path = bytes_leg(args, dev, rank, need, total, erase, nobj, samples=samples, tag="object_bytes_path") \
        if args.bytes_path else None
    # BASELINE config 5's shape on the fused byte path, per GPU (its worst
    # redo share: 26.8% of uniform 1 GiB objects switch to 1<<31).
    c5n, c5t, c5m, _, _, c5e = PRESETS["c5"]
    bytes_c5 = None
    if args.c5_bytes and (need, total, args.object_mib) != (c5n, c5t, c5m):
        bytes_c5 = bytes_leg(args, dev, rank, c5n, c5t, [int(x) for x in c5e.split(",")], 16, mib=c5m,
                             samples=samples, tag="object_bytes_path_c5")
    if want_host and args.host_order == "after-free":
        host = run_host_leg()
    c5 = None
    is_c5 = (need, total, args.object_mib, args.global_objects) == (10, 14, 1024, 64)
    if args.c5_leg and not is_c5:
        c5 = c5_leg(args, dev, rank, world, samples)

    if rank == 0:
        line = {
            "metric": "RS encode+decode GiB/s device-resident at need=8/total=12, 1/2/4/8 GPUs",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": len(set(bdfs)),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 symbols in [0,p), seeded per rank; MapToGF domain)",
            "config": {
                "workload": f"{shape_label(need, total, args.object_mib)}need={need} total={total}, "
                            f"{args.object_mib} MiB objects x {nobj} per GPU; encode all parity + decode erased {erase}",
                "need": need, "total": total, "object_mib": args.object_mib, "objects_per_gpu": nobj,
                "symbols_per_shard": L, "shard_stride_symbols": SS, "erased": erase, "decode_dst": args.decode_dst,
                "parallelism": f"object-partition x{world} (no RCCL)",
                "allocator": ALLOCATOR_NOTE[args.allocator],
                "placement": placement,
            },
            "encode_gibs": round(obj_bytes / GIB / (enc_ms * 1e-3), 2),
            "decode_gibs": round(obj_bytes / GIB / (dec_ms * 1e-3), 2),
            "kernel_ms": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4),
                          "encode_max_rank": round(enc_ms_max, 4), "decode_max_rank": round(dec_ms_max, 4),
                          "encode_min_max": [round(min(enc_all), 4), round(max(enc_all), 4)],
                          "decode_min_max": [round(min(dec_all), 4), round(max(dec_all), 4)],
                          # SURVEY §8(d) asks for the median of >= 5 runs; the roofline uses the mean
                          "encode_median": round(statistics.median(enc_all), 4),
                          "decode_median": round(statistics.median(dec_all), 4)},
            "verified": bad == 0.0,
            "roofline": {
                "bound": "hbm",
                "kernel": f"{kname}<{need},vec>",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_source,
                "alg_bytes_per_launch": {"encode": enc_alg, "decode": dec_alg},
                "measured_streams": ceilings,
                "achievable_peak": HBM_ACHIEVABLE_GBS,
                "frac_of_achievable": round(achieved / HBM_ACHIEVABLE_GBS, 4),
                "achievable_source": "MI355X_MICROARCH.md: 6.29 TB/s measured float4 copy (79% of the 8 TB/s spec)",
            },
            "cpu_baseline": None,
            "rehearsal": (f"{world} ranks sharing {len(set(bdfs))} GPU(s) (SLIME_BENCH_SHARE_GPU=1): "
                          "a test of the multi-rank path, not a scaling number") if shared_gpu_rehearsal() else None,
            "c5_partitioned": c5,
            "shapes": shapes,
            "object_bytes_path": bytes_path,
            "object_bytes_path_c5": bytes_c5,
            "allocator_probe": alloc_probe,
        }
        line["device"] = board_info(dev)
        if host is not None:
            line["host_path"] = host
        if pooled is not None:  # at every N (the N = 1 host legs above run only at N = 1)
            line.setdefault("host_path", {})["pooled"] = pooled
        if cpu_sample is not None:
            line["cpu_baseline"] = cpu_baseline(cpu_sample, f"object 0 of this run's batch ({args.object_mib} MiB)",
                                                need, total, erase, args.cpu_seconds, samples)
            pin = line["cpu_baseline"]["oracle_pin"]
            # `verified` = round trip of every leg AND, where the oracle ran,
            # bit-exact vs the reference's arithmetic on every object.
            line["verified_objects"] = {k: f"{v['verified_objects']}/{v['objects']}" for k, v in pin.items()}
            line["verified_columns_per_object"] = ORACLE_COLS + 1
            pinned_ok = all(v["verified_objects"] == v["objects"] for v in pin.values())
            line["verified"] = line["verified"] and pinned_ok
            def pinned(leg: dict | None, name: str) -> None:  # the leg's own verdict AND its pin
                if leg is not None and name in pin:
                    leg["verified_objects"] = pin[name]["verified_objects"]
                    leg["verified"] = leg["verified"] and pin[name]["verified_objects"] == pin[name]["objects"]
            for nm, v in shapes.items():
                pinned(v, nm)
            for key in ("c5_partitioned", "object_bytes_path", "object_bytes_path_c5"):
                pinned(line.get(key), key)
            bad = bad or not pinned_ok
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if bad or (c5 is not None and not c5["verified"]) or not all(v["verified"] for v in shapes.values()) or \
            (pooled is not None and not pooled["verified"]) or (bytes_path is not None and not bytes_path["verified"]) or \
            (bytes_c5 is not None and not bytes_c5["verified"]):
        sys.exit(3)


if __name__ == "__main__":
    main()
