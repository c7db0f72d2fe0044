"""bench.py's contract pieces that run without a GPU: refusing more ranks than
visible devices, the BASELINE config labels, and that the committed PMC
traffic summary belongs to the kernel source being shipped (bench.py replays
it only then, and labels it)."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_refuses_more_ranks_than_gpus():
    import torch
    if torch.cuda.device_count() > 0:
        return  # only meaningful on a machine without GPUs
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "one rank per GPU" in r.stderr


def _bench(args, **env):
    e = dict(os.environ, **env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if k not in env:
            e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=e)


def test_gpus_n_launches_n_ranks_that_agree_on_the_partition():
    """`bench.py --gpus 2` outside torchrun starts two ranks itself (a stub
    device count under --dry-run: no GPU here); both rendezvous and report
    their share.  Weak scaling: 128 objects each; the C5 preset: 64 objects
    split 32 + 32."""
    r = _bench(["--gpus", "2", "--dry-run"], SLIME_BENCH_DEVICE_COUNT="2")
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_ranks"] == 2 and line["scaling"] == "weak"
    assert line["partitions"] == [[0, 0, 0, 128], [1, 1, 128, 128]]
    r = _bench(["--gpus", "2", "--dry-run", "--preset", "c5"], SLIME_BENCH_DEVICE_COUNT="2")
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert (line["need"], line["total"], line["object_mib"], line["scaling"]) == (10, 14, 1024, "strong")
    assert line["partitions"] == [[0, 0, 0, 32], [1, 1, 32, 32]]


def test_dry_run_reports_the_c5_partition_at_every_n():
    """Every `bench.py --gpus N` run carries BASELINE config 5 as a second leg:
    64 x 1 GiB objects (10/14) partitioned over the N ranks -- 32 + 32 at
    N = 2, 8 x 8 at N = 8 -- beside the weak-scaling C3 leg."""
    r = _bench(["--gpus", "2", "--dry-run"], SLIME_BENCH_DEVICE_COUNT="2")
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    c5 = line["c5_partitioned"]
    assert (c5["need"], c5["total"], c5["object_mib"], c5["objects"]) == (10, 14, 1024, 64)
    assert c5["partitions"] == [[0, 0, 0, 32], [1, 1, 32, 32]]
    r = _bench(["--gpus", "8", "--dry-run"], SLIME_BENCH_DEVICE_COUNT="8")
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["partitions"] == [[i, i, 128 * i, 128] for i in range(8)]
    assert line["c5_partitioned"]["partitions"] == [[i, i, 8 * i, 8] for i in range(8)]


def test_gpu_count_reads_sysfs_not_hip(tmp_path, monkeypatch):
    """The launcher counts GPUs from the KFD topology (CPU nodes have no SIMDs;
    a GPU whose render node this process cannot open is not counted) and the
    visibility variables, without starting the HIP runtime."""
    bench = _load("bench.py", "bench_mod_kfd")
    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    for i, (simds, minor) in enumerate([(0, None), (1024, 128), (1024, 129), (1024, 130)]):
        d = nodes / str(i)
        d.mkdir(parents=True)
        props = f"cpu_cores_count 64\nsimd_count {simds}\n" + (f"drm_render_minor {minor}\n" if minor else "")
        (d / "properties").write_text(props)
    for minor in (128, 129):  # node 3's render node is not in this container
        (dri / f"renderD{minor}").write_text("")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.kfd_gpus(str(nodes), str(dri)) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.kfd_gpus(str(nodes), str(dri)) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.kfd_gpus(str(nodes), str(dri)) == 0
    assert bench.kfd_gpus(str(tmp_path / "absent"), str(dri)) == 0


def test_gpus_n_beyond_visible_devices_exits_2():
    """--gpus 2 with fewer visible GPUs: exit 2 with a message, never a line
    claiming one GPU for a multi-GPU request."""
    r = _bench(["--gpus", "2", "--dry-run"], SLIME_BENCH_DEVICE_COUNT="1")
    assert r.returncode == 2 and "one rank per GPU" in r.stderr, r.stdout + r.stderr
    assert r.stdout.strip() == ""
    import torch
    if torch.cuda.device_count() < 2:
        r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
        assert r.returncode == 2 and "one rank per GPU" in r.stderr, r.stdout + r.stderr
        assert "n_gpus" not in r.stdout


def test_presets_fill_the_baseline_shapes_and_flags_win():
    bench = _load("bench.py", "bench_mod3")
    a = bench.parse(["--preset", "c2"])
    assert (a.need, a.total, a.object_mib, a.objects, a.global_objects, a.erase) == (4, 6, 64, 32, 0, "0,1")
    a = bench.parse(["--preset", "c5", "--global-objects", "16"])
    assert (a.need, a.total, a.object_mib, a.global_objects) == (10, 14, 1024, 16)
    a = bench.parse([])
    assert (a.need, a.total, a.object_mib, a.objects) == (8, 12, 256, 128)


def test_shape_labels_name_baseline_configs():
    bench = _load("bench.py", "bench_mod")
    assert bench.shape_label(8, 12, 256).startswith("C3+C4")
    assert bench.shape_label(4, 6, 64).startswith("C2")
    assert bench.shape_label(10, 14, 1024).startswith("C5")
    assert bench.shape_label(8, 12, 512).startswith("north-star")
    assert bench.shape_label(3, 5, 7) == ""


def test_committed_traffic_matches_shipped_kernel_code():
    """The PMC summary bench.py replays was measured on the machine code the
    built library runs (slime_amd/codeobj.py hashes the kernel's gfx950
    instructions), and its traffic is the algorithmic bytes."""
    import sys
    sys.path.insert(0, ROOT)
    from slime_amd.codeobj import kernel_code_id
    tj = json.load(open(os.path.join(ROOT, "profiles", "r04", "pmc_traffic.json")))
    assert tj["config"] == "8/12 L=8388608 nobj=128" and tj["kernel"] == "rs_apply_queue_kernel"
    lib = os.path.join(ROOT, "slime_amd", "lib", "libslime_rs.so")
    code = kernel_code_id(lib, ("rs_apply_queue_kernelILi8E",))
    assert code is not None
    assert tj["kernel_code"] == code, \
        "apply kernel's machine code changed since its PMC passes: re-run tools/gpu_r04.sh pmc_fetch pmc_write, then tools/pmc_traffic.py"
    alg = 128 * 4 * 8388608 * 12
    assert abs(tj["hbm_bytes_per_launch"] / alg - 1) < 0.01  # no wasted re-reads


def test_committed_byte_traffic_matches_shipped_kernel_code():
    """The byte path's PMC summary (profiles/r06/pmc_bytes.json, replayed into
    object_bytes_path and object_bytes_path_c5) covers C3 and C5 on 256 B
    chunk strides, was measured on the machine code of every kernel it names,
    and the first pass and repair move their algorithmic bytes 4L(k+r) /
    4L(k+e) -- C5's first pass plus the K/8 bytes a column of top bits it
    stores for the second pass's correction (rs_bytes_launch.hpp).  Older
    rounds' summaries name machine code since changed; bench.py skips them."""
    rnd = "r06"
    import sys
    sys.path.insert(0, ROOT)
    from slime_amd.codeobj import kernel_code_id
    entries = json.load(open(os.path.join(ROOT, "profiles", rnd, "pmc_bytes.json")))
    lib = os.path.join(ROOT, "slime_amd", "lib", "libslime_rs.so")
    shapes = {"8/12 S=268435456 nobj=128 cs=33554432": (8, 12, 8388608, 128),
              "10/14 S=1073741824 nobj=16 cs=107374336": (10, 14, 26843546, 16)}
    assert {e["config"] for e in entries} == set(shapes)
    for e in entries:
        need, total, L, nobj = shapes[e["config"]]
        ks = e["kernels"]
        for name, k in ks.items():
            assert k["kernel_code"] == kernel_code_id(lib, (f"{name}ILi{need}E",)), \
                f"{name}<{need}> changed since its PMC passes: re-run tools/gpu_r04.sh bpmc_c3 bpmc_c5"
        alg = nobj * 4 * L * total
        if "encode_bytes_queue_bits_kernel" in ks:  # C5: >= 1 GiB objects store top bits
            assert "encode_bytes_fix_kernel" in ks and "encode_bytes_queue_kernel" not in ks
            bits = nobj * L * need / 8
            assert abs(ks["encode_bytes_queue_bits_kernel"]["hbm_bytes"] / (alg + bits) - 1) < 0.01
        else:
            assert abs(ks["encode_bytes_queue_kernel"]["hbm_bytes"] / alg - 1) < 0.01
        assert abs(ks["decode_bytes_queue_kernel"]["hbm_bytes"] / (nobj * 4 * L * (need + 4)) - 1) < 0.01


def test_kernel_code_ids_name_one_kernel_each():
    """slime_amd/codeobj.py finds exactly one gfx950 kernel per fragment bench.py
    asks for (the apply and byte-path kernels of the BASELINE shapes), and
    distinct kernels hash differently."""
    import sys
    sys.path.insert(0, ROOT)
    from slime_amd.codeobj import kernel_code_id
    lib = os.path.join(ROOT, "slime_amd", "lib", "libslime_rs.so")
    ids = {}
    for need in (4, 8, 10):
        for k in ("rs_apply_queue_kernel", "encode_bytes_queue_kernel", "encode_bytes_redo_kernel",
                  "decode_bytes_queue_kernel", "encode_bytes_queue_bits_kernel", "encode_bytes_fix_kernel"):
            ids[(k, need)] = kernel_code_id(lib, (f"{k}ILi{need}E",))
            assert ids[(k, need)] is not None, (k, need)
    assert len(set(ids.values())) == len(ids)
    assert kernel_code_id(lib, ("no_such_kernel",)) is None


def test_matrix_core_labels_follow_the_library_rule():
    """bench.py labels a wide-code line with the matrix-core kernels exactly
    where the library routes it there (rs_apply_mfma.hip mfma_wanted: k >= 33,
    or 17 <= k <= 32 with k x rows >= 128; at most 32 rows, k <= 112)."""
    bench = _load("bench.py", "bench_mod_mfma")
    yes = [(64, 16), (33, 1), (99, 1), (112, 32), (24, 8), (32, 4), (17, 8)]
    no = [(8, 4), (10, 4), (16, 16), (20, 4), (17, 7), (64, 33), (113, 4), (40, 0)]
    assert all(bench._matrix_cores(k, r) for k, r in yes)
    assert not any(bench._matrix_cores(k, r) for k, r in no)


def test_dry_run_plans_the_c2_and_north_star_shape_legs():
    """Every line carries BASELINE config 2 (4/6, 32 x 64 MiB) and the north
    star's 64 MiB-shard shape (8/12, 64 x 512 MiB) per GPU beside C3+C4; a
    run whose main shape is one of them does not repeat it."""
    r = _bench(["--gpus", "2", "--dry-run"], SLIME_BENCH_DEVICE_COUNT="2")
    assert r.returncode == 0, r.stdout + r.stderr
    sh = json.loads(r.stdout.strip().splitlines()[-1])["shapes"]
    assert sh["c2"] == {"need": 4, "total": 6, "object_mib": 64, "objects_per_rank": 32, "scaling": "weak"}
    assert sh["ns64"] == {"need": 8, "total": 12, "object_mib": 512, "objects_per_rank": 64, "scaling": "weak"}
    r = _bench(["--dry-run", "--preset", "c2"], SLIME_BENCH_DEVICE_COUNT="1")
    sh = json.loads(r.stdout.strip().splitlines()[-1])["shapes"]
    assert set(sh) == {"ns64"}
    # ns64 re-lays the C3 batch's buffer: exactly the same number of words
    bench = _load("bench.py", "bench_mod_ns64")
    c3 = 128 * 12 * bench.ceil_div(bench.ceil_div(256 << 20, 4), 8)
    ns = 64 * 12 * bench.ceil_div(bench.ceil_div(512 << 20, 4), 8)
    assert c3 == ns


def test_dry_run_plans_the_pooled_proxy_leg_at_every_n():
    """At every N, rank 0 drives the host entry points as one proxy does (25
    concurrent PUT + GET requests, SLIME_RS_ANY_DEVICE) over the GPUs of all
    N ranks: the device pool is restricted to exactly those GPUs."""
    for n in (1, 2, 8):
        args = ["--gpus", str(n), "--dry-run"] if n > 1 else ["--dry-run"]
        r = _bench(args, SLIME_BENCH_DEVICE_COUNT=str(n))
        assert r.returncode == 0, r.stdout + r.stderr
        pooled = json.loads(r.stdout.strip().splitlines()[-1])["host_path.pooled"]
        assert pooled["driver_rank"] == 0 and pooled["threads"] == 25
        assert pooled["devices"] == list(range(n))
        assert pooled["pool_env"] == ",".join(str(d) for d in range(n))
        assert pooled["workloads"] == ["fused_64mib", "fused_1mib", "unchanged_caller_64mib"]


def test_proxy_load_library_exports_its_entry_point():
    """tools/libproxy_load.so (built by make) links the C-ABI and exports
    proxy_load; argument errors return SLIME_RS_ERR_INVALID_ARG without
    touching a GPU."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libproxy_load.so"))
    f = lib.proxy_load
    f.restype = ctypes.c_int
    out = (ctypes.c_double * 10)()
    have = (ctypes.c_int * 8)(*range(4, 12))
    assert f(0, ctypes.c_uint64(1 << 20), 8, 12, have, 0, ctypes.c_double(1.0), ctypes.c_uint64(1), out) == 9
    assert f(4, ctypes.c_uint64(1 << 20), 8, 12, have, 2, ctypes.c_double(1.0), ctypes.c_uint64(1), out) == 9


def test_proxy_load_fails_loudly_without_a_gpu():
    """No GPU: every request's device calls return SLIME_RS_ERR_NO_DEVICE (10)
    and the run is not verified -- there is no CPU fallback to hide behind."""
    import ctypes
    import torch
    if torch.cuda.device_count() > 0:
        return
    sys.path.insert(0, ROOT)
    import slime_amd  # noqa: F401  (loads libslime_rs.so first, as bench.py does)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libproxy_load.so"))
    lib.proxy_load.restype = ctypes.c_int
    out = (ctypes.c_double * 10)()
    have = (ctypes.c_int * 8)(*range(4, 12))
    for pattern in (0, 1):
        rc = lib.proxy_load(2, ctypes.c_uint64(4096), 8, 12, have, pattern, ctypes.c_double(0.05),
                            ctypes.c_uint64(1), out)
        assert rc == 10 and out[2] == 0.0 and out[8] > 0


def test_committed_traffic_per_shape_matches_shipped_kernel_code():
    """profiles/r06/pmc_traffic.json holds one PMC summary per BASELINE shape
    the line reports (C3, C2, the north star's 64 MiB shards); each was
    measured on the machine code the built library runs, and each moves its
    algorithmic bytes 4L(k+r) per launch to within 1%.  Its C2 entry is the
    pass after the three-tile units at k <= 4 (s31); older rounds' files name
    machine code since changed, and bench.py skips them."""
    rnd = "r06"
    import sys
    sys.path.insert(0, ROOT)
    from slime_amd.codeobj import kernel_code_id
    entries = json.load(open(os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json")))
    lib = os.path.join(ROOT, "slime_amd", "lib", "libslime_rs.so")
    shapes = {"8/12 L=8388608 nobj=128": (8, 12, 8388608, 128), "4/6 L=4194304 nobj=32": (4, 6, 4194304, 32),
              "8/12 L=16777216 nobj=64": (8, 12, 16777216, 64)}
    assert {e["config"] for e in entries} == set(shapes)
    for e in entries:
        need, total, L, nobj = shapes[e["config"]]
        assert e["kernel"] == "rs_apply_queue_kernel"
        assert e["kernel_code"] == kernel_code_id(lib, (f"rs_apply_queue_kernelILi{need}E",)), e["config"]
        assert abs(e["hbm_bytes_per_launch"] / (nobj * 4 * L * total) - 1) < 0.01, e["config"]


def test_oracle_pin_counts_every_object_and_catches_one_bad_word():
    """bench.py's oracle pin: column_sample gathers a seeded
    window plus the last column of every object; oracle_pin re-encodes each
    object's sampled data columns with the oracle and recovers them from the
    survivors.  A batch the oracle itself encoded pins every object, in the
    symbol domain and in the byte domain (big-endian words XOR the mapping);
    one flipped parity word, or one flipped rebuilt data word, fails exactly
    that object."""
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from oracle import oracle_c as OC
    bench = _load("bench.py", "bench_mod_pin")
    need, total, L, SS, nobj = 4, 6, 9000, 9024, 5
    erase = [0, 1]
    have = [i for i in range(total) if i not in erase][:need]
    rng = np.random.default_rng(7)
    buf = np.zeros((nobj, total, SS), dtype=np.uint32)
    for o in range(nobj):
        sh = np.zeros((total, L), dtype=np.uint32)
        sh[:need] = rng.integers(0, 2**32 - 5, size=(need, L), dtype=np.uint32)
        OC.encode_object(sh, need, total)
        buf[o, :, :L] = sh
    v3 = torch.from_numpy(buf.view(np.int32))
    smp = bench.column_sample(v3, L, 11, ncols=1024)
    assert smp["cols"].shape == (nobj, total, 1025) and smp["window"] == 1024
    for o in range(nobj):  # the window at its offset, then column L-1
        off = smp["offsets"][o]
        assert np.array_equal(smp["cols"][o, :, :1024], buf[o, :, off:off + 1024])
        assert np.array_equal(smp["cols"][o, :, 1024], buf[o, :, L - 1])
    smp.update(need=need, total=total, have=have)
    pin = bench.oracle_pin({"sym": smp})
    assert pin["sym"]["verified_objects"] == nobj and pin["sym"]["columns_per_object"] == 1025
    bad = dict(smp, cols=smp["cols"].copy())
    bad["cols"][2, need, 17] ^= 1          # a parity word of object 2
    bad["cols"][4, erase[1], 1024] ^= 4    # a rebuilt data word of object 4 (the last column)
    assert bench.oracle_pin({"sym": bad})["sym"]["verified_objects"] == nobj - 2
    # byte domain: slot words are big-endian bytes of symbol ^ mapping
    ms = np.array([0, 1 << 31, 0x12345, 0, 1 << 31], dtype=np.uint32)
    wire = (smp["cols"] ^ ms[:, None, None]).byteswap()
    pin = bench.oracle_pin({"b": dict(smp, cols=wire, mapping=ms)})
    assert pin["b"]["verified_objects"] == nobj and pin["b"]["domain"] == "bytes"
    assert bench.oracle_pin({"b": dict(smp, cols=wire, mapping=ms ^ np.uint32(1))})["b"]["verified_objects"] == 0
