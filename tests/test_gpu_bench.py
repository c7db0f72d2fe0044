"""GPU tests of bench.py's host-memory legs at small sizes: the proxy-level
pooled driver (tools/proxy_load.cpp, host_path.pooled) and the unchanged Go
caller's split.  Both run the product through the C-ABI; the round trips and
the chunk comparisons are their checks (the parity itself is pinned against
the oracle in test_gpu_parity.py)."""
import ctypes
import importlib.util
import os

import numpy as np
import pytest

from slime_amd import _native as N
from slime_amd import objects

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_gpu_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _proxy():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libproxy_load.so"))
    lib.proxy_load.restype = ctypes.c_int
    lib.proxy_load.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_double, ctypes.c_uint64,
                               ctypes.POINTER(ctypes.c_double)]
    return lib


@pytest.mark.parametrize("pattern", [0, 1])
@pytest.mark.parametrize("size,need,total,have", [
    (256 << 10, 8, 12, [4, 5, 6, 7, 8, 9, 10, 11]),
    ((1 << 20) + 13, 4, 6, [1, 2, 4, 5]),
    (4099, 10, 14, [0, 2, 4, 6, 8, 9, 10, 11, 12, 13]),
])
def test_proxy_load_round_trips_under_concurrency(pattern, size, need, total, have):
    """8 concurrent requests, PUT + GET each, through the *_ex forms with
    SLIME_RS_ANY_DEVICE: every GET returns its object, chunks are stable, the
    unchanged caller's chunks equal the fused entry point's, and the device
    pool counted every call on a GPU."""
    lib = _proxy()
    n = N.lib.slime_rs_device_count()
    before = [N.pool_calls(d)[0] for d in range(n)]
    out = (ctypes.c_double * 10)()
    c_have = (ctypes.c_int * need)(*have)
    rc = lib.proxy_load(8, size, need, total, c_have, pattern, 0.3, 77 + pattern, out)
    after = [N.pool_calls(d)[0] for d in range(n)]
    assert rc == 0 and out[8] == 0, (rc, list(out))
    assert out[2] == 1.0, "a GET did not return its object or the chunks changed"
    assert out[0] >= 8 and out[1] > 0
    # device-routed calls: fused 2 per request; unchanged r CreateParity + 1 RecoverData
    # per request (the codec calls run on the host cores and take no device)
    assert sum(a - b for a, b in zip(after, before)) >= out[0] * (2 if pattern == 0 else 1)


def test_unchanged_caller_split_adds_up():
    """The unchanged caller's line: phases + other = total for the median call,
    total min <= median <= max over >= 7 reps, and both directions verified
    (the write's chunks equal the fused entry point's)."""
    bench = _bench()
    need, total, erase = 8, 12, [0, 1, 2, 3]
    have = [i for i in range(total) if i not in erase][:need]
    data = np.random.default_rng(5).integers(0, 256, size=(2 << 20) + 7, dtype=np.uint8)
    chunks = [np.zeros(objects.chunk_size(data.size, need), dtype=np.uint8) for _ in range(total)]
    m, _ = objects.write_chunks(data, need, total, out=chunks)
    u = bench.unchanged_caller(data, need, total, have, chunks, m, m, 7)
    assert u["verified"]
    for side in ("write", "read"):
        s = u[side]["split_ms"]
        parts = sum(v for k, v in s.items() if k != "total")
        assert abs(parts - s["total"]) < 0.01, s
        t = u[side]["total_ms"]
        assert t["min"] <= t["median"] <= t["max"] and len(u[side]["reps_ms"]) == 7
    assert "map_from_gf_x12_concurrent" in u["write"]["split_ms"]


def test_callers_beyond_the_host_call_slots_queue_and_finish():
    """More concurrent callers than host-call slots (slime_rs_host_call_slots):
    the surplus waits asleep for a slot and every request still completes and
    verifies; the slots pass in arrival order, so no caller's worst request
    waits more than a few rounds of everyone else's."""
    lib = _proxy()
    slots = N.lib.slime_rs_host_call_slots()
    assert slots >= 4
    threads = 3 * slots
    out = (ctypes.c_double * 10)()
    have = (ctypes.c_int * 8)(*range(4, 12))
    rc = lib.proxy_load(threads, 96 << 10, 8, 12, have, 0, 0.5, 5, out)
    assert rc == 0 and out[2] == 1.0 and out[8] == 0, list(out)
    assert out[0] >= threads
    put_p50, put_p99 = out[4], out[5]
    assert put_p99 < max(20 * put_p50, 25.0), (put_p50, put_p99)  # no starved caller (ms)


@pytest.mark.parametrize("alloc", ["torch", "vmm"])
def test_device_legs_pin_every_object_to_the_oracle(alloc):
    """bench.py's device legs at small sizes, end to end on the GPU: a symbol
    batch (SymbolBatch.run, then .sample) at 4/6 and 10/14, and the fused byte
    leg at 10/14 through the phased encode, each sampled and pinned by
    oracle_pin -- every object verified, the byte leg's pass split adding up.
    (Few 8 MiB objects switch to 1<<31; the switch and its redo are pinned by
    test_gpu_parity.py's mid-object-switch and phased-event tests.)"""
    import types

    import torch
    bench = _bench()
    args = types.SimpleNamespace(object_mib=8, chunk_align=256, allocator=alloc, warmup=1, steps=2, shard_align=64,
                                 traffic="")
    samples = {}
    for name, (need, total, erase, nobj) in {"s46": (4, 6, [0, 1], 5), "s1014": (10, 14, [0, 3, 10, 13], 3)}.items():
        sb = bench.SymbolBatch(args, 0, 0x5A5A + need, need, total, (8 << 20) + 12, nobj, erase)
        res = sb.run(2, 1)
        assert res["ok"]
        samples[name] = sb.sample(7 + need)
        assert samples[name]["cols"].shape == (nobj, total, 4097)
        sb.free()
    leg = bench.bytes_leg(args, 0, 0, 10, 14, [0, 1, 2, 3], 6, mib=8, samples=samples, tag="bytes")
    assert leg["verified"] and leg["n_ranks"] == 1
    km = leg["kernel_ms"]
    assert 0 < km["encode_pass0"] <= km["encode_both_passes"] and km["encode_redo"] >= 0
    pin = bench.oracle_pin(samples)
    assert {k: (v["verified_objects"], v["objects"]) for k, v in pin.items()} == \
        {"s46": (5, 5), "s1014": (3, 3), "bytes": (6, 6)}
    assert pin["bytes"]["domain"] == "bytes"
    torch.cuda.synchronize()
