"""slime_rs_device_alloc / slime_rs_device_free (device batch buffers built
from physical chunks) and the torch wrapper device.device_empty: the buffers
hold what the kernels write, exactly as hipMalloc'd ones do, are returned to
the device when freed, and misuse is refused."""
import ctypes
import threading

import numpy as np
import pytest

from slime_amd import _native as N
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


def test_alloc_rejects_misuse(torch_dev):
    p = ctypes.c_void_p()
    assert N.lib.slime_rs_device_alloc(0, 0, ctypes.byref(p)) != 0
    assert N.lib.slime_rs_device_alloc(0, 1 << 20, None) != 0
    assert N.lib.slime_rs_device_alloc(999, 1 << 20, ctypes.byref(p)) != 0
    assert N.lib.slime_rs_device_free(ctypes.c_void_p(0x1000)) != 0
    assert N.lib.slime_rs_device_alloc(0, 5, ctypes.byref(p)) == 0 and p.value
    assert N.lib.slime_rs_device_free(p) == 0
    assert N.lib.slime_rs_device_free(p) != 0  # freed once only


@pytest.mark.parametrize("need,total,L,nobj", [(8, 12, 4099, 7), (4, 6, 1 << 20, 3), (10, 14, 3 * 4096 + 5, 5)])
def test_device_empty_batch_matches_oracle(torch_dev, need, total, L, nobj):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(L + need)
    h = rng.integers(0, 2**32, size=(nobj, total, L), dtype=np.uint64).astype(np.uint32)
    buf = D.device_empty(nobj * total * L, torch.int32)
    assert buf.is_cuda and buf.numel() == nobj * total * L
    buf.copy_(torch.from_numpy(h.view(np.int32).reshape(-1)))
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
    for o in range(nobj):
        ref = np.ascontiguousarray(h[o])
        OC.encode_object(ref, need, total)
        assert np.array_equal(got[o], ref), o


def test_device_empty_byte_slots_and_views(torch_dev):
    torch = torch_dev
    from slime_amd import device as D
    b = D.device_empty(3 * (1 << 20) + 7, torch.uint8)
    b.fill_(0xA5)
    w = b[: 3 << 20].view(torch.int32)
    D.fill_symbols(w, 9)
    ref = torch.empty(3 << 18, dtype=torch.int32, device="cuda")
    D.fill_symbols(ref, 9)
    torch.cuda.synchronize()
    assert torch.equal(w, ref) and int(b[-1].item()) == 0xA5


def test_buffers_are_returned_to_the_device(torch_dev):
    """Sixteen rounds of a 24 GiB buffer (384 GiB in all, more than the device
    holds): each is freed when its last tensor goes."""
    torch = torch_dev
    from slime_amd import device as D
    free0, _ = torch.cuda.mem_get_info()
    for i in range(16):
        t = D.device_empty(6 << 30, torch.int32)
        t[:: 1 << 24].fill_(i)
        del t
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free1 > free0 - (1 << 30)


def test_concurrent_alloc_free(torch_dev):
    errors = []

    def worker(seed):
        try:
            for k in range(20):
                p = ctypes.c_void_p()
                rc = N.lib.slime_rs_device_alloc(0, (seed + k) * (1 << 20) + 123, ctypes.byref(p))
                assert rc == 0 and p.value
                assert N.lib.slime_rs_device_free(p) == 0
        except AssertionError as e:  # pragma: no cover - reported below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(s,)) for s in range(1, 9)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors


def test_placement_probe_keeps_the_fastest_candidate(torch_dev, monkeypatch):
    """A 16 GiB buffer with an unreachable probe target: the allocator probes
    its first placement and both alternatives (1 GiB chunks, hipMalloc), keeps
    the fastest, releases the others, and the buffer it returns computes
    exactly like any other."""
    torch = torch_dev
    from slime_amd import device as D
    monkeypatch.setenv("SLIME_RS_PLACEMENT_MIN_GBS", "1e9")
    free0, _ = torch.cuda.mem_get_info()
    buf = D.device_empty(4 << 30, torch.int32)  # 16 GiB
    info = D.placement(buf)
    assert info["retries"] == 2 and len(info["probes"]) == 3, info
    rates = [p["probe_gbs"] for p in info["probes"]]
    assert all(r > 1000 for r in rates), info
    assert info["chosen"] == rates.index(max(rates))
    assert info["kept"] == info["probes"][info["chosen"]]["placement"]
    free1, _ = torch.cuda.mem_get_info()
    assert free0 - free1 < (16 << 30) + (2 << 30), "the losing placements were released"
    need, total, L, nobj = 8, 12, 4099, 5
    rng = np.random.default_rng(3)
    h = rng.integers(0, 2**32, size=(nobj, total, L), dtype=np.uint64).astype(np.uint32)
    off = (3 << 30) + 12345  # somewhere past the first GiB
    buf[off: off + h.size].copy_(torch.from_numpy(h.view(np.int32).reshape(-1)))
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, src_offset=off, dst_offset=off + need * L)
    torch.cuda.synchronize()
    got = buf[off: off + h.size].cpu().numpy().view(np.uint32).reshape(nobj, total, L)
    for o in range(nobj):
        ref = np.ascontiguousarray(h[o])
        OC.encode_object(ref, need, total)
        assert np.array_equal(got[o], ref), o
    del buf
    torch.cuda.synchronize()


def test_placement_probe_skips_small_buffers_and_fast_ones(torch_dev, monkeypatch):
    torch = torch_dev
    from slime_amd import device as D
    small = D.device_empty(1 << 20, torch.int32)
    assert D.placement(small)["probes"] == [] and D.placement(small)["retries"] == 0
    monkeypatch.setenv("SLIME_RS_PLACEMENT_MIN_GBS", "1")  # any placement is fast enough
    big = D.device_empty(4 << 30, torch.int32)
    info = D.placement(big)
    assert len(info["probes"]) == 1 and info["retries"] == 0 and info["chosen"] == 0


def test_probe_placement_of_caller_buffers(torch_dev, caplog):
    """slime_rs_probe_placement over a caller's fresh buffer: the library's
    buffer (probed and re-placed when created) ranks at least as fast as a
    torch.empty (hipMalloc) buffer of the same size, within noise; a slow
    caller buffer is logged; ranges outside an allocation are refused."""
    import logging
    torch = torch_dev
    from slime_amd import device as D
    n = (20 << 30) // 4
    lib_buf = D.device_empty(n, torch.int32, 0)
    lib_gbs = D.probe_placement(lib_buf)
    lib_info = D.placement(lib_buf)
    del lib_buf
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    with caplog.at_level(logging.WARNING, logger="slime_amd"):
        t_gbs = D.probe_placement(t)
    want = float(N.lib.slime_rs_placement_threshold())
    assert lib_gbs > 0 and t_gbs > 0
    # The library's promise: its buffer is re-placed until it probes at the
    # threshold, keeping the fastest of its tries when none does (the default
    # threshold sits at the top of the rates seen, so it nearly always tries
    # all three).  So it matches the hipMalloc buffer within noise, or it
    # clears the threshold within noise (fast placements differ by up to ~4%:
    # 5950-6370 GB/s across this project's boxes), or every try was below it.
    rates = [p["probe_gbs"] for p in lib_info["probes"]]
    assert lib_info["chosen"] == rates.index(max(rates)), lib_info
    every_try_slow = len(rates) > 1 and all(r < want for r in rates)
    assert lib_gbs >= 0.97 * t_gbs or lib_gbs >= 0.98 * want or every_try_slow, (lib_gbs, t_gbs, lib_info)
    slow = D.SLOW_PLACEMENT * want
    assert (t_gbs < slow) == any("probes" in r.getMessage() for r in caplog.records), (t_gbs, slow)
    gbs = ctypes.c_double()
    # past the end of the allocation: refused before any launch
    rc = N.lib.slime_rs_probe_placement(ctypes.c_void_p(t.data_ptr()), t.numel() * 4 + (64 << 20), 0,
                                        ctypes.byref(gbs))
    assert rc == N.ERR_INVALID_ARG and gbs.value == 0
    host = np.zeros(1 << 20, dtype=np.uint8)
    assert N.lib.slime_rs_probe_placement(ctypes.c_void_p(host.ctypes.data), host.size, 0,
                                          ctypes.byref(gbs)) == N.ERR_INVALID_ARG
    # a small range: nothing to measure, no launch
    small = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    assert D.probe_placement(small) == 0.0
    del t
    torch.cuda.empty_cache()


def test_plan_warns_once_about_an_unprobed_large_buffer(torch_dev, caplog):
    """A >= 16 GiB caller buffer handed to a plan without a placement probe is
    logged once (its placement decides the kernels' speed); device_empty
    buffers are not."""
    import logging
    torch = torch_dev
    from slime_amd import device as D
    need, total, nobj = 8, 12, 16
    L = (17 << 30) // 4 // (nobj * total)
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    with caplog.at_level(logging.WARNING, logger="slime_amd"):
        t = torch.zeros(nobj * total * L, dtype=torch.int32, device="cuda")
        plan(t, lay, t, lay, L, nobj, dst_offset=need * L)
        plan(t, lay, t, lay, L, nobj, dst_offset=need * L)
        torch.cuda.synchronize()
        warned = [r for r in caplog.records if "unprobed" in r.getMessage()]
        assert len(warned) == 1
        del t
        torch.cuda.empty_cache()
        b = D.device_empty(nobj * total * L, torch.int32, 0)
        plan(b, lay, b, lay, L, nobj, dst_offset=need * L)
        torch.cuda.synchronize()
        assert len([r for r in caplog.records if "unprobed" in r.getMessage()]) == 1
        del b
