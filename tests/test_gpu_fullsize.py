"""Full-symbol parity at BASELINE sizes: every output symbol of the HIP path
against the C oracle (oracle/rs_oracle.c, the reference's arithmetic), not a
sample and not a round trip.

  C3: need=8 total=12, 256 MiB objects -- encode (all parity rows,
      internal/rs/vector.go:90-102 via CreateParity x r, multi_store.go:528-531)
  C4: the same objects, data shards {0,1,2,3} erased, and the mixed set
      {0,3,8,11} (RecoverData, vector.go:50-88, + CreateParity for parity rows)
  C5: need=10 total=14, 1 GiB objects (L = 26843546, 4 padding symbols)
  C2: need=4 total=6, 64 MiB objects in a batch of 32 (the queue kernels'
      4-tile units and 2-segment spread), decodes of {0,1} and {0,5}
and the fused byte path (writeChunks / reconstruct framing,
multi_store.go:526-557 and :194-242) at C3, C5 and C2 (in its 32-object
batch), including objects mapped with 1<<31 (map.go:47-62).  The oracle runs threaded over column ranges
(every output column is independent), so a 1 GiB object checks in seconds.
"""
import ctypes
import os
import threading

import numpy as np
import pytest

from slime_amd import rs
from oracle import oracle_c as OC
from oracle import oracle_py as OP

pytestmark = pytest.mark.gpu

P = 4294967291
NTHREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


def _threads(n_cols: int, fn):
    """fn(c0, c1) over NTHREADS contiguous column ranges, in parallel (ctypes drops the GIL)."""
    step = -(-n_cols // NTHREADS)
    ts = [threading.Thread(target=fn, args=(c0, min(n_cols, c0 + step))) for c0 in range(0, n_cols, step)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def oracle_apply(mat, ins):
    """out[i] = sum_j mat[i][j] * ins[j] mod p (oracle_apply_matrix, vector.go:90-102), threaded."""
    mat = np.ascontiguousarray(mat, dtype=np.uint32)
    rows, k = mat.shape
    L = ins[0].size
    assert all(x.flags.c_contiguous and x.size == L for x in ins)
    outs = [np.empty(L, dtype=np.uint32) for _ in range(rows)]

    def work(c0, c1):
        ip = (ctypes.c_void_p * k)(*[x.ctypes.data + 4 * c0 for x in ins])
        op = (ctypes.c_void_p * rows)(*[o.ctypes.data + 4 * c0 for o in outs])
        OC.lib.oracle_apply_matrix(mat.ctypes.data, rows, k, ip, op, c1 - c0)

    _threads(L, work)
    return outs


def oracle_recover(chunks, have):
    """RecoverData(chunks, have) (oracle_recover_data, vector.go:50-88), threaded over columns."""
    n = len(chunks)
    L = chunks[0].size
    outs = [np.empty(L, dtype=np.uint32) for _ in range(n)]
    idx = (ctypes.c_int * n)(*have)
    rcs = []

    def work(c0, c1):
        ip = (ctypes.c_void_p * n)(*[x.ctypes.data + 4 * c0 for x in chunks])
        op = (ctypes.c_void_p * n)(*[o.ctypes.data + 4 * c0 for o in outs])
        lens = (ctypes.c_uint64 * n)(*([c1 - c0] * n))
        rcs.append(OC.lib.oracle_recover_data(ip, lens, idx, n, n, op))

    _threads(L, work)
    assert rcs and all(rc == 0 for rc in rcs)
    return outs


def _symbol_case(torch, need, total, mib, nobj, check_obj, erasures=None):
    from slime_amd import device as D
    L = -(-(-(-(mib << 20) // 4)) // need)
    SS = -(-L // 64) * 64  # bench.py's device layout (256 B shard stride)
    lay = D.layout_of(total, L, SS)
    buf = torch.empty(nobj * total * SS, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, 0xF011 + need)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * SS)
    torch.cuda.synchronize()
    h = buf.view(nobj, total, SS)[check_obj, :, :L].cpu().numpy().view(np.uint32)
    shards = [np.ascontiguousarray(h[s]) for s in range(total)]
    del h
    # encode: every parity symbol
    pm = rs.ParityMatrix(need, total - need)[need:]
    ref = oracle_apply(pm, shards[:need])
    for i in range(total - need):
        assert np.array_equal(shards[need + i], ref[i]), f"parity row {need + i}"
    del ref
    # decode: two erasure sets, rebuilt into a separate buffer
    for erase in erasures or ([0, 1, 2, 3], [0, 3, need, total - 1]):
        have = [i for i in range(total) if i not in erase][:need]
        out = torch.empty(nobj * len(erase) * SS, dtype=torch.int32, device="cuda")
        D.Plan.reconstruct(need, total, have, erase)(buf, lay, out, D.layout_of(len(erase), L, SS), L, nobj)
        torch.cuda.synchronize()
        got = out.view(nobj, len(erase), SS)[check_obj, :, :L].cpu().numpy().view(np.uint32)
        del out
        data = oracle_recover([shards[i] for i in have], have)  # all need data rows, as the reference computes
        par = oracle_apply(pm, data)
        for i, t in enumerate(erase):
            want = data[t] if t < need else par[t - need]
            assert np.array_equal(got[i], want), (erase, t)
            assert np.array_equal(got[i], shards[t]), (erase, t)
    del buf
    torch.cuda.empty_cache()


def test_c3_c4_every_symbol_vs_oracle(torch_dev):
    """C3 encode + C4 decode of one whole 256 MiB object (object 1 of 2 in the batch)."""
    _symbol_case(torch_dev, 8, 12, 256, 2, 1)


def test_c5_every_symbol_vs_oracle(torch_dev):
    """C5 (10/14, 1 GiB object, L = 26843546) encode + two decodes, every symbol."""
    _symbol_case(torch_dev, 10, 14, 1024, 1, 0)


def test_c2_every_symbol_vs_oracle(torch_dev):
    """C2 (4/6, 64 MiB objects, a batch of 32: the launch geometry of
    BASELINE's C2) encode + decodes of {0,1} and {0,5}, every symbol of
    in-batch object 17."""
    _symbol_case(torch_dev, 4, 6, 64, 32, 17, erasures=([0, 1], [0, 5]))


# ------------------------------------------------------------ fused byte path

def _oracle_chunks_threaded(obj: bytes, need: int, total: int, cands=()):
    """writeChunks' framing (multi_store.go:526-554) via the oracle, parity threaded."""
    rc, m, words = OC.map_to_gf(obj, list(cands))
    assert rc == 0
    parts = [np.ascontiguousarray(p) for p in OP.split_vector(words, need)]
    parity = oracle_apply(rs.ParityMatrix(need, total - need)[need:], parts)
    return m, [OC.map_from_gf(m, p) for p in parts + parity]


def _bytes_case(torch, need, total, mib, nobj=2, at=(0, 1), erasures=None, align=1):
    """Objects at[0] (uniform random) and at[1] (forced to mapping 1<<31) of an
    nobj-object batch, every chunk byte against the oracle's framing; the
    other objects are random bytes drawn on the device.  align > 1: chunks
    `cs` = roundup(4L, align) apart (the _chunked entry points), object byte i
    at chunk i // 4L, offset i % 4L."""
    from slime_amd import device as D
    S = mib << 20
    L, cs, slot = D.slot_geometry(S, need, total, chunk_align=align)
    chunk = 4 * L
    cstride = cs if align > 1 else 0
    rng = np.random.default_rng(mib * 131 + need)
    objs = [rng.integers(0, 256, size=S, dtype=np.uint8) for _ in range(2)]
    # at[1]: a word >= p and no word that 1<<31 would map to >= p, so MapToGF
    # picks 1<<31 (map.go:47-62).  at[0] stays uniform random (at 1 GiB about
    # a quarter of such objects need 1<<31 or the random fallback).
    w = objs[1].view(">u4")
    w[(w >= 0x7FFFFFFB) & (w <= 0x7FFFFFFF)] = 0x12345678
    w[0] = 0xFFFFFFFF
    if nobj == 2:
        host = np.zeros(2 * slot, dtype=np.uint8)
        slots = None
    else:
        gen = torch.Generator(device="cuda").manual_seed(mib + nobj)
        slots = torch.randint(0, 256, (nobj * slot,), dtype=torch.uint8, device="cuda", generator=gen)
    for i, o in enumerate(at):
        for j in range(need):  # data chunk j: object bytes [4jL, 4(j+1)L) at slot + j*cs
            part = objs[i][j * chunk: (j + 1) * chunk]
            at_ = o * slot + j * cs
            if slots is None:
                host[at_: at_ + part.size] = part
            else:
                slots[at_: at_ + part.size].copy_(torch.from_numpy(part))
    if slots is None:
        slots = torch.from_numpy(host).cuda()
        del host
    enc = D.Plan.encode(need, total)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    D.encode_objects(enc, slots, slot, S, nobj, mapping, status, chunk_stride=cstride)
    torch.cuda.synchronize()
    st = status.cpu().numpy().tolist()
    assert st[at[1]] == 0
    if any(st):  # MapToGF's random fallback (map.go:64-66): resolved on the device
        assert D.resolve_fallbacks(enc, slots, slot, S, nobj, mapping, status, chunk_stride=cstride) == sum(st)
    ms = mapping.cpu().numpy().view(np.uint32).tolist()
    truth = {}
    for i, o in enumerate(at):
        cands = [ms[o]] if ms[o] not in (0, 1 << 31) else []
        m, want = _oracle_chunks_threaded(objs[i].tobytes(), need, total, cands)
        assert ms[o] == m, o
        got = slots[o * slot: (o + 1) * slot].cpu().numpy()
        for c in range(total):
            assert got[c * cs: c * cs + chunk].tobytes() == want[c], (o, c)
        if i == 1:
            assert m == 1 << 31
        truth[o] = want
    # repair of every object; compare the rebuilt chunk bytes of both checked objects
    for erase in erasures or ([0, 1, 2, 3], [0, 3, need, total - 1]):
        have = [i for i in range(total) if i not in erase][:need]
        rec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
        v = slots.view(nobj, slot)[:, : total * cs].view(nobj, total, cs)
        v[:, erase, :chunk] = 0x5A
        D.decode_objects(rec, slots, slot, L, nobj, mapping, chunk_stride=cstride)
        torch.cuda.synchronize()
        for o in at:
            got = slots[o * slot: (o + 1) * slot].cpu().numpy()
            for c in erase:
                assert got[c * cs: c * cs + chunk].tobytes() == truth[o][c], (o, erase, c)
    del slots
    torch.cuda.empty_cache()


def test_c3_bytes_every_byte_vs_oracle(torch_dev):
    _bytes_case(torch_dev, 8, 12, 256)


def test_c5_bytes_every_byte_vs_oracle(torch_dev):
    _bytes_case(torch_dev, 10, 14, 1024)


def test_c5_bytes_aligned_chunks_every_byte_vs_oracle(torch_dev):
    """The bench's byte-path layout at C5: 16 x 1 GiB objects on 256 B-aligned
    chunk strides (4L = 107,374,184 B -> 107,374,336), objects 3 (random) and
    11 (1<<31) of the batch, every byte of encode and both repairs."""
    _bytes_case(torch_dev, 10, 14, 1024, nobj=16, at=(3, 11), align=256)


def test_c2_bytes_every_byte_vs_oracle(torch_dev):
    """C2's batch (4/6, 32 x 64 MiB): objects 5 (random) and 22 (1<<31) of the
    batch, encode and the repairs of {0,1} and {0,5}, every byte."""
    _bytes_case(torch_dev, 4, 6, 64, nobj=32, at=(5, 22), erasures=([0, 1], [0, 5]))
