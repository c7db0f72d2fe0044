"""GPU parity: the gfx950 HIP path (through the C-ABI) against the oracle.

Bit-exact comparisons (integer field arithmetic) on seeded inputs at sizes the
C oracle finishes in seconds, the committed golden vectors, the reference's
KATs, and size-independent properties at full BASELINE sizes (encode -> erase
-> reconstruct round trips, linearity).  Edge cases the reference admits:
empty and ragged vectors, non-canonical symbols (x >= p, 0xFFFFFFFF), every
erasure pattern at 4/6, unaligned layouts, k > 16 (generic kernel).
"""
import ctypes
import itertools
import random

import numpy as np
import pytest

import slime_amd
from slime_amd import _native as N
from slime_amd import gf, rs
from oracle import oracle_c as OC
from oracle import oracle_py as OP

pytestmark = pytest.mark.gpu

P = gf.MaxVal
EDGES = np.array([0, 1, 2, P - 1, P, P + 1, P + 4, 0xFFFFFFFF, 0x7FFFFFFF, 0x80000000], dtype=np.uint32)


def rand_vecs(rng, k, L, canonical=False, edges=True):
    hi = P if canonical else 2**32
    vs = [rng.integers(0, hi, size=L, dtype=np.uint64).astype(np.uint32) for _ in range(k)]
    if edges and not canonical:
        for v in vs:
            n = min(L, EDGES.size)
            v[rng.choice(L, size=n, replace=False)] = EDGES[:n]
    return vs


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    assert N.device_count() > 0
    return torch


# ---------------------------------------------------------------- Go-API layer

def test_create_parity_kats(kats):
    for case in kats["create_parity"]:
        assert rs.CreateParity(case["data"], case["index"]).tolist() == case["out"]


def test_golden_encode_decode(golden):
    for case in golden["encode"]:
        for i, row in enumerate(case["parity"]):
            assert rs.CreateParity(case["data"], case["need"] + i).tolist() == row
        assert [r.tolist() for r in rs.CreateParities(case["data"], case["total"])] == case["parity"]
    for case in golden["decode"]:
        assert [r.tolist() for r in rs.RecoverData(case["chunks"], case["have"])] == case["data"]


@pytest.mark.parametrize("need,total", [(1, 2), (2, 3), (3, 5), (4, 6), (6, 8), (8, 12), (10, 14), (16, 20),
                                        (17, 20), (20, 24), (32, 36)])
@pytest.mark.parametrize("L", [1, 3, 4, 5, 7, 64, 1001, 4096 + 3])
def test_create_parity_vs_oracle(need, total, L):
    rng = np.random.default_rng(need * 1000 + L)
    data = rand_vecs(rng, need, L)
    for idx in [0, need - 1] + list(range(need, total)):
        rc, want = OC.create_parity(data, idx)
        assert rc == 0
        got = rs.CreateParity(data, idx)
        assert np.array_equal(got, want), (need, total, L, idx)
    allp = rs.CreateParities(data, total)
    for i, row in enumerate(allp):
        assert np.array_equal(row, OC.create_parity(data, need + i)[1])


def test_create_parity_reuses_out_buffer():
    data = [np.arange(10, dtype=np.uint32), np.arange(10, dtype=np.uint32) * 3]
    buf = np.full(32, 7, dtype=np.uint32)
    out = rs.CreateParity(data, 2, buf)
    assert out.base is buf or out.ctypes.data == buf.ctypes.data
    assert np.array_equal(out, OC.create_parity(data, 2)[1])
    assert np.all(buf[10:] == 7)


@pytest.mark.parametrize("need,total", [(2, 3), (4, 6), (8, 12), (10, 14), (17, 21), (33, 50), (64, 80)])
def test_recover_data_vs_oracle(need, total):
    rng = np.random.default_rng(need)
    L = 777
    data = rand_vecs(rng, need, L, canonical=True, edges=False)
    code = data + [OC.create_parity(data, need + i)[1] for i in range(total - need)]
    pyrng = random.Random(total)
    if total <= 24:
        sets = list(itertools.combinations(range(total), need))
        pyrng.shuffle(sets)
    else:  # too many subsets to list: sample them
        sets = [pyrng.sample(range(total), need) for _ in range(12)]
    for have in sets[:40]:
        have = list(have)
        pyrng.shuffle(have)  # any order, as RecoverData allows
        chunks = [code[i] for i in have]
        got = rs.RecoverData(chunks, have)
        rc, want = OC.recover_data(chunks, have)
        assert rc == 0
        for g, w, d in zip(got, want, data):
            assert np.array_equal(g, w) and np.array_equal(g, d)


def test_recover_data_noncanonical_survivors_match_reference():
    # Surviving data rows go through applyMatrix in the reference: x*1 mod p.
    chunks = [np.array([P, P + 3, 0xFFFFFFFF, 5], dtype=np.uint32), np.array([1, 2, 3, 4], dtype=np.uint32)]
    got = rs.RecoverData(chunks, [0, 2])
    rc, want = OC.recover_data(chunks, [0, 2])
    assert rc == 0
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    assert got[0].tolist() == [0, 3, 4, 5]


def test_recover_data_ragged_longer_chunks():
    a = np.arange(1, 9, dtype=np.uint32)
    b = np.arange(1, 13, dtype=np.uint32)  # longer than chunks[0]: extra ignored (vector.go:80-85)
    got = rs.RecoverData([a, b], [0, 2])
    rc, want = OC.recover_data([a, b], [0, 2])
    assert rc == 0 and all(np.array_equal(g, w) for g, w in zip(got, want))
    assert all(g.size == 8 for g in got)


@pytest.mark.parametrize("need,total,L", [(8, 12, 700001), (4, 6, 3 * 262144 + 5), (16, 20, 500003), (8, 12, 4099)])
def test_host_pipeline_multi_chunk(need, total, L):
    # The Go-API entry points stream host buffers through a 3-deep ring of
    # ~8 MiB stages: these sizes span >3 chunks with a ragged last chunk.
    rng = np.random.default_rng(L)
    data = rand_vecs(rng, need, L)
    par = rs.CreateParities(data, total)
    for i, row in enumerate(par):
        assert np.array_equal(row, OC.create_parity(data, need + i)[1]), i
    code = [OC.create_parity(data, t)[1] for t in range(total)]  # canonical data rows via identity rows
    have = list(range(total - need, total))[::-1]
    got = rs.RecoverData([code[i] for i in have], have)
    rc, want = OC.recover_data([code[i] for i in have], have)
    assert rc == 0
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


def test_host_pipeline_read_only_and_shared_inputs():
    # Read-only rows (np.frombuffer of bytes) and one row passed twice: the
    # staged pipeline only reads them.
    need, total, L = 4, 7, 300007
    rng = np.random.default_rng(5)
    base = rand_vecs(rng, need, L)
    data = [np.frombuffer(base[0].tobytes(), dtype=np.uint32), base[1], base[1], base[3]]
    assert not data[0].flags.writeable
    par = rs.CreateParities(data, total)
    for i, row in enumerate(par):
        assert np.array_equal(row, OC.create_parity([np.array(d) for d in data], need + i)[1])


def test_host_pipeline_concurrent_callers():
    # Several host threads share the workspace pool and the copy pool.
    import concurrent.futures as cf
    need, total, L = 8, 12, 400009
    rng = np.random.default_rng(9)
    jobs = [rand_vecs(rng, need, L) for _ in range(6)]
    with cf.ThreadPoolExecutor(4) as ex:
        outs = list(ex.map(lambda d: rs.CreateParities(d, total), jobs))
    for d, par in zip(jobs, outs):
        for i, row in enumerate(par):
            assert np.array_equal(row, OC.create_parity(d, need + i)[1])


@pytest.fixture(params=[0, 1], ids=["host_codec", "device_codec"])
def codec_place(request):
    """Both placements of the host-memory codec calls (slime_gf_codec_placement)."""
    prev = N.lib.slime_gf_codec_placement(-1)
    N.check(N.lib.slime_gf_codec_placement(request.param))
    yield request.param
    N.check(N.lib.slime_gf_codec_placement(prev))


def test_map_kats_on_gpu(kats, codec_place):
    for case in kats["map_trivial"]:
        data = bytes(case["in"])
        n, v = gf.MapToGF(data)
        assert n == case["n"] and v.tolist() == case["v"]
        assert gf.MapFromGF(n, v)[: len(data)] == data
    gf.Seed(99)
    for case in kats["map_tricky"]:
        data = bytes(case)
        n, v = gf.MapToGF(data)
        assert all(int(x) < P for x in v)
        assert gf.MapFromGF(n, v)[: len(data)] == data
        assert np.array_equal(gf.MapToGFWith(data, n), v)


def test_map_golden_and_random(golden, codec_place):
    for case in golden["map"]:
        data = bytes(case["bytes"])
        n, v = gf.MapToGF(data)
        assert n == case["n"] and v.tolist() == case["words"]
        assert list(gf.MapFromGF(n, v)) == case["back"]
    rng = np.random.default_rng(5)
    for length in [1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 100003]:
        data = rng.integers(0, 256, size=length, dtype=np.uint8).tobytes()
        for m in (0, 1 << 31, 0x12345678):
            assert np.array_equal(gf.MapToGFWith(data, m), OC.map_to_gf_with(data, m))
        n, v = gf.MapToGF(data)
        rc, n2, v2 = OC.map_to_gf(data)
        assert rc == 0 and n == n2 and np.array_equal(v, v2)
        assert gf.MapFromGF(n, v) == OC.map_from_gf(n, v)


def test_map_to_gf_high_bit_mapping(codec_place):
    # Every word >= p forces mapping 1<<31 (map.go:47-62).
    data = bytes([0xFF, 0xFF, 0xFF, 0xFB]) * 1000 + bytes([1, 2])
    n, v = gf.MapToGF(data)
    rc, n2, v2 = OC.map_to_gf(data)
    assert rc == 0 and n == n2 == 1 << 31 and np.array_equal(v, v2)


def test_map_to_gf_seeded_fallbacks_agree_across_placements():
    """Objects that need MapToGF's random fallback (map.go:64-66: a word in
    [p, 2^32) and one in [p ^ 1<<31, 2^31)) draw from the library's seeded
    candidate stream in batches of the same size on the host and on the
    device, first fit wins: after slime_gf_seed, a SEQUENCE of fallback
    objects gets the same mappings on both placements, and every mapping
    fits (every word < p)."""
    rng = np.random.default_rng(31)
    objs = []
    for i in range(4):
        w = rng.integers(0, 2**32, size=5000 + 997 * i, dtype=np.uint64).astype(np.uint32)
        w[7] = 0xFFFFFFFF
        w[11] = 0x7FFFFFFE
        objs.append(w.byteswap().tobytes() + bytes(i))  # big-endian words, ragged tail
    got = {}
    prev = N.lib.slime_gf_codec_placement(-1)
    try:
        for place in (0, 1):
            N.check(N.lib.slime_gf_codec_placement(place))
            gf.Seed(2024)
            got[place] = [gf.MapToGF(o) for o in objs]
    finally:
        N.check(N.lib.slime_gf_codec_placement(prev))
    for (m0, v0), (m1, v1), o in zip(got[0], got[1], objs):
        assert m0 == m1 and m0 not in (0, 1 << 31)
        assert np.array_equal(v0, v1) and int(v0.max()) < P
        assert gf.MapFromGF(m0, v0)[: len(o)] == o


@pytest.mark.parametrize("alias", ["inplace_parity_slots", "shifted_overlap"])
def test_recover_data_outputs_overlapping_chunks(alias):
    """RecoverData whose output rows overlap survivor chunks (a C caller's
    in-place repair): the erased rows are computed before anything the unit
    rows read is overwritten -- identical to the oracle on fresh buffers."""
    need, total, L = 6, 9, 70001
    rng = np.random.default_rng(17)
    data = rand_vecs(rng, need, L, canonical=True)
    code = [OC.create_parity(data, t)[1] for t in range(total)]
    have = [2, 3, 4, 6, 7, 8]  # data rows 0, 1, 5 erased
    want = OC.recover_data([code[i] for i in have], have)[1]
    if alias == "inplace_parity_slots":
        # erased data rows 0, 1, 5 are written over the parity survivors' own buffers
        chunks = [np.array(code[i]) for i in have]
        out = [None] * need
        out[0], out[1], out[5] = chunks[3], chunks[4], chunks[5]
        for t in (2, 3, 4):
            out[t] = chunks[have.index(t)]  # unit rows in place
    else:
        # one arena: each output row starts half a row into a survivor chunk
        arena = np.zeros((need + 1) * L, dtype=np.uint32)
        for q, i in enumerate(have):
            arena[q * L:(q + 1) * L] = code[i]
        chunks = [arena[q * L:(q + 1) * L] for q in range(need)]
        out = [arena[t * L + L // 2:(t + 1) * L + L // 2] for t in range(need)]
    ptr = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])  # noqa: E731
    lens = (ctypes.c_uint64 * need)(*([L] * need))
    idx = (ctypes.c_int * need)(*have)
    N.check(N.lib.slime_rs_recover_data(ptr(chunks), lens, need, idx, need, ptr(out)))
    for t in range(need):
        assert np.array_equal(out[t], want[t]), t


# ------------------------------------------------------- device-resident batch API

def _objects(torch, nobj, n, L, seed):
    from slime_amd import device as D
    buf = torch.empty(nobj * n * L, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, seed)
    return buf


def _host(t, nobj, n, L):
    return t.cpu().numpy().view(np.uint32).reshape(nobj, n, L)


@pytest.mark.parametrize("need,total,L,nobj", [(2, 3, 1000, 3), (4, 6, 4096, 5), (8, 12, 12345, 4),
                                               (10, 14, 8191, 3), (8, 12, 3, 7), (16, 20, 1024, 2),
                                               (20, 24, 999, 2), (17, 21, 4100, 3), (33, 40, 5003, 2),
                                               (40, 60, 4096 + 7, 2), (50, 100, 2051, 2), (20, 24, 3 * 4096, 5)])
def test_plan_encode_vs_oracle(torch_dev, need, total, L, nobj):
    torch = torch_dev
    from slime_amd import device as D
    buf = _objects(torch, nobj, total, L, seed=need * 7919 + L)
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    h = _host(buf, nobj, total, L)
    for o in range(nobj):
        ref = np.ascontiguousarray(h[o].copy())
        OC.encode_object(ref, need, total)
        assert np.array_equal(h[o], ref), o


@pytest.mark.parametrize("need,total,L", [(8, 12, 1 << 20), (10, 14, 26843546 // 32), (4, 6, 99991)])
def test_column_ranges_compose(torch_dev, need, total, L):
    """one object split by column ranges [b0, b1) -- the
    partition of a single huge object over GPUs, no exchange -- gives exactly
    the whole-object launch: each range is the same layout at a column offset
    with L = b1 - b0 (ranges of 1, odd and vector-multiple widths)."""
    torch = torch_dev
    from slime_amd import device as D
    nobj = 2
    buf = _objects(torch, nobj, total, L, seed=L + need)
    whole = buf.clone()
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    plan(whole, lay, whole, lay, L, nobj, dst_offset=need * L)
    cuts = sorted({0, 1, 4 * 1000 + 3, L // 3, L // 2 + 1, L - 5, L})
    for b0, b1 in zip(cuts, cuts[1:]):
        plan(buf, lay, buf, lay, b1 - b0, nobj, src_offset=b0, dst_offset=need * L + b0)
    torch.cuda.synchronize()
    assert torch.equal(buf, whole)
    h = _host(buf, nobj, total, L)[0]
    ref = np.ascontiguousarray(h.copy())
    OC.encode_object(ref, need, total)
    assert np.array_equal(h, ref)


@pytest.mark.parametrize("need,total", [(4, 6), (8, 12), (10, 14), (20, 24)])
@pytest.mark.parametrize("L", [4 * 262145, 4 * 262145 + 3])
@pytest.mark.parametrize("align", [1, 64])
def test_segment_rounding_empty_trailing_segments(torch_dev, need, total, L, align):
    """One object of 262145+ vectors per shard: 256 column segments whose 1 KiB
    rounding (segment_vectors, rs_apply_kernel.hpp) leaves the trailing
    segments empty, plus tail columns past the last vector; packed and 256 B
    shard strides (the recommended layout).  Encode and in-place repair of r
    erased shards, bit-exact against the oracle."""
    torch = torch_dev
    from slime_amd import device as D
    SS = (L + align - 1) // align * align
    buf = torch.empty(total * SS, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, 0xE5E6 + need * 131 + L + align)
    lay = D.layout_of(total, L, SS)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, 1, dst_offset=need * SS)
    torch.cuda.synchronize()
    h = buf.cpu().numpy().view(np.uint32).reshape(total, SS)[:, :L]
    ref = np.ascontiguousarray(h.copy())
    OC.encode_object(ref, need, total)
    assert np.array_equal(h, ref)
    erase = list(range(total - need - 1)) + [need]  # r erasures: data 0..r-2 and the first parity
    have = [i for i in range(total) if i not in erase][:need]
    buf.view(total, SS)[erase, :L] = 0
    D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)(buf, lay, buf, lay, L, 1)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint32).reshape(total, SS)[:, :L]
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("need,total", [(4, 6), (8, 12)])
def test_plan_reconstruct_every_pattern(torch_dev, need, total):
    torch = torch_dev
    from slime_amd import device as D
    nobj, L = 2, 2052
    buf = _objects(torch, nobj, total, L, seed=total)
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    h = _host(buf, nobj, total, L)
    sets = list(itertools.combinations(range(total), need))
    if len(sets) > 60:
        random.Random(1).shuffle(sets)
        sets = sets[:60] + [tuple(range(4, 12)), (1, 2, 4, 5, 6, 7, 9, 10)]
    for have in sets:
        want = [i for i in range(total) if i not in have]  # every lost shard, data and parity
        plan = D.Plan.reconstruct(need, total, list(have), want)
        out = torch.empty(nobj * len(want) * L, dtype=torch.int32, device="cuda")
        plan(buf, lay, out, D.layout_of(len(want), L), L, nobj)
        torch.cuda.synchronize()
        got = _host(out, nobj, len(want), L)
        for o in range(nobj):
            for w_i, t in enumerate(want):
                assert np.array_equal(got[o, w_i], h[o, t]), (have, t)


def test_plan_reconstruct_in_place_repair(torch_dev):
    """Rebuilt shards written back into their erased slots (slime_rs_plan_set_outputs)."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, L, nobj = 8, 12, 5003, 3
    buf = _objects(torch, nobj, total, L, seed=77)
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    truth = buf.clone()
    for erase in ([0, 1, 2, 3], [0, 3, 8, 11], [11], [2, 9]):
        have = [i for i in range(total) if i not in erase][:need]
        v = buf.view(nobj, total, L)
        v[:, erase, :] = -1  # destroy the erased shards
        plan = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
        plan(buf, lay, buf, lay, L, nobj)
        torch.cuda.synchronize()
        assert torch.equal(buf, truth), erase


def test_plan_matrix_unaligned_layouts_and_noncanonical(torch_dev):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(11)
    k, rows, L, nobj = 5, 3, 1031, 3
    shard, objs = L + 1, (L + 1) * k + 3  # odd strides: forces the one-column path
    host = rng.integers(0, 2**32, size=nobj * objs + 1, dtype=np.uint64).astype(np.uint32)
    host[:EDGES.size] = EDGES
    src = torch.from_numpy(host.view(np.int32)).cuda()
    coeff = rng.integers(0, P, size=(rows, k), dtype=np.uint64).astype(np.uint32)
    coeff[0] = P - 1
    plan = D.Plan.matrix(coeff, list(range(k)))
    dst = torch.zeros(nobj * rows * L + 1, dtype=torch.int32, device="cuda")
    plan(src, D.N.Layout(objs, shard), dst, D.N.Layout(rows * L, L), L, nobj, src_offset=1, dst_offset=1)
    torch.cuda.synchronize()
    got = dst.cpu().numpy().view(np.uint32)[1:].reshape(nobj, rows, L)
    for o in range(nobj):
        ins = [host[1 + o * objs + j * shard: 1 + o * objs + j * shard + L] for j in range(k)]
        want = OC.apply_matrix(coeff, ins)
        for i in range(rows):
            assert np.array_equal(got[o, i], want[i])


@pytest.mark.parametrize("need,total", [(8, 12), (10, 14), (4, 6)])
@pytest.mark.parametrize("L", [5 * 1024 + 1, 3 * 1024 + 2, 2 * 1024 + 3, 4097, 65, 7])
def test_realigned_layouts_vs_oracle(torch_dev, need, total, L):
    """Shard bases off 16-byte boundaries by 1..3 words (realigned loads and
    stores, tile and shard boundaries, in-place parity and a separate
    destination at every base offset)."""
    torch = torch_dev
    from slime_amd import device as D
    nobj = 3
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    for off in range(4):
        buf = torch.empty(off + nobj * total * L + 3, dtype=torch.int32, device="cuda")
        D.fill_symbols(buf, seed=L * 13 + off)
        before = buf.clone()
        plan(buf, lay, buf, lay, L, nobj, src_offset=off, dst_offset=off + need * L)
        torch.cuda.synchronize()
        whole = buf.cpu().numpy().view(np.uint32)
        # nothing outside the parity stripes moved (partial granules at both ends)
        mask = np.ones(whole.size, dtype=bool)
        for o in range(nobj):
            s0 = off + o * total * L + need * L
            mask[s0: s0 + (total - need) * L] = False
        assert np.array_equal(whole[mask], before.cpu().numpy().view(np.uint32)[mask]), off
        h = whole[off: off + nobj * total * L].reshape(nobj, total, L)
        for o in range(nobj):
            ref = np.ascontiguousarray(h[o].copy())
            OC.encode_object(ref, need, total)
            assert np.array_equal(h[o], ref), (off, o)
        # rebuild a data and a parity shard into a separate buffer at every offset
        erase = [1, need]
        have = [i for i in range(total) if i not in erase][:need]
        rec = D.Plan.reconstruct(need, total, have, erase)
        for doff in range(4):
            out = torch.zeros(doff + nobj * len(erase) * L + 2, dtype=torch.int32, device="cuda")
            rec(buf, lay, out, D.layout_of(len(erase), L), L, nobj, src_offset=off, dst_offset=doff)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            assert not got[:doff].any() and not got[doff + nobj * len(erase) * L:].any()
            got = got[doff: doff + nobj * len(erase) * L].reshape(nobj, len(erase), L)
            for o in range(nobj):
                for i, t in enumerate(erase):
                    assert np.array_equal(got[o, i], h[o, t]), (off, doff, o, t)


def test_full_size_c5_roundtrip(torch_dev):
    """BASELINE C5 shape (10/14, 1 GiB objects, L = 26843546: shard bases 8 bytes
    off 16-byte boundaries) on two objects: encode, erase, rebuild in place."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, nobj = 10, 14, 2
    L = -(-(1 << 30) // 4 // need)
    assert L % 4 == 2
    buf = _objects(torch, nobj, total, L, seed=0xC5)
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    v = buf.view(nobj, total, L)
    h = v[1].cpu().numpy().view(np.uint32)
    cols = np.sort(np.concatenate([np.arange(0, 1100), np.arange(L - 1100, L),
                                   np.random.default_rng(5).choice(L, size=4096, replace=False)]))
    ref = OC.apply_matrix(rs.ParityMatrix(need, total - need)[need:], [h[j, cols] for j in range(need)])
    for i in range(total - need):
        assert np.array_equal(h[need + i, cols], ref[i])
    for erase in ([0, 1, 2, 3], [0, 5, 10, 13]):
        truth = v[:, erase, :].clone()
        v[:, erase, :] = -1
        have = [i for i in range(total) if i not in erase][:need]
        D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)(buf, lay, buf, lay, L, nobj)
        torch.cuda.synchronize()
        assert torch.equal(v[:, erase, :], truth), erase
        del truth
    del buf, v
    torch.cuda.empty_cache()


def test_full_size_roundtrip_and_linearity(torch_dev):
    """BASELINE C3/C4 shape (8/12, 256 MiB objects) on a few objects: properties."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, nobj = 8, 12, 2
    L = (256 << 20) // 4 // need
    buf = _objects(torch, nobj, total, L, seed=0x5113E)
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    # erase data {0,1,2,3}: rebuild from 4..11 (C4 worst case)
    have, want = list(range(4, 12)), [0, 1, 2, 3]
    out = torch.empty(nobj * 4 * L, dtype=torch.int32, device="cuda")
    D.Plan.reconstruct(need, total, have, want)(buf, lay, out, D.layout_of(4, L), L, nobj)
    torch.cuda.synchronize()
    v = buf.view(nobj, total, L)
    r = out.view(nobj, 4, L)
    assert torch.equal(r, v[:, :4, :])
    # mixed erasure {0,3,8,11}
    have2 = [1, 2, 4, 5, 6, 7, 9, 10]
    out2 = torch.empty(nobj * 4 * L, dtype=torch.int32, device="cuda")
    D.Plan.reconstruct(need, total, have2, [0, 3, 8, 11])(buf, lay, out2, D.layout_of(4, L), L, nobj)
    torch.cuda.synchronize()
    r2 = out2.view(nobj, 4, L)
    for i, t in enumerate([0, 3, 8, 11]):
        assert torch.equal(r2[:, i, :], v[:, t, :])
    # sampled columns against the C oracle
    h = v[0].cpu().numpy().view(np.uint32)
    cols = np.random.default_rng(0).choice(L, size=4096, replace=False)
    ref = OC.apply_matrix(rs.ParityMatrix(need, total - need)[need:], [h[j, cols] for j in range(need)])
    for i in range(total - need):
        assert np.array_equal(h[need + i, cols], ref[i])
    del buf, out, out2
    torch.cuda.empty_cache()


def test_codec_device_roundtrip(torch_dev):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(2)
    for n in (1, 3, 4, 17, 1 << 20, (1 << 20) + 5):
        raw = rng.integers(0, 256, size=n, dtype=np.uint8)
        src = torch.from_numpy(raw).cuda()
        words = torch.empty((n + 3) // 4, dtype=torch.int32, device="cuda")
        flags = torch.zeros(1, dtype=torch.int32, device="cuda")
        D.pack_bytes(src, 0x80000000, words, flags)
        back = torch.empty(4 * words.numel(), dtype=torch.uint8, device="cuda")
        D.unpack_words(words, 0x80000000, back)
        torch.cuda.synchronize()
        assert np.array_equal(words.cpu().numpy().view(np.uint32), OC.map_to_gf_with(raw.tobytes(), 0x80000000))
        assert back.cpu().numpy()[:n].tobytes() == raw.tobytes()


def test_fill_symbols_deterministic_and_canonical(torch_dev):
    torch = torch_dev
    from slime_amd import device as D
    a = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    b = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    D.fill_symbols(a, 42)
    D.fill_symbols(b, 42)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert int(a.cpu().numpy().view(np.uint32).max()) < P


# ------------------------------------------- fused byte-domain object pipeline

def _oracle_chunks(obj: bytes, need: int, total: int, cands=()):
    """The reference's writeChunks framing (multi_store.go:526-554) via the oracle."""
    rc, m, words = OC.map_to_gf(obj, list(cands))
    assert rc == 0
    parts = OP.split_vector(words, need)
    parity = [OC.create_parity(parts, need + i)[1] for i in range(total - need)]
    return m, [OC.map_from_gf(m, p) for p in parts + parity]


def _make_slots(torch, objs, need, total, extra=0):
    from slime_amd import device as D
    S = len(objs[0])
    L, chunk, slot = D.slot_geometry(S, need, total)
    stride = slot + extra
    host = np.zeros(len(objs) * stride, dtype=np.uint8)
    for o, b in enumerate(objs):
        host[o * stride: o * stride + S] = np.frombuffer(b, dtype=np.uint8)
        host[o * stride + S: (o + 1) * stride] = 0xA5  # garbage past the object
    return torch.from_numpy(host).cuda(), L, chunk, stride


@pytest.fixture(params=[("1", 1), ("1", 0), ("0", 1)], ids=["queue", "pipelined", "fallback"])
def kernel_form(request):
    """Byte kernels: the product form (pipelined, dynamic schedule), the
    pipelined form with static shares (slime_rs_kernel_schedule(0)) and the
    non-pipelined form (chunks >= 4 GiB), selected process-wide by
    slime_rs_kernel_pipeline / slime_rs_kernel_schedule."""
    pipe, sched = request.param
    before = N.lib.slime_rs_kernel_pipeline(-1), N.lib.slime_rs_kernel_schedule(-1)
    assert N.lib.slime_rs_kernel_pipeline(int(pipe)) == 0
    assert N.lib.slime_rs_kernel_schedule(sched) == 0
    yield pipe
    N.lib.slime_rs_kernel_pipeline(before[0])
    N.lib.slime_rs_kernel_schedule(before[1])


@pytest.fixture
def switch_bits(request):
    """The second pass of the byte encode (slime_rs_switch_bits): mode 0 by
    object size (objects under 1 GiB here: the re-encode), 1 = always the
    top-bit correction.  Restored afterwards."""
    before = N.lib.slime_rs_switch_bits(-1)
    yield lambda m: N.lib.slime_rs_switch_bits(m)
    N.lib.slime_rs_switch_bits(before)


def test_switch_bits_mode_round_trip(torch_dev, switch_bits):
    assert switch_bits(-1) == 0
    for m in (1, 2, 0):
        assert switch_bits(m) == 0 and switch_bits(-1) == m
    assert switch_bits(3) == N.ERR_INVALID_ARG and switch_bits(-1) == 0


@pytest.mark.parametrize("bits", [0, 1], ids=["by_size", "topbits"])
@pytest.mark.parametrize("need,total", [(2, 3), (4, 6), (8, 12), (10, 14), (3, 5), (16, 20), (17, 20), (33, 50)])
@pytest.mark.parametrize("S", [1, 3, 4, 5, 31, 32, 33, 1000, 4096, 65537, 1 << 20, 3 * (1 << 20) + 7])
def test_encode_objects_matches_write_chunks(torch_dev, kernel_form, switch_bits, bits, need, total, S):
    """Device writeChunks against the reference framing, every chunk byte, in
    every kernel form; `topbits` corrects the switched units from stored top
    bits (need <= 10) instead of re-encoding them."""
    if bits and need > 10:
        pytest.skip("the top-bit correction takes need <= 10")
    assert switch_bits(bits) == 0
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(S * 31 + need)
    objs = [rng.integers(0, 256, size=S, dtype=np.uint8).tobytes() for _ in range(3)]
    # object 1 forces mapping 1<<31 (a word >= p, no word in 0x7FFFFFFB..0x7FFFFFFF)
    if S >= 4:
        b = bytearray(objs[1]); b[0:4] = b"\xff\xff\xff\xfd"; objs[1] = bytes(b)
    slots, L, chunk, stride = _make_slots(torch, objs, need, total, extra=12)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(3, dtype=torch.int32, device="cuda")
    status = torch.empty(3, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, 3, mapping, status)
    torch.cuda.synchronize()
    h = slots.cpu().numpy()
    ms = mapping.cpu().numpy().view(np.uint32)
    assert status.cpu().numpy().tolist() == [0, 0, 0]
    for o, obj in enumerate(objs):
        m, chunks = _oracle_chunks(obj, need, total)
        assert ms[o] == m
        for c in range(total):
            got = h[o * stride + c * chunk: o * stride + (c + 1) * chunk].tobytes()
            assert got == chunks[c], (o, c)
    if S >= 4:
        assert ms[1] == 1 << 31


@pytest.mark.parametrize("need,total,S,nobj", [(8, 12, 16 << 20, 12), (10, 14, (8 << 20) + 5, 12),
                                               (4, 6, (6 << 20) + 3, 18), (20, 24, (4 << 20) + 1, 6),
                                               (3, 5, 1 << 20, 36), (16, 20, (5 << 20) + 2, 6),
                                               # more than four parity rows (the correction's table is
                                               # rebuilt per four rows), and need 1 / 9 (narrow and odd
                                               # bit fields)
                                               (6, 14, (3 << 20) + 1, 8), (2, 9, (2 << 20) + 6, 8),
                                               (1, 3, (1 << 20) + 2, 8), (9, 16, (4 << 20) + 3, 8),
                                               # the matrix-core encode's switch (rs_bytes_mfma.hip): 2..5 K
                                               # steps, four- and two-column lane tiles, many segments
                                               (25, 32, (3 << 20) + 1, 8), (40, 48, (4 << 20) + 2, 8),
                                               (64, 80, (8 << 20) + 3, 8), (80, 100, (6 << 20) + 1, 8),
                                               (33, 40, (2 << 20) + 7, 16), (72, 90, (5 << 20) + 2, 8)])
@pytest.mark.parametrize("bits", [0, 1], ids=["by_size", "topbits"])
def test_encode_objects_mid_object_switch(torch_dev, switch_bits, bits, need, total, S, nobj):
    """The dynamic-schedule encode (and the matrix-core encode of wide codes)
    switches an object to 1<<31 as soon as a word >= p has been seen and the
    second pass redoes only the units (tiles) encoded before that
    (rs_bytes_kernel.hpp, rs_bytes_mfma.hip).  Objects with that word at the start,
    a quarter, half, 90 % and the last whole word, two such words, none, and
    one that needs the random fallback (a word >= p after a word 1<<31 cannot
    map); every chunk byte against the reference framing (map.go:15-67,
    multi_store.go:526-554).  `topbits`: the second pass corrects the listed
    units from the top bits the first pass stored (slime_rs_switch_bits(1))."""
    if bits and need > 10:
        pytest.skip("the top-bit correction takes need <= 10")
    assert switch_bits(bits) == 0
    torch = torch_dev
    from slime_amd import device as D
    assert N.lib.slime_rs_kernel_pipeline(-1) == 1 and N.lib.slime_rs_kernel_schedule(-1) == 1
    rng = np.random.default_rng(S + nobj)
    nfull = S // 4  # whole words
    kinds = [None, 0.0, 0.25, 0.5, 0.9, "last", (0.3, 0.8), "fallback"]
    objs = []
    for o in range(nobj):
        b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
        w = np.frombuffer(b, dtype=">u4", count=nfull).copy()
        w[(w >= 0x7FFFFFFB) & (w < 0x80000000)] ^= 0x00100000  # no accidental fallback
        w[w >= 4294967291] = 0x01020304  # no accidental 1<<31 either
        b[:4 * nfull] = w.astype(">u4").tobytes()
        k = kinds[o % len(kinds)]
        at = []
        if k == "last":
            at = [nfull - 1]
        elif k == "fallback":
            at = [int(0.6 * (nfull - 1))]
            b[4 * int(0.1 * nfull): 4 * int(0.1 * nfull) + 4] = b"\x7f\xff\xff\xfd"
        elif isinstance(k, tuple):
            at = [int(f * (nfull - 1)) for f in k]
        elif k is not None:
            at = [int(k * (nfull - 1))]
        for a in at:
            b[4 * a: 4 * a + 4] = b"\xff\xff\xff\xfd"
        objs.append(bytes(b))
    slots, L, chunk, stride = _make_slots(torch, objs, need, total, extra=64)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, nobj, mapping, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().tolist()
    assert st == [1 if kinds[o % len(kinds)] == "fallback" else 0 for o in range(nobj)]
    if any(st):
        assert D.resolve_fallbacks(plan, slots, stride, S, nobj, mapping, status) == sum(st)
    ms = mapping.cpu().numpy().view(np.uint32)
    h = slots.cpu().numpy()
    for o, obj in enumerate(objs):
        k = kinds[o % len(kinds)]
        cands = [int(ms[o])] if k == "fallback" else []
        m, chunks = _oracle_chunks(obj, need, total, cands)
        assert ms[o] == m and (k is None) == (m == 0), (o, k)
        for c in range(total):
            got = h[o * stride + c * chunk: o * stride + (c + 1) * chunk].tobytes()
            assert got == chunks[c], (o, k, c)
        assert (h[o * stride + total * chunk: (o + 1) * stride] == 0xA5).all(), "wrote past the chunks"


@pytest.mark.parametrize("need,total", [(8, 12), (10, 14), (40, 56)])
def test_encode_objects_phased_event_splits_the_passes(torch_dev, need, total):
    """slime_rs_encode_objects_phased (bench.py's redo share): the same chunks
    as the plain call, byte for byte, with objects that switch to 1<<31; the
    event it records lies between the call's start and end on the stream, so
    pass 0 + redo = the whole encode."""
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(need)
    S, nobj = (4 << 20) + 4, 8
    objs = []
    for o in range(nobj):
        b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
        if o % 2:
            b[4 * (o * 1000): 4 * (o * 1000) + 4] = b"\xff\xff\xff\xfd"
        objs.append(bytes(b))
    plan = D.Plan.encode(need, total)
    outs = []
    for phased in (False, True):
        slots, L, chunk, stride = _make_slots(torch, objs, need, total)
        mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
        status = torch.empty(nobj, dtype=torch.int32, device="cuda")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[1].record()
        ev[0].record()
        D.encode_objects(plan, slots, stride, S, nobj, mapping, status, phase_event=ev[1] if phased else None)
        ev[2].record()
        torch.cuda.synchronize()
        assert status.cpu().numpy().tolist() == [0] * nobj
        if phased:
            a, b = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
            assert a > 0 and b > 0 and abs(a + b - ev[0].elapsed_time(ev[2])) < 1e-3
        outs.append((slots.cpu().numpy(), mapping.cpu().numpy().view(np.uint32)))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert (outs[1][1][1::2] == 1 << 31).all()
    with pytest.raises(ValueError):
        D.encode_objects(plan, slots, stride, S, nobj, mapping, status,
                         phase_event=torch.cuda.Event(enable_timing=True))  # never recorded: no handle yet


def test_encode_objects_random_fallback(torch_dev):
    torch = torch_dev
    from slime_amd import device as D
    need, total, S = 4, 6, 4096
    rng = np.random.default_rng(9)
    b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
    b[0:8] = b"\xff\xff\xff\xff\x7f\xff\xff\xff"  # neither 0 nor 1<<31 fits (map_test.go TestMapTricky)
    objs = [bytes(b), rng.integers(0, 256, size=S, dtype=np.uint8).tobytes()]
    slots, L, chunk, stride = _make_slots(torch, objs, need, total)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(2, dtype=torch.int32, device="cuda")
    status = torch.empty(2, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, 2, mapping, status)
    torch.cuda.synchronize()
    assert status.cpu().numpy().tolist() == [1, 0]
    assert D.resolve_fallbacks(plan, slots, stride, S, 2, mapping, status) == 1
    m = int(mapping.cpu().numpy().view(np.uint32)[0])
    assert status.cpu().numpy().tolist() == [0, 0]
    # the chosen mapping is valid and the chunks are the reference's for that mapping
    rc, m2, _ = OC.map_to_gf(objs[0], [m])
    assert rc == 0 and m2 == m
    _, chunks = _oracle_chunks(objs[0], need, total, [m])
    h = slots.cpu().numpy()
    for c in range(total):
        assert h[c * chunk:(c + 1) * chunk].tobytes() == chunks[c]


@pytest.mark.parametrize("need,total,S", [(4, 6, 5000), (8, 12, 1 << 20), (8, 12, 999999), (10, 14, 77777),
                                          (2, 3, 3), (20, 24, 300001), (40, 60, 123457), (6, 9, 5 * (1 << 20) + 3),
                                          (12, 16, 3 * (1 << 20) + 1), (16, 20, 2 * (1 << 20))])
def test_decode_objects_repairs_chunks(torch_dev, kernel_form, need, total, S):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(S)
    objs = [rng.integers(0, 256, size=S, dtype=np.uint8).tobytes() for _ in range(4)]
    if S >= 4:
        b = bytearray(objs[2]); b[0:4] = b"\xff\xff\xff\xfe"; objs[2] = bytes(b)  # mapping 1<<31
    slots, L, chunk, stride = _make_slots(torch, objs, need, total)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(4, dtype=torch.int32, device="cuda")
    status = torch.empty(4, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, 4, mapping, status)
    torch.cuda.synchronize()
    truth = slots.clone()
    r = total - need
    for erase in (list(range(min(r, need))), [0, total - 1][:r], [need - 1]):
        have = [i for i in range(total) if i not in erase][:need]
        rec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
        v = slots.view(4, stride)[:, : total * chunk].view(4, total, chunk)
        v[:, erase, :] = 0x5A
        D.decode_objects(rec, slots, stride, L, 4, mapping)
        torch.cuda.synchronize()
        assert torch.equal(slots, truth), erase
    # the object bytes are the first S bytes of each slot (reconstruct's data[:Size])
    h = slots.cpu().numpy()
    for o, obj in enumerate(objs):
        assert h[o * stride: o * stride + S].tobytes() == obj


def _make_chunked_slots(torch, objs, need, total, align):
    """Slots whose chunks sit `cs` = roundup(4L, align) bytes apart: object byte
    i at chunk i // 4L, offset i % 4L; every other byte 0xA5."""
    from slime_amd import device as D
    S = len(objs[0])
    L, cs, slot = D.slot_geometry(S, need, total, chunk_align=align)
    stride = slot + 64
    host = np.full(len(objs) * stride, 0xA5, dtype=np.uint8)
    for o, b in enumerate(objs):
        a = np.frombuffer(b, dtype=np.uint8)
        for j in range(need):
            part = a[j * 4 * L: (j + 1) * 4 * L]
            host[o * stride + j * cs: o * stride + j * cs + part.size] = part
    return torch.from_numpy(host).cuda(), L, cs, stride


@pytest.mark.parametrize("need,total,S,nobj", [(8, 12, (2 << 20) + 5, 9), (4, 6, 4097, 5), (10, 14, 999999, 8),
                                               (16, 20, (1 << 20) + 3, 4), (20, 24, 300001, 3), (2, 3, 7, 3)])
@pytest.mark.parametrize("align", [256, 4096])
def test_objects_chunk_stride_layout(torch_dev, kernel_form, need, total, S, nobj, align):
    """encode/resolve/decode over a slot layout with padded chunk stride
    (slime_rs_*_objects_chunked): every chunk equals the reference framing
    (map.go:15-67, multi_store.go:526-554), the padding between chunks is
    untouched, and erased chunks come back bit-exact."""
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(S + align + nobj)
    objs = []
    for o in range(nobj):
        b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
        if S >= 8 and o % 3 == 1:
            at = 4 * ((S // 4) * 2 // 3)
            b[at: at + 4] = b"\xff\xff\xff\xfd"  # mid-object switch to 1<<31
        if S >= 8 and o == nobj - 1:
            b[0:8] = b"\xff\xff\xff\xff\x7f\xff\xff\xff"  # random fallback (map_test.go TestMapTricky)
        objs.append(bytes(b))
    slots, L, cs, stride = _make_chunked_slots(torch, objs, need, total, align)
    assert cs % align == 0 and cs >= 4 * L
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, nobj, mapping, status, chunk_stride=cs)
    torch.cuda.synchronize()
    st = status.cpu().numpy().tolist()
    if any(st):
        assert D.resolve_fallbacks(plan, slots, stride, S, nobj, mapping, status, chunk_stride=cs) == sum(st)
    torch.cuda.synchronize()
    ms = mapping.cpu().numpy().view(np.uint32)
    h = slots.cpu().numpy()
    for o, obj in enumerate(objs):
        m, chunks = _oracle_chunks(obj, need, total, [int(ms[o])] if st[o] else [])
        assert ms[o] == m, o
        base = o * stride
        for c in range(total):
            assert h[base + c * cs: base + c * cs + 4 * L].tobytes() == chunks[c], (o, c)
            assert (h[base + c * cs + 4 * L: base + (c + 1) * cs] == 0xA5).all(), ("gap", o, c)
        assert (h[base + total * cs: base + stride] == 0xA5).all(), ("tail", o)
    truth = slots.clone()
    r = total - need
    for erase in (list(range(min(r, need))), [need - 1, total - 1][:r]):
        have = [i for i in range(total) if i not in erase][:need]
        rec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
        v = slots.view(nobj, stride)
        for e in erase:
            v[:, e * cs: e * cs + 4 * L] = 0x5A
        D.decode_objects(rec, slots, stride, L, nobj, mapping, chunk_stride=cs)
        torch.cuda.synchronize()
        assert torch.equal(slots, truth), erase


def test_objects_chunk_stride_rejects_bad_layouts(torch_dev):
    """The _chunked entry points refuse a chunk stride below 4L or not a
    multiple of 4, and a slot stride that cannot hold total chunks at it
    (SLIME_RS_ERR_INVALID_ARG, nothing launched); 0 is the wire layout."""
    torch = torch_dev
    import ctypes
    from slime_amd import device as D
    need, total, S, nobj = 4, 6, 4000, 2
    L, _, _ = D.slot_geometry(S, need, total)
    plan = D.Plan.encode(need, total)
    cs = 4 * L + 256
    slots = torch.zeros(nobj * total * cs, dtype=torch.uint8, device="cuda")
    mapping = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    p, mp, sp = (ctypes.c_void_p(t.data_ptr()) for t in (slots, mapping, status))
    enc = N.lib.slime_rs_encode_objects_chunked
    for bad_cs, stride in ((4 * L - 4, total * cs), (4 * L + 2, total * cs), (cs, total * cs - 4)):
        assert enc(plan._h, p, stride, bad_cs, S, nobj, mp, sp, None) == N.ERR_INVALID_ARG, (bad_cs, stride)
        if bad_cs != cs:
            assert N.lib.slime_rs_decode_objects_chunked(plan._h, p, stride, bad_cs, L, nobj, mp, None) == \
                N.ERR_INVALID_ARG, bad_cs
    assert enc(plan._h, p, total * cs, cs, S, nobj, mp, sp, None) == 0
    assert enc(plan._h, p, total * cs, 0, S, nobj, mp, sp, None) == 0
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        D.encode_objects(plan, slots, total * cs, S, nobj, mapping, status, chunk_stride=4 * L - 4)


# ------------------------------------------------- object entry points (host memory)

def _obj_bytes(rng, S, kind):
    b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
    if kind == "high" and S >= 4:
        b[0:4] = b"\xff\xff\xff\xff"  # mapping 1<<31 (map.go:47)
    if kind == "fallback" and S >= 8:
        b[0:8] = b"\xff\xff\xff\xff\x7f\xff\xff\xff"  # neither 0 nor 1<<31 (TestMapTricky)
    return bytes(b)


def _oracle_reconstruct(chunks, have, mapping, need, size):
    """multi_store.go:215-241 via the oracle: MapToGFWith, RecoverData, MapFromGF, [:Size]."""
    vecs = [OC.map_to_gf_with(bytes(c), mapping) for c in chunks]
    rc, data = OC.recover_data(vecs, have)
    assert rc == 0
    out = b"".join(OC.map_from_gf(mapping, v) for v in data)
    return (out + bytes(max(0, size - len(out))))[:size]


@pytest.mark.parametrize("need,total", [(2, 3), (4, 6), (8, 12), (10, 14), (16, 20), (20, 24), (40, 56)])
@pytest.mark.parametrize("S", [1, 3, 4, 5, 33, 4096, 100003, 3 * (8 << 20) + 13])
@pytest.mark.parametrize("kind", ["plain", "high", "fallback"])
def test_write_chunks_and_reconstruct_vs_oracle(need, total, S, kind):
    # Objects of 3 x 8 MiB + 13 span several pinned ring stages each way.
    from slime_amd import objects
    rng = np.random.default_rng(S * 31 + need)
    obj = _obj_bytes(rng, S, kind)
    m, chunks = objects.write_chunks(obj, need, total)
    if kind == "plain":
        assert m in (0, 1 << 31)
    if kind == "high" and S >= 4:
        assert m == 1 << 31
    # the reference's chunks for the mapping it would pick (the random draw is the library's)
    m_ref, want = _oracle_chunks(obj, need, total, [m] if kind == "fallback" and S >= 8 else [])
    assert m == m_ref
    assert [c.tobytes() for c in chunks] == want
    # reconstruct from the last `need` chunks, and from a mixed set
    for have in (list(range(total - need, total)), sorted(rng.choice(total, size=need, replace=False).tolist())):
        got = objects.reconstruct([chunks[i] for i in have], have, m, S)
        assert got.tobytes() == obj
    assert objects.reconstruct([chunks[i] for i in have], have, m, S).tobytes() == \
        _oracle_reconstruct([chunks[i] for i in have], have, m, need, S)


@pytest.mark.parametrize("need,total", [(8, 12), (10, 14), (3, 5)])
@pytest.mark.parametrize("S", [(2 << 20) + 1, (4 << 20) - 3, (4 << 20) + 5, (6 << 20) + 7])
@pytest.mark.parametrize("kind", ["plain", "high"])
def test_host_windows_either_side_of_the_copy_kernel_threshold(need, total, S, kind):
    """A window moving <= 4 MiB each way crosses PCIe as one copy kernel over
    the pinned ring (host_blit.hip), a larger one through the copy engines
    (rs_capi.cpp dma_spans): objects on both sides of that line, odd sizes
    (4-byte-aligned but not 16-byte-aligned chunk offsets, a partial last
    word), one-window 1<<31 objects (the host sees the flags and the device
    re-encodes), and the Go-API rows at L on both sides."""
    from slime_amd import objects
    rng = np.random.default_rng(S + need)
    obj = _obj_bytes(rng, S, kind)
    m, chunks = objects.write_chunks(obj, need, total)
    m_ref, want = _oracle_chunks(obj, need, total, [])
    assert m == m_ref == (1 << 31 if kind == "high" else m)
    assert [c.tobytes() for c in chunks] == want
    have = sorted(rng.choice(total, size=need, replace=False).tolist())
    got = objects.reconstruct([chunks[i] for i in have], have, m, S)
    assert got.tobytes() == obj
    if kind == "plain":  # the rows path at the same L (CreateParity / RecoverData)
        L = len(chunks[0]) // 4
        data = [np.frombuffer(chunks[j], dtype=">u4").astype(np.uint32) for j in range(need)]
        for idx in (need, total - 1):
            assert np.array_equal(rs.CreateParity(data, idx), OC.create_parity(data, idx)[1])
        code = data + [OC.create_parity(data, need + i)[1] for i in range(total - need)]
        rec = rs.RecoverData([code[i] for i in have], have)
        for g, d in zip(rec, data):
            assert g.size == L and np.array_equal(g, d)


def test_reconstruct_every_pattern_4_6():
    from slime_amd import objects
    rng = np.random.default_rng(46)
    S = 77777
    obj = _obj_bytes(rng, S, "high")
    m, chunks = objects.write_chunks(obj, 4, 6)
    for have in itertools.combinations(range(6), 4):
        assert objects.reconstruct([chunks[i] for i in have], list(have), m, S).tobytes() == obj


def test_reconstruct_corrupt_noncanonical_survivor_matches_reference():
    # A surviving data chunk whose words unmap to values >= p: the reference
    # reduces them mod p (RecoverData applies unit rows); so must we.
    from slime_amd import objects
    need, total, S = 4, 6, 4000
    rng = np.random.default_rng(7)
    obj = _obj_bytes(rng, S, "plain")
    m, chunks = objects.write_chunks(obj, need, total)
    bad = chunks[1].copy()
    bad[0:8] = np.frombuffer(b"\xff\xff\xff\xff\xff\xff\xff\xfb", dtype=np.uint8)
    assert m == 0  # so the corrupt words unmap to 0xFFFFFFFF and 0xFFFFFFFB, both >= p
    have = [0, 1, 4, 5]
    surv = [chunks[0], bad, chunks[4], chunks[5]]
    assert objects.reconstruct(surv, have, m, S).tobytes() == _oracle_reconstruct(surv, have, m, need, S)


def test_reconstruct_size_past_chunks_is_zero_padded():
    from slime_amd import objects
    m, chunks = objects.write_chunks(b"abcdefgh" * 3, 2, 3)
    got = objects.reconstruct([chunks[1], chunks[2]], [1, 2], m, 40).tobytes()
    assert got[:24] == b"abcdefgh" * 3 and got[24:] == bytes(16)


def test_object_entry_points_reuse_caller_buffers():
    from slime_amd import objects
    rng = np.random.default_rng(3)
    obj = rng.integers(0, 256, size=123457, dtype=np.uint8).tobytes()
    cb = objects.chunk_size(len(obj), 4)
    bufs = [np.full(cb + 9, 0xAB, dtype=np.uint8) for _ in range(6)]
    m, chunks = objects.write_chunks(obj, 4, 6, out=bufs)
    assert all(c.ctypes.data == b.ctypes.data for c, b in zip(chunks, bufs))
    assert all((b[cb:] == 0xAB).all() for b in bufs)
    assert [c.tobytes() for c in chunks] == _oracle_chunks(obj, 4, 6)[1]
    dst = np.full(len(obj) + 5, 0xCD, dtype=np.uint8)
    got = objects.reconstruct([chunks[i] for i in (1, 3, 4, 5)], [1, 3, 4, 5], m, len(obj), out=dst)
    assert got.ctypes.data == dst.ctypes.data and got.tobytes() == obj and (dst[len(obj):] == 0xCD).all()


def test_fuzz_random_shapes_and_layouts(torch_dev):
    """Seeded random shapes across every kernel form (k = 1..16 templates, the
    wide kernel, column segments, padded and misaligned strides): encode in
    place, then rebuild a random erasure set into a separate buffer."""
    torch = torch_dev
    from slime_amd import device as D
    rng = random.Random(0xF022)
    for case in range(48):
        need = rng.choice([1, 2, 3, 4, 5, 7, 8, 9, 10, 12, 15, 16, 17, 24, 31, 33, 40])
        total = need + rng.randint(1, min(12, 100 - need))
        L = rng.choice([1, 2, 3, 5, 63, 64, 255, 1024, 4099, 8192 + rng.randint(0, 7), rng.randint(1, 30000)])
        nobj = rng.randint(1, 5)
        pad = rng.choice([0, 0, 1, 3, 4, 64])
        off = rng.randint(0, 3)
        SS = L + pad
        lay = D.layout_of(total, L, SS)
        buf = torch.empty(off + nobj * total * SS, dtype=torch.int32, device="cuda")
        D.fill_symbols(buf, seed=case)
        D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, src_offset=off, dst_offset=off + need * SS)
        torch.cuda.synchronize()
        h = buf.cpu().numpy().view(np.uint32)[off:].reshape(nobj, total, SS)[:, :, :L]
        for o in range(nobj):
            ref = np.ascontiguousarray(h[o].copy())
            OC.encode_object(ref, need, total)
            assert np.array_equal(h[o], ref), (case, need, total, L, nobj, pad, off, o)
        e = rng.randint(1, total - need)
        erase = sorted(rng.sample(range(total), e))
        have = [i for i in range(total) if i not in erase][:need]
        out = torch.zeros(nobj * e * L + 1, dtype=torch.int32, device="cuda")
        D.Plan.reconstruct(need, total, have, erase)(buf, lay, out, D.layout_of(e, L), L, nobj, src_offset=off,
                                                     dst_offset=1)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)[1:].reshape(nobj, e, L)
        for o in range(nobj):
            for i, t in enumerate(erase):
                assert np.array_equal(got[o, i], h[o, t]), (case, need, total, L, erase, o, t)


def test_fuzz_byte_path_random_shapes(torch_dev):
    """Seeded random shapes on the fused byte path (writeChunks / reconstruct on
    device, multi_store.go:526-557 and 185-242): the VALU, k-template and
    matrix-core encodes with the mid-object switch, a word >= p planted at the
    start, a random place or the last whole word (an edge column) of half the
    objects, object sizes with every remainder mod 4, then a random erasure set
    repaired in place from shuffled survivors; every chunk byte against the
    oracle's framing."""
    torch = torch_dev
    from slime_amd import device as D
    rng = random.Random(0xB17E)
    for case in range(24):
        need = rng.choice([1, 2, 3, 4, 8, 10, 12, 16, 17, 24, 25, 32, 33, 40, 48, 64, 65, 72, 80, 96])
        total = need + rng.randint(1, min(20, 100 - need))
        S = rng.choice([1, 3, 4, 17, 4097, rng.randint(1, 1 << 16), rng.randint(1 << 18, 3 << 20)])
        nobj = rng.randint(1, 6)
        nrng = np.random.default_rng(case)
        objs = []
        for _ in range(nobj):
            b = bytearray(nrng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
            nfull = S // 4
            if nfull:
                w = np.frombuffer(b, dtype=">u4", count=nfull).copy()
                w[(w >= 0x7FFFFFFB) & (w < 0x80000000)] ^= 0x00100000  # no random fallback
                w[w >= 4294967291] = 0x01020304
                b[:4 * nfull] = w.astype(">u4").tobytes()
                if rng.random() < 0.5:
                    a = rng.choice([0, rng.randrange(nfull), nfull - 1])
                    b[4 * a: 4 * a + 4] = b"\xff\xff\xff\xfd"
            objs.append(bytes(b))
        slots, L, chunk, stride = _make_slots(torch, objs, need, total, extra=64)
        mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
        status = torch.empty(nobj, dtype=torch.int32, device="cuda")
        D.encode_objects(D.Plan.encode(need, total), slots, stride, S, nobj, mapping, status)
        torch.cuda.synchronize()
        assert status.cpu().numpy().tolist() == [0] * nobj, (case, need, total, S)
        ms = mapping.cpu().numpy().view(np.uint32)
        h = slots.cpu().numpy()
        for o, obj in enumerate(objs):
            m, chunks = _oracle_chunks(obj, need, total)
            assert ms[o] == m, (case, need, total, S, o)
            for c in range(total):
                got = h[o * stride + c * chunk: o * stride + (c + 1) * chunk].tobytes()
                assert got == chunks[c], (case, need, total, S, o, c)
            assert (h[o * stride + total * chunk: (o + 1) * stride] == 0xA5).all(), (case, "wrote past the chunks")
        truth = slots.clone()
        erase = sorted(rng.sample(range(total), rng.randint(1, total - need)))
        have = [i for i in range(total) if i not in erase]
        rng.shuffle(have)
        rec = D.Plan.reconstruct(need, total, have[:need], erase).set_outputs(erase)
        slots.view(nobj, stride)[:, : total * chunk].view(nobj, total, chunk)[:, erase, : 4 * L] = 0x5A
        D.decode_objects(rec, slots, stride, L, nobj, mapping)
        torch.cuda.synchronize()
        assert torch.equal(slots, truth), (case, need, total, S, erase)


@pytest.mark.gpu
@pytest.mark.parametrize("need,total", [(4, 6), (8, 12), (10, 14), (16, 20), (20, 24), (17, 30), (40, 56)])
def test_fallback_kernel_vs_oracle(torch_dev, need, total):
    """The non-pipelined apply kernel (shards >= 4 GiB; kernel_pipeline(0)) at
    small sizes: encode in place, misaligned bases, reconstruct into a
    separate buffer -- and the pipelined product form on the same inputs."""
    torch = torch_dev
    from slime_amd import device as D
    nobj, L = 3, 3 * 1024 + 5
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    erase = [0, need]
    have = [i for i in range(total) if i not in erase][:need]
    rec = D.Plan.reconstruct(need, total, have, erase)
    outs = {}
    before = N.lib.slime_rs_kernel_pipeline(-1)
    for pipe in ("0", "1"):
        N.lib.slime_rs_kernel_pipeline(int(pipe))
        for off in (0, 1):
            buf = torch.empty(off + nobj * total * L, dtype=torch.int32, device="cuda")
            D.fill_symbols(buf, seed=need * 31 + off)
            plan(buf, lay, buf, lay, L, nobj, src_offset=off, dst_offset=off + need * L)
            out = torch.zeros(nobj * len(erase) * L, dtype=torch.int32, device="cuda")
            rec(buf, lay, out, D.layout_of(len(erase), L), L, nobj, src_offset=off)
            torch.cuda.synchronize()
            h = buf.cpu().numpy().view(np.uint32)[off:].reshape(nobj, total, L)
            got = out.cpu().numpy().view(np.uint32).reshape(nobj, len(erase), L)
            for o in range(nobj):
                ref = np.ascontiguousarray(h[o].copy())
                OC.encode_object(ref, need, total)
                assert np.array_equal(h[o], ref), (pipe, off, o)
                for i, t in enumerate(erase):
                    assert np.array_equal(got[o, i], h[o, t]), (pipe, off, o, t)
            outs[(pipe, off)] = h.copy()
    N.lib.slime_rs_kernel_pipeline(before)
    for off in (0, 1):
        assert np.array_equal(outs[("0", off)], outs[("1", off)])


# ------------------------------------------------- round-2 boundary behaviour

@pytest.mark.parametrize("need", [1, 3, 8])
@pytest.mark.parametrize("S", [1, 5, 4096, 100003])
@pytest.mark.parametrize("kind", ["plain", "high", "fallback"])
def test_write_chunks_without_parity_vs_oracle(need, S, kind):
    """need == total (checkConfig, multi_config.go:36; 1-of-1 in multi_test.go:179):
    chunks are the reference's MapFromGF(m, splitVector parts) and the object
    reconstructs from them."""
    from slime_amd import objects
    rng = np.random.default_rng(S * 7 + need)
    obj = _obj_bytes(rng, S, kind)
    m, chunks = objects.write_chunks(obj, need, need)
    m_ref, want = _oracle_chunks(obj, need, need, [m] if kind == "fallback" and S >= 8 else [])
    assert m == m_ref
    assert [c.tobytes() for c in chunks] == want
    assert objects.reconstruct(chunks, list(range(need)), m, S).tobytes() == obj


@pytest.mark.parametrize("cut", [1, 2, 3])
def test_reconstruct_partial_word_chunks_vs_oracle(cut):
    """Survivors whose length is not a multiple of 4 (truncated stored chunks):
    MapToGFWith zero-pads the partial word (map.go:16-33) and every recovered
    row is that long (vector.go:80-85), as the reference computes."""
    from slime_amd import objects
    rng = np.random.default_rng(cut)
    need, total, S = 4, 6, 40000
    obj = _obj_bytes(rng, S, "high")
    m, chunks = objects.write_chunks(obj, need, total)
    have = [1, 2, 4, 5]
    surv = [chunks[i][:-cut].tobytes() for i in have]
    for size in (S, S + 100):
        got = objects.reconstruct(surv, have, m, size).tobytes()
        assert got == _oracle_reconstruct(surv, have, m, need, size)


def test_plan_cache_stays_bounded_on_device():
    """RecoverData over many distinct survivor sets (20/40): the host plan cache
    stays at its capacity and evicted plans free their device tables
    (vector.go:69-77 inverts per survivor set)."""
    import itertools as it
    rng = np.random.default_rng(2040)
    N.set_plan_cache_capacity(8)
    try:
        need, total, L = 20, 40, 37
        data = rand_vecs(rng, need, L, canonical=True, edges=False)
        code = data + [OC.create_parity(data, need + i)[1] for i in range(total - need)]
        base = N.plan_cache_stats()
        seen = 0
        for have in it.islice(it.combinations(range(total), need), 0, 100000, 997):
            got = rs.RecoverData([code[i] for i in have], list(have))
            assert all(np.array_equal(g, d) for g, d in zip(got, data))
            seen += 1
        st = N.plan_cache_stats()
        assert seen >= 60
        assert st["live"] <= 8 and st["capacity"] == 8
        assert st["evictions"] - base["evictions"] >= seen - 8
        assert st["device_tables"] <= base["device_tables"] + 8
    finally:
        N.set_plan_cache_capacity(256)


def test_set_outputs_refused_after_launch(torch_dev):
    """A plan's output table is fixed once it has launched (launches in flight read it)."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, L = 4, 6, 1024
    buf = _objects(torch, 1, total, L, seed=3)
    lay = D.layout_of(total, L)
    rec = D.Plan.reconstruct(need, total, [2, 3, 4, 5], [0, 1]).set_outputs([0, 1])  # before: fine
    rec(buf, lay, buf, lay, L, 1)
    torch.cuda.synchronize()
    with pytest.raises(slime_amd.NativeError) as e:
        rec.set_outputs([1, 0])
    assert e.value.code == N.ERR_INVALID_ARG


def test_device_pool_routes_unpinned_calls():
    """Host calls that name no device go through the device pool; on a 1-GPU box
    every call lands on device 0 (8-GPU behaviour: DESIGN.md, unmeasured)."""
    n = N.device_count()
    before = [N.pool_calls(d)[0] for d in range(n)]
    for _ in range(6):
        assert rs.CreateParity([[0, 0, 0], [1, 2, 3]], 2).tolist() == [3, 6, 9]
    after = [N.pool_calls(d) for d in range(n)]
    assert sum(a[0] - b for a, b in zip(after, before)) == 6
    assert all(a[1] == 0 for a in after)
    if n == 1:
        assert after[0][0] - before[0] == 6
    # a pinned call bypasses the pool's choice but still counts on its device
    buf = ctypes.create_string_buffer(128)
    call = N.Call(0, ctypes.cast(buf, ctypes.c_char_p), 128)
    x = np.array([1, 2, 3], dtype=np.uint32)
    out = np.zeros(3, dtype=np.uint32)
    ptrs = (ctypes.c_void_p * 2)(x.ctypes.data, x.ctypes.data)
    lens = (ctypes.c_uint64 * 2)(3, 3)
    assert N.lib.slime_rs_create_parity_ex(ctypes.byref(call), ptrs, lens, 2, 2, out.ctypes.data) == 0
    assert buf.value == b"" and out.tolist() == OC.create_parity([x, x], 2)[1].tolist()


def test_concurrent_host_callers_match_oracle():
    """The reference's callers are concurrent (25 HTTP goroutines by default,
    main.go:107-109; scrubbers, multi.go:54-58).  Eight threads run the object
    entry points and the Go-API data path at once, on mixed shapes and survivor
    sets, with the plan cache capped below the number of live survivor sets, so
    workspaces, the copy pool, the device pool and plan eviction all run under
    contention.  Every result is checked against the oracle's framing."""
    import threading
    from slime_amd import objects
    N.set_plan_cache_capacity(4)
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(1000 + t)
            for it in range(6):
                need = int(rng.choice([2, 4, 8, 10, 17]))
                total = need + int(rng.integers(0, 5))
                S = int(rng.choice([5, 4096, 100003, 3 << 20]))
                obj = _obj_bytes(rng, S, "high" if it % 3 == 0 else "plain")
                m, chunks = objects.write_chunks(obj, need, total)
                m_ref, want = _oracle_chunks(obj, need, total)
                if m != m_ref or [c.tobytes() for c in chunks] != want:
                    errors.append(("write_chunks", t, it, need, total, S))
                    continue
                have = sorted(rng.choice(total, size=need, replace=False).tolist())
                got = objects.reconstruct([chunks[i] for i in have], have, m, S)
                if got.tobytes() != obj:
                    errors.append(("reconstruct", t, it, need, total, S, have))
                L = 1 + int(rng.integers(0, 5000))
                data = rand_vecs(rng, need, L)
                idx = need + int(rng.integers(0, max(1, total - need) + 1))
                if not np.array_equal(rs.CreateParity(data, idx), OC.create_parity(data, idx)[1]):
                    errors.append(("CreateParity", t, it, need, idx))
                code = [np.ascontiguousarray(OC.create_parity(data, i)[1]) for i in range(need + 3)]
                hv = sorted(rng.choice(need + 3, size=need, replace=False).tolist())
                rec = rs.RecoverData([code[i] for i in hv], hv)
                ref = OC.recover_data([code[i] for i in hv], hv)[1]
                if not all(np.array_equal(a, b) for a, b in zip(rec, ref)):
                    errors.append(("RecoverData", t, it, need, hv))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(("exception", t, repr(e)))

    try:
        ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for th in ts:
            th.start()
        for th in ts:
            th.join()
    finally:
        N.set_plan_cache_capacity(256)
    assert not errors, errors[:5]
    st = N.plan_cache_stats()
    assert st["live"] <= 256


@pytest.mark.parametrize("need", list(range(17, 33)))
def test_k17_to_32_pipelined_kernel_vs_oracle(torch_dev, need):
    """17 <= k <= 32 runs the k-template pipelined kernel (rs_apply_k32.hip):
    every k, non-canonical inputs (x >= p, 0xFFFFFFFF), a column tail past the
    last 16-byte vector, 1..r output rows, encode in place and a reconstruct of
    data and parity rows into a separate buffer."""
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(need)
    r = 1 + need % 5
    total, nobj = need + r, 2
    L = 4 * 1024 + 1 + need % 3  # tail columns
    h = np.stack([np.stack(rand_vecs(rng, total, L)) for _ in range(nobj)])  # [obj][shard][L]
    buf = torch.from_numpy(h.reshape(-1).view(np.int32).copy()).cuda()
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
    for o in range(nobj):
        ref = np.ascontiguousarray(h[o].copy())
        OC.encode_object(ref, need, total)
        assert np.array_equal(got[o], ref), o
    erase = sorted(rng.choice(total, size=r, replace=False).tolist())
    have = [i for i in range(total) if i not in erase][:need]
    out = torch.zeros(nobj * r * L, dtype=torch.int32, device="cuda")
    D.Plan.reconstruct(need, total, have, erase)(buf, lay, out, D.layout_of(r, L), L, nobj)
    torch.cuda.synchronize()
    rec = out.cpu().numpy().view(np.uint32).reshape(nobj, r, L)
    for o in range(nobj):
        for i, t in enumerate(erase):
            # RecoverData returns canonical residues: a non-canonical data symbol x comes back as x mod p
            want = (got[o, t].astype(np.uint64) % P).astype(np.uint32)
            assert np.array_equal(rec[o, i], want), (o, t)


@pytest.mark.parametrize("need,total", [(17, 18), (19, 24), (24, 30), (27, 32), (31, 36), (32, 40)])
@pytest.mark.parametrize("S", [33, 65537, (1 << 20) + 7])
def test_k17_to_32_byte_kernels_vs_oracle(torch_dev, kernel_form, need, total, S):
    """17 <= need <= 32 byte kernels (rs_bytes_k32.hip in the pipelined form):
    encode_objects against the oracle's writeChunks framing (mappings 0 and
    1<<31), then repair of erased data and parity chunks in place."""
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(S + need)
    objs = [rng.integers(0, 256, size=S, dtype=np.uint8).tobytes() for _ in range(2)]
    b = bytearray(objs[1]); b[0:4] = b"\xff\xff\xff\xfd"; objs[1] = bytes(b)  # mapping 1<<31
    slots, L, chunk, stride = _make_slots(torch, objs, need, total, extra=8)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(2, dtype=torch.int32, device="cuda")
    status = torch.empty(2, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, 2, mapping, status)
    torch.cuda.synchronize()
    assert status.cpu().numpy().tolist() == [0, 0]
    h = slots.cpu().numpy()
    ms = mapping.cpu().numpy().view(np.uint32)
    for o, obj in enumerate(objs):
        m, chunks = _oracle_chunks(obj, need, total)
        assert ms[o] == m
        for c in range(total):
            assert h[o * stride + c * chunk: o * stride + (c + 1) * chunk].tobytes() == chunks[c], (o, c)
    truth = slots.clone()
    r = total - need
    erase = sorted(set([0, need - 1] + list(range(need, total))[:max(0, r - 2)]))[:r]
    have = [i for i in range(total) if i not in erase][:need]
    rec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
    v = slots.view(2, stride)[:, : total * chunk].view(2, total, chunk)
    v[:, erase, :] = 0x5A
    D.decode_objects(rec, slots, stride, L, 2, mapping)
    torch.cuda.synchronize()
    assert torch.equal(slots, truth), erase


def test_on_device_restores_the_threads_previous_selection():
    """N.on_device restores whatever the thread had selected before the block:
    a direct slime_rs_select_device call, an enclosing block, or nothing."""
    assert N.lib.slime_rs_selected_device() == N.ANY_DEVICE
    N.check(N.lib.slime_rs_select_device(0))
    try:
        with N.on_device(0):
            with N.on_device(0):
                assert N.lib.slime_rs_selected_device() == 0
            assert N.lib.slime_rs_selected_device() == 0
        assert N.lib.slime_rs_selected_device() == 0, "the direct selection survives the block"
    finally:
        N.check(N.lib.slime_rs_select_device(N.ANY_DEVICE))
    with N.on_device(0):
        pass
    assert N.lib.slime_rs_selected_device() == N.ANY_DEVICE


_SMALL_CALLS = r'''
import hashlib, json, sys
import numpy as np
from slime_amd import objects, rs
out = []
for need, total, S, kind in json.loads(sys.argv[1]):
    rng = np.random.default_rng(S * 13 + need)
    b = bytearray(rng.integers(0, 256, size=S, dtype=np.uint8).tobytes())
    if kind == "high" and S >= 4:
        b[0:4] = b"\xff\xff\xff\xff"
    if kind == "fallback" and S >= 8:
        b[0:8] = b"\xff\xff\xff\xff\x7f\xff\xff\xff"
    m, chunks = objects.write_chunks(bytes(b), need, total)
    have = list(range(total - need, total))
    back = objects.reconstruct([chunks[i] for i in have], have, m, S).tobytes() == bytes(b)
    rows = [np.frombuffer(chunks[j], dtype=np.uint32).copy() for j in range(need)]
    par = rs.CreateParity(rows, total - 1)
    out.append([m, [hashlib.sha256(c.tobytes()).hexdigest() for c in chunks], back,
                hashlib.sha256(np.ascontiguousarray(par).tobytes()).hexdigest()])
print(json.dumps(out))
'''


def test_small_calls_same_with_direct_and_tiny_rules_off():
    """The small-call rules (rs_capi.cpp run_windows "direct": a one-window
    call's kernel on the mapped pinned stage; kernels.hpp queue_spread: one
    block's units, or one object's up to 1024, on the static kernels) change no
    byte: a child process with them off (SLIME_RS_DIRECT_KIB=0,
    SLIME_RS_TINY_UNITS=0, SLIME_RS_ONE_OBJECT_UNITS=0: copy kernels and the
    dynamic schedule; one-window objects of 4-6 MiB take the copy kernel or the
    copy engines) gives the same mappings, chunks, round trips and parity
    rows as this process, and this process matches the oracle.  "fallback"
    objects draw their mapping at random, so only plain and 1<<31 objects are
    compared across processes."""
    import hashlib
    import json
    import os
    import subprocess
    import sys
    cases = [[need, total, S, kind] for need, total in ((4, 6), (8, 12), (10, 14))
             for S in (1, 5, 4096, 65536 + 3, 200003, (3 << 20) + 1) for kind in ("plain", "high")]
    # one-window objects either side of the copy kernel's 4 MiB upload limit (direct off in the child)
    cases += [[8, 12, S, kind] for S in ((4 << 20) - 3, (6 << 20) + 7) for kind in ("plain", "high")]
    env = dict(os.environ, SLIME_RS_DIRECT_KIB="0", SLIME_RS_TINY_UNITS="0", SLIME_RS_ONE_OBJECT_UNITS="0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-c", _SMALL_CALLS, json.dumps(cases)], env=env, cwd=root,
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    child = json.loads(res.stdout.strip().splitlines()[-1])
    from slime_amd import objects
    for (need, total, S, kind), (cm, chashes, cback, cpar) in zip(cases, child):
        rng = np.random.default_rng(S * 13 + need)
        obj = _obj_bytes(rng, S, kind)
        m, chunks = objects.write_chunks(obj, need, total)
        m_ref, want = _oracle_chunks(obj, need, total, [])
        assert m == m_ref == cm, (need, S, kind)
        assert [c.tobytes() for c in chunks] == want
        assert [hashlib.sha256(w).hexdigest() for w in want] == chashes, (need, S, kind)
        assert cback, (need, S, kind)
        rows = [np.frombuffer(chunks[j], dtype=np.uint32).copy() for j in range(need)]
        par = rs.CreateParity(rows, total - 1)
        _, par_ref = OC.create_parity(rows, total - 1)
        assert np.array_equal(np.asarray(par, dtype=np.uint32), np.asarray(par_ref, dtype=np.uint32))
        assert hashlib.sha256(np.ascontiguousarray(par).tobytes()).hexdigest() == cpar, (need, S, kind)
