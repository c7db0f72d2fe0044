"""GPU parity of the matrix-core apply kernel (rs_apply_mfma.hip): wide codes
(k >= 33, and 17 <= k <= 32 with k x rows >= 128; up to 32 output rows) as an
exact int8-limb product on
v_mfma_i32_16x16x64_i8, against the C oracle (applyMatrix,
internal/rs/vector.go:90-102) and against the VALU kernels in the same process
(slime_rs_kernel_matrix_cores 0/1).  Bit-exact: integer field arithmetic.

Cases: every K-step count 3..7 (k = 33..112), 1..32 output rows (M-tile
padding), column tails past the last 16-byte vector and partial wave tiles,
non-canonical inputs (x >= p, 0xFFFFFFFF), arbitrary coefficient matrices
including non-canonical coefficients, shuffled survivor indices, padded shard
strides, a separate destination, and rows > 32 (the VALU kernels take over).
"""
import numpy as np
import pytest

from slime_amd import _native as N
from slime_amd import gf
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu

P = gf.MaxVal
EDGES = np.array([0, 1, 2, P - 1, P, P + 1, P + 4, 0xFFFFFFFF, 0x7FFFFFFF, 0x80000000, 0x80808080],
                 dtype=np.uint32)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


@pytest.fixture(params=[1, 0], ids=["mfma", "valu"])
def matrix_cores(request):
    """Matrix cores (product for k >= 33) and the VALU kernels."""
    prev = N.lib.slime_rs_kernel_matrix_cores(-1)
    N.check(N.lib.slime_rs_kernel_matrix_cores(request.param))
    yield request.param
    N.check(N.lib.slime_rs_kernel_matrix_cores(prev))


def _rand(rng, shape):
    x = rng.integers(0, 2**32, size=shape, dtype=np.uint64).astype(np.uint32)
    flat = x.reshape(-1)
    n = min(flat.size, 64)
    flat[rng.choice(flat.size, size=n, replace=False)] = rng.choice(EDGES, size=n)
    return x


def _apply_ref(coeff, x):
    """out[i] = sum_j coeff[i][j] * x[j] mod p over columns (exact, numpy uint64 in pieces)."""
    c = coeff.astype(np.uint64) % P
    xs = x.astype(np.uint64) % P
    out = np.zeros((c.shape[0], x.shape[1]), dtype=np.uint64)
    for j in range(c.shape[1]):
        out = (out + (c[:, j:j + 1] * xs[j:j + 1]) % P) % P
    return out.astype(np.uint32)


@pytest.mark.parametrize("need,total", [(33, 34), (33, 50), (40, 56), (47, 48), (48, 64), (64, 80), (80, 100),
                                        (64, 96), (99, 100), (17, 25), (24, 32), (31, 40), (20, 24),
                                        # five K steps with a clamped last step (uniform offsets); six, seven
                                        (72, 90), (65, 81), (90, 100), (100, 116)])
@pytest.mark.parametrize("L", [1, 5, 64, 67, 1001, 4096 + 3])
def test_encode_vs_oracle(torch_dev, matrix_cores, need, total, L):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(need * 131 + L)
    nobj = 2
    h = _rand(rng, (nobj, total, L))
    buf = torch.from_numpy(h.reshape(-1).view(np.int32).copy()).cuda()
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
    for o in range(nobj):
        ref = np.ascontiguousarray(h[o].copy())
        OC.encode_object(ref, need, total)
        assert np.array_equal(got[o], ref), (o, need, total, L)


@pytest.mark.parametrize("need,total,L,nobj", [(80, 100, 200, 300), (40, 56, 64, 500), (64, 80, 1500, 40),
                                               (33, 50, 7, 200), (72, 90, 3, 64), (96, 100, 2047, 9)])
def test_many_short_objects_vs_oracle(torch_dev, need, total, L, nobj):
    """Batches of many short objects (at most 32 tiles each: the matrix-core
    kernel's flat walk over every object's tiles, rs_apply_mfma_kernel): encode
    in place, then rebuild a data-and-parity erasure set into a separate
    buffer; every object against the oracle."""
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(need * 7 + L + nobj)
    h = _rand(rng, (nobj, total, L))
    buf = torch.from_numpy(h.reshape(-1).view(np.int32).copy()).cuda()
    lay = D.layout_of(total, L)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
    for o in range(nobj):
        ref = np.ascontiguousarray(h[o].copy())
        OC.encode_object(ref, need, total)
        assert np.array_equal(got[o], ref), (o, need, total, L)
    erase = sorted({0, need - 1, need, total - 1})
    have = [i for i in range(total) if i not in erase][:need]
    e = len(erase)
    out = torch.zeros(nobj * e * L, dtype=torch.int32, device="cuda")
    D.Plan.reconstruct(need, total, have, erase)(buf, lay, out, D.layout_of(e, L), L, nobj)
    torch.cuda.synchronize()
    rec = out.cpu().numpy().view(np.uint32).reshape(nobj, e, L)
    for o in range(nobj):
        for i, t in enumerate(erase):  # rebuilt as canonical residues (the data holds words >= p)
            assert np.array_equal(rec[o, i], got[o, t] % P), (o, t)


@pytest.mark.parametrize("need,total,nerase", [(64, 80, 16), (40, 56, 5), (50, 82, 32), (96, 100, 4), (33, 50, 17),
                                               (72, 90, 18), (80, 100, 20), (90, 100, 10), (100, 116, 16)])
def test_reconstruct_shuffled_survivors_separate_dst(torch_dev, matrix_cores, need, total, nerase):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(total * 7 + nerase)
    L, nobj, ss = 3 * 1024 + 7, 3, 3 * 1024 + 64  # padded shard stride
    data = _rand(rng, (nobj, need, L)) % P
    code = np.zeros((nobj, total, ss), dtype=np.uint32)
    for o in range(nobj):
        ref = np.zeros((total, L), dtype=np.uint32)
        ref[:need] = data[o]
        OC.encode_object(ref, need, total)
        code[o, :, :L] = ref
    buf = torch.from_numpy(code.reshape(-1).view(np.int32).copy()).cuda()
    erase = sorted(rng.choice(total, size=nerase, replace=False).tolist())
    have = [i for i in range(total) if i not in erase]
    rng.shuffle(have)
    have = have[:need]
    out = torch.zeros(nobj * nerase * L, dtype=torch.int32, device="cuda")
    D.Plan.reconstruct(need, total, have, erase)(buf, D.layout_of(total, L, ss), out, D.layout_of(nerase, L), L, nobj)
    torch.cuda.synchronize()
    rec = out.cpu().numpy().view(np.uint32).reshape(nobj, nerase, L)
    for o in range(nobj):
        for i, t in enumerate(erase):
            assert np.array_equal(rec[o, i], code[o, t, :L]), (o, t)


@pytest.mark.parametrize("rows,k", [(1, 33), (3, 47), (5, 64), (17, 70), (31, 99), (32, 112), (33, 64), (40, 100)])
def test_arbitrary_matrix_noncanonical_coefficients(torch_dev, matrix_cores, rows, k):
    """Plan.matrix with random coefficients, a quarter of them >= p or at the
    digit window's edges; rows 33 and 40 exceed the matrix-core table (VALU)."""
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(rows * 1000 + k)
    coeff = rng.integers(0, 2**32, size=(rows, k), dtype=np.uint64).astype(np.uint32)
    edge = np.array([0, 1, P - 1, P, 0xFFFFFFFF, 2139062143, 2139062144, 2155905147, 256], dtype=np.uint32)
    mask = rng.random((rows, k)) < 0.25
    coeff[mask] = rng.choice(edge, size=int(mask.sum()))
    L, nobj = 2 * 1024 + 3, 2
    shards = [int(s) for s in rng.permutation(k + 5)[:k]]  # k input shards out of k + 5, any order
    src = _rand(rng, (nobj, k + 5, L))
    sbuf = torch.from_numpy(src.reshape(-1).view(np.int32).copy()).cuda()
    dbuf = torch.zeros(nobj * rows * L, dtype=torch.int32, device="cuda")
    D.Plan.matrix(coeff, shards)(sbuf, D.layout_of(k + 5, L), dbuf, D.layout_of(rows, L), L, nobj)
    torch.cuda.synchronize()
    got = dbuf.cpu().numpy().view(np.uint32).reshape(nobj, rows, L)
    for o in range(nobj):
        want = _apply_ref(coeff, src[o][shards])
        assert np.array_equal(got[o], want), o


def test_matrix_cores_match_valu_large(torch_dev):
    """64/80 on 3 objects of 4 Mi symbols per shard: the two kernel families
    agree on every symbol; one object's first 64 Ki columns vs the oracle."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, L, nobj = 64, 80, 1 << 22, 3
    lay = D.layout_of(total, L)
    buf = D.device_empty(nobj * total * L, torch.int32, 0)
    D.fill_symbols(buf, 4242)
    prev = N.lib.slime_rs_kernel_matrix_cores(-1)
    try:
        outs = []
        for mode in (1, 0):
            N.check(N.lib.slime_rs_kernel_matrix_cores(mode))
            out = torch.zeros(nobj * (total - need) * L, dtype=torch.int32, device="cuda")
            D.Plan.encode(need, total)(buf, lay, out, D.layout_of(total - need, L), L, nobj)
            torch.cuda.synchronize()
            outs.append(out)
        assert torch.equal(outs[0], outs[1])
    finally:
        N.check(N.lib.slime_rs_kernel_matrix_cores(prev))
    cols = 1 << 16
    h = buf.view(nobj, total, L)[1, :need, :cols].cpu().numpy().view(np.uint32)
    ref = np.zeros((total, cols), dtype=np.uint32)
    ref[:need] = h
    OC.encode_object(ref, need, total)
    got = outs[0].view(nobj, total - need, L)[1, :, :cols].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, ref[need:])


def test_matrix_cores_switch():
    assert N.lib.slime_rs_kernel_matrix_cores(-1) in (0, 1)
    assert N.lib.slime_rs_kernel_matrix_cores(2) != 0


# ---------------------------------------------------------------- byte path
# writeChunks / reconstruct on chunk bytes (rs_bytes_mfma.hip): the encode's
# matrix-core interior tiles with MapToGF flags and the VALU edge step, the
# re-encode of 1<<31 objects, the decode; every chunk byte vs the oracle's
# framing (map.go:15-113, multi_store.go:185-242, 526-557).

def _byte_objects(rng, S, n):
    objs = [rng.integers(0, 256, size=S, dtype=np.uint8).tobytes() for _ in range(n)]
    nfull = S // 4
    if nfull >= 8:
        b = bytearray(objs[1]); a = int(0.6 * (nfull - 1)); b[4 * a: 4 * a + 4] = b"\xff\xff\xff\xfd"
        objs[1] = bytes(b)  # a word >= p mid-object: mapping 1<<31
        b = bytearray(objs[2]); b[4 * (nfull - 1): 4 * nfull] = b"\xff\xff\xff\xfe"
        objs[2] = bytes(b)  # on the last whole word (an edge step)
    return objs


@pytest.mark.parametrize("need,total,S", [(33, 50, (1 << 20) + 7), (40, 56, 3 * (1 << 20) + 3), (64, 80, (4 << 20) + 1),
                                          (80, 100, 2 << 20), (99, 100, 99999), (47, 48, 65537), (64, 96, 5 << 20),
                                          (48, 64, 777), (32, 40, (1 << 20) + 3), (28, 36, 77777), (25, 33, 4096),
                                          (72, 90, (3 << 20) + 2), (65, 70, 123457)])
def test_bytes_encode_objects_vs_oracle(torch_dev, matrix_cores, need, total, S):
    torch = torch_dev
    from slime_amd import device as D
    from test_gpu_parity import _make_slots, _oracle_chunks
    rng = np.random.default_rng(S + need)
    objs = _byte_objects(rng, S, 4)
    slots, L, chunk, stride = _make_slots(torch, objs, need, total, extra=64)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(4, dtype=torch.int32, device="cuda")
    status = torch.empty(4, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, 4, mapping, status)
    torch.cuda.synchronize()
    assert status.cpu().numpy().tolist() == [0, 0, 0, 0]
    ms = mapping.cpu().numpy().view(np.uint32)
    h = slots.cpu().numpy()
    for o, obj in enumerate(objs):
        m, chunks = _oracle_chunks(obj, need, total)
        assert ms[o] == m, o
        for c in range(total):
            assert h[o * stride + c * chunk: o * stride + (c + 1) * chunk].tobytes() == chunks[c], (o, c)
        assert (h[o * stride + total * chunk: (o + 1) * stride] == 0xA5).all(), "wrote past the chunks"
    if S // 4 >= 8:
        assert ms[1] == 1 << 31 and ms[2] == 1 << 31


@pytest.mark.parametrize("need,total,S,align", [(64, 80, (2 << 20) + 5, 256), (40, 56, 300001, 4096),
                                                (80, 100, 1 << 20, 0), (33, 49, 123457, 0), (24, 32, 300001, 0),
                                                (32, 40, 1 << 20, 256), (17, 25, 65537, 0), (72, 90, (1 << 20) + 3, 256),
                                                (96, 100, 300001, 0), (100, 116, (1 << 20) + 1, 256)])
def test_bytes_decode_objects_repairs_chunks(torch_dev, matrix_cores, need, total, S, align):
    torch = torch_dev
    from slime_amd import device as D
    from test_gpu_parity import _make_chunked_slots, _make_slots
    rng = np.random.default_rng(S + total)
    objs = _byte_objects(rng, S, 3)
    if align:
        slots, L, chunk, stride = _make_chunked_slots(torch, objs, need, total, align)
        cs = dict(chunk_stride=chunk)
    else:
        slots, L, chunk, stride = _make_slots(torch, objs, need, total)
        cs = {}
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(3, dtype=torch.int32, device="cuda")
    status = torch.empty(3, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, 3, mapping, status, **cs)
    torch.cuda.synchronize()
    # The chunks the repair must restore are pinned to the oracle's framing
    # (map.go:15-113, multi_store.go:526-557) first, so every repaired byte is
    # checked against the oracle, not only against the kernel's own encode.
    from test_gpu_parity import _oracle_chunks
    h = slots.cpu().numpy()
    ms = mapping.cpu().numpy().view(np.uint32)
    for o, obj in enumerate(objs):
        m, want = _oracle_chunks(obj, need, total)
        assert ms[o] == m, o
        for c in range(total):
            assert h[o * stride + c * chunk: o * stride + c * chunk + 4 * L].tobytes() == want[c], (o, c)
    truth = slots.clone()
    r = total - need
    for erase in (list(range(min(r, 16))), sorted(rng.choice(total, size=min(r, 20), replace=False).tolist()),
                  [need - 1, total - 1][: r]):
        have = [i for i in range(total) if i not in erase]
        rng.shuffle(have)
        have = have[:need]
        rec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
        v = slots.view(3, stride)[:, : total * chunk].view(3, total, chunk)
        v[:, erase, : 4 * L] = 0x5A
        D.decode_objects(rec, slots, stride, L, 3, mapping, **cs)
        torch.cuda.synchronize()
        assert torch.equal(slots, truth), erase


@pytest.mark.parametrize("need,total,S,nobj", [(80, 100, 65536, 120), (40, 56, 3001, 300), (33, 50, 777, 200),
                                               (96, 100, 20001, 64), (64, 80, 131075, 40), (72, 90, 9, 50)])
def test_bytes_many_short_objects_round_trip(torch_dev, matrix_cores, need, total, S, nobj):
    """Batches of short objects (a few tiles a chunk) take the flat walk in
    the matrix-core byte decode (rs_bytes_mfma.hip dec_ks): encode, pin a
    sample of objects to the oracle's framing (multi_store.go:526-557), erase
    and rebuild every object's chunks byte for byte."""
    torch = torch_dev
    from slime_amd import device as D
    from test_gpu_parity import _make_slots, _oracle_chunks
    rng = np.random.default_rng(S * 7 + nobj)
    objs = _byte_objects(rng, S, nobj)
    slots, L, chunk, stride = _make_slots(torch, objs, need, total)
    plan = D.Plan.encode(need, total)
    mapping = torch.empty(nobj, dtype=torch.int32, device="cuda")
    status = torch.empty(nobj, dtype=torch.int32, device="cuda")
    D.encode_objects(plan, slots, stride, S, nobj, mapping, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    h = slots.cpu().numpy()
    ms = mapping.cpu().numpy().view(np.uint32)
    for o in sorted({0, 1, 2, nobj // 2, nobj - 1}):
        m, want = _oracle_chunks(objs[o], need, total)
        assert ms[o] == m, o
        for c in range(total):
            assert h[o * stride + c * chunk: o * stride + c * chunk + 4 * L].tobytes() == want[c], (o, c)
    truth = slots.clone()
    r = total - need
    for erase in (list(range(min(r, 16))), sorted(rng.choice(total, size=min(r, 20), replace=False).tolist())):
        have = [i for i in range(total) if i not in erase]
        rng.shuffle(have)
        rec = D.Plan.reconstruct(need, total, have[:need], erase).set_outputs(erase)
        v = slots.view(nobj, stride)[:, : total * chunk].view(nobj, total, chunk)
        v[:, erase, : 4 * L] = 0x5A
        D.decode_objects(rec, slots, stride, L, nobj, mapping)
        torch.cuda.synchronize()
        assert torch.equal(slots, truth), erase


def test_objects_over_4gib_take_the_valu_kernels(torch_dev):
    """The matrix-core kernel addresses an object with 32-bit byte offsets; a
    layout whose object spans 4 GiB or more (here 40 shards 128 MiB + 256 B
    apart: 5 GiB) must take the VALU kernels and still be exact."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, L = 40, 44, 4099
    SS = (1 << 25) + 64  # shard stride in symbols
    rng = np.random.default_rng(44)
    buf = torch.zeros(total * SS, dtype=torch.int32, device="cuda")
    data = _rand(rng, (need, L)) % P
    for j in range(need):
        buf[j * SS: j * SS + L] = torch.from_numpy(data[j].view(np.int32).copy()).cuda()
    lay = D.layout_of(total, L, SS)
    D.Plan.encode(need, total)(buf, lay, buf, lay, L, 1, dst_offset=need * SS)
    torch.cuda.synchronize()
    ref = np.zeros((total, L), dtype=np.uint32)
    ref[:need] = data
    OC.encode_object(ref, need, total)
    for i in range(need, total):
        got = buf[i * SS: i * SS + L].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, ref[i]), i
    del buf
    torch.cuda.empty_cache()
