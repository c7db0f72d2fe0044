"""GPU parity of the apply kernels' work schedules (slime_rs_kernel_schedule):
static shares per wave (rs_apply_pipe_kernel) and the dynamic ticket schedule
(rs_apply_queue_kernel), both against the C oracle (applyMatrix,
internal/rs/vector.go:90-102) and against each other, bit-exact.

The dynamic schedule deals units of tiles over eight ticket counters; the cases
here cover units that straddle object ends, empty sub-units, objects shorter
than one tile (only column tails), many objects per counter, and consecutive
launches on one stream and on two streams.  Every launch leaves its counter
set zero and the library hands a set only to a launch no unfinished launch
shares it with, whatever the stream: hipStreamPerThread from two threads, a
stream destroyed with its launch in flight and its handle reused, and a
launch captured into a graph and replayed are all exact.  Graph captures take
the static kernels by default (mode 1) and the dynamic ones under mode 2,
whose sets go back to the pool when the graph and its execs die.
"""
import ctypes
import threading

import numpy as np
import pytest

from slime_amd import _native as N
from slime_amd import gf
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu

P = gf.MaxVal
EDGES = np.array([0, 1, P - 1, P, P + 4, 0xFFFFFFFF, 0x80000000], dtype=np.uint32)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


@pytest.fixture
def schedule():
    before = N.lib.slime_rs_kernel_schedule(-1)
    yield lambda m: N.lib.slime_rs_kernel_schedule(m)
    N.lib.slime_rs_kernel_schedule(before)


def _objects(rng, nobj, total, L):
    h = rng.integers(0, 2**32, size=(nobj, total, L), dtype=np.uint64).astype(np.uint32)
    flat = h.reshape(-1)
    n = min(flat.size, 64)
    flat[rng.choice(flat.size, size=n, replace=False)] = np.resize(EDGES, n)
    return h


def _encode_ref(h, need, total):
    ref = h.copy()
    for o in range(ref.shape[0]):
        obj = np.ascontiguousarray(ref[o])
        OC.encode_object(obj, need, total)
        ref[o] = obj
    return ref


def test_schedule_switch_rejects_unknown_modes(schedule):
    assert schedule(-1) in (0, 1, 2)
    for m in (0, 1, 2):
        assert schedule(3) != 0 and schedule(-1) in (0, 1, 2)
        assert schedule(m) == 0 and schedule(-1) == m


@pytest.mark.parametrize("need,total", [(1, 2), (3, 5), (4, 6), (5, 8), (8, 12), (10, 14), (12, 16), (13, 17),
                                        (16, 20), (17, 20), (24, 28), (25, 30), (32, 40)])
@pytest.mark.parametrize("L,nobj", [(1, 3), (3, 2), (4, 5), (191, 3), (768 + 4, 9), (6 * 768 * 4 + 17, 7),
                                    (65536 + 3, 2)])
def test_encode_every_schedule_vs_oracle(torch_dev, schedule, need, total, L, nobj):
    torch = torch_dev
    from slime_amd import device as D
    rng = np.random.default_rng(need * 1000 + L + nobj)
    h = _objects(rng, nobj, total, L)
    ref = _encode_ref(h, need, total)
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    outs = []
    for m in (0, 1):
        assert schedule(m) == 0
        buf = torch.from_numpy(h.view(np.int32).reshape(-1).copy()).cuda()
        plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
        torch.cuda.synchronize()
        got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
        assert np.array_equal(got, ref), m
        outs.append(got)


@pytest.mark.parametrize("need,total,erase", [(8, 12, [0, 1, 2, 3]), (8, 12, [0, 3, 8, 11]), (10, 14, [1, 12]),
                                              (4, 6, [0, 5]), (20, 24, [0, 1, 2, 3]), (32, 40, [5, 33])])
def test_reconstruct_every_schedule_vs_oracle(torch_dev, schedule, need, total, erase):
    torch = torch_dev
    from slime_amd import device as D
    nobj, L = 11, 4 * 768 * 3 + 9
    rng = np.random.default_rng(sum(erase) + need)
    h = _encode_ref(_objects(rng, nobj, total, L), need, total)
    have = [i for i in range(total) if i not in erase][:need]
    rec = D.Plan.reconstruct(need, total, have, erase)
    for m in (0, 1):
        assert schedule(m) == 0
        src = torch.from_numpy(h.view(np.int32).reshape(-1).copy()).cuda()
        out = torch.zeros(nobj * len(erase) * L, dtype=torch.int32, device="cuda")
        rec(src, D.layout_of(total, L), out, D.layout_of(len(erase), L), L, nobj)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32).reshape(nobj, len(erase), L)
        for i, t in enumerate(erase):
            # RecoverData yields canonical residues; the inputs hold symbols >= p.
            assert np.array_equal(got[:, i], (h[:, t].astype(np.uint64) % P).astype(np.uint32)), (m, t)


def test_consecutive_launches_one_stream_and_two_streams(torch_dev, schedule):
    """Each launch zeroes the counter set of the next launch on its stream:
    back-to-back launches of different sizes on one stream, and two streams
    interleaved, all exact."""
    torch = torch_dev
    from slime_amd import device as D
    need, total = 8, 12
    plan = D.Plan.encode(need, total)
    assert schedule(1) == 0
    rng = np.random.default_rng(7)
    cases = [(5, 3 * 768 * 4 + 1), (1, 1000), (17, 2 * 768 * 4), (2, 7), (9, 768 * 4 * 5 + 33)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(2):
        bufs = []
        for ci, (nobj, L) in enumerate(cases):
            h = _objects(rng, nobj, total, L)
            buf = torch.from_numpy(h.view(np.int32).reshape(-1).copy()).cuda()
            torch.cuda.synchronize()
            s = streams[ci % 2] if rep else torch.cuda.current_stream()
            plan(buf, D.layout_of(total, L), buf, D.layout_of(total, L), L, nobj, stream=s, dst_offset=need * L)
            bufs.append((h, buf, nobj, L))
        torch.cuda.synchronize()
        for h, buf, nobj, L in bufs:
            got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
            assert np.array_equal(got, _encode_ref(h, need, total)), (rep, nobj, L)


def test_dynamic_schedule_full_batch_matches_static(torch_dev, schedule):
    """A C3-sized launch (8/12, 128 x 256 MiB) under both schedules: identical
    parity shards (compared on the device)."""
    torch = torch_dev
    from slime_amd import device as D
    need, total, nobj = 8, 12, 128
    L = (256 << 20) // 4 // need
    lay = D.layout_of(total, L)
    buf = torch.empty(nobj * total * L, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, seed=11)
    plan = D.Plan.encode(need, total)
    first = None
    for m in (0, 1):
        assert schedule(m) == 0
        buf.view(nobj, total, L)[:, need:].zero_()
        plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
        if first is None:
            first = buf.view(nobj, total, L)[:, need:].clone()
    torch.cuda.synchronize()
    assert torch.equal(first, buf.view(nobj, total, L)[:, need:])


@pytest.mark.parametrize("mode", [1, 2])
def test_graph_captured_launches_replay_exactly(torch_dev, schedule, mode):
    """A captured launch replays with the same arguments.  Mode 1 (default)
    captures the static kernels (no counter set bound to the graph); mode 2
    captures the dynamic ones, each holding its counter set for the graph's
    life (every replay leaves it zero for the next).  Replay a captured encode
    and repair three times over changing data, every time exact; destroying
    the graph gives mode 2's sets back."""
    torch = torch_dev
    from slime_amd import device as D
    assert schedule(mode) == 0
    need, total, nobj, L = 8, 12, 9, 3 * 768 * 4 + 5
    erase = [0, 3, 8, 11]
    have = [i for i in range(total) if i not in erase][:need]
    lay = D.layout_of(total, L)
    enc = D.Plan.encode(need, total)
    rec = D.Plan.reconstruct(need, total, have, erase)
    buf = torch.zeros(nobj * total * L, dtype=torch.int32, device="cuda")
    out = torch.zeros(nobj * len(erase) * L, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm the plans' launch path outside the capture
        enc(buf, lay, buf, lay, L, nobj, stream=s, dst_offset=need * L)
    torch.cuda.synchronize()
    _, held0 = N.ticket_sets(0)
    dyn0, fb0 = N.schedule_counts(0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        enc(buf, lay, buf, lay, L, nobj, stream=s, dst_offset=need * L)
        rec(buf, lay, out, D.layout_of(len(erase), L), L, nobj, stream=s)
    torch.cuda.synchronize()
    _, held1 = N.ticket_sets(0)
    dyn1, fb1 = N.schedule_counts(0)
    if mode == 2:
        assert held1 == held0 + 2 and dyn1 == dyn0 + 2, "both captured launches took the dynamic schedule"
    else:
        assert held1 == held0 and dyn1 == dyn0, "both captured launches took the static kernels"
    rng = np.random.default_rng(5)
    for _ in range(3):
        h = _objects(rng, nobj, total, L)
        buf.copy_(torch.from_numpy(h.view(np.int32).reshape(-1)))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ref = _encode_ref(h, need, total)
        got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
        assert np.array_equal(got, ref)
        r = out.cpu().numpy().view(np.uint32).reshape(nobj, len(erase), L)
        for i, t in enumerate(erase):
            assert np.array_equal(r[:, i], (ref[:, t].astype(np.uint64) % P).astype(np.uint32)), t
    del g
    torch.cuda.synchronize()
    assert _held_settles(held0), "the destroyed graph's counter sets went back to the pool"


def _held_settles(want, tries=200):
    """Sets held, polled until it equals `want` (a user object's destructor may
    run on a runtime thread shortly after the graph is destroyed)."""
    import time
    for _ in range(tries):
        if N.ticket_sets(0)[1] == want:
            return True
        time.sleep(0.01)
    return False


class _Graphs:
    """Stream capture and graph execs through the HIP runtime torch loaded."""

    def __init__(self):
        h = _hip()
        V, P_ = ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)
        for name, args in [("hipStreamBeginCapture", [V, ctypes.c_int]), ("hipStreamEndCapture", [V, P_]),
                           ("hipGraphInstantiate", [P_, V, V, V, ctypes.c_size_t]), ("hipGraphLaunch", [V, V]),
                           ("hipGraphExecDestroy", [V]), ("hipGraphDestroy", [V])]:
            getattr(h, name).argtypes = args
        self.h = h

    def capture(self, stream, fn):
        g = ctypes.c_void_p()
        assert self.h.hipStreamBeginCapture(ctypes.c_void_p(stream), 2) == 0  # hipStreamCaptureModeRelaxed
        fn()
        assert self.h.hipStreamEndCapture(ctypes.c_void_p(stream), ctypes.byref(g)) == 0
        return g.value

    def instantiate(self, graph):
        e = ctypes.c_void_p()
        assert self.h.hipGraphInstantiate(ctypes.byref(e), ctypes.c_void_p(graph), None, None, 0) == 0
        return e.value

    def launch(self, exec_, stream):
        assert self.h.hipGraphLaunch(ctypes.c_void_p(exec_), ctypes.c_void_p(stream)) == 0

    def destroy(self, graph=None, exec_=None):
        if exec_ is not None:
            assert self.h.hipGraphExecDestroy(ctypes.c_void_p(exec_)) == 0
        if graph is not None:
            assert self.h.hipGraphDestroy(ctypes.c_void_p(graph)) == 0


def test_graph_held_sets_return_when_graphs_die(torch_dev, schedule):
    """Mode 2: capture, replay and destroy 2000 single-launch graphs.  Each
    captured launch's counter set is bound to its graph by a user object and
    comes back when the graph dies, so the held count returns to its baseline,
    the pool does not grow past its first slabs, and a later uncaptured launch
    still takes the dynamic schedule (rs_apply_queue_kernel)."""
    torch = torch_dev
    from slime_amd import device as D
    assert schedule(2) == 0
    G = _Graphs()
    need, total, nobj, L = 4, 6, 2, 4096 + 4
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    rng = np.random.default_rng(77)
    h = _objects(rng, nobj, total, L)
    buf = torch.from_numpy(h.view(np.int32).reshape(-1).copy()).cuda()
    ref = _encode_ref(h, need, total)
    s = torch.cuda.Stream()
    plan(buf, lay, buf, lay, L, nobj, stream=s, dst_offset=need * L)  # warm
    torch.cuda.synchronize()
    sets0, held0 = N.ticket_sets(0)
    for i in range(2000):
        buf.view(nobj, total, L)[:, need:].zero_()
        torch.cuda.synchronize()
        g = G.capture(s.cuda_stream, lambda: plan(buf, lay, buf, lay, L, nobj, stream=s.cuda_stream,
                                                    dst_offset=need * L))
        e = G.instantiate(g)
        G.launch(e, s.cuda_stream)
        torch.cuda.synchronize()
        if i % 250 == 0:
            assert np.array_equal(buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L), ref), i
        G.destroy(graph=g, exec_=e)
    torch.cuda.synchronize()
    assert _held_settles(held0), (N.ticket_sets(0), held0)
    sets1, _ = N.ticket_sets(0)
    assert sets1 == sets0, "the sets came back: no new slabs for 2000 graphs"
    dyn0, _ = N.schedule_counts(0)
    buf.view(nobj, total, L)[:, need:].zero_()
    plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    dyn1, _ = N.schedule_counts(0)
    assert dyn1 == dyn0 + 1, "an uncaptured launch after the graphs still runs the dynamic schedule"
    assert np.array_equal(buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L), ref)


def test_graph_exec_keeps_its_set_after_the_graph_is_destroyed(torch_dev, schedule):
    """Mode 2, the torch pattern: the graph is destroyed right after it is
    instantiated, and the exec alone holds the captured set.  Two execs of one
    graph replayed one after the other, with uncaptured launches on another
    stream in between, are exact; the set is held until the last exec dies."""
    torch = torch_dev
    from slime_amd import device as D
    assert schedule(2) == 0
    G = _Graphs()
    need, total, nobj, L = 8, 12, 5, 3 * 768 * 4 + 7
    plan = D.Plan.encode(need, total)
    lay = D.layout_of(total, L)
    rng = np.random.default_rng(78)
    buf = torch.zeros(nobj * total * L, dtype=torch.int32, device="cuda")
    s, other = torch.cuda.Stream(), torch.cuda.Stream()
    plan(buf, lay, buf, lay, L, nobj, stream=s, dst_offset=need * L)  # warm
    torch.cuda.synchronize()
    _, held0 = N.ticket_sets(0)
    g = G.capture(s.cuda_stream, lambda: plan(buf, lay, buf, lay, L, nobj, stream=s.cuda_stream,
                                                dst_offset=need * L))
    e1, e2 = G.instantiate(g), G.instantiate(g)
    G.destroy(graph=g)
    torch.cuda.synchronize()
    assert _held_settles(held0 + 1, tries=20), "the execs keep the captured set"
    side = [(_objects(rng, 3, total, 999), 3, 999) for _ in range(4)]
    for rep, ex in enumerate([e1, e2, e1, e2]):
        h = _objects(rng, nobj, total, L)
        buf.copy_(torch.from_numpy(h.view(np.int32).reshape(-1)))
        sh, sn, sL = side[rep]
        sbuf = torch.from_numpy(sh.view(np.int32).reshape(-1).copy()).cuda()
        torch.cuda.synchronize()
        G.launch(ex, s.cuda_stream)
        plan(sbuf, D.layout_of(total, sL), sbuf, D.layout_of(total, sL), sL, sn, stream=other,
             dst_offset=need * sL)  # uncaptured, concurrent: must get another set
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L), _encode_ref(h, need, total))
        assert np.array_equal(sbuf.cpu().numpy().view(np.uint32).reshape(sn, total, sL), _encode_ref(sh, need, total))
    G.destroy(exec_=e1)
    torch.cuda.synchronize()
    assert _held_settles(held0 + 1, tries=20), "one exec is still alive"
    G.destroy(exec_=e2)
    torch.cuda.synchronize()
    assert _held_settles(held0), "the last exec died: the set is back"


@pytest.mark.parametrize("need,total,nobj,S", [(10, 14, 6, (24 << 20) + 5), (40, 56, 6, (24 << 20) + 5),
                                               (80, 100, 6, (24 << 20) + 5), (80, 100, 64, 65541),
                                               (40, 56, 96, 9005)])
def test_graph_captured_byte_path_replays_exactly(torch_dev, need, total, nobj, S):
    """The fused byte path captured into a graph: encode_objects (no scratch
    inside a capture, so no mid-object switch: objects mapped with 1<<31 are
    re-encoded whole -- the VALU queue kernel at 10/14, the matrix cores'
    whole-object re-encode at 40/56 and 80/100) and decode_objects on 256 B
    chunk strides, replayed three times over fresh objects, each time equal to
    the uncaptured calls.  Batches of short objects walk flat (phase 0 with
    and without the switch record: the uncaptured calls have one)."""
    torch = torch_dev
    from slime_amd import device as D
    L, cs, slot = D.slot_geometry(S, need, total, chunk_align=256)
    erase = [0, 3, need, total - 1]
    have = [i for i in range(total) if i not in erase][:need]
    enc = D.Plan.encode(need, total)
    rec = D.Plan.reconstruct(need, total, have, erase).set_outputs(erase)
    slots = torch.zeros(nobj * slot, dtype=torch.uint8, device="cuda")
    mapping = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    chunks = slots.view(nobj, total, cs)[:, :, : 4 * L]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def fill(seed):
        g = torch.Generator(device="cuda").manual_seed(seed)
        slots.copy_(torch.randint(0, 256, slots.shape, dtype=torch.uint8, device="cuda", generator=g))
        words = chunks[:, :need].view(torch.int32)
        words[1:3] &= 0x7F7F7F7F  # objects 1 and 2: every word below 2^31 (mapping 0)
        slots.view(nobj, slot)[2, :4] = torch.tensor([255, 255, 255, 253], dtype=torch.uint8)  # 2: now 1<<31

    def calls():
        D.encode_objects(enc, slots, slot, S, nobj, mapping, status, s, cs)
        for e in erase:  # basic slices: a fill kernel, capturable (a list index would upload it)
            chunks[:, e].fill_(0x5A)
        D.decode_objects(rec, slots, slot, L, nobj, mapping, s, cs)

    with torch.cuda.stream(s):
        fill(1)
        calls()  # warm the launch paths outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        calls()
    for seed in (2, 3, 4):
        with torch.cuda.stream(s):
            fill(seed)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        got, gm, gs = chunks.clone(), mapping.clone(), status.clone()
        with torch.cuda.stream(s):
            fill(seed)
            calls()
        torch.cuda.synchronize()
        ok = (status == 0).nonzero().flatten()
        assert torch.equal(gs, status) and torch.equal(gm, mapping), seed
        assert int(mapping[2]) == -2**31
        assert torch.equal(got[ok], chunks[ok]), seed


HIP_STREAM_PER_THREAD = 2  # (hipStream_t)2, hip_runtime_api.h


def _hip():
    """The HIP runtime torch loaded (same soname, so dlopen returns it)."""
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return hip


def test_stream_per_thread_from_two_threads(torch_dev, schedule):
    """Two host threads launch interleaved encodes on hipStreamPerThread: one
    handle, a different stream per thread, so the launches are unordered
    against each other.  Every object exact, and every counter set is back in
    the pool once the device is idle."""
    torch = torch_dev
    from slime_amd import device as D
    assert schedule(1) == 0
    need, total = 8, 12
    plan = D.Plan.encode(need, total)
    rng = np.random.default_rng(21)
    shapes = [(7, 3 * 768 * 4 + 11), (3, 96 * 1024 + 5), (12, 2 * 768 * 4), (1, 4099)]
    jobs = []
    for t in range(2):
        mine = []
        for rep in range(6):
            nobj, L = shapes[(t + rep) % len(shapes)]
            h = _objects(rng, nobj, total, L)
            mine.append((h, torch.from_numpy(h.view(np.int32).reshape(-1).copy()).cuda(), nobj, L))
        jobs.append(mine)
    torch.cuda.synchronize()
    _, held0 = N.ticket_sets(0)
    errors = []
    barrier = threading.Barrier(2)

    def run(mine):
        try:
            torch.cuda.set_device(0)
            barrier.wait()
            for h, buf, nobj, L in mine:
                lay = D.layout_of(total, L)
                plan(buf, lay, buf, lay, L, nobj, stream=HIP_STREAM_PER_THREAD, dst_offset=need * L)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ts = [threading.Thread(target=run, args=(mine,)) for mine in jobs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    torch.cuda.synchronize()
    for mine in jobs:
        for h, buf, nobj, L in mine:
            got = buf.cpu().numpy().view(np.uint32).reshape(nobj, total, L)
            assert np.array_equal(got, _encode_ref(h, need, total)), (nobj, L)
    # The device is idle: every set the 12 launches took is back in the pool.
    _, held1 = N.ticket_sets(0)
    assert held1 == held0


def test_stream_destroyed_in_flight_and_handle_reused(torch_dev, schedule):
    """A stream destroyed while its launch still runs, then a new stream (the
    runtime may hand back the same handle) launching at once: the two launches
    are unordered, and both results are exact."""
    torch = torch_dev
    from slime_amd import device as D
    assert schedule(1) == 0
    hip = _hip()
    need, total = 8, 12
    plan = D.Plan.encode(need, total)
    rng = np.random.default_rng(33)
    big_n, big_L = 24, 256 * 1024  # a launch long enough to still run at the destroy
    big = _objects(rng, big_n, total, big_L)
    small = [(_objects(rng, n, total, L), n, L) for n, L in [(5, 3 * 768 * 4 + 1), (9, 40000), (2, 7)]]
    bufs = [torch.from_numpy(big.view(np.int32).reshape(-1).copy()).cuda()]
    bufs += [torch.from_numpy(h.view(np.int32).reshape(-1).copy()).cuda() for h, _, _ in small]
    torch.cuda.synchronize()
    handles = []
    for rep in range(3):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0  # hipStreamNonBlocking
        handles.append(s.value)
        if rep == 0:
            plan(bufs[0], D.layout_of(total, big_L), bufs[0], D.layout_of(total, big_L), big_L, big_n,
                 stream=s.value, dst_offset=need * big_L)
        h, n, L = small[rep]
        plan(bufs[1 + rep], D.layout_of(total, L), bufs[1 + rep], D.layout_of(total, L), L, n, stream=s.value,
             dst_offset=need * L)
        assert hip.hipStreamDestroy(ctypes.c_void_p(s.value)) == 0  # launches still in flight
    torch.cuda.synchronize()
    got = bufs[0].cpu().numpy().view(np.uint32).reshape(big_n, total, big_L)
    assert np.array_equal(got, _encode_ref(big, need, total))
    for (h, n, L), buf in zip(small, bufs[1:]):
        got = buf.cpu().numpy().view(np.uint32).reshape(n, total, L)
        assert np.array_equal(got, _encode_ref(h, need, total)), (n, L)


def test_counter_sets_are_reused_not_grown(torch_dev, schedule):
    """Sequential launches on one stream reuse the pool's sets: 200 launches
    allocate no new slab once the first exists."""
    torch = torch_dev
    from slime_amd import device as D
    assert schedule(1) == 0
    need, total, nobj, L = 4, 6, 3, 4096
    plan = D.Plan.encode(need, total)
    buf = torch.zeros(nobj * total * L, dtype=torch.int32, device="cuda")
    D.fill_symbols(buf, seed=3)
    lay = D.layout_of(total, L)
    plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    sets0, _ = N.ticket_sets(0)
    for _ in range(200):
        plan(buf, lay, buf, lay, L, nobj, dst_offset=need * L)
    torch.cuda.synchronize()
    sets1, _ = N.ticket_sets(0)
    assert sets1 == sets0
