"""Multi-rank control plane on the CPU (gloo, world size 2).

The data path shards objects across GPUs with no collective; what must be
right for N > 1 is the partition (every object exactly once) and the
max-over-ranks timing reduction bench.py reports.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from slime_amd import batch


def test_partition_tiles_every_object_once():
    for nobj in (0, 1, 7, 8, 63, 64, 65, 128, 1000):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                s, c = batch.partition(nobj, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(nobj))
    assert batch.partition(64, 8, 3) == (24, 8)  # C5: 8 objects per GPU


def test_partition_rejects_bad_rank():
    with pytest.raises(ValueError):
        batch.partition(10, 2, 2)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, count = batch.partition(64, world, rank)
        batch.barrier()
        # rank r "took" 1+r seconds and processed `count` objects
        elapsed, objs = batch.max_over_ranks([1.0 + rank, float(count)])
        t = torch.tensor([float(count)], dtype=torch.float64)
        dist.all_reduce(t)
        # bench.py's n_gpus: distinct device addresses over ranks (two ranks
        # reporting one PCI address count as one GPU)
        bdfs = batch.gather_strings(f"0000:{rank:02x}:00.0")
        shared = batch.gather_strings("0000:5d:00.0")
        q.put((rank, start, count, elapsed, objs, t.item(), len(set(bdfs)), len(set(shared)), bdfs))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_partition_and_max_timing():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 32), (32, 32)]
    assert all(r[3] == 2.0 for r in res)  # max over ranks
    assert all(r[5] == 64.0 for r in res)  # every object once
    assert all(r[6] == 2 and r[7] == 1 for r in res)  # n_gpus counts distinct devices
    assert all(r[8] == ["0000:00:00.0", "0000:01:00.0"] for r in res)  # rank order


def _pooled_worker(rank, world, port, q):
    """bench.py's pooled leg at world 2 on the CPU: every rank enters, rank 0
    drives the proxy load (no GPU here: every device call fails with
    SLIME_RS_ERR_NO_DEVICE, quickly), rank 1 waits at the barrier and gets
    None; nobody deadlocks."""
    import importlib.util
    import sys
    import types
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    spec = importlib.util.spec_from_file_location("bench_pooled", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = types.SimpleNamespace(pool_threads=2, pool_seconds=0.05)
        out = bench.pooled_leg(args, rank, world, bench.pool_devices(world, 1))
        q.put((rank, None if out is None else
               (out["devices"], out["verified"], sorted(out["workloads"]),
                {w["status"] for w in out["workloads"].values()})))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_pooled_leg_runs_on_rank0_only():
    if torch.cuda.device_count() > 0:
        pytest.skip("the CPU form of the check; on a GPU box bench.py runs the pooled leg for real")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pooled_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] == (1, None)
    devices, verified, names, statuses = res[0][1]
    assert devices == [0] and verified is False
    assert names == ["fused_1mib", "fused_64mib", "unchanged_caller_64mib"]
    assert statuses == {10}  # SLIME_RS_ERR_NO_DEVICE: no CPU fallback
