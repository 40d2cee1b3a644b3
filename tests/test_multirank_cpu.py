"""The N > 1 path on CPU: world-size-2 gloo process group, frames sharded by
index (shard.frame_range), each rank demodulating its own frames, decoded
payloads gathered (shard.gather_payloads) and compared on every rank with the
whole batch's payloads.  The CPU oracle stands in for the per-rank HIP
launch here (test infrastructure); the GPU path is the same C-ABI call per
rank (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frames(oracle, total, sf, plen):
    rng = np.random.default_rng(99)
    pays = rng.integers(0, 256, (total, plen), dtype=np.uint8)
    return pays, [oracle.modulate(oracle.encode(p.tobytes()), sf) for p in pays]


def _worker(rank, world, port, total, sf, plen, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from checkers import Oracle
        o = Oracle()
        pays, iqs = _frames(o, total, sf, plen)
        first, count = shard.frame_range(total, world, rank)
        local = np.zeros((count, plen), np.uint8)
        for i in range(count):
            x = o.dechirp(iqs[first + i], sf)
            r, syms, sync, _ = o.lora_demodulate(x, sf)
            local[i] = o.lora_decode(syms)[1]
        got = shard.gather_payloads(torch.from_numpy(local.reshape(-1).copy()), count, plen, total)
        q.put((rank, bool(np.array_equal(got.numpy().reshape(total, plen), pays))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 7])
def test_two_rank_shard_and_gather(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, 7, 8, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: True, 1: True}


@pytest.mark.parametrize("total,world", [(10, 3), (65536, 8), (1, 2), (0, 4), (1000000, 8)])
def test_frame_range_partitions(total, world):
    spans = [shard.frame_range(total, world, r) for r in range(world)]
    assert spans[0][0] == 0
    for (a, n), (b, _) in zip(spans, spans[1:]):
        assert a + n == b
    assert sum(n for _, n in spans) == total
    assert max(n for _, n in spans) - min(n for _, n in spans) <= 1


def _varlen_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = torch.arange(3 + 4 * rank, dtype=torch.uint8)
        parts = shard.gather_varlen(local)
        q.put((rank, [p.tolist() for p in parts]))
    finally:
        dist.destroy_process_group()


def test_gather_varlen_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_varlen_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [list(range(3)), list(range(7))]
    assert res == {0: want, 1: want}


@pytest.mark.parametrize("world", [1, 2, 8])
def test_balanced_ranges_by_cost(world):
    rng = np.random.default_rng(3)
    sfs = rng.integers(7, 13, 20000)
    cost = (1 << sfs) * sfs.astype(np.float64)
    spans = shard.balanced_ranges(cost, world)
    assert spans[0][0] == 0 and sum(n for _, n in spans) == sfs.size
    for (a, n), (b, _) in zip(spans, spans[1:]):
        assert a + n == b
    loads = [cost[a:a + n].sum() for a, n in spans]
    assert max(loads) - min(loads) <= 2.5 * cost.max()  # within a couple of frames
