"""world_size-2 gloo test of the multi-GPU path's host logic (sharding, return gather,
max-over-ranks timing, inner-step sum) on CPU tensors."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fancy_gym_crowd_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 16
    lo, hi = shard.shard_range(n, rank, world)
    allp = np.random.default_rng(1234).standard_normal((n * world, 3), dtype=np.float32)
    mine = shard.shard_rows(allp, rank, world)
    # a stand-in "return" that depends on the global env index and the env's parameter row
    ret = torch.from_numpy(mine.sum(1).astype(np.float64)) + torch.arange(lo, hi, dtype=torch.float64)
    all_ret = shard.gather_returns(ret)
    # bench.py's per-BB-step form: one all_gather_into_tensor into a preallocated buffer
    buf = torch.empty(n * world, dtype=torch.float64)
    assert shard.gather_returns_into(buf, ret) is buf
    assert torch.equal(buf, all_ret)
    try:
        shard.gather_returns_into(torch.empty(n, dtype=torch.float64), ret)
        raise AssertionError("short gather buffer accepted")
    except ValueError:
        pass
    t = shard.max_over_ranks(1.0 + rank, "cpu")
    s = shard.sum_over_ranks(200 * n, "cpu")
    q.put((rank, lo, hi, all_ret.numpy(), t, s))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    n = 16
    allp = np.random.default_rng(1234).standard_normal((n * world, 3), dtype=np.float32)
    expect = allp.sum(1).astype(np.float64) + np.arange(n * world)
    for rank, lo, hi, all_ret, t, s in res:
        assert (lo, hi) == (rank * n, (rank + 1) * n)
        np.testing.assert_array_equal(all_ret, expect)       # global env order, bit-exact
        assert t == 2.0                                      # max over ranks
        assert s == 200 * n * world                          # sum of inner steps


def test_shard_rows_requires_even_split():
    import pytest
    with pytest.raises(ValueError):
        shard.shard_rows(np.zeros((5, 2)), 0, 2)
