"""CPU multi-process test (gloo, world_size 2) of the bench's N>1 path: disjoint contiguous
shards and the max-over-ranks timing reduction."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from smartbft_amd.dist import reduce_timing, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(rank, world, 1000)
    elapsed = 1.0 + rank  # rank 1 is slower
    t, m = reduce_timing(elapsed, mismatches=rank)
    dist.barrier()
    out[rank] = (lo, hi, t, m)
    dist.destroy_process_group()


def test_two_rank_shards_and_max_time():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    assert out[0][:2] == (0, 1000) and out[1][:2] == (1000, 2000)
    assert out[0][2] == out[1][2] == 2.0  # max over ranks
    assert out[0][3] == out[1][3] == 1    # summed mismatches


def test_shard_range_single():
    assert shard_range(0, 1, 7) == (0, 7)
    with pytest.raises(AssertionError):
        shard_range(2, 2, 7)
