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


@pytest.mark.parametrize("nd", [2, 4, 8])
@pytest.mark.parametrize("n", [0, 1, 7, 65535, 65536, 65537, 1_000_000, 8_000_003, 10_000])
def test_library_plan_split(nd, n):
    """The engine's in-process multi-GPU split (sbft_gv_plan_split, used by every host-buffer
    call: one contiguous share per device, each driven by its own host thread and stream).
    Shares tile [0, n) in device order and differ by at most one tuple; batches below
    min_split (65,536 by default) stay whole on one device."""
    from smartbft_amd.gpuverify import plan_split
    parts = plan_split(n, nd)
    if n < 65536:
        assert parts == [(0, n)]
        return
    assert len(parts) == nd
    assert parts[0][0] == 0 and sum(c for _, c in parts) == n
    for (b0, c0), (b1, _) in zip(parts, parts[1:]):
        assert b0 + c0 == b1
    counts = [c for _, c in parts]
    assert max(counts) - min(counts) <= 1


def test_library_plan_split_min_split_and_tiny_shares():
    from smartbft_amd.gpuverify import plan_split
    assert plan_split(100, 8, min_split=1) == [(0, 12), (12, 13), (25, 12), (37, 13), (50, 12), (62, 13),
                                               (75, 12), (87, 13)]
    # fewer tuples than devices: empty shares are left out
    assert plan_split(3, 8, min_split=1) == [(0, 1), (1, 1), (2, 1)]
    assert plan_split(10, 1, min_split=1) == [(0, 10)]
    assert plan_split(10, 0) == []


@pytest.mark.parametrize("nd", [2, 4, 8])
def test_config3_split_shares_fit_the_wide_kernel(nd):
    """The engine's default min_split with the wide half kernel on (halfq_max + 1; 24 x 256 CUs + 1 =
    6,145 on an MI355X): a 10k-request proposal on nd devices is cut into nd contiguous shares, each
    at most halfq_max tuples, so every device runs the wide kernel; on one device it stays whole."""
    from smartbft_amd.gpuverify import plan_split
    halfq = 24 * 256
    parts = plan_split(10_000, nd, min_split=halfq + 1)
    assert len(parts) == nd and max(c for _, c in parts) <= halfq
    assert sum(c for _, c in parts) == 10_000 and parts[0][0] == 0
    assert plan_split(10_000, 1, min_split=halfq + 1) == [(0, 10_000)]
    assert plan_split(halfq, nd, min_split=halfq + 1) == [(0, halfq)]


def _gloo_wait_worker(rank, world, port, out):
    # bench.py's end at N > 1: rank 0 runs config 3 across the GPUs while the others wait on a
    # gloo group's barrier (no collective kernel on their devices), then all leave together
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = dist.new_group(backend="gloo")
    if rank == 0:
        import time
        time.sleep(0.5)
    dist.barrier(group=g)
    out[rank] = True
    dist.destroy_process_group()


def test_two_rank_cpu_side_final_barrier():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gloo_wait_worker, args=(world, port, out), nprocs=world, join=True)
    assert dict(out) == {0: True, 1: True}
