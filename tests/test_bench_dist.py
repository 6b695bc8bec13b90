"""The bench's multi-rank logic on CPU: two gloo ranks (the GPU bench uses the same helpers over
RCCL). Job time is the max over ranks, bit errors are summed, value is whole-job Mbps."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    el, err = bench.reduce_over_ranks(dist, torch.device("cpu"), 1.0 + rank, 3 * rank)
    q.put((rank, el, err, bench.decoded_mbps(world, bench.NCB, bench.K, 10, el)))
    dist.destroy_process_group()


def test_two_rank_reduction_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import bench  # noqa: E402
    for rank, el, err, mbps in out:
        assert el == 2.0 and err == 3
        assert mbps == pytest.approx(2 * bench.NCB * bench.K * 10 / 2.0 / 1e6)


def test_single_process_identity():
    sys.path.insert(0, REPO)
    import bench
    assert bench.reduce_over_ranks(None, None, 1.5, 7) == (1.5, 7)
