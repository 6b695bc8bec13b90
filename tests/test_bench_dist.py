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


def test_bench_spawns_ranks_and_gathers(tmp_path):
    """bench.py --gpus 2 with no launcher starts two ranks itself (one process per GPU on the box);
    the distcheck leg runs the legs' partitions and the gather to rank 0 over gloo, and rank 0
    verifies every gathered record byte for byte"""
    import json
    import subprocess
    detail = tmp_path / "detail.json"
    env = dict(os.environ, SRSGPU_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--legs", "distcheck",
                        "--detail", str(detail)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    dc = json.load(open(detail))["distcheck"]
    assert sorted(p["rank"] for p in dc["ranks"]) == [0, 1]
    assert len({p["pid"] for p in dc["ranks"]}) == 2
    assert sorted(p["local_rank"] for p in dc["ranks"]) == [0, 1]
    for leg in ("c3", "tm3", "c5"):
        rec = dc["legs"][leg]
        assert rec["units"] == 2048 and sum(rec["units_per_rank"]) == 2048
        assert rec["gathered_ok"] == rec["units"], (leg, rec)
    assert dc["legs"]["c3"]["units_per_rank"] == [1024, 1024]
    assert dc["legs"]["c5"]["balance"] <= 1.1


def test_bench_refuses_mismatched_world_size():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--legs", "distcheck"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_compact_summary_fits_driver_capture():
    """the last stdout line stays far below the driver's 8 KB capture with every leg present (the
    round-4 record, whose one-line form was 20.7 KB)"""
    import json
    sys.path.insert(0, REPO)
    import bench
    rec = json.load(open(os.path.join(REPO, "profiles", "r04_s17_bench.json")))
    line = bench.compact_summary(rec, "bench_detail.json")
    assert len(line) <= 6000
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "valu_roofline", "cpu_baseline", "legs"):
        assert k in out
    assert out["value"] == rec["value"] and out["roofline"]["frac"] == rec["roofline"]["frac"]
    assert out["config"]["workload"] == rec["config"]["workload"]
    big = dict(rec, cpu_baseline=dict(rec["cpu_baseline"], sample="x" * 20000))
    assert len(bench.compact_summary(big, "d.json")) <= 6000
