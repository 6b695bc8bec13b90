"""Multi-rank partition + gather on CPU: the native partitioner
(include/srsgpu/shard.h) and srsgpu_shard.gather_records over two gloo ranks.

The C5-style job: mixed-size transport blocks (K from 40 to 6144 across TBS values of the 36.213
tables) at SNRs where some fail and iteration counts vary. Each rank decodes only the TBs the
weighted partition gives it — with the CPU oracle (the sch.c decode_tb restatement) standing in for
the GPU decode, since this runs without a GPU — then the results go to rank 0 in one grouped
send/recv batch. Rank 0's gathered results must equal a single-process decode of the whole job, and
the partition must balance the decoding cost within 10 %."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import REPO

HERE = os.path.dirname(os.path.abspath(__file__))
MAXH = 8


def _job(n_tb=36, seed=5):
    """(tbs, Qm, nbits, rv, llr) per TB: random PRB count and MCS from the C5 tables"""
    from srsgpu_testlib import DlschOracle, Oracle
    table = json.load(open(os.path.join(HERE, "golden", "c5_traffic.json")))
    orc = Oracle()
    dl = DlschOracle(orc)
    rng = np.random.default_rng(seed)
    qm_of = {1: 2, 2: 4, 3: 6}
    job = []
    while len(job) < n_tb:
        prb = int(rng.choice([6, 25, 50, 100]))
        L, mcs = int(rng.integers(1, prb + 1)), int(rng.integers(0, 29))
        tbs, qm = table["tbs_by_prb_mcs"][L - 1][mcs], qm_of[table["mod_by_mcs"][mcs]]
        C = table["cbsegm_C_C1_K1_C2_K2_F"][str(tbs)][0]
        nb = 136 * L * qm  # ~ PDSCH REs of L PRB x bits per symbol
        if tbs + 24 > 0.9 * nb or table["cbsegm_C_C1_K1_C2_K2_F"][str(tbs)][5]:
            continue
        nb = max(nb - nb % qm, qm * C)
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        e = dl.encode(tbs, 0, qm, nb, data)
        snr = float(rng.uniform(0.0, 5.0))
        y = np.where(e == 1, 1.0, -1.0) + 10 ** (-snr / 20) * rng.standard_normal(e.size)
        job.append((tbs, qm, nb, (100 * y).astype(np.float32).astype(np.int16)))
    return table, job


def _decode(job, units):
    from srsgpu_testlib import DlschOracle, Oracle
    dl = DlschOracle(Oracle())
    import srsgpu_shard as sh
    recs = []
    sb = dl.softbuffer(13)
    for u in units:
        tbs, qm, nb, llr = job[u]
        dl.reset(sb)
        r, data, noi, cb_crc = dl.decode(sb, tbs, 0, qm, llr, MAXH)
        recs.append(sh.pack_tb_record(r, noi, data, cb_crc, tbs))
    dl.free(sb)
    return recs


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
    import srsgpu_shard as sh
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        table, job = _job()
        w = [sh.tb_weight(table["cbsegm_C_C1_K1_C2_K2_F"][str(t[0])], MAXH) for t in job]
        owner, load = sh.weighted(w, world)
        mine = [u for u in range(len(job)) if owner[u] == rank]
        recs = _decode(job, mine)
        local = torch.from_numpy(np.concatenate(recs) if recs else np.zeros(0, np.uint8))
        sizes = [sh.tb_record_len(t[0]) for t in job]
        out = sh.gather_records(dist, torch, torch.device("cpu"), owner, sizes, local)
        q.put((rank, None if out is None else [r.tobytes() for r in out], list(map(int, load)),
               list(map(int, owner))))
    finally:
        dist.destroy_process_group()


def test_contiguous_ranges():
    import srsgpu_shard as sh
    for n, world in [(4096, 1), (8192, 8), (13, 4), (3, 8), (0, 2)]:
        f = sh.contiguous(n, world)
        assert f[0] == 0 and f[-1] == n and len(f) == world + 1
        sizes = np.diff(f)
        assert sizes.min() >= 0 and sizes.max() - sizes.min() <= 1


def test_weighted_balance_c5_mix():
    """LPT over a C5-like TB mix: 1024 subframes of random PRB / MCS, weights sum(K) x 8"""
    import srsgpu_shard as sh
    table = json.load(open(os.path.join(HERE, "golden", "c5_traffic.json")))
    rng = np.random.default_rng(1)
    w = []
    for i in range(1024):
        prb = (6, 25, 50, 100)[i % 4]
        L, mcs = int(rng.integers(1, prb + 1)), int(rng.integers(0, 29))
        tbs = table["tbs_by_prb_mcs"][L - 1][mcs]
        w.append(sh.tb_weight(table["cbsegm_C_C1_K1_C2_K2_F"][str(tbs)], 8))
    for world in (2, 4, 8):
        owner, load = sh.weighted(w, world)
        assert set(owner.tolist()) == set(range(world))
        assert int(load.sum()) == sum(w)
        assert sh.balance(load) <= 1.01, (world, load)  # many units: LPT is near perfect
        for r in range(world):  # load is what the owner vector says
            assert int(load[r]) == sum(x for x, o in zip(w, owner) if o == r)
    owner, load = sh.weighted([5, 4, 3, 3, 3], 2)  # LPT worst-case shape: 4/3 of optimum 9
    assert max(load) <= 12 and sorted(load.tolist()) == [8, 10]


def test_two_rank_c5_partition_gather_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    root = got[0]
    assert root[0] == 0 and got[1][1] is None
    table, job = _job()
    single = _decode(job, range(len(job)))
    import srsgpu_shard as sh
    assert len(root[1]) == len(job)
    rets, nois = set(), set()
    for u, (a, b) in enumerate(zip(root[1], single)):
        assert a == b.tobytes(), u
        r, n, _crc, _d = sh.unpack_tb_record(b, job[u][0])
        rets.add(r)
        nois.add(n)
    assert len(rets) > 1 and len(nois) > 2  # failures and varied iteration counts
    owner, load = np.array(root[3]), np.array(root[2])
    assert set(owner.tolist()) == {0, 1}
    assert sh.balance(load) <= 1.10, load
    ks = {table["cbsegm_C_C1_K1_C2_K2_F"][str(t[0])][2] for t in job}
    assert len(ks) >= 10  # mixed K


def _rank_tm3(rank, world, port, q):
    """BASELINE configs[3]'s multi-GPU form: a global job of TM3 subframes (two codewords each),
    split in contiguous subframe ranges (srsgpu_shard_contiguous, as bench.py's pipeline_tm3 leg
    splits nranks x 1024 subframes); each rank decodes its own subframes' two TBs and gathers one
    record per subframe (the two TB records back to back) to rank 0."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
    import srsgpu_shard as sh
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _table, job = _job(n_tb=2 * TM3_SF, seed=7)
        first = sh.contiguous(TM3_SF, world)
        owner = np.repeat(np.arange(world), np.diff(first))
        mine = range(first[rank], first[rank + 1])
        recs = [np.concatenate(_decode(job, [2 * i, 2 * i + 1])) for i in mine]
        local = torch.from_numpy(np.concatenate(recs) if recs else np.zeros(0, np.uint8))
        sizes = [sh.tb_record_len(job[2 * i][0]) + sh.tb_record_len(job[2 * i + 1][0]) for i in range(TM3_SF)]
        out = sh.gather_records(dist, torch, torch.device("cpu"), owner, sizes, local)
        q.put((rank, None if out is None else [r.tobytes() for r in out], list(map(int, first))))
    finally:
        dist.destroy_process_group()


TM3_SF = 11  # odd: the two ranks get 5 and 6 subframes


def test_two_rank_tm3_subframe_partition_gather_gloo():
    """The TM3 job's partition and gather over two gloo ranks (the DL-SCH decode of each codeword
    by the CPU oracle stands in for the GPU receive chain): rank 0's gathered per-subframe records
    equal a single-process decode of the whole job, in subframe order."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30700 + os.getpid() % 1000
    procs = [ctx.Process(target=_rank_tm3, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    root = got[0]
    assert root[0] == 0 and got[1][1] is None
    assert root[2] == [0, 5, 11]
    _table, job = _job(n_tb=2 * TM3_SF, seed=7)
    import srsgpu_shard as sh
    assert len(root[1]) == TM3_SF
    rets = set()
    for i, rec in enumerate(root[1]):
        single = np.concatenate(_decode(job, [2 * i, 2 * i + 1]))
        assert rec == single.tobytes(), i
        n0 = sh.tb_record_len(job[2 * i][0])
        rets.add(sh.unpack_tb_record(single[:n0], job[2 * i][0])[0])
        rets.add(sh.unpack_tb_record(single[n0:], job[2 * i + 1][0])[0])
    assert len(rets) > 1  # acked and failed codewords both present
