"""Multi-GPU receive jobs: partition, per-rank decode, gather.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo" for the CPU tests).
A job of independent units — code blocks, transport blocks, subframes — is split by the native
partitioner (include/srsgpu/shard.h): contiguous ranges for equal-cost units (C2-C4) and a global
longest-first queue over unit weights for mixed sizes (C5: weight = sum of K over the unit's code
blocks x the half-iteration budget). Every rank computes the same partition, so the split needs no
message. Each rank decodes its own units where they lie; the only data-path communication is the
gather of results to one rank, as ONE grouped batch of point-to-point receives on the root
(torch.distributed.batch_isend_irecv, i.e. a grouped ncclSend / ncclRecv over xGMI on the GPU box).

Reference analogue: srsUE's PHY worker pool hands whole subframes to idle workers
(srsue/src/phy/phy.cc:141-168); the result of every worker goes to the one MAC.
"""
import numpy as np

import srsgpu_phy as s


def contiguous(n, world):
    """[first_0, ..., first_world]: rank r owns units first[r] .. first[r + 1] - 1"""
    return s.shard_contiguous(n, world)


def weighted(weights, world):
    """(owner[unit], load[rank]) from the global longest-first queue"""
    return s.shard_weighted(weights, world)


def tb_weight(cbsegm_row, max_halfits):
    """decoding cost of one transport block: sum of K over its code blocks x the half-iteration
    budget (cbsegm_row = [C, C1, K1, C2, K2, F] as srslte_cbsegm fills it)"""
    C, _c1, K1, C2, K2, _f = cbsegm_row
    return int(sum(K2 if i < C2 else K1 for i in range(C)) * max_halfits)


def balance(load):
    """max / mean load (1.0 = perfect)"""
    load = np.asarray(load, np.float64)
    return float(load.max() / load.mean()) if load.size and load.mean() > 0 else 1.0


def gather_records(dist, torch, device, owner, sizes, local, root=0):
    """Gather per-unit byte records to `root`.

    owner[i]: the rank that holds unit i; sizes[i]: unit i's record length in bytes (known to every
    rank); local: this rank's records of its own units in ascending unit order, concatenated, as a
    uint8 tensor on `device` (CUDA for RCCL, CPU for gloo). On the root, returns the list of all
    units' records (numpy uint8 arrays) in unit order; elsewhere None. All receives are posted as
    one grouped batch on the root."""
    rank, world = dist.get_rank(), dist.get_world_size()
    owner = np.asarray(owner)
    sizes = np.asarray(sizes, np.int64)
    per_rank = [np.flatnonzero(owner == r) for r in range(world)]
    nbytes = [int(sizes[u].sum()) for u in per_rank]
    if int(local.numel()) != nbytes[rank]:
        raise ValueError("rank %d: %d bytes of records, partition says %d" % (rank, local.numel(), nbytes[rank]))
    if rank != root:
        if nbytes[rank]:
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, local, root)]):
                req.wait()
        return None
    bufs = {r: (local if r == root else torch.empty(nbytes[r], dtype=torch.uint8, device=device))
            for r in range(world) if nbytes[r]}
    ops = [dist.P2POp(dist.irecv, b, r) for r, b in bufs.items() if r != root]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    out = [None] * len(owner)
    for r, b in bufs.items():
        host = b.cpu().numpy()
        off = 0
        for u in per_rank[r]:
            out[u] = host[off:off + sizes[u]]
            off += sizes[u]
    return out


def pack_tb_record(ret, noi, data, cb_crc, tbs, max_cb=13):
    """one TB's result as bytes: int32 return code, uint32 nof_iterations, max_cb cb_crc flags,
    the TB's tbs/8 data bytes"""
    rec = np.zeros(8 + max_cb + tbs // 8, np.uint8)
    rec[:4] = np.frombuffer(np.int32(ret).tobytes(), np.uint8)
    rec[4:8] = np.frombuffer(np.uint32(noi).tobytes(), np.uint8)
    c = np.asarray(cb_crc, np.uint8)[:max_cb]
    rec[8:8 + c.size] = c
    rec[8 + max_cb:] = np.asarray(data, np.uint8)[:tbs // 8]
    return rec


def unpack_tb_record(rec, tbs, max_cb=13):
    ret = int(np.frombuffer(rec[:4].tobytes(), np.int32)[0])
    noi = int(np.frombuffer(rec[4:8].tobytes(), np.uint32)[0])
    return ret, noi, rec[8:8 + max_cb].copy(), rec[8 + max_cb:8 + max_cb + tbs // 8].copy()


def tb_record_len(tbs, max_cb=13):
    return 8 + max_cb + tbs // 8
