"""One PDSCH engine whose DL-SCH runs its early-stop tail on a tail stream
(srsgpu_dlsch_set_tail_stream on srsgpu_pdsch_get_dlsch()). The tail of call N reads the PDSCH's own
LLR buffer (the rows of failed TBs are written from it, k_derm_late), and call N+1's LLR stage
rewrites that buffer on the engine's stream: srsgpu_pdsch_decode_dev must make its stream wait for
the tail first (srsgpu_dlsch_join_tail). Two different batches decoded back to back with no host
wait must leave exactly what the same engine without a tail stream leaves: return codes, TB bytes,
nof_iterations, cb_crc and every softbuffer row of both batches' TBs."""
import ctypes
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batches(torch, dev, n, stream):
    import srsgpu_traffic as tr
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    out = []
    # 15 / 15.5 dB, in the waterfall: TBs that ack after several half-iterations and TBs that fail
    # (their rows are the tail's deferred writes); two seeds: two different received batches
    for seed, snr in ((22, 15.0), (23, 15.5)):
        m = tr.MixedCells(table, n, torch, dev, seed=seed, snr_db=snr, prbs=(100,), mcs=28, full_band=True,
                          stream=stream)
        m.front_end()
        torch.cuda.synchronize()
        out.append(m)
    return out


def _decode_pair(s, torch, dev, ms, stream, tail):
    c0 = ms[0].cells[0]
    n = c0["n"]
    pd = s.Pdsch(100, c0["id"], nof_softbuffers=2 * n, max_cb=13, max_sf=n, stream=stream.cuda_stream)
    pd.set_ce_rows(4)
    dl = ctypes.c_void_p(pd.dlsch_q)
    if tail is not None:
        assert s._lib.srsgpu_dlsch_set_tail_stream(dl, ctypes.c_void_p(tail.cuda_stream)) == 0
    pd.reset_softbuffer(0, 2 * n)
    res = []
    bufs = []
    for b, m in enumerate(ms):
        c = m.cells[0]
        sfs = []
        for j in range(n):
            sf = s.srsgpu_pdsch_sf_t.from_buffer_copy(c["sfs"][j])
            sf.softbuffer[0] = j + b * n
            sfs.append(sf)
        d_data = torch.zeros(m.d_data.numel(), dtype=torch.uint8, device=dev)
        d_ret = torch.zeros(n, dtype=torch.int32, device=dev)
        d_noi = torch.zeros(n, dtype=torch.int32, device=dev)
        pd.set_noise_dev(c["noise"].data_ptr())
        # no host wait between the two batches: batch 1's LLR stage follows batch 0's decode at once
        assert pd.decode_dev(sfs, c["grid"].data_ptr(), c["ce"].data_ptr(), c["gsz"], d_data.data_ptr(), 8,
                             d_ret.data_ptr(), d_noi.data_ptr()) == 0
        bufs.append((d_data, d_ret, d_noi))
    torch.cuda.synchronize()
    for b, (d_data, d_ret, d_noi) in enumerate(bufs):
        rows = np.zeros((n, 13, s.SOFTBUFFER_SIZE), np.int16)
        crc = np.zeros((n, 13), np.uint8)
        for j in range(n):
            assert s._lib.srsgpu_dlsch_softbuffer_read(dl, j + b * n, s._i16(rows[j]), s._u8(crc[j])) == 0
        res.append((d_ret.cpu().numpy(), d_noi.cpu().numpy(), d_data.cpu().numpy(), crc, rows))
    pd.close()
    return res


def test_pdsch_tail_stream_reused_llr_buffer():
    import torch
    import srsgpu_phy as s
    dev = torch.device("cuda:0")
    main = torch.cuda.Stream(dev)
    tail = torch.cuda.Stream(dev)
    ms = _batches(torch, dev, 48, main.cuda_stream)
    keep = s.get_schedule()
    s.set_schedule(es_fused=3, es_chunk=8)  # hybrid: the tail splits after the first half-iteration
    try:
        want = _decode_pair(s, torch, dev, ms, main, None)
        for rep in range(2):
            got = _decode_pair(s, torch, dev, ms, main, tail)
            rets = np.concatenate([want[0][0], want[1][0]])
            assert (rets == 0).any() and (rets != 0).any(), "the batches should mix acked and failed TBs"
            for b in range(2):
                for k, (x, y) in enumerate(zip(got[b], want[b])):
                    assert (x == y).all(), (rep, b, k)
    finally:
        s.set_schedule(**keep)
        for m in ms:
            m.close()
