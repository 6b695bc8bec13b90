"""C5 (BASELINE configs[4]): mixed-bandwidth multi-cell subframes — cells of 6/25/50/100 PRB,
random allocations and MCS 0..28 (K = 40..6144) — through the GPU transmitter and receiver, with
all cells' transport blocks decoded in ONE DL-SCH call (mixed K). Parity: every TB the GPU decodes
from its own LLRs equals the CPU oracle's decode of the same LLRs (return code, bytes,
nof_iterations), at an SNR where some TBs fail and iteration counts vary."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def table():
    return json.load(open(os.path.join(HERE, "golden", "c5_traffic.json")))


def test_c5_tx_rx_all_ack(table):
    import torch
    import srsgpu_traffic as tr
    m = tr.MixedCells(table, 96, torch, torch.device("cuda", 0), seed=11, snr_db=35.0)
    m.step()
    torch.cuda.synchronize()
    acks, good, noi = m.check()
    assert acks == m.ntb and good == m.ntb, (acks, good, m.ntb)
    assert noi <= 3.0
    m.close()


def test_c5_mixed_k_decode_vs_oracle(table, oracle):
    """LLRs from the GPU front end at 6 dB; the GPU's one-call mixed-K decode vs the CPU oracle
    (sch.c decode_tb restatement) TB by TB"""
    import torch
    import srsgpu_traffic as tr
    m = tr.MixedCells(table, 40, torch, torch.device("cuda", 0), seed=12, snr_db=6.0)
    m.step()
    torch.cuda.synchronize()
    e = m.d_e.cpu().numpy()
    ret = m.d_ret.cpu().numpy()
    noi = m.d_noi.cpu().numpy()
    data = m.d_data.cpu().numpy()
    dl = DlschOracle(oracle)
    ks = set()
    for i, t in enumerate(m.tb_list):
        sb = dl.softbuffer(13)
        dl.reset(sb)
        r, d, n, _ = dl.decode(sb, t["tbs"], t["rv"], t["Qm"],
                               e[t["e_offset"]:t["e_offset"] + t["nof_e_bits"]], 8)
        dl.free(sb)
        assert (r, n) == (ret[i], noi[i]), (i, t, r, n, ret[i], noi[i])
        if r == 0:
            o = t["data_offset"]
            assert (d[:t["tbs"] // 8] == data[o:o + t["tbs"] // 8]).all(), i
        ks.add(table["cbsegm_C_C1_K1_C2_K2_F"][str(t["tbs"])][2])
    assert len(set(ret.tolist())) > 1 and len(set(noi.tolist())) > 2  # failures and varied noi
    assert len(ks) > 10
    m.close()


def test_c5_decode_identical_under_every_schedule(table):
    """srsgpu_tdec_set_schedule changes only how the decoders are launched: the same mixed-K job
    (window and SSE kinds, failures and varied nof_iterations at 6 dB) decodes to the same return
    codes, nof_iterations, bytes and cb_crc under the auto, fused (1 and 8 half-iterations per
    launch), per-half-iteration, hybrid (first half-iteration per launch, the rest fused; with the
    one-wave SSE decoder the hybrid falls back) and one-wave SSE schedules."""
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    keep = s.get_schedule()
    m = tr.MixedCells(table, 40, torch, torch.device("cuda", 0), seed=13, snr_db=6.0)
    try:
        m.front_end()
        torch.cuda.synchronize()
        outs = {}
        for name, sch in {"auto": dict(es_fused=2, es_chunk=8, sse_bidir=1),
                          "fused1": dict(es_fused=1, es_chunk=1, sse_bidir=1),
                          "fused8": dict(es_fused=1, es_chunk=8, sse_bidir=1),
                          "per_halfit": dict(es_fused=0, sse_bidir=1),
                          "hybrid": dict(es_fused=3, es_chunk=8, sse_bidir=1),
                          "hybrid_one_wave": dict(es_fused=3, es_chunk=8, sse_bidir=0),
                          "sse_one_wave": dict(es_fused=0, sse_bidir=0)}.items():
            s.set_schedule(**sch)
            m.d_data.zero_()
            m.decode()
            torch.cuda.synchronize()
            crc = [bytes(m.dlsch.read_cb_crc(t["softbuffer"])) for t in m.tb_list]
            outs[name] = (m.d_ret.cpu().numpy(), m.d_noi.cpu().numpy(), m.d_data.cpu().numpy(), crc)
        ref = outs["auto"]
        assert len(set(ref[0].tolist())) > 1 and len(set(ref[1].tolist())) > 2
        for name, o in outs.items():
            assert (o[0] == ref[0]).all() and (o[1] == ref[1]).all(), name
            assert (o[2] == ref[2]).all() and o[3] == ref[3], name
    finally:
        s.set_schedule(**keep)
        m.close()
