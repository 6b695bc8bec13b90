"""srsgpu_dlsch_set_tail_stream: the early-stop tail of each DL-SCH call (the half-iterations after
the first, the bytes, the TB CRC) on a second stream, two engines alternating per batch, must give
exactly what the single-stream decode gives — return codes, TB bytes, nof_iterations and cb_crc —
on coded C3 subframes at SNRs where code blocks need one, two or more extra half-iterations, and
where TBs fail (their softbuffer rows are written in the tail). With fe_stream the front end runs on a
third stream, ordered against the DL-SCH call and the engine's previous tail by events (the headline's
form: bench.py --fe-stream 1), and must give the same again."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _results(m):
    ret = m.d_ret.cpu().numpy().copy()
    noi = m.d_noi.cpu().numpy().copy()
    data = m.d_data.cpu().numpy().copy()
    crc = np.stack([m.dlsch.read_cb_crc(m.softbuffer_of(t)) for t in m.tb_list])
    return ret, noi, data, crc


@pytest.mark.parametrize("fe", [0, 1])
@pytest.mark.parametrize("es_fused", [3])
@pytest.mark.parametrize("snr_db", [14.0, 16.5, 20.0])
def test_tail_stream_equals_single_stream(snr_db, es_fused, fe):
    """es_fused 3 (hybrid: first half-iteration, k_decide, the rest in one early-stop launch, as the
    headline's batches run): the split comes right after the first half-iteration (SRSGPU_SPLIT_EARLY)"""
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    dev = torch.device("cuda:0")
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    kw = dict(seed=22, snr_db=snr_db, prbs=(100,), mcs=28, full_band=True)
    main = torch.cuda.Stream(dev)
    tail = torch.cuda.Stream(dev)
    ref = tr.MixedCells(table, 96, torch, dev, stream=main.cuda_stream, **kw)
    fes = torch.cuda.Stream(dev) if fe else None
    two = tr.MixedCells(table, 96, torch, dev, stream=main.cuda_stream, engines=2, tail_stream=tail.cuda_stream,
                        fe_stream=fes.cuda_stream if fe else None, **kw)
    torch.cuda.synchronize()
    ref.step()  # default schedule (auto: this small job runs fused)
    torch.cuda.synchronize()
    want = _results(ref)
    keep = s.get_schedule()
    s.set_schedule(es_fused=es_fused, es_chunk=8)
    # 14 dB: every TB fails (the failed TBs' deferred rows, k_derm_late, run in the tail); 16.5 dB: mixed
    for k in range(4):  # both engines twice, back to back without a host wait between the steps
        two.step()
        if k % 2 == 1:
            torch.cuda.synchronize()
            for e in (0, 1):  # both engines' last batch
                two.eng = e
                for a, b in zip(_results(two), want):
                    assert (a == b).all(), (k, e)
            two.eng = 0
    torch.cuda.synchronize()
    s.set_schedule(**keep)
    ref.close()
    two.close()
