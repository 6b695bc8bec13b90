"""Compact channel estimates (srsgpu_chest_set_ce_rows + srsgpu_pdsch_set_ce_rows): the estimator
writes only the rows the reference's time interpolation starts from (chest_dl.c:397-421: the
frequency-interpolated CRS symbols 0 / 4 / 7 / 11, or the averaged row with average_subframe) and
the PDSCH stage interpolates per resource element with the same operations. Pinned against the
full-plane path, which tests/test_chest.py pins to the reference's chest_dl.c: the rows equal the
full planes at their symbols bit for bit, and LLRs / decoded transport blocks are identical."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def table():
    return json.load(open(os.path.join(HERE, "golden", "c5_traffic.json")))


@pytest.mark.parametrize("ports", [1, 2])
@pytest.mark.parametrize("mode", ["per_symbol", "average", "average_auto"])
def test_chest_rows_equal_full_planes(ports, mode):
    import torch
    import srsgpu_phy as s
    prb, n = 50, 12
    nsc, gsz = 12 * prb, 14 * 12 * prb
    rng = np.random.default_rng(3 + ports)
    grid = (rng.standard_normal((n, gsz)) + 1j * rng.standard_normal((n, gsz))).astype(np.complex64)
    d_grid = torch.from_numpy(grid.reshape(-1)).cuda()
    sf_idx = [int(i % 10) for i in range(n)]
    outs = {}
    for rows in (False, True):
        c = s.Chest(prb, 7, max_grids=n, nof_ports=ports)
        if mode != "per_symbol":
            c.set_cfg(average_subframe=True, smooth_filter_auto=(mode == "average_auto"))
        c.set_ce_rows(rows)
        ce = torch.zeros(n * ports * gsz, dtype=torch.complex64, device="cuda")
        noise = torch.zeros(n * ports, dtype=torch.float32, device="cuda")
        assert c.estimate_dev(sf_idx, d_grid.data_ptr(), gsz, ce.data_ptr(), noise.data_ptr()) == 0
        torch.cuda.synchronize()
        outs[rows] = (ce.cpu().numpy().reshape(n * ports, 14, nsc), noise.cpu().numpy())
        c.close()
    full, rows = outs[False][0], outs[True][0]
    assert (outs[False][1] == outs[True][1]).all()
    if mode == "per_symbol":
        for l, sym in enumerate((0, 4, 7, 11)):
            assert (rows[:, l] == full[:, sym]).all(), sym
    else:
        for sym in range(14):
            assert (rows[:, 0] == full[:, sym]).all(), sym


@pytest.mark.parametrize("average", [False, True])
def test_siso_llrs_identical(table, average):
    """MixedCells (6/25/50/100 PRB cells, random allocations and MCS) at 8 dB: the LLRs of every TB
    from compact rows equal those from full planes."""
    import torch
    import srsgpu_traffic as tr
    m = tr.MixedCells(table, 24, torch, torch.device("cuda", 0), seed=9, snr_db=8.0)
    try:
        llrs = {}
        for rows in (True, False):
            for c in m.cells:
                if average:
                    c["chest"].set_cfg(average_subframe=True)
                c["chest"].set_ce_rows(rows)
                c["pd"].set_ce_rows((1 if average else 4) if rows else 0)
            m.d_e.zero_()
            m.front_end()
            torch.cuda.synchronize()
            llrs[rows] = m.d_e.cpu().numpy().copy()
        assert np.abs(llrs[True]).sum() > 0
        assert (llrs[True] == llrs[False]).all()
    finally:
        m.close()


@pytest.mark.parametrize("mimo", ["cdd", "txdiv", "mux"])
def test_two_port_decode_identical(mimo):
    """Two-port cells with 2 rx antennas (TM3 CDD, TM2 transmit diversity, TM4 codebook 1) at an SNR
    where TBs fail and nof_iterations vary: return codes, nof_iterations and bytes are identical
    with compact rows and with full planes."""
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    kind = {"cdd": s.MIMO_CDD, "txdiv": s.MIMO_TX_DIVERSITY, "mux": s.MIMO_SPATIAL_MULTIPLEX}[mimo]
    snr = {"cdd": 21.0, "txdiv": 12.0, "mux": 21.0}[mimo]
    m = tr.MimoSubframes(torch, torch.device("cuda", 0), 16, seed=41, snr_db=snr, mimo=kind)
    try:
        res = {}
        for rows in (True, False):
            m.chest.set_ce_rows(rows)
            m.pd.set_ce_rows(4 if rows else 0)
            m.d_data.zero_()
            m.step()
            torch.cuda.synchronize()
            res[rows] = (m.d_ret.cpu().numpy().copy(), m.d_noi.cpu().numpy().copy(), m.d_data.cpu().numpy().copy())
        for a, b in zip(res[True], res[False]):
            assert (a == b).all()
    finally:
        m.close()
