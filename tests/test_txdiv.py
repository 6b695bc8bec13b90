"""TM2 transmit diversity (2 CRS ports, SFBC over RE pairs; srslte_predecoding_diversity_multi +
srslte_layerdemap_diversity, precoding.c:356-685, layermap.c:143-151): the oracle restatement
(oracle/pdsch_oracle.c orc_predecode_txdiv) against golden vectors recorded from the reference
(tests/golden/make_txdiv_golden.py) and, with oracle/_ref, against the reference on random cases
(CPU); the GPU receiver's LLRs against the oracle chain bit for bit (GPU)."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import BITS_PER_SYMBOL, PdschOracle, Ref, have_ref, predecode_txdiv

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "txdiv_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def _case(z, c):
    y = [z[c["key"] + "_y%d" % a] for a in range(c["nrx"])]
    h = [[z[c["key"] + "_h%d%d" % (p, a)] for a in range(c["nrx"])] for p in range(c.get("ports", 2))]
    return y, h


def test_golden_txdiv(oracle, gold):
    z, man = gold
    assert len(man) == 24 + 16
    for c in man:
        y, h = _case(z, c)
        out = predecode_txdiv(oracle, y, h, c["scaling"], c["csi"])
        d = out[0] if c["csi"] else out
        assert (d.view(np.uint64) == z[c["key"] + "_d"].view(np.uint64)).all(), c["key"]
        if c["csi"]:
            assert (out[1] == z[c["key"] + "_csi"]).all(), c["key"]


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_random_txdiv4_vs_reference(oracle):
    """4 ports: RE quadruplets on ports 0/2 and 1/3 (precoding.c:388-423, 604-662)"""
    ref = Ref()
    rng = np.random.default_rng(44)
    for n in (8, 32, 40, 404):
        for nrx in (1, 2):
            for csi in (False, True):
                y = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                h = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
                      for _ in range(nrx)] for _ in range(4)]
                a = predecode_txdiv(oracle, y, h, 0.9, csi)
                b = predecode_txdiv(ref, y, h, 0.9, csi, ref=True)
                if csi:
                    assert (a[0].view(np.uint64) == b[0].view(np.uint64)).all() and (a[1] == b[1]).all()
                else:
                    assert (a.view(np.uint64) == b.view(np.uint64)).all()


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_random_txdiv_vs_reference(oracle):
    ref = Ref()
    rng = np.random.default_rng(9)
    for n in (2, 30, 36, 102, 600):
        for nrx in (1, 2):
            for csi in (False, True):
                y = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                h = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
                      for _ in range(nrx)] for _ in range(2)]
                a = predecode_txdiv(oracle, y, h, 0.9, csi)
                b = predecode_txdiv(ref, y, h, 0.9, csi, ref=True)
                if csi:
                    assert (a[0].view(np.uint64) == b[0].view(np.uint64)).all() and (a[1] == b[1]).all()
                else:
                    assert (a.view(np.uint64) == b.view(np.uint64)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id,nrx,csi,nports", [(100, 1, 1, False, 2), (25, 17, 2, False, 2),
                                                            (50, 300, 2, True, 2), (6, 501, 1, True, 2),
                                                            (100, 7, 2, False, 4), (50, 33, 1, True, 4),
                                                            (6, 2, 2, True, 4), (16, 401, 1, False, 4)])
def test_gpu_txdiv_llr_vs_oracle(oracle, nof_prb, cell_id, nrx, csi, nports):
    """random grids and 2- or 4-port channels, QPSK/16QAM/64QAM, subframes 0/1/5, random PRB masks:
    descrambled (CSI-weighted) int16 LLRs equal the oracle chain"""
    import torch
    import srsgpu_phy as s
    po = PdschOracle(oracle)
    rng = np.random.default_rng(nof_prb + cell_id + nrx)
    size = nof_prb * 12 * 14
    n_sf = 6
    y = (rng.standard_normal((n_sf, nrx, size)) + 1j * rng.standard_normal((n_sf, nrx, size))).astype(np.complex64)
    h = (rng.standard_normal((n_sf, nrx, nports, size)) +
         1j * rng.standard_normal((n_sf, nrx, nports, size))).astype(np.complex64)
    p = s.Pdsch(nof_prb, cell_id, nof_ports=nports, nof_rx_ant=nrx, max_sf=n_sf)
    p.set_csi(csi)
    sfs, expect, offs, off = [], [], [], 0
    for i in range(n_sf):
        sf_idx = [0, 1, 5][i % 3]
        lstart = 1 + i % 3
        mask = np.ones((2, nof_prb), np.uint8) if i % 2 == 0 else (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
        mod = [1, 2, 3][i % 3]
        rnti = int(rng.integers(1, 65535))
        scaling = 1.0 if i % 2 else 0.7943
        idx = po.re_map(nof_prb, cell_id, nports, lstart, sf_idx, mask)
        sfs.append(s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mod,
                             nof_re=idx.size, rnti=rnti, scaling=scaling, mimo=s.MIMO_TX_DIVERSITY,
                             grid_offset=i * nrx * size, ce_offset=i * nrx * nports * size))
        out = predecode_txdiv(oracle, [y[i, a][idx] for a in range(nrx)],
                              [[h[i, a, pp][idx] for a in range(nrx)] for pp in range(nports)], scaling, csi)
        d = out[0] if csi else out
        llr = po.scramble(po.seed(rnti, 0, 2 * sf_idx, cell_id), po.demod(mod, d))
        expect.append(po.csi_correction(mod, out[1], llr) if csi else llr)
        offs.append(off)
        off += idx.size * BITS_PER_SYMBOL[mod]
    d_y = torch.from_numpy(y.reshape(-1)).cuda()
    d_h = torch.from_numpy(h.reshape(-1)).cuda()
    d_e = torch.zeros(off + 8, dtype=torch.int16, device="cuda")
    assert p.llr_dev(sfs, d_y.data_ptr(), d_h.data_ptr(), size, d_e.data_ptr(), offs) == 0
    torch.cuda.synchronize()
    e = d_e.cpu().numpy()
    for i in range(n_sf):
        got = e[offs[i]:offs[i] + expect[i].size]
        assert (got == expect[i]).all(), (i, np.nonzero(got != expect[i])[0][:5])
    p.close()


@pytest.mark.gpu
def test_gpu_txdiv_needs_two_ports():
    import torch
    import srsgpu_phy as s
    p = s.Pdsch(25, 1, nof_ports=1, max_sf=1)
    d = torch.zeros(25 * 12 * 14 * 2, dtype=torch.float32, device="cuda")
    sf = s.make_sf(sf_idx=1, lstart=1, nof_prb=25, mod=1, nof_re=1, mimo=s.MIMO_TX_DIVERSITY)
    assert p.llr_dev([sf], d.data_ptr(), d.data_ptr(), 25 * 12 * 14, d.data_ptr(), [0]) == -1
    p.close()



def test_txdiv4_grants_are_whole_quadruplets(oracle):
    """with 4 CRS ports every normal-CP PDSCH grant has a multiple of 4 REs (full PRBs give 12 or 8 per
    symbol, the half PRBs around PBCH / sync 6 + 6, 4 + 4 and 6 + 6 over symbol pairs), so the
    reference's 4 floor(n / 4) layer symbols always cover the grant"""
    po = PdschOracle(oracle)
    rng = np.random.default_rng(5)
    for nof_prb in (6, 15, 25, 75, 100):
        for sf in (0, 1, 5):
            for lstart in (1, 2, 3, 4):
                for _ in range(3):
                    mask = (rng.random((2, nof_prb)) < 0.5).astype(np.uint8)
                    assert po.re_map(nof_prb, 7, 4, lstart, sf, mask).size % 4 == 0
