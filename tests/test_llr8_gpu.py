"""Parity of the 8-bit LLR receive chain on the GPU (srslte_pdsch_t / srslte_sch_t llr_is_8bit:
pdsch.c:795-806, sch.c:344-364): int8 demapping + scrambling + CSI (srsgpu_pdsch_set_llr_8bit),
8-bit de-rate-matching (srsgpu_rm_turbo_rx_8bit_dev) and the DL-SCH decode on int8 softbuffer
rows, against golden vectors recorded from the reference (tests/golden/make_llr8_golden.py) and
the oracle chain (itself pinned to the reference, tests/test_llr8_oracle.py)."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import BITS_PER_SYMBOL, DlschOracle, Llr8, PdschOracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def s():
    import srsgpu_phy
    return srsgpu_phy


@pytest.fixture(scope="module")
def po(oracle):
    return PdschOracle(oracle)


@pytest.fixture(scope="module")
def l8(oracle):
    return Llr8(oracle)


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "llr8_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def _oracle_llr8(po, l8, y, h, idx, mod, rnti, sf_idx, cell_id, noise, csi=False):
    x = po.predecode(y[idx], h[idx], 1.0, noise, csi)
    c = None
    if csi:
        x, c = x
    llr = l8.scramble(rnti, 0, 2 * sf_idx, cell_id, l8.demod(mod, x))
    return l8.csi_correction(mod, c, llr) if csi else llr


@pytest.mark.parametrize("nof_prb,cell_id", [(100, 1), (25, 17), (6, 500)])
def test_llr8_vs_oracle(s, po, l8, nof_prb, cell_id):
    """Random grids and channels, QPSK/16QAM/64QAM, subframes 0/1/5, random PRB masks (odd symbol
    counts reach the C tails): int8 LLRs equal the oracle bit for bit."""
    import torch
    rng = np.random.default_rng(100 + nof_prb + cell_id)
    size = nof_prb * 12 * 14
    n_sf = 9
    y = (rng.standard_normal((n_sf, size)) + 1j * rng.standard_normal((n_sf, size))).astype(np.complex64)
    h = (rng.standard_normal((n_sf, size)) + 1j * rng.standard_normal((n_sf, size))).astype(np.complex64)
    y *= np.float32(3.0)  # some symbols saturate the int8 range
    p = s.Pdsch(nof_prb, cell_id, max_sf=n_sf)
    p.set_llr_8bit(True)
    sfs, expect, offs, off = [], [], [], 0
    for i in range(n_sf):
        sf_idx = [0, 1, 5][i % 3]
        lstart = 1 + i % 3
        mask = np.ones((2, nof_prb), np.uint8) if i % 3 == 0 else (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
        mod = [1, 2, 3][i % 3]
        noise = 0.0 if i % 2 else 0.05
        rnti = int(rng.integers(1, 65535))
        idx = po.re_map(nof_prb, cell_id, 1, lstart, sf_idx, mask)
        sfs.append(s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mod,
                             nof_re=idx.size, rnti=rnti, noise=noise, grid_offset=i * size))
        expect.append(_oracle_llr8(po, l8, y[i], h[i], idx, mod, rnti, sf_idx, cell_id, noise))
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
        assert (got == expect[i].astype(np.int16)).all(), (i, np.nonzero(got != expect[i])[0][:5])
    p.close()


@pytest.mark.parametrize("mod", [1, 2, 3])
def test_llr8_csi_mode(s, po, l8, mod):
    """8-bit CSI weighting (pdsch.c:707-713) on the oracle's exact-reciprocal CSI"""
    import torch
    rng = np.random.default_rng(50 + mod)
    nof_prb, cell_id, size = 50, 3, 50 * 12 * 14
    y = (rng.standard_normal(size) + 1j * rng.standard_normal(size)).astype(np.complex64)
    h = ((rng.standard_normal(size) + 1j * rng.standard_normal(size)) * (0.2 + rng.random(size))).astype(np.complex64)
    p = s.Pdsch(nof_prb, cell_id, max_sf=1)
    p.set_csi(True)
    p.set_llr_8bit(True)
    mask = np.ones((2, nof_prb), np.uint8)
    mask[1, 7] = 0
    idx = po.re_map(nof_prb, cell_id, 1, 2, 1, mask)
    sf = s.make_sf(sf_idx=1, lstart=2, prb=mask, nof_prb=nof_prb, mod=mod, nof_re=idx.size,
                   rnti=77, noise=0.1)
    d_y, d_h = torch.from_numpy(y).cuda(), torch.from_numpy(h).cuda()
    d_e = torch.zeros(idx.size * BITS_PER_SYMBOL[mod], dtype=torch.int16, device="cuda")
    assert p.llr_dev([sf], d_y.data_ptr(), d_h.data_ptr(), size, d_e.data_ptr(), [0]) == 0
    torch.cuda.synchronize()
    want = _oracle_llr8(po, l8, y, h, idx, mod, 77, 1, cell_id, 0.1, csi=True)
    assert (d_e.cpu().numpy() == want.astype(np.int16)).all()
    p.close()


def test_rm8_dev_golden(s, gold):
    """srsgpu_rm_turbo_rx_8bit_dev == the reference's srslte_rm_turbo_rx_lut_8bit"""
    import torch
    z, man = gold
    g = s.Dlsch(1, 4, 16)
    for c in (c for c in man if c["kind"] == "rm"):
        e = torch.from_numpy(z[c["key"] + "_e"].astype(np.int16)).cuda()
        init = z[c["key"] + "_init"]
        out = torch.zeros(18600, dtype=torch.int16, device="cuda")
        out[:init.size] = torch.from_numpy(init.astype(np.int16)).cuda()
        assert g.rm_rx_8bit_dev(e.data_ptr(), out.data_ptr(), e.numel(), c["K"], c["rv"]) == 0
        torch.cuda.synchronize()
        got = out.cpu().numpy()[:init.size]
        assert (got == z[c["key"] + "_out"].astype(np.int16)).all(), c["key"]
    g.close()


def test_dlsch8_golden_harq_sequences(s, gold):
    """Each golden 8-bit TB in its own softbuffer: every transmission's return code, noi, bytes
    and cb_crc equal the reference's srslte_dlsch_decode2 with llr_is_8bit."""
    z, man = gold
    tbc = [c for c in man if c["kind"] == "tb"]
    g = s.Dlsch(len(tbc), 16, 64)
    g.set_llr_8bit(True)
    for slot, c in enumerate(tbc):
        g.reset(slot)
        for t in c["tx"]:
            llr = z[t["key"] + "_llr"].astype(np.int16)
            ret, data, noi = g.decode([dict(tbs=c["tbs"], rv=t["rv"], Qm=c["Qm"], nof_e_bits=c["nbits"],
                                            softbuffer=slot)], [llr], 8)
            assert (ret[0], int(noi[0])) == (t["ret"], t["noi"]), (t["key"], ret, noi)
            nb = (c["tbs"] + 24) // 8
            if ret[0] == 0:
                assert (data[0][:nb] == z[t["key"] + "_data"]).all(), t["key"]
            crc = g.read_cb_crc(slot)
            C = z[t["key"] + "_cbcrc"].size
            assert (crc[:C] == z[t["key"] + "_cbcrc"]).all(), t["key"]
    g.close()


def test_dlsch8_one_call_vs_oracle(s, oracle, l8, gold):
    """All golden first transmissions in ONE 8-bit call (mixed K: AVX8 / SSE8 windows and the 16-bit
    fallback) against the oracle's orc_dlsch_decode8, data bytes included for failed TBs."""
    z, man = gold
    dl = DlschOracle(oracle)
    tbc = [c for c in man if c["kind"] == "tb"]
    g = s.Dlsch(len(tbc), 16, 128)
    g.set_llr_8bit(True)
    for slot in range(len(tbc)):
        g.reset(slot)
    tbl = [dict(tbs=c["tbs"], rv=c["tx"][0]["rv"], Qm=c["Qm"], nof_e_bits=c["nbits"], softbuffer=i)
           for i, c in enumerate(tbc)]
    ret, data, noi = g.decode(tbl, [z[c["tx"][0]["key"] + "_llr"].astype(np.int16) for c in tbc], 8)
    for i, c in enumerate(tbc):
        sb = dl.softbuffer(16)
        dl.reset(sb)
        r, od, onoi, _ = l8.decode(sb, c["tbs"], c["tx"][0]["rv"], c["Qm"], z[c["tx"][0]["key"] + "_llr"], 8)
        dl.free(sb)
        assert (ret[i], int(noi[i])) == (r, onoi), c["key"]
        nb = (c["tbs"] + 24) // 8
        assert (data[i][:nb] == od[:nb]).all(), c["key"]
    g.close()


def test_dlsch8_refuses_undefined_sizes(s):
    """400 < K <= 800 has no defined 8-bit result in the reference: -2, other TBs unaffected"""
    g = s.Dlsch(2, 4, 16)
    g.set_llr_8bit(True)
    g.reset(0)
    g.reset(1)
    ones = np.ones(1200, np.int16)
    ret, _, _ = g.decode([dict(tbs=456, rv=0, Qm=2, nof_e_bits=1200, softbuffer=0),
                          dict(tbs=120, rv=0, Qm=2, nof_e_bits=1200, softbuffer=1)], [ones, ones], 8)
    assert ret[0] == -2 and ret[1] in (0, -1)
    g.close()


def test_full_chain_grid_to_tb_8bit(s, po, l8, oracle):
    """TB -> encode -> scramble -> 16QAM -> grid with channel + AWGN -> GPU 8-bit chain; equal to the
    oracle's 8-bit chain (ret / noi / bytes) and error-free at high SNR"""
    import torch
    from test_pdsch_gpu import _modulate
    dl = DlschOracle(oracle)
    rng = np.random.default_rng(21)
    nof_prb, cell_id, size, n_sf, tbs = 50, 7, 50 * 12 * 14, 4, 20616
    p = s.Pdsch(nof_prb, cell_id, nof_softbuffers=n_sf, max_sf=n_sf)
    p.set_llr_8bit(True)
    ys, hs, sfs, datas = [], [], [], []
    dlen = tbs // 8 + 6
    for i in range(n_sf):
        sf_idx = 1 + i
        idx = po.re_map(nof_prb, cell_id, 1, 1, sf_idx, np.ones((2, nof_prb), np.uint8))
        nbits = idx.size * 4
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        e = dl.encode(tbs, 0, 4, nbits, data)
        c = po.sequence(po.seed(1234, 0, 2 * sf_idx, cell_id), nbits)
        sym = _modulate(e ^ c, 2).astype(np.complex64)
        hgrid = ((1 + 0.1 * rng.standard_normal(size)) * np.exp(1j * rng.uniform(0, 6.28, size))).astype(np.complex64)
        grid = np.zeros(size, np.complex64)
        grid[idx] = sym
        snr_db = 30.0 if i < 2 else 9.0
        noise = (10 ** (-snr_db / 20) / np.sqrt(2)) * (rng.standard_normal(size) + 1j * rng.standard_normal(size))
        ys.append((hgrid * grid + noise).astype(np.complex64))
        hs.append(hgrid)
        datas.append(data)
        sfs.append(s.make_sf(sf_idx=sf_idx, lstart=1, nof_prb=nof_prb, mod=2, nof_re=idx.size, rnti=1234,
                             noise=float(10 ** (-snr_db / 10)), tbs=tbs, rv=0, softbuffer=i,
                             grid_offset=i * size, data_offset=i * dlen))
        p.reset_softbuffer(i)
    d_y = torch.from_numpy(np.stack(ys).reshape(-1)).cuda()
    d_h = torch.from_numpy(np.stack(hs).reshape(-1)).cuda()
    d_data = torch.zeros(n_sf * dlen, dtype=torch.uint8, device="cuda")
    d_ret = torch.full((n_sf,), 9, dtype=torch.int32, device="cuda")
    d_noi = torch.zeros(n_sf, dtype=torch.int32, device="cuda")
    assert p.decode_dev(sfs, d_y.data_ptr(), d_h.data_ptr(), size, d_data.data_ptr(), 8,
                        d_ret.data_ptr(), d_noi.data_ptr()) == 0
    torch.cuda.synchronize()
    ret, noi = d_ret.cpu().numpy(), d_noi.cpu().numpy()
    out = d_data.cpu().numpy().reshape(n_sf, dlen)
    sb = dl.softbuffer(16)
    for i in range(n_sf):
        idx = po.re_map(nof_prb, cell_id, 1, 1, 1 + i, np.ones((2, nof_prb), np.uint8))
        llr = _oracle_llr8(po, l8, ys[i], hs[i], idx, 2, 1234, 1 + i, cell_id, sfs[i].noise_estimate)
        dl.reset(sb)
        r, od, onoi, _ = l8.decode(sb, tbs, 0, 4, llr, 8)
        assert ret[i] == r and noi[i] == onoi, (i, ret[i], r, noi[i], onoi)
        assert (out[i][:(tbs + 24) // 8] == od[:(tbs + 24) // 8]).all(), i
        if i < 2:
            assert r == 0 and (out[i][:tbs // 8] == datas[i]).all(), i
    dl.free(sb)
    p.close()
