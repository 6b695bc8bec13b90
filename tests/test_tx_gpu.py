"""Transmit side on the GPU (traffic synthesis): PDSCH modulation + scrambling + RE mapping of
the DL-SCH codeword against the oracle's receive-side restatements run in reverse, CRS placement
against the channel-estimation oracle, OFDM TX against numpy's inverse FFT, and the whole
transmitter into the receiver (time domain -> transport blocks) at full C3 size."""
import os
import sys

import numpy as np
import pytest

from srsgpu_testlib import BITS_PER_SYMBOL, DlschOracle, PdschOracle

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402
import ofdm_oracle as oo  # noqa: E402

pytestmark = pytest.mark.gpu

# modem/lte_tables.c constellations, computed independently from 36.211 7.1 tables
_L16 = {0: 1, 1: 3}
_L64 = {0: 3, 1: 1, 2: 5, 3: 7}


def _modulate(bits, qm):
    b = bits.reshape(-1, qm).astype(np.int64)
    if qm == 2:
        re, im = 1 - 2 * b[:, 0], 1 - 2 * b[:, 1]
        return ((re + 1j * im) / np.sqrt(2)).astype(np.complex64)
    if qm == 4:
        re = (1 - 2 * b[:, 0]) * np.vectorize(_L16.get)(b[:, 2])
        im = (1 - 2 * b[:, 1]) * np.vectorize(_L16.get)(b[:, 3])
        return (re / np.sqrt(10) + 1j * im / np.sqrt(10)).astype(np.complex64)
    re = (1 - 2 * b[:, 0]) * np.vectorize(_L64.get)(2 * b[:, 2] + b[:, 4])
    im = (1 - 2 * b[:, 1]) * np.vectorize(_L64.get)(2 * b[:, 3] + b[:, 5])
    return (re / np.sqrt(42) + 1j * im / np.sqrt(42)).astype(np.complex64)


@pytest.fixture(scope="module")
def s():
    import srsgpu_phy
    return srsgpu_phy


def test_pdsch_encode_vs_oracle(s, oracle):
    """codeword bits (oracle encoder) -> scrambled (oracle Gold sequence) -> modulated -> mapped
    (oracle RE map) equals the GPU grid; REs outside the grant stay untouched"""
    import torch
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(3)
    nof_prb, cell_id = 25, 77
    size = nof_prb * 12 * 14
    p = s.Pdsch(nof_prb, cell_id, max_sf=6)
    sfs, expect, datas = [], [], []
    doff = 0
    for i, (mod, tbs, sf_idx, lstart) in enumerate(((1, 1800, 1, 1), (2, 5736, 0, 2), (3, 12216, 5, 3),
                                                     (3, 18336, 4, 1), (2, 2600, 9, 2), (1, 392, 3, 3))):
        mask = np.ones((2, nof_prb), np.uint8) if i % 2 == 0 else (rng.random((2, nof_prb)) < 0.7).astype(np.uint8)
        idx = po.re_map(nof_prb, cell_id, 1, lstart, sf_idx, mask)
        qm = BITS_PER_SYMBOL[mod]
        rnti, rv = int(rng.integers(1, 65535)), i % 4
        data = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        sfs.append(s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mod,
                             nof_re=idx.size, rnti=rnti, tbs=tbs, rv=rv, grid_offset=i * size,
                             data_offset=doff))
        datas.append((doff, data))
        doff += tbs // 8 + 8
        e = dl.encode(tbs, rv, qm, idx.size * qm, data)
        c = po.sequence(po.seed(rnti, 0, 2 * sf_idx, cell_id), e.size)
        g = np.full(size, 5 + 5j, np.complex64)
        g[idx] = _modulate(e ^ c, qm)
        expect.append(g)
    d_data = torch.zeros(doff, dtype=torch.uint8, device="cuda")
    for off, d in datas:
        d_data[off:off + d.size] = torch.from_numpy(d)
    d_grid = torch.full((6 * size,), 5 + 5j, dtype=torch.complex64, device="cuda")
    assert p.encode_dev(sfs, d_data.data_ptr(), d_grid.data_ptr()) == 0
    got = d_grid.cpu().numpy().reshape(6, size)
    for i in range(6):
        assert (got[i] == expect[i]).all(), (i, np.nonzero(got[i] != expect[i])[0][:5])
    p.close()


@pytest.mark.parametrize("nof_ports", [1, 2])
def test_crs_put(s, nof_ports):
    import torch
    nof_prb, cell_id = 50, 211
    size = nof_prb * 12 * 14
    c = s.Chest(nof_prb, cell_id, max_grids=4, nof_ports=nof_ports)
    d = torch.zeros(4 * nof_ports * size, dtype=torch.complex64, device="cuda")
    assert c.put_crs_dev([0, 3, 7, 9], d.data_ptr(), size) == 0
    got = d.cpu().numpy().reshape(4, nof_ports, 14, 12 * nof_prb)
    for i, sf in enumerate((0, 3, 7, 9)):
        pil = co.crs_pilots(nof_prb, cell_id, sf)
        for p in range(nof_ports):
            exp = np.zeros((14, 12 * nof_prb), np.complex64)
            for l, sym in enumerate(co.SYMS):
                exp[sym, co.fidx(cell_id, l, p) + 6 * np.arange(2 * nof_prb)] = pil[l]
            assert np.allclose(got[i, p], exp, atol=1e-7), (i, p)
    c.close()


@pytest.mark.parametrize("nof_prb,standard", [(100, True), (25, False), (6, False), (75, False)])
def test_ofdm_tx_vs_numpy_and_roundtrip(s, nof_prb, standard):
    import torch
    N = s.symbol_sz(nof_prb, standard)
    rng = np.random.default_rng(N)
    n = 3
    nre = 12 * nof_prb
    g = (rng.standard_normal((n, 14 * nre)) + 1j * rng.standard_normal((n, 14 * nre))).astype(np.complex64)
    o = s.OfdmRx(nof_prb, N)
    d_g = torch.from_numpy(g.reshape(-1)).cuda()
    d_x = torch.zeros(n * 15 * N, dtype=torch.complex64, device="cuda")
    assert o.tx_dev(n, d_g.data_ptr(), 14 * nre, d_x.data_ptr(), 15 * N) == 0
    d_back = torch.zeros_like(d_g)
    assert o.rx_dev(n, d_x.data_ptr(), 15 * N, d_back.data_ptr(), 14 * nre) == 0
    torch.cuda.synchronize()
    x = d_x.cpu().numpy().reshape(n, -1)
    for i in range(n):
        ref = oo.tx_sf(g[i].astype(np.complex128), nof_prb, N)
        assert np.abs(x[i] - ref).max() < 1e-4 * np.abs(ref).max(), i
    back = d_back.cpu().numpy().reshape(n, -1)
    assert np.abs(back - g * N).max() < 1e-3 * N  # rx(tx(g)) = N g (both unnormalised)
    o.close()


def test_tx_to_rx_c3_full_size(s):
    """1024 random 20 MHz TBs (TBS 75376, 64QAM) through the GPU transmitter (DL-SCH + PDSCH
    encoding, CRS, OFDM TX), light AWGN, then the GPU receiver (OFDM RX, channel estimation,
    PDSCH + DL-SCH with early stop): every TB acks with its bytes, mostly in one half-iteration."""
    import torch
    n, nprb, cell, tbs = 1024, 100, 1, 75376
    N = s.symbol_sz(nprb, True)
    gsz = 14 * 12 * nprb
    ofdm = s.OfdmRx(nprb, N)
    chest = s.Chest(nprb, cell, max_grids=n)
    pd = s.Pdsch(nprb, cell, nof_softbuffers=n, max_cb=13, max_sf=n)
    sfi = [1 + (i % 4) for i in range(n)]
    nre = pd.nof_re(s.make_sf(sf_idx=1, lstart=1, nof_prb=nprb, mod=3))
    dlen = tbs // 8 + 6
    sfs = [s.make_sf(sf_idx=sfi[i], lstart=1, nof_prb=nprb, mod=3, nof_re=nre, rnti=1234, tbs=tbs,
                     softbuffer=i, grid_offset=i * gsz, data_offset=i * dlen) for i in range(n)]
    data = torch.randint(0, 256, (n * dlen,), dtype=torch.uint8, device="cuda")
    grid = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    assert pd.encode_dev(sfs, data.data_ptr(), grid.data_ptr()) == 0
    assert chest.put_crs_dev(sfi, grid.data_ptr(), gsz) == 0
    x = torch.zeros(n * 15 * N, dtype=torch.complex64, device="cuda")
    assert ofdm.tx_dev(n, grid.data_ptr(), gsz, x.data_ptr(), 15 * N) == 0
    torch.cuda.synchronize()
    p = x.abs().pow(2).mean().item()
    x += (np.sqrt(p / 10 ** 3.0 / 2) * torch.randn(x.shape, dtype=torch.complex64, device="cuda")).to(torch.complex64)
    rx = torch.zeros_like(grid)
    ce = torch.zeros_like(grid)
    noise = torch.zeros(n, dtype=torch.float32, device="cuda")
    out = torch.zeros(n * dlen, dtype=torch.uint8, device="cuda")
    ret = torch.zeros(n, dtype=torch.int32, device="cuda")
    noi = torch.zeros(n, dtype=torch.int32, device="cuda")
    pd.set_noise_dev(noise.data_ptr())
    assert ofdm.rx_dev(n, x.data_ptr(), 15 * N, rx.data_ptr(), gsz) == 0
    assert chest.estimate_dev(sfi, rx.data_ptr(), gsz, ce.data_ptr(), noise.data_ptr()) == 0
    assert pd.decode_dev(sfs, rx.data_ptr(), ce.data_ptr(), gsz, out.data_ptr(), 8, ret.data_ptr(),
                         noi.data_ptr()) == 0
    torch.cuda.synchronize()
    r = ret.cpu().numpy()
    assert (r == 0).all(), (r != 0).sum()
    got = out.cpu().numpy().reshape(n, dlen)[:, :tbs // 8]
    assert (got == data.cpu().numpy().reshape(n, dlen)[:, :tbs // 8]).all()
    assert noi.cpu().numpy().mean() <= 2.0
    for o in (ofdm, chest, pd):
        o.close()
