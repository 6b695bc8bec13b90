"""Parity of the MI355X PDSCH receiver (srsgpu_pdsch_*): descrambled int16 LLRs bit-exact with the
CPU oracle (RE map + equaliser + demapper + scrambling, itself pinned to the srsLTE reference),
CSI mode within the reference's rcpps tolerance, and the full grid -> transport block chain."""
import numpy as np
import pytest

from srsgpu_testlib import BITS_PER_SYMBOL, DlschOracle, PdschOracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s():
    import srsgpu_phy
    return srsgpu_phy


@pytest.fixture(scope="module")
def po(oracle):
    return PdschOracle(oracle)


def _grids(rng, n_sf, size, nrx=1):
    y = (rng.standard_normal((n_sf, nrx, size)) + 1j * rng.standard_normal((n_sf, nrx, size))).astype(np.complex64)
    h = (rng.standard_normal((n_sf, nrx, size)) + 1j * rng.standard_normal((n_sf, nrx, size))).astype(np.complex64)
    return y, h


def _oracle_llr(po, y, h, idx, mod, seed, noise, csi=False):
    x = po.predecode(y[idx], h[idx], 1.0, noise, csi)
    if csi:
        x = x[0]
    return po.scramble(seed, po.demod(mod, x))


@pytest.mark.parametrize("nof_prb,cell_id", [(100, 1), (25, 17), (6, 500), (75, 11)])
def test_llr_vs_oracle(s, po, nof_prb, cell_id):
    """Random grids/channels, all modulations, subframes 0/1/5, random PRB masks and CFI:
    LLRs equal the oracle bit for bit (ZF and MMSE)."""
    import torch
    rng = np.random.default_rng(nof_prb + cell_id)
    size = nof_prb * 12 * 14
    n_sf = 12
    y, h = _grids(rng, n_sf, size)
    p = s.Pdsch(nof_prb, cell_id, max_sf=n_sf)
    sfs, expect, offs, off = [], [], [], 0
    for i in range(n_sf):
        sf_idx = [0, 1, 5, 3][i % 4]
        lstart = 1 + i % 3
        mask = np.ones((2, nof_prb), np.uint8) if i % 3 == 0 else (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
        mod = [1, 2, 3, 3][i % 4]
        noise = 0.0 if i % 2 else 0.05
        rnti = int(rng.integers(1, 65535))
        idx = po.re_map(nof_prb, cell_id, 1, lstart, sf_idx, mask)
        sf = s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mod,
                       nof_re=idx.size, rnti=rnti, noise=noise, grid_offset=i * size)
        assert p.nof_re(sf) == idx.size
        sfs.append(sf)
        expect.append(_oracle_llr(po, y[i, 0], h[i, 0], idx, mod, po.seed(rnti, 0, 2 * sf_idx, cell_id), noise))
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


@pytest.mark.parametrize("mod", [1, 2, 3])
def test_llr_csi_mode(s, po, mod):
    """CSI weighting (srsUE default, pdsch.c:676-776): bit-exact with the oracle's restatement.
    (The oracle's equaliser uses an exact reciprocal where the reference uses rcpps; see
    test_pdsch_oracle.py for that tolerance.)"""
    import torch
    rng = np.random.default_rng(5 + mod)
    nof_prb, cell_id, size = 50, 3, 50 * 12 * 14
    y, h = _grids(rng, 1, size)
    h[0, 0] *= (0.2 + rng.random(size)).astype(np.float32)
    p = s.Pdsch(nof_prb, cell_id, max_sf=1)
    p.set_csi(True)
    mask = np.ones((2, nof_prb), np.uint8)
    mask[1, 7] = 0  # odd symbol count: exercises the C tails
    idx = po.re_map(nof_prb, cell_id, 1, 2, 1, mask)
    sf = s.make_sf(sf_idx=1, lstart=2, prb=mask, nof_prb=nof_prb, mod=mod, nof_re=idx.size, rnti=77,
                   noise=0.1)
    q = BITS_PER_SYMBOL[mod]
    d_y = torch.from_numpy(y.reshape(-1)).cuda()
    d_h = torch.from_numpy(h.reshape(-1)).cuda()
    d_e = torch.zeros(idx.size * q, dtype=torch.int16, device="cuda")
    assert p.llr_dev([sf], d_y.data_ptr(), d_h.data_ptr(), size, d_e.data_ptr(), [0]) == 0
    torch.cuda.synchronize()
    x, csi = po.predecode(y[0, 0][idx], h[0, 0][idx], 1.0, 0.1, True)
    llr = po.scramble(po.seed(77, 0, 2, cell_id), po.demod(mod, x))
    assert (d_e.cpu().numpy() == po.csi_correction(mod, csi, llr)).all()
    p.close()


def _modulate(bits, mod):
    """36.211 7.1 mapping consistent with the soft demapper's sign/offset conventions."""
    b = bits.reshape(-1, {1: 2, 2: 4, 3: 6}[mod]).astype(np.float32)
    if mod == 1:
        return ((1 - 2 * b[:, 0]) + 1j * (1 - 2 * b[:, 1])) / np.sqrt(2)
    if mod == 2:
        return ((1 - 2 * b[:, 0]) * (1 + 2 * b[:, 2]) + 1j * (1 - 2 * b[:, 1]) * (1 + 2 * b[:, 3])) / np.sqrt(10)
    amp = lambda hi, lo: np.where(hi == 0, np.where(lo == 0, 3, 1), np.where(lo == 0, 5, 7))
    return ((1 - 2 * b[:, 0]) * amp(b[:, 2], b[:, 4]) + 1j * (1 - 2 * b[:, 1]) * amp(b[:, 3], b[:, 5])) / np.sqrt(42)


def test_full_chain_grid_to_tb(s, po, oracle):
    """TB -> DL-SCH encode -> scramble -> 64QAM -> RE map -> Rayleigh-ish channel + AWGN grid;
    the GPU decodes every subframe's TB and agrees with the oracle chain on ret / bytes / noi."""
    import torch
    dl = DlschOracle(oracle)
    rng = np.random.default_rng(11)
    nof_prb, cell_id, size, n_sf = 100, 1, 100 * 12 * 14, 6
    tbs = 75376
    p = s.Pdsch(nof_prb, cell_id, nof_softbuffers=n_sf, max_sf=n_sf)
    ys, hs, sfs, datas = [], [], [], []
    dlen = tbs // 8 + 6
    for i in range(n_sf):
        sf_idx = 1 + i
        idx = po.re_map(nof_prb, cell_id, 1, 1, sf_idx, np.ones((2, nof_prb), np.uint8))
        nbits = idx.size * 6
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        e = dl.encode(tbs, 0, 6, nbits, data)
        c = po.sequence(po.seed(1234, 0, 2 * sf_idx, cell_id), nbits)
        sym = _modulate(e ^ c, 3).astype(np.complex64)
        hgrid = ((1 + 0.1 * rng.standard_normal(size)) * np.exp(1j * rng.uniform(0, 6.28, size))).astype(np.complex64)
        grid = np.zeros(size, np.complex64)
        grid[idx] = sym
        snr_db = 32.0 if i < 4 else 18.0
        noise = (10 ** (-snr_db / 20) / np.sqrt(2)) * (rng.standard_normal(size) + 1j * rng.standard_normal(size))
        ys.append((hgrid * grid + noise).astype(np.complex64))
        hs.append(hgrid)
        datas.append(data)
        sfs.append(s.make_sf(sf_idx=sf_idx, lstart=1, nof_prb=nof_prb, mod=3, nof_re=idx.size, rnti=1234,
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
        llr = _oracle_llr(po, ys[i], hs[i], idx, 3, po.seed(1234, 0, 2 * (1 + i), cell_id), sfs[i].noise_estimate)
        dl.reset(sb)
        r, od, onoi, _ = dl.decode(sb, tbs, 0, 6, llr, 8)
        assert ret[i] == r and noi[i] == onoi, (i, ret[i], r, noi[i], onoi)
        assert (out[i][:(tbs + 24) // 8] == od[:(tbs + 24) // 8]).all(), i
        if i < 4:
            assert r == 0 and (out[i][:tbs // 8] == datas[i]).all(), i
    dl.free(sb)
    p.close()


def test_re_count_mismatch_is_an_error(s):
    p = s.Pdsch(25, 1, max_sf=1)
    import torch
    d = torch.zeros(25 * 12 * 14 * 2, dtype=torch.float32, device="cuda")
    sf = s.make_sf(sf_idx=1, lstart=1, nof_prb=25, mod=1, nof_re=123)
    assert p.llr_dev([sf], d.data_ptr(), d.data_ptr(), 25 * 12 * 14, d.data_ptr(), [0]) == -1
    p.close()


@pytest.mark.parametrize("nof_prb,cell_id,swap,csi", [(100, 3, 0, False), (25, 101, 1, False),
                                                       (50, 7, 0, True), (15, 400, 1, True)])
def test_llr_cdd_vs_oracle(s, po, nof_prb, cell_id, swap, csi):
    """TM3 CDD 2x2 MMSE (2 ports, 2 rx, 2 TBs per subframe): every TB's LLRs equal the oracle
    (exact-reciprocal restatement of srslte_mat_2x2_mmse_csi_gen) bit for bit, codeword / layer /
    scrambling q chosen through tb_cw_swap as pdsch.c:959-995 does; CSI weighting per codeword."""
    import torch
    rng = np.random.default_rng(3 * nof_prb + cell_id)
    size = nof_prb * 12 * 14
    n_sf = 6
    y = (rng.standard_normal((n_sf, 2, size)) + 1j * rng.standard_normal((n_sf, 2, size))).astype(np.complex64)
    h = (rng.standard_normal((n_sf, 2, 2, size)) + 1j * rng.standard_normal((n_sf, 2, 2, size))).astype(np.complex64)
    p = s.Pdsch(nof_prb, cell_id, nof_ports=2, nof_rx_ant=2, max_sf=n_sf)
    p.set_csi(csi)
    sfs, expect, offs, off = [], [], [], 0
    for i in range(n_sf):
        sf_idx = [0, 1, 5][i % 3]
        lstart = 1 + i % 3
        mask = np.ones((2, nof_prb), np.uint8) if i % 2 == 0 else (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
        mods = ([3, 2], [1, 3], [2, 2])[i % 3]
        noise = 0.05 + 0.05 * (i % 2)
        rnti = int(rng.integers(1, 65535))
        idx = po.re_map(nof_prb, cell_id, 2, lstart, sf_idx, mask)
        sf = s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mods,
                       nof_re=idx.size, rnti=rnti, noise=noise, grid_offset=i * 2 * size,
                       ce_offset=i * 4 * size, mimo=s.MIMO_CDD, tb_cw_swap=swap)
        assert p.nof_re(sf) == idx.size
        sfs.append(sf)
        # h[sf][rx][port] planes on the device; the oracle takes h[port][rx]
        hp = [[h[i, a, port][idx] for a in (0, 1)] for port in (0, 1)]
        xs = po.predecode_ccd([y[i, 0][idx], y[i, 1][idx]], hp, 1.0, noise, csi)
        x, c = (xs if csi else (xs, None))
        for tb in (0, 1):
            cw = tb ^ swap
            e = po.demod(mods[tb], x[cw])
            e = po.scramble(po.seed(rnti, cw, 2 * sf_idx, cell_id), e)
            if csi:
                e = po.csi_correction(mods[tb], c[cw], e)
            expect.append(e)
            offs.append(off)
            off += e.size
    d_y = torch.from_numpy(y.reshape(-1)).cuda()
    d_h = torch.from_numpy(h.reshape(-1)).cuda()
    d_e = torch.zeros(off + 8, dtype=torch.int16, device="cuda")
    assert p.llr_dev(sfs, d_y.data_ptr(), d_h.data_ptr(), size, d_e.data_ptr(), offs) == 0
    torch.cuda.synchronize()
    e = d_e.cpu().numpy()
    for k in range(len(expect)):
        got = e[offs[k]:offs[k] + expect[k].size]
        assert (got == expect[k]).all(), (k, np.nonzero(got != expect[k])[0][:5])
    p.close()


def test_cdd_needs_two_port_cell(s):
    """a CDD subframe on a 1-port cell is refused (precoding.c:1085-1097)"""
    import torch
    p = s.Pdsch(25, 1, max_sf=1)
    sf = s.make_sf(sf_idx=1, lstart=1, nof_prb=25, mod=(1, 1), nof_re=1, mimo=s.MIMO_CDD)
    d = torch.zeros(25 * 12 * 14 * 4, dtype=torch.complex64, device="cuda")
    d_e = torch.zeros(100000, dtype=torch.int16, device="cuda")
    assert p.llr_dev([sf], d.data_ptr(), d.data_ptr(), 25 * 12 * 14, d_e.data_ptr(), [0, 0]) == -1
    p.close()
