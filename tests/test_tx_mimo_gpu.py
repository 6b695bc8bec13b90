"""The two-port transmitter (srsgpu_pdsch_encode_ports_dev) and TM2 / TM3 / TM4 traffic end to end.

  - the GPU transmitter against the reference's own srslte_pdsch_encode (pdsch.c:1048-1131 with
    srslte_layermap_type / srslte_precoding_type, compiled into oracle/_ref): transmit diversity, CDD
    with and without the codeword swap, spatial multiplexing of 1 layer (codebooks 0-3) and 2 layers
    (codebooks 1-2), several cells and subframes (0 and 5 included), equal grids on every port;
  - BASELINE configs[3] at full size: 1024 coded TM3 subframes (two MCS-28 TBs each) built on the GPU,
    through a 2x2 channel, received by the GPU pipeline (FFT, 2-port channel estimation, CDD 2x2 MMSE,
    DL-SCH): every TB acks with its transmitted bytes, and sampled subframes decoded by the reference's
    srslte_pdsch_decode on the same grids and estimates give the same acks, bytes and nof_iterations;
  - TM2 and TM4 traffic the same way at a smaller size.
"""
import ctypes

import numpy as np
import pytest

from srsgpu_testlib import Oracle, PdschOracle, Ref, have_ref

pytestmark = pytest.mark.gpu

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)


def _ref_sigs(L):
    u32 = ctypes.c_uint32
    L.ref_pdsch_encode.argtypes = [u32] * 5 + [ctypes.c_uint16] + [u32] * 4 + [_u32p, _u32p, _u8p, _u8p, _f32p]
    L.ref_pdsch_decode_mimo.argtypes = ([u32] * 6 + [ctypes.c_uint16] + [u32] * 4 + [_u32p, _u32p, ctypes.c_float,
                                        _f32p, _f32p, _u8p, _u8p, _i32p, _u32p])
    L.ref_mcs_tbs.argtypes = [u32, u32, _u32p]
    return L


def _p(a, t):
    return a.ctypes.data_as(t)


def _mcs_tbs(L, mcs, nof_prb):
    mod = ctypes.c_uint32(0)
    tbs = L.ref_mcs_tbs(mcs, nof_prb, ctypes.byref(mod))
    return tbs, mod.value


CASES = [  # (nof_prb, cell_id, mimo, ntb, pmi, swap, mcs)
    (25, 3, 1, 1, 0, 0, (12, 0)),     # transmit diversity
    (6, 501, 1, 1, 0, 0, (5, 0)),
    (100, 1, 3, 2, 0, 0, (28, 28)),   # TM3 CDD
    (50, 77, 3, 2, 0, 1, (20, 9)),    # CDD, codeword swap, different modulations
    (25, 9, 2, 1, 0, 0, (15, 0)),     # TM4, one layer, codebooks 0..3
    (25, 9, 2, 1, 1, 0, (15, 0)),
    (25, 9, 2, 1, 2, 0, (15, 0)),
    (25, 9, 2, 1, 3, 0, (15, 0)),
    (50, 140, 2, 2, 0, 0, (24, 17)),  # TM4, two layers, codebooks 1 and 2
    (50, 140, 2, 2, 1, 1, (24, 17)),
]
CASES = [c + (2,) for c in CASES] + [
    # transmit diversity at MCS 28: the codeword's E bits split over 13 blocks with Qm x Nl = 12
    # (sch.c:535-545), which differs from a split by Qm in these subframes
    (100, 41, 1, 1, 0, 0, (28, 0), 2),
    # 4-port transmit diversity (precoding.c:1863-1889)
    (25, 3, 1, 1, 0, 0, (12, 0), 4), (100, 41, 1, 1, 0, 0, (28, 0), 4), (15, 502, 1, 1, 0, 0, (7, 0), 4)]


@pytest.mark.skipif(not have_ref(), reason="needs the reference build (oracle/_ref)")
@pytest.mark.parametrize("nof_prb,cell_id,mimo,ntb,pmi,swap,mcs,nports", CASES)
def test_encode_ports_vs_reference(nof_prb, cell_id, mimo, ntb, pmi, swap, mcs, nports):
    import torch
    import srsgpu_phy as s
    L = _ref_sigs(Ref().lib)
    rng = np.random.default_rng(nof_prb + 7 * mimo + pmi)
    gsz = 14 * 12 * nof_prb
    sfs_idx = [0, 1, 5, 8]
    cfi = 2 if nof_prb > 10 else 3
    pd = s.Pdsch(nof_prb, cell_id, nof_ports=nports, nof_rx_ant=2, max_sf=len(sfs_idx))
    tb = [_mcs_tbs(L, m, nof_prb) for m in mcs]
    dlen = s.dlsch_data_len(max(t[0] for t in tb)) + 2
    data = rng.integers(0, 256, (len(sfs_idx), 2, dlen)).astype(np.uint8)
    sfs, refs = [], []
    for j, sf_idx in enumerate(sfs_idx):
        sf = s.make_sf(sf_idx=sf_idx, lstart=cfi + 1 if nof_prb < 10 else cfi, nof_prb=nof_prb, mod=(tb[0][1], tb[1][1]), rnti=0x3321,
                       tbs=(tb[0][0], tb[1][0] if ntb == 2 else 0), rv=(0, 0), mimo=mimo,
                       grid_offset=j * nports * gsz, data_offset=((2 * j) * dlen, (2 * j + 1) * dlen), tb_cw_swap=swap,
                       codebook_idx=pmi + (1 if (mimo == 2 and ntb == 2) else 0))
        sf.nof_re = pd.nof_re(sf)
        sfs.append(sf)
        g = np.zeros(nports * gsz, np.complex64)
        mc = np.array(mcs, np.uint32)
        rv = np.zeros(2, np.uint32)  # the reference encodes a fresh softbuffer only at rv 0 (sch.c)
        nre = L.ref_pdsch_encode(nof_prb, cell_id, nports, cfi, sf_idx, 0x3321, mimo, pmi, swap, ntb, _p(mc, _u32p),
                                 _p(rv, _u32p), _p(data[j, 0], _u8p), _p(data[j, 1], _u8p), _p(g, _f32p))
        assert nre == sf.nof_re, (nre, sf.nof_re)
        refs.append(g)
    d_data = torch.from_numpy(data.reshape(-1)).cuda()
    d_grid = torch.zeros(len(sfs_idx) * nports * gsz, dtype=torch.complex64, device="cuda")
    assert pd.encode_dev(sfs, d_data.data_ptr(), d_grid.data_ptr(), port_stride=gsz) == 0
    torch.cuda.synchronize()
    got = d_grid.cpu().numpy().reshape(len(sfs_idx), nports * gsz)
    po = PdschOracle(Oracle())
    for j in range(len(sfs_idx)):
        want = refs[j].copy()
        n = sfs[j].nof_re
        if mimo == 3 and n % 4:
            # the reference's AVX CDD precoder (precoding.c:1898-1917) leaves the last nof_re mod 4
            # symbols of each port as whatever its buffer held: those REs are not compared
            idx = po.re_map(nof_prb, cell_id, 2, sfs[j].lstart, sfs_idx[j], np.ones((2, nof_prb), np.uint8))
            assert idx.size == n
            for p in range(2):
                want[p * gsz + idx[4 * (n // 4):]] = got[j][p * gsz + idx[4 * (n // 4):]]
        assert np.array_equal(got[j].view(np.uint64), want.view(np.uint64)), \
            (j, np.max(np.abs(got[j] - want)), np.count_nonzero(got[j] != want))
    pd.close()


def _ref_decode(L, m, j, mimo, pmi, ntb, mcs):
    """the reference's srslte_pdsch_decode of subframe j of a MimoSubframes m on its grids / estimates"""
    gsz, P = m.gsz, m.nports
    y = m.grid.cpu().numpy().reshape(m.n, 2, gsz)[j]
    ce = m.ce.cpu().numpy().reshape(m.n, 2, P, gsz)[j]          # [rx][port]
    h = np.ascontiguousarray(np.transpose(ce, (1, 0, 2)))        # [port][rx]
    nz = m.noise.cpu().numpy().reshape(m.n, 2, P)[j]  # [rx][port]
    f = np.float32  # srslte_chest_dl_get_noise_estimate's float order (chest_dl.c:741-750)
    acc = f(0)
    for a in range(2):
        sa = f(0)
        for p in range(P):
            sa = f(sa + nz[a, p])
        acc = f(acc + sa / f(P))
    noise = float(acc / f(2))
    sf = m.sfs[j]
    d0 = np.zeros(m.tbs // 8 + 8, np.uint8)
    d1 = np.zeros(m.tbs // 8 + 8, np.uint8)
    ok = np.zeros(2, np.int32)
    noi = np.zeros(2, np.uint32)
    mc = np.array(mcs, np.uint32)
    rv = np.zeros(2, np.uint32)
    r = L.ref_pdsch_decode_mimo(m.nof_prb, m.cell_id, P, 2, sf.lstart, sf.sf_idx, sf.rnti, mimo, pmi, sf.tb_cw_swap,
                                ntb, _p(mc, _u32p), _p(rv, _u32p), noise, _p(np.ascontiguousarray(y), _f32p),
                                _p(h, _f32p), _p(d0, _u8p), _p(d1, _u8p), _p(ok, _i32p), _p(noi, _u32p))
    assert r == 0
    return ok[:ntb], (d0, d1)[:ntb], noi[:ntb]


@pytest.mark.skipif(not have_ref(), reason="needs the reference build (oracle/_ref)")
def test_tm3_full_size_tx_rx():
    """BASELINE configs[3] per-GPU shard at full size: 1024 TM3 subframes, 2048 TBs"""
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    L = _ref_sigs(Ref().lib)
    # full estimate planes: the reference decoder below reads them (compact rows: test_ce_rows_gpu.py)
    m = tr.MimoSubframes(torch, torch.device("cuda"), 1024, seed=5, snr_db=30.0, ce_rows=False)
    m.step()
    torch.cuda.synchronize()
    acks, good, noi = m.check()
    assert acks == 2048 and good == 2048, (acks, good)
    ret = m.d_ret.cpu().numpy()
    nois = m.d_noi.cpu().numpy()
    data = m.d_data.cpu().numpy()
    for j in (0, 1, 513, 1023):  # both codeword orders
        ok, dref, noiref = _ref_decode(L, m, j, s.MIMO_CDD, 0, 2, (28, 28))
        for t in range(2):
            o = (2 * j + t) * m.dlen
            assert ok[t] == 1 and ret[2 * j + t] == 0, (j, t)
            assert (data[o:o + m.tbs // 8] == dref[t][:m.tbs // 8]).all(), (j, t)
            assert nois[2 * j + t] == noiref[t], (j, t, nois[2 * j + t], noiref[t])
    m.close()


@pytest.mark.skipif(not have_ref(), reason="needs the reference build (oracle/_ref)")
@pytest.mark.parametrize("mimo,ntb,codebook,mcs", [(1, 1, 0, 16), (2, 2, 1, 26), (2, 2, 2, 22), (2, 1, 3, 14),
                                                   (2, 1, 0, 20)])
def test_tm2_tm4_tx_rx(mimo, ntb, codebook, mcs):
    """transmit diversity and spatial multiplexing traffic: every TB acks with its bytes; two subframes
    decoded by the reference on the same grids and estimates agree"""
    import torch
    import srsgpu_traffic as tr
    L = _ref_sigs(Ref().lib)
    m = tr.MimoSubframes(torch, torch.device("cuda"), 64, seed=9 + codebook, snr_db=32.0, mimo=mimo, mcs=mcs,
                         nof_prb=50, cell_id=88, codebook=codebook, nof_tb=ntb, ce_rows=False)
    m.step()
    torch.cuda.synchronize()
    acks, good, _ = m.check()
    assert acks == good == 64 * m.ntb, (acks, good)
    ret, nois, data = m.d_ret.cpu().numpy(), m.d_noi.cpu().numpy(), m.d_data.cpu().numpy()
    pmi = codebook - 1 if (mimo == 2 and ntb == 2) else codebook
    for j in (0, 37):
        ok, dref, noiref = _ref_decode(L, m, j, mimo, pmi, m.ntb, (mcs, mcs))
        for t in range(m.ntb):
            k = 2 * j + t if m.ntb == 2 else j
            o = (2 * j + t) * m.dlen
            assert ok[t] == 1 and ret[k] == 0 and nois[k] == noiref[t], (j, t)
            assert (data[o:o + m.tbs // 8] == dref[t][:m.tbs // 8]).all(), (j, t)
    m.close()


@pytest.mark.skipif(not have_ref(), reason="needs the reference build (oracle/_ref)")
@pytest.mark.parametrize("nof_prb,cell_id,mcs,csi", [(50, 21, 20, False), (100, 6, 27, True)])
def test_tm2_four_ports_tx_rx(nof_prb, cell_id, mcs, csi):
    """4-port transmit diversity end to end: GPU encoder (RE quadruplets on port pairs 0/2 and 1/3), the
    CRS of ports 0-3, OFDM, a 2x4 channel; GPU OFDM / channel estimation of all four ports / SFBC
    predecoding / DL-SCH: every TB acks with its bytes, and the reference's srslte_pdsch_decode on the
    same grids and estimates of two subframes agrees (ack, bytes, nof_iterations)"""
    import torch
    import srsgpu_traffic as tr
    L = _ref_sigs(Ref().lib)
    m = tr.MimoSubframes(torch, torch.device("cuda"), 48, seed=13 + nof_prb, snr_db=30.0, mimo=1, mcs=mcs,
                         nof_prb=nof_prb, cell_id=cell_id, nof_tb=1, ce_rows=False, nof_ports=4)
    m.pd.set_csi(csi)
    m.step()
    torch.cuda.synchronize()
    acks, good, _ = m.check()
    assert acks == good == 48, (acks, good)
    ret, nois, data = m.d_ret.cpu().numpy(), m.d_noi.cpu().numpy(), m.d_data.cpu().numpy()
    if not csi:  # the reference harness decodes with CSI off
        for j in (0, 29):
            ok, dref, noiref = _ref_decode(L, m, j, 1, 0, 1, (mcs, mcs))
            o = 2 * j * m.dlen
            assert ok[0] == 1 and ret[j] == 0 and nois[j] == noiref[0], (j, nois[j], noiref[0])
            assert (data[o:o + m.tbs // 8] == dref[0][:m.tbs // 8]).all(), j
    m.close()
