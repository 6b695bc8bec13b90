"""Extended cyclic prefix (SRSLTE_CP_EXT, 6 OFDM symbols per slot) along the receive path: OFDM
(ofdm.c:75-76), CRS and channel estimation (refsignal_dl.c:112-122, 265-318; chest_dl.c:433-441),
PDSCH RE order (pdsch.c:95-234), PDCCH REGs (regs.c:587-616) and, on the GPU, coded subframes sent
and received end to end.

CPU: the oracle restatements (with 256 added to nof_ports for an extended-CP cell) against golden
vectors recorded from the reference build (tests/golden/make_extcp_golden.py) and, with oracle/_ref,
against the reference live. GPU: every stage against the same golden data / the oracle chain."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402
import ofdm_oracle as oo  # noqa: E402
from srsgpu_testlib import (BITS_PER_SYMBOL, PdschOracle, Ref, have_ref, have_ref_front, pdcch_map,  # noqa: E402
                            predecode_txdiv, ref_front_chest)

HERE = os.path.dirname(os.path.abspath(__file__))
EXT = 256
ALG = {0: "refs", 1: "pss", 2: "empty"}


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "extcp_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_re_maps(oracle, gold):
    z, man = gold
    po = PdschOracle(oracle)
    assert len(man["re_maps"]) == 72
    for m in man["re_maps"]:
        got = po.re_map(m["nof_prb"], m["cell_id"], m["nports"] | EXT, m["lstart"], m["sf_idx"], z[m["key"] + "_mask"])
        assert np.array_equal(got, z[m["key"]]), m


def test_golden_pdcch_maps(oracle, gold):
    z, man = gold
    for m in man["pdcch_maps"]:
        idx, ncce = pdcch_map(oracle, m["nof_prb"], m["cell_id"], m["nports"] | EXT, m["phich_len"], m["phich_res"],
                              m["cfi"])
        assert ncce == m["nof_cce"] and np.array_equal(idx, z[m["key"]]), m
    # symbol 3 of the 4-symbol regions below 11 PRB has CRS with extended CP: other REG orders
    m = [c for c in man["pdcch_maps"] if c["nof_prb"] == 6 and c["cfi"] == 3][0]
    idx_n, _ = pdcch_map(oracle, m["nof_prb"], m["cell_id"], m["nports"], m["phich_len"], m["phich_res"], 3)
    assert not np.array_equal(idx_n, z[m["key"]])


def test_golden_crs(gold):
    z, man = gold
    for m in man["crs"]:
        want = z[m["key"]]
        got = co.crs_pilots(m["nof_prb"], m["cell_id"], m["sf_idx"], 2 * m["pair"], cp=1).astype(np.complex64)
        assert np.array_equal(got.reshape(-1), want), m


def _noise_before(z, c, i):
    """q->noise_estimate before subframe i of the recorded sequence"""
    if i == 0:
        return np.full((c["nrx"], c["nports"]), c["noise_init"], np.float32)
    return z["%s_%d_noise" % (c["key"], i - 1)]


def _filt(c):
    return co.gauss_filter(*c["gauss"]) if c["gauss"] else (0.1, 0.8, 0.1)


def test_golden_chest_oracle(gold):
    z, man = gold
    for c in man["chest"]:
        for i, sf in enumerate(c["sfs"]):
            nb = _noise_before(z, c, i)
            for a in range(c["nrx"]):
                g = z["%s_%d_y%d" % (c["key"], i, a)].astype(np.complex128)
                for p in range(c["nports"]):
                    ce, nz = co.estimate_full(g, c["nof_prb"], c["cell_id"], sf, _filt(c), p, c["average"],
                                              ALG[c["noise_alg"]], c["smooth_auto"], float(nb[a, p]), c["nports"], cp=1)
                    want = z["%s_%d_ce" % (c["key"], i)][a, p]
                    assert np.max(np.abs(ce - want)) / np.max(np.abs(want)) < 1e-4, (c["key"], sf, a, p)
                    rn = float(z["%s_%d_noise" % (c["key"], i)][a, p])
                    assert abs(nz - rn) <= 1e-4 * abs(rn) + 1e-9, (c["key"], sf, a, p)
                    m = co.measurements(g, c["nof_prb"], c["cell_id"], sf, p, c["symbol_sz"], cp=1)
                    for v, f in zip((m[0], m[1], m[3]), ("rsrp", "rssi", "cfo")):
                        w = float(z["%s_%d_%s" % (c["key"], i, f)][a, p])
                        assert abs(v - w) <= 1e-4 * abs(w) + 1e-7, (c["key"], f, v, w)


@pytest.mark.skipif(not (have_ref() and have_ref_front()), reason="oracle/_ref not built")
def test_live_vs_reference(oracle):
    """random cells, grants and grids: RE and REG orders and estimates against the reference run here"""
    ref = Ref()
    po = PdschOracle(oracle)
    rng = np.random.default_rng(77)
    get = ref.lib.ref_pdsch_get
    get.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_void_p] * 3
    for nof_prb in (6, 9, 27, 100):
        for nports in (1, 2, 4):
            cid = int(rng.integers(0, 504))
            for sf in (0, 5, 7):
                mask = (rng.random((2, nof_prb)) < 0.5).astype(np.uint8)
                g = np.arange(12 * 12 * nof_prb).astype(np.complex64)
                out = np.zeros_like(g)
                n = get(nof_prb, cid, nports | EXT, 2, sf, mask.ctypes.data, g.ctypes.data, out.ctypes.data)
                assert np.array_equal(po.re_map(nof_prb, cid, nports | EXT, 2, sf, mask), out[:n].real.astype(np.uint32))
            for cfi in (1, 3):
                a = pdcch_map(oracle, nof_prb, cid, nports | EXT, 1, 1, cfi)
                b = pdcch_map(ref, nof_prb, cid, nports | EXT, 1, 1, cfi, ref=True)
                assert np.array_equal(a[0], b[0]) and a[1] == b[1]
    nof_prb, nports, nrx = 15, 4, 2
    cid = int(rng.integers(0, 504))
    sfs = [0, 3]
    n = 12 * 12 * nof_prb
    grids = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
             for _ in sfs]
    out = ref_front_chest(nof_prb, cid, nports, nrx, sfs, grids, cp=1)
    for i, sf in enumerate(sfs):
        for a in range(nrx):
            for p in range(nports):
                ce, _ = co.estimate_full(grids[i][a].astype(np.complex128), nof_prb, cid, sf, port=p, nof_ports=nports,
                                         cp=1)
                want = out[i]["ce"][a, p]
                assert np.max(np.abs(ce - want)) / np.max(np.abs(want)) < 1e-4


def test_ofdm_oracle_roundtrip():
    """12-symbol grids through the oracle transmitter and receiver; every CP is a copy of its symbol's
    tail and the 6 symbols of a slot fill 7.5 N samples"""
    rng = np.random.default_rng(3)
    for nof_prb, N in ((6, 128), (25, 384), (100, 2048)):
        g = rng.standard_normal(12 * 12 * nof_prb) + 1j * rng.standard_normal(12 * 12 * nof_prb)
        x = oo.tx_sf(g, nof_prb, N, ext=True)
        assert np.allclose(oo.rx_sf(x, nof_prb, N, ext=True), N * g)  # unnormalised DFT pair
        st = oo.symbol_starts(N, ext=True)
        assert st[6] == N * 15 // 2 + N // 4 and st[-1] + N == 15 * N
        assert np.allclose(x[st[1] - N // 4:st[1]], x[st[1] + 3 * N // 4:st[1] + N])


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,standard", [(100, True), (25, False), (6, False), (75, True)])
def test_gpu_ofdm_ext(nof_prb, standard):
    """receive against numpy's FFT on the extended-CP symbol layout, and transmit -> receive"""
    import torch
    import srsgpu_phy as s
    N = s.symbol_sz(nof_prb, standard)
    rng = np.random.default_rng(nof_prb + N)
    n, gsz = 4, 12 * 12 * nof_prb
    x = (rng.standard_normal((n, 15 * N)) + 1j * rng.standard_normal((n, 15 * N))).astype(np.complex64)
    o = s.OfdmRx(nof_prb, N, cp=1)
    d_x = torch.from_numpy(x.reshape(-1)).cuda()
    d_g = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    assert o.rx_dev(n, d_x.data_ptr(), 15 * N, d_g.data_ptr(), gsz) == 0
    torch.cuda.synchronize()
    got = d_g.cpu().numpy().reshape(n, -1)
    for i in range(n):
        want = oo.rx_sf(x[i], nof_prb, N, ext=True)
        rms = np.sqrt(np.mean(np.abs(want) ** 2))
        assert np.max(np.abs(got[i] - want)) / rms < 1e-4, i
    g = (rng.standard_normal((n, gsz)) + 1j * rng.standard_normal((n, gsz))).astype(np.complex64)
    d_g.copy_(torch.from_numpy(g.reshape(-1)))
    assert o.tx_dev(n, d_g.data_ptr(), gsz, d_x.data_ptr(), 15 * N) == 0
    torch.cuda.synchronize()
    xt = d_x.cpu().numpy().reshape(n, -1)
    for i in range(n):
        want = oo.tx_sf(g[i], nof_prb, N, ext=True)
        rms = np.sqrt(np.mean(np.abs(want) ** 2))
        assert np.max(np.abs(xt[i] - want)) / rms < 1e-4, i
    assert o.rx_dev(n, d_x.data_ptr(), 15 * N, d_g.data_ptr(), gsz - 1) == -1  # grid stride below 12 symbols
    o.close()


@pytest.mark.gpu
def test_gpu_chest_ext_vs_golden(gold):
    """the GPU estimator of an extended-CP cell against chest_dl.c's recordings, one call per subframe
    (rx antennas as separate grids) with the recorded noise state before it"""
    import torch
    import srsgpu_phy as s
    z, man = gold
    for c in man["chest"]:
        nprb, npt, nrx = c["nof_prb"], c["nports"], c["nrx"]
        size = 12 * 12 * nprb
        ch = s.Chest(nprb, c["cell_id"], max_grids=nrx, nof_ports=npt, cp=1)
        if c["gauss"]:
            ch.set_filter_gauss(int(c["gauss"][0]), float(c["gauss"][1]))
        else:
            ch.set_filter([0.1, 0.8, 0.1])
        ch.set_cfg(average_subframe=c["average"], noise_alg=c["noise_alg"], smooth_filter_auto=c["smooth_auto"],
                   rsrp_neighbour=True, cfo_enable=True, cfo_mask=0x3FF)
        for i, sf in enumerate(c["sfs"]):
            g = np.stack([z["%s_%d_y%d" % (c["key"], i, a)] for a in range(nrx)])
            d_g = torch.from_numpy(g.reshape(-1)).cuda()
            d_ce = torch.zeros(npt * nrx * size, dtype=torch.complex64, device="cuda")
            d_n = torch.from_numpy(_noise_before(z, c, i).reshape(-1).astype(np.float32)).cuda()
            d_m = torch.zeros(nrx * npt * 4, dtype=torch.float32, device="cuda")
            assert ch.estimate_meas_dev([sf] * nrx, d_g.data_ptr(), size, d_ce.data_ptr(), d_n.data_ptr(),
                                        d_m.data_ptr()) == 0
            torch.cuda.synchronize()
            ce = d_ce.cpu().numpy().reshape(nrx, npt, size)
            nz = d_n.cpu().numpy().reshape(nrx, npt)
            me = d_m.cpu().numpy().reshape(nrx, npt, 4)
            want = z["%s_%d_ce" % (c["key"], i)]
            for a in range(nrx):
                for p in range(npt):
                    w = want[a, p]
                    assert np.max(np.abs(ce[a, p] - w)) / np.max(np.abs(w)) < 1e-4, (c["key"], sf, a, p)
                    rn = float(z["%s_%d_noise" % (c["key"], i)][a, p])
                    assert abs(nz[a, p] - rn) <= 1e-4 * abs(rn) + 1e-9, (c["key"], sf, a, p, nz[a, p], rn)
                    for j, f in ((0, "rsrp"), (1, "rssi"), (3, "cfo")):
                        wv = float(z["%s_%d_%s" % (c["key"], i, f)][a, p])
                        assert abs(me[a, p, j] - wv) <= 1e-4 * abs(wv) + 1e-7, (c["key"], f, me[a, p, j], wv)
        ch.close()


@pytest.mark.gpu
def test_gpu_pdcch_cell_map_ext(gold):
    import srsgpu_phy as s
    z, man = gold
    for m in man["pdcch_maps"]:
        idx, ncce = s.pdcch_cell_map(m["nof_prb"], m["cell_id"], m["nports"], m["phich_len"], m["phich_res"],
                                     m["cfi"], cp=1)
        assert ncce == m["nof_cce"] and np.array_equal(np.asarray(idx, np.uint32), z[m["key"]]), m


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id,nrx,csi,nports", [(100, 3, 1, False, 1), (25, 40, 1, True, 1),
                                                            (50, 301, 2, False, 2), (6, 9, 1, True, 4),
                                                            (15, 402, 2, False, 4)])
def test_gpu_pdsch_ext_llr_vs_oracle(oracle, nof_prb, cell_id, nrx, csi, nports):
    """random 12-symbol grids and channels, QPSK/16QAM/64QAM, subframes 0/1/5, random PRB masks; 1 port
    SISO (1 rx), 2 / 4 ports transmit diversity: the GPU's descrambled int16 LLRs equal the oracle chain"""
    import torch
    import srsgpu_phy as s
    po = PdschOracle(oracle)
    rng = np.random.default_rng(nof_prb + cell_id)
    size = nof_prb * 12 * 12
    n_sf = 6
    y = (rng.standard_normal((n_sf, nrx, size)) + 1j * rng.standard_normal((n_sf, nrx, size))).astype(np.complex64)
    h = (rng.standard_normal((n_sf, nrx, nports, size)) +
         1j * rng.standard_normal((n_sf, nrx, nports, size))).astype(np.complex64)
    p = s.Pdsch(nof_prb, cell_id, nof_ports=nports, nof_rx_ant=nrx, max_sf=n_sf, cp=1)
    p.set_csi(csi)
    sfs, expect, offs, off = [], [], [], 0
    ragged = []
    for i in range(n_sf):
        sf_idx = [0, 1, 5][i % 3]
        lstart = 1 + i % 3
        mask = np.ones((2, nof_prb), np.uint8) if i % 2 == 0 else (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
        mod = [1, 2, 3][i % 3]
        rnti = int(rng.integers(1, 65535))
        scaling = 1.0 if i % 2 else 0.7943
        idx = po.re_map(nof_prb, cell_id, nports | EXT, lstart, sf_idx, mask)
        mimo = s.MIMO_SINGLE_ANTENNA if nports == 1 else s.MIMO_TX_DIVERSITY
        if nports == 4 and idx.size % 4:  # a ragged 4-port grant (one half PRB beside the PBCH): refused
            bad = s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mod, nof_re=idx.size,
                            mimo=mimo)
            ragged.append(bad)
            mask[:] = 1
            idx = po.re_map(nof_prb, cell_id, nports | EXT, lstart, sf_idx, mask)
        sfs.append(s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mod, nof_re=idx.size,
                             rnti=rnti, scaling=scaling, mimo=mimo, grid_offset=i * nrx * size,
                             ce_offset=i * nrx * nports * size))
        if nports == 1:  # one rx antenna (srslte_predecoding_single)
            out = po.predecode(y[i, 0][idx], h[i, 0, 0][idx], scaling, 0.0, csi)
        else:
            out = predecode_txdiv(oracle, [y[i, a][idx] for a in range(nrx)],
                                  [[h[i, a, pp][idx] for a in range(nrx)] for pp in range(nports)], scaling, csi)
        d = out[0] if csi else out
        llr = po.scramble(po.seed(rnti, 0, 2 * sf_idx, cell_id), po.demod(mod, d))
        expect.append(po.csi_correction(mod, out[1], llr) if csi else llr)
        offs.append(off)
        off += idx.size * BITS_PER_SYMBOL[mod]
        assert p.nof_re(sfs[-1]) == idx.size
    d_y = torch.from_numpy(y.reshape(-1)).cuda()
    d_h = torch.from_numpy(h.reshape(-1)).cuda()
    d_e = torch.zeros(off + 8, dtype=torch.int16, device="cuda")
    for bad in ragged:
        assert p.llr_dev([bad], d_y.data_ptr(), d_h.data_ptr(), size, d_e.data_ptr(), [0]) == -1
    assert p.llr_dev(sfs, d_y.data_ptr(), d_h.data_ptr(), size, d_e.data_ptr(), offs) == 0
    torch.cuda.synchronize()
    e = d_e.cpu().numpy()
    for i in range(n_sf):
        got = e[offs[i]:offs[i] + expect[i].size]
        assert (got == expect[i]).all(), (i, np.nonzero(got != expect[i])[0][:5])
    p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mimo,nports", [(0, 1), (1, 2), (1, 4), (3, 2)])
def test_gpu_ext_tx_rx(mimo, nports):
    """coded extended-CP subframes end to end on the GPU: DL-SCH encode, precoding, CRS, OFDM TX, a flat
    2 x P channel at 30 dB, OFDM RX, channel estimation, PDSCH and DL-SCH: every TB acks with its bytes"""
    import torch
    import srsgpu_traffic as tr
    m = tr.MimoSubframes(torch, torch.device("cuda"), 24, seed=17 + nports, snr_db=30.0, mimo=mimo, mcs=20,
                         nof_prb=50, ce_rows=False, nof_ports=nports, cp=1)
    m.step()
    torch.cuda.synchronize()
    acked, good, _ = m.check()
    assert acked == good == m.ntb * m.n, (acked, good, m.ntb * m.n)
    m.close()


@pytest.mark.gpu
def test_gpu_ext_queue():
    """an extended-CP cell through the subframe queue (srsgpu_rxq_*: OFDM, channel estimation and the
    PDSCH of the cell's CP): SISO subframes on 2 rx antennas decode as the direct batch call does"""
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    m = tr.MimoSubframes(torch, torch.device("cuda"), 12, seed=23, snr_db=30.0, mimo=s.MIMO_SINGLE_ANTENNA, mcs=20,
                         nof_prb=25, ce_rows=False, nof_ports=1, cp=1)
    m.step()
    torch.cuda.synchronize()
    acked, good, _ = m.check()
    assert acked == good == m.n
    x = m.x.cpu().numpy().reshape(m.n, 2, 15 * m.N)
    q = s.RxQueue(25, m.cell_id, m.N, nof_ports=1, nof_rx_ant=2, nof_softbuffers=m.n, max_batch=4,
                  max_wait_us=2000, cp=1)
    tx = m.d_data_tx.cpu().numpy().reshape(m.n, 2, m.dlen)
    nb = m.tbs // 8
    for j, i in enumerate(m.kept):
        td = [np.ascontiguousarray(x[j, a]) for a in range(2)]
        out = np.zeros(m.dlen, np.uint8)
        sf = s.make_sf(sf_idx=1 + (i % 4), lstart=1, nof_prb=25, mod=3, rnti=1234, tbs=m.tbs, softbuffer=j)
        sf.nof_re = m.pd.nof_re(sf)
        it = q.item(td, sf, [out])
        assert q.decode(it) == 0 and it.ret[0] == 0, j
        assert (out[:nb] == tx[j, 0, :nb]).all(), j
    q.close()
    m.close()
