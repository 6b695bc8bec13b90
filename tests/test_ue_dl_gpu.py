"""srslte_ue_dl_decode_rnti on the batch queue (ue_dl.c:467-620): worker threads
submit time-domain subframes that carry a control region (PCFICH with the subframe's CFI, a PDCCH
Format 1A DCI for the UE's C-RNTI at a UE-specific location, encoded by the reference's
srslte_pdcch_encode) and the PDSCH of that DCI's grant; the queue runs FFT -> channel estimation ->
PCFICH -> PDCCH LLRs + DL DCI search -> grant -> PDSCH / DL-SCH per batch.

Checked per subframe: the detected CFI, the found DCI (format, location, message bits), the grant,
the return value (TB 0's size), the ack and the transmitted bytes; and every stage against the
direct batch APIs run on the same samples (PCFICH CFI / correlation, the DCI search result, the
PDSCH's TB bytes and nof_iterations), bit for bit. Subframes addressed to another RNTI return 0 with
no PDSCH decode, and grant items share the batches. The DCI packer is the reference's
(oracle/_ref, tests only)."""
import os
import sys
import threading

import numpy as np
import pytest

from srsgpu_testlib import (F1A, DlschOracle, PdschOracle, dci_pack_dl_ref, have_ref, pcfich_re_map,
                            pdcch_encode)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402
import ofdm_oracle as oo  # noqa: E402
from test_pdsch_gpu import _modulate  # noqa: E402

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not have_ref(), reason="needs the reference DCI packer")]

PHICH_LEN, PHICH_RES = 0, 2  # normal, Ng = 1


def _riv(L, start, N):
    return (L - 1) * N + start if L - 1 <= N // 2 else N * (N - L + 1) + (N - 1 - start)


def _pcfich_symbols(po, nof_prb, cell_id, sf_idx, cfi):
    """36.212 5.3.4 CFI codeword, 36.211 6.7.1 scrambling and QPSK (pcfich.c:244-290's encoder)"""
    b = np.array([(i % 3 != 0) if cfi == 1 else (i % 3 != 1) if cfi == 2 else (i % 3 != 2) for i in range(32)],
                 np.uint8)
    c = po.sequence(((sf_idx + 1) * (2 * cell_id + 1) << 9) + cell_id, 32)
    z = b ^ c
    return ((1 - 2.0 * z[0::2]) + 1j * (1 - 2.0 * z[1::2])) / np.sqrt(2)


def build_ue_subframe(s, ref, oracle, po, dl, rng, nof_prb, cell_id, N, tti, rnti, cfi, snr_db, flat=False,
                      ul=None):
    """(time-domain subframe, tx data, DCI bits, (L, ncce), grant) of one TM1 subframe (flat: no
    frequency-selective channel). ul: a format 0 message for the same RNTI, placed at another free
    UE-specific location (the UL grant phch_worker looks for after the DL one)"""
    sf_idx = tti % 10
    _, nof_cce = s.pdcch_cell_map(nof_prb, cell_id, 1, PHICH_LEN, PHICH_RES, cfi)
    locs = [lc for lc in s.pdcch_locations(nof_cce, sf_idx, rnti) if lc[1] <= 87]
    L, ncce = locs[int(rng.integers(0, len(locs)))]
    msgs = []
    if ul is not None:
        free = [lc for lc in locs if lc[1] + (1 << lc[0]) <= ncce or lc[1] >= ncce + (1 << L)]
        if free:
            uL, uc = free[int(rng.integers(0, len(free)))]
            msgs.append((ul, uL, uc, rnti))
    Lcrb = int(rng.integers(2, nof_prb + 1))
    start = int(rng.integers(0, nof_prb - Lcrb + 1))
    mcs = int(rng.integers(0, 17))
    f = [0] * 30
    f[0], f[5], f[6], f[7], f[12], f[23] = 2, _riv(Lcrb, start, nof_prb), Lcrb, start, mcs, 1
    bits = dci_pack_dl_ref(ref, F1A, nof_prb, 1, True, f)
    r, _, g = s.dci_msg_to_dl_grant(bits, F1A, rnti, nof_prb, 1)
    assert r == 0 and g.tb_en[0]
    tbs, mod = int(g.tbs[0]), int(g.mod[0])
    qm = {1: 2, 2: 4, 3: 6}[mod]
    mask = np.array([[g.prb_idx[sl][p] for p in range(nof_prb)] for sl in range(2)], np.uint8)
    idx = po.re_map(nof_prb, cell_id, 1, cfi, sf_idx, mask)
    nbits = idx.size * qm
    data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
    e = dl.encode(tbs, 0, qm, nbits, data)
    c = po.sequence(po.seed(rnti, 0, 2 * sf_idx, cell_id), nbits)
    grid = np.zeros(14 * 12 * nof_prb, np.complex128)
    grid[idx] = _modulate(e ^ c, mod)
    grid += pdcch_encode(ref, nof_prb, cell_id, 1, PHICH_LEN, PHICH_RES, cfi, sf_idx,
                         [(bits, L, ncce, rnti)] + msgs)[0]
    grid[pcfich_re_map(oracle, nof_prb, cell_id)] = _pcfich_symbols(po, nof_prb, cell_id, sf_idx, cfi)
    g2 = grid.reshape(14, -1)
    pil = co.crs_pilots(nof_prb, cell_id, sf_idx)
    for l, sy in enumerate(co.SYMS):
        g2[sy, co.fidx(cell_id, l) + 6 * np.arange(2 * nof_prb)] = pil[l]
    k = np.arange(12 * nof_prb)
    ph = rng.uniform(0, 6.28)
    h = 1.0 if flat else np.tile((1 + 0.3 * np.cos(2 * np.pi * k / k.size + ph)) * np.exp(1j * (ph + 0.5 * np.sin(2 * np.pi * k / k.size))), 14)
    x = oo.tx_sf(grid * h, nof_prb, N) / N
    sig = 10 ** (-snr_db / 20) / np.sqrt(2 * N)
    x = x + sig * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
    return x.astype(np.complex64), data, bits, (L, ncce), g, bool(msgs)


def _direct(s, torch, xs, ttis, rntis, nof_prb, cell_id, N):
    """the same subframes through the batch APIs one stage at a time: CFI, correlation, DCI results"""
    n, gsz = len(xs), 14 * 12 * nof_prb
    ofdm, chest = s.OfdmRx(nof_prb, N), s.Chest(nof_prb, cell_id, max_grids=n)
    d_x = torch.from_numpy(np.stack(xs).reshape(-1)).cuda()
    d_grid = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    d_ce = torch.zeros_like(d_grid)
    d_noise = torch.zeros(n, dtype=torch.float32, device="cuda")
    assert ofdm.rx_dev(n, d_x.data_ptr(), 15 * N, d_grid.data_ptr(), gsz) == 0
    assert chest.estimate_dev([t % 10 for t in ttis], d_grid.data_ptr(), gsz, d_ce.data_ptr(),
                              d_noise.data_ptr()) == 0
    torch.cuda.synchronize()
    noise = d_noise.cpu().numpy()
    pc = s.Pcfich(nof_prb, cell_id)
    d_cfi = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_corr = torch.zeros(n, dtype=torch.float32, device="cuda")
    sfs = [(i * gsz, i * gsz, ttis[i] % 10, float(noise[i])) for i in range(n)]
    assert pc.decode_dev(sfs, d_grid.data_ptr(), d_ce.data_ptr(), gsz, d_cfi.data_ptr(), d_corr.data_ptr()) == 0
    torch.cuda.synchronize()
    cfi, corr = d_cfi.cpu().numpy(), d_corr.cpu().numpy()
    pd = s.Pdcch(nof_prb, cell_id, 1, 1, PHICH_LEN, PHICH_RES)
    stride = 72 * 88
    d_llr = torch.zeros(n * stride, dtype=torch.float32, device="cuda")
    psf = [(i * gsz, i * gsz, i * stride, ttis[i] % 10, int(cfi[i]), float(noise[i])) for i in range(n)]
    assert pd.extract_llr_dev(psf, d_grid.data_ptr(), d_ce.data_ptr(), gsz, d_llr.data_ptr()) == 0
    se = [(i * stride, ttis[i] % 10, int(cfi[i]), rntis[i], 0, -1, rntis[i]) for i in range(n)]
    d_res = torch.zeros(n * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    d_ul = torch.zeros(n * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    assert pd.find_dci_dev(se, d_llr.data_ptr(), d_res.data_ptr(), d_ul.data_ptr()) == 0
    torch.cuda.synchronize()
    res = s.Pdcch.parse_results(d_res.cpu().numpy().tobytes())
    ul = s.Pdcch.parse_results(d_ul.cpu().numpy().tobytes())
    for h in (ofdm, chest):
        h.close()
    return cfi, corr, res, noise, ul


def test_decode_rnti_through_the_queue(oracle):
    """every item also runs phch_worker's UL search for its RNTI (srslte_ue_dl_find_ul_dci): two thirds of
    the subframes carry a format 0 message, whose grant must come back unpacked as the reference's
    srslte_dci_msg_to_ul_grant unpacks the transmitted bits"""
    import torch
    import srsgpu_phy as s
    from srsgpu_testlib import Ref, dci_to_ul_grant_ref, random_ul_msg
    ref = Ref()
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(31)
    nof_prb, cell_id, rnti = 25, 77, 0x4601
    N = s.symbol_sz(nof_prb, True)
    n, nthreads = 24, 4
    xs, datas, dcis, ttis, rntis, grants, uls = [], [], [], [], [], [], []
    for i in range(n):
        tti = 1000 + 7 * i + (1 if (1000 + 7 * i) % 10 in (0, 5) else 0)  # not 0 / 5: no PSS / SSS
        cfi = 1 + i % 3
        ulb = random_ul_msg(ref, rng, nof_prb, hop_p=0.3) if i % 3 else None
        x, data, bits, loc, g, placed = build_ue_subframe(s, ref, oracle, po, dl, rng, nof_prb, cell_id, N, tti,
                                                          rnti, cfi, 28.0 if i % 4 else 20.0, ul=ulb)
        uls.append(ulb if placed else None)
        xs.append(x)
        datas.append(data)
        dcis.append((bits, loc, cfi))
        ttis.append(tti)
        rntis.append(rnti if i % 6 != 5 else rnti + 1)  # every 6th worker call looks for another UE
        grants.append(g)
    cfi_d, corr_d, res_d, noise_d, ul_d = _direct(s, torch, xs, ttis, rntis, nof_prb, cell_id, N)

    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=2 * n, max_batch=8, max_wait_us=3000)
    q.set_phich(PHICH_LEN, PHICH_RES)
    outs = [np.zeros(int(g.tbs[0]) // 8 + 6, np.uint8) for g in grants]
    items = [q.ue_item([xs[i]], ttis[i], rntis[i], [outs[i]], softbuffer=(2 * i, 2 * i + 1), ul_rnti=rntis[i],
                       n_rb_ho=2 * (i % 2)) for i in range(n)]
    rcs = [None] * n

    def worker(w):
        for i in range(w, n, nthreads):
            rcs[i] = q.decode_rnti(items[i])

    th = [threading.Thread(target=worker, args=(w,)) for w in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert rcs == [0] * n
    batches, done = q.stats()
    assert done == n and batches < n
    found = nul = 0
    for i, u in enumerate(items):
        bits, (L, ncce), cfi = dcis[i]
        # the UL search: as the direct search call, and the transmitted format 0 message where there is one
        assert u.ul_found == ul_d[i][0] and (u.ul_found < 1 or (u.ul_L, u.ul_ncce) == ul_d[i][2:4]), i
        if uls[i] is not None and rntis[i] == rnti:
            assert u.ul_found == 1 and list(u.ul_data[:len(uls[i])]) == list(uls[i]), i
            r, d, g = dci_to_ul_grant_ref(ref, uls[i], nof_prb, 2 * (i % 2))
            assert u.ul_grant_ret == r and u.ul_dci.fields11() == list(d), i
            assert r or u.ul_grant.fields10() == list(g), i
            nul += 1
        elif rntis[i] != rnti or uls[i] is None:
            assert u.ul_found == 0 and u.ul_grant_ret == -1, i
        # every stage equals the direct batch APIs on the same samples
        assert u.cfi == cfi_d[i] and u.cfi_corr == corr_d[i], i
        assert abs(u.noise - noise_d[i]) <= 1e-6 * max(1.0, abs(noise_d[i])), i
        r_found, r_fmt, r_L, r_ncce, r_buf = res_d[i]
        assert u.found == r_found, i
        assert u.cfi == cfi, (i, u.cfi, cfi)
        if rntis[i] != rnti:
            assert u.found == 0 and u.ret == 0 and not u.acks[0], i
            continue
        # the location is the search's first match, which may be a larger candidate covering the
        # transmitted one (its extra CCEs carry no energy, so the soft combining decodes the same)
        assert u.found == 1 and u.format == F1A == r_fmt and (u.L, u.ncce) == (r_L, r_ncce), i
        assert u.ncce <= ncce and ncce + (1 << L) <= u.ncce + (1 << u.L), (i, u.L, u.ncce, L, ncce)
        assert r_buf[:len(bits)].tolist() == list(bits), i
        g = u.grant
        assert g.fields13() == grants[i].fields13(), i
        assert u.rv[0] == 0 and u.mimo_type == s.MIMO_SINGLE_ANTENNA
        assert u.ret == int(grants[i].tbs[0]), (i, u.ret)
        assert u.acks[0] == 1 and (outs[i][:len(datas[i])] == datas[i]).all(), i
        found += 1
    assert found >= n - n // 6 - 1 and nul >= 10


def test_mixed_grant_and_ue_dl_items(oracle):
    """grant items (srsgpu_rxq_submit) and ue_dl items in the same batches: each kind's results are
    the ones it gets alone"""
    import torch  # noqa: F401
    import srsgpu_phy as s
    from srsgpu_testlib import Ref
    ref = Ref()
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(8)
    nof_prb, cell_id, rnti = 15, 12, 0x1234
    N = s.symbol_sz(nof_prb, True)
    n = 10
    built = [build_ue_subframe(s, ref, oracle, po, dl, rng, nof_prb, cell_id, N, 2 + i, rnti, 2, 30.0)[:5]
             for i in range(n)]
    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=2 * n, max_batch=4, max_wait_us=100000)
    q.set_phich(PHICH_LEN, PHICH_RES)
    outs = [np.zeros(int(b[4].tbs[0]) // 8 + 6, np.uint8) for b in built]
    ue_items, gr_items = [], []
    for i, (x, data, bits, loc, g) in enumerate(built):
        if i % 2 == 0:
            ue_items.append((i, q.ue_item([x], 2 + i, rnti, [outs[i]], softbuffer=(2 * i, 2 * i + 1))))
        else:
            mask = np.array([[g.prb_idx[sl][p] for p in range(nof_prb)] for sl in range(2)], np.uint8)
            sf = s.make_sf(sf_idx=(2 + i) % 10, lstart=2, prb=mask, nof_prb=nof_prb, mod=int(g.mod[0]),
                           rnti=rnti, tbs=int(g.tbs[0]), softbuffer=2 * i)
            sf.nof_re = s._lib.srsgpu_pdsch_nof_re(s.ctypes.byref(s.srsgpu_cell_t(nof_prb, cell_id, 1, 1)),
                                                   s.ctypes.byref(sf))
            gr_items.append((i, q.item([x], sf, [outs[i]])))
    tickets = []
    for i in range(n):
        it = dict(ue_items).get(i) or dict(gr_items).get(i)
        tickets.append(q.submit_ue_dl(it) if i % 2 == 0 else q.submit(it))
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    for i, u in ue_items:
        assert u.found == 1 and u.cfi == 2 and u.ret == int(built[i][4].tbs[0]) and u.acks[0], i
    for i, it in gr_items:
        assert it.ret[0] == 0, i
    for i in range(n):
        assert (outs[i][:len(built[i][1])] == built[i][1]).all(), i
    q.close()


def test_acked_tb_is_left_alone(oracle):
    """srslte_pdsch_decode skips a TB whose ack the caller already set (pdsch.c:946-947): through the queue
    its data buffer, nof_iterations and softbuffer stay untouched while the other items decode"""
    import srsgpu_phy as s
    from srsgpu_testlib import Ref
    ref = Ref()
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(12)
    nof_prb, cell_id, rnti = 25, 5, 0x2222
    N = s.symbol_sz(nof_prb, True)
    n = 6
    built = [build_ue_subframe(s, ref, oracle, po, dl, rng, nof_prb, cell_id, N, 11 + i, rnti, 2, 30.0)[:5]
             for i in range(n)]
    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=2 * n, max_batch=n, max_wait_us=100000)
    q.set_phich(PHICH_LEN, PHICH_RES)
    sentinel = 0xA5
    outs = [np.full(int(b[4].tbs[0]) // 8 + 6, sentinel, np.uint8) for b in built]
    items = [q.ue_item([b[0]], 11 + i, rnti, [outs[i]], softbuffer=(2 * i, 2 * i + 1), acks=(i % 2, 0))
             for i, b in enumerate(built)]
    for u in items:
        u.noi[0] = 77
    tickets = [q.submit_ue_dl(u) for u in items]
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    for i, u in enumerate(items):
        assert u.found == 1 and u.ret == int(built[i][4].tbs[0]), i
        if i % 2:
            assert u.acks[0] == 1 and u.noi[0] == 77 and (outs[i] == sentinel).all(), i
        else:
            assert u.acks[0] == 1 and u.noi[0] >= 1 and (outs[i][:len(built[i][1])] == built[i][1]).all(), i
    # a later retransmission into an acked item's softbuffer decodes as if that softbuffer were fresh
    # (the skipped TB never touched it): the same subframe with acks cleared decodes
    items2 = [q.ue_item([built[i][0]], 11 + i, rnti, [outs[i]], softbuffer=(2 * i, 2 * i + 1)) for i in (1, 3)]
    t2 = [q.submit_ue_dl(u) for u in items2]
    q.flush()
    assert all(q.wait(t) == 0 for t in t2)
    for j, i in enumerate((1, 3)):
        assert items2[j].acks[0] == 1 and (outs[i][:len(built[i][1])] == built[i][1]).all(), i
    q.close()
