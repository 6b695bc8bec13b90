"""PDCCH reception (§8(f) rank 1: the control channel every subframe's PDSCH decode depends on,
include/srsgpu/pdcch_batch.h):

  - the cell's PDCCH symbol order (srslte_regs_init + srslte_regs_pdcch_get, regs.c) and the search
    space locations (pdcch.c:227-300) against golden maps recorded from the reference
    (tests/golden/make_pdcch_golden.py) and, with oracle/_ref, the reference build on more cells (CPU);
  - srsgpu_pdcch_extract_llr_dev against srslte_pdcch_extract_llr_multi (pdcch.c:424-506), bit-exact
    in every float LLR, one subframe per launch and many subframes of mixed CFI / subframe index /
    noise estimate per launch (GPU);
  - srsgpu_pdcch_find_dci_dev against the reference's own ue_dl.c (oracle/_ref/ref_front):
    srslte_ue_dl_find_dl_dci(_type) then srslte_ue_dl_find_ul_dci (ue_dl.c:768-932, phch_worker's
    order): found / format / location / message buffer of both searches, for C-, SI- and RA-RNTIs,
    absent RNTIs, explicit RNTI types, format 0 set aside by the 1A search and taken by the UL search,
    and the found messages through srsgpu_dci_msg_to_dl_grant / _ul_grant (GPU)."""
import json
import os

import numpy as np
import pytest

import srsgpu_phy as s
from srsgpu_testlib import (Ref, dci_to_dl_grant_ref, find_dci_ref, have_ref, have_ref_front, pdcch_llr,
                            pdcch_locations, pdcch_map, pdcch_subframe)

HERE = os.path.dirname(os.path.abspath(__file__))
LLR_STRIDE = 72 * 128  # per-subframe LLR slots (NOF_CCE reaches 96 at 110 PRB)


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "pdcch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def _case(z, c):
    y = [z["%s_y%d" % (c["key"], a)] for a in range(c["nrx"])]
    h = [[z["%s_h%d%d" % (c["key"], p, a)] for a in range(c["nrx"])] for p in range(c["nports"])]
    return y, h


def test_golden_cell_maps(gold):
    z, man = gold
    assert len(man["maps"]) >= 100
    for m in man["maps"]:
        idx, ncce = s.pdcch_cell_map(m["nof_prb"], m["cell_id"], m["nports"], m["phich_len"], m["phich_res"],
                                     m["cfi"])
        assert ncce == m["nof_cce"] and (idx == z[m["key"]]).all(), m


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_cell_maps_vs_reference():
    ref = Ref()
    rng = np.random.default_rng(11)
    for nof_prb in (6, 7, 9, 10, 11, 12, 15, 19, 20, 25, 26, 27, 39, 44, 45, 49, 50, 52, 63, 64, 75, 79, 80, 100,
                    110):
        for _ in range(3):
            cell_id, nports = int(rng.integers(0, 504)), int(rng.integers(1, 3))
            pl, pr = int(rng.integers(0, 2)), int(rng.integers(0, 4))
            for cfi in (1, 2, 3):
                a = s.pdcch_cell_map(nof_prb, cell_id, nports, pl, pr, cfi)
                b = pdcch_map(ref, nof_prb, cell_id, nports, pl, pr, cfi, ref=True)
                assert a[1] == b[1] and (a[0] == b[0]).all(), (nof_prb, cell_id, nports, pl, pr, cfi)


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_locations_vs_reference():
    ref = Ref()
    rng = np.random.default_rng(3)
    for nof_cce in list(range(0, 30)) + [41, 43, 62, 84, 87]:
        assert s.pdcch_locations(nof_cce, common=True) == pdcch_locations(ref, nof_cce, 0, 0, True)
        for sf in range(10):
            rnti = int(rng.integers(1, 0x10000))
            assert s.pdcch_locations(nof_cce, sf, rnti) == pdcch_locations(ref, nof_cce, sf, rnti, False)


def test_golden_search_spaces_cover_the_cases(gold):
    """the fixture exercises C-, SI- and RA-RNTI finds, misses, and every UE format family"""
    _, man = gold
    res = [r for c in man["cases"] for r in c["searches"]]
    found = [r for r in res if r["found"]]
    assert len(found) >= 60 and len(res) - len(found) >= 60
    fmts = {r["format"] for r in found}
    assert fmts >= {1, 2, 3} and len(fmts & {4, 5, 6, 7, 8}) >= 3
    assert any(r["rnti"] == 0xFFFF for r in found) and any(r["rnti"] <= 10 for r in found)
    assert sum(r["found"] < 0 for r in res) >= 4  # searches the reference ends with SRSLTE_ERROR


@pytest.mark.parametrize("nof_prb,cell_id,nports,nrx,pl,pr", [(5, 0, 1, 1, 0, 0), (111, 0, 1, 1, 0, 0),
                                                             (6, 504, 1, 1, 0, 0), (6, 0, 3, 1, 0, 0),
                                                             (6, 0, 1, 3, 0, 0), (6, 0, 1, 1, 2, 0),
                                                             (6, 0, 1, 1, 0, 4)])
def test_create_rejects_invalid_cells(nof_prb, cell_id, nports, nrx, pl, pr):
    """srsgpu_pdcch_create validates the cell before touching the device (runs without a GPU)"""
    with pytest.raises(RuntimeError):
        s.Pdcch(nof_prb, cell_id, nports, nrx, pl, pr)


# ------------------------------------------------------------------------------------ GPU ----
class _Dev:
    """subframes of one cell on the device, laid out as the PDSCH path's grids: [sf][rx] grid planes,
    [sf][rx][port] estimate planes, 14 * 12 nof_prb complex each; LLRs at LLR_STRIDE floats per subframe"""

    def __init__(self, torch, nof_prb, nports, nrx, subframes):
        self.torch = torch
        self.stride = 14 * 12 * nof_prb
        ns = len(subframes)
        grid = np.zeros((ns, nrx, self.stride), np.complex64)
        ce = np.zeros((ns, nrx * nports, self.stride), np.complex64)
        for i, (y, h) in enumerate(subframes):
            for a in range(nrx):
                grid[i, a, :y[a].size] = y[a]
                for p in range(nports):
                    ce[i, a * nports + p, :h[p][a].size] = h[p][a]
        self.g = torch.from_numpy(grid.view(np.float32)).cuda()
        self.c = torch.from_numpy(ce.view(np.float32)).cuda()
        self.llr = torch.full((ns * LLR_STRIDE,), float("nan"), dtype=torch.float32, device="cuda")
        self.nrx, self.nports = nrx, nports

    def sf(self, i, sf_idx, cfi, noise):
        return (i * self.nrx * self.stride, i * self.nrx * self.nports * self.stride, i * LLR_STRIDE, sf_idx, cfi, noise)


def _search_gpu(torch, q, searches, d_llr):
    """searches: [(llr_offset, sf_idx, cfi, rnti, tm, rnti_type, ul_rnti)] -> [(dl, ul)] parsed results"""
    res = torch.zeros(len(searches) * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    ul = torch.zeros(len(searches) * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    assert q.find_dci_dev(searches, d_llr, res.data_ptr(), ul.data_ptr()) == 0
    torch.cuda.synchronize()
    return list(zip(s.Pdcch.parse_results(res.cpu().numpy().tobytes()),
                    s.Pdcch.parse_results(ul.cpu().numpy().tobytes())))


def _ul_want(r, z, key, j):
    return dict(found=r["ul_found"], format=r["ul_format"], L=r["ul_L"], ncce=r["ul_ncce"], nof_bits=r["ul_nof_bits"],
                bits=z["%s_s%d_ulbits" % (key, j)])


def _check_ul_grant(got, r, nof_prb, what):
    """a found UL DCI unpacked as phch_worker does (srslte_dci_msg_to_ul_grant, hopping offset 0)"""
    ret, d, g = s.dci_msg_to_ul_grant(got[4], nof_prb, 0, r["ul_nof_bits"])
    assert ret == r["ul_grant_ret"] and d.fields11() == r["ul_dci"], what
    assert ret or g.fields10() == r["ul_grant"], what


def _same_result(got, want, what):
    found, fmt, L, ncce, buf = got
    assert found == want["found"], what
    if found > 0:
        nb = want["nof_bits"]
        assert (fmt, L, ncce) == (want["format"], want["L"], want["ncce"]), (what, got[:4], want)
        assert (buf[:nb + 16] == want["bits"][:nb + 16]).all() and not buf[nb + 16:].any(), what


@pytest.mark.gpu
def test_gpu_golden_subframes(gold):
    """every golden subframe: LLRs bit-exact, every search's result identical, and the found messages
    unpacked to the reference's grants"""
    import torch
    z, man = gold
    grants = {(g["format"], g["rnti"], g["nof_prb"], g["nports"], z[g["key"] + "_bits"].tobytes()): g
              for g in man["grants"]}
    nfound = nul = 0
    for c in man["cases"]:
        if c["group"] == "batch":
            continue
        y, h = _case(z, c)
        q = s.Pdcch(c["nof_prb"], c["cell_id"], c["nports"], c["nrx"], c["phich_len"], c["phich_res"])
        dev = _Dev(torch, c["nof_prb"], c["nports"], c["nrx"], [(y, h)])
        torch.cuda.synchronize()
        assert q.extract_llr_dev([dev.sf(0, c["sf_idx"], c["cfi"], c["noise"])], dev.g.data_ptr(),
                                 dev.c.data_ptr(), dev.stride, dev.llr.data_ptr()) == 0
        torch.cuda.synchronize()
        want = z[c["key"] + "_llr"]
        got = dev.llr[:want.size].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), c["key"]
        assert torch.isnan(dev.llr[want.size:]).all()  # nothing written past NOF_CCE(cfi)
        srch = [(0, c["sf_idx"], c["cfi"], r["rnti"], r["tm"], r["rnti_type"], r["ul_rnti"]) for r in c["searches"]]
        res = _search_gpu(torch, q, srch, dev.llr.data_ptr())
        for j, (r, (got, gul)) in enumerate(zip(c["searches"], res)):
            want = dict(r, bits=z["%s_s%d_bits" % (c["key"], j)])
            _same_result(got, want, (c["key"], j))
            _same_result(gul, _ul_want(r, z, c["key"], j), (c["key"], j, "UL"))
            if gul[0] > 0:
                nul += 1
                _check_ul_grant(gul, r, c["nof_prb"], (c["key"], j))
            if got[0] > 0:
                nfound += 1
                g = grants[(r["format"], r["rnti"], c["nof_prb"], c["nports"], want["bits"].tobytes())]
                ret, d, gr = s.dci_msg_to_dl_grant(got[4], got[1], r["rnti"], c["nof_prb"], c["nports"],
                                                   r["nof_bits"])
                assert ret == g["ret"] and (ret or d.fields30() == g["dci"]), (c["key"], j)
    assert nfound >= 50 and nul >= 25


@pytest.mark.gpu
def test_gpu_golden_batch(gold):
    """the batch group (one 2x2 cell, subframes of mixed CFI and subframe index) in one extraction
    launch and one search call over all subframes' searches"""
    import torch
    z, man = gold
    cs = [c for c in man["cases"] if c["group"] == "batch"]
    assert len(cs) >= 6
    c0 = cs[0]
    q = s.Pdcch(c0["nof_prb"], c0["cell_id"], c0["nports"], c0["nrx"], c0["phich_len"], c0["phich_res"])
    dev = _Dev(torch, c0["nof_prb"], c0["nports"], c0["nrx"], [_case(z, c) for c in cs])
    torch.cuda.synchronize()
    sfs = [dev.sf(i, c["sf_idx"], c["cfi"], c["noise"]) for i, c in enumerate(cs)]
    assert q.extract_llr_dev(sfs, dev.g.data_ptr(), dev.c.data_ptr(), dev.stride, dev.llr.data_ptr()) == 0
    srch, want = [], []
    for i, c in enumerate(cs):
        for j, r in enumerate(c["searches"]):
            srch.append((i * LLR_STRIDE, c["sf_idx"], c["cfi"], r["rnti"], r["tm"], r["rnti_type"], r["ul_rnti"]))
            want.append((dict(r, bits=z["%s_s%d_bits" % (c["key"], j)]), _ul_want(r, z, c["key"], j), (c["key"], j)))
    res = _search_gpu(torch, q, srch, dev.llr.data_ptr())
    llr = dev.llr.cpu().numpy()
    for i, c in enumerate(cs):
        w = z[c["key"] + "_llr"]
        assert np.array_equal(llr[i * LLR_STRIDE:i * LLR_STRIDE + w.size].view(np.uint32), w.view(np.uint32)), c["key"]
    for (got, gul), (w, wu, what) in zip(res, want):
        _same_result(got, w, what)
        _same_result(gul, wu, what + ("UL",))


@pytest.mark.gpu
@pytest.mark.skipif(not (have_ref() and have_ref_front()), reason="oracle/_ref not built")
@pytest.mark.parametrize("nof_prb,nports,nrx", [(6, 1, 1), (9, 2, 2), (10, 1, 2), (15, 2, 1), (25, 1, 2), (50, 2, 2), (75, 1, 1),
                                                (100, 2, 2), (110, 2, 1), (25, 4, 2), (100, 4, 1)])
def test_gpu_random_vs_reference(nof_prb, nports, nrx):
    """random cells and subframes generated live with the reference's encoder; 40 subframes in one launch,
    back-to-back extraction / search calls on one stream with no host sync in between"""
    import torch
    ref = Ref()
    rng = np.random.default_rng(nof_prb * 10 + nports + nrx)
    cell_id, pl, pr = int(rng.integers(0, 504)), int(rng.integers(0, 2)), int(rng.integers(0, 4))
    q = s.Pdcch(nof_prb, cell_id, nports, nrx, pl, pr)
    subs, meta = [], []
    for i in range(40):
        cfi, sf_idx, tm = int(rng.integers(1, 4)), i % 10, int(rng.integers(0, 8))
        y, h, searches, noise = pdcch_subframe(ref, rng, nof_prb, cell_id, nports, nrx, pl, pr, cfi, sf_idx, tm,
                                               snr_db=float(rng.choice([3.0, 10.0, 40.0])))
        subs.append((y, h))
        meta.append((cfi, sf_idx, noise, searches, y, h))
    dev = _Dev(torch, nof_prb, nports, nrx, subs)
    torch.cuda.synchronize()
    # two extraction calls and two search calls back to back (the double-buffered descriptor uploads)
    half = 20
    results = []
    for lo, hi in ((0, half), (half, 40)):
        sfs = [dev.sf(i, meta[i][1], meta[i][0], meta[i][2]) for i in range(lo, hi)]
        assert q.extract_llr_dev(sfs, dev.g.data_ptr(), dev.c.data_ptr(), dev.stride, dev.llr.data_ptr()) == 0
    bufs = []
    for lo, hi in ((0, half), (half, 40)):
        srch = [(i * LLR_STRIDE, meta[i][1], meta[i][0], r, t, rt, u) for i in range(lo, hi)
                for (r, t, rt, u) in meta[i][3]]
        res = torch.zeros(len(srch) * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
        rul = torch.zeros(len(srch) * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
        assert q.find_dci_dev(srch, dev.llr.data_ptr(), res.data_ptr(), rul.data_ptr()) == 0
        bufs.append((srch, res, rul))
    torch.cuda.synchronize()
    for srch, res, rul in bufs:
        results += list(zip(srch, s.Pdcch.parse_results(res.cpu().numpy().tobytes()),
                            s.Pdcch.parse_results(rul.cpu().numpy().tobytes())))
    llr = dev.llr.cpu().numpy()
    nfound = nul = 0
    k = 0
    for i, (cfi, sf_idx, noise, searches, y, h) in enumerate(meta):
        w, found = find_dci_ref(nof_prb, cell_id, nports, nrx, pl, pr, cfi, sf_idx, noise, y, h, searches)
        assert np.array_equal(llr[i * LLR_STRIDE:i * LLR_STRIDE + w.size].view(np.uint32), w.view(np.uint32)), i
        for (rnti, tm, rt, ur), (dl, ul, ulg) in zip(searches, found):
            f, fmt, L, ncce, nb, buf = dl
            _same_result(results[k][1], dict(found=f, format=fmt, L=L, ncce=ncce, nof_bits=nb, bits=buf), (i, rnti))
            _same_result(results[k][2], dict(found=ul[0], format=ul[1], L=ul[2], ncce=ul[3], nof_bits=ul[4],
                                             bits=ul[5]), (i, rnti, "UL"))
            if ul[0] > 0:
                nul += 1
                a = s.dci_msg_to_ul_grant(ul[5], nof_prb, 0, ul[4])
                assert a[0] == ulg[0] and a[1].fields11() == list(ulg[1]), (i, ur)
            if f > 0:
                nfound += 1
                a = s.dci_msg_to_dl_grant(buf, fmt, rnti, nof_prb, nports, nb)
                b = dci_to_dl_grant_ref(ref, buf, fmt, rnti, nof_prb, nports, nof_bits=nb)
                assert a[0] == b[0] and (a[0] or a[1].fields30() == list(b[1])), (i, rnti)
            k += 1
    assert nfound >= 20 and nul >= 5


@pytest.mark.gpu
def test_gpu_invalid_requests():
    import torch
    q = s.Pdcch(25, 1, 1, 1)
    buf = torch.zeros(1 << 20, dtype=torch.float32, device="cuda")
    p = buf.data_ptr()
    stride = 14 * 12 * 25
    assert q.extract_llr_dev([(0, 0, 0, 10, 1, 0.0)], p, p, stride, p) == -1   # sf_idx > 9
    assert q.extract_llr_dev([(0, 0, 0, 1, 4, 0.0)], p, p, stride, p) == -1    # cfi 4
    assert q.extract_llr_dev([(0, 0, 1, 1, 1, 0.0)], p, p, stride, p) == -1    # odd llr offset
    assert q.extract_llr_dev([(0, 0, 0, 1, 1, 0.0)], p, p, stride - 1, p) == -1
    assert q.extract_llr_dev([], p, p, stride, p) == 0
    res = torch.zeros(4 * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    for bad in [(0, 0, 1, 0, 0), (0, 0, 0, 0x1234, 0), (0, 10, 1, 0x1234, 0), (0, 0, 1, 0x1234, 8),
                (0, 0, 1, 0x1234, 0, 7)]:
        assert q.find_dl_dci_dev([bad], p, res.data_ptr()) == -1, bad
    assert q.find_dl_dci_dev([], p, res.data_ptr()) == 0
    ul = torch.zeros(4 * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    assert q.find_dci_dev([(0, 0, 1, 0, 0, -1, 0)], p, res.data_ptr(), ul.data_ptr()) == -1  # no search at all
    assert q.find_dci_dev([(0, 0, 1, 0x1234, 0, -1, 0x10000)], p, res.data_ptr(), ul.data_ptr()) == -1
    # a UL search alone: the DL result reports the reference's "RNTI not specified" error
    p0 = torch.zeros(72 * 128, dtype=torch.float32, device="cuda")
    got = _search_gpu(torch, q, [(0, 3, 2, 0, 0, -1, 0x4321)], p0.data_ptr())
    assert got[0][0][0] == -1 and got[0][1][0] == 0
    torch.cuda.synchronize()
