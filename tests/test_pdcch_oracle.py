"""The PDCCH oracle (oracle/pdcch_oracle.c: REG map, LLR extraction, candidate locations, the DL blind
search and the UL (format 0) search after it, restated in scalar C) against the golden receptions recorded
from the reference build and its own ue_dl.c (tests/golden/make_pdcch_golden.py, oracle/_ref/ref_front)
and, with oracle/_ref, against the reference on random cells and subframes. CPU only: this pins the
checker the GPU tests can fall back on."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import (Ref, find_dci, find_dci_ref, have_ref, have_ref_front, pdcch_llr, pdcch_locations,
                            pdcch_map, pdcch_subframe)

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "pdcch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_maps(oracle, gold):
    z, man = gold
    for m in man["maps"]:
        idx, ncce = pdcch_map(oracle, m["nof_prb"], m["cell_id"], m["nports"], m["phich_len"], m["phich_res"],
                              m["cfi"])
        assert ncce == m["nof_cce"] and np.array_equal(idx, z[m["key"]]), m


def test_golden_llrs_and_searches(oracle, gold):
    z, man = gold
    nfound = nref = nul = 0
    for c in man["cases"]:
        y = [z["%s_y%d" % (c["key"], a)] for a in range(c["nrx"])]
        h = [[z["%s_h%d%d" % (c["key"], p, a)] for a in range(c["nrx"])] for p in range(c["nports"])]
        args = (c["nof_prb"], c["cell_id"], c["nports"], c["phich_len"], c["phich_res"])
        llr = pdcch_llr(oracle, *args, c["nrx"], c["cfi"], c["sf_idx"], c["noise"], y, h)
        want = z[c["key"] + "_llr"]
        assert np.array_equal(llr.view(np.uint32), want.view(np.uint32)), c["key"]
        for j, r in enumerate(c["searches"]):
            dl, ul = find_dci(oracle, *args, c["cfi"], c["sf_idx"], llr, r["rnti"], r["tm"], r["rnti_type"],
                              r["ul_rnti"])
            f, fmt, L, ncce, nb, buf = dl
            assert f == r["found"], (c["key"], j)
            if f > 0:
                nfound += 1
                assert (fmt, L, ncce, nb) == (r["format"], r["L"], r["ncce"], r["nof_bits"]), (c["key"], j)
                # the payload and CRC bits; past them the reference's buffer holds earlier candidates' bits
                assert np.array_equal(buf[:nb + 16], z["%s_s%d_bits" % (c["key"], j)][:nb + 16]), (c["key"], j)
            nref += f < 0
            f, fmt, L, ncce, nb, buf = ul
            assert f == r["ul_found"], (c["key"], j, "UL")
            if f > 0:
                nul += 1
                assert (fmt, L, ncce, nb) == (r["ul_format"], r["ul_L"], r["ul_ncce"], r["ul_nof_bits"]), (c["key"], j)
                assert np.array_equal(buf[:nb + 16], z["%s_s%d_ulbits" % (c["key"], j)][:nb + 16]), (c["key"], j)
    assert nfound >= 60 and nref >= 4 and nul >= 30


@pytest.mark.skipif(not (have_ref() and have_ref_front()), reason="oracle/_ref not built")
def test_random_vs_reference(oracle):
    ref = Ref()
    rng = np.random.default_rng(77)
    for nof_prb, nports, nrx in ((6, 2, 2), (10, 1, 1), (11, 1, 2), (27, 2, 1), (63, 1, 1), (80, 2, 2),
                                 (110, 1, 2)):
        cell_id, pl, pr = int(rng.integers(0, 504)), int(rng.integers(0, 2)), int(rng.integers(0, 4))
        for cfi in (1, 2, 3):
            a = pdcch_map(oracle, nof_prb, cell_id, nports, pl, pr, cfi)
            b = pdcch_map(ref, nof_prb, cell_id, nports, pl, pr, cfi, ref=True)
            assert a[1] == b[1] and np.array_equal(a[0], b[0])
            assert pdcch_locations(oracle, a[1], 0, 0, True, ref=False) == pdcch_locations(ref, a[1], 0, 0, True)
            for sf in range(10):
                rnti = int(rng.integers(1, 0x10000))
                assert (pdcch_locations(oracle, a[1], sf, rnti, False, ref=False)
                        == pdcch_locations(ref, a[1], sf, rnti, False))
        for k in range(6):
            cfi, sf, tm = int(rng.integers(1, 4)), int(rng.integers(0, 10)), int(rng.integers(0, 8))
            y, h, searches, noise = pdcch_subframe(ref, rng, nof_prb, cell_id, nports, nrx, pl, pr, cfi, sf, tm,
                                                   snr_db=float(rng.choice([4.0, 15.0])))
            args = (nof_prb, cell_id, nports, pl, pr)
            la = pdcch_llr(oracle, *args, nrx, cfi, sf, noise, y, h)
            lb, found = find_dci_ref(nof_prb, cell_id, nports, nrx, pl, pr, cfi, sf, noise, y, h, searches)
            assert np.array_equal(la.view(np.uint32), lb.view(np.uint32)), (nof_prb, k)
            for (rnti, t, rt, ur), (rdl, rul, _) in zip(searches, found):
                for got, want in zip(find_dci(oracle, *args, cfi, sf, la, rnti, t, rt, ur), (rdl, rul)):
                    nb = got[4]
                    assert got[:5] == want[:5] and np.array_equal(got[5][:nb + 16], want[5][:nb + 16]), \
                        (nof_prb, k, rnti, ur)
