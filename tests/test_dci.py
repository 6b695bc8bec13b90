"""DCI handling on the host (include/srsgpu/dci.h, the step between the PDCCH blind search and the
PDSCH decode): srsgpu_dci_format_sizeof, srsgpu_dci_msg_to_dl_grant and the 36.213 TBS tables against
golden unpackings recorded from the reference (tests/golden/make_pdcch_golden.py:
srslte_dci_msg_to_dl_grant, dci.c:49-90 with ra.c) and, with oracle/_ref, against the reference build
on random packed and random-bit messages. Pure host code: runs without a GPU."""
import json
import os

import numpy as np
import pytest

import srsgpu_phy as s
from srsgpu_testlib import (F1, F1A, F1B, F1C, F1D, F2, F2A, F2B, Ref, dci_sizeof_ref, dci_to_dl_grant_ref,
                            have_ref, random_dl_msg)

HERE = os.path.dirname(os.path.abspath(__file__))
DL_FORMATS = (F1, F1A, F1C, F1B, F1D, F2, F2A, F2B)


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "pdcch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def _check(bits, fmt, rnti, nof_prb, nports, ret, dci, grant, prb, what, nof_bits=None):
    r, d, g = s.dci_msg_to_dl_grant(bits, fmt, rnti, nof_prb, nports, nof_bits)
    assert r == ret, (what, r, ret)
    if ret != 0:
        return
    assert d.fields30() == list(dci), (what, d.fields30(), list(dci))
    if dci[25]:  # a random-access order carries no grant (dci.c:58-62)
        return
    assert g.fields13() == list(grant), (what, g.fields13(), list(grant))
    assert (np.frombuffer(bytes(g.prb_idx), np.uint8).reshape(2, 110) == prb).all(), what


def test_golden_grants(gold):
    z, man = gold
    gs = man["grants"]
    assert len(gs) >= 400 and sum(g["ret"] == 0 for g in gs) >= 300
    assert {g["format"] for g in gs if g["ret"] == 0} >= {F1, F1A, F1C, F1B, F1D, F2, F2A, F2B}
    for g in gs:
        _check(z[g["key"] + "_bits"], g["format"], g["rnti"], g["nof_prb"], g["nports"], g["ret"], g["dci"],
               g["grant"], z[g["key"] + "_prb"], g["key"], g["nof_bits"])


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_sizeof_vs_reference():
    ref = Ref()
    for nof_prb in list(range(6, 111, 1)):
        for nports in (1, 2, 4):
            for fmt in (0,) + DL_FORMATS:
                assert s.dci_format_sizeof(fmt, nof_prb, nports) == dci_sizeof_ref(ref, fmt, nof_prb, nports), \
                    (fmt, nof_prb, nports)


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_tbs_tables_vs_reference():
    ref = Ref()
    import ctypes
    f = ref.lib.ref_tbs_from_idx
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    g = ref.lib.ref_tbs_idx_from_mcs
    g.argtypes = [ctypes.c_uint32]
    for idx in range(0, 28):
        for nprb in (0, 1, 2, 50, 110, 111):
            assert s._lib.srsgpu_ra_tbs_from_idx(idx, nprb) == f(idx, nprb), (idx, nprb)
    for mcs in range(0, 33):
        assert s._lib.srsgpu_ra_tbs_idx_from_mcs(mcs) == g(mcs), mcs


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
@pytest.mark.parametrize("nof_prb", [6, 7, 15, 25, 27, 50, 64, 75, 100, 110])
def test_random_messages_vs_reference(nof_prb):
    """packed messages of every format the reference packs, and random bits of every DL format's size
    (invalid allocations, MCS 29-31, RA orders, 2A/2B swap and disabled blocks), under C-, SI-, P- and
    RA-RNTIs"""
    ref = Ref()
    rng = np.random.default_rng(nof_prb)
    n = 0
    for nports in (1, 2):
        for fmt in DL_FORMATS:
            for k in range(24):
                rnti = [0x1234, 0xFFFF, 0xFFFE, 0x0001, 0x000A, 0x000B, 0xFFF3][k % 7]
                crnti = rnti >= 0x000B and rnti <= 0xFFF3
                bits = (random_dl_msg(ref, rng, fmt, nof_prb, nports, crc_is_crnti=crnti) if k % 2 else
                        rng.integers(0, 2, dci_sizeof_ref(ref, fmt, nof_prb, nports)).astype(np.uint8))
                ret, d, g, p = dci_to_dl_grant_ref(ref, bits, fmt, rnti, nof_prb, nports)
                _check(bits, fmt, rnti, nof_prb, nports, ret, d, g, p, (fmt, nports, k))
                n += ret == 0
    assert n > 100


def _check_ul(bits, nof_prb, n_rb_ho, ret, dci, grant, what, nof_bits=None):
    r, d, g = s.dci_msg_to_ul_grant(bits, nof_prb, n_rb_ho, nof_bits)
    assert r == ret, (what, r, ret)
    assert d.fields11() == list(dci), (what, d.fields11(), list(dci))
    if ret == 0:
        assert g.fields10() == list(grant), (what, g.fields10(), list(grant))


def test_golden_ul_grants(gold):
    """srsgpu_dci_msg_to_ul_grant against the reference's srslte_dci_msg_to_ul_grant (dci.c:165-197):
    format 0 messages the reference packed and the UL DCIs its ue_dl.c search found, with and without a
    PUSCH hopping offset"""
    z, man = gold
    gs = man["ul_grants"]
    assert len(gs) >= 150 and sum(g["ret"] == 0 for g in gs) >= 100
    assert {g["dci"][0] for g in gs} >= {-1, 0, 1, 2, 3}  # every hopping kind
    for g in gs:
        _check_ul(z[g["key"] + "_bits"], g["nof_prb"], g["n_rb_ho"], g["ret"], g["dci"], g["grant"], g["key"])
    # the grants of the UL searches of the recorded subframes (as ue_dl.c's caller unpacks them)
    n = 0
    for c in man["cases"]:
        for j, r in enumerate(c["searches"]):
            if r["ul_found"] > 0:
                b = z["%s_s%d_ulbits" % (c["key"], j)][:r["ul_nof_bits"]]
                _check_ul(b, c["nof_prb"], 0, r["ul_grant_ret"], r["ul_dci"], r["ul_grant"], (c["key"], j))
                n += 1
    assert n >= 30


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_ul_grants_vs_reference():
    """random reference-packed and random-bit format 0 messages of every bandwidth and hopping offset"""
    from srsgpu_testlib import dci_to_ul_grant_ref, random_ul_msg
    ref = Ref()
    rng = np.random.default_rng(5)
    for nof_prb in list(range(6, 111, 7)) + [100, 110]:
        for k in range(8):
            if k < 5:
                b = random_ul_msg(ref, rng, nof_prb)
            else:
                b = rng.integers(0, 2, s.dci_format_sizeof(0, nof_prb, 1)).astype(np.uint8)
                b[0] = int(k == 7)  # a 1A look-alike is refused
            for n_rb_ho in (0, 3, int(rng.integers(0, nof_prb // 2 + 1))):
                r, d, g = dci_to_ul_grant_ref(ref, b, nof_prb, n_rb_ho)
                _check_ul(b, nof_prb, n_rb_ho, r, d, g, (nof_prb, k, n_rb_ho))
    # wrong length: refused
    r, _, _ = s.dci_msg_to_ul_grant(np.zeros(10, np.uint8), 50)
    assert r == -1
