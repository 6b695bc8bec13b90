"""CPU checks of the PDSCH front-end oracle (oracle/pdsch_oracle.c): RE extraction maps, the SISO
equaliser (bit-exact without CSI; with CSI within the reference's rcpps error), the int16 soft
demapper and PDSCH scrambling, against golden vectors recorded from the srsLTE reference and,
where oracle/_ref exists, against the reference on random cases."""
import ctypes
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import PdschOracle, Ref, have_ref, ref_pdsch

HERE = os.path.dirname(os.path.abspath(__file__))
f32 = ctypes.POINTER(ctypes.c_float)
u8 = ctypes.POINTER(ctypes.c_uint8)
i16 = ctypes.POINTER(ctypes.c_int16)


@pytest.fixture(scope="module")
def po(oracle):
    return PdschOracle(oracle)


@pytest.fixture(scope="module")
def pgold():
    z = np.load(os.path.join(HERE, "golden", "pdsch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_re_maps(po, pgold):
    z, man = pgold
    for c in (c for c in man if c["kind"] == "map"):
        idx = po.re_map(c["nof_prb"], c["cell_id"], c["ports"], c["lstart"], c["sf_idx"],
                        z[c["key"] + "_mask"])
        assert (idx == z[c["key"] + "_idx"]).all(), c["key"]


def test_golden_equaliser(po, pgold):
    z, man = pgold
    for c in (c for c in man if c["kind"] == "eq"):
        y, h, x = z[c["key"] + "_y"], z[c["key"] + "_h"], z[c["key"] + "_x"]
        if c["csi"]:
            xo, co = po.predecode(y, h, 1.0, c["noise"], True)
            assert (co == z[c["key"] + "_csi"]).all()
            # the reference multiplies by _mm256_rcp_ps (12-bit): 1e-3 relative
            assert np.max(np.abs(xo - x) / np.maximum(np.abs(x), 1e-6)) < 1e-3
        else:
            assert (po.predecode(y, h, 1.0, c["noise"]) == x).all(), c["key"]


def test_golden_demapper(po, pgold):
    z, man = pgold
    for c in (c for c in man if c["kind"] == "demod"):
        assert (po.demod(c["mod"], z[c["key"] + "_sym"]) == z[c["key"] + "_llr"]).all(), c["key"]


def test_golden_scrambling(po, pgold):
    z, man = pgold
    for c in (c for c in man if c["kind"] == "scramble"):
        seed = po.seed(c["rnti"], c["q"], c["nslot"], c["cell_id"])
        assert (po.scramble(seed, z[c["key"] + "_in"]) == z[c["key"] + "_out"]).all()


needs_ref = pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (build container only)")


@needs_ref
def test_re_maps_vs_reference(po):
    L = ref_pdsch(Ref())
    rng = np.random.default_rng(1)
    for nprb in (6, 15, 25, 50, 75, 100):
        for ports in (1, 2, 4):
            for sf in (0, 1, 5):
                for lstart in (1, 2, 3, 4):
                    cid = int(rng.integers(504))
                    mask = (rng.random((2, nprb)) < 0.6).astype(np.uint8)
                    idx = po.re_map(nprb, cid, ports, lstart, sf, mask)
                    grid = np.zeros(nprb * 12 * 14, np.complex64)
                    grid.real = np.arange(grid.size)
                    out = np.zeros(grid.size, np.complex64)
                    n = L.ref_pdsch_get(nprb, cid, ports, lstart, sf, mask.ctypes.data_as(u8),
                                        grid.ctypes.data_as(f32), out.ctypes.data_as(f32))
                    assert n == idx.size and (out[:n].real.astype(np.uint32) == idx).all()


@needs_ref
def test_equaliser_and_demapper_vs_reference(po):
    L = ref_pdsch(Ref())
    rng = np.random.default_rng(2)
    for n in (1, 7, 16, 17, 33, 1000, 15000, 15007):
        y = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        h = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        for noise in (0.0, 0.1):
            x = np.zeros_like(y)
            L.ref_predecode_single(y.ctypes.data_as(f32), h.ctypes.data_as(f32),
                                   x.ctypes.data_as(f32), None, n, 1.0, noise)
            assert (po.predecode(y, h, 1.0, noise) == x).all(), (n, noise)
        for mod, bps in ((0, 1), (1, 2), (2, 4), (3, 6)):
            for sc in (0.5, 2.0, 90.0):
                s = (x * sc).astype(np.complex64)
                llr = np.zeros(n * bps, np.int16)
                L.ref_demod_s(mod, s.ctypes.data_as(f32), n, llr.ctypes.data_as(i16))
                assert (po.demod(mod, s) == llr).all(), (n, mod, sc)


@needs_ref
def test_cdd_equaliser_vs_reference(po):
    """TM3 CDD 2x2 MMSE (precoding.c:930-1072). The reference's C tail (the last n % 8 REs) is
    the oracle's formula and must agree bit for bit; its AVX body uses rcpps and must agree to
    the rcpps tolerance (<= 1e-3 relative)."""
    from srsgpu_testlib import ref_predecode_ccd
    L = ref_pdsch(Ref())
    rng = np.random.default_rng(5)
    for n in (2, 6, 8, 14, 1000, 14406):
        y = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(2)]
        h = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
              for _ in range(2)] for _ in range(2)]
        for noise, scaling, csi in ((0.1, 1.0, False), (0.01, 0.8, True), (0.5, 1.0, True)):
            got = po.predecode_ccd(y, h, scaling, noise, csi)
            ref = ref_predecode_ccd(L, y, h, scaling, noise, csi)
            xg, xr = (got[0], ref[0]) if csi else (got, ref)
            tail = 8 * (n // 8)
            for lay in (0, 1):
                assert (xg[lay][tail:] == xr[lay][tail:]).all(), (n, lay)
                scale = np.abs(xr[lay][:tail]) + 1.0
                assert (np.abs(xg[lay][:tail] - xr[lay][:tail]) / scale).max(initial=0) < 1e-3, (n, lay)
                if csi:
                    cg, cr = got[1][lay], ref[1][lay]
                    assert (cg[tail:] == cr[tail:]).all()
                    assert (np.abs(cg[:tail] - cr[:tail]) / np.abs(cr[:tail])).max(initial=0) < 2e-3
