"""TM4 closed-loop spatial multiplexing (srslte_predecoding_multiplex, precoding.c:1715-1760, reached
from srslte_pdsch_decode with SRSLTE_MIMO_TYPE_SPATIAL_MULTIPLEX: 2 TBs on 2 layers through the 2x2
MMSE of codebook 0-2, or 1 TB on 1 layer through the 2x1 MRC of codebook 0-3).

CPU: the oracle restatement against the reference build — bit-exact where the reference runs its C
loops (fewer REs than one AVX vector, and every RE past the last whole vector), within the rcpps
tolerance on the AVX bodies (the reference's approximate reciprocal, model-dependent), with and
without CSI. GPU: the PDSCH LLRs of TM4 subframes (srsgpu_pdsch_llr_dev) equal the oracle chain
(predecode -> demap -> descramble) bit for bit, and full decodes of precoded codewords ack."""
import numpy as np
import pytest

from srsgpu_testlib import PdschOracle, Ref, have_ref

SIMD_CF = 8  # SRSLTE_SIMD_CF_SIZE of the AVX2 reference build


def _chan(rng, n):
    y = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(2)]
    h = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(2)]
         for _ in range(2)]
    return y, h


@pytest.mark.skipif(not have_ref(), reason="reference build (oracle/_ref) absent")
@pytest.mark.parametrize("layers,codebooks", [(2, (0, 1, 2)), (1, (0, 1, 2, 3))])
def test_oracle_vs_reference(oracle, layers, codebooks):
    po, ref = PdschOracle(oracle), Ref()
    rng = np.random.default_rng(40 + layers)
    for cb in codebooks:
        for csi in (False, True):
            for n, scaling, noise in [(7, 1.0, 0.05), (5, 0.8, 0.0), (203, 1.0, 0.1), (1200, 1.25, 0.02)]:
                y, h = _chan(rng, n)
                a = po.predecode_multiplex(y, h, cb, layers, scaling, noise, csi)
                b = po.predecode_multiplex(y, h, cb, layers, scaling, noise, csi, lib=ref)
                xa, xb = (a[0], b[0]) if csi else (a, b)
                tail = (n // SIMD_CF) * SIMD_CF
                for la in range(layers):
                    # C loop of the reference: bit-exact
                    assert (xa[la][tail:].view(np.uint32) == xb[la][tail:].view(np.uint32)).all(), (cb, n, la)
                    # AVX body (rcpps): relative tolerance
                    d = np.abs(xa[la][:tail] - xb[la][:tail]) / np.maximum(np.abs(xb[la][:tail]), 1e-3)
                    assert d.size == 0 or d.max() < 3e-3, (cb, n, la, d.max())
                if csi:
                    for la in range(layers):
                        ca, cb_ = a[1][la], b[1][la]
                        assert (ca[tail:].view(np.uint32) == cb_[tail:].view(np.uint32)).all(), (cb, n)
                        d = np.abs(ca[:tail] - cb_[:tail]) / np.maximum(np.abs(cb_[:tail]), 1e-3)
                        assert d.size == 0 or d.max() < 3e-3, (cb, n, d.max())


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id,layers,csi", [(100, 3, 2, False), (25, 101, 2, True), (50, 7, 1, False),
                                                        (15, 400, 1, True)])
def test_gpu_llr_vs_oracle(oracle, nof_prb, cell_id, layers, csi):
    """TM4 subframes (2 ports, 2 rx) through srsgpu_pdsch_llr_dev: every TB's LLRs equal the oracle
    chain (orc_predecode_multiplex -> demap -> descramble -> CSI) bit for bit, every codebook,
    codeword swap with two TBs"""
    import torch
    import srsgpu_phy as s
    po = PdschOracle(oracle)
    rng = np.random.default_rng(7 * nof_prb + cell_id + layers)
    size = nof_prb * 12 * 14
    n_sf = 8
    y = (rng.standard_normal((n_sf, 2, size)) + 1j * rng.standard_normal((n_sf, 2, size))).astype(np.complex64)
    h = (rng.standard_normal((n_sf, 2, 2, size)) + 1j * rng.standard_normal((n_sf, 2, 2, size))).astype(np.complex64)
    p = s.Pdsch(nof_prb, cell_id, nof_ports=2, nof_rx_ant=2, max_sf=n_sf)
    p.set_csi(csi)
    sfs, expect, offs, off = [], [], [], 0
    for i in range(n_sf):
        sf_idx = [0, 1, 5, 7][i % 4]
        lstart = 1 + i % 3
        cb = i % (3 if layers == 2 else 4)
        swap = (i // 2) % 2 if layers == 2 else 0
        mask = np.ones((2, nof_prb), np.uint8) if i % 2 == 0 else (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
        mods = ([3, 2], [1, 3], [2, 2])[i % 3]
        noise = 0.05 + 0.05 * (i % 2)
        rnti = int(rng.integers(1, 65535))
        idx = po.re_map(nof_prb, cell_id, 2, lstart, sf_idx, mask)
        tbs = (1000, 1000) if layers == 2 else (1000, 0)
        sf = s.make_sf(sf_idx=sf_idx, lstart=lstart, prb=mask, nof_prb=nof_prb, mod=mods if layers == 2 else mods[0],
                       nof_re=idx.size, rnti=rnti, noise=noise, grid_offset=i * 2 * size, ce_offset=i * 4 * size,
                       mimo=s.MIMO_SPATIAL_MULTIPLEX, tb_cw_swap=swap, tbs=tbs, codebook_idx=cb)
        assert p.nof_re(sf) == idx.size
        sfs.append(sf)
        hp = [[h[i, a, port][idx] for a in (0, 1)] for port in (0, 1)]
        xs = po.predecode_multiplex([y[i, 0][idx], y[i, 1][idx]], hp, cb, layers, 1.0, noise, csi)
        x, c = (xs if csi else (xs, None))
        for tb in range(layers):
            cw = tb ^ swap if layers == 2 else 0
            e = po.demod(mods[tb] if layers == 2 else mods[0], x[cw])
            e = po.scramble(po.seed(rnti, cw, 2 * sf_idx, cell_id), e)
            if csi:
                e = po.csi_correction(mods[tb] if layers == 2 else mods[0], c[cw], e)
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


@pytest.mark.gpu
def test_gpu_spatial_multiplexing_refusals():
    """spatial multiplexing needs 2 ports and 2 rx antennas and a codebook the reference accepts"""
    import torch
    import srsgpu_phy as s
    d = torch.zeros(25 * 12 * 14 * 4, dtype=torch.complex64, device="cuda")
    d_e = torch.zeros(100000, dtype=torch.int16, device="cuda")
    for nports, nrx, cb, tbs in [(2, 1, 0, (100, 100)), (1, 2, 0, (100, 100)), (2, 2, 3, (100, 100)),
                                 (2, 2, 4, (100, 0))]:
        p = s.Pdsch(25, 1, nof_ports=nports, nof_rx_ant=nrx, max_sf=1)
        sf = s.make_sf(sf_idx=1, lstart=1, nof_prb=25, mod=(1, 1), nof_re=1, mimo=s.MIMO_SPATIAL_MULTIPLEX,
                       tbs=tbs, codebook_idx=cb)
        assert p.llr_dev([sf], d.data_ptr(), d.data_ptr(), 25 * 12 * 14, d_e.data_ptr(), [0, 0]) == -1
        p.close()
