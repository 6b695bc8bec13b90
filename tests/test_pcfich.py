"""PCFICH decoding (§8(f) rank 1: the CFI detection srslte_pcfich_decode_multi runs on every
subframe before the PDCCH search, pcfich.c:178-241): the oracle restatement
(oracle/pdsch_oracle.c orc_pcfich_re_map / orc_pcfich_decode) against golden decodes recorded from
the reference (tests/golden/make_pcfich_golden.py) and, with oracle/_ref, random cases (CPU); the
batched GPU decoder (include/srsgpu/pcfich_batch.h) against both, bit-exact in the CFI and the
correlation value (GPU)."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import Ref, have_ref, pcfich_decode, pcfich_re_map

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "pcfich_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def _case(z, c):
    y = [z["%s_y%d" % (c["key"], a)] for a in range(c["nrx"])]
    h = [[z["%s_h%d%d" % (c["key"], p, a)] for a in range(c["nrx"])] for p in range(c["nports"])]
    return y, h


def test_golden_oracle(oracle, gold):
    z, man = gold
    assert len(man) == 72 + 24  # 24 of them with 4 CRS ports
    assert sum(c["cfi"] == c["sent_cfi"] for c in man) >= 60  # the fixture exercises real detection
    for c in man:
        assert (pcfich_re_map(oracle, c["nof_prb"], c["cell_id"]) == z[c["key"] + "_idx"]).all()
        y, h = _case(z, c)
        cfi, corr = pcfich_decode(oracle, c["nof_prb"], c["cell_id"], c["nports"], c["nrx"], y, h,
                                  c["noise"], c["sf_idx"])
        assert cfi == c["cfi"] and np.float32(corr) == np.float32(c["corr"]), c["key"]


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_random_vs_reference(oracle):
    ref = Ref()
    rng = np.random.default_rng(5)
    for nof_prb in (6, 25, 100):
        for cell_id in (0, 1, 2, 301, 503):
            assert (pcfich_re_map(oracle, nof_prb, cell_id) == pcfich_re_map(ref, nof_prb, cell_id, ref=True)).all()
            for nports in (1, 2, 4):
                for nrx in (1, 2):
                    n0 = nof_prb * 12
                    y = [(rng.standard_normal(n0) + 1j * rng.standard_normal(n0)).astype(np.complex64)
                         for _ in range(nrx)]
                    h = [[(rng.standard_normal(n0) + 1j * rng.standard_normal(n0)).astype(np.complex64)
                          for _ in range(nrx)] for _ in range(nports)]
                    sf, noise = int(rng.integers(0, 10)), float(rng.choice([0.0, 0.3]))
                    a = pcfich_decode(oracle, nof_prb, cell_id, nports, nrx, y, h, noise, sf)
                    b = pcfich_decode(ref, nof_prb, cell_id, nports, nrx, y, h, noise, sf, ref=True)
                    assert a[0] == b[0] and np.float32(a[1]) == np.float32(b[1])


def _gpu_decode(torch, s, nof_prb, cell_id, nports, nrx, subframes):
    """subframes: list of (y[a], h[p][a] symbol-0 arrays, noise, sf_idx) -> (cfi, corr) arrays"""
    n0, stride = nof_prb * 12, nof_prb * 12 * 14
    ns = len(subframes)
    grid = np.zeros((ns, nrx, stride), np.complex64)
    ce = np.zeros((ns, nrx * nports, stride), np.complex64)
    for i, (y, h, _, _) in enumerate(subframes):
        for a in range(nrx):
            grid[i, a, :n0] = y[a]
            for p in range(nports):
                ce[i, a * nports + p, :n0] = h[p][a]
    d_grid = torch.from_numpy(grid.view(np.float32)).cuda()
    d_ce = torch.from_numpy(ce.view(np.float32)).cuda()
    d_cfi = torch.zeros(ns, dtype=torch.int32, device="cuda")
    d_corr = torch.zeros(ns, dtype=torch.float32, device="cuda")
    q = s.Pcfich(nof_prb, cell_id, nports, nrx)
    sfs = [(i * nrx * stride, i * nrx * nports * stride, sf, noise) for i, (_, _, noise, sf) in enumerate(subframes)]
    torch.cuda.synchronize()
    assert q.decode_dev(sfs, d_grid.data_ptr(), d_ce.data_ptr(), stride, d_cfi.data_ptr(), d_corr.data_ptr()) == 0
    torch.cuda.synchronize()
    return q, d_cfi.cpu().numpy(), d_corr.cpu().numpy()


@pytest.mark.gpu
def test_gpu_golden(gold):
    import torch
    import srsgpu_phy as s
    z, man = gold
    for c in man:
        y, h = _case(z, c)
        q, cfi, corr = _gpu_decode(torch, s, c["nof_prb"], c["cell_id"], c["nports"], c["nrx"],
                                   [(y, h, c["noise"], c["sf_idx"])])
        assert (np.array(q.re_map(), np.uint32) == z[c["key"] + "_idx"]).all()
        assert cfi[0] == c["cfi"] and corr[0] == np.float32(c["corr"]), c["key"]


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id,nports,nrx", [(6, 11, 1, 1), (25, 200, 1, 2), (50, 7, 2, 1),
                                                        (100, 503, 2, 2)])
def test_gpu_batch_vs_oracle(oracle, nof_prb, cell_id, nports, nrx):
    """400 subframes in one launch (all ten subframe indices, mixed SNR and noise estimates)"""
    import torch
    import srsgpu_phy as s
    rng = np.random.default_rng(nof_prb + cell_id)
    n0 = nof_prb * 12
    subs = []
    for i in range(400):
        amp = float(rng.choice([0.1, 1.0, 10.0]))
        y = [(amp * (rng.standard_normal(n0) + 1j * rng.standard_normal(n0))).astype(np.complex64) for _ in range(nrx)]
        h = [[(rng.standard_normal(n0) + 1j * rng.standard_normal(n0)).astype(np.complex64) for _ in range(nrx)]
             for _ in range(nports)]
        if i % 50 == 0:  # a dead channel: the reference's 1e-4 guard (2 ports) / 0 + noise (1 port)
            for p in range(nports):
                for a in range(nrx):
                    h[p][a][:] = 0
        subs.append((y, h, float(rng.choice([0.0, 0.05, 1.0])), i % 10))
    _, cfi, corr = _gpu_decode(torch, s, nof_prb, cell_id, nports, nrx, subs)
    for i, (y, h, noise, sf) in enumerate(subs):
        w = pcfich_decode(oracle, nof_prb, cell_id, nports, nrx, y, h, noise, sf)
        if not np.isfinite(w[1]):
            assert not np.isfinite(corr[i]) or corr[i] == np.float32(w[1]), i
            continue
        assert cfi[i] == w[0] and corr[i] == np.float32(w[1]), (i, cfi[i], corr[i], w)


@pytest.mark.parametrize("nof_prb,cell_id,nports,nrx", [(5, 0, 1, 1), (111, 0, 1, 1), (6, 504, 1, 1),
                                                        (6, 0, 4, 1), (6, 0, 0, 1), (6, 0, 1, 3)])
def test_create_rejects_invalid_cells(nof_prb, cell_id, nports, nrx):
    """srsgpu_pcfich_create validates the cell before touching the device (runs without a GPU):
    the GPU path covers 6-110 PRB, N_ID 0-503, 1-2 ports, 1-2 rx antennas, and refuses the rest
    loudly instead of falling back"""
    import srsgpu_phy as s
    with pytest.raises(RuntimeError):
        s.Pcfich(nof_prb, cell_id, nports, nrx)


@pytest.mark.gpu
def test_gpu_back_to_back_calls_and_streams(oracle):
    """srsgpu_pcfich_decode_dev reuses its pinned descriptor buffer: several calls back to back with
    different descriptor contents and counts, no host sync in between, on one stream and then on a
    second stream (the call waits for the previous upload, or for the previous stream), plus one
    call with the noise estimates taken from device memory (srsgpu_pcfich_set_noise_dev). Every
    result equals the oracle."""
    import torch
    import srsgpu_phy as s
    nof_prb, cell_id, nports, nrx = 25, 33, 1, 2  # one port: the noise estimate enters the equaliser
    rng = np.random.default_rng(9)
    n0, stride = nof_prb * 12, nof_prb * 12 * 14
    ns = 48
    subs = []
    for i in range(ns):
        y = [(rng.standard_normal(n0) + 1j * rng.standard_normal(n0)).astype(np.complex64) for _ in range(nrx)]
        h = [[(rng.standard_normal(n0) + 1j * rng.standard_normal(n0)).astype(np.complex64) for _ in range(nrx)]
             for _ in range(nports)]
        subs.append((y, h, float(rng.choice([0.0, 0.3])), i % 10))
    grid = np.zeros((ns, nrx, stride), np.complex64)
    ce = np.zeros((ns, nrx * nports, stride), np.complex64)
    for i, (y, h, _, _) in enumerate(subs):
        for a in range(nrx):
            grid[i, a, :n0] = y[a]
            for p in range(nports):
                ce[i, a * nports + p, :n0] = h[p][a]
    d_grid = torch.from_numpy(grid.view(np.float32)).cuda()
    d_ce = torch.from_numpy(ce.view(np.float32)).cuda()
    q = s.Pcfich(nof_prb, cell_id, nports, nrx)
    st1, st2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    # calls of 7, 16, 25 subframes (different windows of the batch) into separate outputs
    windows = [(0, 7), (5, 21), (20, 45), (30, 48)]
    outs = []
    for k, (a, b) in enumerate(windows):
        st = st1 if k < 3 else st2
        d_cfi = torch.full((b - a,), 9, dtype=torch.int32, device="cuda")
        d_corr = torch.zeros(b - a, dtype=torch.float32, device="cuda")
        sfs = [(i * nrx * stride, i * nrx * nports * stride, subs[i][3], subs[i][2]) for i in range(a, b)]
        assert q.decode_dev(sfs, d_grid.data_ptr(), d_ce.data_ptr(), stride, d_cfi.data_ptr(), d_corr.data_ptr(),
                            stream=st.cuda_stream) == 0
        outs.append((a, b, d_cfi, d_corr))
    # device-resident noise for the last window, on the first stream again
    d_noise = torch.tensor([subs[i][2] for i in range(ns)], dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    s._lib.srsgpu_pcfich_set_noise_dev(q.q, s._vp(d_noise.data_ptr()))
    d_cfi = torch.full((ns,), 9, dtype=torch.int32, device="cuda")
    d_corr = torch.zeros(ns, dtype=torch.float32, device="cuda")
    sfs = [(i * nrx * stride, i * nrx * nports * stride, subs[i][3], -1.0) for i in range(ns)]  # noise ignored
    assert q.decode_dev(sfs, d_grid.data_ptr(), d_ce.data_ptr(), stride, d_cfi.data_ptr(), d_corr.data_ptr(),
                        stream=st1.cuda_stream) == 0
    outs.append((0, ns, d_cfi, d_corr))
    torch.cuda.synchronize()
    s._lib.srsgpu_pcfich_set_noise_dev(q.q, None)
    for a, b, d_cfi, d_corr in outs:
        cfi, corr = d_cfi.cpu().numpy(), d_corr.cpu().numpy()
        for j, i in enumerate(range(a, b)):
            y, h, noise, sf = subs[i]
            w = pcfich_decode(oracle, nof_prb, cell_id, nports, nrx, y, h, noise, sf)
            assert cfi[j] == w[0] and corr[j] == np.float32(w[1]), (a, b, i)
