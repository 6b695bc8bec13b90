"""The reference's own over-the-air recordings (lib/src/phy/phch/test/signal.10M.dat and
signal.1.92M.amar.dat, the inputs of its ctest cases pcfich_file_test / pdcch_file_test /
pdsch_pdcch_file_test, CMakeLists.txt:213-216) through the GPU receive chain, from the time-domain
samples: OFDM FFT -> CRS channel estimation -> PCFICH -> PDCCH + DCI blind search -> PDSCH / DL-SCH.

These are the reference's only evidence for the OFDM stage on real signals. The expected values
(tests/golden/recorded_golden.npz, tests/golden/make_recorded_golden.py) are the reference's own
chest_dl.c / pcfich.c / pdcch.c / ue_dl.c / pdsch.c run on the numpy OFDM oracle's grids (FFTW, which
the reference's ofdm.c needs, is absent). The GPU must meet the reference tests' pass criteria and
equal those outputs: the grid within 1e-4 of the numpy OFDM (relative to the grid's peak), the channel
estimates within 1e-4, CFI / DCI / TB bytes / ack exactly, the PCFICH correlation within 1e-4."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "oracle"))
import ofdm_oracle as oo  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden", "recorded_golden.npz")
SIRNTI = 0xFFFF


def _load():
    z = np.load(GOLD)
    return z, json.loads(bytes(z["manifest"]).decode())


def _padded(x, N, nsf):
    """the subframes of a recording, zero-padded as srslte_ofdm_init_ leaves the input buffer (ofdm.c:84-88)"""
    L = 15 * N
    out = np.zeros(nsf * L, np.complex64)
    out[:min(x.size, out.size)] = x[:out.size]
    return out.reshape(nsf, L)


def test_golden_meets_reference_pass_criteria():
    """the recorded expectations are the reference tests' passes: pcfich_file_test.c:244-256 (CFI 1,
    correlation > 2.8) and pdsch_pdcch_file_test.c:186-210 (a subframe with a DCI and a decoded PDSCH)"""
    z, man = _load()
    assert int(z["s10m_cfi"][0]) == 1 and float(z["s10m_corr"][0]) > 2.8
    ok = np.flatnonzero(z["amar_ret"] > 0)
    assert ok.size >= 1 and all(z["amar_ack"][ok] == 1)
    assert all(z["amar_dl"][ok, 0] == 1)
    assert man["amar"]["subframes"] == 10 and z["amar_x"].size == 10 * 15 * 128
    assert z["s10m_x"].size == man["s10m"]["samples"] == 7681  # half a subframe: the rest is zeros


def test_numpy_chest_oracle_on_recordings():
    """the numpy estimator restatement (oracle/chest_oracle.py, the default 3-tap smoothing, REFS noise)
    on the numpy OFDM grids equals the reference's estimates on the same grids"""
    import chest_oracle as co
    z, man = _load()
    for name in ("s10m", "amar"):
        m = man[name]
        xs = _padded(z[name + "_x"], m["N"], m["subframes"])
        for i in range(m["subframes"]):
            g = oo.rx_sf(xs[i], m["nof_prb"], m["N"]).reshape(-1)
            for p in range(m["nof_ports"]):
                ce, _ = co.estimate(g, m["nof_prb"], m["cell_id"], i % 10, port=p)
                ref = z[name + "_ce"][i, p, 0]
                assert np.abs(ce - ref).max() <= 1e-4 * np.abs(ref).max(), (name, i, p)


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "ref_front")),
                    reason="needs the reference build (this container only)")
def test_golden_equals_live_reference():
    from srsgpu_testlib import ref_front_ue_dl
    z, man = _load()
    for name in ("s10m", "amar"):
        m = man[name]
        xs = _padded(z[name + "_x"], m["N"], m["subframes"])
        grids = [[oo.rx_sf(xs[i], m["nof_prb"], m["N"]).reshape(-1).astype(np.complex64)] for i in range(m["subframes"])]
        res = ref_front_ue_dl(m["nof_prb"], m["cell_id"], m["nof_ports"], 1, m["phich_length"], m["phich_resources"],
                              m["max_prb"], m["rnti"], m["tm"], list(range(m["subframes"])), grids)
        for i, r in enumerate(res):
            assert r["cfi"] == z[name + "_cfi"][i] and r["ret"] == z[name + "_ret"][i], (name, i)
            assert r["corr"] == z[name + "_corr"][i] and r["dl"][0] == z[name + "_dl"][i, 0], (name, i)


def _gpu_front(s, torch, name, z, m):
    """GPU OFDM + channel estimation (default configuration, as the reference tests' estimators) of a
    recording -> (grids [nsf][n], ce [nsf][port][n], noise [nsf])"""
    nof_prb, N, nsf, P = m["nof_prb"], m["N"], m["subframes"], m["nof_ports"]
    n = 14 * 12 * nof_prb
    xs = _padded(z[name + "_x"], N, nsf)
    ofdm = s.OfdmRx(nof_prb, N)
    chest = s.Chest(nof_prb, m["cell_id"], max_grids=nsf, nof_ports=P)
    d_x = torch.from_numpy(xs.reshape(-1)).cuda()
    d_grid = torch.zeros(nsf * n, dtype=torch.complex64, device="cuda")
    d_ce = torch.zeros(nsf * P * n, dtype=torch.complex64, device="cuda")
    d_noise = torch.zeros(nsf * P, dtype=torch.float32, device="cuda")
    assert ofdm.rx_dev(nsf, d_x.data_ptr(), 15 * N, d_grid.data_ptr(), n) == 0
    assert chest.estimate_dev([i % 10 for i in range(nsf)], d_grid.data_ptr(), n, d_ce.data_ptr(),
                              d_noise.data_ptr()) == 0
    torch.cuda.synchronize()
    out = (d_grid.cpu().numpy().reshape(nsf, n), d_ce.cpu().numpy().reshape(nsf, P, n),
           d_noise.cpu().numpy().reshape(nsf, P))
    ofdm.close()
    chest.close()
    return xs, d_grid, d_ce, out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["s10m", "amar"])
def test_gpu_ofdm_and_chest_on_recordings(name):
    import torch
    import srsgpu_phy as s
    z, man = _load()
    m = man[name]
    xs, _, _, (grid, ce, _) = _gpu_front(s, torch, name, z, m)
    for i in range(m["subframes"]):
        ref = oo.rx_sf(xs[i], m["nof_prb"], m["N"]).reshape(-1)
        assert np.abs(grid[i] - ref).max() <= 1e-4 * np.abs(ref).max(), (name, i)
        for p in range(m["nof_ports"]):
            r = z[name + "_ce"][i, p, 0]
            assert np.abs(ce[i, p] - r).max() <= 1e-4 * np.abs(r).max(), (name, i, p)


@pytest.mark.gpu
def test_gpu_pcfich_file_test():
    """pcfich_file_test -c 150 -n 50 -p 2 -i signal.10M.dat: the GPU chain's CFI is 1 with correlation
    > 2.8, and equals the reference's on the same samples"""
    import torch
    import srsgpu_phy as s
    z, man = _load()
    m = man["s10m"]
    n = 14 * 12 * m["nof_prb"]
    _, d_grid, d_ce, (_, _, noise) = _gpu_front(s, torch, "s10m", z, m)
    pc = s.Pcfich(m["nof_prb"], m["cell_id"], m["nof_ports"], 1)
    d_cfi = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_corr = torch.zeros(1, dtype=torch.float32, device="cuda")
    assert pc.decode_dev([(0, 0, 0, float(noise[0].mean()))], d_grid.data_ptr(), d_ce.data_ptr(), n,
                         d_cfi.data_ptr(), d_corr.data_ptr()) == 0
    torch.cuda.synchronize()
    cfi, corr = int(d_cfi.item()), float(d_corr.item())
    assert cfi == 1 and corr > 2.8
    assert cfi == int(z["s10m_cfi"][0]) and abs(corr - float(z["s10m_corr"][0])) <= 1e-4 * abs(corr)


@pytest.mark.gpu
def test_gpu_pdsch_pdcch_file_test():
    """pdsch_pdcch_file_test -c 1 -f 3 -n 6 -p 1 -i signal.1.92M.amar.dat (and pdcch_file_test on the same
    capture): the ten recorded subframes as srslte_ue_dl_decode calls with the SI-RNTI on the GPU queue
    (FFT -> chest -> PCFICH -> PDCCH search -> grant -> PDSCH); every subframe's CFI, DCI search result,
    return value, ack and SIB bytes equal the reference's, and the reference test's pass (a DCI found and
    its PDSCH decoded) is met"""
    import torch  # noqa: F401
    import srsgpu_phy as s
    z, man = _load()
    m = man["amar"]
    nsf, N = m["subframes"], m["N"]
    xs = _padded(z["amar_x"], N, nsf)
    q = s.RxQueue(m["nof_prb"], m["cell_id"], N, nof_softbuffers=2 * nsf, max_batch=nsf, max_wait_us=100000)
    q.set_phich(m["phich_length"], m["phich_resources"])
    outs = [np.zeros(12000, np.uint8) for _ in range(nsf)]
    items = [q.ue_item([xs[i]], i, SIRNTI, [outs[i]], tm=0, softbuffer=(2 * i, 2 * i + 1)) for i in range(nsf)]
    tickets = [q.submit_ue_dl(u) for u in items]
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    decoded = 0
    for i, u in enumerate(items):
        assert u.cfi == int(z["amar_cfi"][i]) == 3, (i, u.cfi)
        assert abs(u.cfi_corr - float(z["amar_corr"][i])) <= 1e-4 * abs(u.cfi_corr), i
        found, fmt, L, ncce, nbits = (int(v) for v in z["amar_dl"][i])
        assert u.found == found, i
        assert u.ret == int(z["amar_ret"][i]), (i, u.ret)
        if found == 1:
            assert (u.format, u.L, u.ncce) == (fmt, L, ncce), i
            assert u.dci_nof_bits == nbits and u.dci_bits() == list(z["amar_msg"][i][:nbits]), i
            assert int(u.grant.tbs[0]) == int(z["amar_tbs"][i]) and int(u.grant.mod[0]) == int(z["amar_mod"][i]), i
            assert int(u.acks[0]) == int(z["amar_ack"][i]) and u.rv[0] == int(z["amar_rv"][i]), i
            nb = int(z["amar_tbs"][i]) // 8
            assert (outs[i][:nb] == z["amar_data"][i][:nb]).all(), i
            decoded += int(u.ret > 0 and u.acks[0])
    assert decoded >= 1
    q.close()
