"""Golden per-subframe measurements and TM3 / TM4 feedback from the reference (oracle/_ref/ref_front ue_dl,
this container only): what srsUE's PHY worker reads after each subframe — srslte_chest_dl_get_noise_estimate
/ _get_snr / _get_rssi / _get_rsrq / _get_rsrp / _get_rsrp_neighbour / _get_cfo (chest_dl.c:737-846;
phch_worker.cc:226-241, 301, 313, 1618-1628) and its compute_ri (phch_worker.cc:522-540):
srslte_ue_dl_ri_select (condition number, TM3 rank) and srslte_ue_dl_ri_pmi_select (TM4 rank / PMI /
per-codebook SINR), ue_dl.c:684-764.

Synthetic two-port cells: the CRS of ports 0 and 1 (each port's pilots, the other port's pilot REs left
empty, 36.211 6.10.1.2) and random QPSK elsewhere, through a frequency-selective 2 x P channel per
subframe, OFDM (numpy), a carrier offset and AWGN. The time-domain samples are the fixture; the reference
runs on the numpy OFDM oracle's grids (FFTW is absent) with srsUE's estimator settings or the
srslte_chest_dl_init defaults, CFO estimation on all or some subframes (the value carries over the
others, as the estimator object keeps it).

    python tests/golden/make_feedback_golden.py   -> tests/golden/feedback_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import chest_oracle as co  # noqa: E402
import ofdm_oracle as oo  # noqa: E402
from srsgpu_testlib import ref_front_ue_dl  # noqa: E402

SRSUE = dict(gauss=(4, 1.0), average=True, rsrp_neighbour=True, cfo_enable=True, cfo_mask=0x3FF)
INIT = dict(gauss=None, average=False, rsrp_neighbour=False, cfo_enable=True, cfo_mask=(1 << 0) | (1 << 5))
# name: nof_prb, cell_id, nrx, N, subframes (tti), snr_db, cfo_hz, estimator settings, rnti
CASES = {
    "tm4_25_2x2": (25, 7, 2, 512, [0, 1, 2, 3], 25.0, 150.0, SRSUE, 0x4601),
    "tm4_6_2x1": (6, 3, 1, 128, [4, 5, 6], 22.0, -80.0, INIT, 0x1234),
    "tm3_50_2x2": (50, 301, 2, 1024, [5, 6, 7], 28.0, 60.0, INIT, 0x2222),
}


def synth(rng, nof_prb, cell_id, nrx, N, sf_idx, snr_db, cfo_hz):
    """time-domain subframe [nrx][15 N] of a 2-port cell"""
    nsc = 12 * nof_prb
    qpsk = (rng.choice([-1.0, 1.0], (2, 14, nsc)) + 1j * rng.choice([-1.0, 1.0], (2, 14, nsc))) / np.sqrt(2)
    X = qpsk.astype(np.complex128)
    pil = [co.crs_pilots(nof_prb, cell_id, sf_idx, port=p) for p in (0, 1)]
    for p in (0, 1):
        for l, sy in enumerate(co.syms(p)):
            pos = co.fidx(cell_id, l, p) + 6 * np.arange(2 * nof_prb)
            X[p, sy, pos] = pil[p][l]
            X[1 - p, sy, pos] = 0.0  # the other port leaves its pilot REs empty
    k = np.arange(nsc)
    x = np.zeros((nrx, 15 * N), np.complex128)
    for a in range(nrx):
        Y = np.zeros((14, nsc), np.complex128)
        for p in (0, 1):
            ph, amp = rng.uniform(0, 2 * np.pi), rng.uniform(0.4, 1.0)
            d = rng.uniform(0.5, 4.0)
            h = amp * (1 + 0.3 * np.cos(2 * np.pi * d * k / nsc + ph)) * np.exp(1j * (ph + 0.7 * np.sin(2 * np.pi * k / nsc)))
            Y += X[p] * h[None, :]
        x[a] = oo.tx_sf(Y.reshape(-1), nof_prb, N) / N
    n = np.arange(15 * N)
    x *= np.exp(2j * np.pi * cfo_hz * n / (15000.0 * N))[None, :]
    sig = np.sqrt(np.mean(np.abs(x) ** 2)) * 10 ** (-snr_db / 20) / np.sqrt(2)
    x += sig * (rng.standard_normal(x.shape) + 1j * rng.standard_normal(x.shape))
    return x.astype(np.complex64)


def main():
    rng = np.random.default_rng(77)
    arrays, man = {}, {}
    for name, (nof_prb, cell_id, nrx, N, ttis, snr, cfo, cfg, rnti) in CASES.items():
        xs = np.stack([synth(rng, nof_prb, cell_id, nrx, N, t % 10, snr, cfo) for t in ttis])
        grids = [[oo.rx_sf(xs[i, a], nof_prb, N).reshape(-1).astype(np.complex64) for a in range(nrx)]
                 for i in range(len(ttis))]
        res = ref_front_ue_dl(nof_prb, cell_id, 2, nrx, 0, 2, nof_prb, rnti, 3, ttis, grids,
                              gauss=cfg["gauss"], filt=None if cfg["gauss"] else (0.1, 0.8, 0.1),
                              average=cfg["average"], rsrp_neighbour=cfg["rsrp_neighbour"],
                              cfo_enable=cfg["cfo_enable"], cfo_mask=cfg["cfo_mask"])
        arrays[name + "_x"] = xs
        arrays[name + "_getters"] = np.stack([r["getters"] for r in res])
        arrays[name + "_cn"] = np.array([r["cn"] for r in res], np.float32)
        arrays[name + "_sinr"] = np.stack([r["sinr"] for r in res])
        for k in ("ri_tm3", "ret_cn", "ri", "pmi", "ret_pmi"):
            arrays["%s_%s" % (name, k)] = np.array([r[k] for r in res], np.int32)
        arrays[name + "_pmi_l"] = np.array([r["pmi_l"] for r in res], np.int32)
        man[name] = dict(nof_prb=nof_prb, cell_id=cell_id, nof_ports=2, nrx=nrx, N=N, ttis=ttis, snr_db=snr,
                         cfo_hz=cfo, rnti=rnti, gauss=cfg["gauss"], average=cfg["average"],
                         rsrp_neighbour=cfg["rsrp_neighbour"], cfo_enable=cfg["cfo_enable"],
                         cfo_mask=cfg["cfo_mask"])
        for r in res:
            print(name, np.round(r["getters"], 5).tolist(), round(r["cn"], 3), r["ri_tm3"], r["ri"], r["pmi"],
                  r["pmi_l"], np.round(r["sinr"], 3).tolist())
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "feedback_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
