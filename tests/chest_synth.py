"""Synthetic CRS grids for the channel-estimation tests and golden generator (test infrastructure).

smooth_channel / crs_grid follow the reference's chest_test_dl.c channel; sync_grid adds the PSS / SSS
of subframes 0 and 5 with their empty subcarriers (pss.c:386-392) and a per-port channel.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402


def smooth_channel(nof_prb):
    """chest_test_dl.c:158-164 channel: h = (3 + x) exp(jx), x = -1 + i/7 + cos(2 pi j / (12 nprb))"""
    i = np.arange(14)[:, None]
    j = np.arange(12 * nof_prb)[None, :]
    x = -1 + i / 7 + np.cos(2 * np.pi * j / nof_prb / 12)
    return ((3 + x) * np.exp(1j * x)).reshape(-1)


def crs_grid(nof_prb, cell_id, sf_idx, rng, port=0):
    """random data REs with the CRS of `port` placed (refsignal_cs_put_sf)"""
    g = ((0.5 - rng.random((14, 12 * nof_prb))) + 1j * (0.5 - rng.random((14, 12 * nof_prb))))
    pil = co.crs_pilots(nof_prb, cell_id, sf_idx, port)
    for l, s in enumerate(co.syms(port)):
        g[s, co.fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] = pil[l]
    return g.reshape(-1)


def sync_grid(nof_prb, cell_id, sf_idx, nports, rng, sigma=0.02, flat=False):
    """every port's CRS through its own channel; in subframes 0 / 5 the PSS (symbol 6) and a random
    SSS (symbol 5) at the band centre with their 5 empty subcarriers either side (pss.c:386-392)"""
    size = 14 * 12 * nof_prb
    nsc = 12 * nof_prb
    g = np.zeros(size, np.complex128)
    hs = []
    for port in range(nports):
        h = smooth_channel(nof_prb) * np.exp(1j * rng.uniform(0, 6.3)) * (0.5 + port)
        if flat:
            h = np.tile(h.reshape(14, -1)[0], 14)
        hs.append(h)
        x = crs_grid(nof_prb, cell_id, sf_idx, rng, port)
        mask = np.zeros((14, nsc), bool)
        for l, sy in enumerate(co.syms(port)):
            mask[sy, co.fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] = True
        g += np.where(mask.reshape(-1), x * h, 0)
    if sf_idx in (0, 5):
        k0 = nsc // 2 - 31
        for s, seq in ((6, co.pss_sequence(cell_id % 3)), (5, np.sign(rng.standard_normal(62)) + 0j)):
            k = s * nsc + k0
            g[k - 5:k] = 0
            g[k + 62:k + 67] = 0
            g[k:k + 62] = seq * hs[0][k:k + 62]
    g += sigma * (rng.standard_normal(size) + 1j * rng.standard_normal(size))
    return g.astype(np.complex64)
