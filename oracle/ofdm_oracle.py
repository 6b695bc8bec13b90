"""CPU ORACLE — TEST INFRASTRUCTURE ONLY. numpy (float64) restatement of srsLTE's normal- and extended-CP OFDM
modulator / demodulator (paths relative to /root/reference/lib/src/phy):

  rx_sf   dft/ofdm.c:401-470 srslte_ofdm_rx_sf with the guru plan of :86-104: per symbol the N
          samples after its CP (ceil(160 N/2048) for symbol 0 of a slot, ceil(144 N/2048) after),
          forward DFT, bins [N - nre/2, N) ++ [1, 1 + nre/2), optional 1/sqrt(N)
  tx_sf   dft/ofdm.c:491-598 srslte_ofdm_tx_sf: the inverse mapping, inverse DFT, CP = tail copy

The reference DFT is FFTW (dft/dft_fftw.c), which this image lacks, so the reference OFDM cannot
be compiled: parity is pinned to numpy's float64 FFT, checked with a tolerance.
Only tests/ and bench.py's CPU baseline may import this module.
"""
import math

import numpy as np


def cp_lens(N, ext=False):
    """(first, other) CP lengths of a slot (ofdm.c:75-76): normal ceil(160 N/2048), ceil(144 N/2048);
    extended ceil(512 N/2048) for all 6 symbols"""
    if ext:
        return math.ceil(512 * N / 2048), math.ceil(512 * N / 2048)
    return math.ceil(160 * N / 2048), math.ceil(144 * N / 2048)


def symbol_starts(N, ext=False):
    cp0, cp = cp_lens(N, ext)
    ns = 6 if ext else 7
    return [s * (N * 15 // 2) + cp0 + l * (N + cp) for s in range(2) for l in range(ns)]


def rx_sf(x, nof_prb, N, normalize=False, ext=False):
    nre = 12 * nof_prb
    h = nre // 2
    out = np.zeros((12 if ext else 14, nre), np.complex128)
    for i, st in enumerate(symbol_starts(N, ext)):
        X = np.fft.fft(np.asarray(x[st:st + N], np.complex128))
        out[i, :h] = X[N - h:]
        out[i, h:] = X[1:1 + h]
    if normalize:
        out /= math.sqrt(N)
    return out.reshape(-1)


def tx_sf(grid, nof_prb, N, ext=False):
    nre = 12 * nof_prb
    h = nre // 2
    ns = 6 if ext else 7
    g = np.asarray(grid).reshape(2 * ns, nre)
    cp0, cp = cp_lens(N, ext)
    out = np.zeros(15 * N, np.complex128)
    for i, st in enumerate(symbol_starts(N, ext)):
        X = np.zeros(N, np.complex128)
        X[N - h:] = g[i, :h]
        X[1:1 + h] = g[i, h:]
        t = np.fft.ifft(X) * N
        c = cp0 if i % ns == 0 else cp
        out[st - c:st] = t[N - c:]
        out[st:st + N] = t
    return out
