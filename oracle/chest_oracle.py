"""CPU ORACLE — TEST INFRASTRUCTURE ONLY. numpy (float64) restatement of srsLTE's downlink CRS
channel estimation for CRS ports 0 and 1, normal CP, per-symbol mode (paths relative to
/root/reference/lib/src/phy):

  crs_pilots        ch_estimation/refsignal_dl.c:265-318 (Gold sequence per slot/symbol)
  ls_estimates      refsignal_dl.c:404-430 + chest_dl.c:648-650 (received * conj(CRS))
  noise_refs        chest_dl.c:268-329 estimate_noise_pilots (only the last symbol's residual
                    power is kept: the loop assigns, it does not accumulate)
  smooth            utils/convolution.c:172-211 srslte_conv_same_cf with extrapolated extremes
  interp_freq       resampling/interp.c:245-272 srslte_interp_linear_offset (M = 6)
  interp_time       chest_dl.c:392-397 + interp.c:150-173 (running sums of (b - a) / d)

The reference chest (chest_dl.c) cannot be compiled here: through sync/pss.c and
utils/convolution.c it needs the FFTW-backed DFT, which the image lacks. Its CRS generation and
pilot extraction (refsignal_dl.c) do compile and pin crs_pilots / ls_estimates; the rest is
parity-unpinned restatement (float stage, compared with a tolerance).
Only tests/ may import this module.
"""
import numpy as np

NC = 1600


def gold(cinit, n):
    x1 = np.zeros(NC + n + 31, np.uint8)
    x2 = np.zeros(NC + n + 31, np.uint8)
    x1[0] = 1
    for i in range(31):
        x2[i] = (cinit >> i) & 1
    for i in range(NC + n):
        x1[i + 31] = x1[i + 3] ^ x1[i]
        x2[i + 31] = x2[i + 3] ^ x2[i + 2] ^ x2[i + 1] ^ x2[i]
    return x1[NC:NC + n] ^ x2[NC:NC + n]


def crs_pilots(nof_prb, cell_id, sf_idx):
    """[4 CRS symbols (0, 4, 7, 11)][2*nof_prb] complex pilots of ports 0/1."""
    out = np.zeros((4, 2 * nof_prb), np.complex128)
    m = np.arange(2 * nof_prb) + 110 - nof_prb
    for s in range(2):
        ns = 2 * sf_idx + s
        for li, lp in enumerate((0, 4)):
            cinit = 1024 * (7 * (ns + 1) + lp + 1) * (2 * cell_id + 1) + 2 * cell_id + 1
            c = gold(cinit, 4 * 110).astype(np.float64)
            out[2 * s + li] = ((1 - 2 * c[2 * m]) + 1j * (1 - 2 * c[2 * m + 1])) / np.sqrt(2)
    return out


SYMS = (0, 4, 7, 11)


def fidx(cell_id, l, port=0):
    """refsignal_dl.c:40-95: v = 0 / 3 alternating over the CRS symbols, port 1 shifted by 3"""
    return ((3 if (l % 2) ^ port else 0) + cell_id % 6) % 6


def ls_estimates(grid, nof_prb, cell_id, sf_idx, port=0):
    g = grid.reshape(14, 12 * nof_prb)
    pil = crs_pilots(nof_prb, cell_id, sf_idx)  # ports 0 and 1 share the sequence (pilots[p/2])
    est = np.zeros_like(pil)
    for l, s in enumerate(SYMS):
        est[l] = g[s, fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] * np.conj(pil[l])
    return est


def noise_refs(est, cell_id, port=0):
    n = est.shape[1]
    row3, prev, nxt = est[3], est[2], 2 * est[2] - est[0]
    off = 0 if fidx(cell_id, 0, port) < 3 else 1
    tmp = row3.copy()
    for r in (prev, nxt):
        tmp[off:] += r[:n - off]
        tmp[:n + off - 1] += r[1 - off:]
        if off:
            tmp[0] += 2 * r[0] - r[1]
        else:
            tmp[n - 1] += 2 * r[n - 2] - r[n - 1]
    tmp = row3 - tmp / 5.0
    return np.mean(np.abs(tmp) ** 2) / 4.0 * np.sqrt(5.0)


def smooth(x, filt):
    M, h, N = len(filt), len(filt) // 2, len(x)
    if M == 0:
        return x.copy()
    first = np.array([(2 + h - q) * x[1] - (1 + h - q) * x[0] if q < h else x[q - h]
                      for q in range(M + h)])
    last = np.array([(2 + q - h) * x[N - 1] - (1 + q - h) * x[N - 2] if q >= M - 1 else x[N - M + q + 1]
                     for q in range(M + h)])
    out = np.zeros(N, np.complex128)
    for i in range(h):
        out[i] = np.dot(first[i:i + M], filt)
    for i in range(h, N - h):
        out[i] = np.dot(x[i - h:i - h + M], filt)
    for j, i in enumerate(range(N - h, N)):
        out[i] = np.dot(last[j:j + M], filt)
    return out


def interp_freq(x, off_st, M=6):
    n = len(x)
    out = np.zeros(n * M, np.complex128)
    for j in range(off_st):
        out[off_st - j - 1] = x[0] - (j + 1) * (x[1] - x[0]) / M
    for i in range(n - 1):
        for j in range(M):
            out[i * M + j + off_st] = x[i] + j * (x[i + 1] - x[i]) / M
    d = x[n - 1] - x[n - 2]
    for j in range(M - off_st):
        out[(n - 1) * M + j + off_st] = x[n - 1] + j * d / M
    return out


def estimate(grid, nof_prb, cell_id, sf_idx, filt=(0.1, 0.8, 0.1), port=0):
    """-> (ce grid [14 * 12*nof_prb] complex128, noise estimate) of CRS port `port`"""
    est = ls_estimates(grid, nof_prb, cell_id, sf_idx, port)
    noise = noise_refs(est, cell_id, port)
    f = np.asarray(filt, np.float64)
    sm = est if (len(f) == 0 or (len(f) == 3 and f[0] == 0)) else np.stack([smooth(r, f) for r in est])
    ce = np.zeros((14, 12 * nof_prb), np.complex128)
    for l, s in enumerate(SYMS):
        ce[s] = interp_freq(sm[l], fidx(cell_id, l, port))
    for a, b, d, first, cnt in ((0, 4, 4, 1, 3), (4, 7, 3, 5, 2), (7, 11, 4, 8, 3), (7, 11, 4, 12, 2)):
        diff = (ce[b] - ce[a]) / d
        prev = ce[b] if first == 12 else ce[a]
        for k in range(cnt):
            prev = prev + diff
            ce[first + k] = prev
    return ce.reshape(-1), noise
