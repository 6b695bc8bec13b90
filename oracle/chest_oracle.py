"""CPU ORACLE — TEST INFRASTRUCTURE ONLY. numpy (float64) restatement of srsLTE's downlink CRS
channel estimation for CRS ports 0-3, normal and extended CP (cp=1: 6 symbols per slot; paths relative to
/root/reference/lib/src/phy):

  crs_pilots        ch_estimation/refsignal_dl.c:265-318 (Gold sequence per slot/symbol)
  ls_estimates      refsignal_dl.c:404-430 + chest_dl.c:648-650 (received * conj(CRS))
  noise_refs        chest_dl.c:268-329 estimate_noise_pilots (only the last symbol's residual
                    power is kept: the loop assigns, it does not accumulate)
  smooth            utils/convolution.c:172-211 srslte_conv_same_cf with extrapolated extremes
  interp_freq       resampling/interp.c:245-272 srslte_interp_linear_offset (M = 6)
  interp_time       chest_dl.c:421-431 + interp.c:150-173 (running sums of (b - a) / d); ports 2 / 3
                    (CRS in symbols 1 and 8 only): symbol 0 extrapolated back from 1, symbols 2-7
                    forward from 1 with (c8 - c1) / 7, and 9-13 forward from symbol 1 again (the
                    reference's in0 is c1 for that segment, so they repeat 2-6)
  average_row       chest_dl.c:528-548 average_pilots with average_subframe (srsUE's default,
                    srsue/src/main.cc:287-289): the 4 CRS symbols folded into one row of 4*nof_prb
                    pilots at spacing 3, interpolated with M = 3 (chest_dl.c:393-399) and copied to
                    all 14 symbols (chest_dl.c:410-414)
  gauss_filter      chest_dl.c:471-490 srslte_chest_dl_set_smooth_filter_gauss (smooth_filter_auto,
                    chest_dl.c:616-618: order 4, std dev = noise estimate x 200)
  noise_pss         chest_dl.c:332-348 estimate_noise_pss (sync/pss.c:354-398 sequence / slot)
  noise_empty       chest_dl.c:351-361 estimate_noise_empty_sc; both only in subframes 0 and 5
  measurements      chest_dl.c:500-515 rssi, :562-587 CFO, :652-657 RSRP / RSRP correlation

Pinned to the reference: chest_dl.c itself (with sync/pss.c, utils/convolution.c, resampling/interp.c)
is compiled where it lies into oracle/_ref/ref_front (srslte_dft_* left unresolved: the estimation path
never calls them). tests/golden/chest_golden.npz holds its outputs (tests/golden/make_chest_golden.py)
and tests/test_chest.py checks this restatement against them (and against live runs in the build
container) within 1e-4 relative; CRS generation and pilot extraction equal refsignal_dl.c bit for bit.
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


def nsymb(cp=0):
    """SRSLTE_CP_NSYMB: OFDM symbols per slot"""
    return 6 if cp else 7


def syms(port=0, cp=0):
    """srslte_refsignal_cs_nsymbol (refsignal_dl.c:112-122): the CRS symbols of a port in a subframe,
    normal CP 0 / 4 / 7 / 11 or 1 / 8, extended CP 0 / 3 / 6 / 9 or 1 / 7"""
    n = nsymb(cp)
    return (0, n - 3, n, 2 * n - 3) if port < 2 else (1, n + 1)


SYMS = syms(0)


def crs_pilots(nof_prb, cell_id, sf_idx, port=0, cp=0):
    """[CRS symbols][2*nof_prb] complex pilots of ports 0/1 or 2/3: csr_refs.pilots[port / 2]
    (refsignal_dl.c:291-313, l' = 0 / nsymb - 3 or 1 in each slot, N_cp = 1 normal, 0 extended)"""
    lps = (0, nsymb(cp) - 3) if port < 2 else (1,)
    out = np.zeros((2 * len(lps), 2 * nof_prb), np.complex128)
    m = np.arange(2 * nof_prb) + 110 - nof_prb
    for s in range(2):
        ns = 2 * sf_idx + s
        for li, lp in enumerate(lps):
            cinit = 1024 * (7 * (ns + 1) + lp + 1) * (2 * cell_id + 1) + 2 * cell_id + (0 if cp else 1)
            c = gold(cinit, 4 * 110).astype(np.float64)
            out[len(lps) * s + li] = ((1 - 2 * c[2 * m]) + 1j * (1 - 2 * c[2 * m + 1])) / np.sqrt(2)
    return out




def fidx(cell_id, l, port=0):
    """refsignal_dl.c:40-95: v = 0 / 3 alternating over the CRS symbols, ports 1 and 3 shifted by 3"""
    return ((3 if (l % 2) ^ (port % 2) else 0) + cell_id % 6) % 6


def ls_estimates(grid, nof_prb, cell_id, sf_idx, port=0, cp=0):
    g = grid.reshape(2 * nsymb(cp), 12 * nof_prb)
    pil = crs_pilots(nof_prb, cell_id, sf_idx, port, cp)  # ports 2p and 2p+1 share pilots[p]
    est = np.zeros_like(pil)
    for l, s in enumerate(syms(port, cp)):
        est[l] = g[s, fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] * np.conj(pil[l])
    return est


def noise_refs(est, cell_id, port=0):
    """the last CRS symbol's residual against its neighbours: with 4 symbols est[2] and the
    extrapolated 2 est[2] - est[0]; with 2 (ports 2 / 3) est[0] on both sides (chest_dl.c:285-299)"""
    n, ns = est.shape[1], est.shape[0]
    last = est[ns - 1]
    prev, nxt = (est[2], 2 * est[2] - est[0]) if ns == 4 else (est[0], est[0])
    off = 0 if fidx(cell_id, 0, port) < 3 else 1
    tmp = last.copy()
    for r in (prev, nxt):
        tmp[off:] += r[:n - off]
        tmp[:n + off - 1] += r[1 - off:]
        if off:
            tmp[0] += 2 * r[0] - r[1]
        else:
            tmp[n - 1] += 2 * r[n - 2] - r[n - 1]
    tmp = last - tmp / 5.0
    return np.mean(np.abs(tmp) ** 2) / ns * np.sqrt(5.0)


def interp_time(ce, port=0, cp=0):
    """chest_dl.c:421-442 on a [14][nsc] (extended CP [12][nsc]) grid whose CRS rows are filled;
    segments (a, b, d, first, count, start): rows first .. first+count-1 = running sums of (b - a) / d
    from row start"""
    if cp:  # chest_dl.c:433-441
        segs = (((0, 3, 3, 1, 2, 0), (3, 6, 3, 4, 2, 3), (6, 9, 3, 7, 2, 6), (6, 9, 3, 10, 2, 9)) if port < 2 else
                ((7, 1, 6, 0, 1, 1), (1, 7, 6, 2, 5, 1), (1, 7, 6, 8, 4, 1)))
    elif port < 2:
        segs = ((0, 4, 4, 1, 3, 0), (4, 7, 3, 5, 2, 4), (7, 11, 4, 8, 3, 7), (7, 11, 4, 12, 2, 11))
    else:
        segs = ((8, 1, 7, 0, 1, 1), (1, 8, 7, 2, 6, 1), (1, 8, 7, 9, 5, 1))
    for a, b, d, first, cnt, start in segs:
        diff = (ce[b] - ce[a]) / d
        prev = ce[start]
        for k in range(cnt):
            prev = prev + diff
            ce[first + k] = prev


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


def estimate(grid, nof_prb, cell_id, sf_idx, filt=(0.1, 0.8, 0.1), port=0, cp=0):
    """-> (ce grid [14 (12) * 12*nof_prb] complex128, noise estimate) of CRS port `port`"""
    est = ls_estimates(grid, nof_prb, cell_id, sf_idx, port, cp)
    noise = noise_refs(est, cell_id, port)
    f = np.asarray(filt, np.float64)
    sm = est if (len(f) == 0 or (len(f) == 3 and f[0] == 0)) else np.stack([smooth(r, f) for r in est])
    ce = np.zeros((2 * nsymb(cp), 12 * nof_prb), np.complex128)
    for l, s in enumerate(syms(port, cp)):
        ce[s] = interp_freq(sm[l], fidx(cell_id, l, port))
    interp_time(ce, port, cp)
    return ce.reshape(-1), noise


def average_row(est, cell_id, port=0):
    """chest_dl.c:528-548: slot-pair interleave of the CRS symbols, scaled by 2 / nsymbols"""
    n, ns = est.shape[1], est.shape[0]
    a, b = (0, 1) if fidx(cell_id, 0, port) < 3 else (1, 0)
    t = np.zeros(2 * n, np.complex128)
    t[0::2] = est[a] + est[a + 2] if ns == 4 else est[a]
    t[1::2] = est[b] + est[b + 2] if ns == 4 else est[b]
    return t * (2.0 / ns)


def gauss_filter(order, std_dev):
    """chest_dl.c:471-490 (float32 as the reference computes it)"""
    L, c = order + 1, order // 2
    f = np.array([np.exp(np.float32(-float((i - c) ** 2)) / np.float32(2.0 * np.float32(std_dev) ** 2))
                  for i in range(L)], np.float32)
    norm = np.float32(0)
    for v in f:
        norm = np.float32(norm + v)
    return (f * np.float32(1.0 / norm)).astype(np.float64)


def pss_sequence(n_id_2):
    """sync/pss.c:354-382: length-62 Zadoff-Chu, roots 25 / 29 / 34"""
    u = (25.0, 29.0, 34.0)[n_id_2]
    i = np.arange(62, dtype=np.float64)
    arg = np.where(i < 31, -np.pi * u * i * (i + 1) / 63.0, -np.pi * u * (i + 2) * (i + 1) / 63.0)
    return np.exp(1j * arg.astype(np.float32).astype(np.float64))  # pss.c stores the argument as float


def _avg_power(x):
    return float(np.mean(np.abs(x) ** 2))


def noise_pss(grid, ce, nof_prb, cell_id, nof_ports, cp=0):
    nsc = 12 * nof_prb
    k = (nsymb(cp) - 1) * nsc + nsc // 2 - 31  # srslte_pss_get_slot: last symbol of slot 0
    r = ce[k:k + 62] * pss_sequence(cell_id % 3) - grid[k:k + 62]
    return nof_ports * _avg_power(r) / np.sqrt(2)


def noise_empty(grid, nof_prb, cp=0):
    nsc = 12 * nof_prb
    ks = (nsymb(cp) - 2) * nsc + nsc // 2 - 31
    kp = (nsymb(cp) - 1) * nsc + nsc // 2 - 31
    return (_avg_power(grid[ks - 5:ks]) + _avg_power(grid[ks + 62:ks + 67]) +
            _avg_power(grid[kp - 5:kp]) + _avg_power(grid[kp + 62:kp + 67]))


def measurements(grid, nof_prb, cell_id, sf_idx, port=0, symbol_sz=1536, cp=0):
    """(rsrp, rssi, rsrp_corr, cfo) as srslte_chest_dl_estimate_port leaves them in q. The CFO
    (chest_dl.c:583-603) always reads 4 rows of the shared pilot buffer: for ports 2 / 3, which
    fill only the first 2, rows 2 and 3 still hold port 1's estimates of the same rx antenna
    (srslte_chest_dl_estimate_multi runs the ports in order)"""
    g = grid.reshape(2 * nsymb(cp), 12 * nof_prb)
    sy = syms(port, cp)
    recv = np.stack([g[s, fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] for l, s in enumerate(sy)])
    est = ls_estimates(grid, nof_prb, cell_id, sf_idx, port, cp)
    rsrp = _avg_power(recv)
    rssi = float(sum(np.sum(np.abs(g[s]) ** 2) for s in sy) / len(sy))
    corr = abs(est.sum() / est.size) ** 2
    e4 = est if port < 2 else np.concatenate([est, ls_estimates(grid, nof_prb, cell_id, sf_idx, 1, cp)[2:]])
    acc = np.sum(e4[0] * np.conj(e4[2])) + np.sum(e4[1] * np.conj(e4[3]))
    n = float(symbol_sz)
    ng = float(np.ceil(144 * n / 2048))
    cfo = -np.angle(acc) * n / (nsymb(cp) * (n + ng)) / 2 / np.pi
    return rsrp, rssi, corr, cfo


def estimate_full(grid, nof_prb, cell_id, sf_idx, filt=(0.1, 0.8, 0.1), port=0, average=False,
                  noise_alg="refs", filt_auto=False, noise_in=0.0, nof_ports=1, cp=0):
    """chest_interpolate_noise_est (chest_dl.c:606-639) in any of srsUE's configurations.
    -> (ce, noise): noise is the value q->noise_estimate[rx][port] holds afterwards (noise_in when
    the algorithm leaves it alone: PSS / EMPTY outside subframes 0 and 5)"""
    est = ls_estimates(grid, nof_prb, cell_id, sf_idx, port, cp)
    noise = noise_refs(est, cell_id, port) if noise_alg == "refs" else noise_in
    f = gauss_filter(4, noise * 200.0) if filt_auto else np.asarray(filt, np.float64)
    smoothing = not (len(f) == 0 or (len(f) == 3 and f[0] == 0))
    nsc = 12 * nof_prb
    ce = np.zeros((2 * nsymb(cp), nsc), np.complex128)
    if average:
        # without smoothing the reference interpolates the raw pilot buffer (symbols 0 and 4
        # back to back) as if it were the averaged row (chest_dl.c:619-621 + 393-399)
        row = smooth(average_row(est, cell_id, port), f) if smoothing else est[:2].reshape(-1)
        ce[:] = interp_freq(row, cell_id % 3, M=3)[None, :]
    else:
        sm = np.stack([smooth(r, f) for r in est]) if smoothing else est
        for l, s in enumerate(syms(port, cp)):
            ce[s] = interp_freq(sm[l], fidx(cell_id, l, port))
        interp_time(ce, port, cp)
    ce = ce.reshape(-1)
    if noise_alg != "refs" and sf_idx in (0, 5):
        noise = (noise_pss(grid, ce, nof_prb, cell_id, nof_ports, cp) if noise_alg == "pss"
                 else noise_empty(grid, nof_prb, cp))
    return ce, noise
