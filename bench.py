#!/usr/bin/env python3
"""Benchmark of the MI355X PDSCH receive path on BASELINE.json's metric configuration, configs[2]:
20 MHz (2048-point FFT) SISO 64QAM subframes, 1024 per GPU per step, time domain -> TB bytes (OFDM FFT,
CRS channel estimation, MMSE, 64QAM demapping, descrambling, de-rate-matching, turbo decoding with CRC
early stop up to 8 half-iterations, TB CRC), coded traffic from the GPU transmitter at 20 dB, inputs
resident in HBM. value = decoded Mbps (the sum of K over CRC-passing code blocks per
second); config carries subframes/s. The CPU baseline is the reference's own srslte_chest_dl_estimate
+ srslte_pdsch_decode (oracle/_ref/ref_front) on the same received grids, FFT excluded.

Further legs on the same JSON line: BASELINE configs[1] (4096 x K=6144 code blocks, 8 half-iterations:
decoder_c2, with its own roofline and the reference AVX2 decoder as its CPU baseline), the same C3
subframes with all 8 half-iterations (no early stop), an SNR sweep into the waterfall, the 1536-point
FFT, TM3 (configs[3] shard), mixed bandwidths (configs[4] shard), the 8-bit decoders, PDCCH / PCFICH,
the subframe queue and the per-call drop-in.

    python bench.py [--gpus N] [--steps K] [--warmup W]
For N > 1, one rank per GPU: under torch.distributed.run (WORLD_SIZE must equal N), or started by
bench.py itself when WORLD_SIZE is unset (N child processes, rank r on GPU r). Each rank decodes its
own shard of the global job (independent subframes, no data-path collective; results gathered to
rank 0) -> weak scaling. Rank 0 writes the full record to bench_detail.json and prints ONE compact
JSON line (<= 6 KB: the contract's keys, roofline, valu_roofline, cpu_baseline, one number per leg).
"""
import argparse
import ctypes
import gc
import json
import re
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))

METRIC = "turbo-decoded Mbps + subframes/s, 20 MHz 64QAM, 1/2/4/8 MI355X"
K = 6144
NCB = 4096
NHALF = 8
NSTREAMS = 3  # batches in flight in the streaming measurement
EBNO_DB = 4.5            # reference convention (noise std sqrt(1/(Es/N0))), error-free region
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SF_BITS = 75376          # 20 MHz, MCS 28 transport block (13 x K=5824): subframe equivalent
# SURVEY §8(d) compulsory HBM bytes of one code block's whole decode: the int16 input in the
# reference's sub-block layout, (3(K+32)+12) * 2 B, plus K/8 decision bytes = 37,848 B at K=6144.
# One half-iteration launch is charged 1/NHALF of it (roofline.achieved).
COMPULSORY_BYTES_PER_CB = (3 * (K + 32) + 12) * 2 + K // 8
# SURVEY §8(d) algorithmic work: ~90 int16 operations per info bit per half-iteration (beta ~25.5,
# alpha ~56.5, estimation pre-passes ~4.8, extrinsic subtraction + scatter ~3)
ALG_OPS_PER_BIT_HALFIT = 90
# SURVEY §8(d) VALU peak for packed int16: 256 CUs x 64 lanes x 2 packed halves x 2.4 GHz
# = 78.6 T int16-ops/s. The issue rate measured on the MI355X (tools/dbg/vrate16.hip,
# profiles/r02_vrate16.txt) is lower: 1024 SIMDs x 128 ops / 1.96 ns = 66.9 T at 4 waves per
# SIMD, 51.4 T (2.55 ns) at the decoder's one wave per SIMD with 8 independent chains.
VALU_INT16_PEAK_T = 78.6
VALU_INT16_MEASURED_T = {"4_waves_per_simd": 66.9, "1_wave_per_simd_ilp8": 51.4}


def make_inputs(n, seed, tcod, first=0):
    """Code blocks first .. first+n-1 of the global job (a rank's contiguous shard): random bits
    (256 templates, the same on every rank), srslte_tcod_encode (product encoder), AWGN (noise
    seeded by the shard), int16 LLRs."""
    rng = np.random.default_rng(seed)
    ntmpl = 256
    bits = rng.integers(0, 2, (ntmpl, K), dtype=np.uint8)
    coded = np.stack([tcod.encode(b) for b in bits])
    rng = np.random.default_rng(seed + 1 + first)
    idx = (first + np.arange(n)) % ntmpl
    esno = EBNO_DB + 10 * np.log10(1.0 / 3.0)
    sigma = np.float32(np.sqrt(1.0 / 10 ** (esno / 10)))
    llr = np.empty((n, 3 * K + 12), np.int16)
    for c0 in range(0, n, 512):
        c1 = min(n, c0 + 512)
        sym = np.where(coded[idx[c0:c1]].astype(bool), np.float32(1), np.float32(-1))
        y = sym + sigma * rng.standard_normal(sym.shape, dtype=np.float32)
        llr[c0:c1] = (np.float32(100) * y).astype(np.int16)
    return bits, idx, llr


def physical_cpus():
    """One logical CPU per physical core among the CPUs this process may run on (SMT siblings
    from /sys/devices/system/cpu/cpu*/topology/thread_siblings_list)."""
    out, seen = [], set()
    for c in sorted(os.sched_getaffinity(0)):
        try:
            sib = open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c).read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            out.append(c)
    return out


def quiet_cpus(n, sample_s=0.3):
    """n physical cores (one logical CPU each) among this process's CPUs, the least busy first, from two
    /proc/stat samples sample_s apart (a core's load = its busiest SMT sibling). The GPU box shares its
    host's cores with other jobs: a thread pinned to a core another process keeps busy waits behind it
    (r06_s7: the first paced point on CPUs 0-7 saw 35-95 ms stalls without any quota throttling).
    Returns (cpus, busy fraction of each)."""
    def snap():
        out = {}
        try:
            for line in open("/proc/stat"):
                if line.startswith("cpu") and line[3].isdigit():
                    f = line.split()
                    v = [int(x) for x in f[1:]]
                    out[int(f[0][3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
        except OSError:
            pass
        return out
    a = snap()
    time.sleep(sample_s)
    b = snap()
    busy = {}
    for c in os.sched_getaffinity(0):
        if c in a and c in b and b[c][0] > a[c][0]:
            busy[c] = 1.0 - (b[c][1] - a[c][1]) / (b[c][0] - a[c][0])
        else:
            busy[c] = 0.5
    cores = {}
    for c in sorted(busy):
        try:
            sib = open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c).read().strip()
        except OSError:
            sib = str(c)
        cores.setdefault(sib, []).append(c)
    ranked = sorted(cores.values(), key=lambda cs: (max(busy[c] for c in cs), cs[0]))[:n]
    return [cs[0] for cs in ranked], [round(max(busy[c] for c in cs), 3) for cs in ranked]


def ref8_sample(d_in8, d_out, expect, stride, nsample=64):
    """The reference's own 8-bit decoder (srslte_tdec_iteration_8bit, AUTO -> AVX8, oracle/_ref) on
    `nsample` of the 8-bit leg's code blocks (the same int8 LLRs): its bit errors against the
    transmitted bits beside the GPU's on the same blocks, and whether every decision is equal"""
    ref = os.path.join(REPO, "oracle", "_ref", "libsrsref.so")
    if not os.path.exists(ref):
        return None
    lib = ctypes.CDLL(ref)
    fn = lib.ref_tdec8_run
    i8p, u8p = ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(ctypes.c_uint8)
    fn.argtypes = [ctypes.c_int, ctypes.c_int, i8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, u8p]
    ins = d_in8.cpu().numpy().reshape(-1, stride)
    outs = d_out.cpu().numpy()
    idx = np.linspace(0, ins.shape[0] - 1, nsample).astype(int)
    e_ref = e_gpu = same = 0
    for i in idx:
        x = np.ascontiguousarray(ins[i, :3 * K + 12].astype(np.int8))
        dec = np.zeros((NHALF, K // 8), np.uint8)
        if fn(0, 0, x.ctypes.data_as(i8p), x.size, K, NHALF, dec.ctypes.data_as(u8p)) != 0:
            return None
        e_ref += int(np.unpackbits(dec[-1] ^ expect[i]).sum())
        e_gpu += int(np.unpackbits(outs[i] ^ expect[i]).sum())
        same += int((dec[-1] == outs[i]).all())
    return {"code_blocks": int(idx.size), "reference_bit_errors": e_ref, "gpu_bit_errors": e_gpu,
            "identical_decisions": "%d/%d" % (same, idx.size),
            "reference": "oracle/_ref srslte_tdec_iteration_8bit (AUTO -> AVX8), same int8 LLRs"}


def cpu_baseline(llr, nthreads=None):
    """Reference AVX2 AUTO decoder (oracle/_ref, compiled from the reference's own sources) on
    the host cores: one srslte_tdec_t per thread, each thread pinned to its own physical core
    (SURVEY §8(d)), srslte_tdec_run_all over a bounded sample of the same code blocks. Threads =
    every physical core this process may use, capped by the host's CPU share for this job
    (OMP_NUM_THREADS, 16 per GPU on the GPU box) or SRSGPU_CPU_THREADS. Falls back to the scalar
    oracle port if _ref is absent."""
    cores = physical_cpus()
    cap = int(os.environ.get("SRSGPU_CPU_THREADS", os.environ.get("OMP_NUM_THREADS", len(cores))))
    if nthreads is None:
        nthreads = max(1, min(len(cores), cap))
    pin = quiet_cpus(nthreads)[0]  # the least busy physical cores of the shared host
    ref = os.path.join(REPO, "oracle", "_ref", "libsrsref.so")
    port = os.path.join(REPO, "oracle", "liboracle.so")
    kind = "reference" if os.path.exists(ref) else "port"
    lib = ctypes.CDLL(ref if kind == "reference" else port)
    i16p = ctypes.POINTER(ctypes.c_int16)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    if kind == "reference":
        fn = lib.ref_tdec_run_all_many
        fn.argtypes = [ctypes.c_int, i16p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                       ctypes.c_uint32, u8p]

        def work(rows, out):
            fn(0, rows.ctypes.data_as(i16p), rows.shape[1], K, rows.shape[0], NHALF,
               out.ctypes.data_as(u8p))
    else:
        fn = lib.orc_tdec_run
        fn.argtypes = [ctypes.c_int, ctypes.c_int, i16p, ctypes.c_uint32, ctypes.c_uint32, u8p,
                       i16p, i16p]
        dec = np.zeros((NHALF, K // 8), np.uint8)

        def work(rows, out):
            for r in rows:
                fn(0, 0, r.ctypes.data_as(i16p), K, NHALF, dec.ctypes.data_as(u8p), None, None)
    # size the sample to ~20 s of CPU work (thread-seconds): one threaded pass over the batch
    # calibrates, then the timed run repeats it R times
    scratch = np.zeros((1, K // 8), np.uint8)
    work(llr[:1], scratch)  # first call pays the decoder's table set-up
    per_thread = max(1, llr.shape[0] // nthreads)
    outs = [np.zeros((per_thread, K // 8), np.uint8) for _ in range(nthreads)]

    def threaded(reps):
        def thread_fn(i):
            if i < len(pin):
                os.sched_setaffinity(0, {pin[i]})  # Linux: pins the calling thread
            rows = llr[i * per_thread:(i + 1) * per_thread]
            for _ in range(reps):
                work(rows, outs[i])
        ths = [threading.Thread(target=thread_fn, args=(i,)) for i in range(nthreads)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        return time.perf_counter() - t0

    reps = 1
    while True:  # grow R until one timed run holds >= 10 thread-seconds (target 20)
        wall = threaded(reps)
        if wall * nthreads >= 10.0 or reps >= 400:
            break
        reps = int(min(400, max(reps + 1, np.ceil(reps * 20.0 / (wall * nthreads)))))
    ncb = per_thread * nthreads * reps
    return {"value": round(ncb * K / wall / 1e6, 2), "unit": "Mbps", "cores": nthreads,
            "kind": kind, "pinned_cpus": pin, "physical_cores_available": len(cores),
            "sample": "%d CB decodes of K=%d (%d threads x %d CBs x %d passes), %d half-iterations, "
                      "AUTO (AVX2) decoder, natural layout, one srslte_tdec_t per thread, each thread "
                      "pinned to its own physical core (%d physical cores in the affinity set, CPU "
                      "share cap %d), %.1f s wall (%.0f thread-seconds)"
                      % (ncb, K, nthreads, per_thread, reps, NHALF, len(cores), cap, wall,
                         wall * nthreads)}


# ---------------------------------------------------------------- C3 subframe pipeline ----
C3_PRB, C3_CELL, C3_TBS, C3_SF = 100, 1, 75376, 1024   # BASELINE configs[2]: 20 MHz SISO 64QAM


def pipeline_inputs(s, n_sf, rng, nrx=1, nports=1, first=0, noise_seed=None):
    """Subframes first .. first+n_sf-1 of a global job (a rank's contiguous shard), each
    time-domain 20 MHz subframe per rx antenna (N = 2048, 15 N samples): random 64QAM symbols on
    every RE of each layer through frequency-selective channels plus AWGN, built with numpy only ->
    [n_sf][nrx][15 N]. Global subframe i uses template i % 16 (templates drawn from `rng`, the
    same on every rank); the noise is seeded by the shard. The symbols are not codewords, so
    every code block runs the full 8 half-iterations (the fixed-8 throughput case; early stop
    never triggers)."""
    N = s.symbol_sz(C3_PRB, True)
    nsc = 12 * C3_PRB
    k = np.arange(nsc)
    lev = np.array([-7, -5, -3, -1, 1, 3, 5, 7], np.float32) / np.sqrt(42)
    cp0, cp = int(np.ceil(160 * N / 2048)), int(np.ceil(144 * N / 2048))
    ntmpl = 16
    tmpl = np.zeros((ntmpl, nrx, 15 * N), np.complex64)
    for t in range(ntmpl):
        layers = [lev[rng.integers(0, 8, (14, nsc))] + 1j * lev[rng.integers(0, 8, (14, nsc))]
                  for _ in range(nports)]
        for a in range(nrx):
            g = np.zeros((14, nsc), np.complex128)
            for p, lay in enumerate(layers):
                ph = 0.5 + 0.7 * a + 1.3 * p
                h = (1 + 0.3 * np.cos(2 * np.pi * k / nsc + ph)) * np.exp(0.5j * np.sin(2 * np.pi * k / nsc + ph))
                g += lay * h / np.sqrt(nports)
            X = np.zeros((14, N), np.complex64)
            X[:, N - nsc // 2:] = g[:, :nsc // 2]
            X[:, 1:1 + nsc // 2] = g[:, nsc // 2:]
            sym = np.fft.ifft(X, axis=1).astype(np.complex64)
            pos = 0
            for i in range(14):
                c = cp0 if i % 7 == 0 else cp
                tmpl[t, a, pos:pos + c] = sym[i, N - c:]
                tmpl[t, a, pos + c:pos + c + N] = sym[i]
                pos += c + N
    x = tmpl[(first + np.arange(n_sf)) % ntmpl]
    nrng = rng if noise_seed is None else np.random.default_rng(noise_seed)
    x += (1e-3 / np.sqrt(N)) * (nrng.standard_normal(x.shape) + 1j * nrng.standard_normal(x.shape)).astype(np.complex64)
    return N, x


STAGES = ("k_ofdm_rx", "k_chest", "k_gold", "k_pdsch_llr", "k_derm", "k_load", "k_ldderm", "k_rows_late", "k_win_bidir",
          "k_sse_halfit", "k_decide", "k_tb_finish")
# kernels of the coded subframe legs, for the per-kernel table and the roofline of the dominant one
# (names as the library's ProfScope records them; prof_get matches substrings, so the decoder's
# early-stop launches are asked for by their full name)
KERNELS = ("k_ofdm_rx", "k_chest", "k_gold", "k_pdsch_llr", "k_derm", "k_load", "k_ldderm", "k_rows_late",
           "k_win_bidir_h0", "k_win_bidir_es",
           "k_sse_es", "k_es_bytes", "k_win_bidir_run", "k_win_bidir", "k_decide", "k_tb_finish")


_LANE_STREAMS = {}


def lane_stream(torch, dev, li, priority=0):
    """lane li's HIP stream, created once and shared by every leg: each leg then runs on the same
    streams (and so the same hardware queues) as the headline. Fresh streams per leg land on other
    hardware queues of the process (4 on the box), and two lanes on one queue run one after the other.
    priority < 0: a high-priority stream (its hardware queue's dispatches go first)."""
    key = (li, priority)
    if key not in _LANE_STREAMS:
        _LANE_STREAMS[key] = torch.cuda.Stream(dev, priority=priority) if priority else torch.cuda.Stream(dev)
    return _LANE_STREAMS[key]


def stage_profile(s, torch, step, steps, kernels=None):
    """Per-stage device time per batch, from HIP events around every launch (srsgpu_prof_*), in
    a separate pass after the timed loop: creating and recording the events costs host time that
    would otherwise show in the host-bound legs' wall clock. With several streams the spans of
    concurrent launches overlap, so the stage sums then exceed the wall time per batch.
    kernels: also return {name: (total ms per batch, launches per batch)} for these names."""
    s.prof_reset()
    s.prof_enable(True)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    s.prof_enable(False)
    out = {}
    for name in STAGES:
        ms, cnt = s.prof_get(name)
        if cnt:
            out[name] = round(ms / steps, 4)
    if kernels is None:
        return out
    kt = {}
    for name in kernels:
        ms, cnt = s.prof_get(name)
        if cnt:
            kt[name] = (ms / steps, cnt / steps)
    return out, kt


def warm_up(torch, step, warmup, seconds=0.25):
    """The leg's warmup steps, then more until `seconds` of decoding have run: the legs are set up
    on the host for seconds with the GPU idle, and a GPU ramps its clock over the first tens of ms
    of load (the first timed loop after two warmup steps ran up to 1.8x slower than the same steps
    a moment later: profiles/r03_s13_sched_ab.json, ms_per_batch against the schedule rounds). As
    the headline's pre-heat, this times the steady clock of a receiver that decodes continuously."""
    t0 = time.perf_counter()
    n = 0
    while n < warmup or time.perf_counter() - t0 < seconds:
        step()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def schedule_ab(s, torch, step, steps, schedules, reps=3):
    """A/B of decoder launch schedules (srsgpu_tdec_set_schedule; results are identical under all)
    in one process on the same inputs: reps rounds, each timing `steps` steps per schedule in turn
    after one warm-up step; ms per batch per schedule, then the schedule in force before is restored."""
    if not schedules:
        return None
    keep = s.get_schedule()
    res = {name: [] for name in schedules}
    for _ in range(reps):
        for name, sch in schedules.items():
            s.set_schedule(**sch)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            res[name].append(round((time.perf_counter() - t0) / steps * 1e3, 3))
    s.set_schedule(**keep)
    return {name: {"ms_per_batch": v, "median": float(np.median(v))} for name, v in res.items()}


def run_pipeline(s, torch, dev, steps, warmup, tm=1, lanes=2, dist=None, schedules=None):
    """tm 1 — BASELINE configs[2]: one step = 1024 subframes through OFDM FFT -> CRS channel
    estimation -> PDSCH (RE extraction, MMSE, 64QAM demap, descramble) -> DL-SCH (de-RM, turbo
    decoding with CRC early stop up to 8 half-iterations, TB CRC) for TBS 75376 (13 x K=5824).
    tm 3 — the per-GPU shard of BASELINE configs[3]: 1024 TM3 subframes (2 CRS ports, 2 rx
    antennas, CDD 2x2 MMSE, two MCS-28 TBs per subframe) through the same stages.
    lanes: the batch is split over that many HIP streams, each with its own OFDM / estimator /
    PDSCH handles (a worker per stream, as srsUE runs one phch_worker per subframe): one lane's
    front end and small kernels fill the SIMDs the other lane's decoder leaves idle.
    Multi-GPU (BASELINE configs[3] "8192-subframe batch sharded across 8 GPUs"): the
    job is nranks x 1024 subframes, split in contiguous subframe ranges by the native partitioner
    (srsgpu_shard_contiguous, the analogue of srsUE's worker pool handing out whole subframes,
    phy.cc:141-168); every rank synthesises and decodes its own range, then the results of every
    subframe (per TB: return code, nof_iterations, cb_crc, TB bytes) go to rank 0 in one grouped
    send/recv batch (srsgpu_shard.gather_records), timed separately as gather_ms."""
    import srsgpu_shard as sh
    rank = dist.get_rank() if dist else 0
    nranks = dist.get_world_size() if dist else 1
    n_global = C3_SF * nranks
    first = sh.contiguous(n_global, nranks)
    assert first[rank + 1] - first[rank] == C3_SF
    nrx = nports = 2 if tm == 3 else 1
    ntb = 2 if tm == 3 else 1
    rng = np.random.default_rng(99)
    N, x = pipeline_inputs(s, C3_SF, rng, nrx, nports, first=first[rank], noise_seed=1000 + rank)
    gsz = 14 * 12 * C3_PRB
    nsf = C3_SF // lanes
    ngrid = nsf * nrx
    d_x = torch.from_numpy(x.reshape(-1)).to(dev)
    del x
    dlen = C3_TBS // 8 + 6
    sf_idx = [1 + (i % 4) for i in range(nsf)]  # subframes without PSS/SSS/PBCH
    mimo = s.MIMO_CDD if tm == 3 else s.MIMO_SINGLE_ANTENNA
    L = []
    for li in range(lanes):
        st = lane_stream(torch, dev, li) if lanes > 1 else torch.cuda.current_stream(dev)
        o = {"st": st, "x": d_x[li * ngrid * 15 * N:(li + 1) * ngrid * 15 * N]}
        o["ofdm"] = s.OfdmRx(C3_PRB, N, stream=st.cuda_stream)
        o["chest"] = s.Chest(C3_PRB, C3_CELL, max_grids=ngrid, stream=st.cuda_stream, nof_ports=nports)
        o["pd"] = s.Pdsch(C3_PRB, C3_CELL, nof_ports=nports, nof_rx_ant=nrx, nof_softbuffers=nsf * ntb,
                          max_cb=13, max_sf=nsf, stream=st.cuda_stream)
        o["grid"] = torch.zeros(ngrid * gsz, dtype=torch.complex64, device=dev)
        o["ce"] = torch.zeros(ngrid * nports * gsz, dtype=torch.complex64, device=dev)
        o["noise"] = torch.zeros(ngrid * nports, dtype=torch.float32, device=dev)
        o["data"] = torch.zeros(nsf * ntb * dlen, dtype=torch.uint8, device=dev)
        o["ret"] = torch.zeros(nsf * ntb, dtype=torch.int32, device=dev)
        o["noi"] = torch.zeros(nsf * ntb, dtype=torch.int32, device=dev)
        o["pd"].set_noise_dev(o["noise"].data_ptr())
        nre = o["pd"].nof_re(s.make_sf(sf_idx=1, lstart=1, nof_prb=C3_PRB, mod=3))
        sfs = [s.make_sf(sf_idx=sf_idx[i], lstart=1, nof_prb=C3_PRB, mod=(3, 3), nof_re=nre, rnti=1234,
                         tbs=(C3_TBS, C3_TBS), softbuffer=(ntb * i, ntb * i + 1), mimo=mimo,
                         grid_offset=i * nrx * gsz, ce_offset=i * nrx * nports * gsz,
                         data_offset=(ntb * i * dlen, (ntb * i + 1) * dlen))
               for i in range(nsf)]
        grid_sf = [v for v in sf_idx for _ in range(nrx)]
        o["sfs"], o["grid_sf"] = s.make_sf_array(sfs), (ctypes.c_uint32 * len(grid_sf))(*grid_sf)  # built once
        L.append(o)
    torch.cuda.synchronize()

    def step():
        for o in L:
            o["pd"].reset_softbuffer(0, nsf * ntb)  # new TBs: one softbuffer reset pass
            assert o["ofdm"].rx_dev(ngrid, o["x"].data_ptr(), 15 * N, o["grid"].data_ptr(), gsz) == 0
            assert o["chest"].estimate_dev(o["grid_sf"], o["grid"].data_ptr(), gsz, o["ce"].data_ptr(),
                                           o["noise"].data_ptr()) == 0
            assert o["pd"].decode_dev(o["sfs"], o["grid"].data_ptr(), o["ce"].data_ptr(), gsz,
                                      o["data"].data_ptr(), 8, o["ret"].data_ptr(), o["noi"].data_ptr()) == 0

    warm_up(torch, step, warmup)
    if dist:
        dist.barrier()
    gc.disable()  # the host-bound legs must not pay a collector pause inside the timed loop
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    gc.enable()
    stages = stage_profile(s, torch, step, steps)
    ab = schedule_ab(s, torch, step, steps, schedules)
    noi = np.concatenate([o["noi"].cpu().numpy() for o in L])
    # results of this rank's subframes (lane li holds subframes li*nsf .. of the range), one record
    # per subframe = its TBs' records, then the gather to rank 0
    recs = []
    for o in L:
        ret, noiv, data = o["ret"].cpu().numpy(), o["noi"].cpu().numpy(), o["data"].cpu().numpy()
        for i in range(nsf):
            recs.append(np.concatenate([
                sh.pack_tb_record(ret[ntb * i + t], noiv[ntb * i + t],
                                  data[(ntb * i + t) * dlen:(ntb * i + t) * dlen + C3_TBS // 8],
                                  o["pd"].read_cb_crc(ntb * i + t), C3_TBS) for t in range(ntb)]))
    gdev = dev if (dist and dist.get_backend() == "nccl") else torch.device("cpu")  # gloo: host tensors
    local = torch.from_numpy(np.concatenate(recs)).to(gdev)
    gather_ms, gathered = None, None
    if dist:
        owner = np.repeat(np.arange(nranks), np.diff(first))
        sizes = [ntb * sh.tb_record_len(C3_TBS)] * n_global
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        got = sh.gather_records(dist, torch, gdev, owner, sizes, local)
        torch.cuda.synchronize()
        gather_ms = round((time.perf_counter() - tg) * 1e3, 3)
        if got is not None:
            gathered = sum(1 for r in got if r is not None and r.size == sizes[0])
    for o in L:
        for k in ("ofdm", "chest", "pd"):
            o[k].close()
    name = "c3_pdsch_pipeline" if tm == 1 else "c4_tm3_cdd2x2_pipeline"
    return {"workload": "%s_%dsf_20MHz_64QAM_%dx_tbs%d" % (name, C3_SF, ntb, C3_TBS),
            "subframes_per_s": round(C3_SF * steps / el, 1),
            "processing_mbps": round(C3_SF * ntb * steps * C3_TBS / el / 1e6, 1),
            "ms_per_batch": round(el / steps * 1e3, 3), "symbol_size": N, "rx_antennas": nrx,
            "streams": lanes, "nof_iterations_mean": float(noi.mean()), "stage_ms_per_batch": stages,
            "global_subframes": n_global, "partition": {"kind": "contiguous", "balance": 1.0},
            "subframes_this_rank": C3_SF, "gather_ms": gather_ms, "gathered_subframes": gathered,
            "result_bytes_per_rank": int(local.numel()), "schedule_ab": ab,
            "data": "synthetic 64QAM symbols (not codewords: every CB runs the full 8 half-iterations "
                    "and fails its CRC, so this is the fixed-8 processing rate in TB bits per second, "
                    "not decoded Mbps; see c3_coded_sweep for SURVEY 8(d)'s decoded Mbps)"}


def cb_sizes(table, tbs):
    """K of each code block of a TB (cbsegm.c order: C2 blocks of K2, then K1)"""
    C, _c1, K1, C2, K2, _f = table["cbsegm_C_C1_K1_C2_K2_F"][str(tbs)]
    return [K2 if i < C2 else K1 for i in range(C)]


def run_traffic(s, torch, dev, steps, warmup, kind, lanes=2, snr_db=None, dist=None, schedules=None,
                standard_rate=True, early_stop=True, cpu_sample=0, warm_seconds=0.25, rotate=1, tail=0,
                tail_prio=True, fe_split=False):
    """Coded traffic made on the GPU by the transmit chain (srsgpu_traffic.MixedCells), received
    with CRC early stop (max 8 half-iterations, srsUE's default):
    kind "c5" — BASELINE configs[4] per-GPU shard: 1024 subframes per GPU interleaved over cells of
      6/25/50/100 PRB, random allocation and MCS 0..28 (K 40..6144), all cells' TBs in one
      DL-SCH call per stream; AWGN at 20 dB.
    kind "c3_coded" — the C3 subframe (100 PRB, MCS 28, TBS 75376) as real codewords at snr_db
      (default 30 dB, the operating point of a loaded 20 MHz cell) rather than the fixed-8 worst
      case.
    Multi-GPU: the job is nranks x 1024 subframes, planned identically on every
    rank (srsgpu_traffic.plan) and split by the native partitioner: C5 by decoding cost from one
    global longest-first queue, C3 in contiguous ranges. After the timed loop the results of every
    rank (TB bytes, return code, nof_iterations, cb_crc) go to rank 0 in one grouped send/recv
    batch (srsgpu_shard.gather_records), timed separately as gather_ms.
    lanes: a rank's subframes are split over that many HIP streams (run_pipeline).
    decoded_mbps is SURVEY §8(d)'s metric: the sum of K over CRC-passing code blocks per second.
    standard_rate False: srsLTE's 1536-point FFT at 20 MHz instead of 2048. early_stop False: every
    code block runs all 8 half-iterations (srsgpu_dlsch_set_early_stop, the fixed-8 rate on real
    codewords). cpu_sample > 0: the first cpu_sample received resource grids of lane 0 (after the
    FFT) come back as host arrays for the CPU baseline ("_cpu_grids", "_cpu_sf_idx").
    rotate R > 1: successive steps cycle through R descriptor sets with different softbuffers
    (MixedCells rotate), so the PDSCH / DL-SCH repeat-call caches never hit and every step pays the
    per-code-block host work a receiver with changing grants pays. host_ms_per_step is the host
    time spent inside the step calls (enqueue side; the GPU runs asynchronously).
    tail 1 / 2: each lane alternates between two DL-SCH engines whose early-stop tails run on a tail
    stream (srsgpu_dlsch_set_tail_stream; 1: one tail stream shared by the lanes, 2: one per lane), so
    a lane's next batch starts while the last one's straggling code blocks finish; tail_prio: the tail
    streams are high-priority streams; fe_split: each lane's front end on a stream of its own."""
    import srsgpu_shard as sh
    import srsgpu_traffic as tr
    rank = dist.get_rank() if dist else 0
    nranks = dist.get_world_size() if dist else 1
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    n_global = C3_SF * nranks
    if kind == "c5":
        snr, seed, kw = (20.0 if snr_db is None else snr_db), 21, {}
        sf_plan = tr.plan(table, n_global, seed=seed)
        owner, load = sh.weighted(tr.tb_weights(table, sf_plan), nranks)
        part = {"kind": "weighted (global longest-first queue over sum K x 8)", "balance": sh.balance(load)}
    else:
        snr, seed, kw = (30.0 if snr_db is None else snr_db), 22, dict(prbs=(100,), mcs=28, full_band=True)
        sf_plan = tr.plan(table, n_global, seed=seed, **kw)
        f = sh.contiguous(n_global, nranks)
        owner = np.repeat(np.arange(nranks), np.diff(f))
        part = {"kind": "contiguous", "balance": 1.0}
    mine = [i for i in range(n_global) if owner[i] == rank]
    ms = []
    for li in range(lanes):
        st = (lane_stream(torch, dev, li) if lanes > 1 else torch.cuda.current_stream(dev)).cuda_stream
        tk = {}
        if tail:
            # tail_prio: the tail streams at high priority (their straggler workgroups dispatched first)
            tp = -1 if tail_prio else 0
            tk = dict(engines=2, tail_stream=lane_stream(torch, dev, "tail" if tail == 1 else "tail%d" % li,
                                                         priority=tp).cuda_stream)
            if fe_split:  # the front end on a stream of its own (MixedCells fe_stream)
                tk["fe_stream"] = lane_stream(torch, dev, "fe%d" % li).cuda_stream
        ms.append(tr.MixedCells(table, n_global, torch, dev, seed=seed, stream=st, snr_db=snr,
                                keep=mine[li::lanes], standard_rate=standard_rate, early_stop=early_stop,
                                rotate=rotate, **tk, **kw))  # one plan: the same seed everywhere
    torch.cuda.synchronize()

    def step():
        for m in ms:
            m.step()

    warm_up(torch, step, warmup, warm_seconds)
    if dist:
        dist.barrier()
    gc.disable()
    host = 0.0
    for m in ms:
        m.host_s = [0.0, 0.0]
    t0 = time.perf_counter()
    for _ in range(steps):
        th = time.perf_counter()
        step()
        host += time.perf_counter() - th
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    gc.enable()
    host_split = [sum(m.host_s[i] for m in ms) for i in (0, 1)]
    stages, ktab = stage_profile(s, torch, step, steps, KERNELS)
    ab = schedule_ab(s, torch, step, steps, schedules)
    chk = [m.check() for m in ms]
    # decoder work of the last batch: the half-iterations each code block ran (srsgpu_dlsch_cb_halfits)
    # weighted by its K, for the VALU roofline of the whole decoder (first + early-stop launches)
    # (one block size only: the decoder's block order groups blocks by K, not by TB)
    halfit_bits = 0
    for m in ms:
        h = m.dlsch.cb_halfits()
        ks_cb = [k for t in m.tb_list for k in cb_sizes(table, t["tbs"])]
        assert len(ks_cb) == h.size, (len(ks_cb), h.size)
        if halfit_bits is None or len(set(ks_cb)) != 1:
            halfit_bits = None
            continue
        halfit_bits += int(h.astype(np.int64).sum()) * ks_cb[0]
    acks, good = sum(c[0] for c in chk), sum(c[1] for c in chk)
    noi = float(np.mean([c[2] for c in chk]))
    tbl = [t for m in ms for t in m.tb_list]
    ks = sorted({int(table["cbsegm_C_C1_K1_C2_K2_F"][str(t["tbs"])][2]) for t in tbl})
    bits = sum(m.bits for m in ms)
    cb_bits = sum(m.decoded_bits(table) for m in ms)
    acked_bits = sum(t["tbs"] for m in ms for t, r in zip(m.tb_list, m.d_ret.cpu().numpy()) if r == 0)
    # gather of the results to rank 0 (RCCL grouped send/recv on the GPU box)
    recs = {}
    for m in ms:
        ret, noiv, data = m.d_ret.cpu().numpy(), m.d_noi.cpu().numpy(), m.d_data.cpu().numpy()
        for t, r, n in zip(m.tb_list, ret, noiv):
            o = t["data_offset"]
            recs[t["sf"]] = sh.pack_tb_record(r, n, data[o:o + t["tbs"] // 8], m.dlsch.read_cb_crc(m.softbuffer_of(t)),
                                              t["tbs"])
    gdev = dev if (dist and dist.get_backend() == "nccl") else torch.device("cpu")  # gloo: host tensors
    local = torch.from_numpy(np.concatenate([recs[i] for i in mine])).to(gdev)
    sizes = [sh.tb_record_len(p["tbs"]) for p in sf_plan]
    gather_ms = None
    if dist:
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        sh.gather_records(dist, torch, gdev, owner, sizes, local)
        torch.cuda.synchronize()
        gather_ms = round((time.perf_counter() - tg) * 1e3, 3)
    out = {"workload": ("c5_mixed_bw_%dsf_per_gpu_6-25-50-100prb_mcs0-28" % C3_SF if kind == "c5" else
                        "c3_coded_%dsf_per_gpu_20MHz_64QAM_tbs%d" % (C3_SF, C3_TBS)),
           "snr_db": snr, "subframes_per_s": round(len(mine) * steps / el, 1),
           "decoded_mbps": round(cb_bits * steps / el / 1e6, 1),
           "acked_tb_mbps": round(acked_bits * steps / el / 1e6, 1),
           "offered_tb_mbps": round(bits * steps / el / 1e6, 1), "ms_per_batch": round(el / steps * 1e3, 3),
           "streams": lanes, "code_blocks": sum(m.ncb for m in ms), "distinct_K": len(ks),
           "K_range": [ks[0], ks[-1]], "acked_tbs": acks, "tbs_bytes_ok": good, "tbs": len(tbl),
           "nof_iterations_mean": noi, "stage_ms_per_batch": stages, "partition": part,
           "subframes_this_rank": len(mine), "gather_ms": gather_ms,
           "result_bytes_per_rank": int(local.numel()), "schedule_ab": ab,
           "symbol_size": ms[0].cells[0]["N"], "early_stop": early_stop,
           "host_ms_per_step": round(host / steps * 1e3, 3), "descriptor_sets": rotate,
           "halfit_bits_per_batch": halfit_bits,
           "host_ms_front_end": round(host_split[0] / steps * 1e3, 3),
           "host_ms_dlsch": round(host_split[1] / steps * 1e3, 3),
           "kernels_per_batch": {k: {"ms": round(v[0], 4), "launches": v[1]} for k, v in ktab.items()},
           "data": "synthetic coded subframes (GPU transmitter, AWGN %s dB)" % snr}
    if cpu_sample:
        c = ms[0].cells[0]
        n = min(cpu_sample, c["n"])
        out["_cpu_grids"] = c["grid"][:n * c["gsz"]].cpu().numpy().reshape(n, c["gsz"])
        out["_cpu_sf_idx"] = [int(c["sf_idx"][i]) for i in range(n)]
    for m in ms:
        m.close()
    return out


def run_tm3_coded(s, torch, dev, steps, warmup, snr_db=30.0, lanes=2, dist=None):
    """BASELINE configs[3] per-GPU shard as real codewords: 1024 TM3 subframes per GPU (20 MHz, 2 CRS
    ports, 2 rx antennas, large-delay CDD with two MCS-28 TBs of TBS 75376 = 26 code blocks per
    subframe) from the GPU transmitter (srsgpu_traffic.MimoSubframes: pdsch_encode_ports, CRS of both
    ports, OFDM TX, a 2x2 flat channel, AWGN at snr_db). Timed step: OFDM FFT of both antennas, channel
    estimation of both ports on each antenna, CDD 2x2 MMSE PDSCH and DL-SCH with CRC early stop (max 8
    half-iterations). Multi-GPU: the job is nranks x 1024 subframes in contiguous ranges (subframe i's
    content depends only on i); no data-path collective. decoded_mbps = sum of K over CRC-passing
    code blocks per second, whole job over the slowest rank's time."""
    import srsgpu_shard as sh
    import srsgpu_traffic as tr
    rank = dist.get_rank() if dist else 0
    nranks = dist.get_world_size() if dist else 1
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    n_global = C3_SF * nranks
    f = sh.contiguous(n_global, nranks)
    mine = list(range(int(f[rank]), int(f[rank + 1])))
    ms = []
    for li in range(lanes):
        st = (lane_stream(torch, dev, li) if lanes > 1 else torch.cuda.current_stream(dev)).cuda_stream
        ms.append(tr.MimoSubframes(torch, dev, n_global, seed=5, stream=st, snr_db=snr_db, keep=mine[li::lanes]))
    torch.cuda.synchronize()

    def step():
        for m in ms:
            m.step()

    warm_up(torch, step, warmup, 0.5)
    if dist:
        dist.barrier()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    gc.enable()
    stages, ktab = stage_profile(s, torch, step, steps, KERNELS)
    chk = [m.check() for m in ms]
    acks, good = sum(c[0] for c in chk), sum(c[1] for c in chk)
    noi = float(np.mean([c[2] for c in chk]))
    cb_bits = sum(m.decoded_bits(table) for m in ms)
    ntb = sum(m.ntb * m.n for m in ms)
    el_job, _ = reduce_over_ranks(dist, dev, el, 0)
    bits_job, _ = reduce_over_ranks(dist, dev, float(cb_bits), 0, op="sum")
    acked_job, _ = reduce_over_ranks(dist, dev, float(acks * C3_TBS), 0, op="sum")
    for m in ms:
        m.close()
    return {"workload": "c3_tm3_coded_%dsf_per_gpu_20MHz_2x2_cdd_64QAM_2x_tbs%d" % (C3_SF, C3_TBS),
            "baseline_config": "BASELINE configs[3] (per-GPU shard)", "snr_db": snr_db,
            "decoded_mbps": round(bits_job * steps / el_job / 1e6, 1),
            "acked_tb_mbps": round(acked_job * steps / el_job / 1e6, 1),
            "subframes_per_s": round(n_global * steps / el_job, 1), "ms_per_batch": round(el_job / steps * 1e3, 3),
            "streams": lanes, "tbs": ntb, "acked_tbs": acks, "tbs_bytes_ok": good, "nof_iterations_mean": noi,
            "code_blocks_per_subframe": 26, "stage_ms_per_batch": stages,
            "kernels_per_batch": {k: {"ms": round(v[0], 4), "launches": v[1]} for k, v in ktab.items()},
            "partition": "contiguous", "data": "synthetic coded TM3 subframes (GPU transmitter, 2x2 flat channel, "
                                               "AWGN %.0f dB)" % snr_db}


def reduce_over_ranks(dist, dev, elapsed, bit_errors, op="max"):
    """Job time = the slowest rank's timed region (it is bracketed by barriers); bit errors are
    summed (op="sum" sums the first value too). Identity on a single process."""
    if not dist:
        return elapsed, bit_errors
    import torch
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    e = torch.tensor([bit_errors], device=dev, dtype=torch.int64)
    dist.all_reduce(e)
    return float(t.item()), int(e.item())


def decoded_mbps(nranks, ncb, k, steps, elapsed):
    """Whole-job decoded Mbps: every rank decodes its own ncb code blocks per step (weak scaling)."""
    return nranks * ncb * k * steps / elapsed / 1e6


def load_profile_json(workload, tag="pmc_traffic"):
    """Per-launch figures of the dominant kernel from a committed profile summary
    (profiles/*<tag>*.json): HBM bytes from rocprofv3 FETCH/WRITE passes (tools/pmc_traffic.py),
    or VALU instructions per launch and the measured packed-int16 issue peak (tag "valu")."""
    pdir = os.path.join(REPO, "profiles")
    best = None
    if os.path.isdir(pdir):
        # natural order (r02_s13 after r02_s7): the newest matching record wins
        natural = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]
        for f in sorted(os.listdir(pdir), key=natural):
            if tag in f and f.endswith(".json"):
                try:
                    d = json.load(open(os.path.join(pdir, f)))
                except Exception:
                    continue
                if d.get("workload") == workload:
                    best = dict(d, source="profiles/" + f)  # the committed file the figures come from
    return best


def dci_blind_decode(s, torch, steps, nsf=1024, per_sf=44):
    """PDCCH blind decoding: per subframe srsUE tries up to 44 candidates
    (common + UE-specific search spaces over the aggregation levels, two DCI sizes); each is
    srslte_pdcch_decode_msg's candidate decode (mean check, srslte_rm_conv_rx, tail-biting Viterbi
    of nof_bits + 16, CRC16 remainder). nsf subframes' candidates per launch (srsgpu_dci_decode_dev),
    random LLRs of the PDCCH formats, 20 MHz DCI sizes (1A / 1: 27 / 31 bits)."""
    rng = np.random.default_rng(3)
    n = nsf * per_sf
    Ls = rng.choice([72, 144, 288, 576], n)
    nbs = rng.choice([27, 31], n)
    arr = (s.srsgpu_dci_cand_t * n)()
    lo = oo = 0
    for i in range(n):
        arr[i].llr_offset, arr[i].out_offset, arr[i].E, arr[i].nof_bits = lo, oo, int(Ls[i]), int(nbs[i])
        lo += int(Ls[i])
        oo += int(nbs[i]) + 16
    llr = (rng.standard_normal(lo) + np.where(rng.random(lo) < 0.5, 1.0, -1.0)).astype(np.float32)
    d_c = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    d_llr = torch.from_numpy(llr).cuda()
    d_out = torch.zeros(oo, dtype=torch.uint8, device="cuda")
    d_crc = torch.zeros(n, dtype=torch.int16, device="cuda")
    d_dec = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()

    def step():
        if s._lib.srsgpu_dci_decode_dev(s._vp(d_c.data_ptr()), n, s._vp(d_llr.data_ptr()),
                                        s._vp(d_out.data_ptr()), s._vp(d_crc.data_ptr()),
                                        s._vp(d_dec.data_ptr()), s._vp(st)) != 0:
            raise RuntimeError("srsgpu_dci_decode_dev failed")

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"workload": "pdcch_dci_blind_decode_%dsf_x%d_candidates" % (nsf, per_sf),
            "candidates_per_launch": n, "ms_per_launch": round(el / steps * 1e3, 3),
            "candidates_per_s": round(n * steps / el, 1),
            "subframes_per_s": round(nsf * steps / el, 1),
            "decoded_fraction": round(float(d_dec.float().mean().item()), 3)}


# registered-sample ingest of the queue (srsgpu_rxq, rx_queue.hip stage()): DMA from the caller's
# memory on the copy stream (default), or the ingest kernel reading the samples over the bus
INGEST_VARIANTS = {"dma": {}, "busread": {"SRSGPU_RXQ_INGEST": "kernel"}}


def cpu_probe():
    """(wall s, this process's CPU s, cgroup throttled usec, cgroup nr_throttled): the GPU box gives a
    command a CFS quota (/sys/fs/cgroup/cpu.max, 16 CPUs over 256 visible cores), so a process that
    burns more than its quota in a 100 ms period stalls every thread until the next one"""
    import resource
    r = resource.getrusage(resource.RUSAGE_SELF)
    thr = nr = None
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k == "throttled_usec":
                thr = int(v)
            elif k == "nr_throttled":
                nr = int(v)
    except OSError:
        pass
    return time.perf_counter(), r.ru_utime + r.ru_stime, thr, nr


def cpu_delta(a, b):
    """CPU use between two cpu_probe() samples: cores busy on average, ms of quota throttling"""
    out = {"cpu_cores_busy": round((b[1] - a[1]) / max(b[0] - a[0], 1e-9), 2)}
    if a[2] is not None and b[2] is not None:
        out["cgroup_throttled_ms"] = round((b[2] - a[2]) / 1e3, 1)
        out["cgroup_nr_throttled"] = b[3] - a[3]
    return out


def cpu_quota():
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def paced_record(lat, slat, status, acked, late, ns, ticks, nb, done, tmg, budget_ms, sf_bytes):
    """one paced point: latency from the tick (what the HARQ budget sees) and from the actual submission
    (the queue's own latency, without the producer threads' lateness behind the tick)"""
    ok = slat >= 0
    p99 = float(np.percentile(lat, 99))
    rec = {"latency_ms_p50": round(float(np.percentile(lat, 50)), 3), "latency_ms_p99": round(p99, 3),
           "latency_ms_max": round(float(lat.max()), 3),
           "submit_latency_ms_p50": round(float(np.percentile(slat[ok], 50)), 3) if ok.any() else None,
           "submit_latency_ms_p99": round(float(np.percentile(slat[ok], 99)), 3) if ok.any() else None,
           "producer_late_ms_max": round(late, 3),
           "producer_late_ms_p99": round(float(np.percentile(lat[ok] - slat[ok], 99)), 3) if ok.any() else None,
           "acked": "%d/%d" % (acked, ns * ticks), "failed": int((status != 0).sum()),
           "mean_batch": round(done / max(nb, 1), 1), "subframes_per_s": round(ns * 1000.0, 1),
           "dispatcher_us_per_sf": {k: round(v / max(done, 1) * 1e6, 3) for k, v in tmg.items()},
           "ingest_GBps": round(ns * 1000.0 * sf_bytes / 1e9, 2)}
    rec["within_budget"] = bool(p99 <= budget_ms and rec["failed"] == 0 and acked == ns * ticks)
    rec["worst_tick"] = int(np.argmax(lat)) // ns  # where the largest latency fell in the run
    return rec


def rx_queue_leg(s, torch, dev, nsf=4096, batches=(256, 1024), producers=8, snr_db=30.0, min_batches=16,
                 paced_streams=(32, 64, 128, 192, 256, 320, 384, 448, 512, 640), ticks=300, depth=3,
                 budget_ms=3.0, paced_fft=(2048, 1536), paced_workers=4):
    """The real srsUE caller path: host threads hand single time-domain C3
    subframes (20 MHz, MCS 28 codewords from the GPU transmitter at snr_db, copied to host memory
    once) to the subframe batch queue (include/srsgpu/rx_queue.h). The threads are native
    (srsgpu_rxq_drive / _drive_paced_ex), as srsUE's PHY workers are.

    Host memory: the samples a queue reads in place and the TB outputs the decoder writes in place lie
    in queue-owned blocks (srsgpu_rxq_alloc_host), filled from the caller's arrays and freed by the
    queue; the caller's own memory is never pinned (the r05_s39 / r05_s46 fault followed
    the free of caller memory the queue had pinned).

    saturated: `producers` threads submit max(nsf, min_batches * B) subframes as fast as the queue
    takes them (at least min_batches batches: the pipeline's first transfer and last decode do not
    overlap anything), per batch size and ingest mode — staged (each submission copies its samples
    into the queue's pinned staging, then one DMA per batch), zero-copy (the samples lie in a
    queue-owned block: DMA'd from there, one copy per run of address-contiguous subframes), zero-copy
    SC16 (the radio's int16 I/Q, half the bytes, converted on the GPU) and zero-copy SC16 bus-read
    (the batch's ingest kernel reads the samples over PCIe in place, SRSGPU_RXQ_INGEST=kernel).
    ingest_GBps = sample bytes handed over / wall time.

    paced: N streams each hand over one SC16 subframe per 1 ms TTI (srsgpu_rxq_drive_paced_ex,
    zero-copy, batch = N, depth HARQ slots per stream) for `ticks` TTIs, at the 3GPP 2048-point rate
    and at srsLTE's default 1536-point rate (phy_common.c:37-41, 25 % fewer bytes). The queue's three
    threads, the collector and `paced_workers` producers are pinned to distinct physical cores.
    latency = results written - TTI start (the HARQ budget's view) and - actual submission (the
    queue's own); real_time_streams = the largest N whose p99 latency from the tick is within
    budget_ms with every TB acked (the sweep stops at the second miss in a row; srsUE must send the
    HARQ ACK in subframe n + 4: HARQ_DELAY_MS, lib/include/srslte/common/common.h:49, leaving ~3 ms
    for the decode). The first miss is kept whole in `first_miss`."""
    import srsgpu_traffic as tr
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    srcs = {}
    for fft in sorted(set((2048,) + tuple(paced_fft))):
        m = tr.MixedCells(table, 1024, torch, dev, seed=22, snr_db=snr_db, prbs=(100,), mcs=28, full_band=True,
                          standard_rate=(fft == 2048))
        c = m.cells[0]
        assert c["N"] == fft, (c["N"], fft)
        x_cf = c["x"].cpu().numpy().reshape(c["n"], 15 * fft)
        base = c["sfs"]
        m.close()
        torch.cuda.synchronize()
        scale = float(np.abs(x_cf.view(np.float32)).max()) / 32000.0
        x_sc = np.round(x_cf.view(np.float32) / scale).astype(np.int16)  # [n_src][15 N * 2]
        srcs[fft] = {"cf": x_cf, "sc": x_sc, "scale": scale, "sfs": base, "n": c["n"]}
    # the queue's closer / dispatcher / completer, then the collector and the producers (paced), each on
    # its own physical core, the least busy ones of the host
    cpus, cpu_busy = quiet_cpus(4 + paced_workers)
    q_cpus, d_cpus = cpus[:3], cpus[3:4 + paced_workers] or cpus[:1]
    out = {"workload": "c3_coded_queue_20MHz_64QAM_tbs%d" % C3_TBS, "snr_db": snr_db,
           "producers": producers, "saturated": {}, "paced": {},
           "host_memory": "queue-owned (srsgpu_rxq_alloc_host)",
           "cpus": {"available": len(os.sched_getaffinity(0)), "physical": len(physical_cpus()), "quota": cpu_quota(),
                    "queue_threads": q_cpus, "paced_threads": d_cpus, "busy_when_chosen": cpu_busy}}

    def owned(q, x):
        """the caller's sample ring in queue-owned device-visible memory"""
        a = q.alloc_host(x.shape, x.dtype)
        a[...] = x
        return a

    def make_items(q, count, nsb, src, sfs, n_src):
        """TB outputs in one queue-owned block: the decoder writes the TB bytes into it over PCIe"""
        dl = (C3_TBS // 8 + 6 + 63) // 64 * 64
        block = q.alloc_host((nsb, dl), np.uint8)
        outs = [block[k, :C3_TBS // 8 + 6] for k in range(nsb)]
        items = []
        for i in range(count):
            j = i % n_src
            sf = sfs[j]
            sf.softbuffer[0] = i % nsb
            items.append(q.item([src[j]], sf, [outs[i % nsb]]))
        return items, outs, block

    def queue(variant, *a, **kw):
        """a queue under one registered-ingest variant (the env is read when the queue is created)"""
        env = INGEST_VARIANTS[variant]
        os.environ.update(env)
        try:
            q = s.RxQueue(*a, **kw)
        finally:
            for k in env:
                os.environ.pop(k, None)
        q.set_affinity(q_cpus)
        return q

    # BENCH_RXQ_VARIANTS=a,b: only these ingest variants (diagnosis runs)
    variants = [v for v in os.environ.get("BENCH_RXQ_VARIANTS", ",".join(INGEST_VARIANTS)).split(",") if v]
    sf_bytes = {"cf32": 8 * 15 * 2048, "sc16": 4 * 15 * 2048}
    S = srcs[2048]
    for B in batches:
        modes = [("staged", "dma"), ("zero_copy", "dma")] + [("zero_copy_sc16", v) for v in variants]
        for mode, variant in modes:
            print("rx_queue: saturated %s %s b%d" % (mode, variant, B), file=sys.stderr, flush=True)
            q = queue(variant, C3_PRB, 1, 2048, nof_softbuffers=4 * B, max_batch=B, max_wait_us=2000)
            x = S["sc"] if "sc16" in mode else S["cf"]
            if "sc16" in mode:
                q.set_input_format(q.SC16, S["scale"])
            src = x if mode == "staged" else owned(q, x)
            count = max(nsf, min_batches * B)
            items, outs, block = make_items(q, count, 4 * B, src, S["sfs"], S["n"])
            warm = [q.submit(items[i]) for i in range(min(B, count))]
            q.flush()
            assert all(q.wait(t) == 0 for t in warm)
            nb0, done0 = q.stats()
            c0 = cpu_probe()
            t0 = time.perf_counter()
            t_sub, t_done, status = q.drive(items, producers, reuse=4 * B)
            el = time.perf_counter() - t0
            c1 = cpu_probe()
            nb, done = q.stats()
            nb, done = nb - nb0, done - done0
            lat = (t_done - t_sub) * 1e3
            acked = sum(1 for it in items[-min(count, 4 * B):] if it.ret[0] == 0)
            zc, st = q.ingest_stats()
            tmg = q.timing()
            key = "%s_b%d" % (mode, B) if mode != "zero_copy_sc16" or variant == "dma" else \
                "%s_%s_b%d" % (mode, variant, B)
            out["saturated"][key] = {
                "dispatcher_us_per_sf": {k: round(v / max(done, 1) * 1e6, 3) for k, v in tmg.items()},
                "subframes": count, "subframes_per_s": round(count / el, 1),
                "ingest_GBps": round(count * sf_bytes["sc16" if "sc16" in mode else "cf32"] / el / 1e9, 2),
                "latency_ms_p50": round(float(np.percentile(lat, 50)), 3),
                "latency_ms_p99": round(float(np.percentile(lat, 99)), 3),
                "mean_batch": round(done / max(nb, 1), 1), "failed": int((status != 0).sum()),
                "zero_copy_rows": zc, "staged_rows": st, "ingest": variant,
                "acked_of_last": "%d/%d" % (acked, min(count, 4 * B)), **cpu_delta(c0, c1)}
            del items, outs, block, src  # views of the queue's blocks: gone before the queue frees them
            q.close()
            torch.cuda.synchronize()  # a fault of this queue's work is reported here, not by the next one
    # paced real-time streams (zero-copy SC16 by DMA), per FFT size
    for fft in paced_fft:
        S = srcs[fft]
        key = "paced" if fft == 2048 else "paced_%d" % fft
        paced = out.setdefault(key, {})
        best, best_q, misses, first_miss = 0, 0, 0, None

        def point(ns):
            q = queue("dma", C3_PRB, 1, fft, nof_softbuffers=ns * depth, max_batch=ns, max_wait_us=800)
            q.set_input_format(q.SC16, S["scale"])
            src = owned(q, S["sc"])
            items, outs, block = make_items(q, ns * depth, ns * depth, src, S["sfs"], S["n"])
            warm = [q.submit(items[i]) for i in range(ns)]
            q.flush()
            assert all(q.wait(t) == 0 for t in warm)
            nb0, done0 = q.stats()
            c0 = cpu_probe()
            lat, slat, status, acked, late = q.drive_paced_ex(items, ns, depth, ticks, 1000,
                                                              workers=min(paced_workers, ns), cpus=d_cpus)
            c1 = cpu_probe()
            nb, done = q.stats()
            rec = paced_record(lat, slat, status, acked, late, ns, ticks, nb - nb0, done - done0, q.timing(),
                               budget_ms, 4 * 15 * fft)
            rec.update(cpu_delta(c0, c1))
            del items, outs, block, src
            q.close()
            torch.cuda.synchronize()
            return rec

        # an unrecorded first point: the sweep's first queue met one-time stalls of 35-95 ms (r06_s7)
        print("rx_queue: paced N=%d warm-up" % fft, file=sys.stderr, flush=True)
        warm_rec = point(paced_streams[0])
        paced["warm_up"] = {k: warm_rec[k] for k in ("latency_ms_p99", "producer_late_ms_max", "worst_tick")}
        for ns in paced_streams:
            print("rx_queue: paced N=%d %d streams" % (fft, ns), file=sys.stderr, flush=True)
            rec = point(ns)
            attempts = []
            while not rec["within_budget"] and (rec["producer_late_ms_p99"] or 0) > 1.0 and len(attempts) < 2:
                # the load generator fell behind its ticks (the producer threads descheduled on a shared
                # host): measured again, at most twice, every attempt kept
                attempts.append({k: rec[k] for k in ("latency_ms_p99", "submit_latency_ms_p99", "producer_late_ms_max",
                                                     "producer_late_ms_p99", "worst_tick")})
                rec = point(ns)
            if attempts:
                rec["earlier_attempts"] = attempts
            paced[str(ns)] = rec
            if rec["failed"] == 0 and rec["acked"] == "%d/%d" % (ns * ticks, ns * ticks) and \
                    (rec["submit_latency_ms_p99"] or 1e9) <= budget_ms:
                best_q = max(best_q, ns)
            if rec["within_budget"]:
                misses = 0
                best = max(best, ns)
            else:
                # a miss can be a host hiccup (the shared host stalled this process for 30-90 ms in
                # r06_s7 / r06_s8 at 32 streams, with every later point met): the sweep stops at the
                # second miss in a row once some N has met the budget; real_time_streams is the largest
                # N that met it
                misses += 1
                if first_miss is None:
                    first_miss = dict(rec, streams=ns)
                if misses >= 2 and best > 0:
                    break
        out["real_time_streams" if fft == 2048 else "real_time_streams_%d" % fft] = best
        # the queue's own capacity: latency from each subframe's actual submission within the budget
        out["queue_streams" if fft == 2048 else "queue_streams_%d" % fft] = best_q
        out["first_miss" if fft == 2048 else "first_miss_%d" % fft] = first_miss
    out["paced_cfg"] = {"ticks": ticks, "tti_us": 1000, "depth": depth, "input": "sc16 zero-copy (DMA)",
                        "batch": "one TTI of all streams", "p99_budget_ms": budget_ms, "producers": paced_workers,
                        "fft": list(paced_fft)}
    return out


def pcfich_cfi(s, torch, steps, nsf=4096, nof_prb=100):
    """PCFICH CFI detection: srslte_pcfich_decode_multi for nsf subframes of
    a 20 MHz 2-port cell with 2 rx antennas (transmit diversity) per launch (srsgpu_pcfich_decode_dev),
    random grids and estimates laid out as the receiver's full subframe planes. Per call: the
    descriptor fill and upload and the launch; the API waits only for the previous call's
    descriptor upload (it reuses its pinned descriptor buffer)."""
    rng = np.random.default_rng(4)
    stride, nrx, nports = nof_prb * 12 * 14, 2, 2
    n0 = nof_prb * 12
    grid = torch.zeros((nsf, nrx, stride, 2), dtype=torch.float32, device="cuda")
    ce = torch.zeros((nsf, nrx * nports, stride, 2), dtype=torch.float32, device="cuda")
    grid[:, :, :n0] = torch.from_numpy(rng.standard_normal((nsf, nrx, n0, 2)).astype(np.float32)).cuda()
    ce[:, :, :n0] = torch.from_numpy(rng.standard_normal((nsf, nrx * nports, n0, 2)).astype(np.float32)).cuda()
    d_cfi = torch.zeros(nsf, dtype=torch.int32, device="cuda")
    d_corr = torch.zeros(nsf, dtype=torch.float32, device="cuda")
    q = s.Pcfich(nof_prb, 1, nports, nrx)
    sfs = [(i * nrx * stride, i * nrx * nports * stride, i % 10, 0.01) for i in range(nsf)]
    sfs = (q.make_sf_array(sfs), nsf)  # the host descriptor array a caller keeps between subframes
    st = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()

    def step():
        if q.decode_dev(sfs, grid.data_ptr(), ce.data_ptr(), stride, d_cfi.data_ptr(), d_corr.data_ptr(), st) != 0:
            raise RuntimeError("srsgpu_pcfich_decode_dev failed")

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    del grid, ce
    return {"workload": "pcfich_cfi_%dsf_%dprb_2ports_2rx" % (nsf, nof_prb),
            "ms_per_launch": round(el / steps * 1e3, 3), "subframes_per_s": round(nsf * steps / el, 1)}


def pdcch_receive(s, torch, steps, nsf=1024, nof_prb=100):
    """The PDCCH receive of srslte_ue_dl_decode_rnti for nsf subframes of a
    20 MHz 2-port cell with 2 rx antennas: srslte_pdcch_extract_llr_multi (transmit diversity, one
    launch for all subframes, srsgpu_pdcch_extract_llr_dev) and the srslte_ue_dl_find_dl_dci search
    for a C-RNTI (TM3: 1A and 2A in the UE-specific space, 1A in the common space) and the SI-RNTI
    (1A and 1C in the common space) per subframe (srsgpu_pdcch_find_dl_dci_dev: host candidate lists,
    one decode launch for every candidate, one selection launch). Random grids: nothing is found, so
    every candidate is decoded and every search runs to its end (the search's worst case)."""
    rng = np.random.default_rng(5)
    stride, nrx, nports = nof_prb * 12 * 14, 2, 2
    n3 = 3 * nof_prb * 12
    grid = torch.zeros((nsf, nrx, stride, 2), dtype=torch.float32, device="cuda")
    ce = torch.zeros((nsf, nrx * nports, stride, 2), dtype=torch.float32, device="cuda")
    grid[:, :, :n3] = torch.from_numpy(rng.standard_normal((nsf, nrx, n3, 2)).astype(np.float32)).cuda()
    ce[:, :, :n3] = torch.from_numpy(rng.standard_normal((nsf, nrx * nports, n3, 2)).astype(np.float32)).cuda()
    q = s.Pdcch(nof_prb, 1, nports, nrx, 0, 1)
    llr_stride = 72 * 128
    d_llr = torch.zeros(nsf * llr_stride, dtype=torch.float32, device="cuda")
    sfs = [(i * nrx * stride, i * nrx * nports * stride, i * llr_stride, i % 10, 3, 0.01) for i in range(nsf)]
    sfs = (q.make_sf_array(sfs), nsf)
    searches = []
    for i in range(nsf):
        searches.append((i * llr_stride, i % 10, 3, 0x3000 + 17 * i, 2))
        searches.append((i * llr_stride, i % 10, 3, 0xFFFF, 2))
    d_res = torch.zeros(len(searches) * s.Pdcch.RESULT_SIZE, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ncand = sum(len(s.pdcch_locations(q.nof_cce(3), i % 10, 0x3000 + 17 * i)) * 2 for i in range(nsf)) + \
        len(s.pdcch_locations(q.nof_cce(3), common=True)) * 3 * nsf
    torch.cuda.synchronize()

    def step():
        if q.extract_llr_dev(sfs, grid.data_ptr(), ce.data_ptr(), stride, d_llr.data_ptr(), st) != 0:
            raise RuntimeError("srsgpu_pdcch_extract_llr_dev failed")
        if q.find_dl_dci_dev(searches, d_llr.data_ptr(), d_res.data_ptr(), st) != 0:
            raise RuntimeError("srsgpu_pdcch_find_dl_dci_dev failed")

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    found = sum(r[0] for r in s.Pdcch.parse_results(d_res.cpu().numpy().tobytes()))
    del grid, ce
    return {"workload": "pdcch_receive_%dsf_%dprb_2ports_2rx_cfi3" % (nsf, nof_prb),
            "searches_per_step": len(searches), "candidates_per_step": ncand,
            "ms_per_step": round(el / steps * 1e3, 3), "subframes_per_s": round(nsf * steps / el, 1),
            "found": int(found)}


def dropin_latency(s, llr, ncb=16):
    """The drop-in srslte_tdec_iteration path (include/srslte/phy/fec/turbodecoder.h) as an
    unmodified decode_tb_cb loop drives it (sch.c:356-391): per code block srslte_tdec_new_cb, then
    one call per half-iteration, each a GPU launch for ONE code block, a stream synchronisation and
    the decision bytes copied back. Latency-bound by construction; reported so the cost of the
    compatibility path is on record (host-pointer rate, never `value`)."""
    d = s.Tdec(K)
    d.force_not_sb()  # the bench's LLRs are in natural [s, p0, p1] order
    out = np.zeros(K // 8, np.uint8)
    rows = [np.ascontiguousarray(llr[i]) for i in range(ncb)]
    for r in rows[:2]:  # warm-up: tables, first launches
        d.new_cb(K)
        for _ in range(NHALF):
            d.iteration(r, out)
    t0 = time.perf_counter()
    for r in rows:
        d.new_cb(K)
        for _ in range(NHALF):
            d.iteration(r, out)
    el = time.perf_counter() - t0
    d.free()
    return {"K": K, "code_blocks": ncb, "half_iterations": NHALF,
            "us_per_halfit_call": round(el / (ncb * NHALF) * 1e6, 2),
            "mbps": round(ncb * K / el / 1e6, 2),
            "note": "one code block per srslte_tdec_iteration call (host buffers, synchronous); the "
                    "batch APIs carry the throughput"}


# SURVEY §8(d) per-subframe algorithmic HBM bytes of the C3 (20 MHz SISO, 100 PRB, MCS 28, CFI 1,
# N = 2048) kernels: what each must read and write at least, per subframe
C3_NRE, C3_NLLR, C3_GRID = 15000, 90000, 14 * 12 * 100
C3_KS = [5824] * 13
ALG_BYTES_PER_SF = {
    # 14 symbols of N complex-float samples in (CPs skipped), the 16,800-RE grid out
    "k_ofdm_rx": lambda N: 14 * N * 8 + C3_GRID * 8,
    # 4 x 200 CRS pilots in, the estimator's compact rows (4 x 1200 RE: srsgpu_chest_set_ce_rows, the
    # traffic legs' form) and the noise estimate out
    "k_chest": lambda N: 800 * 8 + 4 * 1200 * 8 + 4,
    # the subframe's Gold sequence bits out
    "k_gold": lambda N: C3_NLLR // 8,
    # grid of the 15,000 PDSCH REs and the 4 estimate rows in, 90,000 int16 LLRs out
    "k_pdsch_llr": lambda N: C3_NRE * 8 + 4 * 1200 * 8 + C3_NLLR * 2,
    # LLRs in, the 13 softbuffer rows (3(K+32)+12 int16) out
    "k_derm": lambda N: C3_NLLR * 2 + sum((3 * (k + 32) + 12) * 2 for k in C3_KS),
    # rows in, the decoder's systematic / parity planes out: 6 B + 6 B per info bit
    "k_load": lambda N: 12 * sum(C3_KS),
    # direct de-rate-matching (fresh softbuffers): LLRs in, the decoder's planes out (6 B per info bit)
    "k_ldderm": lambda N: C3_NLLR * 2 + 6 * sum(C3_KS),
    # (3(K+32)+12)*2 + K/8 B per code block per decode
    "k_win_bidir_es": lambda N: sum((3 * (k + 32) + 12) * 2 + k // 8 for k in C3_KS),
    "k_win_bidir_run": lambda N: sum((3 * (k + 32) + 12) * 2 + k // 8 for k in C3_KS),
    # one half-iteration of the windowed decoder (per-half-iteration launches of an early-stop job;
    # "k_win_bidir" also matches the fused forms, which a job uses instead): 6 B per info bit
    "k_win_bidir": lambda N: 6 * sum(C3_KS),
    # packed decisions in (2 bits per info bit pair), natural-order bytes out
    "k_decide": lambda N: sum(k // 4 + k // 8 for k in C3_KS),
    # decision bytes in, TB bytes out
    "k_es_bytes": lambda N: 2 * sum(k // 8 for k in C3_KS),
    "k_tb_finish": lambda N: sum(k // 8 for k in C3_KS) + C3_TBS // 8,
}
HEADLINE_SNR_DB = 20.0
# descriptor sets the headline cycles through (a new grant every step: no repeat-call cache hits)
HEADLINE_DESCRIPTOR_SETS = 4
HEADLINE_FE_STREAM = 1  # r06_s16: 0.695 against 0.712 ms per batch (three alternated pairs)
HEADLINE_TAIL = 1  # r06_s7: 0.770 against 0.845 ms per batch (three alternated pairs, four descriptor sets)
# decoder early-stop launch schedules (srsgpu_tdec_set_schedule) compared by --ab-headline
HEADLINE_AB = {"auto": {"es_fused": 2, "es_chunk": 8}, "per_halfit": {"es_fused": 0},
               "fused_c8": {"es_fused": 1, "es_chunk": 8}, "hybrid": {"es_fused": 3, "es_chunk": 8}}


def decoder_valu_roofline(leg):
    """VALU roofline of the WHOLE turbo decoder of a coded leg: SURVEY 8(d)'s 90 int16 ops per info
    bit per half-iteration, over every half-iteration every code block ran in the batch (the first,
    k_win_bidir_h0, for all blocks; the early-stop continuation, k_win_bidir_es, for the blocks
    still running; srsgpu_dlsch_cb_halfits), divided by the device time of all decoder launches of
    the batch (HIP events on the lane streams). The per-launch-class split stays in `launches`."""
    kt = leg["kernels_per_batch"]
    h0, es = kt.get("k_win_bidir_h0"), kt.get("k_win_bidir_es")
    bits = leg.get("halfit_bits_per_batch")
    if not (h0 and h0["launches"]) or not bits:
        return None
    first_bits = sum(C3_KS) * C3_SF
    ms = h0["ms"] + (es["ms"] if es else 0.0)
    ops = ALG_OPS_PER_BIT_HALFIT * bits
    rate = ops / (ms / 1e3) / 1e12
    split = {"k_win_bidir_h0": {"ms_per_batch": h0["ms"], "launches": h0["launches"],
                                "ops": ALG_OPS_PER_BIT_HALFIT * first_bits,
                                "T_ops": round(ALG_OPS_PER_BIT_HALFIT * first_bits / (h0["ms"] / 1e3) / 1e12, 2)}}
    if es and es["launches"]:
        rest = ALG_OPS_PER_BIT_HALFIT * max(bits - first_bits, 0)
        split["k_win_bidir_es"] = {"ms_per_batch": es["ms"], "launches": es["launches"], "ops": rest,
                                   "T_ops": round(rest / (es["ms"] / 1e3) / 1e12, 3)}
    return {"bound": "valu (packed int16)", "kernel": "turbo decoder, all launches (k_win_bidir_h0 + k_win_bidir_es)",
            "achieved": round(rate, 2), "peak": VALU_INT16_PEAK_T, "unit": "T int16-ops/s",
            "frac": round(rate / VALU_INT16_PEAK_T, 4), "alg_ops_per_batch": int(ops),
            "halfits_per_cb_mean": round(bits / first_bits, 4), "decoder_ms_per_batch": round(ms, 4),
            "avg_launch_ms": round(ms / (h0["launches"] + (es["launches"] if es else 0)), 4), "launches": split}


def pipeline_roofline(leg, nsf_per_batch):
    """roofline of the leg's dominant kernel (the largest device time per batch among the ones with
    §8(d) algorithmic bytes): achieved = algorithmic bytes per launch / average launch time (HIP
    events on the launch stream, stage_profile); plus the whole per-kernel table"""
    N = leg["symbol_size"]
    table = {}
    for k, v in leg["kernels_per_batch"].items():
        if k not in ALG_BYTES_PER_SF or not v["launches"] or k == "k_win_bidir_h0":
            continue
        alg = ALG_BYTES_PER_SF[k](N) * nsf_per_batch / v["launches"]
        avg = v["ms"] / v["launches"]
        table[k] = {"ms_per_batch": v["ms"], "launches_per_batch": v["launches"], "avg_launch_ms": round(avg, 4),
                    "alg_bytes_per_launch": int(alg), "achieved_GBs": round(alg / (avg / 1e3) / 1e9, 1),
                    "frac": round(alg / (avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    if not table:
        return None, table
    dom = max(table, key=lambda k: table[k]["ms_per_batch"])
    t = table[dom]
    pmc = load_profile_json(leg["workload"] + ":" + dom)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    src = pmc.get("source") if pmc else None
    if traffic is None:
        traffic, src = pipeline_pmc_traffic(dom)
    roof = {"bound": "hbm", "kernel": dom, "achieved": t["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": t["frac"], "traffic": traffic,
            "traffic_over_alg": round(traffic / t["alg_bytes_per_launch"], 2) if traffic else None,
            "traffic_source": src,
            "alg_bytes_per_launch": t["alg_bytes_per_launch"], "avg_launch_ms": t["avg_launch_ms"],
            "launches_per_batch": t["launches_per_batch"],
            "alg_bytes_def": "SURVEY 8(d) per-subframe algorithmic bytes of %s (bench.py ALG_BYTES_PER_SF) x "
                             "%d subframes per launch" % (dom, nsf_per_batch / t["launches_per_batch"])}
    return roof, table


# library scope name -> rocprof kernel name prefixes (tools/pmc_pipeline.py keys)
PMC_NAMES = {"k_ldderm": ("k_load_derm",), "k_ofdm_rx": ("k_ofdm_rx_p", "k_ofdm_rx_c"),
             "k_win_bidir": ("k_win_bidir<", "k_win_bidir_es<")}


def pipeline_pmc_traffic(kernel):
    """HBM bytes per launch of a pipeline kernel from the newest committed
    profiles/*pmc_pipeline.json (tools/pmc_pipeline.py: FETCH_SIZE x2 + WRITE_SIZE per dispatch,
    separate passes), averaged over its variants by dispatch count; (None, None) without one"""
    pdir = os.path.join(REPO, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    natural = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]  # noqa: E731
    files = sorted((f for f in os.listdir(pdir) if f.endswith("pmc_pipeline.json")), key=natural)
    if not files:
        return None, None
    d = json.load(open(os.path.join(pdir, files[-1])))
    pre = PMC_NAMES.get(kernel, (kernel,))
    tot = n = 0
    for k, r in d.items():
        if any(k.startswith(p) for p in pre):
            c = max(r["dispatches"])
            tot += (r["fetch_bytes_x2"] + r["write_bytes"]) * c
            n += c
    return (int(tot / n), "profiles/" + files[-1]) if n else (None, None)


def cpu_baseline_pipeline(grids, sf_idx, snr_db, nthreads=None, target_thread_s=15.0):
    """BASELINE configs[2] on the host: the reference's own srslte_chest_dl_estimate +
    srslte_pdsch_decode (CRC early stop, max 8 half-iterations), compiled from its sources into
    oracle/_ref/ref_front, one chest / PDSCH / softbuffer per pthread, each pinned to its own physical
    core, on the GPU leg's own received grids (after its FFT: FFTW is absent, so the OFDM stage is
    excluded here and stated). Threads as cpu_baseline. None if the executable is absent."""
    import subprocess
    import tempfile
    exe = os.path.join(REPO, "oracle", "_ref", "ref_front")
    if not os.path.exists(exe):
        return None
    cores = physical_cpus()
    cap = int(os.environ.get("SRSGPU_CPU_THREADS", os.environ.get("OMP_NUM_THREADS", len(cores))))
    if nthreads is None:
        nthreads = max(1, min(len(cores), cap))
    pin = quiet_cpus(nthreads)[0]  # the least busy physical cores of the shared host
    nsf = len(sf_idx)

    def run(reps):
        head = np.array([C3_PRB, C3_CELL, 1, 1234, 28, 8, nthreads, reps, nsf, len(pin)] + list(pin), np.uint32)
        body = b"".join(np.array([sf], np.uint32).tobytes() + np.ascontiguousarray(g, np.complex64).tobytes()
                        for sf, g in zip(sf_idx, grids))
        with tempfile.TemporaryDirectory() as d:
            fi, fo = os.path.join(d, "in.bin"), os.path.join(d, "out.json")
            with open(fi, "wb") as f:
                f.write(head.tobytes() + body)
            r = subprocess.run([exe, "pdsch_bench", fi, fo], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError("ref_front pdsch_bench failed: " + r.stderr[-400:])
            return json.load(open(fo))

    reps = 1
    while True:  # grow the passes until one timed run holds >= 10 thread-seconds (target 15)
        res = run(reps)
        wall = res["wall_s"]
        if wall * nthreads >= 10.0 or reps >= 20000:
            break
        reps = int(min(20000, max(reps + 1, np.ceil(reps * target_thread_s / max(wall * nthreads, 1e-6)))))
    return {"value": round(res["cb_bits_ok"] / wall / 1e6, 2), "unit": "Mbps", "cores": nthreads, "kind": "reference",
            "subframes_per_s": round(res["subframes"] / wall, 1), "acked_tbs": res["acked"],
            "subframes": res["subframes"], "nof_iterations_mean": res["noi_mean"], "pinned_cpus": pin,
            "physical_cores_available": len(cores),
            "sample": "%d subframe decodes (%d distinct received grids of the GPU headline leg at %.0f dB x %d "
                      "passes) through the reference's srslte_chest_dl_estimate + srslte_pdsch_decode "
                      "(oracle/_ref/ref_front, compiled from the reference's sources, AVX2, CRC early stop max 8 "
                      "half-iterations), %d threads each pinned to its own physical core (%d physical cores in "
                      "the affinity set, CPU share cap %d), %.2f s wall (%.0f thread-seconds); OFDM FFT excluded "
                      "(FFTW absent)" % (res["subframes"], nsf, snr_db, reps, nthreads, len(cores), cap, wall,
                                         wall * nthreads)}


def decoder_leg(s, torch, dev, args, dist, rank, nranks):
    """BASELINE configs[1]: 4096 x K=6144 code blocks per GPU, 8 half-iterations, AUTO decoder (AVX16
    window), inputs resident in HBM; one step = one srsgpu_tdec_batch_run_dev. Returns (dict, llr) —
    the dict carries its own roofline (compulsory HBM bytes) and VALU roofline."""
    import srsgpu_shard as sh
    tcod = s.Tcod(K)
    first = sh.contiguous(nranks * NCB, nranks)
    assert first[rank + 1] - first[rank] == NCB
    bits, idx, llr = make_inputs(NCB, 1234, tcod, first=first[rank])
    d_in = torch.from_numpy(llr).to(dev)
    d_out = torch.zeros((NCB, K // 8), dtype=torch.uint8, device=dev)
    # a dedicated stream: launches on the null stream carry HIP's implicit cross-stream
    # synchronisation and cost ~6 % of the step here
    stream = lane_stream(torch, dev, 0)
    batch = s.TdecBatch(NCB, K, stream=stream.cuda_stream)
    stride = 3 * K + 12

    def step():
        if batch.run_dev(0, 0, d_in.data_ptr(), stride, K, NCB, NHALF, d_out.data_ptr(), K // 8) != 0:
            raise RuntimeError("srsgpu_tdec_batch_run_dev failed")

    # pre-heat: ~0.3 s of decoding so the timed steps see the steady clock of a receiver that decodes
    # continuously (a cold GPU ramps its clock over the first few ms of load)
    t_heat = time.perf_counter()
    while time.perf_counter() - t_heat < 0.3:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    expect = np.packbits(bits, axis=1)[idx]
    bit_errors = int(np.unpackbits(d_out.cpu().numpy() ^ expect).sum())
    steps = args.steps
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    # the decoder kernel's launch duration: HIP events around every launch on the batch stream,
    # over the same number of steps right after the timed loop
    s.prof_reset()
    s.prof_enable(True)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    s.prof_enable(False)
    kern_name, halfits_per_launch = "k_win_bidir_run", NHALF
    kern_ms, kern_n = s.prof_get(kern_name)
    if not kern_n:
        kern_name, halfits_per_launch = "k_win_bidir", 1
        kern_ms, kern_n = s.prof_get(kern_name)
    elapsed, bit_errors = reduce_over_ranks(dist, dev, elapsed, bit_errors)
    gather = None
    if dist:  # decoded bytes to rank 0 in one grouped send/recv batch (not in the step)
        gdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        local_out = d_out.reshape(-1) if gdev.type == "cuda" else d_out.reshape(-1).cpu()
        owner = np.repeat(np.arange(nranks), np.diff(first))
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        got = sh.gather_records(dist, torch, gdev, owner, [K // 8] * (nranks * NCB), local_out)
        torch.cuda.synchronize()
        gather = {"gather_ms": round((time.perf_counter() - tg) * 1e3, 3), "bytes_per_rank": NCB * K // 8,
                  "gathered_code_blocks": (sum(1 for r in got if r is not None) if got is not None else None)}
    workload = "batched_turbo_decode_%dxK%d_%dhalfits" % (NCB, K, NHALF)
    avg_launch_ms = kern_ms / max(kern_n, 1)
    alg_bytes = COMPULSORY_BYTES_PER_CB * NCB / NHALF * halfits_per_launch
    achieved = alg_bytes / (avg_launch_ms / 1e3) / 1e9 if kern_n else None
    pmc = load_profile_json(workload)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc and pmc.get("kernel") == kern_name else None
    out = {"workload": workload, "config": "BASELINE configs[1]", "mbps": round(decoded_mbps(nranks, NCB, K, steps, elapsed), 2),
           "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "code_blocks_per_gpu": NCB, "K": K,
           "half_iterations": NHALF, "decoder": "AUTO (AVX16 window, 16 sub-blocks)", "ebno_db_ref_convention": EBNO_DB,
           "bit_errors": bit_errors, "decoder_schedule": s.get_schedule(),
           "roofline": {"bound": "hbm", "kernel": kern_name, "achieved": round(achieved, 1) if achieved else None,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                        "traffic": traffic, "traffic_over_compulsory": round(traffic / alg_bytes, 2) if traffic else None,
                        "traffic_source": pmc.get("source") if pmc else None, "alg_bytes_per_launch": int(alg_bytes),
                        "alg_bytes_def": "SURVEY 8(d): (3(K+32)+12)*2 + K/8 = %d B per CB per decode" % COMPULSORY_BYTES_PER_CB,
                        # what an iterative decoder must stream every half-iteration (its state does not fit
                        # the caches: 4096 x K=6144 x 10 B = 252 MB): DEC1 reads SP0 + A (6 B per CB and info
                        # bit) and writes X2 (2 B), DEC2 reads X2 + P1 (4 B) and writes A (2 B)
                        "working_set_bytes_per_launch": int(7 * NCB * K * halfits_per_launch),
                        "traffic_over_working_set": round(traffic / (7 * NCB * K * halfits_per_launch), 2) if traffic else None,
                        "avg_launch_ms": round(avg_launch_ms, 4), "launches": kern_n,
                        "halfits_per_launch": halfits_per_launch, "avg_halfit_ms": round(avg_launch_ms / halfits_per_launch, 4)}}
    if kern_n:
        ops = ALG_OPS_PER_BIT_HALFIT * NCB * K * halfits_per_launch
        rate_t = ops / (avg_launch_ms / 1e3) / 1e12
        out["valu_roofline"] = {
            "bound": "valu (packed int16)", "kernel": kern_name, "achieved": round(rate_t, 2), "peak": VALU_INT16_PEAK_T,
            "unit": "T int16-ops/s", "frac": round(rate_t / VALU_INT16_PEAK_T, 4), "alg_ops_per_launch": ops,
            "alg_ops_def": "SURVEY 8(d): %d int16 ops per info bit per half-iteration" % ALG_OPS_PER_BIT_HALFIT,
            "measured_issue_peaks_T": VALU_INT16_MEASURED_T,
            "frac_of_1wave_issue_peak": round(rate_t / VALU_INT16_MEASURED_T["1_wave_per_simd_ilp8"], 4)}
    if gather:
        out["gather"] = gather
    out["_batch"], out["_d_in"], out["_d_out"], out["_expect"], out["_stride"] = batch, d_in, d_out, expect, stride
    return out, llr


def spawn_ranks(n, argv):
    """bench.py --gpus N without a launcher (WORLD_SIZE unset): start N child processes of this
    script, rank r on GPU r (LOCAL_RANK), rendezvous on 127.0.0.1 at a free port, and wait for all.
    Called before anything touches the GPU; the parent never initialises HIP and never re-execs.
    Rank 0's stdout is the parent's, so its JSON line is the last line printed. If one rank fails
    the others are stopped (they would wait in a collective) and the exit code is non-zero."""
    import signal
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL, start_new_session=True))
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print("bench.py: a rank exited with %d; stopping the others" % c, file=sys.stderr, flush=True)
                for q in procs:
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
    return rc


def dist_check(dist, torch, rank, nranks):
    """The multi-rank plumbing of the bench without a GPU (--legs distcheck, gloo): every rank
    reports its process, plans the legs' global jobs (C3 / TM3 contiguous subframe ranges, the C5
    mixed-bandwidth plan by the weighted longest-first partition), builds one result record per unit
    it owns — bytes derived from the unit index, so rank 0 can verify every byte — and gathers them
    to rank 0 with srsgpu_shard.gather_records, as the GPU legs do after their timed loop."""
    import srsgpu_shard as sh
    import srsgpu_traffic as tr
    procs = [None] * nranks
    dist.all_gather_object(procs, {"rank": rank, "pid": os.getpid(), "local_rank": int(os.environ.get("LOCAL_RANK", 0))})
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    n_global = C3_SF * nranks
    out = {"ranks": procs, "backend": dist.get_backend(), "legs": {}}

    def record(u, tbs):
        rng = np.random.default_rng(1000003 * u + tbs)
        return sh.pack_tb_record(0, 1 + u % 8, rng.integers(0, 256, tbs // 8, dtype=np.uint8),
                                 np.ones(13, np.uint8), tbs)

    for leg, plan_tbs, part in (("c3", [C3_TBS] * n_global, "contiguous"),
                                ("tm3", [2 * C3_TBS] * n_global, "contiguous"),
                                ("c5", None, "weighted")):
        if part == "contiguous":
            f = sh.contiguous(n_global, nranks)
            owner = np.repeat(np.arange(nranks), np.diff(f))
            tbs_of = plan_tbs
            bal = 1.0
        else:
            sf_plan = tr.plan(table, n_global, seed=21)
            owner, load = sh.weighted(tr.tb_weights(table, sf_plan), nranks)
            tbs_of = [p["tbs"] for p in sf_plan]
            bal = sh.balance(load)
        sizes = [sh.tb_record_len(t) for t in tbs_of]
        mine = [u for u in range(n_global) if owner[u] == rank]
        local = torch.from_numpy(np.concatenate([record(u, tbs_of[u]) for u in mine]) if mine
                                 else np.zeros(0, np.uint8))
        t0 = time.perf_counter()
        got = sh.gather_records(dist, torch, torch.device("cpu"), owner, sizes, local)
        ms = (time.perf_counter() - t0) * 1e3
        if rank == 0:
            ok = sum(1 for u, r in enumerate(got) if r is not None and np.array_equal(r, record(u, tbs_of[u])))
            out["legs"][leg] = {"units": n_global, "units_per_rank": np.bincount(owner, minlength=nranks).tolist(),
                                "partition": part, "balance": round(bal, 4), "gathered_ok": ok,
                                "gather_ms": round(ms, 3)}
    return out


# keys of a leg's result reported in the compact summary line (one or two numbers per leg)
LEG_SUMMARY = (
    ("c3_fixed8_codewords", "fixed8", ("subframes_per_s", "decoded_mbps", "ms_per_batch")),
    ("c3_cached", "cached", ("subframes_per_s", "decoded_mbps", "ms_per_batch", "host_ms_per_step")),
    ("pipeline_tm3_coded", "tm3_coded", ("subframes_per_s", "decoded_mbps")),
    ("pipeline_c5", "c5", ("subframes_per_s", "decoded_mbps")),
    ("pipeline_coded", "coded30", ("subframes_per_s", "decoded_mbps")),
    ("c3_fft1536", "n1536", ("subframes_per_s", "decoded_mbps")),
    ("pipeline", "c3_random_fixed8", ("subframes_per_s",)),
    ("pipeline_tm3", "tm3_random_fixed8", ("subframes_per_s",)),
    ("pdcch", "pdcch", ("subframes_per_s",)),
    ("pcfich", "pcfich", ("subframes_per_s",)),
    ("pdcch_dci", "dci", ("candidates_per_s",)),
    ("dropin_latency", "dropin", ("us_per_halfit_call",)),
    ("distcheck", "distcheck", ("backend",)),
)


def compact_summary(result, detail_name, limit=6000):
    """The driver-facing last stdout line: the contract's keys, the headline's roofline /
    valu_roofline / cpu_baseline, and one or two numbers per leg; everything else stays in the
    detail file. Trimmed to `limit` bytes (the driver keeps the tail of stdout)."""
    top = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
           "vs_baseline", "dtype", "data", "value_def")
    out = {k: result[k] for k in top if k in result}
    cfg = result.get("config", {})
    out["config"] = {k: cfg[k] for k in ("workload", "baseline_config", "subframes_per_batch_per_gpu", "nof_prb",
                                         "fft_size", "mcs", "tbs", "code_blocks_per_subframe", "K", "snr_db",
                                         "early_stop_max_halfits", "descriptor_sets", "lanes", "fe_stream", "tail_stream",
                                         "subframes_per_s", "nof_iterations_mean",
                                         "acked_tbs", "tbs_bytes_ok", "parallelism") if k in cfg}
    for key, fields in (("roofline", ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                                      "traffic_over_alg", "traffic_source", "alg_bytes_per_launch", "avg_launch_ms",
                                      "launches_per_batch")),
                        ("valu_roofline", ("bound", "kernel", "achieved", "peak", "unit", "frac", "avg_launch_ms")),
                        ("cpu_baseline", ("value", "unit", "cores", "kind", "subframes_per_s", "nof_iterations_mean",
                                          "sample"))):
        if result.get(key):
            out[key] = {f: result[key][f] for f in fields if f in result[key]}
    legs = {}
    dec = result.get("decoder_c2")
    if dec:
        legs["decoder_c2"] = {"mbps": dec.get("mbps"), "ms_per_step": dec.get("ms_per_step"),
                              "valu_frac": (dec.get("valu_roofline") or {}).get("frac"),
                              "hbm_frac": (dec.get("roofline") or {}).get("frac"),
                              "cpu_mbps": (dec.get("cpu_baseline") or {}).get("value")}
    for key, name, fields in LEG_SUMMARY:
        if result.get(key):
            legs[name] = {f: result[key].get(f) for f in fields}
    sw = result.get("c3_coded_sweep")
    if sw:
        legs["sweep_decoded_mbps"] = {"%g" % p["snr_db"]: p["decoded_mbps"] for p in sw["points"]}
    rq = result.get("rx_queue")
    if rq:
        sat = rq.get("saturated", {})
        top = max(sat, key=lambda k: sat[k]["subframes_per_s"], default=None)
        def miss(fm):
            return None if not fm else {k: fm.get(k) for k in (
                "streams", "latency_ms_p99", "submit_latency_ms_p99", "producer_late_ms_max", "producer_late_ms_p99",
                "failed", "acked", "mean_batch", "cpu_cores_busy", "cgroup_throttled_ms")}

        legs["rx_queue"] = {"real_time_streams": rq.get("real_time_streams"),
                            "real_time_streams_1536": rq.get("real_time_streams_1536"),
                            "queue_streams": rq.get("queue_streams"),
                            "queue_streams_1536": rq.get("queue_streams_1536"),
                            "first_miss": miss(rq.get("first_miss")),
                            "first_miss_1536": miss(rq.get("first_miss_1536")),
                            "saturated_max_sfps": sat[top]["subframes_per_s"] if top else None,
                            "saturated_max_mode": top, "cpu_quota": (rq.get("cpus") or {}).get("quota")}
    hd = result.get("headline_detail") or {}
    if hd.get("gather_ms") is not None:
        legs["headline_gather_ms"] = hd["gather_ms"]
    out["legs"] = legs
    out["detail"] = detail_name
    line = json.dumps(out, separators=(",", ":"))
    for drop in ("sample", "legs"):  # over the limit: shorten the free text, then the legs
        if len(line) <= limit:
            break
        if drop == "sample" and "cpu_baseline" in out:
            out["cpu_baseline"]["sample"] = out["cpu_baseline"].get("sample", "")[:200]
        elif drop == "legs":
            out["legs"] = {k: legs[k] for k in ("decoder_c2", "fixed8", "tm3_coded", "c5", "rx_queue") if k in legs}
        line = json.dumps(out, separators=(",", ":"))
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="headline and configs[1] decoder only")
    ap.add_argument("--coded-snr", type=float, default=None,
                    help="SNR of the coded C3 leg (default 30 dB; profiling aid)")
    # one lane: with the early-stop tails on the tail stream, a second lane no longer pays
    # (r06_s12: 0.743 against 0.754 ms per batch, three alternated pairs)
    ap.add_argument("--lanes", type=int, default=1, help="HIP streams per rank for the headline leg")
    ap.add_argument("--fe-stream", type=int, default=HEADLINE_FE_STREAM,
                    help="1: the headline's front end on a stream of its own, beside the previous batch's decoder")
    ap.add_argument("--tail", type=int, default=HEADLINE_TAIL,
                    help="headline early-stop tails: 0 on the lane's stream, 1 on one high-priority tail stream")
    ap.add_argument("--ab-headline", action="store_true",
                    help="A/B the decoder's early-stop launch schedules on the headline workload")
    ap.add_argument("--legs", default="c2,fixed8,cached,c3,tm3,tm3c,coded,sweep,n1536,c5,d8,dropin,dci,pcfich,pdcch,rxq",
                    help="legs after the headline (profiling aid); 'distcheck' alone rehearses the multi-rank "
                         "partition and gather on the CPU (gloo), without a GPU")
    ap.add_argument("--detail", default=os.path.join(REPO, "bench_detail.json"),
                    help="file for the full per-leg record (the last stdout line is the compact summary)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))  # before any GPU call
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%d but --gpus %d; launch one rank per GPU" % (world, args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nranks = max(1, world)
    legs = set() if args.no_pipeline else set(args.legs.split(","))
    if args.no_pipeline:
        legs = {"c2"}

    import torch

    if legs == {"distcheck"}:  # CPU rehearsal of the multi-rank path: no GPU, no headline
        import torch.distributed as dist
        dist.init_process_group(os.environ.get("SRSGPU_DIST_BACKEND", "gloo"))
        dc = dist_check(dist, torch, rank, nranks)
        if rank == 0:
            result = {"metric": METRIC, "value": None, "unit": "Mbps", "n_gpus": nranks, "steps": args.steps,
                      "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
                      "vs_baseline": None, "dtype": "fp32+int16", "data": "none (multi-rank plumbing rehearsal)",
                      "config": {"workload": "distcheck", "parallelism": "dp%d" % nranks}, "distcheck": dc}
            with open(args.detail, "w") as f:
                json.dump(result, f)
            print(compact_summary(result, os.path.basename(args.detail)), flush=True)
        dist.destroy_process_group()
        return

    import srsgpu_phy as s

    dist = None
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU over RCCL; SRSGPU_DIST_BACKEND=gloo rehearses several ranks on one card
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(os.environ.get("SRSGPU_DIST_BACKEND", "nccl"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    def scale_ranks(r):
        if dist:  # whole job: every rank's bits and subframes over the slowest rank's batch time
            ms, _ = reduce_over_ranks(dist, dev, r["ms_per_batch"], 0)
            for key in ("decoded_mbps", "acked_tb_mbps", "offered_tb_mbps"):
                tot, _ = reduce_over_ranks(dist, dev, r[key] * r["ms_per_batch"], 0, op="sum")
                r[key] = round(tot / ms, 1)
            r["subframes_per_s"] = round(nranks * C3_SF / (ms / 1e3), 1)
        return r

    # ---- headline: BASELINE configs[2] (the metric's own configuration) ----
    # 1024 coded 20 MHz SISO 64QAM subframes per GPU (MCS 28, TBS 75376, 13 x K=5824) from the GPU
    # transmitter at 20 dB, time domain -> TB bytes: OFDM FFT, CRS channel estimation, PDSCH (RE
    # extraction, MMSE, 64QAM demap, descramble), DL-SCH (de-RM, turbo decoding with CRC early stop up
    # to 8 half-iterations as srsUE runs it, TB CRC). One step = one 1024-subframe batch.
    # The descriptors change every step (four sets with different softbuffers in turn, rotate=4), as a
    # receiver's grants do (pdsch.c:868-1007 is called with a fresh cfg per subframe): the PDSCH / DL-SCH
    # repeat-call caches never hit, every step pays its per-code-block host work
    head = scale_ranks(run_traffic(s, torch, dev, args.steps, args.warmup, "c3_coded", snr_db=HEADLINE_SNR_DB,
                                   dist=dist, cpu_sample=64 if (rank == 0 and nranks == 1) else 0, lanes=args.lanes,
                                   warm_seconds=1.0, schedules=HEADLINE_AB if args.ab_headline else None,
                                   rotate=HEADLINE_DESCRIPTOR_SETS, tail=args.tail, fe_split=bool(args.fe_stream)))
    cpu_grids, cpu_sf = head.pop("_cpu_grids", None), head.pop("_cpu_sf_idx", None)
    result = None
    if rank == 0:
        roof, ktable = pipeline_roofline(head, C3_SF)
        head["kernel_table"] = ktable
        valu = decoder_valu_roofline(head)
        result = {
            "metric": METRIC, "value": head["decoded_mbps"], "unit": "Mbps", "n_gpus": nranks, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_batch"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32+int16",
            "data": "synthetic (coded subframes from the GPU transmitter, AWGN %.0f dB)" % HEADLINE_SNR_DB,
            "config": {"workload": "pdsch_test_c3_20MHz_siso_64qam_%dsf_snr%d_earlystop8" % (C3_SF, HEADLINE_SNR_DB),
                       "baseline_config": "BASELINE configs[2]", "subframes_per_batch_per_gpu": C3_SF,
                       "nof_prb": C3_PRB, "fft_size": head["symbol_size"], "mcs": 28, "tbs": C3_TBS,
                       "code_blocks_per_subframe": 13, "K": 5824, "snr_db": HEADLINE_SNR_DB,
                       "early_stop_max_halfits": 8, "descriptor_sets": HEADLINE_DESCRIPTOR_SETS,
                       "tail_stream": args.tail, "lanes": args.lanes, "fe_stream": args.fe_stream,
                       "subframes_per_s": head["subframes_per_s"],
                       "nof_iterations_mean": head["nof_iterations_mean"], "acked_tbs": head["acked_tbs"],
                       "tbs_bytes_ok": head["tbs_bytes_ok"], "parallelism": "dp%d" % nranks},
            "value_def": "decoded Mbps = sum of K over CRC-passing code blocks per second (SURVEY 8(d)), whole "
                         "job over the slowest rank's batch time",
            "roofline": roof,
            "valu_roofline": valu,
            "headline_detail": head,
        }
    # ---- further legs ----
    dec = None
    llr = None
    if "c2" in legs:
        dec, llr = decoder_leg(s, torch, dev, args, dist, rank, nranks)
    extra = {}
    if "fixed8" in legs:
        # the same coded subframes with every code block running all 8 half-iterations (no early stop):
        # the worst-case processing rate on real codewords
        extra["fixed8"] = scale_ranks(run_traffic(s, torch, dev, max(8, args.steps), 2, "c3_coded",
                                                  snr_db=HEADLINE_SNR_DB, dist=dist, early_stop=False))
    if "envab" in legs:
        # the headline workload with and without an environment setting (BENCH_AB_ENV="NAME=VALUE"), in
        # turn in one process: A/B of a launch knob (wave_prio.h; srsgpu_knobs_reload after each change)
        name, _, val = os.environ.get("BENCH_AB_ENV", "SRSGPU_LLR_GENERIC=1").partition("=")
        for on in (0, 1, 0, 1, 0, 1):
            if on:
                os.environ[name] = val
            s.knobs_reload()
            r = run_traffic(s, torch, dev, max(10, args.steps), 3, "c3_coded", snr_db=HEADLINE_SNR_DB, dist=dist,
                            lanes=args.lanes, rotate=int(os.environ.get("BENCH_AB_ROTATE", str(HEADLINE_DESCRIPTOR_SETS))),
                            tail=args.tail, fe_split=bool(args.fe_stream))
            os.environ.pop(name, None)
            s.knobs_reload()
            extra.setdefault("envab", []).append({name: val if on else None, "ms_per_batch": r["ms_per_batch"],
                                                  "stage_ms": r["stage_ms_per_batch"], "acked_tbs": r["acked_tbs"],
                                                  "tbs_bytes_ok": r["tbs_bytes_ok"]})
    if "tailab" in legs:
        # the headline workload with the early-stop tails on tail streams (two engines per lane)
        # (BENCH_AB_ROTATE descriptor sets, BENCH_TAIL_PRIO=0: tail streams at normal priority)
        for t in (0, 1, 0, 1, 0, 1):
            r = run_traffic(s, torch, dev, max(10, args.steps), 3, "c3_coded", snr_db=HEADLINE_SNR_DB, dist=dist,
                            tail=t, lanes=args.lanes, rotate=int(os.environ.get("BENCH_AB_ROTATE", "1")),
                            tail_prio=os.environ.get("BENCH_TAIL_PRIO", "1") == "1")
            extra.setdefault("tailab", []).append({"tail": t, "ms_per_batch": r["ms_per_batch"],
                                                   "decoded_mbps": r["decoded_mbps"], "acked_tbs": r["acked_tbs"],
                                                   "tbs_bytes_ok": r["tbs_bytes_ok"]})
    if "feab" in legs:
        # the headline with and without a front-end stream of its own, in turn
        for fe in (0, 1, 0, 1, 0, 1):
            r = run_traffic(s, torch, dev, max(10, args.steps), 3, "c3_coded", snr_db=HEADLINE_SNR_DB, dist=dist,
                            lanes=args.lanes, rotate=HEADLINE_DESCRIPTOR_SETS, tail=args.tail, fe_split=bool(fe))
            extra.setdefault("feab", []).append({"fe_stream": fe, "ms_per_batch": r["ms_per_batch"],
                                                 "stage_ms": r["stage_ms_per_batch"], "acked_tbs": r["acked_tbs"],
                                                 "tbs_bytes_ok": r["tbs_bytes_ok"]})
    if "laneab" in legs:
        # the headline workload on one and on two lane streams, in turn (with the tail stream)
        for ln in (1, 2, 1, 2, 1, 2):
            r = run_traffic(s, torch, dev, max(10, args.steps), 3, "c3_coded", snr_db=HEADLINE_SNR_DB, dist=dist,
                            lanes=ln, rotate=HEADLINE_DESCRIPTOR_SETS, tail=args.tail)
            extra.setdefault("laneab", []).append({"lanes": ln, "ms_per_batch": r["ms_per_batch"],
                                                   "stage_ms": r["stage_ms_per_batch"], "acked_tbs": r["acked_tbs"],
                                                   "tbs_bytes_ok": r["tbs_bytes_ok"]})
    if "cached" in legs:
        # the headline workload with ONE descriptor set repeated every step, so the PDSCH / DL-SCH
        # repeat-call caches hit (no per-code-block host work): what a receiver never sees, kept as the
        # upper bound beside the headline, whose descriptors change every step
        extra["cached"] = scale_ranks(run_traffic(s, torch, dev, max(8, args.steps), 2, "c3_coded",
                                                  snr_db=HEADLINE_SNR_DB, dist=dist, rotate=1, tail=args.tail,
                                                  lanes=args.lanes))
    if "n1536" in legs:
        # srsLTE's reduced 20 MHz sampling (1536-point FFT, SURVEY 8(d) "N=1536")
        extra["n1536"] = scale_ranks(run_traffic(s, torch, dev, max(8, args.steps), 2, "c3_coded",
                                                 snr_db=HEADLINE_SNR_DB, dist=dist, standard_rate=False,
                                                 lanes=args.lanes, tail=args.tail, rotate=HEADLINE_DESCRIPTOR_SETS))
    pipe = None
    if "c3" in legs:
        pipe = run_pipeline(s, torch, dev, max(2, args.steps // 2), 2, dist=dist)
        if dist:
            ms, _ = reduce_over_ranks(dist, dev, pipe["ms_per_batch"], 0)
            pipe["subframes_per_s"] = round(nranks * C3_SF / (ms / 1e3), 1)
            pipe["processing_mbps"] = round(pipe["subframes_per_s"] * C3_TBS / 1e6, 1)
    pipe3 = None
    if "tm3" in legs:
        pipe3 = run_pipeline(s, torch, dev, max(2, args.steps // 2), 2, tm=3, dist=dist)
        if dist:
            ms, _ = reduce_over_ranks(dist, dev, pipe3["ms_per_batch"], 0)
            pipe3["subframes_per_s"] = round(nranks * C3_SF / (ms / 1e3), 1)
            pipe3["processing_mbps"] = round(pipe3["subframes_per_s"] * 2 * C3_TBS / 1e6, 1)
    tm3c = None
    if "tm3c" in legs:
        tm3c = run_tm3_coded(s, torch, dev, max(8, args.steps // 2), 2, dist=dist)
    for kind in ("c3_coded", "c5"):
        if kind.split("_")[-1] in legs:
            extra[kind] = scale_ranks(run_traffic(s, torch, dev, max(8, args.steps), 2, kind, dist=dist,
                                                  snr_db=args.coded_snr if kind == "c3_coded" else None))
    sweep = None
    if "sweep" in legs:
        # SURVEY §8(d) C3 points with CRC early stop (max 8 half-iterations), down into the waterfall
        # (14-16 dB: 2..8 half-iterations, failing TBs) and up to 30 dB
        sweep = []
        for snr in (14.0, 15.0, 16.0, 18.0, 20.0, 25.0, 30.0):
            r = scale_ranks(run_traffic(s, torch, dev, max(8, args.steps // 2), 2, "c3_coded", snr_db=snr, dist=dist,
                                        lanes=args.lanes, tail=args.tail, rotate=HEADLINE_DESCRIPTOR_SETS))
            sweep.append({k: r[k] for k in ("snr_db", "decoded_mbps", "acked_tb_mbps", "offered_tb_mbps",
                                             "subframes_per_s", "ms_per_batch", "nof_iterations_mean",
                                             "acked_tbs", "tbs")})
    dec8 = None
    if "d8" in legs and dec:
        # the reference's 8-bit path (srslte_tdec_iteration_8bit: AUTO -> int8 AVX8 window, 32 sub-blocks
        # at K = 6144) on the same code blocks, LLRs requantised to int8
        batch, d_in, d_out, expect, stride = dec["_batch"], dec["_d_in"], dec["_d_out"], dec["_expect"], dec["_stride"]
        d_in8 = torch.clamp(torch.div(d_in, 6, rounding_mode="trunc"), -128, 127).contiguous()
        torch.cuda.synchronize()

        def step8():
            if batch.run_dev(s.SRSGPU_TDEC_AUTO_8BIT, 0, d_in8.data_ptr(), stride, K, NCB, NHALF,
                             d_out.data_ptr(), K // 8) != 0:
                raise RuntimeError("srsgpu_tdec_batch_run_dev (8-bit) failed")

        for _ in range(args.warmup):
            step8()
        torch.cuda.synchronize()
        err8 = int(np.unpackbits(d_out.cpu().numpy() ^ expect).sum())
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        gc.disable()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step8()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el8 = time.perf_counter() - t0
        gc.enable()
        el8, err8 = reduce_over_ranks(dist, dev, el8, err8)
        dec8 = {"decoder": "AUTO 8-bit (int8 AVX8 window, 32 sub-blocks)",
                "mbps": round(decoded_mbps(nranks, NCB, K, args.steps, el8), 1),
                "ms_per_step": round(el8 / args.steps * 1e3, 3), "bit_errors": err8}
        if rank == 0:
            dec8["reference_sample"] = ref8_sample(d_in8, d_out, expect, stride)
    dci = pcf = pdc = rxq = dropin = None
    if "dci" in legs and rank == 0:
        dci = dci_blind_decode(s, torch, max(4, args.steps // 4))
    if "pcfich" in legs and rank == 0:
        pcf = pcfich_cfi(s, torch, max(4, args.steps // 4))
    if "pdcch" in legs and rank == 0:
        pdc = pdcch_receive(s, torch, max(4, args.steps // 4))
    if "rxq" in legs and rank == 0:
        rxq = rx_queue_leg(s, torch, dev)
    if "dropin" in legs and rank == 0 and llr is not None:
        dropin = dropin_latency(s, llr)
    if dec:
        dec.pop("_batch").close()
        for k in ("_d_in", "_d_out", "_expect", "_stride"):
            dec.pop(k)
    if rank == 0:
        if dec:
            result["decoder_c2"] = dec
        for key, val in (("dropin_latency", dropin), ("pdcch_dci", dci), ("pcfich", pcf), ("pdcch", pdc),
                         ("rx_queue", rxq), ("decoder_8bit", dec8)):
            if val:
                result[key] = val
        if "fixed8" in extra:
            result["c3_fixed8_codewords"] = extra["fixed8"]
            result["config"]["subframes_per_s_fixed8"] = extra["fixed8"]["subframes_per_s"]
        if "n1536" in extra:
            result["c3_fft1536"] = extra["n1536"]
        if "cached" in extra:
            result["c3_cached"] = extra["cached"]
        if "tailab" in extra:
            result["tail_ab"] = extra["tailab"]
        if "laneab" in extra:
            result["lane_ab"] = extra["laneab"]
        if "feab" in extra:
            result["fe_ab"] = extra["feab"]
        if "envab" in extra:
            result["env_ab"] = extra["envab"]
        if pipe:
            result["config"]["subframes_per_s_random_symbols_fixed8"] = pipe["subframes_per_s"]
            result["pipeline"] = pipe
        if pipe3:
            result["config"]["subframes_per_s_tm3"] = pipe3["subframes_per_s"]
            result["pipeline_tm3"] = pipe3
        if tm3c:
            result["config"]["tm3_coded_decoded_mbps"] = tm3c["decoded_mbps"]
            result["pipeline_tm3_coded"] = tm3c
        if sweep:
            result["c3_coded_sweep"] = {"workload": "c3_coded_%dsf_20MHz_64QAM_tbs%d" % (C3_SF, C3_TBS),
                                        "early_stop_max_halfits": 8, "points": sweep}
        for kind, key in (("c3_coded", "coded"), ("c5", "c5")):
            if kind in extra:
                result["config"]["subframes_per_s_" + key] = extra[kind]["subframes_per_s"]
                result["pipeline_" + key] = extra[kind]
    if rank == 0 and not args.no_cpu_baseline and nranks == 1:
        if cpu_grids is not None:
            result["cpu_baseline"] = cpu_baseline_pipeline(cpu_grids, cpu_sf, HEADLINE_SNR_DB)
        if llr is not None:
            result["decoder_c2"]["cpu_baseline"] = cpu_baseline(llr)
            if dropin:  # the reference's own per-call cost on one pinned thread, for comparison
                cb = result["decoder_c2"]["cpu_baseline"]
                dropin["cpu_reference_us_per_halfit_one_thread"] = round(K / (cb["value"] / max(cb["cores"], 1)) / NHALF, 2)
    if rank == 0:
        # the full record to the detail file; the last stdout line is the compact summary (the driver
        # keeps only the tail of stdout)
        with open(args.detail, "w") as f:
            json.dump(result, f)
        print(compact_summary(result, os.path.basename(args.detail)), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
