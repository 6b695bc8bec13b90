"""Reference-side binding (integration/srslte_gpu_shim.c).

CPU: the shim type-checks against the reference's own headers (when /root/reference exists).
GPU: oracle/_ref/shim_check decodes every subframe with the reference's CPU srslte_pdsch_decode
(pdsch.c:868-1007) and with the shim's GPU version on the same srslte_pdsch_t, grids and HARQ
sequence (rv 0, 2, 3, 1), and requires identical return value, ack, data bytes,
last_nof_iterations and softbuffer cb_crc / tb_crc for every transmission of TM1 without CSI.
With CSI, and in TM3 (whose MMSE inverts with rcpps in the reference), the reference's
approximate reciprocal makes LLRs agree only to its tolerance: data bytes must agree whenever
both decoders ack, and ack / iteration-count differences at the decoding threshold ("soft") must
stay rare.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_INC = "/root/reference/lib/include"
SHIM = os.path.join(REPO, "integration", "srslte_gpu_shim.c")
CHECK = os.path.join(REPO, "oracle", "_ref", "shim_check")


@pytest.mark.skipif(not os.path.isdir(REF_INC), reason="reference headers not present")
def test_shim_typechecks_against_reference_headers():
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-std=gnu99",
                        "-I" + REF_INC, "-I" + os.path.join(REPO, "include"), SHIM],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


# nof_prb, cell_id, mcs, cfi, nof_rx, csi, nof_tb, snr_db, seed, tm
CASES = [
    (6, 1, 9, 3, 1, 0, 8, 3.0, 1, 1),      # QPSK, 6 PRB, includes subframes 0 and 5
    (15, 77, 16, 2, 2, 1, 8, 9.0, 2, 1),   # 16QAM, odd PRB count (PBCH half PRBs), 2 rx, CSI
    (25, 301, 22, 1, 1, 0, 6, 14.0, 3, 1),  # 64QAM, 25 PRB
    (15, 77, 16, 2, 2, 0, 8, 9.0, 6, 1),   # 2 rx without CSI: every transmission bit-exact
    (50, 503, 27, 2, 2, 1, 4, 18.0, 4, 1),  # 64QAM, 2 rx, CSI, several code blocks
    (100, 12, 28, 2, 1, 0, 4, 21.0, 5, 1),  # 100 PRB, 13 code blocks
    (25, 7, 16, 2, 2, 0, 8, 16.0, 7, 3),   # TM3 CDD 2x2, two 16QAM TBs
    (50, 150, 26, 1, 2, 1, 6, 25.0, 8, 3),  # TM3, 64QAM, CSI
    (100, 1, 28, 1, 2, 0, 4, 27.0, 9, 3),  # TM3 20 MHz, two 64QAM TBs (BASELINE configs[3] shape)
    (6, 3, 9, 3, 2, 0, 8, 4.0, 21, 2),     # TM2 transmit diversity, QPSK, 2 rx (SIB-like)
    (25, 33, 16, 2, 1, 0, 6, 12.0, 22, 2),  # TM2, 16QAM, 1 rx
    (50, 211, 27, 1, 2, 1, 4, 20.0, 23, 2),  # TM2, 64QAM, 2 rx, CSI
    (25, 9, 16, 2, 2, 0, 8, 18.0, 31, 4),   # TM4 spatial multiplexing, 2 TBs on 2 layers, codebook 1-2
    (50, 140, 22, 1, 2, 1, 6, 22.0, 32, 4),  # TM4, 2 layers, CSI
    (25, 61, 16, 2, 2, 0, 8, 14.0, 33, 5),  # TM4 rank 1: one TB on one layer, codebook 0-3 (2x1 MRC)
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES,
                         ids=[f"tm{c[9]}_prb{c[0]}_mcs{c[2]}_rx{c[4]}_csi{c[5]}" for c in CASES])
def test_shim_pdsch_decode_matches_reference(case):
    if not os.path.exists(CHECK):
        pytest.skip("oracle/_ref/shim_check not built (needs /root/reference at build time)")
    r = subprocess.run([CHECK] + [str(v) for v in case], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    stats = dict(kv.split("=") for kv in r.stdout.split())
    assert int(stats["mismatches"]) == 0 and int(stats["tx"]) >= case[6]
    assert int(stats["soft"]) <= max(1, int(stats["tx"]) // 10), r.stdout + r.stderr
    assert int(stats["acks"]) > 0
    # reference-named DL-SCH drop-ins (srslte_dlsch_decode2, srslte_softbuffer_rx_*,
    # srslte_rm_turbo_rx_lut) on the same LLRs: exact in every configuration
    assert int(stats["dlsch"]) >= case[6] and int(stats["dlsch_mismatches"]) == 0, r.stdout + r.stderr
    assert int(stats["rm_mismatches"]) == 0, r.stdout + r.stderr
    # srslte_pcfich_decode_multi drop-in on this cell's ports / rx antennas: CFI and correlation exact
    assert int(stats["pcfich_mismatches"]) == 0, r.stdout + r.stderr
    # srslte_pdcch_extract_llr_multi / srslte_pdcch_decode_msg drop-ins: q->llr and every candidate's
    # message, CRC remainder and return value exact
    assert int(stats["pdcch"]) >= 100 and int(stats["pdcch_mismatches"]) == 0, r.stdout + r.stderr
    assert int(stats["pdcch_found"]) >= 1, r.stdout + r.stderr
    # srslte_ulsch_decode drop-in (PUSCH data at this cell's bandwidth, QPSK / 16QAM / 64QAM, with
    # and without SRS, HARQ rv 0-2-3-1): return code, data, g bits, noi and cb_crc exact
    assert int(stats["ulsch"]) >= 6 and int(stats["ulsch_mismatches"]) == 0, r.stdout + r.stderr
    assert int(stats["ulsch_ok"]) >= 1, r.stdout + r.stderr


# the 8-bit LLR chain (llr_is_8bit on the PDSCH and its DL-SCH, pdsch.c:795-806, sch.c:344-364):
# same arguments plus llr8 = 1. The 8-bit HARQ combining wraps at 8 bits, as the reference's does.
CASES8 = [
    (25, 301, 16, 1, 1, 0, 6, 12.0, 11, 1),  # 16QAM, 25 PRB (AVX8 window at K = 6144 / 3136...)
    (50, 503, 27, 2, 2, 1, 4, 18.0, 12, 1),  # 64QAM, 2 rx, CSI (8-bit weighting)
    (100, 12, 28, 2, 1, 0, 3, 21.0, 13, 1),  # 20 MHz, 13 code blocks
    (25, 7, 16, 2, 2, 0, 6, 16.0, 14, 3),    # TM3 CDD 2x2, two 16QAM TBs
    (15, 41, 22, 2, 2, 1, 6, 16.0, 15, 2),   # TM2 transmit diversity, CSI
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES8,
                         ids=[f"llr8_tm{c[9]}_prb{c[0]}_mcs{c[2]}_rx{c[4]}_csi{c[5]}" for c in CASES8])
def test_shim_pdsch_decode_8bit_matches_reference(case):
    if not os.path.exists(CHECK):
        pytest.skip("oracle/_ref/shim_check not built (needs /root/reference at build time)")
    r = subprocess.run([CHECK] + [str(v) for v in case] + ["1"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    stats = dict(kv.split("=") for kv in r.stdout.split())
    assert int(stats["mismatches"]) == 0 and int(stats["tx"]) >= case[6], r.stdout + r.stderr
    assert int(stats["soft"]) <= max(1, int(stats["tx"]) // 10), r.stdout + r.stderr
    assert int(stats["dlsch_mismatches"]) == 0 and int(stats["rm_mismatches"]) == 0, r.stdout + r.stderr


FRONT = os.path.join(REPO, "oracle", "_ref", "shim_front")
# nof_prb_a, nof_prb_b, cell_id, mcs, nof_rx, nof_sf, snr_db, seed
FRONT_CASES = [
    (25, 6, 33, 16, 2, 10, 24.0, 1),   # 5 MHz -> 1.4 MHz, 2 rx
    (100, 50, 400, 22, 1, 10, 26.0, 2),  # 20 MHz -> 10 MHz
    (6, 15, 502, 9, 2, 10, 20.0, 3),   # 1.4 MHz -> 3 MHz (odd PRB count), cell id 502 -> 503
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", FRONT_CASES, ids=[f"prb{c[0]}to{c[1]}_rx{c[4]}" for c in FRONT_CASES])
def test_shim_front_end_time_domain(case):
    """shim srslte_ofdm_rx_sf -> srslte_chest_dl_estimate_multi -> srslte_pdsch_decode on a time
    signal (oracle/shim_front.c): OFDM grid within 1e-4 of the transmitted one, channel estimate
    close to the true channel, noise / RSRP / RSSI / CFO written back into the reference object
    (EMPTY noise only in subframes 0 and 5), the PDSCH decode bit-exact with the reference CPU
    decoder on the same grids and estimates, GPU handles recreated after the cell change and all
    released through srsgpu_shim_release"""
    if not os.path.exists(FRONT):
        pytest.skip("oracle/_ref/shim_front not built (needs /root/reference at build time)")
    r = subprocess.run([FRONT] + [str(v) for v in case], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    stats = dict(kv.split("=") for kv in r.stdout.split())
    assert int(stats["mismatches"]) == 0 and int(stats["sf"]) == 2 * case[5]
    assert float(stats["ofdm_err"]) < 1e-4 and float(stats["ce_err"]) < 0.2, r.stdout
    assert int(stats["recreated"]) == 1 and int(stats["live"]) == 0
    assert int(stats["acks"]) >= case[5]  # at least the high-SNR phase decodes


FAULT = os.path.join(REPO, "oracle", "_ref", "shim_fault")


@pytest.mark.gpu
def test_shim_error_paths_and_harq_growth():
    """oracle/_ref/shim_fault: every device allocation the shim makes is failed once in turn (the
    drop-in must return SRSLTE_ERROR and work again on the next call), and one srslte_sch_t decodes
    two HARQ processes whose grants differ in size, interleaved, exactly as the reference does
    (the larger grant must not drop the other process's combined soft bits)."""
    if not os.path.exists(FAULT):
        pytest.skip("oracle/_ref/shim_fault not built (needs /root/reference at build time)")
    r = subprocess.run([FAULT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    stats = dict(kv.split("=") for kv in r.stdout.split())
    assert int(stats["fault_cases"]) >= 8 and int(stats["fault_failures"]) == 0, r.stdout + r.stderr
    assert int(stats["harq_tx"]) == 36 and int(stats["harq_mismatches"]) == 0, r.stdout + r.stderr
