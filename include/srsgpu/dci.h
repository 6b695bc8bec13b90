/*
 * srsgpu DCI handling on the host — sizes, unpacking and the DL grant of a decoded DCI message
 * (the step between the PDCCH blind search, srsgpu/pdcch_batch.h, and the PDSCH decode).
 *
 * Restates (reference paths relative to /root/reference/lib):
 *   srslte_dci_format_sizeof          src/phy/phch/dci.c:223-360, :463-493
 *   srslte_dci_msg_unpack_pdsch       src/phy/phch/dci.c:1332-1356 with the format unpackers
 *                                     (1 :680, 1A :829, 1B :933, 1C :1035, 1D :1076, 2/2A/2B :1205)
 *   srslte_dci_msg_to_dl_grant        src/phy/phch/dci.c:49-90
 *   srslte_ra_dl_dci_to_grant         src/phy/phch/ra.c:292-425 (PRB allocation types 0, 1, 2
 *                                     localised and distributed), :427-455, :509-561, :583-612
 *   srslte_ra_tbs_from_idx            src/phy/phch/ra.c:725 (36.213 Table 7.1.7.2.1-1)
 *   srslte_dci_msg_to_ul_grant        src/phy/phch/dci.c:165-197 with dci_format0_unpack (:571-626),
 *                                     srslte_ra_ul_dci_to_grant (ra.c:118-245: PUSCH hopping type 1 / 2,
 *                                     MCS / TBS / redundancy version of 36.213 8.6)
 * with the reference's field semantics and error returns; tests/test_dci.py checks every function
 * against the reference build. Pure host code: no GPU needed.
 */
#ifndef SRSGPU_DCI_H
#define SRSGPU_DCI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* srslte_dci_format_t order */
enum {
  SRSGPU_DCI_FORMAT0 = 0,
  SRSGPU_DCI_FORMAT1,
  SRSGPU_DCI_FORMAT1A,
  SRSGPU_DCI_FORMAT1C,
  SRSGPU_DCI_FORMAT1B,
  SRSGPU_DCI_FORMAT1D,
  SRSGPU_DCI_FORMAT2,
  SRSGPU_DCI_FORMAT2A,
  SRSGPU_DCI_FORMAT2B,
  SRSGPU_DCI_NOF_FORMATS
};

/* srslte_ra_dl_dci_t (ra.h); the reference keeps the three allocation types in a union, here they
 * are separate fields and only the decoded type's are set */
typedef struct {
  uint32_t alloc_type;                   /* 0, 1, 2 */
  uint32_t rbg_bitmask;                  /* type 0 */
  uint32_t vrb_bitmask, rbg_subset, shift; /* type 1 */
  uint32_t riv, L_crb, RB_start, n_prb1a, n_gap, mode; /* type 2 (mode 0 localised, 1 distributed) */
  uint32_t harq_process, mcs_idx;
  int32_t rv_idx;
  uint32_t ndi, mcs_idx_1;
  int32_t rv_idx_1;
  uint32_t ndi_1, tb_cw_swap, sram_id, pinfo, pconf, power_offset;
  uint32_t tb_en[2];
  uint32_t is_ra_order, ra_preamble, ra_mask_idx, dci_is_1a, dci_is_1c;
} srsgpu_ra_dl_dci_t;

/* srslte_ra_dl_grant_t (ra.h): prb_idx[slot][prb] as bytes */
typedef struct {
  uint8_t prb_idx[2][110];
  uint32_t nof_prb;
  uint32_t Qm[2];
  uint32_t mod[2];  /* srslte_mod_t: 0 BPSK, 1 QPSK, 2 16QAM, 3 64QAM */
  int32_t tbs[2];
  uint32_t mcs_idx[2];
  uint32_t tb_en[2];
  uint32_t pinfo, tb_cw_swap;
} srsgpu_ra_dl_grant_t;

/* srslte_ra_ul_dci_t (ra.h:172-194), format 0 */
typedef struct {
  int32_t freq_hop_fl;      /* -1 disabled, 0 quarter, 1 minus quarter, 2 half, 3 type 2 */
  uint32_t riv, L_crb, RB_start;
  uint32_t mcs_idx, rv_idx, n_dmrs, ndi, cqi_request, tpc_pusch;
} srsgpu_ra_ul_dci_t;

/* srslte_ra_ul_grant_t (ra.h:150-169) */
typedef struct {
  uint32_t L_prb, n_prb[2], freq_hopping, M_sc, M_sc_init, Qm;
  uint32_t mod;             /* srslte_mod_t; 4 = SRSLTE_MOD_LAST (mcs 29-31: keep the last one) */
  int32_t tbs;              /* -1 with SRSLTE_MOD_LAST */
  uint32_t mcs_idx, ncs_dmrs;
} srsgpu_ra_ul_grant_t;

uint32_t srsgpu_dci_format_sizeof(uint32_t format, uint32_t nof_prb, uint32_t nof_ports);
/* srslte_dci_msg_to_dl_grant: bits is the message buffer as srslte_dci_msg_t.data holds it
 * (SRSGPU_DCI_MAX_BITS = 128 bytes, one bit per byte: nof_bits payload bits, then what the decoder
 * left there — srsgpu_dci_result_t.data carries the CRC bits), format the one the search reported.
 * The unpackers read as dci.c does, which for Format 1C with N_gap,2 goes past the payload. -1 (SRSLTE_ERROR) if the message does not unpack; else 0,
 * also when the grant itself is invalid (dci.c:71-76 returns the unpack's status then, with the
 * grant as far as ra.c filled it: check it with srsgpu_ra_dl_dci_to_grant). A random-access order
 * (1A) returns 0 with dci->is_ra_order set and no grant. */
int srsgpu_dci_msg_to_dl_grant(const uint8_t *bits, uint32_t nof_bits, uint32_t format, uint16_t rnti,
                               uint32_t nof_prb, uint32_t nof_ports, srsgpu_ra_dl_dci_t *dci,
                               srsgpu_ra_dl_grant_t *grant);
/* srslte_ra_dl_dci_to_grant (ra.c:583-612): the PRB allocation and MCS / TBS of an unpacked DCI;
 * 0, or -1 on an invalid allocation or MCS (grant filled up to the failing step). A Format 1C for
 * RA- or P-RNTI sets dci->rv_idx = 0 (36.213 7.1.7.3). */
int srsgpu_ra_dl_dci_to_grant(srsgpu_ra_dl_dci_t *dci, uint32_t nof_prb, uint16_t rnti,
                              srsgpu_ra_dl_grant_t *grant);
/* srslte_dci_msg_to_ul_grant (dci.c:165-197): unpack a format 0 message (bits / nof_bits as above) and
 * compute its PUSCH grant with hopping offset n_rb_ho (pusch_hopping.hopping_offset). -1 (SRSLTE_ERROR)
 * if the message is not a format 0 of this bandwidth or the allocation does not fit (dci / grant as far
 * as the reference filled them), else 0. */
int srsgpu_dci_msg_to_ul_grant(const uint8_t *bits, uint32_t nof_bits, uint32_t nof_prb, uint32_t n_rb_ho,
                               srsgpu_ra_ul_dci_t *dci, srsgpu_ra_ul_grant_t *grant);
/* 36.213 Table 7.1.7.2.1-1: -1 outside tbs_idx < 27, 1 <= nof_prb <= 110 */
int srsgpu_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t nof_prb);
/* srslte_ra_tbs_idx_from_mcs (ra.c:697): -1 for mcs >= 29 */
int srsgpu_ra_tbs_idx_from_mcs(uint32_t mcs);

#ifdef __cplusplus
}
#endif
#endif
