/*
 * srsgpu batched PDSCH receiver — C ABI of the MI355X (gfx950) path from the received resource
 * grid and its channel estimate to decoded transport blocks.
 *
 * Per subframe and codeword, this follows the reference's srslte_pdsch_decode
 * (reference: lib/src/phy/phch/pdsch.c:868-1007, srslte_pdsch_codeword_decode :778-835):
 *   - RE extraction of the grant (srslte_pdsch_get, pdsch.c:95-234);
 *   - SISO ZF/MMSE equalisation over 1-2 rx antennas (srslte_predecoding_single_multi,
 *     mimo/precoding.c:243-352), or TM3 large-delay CDD 2x2 MMSE over 2 ports and 2 rx antennas
 *     (srslte_predecoding_ccd_mmse, precoding.c:930-1097), or TM2 transmit diversity over 2 or 4
 *     ports and 1-2 rx antennas (srslte_predecoding_diversity_multi + srslte_layerdemap_diversity,
 *     precoding.c:356-685, layermap.c:143-151; with 4 ports over RE quadruplets, which normal-CP
 *     grants always fill), optionally with CSI;
 *   - soft demapping to int16 LLRs (srslte_demod_soft_demodulate_s, modem/demod_soft.c);
 *   - descrambling with the PDSCH Gold sequence (scrambling.c:48-51, sequences.c:64-66);
 *   - optional CSI weighting (csi_correction, pdsch.c:676-776);
 *   - DL-SCH decoding into the softbuffers of include/srsgpu/dlsch_batch.h.
 * Everything for a batch of subframes runs as a few fused kernel launches on the handle's
 * stream.
 *
 * Grid layout (as srslte_ofdm_rx_sf produces and srslte_chest_dl_estimate consumes): per
 * subframe and rx antenna, 14 OFDM symbols x nof_prb*12 subcarriers of complex float. Channel
 * estimates use the same plane layout, one plane per (rx antenna, port) in that order, which is
 * the order srsgpu_chest_estimate_dev writes them. Plane a of the grid starts at
 * d_grid + grid_offset + a*ant_stride; plane (a, p) of the estimate at
 * d_ce + ce_offset + (a*nof_ports + p)*ant_stride.
 *
 * Transport blocks of a call are numbered in subframe order, TB 0 then TB 1 of a CDD subframe:
 * d_ret / d_noi / e_offset have one entry per TB in that order.
 */
#ifndef SRSGPU_PDSCH_BATCH_H
#define SRSGPU_PDSCH_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "srsgpu/dlsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_pdsch srsgpu_pdsch_t;

typedef struct {
  uint32_t nof_prb;    /* cell bandwidth in PRB (6..110) */
  uint32_t id;         /* physical cell id (0..503) */
  uint32_t nof_ports;  /* CRS ports: the RE map skips their reference signals; SISO decoding
                          needs 1 port */
  uint32_t nof_rx_ant; /* 1 or 2 */
  uint32_t cp;         /* srslte_cp_t: 0 normal (7 symbols per slot), 1 extended (6 symbols per slot,
                          CRS in symbols 0 / 3 of each slot, srslte_refsignal_cs_nsymbol) */
} srsgpu_cell_t;

/* srslte_mimo_type_t values accepted by the GPU receiver */
#define SRSGPU_MIMO_SINGLE_ANTENNA 0 /* 1 CRS port, 1 layer, 1 TB (TM1), 1-2 rx antennas */
#define SRSGPU_MIMO_TX_DIVERSITY 1   /* TM2 / DCI 1A on 2-port cells: SFBC over RE pairs, 1 TB, 1-2 rx */
#define SRSGPU_MIMO_SPATIAL_MULTIPLEX 2 /* TM4 closed-loop spatial multiplexing: 2 ports, 2 rx antennas;
                                          2 TBs on 2 layers (2x2 MMSE, codebook_idx 0..2) or 1 TB on
                                          1 layer (2x1 MRC, codebook_idx 0..3) */
#define SRSGPU_MIMO_CDD 3            /* TM3 large-delay CDD: 2 ports, 2 layers, 2 TBs, 2 rx antennas */

typedef struct {
  uint32_t sf_idx;          /* subframe index 0..9 */
  uint32_t lstart;          /* first PDSCH OFDM symbol (srslte_ra_nbits_t.lstart) */
  uint8_t prb_idx[2][110];  /* srslte_ra_dl_grant_t.prb_idx: PRB allocation per slot */
  uint32_t nof_re;          /* srslte_ra_nbits_t.nof_re: must equal the grant's RE count */
  uint16_t rnti;
  float noise_estimate;     /* MMSE term (0 = ZF) */
  float scaling;            /* pdsch_scaling (rho_a, 1.0 by default) */
  uint32_t mimo_type;       /* SRSGPU_MIMO_SINGLE_ANTENNA, SRSGPU_MIMO_TX_DIVERSITY or SRSGPU_MIMO_CDD */
  uint32_t tb_cw_swap;      /* srslte_pdsch_cfg_t.tb_cw_swap (CDD): TB 0 on codeword 1 */
  /* per transport block (index 1 only with CDD) */
  uint32_t mod[2];          /* srslte_mod_t: 0 BPSK, 1 QPSK, 2 16QAM, 3 64QAM */
  uint32_t tbs[2], rv[2], softbuffer[2];
  uint64_t grid_offset;     /* this subframe's [rx antenna] grid planes in d_grid (complex elements) */
  uint64_t ce_offset;       /* this subframe's [rx antenna][port] estimate planes in d_ce */
  uint64_t data_offset[2];  /* first output byte of each TB in d_data */
  uint32_t codebook_idx;    /* srslte_pdsch_cfg_t.codebook_idx (spatial multiplexing only; with
                               tbs[1] > 0 two TBs on two layers, else one TB on one layer) */
  uint32_t skip_tb;         /* bit t set: TB t is not decoded, as srslte_pdsch_decode skips a TB whose
                               acks[t] is already true (pdsch.c:946-947). Its softbuffer and data bytes
                               are not touched; its d_ret / d_noi entries are written as 0. The
                               subframe's equalisation still runs (a 2-layer equaliser needs both). */
} srsgpu_pdsch_sf_t;

/* nof_softbuffers HARQ softbuffers of max_cb code blocks; up to max_sf subframes per call. */
int srsgpu_pdsch_create(srsgpu_pdsch_t **q, const srsgpu_cell_t *cell, uint32_t nof_softbuffers,
                        uint32_t max_cb, uint32_t max_sf);
void srsgpu_pdsch_destroy(srsgpu_pdsch_t *q);
void srsgpu_pdsch_set_stream(srsgpu_pdsch_t *q, void *hip_stream);
void srsgpu_pdsch_set_csi(srsgpu_pdsch_t *q, int enable); /* srslte_pdsch_enable_csi */
/* srslte_pdsch_t.llr_is_8bit (+ srslte_sch_t.llr_is_8bit of its DL-SCH): int8 soft demapping
 * (srslte_demod_soft_demodulate_b), int8 scrambling (srslte_scrambling_sb_offset), the 8-bit CSI
 * weighting (pdsch.c:707-713), 8-bit de-rate-matching and decoders (pdsch.c:795-806,
 * sch.c:344-364). The LLRs stay int16 elements holding int8 values. */
void srsgpu_pdsch_set_llr_8bit(srsgpu_pdsch_t *q, int enable);
/* The estimate planes passed to srsgpu_pdsch_decode(_dev) hold the compact rows of
 * srsgpu_chest_set_ce_rows: rows = 4 (per-symbol estimation: the CRS symbols' rows, time
 * interpolation done per resource element with the estimator's operations, so the LLRs are
 * identical), 1 (average_subframe: the averaged row), 0 (default: full 14-symbol planes).
 * Returns -1 for any other value, and for rows = 4 on an extended-CP cell or a cell of more than
 * 2 ports (the estimator writes compact rows only for those it can: chest_batch.h). */
int srsgpu_pdsch_set_ce_rows(srsgpu_pdsch_t *q, int rows);
/* Take the MMSE noise term from device memory instead of sf[i].noise_estimate: subframe i of a
 * call uses the mean of d_noise[i*nof_rx_ant + a] (the channel estimator's per-antenna outputs,
 * as srslte_chest_dl_get_noise_estimate averages them). NULL restores sf[i].noise_estimate. */
void srsgpu_pdsch_set_noise_dev(srsgpu_pdsch_t *q, const float *d_noise);
/* the DL-SCH engine owning the softbuffers (reset them with srsgpu_dlsch_softbuffer_reset) */
srsgpu_dlsch_t *srsgpu_pdsch_get_dlsch(srsgpu_pdsch_t *q);

/* LLRs only: d_e receives nof_re * Qm descrambled int16 LLRs per TB at e_offset[tb] (host array,
 * one entry per TB of the call). */
int srsgpu_pdsch_llr_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t nof_sf,
                         const float *d_grid, const float *d_ce, size_t ant_stride, int16_t *d_e,
                         const uint64_t *e_offset);

/* Full decode: LLRs then DL-SCH. d_ret[t] = srslte_dlsch_decode2's result for TB t (0: decoded
 * with a good CRC, i.e. ack; -1: CRC error; -2: invalid TB), d_noi[t] = nof_iterations. Returns
 * -1 on invalid input (RE count mismatch: pdsch.c:886-890; a MIMO type the cell cannot carry). */
int srsgpu_pdsch_decode_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t nof_sf,
                            const float *d_grid, const float *d_ce, size_t ant_stride,
                            uint8_t *d_data, uint32_t max_halfits, int32_t *d_ret, uint32_t *d_noi);

/* As srsgpu_pdsch_decode_dev with TB t of the call (subframe order, TB 0 then TB 1) written at d_out[t]
 * (data_offset ignored): device memory or host memory the device can address (srsgpu_dlsch_decode_out_dev). */
int srsgpu_pdsch_decode_out_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t nof_sf,
                                const float *d_grid, const float *d_ce, size_t ant_stride,
                                uint8_t *const *d_out, uint32_t max_halfits, int32_t *d_ret, uint32_t *d_noi);

/* Transmit side, used to synthesise traffic on the device (srslte_pdsch_encode, pdsch.c:1048-1131,
 * single antenna port): per subframe, DL-SCH encoding of TB 0 (srsgpu_dlsch_encode_dev, rv from
 * sf[i].rv[0]), scrambling, modulation (modem/lte_tables.c), rho_a scaling and RE mapping into
 * the port-0 grid at d_grid + grid_offset. REs outside the grant (CRS, control region) are left
 * as they are: srsgpu_chest_put_crs_dev writes the CRS. */
int srsgpu_pdsch_encode_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t nof_sf,
                            const uint8_t *d_data, float *d_grid);
/* The same for every MIMO type of the receiver (srslte_pdsch_encode with srslte_layermap_type and
 * srslte_precoding_type, pdsch.c:1048-1131, layermap.c:43-130, precoding.c:1849-2143): per TB the DL-SCH
 * encoding (rv, data at data_offset[tb]), each codeword (cw = tb ^ tb_cw_swap with two TBs) scrambled
 * with its own sequence and modulated, then single antenna, transmit diversity (2-port SFBC or 4-port
 * SFBC over RE quadruplets on port pairs 0/2 and 1/3, precoding.c:1863-1889), large-delay
 * CDD (2 ports, 2 TBs) or codebook precoding (2 ports, codebook_idx; 1 TB on 1 layer or 2 TBs on 2
 * layers), rho_a scaling, and the RE mapping of every port: port p of subframe i at
 * d_grid + sf[i].grid_offset + p * port_stride. Transmit diversity with an odd RE count leaves the last
 * RE of each port as it is (the reference precodes 2 floor(n / 2) symbols). */
int srsgpu_pdsch_encode_ports_dev(srsgpu_pdsch_t *q, const srsgpu_pdsch_sf_t *sf, uint32_t nof_sf,
                                  const uint8_t *d_data, float *d_grid, size_t port_stride);

/* TM3 / TM4 feedback from a subframe's channel estimates, as srsUE's PHY worker computes it for its
 * uplink control information (phch_worker.cc:522-540):
 *   - condition number (srslte_pdsch_cn_compute -> srslte_precoding_cn, precoding.c:2889-2922: the mean
 *     over every 24th estimate of 10 log10(lambda_max / lambda_min) of H H', 2 ports x 2 rx antennas only)
 *     and the TM3 rank of srslte_ue_dl_ri_select (ue_dl.c:747-764: 1 below 17 dB);
 *   - the per-layer PMI choice of srslte_pdsch_pmi_select (pdsch.c:1009-1041 ->
 *     srslte_precoding_pmi_select_1l / _2l, precoding.c:2335-2860, AVX forms: four estimates every 96,
 *     every 24 apart) and the rank / PMI of srslte_ue_dl_ri_pmi_select (ue_dl.c:684-745), 2 ports, 1-2 rx.
 * The one-layer SINRs follow the reference's operations (FMA complex products) exactly; the two-layer
 * ones use exact reciprocals where the reference uses _mm256_rcp_ps (relative error <= 1.5 * 2^-12), and
 * the condition number the device log10f. A codebook whose SINR never exceeds 0 leaves its PMI at 0 (the
 * reference keeps the value its object held). */
typedef struct {
  uint64_t ce_offset;   /* the subframe's full [rx antenna][port] estimate planes in d_ce (complex elements) */
  float noise_estimate; /* srslte_chest_dl_get_noise_estimate of the subframe */
  uint32_t flags;       /* SRSGPU_FEEDBACK_CN | SRSGPU_FEEDBACK_PMI */
} srsgpu_feedback_sf_t;
#define SRSGPU_FEEDBACK_CN 1u  /* condition number + TM3 rank (2 ports, 2 rx antennas) */
#define SRSGPU_FEEDBACK_PMI 2u /* per-layer PMI / SINR + TM4 rank / PMI (2 ports) */
typedef struct {
  float cn;             /* dB; 0 when not computed */
  uint32_t ri_tm3;      /* srslte_ue_dl_ri_select: 1 (two layers) when cn < 17 dB */
  int32_t ret_cn;       /* 0, or -1 where the reference's call fails (not 2 x 2) or it was not asked */
  uint32_t ri, pmi;     /* srslte_ue_dl_ri_pmi_select's rank index (layers - 1) and PMI */
  uint32_t pmi_l[2];    /* srslte_precoding_pmi_select's PMI for 1 and 2 layers */
  int32_t ret_pmi;      /* 0, or -1 (not 2 ports, or not asked) */
  float sinr[2][4];     /* q->sinr[layers - 1][codebook]; layers above the rx antennas: -inf; the two-layer
                           codebooks 2, 3: 0 */
} srsgpu_feedback_t;
/* nof_sf subframes of the cell's estimate planes (ant_stride complex elements apart) -> d_out[nof_sf]
 * (device memory), one launch on the handle's stream. d_noise (may be NULL): subframe i's noise estimate
 * is d_noise[i] instead of sf[i].noise_estimate. */
int srsgpu_pdsch_feedback_dev(srsgpu_pdsch_t *q, const srsgpu_feedback_sf_t *sf, uint32_t nof_sf,
                              const float *d_ce, size_t ant_stride, const float *d_noise, srsgpu_feedback_t *d_out);

/* RE count of a grant (srslte_pdsch_get's return value). */
int srsgpu_pdsch_nof_re(const srsgpu_cell_t *cell, const srsgpu_pdsch_sf_t *sf);

#ifdef __cplusplus
}
#endif
#endif
