/*
 * srsgpu batched PDCCH receiver — C ABI of the MI355X (gfx950) control-channel search that turns
 * a subframe's equalised control region into the UE's DL DCI (reference
 * paths relative to /root/reference/lib):
 *   - srslte_regs_init / regs_pdcch_init (src/phy/phch/regs.c:82-158, :681-763): the REG grid,
 *     PCFICH and PHICH REGs (:256-331, :477-512) and the interleaved, cyclically shifted PDCCH REG
 *     order for each CFI; srslte_pdcch_set_cell (src/phy/phch/pdcch.c:177-208): NOF_CCE(cfi)
 *     and the ten subframe scrambling sequences (sequences.c:57-59);
 *   - srslte_pdcch_extract_llr_multi (pdcch.c:424-506) for many subframes per launch: REG
 *     gather, 1-port or transmit-diversity predecoding, float QPSK demapping, descrambling;
 *   - the DL blind search of srslte_ue_dl_find_dl_dci (src/phy/ue/ue_dl.c:768-923): candidate
 *     locations (pdcch.c:227-300), srslte_pdcch_decode_msg on every candidate (the batched
 *     decoder of srsgpu/viterbi_batch.h), RNTI match on the CRC remainder and the reference's
 *     search order (UE-specific formats of the transmission mode, then the common 1A; 1A and 1C
 *     in the common space for SI / P / RA-RNTI), first match wins.
 * Bit-exact with the reference in LLRs and found DCIs (tests/test_pdcch.py).
 * Grid / estimate layout as srsgpu/pdsch_batch.h: plane a of the grid at d_grid + grid_offset +
 * a * ant_stride, plane (a, p) of the estimate at d_ce + ce_offset + (a * nof_ports + p) * ant_stride.
 */
#ifndef SRSGPU_PDCCH_BATCH_H
#define SRSGPU_PDCCH_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "srsgpu/pdsch_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct srsgpu_pdcch srsgpu_pdcch_t;

/* srslte_pdcch_init_ue + srslte_pdcch_set_cell on srslte_regs_init(cell): phich_length 0 normal /
 * 1 extended, phich_resources 0..3 = 1/6, 1/2, 1, 2 (srslte_phich_length_t /
 * srslte_phich_resources_t). -1 on an invalid cell (1-2 ports, 1-2 rx antennas, 6-110 PRB). */
int srsgpu_pdcch_create(srsgpu_pdcch_t **q, const srsgpu_cell_t *cell, uint32_t phich_length,
                        uint32_t phich_resources);
void srsgpu_pdcch_destroy(srsgpu_pdcch_t *q);
/* The same map for a cell without a GPU object (host only): the symbol count, NOF_CCE(cfi) in
 * *nof_cce; idx may be NULL to ask for the count. -1 on invalid input. */
int srsgpu_pdcch_cell_map(const srsgpu_cell_t *cell, uint32_t phich_length, uint32_t phich_resources,
                          uint32_t cfi, uint32_t *idx, uint32_t max, uint32_t *nof_cce);
/* NOF_CCE(cfi) of pdcch.c (0 for cfi outside 1..3) */
uint32_t srsgpu_pdcch_nof_cce(const srsgpu_pdcch_t *q, uint32_t cfi);
/* Take each subframe's noise estimate from device memory instead of sf[i].noise_estimate: subframe
 * i of a srsgpu_pdcch_extract_llr_dev call uses d_noise[i]. NULL restores sf[i].noise_estimate. */
void srsgpu_pdcch_set_noise_dev(srsgpu_pdcch_t *q, const float *d_noise);
/* the 36 NOF_CCE(cfi) grid indices (l * 12 nof_prb + k) in srslte_regs_pdcch_get order; returns
 * their count, or -1 if max is too small */
int srsgpu_pdcch_re_map(const srsgpu_pdcch_t *q, uint32_t cfi, uint32_t *idx, uint32_t max);

typedef struct {
  uint64_t grid_offset; /* this subframe's [rx antenna] grid planes (complex elements) */
  uint64_t ce_offset;   /* this subframe's [rx antenna][port] estimate planes */
  uint64_t llr_offset;  /* first of its 72 NOF_CCE(cfi) float LLRs in d_llr (even) */
  uint32_t sf_idx;      /* subframe 0..9 */
  uint32_t cfi;         /* 1..3 (from the PCFICH) */
  float noise_estimate; /* srslte_pdcch_extract_llr_multi's noise_estimate */
  uint32_t reserved;
} srsgpu_pdcch_sf_t;

/* srslte_pdcch_extract_llr_multi for nof_sf subframes (sf: host array). Asynchronous on
 * hip_stream (NULL: the null stream). 0, or -1 on invalid input. */
int srsgpu_pdcch_extract_llr_dev(srsgpu_pdcch_t *q, const srsgpu_pdcch_sf_t *sf, uint32_t nof_sf,
                                 const float *d_grid, const float *d_ce, size_t ant_stride,
                                 float *d_llr, void *hip_stream);

typedef struct {
  uint32_t L;    /* aggregation level index: 2^L CCEs */
  uint32_t ncce; /* first CCE */
} srsgpu_dci_location_t;
/* srslte_pdcch_ue_locations_ncce (pdcch.c:227-266) / srslte_pdcch_common_locations_ncce
 * (:274-300): candidate locations in the reference's order; return their count */
uint32_t srsgpu_pdcch_ue_locations(uint32_t nof_cce, uint32_t sf_idx, uint16_t rnti,
                                   srsgpu_dci_location_t *c, uint32_t max);
uint32_t srsgpu_pdcch_common_locations(uint32_t nof_cce, srsgpu_dci_location_t *c, uint32_t max);

/* One DL DCI search (srslte_ue_dl_find_dl_dci / _find_dl_dci_type, ue_dl.c:840-923): a subframe's
 * LLRs (extracted with this cfi) and the RNTI the UE looks for. tm is the reference's argument: the
 * row of ue_dci_formats (ue_dl.c:41-50), 0..7 for transmission modes 1..8 (srsUE passes the RRC
 * tx_mode enum, phch_worker.cc:626). rnti_type < 0 derives the search from the RNTI value as
 * srslte_ue_dl_find_dl_dci does; otherwise it is a srslte_rnti_type_t as _find_dl_dci_type takes
 * it (SI = 1, RAR = 2, PCH = 5: common space 1A then 1C; any other: the C-RNTI search). */
typedef struct {
  uint64_t llr_offset;
  uint32_t sf_idx, cfi;
  uint32_t rnti;       /* the DL search's RNTI (srsgpu_pdcch_find_dci_dev: 0 = no DL search) */
  uint32_t tm;
  int32_t rnti_type;
  uint32_t ul_rnti;    /* srsgpu_pdcch_find_dci_dev only: the UL search's RNTI, 0 = none */
} srsgpu_dci_search_t;

/* result: found 1 / 0, or -1 where the reference's search returns SRSLTE_ERROR (it reaches a
 * location with nCCE > 87, which srslte_pdcch_decode_msg refuses: dci.c:215-221, possible in cells
 * with more than 88 CCEs); format (srsgpu/dci.h SRSGPU_DCI_FORMAT*), location; data is the message
 * buffer as the reference's srslte_dci_msg_t.data holds it after srslte_pdcch_decode_msg: nof_bits
 * payload bits, the 16 CRC bits after them (dci_decode decodes nof_bits + 16), zeros after those */
typedef struct {
  int32_t found;
  uint32_t format, L, ncce, nof_bits;
  uint8_t data[128];
} srsgpu_dci_result_t;

/* srslte_ue_dl_find_dl_dci for nof_search searches (host array) on device LLRs; d_res: device
 * array of nof_search results. Asynchronous on hip_stream. 0, or -1 on invalid input (ul_rnti is
 * ignored). */
int srsgpu_pdcch_find_dl_dci_dev(srsgpu_pdcch_t *q, const srsgpu_dci_search_t *s, uint32_t nof_search,
                                 const float *d_llr, srsgpu_dci_result_t *d_res, void *hip_stream);
/* srsUE's per-subframe PDCCH searches (phch_worker.cc:548-806 then :938-967): the DL search of
 * srslte_ue_dl_find_dl_dci(_type) for rnti (none if 0: d_res then reports -1, the reference's "RNTI not
 * specified" error, ue_dl.c:805-807), then srslte_ue_dl_find_ul_dci for ul_rnti (none if 0: found 0),
 * format 0 in the UE-specific space (ue_dl.c:811-838). A format 0 message the DL 1A search passed over
 * (ue_dl.c:785-792) is the UL result when ul_rnti equals rnti; the search keeps no state between calls
 * (the reference's ue_dl object carries such a message to a later UL search of that RNTI when this
 * subframe's UL search is for another one). d_res_ul: nof_search results (format 0, same layout). */
int srsgpu_pdcch_find_dci_dev(srsgpu_pdcch_t *q, const srsgpu_dci_search_t *s, uint32_t nof_search,
                              const float *d_llr, srsgpu_dci_result_t *d_res, srsgpu_dci_result_t *d_res_ul,
                              void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
