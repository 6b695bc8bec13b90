// srsgpu DCI host functions (include/srsgpu/dci.h): DCI sizes, DL unpacking and the DL grant.
// Restated from the reference (paths relative to /root/reference/lib): src/phy/phch/dci.c and
// src/phy/phch/ra.c, cited per function. Host code: the PDCCH blind search (csrc/pdcch.hip) finds
// the message on the GPU, this turns it into the PDSCH grant.
#include <math.h>
#include <string.h>

#include "lte_tables.h"
#include "srsgpu/dci.h"

namespace {

constexpr uint32_t kHarqPidLen = 3;              // dci.c:45
constexpr uint16_t kCrntiStart = 0x000B, kCrntiEnd = 0xFFF3; // phy_common.h:73-74
constexpr uint16_t kRarntiStart = 0x0001, kRarntiEnd = 0x000A, kPrnti = 0xFFFE;

// srslte_bit_pack: n bits MSB first
uint32_t bit_pack(const uint8_t **y, int n) {
  uint32_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 1) | ((*y)[i] & 1u);
  *y += n;
  return v;
}

// dci.c:223-240
uint32_t riv_nbits(uint32_t nof_prb) {
  return (uint32_t)ceilf(log2f((float)nof_prb * ((float)nof_prb + 1) / 2));
}
bool is_ambiguous_size(uint32_t size) {
  static const uint32_t amb[10] = {12, 14, 16, 20, 24, 26, 32, 40, 44, 56};
  for (uint32_t a : amb)
    if (size == a) return true;
  return false;
}

// ra.c:614-695
uint32_t ra_type0_P(uint32_t nof_prb) { return nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4; }
uint32_t ra_type1_N_rb(uint32_t nof_prb) {
  const uint32_t P = ra_type0_P(nof_prb);
  return (uint32_t)ceilf((float)nof_prb / P) - (uint32_t)ceilf(log2f((float)P)) - 1;
}
void ra_type2_from_riv(uint32_t riv, uint32_t *L_crb, uint32_t *RB_start, uint32_t nof_prb, uint32_t nof_vrb) {
  *L_crb = riv / nof_prb + 1;
  *RB_start = riv % nof_prb;
  if (*L_crb > nof_vrb - *RB_start) {
    *L_crb = nof_prb - (int)(riv / nof_prb) + 1;
    *RB_start = nof_prb - riv % nof_prb - 1;
  }
}
uint32_t ra_type2_ngap(uint32_t nof_prb, bool ngap_is_1) {
  if (nof_prb <= 10) return nof_prb / 2;
  if (nof_prb == 11) return 4;
  if (nof_prb <= 19) return 8;
  if (nof_prb <= 26) return 12;
  if (nof_prb <= 44) return 18;
  if (nof_prb <= 49) return 27;
  if (nof_prb <= 63) return ngap_is_1 ? 27 : 9;
  if (nof_prb <= 79) return ngap_is_1 ? 32 : 16;
  return ngap_is_1 ? 48 : 16;
}
uint32_t ra_type2_n_rb_step(uint32_t nof_prb) { return nof_prb < 50 ? 2 : 4; }
uint32_t ra_type2_n_vrb_dl(uint32_t nof_prb, bool ngap_is_1) {
  const uint32_t ngap = ra_type2_ngap(nof_prb, ngap_is_1);
  if (ngap_is_1) return 2 * (ngap < nof_prb - ngap ? ngap : nof_prb - ngap);
  return (nof_prb / ngap) * 2 * ngap;
}

// dci.c:242-360: payload sizes
uint32_t f0_sizeof_(uint32_t nof_prb) { return 1 + 1 + riv_nbits(nof_prb) + 5 + 1 + 2 + 3 + 1; }
uint32_t f1A_sizeof(uint32_t nof_prb) {
  uint32_t n = 1 + 1 + riv_nbits(nof_prb) + 5 + kHarqPidLen + 1 + 2 + 2;
  while (n < f0_sizeof_(nof_prb)) n++;
  if (is_ambiguous_size(n)) n++;
  return n;
}
uint32_t f0_sizeof(uint32_t nof_prb) {
  uint32_t n = f0_sizeof_(nof_prb);
  while (n < f1A_sizeof(nof_prb)) n++;
  return n;
}
uint32_t f1_sizeof(uint32_t nof_prb) {
  uint32_t n = (uint32_t)ceilf((float)nof_prb / ra_type0_P(nof_prb)) + 5 + kHarqPidLen + 1 + 2 + 2;
  if (nof_prb > 10) n++;
  while (n == f0_sizeof(nof_prb) || n == f1A_sizeof(nof_prb) || is_ambiguous_size(n)) n++;
  return n;
}
uint32_t f1C_sizeof(uint32_t nof_prb) {
  const uint32_t gap1 = ra_type2_n_vrb_dl(nof_prb, true), step = ra_type2_n_rb_step(nof_prb);
  uint32_t n = riv_nbits(gap1 / step) + 5;
  if (nof_prb >= 50) n++;
  return n;
}
uint32_t tpmi_bits(uint32_t nof_ports) { return nof_ports <= 2 ? 2 : 4; }
uint32_t f1B_sizeof(uint32_t nof_prb, uint32_t nof_ports) {
  uint32_t n = f1A_sizeof(nof_prb) - 1 + tpmi_bits(nof_ports) + 1;
  while (is_ambiguous_size(n)) n++;
  return n;
}
uint32_t precoding_bits_f2(uint32_t nof_ports) { return nof_ports <= 2 ? 3 : 6; }
uint32_t precoding_bits_f2a(uint32_t nof_ports) { return nof_ports <= 2 ? 0 : 2; }
uint32_t f2x_sizeof(uint32_t nof_prb, uint32_t precoding_bits) {
  uint32_t n = (uint32_t)ceilf((float)nof_prb / ra_type0_P(nof_prb)) + 2 + kHarqPidLen + 1 + 2 * (5 + 1 + 2) +
               precoding_bits;
  if (nof_prb > 10) n++;
  while (is_ambiguous_size(n)) n++;
  return n;
}

// dci.c:680-735 (format 1) and :1205-1303 (formats 2 / 2A / 2B): resource allocation type 0 or 1
bool unpack_type01(const uint8_t **y, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb) {
  d->alloc_type = nof_prb > 10 ? *(*y)++ : 0u;
  const uint32_t P = ra_type0_P(nof_prb), alloc_size = (uint32_t)ceilf((float)nof_prb / P);
  if (d->alloc_type == 0) {
    d->rbg_bitmask = bit_pack(y, (int)alloc_size);
  } else if (d->alloc_type == 1) {
    const int lp = (int)ceilf(log2f((float)P));
    d->rbg_subset = bit_pack(y, lp);
    d->shift = *(*y)++ ? 1u : 0u;
    d->vrb_bitmask = bit_pack(y, (int)alloc_size - lp - 1);
  } else {
    return false;
  }
  return true;
}

// the type-2 RIV of formats 1A / 1B / 1D (dci.c:865-885, :941-960, :1084-1103)
void unpack_type2_riv(const uint8_t **y, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb, bool gap_bit) {
  uint32_t nb_gap = 0;
  if (gap_bit && d->mode == 1 && nof_prb >= 50) {
    nb_gap = 1;
    d->n_gap = *(*y)++;
  }
  const uint32_t nof_vrb = d->mode == 0 ? nof_prb : ra_type2_n_vrb_dl(nof_prb, d->n_gap == 0);
  const uint32_t riv = bit_pack(y, (int)(riv_nbits(nof_prb) - nb_gap));
  ra_type2_from_riv(riv, &d->L_crb, &d->RB_start, nof_prb, nof_vrb);
  d->riv = riv;
}

int unpack_1(const uint8_t *bits, uint32_t nof_bits, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb) {
  if (nof_bits != f1_sizeof(nof_prb)) return -1;
  const uint8_t *y = bits;
  if (!unpack_type01(&y, d, nof_prb)) return -1;
  d->mcs_idx = bit_pack(&y, 5);
  d->harq_process = bit_pack(&y, kHarqPidLen);
  d->ndi = *y++ ? 1u : 0u;
  d->rv_idx = (int32_t)bit_pack(&y, 2);
  d->tb_en[0] = 1;
  d->tb_en[1] = 0;
  return 0;
}

int unpack_1A(const uint8_t *bits, uint32_t nof_bits, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb, bool crnti) {
  if (nof_bits != f1A_sizeof(nof_prb)) return -1;
  const uint8_t *y = bits;
  if (*y++ != 1) return -1; // format 0
  d->dci_is_1a = 1;
  if (*y == 0) { // random access by PDCCH order (dci.c:848-870)
    const int nb = (int)riv_nbits(nof_prb);
    int i = 0;
    while (i < nb && y[1 + i] == 1) i++;
    if (i == nb) {
      i = 1 + 10 + nb;
      while (i < (int)nof_bits - 1 && y[i] == 0) i++;
      if (i == (int)nof_bits - 1) {
        y += 1 + nb;
        d->is_ra_order = 1;
        d->ra_preamble = bit_pack(&y, 6);
        d->ra_mask_idx = bit_pack(&y, 4);
        return 0;
      }
    }
  }
  d->is_ra_order = 0;
  d->alloc_type = 2;
  d->mode = *y++;
  d->n_gap = 0;
  unpack_type2_riv(&y, d, nof_prb, crnti);
  d->mcs_idx = bit_pack(&y, 5);
  d->harq_process = bit_pack(&y, kHarqPidLen);
  if (!crnti) {
    if (nof_prb >= 50 && d->mode == 1)
      d->n_gap = *y++;
    else
      y++; // NDI reserved
  } else {
    d->ndi = *y++ ? 1u : 0u;
  }
  d->rv_idx = (int32_t)bit_pack(&y, 2);
  if (crnti) {
    y += 2; // TPC
  } else {
    y++;                // MSB of TPC reserved
    d->n_prb1a = *y++;  // N_prb_1a for the TBS
  }
  d->tb_en[0] = 1;
  d->tb_en[1] = 0;
  return 0;
}

int unpack_1BD(const uint8_t *bits, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb, uint32_t nof_ports, bool is_1d) {
  const uint8_t *y = bits;
  d->alloc_type = 2;
  d->mode = *y++;
  d->n_gap = 0;
  unpack_type2_riv(&y, d, nof_prb, true);
  d->mcs_idx = bit_pack(&y, 5);
  d->harq_process = bit_pack(&y, kHarqPidLen);
  d->ndi = *y++ ? 1u : 0u;
  d->rv_idx = (int32_t)bit_pack(&y, 2);
  y += 2; // TPC for PUCCH
  d->pinfo = bit_pack(&y, (int)tpmi_bits(nof_ports));
  if (is_1d)
    d->power_offset = *y++ ? 1u : 0u;
  else
    d->pconf = *y++ ? 1u : 0u;
  d->tb_en[0] = 1;
  d->tb_en[1] = 0;
  return 0;
}

int unpack_1C(const uint8_t *bits, uint32_t nof_bits, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb) {
  if (nof_bits != f1C_sizeof(nof_prb)) return -1;
  const uint8_t *y = bits;
  d->dci_is_1c = 1;
  d->alloc_type = 2;
  d->mode = 1;
  if (nof_prb >= 50) d->n_gap = *y++;
  const uint32_t n_step = ra_type2_n_rb_step(nof_prb);
  const uint32_t n_vrb_dl = ra_type2_n_vrb_dl(nof_prb, d->n_gap == 0);
  const uint32_t riv = bit_pack(&y, (int)riv_nbits(n_vrb_dl / n_step));
  const uint32_t n_vrb_p = n_vrb_dl / n_step;
  uint32_t L_p, RB_p;
  ra_type2_from_riv(riv, &L_p, &RB_p, n_vrb_p, n_vrb_p);
  d->L_crb = L_p * n_step;
  d->RB_start = RB_p * n_step;
  d->riv = riv;
  d->mcs_idx = bit_pack(&y, 5);
  d->rv_idx = -1;
  d->tb_en[0] = 1;
  d->tb_en[1] = 0;
  return 0;
}

int unpack_2x(const uint8_t *bits, uint32_t format, srsgpu_ra_dl_dci_t *d, uint32_t nof_prb, uint32_t nof_ports) {
  const uint8_t *y = bits;
  if (!unpack_type01(&y, d, nof_prb)) return -1;
  y += 2; // TPC for PUCCH
  d->harq_process = bit_pack(&y, kHarqPidLen);
  if (format == SRSGPU_DCI_FORMAT2B)
    d->sram_id = *y++ ? 1u : 0u;
  else
    d->tb_cw_swap = *y++ ? 1u : 0u;
  d->mcs_idx = bit_pack(&y, 5);
  d->ndi = *y++ ? 1u : 0u;
  d->rv_idx = (int32_t)bit_pack(&y, 2);
  d->tb_en[0] = !(d->mcs_idx == 0 && d->rv_idx == 1);
  d->mcs_idx_1 = bit_pack(&y, 5);
  d->ndi_1 = *y++ ? 1u : 0u;
  d->rv_idx_1 = (int32_t)bit_pack(&y, 2);
  d->tb_en[1] = !(d->mcs_idx_1 == 0 && d->rv_idx_1 == 1);
  if (format == SRSGPU_DCI_FORMAT2)
    d->pinfo = bit_pack(&y, (int)precoding_bits_f2(nof_ports));
  else if (format == SRSGPU_DCI_FORMAT2A)
    d->pinfo = bit_pack(&y, (int)precoding_bits_f2a(nof_ports));
  if (d->tb_en[0] && d->tb_en[1] && d->tb_cw_swap) { // Table 5.3.3.1.5-1
    uint32_t t = (uint32_t)d->rv_idx;
    d->rv_idx = d->rv_idx_1;
    d->rv_idx_1 = (int32_t)t;
    t = d->mcs_idx;
    d->mcs_idx = d->mcs_idx_1;
    d->mcs_idx_1 = t;
    t = d->ndi;
    d->ndi = d->ndi_1;
    d->ndi_1 = t;
  }
  if (!d->tb_en[0]) { // Table 5.3.3.1.5-2
    d->rv_idx = d->rv_idx_1;
    d->mcs_idx = d->mcs_idx_1;
    d->ndi = d->ndi_1;
    d->tb_en[1] = 0;
  }
  return 0;
}

// ra.c:292-425
int dl_prb_allocation(const srsgpu_ra_dl_dci_t *d, srsgpu_ra_dl_grant_t *g, uint32_t nof_prb) {
  const uint32_t P = ra_type0_P(nof_prb);
  switch (d->alloc_type) {
  case 0: {
    const int nb = (int)ceilf((float)nof_prb / P);
    for (int i = 0; i < nb; i++)
      if (d->rbg_bitmask & (1u << (nb - i - 1)))
        for (uint32_t j = 0; j < P; j++)
          if (i * P + j < nof_prb) {
            g->prb_idx[0][i * P + j] = 1;
            g->nof_prb++;
          }
    memcpy(g->prb_idx[1], g->prb_idx[0], 110);
    return 0;
  }
  case 1: {
    if (d->rbg_subset >= P) return -1;
    const uint32_t n_rb_type1 = ra_type1_N_rb(nof_prb), temp = ((nof_prb - 1) / P) % P;
    uint32_t n_rb_rbg_subset;
    if (d->rbg_subset < temp)
      n_rb_rbg_subset = ((nof_prb - 1) / (P * P)) * P + P;
    else if (d->rbg_subset == temp)
      n_rb_rbg_subset = ((nof_prb - 1) / (P * P)) * P + ((nof_prb - 1) % P) + 1;
    else
      n_rb_rbg_subset = ((nof_prb - 1) / (P * P)) * P;
    const int shift = d->shift ? (int)(n_rb_rbg_subset - n_rb_type1) : 0;
    for (int i = 0; i < (int)n_rb_type1; i++)
      if (d->vrb_bitmask & (1u << (n_rb_type1 - i - 1))) {
        const uint32_t idx = ((i + shift) / P) * P * P + d->rbg_subset * P + (i + shift) % P;
        if (idx >= nof_prb) return -1;
        g->prb_idx[0][idx] = 1;
        g->nof_prb++;
      }
    memcpy(g->prb_idx[1], g->prb_idx[0], 110);
    return 0;
  }
  case 2: {
    if (d->mode == 0) {
      for (uint32_t i = 0; i < d->L_crb; i++) {
        // the reference writes bool prb_idx[0][RB_start + i] unchecked (ra.c:342-345)
        if (i + d->RB_start < 110) g->prb_idx[0][i + d->RB_start] = 1;
        g->nof_prb++;
      }
      memcpy(g->prb_idx[1], g->prb_idx[0], 110);
      return 0;
    }
    // 36.211 6.2.3.2 distributed VRB -> PRB (ra.c:347-418)
    int N_gap, N_tilde_vrb;
    if (d->n_gap == 0) {
      N_tilde_vrb = (int)ra_type2_n_vrb_dl(nof_prb, true);
      N_gap = (int)ra_type2_ngap(nof_prb, true);
    } else {
      N_tilde_vrb = 2 * (int)ra_type2_n_vrb_dl(nof_prb, true);
      N_gap = (int)ra_type2_ngap(nof_prb, false);
    }
    const int N_row = (int)ceilf((float)N_tilde_vrb / (4 * P)) * (int)P;
    const int N_null = 4 * N_row - N_tilde_vrb;
    for (int i = 0; i < (int)d->L_crb; i++) {
      const int n_vrb = i + (int)d->RB_start;
      const int n_tilde_vrb = n_vrb % N_tilde_vrb;
      const int n_tilde_prb = 2 * N_row * (n_tilde_vrb % 2) + n_tilde_vrb / 2 + N_tilde_vrb * (n_vrb / N_tilde_vrb);
      const int n_tilde2_prb = N_row * (n_tilde_vrb % 4) + n_tilde_vrb / 4 + N_tilde_vrb * (n_vrb / N_tilde_vrb);
      int odd;
      if (N_null != 0 && n_tilde_vrb >= (N_tilde_vrb - N_null) && (n_tilde_vrb % 2) == 1)
        odd = n_tilde_prb - N_row;
      else if (N_null != 0 && n_tilde_vrb >= (N_tilde_vrb - N_null) && (n_tilde_vrb % 2) == 0)
        odd = n_tilde_prb - N_row + N_null / 2;
      else if (N_null != 0 && n_tilde_vrb < (N_tilde_vrb - N_null) && (n_tilde_vrb % 4) >= 2)
        odd = n_tilde2_prb - N_null / 2;
      else
        odd = n_tilde2_prb;
      const int even = (odd + N_tilde_vrb / 2) % N_tilde_vrb + N_tilde_vrb * (n_vrb / N_tilde_vrb);
      for (int s = 0; s < 2; s++) {
        const int v = s ? even : odd;
        const int prb = v < N_tilde_vrb / 2 ? v : v + N_gap - N_tilde_vrb / 2;
        if (prb >= (int)nof_prb || prb < 0) return -1;
        g->prb_idx[s][prb] = 1;
        if (s == 0) g->nof_prb++;
      }
    }
    return 0;
  }
  default:
    return -1;
  }
}

// ra.c:427-455
int fill_ra_mcs(uint32_t idx, uint32_t nprb, uint32_t *mod, int32_t *tbs_out) {
  int i_tbs = -1;
  if (idx < 10) {
    *mod = 1;
    i_tbs = (int)idx;
  } else if (idx < 17) {
    *mod = 2;
    i_tbs = (int)idx - 1;
  } else if (idx < 29) {
    *mod = 3;
    i_tbs = (int)idx - 2;
  } else if (idx == 29) {
    *mod = 1;
  } else if (idx == 30) {
    *mod = 2;
  } else if (idx == 31) {
    *mod = 3;
  }
  int tbs = -1;
  if (i_tbs >= 0) {
    tbs = srsgpu_ra_tbs_from_idx((uint32_t)i_tbs, nprb);
    *tbs_out = tbs;
  }
  return tbs;
}

uint32_t mod_bits(uint32_t mod) { return mod == 0 ? 1 : mod == 1 ? 2 : mod == 2 ? 4 : 6; }

} // namespace

extern "C" {

int srsgpu_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t nof_prb) {
  if (tbs_idx < 27 && nof_prb > 0 && nof_prb <= 110) return srsgpu::kTbsTable[tbs_idx][nof_prb - 1];
  return -1;
}

int srsgpu_ra_tbs_idx_from_mcs(uint32_t mcs) { return mcs < 29 ? srsgpu::kMcsTbsIdx[mcs] : -1; }

uint32_t srsgpu_dci_format_sizeof(uint32_t format, uint32_t nof_prb, uint32_t nof_ports) {
  switch (format) {
  case SRSGPU_DCI_FORMAT0: return f0_sizeof(nof_prb);
  case SRSGPU_DCI_FORMAT1: return f1_sizeof(nof_prb);
  case SRSGPU_DCI_FORMAT1A: return f1A_sizeof(nof_prb);
  case SRSGPU_DCI_FORMAT1C: return f1C_sizeof(nof_prb);
  case SRSGPU_DCI_FORMAT1B:
  case SRSGPU_DCI_FORMAT1D: return f1B_sizeof(nof_prb, nof_ports);
  case SRSGPU_DCI_FORMAT2: return f2x_sizeof(nof_prb, precoding_bits_f2(nof_ports));
  case SRSGPU_DCI_FORMAT2A: return f2x_sizeof(nof_prb, precoding_bits_f2a(nof_ports));
  case SRSGPU_DCI_FORMAT2B: return f2x_sizeof(nof_prb, 0);
  default: return 0;
  }
}

// dci.c:49-90 -> dci.c:1332 (unpack) and ra.c:583-612 (grant)
int srsgpu_dci_msg_to_dl_grant(const uint8_t *bits, uint32_t nof_bits, uint32_t format, uint16_t rnti,
                               uint32_t nof_prb, uint32_t nof_ports, srsgpu_ra_dl_dci_t *d,
                               srsgpu_ra_dl_grant_t *g) {
  if (!bits || !d || !g || nof_prb < 1 || nof_prb > 110) return -1;
  memset(d, 0, sizeof(*d));
  memset(g, 0, sizeof(*g));
  const bool crnti = rnti >= kCrntiStart && rnti <= kCrntiEnd;
  int r;
  switch (format) {
  case SRSGPU_DCI_FORMAT1: r = unpack_1(bits, nof_bits, d, nof_prb); break;
  case SRSGPU_DCI_FORMAT1A: r = unpack_1A(bits, nof_bits, d, nof_prb, crnti); break;
  case SRSGPU_DCI_FORMAT1B: r = unpack_1BD(bits, d, nof_prb, nof_ports, false); break;
  case SRSGPU_DCI_FORMAT1C: r = unpack_1C(bits, nof_bits, d, nof_prb); break;
  case SRSGPU_DCI_FORMAT1D: r = unpack_1BD(bits, d, nof_prb, nof_ports, true); break;
  case SRSGPU_DCI_FORMAT2:
  case SRSGPU_DCI_FORMAT2A:
  case SRSGPU_DCI_FORMAT2B: r = unpack_2x(bits, format, d, nof_prb, nof_ports); break;
  default: r = -1;
  }
  if (r) return -1;
  // dci.c:71-76: a grant that fails to compute still returns the unpack's SRSLTE_SUCCESS, with the
  // grant as far as ra.c filled it before failing
  if (!d->is_ra_order) (void)srsgpu_ra_dl_dci_to_grant(d, nof_prb, rnti, g);
  return 0;
}

// ra.c:583-612 with :292-425 (PRB allocation) and :509-561 (MCS / TBS)
int srsgpu_ra_dl_dci_to_grant(srsgpu_ra_dl_dci_t *d, uint32_t nof_prb, uint16_t rnti, srsgpu_ra_dl_grant_t *g) {
  if (!d || !g || nof_prb < 1 || nof_prb > 110) return -1;
  const bool crnti = rnti >= kCrntiStart && rnti <= kCrntiEnd;
  memset(g, 0, sizeof(*g));
  if (dl_prb_allocation(d, g, nof_prb)) return -1;
  if (!crnti) {
    int tbs = -1;
    if (d->dci_is_1a) {
      tbs = srsgpu_ra_tbs_from_idx(d->mcs_idx, d->n_prb1a == 0 ? 2 : 3);
    } else if (d->dci_is_1c) {
      if (d->mcs_idx < 32) tbs = srsgpu::kTbsFormat1C[d->mcs_idx];
    } else {
      return -1; // P / SI / RA-RNTI take formats 1A / 1C only
    }
    g->mod[0] = 1;
    g->tbs[0] = tbs;
    g->mcs_idx[0] = d->mcs_idx;
  } else {
    if (d->tb_en[0]) {
      g->mcs_idx[0] = d->mcs_idx;
      g->tbs[0] = fill_ra_mcs(d->mcs_idx, g->nof_prb, &g->mod[0], &g->tbs[0]);
    } else {
      g->tbs[0] = 0;
    }
    if (d->tb_en[1]) {
      g->mcs_idx[1] = d->mcs_idx_1;
      g->tbs[1] = fill_ra_mcs(d->mcs_idx_1, g->nof_prb, &g->mod[1], &g->tbs[1]);
    } else {
      g->tbs[1] = 0;
    }
  }
  for (int t = 0; t < 2; t++) {
    g->tb_en[t] = d->tb_en[t];
    if (d->tb_en[t]) g->Qm[t] = mod_bits(g->mod[t]);
  }
  g->pinfo = d->pinfo;
  g->tb_cw_swap = d->tb_cw_swap;
  if (g->tbs[0] < 0 || g->tbs[1] < 0) return -1;
  // 7.1.7.3: RA-RNTI and P-RNTI 1C take rv 0
  if (d->dci_is_1c && ((rnti >= kRarntiStart && rnti <= kRarntiEnd) || rnti == kPrnti)) d->rv_idx = 0;
  return 0;
}

// dci.c:165-197: dci_format0_unpack (:571-626), then srslte_ra_ul_dci_to_grant (ra.c:228-245) with the
// PRB allocation of ra.c:118-187 and the MCS of ra.c:189-218
int srsgpu_dci_msg_to_ul_grant(const uint8_t *bits, uint32_t nof_bits, uint32_t nof_prb, uint32_t n_rb_ho,
                               srsgpu_ra_ul_dci_t *d, srsgpu_ra_ul_grant_t *g) {
  if (!bits || !d || !g || nof_prb < 1 || nof_prb > 110) return -1;
  memset(d, 0, sizeof(*d));
  memset(g, 0, sizeof(*g));
  // format 0 unpack: size, format flag, hopping flag and bits (36.213 Table 8.4-1), RIV, MCS, NDI, TPC,
  // DMRS cyclic shift, CQI request
  if (nof_bits != f0_sizeof(nof_prb) || bits[0] != 0) return -1;
  const uint8_t *y = bits + 1;
  uint32_t n_ul_hop = 0;
  if (*y++ == 0) {
    d->freq_hop_fl = -1;
  } else if (nof_prb < 50) {
    n_ul_hop = 1;
    d->freq_hop_fl = *y++;
  } else {
    n_ul_hop = 2;
    d->freq_hop_fl = y[0] << 1 | y[1];
    y += 2;
  }
  const uint32_t riv = bit_pack(&y, (int)(riv_nbits(nof_prb) - n_ul_hop));
  ra_type2_from_riv(riv, &d->L_crb, &d->RB_start, nof_prb, nof_prb);
  d->riv = riv;
  d->mcs_idx = bit_pack(&y, 5);
  d->ndi = *y++ ? 1 : 0;
  d->tpc_pusch = bit_pack(&y, 2);
  d->n_dmrs = bit_pack(&y, 3);
  d->cqi_request = *y++ ? 1 : 0;
  // PRB allocation (8.1 and 8.4 of 36.213)
  g->ncs_dmrs = d->n_dmrs;
  g->L_prb = d->L_crb;
  const uint32_t n_prb_1 = d->RB_start;
  if (n_rb_ho % 2) n_rb_ho++;
  if (d->freq_hop_fl == -1 || d->freq_hop_fl == 3) {
    g->n_prb[0] = g->n_prb[1] = n_prb_1; // type 2 hopping is applied at resource mapping
    g->freq_hopping = d->freq_hop_fl == -1 ? 0 : 2;
  } else { // type 1: a fixed offset between the slots
    const uint32_t n_rb_pusch = nof_prb - n_rb_ho - (nof_prb % 2);
    g->n_prb[0] = n_prb_1;
    if (n_prb_1 < n_rb_ho / 2) return -1;
    switch (d->freq_hop_fl) {
    case 0: g->n_prb[1] = (n_rb_pusch / 4 + n_prb_1) % n_rb_pusch; break;
    case 1: g->n_prb[1] = n_prb_1 < n_rb_pusch / 4 ? n_rb_pusch + n_prb_1 - n_rb_pusch / 4 : n_prb_1 - n_rb_pusch / 4; break;
    case 2: g->n_prb[1] = (n_rb_pusch / 2 + n_prb_1) % n_rb_pusch; break;
    default: break;
    }
    g->freq_hopping = 1;
  }
  if (!(g->n_prb[0] + g->L_prb <= nof_prb && g->n_prb[1] + g->L_prb <= nof_prb)) return -1;
  // MCS (8.6.1 / 8.6.2)
  if (d->mcs_idx <= 28) {
    const uint32_t off = d->mcs_idx < 11 ? 0 : d->mcs_idx < 21 ? 1 : 2;
    g->mod = d->mcs_idx < 11 ? 1 : d->mcs_idx < 21 ? 2 : 3;
    g->tbs = srsgpu_ra_tbs_from_idx(d->mcs_idx - off, g->L_prb);
  } else if (d->mcs_idx == 29 && d->cqi_request && g->L_prb <= 4) {
    g->mod = 1; // CQI only
    g->tbs = 0;
    d->rv_idx = 1;
  } else {
    g->tbs = -1;
    g->mod = 4; // SRSLTE_MOD_LAST
    d->rv_idx = d->mcs_idx - 28;
  }
  g->mcs_idx = d->mcs_idx;
  g->M_sc = g->L_prb * 12;
  g->M_sc_init = g->M_sc;
  g->Qm = g->mod < 4 ? mod_bits(g->mod) : 0;
  return 0;
}

} // extern "C"
