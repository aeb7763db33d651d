// ewarp_desc.h — validation of an ewh_pta_desc (include/ewarp_hip.h), shared
// by the HIP library (ewarp_hip.hip) and its host twin (ewarp_cpu.cpp): the
// same descriptor is accepted or refused, with the same message, by both.
#pragma once
#include <string>
#include <vector>

#include "ewarp_hip.h"

namespace ewh_desc {

// 0, or a negative EWH_E* code with the reason in msg
inline int desc_check(const ewh_pta_desc* d, std::string& msg) {
  auto fail = [&](int code, const std::string& m) { msg = m; return code; };
  if (!d || d->abi_version != EWH_ABI_VERSION) return fail(EWH_E_INVALID, "bad descriptor / ABI version");
  if (d->n_pulsar <= 0 || !d->pulsars) return fail(EWH_E_INVALID, "no pulsars");
  if (d->n_param < 0) return fail(EWH_E_INVALID, "n_param < 0");
  for (int p = 0; p < d->n_pulsar; ++p) {
    const ewh_pulsar_desc& s = d->pulsars[p];
    const std::string tag = "pulsar " + std::to_string(p) + ": ";
    if (s.n_toa <= 0 || s.n_col < 0 || s.n_lead_const < 0 || s.n_lead_const > s.n_col)
      return fail(EWH_E_INVALID, tag + "bad sizes");
    if ((s.n_col && !s.basis) || !s.resid || !s.toaerr || !s.efac_slot || !s.equad_slot ||
        (s.n_slot && !s.slots) || (s.n_spec && !s.spec))
      return fail(EWH_E_INVALID, tag + "null pointer");
    if (s.n_epoch && (!s.epoch_start || !s.epoch_stop || !s.epoch_slot))
      return fail(EWH_E_INVALID, tag + "null epoch pointer");
    for (int i = 0; i < s.n_slot; ++i)
      if (s.slots[i].idx >= d->n_param) return fail(EWH_E_INVALID, tag + "slot theta index out of range");
    for (int t = 0; t < s.n_toa; ++t) {
      if (s.efac_slot[t] < 0 || s.efac_slot[t] >= s.n_slot) return fail(EWH_E_INVALID, tag + "efac slot out of range");
      if (s.equad_slot[t] >= s.n_slot) return fail(EWH_E_INVALID, tag + "equad slot out of range");
    }
    int prev = 0;
    for (int e = 0; e < s.n_epoch; ++e) {
      if (s.epoch_start[e] < prev || s.epoch_stop[e] <= s.epoch_start[e] + 1 || s.epoch_stop[e] > s.n_toa)
        return fail(EWH_E_INVALID, tag + "epochs must be ordered, disjoint slices of >= 2 TOAs");
      if (s.epoch_slot[e] < 0 || s.epoch_slot[e] >= s.n_slot) return fail(EWH_E_INVALID, tag + "epoch slot out of range");
      prev = s.epoch_stop[e];
    }
    if (s.n_bgroup < 0 || (s.n_bgroup > 0 && (!s.bgroup_idx || !s.col_bgroup || !s.ln_chrom)))
      return fail(EWH_E_INVALID, tag + "bad basis-group tables");
    for (int g = 0; g < s.n_bgroup; ++g)
      if (s.bgroup_idx[g].idx >= d->n_param) return fail(EWH_E_INVALID, tag + "basis-group theta index out of range");
    for (int j = 0; s.n_bgroup > 0 && j < s.n_col; ++j)
      if (s.col_bgroup[j] < -1 || s.col_bgroup[j] >= s.n_bgroup || (j < s.n_lead_const && s.col_bgroup[j] >= 0))
        return fail(EWH_E_INVALID, tag + "bad column basis group");
    std::vector<int> cnt(s.n_col, 0);
    for (int e = 0; e < s.n_spec; ++e) {
      const ewh_spec_entry& sp = s.spec[e];
      if (sp.col < 0 || sp.col >= s.n_col) return fail(EWH_E_INVALID, tag + "spectral column out of range");
      if (sp.kind < EWH_SPEC_POWERLAW || sp.kind > EWH_SPEC_CONST) return fail(EWH_E_INVALID, tag + "bad spectral kind");
      if (sp.p0.idx >= d->n_param || sp.p1.idx >= d->n_param || sp.p2.idx >= d->n_param)
        return fail(EWH_E_INVALID, tag + "spectral theta index out of range");
      if (sp.col < s.n_lead_const && sp.kind != EWH_SPEC_CONST)
        return fail(EWH_E_INVALID, tag + "leading columns must have constant phi");
      cnt[sp.col]++;
    }
    const int ncom = d->common ? s.n_common : 0;
    if (d->common && (s.n_common != d->common->n_col || s.n_common > s.n_col - s.n_lead_const))
      return fail(EWH_E_INVALID, tag + "n_common must equal common->n_col and follow the leading columns");
    if (!d->common && s.n_common != 0) return fail(EWH_E_INVALID, tag + "n_common without a common descriptor");
    for (int j = 0; j < s.n_col - ncom; ++j)
      if (!cnt[j]) return fail(EWH_E_INVALID, tag + "column " + std::to_string(j) + " has no phi entry");
  }
  if (d->common) {
    const ewh_common_desc& c = *d->common;
    if (c.kind != EWH_COMMON_CORRELATED && c.kind != EWH_COMMON_OPTSTAT)
      return fail(EWH_E_INVALID, "common: bad kind");
    if (c.n_col < 1 || c.n_col > 31 || !c.orf || (c.kind == EWH_COMMON_CORRELATED && !c.spec))
      return fail(EWH_E_INVALID, "common: need 1..31 columns, an ORF matrix and spectral entries");
    if (d->n_pulsar > 128) return fail(EWH_E_UNSUPPORTED, "common: at most 128 pulsars");
    for (int g = 0; c.kind == EWH_COMMON_CORRELATED && g < c.n_col; ++g) {
      const ewh_spec_entry& sp = c.spec[g];
      if (sp.col != g || sp.kind < EWH_SPEC_POWERLAW || sp.kind > EWH_SPEC_CONST || sp.p0.idx >= d->n_param ||
          sp.p1.idx >= d->n_param || sp.p2.idx >= d->n_param)
        return fail(EWH_E_INVALID, "common: bad spectral entry " + std::to_string(g));
    }
  }
  return 0;
}

}  // namespace ewh_desc
