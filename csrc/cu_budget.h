// CUs that the one-round GEMM grids are sized for (host side only; no device code here).
//
// The 4-wave ring GEMMs hold a CU's whole register file, so a grid of exactly one round of 256 workgroups needs every
// CU: when other work sits on a few CUs — the RCCL channel blocks of a collective overlapped with the backward at
// N > 1 — the last workgroups wait for a second round (measured with sftamd.cu_hog: 4 held CUs cost the o_proj and
// gate_up input gradients 39-70 %, profiles/r6_cu_contention.md). set_cu_budget(n) makes the split / hybrid decisions
// of those grids use n CUs instead (0 = all of them).
#pragma once

#include <cstdlib>

namespace sftamd {

constexpr int kNumCUs = 256;  // MI355X: 8 XCDs x 32 CUs

inline int& cu_budget_slot() {  // initial value: SFTAMD_CU_BUDGET (0 / unset = all CUs)
  static int b = [] {
    const char* e = std::getenv("SFTAMD_CU_BUDGET");
    return e && e[0] ? std::atoi(e) : 0;
  }();
  return b;
}

inline int cu_budget() {
  const int b = cu_budget_slot();
  return (b > 0 && b < kNumCUs) ? b : kNumCUs;
}

}  // namespace sftamd
