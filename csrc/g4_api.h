// Host entry points of the 4-wave ring GEMMs (csrc/gemm_4w.hip) used by the other GEMM launchers.
#pragma once
#include <vector>

#include "common.h"

namespace sftamd {

// One weight gradient of a multi-problem launch: out (+)= dy^T x (acc), optional norm slots (nrm, capacity cap).
struct WgradJob {
  at::Tensor dy, x, out;
  bool acc;
  float* nrm;
  long cap;
};

void g4_wgrad_multi(const std::vector<WgradJob>& jobs, int split_all, int split_left);

}  // namespace sftamd
