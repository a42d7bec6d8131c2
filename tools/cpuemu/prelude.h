// TEST/DEBUG TOOL ONLY: per-translation-unit LDS backing store for the kernels'
// `extern __shared__ char lds[]` (they live in keto's anonymous namespace).
#pragma once
#include "hip/hip_runtime.h"
namespace keto {
namespace {
alignas(16) char lds[1 << 20];
}
}  // namespace keto
