// TEST/DEBUG TOOL ONLY: per-translation-unit LDS backing store for the kernels'
// `extern __shared__ char lds[]` (they live in keto's anonymous namespace).
#pragma once
#define KETO_CPUEMU 1  // one-lane waves: no block-level kernels (check.hip regroup)
#include "hip/hip_runtime.h"
#ifdef KETO_EMU_TRACE
#include "trace.h"
#endif
namespace keto {
namespace {
alignas(16) char lds[1 << 20];
}
}  // namespace keto
