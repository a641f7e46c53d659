// Host-visible launcher interface of the torcheval_amd HIP kernels.
// Every launcher enqueues on the given HIP stream and returns hipError_t as int (0 = ok,
// -1 = unsupported argument combination, caller must fall back).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "tea_types.h"

namespace tea {

// ------------------------------------------------------------------ K1 classification
struct ClsCountsArgs {
  const void* input = nullptr;  // [n, c] scores (c > 0) or [n] integer labels (c == 0)
  DType in_dt = DType::f32;
  int64_t n = 0;
  int64_t c = 0;
  int64_t row_stride = 0;  // elements between rows of ``input``
  const void* target = nullptr;  // [n] integer labels
  DType tg_dt = DType::i64;
  int k = 1;                     // top-k (k > 1: rank-of-target)
  int64_t num_classes = 0;       // histogram width
  float* micro_correct = nullptr;
  float* micro_total = nullptr;
  float* cls_correct = nullptr;  // [num_classes] correct at target class
  float* cls_label = nullptr;    // [num_classes] samples per target class
  float* cls_pred = nullptr;     // [num_classes] samples per predicted class
  float* confusion = nullptr;    // [num_classes, num_classes] (target, pred)
  int* err = nullptr;            // error bits (1: bad target, 2: bad prediction)
  int check_target = 0;          // flag bad targets even without histograms
  unsigned long long* fold_ws = nullptr;  // tea_fold.h cells (per-stream, self-cleaning)
  int max_blocks = 0;
};
int launch_cls_counts(const ClsCountsArgs& a, hipStream_t stream);

struct BinaryCountsArgs {
  const void* input = nullptr;
  DType in_dt = DType::f32;
  const void* target = nullptr;
  DType tg_dt = DType::f32;
  const void* weight = nullptr;
  DType w_dt = DType::f32;
  int64_t n = 0;
  float threshold = 0.5f;
  int strict_binary = 0;  // non-{0,1} targets count nowhere (1) or as the "other" class (0)
  float* out[4] = {nullptr, nullptr, nullptr, nullptr};  // tp, fp, tn, fn
  float* total = nullptr;  // += n (sample count)
  int max_blocks = 0;
};
int launch_binary_counts(const BinaryCountsArgs& a, hipStream_t stream);

}  // namespace tea
