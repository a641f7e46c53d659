// Host/device-neutral types shared by kernels and the host glue (no device code here).
#pragma once

#include <stdint.h>

namespace tea {

enum class DType : int {
  f32 = 0,
  f16 = 1,
  bf16 = 2,
  f64 = 3,
  i64 = 4,
  i32 = 5,
  u8 = 6,
  b8 = 7,
  i8 = 8,
  i16 = 9,
};

// fold workspace size in u64 cells (tea_fold.h: 64 shards x 64-B stride, 16 value slots)
constexpr int kFoldCells = 64 * 8;

}  // namespace tea
