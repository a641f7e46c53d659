// K5b host twin: the per-row weighted sums of csrc/kernels/rowsums.hip on CPU tensors.
//
// Small CPU batches (BASELINE config: Mean / Sum updates at bs = 8) are dominated by ATen
// dispatch overhead - the reference's Mean.update is mul / sum / numel / tensor / two adds.
// This is the same single pass as the kernel (FP64 sums, outputs merged in their own dtype),
// called once per update.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

#include "tea_kernels.h"
#include "tea_types.h"

namespace tea {

namespace {

double host_load(const void* p, DType dt, int64_t i) {
  switch (dt) {
    case DType::f32: return static_cast<const float*>(p)[i];
    case DType::f64: return static_cast<const double*>(p)[i];
    case DType::i64: return static_cast<double>(static_cast<const int64_t*>(p)[i]);
    case DType::i32: return static_cast<const int32_t*>(p)[i];
    case DType::i16: return static_cast<const int16_t*>(p)[i];
    case DType::i8: return static_cast<const int8_t*>(p)[i];
    case DType::u8: return static_cast<const uint8_t*>(p)[i];
    case DType::b8: return static_cast<const uint8_t*>(p)[i] != 0;
    case DType::f16: {
      const uint16_t h = static_cast<const uint16_t*>(p)[i];
      const uint32_t sign = (h & 0x8000u) << 16, ex = (h >> 10) & 0x1f, man = h & 0x3ff;
      float f;
      if (ex == 0) {
        f = std::ldexp(static_cast<float>(man), -24);
        return sign ? -f : f;
      }
      const uint32_t bits = ex == 31 ? (sign | 0x7f800000u | (man << 13)) : (sign | ((ex + 112) << 23) | (man << 13));
      std::memcpy(&f, &bits, 4);
      return f;
    }
    case DType::bf16: {
      const uint32_t bits = static_cast<uint32_t>(static_cast<const uint16_t*>(p)[i]) << 16;
      float f;
      std::memcpy(&f, &bits, 4);
      return f;
    }
  }
  return 0.0;
}

double nmin(double a, double b) { return (a != a || b != b) ? std::numeric_limits<double>::quiet_NaN() : std::fmin(a, b); }
double nmax(double a, double b) { return (a != a || b != b) ? std::numeric_limits<double>::quiet_NaN() : std::fmax(a, b); }

void store(const RowSumsOut& o, int64_t r, double v) {
  const int64_t i = r * o.stride;
  if (o.dt == DType::f64) {
    double& d = static_cast<double*>(o.p)[i];
    d = o.op == kSet ? v : o.op == kAdd ? d + v : o.op == kMin ? nmin(d, v) : nmax(d, v);
  } else {
    float& d = static_cast<float*>(o.p)[i];
    const float f = static_cast<float>(v);
    d = o.op == kSet ? f : o.op == kAdd ? d + f : static_cast<float>(o.op == kMin ? nmin(d, f) : nmax(d, f));
  }
}

}  // namespace

void row_sums_host(const RowSumsArgs& g) {
  for (int64_t r = 0; r < g.rows; ++r) {
    double v[kRowRaw] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, std::numeric_limits<double>::infinity(),
                         -std::numeric_limits<double>::infinity()};
    const bool f32 = g.x && g.x_dt == DType::f32 && g.x_cs == 1 && (!g.t || (g.t_dt == DType::f32 && g.t_cs == 1)) &&
                     (!g.w || (g.w_dt == DType::f32 && g.w_cs == 1));
    for (int64_t i = 0; i < g.n; ++i) {
      double x, t, w;
      if (f32) {
        x = static_cast<const float*>(g.x)[r * g.x_rs + i];
        t = g.t ? static_cast<const float*>(g.t)[r * g.t_rs + i] : 0.0;
        w = g.w ? static_cast<const float*>(g.w)[r * g.w_rs + i] : g.w_scalar;
      } else {
        x = g.x ? host_load(g.x, g.x_dt, r * g.x_rs + i * g.x_cs) : 0.0;
        t = g.t ? host_load(g.t, g.t_dt, r * g.t_rs + i * g.t_cs) : 0.0;
        w = g.w ? host_load(g.w, g.w_dt, r * g.w_rs + i * g.w_cs) : g.w_scalar;
      }
      v[kWX] += w * x;
      v[kWT] += w * t;
      v[kW] += w;
      const double d = x - t;
      v[kSSE] += d * d;
      v[kWSSE] += w * d * d;
      v[kWTT] += w * t * t;
      if (g.need & ((1 << kTMIN) | (1 << kTMAX))) {
        v[kTMIN] = nmin(v[kTMIN], t);
        v[kTMAX] = nmax(v[kTMAX], t);
      }
    }
    if (!g.w) v[kW] = g.w_scalar * static_cast<double>(g.n);
    double merged_min = 0.0, merged_max = 0.0;
    for (int k = 0; k < g.nout; ++k) {
      const RowSumsOut& o = g.out[k];
      if (o.first_row_only && r != 0) continue;
      const double val = o.stat == kCOUNT ? static_cast<double>(g.n) : o.stat == kRANGE ? merged_max - merged_min : v[o.stat];
      store(o, r, val);
      if (o.stat == kTMIN) merged_min = host_load(o.p, o.dt, r * o.stride);
      if (o.stat == kTMAX) merged_max = host_load(o.p, o.dt, r * o.stride);
    }
  }
}

}  // namespace tea
