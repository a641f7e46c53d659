// K7: fused log-softmax + target gather for perplexity.
//
// Replaces perplexity.py:92-107: softmax over the vocabulary, then ``probs[:, target]
// .diagonal()`` which materialises an (N x N) matrix for N = batch * seq tokens (1.7e7
// elements at N = 4096), then log + sum.  Here one wave64 streams each token's logit row
// once with 16-B loads, keeping a per-lane online (max, sum-exp) pair that is rescaled once per
// 16-value chunk; lanes combine their pairs with xor shuffles; lane 0 adds
//   -log p(target) = logsumexp(row) - row[target]
// in FP64.  Rows that do not start 16-B aligned (odd vocabularies) stream a scalar head, a 16-B
// body and a scalar tail.  ``ignore_index`` rows are skipped and counted out; targets outside [0, V) are
// flagged on device (``err``) instead of the reference's host-synchronising max() check.
#include "tea_common.h"
#include "tea_kernels.h"

#include <cstdlib>

namespace tea {

namespace {

constexpr int kB = 256;
constexpr int kWpb = kB / kWave;

template <int KIND>
__device__ __forceinline__ void load8(const void* row, int64_t col, float (&v)[8]);

template <>
__device__ __forceinline__ void load8<0>(const void* row, int64_t col, float (&v)[8]) {
  const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(row) + col);
  const float4 a = p[0], b = p[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <int KIND>
__device__ __forceinline__ void load8_16(const void* row, int64_t col, float (&v)[8]) {
  const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(row) + col);
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint16_t lo = static_cast<uint16_t>(w[e] & 0xffffu), hi = static_cast<uint16_t>(w[e] >> 16);
    v[2 * e] = KIND == 1 ? bf16_to_f32(lo) : f16_to_f32(lo);
    v[2 * e + 1] = KIND == 1 ? bf16_to_f32(hi) : f16_to_f32(hi);
  }
}
template <>
__device__ __forceinline__ void load8<1>(const void* row, int64_t col, float (&v)[8]) {
  load8_16<1>(row, col, v);
}
template <>
__device__ __forceinline__ void load8<2>(const void* row, int64_t col, float (&v)[8]) {
  load8_16<2>(row, col, v);
}

template <int KIND>
__device__ __forceinline__ float load1(const void* row, int64_t col) {
  if constexpr (KIND == 0) return static_cast<const float*>(row)[col];
  const uint16_t b = static_cast<const uint16_t*>(row)[col];
  return KIND == 1 ? bf16_to_f32(b) : f16_to_f32(b);
}

__device__ __forceinline__ void combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -__builtin_huge_valf()) return;  // both empty
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// One 16-value chunk at p[base .. base + 16) (16-B aligned; the upper 8 only when below n).
template <int KIND>
__device__ __forceinline__ void chunk16(const void* p, int64_t base, int64_t n, float& m, float& s) {
  float v[2][8];
  load8<KIND>(p, base, v[0]);
  if (base + 8 < n) {
    load8<KIND>(p, base + 8, v[1]);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[1][e] = -__builtin_huge_valf();
  }
  float cm = v[0][0];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) cm = fmaxf(cm, v[h][e]);
  float cs = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs += __expf(v[h][e] - cm);
  combine(m, s, cm, cs);
}

// Stream n values (n % 16 == 0, p 16-B aligned) as 16-value chunks per lane.  U2: two chunks a
// wave-stride apart are loaded before either is reduced (four 16-B loads in flight per lane),
// for batches with too few rows to fill the CUs with waves.
template <int KIND, bool U2>
__device__ __forceinline__ void stream_row(const void* p, int64_t n, int lane, float& m, float& s) {
  constexpr int64_t step = kWave * 16;
  int64_t base = static_cast<int64_t>(lane) * 16;
  if constexpr (U2) {
    for (; base + step < n; base += 2 * step) {
      float v[4][8];
      load8<KIND>(p, base, v[0]);
      load8<KIND>(p, base + 8, v[1]);
      load8<KIND>(p, base + step, v[2]);
      load8<KIND>(p, base + step + 8, v[3]);
      float cm = v[0][0];
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) cm = fmaxf(cm, v[h][e]);
      float cs = 0.f;
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) cs += __expf(v[h][e] - cm);
      combine(m, s, cm, cs);
    }
  }
  for (; base < n; base += step) chunk16<KIND>(p, base, n, m, s);
}

// VEC: every row starts 16-B aligned and V % 16 == 0.  Otherwise (odd vocabularies such as
// GPT-2's 50257, or row strides that break 16-B alignment) each row is split into a scalar head
// up to the next 16-B boundary (< 16 / ELS values, one per lane), a 16-B-load body of whole
// 16-value chunks and a scalar tail (< 16 values); rows are element-aligned (checked on the host).
template <int KIND, bool VEC, bool U2>
__global__ __launch_bounds__(kB) void perplexity_kernel(PerplexityArgs a) {
  const int lane = lane_id();
  const int64_t nw = static_cast<int64_t>(gridDim.x) * kWpb;
  constexpr int ELS = KIND == 0 ? 4 : 2;
  double acc = 0.0, cnt = 0.0;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWpb + wave_id(); row < a.rows; row += nw) {
    const int64_t t = load_as_i64(a.target, a.tg_dt, row * a.tg_stride);
    if (a.has_ignore && t == a.ignore_index) continue;
    const void* rp = static_cast<const char*>(a.input) + row * a.row_stride * ELS;
    float m = -__builtin_huge_valf(), s = 0.f;
    if constexpr (VEC) {
      stream_row<KIND, U2>(rp, a.v, lane, m, s);
    } else {
      const uintptr_t addr = reinterpret_cast<uintptr_t>(rp);
      int64_t head = static_cast<int64_t>(((16u - (addr & 15u)) & 15u) / ELS);
      if (head > a.v) head = a.v;
      const int64_t nb = ((a.v - head) / 16) * 16;
      if (lane < head) combine(m, s, load1<KIND>(rp, lane), 1.f);
      const void* bp = static_cast<const char*>(rp) + head * ELS;
      stream_row<KIND, U2>(bp, nb, lane, m, s);
      const int64_t c = head + nb + lane;
      if (c < a.v) combine(m, s, load1<KIND>(rp, c), 1.f);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, kWave);
      const float s2 = __shfl_xor(s, o, kWave);
      combine(m, s, m2, s2);
    }
    if (lane == 0) {
      if (t < 0 || t >= a.v) {
        if (a.err) atomicOr(a.err, 1);
      } else {
        const double lse = static_cast<double>(m) + log(static_cast<double>(s));
        acc += lse - static_cast<double>(load1<KIND>(rp, t));
        cnt += 1.0;
      }
    }
  }
  __shared__ double lds[2][kWpb];
  if (lane == 0) {
    lds[0][threadIdx.x >> 6] = acc;
    lds[1][threadIdx.x >> 6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < kWpb; ++w) tot += lds[threadIdx.x][w];
    if (a.ordered_ws)  // deterministic: per-block partial, folded in block order afterwards
      a.ordered_ws[threadIdx.x * gridDim.x + blockIdx.x] = tot;
    else if (tot != 0.0)
      atomicAdd(a.out + threadIdx.x, tot);
  }
}

template <int KIND>
void launch_kind(const PerplexityArgs& a, int grid, bool vec, bool u2, hipStream_t s) {
  if (vec && u2)
    hipLaunchKernelGGL((perplexity_kernel<KIND, true, true>), dim3(grid), dim3(kB), 0, s, a);
  else if (vec)
    hipLaunchKernelGGL((perplexity_kernel<KIND, true, false>), dim3(grid), dim3(kB), 0, s, a);
  else if (u2)
    hipLaunchKernelGGL((perplexity_kernel<KIND, false, true>), dim3(grid), dim3(kB), 0, s, a);
  else
    hipLaunchKernelGGL((perplexity_kernel<KIND, false, false>), dim3(grid), dim3(kB), 0, s, a);
}

}  // namespace

namespace {

bool vec_ok(const PerplexityArgs& a) {
  const uintptr_t base = reinterpret_cast<uintptr_t>(a.input);
  const int vw = a.in_dt == DType::f32 ? 4 : 8;
  return a.v % 16 == 0 && a.row_stride % vw == 0 && base % 16 == 0;
}

}  // namespace

// Grid cap in 4-wave blocks; rows past cap * 4 waves are grid-strided.  1024 (one row per wave
// up to 4096 rows) except fp32 batches of <= 8192 rows, where 512 (two rows per wave) streams
// faster: measured per shape (profiles/k7_grid_cap_ab_r4.json): 16384 x 32000 bf16 251 -> 189 us,
// 65536 x 4096 fp32 184 -> 177 us with 1024, but 4096 x 32000 fp32 92 vs 99 us, 4096 x 50257
// fp32 139 vs 150 us and 8192 x 1024 fp32 16 vs 19 us with 512.  TORCHEVAL_AMD_PPL_MAXGRID
// overrides (A/B).
int perplexity_blocks(const PerplexityArgs& a) {
  static const int64_t forced = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_PPL_MAXGRID");
    const long v = e ? std::atol(e) : 0;
    return v > 0 ? static_cast<int64_t>(v) : int64_t(0);
  }();
  const int64_t cap = forced > 0 ? forced : (a.in_dt == DType::f32 && a.rows <= 8192 ? 512 : 1024);
  int64_t grid = (a.rows + kWpb - 1) / kWpb;
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  return static_cast<int>(grid);
}

int launch_perplexity(const PerplexityArgs& a, hipStream_t stream) {
  if (a.rows <= 0) return 0;
  const int64_t grid = perplexity_blocks(a);
  const bool vec = vec_ok(a);
  static const int u2_env = [] {  // A/B: TORCHEVAL_AMD_PPL_U2=0/1 forces the unrolled body off/on
    const char* e = std::getenv("TORCHEVAL_AMD_PPL_U2");
    return e ? std::atoi(e) : -1;
  }();
  const int els = a.in_dt == DType::f32 ? 4 : 2;
  // Unrolled body unless the batch already fills the CUs with many short rows (profiles/
  // k7_grid_cap_ab_r4.json: 2048 x 128256 bf16 125 -> 92 us, 65536 x 4096 fp32 177 vs 184 us).
  const bool u2 = u2_env >= 0 ? u2_env != 0 : (a.rows <= 16384 || a.v * els >= 65536);
  if (reinterpret_cast<uintptr_t>(a.input) % els != 0) return -2;  // split path needs element alignment
  switch (a.in_dt) {
    case DType::f32: launch_kind<0>(a, static_cast<int>(grid), vec, u2, stream); break;
    case DType::bf16: launch_kind<1>(a, static_cast<int>(grid), vec, u2, stream); break;
    case DType::f16: launch_kind<2>(a, static_cast<int>(grid), vec, u2, stream); break;
    default: return -1;
  }
  if (a.ordered_ws) return launch_ordered_sum(a.ordered_ws, 2, grid, a.out, stream);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
