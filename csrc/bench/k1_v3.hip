// K1 round-3 A/B harness: bs=8192 x C=1000 fp32 micro-accuracy, every variant interleaved in
// ONE process over the same 8-batch pool (the bench.py shape), back-to-back launches timed
// with events (so the per-launch boundary is included, as in bench.py).
//
// Variants
//   prod          the production launcher (launch_cls_counts, classification.hip)
//   m1<R,E,RPW>   specialised micro kernel: one wave per RPW rows, all loads issued first,
//                 i64 targets by scalar load, no histogram / flag code.
//                 R = 0: DPP max-reduce + target compare (+ ballot for first-index ties)
//                 R = 1: compare-only: a column "beats" the target under torch.argmax order
//                        (NaN greatest, first index wins); correct = no lane sees a beater
//                 E = 0: tea_fold epilogue, 1: per-block slab store, 2: none (side effect only)
//   pipe<G,R>     persistent grid of G blocks, each wave double-buffers rows (next row's
//                 loads in flight while the current one is reduced)
//   smax<RPW>     loads + lane max only (the streaming floor of this read pattern)
//   empty<G>      an empty kernel of G blocks (launch + dispatch floor)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "../kernels/classification.hip"

using namespace tea;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);          \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int N = 8192, C = 1000;
constexpr int STEP = 256;  // columns per wave-load (64 lanes x float4)

__device__ __forceinline__ float fmx(float a, float b) { return __builtin_elementwise_maximum(a, b); }

template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}

// NaN-propagating max over the 64 lanes, returned wave-uniform.
__device__ __forceinline__ float wave_max_dpp(float x) {
  x = fmx(x, dppf<0xB1>(x));   // quad_perm [1,0,3,2]
  x = fmx(x, dppf<0x4E>(x));   // quad_perm [2,3,0,1]
  x = fmx(x, dppf<0x141>(x));  // row_half_mirror
  x = fmx(x, dppf<0x140>(x));  // row_mirror -> every lane holds its 16-lane row max
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
  return fmx(fmx(r0, r1), fmx(r2, r3));
}

struct Row {
  float v[4][4];
};

__device__ __forceinline__ void load_row(const float* __restrict__ rp, int lane, Row& r) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int col = u * STEP + lane * 4;
    const float4 q = *reinterpret_cast<const float4*>(rp + (col < C ? col : 0));
    r.v[u][0] = q.x;
    r.v[u][1] = q.y;
    r.v[u][2] = q.z;
    r.v[u][3] = q.w;
  }
}

// exact torch.argmax == t for one row whose values sit in registers (any NaN / tie pattern)
__device__ __noinline__ bool exact_row(const float* __restrict__ rp, int lane, int64_t t) {
  float bv = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int col = lane; col < C; col += 64) {
    const float v = rp[col];
    if (argmax_better(v, col, bv, bi)) {
      bv = v;
      bi = col;
    }
  }
  wave_argmax(bv, bi);
  return bi == t;
}

__device__ __forceinline__ bool row_correct2(const Row& r, int lane, int64_t t, const float* __restrict__ rp);
template <int R>
__device__ __forceinline__ bool row_correct(Row& r, int lane, int64_t t, const float* __restrict__ rp) {
  if constexpr (R == 2) return row_correct2(r, lane, t, rp);
  const bool t_ok = t >= 0 && t < C;
  const int tu = t_ok ? static_cast<int>(t) : 0;
  const int ut = tu / STEP, et = tu % 4, owner = (tu % STEP) / 4;
  float sel = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const bool in = u * STEP + lane * 4 < C;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r.v[u][e] = in ? r.v[u][e] : -__builtin_huge_valf();
      sel = (u == ut && e == et) ? r.v[u][e] : sel;
    }
  }
  const float xt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), owner));
  if (!t_ok) return false;
  if constexpr (R == 0) {
    float m = r.v[0][0];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmx(m, r.v[u][e]);
    const float wm = wave_max_dpp(m);
    if (__builtin_expect(wm != wm, 0)) return exact_row(rp, lane, t);
    if (xt != wm) return false;
    // the target holds the max: correct iff no earlier column equals it
    bool earlier = false;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) earlier |= (r.v[u][e] == wm) & (u * STEP + lane * 4 + e < tu);
    return !__any(earlier);
  } else {
    if (__builtin_expect(xt != xt, 0)) return exact_row(rp, lane, t);
    // column c beats t iff v > xt, or v is NaN, or (v == xt and c < t)
    bool beat = false;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = r.v[u][e];
        const bool lt = u * STEP + lane * 4 + e < tu;
        beat |= lt ? !(v < xt) : !(v <= xt);
      }
    return !__any(beat);
  }
}


// R2: ~0.6 VALU per element.  Lanes of the last load that are past C re-read columns 0..3 (the
// clamped address), which cannot change the row max; they are masked out of the tie count
// with a uniform lane mask instead of per-element selects.
__device__ __forceinline__ float pick16(const Row& r, int idx) {
  switch (idx) {  // wave-uniform: a scalar branch tree, one v_mov
    case 0: return r.v[0][0]; case 1: return r.v[0][1]; case 2: return r.v[0][2]; case 3: return r.v[0][3];
    case 4: return r.v[1][0]; case 5: return r.v[1][1]; case 6: return r.v[1][2]; case 7: return r.v[1][3];
    case 8: return r.v[2][0]; case 9: return r.v[2][1]; case 10: return r.v[2][2]; case 11: return r.v[2][3];
    case 12: return r.v[3][0]; case 13: return r.v[3][1]; case 14: return r.v[3][2]; default: return r.v[3][3];
  }
}

__device__ __forceinline__ bool row_correct2(const Row& r, int lane, int64_t t, const float* __restrict__ rp) {
  float m0 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(r.v[0][0], r.v[0][1]), r.v[0][2]);
  float m1 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(r.v[0][3], r.v[1][0]), r.v[1][1]);
  float m2 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(r.v[1][2], r.v[1][3]), r.v[2][0]);
  float m3 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(r.v[2][1], r.v[2][2]), r.v[2][3]);
  float m4 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(r.v[3][0], r.v[3][1]), r.v[3][2]);
  float m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m0, m1), m2);
  m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m, m3), m4);
  m = __builtin_elementwise_maximum(m, r.v[3][3]);
  const float wm = wave_max_dpp(m);
  // the NaN test comes first: it needs the row on every path, so the loads stay ahead of the
  // target's range check (else the compiler sinks them behind the scalar target load)
  if (__builtin_expect(wm != wm, 0)) return exact_row(rp, lane, t);
  if (!(t >= 0 && t < C)) return false;
  const int tu = static_cast<int>(t);
  const float sel = pick16(r, (tu >> 8) * 4 + (tu & 3));
  const float xt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), (tu & 255) >> 2));
  if (xt != wm) return false;
  // the target holds the max: correct iff it is the only column holding it (else exact path)
  constexpr int tail_lanes = (C - 768) / 4;  // valid lanes of the last load (C in (768, 1024])
  const uint64_t tail = tail_lanes >= 64 ? ~0ull : ((1ull << tail_lanes) - 1);
  int cnt = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint64_t mk = __ballot(r.v[u][e] == wm);
      if (u == 3) mk &= tail;
      cnt += __builtin_popcountll(mk);
    }
  if (cnt == 1) return true;
  return exact_row(rp, lane, t);
}

template <int E>
__device__ __forceinline__ void epilogue(uint32_t correct_lane0, unsigned long long* ws, float* dst, float* slab) {
  if constexpr (E == 4) {
    if ((threadIdx.x & 63) == 0 && correct_lane0)
      atomicAdd(ws + 4096 + ((blockIdx.x * 4 + (threadIdx.x >> 6)) % 64) * 8, (unsigned long long)correct_lane0);
    return;
  }
  __shared__ uint32_t lds[16];
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = correct_lane0;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += lds[k];
    if constexpr (E == 0) fold_count(ws, s, dst);
    else if constexpr (E == 1) slab[blockIdx.x] = static_cast<float>(s);
    else if constexpr (E == 3) { if (s) atomicAdd(ws + 4096 + (blockIdx.x % 64) * 8, (unsigned long long)s); }
    else if (s == static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst))) slab[0] = 1.f;  // opaque
  }
}

template <int R, int E, int RPW>
__global__ __launch_bounds__(256) void m1(const float* __restrict__ x, const int64_t* __restrict__ y,
                                          unsigned long long* ws, float* dst, float* slab) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + wave_id();
  const int r0 = w * RPW;
  uint32_t correct = 0;
  if (r0 < N) {
    Row rows[RPW];
    int64_t t[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) load_row(x + (size_t)(r0 + k) * C, lane, rows[k]);
#pragma unroll
    for (int k = 0; k < RPW; ++k) t[k] = y[r0 + k];
#pragma unroll
    for (int k = 0; k < RPW; ++k) correct += row_correct<R>(rows[k], lane, t[k], x + (size_t)(r0 + k) * C);
  }
  epilogue<E>(correct, ws, dst, slab);
}

template <int R>
__global__ __launch_bounds__(256) void pipe(const float* __restrict__ x, const int64_t* __restrict__ y,
                                            unsigned long long* ws, float* dst, float* slab) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  int row = blockIdx.x * 4 + wave_id();
  uint32_t correct = 0;
  Row a, b;
  int64_t ta = 0, tb = 0;
  if (row < N) {
    load_row(x + (size_t)row * C, lane, a);
    ta = y[row];
  }
  while (row < N) {
    const int n1 = row + nw;
    if (n1 < N) {
      load_row(x + (size_t)n1 * C, lane, b);
      tb = y[n1];
    }
    correct += row_correct<R>(a, lane, ta, x + (size_t)row * C);
    if (n1 >= N) break;
    const int n2 = n1 + nw;
    if (n2 < N) {
      load_row(x + (size_t)n2 * C, lane, a);
      ta = y[n2];
    }
    correct += row_correct<R>(b, lane, tb, x + (size_t)n1 * C);
    row = n2;
  }
  epilogue<0>(correct, ws, dst, slab);
}


// Isolation kernels: the streaming max plus ONE extra ingredient each.
// T: 0 no target, 1 target by scalar load, 2 target by vector load (every lane, one address)
// RED: 0 lane max only, 1 + DPP wave max, 2 + __shfl_xor wave max;  E: epilogue as above
template <int T, int RED, int E>
__global__ __launch_bounds__(256) void iso(const float* __restrict__ x, const int64_t* __restrict__ y,
                                           unsigned long long* ws, float* dst, float* slab) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave_id();
  uint32_t correct = 0;
  if (row < N) {
    Row r;
    load_row(x + (size_t)row * C, lane, r);
    int64_t t = 0;
    if constexpr (T == 1) t = y[row];
    if constexpr (T == 2) {  // a per-lane address keeps it a vector load (every lane: one row)
      t = y[row + (lane >> 6)];
      t = __builtin_amdgcn_readfirstlane(static_cast<int>(t));
    }
    float m = r.v[0][0];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmx(m, r.v[u][e]);
    if constexpr (RED == 1) m = wave_max_dpp(m);
    if constexpr (RED == 2) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmx(m, __shfl_xor(m, o, 64));
    }
    correct = m > static_cast<float>(t) + 100.f;
  }
  if constexpr (E == 2) {
    if (correct == static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst))) slab[0] = 1.f;  // opaque
  } else {
    epilogue<E>(correct, ws, dst, slab);
  }
}

// R3: R0 compute (lane max3 tree + DPP wave max), the target's own score by a dependent
// scalar load from the row (no per-element select), ballot tie count on candidate rows.
__device__ __forceinline__ bool row_correct3(const Row& r, int lane, int64_t t, float xt_loaded,
                                             const float* __restrict__ rp) {
  float m0 = fmx(fmx(r.v[0][0], r.v[0][1]), r.v[0][2]);
  float m1 = fmx(fmx(r.v[0][3], r.v[1][0]), r.v[1][1]);
  float m2 = fmx(fmx(r.v[1][2], r.v[1][3]), r.v[2][0]);
  float m3 = fmx(fmx(r.v[2][1], r.v[2][2]), r.v[2][3]);
  float m4 = fmx(fmx(r.v[3][0], r.v[3][1]), r.v[3][2]);
  float m = fmx(fmx(m0, m1), m2);
  m = fmx(fmx(m, m3), m4);
  m = fmx(m, r.v[3][3]);
  const float wm = wave_max_dpp(m);
  if (__builtin_expect(wm != wm, 0)) return exact_row(rp, lane, t);
  const bool t_ok = t >= 0 && t < C;
  if (!t_ok || xt_loaded != wm) return false;
  constexpr int tail_lanes = (C - 768) / 4;
  const uint64_t tail = tail_lanes >= 64 ? ~0ull : ((1ull << tail_lanes) - 1);
  int cnt = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint64_t mk = __ballot(r.v[u][e] == wm);
      if (u == 3) mk &= tail;
      cnt += __builtin_popcountll(mk);
    }
  if (cnt == 1) return true;
  return exact_row(rp, lane, t);
}

template <int E>
__global__ __launch_bounds__(256) void m3(const float* __restrict__ x, const int64_t* __restrict__ y,
                                          unsigned long long* ws, float* dst, float* slab) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave_id();
  uint32_t correct = 0;
  if (row < N) {
    const float* rp = x + (size_t)row * C;
    Row r;
    load_row(rp, lane, r);
    const int64_t t = y[row];
    const int64_t tc = t < 0 ? 0 : (t >= C ? C - 1 : t);
    const float xt = rp[tc];
    // the target and its score arrive while the row streams in (one chained scalar round
    // trip beside the row's): the clobber keeps the row loads issued above this point
    asm volatile("" ::"s"(xt) : "memory");
    correct = row_correct3(r, lane, t, xt, rp);
  }
  epilogue<E>(correct, ws, dst, slab);
}


// R4: the row max (max3 tree + DPP), the target's own score by ONE uniform register-indexed
// move (s_set_gpr_idx_on + v_mov: the lane-owner's register) + readlane, and a ballot tie count
// only when the target holds the max.  No per-element selects, no masking: lanes past C in the
// last load re-read columns 0..3 (cannot change the max) and are masked out of the tie count.
typedef float v16f __attribute__((ext_vector_type(16)));

template <int E>
__global__ __launch_bounds__(256) void m4(const float* __restrict__ x, const int64_t* __restrict__ y,
                                          unsigned long long* ws, float* dst, float* slab) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave_id();
  uint32_t correct = 0;
  if (row < N) {
    const float* rp = x + (size_t)row * C;
    float4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int col = u * STEP + lane * 4;
      q[u] = *reinterpret_cast<const float4*>(rp + (col < C ? col : 0));
    }
    const int64_t t = y[row];
    const v16f v = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w,
                    q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w};
    float m = fmx(fmx(v[0], v[1]), v[2]);
    m = fmx(fmx(m, v[3]), v[4]);
    m = fmx(fmx(m, v[5]), v[6]);
    m = fmx(fmx(m, v[7]), v[8]);
    m = fmx(fmx(m, v[9]), v[10]);
    m = fmx(fmx(m, v[11]), v[12]);
    m = fmx(fmx(m, v[13]), v[14]);
    m = fmx(m, v[15]);
    const float wm = wave_max_dpp(m);
    if (__builtin_expect(wm != wm, 0)) {
      correct = exact_row(rp, lane, t);
    } else if (t >= 0 && t < C) {
      const int tu = static_cast<int>(t);
      const float sel = v[((tu >> 8) << 2) | (tu & 3)];
      const float xt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), (tu & 255) >> 2));
      if (xt == wm) {
        constexpr int tail_lanes = (C - 768) / 4;
        const uint64_t tail = tail_lanes >= 64 ? ~0ull : ((1ull << tail_lanes) - 1);
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          uint64_t mk = __ballot(v[e] == wm);
          if (e >= 12) mk &= tail;
          cnt += __builtin_popcountll(mk);
        }
        correct = cnt == 1 ? 1u : static_cast<uint32_t>(exact_row(rp, lane, t));
      }
    }
  }
  epilogue<E>(correct, ws, dst, slab);
}

template <int RPW>
__global__ __launch_bounds__(256) void smax(const float* __restrict__ x, float* slab) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + wave_id()) * RPW;
  float m = -1e30f;
  if (r0 < N) {
    Row rows[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) load_row(x + (size_t)(r0 + k) * C, lane, rows[k]);
#pragma unroll
    for (int k = 0; k < RPW; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) m = fmaxf(m, rows[k].v[u][e]);
  }
  if (m == 12345.f) slab[blockIdx.x] = m;
}

__global__ void empty_k(float* slab) {
  if (threadIdx.x == 1023) slab[0] = 1.f;
}

int main(int argc, char** argv) {
  const int POOL = argc > 1 ? atoi(argv[1]) : 8;
  const int iters = 400;
  std::vector<float> hx((size_t)N * C);
  std::vector<int64_t> hy(N);
  srand(1);
  for (auto& v : hx) v = (rand() / (float)RAND_MAX) * 2.f - 1.f;
  for (int i = 0; i < N; ++i) hy[i] = rand() % C;
  // special rows: full ties, NaN, target = max with an earlier tie, target = first max
  for (int c = 0; c < C; ++c) hx[(size_t)0 * C + c] = 0.5f;
  hy[0] = 0;
  for (int c = 0; c < C; ++c) hx[(size_t)1 * C + c] = 0.5f;
  hy[1] = 7;
  hx[(size_t)2 * C + 500] = NAN;
  hy[2] = 500;
  hx[(size_t)3 * C + 600] = NAN;
  hy[3] = 3;
  hx[(size_t)4 * C + 10] = 5.f;
  hx[(size_t)4 * C + 20] = 5.f;
  hy[4] = 20;
  hx[(size_t)5 * C + 10] = 5.f;
  hx[(size_t)5 * C + 20] = 5.f;
  hy[5] = 10;
  hx[(size_t)6 * C + 999] = 9.f;
  hy[6] = 999;
  const int every = argc > 2 ? atoi(argv[2]) : 5;
  for (int i = 7; every > 0 && i < N; i += every) {  // 1/every of the rows correct
    int bi = 0;
    for (int c = 1; c < C; ++c)
      if (hx[(size_t)i * C + c] > hx[(size_t)i * C + bi]) bi = c;
    hy[i] = bi;
  }
  int ref = 0;
  for (int i = 0; i < N; ++i) {
    int bi = 0;
    float bv = hx[(size_t)i * C];
    for (int c = 1; c < C; ++c) {
      const float v = hx[(size_t)i * C + c];
      if (std::isnan(bv)) break;
      if (std::isnan(v) || v > bv) {
        bv = v;
        bi = c;
      }
    }
    ref += (bi == hy[i]);
  }
  std::vector<float*> xs(POOL);
  std::vector<int64_t*> ys(POOL);
  for (int p = 0; p < POOL; ++p) {
    CK(hipMalloc(&xs[p], hx.size() * 4));
    CK(hipMemcpy(xs[p], hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&ys[p], N * 8));
    CK(hipMemcpy(ys[p], hy.data(), N * 8, hipMemcpyHostToDevice));
  }
  float *dst, *slab;
  unsigned long long* ws;
  CK(hipMalloc(&dst, 16));
  CK(hipMalloc(&slab, 65536 * 4));
  CK(hipMalloc(&ws, kFoldCells * 8 * 4));
  CK(hipMemset(ws, 0, kFoldCells * 8 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  auto prod = [&](int p) {
    ClsCountsArgs a;
    a.input = xs[p];
    a.in_dt = DType::f32;
    a.n = N;
    a.c = C;
    a.row_stride = C;
    a.target = ys[p];
    a.tg_dt = DType::i64;
    a.k = 1;
    a.num_classes = C;
    a.micro_correct = dst;
    a.micro_total = dst + 1;
    a.fold_ws = ws;
    launch_cls_counts(a, 0);
  };
  struct V {
    const char* name;
    std::function<void(int)> fn;
    bool counts;  // accumulates into dst[0]
    std::vector<float> t;
  };
  std::vector<V> vs;
  vs.push_back({"prod (launch_cls_counts)", prod, true, {}});
#define M1(R, E, RPW, G)                                                                           \
  vs.push_back({"m1 R" #R " E" #E " rpw" #RPW, [&](int p) {                                         \
                  hipLaunchKernelGGL((m1<R, E, RPW>), dim3(G), dim3(256), 0, 0, xs[p], ys[p], ws, dst, \
                                     slab);                                                          \
                },                                                                                   \
                E == 0, {}});
  M1(0, 0, 1, 2048)
  M1(0, 2, 1, 2048)
#define ISO(T, RED, E)                                                                              \
  vs.push_back({"iso T" #T " RED" #RED " E" #E, [&](int p) {                                         \
                  hipLaunchKernelGGL((iso<T, RED, E>), dim3(2048), dim3(256), 0, 0, xs[p], ys[p], ws, dst, slab); \
                },                                                                                   \
                false, {}});
  ISO(1, 1, 2)
  ISO(1, 1, 1)
  ISO(1, 1, 0)
  vs.push_back({"m4 E0 (fold)", [&](int p) { hipLaunchKernelGGL((m4<0>), dim3(2048), dim3(256), 0, 0, xs[p], ys[p], ws, dst, slab); }, true, {}});
  vs.push_back({"m4 E1 (slab)", [&](int p) { hipLaunchKernelGGL((m4<1>), dim3(2048), dim3(256), 0, 0, xs[p], ys[p], ws, dst, slab); }, false, {}});
  vs.push_back({"m4 E4 (wave atomics)", [&](int p) { hipLaunchKernelGGL((m4<4>), dim3(2048), dim3(256), 0, 0, xs[p], ys[p], ws, dst, slab); }, false, {}});
  vs.push_back({"smax rpw1 g2048", [&](int p) { hipLaunchKernelGGL((smax<1>), dim3(2048), dim3(256), 0, 0, xs[p], slab); }, false, {}});
  vs.push_back({"smax rpw2 g1024", [&](int p) { hipLaunchKernelGGL((smax<2>), dim3(1024), dim3(256), 0, 0, xs[p], slab); }, false, {}});
  vs.push_back({"empty g2048 b256", [&](int p) { hipLaunchKernelGGL(empty_k, dim3(2048), dim3(256), 0, 0, slab); }, false, {}});
  vs.push_back({"empty g512 b256", [&](int p) { hipLaunchKernelGGL(empty_k, dim3(512), dim3(256), 0, 0, slab); }, false, {}});

  // correctness: one launch per counting variant on batch 0
  for (auto& v : vs) {
    if (!v.counts) continue;
    CK(hipMemset(dst, 0, 16));
    v.fn(0);
    CK(hipDeviceSynchronize());
    float got;
    CK(hipMemcpy(&got, dst, 4, hipMemcpyDeviceToHost));
    printf("check %-26s got %.0f expected %d %s\n", v.name, got, ref, got == ref ? "OK" : "MISMATCH");
  }
  for (int round = 0; round < 5; ++round) {
    for (auto& v : vs) {
      for (int i = 0; i < 20; ++i) v.fn(i % POOL);
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) v.fn(i % POOL);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / iters);
    }
  }
  const double bytes = (double)N * C * 4;
  printf("pool %d batches (%.0f MB), correct rows %d/%d\n", POOL, POOL * bytes / 1e6, ref, N);
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-28s median %6.2f us  min %6.2f us  %5.2f TB/s\n", v.name, v.t[v.t.size() / 2], v.t[0],
           bytes / (v.t[v.t.size() / 2] * 1e-6) / 1e12);
  }
  return 0;
}
