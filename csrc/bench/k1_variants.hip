// Standalone A/B harness for the K1 argmax-accuracy kernel shape (bs=8192, C=1000, fp32).
// Every variant runs interleaved in ONE process on the same data (§5.4 rule 24).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "tea_common.h"
using namespace tea;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int N = 8192, C = 1000, POOL = 8;

// MODE 0: full argmax + atomic per block; 1: argmax + slab store (no atomic);
// 2: loads + plain max only (no index) + slab; 3: loads+sum only + slab
template <int MODE, int RPW, int BLOCK, bool NT>
__global__ __launch_bounds__(BLOCK) void kvar(const float* __restrict__ x, const int64_t* __restrict__ y,
                                             float* out, float* slab, int n) {
  constexpr int WPB = BLOCK / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  int correct = 0;
  for (int64_t r0 = ((int64_t)blockIdx.x * WPB + wave_id()) * RPW; r0 < n; r0 += nw * RPW) {
    float v[RPW][4][4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) ok[u] = (u * 256 + lane * 4) < C;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const float* rp = x + (r0 + r) * C;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ok[u] && r0 + r < n) {
          typedef float f4 __attribute__((ext_vector_type(4)));
          const f4* p = reinterpret_cast<const f4*>(rp + u * 256 + lane * 4);
          f4 q;
          if constexpr (NT) q = __builtin_nontemporal_load(p); else q = *p;
          v[r][u][0] = q.x; v[r][u][1] = q.y; v[r][u][2] = q.z; v[r][u][3] = q.w;
        } else {
          v[r][u][0] = v[r][u][1] = v[r][u][2] = v[r][u][3] = -__builtin_huge_valf();
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      if (r0 + r >= n) break;
      if constexpr (MODE <= 1) {
        float bv = -__builtin_huge_valf(); int bi = 0x7fffffff;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int col = u * 256 + lane * 4 + e;
            if (argmax_better(v[r][u][e], col, bv, bi)) { bv = v[r][u][e]; bi = col; }
          }
        wave_argmax(bv, bi);
        correct += (bi == y[r0 + r]);
      } else if constexpr (MODE == 2) {
        float bv = -__builtin_huge_valf();
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) bv = fmaxf(bv, v[r][u][e]);
        bv = wave_max(bv);
        correct += (bv > 3.f);
      } else {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) s += (v[r][u][e] > -1e30f) ? v[r][u][e] : 0.f;
        s = wave_sum(s);
        correct += (s > 0.f);
      }
    }
  }
  __shared__ int lds[WPB];
  if (lane == 0) lds[threadIdx.x >> 6] = correct;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < WPB; ++w) s += lds[w];
    if (MODE == 0) atomicAdd(out, (float)s); else slab[blockIdx.x] = (float)s;
  }
}


struct FoldWS { float* vals; unsigned* cnts; int shards; };
__device__ __forceinline__ void grid_fold_add(float v, float* dst, FoldWS ws) {
  const int S = ws.shards;
  const int s = blockIdx.x % S;
  const unsigned members = gridDim.x / S + ((int)(gridDim.x % S) > s ? 1u : 0u);
  if (v != 0.f) atomicAdd(ws.vals + s * 16, v);
  const unsigned old = __hip_atomic_fetch_add(ws.cnts + s * 16, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (old == members - 1) {
    const float tot = __hip_atomic_exchange(ws.vals + s * 16, 0.f, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ws.cnts + s * 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tot != 0.f) atomicAdd(dst, tot);
  }
}

// two-phase argmax of 16 lane values at columns base + {u*256 + lane*4 + e}
__device__ __forceinline__ void fast_argmax16(const float (&v)[4][4], int lane, float& bv, int& bi) {
  float m = v[0][0];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) m = __builtin_elementwise_maximum(m, v[u][e]);
  int idx = 0x7fffffff;
#pragma unroll
  for (int u = 3; u >= 0; --u)
#pragma unroll
    for (int e = 3; e >= 0; --e) idx = (v[u][e] == m) ? (u * 256 + lane * 4 + e) : idx;
  bv = m; bi = idx;
}
__device__ __forceinline__ void wave_argmax_fast(float& bv, int& bi) {
  float m = bv;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = __builtin_elementwise_maximum(m, __shfl_xor(m, o, 64));
  int idx = (bv == m) ? bi : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) idx = min(idx, __shfl_xor(idx, o, 64));
  bv = m; bi = idx;
}

// MODE 4: fast argmax; FOLD: 0 slab, 1 hierarchical fold
template <int FOLD, int RPW, int BLOCK>
__global__ __launch_bounds__(BLOCK) void kfast(const float* __restrict__ x, const int64_t* __restrict__ y,
                                             float* out, float* slab, int n, FoldWS ws) {
  constexpr int WPB = BLOCK / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  int correct = 0;
  for (int64_t r0 = ((int64_t)blockIdx.x * WPB + wave_id()) * RPW; r0 < n; r0 += nw * RPW) {
    float v[RPW][4][4];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const float* rp = x + (r0 + r) * C;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int col = u * 256 + lane * 4;
        if (col < C && r0 + r < n) {
          const float4 q = *reinterpret_cast<const float4*>(rp + col);
          v[r][u][0] = q.x; v[r][u][1] = q.y; v[r][u][2] = q.z; v[r][u][3] = q.w;
        } else {
          v[r][u][0] = v[r][u][1] = v[r][u][2] = v[r][u][3] = -__builtin_huge_valf();
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      if (r0 + r >= n) break;
      float bv; int bi;
      fast_argmax16(v[r], lane, bv, bi);
      wave_argmax_fast(bv, bi);
      correct += (bi == y[r0 + r]);
    }
  }
  __shared__ int lds[WPB];
  if (lane == 0) lds[threadIdx.x >> 6] = correct;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < WPB; ++w) s += lds[w];
    if (FOLD == 1) grid_fold_add((float)s, out, ws);
    else if (FOLD == 2) atomicAdd(out, (float)s);
    else if (FOLD == 3) {
      const int S = ws.shards; const int sh = blockIdx.x % S;
      const unsigned members = gridDim.x / S + ((int)(gridDim.x % S) > sh ? 1u : 0u);
      __hip_atomic_fetch_add(ws.vals + sh * 16, (float)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned old = __hip_atomic_fetch_add(ws.cnts + sh * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == members - 1) {
        const float tot = __hip_atomic_exchange(ws.vals + sh * 16, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws.cnts + sh * 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(out, tot);
      }
    }
    else slab[blockIdx.x] = (float)s;
  }
}

template <int FOLD, int RPW, int BLOCK>
float runf(float* const* xs, int64_t* const* ys, float* out, float* slab, int grid, FoldWS ws, hipEvent_t e0, hipEvent_t e1, int iters) {
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((kfast<FOLD, RPW, BLOCK>), dim3(grid), dim3(BLOCK), 0, 0, xs[i % POOL], ys[i % POOL], out, slab, N, ws);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((kfast<FOLD, RPW, BLOCK>), dim3(grid), dim3(BLOCK), 0, 0, xs[i % POOL], ys[i % POOL], out, slab, N, ws);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}

template <int MODE, int RPW, int BLOCK, bool NT>
float run(const char* name, float* const* xs, int64_t* const* ys, float* out, float* slab, int grid, hipEvent_t e0, hipEvent_t e1, int iters) {
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((kvar<MODE, RPW, BLOCK, NT>), dim3(grid), dim3(BLOCK), 0, 0, xs[i % POOL], ys[i % POOL], out, slab, N);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((kvar<MODE, RPW, BLOCK, NT>), dim3(grid), dim3(BLOCK), 0, 0, xs[i % POOL], ys[i % POOL], out, slab, N);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}

int main() {
  std::vector<float> hx((size_t)N * C);
  std::vector<int64_t> hy(N);
  srand(1);
  for (auto& v : hx) v = (rand() / (float)RAND_MAX) * 2.f - 1.f;
  for (auto& v : hy) v = rand() % C;
  float* xs[POOL]; int64_t* ys[POOL];
  for (int p = 0; p < POOL; ++p) {
    CK(hipMalloc(&xs[p], hx.size() * 4)); CK(hipMemcpy(xs[p], hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&ys[p], N * 8)); CK(hipMemcpy(ys[p], hy.data(), N * 8, hipMemcpyHostToDevice));
  }
  float *out, *slab; CK(hipMalloc(&out, 4)); CK(hipMalloc(&slab, 65536 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 400;
  const double bytes = (double)N * C * 4;
  struct R { const char* name; std::vector<float> t; };
  std::vector<R> rs;
  auto rec = [&](const char* name, float us) {
    for (auto& r : rs) if (r.name == name) { r.t.push_back(us); return; }
    rs.push_back({name, {us}});
  };
  float* wsv; unsigned* wsc;
  CK(hipMalloc(&wsv, 64 * 16 * 4)); CK(hipMemset(wsv, 0, 64 * 16 * 4));
  CK(hipMalloc(&wsc, 64 * 16 * 4)); CK(hipMemset(wsc, 0, 64 * 16 * 4));
  FoldWS ws64{wsv, wsc, 64}, ws32{wsv, wsc, 32}, ws8{wsv, wsc, 8};
  // correctness of fold + fast argmax: count correct over one batch vs host
  {
    CK(hipMemset(out, 0, 4));
    hipLaunchKernelGGL((kfast<1, 1, 256>), dim3(2048), dim3(256), 0, 0, xs[0], ys[0], out, slab, N, ws64);
    hipLaunchKernelGGL((kfast<1, 1, 256>), dim3(1000), dim3(256), 0, 0, xs[0], ys[0], out, slab, N, ws32);
    float got; CK(hipMemcpy(&got, out, 4, hipMemcpyDeviceToHost));
    int ref = 0;
    for (int i = 0; i < N; ++i) { int bi = 0; for (int c = 1; c < C; ++c) if (hx[(size_t)i * C + c] > hx[(size_t)i * C + bi]) bi = c; ref += (bi == hy[i]); }
    printf("fold check: got %.0f expected %d\n", got, 2 * ref);
  }
  for (int round = 0; round < 5; ++round) {
    rec("F slab     rpw1 b256 g2048", runf<0, 1, 256>(xs, ys, out, slab, 2048, ws64, e0, e1, iters));
    rec("F atomic   rpw1 b256 g2048", runf<2, 1, 256>(xs, ys, out, slab, 2048, ws64, e0, e1, iters));
    rec("F rlxfold64 rpw1 b256 g2048", runf<3, 1, 256>(xs, ys, out, slab, 2048, ws64, e0, e1, iters));
    rec("F rlxfold8 rpw1 b256 g2048", runf<3, 1, 256>(xs, ys, out, slab, 2048, ws8, e0, e1, iters));
    rec("F slab     rpw2 b1024 g256", runf<0, 2, 1024>(xs, ys, out, slab, 256, ws64, e0, e1, iters));
    rec("F atomic   rpw2 b1024 g256", runf<2, 2, 1024>(xs, ys, out, slab, 256, ws64, e0, e1, iters));
    rec("F atomic   rpw4 b1024 g128", runf<2, 4, 1024>(xs, ys, out, slab, 128, ws64, e0, e1, iters));
    rec("F slab     rpw2 b512 g512 ", runf<0, 2, 512>(xs, ys, out, slab, 512, ws64, e0, e1, iters));
    rec("F atomic   rpw2 b512 g512 ", runf<2, 2, 512>(xs, ys, out, slab, 512, ws64, e0, e1, iters));
    rec("F rlxfold64 rpw2 b512 g512", runf<3, 2, 512>(xs, ys, out, slab, 512, ws64, e0, e1, iters));
    rec("M0 atomic  rpw1 b256 g2048", run<0, 1, 256, false>("", xs, ys, out, slab, 2048, e0, e1, iters));
    rec("M0 atomic  rpw1 b256 g1024", run<0, 1, 256, false>("", xs, ys, out, slab, 1024, e0, e1, iters));
    rec("M1 slab    rpw1 b256 g2048", run<1, 1, 256, false>("", xs, ys, out, slab, 2048, e0, e1, iters));
    rec("M1 slab    rpw2 b256 g1024", run<1, 2, 256, false>("", xs, ys, out, slab, 1024, e0, e1, iters));
    rec("M1 slab    rpw2 b256 g512 ", run<1, 2, 256, false>("", xs, ys, out, slab, 512, e0, e1, iters));
    rec("M1 slab    rpw4 b256 g512 ", run<1, 4, 256, false>("", xs, ys, out, slab, 512, e0, e1, iters));
    rec("M1 slab nt rpw2 b256 g1024", run<1, 2, 256, true>("", xs, ys, out, slab, 1024, e0, e1, iters));
    rec("M1 slab    rpw1 b512 g1024", run<1, 1, 512, false>("", xs, ys, out, slab, 1024, e0, e1, iters));
    rec("M2 max     rpw1 b256 g2048", run<2, 1, 256, false>("", xs, ys, out, slab, 2048, e0, e1, iters));
    rec("M3 sum     rpw1 b256 g2048", run<3, 1, 256, false>("", xs, ys, out, slab, 2048, e0, e1, iters));
    rec("M3 sum     rpw2 b256 g1024", run<3, 2, 256, false>("", xs, ys, out, slab, 1024, e0, e1, iters));
    rec("M3 sum nt  rpw2 b256 g1024", run<3, 2, 256, true>("", xs, ys, out, slab, 1024, e0, e1, iters));
  }
  for (auto& r : rs) {
    std::sort(r.t.begin(), r.t.end());
    printf("%-28s median %7.2f us  min %7.2f us  %6.2f TB/s\n", r.name, r.t[r.t.size() / 2], r.t[0], bytes / (r.t[r.t.size() / 2] * 1e-6) / 1e12);
  }
  return 0;
}
