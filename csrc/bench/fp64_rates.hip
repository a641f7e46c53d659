// Microbenchmark: per-wave issue cost of FP64 VALU FMA vs FP32 FMA vs FP64 MFMA 16x16x4, and the
// latency of an LDS write -> broadcast read round trip, on one wave of one CU (shader clocks,
// s_memtime).  Informs the K9d diagonal-tile design (csrc/kernels/cholesky.hip).
//   hipcc --offload-arch=gfx950 -O3 csrc/bench/fp64_rates.hip -o /tmp/fp64_rates && /tmp/fp64_rates
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

__global__ void fma64_kernel(double* out, unsigned long long* cyc, double seed) {
  double a[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = seed + q + threadIdx.x;
  const double b = 1.0000001, c = 1e-9;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = fma(a[q], b, c);
  }
  const unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += a[q];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void fma32_kernel(float* out, unsigned long long* cyc, float seed) {
  float a[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = seed + q + threadIdx.x;
  const float b = 1.0000001f, c = 1e-9f;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = fmaf(a[q], b, c);
  }
  const unsigned long long t1 = clock64();
  float s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += a[q];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void mfma64_kernel(double* out, unsigned long long* cyc, double seed) {
  f64x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
  const double x = seed + threadIdx.x, y = seed - threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < kIters / 4; ++i) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[q], 0, 0, 0);
  }
  const unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// dependent FP64 chain latency: a = fma(a, b, c) serially
__global__ void chain64_kernel(double* out, unsigned long long* cyc, double seed) {
  double a = seed + threadIdx.x;
  const double b = 1.0000001, c = 1e-9;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < kIters; ++i) a = fma(a, b, c);
  const unsigned long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// LDS: lane-wise write, then every lane reads one broadcast value written by another lane
__global__ void lds_rt_kernel(double* out, unsigned long long* cyc, double seed) {
  __shared__ double col[64];
  double v = seed + threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < kIters / 8; ++i) {
    col[threadIdx.x] = v;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v = col[(i + 1) & 63] + 1.0;
  }
  const unsigned long long t1 = clock64();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// one elimination step's update over 32 slots: r[m] -= u * col[m], the column broadcast from lane
// m's register by v_readlane (2 per double, SGPR operand) - no LDS round trip
__global__ void readlane_elim_kernel(double* out, unsigned long long* cyc, double seed) {
  double r[32];
#pragma unroll
  for (int m = 0; m < 32; ++m) r[m] = seed + m * threadIdx.x;
  double src = seed * threadIdx.x;
  const double u = 1e-3 * threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < 64; ++i) {
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(src), m);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(src), m);
      r[m] = fma(-u, __hiloint2double(hi, lo), r[m]);
    }
    src = r[i & 31];
  }
  const unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int m = 0; m < 32; ++m) s += r[m];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the same update with the column in LDS: write (lanes), one wait, 16 ds_read_b128 broadcasts, 32 FMAs
__global__ void lds_elim_kernel(double* out, unsigned long long* cyc, double seed) {
  __shared__ __attribute__((aligned(16))) double col[64];
  double r[32];
#pragma unroll
  for (int m = 0; m < 32; ++m) r[m] = seed + m * threadIdx.x;
  double src = seed * threadIdx.x;
  const double u = 1e-3 * threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < 64; ++i) {
    col[threadIdx.x] = src;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    double v[32];
#pragma unroll
    for (int m = 0; m < 32; m += 2) {
      const double2 c2 = *reinterpret_cast<const double2*>(&col[m]);
      v[m] = c2.x;
      v[m + 1] = c2.y;
    }
#pragma unroll
    for (int m = 0; m < 32; ++m) r[m] = fma(-u, v[m], r[m]);
    src = r[i & 31];
  }
  const unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int m = 0; m < 32; ++m) s += r[m];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the same two kernels compiled for ONE wave per SIMD (amdgpu_waves_per_eu(1, 1)): the default
// occupancy-driven scheduling keeps 2 loads in flight and waits a full LDS latency per pair
__global__ __attribute__((amdgpu_waves_per_eu(1, 1))) void lds_elim_w1_kernel(double* out, unsigned long long* cyc,
                                                                              double seed) {
  __shared__ __attribute__((aligned(16))) double col[64];
  double r[32];
#pragma unroll
  for (int m = 0; m < 32; ++m) r[m] = seed + m * threadIdx.x;
  double src = seed * threadIdx.x;
  const double u = 1e-3 * threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < 64; ++i) {
    col[threadIdx.x] = src;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    double v[32];
#pragma unroll
    for (int m = 0; m < 32; m += 2) {
      const double2 c2 = *reinterpret_cast<const double2*>(&col[m]);
      v[m] = c2.x;
      v[m + 1] = c2.y;
    }
    __builtin_amdgcn_sched_barrier(0);  // every read issued before the first FMA
#pragma unroll
    for (int m = 0; m < 32; ++m) r[m] = fma(-u, v[m], r[m]);
    src = r[i & 31];
  }
  const unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int m = 0; m < 32; ++m) s += r[m];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ __attribute__((amdgpu_waves_per_eu(1, 1))) void readlane_elim_w1_kernel(double* out, unsigned long long* cyc,
                                                                                   double seed) {
  double r[32];
#pragma unroll
  for (int m = 0; m < 32; ++m) r[m] = seed + m * threadIdx.x;
  double src = seed * threadIdx.x;
  const double u = 1e-3 * threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < 64; ++i) {
    double v[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(src), m);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(src), m);
      v[m] = __hiloint2double(hi, lo);
    }
    __builtin_amdgcn_sched_barrier(0);  // every readlane issued before the first FMA
#pragma unroll
    for (int m = 0; m < 32; ++m) r[m] = fma(-u, v[m], r[m]);
    src = r[i & 31];
  }
  const unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int m = 0; m < 32; ++m) s += r[m];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double* d;
  float* f;
  unsigned long long* c;
  hipMalloc(&d, 64 * sizeof(double));
  hipMalloc(&f, 64 * sizeof(float));
  hipMalloc(&c, 8);
  unsigned long long h = 0;
  auto run = [&](const char* name, auto launch, double per) {
    launch();
    hipDeviceSynchronize();
    launch();
    hipDeviceSynchronize();
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    std::printf("%-28s %8.2f cycles per instruction (wave64)\n", name, static_cast<double>(h) / per);
  };
  run("v_fma_f64 (8 chains)", [&] { fma64_kernel<<<1, 64>>>(d, c, 1.0); }, kIters * 8.0);
  run("v_fma_f32 (8 chains)", [&] { fma32_kernel<<<1, 64>>>(f, c, 1.0f); }, kIters * 8.0);
  run("v_mfma_f64_16x16x4 (4 acc)", [&] { mfma64_kernel<<<1, 64>>>(d, c, 1.0); }, kIters / 4 * 4.0);
  run("v_fma_f64 dependent chain", [&] { chain64_kernel<<<1, 64>>>(d, c, 1.0); }, kIters);
  run("LDS write+bcast read trip", [&] { lds_rt_kernel<<<1, 64>>>(d, c, 1.0); }, kIters / 8.0);
  run("elim 32 slots via readlane", [&] { readlane_elim_kernel<<<1, 64>>>(d, c, 1.0); }, 64.0);
  run("elim 32 slots via LDS", [&] { lds_elim_kernel<<<1, 64>>>(d, c, 1.0); }, 64.0);
  run("elim 32 via LDS, 1 wave/EU", [&] { lds_elim_w1_kernel<<<1, 64>>>(d, c, 1.0); }, 64.0);
  run("elim 32 via readlane, 1w/EU", [&] { readlane_elim_w1_kernel<<<1, 64>>>(d, c, 1.0); }, 64.0);
  return 0;
}
