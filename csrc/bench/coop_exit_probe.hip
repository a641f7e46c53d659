// Control for the exit-time crash under rocprofv3: one trivial
// cooperative launch (and, with argv[1] == "plain", one ordinary launch instead), a device
// synchronize, a normal return from main.  No torch, no torcheval_amd.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void touch(int* p) {
  if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x;
}

int main(int argc, char** argv) {
  const bool plain = argc > 1 && std::strcmp(argv[1], "plain") == 0;
  int* d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 2;
  void* args[] = {&d};
  const hipError_t rc = plain ? hipLaunchKernel(reinterpret_cast<const void*>(&touch), dim3(256), dim3(256), args, 0, 0)
                              : hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&touch), dim3(256), dim3(256),
                                                           args, 0, 0);
  if (rc != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 3;
  int h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  (void)hipFree(d);
  std::printf("done %d\n", h[255]);
  return 0;
}
