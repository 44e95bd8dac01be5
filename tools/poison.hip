// Diagnostic only: fill every CU's LDS and a wave's worth of VGPRs
// with a fixed bit pattern, then exit.  A solve launched after it (serially) that reads state it
// never wrote sees the pattern; comparing solves after two patterns rules stale-state reads in or
// out.  Not on the product path.  Build on the CPU before the gpurun call:
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/poison.hip -o tools/_build/libpoison.so
#include <hip/hip_runtime.h>

#define POISON_LDS_WORDS (160 * 1024 / 4)

__global__ __launch_bounds__(1024) void poison_lds_kernel(unsigned pattern, unsigned* sink) {
  extern __shared__ unsigned s_lds[];
  for (int i = threadIdx.x; i < POISON_LDS_WORDS; i += blockDim.x) s_lds[i] = pattern ^ (unsigned)i;
  __syncthreads();
  if (s_lds[threadIdx.x] == 0x5a5a5a5au && pattern == 0x01234567u) sink[0] = 1u;  // keeps the stores
}

// VGPR fill: 240 live registers per lane, all derived from the pattern, kept live by an empty asm
__global__ __launch_bounds__(256) void poison_vgpr_kernel(unsigned pattern, unsigned* sink) {
  unsigned r[240];
#pragma unroll
  for (int i = 0; i < 240; ++i) {
    r[i] = pattern ^ (unsigned)(i * 0x9e3779b9u);
    asm volatile("" : "+v"(r[i]));
  }
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < 240; ++i) {
    asm volatile("" : "+v"(r[i]));
    acc ^= r[i];
  }
  if (acc == 0x5a5a5a5au && pattern == 0x01234567u) sink[0] = acc;
}

extern "C" int poison_fill(unsigned pattern, int blocks) {
  unsigned* sink = nullptr;
  if (hipMalloc(&sink, 4) != hipSuccess) return 1;
  if (hipFuncSetAttribute((const void*)poison_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024) != hipSuccess)
    return 2;
  hipLaunchKernelGGL(poison_lds_kernel, dim3(blocks), dim3(1024), 160 * 1024, 0, pattern, sink);
  hipLaunchKernelGGL(poison_vgpr_kernel, dim3(blocks * 8), dim3(256), 0, 0, pattern, sink);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipFree(sink);
  return 0;
}
