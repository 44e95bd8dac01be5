// Microbenchmark (diagnostic, not shipped): throughput of the register-resident linearize, the
// part of the persistent / block kernels' round that scales with the items per lane.  Every
// block holds NPT items per lane in registers (as the kernels do) and runs `rounds` linearizes at a
// slightly moving pose, each followed by the wave reduction and one LDS store per wave (the
// kernels' per-round epilogue before the hand-off).  No hand-off: this is the linearize alone.
// build (scalar, the shipped flags):
//   HIPCC=/opt/rocm/bin/hipcc 02-visualodometry_amd/hipcc_nopk.sh -O3 -std=c++17 --offload-arch=gfx950 \
//     -I02-visualodometry_amd/csrc -Iinclude tools/ubench/lin_ubench.hip -o tools/ubench/lin_ubench
// build (packed A/B): /opt/rocm/bin/hipcc -DPICP_ALLOW_PK ... -o tools/ubench/lin_ubench_pk
// usage: lin_ubench [rounds]  -> ns per round and items per second for each variant
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "picp_device.h"
using namespace picp;

template <int NPT, bool PAIRS, int BS>
__global__ __launch_bounds__(BS) void lin(const float* __restrict__ X, const float* __restrict__ Y,
                                          const float* __restrict__ Z, const float* __restrict__ U,
                                          const float* __restrict__ V, int n, int rounds, float* sink) {
  __shared__ float s_wave[BS / 64][PICP_NPART];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_block = NPT * BS;
  const int first = blockIdx.x * per_block;
  const int count = max(0, min(per_block, n - first));
  float xs[NPT], ys[NPT], zs[NPT], us[NPT], vs[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = first + min(tid + k * BS, max(count - 1, 0));
    xs[k] = X[i]; ys[k] = Y[i]; zs[k] = Z[i]; us[k] = U[i]; vs[k] = V[i];
  }
  Cam C;
  C.k00 = 180.0f; C.k01 = 0.0f; C.k02 = 320.0f;
  C.k10 = 0.0f; C.k11 = 180.0f; C.k12 = 240.0f;
  C.k20 = 0.0f; C.k21 = 0.0f; C.k22 = 1.0f;
  C.maxx = 639.0f; C.maxy = 479.0f;
  const float thr = 3000.0f, inv_thr = 1.0f / 3000.0f;
  float check = 0.0f;
  for (int r = 0; r < rounds; ++r) {
    Pose T;
    T.r00 = 1.0f; T.r01 = 1e-4f * r; T.r02 = 0.0f;
    T.r10 = -1e-4f * r; T.r11 = 1.0f; T.r12 = 0.0f;
    T.r20 = 0.0f; T.r21 = 0.0f; T.r22 = 1.0f;
    T.t0 = 1e-5f * r; T.t1 = 0.0f; T.t2 = __builtin_amdgcn_readfirstlane(__float_as_int(check)) == 12345 ? 1.0f : 0.0f;
    float v[PICP_NPART];
    Cnt nc = {0u, 0u};
    if constexpr (PAIRS) {
      Acc2 a;
      acc2_zero(a);
      accumulate_regs<PICP_V_PINHOLE, NPT>(T, C, thr, inv_thr, false, xs, ys, zs, us, vs, tid, BS, count, a, nc);
      acc2_fold(a, v);
    } else {
      Acc a;
      acc_zero(a);
      accumulate_regs1<PICP_V_PINHOLE, NPT>(T, C, thr, inv_thr, false, xs, ys, zs, us, vs, tid, BS, count, a, nc);
      acc_fold(a, v);
    }
    const float wsum = wave_counts(wave_reduce32(v, lane), lane, nc);
    if ((lane & 1) == 0) s_wave[wave][lane >> 1] = wsum;
    __syncthreads();
    check += s_wave[(r + 1) % (BS / 64)][lane & 31];
    __syncthreads();
  }
  if (tid == 0) sink[blockIdx.x] = check;
}

template <int NPT, bool PAIRS, int BS>
static void run(const char* name, float* const* d, int n_per_cu, int cus, int rounds, float* sink) {
  const int per_block = NPT * BS;
  const int blocks = cus * (n_per_cu / per_block);
  const int n = blocks * per_block;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((lin<NPT, PAIRS, BS>), dim3(blocks), dim3(BS), 0, 0, d[0], d[1], d[2], d[3], d[4], n, 4, sink);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((lin<NPT, PAIRS, BS>), dim3(blocks), dim3(BS), 0, 0, d[0], d[1], d[2], d[3], d[4], n, rounds, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  const double ns_round = 1e6 * ms / rounds;
  printf("%-34s blocks %4d  items/lane %d  %8.1f ns/round  %7.3f G item-rounds/s\n", name, blocks, NPT, ns_round,
         (double)n / ns_round);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int n_max = cus * 8192 * 2;
  std::vector<float> h[5];
  for (auto& v : h) v.resize(n_max);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xFFFF) / 65536.0f; };
  for (int i = 0; i < n_max; ++i) {
    const float x = 2.0f * rnd() - 1.0f, y = 1.5f * rnd() - 0.75f, z = 2.0f + 4.0f * rnd();
    h[0][i] = x; h[1][i] = y; h[2][i] = z;
    h[3][i] = 180.0f * x / z + 320.0f + (rnd() - 0.5f);
    h[4][i] = 180.0f * y / z + 240.0f + (rnd() - 0.5f);
    if (i % 10 < 3) h[3][i] += 300.0f;  // 30 % outliers
  }
  float* d[5];
  for (int k = 0; k < 5; ++k) {
    hipMalloc(&d[k], n_max * sizeof(float));
    hipMemcpy(d[k], h[k].data(), n_max * sizeof(float), hipMemcpyHostToDevice);
  }
  float* sink;
  hipMalloc(&sink, 1 << 20);
#if defined(PICP_ALLOW_PK)
  printf("build: packed FP32 allowed\n");
#else
  printf("build: no packed FP32 (shipped)\n");
#endif
  // one 512-thread block per CU, 4096 items per block (C3: 245 blocks x 4082)
  run<8, true, 512>("NPT 8, pairs, 512 thr, 1 blk/CU", d, 4096, cus, rounds, sink);
  run<8, false, 512>("NPT 8, one slot, 512 thr, 1 blk/CU", d, 4096, cus, rounds, sink);
  // the same items per CU as two blocks of NPT 4 (needs <= 128 VGPRs to be co-resident)
  run<4, true, 512>("NPT 4, pairs, 512 thr, 2 blk/CU", d, 4096, cus, rounds, sink);
  run<4, false, 512>("NPT 4, one slot, 512 thr, 2 blk/CU", d, 4096, cus, rounds, sink);
  run<2, false, 512>("NPT 2, one slot, 512 thr, 4 blk/CU", d, 4096, cus, rounds, sink);
  run<4, false, 1024>("NPT 4, one slot, 1024 thr, 1 blk/CU", d, 4096, cus, rounds, sink);
  hipDeviceSynchronize();
  return 0;
}
