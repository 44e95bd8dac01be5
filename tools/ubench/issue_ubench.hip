// Microbenchmark (diagnostic, not shipped): VALU issue rate of one SIMD on MI355X, to calibrate the
// bench line's FP32 vector roofline and issue fraction (VERDICT r04 "What's weak" 1).
//
// Every kernel is launched with 256-thread blocks (one wave on each of a CU's 4 SIMDs) and W
// blocks per CU (__launch_bounds__(256, W)), so up to W waves share every SIMD.  Each wave stamps
// s_memtime (shader cycles) and s_memrealtime (100 MHz) around its loop and records where it ran
// (HW_REG_XCC_ID, HW_REG_HW_ID).  Per SIMD, the span from its first wave's start to its last
// wave's end covers every instruction its waves issued, so
//     SIMD cycles per wave64 instruction = span / (waves on the SIMD x instructions per wave)
// (median over SIMDs), which holds however the dispatcher staggered or spread the waves; the
// per-wave form (median wave duration / (W x instructions)) is printed beside it, and the clock
// s_memtime counts at (its ticks / s_memrealtime's, x 100 MHz).
//   fma<W>   : 8 independent v_fma_f32 chains per lane (inline asm, 64 per iteration)
//   chain<W> : one dependent v_fma_f32 chain per lane
//   mix<NPT, PAIRS, W> : the block kernel's register-resident linearize (accumulate_regs /
//              accumulate_regs1 at the shipped pinhole variant) + wave reduction, NPT items per
//              lane, per round; its VALU instructions per wave come from a separate rocprofv3
//              --pmc SQ_INSTS_VALU SQ_WAVES pass over the same binary (tools/r05/gpu_issue.sh).
// build (the shipped device flags):
//   HIPCC=/opt/rocm/bin/hipcc 02-visualodometry_amd/hipcc_nopk.sh -O3 -std=c++17 --offload-arch=gfx950 \
//     -I02-visualodometry_amd/csrc -Iinclude tools/ubench/issue_ubench.hip -o tools/ubench/issue_ubench
// usage: issue_ubench [iters] [rounds]
#include <algorithm>
#include <cstdio>
#include <map>
#include <cstdlib>
#include <vector>

#include "picp_device.h"
using namespace picp;

#define FMA_ASM(a, b, c) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
// all three sources the destination register itself: no VGPR bank conflict whatever the allocation
#define FMA_SELF(a) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(a))

struct Stamp {
  unsigned long long t0, t1, r0, r1;  // s_memtime, s_memrealtime at loop start / end
  unsigned xcc, hwid;
};
#define STAMP_BEGIN()                                                   \
  const unsigned long long r0_ = __builtin_amdgcn_s_memrealtime();      \
  const unsigned long long t0_ = __builtin_amdgcn_s_memtime()
#define STAMP_END(st)                                                                          \
  do {                                                                                         \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                               \
    const unsigned long long r1_ = __builtin_amdgcn_s_memrealtime();                           \
    if ((threadIdx.x & 63) == 0) {                                                             \
      unsigned xcc_, hw_;                                                                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                        \
      st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = Stamp{t0_, t1_, r0_, r1_, xcc_, hw_}; \
    }                                                                                          \
  } while (0)

template <int W>
__global__ __launch_bounds__(256, W) void fma_stream(float* sink, Stamp* cyc, int iters, float x) {
  float a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  const float b = 1.0000001f, c = 1e-7f;
  STAMP_BEGIN();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      FMA_ASM(a0, b, c); FMA_ASM(a1, b, c); FMA_ASM(a2, b, c); FMA_ASM(a3, b, c);
      FMA_ASM(a4, b, c); FMA_ASM(a5, b, c); FMA_ASM(a6, b, c); FMA_ASM(a7, b, c);
    }
  }
  STAMP_END(cyc);
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int W>
__global__ __launch_bounds__(256, W) void fma_self(float* sink, Stamp* cyc, int iters, float x) {
  float a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  STAMP_BEGIN();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      FMA_SELF(a0); FMA_SELF(a1); FMA_SELF(a2); FMA_SELF(a3);
      FMA_SELF(a4); FMA_SELF(a5); FMA_SELF(a6); FMA_SELF(a7);
    }
  }
  STAMP_END(cyc);
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int W>
__global__ __launch_bounds__(256, W) void fma_chain(float* sink, Stamp* cyc, int iters, float x) {
  float a = x;
  const float b = 1.0000001f, c = 1e-7f;
  STAMP_BEGIN();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 64; ++k) FMA_ASM(a, b, c);
  }
  STAMP_END(cyc);
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// the block kernel's linearize alone: NPT register items per lane, `rounds` rounds at a slowly
// moving pose, each ending in the wave reduction and one LDS store per wave (no hand-off)
template <int NPT, bool PAIRS, int W>
__global__ __launch_bounds__(256, W) void mix(const float* __restrict__ X, const float* __restrict__ Y,
                                              const float* __restrict__ Z, const float* __restrict__ U,
                                              const float* __restrict__ V, int n, int rounds, float* sink,
                                              Stamp* cyc) {
  constexpr int BS = 256;
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
  STAMP_BEGIN();
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
  STAMP_END(cyc);
  if (tid == 0) sink[blockIdx.x] = check;
}

struct Span {
  double per_wave;   // median wave duration (cycles)
  double per_instr;  // median over SIMDs: span / (waves on it x instructions per wave)
  double waves_per_simd;  // mean waves a SIMD ran
  double clock_ghz;  // s_memtime ticks per s_memrealtime tick x 0.1
};

static Span analyse(Stamp* d, int waves, double instr_per_wave) {
  std::vector<Stamp> h(waves);
  hipMemcpy(h.data(), d, waves * sizeof(Stamp), hipMemcpyDeviceToHost);
  std::vector<double> dur, clk;
  std::map<unsigned long long, std::vector<int>> by_simd;
  for (int i = 0; i < waves; ++i) {
    dur.push_back((double)(h[i].t1 - h[i].t0));
    if (h[i].r1 > h[i].r0) clk.push_back(0.1 * (double)(h[i].t1 - h[i].t0) / (double)(h[i].r1 - h[i].r0));
    // HW_ID: simd 5:4, cu 11:8, sh 12, se 15:13 (the wave slot bits 3:0 dropped)
    const unsigned long long key = ((unsigned long long)h[i].xcc << 32) | ((h[i].hwid >> 4) & 0xFFFu);
    by_simd[key].push_back(i);
  }
  std::sort(dur.begin(), dur.end());
  std::sort(clk.begin(), clk.end());
  std::vector<double> per;
  double nw = 0;
  for (auto& kv : by_simd) {
    unsigned long long lo = ~0ull, hi = 0;
    for (int i : kv.second) {
      lo = std::min(lo, h[i].t0);
      hi = std::max(hi, h[i].t1);
    }
    per.push_back((double)(hi - lo) / ((double)kv.second.size() * instr_per_wave));
    nw += kv.second.size();
  }
  std::sort(per.begin(), per.end());
  return Span{dur[waves / 2], per[per.size() / 2], nw / by_simd.size(), clk.empty() ? 0.0 : clk[clk.size() / 2]};
}

// Dynamic LDS that lets exactly W blocks share a CU (160 KB of LDS per CU): the register budget
// alone would let more in, and the dispatcher would then spread the grid unevenly
static size_t lds_for(int W) { return (size_t)(163840 / W - 1024) / 256 * 256; }
template <typename F>
static void pin(F f, int W) {
  hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_for(W));
}

template <int W>
static void run_fma(int cus, int iters, float* sink, Stamp* cyc) {
  const int blocks = cus * W, waves = blocks * 4;
  const double ipw = 64.0 * iters;
  const size_t lds = lds_for(W);
  pin(fma_stream<W>, W);
  pin(fma_self<W>, W);
  pin(fma_chain<W>, W);
  hipLaunchKernelGGL((fma_stream<W>), dim3(blocks), dim3(256), lds, 0, sink, cyc, 4, 1.0f);  // warm
  hipLaunchKernelGGL((fma_stream<W>), dim3(blocks), dim3(256), lds, 0, sink, cyc, iters, 1.0f);
  hipDeviceSynchronize();
  Span s = analyse(cyc, waves, ipw);
  printf("fma_stream  W=%d  SIMD cycles per wave64 v_fma_f32: %6.3f (span, %.2f waves/SIMD)  %6.3f (per wave)  "
         "clock %.3f GHz\n", W, s.per_instr, s.waves_per_simd, s.per_wave / (W * ipw), s.clock_ghz);
  hipLaunchKernelGGL((fma_self<W>), dim3(blocks), dim3(256), lds, 0, sink, cyc, iters, 1.0f);
  hipDeviceSynchronize();
  s = analyse(cyc, waves, ipw);
  printf("fma_self    W=%d  SIMD cycles per wave64 v_fma_f32: %6.3f (span, %.2f waves/SIMD)  %6.3f (per wave)  "
         "clock %.3f GHz\n", W, s.per_instr, s.waves_per_simd, s.per_wave / (W * ipw), s.clock_ghz);
  hipLaunchKernelGGL((fma_chain<W>), dim3(blocks), dim3(256), lds, 0, sink, cyc, 4, 1.0f);
  hipLaunchKernelGGL((fma_chain<W>), dim3(blocks), dim3(256), lds, 0, sink, cyc, iters, 1.0f);
  hipDeviceSynchronize();
  s = analyse(cyc, waves, ipw);
  printf("fma_chain   W=%d  SIMD cycles per wave64 v_fma_f32: %6.3f (span, %.2f waves/SIMD)  %6.3f (per wave)  "
         "one wave's dependent step %.3f cycles  clock %.3f GHz\n", W, s.per_instr, s.waves_per_simd,
         s.per_wave / (W * ipw), s.per_wave / ipw, s.clock_ghz);
}

template <int NPT, bool PAIRS, int W>
static void run_mix(const char* name, float* const* dp, int cus, int rounds, float* sink, Stamp* cyc) {
  const int blocks = cus * W, waves = blocks * 4;
  const int n = blocks * NPT * 256;
  const size_t lds = lds_for(W);
  pin(mix<NPT, PAIRS, W>, W);
  hipLaunchKernelGGL((mix<NPT, PAIRS, W>), dim3(blocks), dim3(256), lds, 0, dp[0], dp[1], dp[2], dp[3], dp[4], n, 4,
                     sink, cyc);
  hipLaunchKernelGGL((mix<NPT, PAIRS, W>), dim3(blocks), dim3(256), lds, 0, dp[0], dp[1], dp[2], dp[3], dp[4], n,
                     rounds, sink, cyc);
  hipDeviceSynchronize();
  // span per item-round: instructions per wave = rounds x NPT x 64 "item-lanes"
  const Span s = analyse(cyc, waves, (double)rounds * NPT * 64);
  printf("mix %-14s W=%d  SIMD cycles per item-round: %6.3f (span, %.2f waves/SIMD)  %6.3f (per wave)  "
         "%8.1f cycles/round/wave  clock %.3f GHz\n", name, W, s.per_instr, s.waves_per_simd,
         s.per_wave / (W * 64.0 * NPT * rounds), s.per_wave / rounds, s.clock_ghz);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 2000;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* sink;
  Stamp* cyc;
  hipMalloc(&sink, (size_t)cus * 8 * 256 * sizeof(float));
  hipMalloc(&cyc, (size_t)cus * 8 * 4 * sizeof(Stamp));
  run_fma<1>(cus, iters, sink, cyc);
  run_fma<2>(cus, iters, sink, cyc);
  run_fma<4>(cus, iters, sink, cyc);
  run_fma<8>(cus, iters, sink, cyc);
  const int n_max = cus * 8 * 256 * 8 * 2;
  std::vector<float> h[5];
  for (auto& v : h) v.resize(n_max);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xFFFF) / 65536.0f; };
  for (int i = 0; i < n_max; ++i) {  // the C4 generator's statistics: all projectable, no outliers
    const float x = 2.0f * rnd() - 1.0f, y = 1.5f * rnd() - 0.75f, z = 2.0f + 4.0f * rnd();
    h[0][i] = x; h[1][i] = y; h[2][i] = z;
    h[3][i] = 180.0f * x / z + 320.0f + (rnd() - 0.5f);
    h[4][i] = 180.0f * y / z + 240.0f + (rnd() - 0.5f);
  }
  float* d[5];
  for (int k = 0; k < 5; ++k) {
    hipMalloc(&d[k], n_max * sizeof(float));
    hipMemcpy(d[k], h[k].data(), n_max * sizeof(float), hipMemcpyHostToDevice);
  }
  // C4 at 1,024 frames: NPT 8 pairs at 2 waves/SIMD; split 4 (128 frames): NPT 4 one slot at 4
  run_mix<8, true, 1>("NPT8 pairs", d, cus, rounds, sink, cyc);
  run_mix<8, true, 2>("NPT8 pairs", d, cus, rounds, sink, cyc);
  run_mix<4, false, 1>("NPT4 one-slot", d, cus, rounds, sink, cyc);
  run_mix<4, false, 2>("NPT4 one-slot", d, cus, rounds, sink, cyc);
  run_mix<4, false, 4>("NPT4 one-slot", d, cus, rounds, sink, cyc);
  run_mix<8, false, 2>("NPT8 one-slot", d, cus, rounds, sink, cyc);
  run_mix<8, false, 4>("NPT8 one-slot", d, cus, rounds, sink, cyc);
  run_mix<4, true, 4>("NPT4 pairs", d, cus, rounds, sink, cyc);
  run_mix<2, false, 4>("NPT2 one-slot", d, cus, rounds, sink, cyc);
  run_mix<2, false, 8>("NPT2 one-slot", d, cus, rounds, sink, cyc);
  hipDeviceSynchronize();
  return 0;
}
