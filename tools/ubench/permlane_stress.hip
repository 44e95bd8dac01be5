// permlane_stress.hip -- diagnostic (never shipped): do gfx950's cross-lane exchanges give the same
// bits whatever else runs on the CU?  A "victim" kernel repeats an exchange pattern on hashed lane
// data and checks every result against its analytic value (or against another exchange form of
// the same sums), while an "aggressor" kernel of a chosen kind is launched over and over on a
// second stream so that its waves share the victim's CUs and SIMDs.
//
//   victim 0: 16 v_permlane32_swap + 8 v_permlane16_swap (the reduction's pattern), every result
//             compared with the value the swap must deliver (integer data)
//   victim 1: wave_reduce32 (swap form, picp_device.h) vs wave_reduce32_bperm on the same floats
//   victim 2: the DPP row stages alone (row_mirror / row_half_mirror / quad_perm), vs ds_bpermute
//   victim 3: transcendental results: v_rcp_f32 / v_rsq_f32 of hashed operands (a new operand every
//             instruction) consumed by FMAs, each checked by its residual (|x*r - 1| <= 2^-21)
//   victim 4: register residency: 96 values per lane loaded once and held live (the block kernel's
//             register-resident items), re-checked every iteration while the wave runs FMA /
//             DPP / permlane / rcp work on other registers; ~150 VGPRs, like picp_block_kernel
//   victim 5: the block kernel's LDS hand-offs: lane 0 of wave 0 writes a 12-float "pose" that
//             changes every iteration, barrier, every lane of every wave reads it back with
//             16-B broadcast loads and checks it (the round-top pose read); then lanes 0-31 of
//             wave 0 write 32 "totals" and the whole wave reads them back at once (the finish's
//             read of s_tot); between them a wave_reduce32 (permlane swaps + DPP) on other data.
//             Mismatches are counted per 16-lane row (victim 6: the same, counts lanes 48-63 only)
//   victim 7: dependent v_rcp_f32 -> FMA chains as the compiler schedules them (the consumer right
//             after the producer's one required wait state), compared bit for bit with the same
//             chain whose every v_rcp_f32 is followed by 16 wait states (inline asm); mismatches
//             counted for lanes 0-47 in the low half of the counter and lanes 48-63 times 2^32
//   victim 8: the same with v_sqrt_f32 / v_rsq_f32 / v_exp_f32 / v_log_f32 producers
//   victim 9: apply_update (picp_device.h: Rx*Ry*Rz compose, packed-FP32 code) on inputs that are
//             the same in every lane: every lane must get lane 0's bits (lanes 0-47 / 48-63 counted
//             as in victim 7); victim 10: the same chain of packed FMAs (v_pk_fma_f32) alone
//   victims 11-16: one packed-FP32 instruction form each (inline asm, dependent chains, inputs the
//             same in every lane, lane agreement as victim 9): 11 v_pk_mul_f32 op_sel_hi:[1,0],
//             12 v_pk_mul_f32 op_sel:[1,1] op_sel_hi:[0,0], 13 v_pk_fma_f32 neg_lo/neg_hi on src2,
//             14 v_pk_fma_f32 op_sel:[0,0,1] op_sel_hi:[1,1,0], 15 v_pk_add_f32, 16 v_pk_fma_f32 plain
//   victims 17-22: a 32-bit VALU write of one half of a register pair, then a packed-FP32 read
//             of the pair after 0 / 1 / 2 wait states (inline asm, explicit v200-v205): 17/18/19
//             the high half written, 20/21/22 the low half written
//   victims 24-27: the form pk_bisect.py isolated (a packed add whose destination is its second
//             source with the halves crossed), its controls and a no-nop variant (inline asm)
//   aggressors: 0 none, 1 MFMA f16, 2 LDS traffic, 3 victim-0 itself, 4 FP32 FMA, 5 FP64 FMA,
//               6 DPP moves, 7 ds_bpermute, 8 v_permlane32_swap, 9 f32 transcendentals,
//               10 f64 transcendentals (v_rcp_f64 / v_sqrt_f64)
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I02-visualodometry_amd/csrc -Iinclude \
//        tools/ubench/permlane_stress.hip -o tools/ubench/permlane_stress
// usage: permlane_stress VICTIM AGGRESSOR [iters]   -> prints mismatches / checks
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "picp_device.h"

using namespace picp;

__device__ __forceinline__ unsigned mix(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// the data of lane L, slot I in iteration it of wave w
__device__ __forceinline__ unsigned val(unsigned w, unsigned it, int L, int I) {
  return mix((w * 0x9E3779B9u) ^ (it * 0x85EBCA6Bu) ^ ((unsigned)L << 8) ^ (unsigned)I);
}

template <int VICTIM>
__global__ __launch_bounds__(512) void victim(int iters, unsigned long long* bad, unsigned long long* checks) {
  const int lane = threadIdx.x & 63;
  const unsigned w = blockIdx.x * 8 + (threadIdx.x >> 6);
  unsigned long long nb = 0, nc = 0;
  for (int it = 0; it < iters; ++it) {
    if (VICTIM == 0) {
      unsigned v[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) v[i] = val(w, it, lane, i);
      // stage 1: v[i] <-> v[i+16] across the half-waves
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const auto r = __builtin_amdgcn_permlane32_swap(v[i], v[i + 16], false, false);
        const bool lo = lane < 32;
        const unsigned e0 = lo ? val(w, it, lane, i) : val(w, it, lane - 32, i + 16);
        const unsigned e1 = lo ? val(w, it, lane + 32, i) : val(w, it, lane, i + 16);
        nb += (r[0] != e0) + (r[1] != e1);
        v[i] = r[0] ^ (r[1] * 3u);
      }
      // stage 2: v[i] <-> v[i+8] across odd/even 16-lane rows
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(v[i], v[i + 8], false, false);
        // what v[i] / v[i+8] held in the partner lane after stage 1
        const int row_odd = (lane >> 4) & 1;
        const int pl = lane ^ 16;
        auto s1 = [&](int L, int I) {  // stage-1 result of lane L, slot I (< 16)
          const bool lo = L < 32;
          const unsigned a = lo ? val(w, it, L, I) : val(w, it, L - 32, I + 16);
          const unsigned b = lo ? val(w, it, L + 32, I) : val(w, it, L, I + 16);
          return a ^ (b * 3u);
        };
        const unsigned e0 = row_odd ? s1(pl, i + 8) : s1(lane, i);
        const unsigned e1 = row_odd ? s1(lane, i + 8) : s1(pl, i);
        nb += (r[0] != e0) + (r[1] != e1);
        v[i] = r[0] + r[1];
      }
      nc += 48;
    } else if (VICTIM == 1) {
      float a[PICP_NPART], b[PICP_NPART];
#pragma unroll
      for (int i = 0; i < PICP_NPART; ++i) {
        const float x = (float)(int)(val(w, it, lane, i) & 0xFFFFF) * 0.001953125f - 1024.0f;
        a[i] = x;
        b[i] = x;
      }
      const float r1 = wave_reduce32(a, lane);
      const float r2 = wave_reduce32_bperm(b, lane);
      nb += (__float_as_uint(r1) != __float_as_uint(r2));
      nc += 1;
    } else if (VICTIM == 5 || VICTIM == 6) {
      __shared__ __attribute__((aligned(16))) float s_pose[12];
      __shared__ float s_tot[32];
      if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < 12; ++i) s_pose[i] = __uint_as_float(val(w, it, 0, i) & 0x3FFFFFFFu);
      }
      __syncthreads();
      float pr[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) pr[i] = s_pose[i];
      unsigned bad_pose = 0;
#pragma unroll
      for (int i = 0; i < 12; ++i) bad_pose |= (__float_as_uint(pr[i]) != (val(w - (threadIdx.x >> 6), it, 0, i) & 0x3FFFFFFFu));
      // (w - wave: the writer was wave 0 of this block)
      float red[PICP_NPART];
#pragma unroll
      for (int i = 0; i < PICP_NPART; ++i) red[i] = pr[i % 12] * (float)(i + 1) + (float)lane;
      const float r = wave_reduce32(red, lane);
      unsigned bad_tot = 0;
      if ((threadIdx.x >> 6) == 0) {
        if (lane < 32) s_tot[lane] = r + (float)lane;
        __builtin_amdgcn_wave_barrier();
        float tw[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) tw[i] = s_tot[i];
        // every lane must see the same 32 words as lane 0 does
#pragma unroll
        for (int i = 0; i < 32; ++i)
          bad_tot |= (__float_as_uint(tw[i]) != (unsigned)__builtin_amdgcn_readfirstlane(__float_as_int(tw[i])));
      }
      const unsigned bad = (bad_pose | bad_tot) ? 1u : 0u;
      nb += (VICTIM == 5) ? bad : ((lane >= 48) ? bad : 0u);
      nc += 1;
      __syncthreads();
    } else if (VICTIM == 7 || VICTIM == 8) {
      float xf = 1.0f + (float)(val(w, it, lane, 0) & 0xFFFFF) * (1.0f / 1048576.0f);
      float xr = xf;
      // the chain as the compiler schedules it: producer, its one wait state, consumer
#pragma unroll 8
      for (int k = 0; k < 64; ++k) {
        float t;
        if (VICTIM == 7) t = __builtin_amdgcn_rcpf(xf);
        else if ((k & 3) == 0) t = __builtin_amdgcn_sqrtf(xf);
        else if ((k & 3) == 1) t = __builtin_amdgcn_rsqf(xf);
        else if ((k & 3) == 2) t = __builtin_amdgcn_exp2f(xf);
        else t = __builtin_amdgcn_logf(xf);
        xf = fmaf(t, 0.375f, 1.0f + 0.0625f * (float)(k & 7));  // back into [1, 2)
      }
      __builtin_amdgcn_sched_barrier(0);
      // the reference: 16 wait states between every producer and its consumer (inline asm)
#pragma unroll 8
      for (int k = 0; k < 64; ++k) {
        const float c = 1.0f + 0.0625f * (float)(k & 7);
        float t;
        if (VICTIM == 7 || (k & 3) == 0 || (k & 3) == 1) {
          if (VICTIM == 7)
            asm volatile("v_rcp_f32 %0, %1\n\ts_nop 7\n\ts_nop 7" : "=v"(t) : "v"(xr));
          else if ((k & 3) == 0)
            asm volatile("v_sqrt_f32 %0, %1\n\ts_nop 7\n\ts_nop 7" : "=v"(t) : "v"(xr));
          else
            asm volatile("v_rsq_f32 %0, %1\n\ts_nop 7\n\ts_nop 7" : "=v"(t) : "v"(xr));
        } else if ((k & 3) == 2) {
          asm volatile("v_exp_f32 %0, %1\n\ts_nop 7\n\ts_nop 7" : "=v"(t) : "v"(xr));
        } else {
          asm volatile("v_log_f32 %0, %1\n\ts_nop 7\n\ts_nop 7" : "=v"(t) : "v"(xr));
        }
        asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(xr) : "v"(t), "v"(0.375f), "v"(c));
      }
      const unsigned long long d = (__float_as_uint(xf) != __float_as_uint(xr)) ? 1ull : 0ull;
      nb += (lane >= 48) ? (d << 32) : d;
      nc += 64;
    } else if (VICTIM == 9) {
      float R[9], t[3], dx[6];
#pragma unroll
      for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0f : 1e-3f * (float)((int)(val(w, it, 0, i) & 63) - 32);
#pragma unroll
      for (int i = 0; i < 3; ++i) t[i] = 1e-2f * (float)((int)(val(w, it, 0, 9 + i) & 255) - 128);
#pragma unroll
      for (int i = 0; i < 6; ++i) dx[i] = 1e-5f * (float)((int)(val(w, it, 0, 12 + i) & 1023) - 512);
      for (int k = 0; k < 8; ++k) {
        apply_update(dx, R, t);
        dx[3] += 1e-7f * R[1];
      }
      bool mism = false;
#pragma unroll
      for (int i = 0; i < 9; ++i) mism |= __float_as_int(R[i]) != __builtin_amdgcn_readfirstlane(__float_as_int(R[i]));
#pragma unroll
      for (int i = 0; i < 3; ++i) mism |= __float_as_int(t[i]) != __builtin_amdgcn_readfirstlane(__float_as_int(t[i]));
      const unsigned long long d = mism ? 1ull : 0ull;
      nb += (lane >= 48) ? (d << 32) : d;
      nc += 8;
    } else if (VICTIM == 10) {
      typedef float f2v __attribute__((ext_vector_type(2)));
      f2v a = {1.0f + 1e-3f * (float)(val(w, it, 0, 0) & 255), 1.0f + 1e-3f * (float)(val(w, it, 0, 1) & 255)};
      f2v b = {0.999f, 1.001f}, c = {1e-3f, -1e-3f};
#pragma unroll 8
      for (int k = 0; k < 256; ++k) {
        a = __builtin_elementwise_fma(a, b, c);
        b = __builtin_elementwise_fma(b, a, c) * 0.5f;
        c = (f2v){c.y, c.x};
      }
      const bool mism = (__float_as_int(a.x) != __builtin_amdgcn_readfirstlane(__float_as_int(a.x))) |
                        (__float_as_int(a.y) != __builtin_amdgcn_readfirstlane(__float_as_int(a.y))) |
                        (__float_as_int(b.x) != __builtin_amdgcn_readfirstlane(__float_as_int(b.x)));
      const unsigned long long d = mism ? 1ull : 0ull;
      nb += (lane >= 48) ? (d << 32) : d;
      nc += 256;
    } else if (VICTIM >= 11 && VICTIM <= 16) {
      typedef float f2v __attribute__((ext_vector_type(2)));
      f2v a = {1.0f + 1e-3f * (float)(val(w, it, 0, 0) & 255), 1.0f - 1e-3f * (float)(val(w, it, 0, 1) & 255)};
      f2v b = {0.75f, 1.25f}, c = {1e-3f, -2e-3f}, r;
#pragma unroll 4
      for (int k = 0; k < 64; ++k) {
        if (VICTIM == 11) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
        else if (VICTIM == 12) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0]" : "=v"(r) : "v"(a), "v"(b));
        else if (VICTIM == 13) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[0,0,1] neg_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
        else if (VICTIM == 14) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
        else if (VICTIM == 15) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
        else asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
        // renormalise into [0.5, 2) with plain VALU (the next producer's operands written right before it)
        a = (f2v){r.x * 0.5f + 0.75f, r.y * 0.5f + 0.5f};
      }
      const bool mism = (__float_as_int(a.x) != __builtin_amdgcn_readfirstlane(__float_as_int(a.x))) |
                        (__float_as_int(a.y) != __builtin_amdgcn_readfirstlane(__float_as_int(a.y)));
      const unsigned long long d = mism ? 1ull : 0ull;
      nb += (lane >= 48) ? (d << 32) : d;
      nc += 64;
    } else if (VICTIM >= 17 && VICTIM <= 22) {
      float x = 1.0f + 1e-3f * (float)(val(w, it, 0, 0) & 255), y = 1.0f - 1e-3f * (float)(val(w, it, 0, 1) & 255);
      float rl = 0.0f, rh = 0.0f;
#define PK_SEQ(WRITE, NOPS)                                                                           \
  asm volatile("v_mov_b32 v200, %2\n\tv_mov_b32 v201, %3\n\tv_mov_b32 v202, 0x3f400000\n\t"             \
               "v_mov_b32 v203, 0x3fa00000\n\ts_nop 7\n\t" WRITE NOPS                                    \
               "v_pk_mul_f32 v[204:205], v[200:201], v[202:203]\n\ts_nop 7\n\t"                          \
               "v_mov_b32 %0, v204\n\tv_mov_b32 %1, v205"                                                \
               : "=v"(rl), "=v"(rh) : "v"(x), "v"(y) : "v200", "v201", "v202", "v203", "v204", "v205")
#pragma unroll 2
      for (int k = 0; k < 64; ++k) {
        if (VICTIM == 17) PK_SEQ("v_add_f32 v203, 0x3fa00000, v200\n\t", "");
        else if (VICTIM == 18) PK_SEQ("v_add_f32 v203, 0x3fa00000, v200\n\t", "s_nop 0\n\t");
        else if (VICTIM == 19) PK_SEQ("v_add_f32 v203, 0x3fa00000, v200\n\t", "s_nop 1\n\t");
        else if (VICTIM == 20) PK_SEQ("v_add_f32 v202, 0x3f400000, v201\n\t", "");
        else if (VICTIM == 21) PK_SEQ("v_add_f32 v202, 0x3f400000, v201\n\t", "s_nop 0\n\t");
        else PK_SEQ("v_add_f32 v202, 0x3f400000, v201\n\t", "s_nop 1\n\t");
        x = rl * 0.25f + 0.75f;
        y = rh * 0.25f + 0.5f;
      }
#undef PK_SEQ
      const bool mism = (__float_as_int(x) != __builtin_amdgcn_readfirstlane(__float_as_int(x))) |
                        (__float_as_int(y) != __builtin_amdgcn_readfirstlane(__float_as_int(y)));
      const unsigned long long d = mism ? 1ull : 0ull;
      nb += (lane >= 48) ? (d << 32) : d;
      nc += 64;
    } else if (VICTIM >= 24 && VICTIM <= 27) {
      // the instruction tools/ubench/pk_bisect.py isolated in victim 9: a packed add whose
      // destination pair is its second source with the halves crossed (lo = a.lo + b.hi,
      // hi = a.hi + b.lo, b = the destination); 25: the same op into a separate pair; 26: the
      // destination as the second source without crossing; 27: as 24 with no s_nop before it
      float x = 1.0f + 1e-3f * (float)(val(w, it, 0, 0) & 255), y = 1.0f - 1e-3f * (float)(val(w, it, 0, 1) & 255);
      float rl = 0.0f, rh = 0.0f;
#define PK_X(PRE, OP)                                                                                 \
  asm volatile("v_mov_b32 v200, %2\n\tv_mov_b32 v201, %3\n\tv_mov_b32 v202, 0x3f400000\n\t"           \
               "v_mov_b32 v203, 0x3fa00000\n\t" PRE OP "\n\ts_nop 7\n\t"                                \
               "v_mov_b32 %0, v200\n\tv_mov_b32 %1, v201"                                              \
               : "=v"(rl), "=v"(rh) : "v"(x), "v"(y) : "v200", "v201", "v202", "v203", "v204", "v205")
#pragma unroll 2
      for (int k = 0; k < 64; ++k) {
        if (VICTIM == 24) PK_X("s_nop 7\n\t", "v_pk_add_f32 v[200:201], v[202:203], v[200:201] op_sel:[0,1] op_sel_hi:[1,0]");
        else if (VICTIM == 25)
          PK_X("s_nop 7\n\t", "v_pk_add_f32 v[204:205], v[202:203], v[200:201] op_sel:[0,1] op_sel_hi:[1,0]\n\t"
                               "s_nop 7\n\tv_mov_b32 v200, v204\n\tv_mov_b32 v201, v205");
        else if (VICTIM == 26) PK_X("s_nop 7\n\t", "v_pk_add_f32 v[200:201], v[202:203], v[200:201]");
        else PK_X("", "v_pk_add_f32 v[200:201], v[202:203], v[200:201] op_sel:[0,1] op_sel_hi:[1,0]");
        x = rl * 0.25f + 0.75f;
        y = rh * 0.25f + 0.5f;
      }
#undef PK_X
      const bool mism = (__float_as_int(x) != __builtin_amdgcn_readfirstlane(__float_as_int(x))) |
                        (__float_as_int(y) != __builtin_amdgcn_readfirstlane(__float_as_int(y)));
      const unsigned long long d = mism ? 1ull : 0ull;
      nb += (lane >= 48) ? (d << 32) : d;
      nc += 64;
    } else if (VICTIM == 4) {
      // (the loop below runs the whole test once; `it` stays 0 here)
      unsigned hold[96];
#pragma unroll
      for (int i = 0; i < 96; ++i) {
        hold[i] = val(w, 7u, lane, i);
        asm volatile("" : "+v"(hold[i]));  // opaque: held in a VGPR, never recomputed
      }
      float acc[24];
#pragma unroll
      for (int i = 0; i < 24; ++i) acc[i] = (float)i;
      for (int k = 0; k < iters; ++k) {
#pragma unroll
        for (int i = 0; i < 24; ++i) {
          acc[i] = fmaf(acc[i], 0.999f, __builtin_amdgcn_rcpf(acc[i] + 3.0f));
          acc[i] += dpp<DPP_ROW_MIRROR>(acc[i]) * 0.001f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i]), __float_as_uint(acc[i + 8]), false, false);
          acc[i] = __uint_as_float(r[0]) * 0.5f + __uint_as_float(r[1]) * 0.5f;
        }
        unsigned bad_here = 0;
        unsigned z = 0;
        asm volatile("" : "+s"(z));  // opaque 0: the expected values are recomputed, not held
#pragma unroll
        for (int i = 0; i < 96; ++i) {
          asm volatile("" : "+v"(hold[i]));  // re-read the register every iteration
          bad_here += (hold[i] != val(w, 7u + z, lane, i));
        }
        nb += bad_here;
        nc += 96;
        if (bad_here && lane >= 0) nb += 0;  // (kept simple: counts only)
        __builtin_amdgcn_s_sleep(1);
      }
      if (acc[0] == 1234.5f) nb += 1000000;  // keep acc alive
      break;
    } else if (VICTIM == 3) {
      // 8 independent operands per iteration, each far from the previous one (a result taken from
      // another operand or an older instruction fails its residual)
      float x[8], r[8], q[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = 1.0f + (float)(val(w, it, lane, i) & 0xFFFFF) * (1.0f / 8192.0f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        r[i] = __builtin_amdgcn_rcpf(x[i]);
        q[i] = __builtin_amdgcn_rsqf(x[i]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float e1 = fabsf(fmaf(x[i], r[i], -1.0f));
        const float e2 = fabsf(fmaf(x[i] * q[i], q[i], -1.0f));
        nb += (e1 > 4.8e-7f) + (e2 > 1e-6f);
      }
      nc += 16;
    } else {
      float a[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = (float)(int)(val(w, it, lane, i) & 0xFFFF) * 0.25f;
      float c[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = a[i];
      bfly_dpp<DPP_ROW_MIRROR, 3, 4>(a, lane);
      bfly_dpp<DPP_ROW_HALF_MIRROR, 2, 2>(a, lane);
      bfly_dpp<DPP_QUAD_XOR2, 1, 1>(a, lane);
      const float r1 = a[0] + dpp<DPP_QUAD_XOR1>(a[0]);
      // the same butterflies through ds_bpermute (partner lanes of the DPP controls)
      auto sh = [&](float x, int partner) { return __shfl(x, partner); };
      {
        const bool hi = (lane >> 3) & 1;
        const int p = (lane & ~15) | (15 - (lane & 15));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float send = hi ? c[i] : c[i + 4], keep = hi ? c[i + 4] : c[i];
          c[i] = keep + sh(send, p);
        }
      }
      {
        const bool hi = (lane >> 2) & 1;
        const int p = (lane & ~7) | (7 - (lane & 7));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float send = hi ? c[i] : c[i + 2], keep = hi ? c[i + 2] : c[i];
          c[i] = keep + sh(send, p);
        }
      }
      {
        const bool hi = (lane >> 1) & 1;
        const int p = lane ^ 2;
        const float send = hi ? c[0] : c[1], keep = hi ? c[1] : c[0];
        c[0] = keep + sh(send, p);
      }
      const float r2 = c[0] + sh(c[0], lane ^ 1);
      nb += (__float_as_uint(r1) != __float_as_uint(r2));
      nc += 1;
    }
  }
  // one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    nb += __shfl_xor(nb, o);
    nc += __shfl_xor(nc, o);
  }
  if (lane == 0) {
    atomicAdd(bad, nb);
    atomicAdd(checks, nc);
  }
}

// victim 23: victim 9 (apply_update, lane agreement) in a kernel compiled without packed FP32
__global__ __launch_bounds__(512) __attribute__((target("no-packed-fp32-ops"))) void victim_nopk(
    int iters, unsigned long long* bad, unsigned long long* checks) {
  const int lane = threadIdx.x & 63;
  const unsigned w = blockIdx.x * 8 + (threadIdx.x >> 6);
  unsigned long long nb = 0, nc = 0;
  for (int it = 0; it < iters; ++it) {
    float R[9], t[3], dx[6];
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0f : 1e-3f * (float)((int)(val(w, it, 0, i) & 63) - 32);
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] = 1e-2f * (float)((int)(val(w, it, 0, 9 + i) & 255) - 128);
#pragma unroll
    for (int i = 0; i < 6; ++i) dx[i] = 1e-5f * (float)((int)(val(w, it, 0, 12 + i) & 1023) - 512);
    for (int k = 0; k < 8; ++k) {
      apply_update(dx, R, t);
      dx[3] += 1e-7f * R[1];
    }
    bool mism = false;
#pragma unroll
    for (int i = 0; i < 9; ++i) mism |= __float_as_int(R[i]) != __builtin_amdgcn_readfirstlane(__float_as_int(R[i]));
#pragma unroll
    for (int i = 0; i < 3; ++i) mism |= __float_as_int(t[i]) != __builtin_amdgcn_readfirstlane(__float_as_int(t[i]));
    const unsigned long long d = mism ? 1ull : 0ull;
    nb += (lane >= 48) ? (d << 32) : d;
    nc += 8;
  }
  for (int o = 32; o > 0; o >>= 1) {
    nb += __shfl_xor(nb, o);
    nc += __shfl_xor(nc, o);
  }
  if (lane == 0) {
    atomicAdd(bad, nb);
    atomicAdd(checks, nc);
  }
}

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ __launch_bounds__(256) void aggressor(int iters, float* sink) {
  const int lane = threadIdx.x & 63;
  __shared__ float lds[4096];
  float acc = (float)lane;
  double dacc = (double)lane;
  if (KIND == 1) {
    half8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = (_Float16)(lane * 0.01f + i);
      b[i] = (_Float16)(i * 0.5f);
    }
    float16v c = {};
    for (int it = 0; it < iters; ++it) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    acc = c[0] + c[15];
  } else if (KIND == 2) {
    for (int it = 0; it < iters; ++it) {
      lds[(threadIdx.x * 17 + it) & 4095] = acc;
      __syncthreads();
      acc += lds[(threadIdx.x * 13 + it * 7) & 4095];
    }
  } else if (KIND == 4) {
    float x = acc, y = 1.0001f, z = 0.5f;
    for (int it = 0; it < iters; ++it) {
      x = fmaf(x, y, z);
      y = fmaf(y, z, x);
      z = fmaf(z, x, y);
    }
    acc = x + y + z;
  } else if (KIND == 5) {
    double x = dacc, y = 1.0001, z = 0.5;
    for (int it = 0; it < iters; ++it) {
      x = fma(x, y, z);
      y = fma(y, z, x);
      z = fma(z, x, y);
    }
    acc = (float)(x + y + z);
  } else if (KIND == 6) {
    for (int it = 0; it < iters; ++it) acc = acc * 0.5f + dpp<DPP_ROW_MIRROR>(acc);
  } else if (KIND == 7) {
    for (int it = 0; it < iters; ++it) acc = acc * 0.5f + __shfl_xor(acc, 32);
  } else if (KIND == 9) {
    float x = 1.5f + lane;
    for (int it = 0; it < iters; ++it) {
      x = __builtin_amdgcn_rcpf(x) + __builtin_amdgcn_rsqf(x + 1.0f) + __builtin_amdgcn_sqrtf(x + 2.0f) + 1.0f;
    }
    acc = x;
  } else if (KIND == 10) {
    double x = 1.5 + lane;
    for (int it = 0; it < iters; ++it) x = 1.0 / x + sqrt(x + 2.0) + 1.0;
    acc = (float)x;
  } else if (KIND == 8) {
    unsigned a = lane, b = lane * 7u;
    for (int it = 0; it < iters; ++it) {
      const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
      a = r[0] + 1u;
      b = r[1] ^ a;
    }
    acc = (float)(a ^ b);
  }
  if (acc == 1234.5678f) sink[0] = acc;  // keep the work alive
}

static void launch_aggr(int kind, hipStream_t s, float* sink) {
  const dim3 g(2048), b(256);
  switch (kind) {
    case 1: hipLaunchKernelGGL(aggressor<1>, g, b, 0, s, 2000, sink); break;
    case 2: hipLaunchKernelGGL(aggressor<2>, g, b, 0, s, 2000, sink); break;
    case 3: {
      static unsigned long long* d = nullptr;
      if (!d) hipMalloc(&d, 16);
      hipLaunchKernelGGL(victim<0>, dim3(512), dim3(512), 0, s, 20, d, d + 1);
      break;
    }
    case 4: hipLaunchKernelGGL(aggressor<4>, g, b, 0, s, 4000, sink); break;
    case 5: hipLaunchKernelGGL(aggressor<5>, g, b, 0, s, 2000, sink); break;
    case 6: hipLaunchKernelGGL(aggressor<6>, g, b, 0, s, 4000, sink); break;
    case 7: hipLaunchKernelGGL(aggressor<7>, g, b, 0, s, 2000, sink); break;
    case 8: hipLaunchKernelGGL(aggressor<8>, g, b, 0, s, 4000, sink); break;
    case 9: hipLaunchKernelGGL(aggressor<9>, g, b, 0, s, 2000, sink); break;
    case 10: hipLaunchKernelGGL(aggressor<10>, g, b, 0, s, 500, sink); break;
    default: break;
  }
}

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

#ifndef STRESS_LIB
int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s VICTIM(0-3) AGGRESSOR(0-10) [iters]\n", argv[0]);
    return 2;
  }
  const int vk = atoi(argv[1]), ak = atoi(argv[2]);
  const int iters = argc > 3 ? atoi(argv[3]) : 2000;
  unsigned long long* d = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&d, 16));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(d, 0, 16));
  hipStream_t sv, sa;
  CK(hipStreamCreateWithFlags(&sv, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  hipEvent_t done;
  CK(hipEventCreate(&done));
  // aggressors first, so that the victim's blocks land among theirs
  for (int k = 0; k < 4; ++k) launch_aggr(ak, sa, sink);
  const dim3 vg(256), vb(512);
  if (vk == 0) hipLaunchKernelGGL(victim<0>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 1) hipLaunchKernelGGL(victim<1>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 3) hipLaunchKernelGGL(victim<3>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 4) hipLaunchKernelGGL(victim<4>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 5) hipLaunchKernelGGL(victim<5>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 6) hipLaunchKernelGGL(victim<6>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 7) hipLaunchKernelGGL(victim<7>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 8) hipLaunchKernelGGL(victim<8>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 9) hipLaunchKernelGGL(victim<9>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 10) hipLaunchKernelGGL(victim<10>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 11) hipLaunchKernelGGL(victim<11>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 12) hipLaunchKernelGGL(victim<12>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 13) hipLaunchKernelGGL(victim<13>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 14) hipLaunchKernelGGL(victim<14>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 15) hipLaunchKernelGGL(victim<15>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 16) hipLaunchKernelGGL(victim<16>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 23) hipLaunchKernelGGL(victim_nopk, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 17) hipLaunchKernelGGL(victim<17>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 18) hipLaunchKernelGGL(victim<18>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 19) hipLaunchKernelGGL(victim<19>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 20) hipLaunchKernelGGL(victim<20>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 21) hipLaunchKernelGGL(victim<21>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 22) hipLaunchKernelGGL(victim<22>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 24) hipLaunchKernelGGL(victim<24>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 25) hipLaunchKernelGGL(victim<25>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 26) hipLaunchKernelGGL(victim<26>, vg, vb, 0, sv, iters, d, d + 1);
  else if (vk == 27) hipLaunchKernelGGL(victim<27>, vg, vb, 0, sv, iters, d, d + 1);
  else hipLaunchKernelGGL(victim<2>, vg, vb, 0, sv, iters, d, d + 1);
  CK(hipGetLastError());
  CK(hipEventRecord(done, sv));
  int n_aggr = 4;
  while (hipEventQuery(done) == hipErrorNotReady && n_aggr < 20000) {
    launch_aggr(ak, sa, sink);
    ++n_aggr;
    if (n_aggr % 8 == 0) hipStreamSynchronize(sa);  // keep the queue short
  }
  CK(hipDeviceSynchronize());
  unsigned long long h[2];
  CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
  if (vk >= 7)
    printf("victim %d aggressor %d: %llu mismatches in lanes 0-47, %llu in lanes 48-63, %llu chain steps (%d aggressor launches)\n",
           vk, ak, h[0] & 0xFFFFFFFFull, h[0] >> 32, h[1], ak ? n_aggr : 0);
  else
    printf("victim %d aggressor %d: %llu mismatches in %llu checks (%d aggressor launches)\n", vk, ak, h[0], h[1],
           ak ? n_aggr : 0);
  return 0;
}

#endif  // STRESS_LIB

// ---- library form (tools/vo_stress.py): the victims launched on a caller's stream ----
extern "C" int stress_launch(int vk, int blocks, int iters, void* stream, unsigned long long* d_counts) {
  const dim3 vg(blocks), vb(512);
  hipStream_t s = (hipStream_t)stream;
  if (vk == 0) hipLaunchKernelGGL(victim<0>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 1) hipLaunchKernelGGL(victim<1>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 3) hipLaunchKernelGGL(victim<3>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 4) hipLaunchKernelGGL(victim<4>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 5) hipLaunchKernelGGL(victim<5>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 6) hipLaunchKernelGGL(victim<6>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 7) hipLaunchKernelGGL(victim<7>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 8) hipLaunchKernelGGL(victim<8>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 9) hipLaunchKernelGGL(victim<9>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else if (vk == 10) hipLaunchKernelGGL(victim<10>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  else hipLaunchKernelGGL(victim<2>, vg, vb, 0, s, iters, d_counts, d_counts + 1);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
