// Microbenchmark (diagnostic, not shipped): cycles of the pieces of finish_round_f on one wave.
#include <cstdio>
#include <vector>
#include "picp_device.h"
using namespace picp;

// ---- experimental finish variants (round 3); not in the product ----
namespace picp {
// The damped 6x6 solve with a short dependency chain (the one-lane form is latency-bound: a
// single wave's dependent VALU ops issue ~8 cycles apart, v_rcp_f32 ~20).  Same elimination as
// ldl6_solve, regrouped so the reciprocal is the only thing each step waits for:
//   forward: a[i][c] -= (a[i][j] a[c][j]) / d_j, rhs[i] -= (a[i][j] rhs[j]) / d_j -- the products
//            are formed while v_rcp_f32(d_j) is in flight, then ONE fma per entry;
//   back:    y_i = rhs_i / d_i and u[k][i] = a[k][i] / d_i formed off the chain, then
//            x_k = y_k, y_i -= u[k][i] x_k -- one fma per step.
// The chain is 2 ops per pivot + 1 per back step (18) instead of 3 + 2 (30).  Rounding differs
// from ldl6_solve in the last bits (a product of two entries before the scale, not after); the
// per-round pose stays within the oracle tolerance (tests/test_gpu_parity.py).
template <bool GUARD>
__device__ __forceinline__ bool ldl6_solve_short(const float* tw, float dx[6]) {
  float a[6][6], rhs[6], id[6];
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int c = 0; c <= i; ++c) a[i][c] = tw[tri_index(c, i)];
    rhs[i] = tw[PICP_P_B + i];
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const float d = a[j][j];
    float inv = __builtin_amdgcn_rcpf(d);
    if (GUARD) inv = (fabsf(d) > FLT_MIN) ? inv : 0.0f;
    else bad |= !(fabsf(d) > FLT_MIN);
    id[j] = inv;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
#pragma unroll
      for (int c = j + 1; c <= i; ++c) a[i][c] = fmaf(-(a[i][j] * a[c][j]), inv, a[i][c]);
      rhs[i] = fmaf(-(a[i][j] * rhs[j]), inv, rhs[i]);
    }
  }
  float y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) y[i] = rhs[i] * id[i];
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const float x = y[k];
    dx[k] = x;
#pragma unroll
    for (int i = 0; i < k; ++i) y[i] = fmaf(-(a[k][i] * id[i]), x, y[i]);
  }
  return bad;
}

__device__ __forceinline__ void ldl6_solve_short(const float* tw, float dx[6]) {
  if (ldl6_solve_short<false>(tw, dx)) ldl6_solve_short<true>(tw, dx);
}

// apply_update for ONE element of the new pose: e in 0..11 of [R column-major | t] (lanes of a
// finishing wave take e = lane & 15, e >= 12 clamped: those lanes publish nothing).  The element's
// products and sums are apply_update's own, in its order, so the value is bit-identical to
// apply_update's R[e] / t[e - 9]; the row of Rd and the column of R it reads are picked by
// per-lane selects.  One third of apply_update's compose per lane, and the pose leaves the finish
// already spread one word per lane, as the publish stores it.
__device__ __forceinline__ float apply_update_elem(const float dx[6], const float R[9], const float t[3], int e) {
  float Rd[3][3];
  update_rotation(dx, Rd);
  e = e < 11 ? e : 11;
  const int j = e / 3, i = e - 3 * j;  // column j of the new pose (3: t), row i
  const float d0 = (i == 0) ? Rd[0][0] : ((i == 1) ? Rd[1][0] : Rd[2][0]);
  const float d1 = (i == 0) ? Rd[0][1] : ((i == 1) ? Rd[1][1] : Rd[2][1]);
  const float d2 = (i == 0) ? Rd[0][2] : ((i == 1) ? Rd[1][2] : Rd[2][2]);
  const float c0 = (j == 0) ? R[0] : ((j == 1) ? R[3] : ((j == 2) ? R[6] : t[0]));
  const float c1 = (j == 0) ? R[1] : ((j == 1) ? R[4] : ((j == 2) ? R[7] : t[1]));
  const float c2 = (j == 0) ? R[2] : ((j == 1) ? R[5] : ((j == 2) ? R[8] : t[2]));
  float s = d0 * c0;
  s = s + d1 * c1;
  s = s + d2 * c2;
  const float di = (i == 0) ? dx[0] : ((i == 1) ? dx[1] : dx[2]);
  return (j == 3) ? s + di : s;
}

// Pose element e (0..11) of [R column-major | t] (e >= 12 clamped to 11).
__device__ __forceinline__ float pose_elem(const float R[9], const float t[3], int e) {
  float w = t[2];
#pragma unroll
  for (int i = 0; i < 9; ++i) w = (e == i) ? R[i] : w;
#pragma unroll
  for (int i = 0; i < 2; ++i) w = (e == 9 + i) ? t[i] : w;
  return w;
}

// finish_round_pose for a whole wave (every lane active) that publishes the pose one word per
// lane: the elimination spread over each 16-lane row (ldl6_solve_wave) and the update of one
// element per lane (apply_update_elem, e = lane & 15).  Bit-identical to finish_round_pose's
// R / t entry e.  R / t: the round's pose (uniform; not updated); returns the new element e.
__device__ __forceinline__ float finish_round_elem(const PicpArgs& A, const float* tw, int j, const float R[9],
                                                   const float t[3], float& chi_prev, RoundOut& o, int e) {
  o.chi_in = tw[PICP_P_CHI_IN];
  o.chi_out = tw[PICP_P_CHI_OUT];
  o.n_in = __float_as_int(tw[PICP_P_N_IN]);
  o.n_proj = __float_as_int(tw[PICP_P_N_PROJ]);
  o.converged = 0;
  if (o.n_in < A.min_inliers) {  // src/picp_solver.cpp:97-100
    o.ok = 0;
    o.done = 1;
    return pose_elem(R, t, e);
  }
  float dx[6];
  ldl6_solve_wave(tw, dx);                       // :96, :102
  const float w = apply_update_elem(dx, R, t, e);  // :103
  o.ok = 1;
  o.done = 0;
  const float prev = chi_prev, cur = o.chi_in;  // exec/icp_test.cpp:99-106
  const float rel = (prev > 1e-10f) ? fabsf(prev - cur) / prev : 0.0f;
  if (rel < A.conv_eps) {
    o.converged = 1;
    o.done = 1;
  } else {
    chi_prev = cur;
  }
  if (j >= A.max_rounds) o.done = 1;
  return w;
}

}  // namespace picp

// MODE 0: finish_round_pose (tw in LDS, loop state in registers), 1: ldl6_solve (tw in LDS),
//      2: apply_update (registers), 3: LDS state copy (s_st -> ns -> s_st), 4: empty loop,
//      5: ldl6_solve_wave (tw in LDS, the elimination over a row's lanes),
//      6: ldl6_solve_short (tw in LDS, the short-chain regrouping),
//      7: the shipped finish + lane 0 storing the 12 pose words to LDS (block kernel),
//      8: finish_round_elem (pose read from LDS, wave solve, one element per lane, lanes 0-11 store)
template <int MODE>
__global__ void bench(PicpArgs A, const float* tot0, int iters, unsigned long long* cyc, float* out) {
  __shared__ float s_tot[PICP_NPART];
  __shared__ PicpState s_st;
  __shared__ float s_pose[12];
  const int lane = threadIdx.x;
  if (lane < PICP_NPART) s_tot[lane] = tot0[lane];
  if (lane < 12) s_pose[lane] = (lane % 4 == 0 && lane < 9) ? 1.0f : 0.0f;
  if (lane == 0) {
    PicpState s{};
    for (int i = 0; i < 9; ++i) s.R[i] = (i % 4 == 0) ? 1.0f : 0.0f;
    s_st = s;
  }
  __syncthreads();
  float R[9], t[3] = {0, 0, 0}, dx[6] = {1e-4f, 2e-4f, 3e-4f, 1e-5f, 2e-5f, 3e-5f};
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0f : 0.0f;
  float acc = 0.0f, chi_prev = 1e30f;
  // the loop-carried LDS word's base value, loaded once: a global load inside the timed loop
  // would put an L2 round trip on every iteration (the round-2 figures included one)
  const float b0 = tot0[PICP_P_B];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {  // the whole finish as the kernels run it (pose + chi_prev in registers)
      RoundOut o;
      finish_round_pose(A, s_tot, it + 1, R, t, chi_prev, o);
      if (lane == 0) s_tot[PICP_P_B] = b0 + R[1] * 1e-30f;  // loop-carried
    } else if (MODE == 1) {
      ldl6_solve(s_tot, dx);
      if (lane == 0) s_tot[PICP_P_B] = b0 + dx[5] * 1e-30f;
    } else if (MODE == 5) {
      ldl6_solve_wave(s_tot, dx);
      if (lane == 0) s_tot[PICP_P_B] = b0 + dx[5] * 1e-30f;
    } else if (MODE == 6) {
      ldl6_solve_short(s_tot, dx);
      if (lane == 0) s_tot[PICP_P_B] = b0 + dx[5] * 1e-30f;
    } else if (MODE == 7) {
      RoundOut o;
      finish_round_pose(A, s_tot, it + 1, R, t, chi_prev, o);
      if (lane == 0) {
        for (int i = 0; i < 9; ++i) s_pose[i] = R[i];
        for (int i = 0; i < 3; ++i) s_pose[9 + i] = t[i];
        s_tot[PICP_P_B] = b0 + R[1] * 1e-30f;
      }
    } else if (MODE == 8) {
      float Rr[9], tr[3];
      for (int i = 0; i < 9; ++i) Rr[i] = s_pose[i];
      for (int i = 0; i < 3; ++i) tr[i] = s_pose[9 + i];
      RoundOut o;
      const float w = finish_round_elem(A, s_tot, it + 1, Rr, tr, chi_prev, o, lane & 15);
      if (lane < 12) s_pose[lane] = w;
      if (lane == 1) s_tot[PICP_P_B] = b0 + w * 1e-30f;
    } else if (MODE == 2) {
      apply_update(dx, R, t);
      dx[3] = R[1] * 1e-3f;
    } else if (MODE == 3) {
      PicpState ns;
      const PicpState& s = s_st;
      for (int i = 0; i < 9; ++i) ns.R[i] = s.R[i];
      for (int i = 0; i < 3; ++i) ns.t[i] = s.t[i];
      ns.chi_prev = s.chi_prev; ns.done = s.done; ns.ok = s.ok; ns.converged = s.converged;
      for (int i = 0; i < 11; ++i) ns.pad[i] = 0;
      ns.chi_in = s_tot[27]; ns.chi_out = s_tot[28]; ns.n_in = it; ns.n_proj = it; ns.rounds = it;
      ns.R[0] += 1e-30f;
      if (lane == 0) s_st = ns;
    }
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  acc = dx[0] + dx[5] + R[0] + t[0] + s_st.R[0];
  if (lane == 0) { cyc[MODE] = (t1 - t0) / iters; out[MODE] = acc; }
}

// ldl6_solve vs ldl6_solve_wave on the same systems: every lane's dx must equal the one-lane
// solve's bits.  System v: the main() system with entry (v % 21) scaled by 1 + v * 1e-3 and b
// perturbed; v >= 60: a zero pivot (row/col 3 zeroed) for the guarded path.
__global__ void check(const float* tot0, int nsys, unsigned* bad, float* maxrel) {
  __shared__ float s_tot[PICP_NPART];
  const int lane = threadIdx.x;
  for (int v = 0; v < nsys; ++v) {
    if (lane < PICP_NPART) {
      float x = tot0[lane];
      if (lane == (v % 21)) x *= 1.0f + 1e-3f * (float)v;
      if (lane >= PICP_P_B && lane < PICP_P_B + 6) x += 1e-4f * (float)((v * 7 + lane) % 13);
      if (v >= 60 && lane < 21) {  // zero row/column 3: a zero pivot
        const int rr[21] = {0,0,0,0,0,0,1,1,1,1,1,2,2,2,2,3,3,3,4,4,5};
        const int cc[21] = {0,1,2,3,4,5,1,2,3,4,5,2,3,4,5,3,4,5,4,5,5};
        if (rr[lane] == 3 || cc[lane] == 3) x = 0.0f;
      }
      s_tot[lane] = x;
    }
    __syncthreads();
    float a[6], b[6], c[6];
    ldl6_solve(s_tot, a);
    ldl6_solve_wave(s_tot, b);
    ldl6_solve_short(s_tot, c);
    bool m = false;
    float amax = 0.0f, dmax = 0.0f;
    for (int i = 0; i < 6; ++i) {
      m |= __float_as_uint(a[i]) != __float_as_uint(b[i]);
      amax = fmaxf(amax, fabsf(a[i]));
      dmax = fmaxf(dmax, fabsf(a[i] - c[i]));
    }
    if (lane == 0 && amax > 0.0f) atomicMax((unsigned*)maxrel, __float_as_uint(dmax / amax));
    const unsigned long long bm = __ballot(m);
    if (lane == 0 && bm) atomicAdd(bad, 1u);
    __syncthreads();
  }
}

// apply_update_elem vs apply_update: every element of every lane, on poses and increments from a
// hash (angles up to ~0.2 rad: both the Taylor and the sincosf branch)
__global__ void check_elem(int n, unsigned* bad) {
  const int lane = threadIdx.x;
  for (int v = 0; v < n; ++v) {
    auto hsh = [&](int k) {
      unsigned x = (unsigned)(v * 977 + k * 131 + 7);
      x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
      return (float)(int)(x & 0xffff) / 32768.0f - 1.0f;
    };
    float R[9], t[3], dx[6], R2[9], t2[3];
    for (int i = 0; i < 9; ++i) R[i] = R2[i] = hsh(i);
    for (int i = 0; i < 3; ++i) t[i] = t2[i] = 3.0f * hsh(9 + i);
    for (int i = 0; i < 6; ++i) dx[i] = ((v & 1) ? 0.2f : 0.01f) * hsh(12 + i);
    apply_update(dx, R2, t2);
    const float w = apply_update_elem(dx, R, t, lane & 15);
    const int e = (lane & 15) < 11 ? (lane & 15) : 11;
    const float ref = e < 9 ? R2[e] : t2[e - 9];
    const unsigned long long bm = __ballot(__float_as_uint(w) != __float_as_uint(ref));
    if (lane == 0 && bm) atomicAdd(bad, 1u);
  }
}

int main() {
  PicpArgs A{};
  A.damping = 1.0f; A.min_inliers = 0; A.max_rounds = 1 << 30; A.conv_eps = -1.0f;
  std::vector<float> tot(PICP_NPART, 0.0f);
  int k = 0;
  for (int r = 0; r < 6; ++r)
    for (int c = r; c < 6; ++c) tot[k++] = (r == c) ? 1e4f + 100.0f * r : 10.0f * (r + c + 1);
  for (int i = 0; i < 6; ++i) tot[PICP_P_B + i] = 1e-3f * (i + 1);
  float* d_tot; unsigned long long* d_cyc; float* d_out;
  hipMalloc(&d_tot, PICP_NPART * 4); hipMalloc(&d_cyc, 16 * 8); hipMalloc(&d_out, 16 * 4);
  hipMemcpy(d_tot, tot.data(), PICP_NPART * 4, hipMemcpyHostToDevice);
  const int iters = 2000;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<4>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<5>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<6>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<7>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipLaunchKernelGGL(bench<8>, dim3(1), dim3(64), 0, 0, A, d_tot, iters, d_cyc, d_out);
    hipDeviceSynchronize();
  }
  unsigned long long cyc[16];
  hipMemcpy(cyc, d_cyc, 16 * 8, hipMemcpyDeviceToHost);
  printf("cycles/iter: finish_round_pose %llu  ldl6_solve %llu  apply_update %llu  state_copy %llu  empty %llu  "
         "ldl6_solve_wave %llu  ldl6_solve_short %llu\n", cyc[0], cyc[1], cyc[2], cyc[3], cyc[4], cyc[5], cyc[6]);
  printf("cycles/iter: shipped finish + lane-0 pose stores %llu  finish_round_elem + lanes 0-11 stores %llu\n",
         cyc[7], cyc[8]);
  unsigned* d_bad; unsigned nbad = 0;
  float* d_rel; float rel = 0.0f;
  hipMalloc(&d_bad, 4); hipMemset(d_bad, 0, 4);
  hipMalloc(&d_rel, 4); hipMemset(d_rel, 0, 4);
  hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, d_tot, 64, d_bad, d_rel);
  hipMemcpy(&nbad, d_bad, 4, hipMemcpyDeviceToHost);
  hipMemcpy(&rel, d_rel, 4, hipMemcpyDeviceToHost);
  printf("ldl6_solve_wave vs ldl6_solve: %u of 64 systems differ (4 with a zero pivot)\n", nbad);
  printf("ldl6_solve_short vs ldl6_solve: max |ddx| / max |dx| = %.3g over the 64 systems\n", rel);
  hipMemset(d_bad, 0, 4);
  hipLaunchKernelGGL(check_elem, dim3(1), dim3(64), 0, 0, 4096, d_bad);
  hipMemcpy(&nbad, d_bad, 4, hipMemcpyDeviceToHost);
  printf("apply_update_elem vs apply_update: %u of 4096 updates differ in some element\n", nbad);
  return 0;
}
