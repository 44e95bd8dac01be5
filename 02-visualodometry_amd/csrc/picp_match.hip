// picp_match.hip -- descriptor matching (reference: match_points, src/my_utilities.h:70-120),
// the producer of the PICP correspondences.
//
// For every descriptor of set 1: the nearest descriptor of set 2 by squared L2 distance and the
// second-nearest distance, updated with strict '<' in set-2 index order exactly as the
// reference loop does; accepted iff best < dist_thr (0.2) and best/second < ratio_thr (0.8)
// (src/my_utilities.h:44-46,100-103).  The distance is summed over the dims in order with FP
// contraction off, so indices, distances and accept flags are bit-identical to the CPU oracle.
//
// Two queries per lane, their descriptors in registers as float2 pairs (the subtract, square and
// in-order accumulation of both written on float2; scalar instructions since the device code is
// built without packed FP32, picp_internal.h -- FMA contraction is off, so the bits equal the
// oracle's);
// set 2 is streamed through LDS in tiles shared by the 512 queries of a block, one broadcast LDS
// read feeding both queries.  Batched: blockIdx.y = problem (ragged sets).
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "picp_internal.h"

#define PICP_MATCH_BLOCK 256
#define PICP_MATCH_QPL 2  // queries per lane: (query A, query B) packed in one float2
#define PICP_MATCH_QPB (PICP_MATCH_BLOCK * PICP_MATCH_QPL)
#define PICP_MATCH_TILE 256
#define PICP_MATCH_MAXD 32

typedef float f2 __attribute__((ext_vector_type(2)));

// The reference's update (src/my_utilities.h:91-97), in index order,
//   if (d < best) { second = best; best = d; bi = j; } else if (d < second) second = d;
// branch-free for d >= 0 or NaN (best <= second always holds; NaN is mapped to +inf, which
// leaves all three unchanged exactly as the reference's comparisons do):
//   second' = med3(best, d, second)   (d < best: best; best <= d < second: d; else second;
//                                       d == best: best == d, as the reference's else-branch)
//   best'   = d < best ? d : best
//   bi'     = d < best ? j : bi       (strict: the first index of the minimum wins)
__device__ inline void match_update(float d, int32_t j, float& best, float& second, int32_t& bi) {
  d = fminf(d, INFINITY);  // a NaN distance never updates anything: make it +inf (IEEE minNum)
  const bool lt = d < best;
  second = __builtin_amdgcn_fmed3f(best, d, second);
  best = lt ? d : best;
  bi = lt ? j : bi;
}

// One query's outputs: best index (relative to the problem's r_off), best and second distance,
// and the reference's accept test (src/my_utilities.h:100-103: best < DISTANCE_THRESHOLD and
// best/second < RATIO_THRESHOLD).  Neither distance is ever NaN (match_update maps NaN to +inf).
__device__ __forceinline__ void match_store(const MatchProblem& P, int64_t o, int32_t bi, float best, float second,
                                            float dist_thr, float ratio_thr, int32_t* best_idx, float* best_dist,
                                            float* second_dist, int32_t* accepted) {
  (void)P;
  best_idx[o] = bi;
  best_dist[o] = best;
  second_dist[o] = second;
  accepted[o] = (bi != -1 && best < dist_thr && best / second < ratio_thr) ? 1 : 0;
}

template <int D>  // D > 0: compile-time dim; D == 0: runtime dim <= PICP_MATCH_MAXD
__global__ __launch_bounds__(PICP_MATCH_BLOCK) void picp_match_kernel(
    const float* __restrict__ q_desc, const float* __restrict__ r_desc,
    const MatchProblem* __restrict__ probs, int dim_rt, float dist_thr, float ratio_thr,
    int32_t* __restrict__ best_idx, float* __restrict__ best_dist,
    float* __restrict__ second_dist, int32_t* __restrict__ accepted) {
  constexpr int DM = D > 0 ? D : PICP_MATCH_MAXD;
  const int dim = D > 0 ? D : dim_rt;
  constexpr int TILE = DM <= 16 ? PICP_MATCH_TILE : PICP_MATCH_TILE / 2;
  __shared__ f2 tile[TILE * DM];  // each value duplicated: one LDS read = both lanes of a pk op
  const MatchProblem P = probs[blockIdx.y];
  const int64_t q0 = (int64_t)blockIdx.x * PICP_MATCH_QPB;
  if (q0 >= P.nq) return;  // whole block past this problem
  const int64_t qa = q0 + threadIdx.x, qb = qa + PICP_MATCH_BLOCK;
  const bool va = qa < P.nq, vb = qb < P.nq;
  f2 q[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    q[k].x = (va && k < dim) ? q_desc[(P.q_off + qa) * dim + k] : 0.0f;
    q[k].y = (vb && k < dim) ? q_desc[(P.q_off + qb) * dim + k] : 0.0f;
  }
  float best_a = FLT_MAX, second_a = FLT_MAX, best_b = FLT_MAX, second_b = FLT_MAX;  // :78-79
  int32_t bi_a = -1, bi_b = -1;
  for (int64_t t0 = 0; t0 < P.nr; t0 += TILE) {
    const int nt = (int)((P.nr - t0) < TILE ? (P.nr - t0) : TILE);
    __syncthreads();
    for (int e = threadIdx.x; e < nt * dim; e += PICP_MATCH_BLOCK) {
      const float r = r_desc[(P.r_off + t0) * dim + e];
      tile[e] = (f2){r, r};
    }
    __syncthreads();
    if (va) {
      for (int j = 0; j < nt; ++j) {
        f2 d = {0.0f, 0.0f};
        {
#pragma clang fp contract(off)
#pragma unroll
          for (int k = 0; k < DM; ++k) {
            if (k < dim) {  // (a - r)^2 summed over the dims in order, per query
              const f2 t = q[k] - tile[j * dim + k];
              d = d + t * t;
            }
          }
        }
        const int32_t jj = (int32_t)(t0 + j);
        match_update(d.x, jj, best_a, second_a, bi_a);
        match_update(d.y, jj, best_b, second_b, bi_b);
      }
    }
  }
  // accepted iff best < DISTANCE_THRESHOLD and best/second < RATIO_THRESHOLD (:100-103)
  if (va)
    match_store(P, P.q_off + qa, bi_a, best_a, second_a, dist_thr, ratio_thr, best_idx, best_dist, second_dist,
                accepted);
  if (vb)
    match_store(P, P.q_off + qb, bi_b, best_b, second_b, dist_thr, ratio_thr, best_idx, best_dist, second_dist,
                accepted);
}

// ---------------------------------------------------------------------------------------
// MFMA pre-filter + exact rescan (same results, bit for bit).
//
// Pass 1: D'(q, r) = |r|^2 - 2 q.r from v_mfma_f32_32x32x16_f16 (fp16 operands, fp32
// accumulation) -- the approximate distance minus the query's constant |q|^2 -- and per query
// the approximate second-smallest s' over all references.  With D = |q|^2 + D' and d the
// reference's float distance (sum of (q_k - r_k)^2 in order), |D - d| <= E_q for every safe
// pair, where (v = 2^-11 fp16 rounding, u = 2^-24)
//   E_q = 1.5 * [(2v + v^2 + 56u)(|q|^2 + Rmax) + 2^-22 (1 + |q|^2 + Rmax)]
// (fp16 quantisation of both operands incl. subnormals, the fp32 accumulation, the fp32 norms,
// the reference's own 12 roundings; 1.5x headroom).  Then every reference that can be the
// exact best or second of q has D' <= s' + 2 E_q: the two smallest-D references have exact
// d <= s' + |q|^2 + E_q, so the exact second s <= s'+|q|^2+E_q, and any r with d_r <= s has
// D'_r <= d_r - |q|^2 + E_q <= s' + 2 E_q.
// Pass 2: the references under that bound ("candidates", typically 2-4) are collected per
// query; the exact update of the reference then runs over them in index order, which yields the
// same best index (first minimum), best and second as scanning all of them.  A query with more
// than MM_CAP candidates, a non-finite or |x| > 60000 component (fp16 range), or < 2 safe
// references takes the exact full scan; an unsafe reference is a candidate for every query.
// ---------------------------------------------------------------------------------------
extern "C" hipError_t picp_launch_match(hipStream_t stream, int n_problems, int64_t max_nq,
                                        const float* q_desc, const float* r_desc,
                                        const MatchProblem* probs, int dim, float dist_thr,
                                        float ratio_thr, int32_t* best_idx, float* best_dist,
                                        float* second_dist, int32_t* accepted);

typedef _Float16 mm_half8 __attribute__((ext_vector_type(8)));
typedef float mm_f16v __attribute__((ext_vector_type(16)));

#ifndef MM_WAVES
#define MM_WAVES 4
#endif
#define MM_BLOCK (64 * MM_WAVES)
// RB (kernel template argument): 32-query MFMA row blocks per wave, sharing every B operand.
// The launcher takes RB = 2 when that still fills a generation of blocks (C5: +3.4 %,
// 1024 x 2000 x 2000: -9 % time) and RB = 1 for small grids (64 x 2000 x 8000: RB = 2 +9 %).
#define MM_CAP 16                 // candidate slots per query
// Reference-range split (ksplit > 1): a problem's references in ranges of mm_kchunk rows, at least
// MM_KMIN (so a range is worth a block's query prologue), whole tiles; mm_nsplit non-empty ranges.
#define MM_KMIN 1024
#define MM_KSPLIT_MAX 16        // the occupancy split's cap (picp_match_ksplit)
#define MM_KSPLIT_MAX2 32       // ... for the folded form at two row blocks per wave
#define MM_KSPLIT_LIMIT 65536   // a launch's hard limit (reference sets up to 2^36 rows in 2^20-row ranges)
__host__ __device__ __forceinline__ int64_t mm_kchunk(int64_t nr, int ksplit) {
  const int64_t c = (nr + ksplit - 1) / ksplit;
  const int64_t t = (c + 255) / 256 * 256;
  return t > MM_KMIN ? t : MM_KMIN;
}
__host__ __device__ __forceinline__ int mm_nsplit(int64_t nr, int ksplit) {
  return nr > 0 ? (int)((nr + mm_kchunk(nr, ksplit) - 1) / mm_kchunk(nr, ksplit)) : 0;
}
#define MM_SAFE 60000.0f

__device__ __forceinline__ float mm_bound(float nq, float rmax) {
  const float v = 1.0f / 2048.0f, u = 1.0f / 16777216.0f;
  const float t = nq + rmax;
  return 1.5f * ((2.0f * v + v * v + 56.0f * u) * t + (1.0f / 4194304.0f) * (1.0f + t));
}

// the reference's distance (src/my_utilities.h:83-90), exactly
__device__ __forceinline__ float mm_exact_dist(const float* q, const float* __restrict__ r, int dim) {
#pragma clang fp contract(off)
  float d = 0.0f;
  for (int k = 0; k < dim; ++k) {
    const float t = q[k] - r[k];
    d = d + t * t;
  }
  return d;
}

// The accept-only (radius) form's constants (see the kernel): the per-pair bound's slope a1 and
// offset b2 (twice mm_bound's headroom) and the radius R = (dist_thr / ratio_thr)(1 + 2^-10).
#define MM_A1 (3.0f * ((2.0f / 2048.0f + 1.0f / (2048.0f * 2048.0f) + 56.0f / 16777216.0f) + 1.0f / 4194304.0f))
#define MM_B2 (3.0f / 4194304.0f)
#define MM_FOLD_MAX 60000.0f  // |x|^2 and |q|^2 bound of the folded form (fp16 range of the halves)
__device__ __forceinline__ float mm_radius(float dist_thr, float ratio_thr) {
  return (dist_thr / ratio_thr) * (1.0f + 1.0f / 1024.0f);
}

// fp16 hi/lo split of x (|x| <= 65504): hi + lo == x to 2^-22 |x| (plus 2^-25 absolute)
__device__ __forceinline__ void mm_split(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

// Prep of n descriptors (float[dim] rows): fp16 rows padded to 16*kch, and the two guard norms
//   n1 = |x|^2, +inf if a component is non-finite or beyond +-60000 (fp16 range): pass 1
//   n2 = |x|^2, -inf for such a row: pass 2 (an unsafe reference is every query's candidate)
// An unsafe row's fp16 values are zeroed so its MFMA products stay finite.
extern "C" __global__ void picp_match_prep_kernel(const float* __restrict__ desc, int64_t n, int dim,
                                                  int kch, _Float16* __restrict__ h,
                                                  float* __restrict__ n1, float* __restrict__ n2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int dp = 16 * kch;
  float nr = 0.0f;
  bool bad = false;
  for (int k = 0; k < dim; ++k) {
    const float x = desc[i * dim + k];
    bad |= !(fabsf(x) <= MM_SAFE);
    nr = fmaf(x, x, nr);
  }
  for (int k = 0; k < dp; ++k) h[i * dp + k] = (_Float16)((k < dim && !bad) ? desc[i * dim + k] : 0.0f);
  if (kch == 1 && dim <= 12) {
    // the folded radius form's reference-side extension (halves dim .. dim+3, which every query
    // A operand zeroes outside that form): [-n2s/2 as hi, lo, 1, 1], n2s = |x|^2 (1 - a1)
    _Float16 hi = (_Float16)0.0f, lo = (_Float16)0.0f;
    if (!bad && nr <= MM_FOLD_MAX) mm_split(-0.5f * (nr * (1.0f - MM_A1)), hi, lo);
    h[i * dp + dim] = hi;
    h[i * dp + dim + 1] = lo;
    h[i * dp + dim + 2] = (_Float16)1.0f;
    h[i * dp + dim + 3] = (_Float16)1.0f;
  }
  n1[i] = bad ? INFINITY : nr;
  n2[i] = bad ? -INFINITY : nr;
}

// The pre-filter kernel.  q_*/r_* prep arrays are indexed like the fp32 descriptors.  The
// references stream through LDS in tiles of MM_RT, double-buffered: the next tile is fetched into
// registers (16 B per lane) while this one is computed and stashed after it.  Rows past the end
// are loaded clamped and masked in registers (norm := +inf).  LDS-DMA (global_load_lds) staging
// was measured 30-40 % slower at full occupancy (C5, 4 blocks per CU: other blocks already hide
// the fetch latency; profiles/r01/match_ab.log).
#ifndef MM_RT
#define MM_RT 256  // reference rows per LDS tile (128: -3.4 % on C5, 512: -7 %; profiles/r01/match_ab.log)
#endif
#ifndef MM_PF
#define MM_PF 1  // tiles of references in flight ahead of the computed one (pass 2): 1, 2 or 3
#endif
static_assert(MM_PF >= 1 && MM_PF <= 3, "MM_PF: 1, 2 or 3");
#ifndef MM_MERGE32
#define MM_MERGE32 0  // 1: splits of 17-32 ranges merged in one 32-range chunk (A/B: 8e equal or
                      // slower than two 16-range chunks, profiles/r06/t37/ab.log)
#endif
#ifndef MM_EARLY
#define MM_EARLY 0  // 1: the next tile's fetch issued at the previous step's end (PF = 1; A/B:
                    // equal at every C5 shape, profiles/r06/t35/ab.log)
#endif
static_assert(!MM_EARLY || MM_PF == 1, "MM_EARLY needs MM_PF = 1");
#ifndef MM_PIPE_RB2
#define MM_PIPE_RB2 1  // 0: the RB = 2 folded loop unpipelined (A/B)
#endif
#ifndef MM_BT
#define MM_BT 4  // folded pass: column blocks whose B operands are read per LDS wait (RB = 1)
#endif
#ifndef MM_BT2
#define MM_BT2 4  // the same for RB = 2
#endif
// Diagnostic build only (-DPICP_STAMPS): [0] queries through the full-scan fallback, [1] total
// candidates rescanned, [2] queries, [3] max candidates of a query (tools/match_stats.py).
// Diagnostic build only (-DMM_TSTAMP): s_memtime phase sums of the folded pass-2 tile loop, lane 0
// of every wave: [0] fold vote + barrier, [1] next tile's fetch issue, [2] compute, [3] fold check +
// stash (waits for the fetch), [4] tiles, [5] whole tile loop (tools/r06/match_tstamp.py).
#ifdef MM_TSTAMP
__device__ unsigned long long picp_match_tstamp[6];
extern "C" hipError_t picp_debug_match_tstamp(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_match_tstamp), sizeof(picp_match_tstamp), 0,
                                     hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) {
    const unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(picp_match_tstamp), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return e;
}
#define MM_TS(v) v = __builtin_amdgcn_s_memtime()
#else
#define MM_TS(v) (void)0
#endif
#ifdef PICP_STAMPS
__device__ unsigned long long picp_match_stats[4];
extern "C" hipError_t picp_debug_match_stats(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_match_stats), sizeof(picp_match_stats), 0,
                                     hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) {
    const unsigned long long z[4] = {0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(picp_match_stats), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return e;
}
#endif

// min(a, b, c) for values that are never NaN (D' = n1 - 2 q.r of finite fp16 products, or +inf):
// one v_min3_f32 -- fminf would add an IEEE canonicalisation (v_max x,x,x) per operand
__device__ __forceinline__ float mm_min3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// m = 2m + (d <= t): the candidate bitmask in two instructions (compare into VCC, shift in as the
// carry); after 16 steps bit 15-i holds element i
__device__ __forceinline__ unsigned mm_shift_in_le(unsigned m, float d, float t) {
  asm("v_cmp_le_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(m) : "v"(d), "v"(t) : "vcc");
  return m;
}

// The 16-element candidate mask of one accumulator (element i >= 0) in 16 instructions, by ROW: bit
// 8k + y is set iff element i = 4k + y is >= 0, and 8k + y = (i & 3) + 8 (i >> 2) is that
// element's row offset within its 32-row half (the caller adds 32 rb + 4 hf), so a candidate's
// row is one add from its bit index.  v_perm_b32 selector 9 / 11 turns the sign bit of src1 /
// src0 into a 0x00 / 0xFF byte: eight perms give two element flags each, four more gather
// W_y = [neg(4k + y), k = 0..3] as bytes, and three bfi merge bit y of byte k from W_y.  The
// selectors and masks sit in SGPRs (no VOP3 literals on gfx9; one SGPR per instruction).  The
// caller has already read every accumulator element (the max tree), so the MFMA result hazard is
// resolved.  (A carry chain, compare into VCC + v_addc per element, took 32: round 3.)
__device__ __forceinline__ unsigned mm_mask16_rows(const mm_f16v& acc) {
  unsigned t, u, v, m;  // W_0 in m, W_y (y > 0) in t, merged as each is done: four temporaries
  asm("v_perm_b32 %[t], %[a4], %[a0], %[s1]\n\t"  // byte 0 = neg(a0), byte 1 = neg(a4)
      "v_perm_b32 %[u], %[a12], %[a8], %[s1]\n\t"  // byte 0 = neg(a8), byte 1 = neg(a12)
      "v_perm_b32 %[v], %[a5], %[a1], %[s1]\n\t"
      "v_perm_b32 %[m], %[u], %[t], %[s2]\n\t"  // W_0 = bytes neg(0), neg(4), neg(8), neg(12)
      "v_perm_b32 %[u], %[a13], %[a9], %[s1]\n\t"
      "v_perm_b32 %[t], %[a6], %[a2], %[s1]\n\t"
      "v_perm_b32 %[v], %[u], %[v], %[s2]\n\t"  // W_1
      "v_perm_b32 %[u], %[a14], %[a10], %[s1]\n\t"
      "v_bfi_b32 %[m], %[k1], %[m], %[v]\n\t"  // bit 0 of each byte from W_0, bits 1.. from W_1
      "v_perm_b32 %[t], %[u], %[t], %[s2]\n\t"  // W_2
      "v_perm_b32 %[v], %[a7], %[a3], %[s1]\n\t"
      "v_perm_b32 %[u], %[a15], %[a11], %[s1]\n\t"
      "v_bfi_b32 %[m], %[k3], %[m], %[t]\n\t"
      "v_perm_b32 %[v], %[u], %[v], %[s2]\n\t"  // W_3
      "v_bfi_b32 %[m], %[k7], %[m], %[v]\n\t"
      "v_bfi_b32 %[m], %[m], 0, %[kf]"  // ~neg & 0x0f0f0f0f: the candidates
      : [t] "=&v"(t), [u] "=&v"(u), [v] "=&v"(v), [m] "=&v"(m)
      : [a0] "v"(acc[0]), [a1] "v"(acc[1]), [a2] "v"(acc[2]), [a3] "v"(acc[3]), [a4] "v"(acc[4]),
        [a5] "v"(acc[5]), [a6] "v"(acc[6]), [a7] "v"(acc[7]), [a8] "v"(acc[8]), [a9] "v"(acc[9]),
        [a10] "v"(acc[10]), [a11] "v"(acc[11]), [a12] "v"(acc[12]), [a13] "v"(acc[13]),
        [a14] "v"(acc[14]), [a15] "v"(acc[15]), [s1] "s"(0x0C0C0B09u), [s2] "s"(0x05040100u),
        [k1] "s"(0x01010101u), [k3] "s"(0x03030303u), [k7] "s"(0x07070707u), [kf] "s"(0x0F0F0F0Fu));
  return m;
}

// mm_mask16_rows' row layout (bit 8k + y = element 4k + y) packed to 16 bits, bit i = element i:
// t = m | m >> 4 puts k = 1 / 3 in the high nibbles of bytes 0 / 2, one v_perm_b32 takes those two
// bytes
__device__ __forceinline__ unsigned mm_pack16(unsigned m) {
  const unsigned t = m | (m >> 4);
  return __builtin_amdgcn_perm(t, t, 0x0C0C0200u);
}

// RAD = 1: the accept-only (radius) form for callers that consume only accepted[] and the
// best_idx of accepted queries (the VO sequence): pass 1 is skipped and the candidates are the
// references within a fixed radius of the query (mm_radius below); best_idx, best_dist and
// second_dist are defined only where accepted[] is 1, accepted[] everywhere.
// RAD = 2: the same candidates with the radius test FOLDED into the MFMA (dim <= 12): the K
// slots dim .. dim+3 carry [1, 1, tau/2 hi, tau/2 lo] on the query side and [-n2s/2 hi, lo, 1, 1]
// on the reference side, so each accumulator element IS S' = q.r - n2s/2 + tau/2 = -S/2 and a
// reference is a candidate iff S' >= 0; a 32x32 block with no candidate costs one max3 tree and
// one wave vote instead of 48 VALU.  Tiles holding a reference outside the fold's range
// (|r|^2 > 60000, unsafe) or past the end take the RAD = 1 compare.
#ifndef MM_MINB
#define MM_MINB 1
#endif
template <int KCH, int RAD, int RB>
__global__ __launch_bounds__(MM_BLOCK, MM_MINB) void picp_match_mfma_kernel(
    const float* __restrict__ q_desc, const float* __restrict__ r_desc,
    const _Float16* __restrict__ q_h, const float* __restrict__ q_n1,
    const _Float16* __restrict__ r_h, const float* __restrict__ r_n1, const float* __restrict__ r_n2,
    const MatchProblem* __restrict__ probs, int dim, float dist_thr, float ratio_thr,
    int32_t* __restrict__ best_idx, float* __restrict__ best_dist,
    float* __restrict__ second_dist, int32_t* __restrict__ accepted, int n_problems, int gx,
    int xcd_map, int ksplit, float4* __restrict__ part, int64_t part_nq, int slot0) {
  constexpr int QPW = 32 * RB;                      // queries per wave
  constexpr int QPB = MM_WAVES * QPW;               // queries per block
  constexpr int BT = (RB == 2) ? MM_BT2 : MM_BT;
  constexpr bool PIPE = MM_PIPE_RB2 && RB == 2;  // the folded loop software-pipelined (below)
  constexpr int DP = 16 * KCH;                      // halves per prepped row
  constexpr int CH = MM_RT * DP / 8;                // 16-B chunks per tile
  constexpr int CPT = CH / MM_BLOCK;                // 16-B chunks per thread per tile
  constexpr int NPN = 2 * MM_RT / MM_BLOCK;        // norms per thread per tile (n1 | n2)
  static_assert(CH % MM_BLOCK == 0 && (2 * MM_RT) % MM_BLOCK == 0, "tile / block shape");
  constexpr int DMAX = 16 * KCH;
  // all of the kernel's LDS in one __shared__ object
  struct Lds {
    mm_half8 t[2][CH];                   // tile rows, 16-B chunks: row*(DP/8) + c*2 + h
    float n[2][2][MM_RT];                // [buf][n1|n2][ref]
    int cnt[MM_WAVES][QPW];
    int nofold[2];  // RAD = 2: 1 + the index of the tile in LDS buffer b that holds an unsafe reference
    int list[MM_WAVES][QPW][MM_CAP];
    float nq[MM_WAVES][QPW];
  };
  __shared__ Lds lds;
  auto& s_t = lds.t;
  auto& s_n = lds.n;
  auto& s_cnt = lds.cnt;
  auto& s_list = lds.list;
  auto& s_nq = lds.nq;

  // XCD-aware block order (cdna_hip_programming.md T1): blocks are dealt round-robin over the
  // 8 XCDs, so block L runs beside blocks L +- 8.  With xcd_map, problem p's query blocks all
  // get L = p (mod 8): every block of a problem shares one XCD's L2, which then holds the
  // references of the ~10 problems in flight there instead of a slice of all of them.
  // With ksplit > 1 (mm_ksplit), group g = pid * ksplit + ks holds the query blocks of problem pid
  // against the ks-th contiguous range of its references (mm_kchunk); the groups take the place of
  // the problems in the XCD map (the blocks that read one reference range share an L2).
  int pid, qblk, ks = 0;
  if (xcd_map) {
    const unsigned L = blockIdx.x, x = L & 7u, sidx = L >> 3;
    const unsigned pq = sidx / (unsigned)gx;
    qblk = (int)(sidx - pq * (unsigned)gx);
    const unsigned g = pq * 8u + x;
    pid = (int)(g / (unsigned)ksplit);
    ks = (int)(g - (unsigned)pid * (unsigned)ksplit);
    if (pid >= n_problems) return;
  } else {
    pid = blockIdx.y;
    qblk = blockIdx.x % gx;
    ks = blockIdx.x / gx;
  }
  MatchProblem P = probs[pid];
  int64_t r_lo = 0;  // this block's references: [r_lo, r_lo + P.nr) of the problem's (P is local)
  if (ksplit > 1) {
    const int64_t kc = mm_kchunk(P.nr, ksplit);
    r_lo = (int64_t)ks * kc;
    if (r_lo >= P.nr) return;  // an empty range (the merge reads only mm_nsplit ranges)
    P.r_off += r_lo;
    P.nr = min(kc, P.nr - r_lo);
  }
  const int64_t q0 = (int64_t)qblk * QPB;
  if (q0 >= P.nq) return;  // whole block past this problem
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int64_t qw = q0 + (int64_t)w * QPW;  // this wave's first query

  mm_half8 qa[RB][KCH];  // A operands: query qw + 32 rb + r, halves [16c + 8 hf, +8)
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int64_t qi = min(qw + 32 * rb + r, P.nq - 1);
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      qa[rb][c] = *reinterpret_cast<const mm_half8*>(q_h + (P.q_off + qi) * DP + 16 * c + 8 * hf);
#pragma unroll
      for (int e = 0; e < 8; ++e)  // the prep's fold extension (halves >= dim) is not a component
        if (16 * c + 8 * hf + e >= dim) qa[rb][c][e] = (_Float16)0.0f;
    }
  }
  if (lane < QPW) {
    const int64_t qi = qw + lane;
    float nq = (qi < P.nq) ? q_n1[P.q_off + qi] : 0.0f;  // +inf: unsafe query
    if (RAD == 2 && !(nq <= MM_FOLD_MAX)) nq = INFINITY;  // outside the fold's range: full scan
    s_nq[w][lane] = nq;
    s_cnt[w][lane] = 0;
    if (tid < 2) lds.nofold[tid] = 0;  // ordered before the first stash by the barrier below
  }

  const int64_t nr_all = P.nr;
  // fetch tile t0 into registers (chunk tid + k*MM_BLOCK; norm tid + k*MM_BLOCK of the tile's
  // [n1 | n2] block), stash them into buffer b
  // the stage registers: MM_PF tiles in flight while tile t is computed (t + 1 .. t + MM_PF), in
  // MM_PF stages whose roles rotate from tile to tile (no register moves)
  mm_half8 stg[CPT], stg2[CPT], stg3[CPT];
  float sn[NPN], sn2[NPN], sn3[NPN];
  auto fetch_to = [&](int64_t t0, mm_half8 (&g)[CPT], float (&gn)[NPN]) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int ch = tid + k * MM_BLOCK;
      const int64_t row = min(t0 + ch / (DP / 8), nr_all - 1);
      g[k] = *reinterpret_cast<const mm_half8*>(r_h + (P.r_off + row) * DP + (ch % (DP / 8)) * 8);
    }
#pragma unroll
    for (int k = 0; k < NPN; ++k) {
      const int idx = tid + k * MM_BLOCK, nt = idx % MM_RT;
      gn[k] = ((idx < MM_RT) ? r_n1 : r_n2)[P.r_off + min(t0 + nt, nr_all - 1)];
    }
  };
  auto fetch = [&](int64_t t0) { fetch_to(t0, stg, sn); };
  // RAD = 2: a tile is folded iff it is whole and every reference in it is inside the fold's
  // range (n1 <= 60000: finite, safe); each thread checks the n1 norms it fetched
  // (RAD = 2: whether a tile folds travels with it through LDS: the stash tags its buffer with the
  // tile's index when a fetched norm is unsafe, and the tile loop's one barrier orders the tag before
  // the read -- a block-wide OR vote cost three barriers per tile, 634-826 cycles per wave and tile:
  // profiles/r06/t22/tstamp.txt)
  auto fold_check_of = [&](const float (&gn)[NPN]) {
    int bad = 0;  // rows past the end are neutralised by the stash (their clamped norms are safe)
#pragma unroll
    for (int k = 0; k < NPN; ++k)
      if (tid + k * MM_BLOCK < MM_RT) bad |= (gn[k] <= MM_FOLD_MAX) ? 0 : 1;
    return bad;
  };
  auto fold_check = [&](int64_t) { return fold_check_of(sn); };
  // The fetched rows go to LDS as loaded, except (RAD = 2) rows past the end: they fold to
  // S' = -65504 + tau/2 < 0 (never a candidate): components zero, -n2s/2 hi = -65504, lo = 0, and
  // its [1, 1] slots zero too -- so a partial tile takes the folded test instead of the compare.
  // The replacement happens HERE, after the compute, not in the fetch: rewriting the loaded
  // registers there made every fetch wait for its own data right after issuing it (an
  // s_waitcnt vmcnt behind the loads, 2,000-7,500 cycles per tile: profiles/r06/t21/tstamp.txt).
  auto stash_from = [&](int b, int64_t t0, const mm_half8 (&g)[CPT], const float (&gn)[NPN]) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int ch = tid + k * MM_BLOCK;
      mm_half8 v = g[k];
      if constexpr (RAD == 2) {
        if (t0 + ch / (DP / 8) >= nr_all) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] = ((ch % (DP / 8)) * 8 + e == dim) ? (_Float16)-65504.0f : (_Float16)0.0f;
        }
      }
      s_t[b][ch] = v;
    }
#pragma unroll
    for (int k = 0; k < NPN; ++k) (&s_n[b][0][0])[tid + k * MM_BLOCK] = gn[k];
  };
  auto stash = [&](int b, int64_t t0) { stash_from(b, t0, stg, sn); };
  auto load_b = [&](int b, int col, mm_half8* bb) {
#pragma unroll
    for (int c = 0; c < KCH; ++c) bb[c] = s_t[b][col * (DP / 8) + 2 * c + hf];
  };

  float tau[RB][16];
  mm_half8 qaf[RB];  // RAD = 2: the folded A operands
  float a1 = 0.0f;  // RAD: n2 is scaled by (1 - a1) before the compare (the per-pair bound)
  int buf = 0;
  // the radius form's threshold of accumulator element i of row block rb
  auto radius_tau = [&](int rb, int i) {
    const int row = 32 * rb + (i & 3) + 8 * (i >> 2) + 4 * hf;
    const float nq = s_nq[w][row];  // +inf (unsafe query): NaN tau, no candidates, full scan
    // rows past the problem's queries (their A operand repeats the last query) take none:
    // a fixed radius around |q|^2 = 0 would admit a large share of the references
    return (qw + row < P.nq) ? (mm_radius(dist_thr, ratio_thr) - nq) + fmaf(MM_A1, nq, MM_B2) : -INFINITY;
  };
  if constexpr (RAD) {
    // Accept-only (radius) candidates.  With R = (dist_thr / ratio_thr)(1 + 2^-10): a query the
    // reference accepts has its best d* < dist_thr <= R, so every reference at d < R -- the
    // best and, when it is < R, the second -- is a candidate, the index-order scan over them
    // gives the reference's best index and best, and a second >= R gives best/second <
    // ratio_thr/(1 + 2^-10), accepted either way; a rejected query (d* >= dist_thr) stays
    // rejected because candidates are a subset.  The pass-1 error bound depends on the pair
    // only through t = |q|^2 + |r|^2 (Rmax above only bounds |r|^2), E(t) = A t + B, so with
    // twice its headroom (a1 = 2A, 2B) the test D' <= R - |q|^2 + 2E(t) is
    //   fma(-2, q.r, n2 (1 - a1)) <= R - |q|^2 + a1 |q|^2 + 2B.
    a1 = MM_A1;
    const float b2 = MM_B2;
    const float R = mm_radius(dist_thr, ratio_thr);
    // RAD = 2 evaluates tau from LDS inside the (rare) tiles that take the compare -- tiles
    // with an unsafe reference -- so no 16 registers stay live across the folded loop
    if constexpr (RAD == 1) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int i = 0; i < 16; ++i) tau[rb][i] = radius_tau(rb, i);
    }
    if constexpr (RAD == 2) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        // A row r of this block: query qw + 32 rb + r (lanes r and 32 + r hold its two halves);
        // unsafe or out-of-range queries get -2 x 65504 (never a candidate; unsafe ones take
        // the full scan whatever their candidates)
        const bool live = qw + 32 * rb + r < P.nq;
        const float nq = s_nq[w][32 * rb + r];
        _Float16 th = (_Float16)-65504.0f, tl = (_Float16)-65504.0f;
        if (live && nq <= MM_FOLD_MAX) mm_split(0.5f * ((R - nq) + fmaf(a1, nq, b2)), th, tl);
        qaf[rb] = qa[rb][0];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = 8 * hf + e;
          qaf[rb][e] = (k == dim || k == dim + 1) ? (_Float16)1.0f
                       : (k == dim + 2) ? th : (k == dim + 3) ? tl : qaf[rb][e];
        }
      }
    }
  } else {
  // ---------------- pass 1: an upper bound on the approximate second-best D' per row ----------
  // Each lane keeps the minimum of D' over its own columns; the second-smallest of the 32 lane
  // minima of a row is >= the row's true approximate second-best s' (equal unless the two
  // smallest share a lane), so tau below can only be looser -- more candidates, same result.
  float b1[RB][16], s1[RB][16];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 16; ++i) b1[rb][i] = s1[rb][i] = INFINITY;
  float rmax = 0.0f;
  if (nr_all > 0) {
    fetch(0);
    stash(0, 0);
  }
  buf = 0;
  for (int64_t t0 = 0; t0 < nr_all; t0 += MM_RT, buf ^= 1) {
    __syncthreads();
    const bool more = t0 + MM_RT < nr_all;
    if (more) fetch(t0 + MM_RT);
#pragma unroll 1
    for (int sub = 0; sub < MM_RT / 32; sub += 2) {  // two column blocks per step: one min3 per row
      const int ca = sub * 32 + r, cb = ca + 32;
      mm_half8 ba[KCH], bbv[KCH];
      load_b(buf, ca, ba);
      load_b(buf, cb, bbv);
      float na = s_n[buf][0][ca], nb = s_n[buf][0][cb];
      na = (t0 + ca < nr_all) ? na : INFINITY;  // past the end: excluded
      nb = (t0 + cb < nr_all) ? nb : INFINITY;
      rmax = (na < INFINITY && na > rmax) ? na : rmax;
      rmax = (nb < INFINITY && nb > rmax) ? nb : rmax;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        mm_f16v acc_a = {}, acc_b = {};
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
          acc_a = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa[rb][c], ba[c], acc_a, 0, 0, 0);
          acc_b = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa[rb][c], bbv[c], acc_b, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)  // n = inf: excluded
          b1[rb][i] = mm_min3(b1[rb][i], fmaf(-2.0f, acc_a[i], na), fmaf(-2.0f, acc_b[i], nb));
      }
    }
    if (more) stash(buf ^ 1, t0 + MM_RT);
  }
  // merge the 32 columns of each row (lanes with equal hf): top-2 of the union
#pragma unroll
  for (int m = 1; m < 32; m <<= 1) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pb = __shfl_xor(b1[rb][i], m), ps = __shfl_xor(s1[rb][i], m);
        s1[rb][i] = fminf(fmaxf(b1[rb][i], pb), fminf(s1[rb][i], ps));
        b1[rb][i] = fminf(b1[rb][i], pb);
      }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) rmax = fmaxf(rmax, __shfl_xor(rmax, m));
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 32 * rb + (i & 3) + 8 * (i >> 2) + 4 * hf;
      tau[rb][i] = s1[rb][i] + 2.0f * mm_bound(s_nq[w][row], rmax);  // inf: every reference
    }
  __syncthreads();  // every wave is past pass 1's last tile before buffer 0 is refilled
  }  // pass 1

  // ---------------- pass 2: collect the candidates ----------------
  // Each lane appends its candidates to its OWN list in LDS -- this wave's s_list words viewed as
  // [64 lanes][LCAP] -- with one plain store per 32 x 32 block in which it holds any: no atomic, no
  // per-candidate loop and no register-indexed buffer inside the MFMA loop.  An entry is the
  // block's 16-element mask (bit i = accumulator element i, row 32 rb + 4 hf + (i & 3) + 8 (i >> 2))
  // under the block's index (tile << 4 | column block << 1 | rb): the lane's own column r gives
  // the reference.  After the pass the wave expands the entries into the per-query lists the
  // rescan reads (~1 candidate per query on C5, so a lane holds a few; a lane that overflows its
  // list sends every query of its wave to the full scan, as does a range past 4,096 tiles).
  constexpr int LCAP = QPW * MM_CAP / 64;  // RB = 2: 16, RB = 1: 8
  static_assert(MM_RT / 32 <= 8, "column block index: 3 bits");
  int* const lane_list = &s_list[w][0][0] + lane * LCAP;
  int c_n = 0;
  // past LCAP the entry overwrites the last slot and c_n > LCAP sends the wave to the full scan,
  // so no kept entry is lost
  auto push_mask = [&](unsigned m16, int64_t t0, int cb, int rb) {
    if (m16) {
      lane_list[min(c_n, LCAP - 1)] = (int)((((unsigned)(t0 / MM_RT) << 4 | (unsigned)cb << 1 | (unsigned)rb) << 16) | m16);
      ++c_n;
    }
  };
  // One tile: fold vote (RAD = 2) and barrier, the next tile's fetch into stage fs, the compute
  // on LDS buffer b, then the stage rs (the same registers: the fetch has landed) into b ^ 1.
#ifdef MM_TSTAMP
  unsigned long long ts_acc[6] = {0, 0, 0, 0, 0, 0}, ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0, tsl0 = 0, tsl1 = 0;
#endif
  auto tile_step = [&](int64_t t0, int b, mm_half8 (&fs)[CPT], float (&fn)[NPN], mm_half8 (&rs)[CPT],
                       float (&rn)[NPN]) {
    const int buf = b;
    bool fold = false;
    MM_TS(ts0);
    __syncthreads();
    if constexpr (RAD == 2) fold = lds.nofold[b] != (int)(t0 / MM_RT) + 1;
    MM_TS(ts1);
    const bool more = t0 + MM_RT < nr_all;
    if (!MM_EARLY && t0 + MM_PF * MM_RT < nr_all) fetch_to(t0 + MM_PF * MM_RT, fs, fn);
    MM_TS(ts2);
    if (RAD == 2 && fold) {
      // folded radius test: element i of the accumulator is S' of (row i, column col)
      // the B operands of BT column blocks first (one LDS wait per group, not per block);
      // BT = 4 instead of the whole tile keeps 16 registers free for a fifth wave per SIMD (RB = 1)
#pragma unroll
      for (int sg = 0; sg < MM_RT / 32; sg += BT) {
        mm_half8 bt[BT];
#pragma unroll
        for (int kb = 0; kb < BT; ++kb) {
          mm_half8 b1[KCH];
          load_b(buf, (sg + kb) * 32 + r, b1);
          bt[kb] = b1[0];
        }
        // RB = 1: the group's MFMA blocks are issued and consumed one at a time (an s_nop 11 after
        // every MFMA); other waves of the SIMD fill the wait.  RB = 2 (PIPE): software-pipelined,
        // block q+1's MFMA issued into a second accumulator before block q's result is tested.
        // Round 3 measured that slower (a wave per SIMD lost: 108 -> 131 VGPRs, profiles/r03/mab/);
        // with the balanced max tree below it fits 120 VGPRs (four waves) and the default C5 shape
        // ran 780k -> 799k frames/s (320 -> 313 us per chain step), the 8e partition +0.5 %; at RB = 1
        // it cost the per-rank shape 1.5 % (profiles/r06/t12/ab.log).  As shipped (RB = 2 only),
        // against the unpipelined build: default C5 774k -> 794k, 8e 44.9k -> 45.5k, the per-rank
        // shape (RB = 1) equal (profiles/r06/t18/ab.log, three interleaved repetitions).
        constexpr int NQB = BT * RB;
        mm_f16v accs[2];
        if constexpr (PIPE) accs[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qaf[0], bt[0], (mm_f16v){}, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < NQB; ++q) {
          const int kb = q / RB, rb = q - kb * RB;
          mm_f16v acc;
          if constexpr (PIPE) {
            if (q + 1 < NQB)
              accs[(q + 1) & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qaf[(q + 1) % RB], bt[(q + 1) / RB],
                                                                          (mm_f16v){}, 0, 0, 0);
            acc = accs[q & 1];
          } else {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(qaf[rb], bt[kb], (mm_f16v){}, 0, 0, 0);
          }
          {
            // S' >= +0 <=> its bits are a non-negative int (S' is never NaN; -0 cannot occur with
            // the tau/2 term, and a true candidate has S' > E/2 anyway).  Integer max3 keeps the
            // reads of the MFMA result visible to the compiler's hazard recognizer (an inline-asm
            // v_max3 here read the accumulator before the MFMA had written it).
            // a balanced max3 tree (dependent depth 3 instead of a chain of 8)
            auto ai = [&](int i) { return __float_as_int(acc[i]); };
            const int m0 = max(max(ai(0), ai(1)), ai(2)), m1 = max(max(ai(3), ai(4)), ai(5));
            const int m2 = max(max(ai(6), ai(7)), ai(8)), m3 = max(max(ai(9), ai(10)), ai(11));
            const int m4 = max(max(ai(12), ai(13)), ai(14));
            const int mx = max(max(max(m0, m1), m2), max(max(m3, m4), ai(15)));
#ifdef MM_DIAG_NOVOTE  // diagnostic timing build only: MFMA + max tree, no vote, no candidates
            if (mx == 0x7fffffff) c_n = 0;
            if (false) {
#elif defined(MM_DIAG_NOCAND)  // diagnostic timing build only: vote, no candidate extraction
            if (__any(mx >= 0)) c_n = 0;
            if (false) {
#else
            if (__any(mx >= 0)) {  // rare: some lane of the wave holds a candidate
#endif
              // the candidate mask in one instruction per element (the max tree above has already
              // read every accumulator, so the asm is not the MFMA result's first reader), packed to
              // 16 bits; a wave vote per element instead (skip the elements no lane has a candidate
              // in) measured 1.6x slower: 16 uniform branches, and 140 VGPRs cost a wave per SIMD
              push_mask(mm_pack16(mm_mask16_rows(acc)), t0, sg + kb, rb);
            }
          }
        }
      }  // column-block group
      MM_TS(ts3);
      if (more) {
        if (fold_check_of(rn)) lds.nofold[buf ^ 1] = (int)(t0 / MM_RT) + 2;  // the fetch has landed by now
        stash_from(buf ^ 1, t0 + MM_RT, rs, rn);
        // MM_EARLY: the tile after next into the stage just freed, before this step's end (and the
        // next step's barrier) rather than after that barrier
        if (MM_EARLY && t0 + 2 * MM_RT < nr_all) fetch_to(t0 + 2 * MM_RT, fs, fn);
      }
#ifdef MM_TSTAMP
      __builtin_amdgcn_s_waitcnt(0);  // the stash issued and landed
      MM_TS(ts4);
      ts_acc[0] += ts1 - ts0;
      ts_acc[1] += ts2 - ts1;
      ts_acc[2] += ts3 - ts2;
      ts_acc[3] += ts4 - ts3;
      ts_acc[4] += 1;
#endif
      return;
    }
#pragma unroll 1
    for (int sub = 0; sub < MM_RT / 32; ++sub) {
      const int col = sub * 32 + r;
      mm_half8 bb[KCH];
      load_b(buf, col, bb);
      float n2 = s_n[buf][1][col];  // -inf: forced candidate
      if constexpr (RAD) n2 *= 1.0f - a1;
      n2 = (t0 + col < nr_all) ? n2 : INFINITY;  // past the end: never a candidate
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        mm_f16v acc = {};
#pragma unroll
        for (int c = 0; c < KCH; ++c) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa[rb][c], bb[c], acc, 0, 0, 0);
        unsigned m = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          m = mm_shift_in_le(m, fmaf(-2.0f, acc[i], n2), RAD == 2 ? radius_tau(rb, i) : tau[rb][i]);
        push_mask(__builtin_bitreverse32(m) >> 16, t0, sub, rb);  // bit 15-i = element i -> bit i
      }
    }
    if (more) {
      if constexpr (RAD == 2)
        if (fold_check_of(rn)) lds.nofold[buf ^ 1] = (int)(t0 / MM_RT) + 2;
      stash_from(buf ^ 1, t0 + MM_RT, rs, rn);
      if (MM_EARLY && t0 + 2 * MM_RT < nr_all) fetch_to(t0 + 2 * MM_RT, fs, fn);
    }
  };
  if (nr_all > 0) {  // an empty reference set (a late part with no new points): no tile
    fetch(0);
    if constexpr (RAD == 2) {
      __syncthreads();  // the tags' initialisation before the first one is set
      if (fold_check(0)) lds.nofold[0] = 1;
    }
    stash(0, 0);
    if (MM_EARLY && MM_RT < nr_all) fetch(MM_RT);
  }
  MM_TS(tsl0);
  if constexpr (MM_PF == 1) {
    for (int64_t t0 = 0, b = 0; t0 < nr_all; t0 += MM_RT, b ^= 1) tile_step(t0, (int)b, stg, sn, stg, sn);
  } else if constexpr (MM_PF == 2) {
    if (MM_RT < nr_all) fetch_to(MM_RT, stg, sn);  // tile 1 in flight
    for (int64_t t0 = 0; t0 < nr_all; t0 += 2 * MM_RT) {
      tile_step(t0, 0, stg2, sn2, stg, sn);
      if (t0 + MM_RT >= nr_all) break;
      tile_step(t0 + MM_RT, 1, stg, sn, stg2, sn2);
    }
  } else {
    if (MM_RT < nr_all) fetch_to(MM_RT, stg, sn);  // tiles 1 and 2 in flight
    if (2 * MM_RT < nr_all) fetch_to(2 * MM_RT, stg2, sn2);
    for (int64_t t0 = 0, b = 0; t0 < nr_all; t0 += 3 * MM_RT, b ^= 1) {
      tile_step(t0, (int)b, stg3, sn3, stg, sn);
      if (t0 + MM_RT >= nr_all) break;
      tile_step(t0 + MM_RT, (int)b ^ 1, stg, sn, stg2, sn2);
      if (t0 + 2 * MM_RT >= nr_all) break;
      tile_step(t0 + 2 * MM_RT, (int)b, stg2, sn2, stg3, sn3);
    }
  }
#ifdef MM_TSTAMP
  MM_TS(tsl1);
  ts_acc[5] = tsl1 - tsl0;
  if (lane == 0)
    for (int k = 0; k < 6; ++k) atomicAdd(&picp_match_tstamp[k], ts_acc[k]);
#endif
  // expand the lane lists into the per-query lists (the same LDS words): every entry of the wave
  // is read into registers and the reads have completed before the first write
  {
    const int ln = min(c_n, LCAP);
    unsigned ent[LCAP];
#pragma unroll
    for (int u = 0; u < LCAP; ++u) ent[u] = (u < ln) ? (unsigned)lane_list[u] : 0u;
    const bool ovf = __any(c_n > LCAP) || nr_all > ((int64_t)MM_RT << 12);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < LCAP; ++u)
      if (u < ln) {
        const unsigned blk = ent[u] >> 16;
        const int ref = (int)(blk >> 4) * MM_RT + (int)((blk >> 1) & 7u) * 32 + r;
        const int rbase = 32 * (int)(blk & 1u) + 4 * hf;
        unsigned m = ent[u] & 0xffffu;
        while (m) {
          const int i = __builtin_ctz(m);
          m &= m - 1;
          const int row = rbase + (i & 3) + 8 * (i >> 2);
          const int slot = atomicAdd(&s_cnt[w][row], 1);
          if (slot < MM_CAP) s_list[w][row][slot] = ref;
        }
      }
    // a dropped entry (full lane list) or a reference range past the packing: the full scan
    if (ovf && lane < QPW) s_cnt[w][lane] = MM_CAP + 1;
  }
  __syncthreads();

  // ---------------- exact update over the candidates, in index order ----------------
  const int64_t qi = qw + lane;
  if (lane < QPW && qi < P.nq) {
    float q[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) q[k] = (k < dim) ? q_desc[(P.q_off + qi) * dim + k] : 0.0f;
    float best = FLT_MAX, second = FLT_MAX;  // :78-79
    int32_t bi = -1;
#ifdef MM_DIAG_NORESCAN  // diagnostic timing build only: no exact rescan
    const int n = 0;
#else
    const int n = s_cnt[w][lane];
#endif
#ifdef PICP_STAMPS
    atomicAdd(&picp_match_stats[2], 1ull);
    atomicAdd(&picp_match_stats[1], (unsigned long long)n);
    atomicMax(&picp_match_stats[3], (unsigned long long)n);
    if (n > MM_CAP || !(s_nq[w][lane] < INFINITY)) atomicAdd(&picp_match_stats[0], 1ull);
#endif
    if (n > MM_CAP || !(s_nq[w][lane] < INFINITY)) {  // slow path: the reference's full scan
      for (int64_t j = 0; j < P.nr; ++j) {
        const float d = mm_exact_dist(q, r_desc + (P.r_off + j) * dim, dim);
        if (d < best) { second = best; best = d; bi = (int32_t)j; }
        else if (d < second) second = d;
      }
    } else {
      // The candidates in LDS are in no particular order (lanes append them with LDS atomics).
      // The reference's in-order strict-'<' scan yields best = the minimum, bi = the FIRST
      // index attaining it, second = the second smallest of the multiset; the update below
      // yields exactly those for ANY visiting order (a tie with the best keeps the smaller
      // index and makes second equal to best; NaN never updates; distances are sums of squares,
      // never -0), so no sort is needed.
      // Candidates in chunks of MM_RQ: every row of a chunk is requested before the first
      // distance (one L2 round trip per chunk instead of one per candidate; ~2-3 candidates per
      // query on C5, so usually one chunk).
      constexpr int MM_RQ = 4;
      for (int k0 = 0; k0 < n; k0 += MM_RQ) {
        float rr[MM_RQ][DMAX];
        int jj[MM_RQ];
#pragma unroll
        for (int u = 0; u < MM_RQ; ++u) {
          jj[u] = (k0 + u < n) ? s_list[w][lane][k0 + u] : -1;
          const float* rp = r_desc + (P.r_off + max(jj[u], 0)) * dim;
#pragma unroll
          for (int k = 0; k < DMAX; ++k) rr[u][k] = (jj[u] >= 0 && k < dim) ? rp[k] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < MM_RQ; ++u) {
          if (jj[u] < 0) continue;
          const int j = jj[u];
          float d = 0.0f;  // mm_exact_dist over the registers (compile-time indices)
          {
#pragma clang fp contract(off)
#pragma unroll
            for (int k = 0; k < DMAX; ++k)
              if (k < dim) {
                const float t = q[k] - rr[u][k];
                d = d + t * t;
              }
          }
          if (d < best) { second = best; best = d; bi = j; }
          else if (d == best) { second = best; bi = min(bi, j); }
          else if (d < second) second = d;
        }
      }
    }
    // indices in the caller's numbering: the range's offset and the problem's idx0
    const int32_t gi = bi >= 0 ? (int32_t)(bi + r_lo + P.idx0) : -1;
    if (ksplit > 1 || slot0 >= 0)  // this range's top-2, merged in range order by picp_match_merge_kernel
      part[((int64_t)(max(slot0, 0) + ks) * n_problems + pid) * part_nq + qi] =
          make_float4(__int_as_float(gi), best, second, 0.0f);
    else
      match_store(P, P.q_off + qi, gi, best, second, dist_thr, ratio_thr, best_idx, best_dist, second_dist,
                  accepted);  // :100-103
  }
}

// The reference ranges of a split launch, merged in index order: the reference's in-order
// strict-'<' scan over range 0, then range 1, ... yields best = the smaller best (a tie keeps the
// earlier range's, i.e. the lower index), second = the second smallest of the union.  Each range's
// (best, first index, second) is exactly its own in-order scan's (index-order-independent update
// above), so the merged triple is the whole scan's.  One thread per query.
template <int MM_MERGE_CHUNK>
__global__ void picp_match_merge_kernel(const MatchProblem* __restrict__ probs, int n_problems,
                                                   int ksplit, const float4* __restrict__ part, int64_t part_nq,
                                                   float dist_thr, float ratio_thr, int32_t* __restrict__ best_idx,
                                                   float* __restrict__ best_dist, float* __restrict__ second_dist,
                                                   int32_t* __restrict__ accepted, int extra) {
  const int pid = blockIdx.y;
  const MatchProblem P = probs[pid];
  const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= P.nq) return;
  // the problem's ranges, then (extra >= 0) slot `extra`: a range of later references (higher
  // indices) written by another launch
  const int nsr = mm_nsplit(P.nr, ksplit);
  const int ns = nsr + (extra >= 0 ? 1 : 0);
  float best = FLT_MAX, second = FLT_MAX;  // src/my_utilities.h:78-79
  int32_t bi = -1;
  // the ranges in chunks of MM_MERGE_CHUNK (4 or 16: the launch's ksplit rounded up), every load of a
  // chunk issued before the first use: the kernel is one short latency chain on the VO world
  // match's path (8e partition: 187 -> 181 us per step with 16, profiles/r06/t4/ab.log)
  for (int k0 = 0; k0 < ns; k0 += MM_MERGE_CHUNK) {
    float4 rr[MM_MERGE_CHUNK];
#pragma unroll
    for (int u = 0; u < MM_MERGE_CHUNK; ++u)  // unconditional (clamped) loads: no branch between them
    {
      const int k = min(k0 + u, ns - 1);
      rr[u] = part[((int64_t)(k < nsr ? k : extra) * n_problems + pid) * part_nq + qi];
    }
#pragma unroll
    for (int u = 0; u < MM_MERGE_CHUNK; ++u) {
      const float4 r = rr[u];
      // a range past ns contributes +inf: never below best or equal to it, and fminf(second, inf)
      // leaves second -- a no-op
      const float b = (k0 + u < ns) ? r.y : INFINITY;
      if (b < best) {
        second = fminf(best, r.z);
        best = b;
        bi = __float_as_int(r.x);
      } else if (b == best) {
        second = best;  // two equal values in the multiset; the earlier index stays
      } else {
        second = fminf(second, b);
      }
    }
  }
  match_store(P, P.q_off + qi, bi, best, second, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
}

extern "C" int picp_match_prep_kch(int dim) { return dim <= 16 ? 1 : 2; }

extern "C" hipError_t picp_launch_match_prep(hipStream_t stream, const float* desc, int64_t n, int dim,
                                             _Float16* h, float* n1, float* n2) {
  if (n <= 0) return hipSuccess;
  if (dim < 1 || dim > PICP_MATCH_MAXD) return hipErrorInvalidValue;
  const int threads = 256;
  hipLaunchKernelGGL(picp_match_prep_kernel, dim3((unsigned)((n + threads - 1) / threads)), dim3(threads), 0,
                     stream, desc, n, dim, picp_match_prep_kch(dim), h, n1, n2);
  return hipGetLastError();
}

// The pre-filtered match over prepped descriptors (picp_launch_match_prep).  form (include/picp_c.h
// PICP_MATCH_FORM_*): bit 0 = the accept-only radius form (only accepted[] and the best index of
// accepted queries are defined), bit 1 = the exact scan (the same results as the full form; for
// A/B checks and the tests).
static hipError_t mm_merge(hipStream_t stream, const MatchProblem* probs, int n_problems, int64_t max_nq, int ksplit,
                           int extra, const float4* part, float dist_thr, float ratio_thr, int32_t* best_idx,
                           float* best_dist, float* second_dist, int32_t* accepted) {
  const dim3 mg((unsigned)((max_nq + 255) / 256), (unsigned)n_problems);
  // (MM_MERGE32: the ranges in one chunk wherever they fit 32 -- measured no faster)
  const int nr = ksplit + (extra >= 0 ? 1 : 0);
  if (nr <= 4)
    hipLaunchKernelGGL(picp_match_merge_kernel<4>, mg, dim3(256), 0, stream, probs, n_problems, ksplit, part, max_nq,
                       dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted, extra);
  else if (nr <= 16 || MM_MERGE32 == 0)
    hipLaunchKernelGGL(picp_match_merge_kernel<16>, mg, dim3(256), 0, stream, probs, n_problems, ksplit, part, max_nq,
                       dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted, extra);
  else
    hipLaunchKernelGGL(picp_match_merge_kernel<32>, mg, dim3(256), 0, stream, probs, n_problems, ksplit, part, max_nq,
                       dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted, extra);
  return hipGetLastError();
}

// slot0 < 0: the whole match (a split launch's ranges merged by a second launch); slot0 >= 0: the
// ranges' partial top-2s only, into scratch slots slot0 .. slot0 + ksplit - 1 (picp_launch_match_merge
// folds them with other launches' ranges)
static hipError_t mm_launch(hipStream_t stream, int n_problems, int64_t max_nq, const float* q_desc,
                            const float* r_desc, const _Float16* q_h, const float* q_n1, const _Float16* r_h,
                            const float* r_n1, const float* r_n2, const MatchProblem* probs, int dim,
                            float dist_thr, float ratio_thr, int32_t* best_idx, float* best_dist,
                            float* second_dist, int32_t* accepted, int form, int ksplit, int slot0, float4* part,
                            int64_t part_cap) {
  if (n_problems <= 0 || max_nq <= 0) return hipSuccess;
  // part_cap: the scratch's capacity in float4; a split launch writes ksplit x n_problems x max_nq
  if (ksplit < 1 || ksplit > MM_KSPLIT_LIMIT || slot0 > MM_KSPLIT_LIMIT) return hipErrorInvalidValue;
  const bool parts = ksplit > 1 || slot0 >= 0;
  if (parts && (!part || (int64_t)(std::max(slot0, 0) + ksplit) * n_problems * max_nq > part_cap))
    return hipErrorInvalidValue;
  const bool accept_only = (form & 1) != 0;
  if (dim < 1 || dim > PICP_MATCH_MAXD || n_problems > 65535) return hipErrorInvalidValue;
  if (slot0 >= 0 && (form & 2)) return hipErrorInvalidValue;  // the exact scan writes no partials
  // the radius argument needs 0 < dist_thr < inf and 0 < ratio_thr <= 1 (else: the full form)
  const bool rad = accept_only && dist_thr > 0.0f && dist_thr < 1e30f && ratio_thr > 0.0f && ratio_thr <= 1.0f;
  // the folded form needs the extension slots (dim <= 12) and tau/2 inside fp16 range
  const char* nf = getenv("PICP_MATCH_NO_FOLD");
  const bool fold = rad && dim <= 12 && (dist_thr / ratio_thr) <= 1000.0f && !(nf && atoi(nf) != 0);
  if (form & 2)
    return picp_launch_match(stream, n_problems, max_nq, q_desc, r_desc, probs, dim, dist_thr, ratio_thr,
                             best_idx, best_dist, second_dist, accepted);
  // RB = 2 (64 queries per wave) halves the tile fetches and LDS B reads per query but also the
  // block count: take it when the grid still holds a full generation (4 blocks per CU at the
  // folded form's 109 VGPRs).  PICP_MATCH_RB=1|2 forces.
  static int num_cu = 0;
  if (!num_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || num_cu <= 0)
      num_cu = 256;
  }
  const int64_t blocks_rb2 = (int64_t)n_problems * ((max_nq + 2 * 32 * MM_WAVES - 1) / (2 * 32 * MM_WAVES));
  // (measured for the folded accept-only form only; the others need 130-224 VGPRs at RB = 2)
  // ... or when an occupancy split of 8+ ranges already multiplies the grid to >= 2 blocks per CU
  // (few problems against long reference sets: the 8e world match's 4 problems x 15 ranges, +1.5-2 %;
  // at the per-rank shape's 4 ranges RB = 2 measured 2.4 % slower, and one problem's 16 ranges at
  // RB = 2 leave half the CUs idle: profiles/r06/t3/ab.log, profiles/r06/final/)
  int rb = (fold && (blocks_rb2 >= 4 * (int64_t)num_cu ||
                     (ksplit >= 8 && blocks_rb2 * ksplit >= 2 * (int64_t)num_cu))) ? 2 : 1;
  if (const char* e = getenv("PICP_MATCH_RB")) rb = (atoi(e) == 2) ? 2 : 1;
  const int qpb = MM_WAVES * 32 * rb;
  const int gx = (int)((max_nq + qpb - 1) / qpb);
  const char* xe = getenv("PICP_MATCH_XCD");
  const int xcd_map = (xe && atoi(xe) == 0) ? 0 : 1;
  const int64_t ngroups = (int64_t)n_problems * ksplit;
  // the kernel decodes blockIdx.x in 32-bit unsigned arithmetic
  if (8 * ((ngroups + 7) / 8) * gx > INT32_MAX || (int64_t)gx * ksplit > INT32_MAX) return hipErrorInvalidValue;
  const dim3 g = xcd_map ? dim3((unsigned)(8 * ((ngroups + 7) / 8) * gx))
                         : dim3((unsigned)(gx * ksplit), (unsigned)n_problems);
  const int64_t part_nq = max_nq;
#define PICP_LAUNCH_MM3(KC, RD, R)                                                                          \
  hipLaunchKernelGGL((picp_match_mfma_kernel<KC, RD, R>), g, dim3(MM_BLOCK), 0, stream, q_desc, r_desc, q_h,  \
                     q_n1, r_h, r_n1, r_n2, probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, \
                     accepted, n_problems, gx, xcd_map, ksplit, part, part_nq, slot0)
#define PICP_LAUNCH_MM(KC, RD)                   \
  {                                              \
    if (rb == 2) PICP_LAUNCH_MM3(KC, RD, 2);     \
    else PICP_LAUNCH_MM3(KC, RD, 1);             \
  }
  if (dim <= 16) {
    if (fold) PICP_LAUNCH_MM(1, 2)
    else if (rad) PICP_LAUNCH_MM(1, 1)
    else PICP_LAUNCH_MM(1, 0)
  } else {
    if (rad) PICP_LAUNCH_MM(2, 1)
    else PICP_LAUNCH_MM(2, 0)
  }
#undef PICP_LAUNCH_MM3
#undef PICP_LAUNCH_MM
  if (ksplit > 1 && slot0 < 0) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return mm_merge(stream, probs, n_problems, max_nq, ksplit, -1, part, dist_thr, ratio_thr, best_idx, best_dist,
                    second_dist, accepted);
  }
  return hipGetLastError();
}

extern "C" hipError_t picp_launch_match_mfma(hipStream_t stream, int n_problems, int64_t max_nq,
                                             const float* q_desc, const float* r_desc,
                                             const _Float16* q_h, const float* q_n1,
                                             const _Float16* r_h, const float* r_n1, const float* r_n2,
                                             const MatchProblem* probs, int dim, float dist_thr,
                                             float ratio_thr, int32_t* best_idx, float* best_dist,
                                             float* second_dist, int32_t* accepted, int form, int ksplit,
                                             float4* part, int64_t part_cap) {
  return mm_launch(stream, n_problems, max_nq, q_desc, r_desc, q_h, q_n1, r_h, r_n1, r_n2, probs, dim, dist_thr,
                   ratio_thr, best_idx, best_dist, second_dist, accepted, form, ksplit, -1, part, part_cap);
}

// The partial top-2s of ksplit ranges of each problem's references into scratch slots slot0 ..
// slot0 + ksplit - 1 (no outputs written; the pre-filtered forms only)
extern "C" hipError_t picp_launch_match_mfma_parts(hipStream_t stream, int n_problems, int64_t max_nq,
                                                   const float* q_desc, const float* r_desc, const _Float16* q_h,
                                                   const float* q_n1, const _Float16* r_h, const float* r_n1,
                                                   const float* r_n2, const MatchProblem* probs, int dim,
                                                   float dist_thr, float ratio_thr, int form, int ksplit, int slot0,
                                                   float4* part, int64_t part_cap) {
  if (slot0 < 0) return hipErrorInvalidValue;
  return mm_launch(stream, n_problems, max_nq, q_desc, r_desc, q_h, q_n1, r_h, r_n1, r_n2, probs, dim, dist_thr,
                   ratio_thr, nullptr, nullptr, nullptr, nullptr, form, ksplit, slot0, part, part_cap);
}

// The outputs of problems probs from scratch: the mm_nsplit(nr, ksplit) ranges of each problem in
// slots 0.., then (extra >= 0) slot extra, whose references all come after the problem's (higher
// indices) -- the reference's in-order scan over the problem's references continued over them
extern "C" hipError_t picp_launch_match_merge(hipStream_t stream, const MatchProblem* probs, int n_problems,
                                              int64_t max_nq, int ksplit, int extra, const float4* part,
                                              int64_t part_cap, float dist_thr, float ratio_thr,
                                              int32_t* best_idx, float* best_dist, float* second_dist,
                                              int32_t* accepted) {
  if (n_problems <= 0 || max_nq <= 0) return hipSuccess;
  if (n_problems > 65535 || ksplit < 1 || ksplit > MM_KSPLIT_LIMIT || extra > MM_KSPLIT_LIMIT || !part)
    return hipErrorInvalidValue;
  if ((int64_t)std::max(ksplit, extra + 1) * n_problems * max_nq > part_cap) return hipErrorInvalidValue;
  return mm_merge(stream, probs, n_problems, max_nq, ksplit, extra, part, dist_thr, ratio_thr, best_idx, best_dist,
                  second_dist, accepted);
}

// The reference-range split a launch of this shape takes (1: none): enough (problem, query block,
// range) blocks for about four per CU, at most MM_KSPLIT_MAX ranges for occupancy -- and always
// enough ranges that none exceeds the candidate entries' 2^20 references (4,096 tiles), however
// many that takes (up to MM_KSPLIT_LIMIT): a range past the packing would send every query to the
// O(nr) full scan.  The caller provides ksplit x n_problems x max_nq float4 of scratch
// (picp_launch_match_mfma's part / part_cap) when > 1.  force > 0 replaces the occupancy choice
// (PICP_MATCH_KSPLIT=n, read by picp_match_ksplit_env; 1: no occupancy split, A/B).  Small problem
// counts against large reference sets (the VO world match of a few long segments: 8 x 2,000
// queries x ~1.9e5 map points) would otherwise run one block per CU or fewer.
extern "C" int picp_match_ksplit_forced(int n_problems, int64_t max_nq, int64_t max_nr, int form, int force) {
  if (form & 2) return 1;  // the exact scan is not split
  static int num_cu = 0;
  if (!num_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || num_cu <= 0)
      num_cu = 256;
  }
  const int64_t base = (int64_t)n_problems * ((max_nq + 32 * MM_WAVES - 1) / (32 * MM_WAVES));
  int64_t k = (4 * (int64_t)num_cu + base - 1) / std::max<int64_t>(base, 1);
  k = std::max<int64_t>(1, std::min<int64_t>(k, MM_KSPLIT_MAX));
  // The folded accept-only form (form bits 0 and 2: the caller's dim <= 12) with few problems runs
  // two row blocks per wave (the launcher's RB rule): there, as many ranges as fill ONE generation
  // of four RB = 2 blocks per CU, up to 32, when every range keeps >= 4,096 rows.  The 8e world
  // match: 4 problems x 9 query blocks x 28 ranges = 1,008 blocks instead of 16 ranges' 576, C5 8e
  // +2.2 % (46.3k / 45.9k -> 47.4k / 46.8k frames/s; 24 ranges equal, 32 -1 %: profiles/r06/t26/).
  if ((form & 1) && (form & 4)) {
    const int64_t b2 = (int64_t)n_problems * ((max_nq + 64 * MM_WAVES - 1) / (64 * MM_WAVES));
    const int64_t k2 = (4 * (int64_t)num_cu) / std::max<int64_t>(b2, 1);
    if (k2 >= 8 && max_nr >= k2 * 4096) k = std::min<int64_t>(k2, MM_KSPLIT_MAX2);
  }
  if (force > 0) k = std::min<int64_t>(force, MM_KSPLIT_LIMIT);  // an A/B count may pass the cap
  // the entries' range: split the largest set at least that far (beyond the occupancy cap)
  const int64_t k_range = (max_nr + ((int64_t)MM_RT << 12) - 1) / ((int64_t)MM_RT << 12);
  return (int)std::min<int64_t>(std::max<int64_t>(k, k_range), MM_KSPLIT_LIMIT);
}

// float4 of scratch a split launch needs: the ranges' partial top-2s (picp_match_merge_kernel
// merges them).  Round 6 measured a fused form (the last-arriving range block merges, arrival
// tickets behind the partials; commit 069e837) slower at every C5 shape: 8e 42.7k-42.9k vs
// 41.9k frames/s, the N = 8 per-rank shape 162.3k vs 156.3k (profiles/r06/t2/ab.log).
extern "C" int64_t picp_match_split_scratch(int ksplit, int n_problems, int64_t max_nq) {
  return ksplit > 1 ? (int64_t)ksplit * n_problems * max_nq : 0;
}

extern "C" int picp_match_ksplit_env(void) {
  const char* e = getenv("PICP_MATCH_KSPLIT");
  return e ? std::max(0, atoi(e)) : 0;
}

extern "C" int picp_match_ksplit(int n_problems, int64_t max_nq, int64_t max_nr, int form) {
  return picp_match_ksplit_forced(n_problems, max_nq, max_nr, form, picp_match_ksplit_env());
}

extern "C" hipError_t picp_launch_match(hipStream_t stream, int n_problems, int64_t max_nq,
                                        const float* q_desc, const float* r_desc,
                                        const MatchProblem* probs, int dim, float dist_thr,
                                        float ratio_thr, int32_t* best_idx, float* best_dist,
                                        float* second_dist, int32_t* accepted) {
  if (n_problems <= 0 || max_nq <= 0) return hipSuccess;
  if (dim < 1 || dim > PICP_MATCH_MAXD || n_problems > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((max_nq + PICP_MATCH_QPB - 1) / PICP_MATCH_QPB), (unsigned)n_problems);
  if (dim == 10)
    hipLaunchKernelGGL(picp_match_kernel<10>, grid, dim3(PICP_MATCH_BLOCK), 0, stream, q_desc, r_desc,
                       probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
  else
    hipLaunchKernelGGL(picp_match_kernel<0>, grid, dim3(PICP_MATCH_BLOCK), 0, stream, q_desc, r_desc,
                       probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
  return hipGetLastError();
}
