// neighbors.hip — exact brute-force k-nearest-neighbour search for every CV split at once.
//
// Reference: KNeighborsClassifier / KNeighborsRegressor are whitelisted estimators that
// sklearn fits per (candidate, fold) on CPU (aws-prod/worker/worker.py:42,49) — a KD/ball
// tree or a brute-force distance pass every time.  Every candidate of a job that shares
// the metric needs the SAME neighbour lists (n_neighbors / weights only change the vote),
// so here ONE pass per job finds the K_max nearest training rows of every test row of
// every split, and all candidates vote from those lists (models/neighbors.py).
//
// Layout / mapping (gfx950, wave64):
//  * one wave owns QPW query rows of one split; the 64 lanes stream over 64 reference
//    rows at a time from a FEATURE-MAJOR copy XT[d, n] (coalesced 256-B loads per
//    feature); the query values are wave-uniform (scalar loads, SGPR operands), so
//    each loaded reference value feeds QPW FMAs;
//  * reference rows whose role in the query's split is not TRAIN get +inf;
//  * the running top-64 of each query is a sorted key per lane (dist_bits<<32 | row):
//    a 64-row batch is merged only when some lane beats the current K-th key (ballot),
//    by a bitonic sort of the batch (descending) + lane-wise min + 6-step bitonic merge
//    — DPP/permlane exchanges only (wave_ops.h), no LDS, no atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave_ops.h"

namespace {

using dml::wave::lane_id;
using dml::wave::shfl_xor;

constexpr int QPW = 8;           // queries per wave
constexpr int WAVES = 4;         // waves per block
constexpr uint64_t kInf = ~0ull;

template <int K, int J>
__device__ __forceinline__ uint64_t bstep(uint64_t key, int lane) {
  const uint64_t other = shfl_xor<J>(key, lane);
  const bool up = (lane & K) == 0;
  const bool lower = (lane & J) == 0;
  const uint64_t mn = key < other ? key : other;
  const uint64_t mx = key < other ? other : key;
  return (lower == up) ? mn : mx;
}

// ascending bitonic sort of 64 u64 keys (one per lane)
__device__ __forceinline__ uint64_t sort64(uint64_t k, int lane) {
  k = bstep<2, 1>(k, lane);
  k = bstep<4, 2>(k, lane); k = bstep<4, 1>(k, lane);
  k = bstep<8, 4>(k, lane); k = bstep<8, 2>(k, lane); k = bstep<8, 1>(k, lane);
  k = bstep<16, 8>(k, lane); k = bstep<16, 4>(k, lane); k = bstep<16, 2>(k, lane); k = bstep<16, 1>(k, lane);
  k = bstep<32, 16>(k, lane); k = bstep<32, 8>(k, lane); k = bstep<32, 4>(k, lane); k = bstep<32, 2>(k, lane);
  k = bstep<32, 1>(k, lane);
  k = bstep<64, 32>(k, lane); k = bstep<64, 16>(k, lane); k = bstep<64, 8>(k, lane); k = bstep<64, 4>(k, lane);
  k = bstep<64, 2>(k, lane); k = bstep<64, 1>(k, lane);
  return k;
}

// sort a bitonic 64-sequence ascending
__device__ __forceinline__ uint64_t merge64(uint64_t k, int lane) {
  k = bstep<64, 32>(k, lane); k = bstep<64, 16>(k, lane); k = bstep<64, 8>(k, lane);
  k = bstep<64, 4>(k, lane); k = bstep<64, 2>(k, lane); k = bstep<64, 1>(k, lane);
  return k;
}

// keep the 64 smallest of (top ascending) U (cand unsorted)
__device__ __forceinline__ uint64_t merge_top(uint64_t top, uint64_t cand, int lane) {
  const uint64_t desc = ~sort64(~cand, lane);           // candidates sorted descending
  const uint64_t m = top < desc ? top : desc;           // bitonic, holds the 64 smallest
  return merge64(m, lane);
}

template <int METRIC>
__device__ __forceinline__ float accum(float acc, float x, float q, float p) {
  const float t = x - q;
  if constexpr (METRIC == 0) return __builtin_fmaf(t, t, acc);   // squared L2
  if constexpr (METRIC == 1) return acc + __builtin_fabsf(t);     // L1
  if constexpr (METRIC == 2) return __builtin_fmaxf(acc, __builtin_fabsf(t));   // Linf
  return acc + __powf(__builtin_fabsf(t), p);                     // general Minkowski (p-th power sum)
}

template <int METRIC>
__global__ __launch_bounds__(64 * WAVES) void k_knn(const float* __restrict__ X, const float* __restrict__ XT,
                                                  int64_t n, int64_t d, const uint8_t* __restrict__ roles,
                                                  const int32_t* __restrict__ qrow, const int32_t* __restrict__ qsplit,
                                                  int64_t nq_groups, float p, int32_t K, float* __restrict__ out_d,
                                                  int32_t* __restrict__ out_i) {
  const int lane = lane_id();
  const int64_t group = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (group >= nq_groups) return;
  // the QPW queries of a group share one split (host pads groups per split)
  const int split = __builtin_amdgcn_readfirstlane(qsplit[group * QPW]);
  int q[QPW];
#pragma unroll
  for (int i = 0; i < QPW; ++i) q[i] = __builtin_amdgcn_readfirstlane(qrow[group * QPW + i]);
  const uint8_t* role = roles + (int64_t)split * n;

  uint64_t top[QPW];
#pragma unroll
  for (int i = 0; i < QPW; ++i) top[i] = kInf;

  for (int64_t base = 0; base < n; base += 64) {
    const int64_t j = base + lane;
    const bool valid = j < n && role[j < n ? j : 0] == 1;
    float acc[QPW];
#pragma unroll
    for (int i = 0; i < QPW; ++i) acc[i] = 0.f;
    if (j < n) {
      for (int64_t f = 0; f < d; ++f) {
        const float x = XT[f * n + j];
#pragma unroll
        for (int i = 0; i < QPW; ++i) {
          const float qv = q[i] >= 0 ? X[(int64_t)q[i] * d + f] : 0.f;
          acc[i] = accum<METRIC>(acc[i], x, qv, p);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < QPW; ++i) {
      const uint64_t key = valid ? (((uint64_t)__builtin_bit_cast(uint32_t, acc[i]) << 32) | (uint32_t)j) : kInf;
      const uint64_t thr = dml::wave::bcast(top[i], K - 1);
      if (__builtin_amdgcn_ballot_w64(key < thr) != 0) top[i] = merge_top(top[i], key, lane);
    }
  }
#pragma unroll
  for (int i = 0; i < QPW; ++i) {
    const int64_t slot = group * QPW + i;
    if (q[i] < 0 || lane >= K) continue;
    const uint64_t k = top[i];
    out_d[slot * K + lane] = k == kInf ? __builtin_inff() : __builtin_bit_cast(float, (uint32_t)(k >> 32));
    out_i[slot * K + lane] = k == kInf ? -1 : (int32_t)(uint32_t)k;
  }
}

// ---- squared-L2 on the matrix cores ---------------------------------------------------
// ||q - r||^2 = ||q||^2 + ||r||^2 - 2 q.r with the dot products on MFMA
// (v_mfma_f32_32x32x16_bf16, bf16x3: x = hi + lo, q.r ~ hi.hi + hi.lo + lo.hi, ~2^-16
// relative): a workgroup owns 32 queries (4 groups of QPW, one per wave) and streams the
// reference rows 128 at a time -- each wave multiplies the 32 queries by its 32
// references into a 32x32 accumulator tile, the tile goes to LDS as distances, and each
// wave then merges its 8 queries' rows of the 32x128 block into their running top-64
// exactly as the scalar kernel does.  The MFMA distances only SELECT candidates: the
// final top-64 of every query is re-ranked by the exact f32 sum of (x - q)^2 in feature
// order -- the scalar kernel's own arithmetic -- so results are those of ``k_knn<0>``
// whenever the true K nearest lie in the approximate 64 nearest (the host uses this
// path for K <= 32: a >= 32-row margin for the 2^-16 selection error).
//
// Operand layout (built once per dataset, models/neighbors.py): XHL = [2][KS][npad][16]
// bf16 (hi, lo planes; 16-feature K-steps; row-padded to 128 with zeros), so lane l of
// a 32x32x16 step reads its 8 features [16s + 8(l>>5), +8) of row (l&31) as one 16-B load.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MQ = 32;          // queries per workgroup (4 waves x QPW)
constexpr int MR = 128;         // reference rows per iteration (4 waves x 32)
constexpr int DL_STRIDE = 136;  // LDS row stride (floats): the two lane halves of a C store hit disjoint banks

__device__ __forceinline__ bf16x8 ld8(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

template <int KS>   // K-steps held in registers (0: stream the query operand from cache)
__global__ __launch_bounds__(256) void k_knn_l2_mfma(const __bf16* __restrict__ XHL, int64_t npad, int ks_n,
                                                     const float* __restrict__ rn, const float* __restrict__ X,
                                                     int64_t n, int64_t d, const uint8_t* __restrict__ roles,
                                                     const int32_t* __restrict__ qrow,
                                                     const int32_t* __restrict__ qsplit, int32_t K,
                                                     float* __restrict__ out_d, int32_t* __restrict__ out_i) {
  __shared__ float Dl[MQ * DL_STRIDE];
  __shared__ float qn_s[MQ];
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t q0 = (int64_t)blockIdx.x * MQ;
  const int64_t plane = (int64_t)ks_n * npad * 16;       // hi -> lo plane offset
  // query (A) operand: row r of this workgroup's 32 queries
  const int qa = qrow[q0 + r];
  const int64_t qa_row = qa >= 0 ? qa : 0;
  bf16x8 ah[KS > 0 ? KS : 1], al[KS > 0 ? KS : 1];
  if constexpr (KS > 0) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const __bf16* p = XHL + ((int64_t)s * npad + qa_row) * 16 + 8 * h;
      ah[s] = ld8(p);
      al[s] = ld8(p + plane);
      if (qa < 0) { ah[s] = bf16x8{}; al[s] = bf16x8{}; }
    }
  }
  if (threadIdx.x < MQ) {
    const int qq = qrow[q0 + threadIdx.x];
    float acc = 0.f;
    if (qq >= 0)
      for (int64_t f = 0; f < d; ++f) { const float x = X[(int64_t)qq * d + f]; acc = __builtin_fmaf(x, x, acc); }
    qn_s[threadIdx.x] = acc;
  }
  // merge-side state: this wave's QPW queries
  const int64_t group = (int64_t)blockIdx.x * WAVES + wave;
  const int split = __builtin_amdgcn_readfirstlane(qsplit[group * QPW]);
  const uint8_t* role = roles + (int64_t)split * n;
  uint64_t top[QPW];
#pragma unroll
  for (int i = 0; i < QPW; ++i) top[i] = kInf;
  __syncthreads();

  for (int64_t base = 0; base < n; base += MR) {
    const int64_t jr = base + 32 * wave + r;              // this lane's reference row in the tile (B col)
    f32x16 acc = {};
    if constexpr (KS > 0) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const __bf16* p = XHL + ((int64_t)s * npad + jr) * 16 + 8 * h;
        const bf16x8 bh = ld8(p), bl = ld8(p + plane);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s], bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bh, acc, 0, 0, 0);
      }
    } else {
      for (int s = 0; s < ks_n; ++s) {
        const __bf16* pa = XHL + ((int64_t)s * npad + qa_row) * 16 + 8 * h;
        const __bf16* pb = XHL + ((int64_t)s * npad + jr) * 16 + 8 * h;
        bf16x8 a_h = ld8(pa), a_l = ld8(pa + plane);
        if (qa < 0) { a_h = bf16x8{}; a_l = bf16x8{}; }
        const bf16x8 bh = ld8(pb), bl = ld8(pb + plane);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, bh, acc, 0, 0, 0);
      }
    }
    // C tile -> distances in LDS: column = reference (lane & 31), row = query
    const float rnj = jr < n ? rn[jr] : 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int qi = (g & 3) + 8 * (g >> 2) + 4 * h;
      const float dist = __builtin_fmaxf(qn_s[qi] + rnj - 2.f * acc[g], 0.f);
      Dl[qi * DL_STRIDE + 32 * wave + r] = dist;
    }
    __syncthreads();
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int64_t j = base + 64 * half + lane;
      const bool valid = j < n && role[j < n ? j : 0] == 1;
#pragma unroll
      for (int i = 0; i < QPW; ++i) {
        const float dist = Dl[(wave * QPW + i) * DL_STRIDE + 64 * half + lane];
        const uint64_t key = valid ? (((uint64_t)__builtin_bit_cast(uint32_t, dist) << 32) | (uint32_t)j) : kInf;
        const uint64_t thr = dml::wave::bcast(top[i], 63);   // keep 64 candidates for the exact re-rank
        if (__builtin_amdgcn_ballot_w64(key < thr) != 0) top[i] = merge_top(top[i], key, lane);
      }
    }
    __syncthreads();
  }
  // exact re-rank of each query's 64 candidates (same arithmetic as k_knn<0>)
#pragma unroll
  for (int i = 0; i < QPW; ++i) {
    const int64_t slot = group * QPW + i;
    const int q = qrow[slot];
    if (q < 0) continue;
    uint64_t key = kInf;
    if (top[i] != kInf) {
      const int64_t row = (int64_t)(uint32_t)top[i];
      float acc = 0.f;
      for (int64_t f = 0; f < d; ++f) {
        const float t = X[row * d + f] - X[(int64_t)q * d + f];
        acc = __builtin_fmaf(t, t, acc);
      }
      key = ((uint64_t)__builtin_bit_cast(uint32_t, acc) << 32) | (uint32_t)row;
    }
    key = sort64(key, lane);
    if (lane < K) {
      out_d[slot * K + lane] = key == kInf ? __builtin_inff() : __builtin_bit_cast(float, (uint32_t)(key >> 32));
      out_i[slot * K + lane] = key == kInf ? -1 : (int32_t)(uint32_t)key;
    }
  }
}

}  // namespace

// qrow/qsplit: [nq_groups * 8] (qrow -1 = padding); out_d/out_i: [nq_groups * 8, K], K <= 64.
// metric: 0 squared-L2, 1 L1, 2 Linf, 3 sum |t|^p.
extern "C" int dml_knn(const float* X, const float* XT, int64_t n, int64_t d, const uint8_t* roles,
                       const int32_t* qrow, const int32_t* qsplit, int64_t nq_groups, int32_t metric, float p,
                       int32_t K, float* out_d, int32_t* out_i, hipStream_t st) {
  if (K < 1 || K > 64 || nq_groups <= 0) return nq_groups == 0 ? 0 : 2;
  const unsigned blocks = (unsigned)((nq_groups + WAVES - 1) / WAVES);
  switch (metric) {
    case 0: k_knn<0><<<blocks, 64 * WAVES, 0, st>>>(X, XT, n, d, roles, qrow, qsplit, nq_groups, p, K, out_d, out_i); break;
    case 1: k_knn<1><<<blocks, 64 * WAVES, 0, st>>>(X, XT, n, d, roles, qrow, qsplit, nq_groups, p, K, out_d, out_i); break;
    case 2: k_knn<2><<<blocks, 64 * WAVES, 0, st>>>(X, XT, n, d, roles, qrow, qsplit, nq_groups, p, K, out_d, out_i); break;
    default: k_knn<3><<<blocks, 64 * WAVES, 0, st>>>(X, XT, n, d, roles, qrow, qsplit, nq_groups, p, K, out_d, out_i); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int dml_knn_qpw() { return QPW; }

// Squared-L2 search on the matrix cores (K <= 64; exact when the true K nearest are among
// the approximate 64 nearest -- the host keeps K <= 32).  XHL: [2][ks_n][npad][16] bf16,
// npad % 128 == 0 and >= n; rn: [n] squared row norms; qrow/qsplit: [nq_groups * 8] with
// nq_groups % 4 == 0 (a workgroup = 4 groups; padding groups use qrow -1).
extern "C" int dml_knn_l2_mfma(const void* XHL, int64_t npad, int32_t ks_n, const float* rn, const float* X, int64_t n,
                               int64_t d, const uint8_t* roles, const int32_t* qrow, const int32_t* qsplit,
                               int64_t nq_groups, int32_t K, float* out_d, int32_t* out_i, hipStream_t st) {
  if (nq_groups == 0) return 0;
  if (K < 1 || K > 64 || nq_groups % WAVES || npad % MR || npad < n || (int64_t)ks_n * 16 < d) return 2;
  const unsigned blocks = (unsigned)(nq_groups / WAVES);
  const __bf16* x = static_cast<const __bf16*>(XHL);
  switch (ks_n) {
    case 1: k_knn_l2_mfma<1><<<blocks, 256, 0, st>>>(x, npad, ks_n, rn, X, n, d, roles, qrow, qsplit, K, out_d, out_i); break;
    case 2: k_knn_l2_mfma<2><<<blocks, 256, 0, st>>>(x, npad, ks_n, rn, X, n, d, roles, qrow, qsplit, K, out_d, out_i); break;
    case 4: k_knn_l2_mfma<4><<<blocks, 256, 0, st>>>(x, npad, ks_n, rn, X, n, d, roles, qrow, qsplit, K, out_d, out_i); break;
    case 8: k_knn_l2_mfma<8><<<blocks, 256, 0, st>>>(x, npad, ks_n, rn, X, n, d, roles, qrow, qsplit, K, out_d, out_i); break;
    default: k_knn_l2_mfma<0><<<blocks, 256, 0, st>>>(x, npad, ks_n, rn, X, n, d, roles, qrow, qsplit, K, out_d, out_i); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
