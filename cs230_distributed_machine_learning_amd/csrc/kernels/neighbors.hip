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
