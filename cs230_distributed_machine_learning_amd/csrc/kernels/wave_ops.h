// wave_ops.h — wave64 cross-lane primitives for gfx950 without LDS round trips.
//
// hipcc lowers __shfl_xor / __shfl_up to ds_bpermute_b32 (an LDS-pipe instruction
// with LDS latency).  The tree kernels are chains of such exchanges (bitonic sorts,
// prefix scans, argmax reductions), so each step here is a VALU instruction instead:
//   xor 1, 2      DPP quad_perm
//   xor 4, 8      DPP row_shl/row_shr (+ select)
//   xor 16, 32    v_permlane16_swap / v_permlane32_swap (gfx950)
//   scans         DPP row_shr:1,2,4,8 + row_bcast:15 + row_bcast:31 (wave64 GCN idiom)
//   shift by 1    DPP wave_shr:1 / wave_shl:1
//   broadcast     v_readlane (uniform source lane)
// tests/test_forest_gpu.py checks every primitive against the ds_bpermute versions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dml {
namespace wave {

constexpr int kQuadXor1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int kRowShl = 0x100;    // + n: lane i <- lane i+n within a 16-lane row
constexpr int kRowShr = 0x110;    // + n: lane i <- lane i-n within a 16-lane row
constexpr int kWaveShl1 = 0x130;  // lane i <- lane i+1 across the wave
constexpr int kWaveShr1 = 0x138;  // lane i <- lane i-1 across the wave
constexpr int kRowBcast15 = 0x142;
constexpr int kRowBcast31 = 0x143;

__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

template <int CTRL, int ROW_MASK = 0xF, bool BOUND_ZERO = true>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, BOUND_ZERO);
}

// value of lane (lane ^ MASK), 32-bit payload
template <int MASK>
__device__ __forceinline__ uint32_t xor32(uint32_t v, int lane) {
  if constexpr (MASK == 1) {
    return dpp<kQuadXor1>(v);
  } else if constexpr (MASK == 2) {
    return dpp<kQuadXor2>(v);
  } else if constexpr (MASK == 4 || MASK == 8) {
    const uint32_t up = dpp<kRowShl + MASK>(v);   // from lane + MASK
    const uint32_t dn = dpp<kRowShr + MASK>(v);   // from lane - MASK
    return (lane & MASK) ? dn : up;
  } else if constexpr (MASK == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((lane >> 4) & 1) ? r[0] : r[1];
  } else {
    static_assert(MASK == 32, "xor mask must be a power of two < 64");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return lane >= 32 ? r[0] : r[1];
  }
}

template <int MASK, typename T>
__device__ __forceinline__ T shfl_xor(T v, int lane) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit payloads only");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, xor32<MASK>(__builtin_bit_cast(uint32_t, v), lane));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = xor32<MASK>((uint32_t)u, lane), hi = xor32<MASK>((uint32_t)(u >> 32), lane);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

// broadcast from a wave-uniform lane
template <typename T>
__device__ __forceinline__ T bcast(T v, int src_lane) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint32_t, v), src_lane));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src_lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src_lane);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

// value of a per-lane source lane (ds_bpermute), 32/64-bit payloads
template <typename T>
__device__ __forceinline__ T bcast_lane(T v, int src_lane) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, (uint32_t)__shfl((int)__builtin_bit_cast(uint32_t, v), src_lane));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)u, src_lane), hi = (uint32_t)__shfl((int)(uint32_t)(u >> 32), src_lane);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

// lane i <- lane i+1 (lane 63 gets `fill`)
template <typename T>
__device__ __forceinline__ T shift_down1(T v, int lane, T fill) {
  static_assert(sizeof(T) == 4, "32-bit payloads only");
  const T r = __builtin_bit_cast(T, dpp<kWaveShl1>(__builtin_bit_cast(uint32_t, v)));
  return lane == 63 ? fill : r;
}

// inclusive prefix sum over the wave (integer or float 32-bit)
template <typename T>
__device__ __forceinline__ T incl_scan(T v) {
  static_assert(sizeof(T) == 4, "32-bit payloads only");
  auto add = [](T a, uint32_t b) { return a + __builtin_bit_cast(T, b); };
  v = add(v, dpp<kRowShr + 1>(__builtin_bit_cast(uint32_t, v)));
  v = add(v, dpp<kRowShr + 2>(__builtin_bit_cast(uint32_t, v)));
  v = add(v, dpp<kRowShr + 4>(__builtin_bit_cast(uint32_t, v)));
  v = add(v, dpp<kRowShr + 8>(__builtin_bit_cast(uint32_t, v)));
  v = add(v, dpp<kRowBcast15, 0xA>(__builtin_bit_cast(uint32_t, v)));
  v = add(v, dpp<kRowBcast31, 0xC>(__builtin_bit_cast(uint32_t, v)));
  return v;
}

// 64-bit unsigned inclusive prefix sum (packed histogram planes)
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t scan_step_u64(uint64_t x) {
  const uint32_t lo = dpp<CTRL, RM>((uint32_t)x), hi = dpp<CTRL, RM>((uint32_t)(x >> 32));
  return x + (((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint64_t incl_scan_u64(uint64_t v) {
  v = scan_step_u64<kRowShr + 1, 0xF>(v);
  v = scan_step_u64<kRowShr + 2, 0xF>(v);
  v = scan_step_u64<kRowShr + 4, 0xF>(v);
  v = scan_step_u64<kRowShr + 8, 0xF>(v);
  v = scan_step_u64<kRowBcast15, 0xA>(v);
  v = scan_step_u64<kRowBcast31, 0xC>(v);
  return v;
}

// exclusive = inclusive shifted by one lane (lane 0 gets 0)
template <typename T>
__device__ __forceinline__ T excl_from_incl(T incl) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp<kWaveShr1>(__builtin_bit_cast(uint32_t, incl)));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, incl);
    const uint32_t lo = dpp<kWaveShr1>((uint32_t)u), hi = dpp<kWaveShr1>((uint32_t)(u >> 32));
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

// ascending bitonic sort of 64 keys, one per lane (ties impossible: callers put the
// lane id in the low bits)
__device__ __forceinline__ uint32_t bitonic64(uint32_t key, int lane) {
#define DML_BITONIC_STEP(K, J)                                  \
  {                                                             \
    const uint32_t other = xor32<J>(key, lane);                 \
    const bool up = (lane & (K)) == 0;                          \
    const bool lower = (lane & (J)) == 0;                       \
    const uint32_t mn = key < other ? key : other;              \
    const uint32_t mx = key < other ? other : key;              \
    key = (lower == up) ? mn : mx;                              \
  }
  DML_BITONIC_STEP(2, 1)
  DML_BITONIC_STEP(4, 2) DML_BITONIC_STEP(4, 1)
  DML_BITONIC_STEP(8, 4) DML_BITONIC_STEP(8, 2) DML_BITONIC_STEP(8, 1)
  DML_BITONIC_STEP(16, 8) DML_BITONIC_STEP(16, 4) DML_BITONIC_STEP(16, 2) DML_BITONIC_STEP(16, 1)
  DML_BITONIC_STEP(32, 16) DML_BITONIC_STEP(32, 8) DML_BITONIC_STEP(32, 4) DML_BITONIC_STEP(32, 2)
  DML_BITONIC_STEP(32, 1)
  DML_BITONIC_STEP(64, 32) DML_BITONIC_STEP(64, 16) DML_BITONIC_STEP(64, 8) DML_BITONIC_STEP(64, 4)
  DML_BITONIC_STEP(64, 2) DML_BITONIC_STEP(64, 1)
#undef DML_BITONIC_STEP
  return key;
}

// argmax over (gain desc, idx asc) — every lane ends with the same pair
__device__ __forceinline__ void argmax(double& g, int& idx, int lane) {
#define DML_ARGMAX_STEP(M)                                           \
  {                                                                  \
    const double og = shfl_xor<M>(g, lane);                          \
    const int oi = shfl_xor<M>(idx, lane);                           \
    if (og > g || (og == g && (unsigned)oi < (unsigned)idx)) {       \
      g = og;                                                        \
      idx = oi;                                                      \
    }                                                                \
  }
  DML_ARGMAX_STEP(32) DML_ARGMAX_STEP(16) DML_ARGMAX_STEP(8) DML_ARGMAX_STEP(4) DML_ARGMAX_STEP(2)
  DML_ARGMAX_STEP(1)
#undef DML_ARGMAX_STEP
}

__device__ __forceinline__ uint64_t min_u64(uint64_t v, int lane) {
#define DML_MIN_STEP(M)                              \
  {                                                  \
    const uint64_t o = shfl_xor<M>(v, lane);         \
    v = o < v ? o : v;                               \
  }
  DML_MIN_STEP(32) DML_MIN_STEP(16) DML_MIN_STEP(8) DML_MIN_STEP(4) DML_MIN_STEP(2) DML_MIN_STEP(1)
#undef DML_MIN_STEP
  return v;
}

// float max over the wave (every lane ends with it)
__device__ __forceinline__ float max_f32(float v, int lane) {
  v = fmaxf(v, shfl_xor<32>(v, lane)); v = fmaxf(v, shfl_xor<16>(v, lane)); v = fmaxf(v, shfl_xor<8>(v, lane));
  v = fmaxf(v, shfl_xor<4>(v, lane)); v = fmaxf(v, shfl_xor<2>(v, lane)); v = fmaxf(v, shfl_xor<1>(v, lane));
  return v;
}

template <typename T>
__device__ __forceinline__ T sum(T v, int lane) {
  v += shfl_xor<32>(v, lane); v += shfl_xor<16>(v, lane); v += shfl_xor<8>(v, lane);
  v += shfl_xor<4>(v, lane); v += shfl_xor<2>(v, lane); v += shfl_xor<1>(v, lane);
  return v;
}

}  // namespace wave
}  // namespace dml
