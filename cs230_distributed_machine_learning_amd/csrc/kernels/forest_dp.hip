// forest_dp.hip — kernels of the row-sharded (data-parallel) forest builder.
//
// The level loop, the per-level histogram all-reduce (RCCL) and the pair compaction run
// in ops/forest_dp.py; every decision is the shared code of forest_dp.h, so the C++
// twin (../runtime/forest_dp_cpu.cpp) and these kernels grow identical trees.
//
// Hot op: the node histograms of a level over this rank's rows.  The (tree, row) pairs
// of the open nodes are kept sorted by node, so every node is one contiguous segment:
//   * a segment of >= kDpSmall pairs is cut into tiles of tile_rows pairs; one 256-thread
//     workgroup per tile privatises the tile's [positions][channels][256] histogram in LDS
//     (lds_feats positions per pass; the tile's rows stay in L2 across passes) and flushes
//     the non-zero bins with one global atomic each;
//   * smaller segments (the many small nodes of deep levels) go straight to global
//     atomics, one wave per node -- an LDS zero + flush of 256 x CH x KR words would cost
//     more than the node's own updates.
// Classification histograms are uint32 (bootstrap weight per class + row count): exact,
// so the sum over ranks is exact and order-independent.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "forest_dp.h"
#include "wave_ops.h"

namespace dml {

constexpr int kDpBlock = 256;

// (tree, local row) -> bootstrap weight (0: not a training row of the tree's split)
__global__ void k_dp_weights(DpArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.T * a.n) return;
  const int t = (int)(idx / a.n);
  const int64_t r = idx - (int64_t)t * a.n;
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[t];
  const uint8_t role = dp_ptr<const uint8_t>(a.roles)[(int64_t)s.split * a.n + r];
  uint32_t w = role == 1 ? boot_weight(s, (uint32_t)(a.r0 + r)) : 0u;
  dp_ptr<uint8_t>(a.wts)[idx] = (uint8_t)(w > 255u ? 255u : w);
}

// local root statistics [T][CH] (doubles; classification sums are integers, exact)
__global__ void k_dp_root_stats(DpArgs a) {
  const int t = blockIdx.y;
  const int CH = (int)a.CH;
  const uint8_t* w8 = dp_ptr<const uint8_t>(a.wts) + (int64_t)t * a.n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (!a.is_reg) {
    // per-lane integer counts in LDS (uint64 atomics are exact)
    __shared__ unsigned long long cnt[kMaxClasses + 1];
    for (int c = threadIdx.x; c < CH; c += blockDim.x) cnt[c] = 0ull;
    __syncthreads();
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
      const uint32_t w = w8[r];
      if (!w) continue;
      atomicAdd(&cnt[dp_ptr<const int32_t>(a.ycls)[r]], (unsigned long long)w);
      atomicAdd(&cnt[CH - 1], 1ull);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < CH; c += blockDim.x)
      if (cnt[c]) atomicAdd(dp_ptr<double>(a.root) + (int64_t)t * CH + c, (double)cnt[c]);
    return;
  }
  // regression: exact integer sums {w, w yq, w y2q, rows} (forest_common.h)
  __shared__ unsigned long long racc[4];
  if (threadIdx.x < 4) racc[threadIdx.x] = 0ull;
  __syncthreads();
  const RegScale q = reg_scale((int)a.yq_e1, (int)a.yq_e2);
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
    const uint32_t w = w8[r];
    if (!w) continue;
    int64_t yq, y2q;
    reg_quantize(dp_target(a, t, r), q, yq, y2q);
    atomicAdd(&racc[0], (unsigned long long)w);
    atomicAdd(&racc[1], (unsigned long long)((int64_t)w * yq));
    atomicAdd(&racc[2], (unsigned long long)((int64_t)w * y2q));
    atomicAdd(&racc[3], 1ull);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 4; c += blockDim.x)
    if (racc[c]) atomicAdd(dp_ptr<unsigned long long>(a.root) + (int64_t)t * 4 + c, racc[c]);
}

__global__ void k_dp_roots(DpArgs a) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.T) return;
  DpSlot sl;
  const int open = dp_root_one(a, t, &sl);
  dp_ptr<DpSlot>(a.next)[t] = sl;
  dp_ptr<int32_t>(a.next_open)[t] = open;
}

// feature of every (searching slot, position) of the round
__global__ void k_dp_feats(DpArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.S * a.KR) return;
  const int s = (int)(idx / a.KR), k = (int)(idx - (int64_t)s * a.KR);
  const DpSlot& sl = dp_ptr<const DpSlot>(a.slots)[dp_ptr<const int32_t>(a.srch)[s]];
  const int p = sl.pos + k;
  dp_ptr<int32_t>(a.feats)[idx] = p < a.d ? feature_at(feat_perm(sl.key, (int)a.d), p, (int)a.d) : -1;
}

// a regression row's three integer histogram terms
struct DpRegRow {
  unsigned long long wr, wy, wyy;
};
__device__ __forceinline__ DpRegRow dp_reg_row(const DpArgs& a, uint32_t w, float fy) {
  int64_t yq, y2q;
  reg_quantize(fy, reg_scale((int)a.yq_e1, (int)a.yq_e2), yq, y2q);
  DpRegRow t;
  t.wr = (unsigned long long)w | (1ull << 32);
  t.wy = (unsigned long long)((int64_t)w * yq);
  t.wyy = (unsigned long long)((int64_t)w * y2q);
  return t;
}

template <bool kReg>
__device__ __forceinline__ void dp_row(const DpArgs& a, int64_t p, int32_t& r, uint32_t& w, int32_t& y, float& fy) {
  r = dp_ptr<const int32_t>(a.act_row)[p];
  const int t = dp_ptr<const int32_t>(a.act_tree)[p];
  w = boot_weight(dp_ptr<const TreeSpec>(a.specs)[t], (uint32_t)(a.r0 + r));
  if (kReg) fy = dp_target(a, t, r);
  else y = dp_ptr<const int32_t>(a.ycls)[r];
}

// LDS-privatised histogram of one tile of a large segment
template <bool kReg>
__global__ void __launch_bounds__(kDpBlock) k_dp_hist_tiles(DpArgs a) {
  extern __shared__ uint32_t lds[];
  const int tile = blockIdx.x;
  const int s = dp_ptr<const int32_t>(a.tile_s)[tile];
  const int slot = dp_ptr<const int32_t>(a.srch)[s];
  const int64_t off = dp_ptr<const int64_t>(a.tile_off)[tile];
  const int64_t seg0 = dp_ptr<const int64_t>(a.seg_start)[slot] + off;
  const int64_t cnt = min((int64_t)a.tile_rows, dp_ptr<const int64_t>(a.seg_cnt)[slot] - off);
  const int CH = (int)a.CH, C = (int)a.C, KR = (int)a.KR, G = (int)a.lds_feats;
  const int32_t* fs = dp_ptr<const int32_t>(a.feats) + (int64_t)s * KR;
  const uint8_t* Xb = dp_ptr<const uint8_t>(a.Xb);
  uint32_t* gh = dp_ptr<uint32_t>(a.hist) + (int64_t)s * dp_hist_words(a);
  unsigned long long* ldr = (unsigned long long*)lds;   // regression: [ng][3][256] u64
  for (int g0 = 0; g0 < KR; g0 += G) {
    const int ng = min(G, KR - g0);
    const int words = kReg ? ng * 3 * 256 * 2 : ng * CH * 256;
    for (int j = threadIdx.x; j < words; j += kDpBlock) lds[j] = 0u;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < cnt; i += kDpBlock) {
      int32_t r, y = 0;
      uint32_t w;
      float fy = 0.f;
      dp_row<kReg>(a, seg0 + i, r, w, y, fy);
      const uint8_t* xr = Xb + (int64_t)r * a.ld;
      DpRegRow q{};
      if (kReg) q = dp_reg_row(a, w, fy);
      for (int k = 0; k < ng; ++k) {
        const int f = fs[g0 + k];
        if (f < 0) break;
        const int b = xr[f];
        if (kReg) {
          unsigned long long* h = ldr + (k * 3) * 256 + b;
          atomicAdd(h, q.wr);
          atomicAdd(h + 256, q.wy);
          atomicAdd(h + 512, q.wyy);
        } else {
          atomicAdd(&lds[(k * CH + y) * 256 + b], w);
          atomicAdd(&lds[(k * CH + C) * 256 + b], 1u);
        }
      }
    }
    __syncthreads();
    if (kReg) {
      unsigned long long* dst = (unsigned long long*)gh + (int64_t)g0 * 3 * 256;
      for (int j = threadIdx.x; j < ng * 3 * 256; j += kDpBlock)
        if (ldr[j]) atomicAdd(dst + j, ldr[j]);
    } else {
      uint32_t* dst = gh + (int64_t)g0 * CH * 256;
      for (int j = threadIdx.x; j < words; j += kDpBlock) {
        const uint32_t v = lds[j];
        if (v) atomicAdd(dst + j, v);
      }
    }
    __syncthreads();
  }
}

// small segments: one wave per node, global atomics, lanes over (pair, position)
template <bool kReg>
__global__ void __launch_bounds__(kDpBlock) k_dp_hist_small(DpArgs a) {
  const int wave = (int)(((int64_t)blockIdx.x * kDpBlock + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= a.n_small) return;
  const int s = dp_ptr<const int32_t>(a.small_s)[wave];
  const int slot = dp_ptr<const int32_t>(a.srch)[s];
  const int64_t seg0 = dp_ptr<const int64_t>(a.seg_start)[slot];
  const int64_t cnt = dp_ptr<const int64_t>(a.seg_cnt)[slot];
  const int CH = (int)a.CH, C = (int)a.C, KR = (int)a.KR;
  const int32_t* fs = dp_ptr<const int32_t>(a.feats) + (int64_t)s * KR;
  const uint8_t* Xb = dp_ptr<const uint8_t>(a.Xb);
  uint32_t* gh = dp_ptr<uint32_t>(a.hist) + (int64_t)s * dp_hist_words(a);
  for (int64_t i = lane; i < cnt; i += 64) {
    int32_t r, y = 0;
    uint32_t w;
    float fy = 0.f;
    dp_row<kReg>(a, seg0 + i, r, w, y, fy);
    const uint8_t* xr = Xb + (int64_t)r * a.ld;
    DpRegRow q{};
    if (kReg) q = dp_reg_row(a, w, fy);
    for (int k = 0; k < KR; ++k) {
      const int f = fs[k];
      if (f < 0) break;
      const int b = xr[f];
      if (kReg) {
        unsigned long long* h = (unsigned long long*)gh + (k * 3) * 256 + b;
        atomicAdd(h, q.wr);
        atomicAdd(h + 256, q.wy);
        atomicAdd(h + 512, q.wyy);
      } else {
        atomicAdd(&gh[(k * CH + y) * 256 + b], w);
        atomicAdd(&gh[(k * CH + C) * 256 + b], 1u);
      }
    }
  }
}

// one thread per searching slot: the sequential feature search of forest_dp.h
__global__ void k_dp_split(DpArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.S) return;
  const int slot = dp_ptr<const int32_t>(a.srch)[s];
  DpSlot sl = dp_ptr<DpSlot>(a.slots)[slot];
  const int64_t hw = dp_hist_words(a);
  dp_eval_slot(a, sl, dp_ptr<double>(a.best_left) + (int64_t)slot * a.CH, dp_ptr<const uint32_t>(a.hist) + s * hw,
               dp_ptr<const int32_t>(a.feats) + (int64_t)s * a.KR);
  dp_ptr<DpSlot>(a.slots)[slot] = sl;
}

// classification: one WAVE per searching slot, each lane owning 4 bins.  Integer prefix
// sums by DPP wave scan (exact, so the same sums as the sequential loop), the same
// per-bin gain code, and an argmax ordered (gain desc, bin asc) -- the sequential loop's
// "first strictly-better bin" -- so the decisions equal dp_eval_slot's.
template <int CHMAX>
__global__ void __launch_bounds__(kDpBlock) k_dp_split_wave(DpArgs a) {
  const int s = (int)(((int64_t)blockIdx.x * kDpBlock + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= a.S) return;
  const int slot = dp_ptr<const int32_t>(a.srch)[s];
  DpSlot sl = dp_ptr<const DpSlot>(a.slots)[slot];
  const TreeSpec& sp = dp_ptr<const TreeSpec>(a.specs)[sl.tree];
  const int C = (int)a.C, CH = (int)a.CH, KR = (int)a.KR, d = (int)a.d;
  const double* cwv = dp_cwv(a, sl.tree);
  double* bl = dp_ptr<double>(a.best_left) + (int64_t)slot * CH;
  const uint32_t* h = dp_ptr<const uint32_t>(a.hist) + (int64_t)s * KR * CH * 256;
  const int32_t* fs = dp_ptr<const int32_t>(a.feats) + (int64_t)s * KR;
  const uint32_t msl = (uint32_t)sp.min_samples_leaf;
  for (int k = 0; k < KR && !sl.done; ++k) {
    const int feat = fs[k];
    if (feat < 0) {
      sl.done = 1;
      break;
    }
    sl.pos += 1;
    uint32_t pre[CHMAX][4], tot[CHMAX];
#pragma unroll
    for (int ch = 0; ch < CHMAX; ++ch) {
      if (ch >= CH) break;
      const uint4 v = ((const uint4*)(h + ((int64_t)k * CH + ch) * 256))[lane];
      const uint32_t c0 = v.x, c1 = c0 + v.y, c2 = c1 + v.z, c3 = c2 + v.w;
      const uint32_t incl = wave::incl_scan<uint32_t>(c3), ex = incl - c3;
      pre[ch][0] = ex + c0; pre[ch][1] = ex + c1; pre[ch][2] = ex + c2; pre[ch][3] = ex + c3;
      tot[ch] = wave::bcast<uint32_t>(incl, 63);
    }
    double best = -INFINITY;
    int bb = -1;
    bool nc = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = lane * 4 + i;
      if (b == 255) break;
      uint32_t rl = 0, rt = 0;
#pragma unroll
      for (int ch = 0; ch < CHMAX; ++ch)
        if (ch == C) { rl = pre[ch][i]; rt = tot[ch]; }
      const uint32_t rr = rt - rl;
      nc |= (rl > 0 && rr > 0);
      if (rl < msl || rr < msl) continue;
      ClsAcc L, R;
      L.init(sp.criterion);
      R.init(sp.criterion);
#pragma unroll
      for (int c = 0; c < CHMAX; ++c) {
        if (c >= C) break;
        const double cw = cwv ? cwv[c] : 1.0;
        const double lc = (double)pre[c][i] * cw, tc = (double)tot[c] * cw;
        L.add(lc);
        R.add(tc - lc);
      }
      if (side_too_light(sp, L.w, R.w)) continue;
      const double g = cls_proxy(L, R, sp.criterion);
      if (g > best) {
        best = g;
        bb = b;
      }
    }
    wave::argmax(best, bb, lane);
    if (__ballot(nc) != 0ull) {
      sl.nonconst += 1;
      if (bb >= 0 && best > sl.best_gain) {
        sl.best_gain = best;
        sl.best_feat = feat;
        sl.best_bin = bb;
        const int src = bb >> 2, sel = bb & 3;
#pragma unroll
        for (int ch = 0; ch < CHMAX; ++ch) {
          if (ch >= CH) break;
          const uint32_t mine = sel == 0 ? pre[ch][0] : sel == 1 ? pre[ch][1] : sel == 2 ? pre[ch][2] : pre[ch][3];
          const uint32_t cv = wave::bcast<uint32_t>(mine, src);
          if (lane == 0) bl[ch] = (double)cv * ((ch < C && cwv) ? cwv[ch] : 1.0);
        }
      }
    }
    if (sl.nonconst >= sp.max_features || sl.pos >= d) sl.done = 1;
  }
  if (lane == 0) dp_ptr<DpSlot>(a.slots)[slot] = sl;
}

__global__ void k_dp_accept(DpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.S_open) return;
  DpSlot* sl = dp_ptr<DpSlot>(a.slots) + i;
  sl->split = dp_accept_one(a, *sl, dp_ptr<const double>(a.best_left) + (int64_t)i * a.CH);
}

__global__ void k_dp_children(DpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.S_open) dp_children_one(a, i);
}

__global__ void k_dp_partition(DpArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.A) dp_ptr<int32_t>(a.new_node)[i] = dp_partition_one(a, i);
}

// smallest right-going bin of every node over this rank's training rows (one thread
// per (tree, local row); the MIN over ranks is an all-reduce in ops/forest_dp.py)
__global__ void k_dp_refine_hi(DpArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.T * a.n) return;
  const int t = (int)(idx / a.n);
  const int64_t r = idx - (int64_t)t * a.n;
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[t];
  if (dp_ptr<const uint8_t>(a.roles)[(int64_t)s.split * a.n + r] != 1 || boot_weight(s, (uint32_t)(a.r0 + r)) == 0) return;
  const uint8_t* xr = dp_ptr<const uint8_t>(a.Xb) + r * a.ld;
  const NodeRec* nodes = dp_ptr<const NodeRec>(a.nodes);
  uint32_t* hi = dp_ptr<uint32_t>(a.hi);
  int node = t;
  NodeRec nr = nodes[node];
  while (nr.split >= 0) {
    const uint32_t b = xr[nr.split >> 8];
    if (b > (uint32_t)(nr.split & 255)) {
      atomicMin(hi + node, b);
      node = nr.left + 1;
    } else {
      node = nr.left;
    }
    nr = nodes[node];
  }
}

__global__ void k_dp_refine_apply(DpArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.P_total) dp_refine_one(a, i);
}

static unsigned blocks(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace dml

using namespace dml;

extern "C" {

int dml_dp_sizeof_args() { return (int)sizeof(DpArgs); }
int dml_dp_sizeof_slot() { return (int)sizeof(DpSlot); }

// step: 0 weights, 1 root stats, 2 roots, 3 feats, 4 hist, 5 split, 6 accept,
//       7 children, 8 partition, 9 refine hi, 10 refine apply
int dml_dp_step(const DpArgs* a, int step, hipStream_t st) {
  switch (step) {
    case 0:
      if (a->T * a->n > 0) k_dp_weights<<<blocks(a->T * a->n, kDpBlock), kDpBlock, 0, st>>>(*a);
      break;
    case 1: {
      if (a->n <= 0 || a->T <= 0) break;
      const unsigned gx = (unsigned)std::min<int64_t>(blocks(a->n, kDpBlock), 64);
      k_dp_root_stats<<<dim3(gx, (unsigned)a->T), kDpBlock, 0, st>>>(*a);
      break;
    }
    case 2:
      if (a->T > 0) k_dp_roots<<<blocks(a->T, 64), 64, 0, st>>>(*a);
      break;
    case 3:
      if (a->S * a->KR > 0) k_dp_feats<<<blocks(a->S * a->KR, kDpBlock), kDpBlock, 0, st>>>(*a);
      break;
    case 4: {
      const size_t lds = (size_t)a->lds_feats * 256 * (a->is_reg ? 3 * 8 : a->CH * 4);
      if (a->n_tiles > 0) {
        if (a->lds_feats <= 0 || lds > 65536) return 2;
        if (a->is_reg) k_dp_hist_tiles<true><<<(unsigned)a->n_tiles, kDpBlock, lds, st>>>(*a);
        else k_dp_hist_tiles<false><<<(unsigned)a->n_tiles, kDpBlock, lds, st>>>(*a);
      }
      if (a->n_small > 0) {
        const unsigned g = blocks(a->n_small * 64, kDpBlock);
        if (a->is_reg) k_dp_hist_small<true><<<g, kDpBlock, 0, st>>>(*a);
        else k_dp_hist_small<false><<<g, kDpBlock, 0, st>>>(*a);
      }
      break;
    }
    case 5:
      if (a->S <= 0) break;
      if (!a->is_reg && a->CH <= 3) k_dp_split_wave<3><<<blocks(a->S * 64, kDpBlock), kDpBlock, 0, st>>>(*a);
      else if (!a->is_reg && a->CH <= 9) k_dp_split_wave<9><<<blocks(a->S * 64, kDpBlock), kDpBlock, 0, st>>>(*a);
      else k_dp_split<<<blocks(a->S, 64), 64, 0, st>>>(*a);   // regression (fp32 bin order) / many classes
      break;
    case 6:
      if (a->S_open > 0) k_dp_accept<<<blocks(a->S_open, 64), 64, 0, st>>>(*a);
      break;
    case 7:
      if (a->S_open > 0) k_dp_children<<<blocks(a->S_open, 64), 64, 0, st>>>(*a);
      break;
    case 8:
      if (a->A > 0) k_dp_partition<<<blocks(a->A, kDpBlock), kDpBlock, 0, st>>>(*a);
      break;
    case 9:
      if (a->T * a->n > 0) k_dp_refine_hi<<<blocks(a->T * a->n, kDpBlock), kDpBlock, 0, st>>>(*a);
      break;
    case 10:
      if (a->P_total > 0) k_dp_refine_apply<<<blocks(a->P_total, kDpBlock), kDpBlock, 0, st>>>(*a);
      break;
    default:
      return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
