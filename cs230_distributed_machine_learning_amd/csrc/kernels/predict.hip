// predict.hip — batched forest inference and fused per-fit scoring (K6 + K10).
//
// The reference predicts once per fit and scores with sklearn metrics
// (aws-prod/worker/worker.py:322-323 accuracy, :336-338 r2/mse, and inside
// cross_val_score :326/:341).  Here one launch predicts the held-out rows of EVERY
// fit of a batch (grid.y = fit), each thread walking all trees of its fit for one
// row against the HBM-resident binned matrix; a second launch reduces per-fit score
// statistics (correct count / SSE / sum y / sum y^2) so the host gets F x 4 doubles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

// int64 argument fields -> GLOBAL address-space pointers (flat loads otherwise)
#define GPTR(T, v) ((T*)(__attribute__((address_space(1))) T*)(uintptr_t)(v))
#include "forest_common.h"

namespace dml {

struct PredictArgs {
  int64_t Xb, ld;
  int64_t nodes, node_val, VC, is_reg, n_classes;
  int64_t fit_tree_off;  // int32[F+1]: trees of fit f are [off[f], off[f+1]) (tree t's root = node t)
  int64_t fit_row_off;   // int64[F+1]: rows of fit f in rows[] are [off[f], off[f+1])
  int64_t rows;          // int32[]: row indices to predict
  int64_t out_pred;      // int32 class id (cls) or float (reg), aligned with rows[]
  int64_t out_proba;     // float [len(rows)][C] or 0
  int64_t F, max_rows;
  int64_t d;          // features (bins per row actually read)
  int64_t lds_pitch;  // set by dml_forest_predict: LDS row stride, 0 = no staging
  int64_t fit_row_off_host;   // optional host copy of fit_row_off (per-fit grid sizes)
  int64_t fit_skip;           // optional int32[F] device mask: fits already predicted (early) are skipped
  int64_t fit_depth_cap;      // optional int32[F]: fit f reads its trees only down to this depth (<= 0: all);
                              // prefix fits of a deeper grown forest (models/base.py prefix_groups)
  int64_t toptab;             // optional NodeRec[trees][kTopSlots]: every tree's first kTopLv levels in heap
                              // order (k_top_fill), walked from LDS; 0 = every level from the node pool
  int64_t max_trees;          // max trees of one fit (k_top_fill grid)
};

// The first kTopLv levels of a tree are shared by every row that walks it: they are
// gathered once per predict into a heap-ordered table (slot s: children 2s+1 / 2s+2;
// a slot under a leaf holds {-1, -1}), and a block copies the table of the U trees it is
// walking into LDS with one coalesced read.  Those levels then cost LDS reads instead of
// dependent 8-B gathers through TA / L2 (the walk's first levels are L2 hits, so the
// saving is address-processing and latency, not HBM bytes).
#ifndef DML_PRED_TOP_LV
#define DML_PRED_TOP_LV 7
#endif
constexpr int kTopLv = DML_PRED_TOP_LV;
constexpr int kTopSlots = 1 << kTopLv;   // 2^kTopLv - 1 used + 1 pad
static_assert(kTopLv >= 1 && kTopSlots <= 256, "ops/forest_ops.py TOP_SLOTS_MAX allocates 256 slots per tree");

// leaf of U consecutive trees [t0, t0 + u_n) for one row, walked in lock-step: the U
// dependent node-load chains are independent, so U requests are in flight per thread
// instead of one (tree traversal is latency-bound)
// top (LDS, [kPredU][kTopSlots]) or nullptr: the group's top-level table (see kTopLv)
template <int kPredU>
__device__ __forceinline__ void leaves_u(const NodeRec* __restrict__ nodes, const uint8_t* __restrict__ xr, int t0,
                                         int u_n, int (&leaf)[kPredU], int cap, const NodeRec* top) {
  NodeRec nr[kPredU];
  int sl[kPredU];
#pragma unroll
  for (int u = 0; u < kPredU; ++u) {
    leaf[u] = t0 + u;
    sl[u] = 0;
    nr[u] = u < u_n ? (top ? top[u * kTopSlots] : nodes[leaf[u]]) : NodeRec{-1, -1};
  }
  for (int steps = 0; steps < cap; ++steps) {   // step s: every unfinished tree at depth s
    bool any = false;
#pragma unroll
    for (int u = 0; u < kPredU; ++u) any |= nr[u].split >= 0;
    if (!any) break;
    if (top && steps + 1 < kTopLv) {   // depth steps + 1 is in the LDS table (uniform branch)
#pragma unroll
      for (int u = 0; u < kPredU; ++u) {
        if (nr[u].split >= 0) {
          const int b = xr[nr[u].split >> 8] > (nr[u].split & 255) ? 1 : 0;
          leaf[u] = nr[u].left + b;
          sl[u] = 2 * sl[u] + 1 + b;
          nr[u] = top[u * kTopSlots + sl[u]];
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < kPredU; ++u) {
        if (nr[u].split >= 0) {
          leaf[u] = nr[u].left + (xr[nr[u].split >> 8] > (nr[u].split & 255) ? 1 : 0);
          nr[u] = nodes[leaf[u]];
        }
      }
    }
  }
}

// the top-level table of every tree of the launch's fits: one wave per tree, one level per
// round (lane i < 2^l fills slot 2^l - 1 + i from its parent's record)
__global__ __launch_bounds__(256) void k_top_fill(PredictArgs a) {
  __shared__ NodeRec recs[4][kTopSlots];
  const int f = blockIdx.y;
  if (a.fit_skip && (GPTR(const int32_t, a.fit_skip))[f]) return;
  const int32_t* toff = GPTR(const int32_t, a.fit_tree_off);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = toff[f] + (int)blockIdx.x * 4 + w;
  if (t >= toff[f + 1]) return;   // wave-uniform; the rounds below synchronise within the wave only
  const NodeRec* nodes = GPTR(const NodeRec, a.nodes);
  NodeRec* r = recs[w];
  if (lane == 0) r[0] = nodes[t];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int l = 1; l < kTopLv; ++l) {
    const int n = 1 << l;
    for (int i = lane; i < n; i += 64) {
      const int s = n - 1 + i;
      const NodeRec pr = r[(s - 1) >> 1];
      r[s] = pr.split >= 0 ? nodes[pr.left + ((s - 1) & 1)] : NodeRec{-1, -1};
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  NodeRec* out = GPTR(NodeRec, a.toptab) + (int64_t)t * kTopSlots;
  for (int s = lane; s < kTopSlots; s += 64) out[s] = s < kTopSlots - 1 ? r[s] : NodeRec{-1, -1};
}

// copy the top tables of trees [t, t + u_n) into LDS (block-wide; every thread of the block calls)
template <int kPredU>
__device__ __forceinline__ void load_top(const PredictArgs& a, NodeRec* top, int t, int u_n) {
  __syncthreads();   // the previous group's walks are done with the table
  const uint4* src = (const uint4*)(GPTR(const NodeRec, a.toptab) + (int64_t)t * kTopSlots);
  uint4* dst = (uint4*)top;
  for (int k = threadIdx.x; k < kPredU * kTopSlots / 2; k += 256)
    if (k < u_n * (kTopSlots / 2)) dst[k] = src[k];
  __syncthreads();
}

// depth cap of fit f (1 << 20: none)
__device__ __forceinline__ int depth_cap(const PredictArgs& a, int f) {
  const int c = a.fit_depth_cap ? (GPTR(const int32_t, a.fit_depth_cap))[f] : 0;
  return c > 0 ? c : 1 << 20;
}

// The block's 256 rows are staged in LDS once (dword stride odd -> a wave whose lanes
// read the same feature hits distinct banks), so the ~25 bin reads per tree walk are LDS
// reads and the only vector-memory traffic of the walk is the node-record chain.
// PredictArgs.lds_pitch = row stride in bytes (multiple of 4, <= ld), 0 = read bins from HBM.
__device__ __forceinline__ const uint8_t* stage_rows(const PredictArgs& a, uint8_t* xs, int64_t r0, int64_t nr) {
  const int P = (int)a.lds_pitch, W = P >> 2;
  const int64_t b0 = (int64_t)blockIdx.x * 256;
  __shared__ int32_t srow[256];
  const int64_t i = b0 + threadIdx.x;
  srow[threadIdx.x] = i < nr ? (GPTR(const int32_t, a.rows))[r0 + i] : -1;
  __syncthreads();
  const uint8_t* X = GPTR(const uint8_t, a.Xb);
  for (int k = threadIdx.x; k < 256 * W; k += 256) {
    const int r = k / W, w = k - r * W;
    const int32_t row = srow[r];
    if (row >= 0) ((uint32_t*)xs)[k] = *(const uint32_t*)(X + (int64_t)row * a.ld + 4 * w);
  }
  __syncthreads();
  return xs + threadIdx.x * P;
}

// byte offset of the top table in the dynamic LDS (after the staged rows, 16-B aligned)
__device__ __forceinline__ int64_t top_lds_off(const PredictArgs& a) { return (a.lds_pitch * 256 + 15) & ~15; }

template <int MAXC, int kPredU>
__global__ __launch_bounds__(256) void k_predict_cls(PredictArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t xs_lds[];
  const int f = blockIdx.y;
  if (a.fit_skip && (GPTR(const int32_t, a.fit_skip))[f]) return;
  const int32_t* toff = GPTR(const int32_t, a.fit_tree_off);
  const int64_t* roff = GPTR(const int64_t, a.fit_row_off);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = roff[f], nr = roff[f + 1] - r0;
  if ((int64_t)blockIdx.x * 256 >= nr) return;
  // with the top table every thread stays to the end (block-wide table loads); a thread
  // past the fit's rows walks nothing and writes nothing
  const bool live = i < nr;
  NodeRec* top = a.toptab ? (NodeRec*)(xs_lds + top_lds_off(a)) : nullptr;
  const uint8_t* xr;
  if (a.lds_pitch) {
    xr = stage_rows(a, xs_lds, r0, nr);
    if (!live && !top) return;
  } else {
    if (!live && !top) return;
    xr = GPTR(const uint8_t, a.Xb) + (int64_t)(GPTR(const int32_t, a.rows))[r0 + (live ? i : 0)] * a.ld;
  }
  const int C = (int)a.n_classes;
  const int cap = depth_cap(a, f);
  const NodeRec* nodes = GPTR(const NodeRec, a.nodes);
  const double* val = GPTR(const double, a.node_val);
  float p[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) p[k] = 0.f;
  const int tend = toff[f + 1];
  for (int t = toff[f]; t < tend; t += kPredU) {
    int leaf[kPredU];
    const int u_all = min(kPredU, tend - t), u_n = live ? u_all : 0;
    if (top) load_top<kPredU>(a, top, t, u_all);
    leaves_u<kPredU>(nodes, xr, t, u_n, leaf, cap, top);
    // accumulate in tree order (bit-identical to the host predictor)
#pragma unroll
    for (int u = 0; u < kPredU; ++u) {
      if (u >= u_n) break;
      const double* v = val + (int64_t)leaf[u] * a.VC;
      double W = 0.0;
#pragma unroll
      for (int k = 0; k < MAXC; ++k)
        if (k < C) W += v[k];
      if (W > 0.0) {
        const double inv = 1.0 / W;
#pragma unroll
        for (int k = 0; k < MAXC; ++k)
          if (k < C) p[k] += (float)(v[k] * inv);
      }
    }
  }
  if (!live) return;
  int best = 0;
  float bv = p[0];
#pragma unroll
  for (int k = 1; k < MAXC; ++k)
    if (k < C && p[k] > bv) { bv = p[k]; best = k; }
  (GPTR(int32_t, a.out_pred))[r0 + i] = best;
  if (a.out_proba) {
    const float nt = (float)(toff[f + 1] - toff[f]);
    float* op = GPTR(float, a.out_proba) + (r0 + i) * C;
#pragma unroll
    for (int k = 0; k < MAXC; ++k)
      if (k < C) op[k] = p[k] / nt;
  }
}

template <int kPredU>
__global__ __launch_bounds__(256) void k_predict_reg(PredictArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t xs_lds[];
  const int f = blockIdx.y;
  if (a.fit_skip && (GPTR(const int32_t, a.fit_skip))[f]) return;
  const int32_t* toff = GPTR(const int32_t, a.fit_tree_off);
  const int64_t* roff = GPTR(const int64_t, a.fit_row_off);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = roff[f], nr = roff[f + 1] - r0;
  if ((int64_t)blockIdx.x * 256 >= nr) return;
  // with the top table every thread stays to the end (block-wide table loads); a thread
  // past the fit's rows walks nothing and writes nothing
  const bool live = i < nr;
  NodeRec* top = a.toptab ? (NodeRec*)(xs_lds + top_lds_off(a)) : nullptr;
  const uint8_t* xr;
  if (a.lds_pitch) {
    xr = stage_rows(a, xs_lds, r0, nr);
    if (!live && !top) return;
  } else {
    if (!live && !top) return;
    xr = GPTR(const uint8_t, a.Xb) + (int64_t)(GPTR(const int32_t, a.rows))[r0 + (live ? i : 0)] * a.ld;
  }
  const NodeRec* nodes = GPTR(const NodeRec, a.nodes);
  const double* val = GPTR(const double, a.node_val);
  const int cap = depth_cap(a, f);
  double acc = 0.0;
  int nt = 0;
  const int tend = toff[f + 1];
  for (int t = toff[f]; t < tend; t += kPredU) {
    int leaf[kPredU];
    const int u_all = min(kPredU, tend - t), u_n = live ? u_all : 0;
    if (top) load_top<kPredU>(a, top, t, u_all);
    leaves_u<kPredU>(nodes, xr, t, u_n, leaf, cap, top);
#pragma unroll
    for (int u = 0; u < kPredU; ++u) {
      if (u >= u_n) break;
      const double* v = val + (int64_t)leaf[u] * a.VC;
      if (v[0] > 0.0) { acc += v[1] / v[0]; ++nt; }
    }
  }
  if (!live) return;
  (GPTR(float, a.out_pred))[r0 + i] = nt ? (float)(acc / nt) : 0.f;
}

// per-fit score statistics: out[f] = {match_count or SSE, sum y, sum y^2, n}
struct ScoreArgs {
  int64_t rows;        // int32[] row ids
  int64_t fit_row_off; // int64[F+1]
  int64_t pred;        // int32 (cls) / float (reg)
  int64_t ycls, yreg, is_reg;
  int64_t out;         // double [F][4]
  int64_t F;
};

__global__ __launch_bounds__(256) void k_scores(ScoreArgs a) {
  const int f = blockIdx.x;
  const int64_t* roff = GPTR(const int64_t, a.fit_row_off);
  const int64_t r0 = roff[f], r1 = roff[f + 1];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  const int32_t* rows = GPTR(const int32_t, a.rows);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
    const int32_t row = rows[i];
    if (a.is_reg) {
      const double y = (GPTR(const float, a.yreg))[row];
      const double e = (double)(GPTR(const float, a.pred))[i] - y;
      s0 += e * e; s1 += y; s2 += y * y;
    } else {
      s0 += (GPTR(const int32_t, a.pred))[i] == (GPTR(const int32_t, a.ycls))[row] ? 1.0 : 0.0;
    }
  }
  __shared__ double red[3][4];
  for (int off = 32; off >= 1; off >>= 1) {
    s0 += __shfl_xor(s0, off); s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = s0; red[1][w] = s1; red[2][w] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* o = GPTR(double, a.out) + 4 * f;
    o[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    o[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    o[2] = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    o[3] = (double)(r1 - r0);
  }
}

// leaf index of every row for every tree (boosting line search / raw-score update):
// leaf[t * n + row]; trees t = t0 .. t0+T-1 have their roots at node t.
__global__ __launch_bounds__(256) void k_apply(const uint8_t* __restrict__ Xb, int64_t ld, int64_t n,
                                               const NodeRec* __restrict__ nodes, int32_t t0,
                                               int32_t* __restrict__ leaf) {
  const int t = blockIdx.y;
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= n) return;
  const uint8_t* xr = Xb + row * ld;
  int node = t0 + t;
  NodeRec nr = nodes[node];
  for (int steps = 0; nr.split >= 0 && steps < 1 << 20; ++steps) {
    node = nr.left + (xr[nr.split >> 8] > (nr.split & 255) ? 1 : 0);
    nr = nodes[node];
  }
  leaf[(int64_t)t * n + row] = node;
}

// ---- sklearn-style split thresholds -------------------------------------------------
// A histogram split "bin <= b_lo" equals sklearn's "x <= (x_left_max + x_right_min) / 2"
// on the training rows; held-out rows between the two values are routed like sklearn
// only if the threshold sits at the midpoint.  For features whose bins are exact values
// (<= 256 distinct), pass 1 finds b_hi = min bin among each internal node's right-going
// in-bag training rows, pass 2 moves the split bin to the last bin value <= midpoint.
__global__ __launch_bounds__(256) void k_refine_hi(const uint8_t* __restrict__ Xb, int64_t ld, int64_t n,
                                                   const NodeRec* __restrict__ nodes,
                                                   const TreeSpec* __restrict__ specs,
                                                   const uint8_t* __restrict__ roles, uint32_t* hi) {
  const int t = blockIdx.y;
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= n) return;
  const TreeSpec& s = specs[t];
  if (roles[(int64_t)s.split * n + row] != 1 || boot_weight(s, (uint32_t)row) == 0) return;
  const uint8_t* xr = Xb + row * ld;
  int node = t;
  NodeRec nr = nodes[node];
  for (int steps = 0; nr.split >= 0 && steps < 1 << 20; ++steps) {
    const uint32_t b = xr[nr.split >> 8];
    if (b > (uint32_t)(nr.split & 255)) {
      if (b < hi[node]) atomicMin(&hi[node], b);
      node = nr.left + 1;
    } else {
      node = nr.left;
    }
    nr = nodes[node];
  }
}

__global__ __launch_bounds__(256) void k_refine_split(NodeRec* nodes, int64_t P, int64_t d, const uint32_t* __restrict__ hi,
                                                      const float* __restrict__ vals, const uint8_t* __restrict__ exact) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const NodeRec nr = nodes[i];
  if (nr.split < 0 || (nr.split >> 8) >= d) return;
  const int f = nr.split >> 8, blo = nr.split & 255;
  const uint32_t bhi = hi[i];
  if (!exact[f] || bhi > 255u || (int)bhi <= blo) return;
  const float* v = vals + (int64_t)f * 256;
  double m = (double)v[blo] / 2.0 + (double)v[bhi] / 2.0;
  if (m == (double)v[bhi] || !(m == m)) m = (double)v[blo];
  int b = blo;
  while (b + 1 < (int)bhi && (double)v[b + 1] <= m) ++b;
  nodes[i].split = f * 256 + b;
}

// U trees walked in lock-step per thread (memory-level parallelism of the dependent
// node-load chains); DML_PRED_U=4/16 select the other widths (A/B)
// LDS row stride for staged predict rows: whole dwords, odd dword count (conflict-free
// when the lanes of a wave read the same feature), within the row pitch; 0 disables
static int64_t predict_pitch(const PredictArgs* a) {
  static const bool off = getenv("DML_PRED_NO_STAGE") != nullptr;
  int64_t w = (a->d + 3) / 4;
  if ((w & 1) == 0) ++w;
  if (off || a->d <= 0 || 4 * ((a->d + 3) / 4) > a->ld || (a->ld & 3) || 256 * 4 * w > 64 * 1024) return 0;
  return 4 * w;
}

template <int U>
static int launch_predict(PredictArgs* a, hipStream_t st) {
  dim3 grid((unsigned)((a->max_rows + 255) / 256), (unsigned)a->F);
  a->lds_pitch = predict_pitch(a);
  size_t lds = (size_t)a->lds_pitch * 256;
  static const bool top_off = getenv("DML_PRED_NO_TOP") != nullptr;
  PredictArgs b = *a;   // the launch's copy: the top table only when it fits the LDS
  const size_t lds_top = ((lds + 15) & ~(size_t)15) + (size_t)U * kTopSlots * sizeof(NodeRec);
  if (top_off || lds_top > 64 * 1024 || a->max_trees <= 0) b.toptab = 0;
  if (b.toptab) {
    k_top_fill<<<dim3((unsigned)((b.max_trees + 3) / 4), (unsigned)b.F), 256, 0, st>>>(b);
    lds = lds_top;
  }
  a = &b;
  if (a->is_reg) {
    k_predict_reg<U><<<grid, 256, lds, st>>>(*a);
  } else {
    const int C = (int)a->n_classes;
    if (C <= 2) k_predict_cls<2, U><<<grid, 256, lds, st>>>(*a);
    else if (C <= 4) k_predict_cls<4, U><<<grid, 256, lds, st>>>(*a);
    else if (C <= 8) k_predict_cls<8, U><<<grid, 256, lds, st>>>(*a);
    else if (C <= 16) k_predict_cls<16, U><<<grid, 256, lds, st>>>(*a);
    else if (C <= 32) k_predict_cls<32, U><<<grid, 256, lds, st>>>(*a);
    else if (C <= 64) k_predict_cls<64, U><<<grid, 256, lds, st>>>(*a);
    else return 5;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// max_leaf_nodes: one lane per limited tree replays sklearn's best-first order over the
// grown tree (forest_common.h best_first_prune); the frontier heap lives in global
// scratch, ``cap`` entries per lane.  Trees with limit 0 are left alone.
__global__ void k_prune_best_first(NodeRec* nodes, const double* vals, int64_t VC, int C, int is_reg,
                                   const TreeSpec* specs, const int32_t* limit, int32_t t0, int32_t T,
                                   FrontierEnt* heap, int64_t cap, int32_t* leaves) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T) return;
  const int t = t0 + i;   // tree t's root is pool node t
  const int L = limit[t];
  if (L <= 0 || L > cap) { if (leaves) leaves[t] = -1; return; }
  const int n = best_first_prune(nodes, vals, VC, C, is_reg != 0, specs[t].criterion, t, L, heap + (int64_t)i * cap);
  if (leaves) leaves[t] = n;
}

}  // namespace dml

using namespace dml;

extern "C" {

int dml_forest_prune(NodeRec* nodes, const double* vals, int64_t VC, int32_t C, int32_t is_reg,
                     const TreeSpec* specs, const int32_t* limit, int32_t t0, int32_t T, void* heap, int64_t cap,
                     int32_t* leaves, hipStream_t st) {
  if (T <= 0) return 0;
  if (cap <= 0 || heap == nullptr) return 2;
  k_prune_best_first<<<(unsigned)((T + 63) / 64), 64, 0, st>>>(nodes, vals, VC, C, is_reg, specs, limit, t0, T,
                                                               static_cast<FrontierEnt*>(heap), cap, leaves);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_forest_refine(const uint8_t* Xb, int64_t ld, int64_t n, int64_t d, NodeRec* nodes, int64_t P,
                      const TreeSpec* specs, int32_t T, const uint8_t* roles, const float* vals, const uint8_t* exact,
                      uint32_t* hi, hipStream_t st) {
  if (P <= 0 || T <= 0) return 0;
  if (hipMemsetAsync(hi, 0xFF, (size_t)P * 4, st) != hipSuccess) return 1;
  dim3 g1((unsigned)((n + 255) / 256), (unsigned)T);
  k_refine_hi<<<g1, 256, 0, st>>>(Xb, ld, n, nodes, specs, roles, hi);
  k_refine_split<<<(unsigned)((P + 255) / 256), 256, 0, st>>>(nodes, P, d, hi, vals, exact);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}


int dml_forest_apply(const uint8_t* Xb, int64_t ld, int64_t n, const dml::NodeRec* nodes, int32_t t0, int32_t T,
                     int32_t* leaf, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  dim3 grid((unsigned)((n + 255) / 256), (unsigned)T);
  dml::k_apply<<<grid, 256, 0, st>>>(Xb, ld, n, nodes, t0, leaf);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_predict_sizeof_args() { return (int)sizeof(PredictArgs); }

int dml_forest_predict(PredictArgs* a, hipStream_t st) {
  if (a->F <= 0 || a->max_rows <= 0) return 0;
  static const int u = [] { const char* e = getenv("DML_PRED_U"); return e ? atoi(e) : 8; }();
  if (u == 16) return launch_predict<16>(a, st);
  if (u == 4) return launch_predict<4>(a, st);
  return launch_predict<8>(a, st);
}

// predict fit f alone (its trees and held-out rows; outputs stay at their absolute rows) --
// the forest builder calls this for a fit whose trees are complete while deeper fits of the
// same build are still growing (forest.hip early predict)
int dml_forest_predict_fit(const PredictArgs* a, int32_t f, hipStream_t st) {
  if (f < 0 || f >= a->F) return 2;
  const int64_t* roff = (const int64_t*)a->fit_row_off_host;
  PredictArgs b = *a;
  b.fit_tree_off = a->fit_tree_off + 4 * (int64_t)f;   // int32[F+1] device array, advanced to fit f
  b.fit_row_off = a->fit_row_off + 8 * (int64_t)f;     // int64[F+1]
  b.F = 1;
  b.fit_skip = 0;
  if (a->fit_depth_cap) b.fit_depth_cap = a->fit_depth_cap + 4 * (int64_t)f;
  b.max_rows = roff ? roff[f + 1] - roff[f] : a->max_rows;
  return dml_forest_predict(&b, st);
}

int dml_scores(ScoreArgs* a, hipStream_t st) {
  if (a->F <= 0) return 0;
  k_scores<<<(unsigned)a->F, 256, 0, st>>>(*a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
