// gbrt.hip — gradient-boosting stage kernels for CDNA4 (gfx950).
//
// The reference fits GradientBoosting{Classifier,Regressor} through sklearn
// (aws-prod/worker/worker.py:41,48 whitelist; sklearn ensemble/_gb.py `_fit_stage`: negative
// gradient, K regression trees, `_update_terminal_regions` line search, raw-score update).
// models/boosting.py grows stage s of EVERY fit of a batch with one call of the batched tree
// builder (forest.hip, regression mode); these kernels are the rest of the stage, fused:
//
//   k_gb_leafsums  every (tree, in-bag row): walk the stage tree, accumulate the Newton
//                  numerator / denominator of the row's leaf in LDS (per workgroup), flush
//                  with one atomic per touched leaf -- replaces apply + boolean masking +
//                  index_add over fits x rows (the float64 atomics of a depth-3 stage queue on
//                  a handful of addresses, profiles/r3_gbrt_config6.md)
//   k_gb_values    one thread per (tree, leaf slot): squared error -> the leaf's node mean
//                  (the builder's exact integer sums), log-loss / exponential -> one Newton step
//   k_gb_update    every (tree, row), train and held-out: raw[fit, k] += lr * value(leaf)
//   k_gb_grad      every (fit, row): the next stage's negative gradient from raw (binomial /
//                  multinomial / exponential / squared error), float64 for the line search and
//                  float32 for the tree builder's target matrix
//
//   k_sel_*        percentile losses (absolute_error / huber / quantile): sklearn's inverted-CDF
//                  percentile of every (tree, leaf)'s residuals -- and huber's delta, the alpha
//                  percentile of every fit's |residual| over its training rows -- by an exact
//                  8-pass radix select on order-preserving 64-bit keys of the float64 values
//                  (one histogram pass + one pick pass per byte), no sort
//
// A leaf is addressed by its PATH SLOT: 1 at the root, 2 s + (went right) per level, so a
// tree of depth <= D has slots in [1, 2^(D+1)) and per-tree leaf arrays need no node index.
// Depths up to 10 (S = 2048: 56 KB of leaf-sum LDS per workgroup, uint16 slot ids).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "forest_common.h"

namespace dml {

enum GbLoss : int32_t { kGbSq = 0, kGbAbs = 1, kGbHuber = 2, kGbQuant = 3, kGbLog = 4, kGbExp = 5 };

struct GbStageArgs {
  int64_t Xb, ld, n;          // uint8 bins [n][ld]
  int64_t nodes, node_val;    // the stage's trees in pool layout (tree j's root = node j), node_val VC = 3
  int64_t J, K, S;            // trees of the stage, classes per fit (1: binary / regression), slots per tree
  int64_t tree_raw;           // int32 [J]: row of `raw` tree j updates (fit * K + class)
  int64_t tree_loss;          // int32 [J] (GbLoss)
  int64_t tree_lr;            // double [J]
  int64_t inbag;              // uint8 [J][n]
  int64_t grad;               // double [J][n]: the stage's negative gradient (tree j's target)
  int64_t ycls;               // int32 [n] class ids (classification)
  int64_t slot_sum;           // double [J][S][2]: (numerator, denominator), zeroed by the caller
  int64_t slot_node;          // int32 [J][S]: leaf node of each slot
  int64_t slot_val;           // double [J][S]
  int64_t raw;                // double [F * K][n]
  int64_t XbT;                // optional feature-major bins uint8 [d][n] (0: walk the row-major Xb)
  // percentile losses (pct_any = 1 when some tree's loss is absolute_error / huber / quantile)
  int64_t pct_any;
  int64_t yreg;               // double [n]
  int64_t slot_of;            // uint16 [J][n] scratch: the in-bag row's leaf slot (0xFFFF: not in-bag)
  int64_t sel_hist;           // uint32 [J * S][256] scratch, zeroed by the caller
  int64_t sel_state;          // uint64 [J * S][4] scratch (prefix, mask, rank, count)
  int64_t tree_q;             // double [J]: the leaf percentile (0.5; quantile: alpha)
  int64_t tree_delta;         // double [J]: huber delta of the tree's fit at this stage
  // 0: the whole stage in one call.  Row-sharded stages run it in phases with all-reduces
  // between them (models/boosting.py): 1 = leaf sums (every leaf slot of the tree table gets its
  // node, rows or not: a rank may hold none of a leaf's in-bag rows), 2 = leaf values + raw
  // update, 3 = huber leaf terms (after the select of dml_gb_sel_step)
  int64_t phase;
};

struct GbGradArgs {
  int64_t n, K, A;            // rows, classes per fit, active fits
  int64_t fit_raw;            // int32 [A]: first raw row of active fit a (fit * K)
  int64_t fit_loss;           // int32 [A]
  int64_t raw;                // double [F * K][n]
  int64_t ycls;               // int32 [n]
  int64_t yreg;               // double [n]
  int64_t grad;               // double [A * K][n] out
  int64_t tgt;                // float [A * K][n] out
  int64_t fit_alpha;          // double [A]: quantile / huber alpha (percentile losses)
  int64_t fit_delta;          // double [A]: huber delta, written by dml_gb_huber_delta
  int64_t fit_train;          // uint8 [A][n]: the fit's training rows (huber delta)
  int64_t sel_hist;           // uint32 [A][256] scratch (huber delta select), zeroed by the caller
  int64_t sel_state;          // uint64 [A][4] scratch
};

#define GB_PTR(T, v) ((T*)(uintptr_t)(v))

// Tree j as a path-slot table in LDS: tsplit[slot] = the split of the node at that slot (-1:
// leaf or unreachable), tnode[slot] = its node index.  Thread t resolves slot t by walking its
// path bits from the root once per workgroup; the rows then walk the table (one LDS read and
// one bin load per level) instead of chasing node records through global memory.
template <int S>
__device__ __forceinline__ void gb_load_tree(const NodeRec* __restrict__ nodes, int j, int32_t* tsplit,
                                             int32_t* tnode) {
  for (int t = threadIdx.x; t < S; t += 256) {
    int node = -1, split = -1;
    if (t >= 1) {
      const int depth = 31 - __clz(t);
      node = j;
      for (int l = depth - 1; l >= 0 && node >= 0; --l) {
        const NodeRec r = nodes[node];
        node = r.split >= 0 ? r.left + ((t >> l) & 1) : -1;
      }
      if (node >= 0) split = nodes[node].split;
    }
    tsplit[t] = split;
    tnode[t] = node;
  }
}

// leaf slot of row r: feature-major bins (XbT, stride n) when given -- the rows of a workgroup
// are consecutive, so lanes at the same node read consecutive bytes of one feature -- else the
// row's line of the row-major table.  A tree of depth D stays below slot 2^(D+1) <= S.
template <int S>
__device__ __forceinline__ int gb_walk(const int32_t* tsplit, const uint8_t* __restrict__ X, int64_t ld,
                                       const uint8_t* __restrict__ XT, int64_t n, int64_t r) {
  int slot = 1;
  int sp = tsplit[1];
  while (sp >= 0) {
    const int f = sp >> 8;
    const int b = XT ? (int)XT[(int64_t)f * n + r] : (int)X[r * ld + f];
    slot = 2 * slot + (b > (sp & 255) ? 1 : 0);
    if (slot >= S) break;   // malformed tree guard (cannot happen for depth < log2 S)
    sp = tsplit[slot];
  }
  return slot < S ? slot : 1;
}

template <int S>
__global__ __launch_bounds__(256) void k_gb_leafsums(GbStageArgs a) {
  __shared__ double num[S], den[S];
  __shared__ int32_t tsplit[S], tnode[S];
  __shared__ int hit[S];
  const int j = blockIdx.y;
  const NodeRec* nodes = GB_PTR(const NodeRec, a.nodes);
  gb_load_tree<S>(nodes, j, tsplit, tnode);
  for (int i = threadIdx.x; i < S; i += 256) { num[i] = 0.0; den[i] = 0.0; hit[i] = 0; }
  __syncthreads();
  const int64_t n = a.n;
  const uint8_t* X = GB_PTR(const uint8_t, a.Xb);
  const uint8_t* XT = GB_PTR(const uint8_t, a.XbT);
  const uint8_t* inb = GB_PTR(const uint8_t, a.inbag) + (int64_t)j * n;
  const double* g = GB_PTR(const double, a.grad) + (int64_t)j * n;
  const int32_t* ycls = GB_PTR(const int32_t, a.ycls);
  const int loss = GB_PTR(const int32_t, a.tree_loss)[j];
  const int K = (int)a.K;
  const int cls = GB_PTR(const int32_t, a.tree_raw)[j] % K;
  const bool newton = loss == kGbLog || loss == kGbExp;
  const int64_t r0 = (int64_t)blockIdx.x * 1024;
  for (int u = 0; u < 4; ++u) {
    const int64_t r = r0 + u * 256 + threadIdx.x;
    if (r >= n) continue;
    if (!inb[r]) {   // (subsampled stages change the in-bag set: every row's entry is rewritten)
      if (a.pct_any) GB_PTR(uint16_t, a.slot_of)[(int64_t)j * n + r] = (uint16_t)0xFFFF;
      continue;
    }
    const int slot = gb_walk<S>(tsplit, X, a.ld, XT, n, r);
    hit[slot] = 1;   // every row of the leaf writes the same flag
    if (a.pct_any) GB_PTR(uint16_t, a.slot_of)[(int64_t)j * n + r] = (uint16_t)slot;
    if (!newton) continue;
    const double gv = g[r];
    double h;
    if (K > 1) {   // multinomial: p_k = y_k - g, hessian p (1 - p)
      const double p = (ycls[r] == cls ? 1.0 : 0.0) - gv;
      h = p * (1.0 - p);
    } else {
      const double yb = (double)ycls[r];
      if (loss == kGbExp) {
        h = yb > 0.5 ? gv : -gv;
      } else {
        const double p = yb - gv;
        h = p * (1.0 - p);
      }
    }
    atomicAdd(&num[slot], gv);
    atomicAdd(&den[slot], h);
  }
  __syncthreads();
  double* ss = GB_PTR(double, a.slot_sum) + (int64_t)j * S * 2;
  int32_t* sn = GB_PTR(int32_t, a.slot_node) + (int64_t)j * S;
  for (int i = threadIdx.x; i < S; i += 256) {
    if (!hit[i] && !(a.phase != 0 && tsplit[i] < 0 && tnode[i] >= 0)) continue;
    sn[i] = tnode[i];
    if (newton) {
      atomicAdd(&ss[2 * i], num[i]);
      atomicAdd(&ss[2 * i + 1], den[i]);
    }
  }
}

// ---- exact radix select ------------------------------------------------------------
constexpr int kSelRows = 8192;   // rows per workgroup of a byte pass (amortises the LDS counters)
// order-preserving 64-bit key of a double (negative values reversed), and back
__device__ __forceinline__ unsigned long long gb_double_key(double v) {
  const unsigned long long u = __double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double gb_key_to_double(unsigned long long k) {
  return __longlong_as_double((k >> 63) ? (long long)(k & 0x7FFFFFFFFFFFFFFFull) : (long long)~k);
}

// one byte pass: every segment member whose key matches the segment's prefix (the bytes fixed
// so far) counts its next byte.  MODE 0: segments (tree j, leaf slot), key = y - raw of tree j's
// in-bag rows of a percentile loss; MODE 1: segments = active fits, key = |y - raw| over the
// fit's training rows (huber delta).  Per-workgroup LDS counters when a grid row's segments fit
// (S <= 64 slots x 256), flushed with one global atomic per nonzero counter.
template <int MODE, int SEGS>
__device__ __forceinline__ void gb_sel_pass(int64_t n, int row_seg, int nseg_row, const double* __restrict__ yreg,
                                            const double* __restrict__ raw, const uint8_t* __restrict__ member,
                                            const uint16_t* __restrict__ slot_of, int loss_ok,
                                            const unsigned long long* __restrict__ state, unsigned int* __restrict__ hist,
                                            int shift) {
  __shared__ unsigned int lh[SEGS > 0 ? SEGS * 256 : 1];
  if (SEGS > 0) {
    for (int i = threadIdx.x; i < SEGS * 256; i += 256) lh[i] = 0u;
    __syncthreads();
  }
  const int64_t r0 = (int64_t)blockIdx.x * kSelRows;
  if (loss_ok) {
    for (int u = 0; u < kSelRows / 256; ++u) {
      const int64_t r = r0 + u * 256 + threadIdx.x;
      if (r >= n) break;
      int local;
      double v;
      if (MODE == 0) {
        const int sl = slot_of[r];
        if (sl == 0xFFFF) continue;
        local = sl;
        v = yreg[r] - raw[r];
      } else {
        if (!member[r]) continue;
        local = 0;
        v = fabs(yreg[r] - raw[r]);
      }
      const int seg = row_seg + local;
      const unsigned long long key = gb_double_key(v);
      const unsigned long long* stt = state + 4 * (int64_t)seg;
      if ((key & stt[1]) != stt[0]) continue;
      const int byte = (int)((key >> shift) & 255ull);
      if (SEGS > 0) atomicAdd(&lh[local * 256 + byte], 1u);
      else atomicAdd(&hist[(int64_t)seg * 256 + byte], 1u);
    }
  }
  if (SEGS > 0) {
    __syncthreads();
    for (int i = threadIdx.x; i < nseg_row * 256 && i < SEGS * 256; i += 256)
      if (lh[i]) atomicAdd(&hist[(int64_t)row_seg * 256 + i], lh[i]);
  }
}

template <int SEGS>
__global__ __launch_bounds__(256) void k_sel_leaf(GbStageArgs a, int shift) {
  const int j = blockIdx.y;
  const int loss = GB_PTR(const int32_t, a.tree_loss)[j];
  const int ok = loss == kGbAbs || loss == kGbQuant || loss == kGbHuber;
  const int64_t n = a.n;
  gb_sel_pass<0, SEGS>(n, j * (int)a.S, (int)a.S, GB_PTR(const double, a.yreg),
                       GB_PTR(const double, a.raw) + (int64_t)GB_PTR(const int32_t, a.tree_raw)[j] * n, nullptr,
                       GB_PTR(const uint16_t, a.slot_of) + (int64_t)j * n, ok,
                       GB_PTR(const unsigned long long, a.sel_state), GB_PTR(unsigned int, a.sel_hist), shift);
}

__global__ __launch_bounds__(256) void k_sel_fit(GbGradArgs a, int shift) {
  const int fa = blockIdx.y;
  const int ok = GB_PTR(const int32_t, a.fit_loss)[fa] == kGbHuber;
  const int64_t n = a.n;
  gb_sel_pass<1, 1>(n, fa, 1, GB_PTR(const double, a.yreg),
                    GB_PTR(const double, a.raw) + (int64_t)GB_PTR(const int32_t, a.fit_raw)[fa] * n,
                    GB_PTR(const uint8_t, a.fit_train) + (int64_t)fa * n, nullptr, ok,
                    GB_PTR(const unsigned long long, a.sel_state), GB_PTR(unsigned int, a.sel_hist), shift);
}

// one wave per segment: the byte holding the target rank (pass 0 also fixes the rank from the
// segment's member count and its percentile q: inverted CDF, k = ceil(q m) - 1, the torch path's
// _segment_percentile); the counters are cleared for the next pass.  state: prefix, mask, rank, m
__global__ __launch_bounds__(64) void k_sel_pick(unsigned long long* state, unsigned int* hist, const double* q,
                                                 int64_t nseg, int64_t q_div, int shift) {
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x;
  unsigned long long* st = state + 4 * i;
  unsigned int* h = hist + i * 256;
  const uint4 c4 = *(const uint4*)(h + 4 * lane);   // bins 4 lane .. 4 lane + 3
  *(uint4*)(h + 4 * lane) = make_uint4(0u, 0u, 0u, 0u);
  const unsigned long long mine = (unsigned long long)c4.x + c4.y + c4.z + c4.w;
  unsigned long long incl = mine;   // inclusive prefix over lanes
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const unsigned long long total = __shfl(incl, 63);
  unsigned long long k;
  if (shift == 56) {   // pass 0: every member counted once
    long long kk = 0;
    if (total > 0) {
      kk = (long long)ceil(q[i / q_div] * (double)total - 1e-12) - 1;
      kk = kk < 0 ? 0 : (kk > (long long)total - 1 ? (long long)total - 1 : kk);
    }
    k = (unsigned long long)kk;
    if (lane == 0) st[3] = total;
  } else {
    k = st[2];
  }
  if (total == 0) {   // empty segment (or no member left): nothing to fix
    if (lane == 0) st[2] = k;
    return;
  }
  const unsigned long long excl = incl - mine;
  const unsigned long long hit = __ballot(k >= excl && k < incl);
  const int src = hit ? __ffsll((long long)hit) - 1 : 63;
  if (lane == src) {
    unsigned long long cum = excl;
    int b = 0;
    const unsigned int cs[4] = {c4.x, c4.y, c4.z, c4.w};
    for (; b < 3; ++b) {
      if (k < cum + cs[b]) break;
      cum += cs[b];
    }
    st[0] |= (unsigned long long)(4 * lane + b) << shift;
    st[1] |= 255ull << shift;
    st[2] = k - cum;
  }
}

__global__ __launch_bounds__(256) void k_sel_init(unsigned long long* state, int64_t nseg) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nseg) return;
  state[4 * i] = 0ull; state[4 * i + 1] = 0ull; state[4 * i + 2] = 0ull; state[4 * i + 3] = 0ull;
}

// huber leaf line search: sum over the leaf's in-bag rows of sign(d) min(delta, |d|), d = resid -
// median, and the member count, into slot_sum (then k_gb_values: median + sum / count)
template <int S>
__global__ __launch_bounds__(256) void k_gb_huber_terms(GbStageArgs a) {
  __shared__ double sm[S], cn[S];
  const int j = blockIdx.y;
  if (GB_PTR(const int32_t, a.tree_loss)[j] != kGbHuber) return;   // workgroup-uniform
  for (int i = threadIdx.x; i < S; i += 256) { sm[i] = 0.0; cn[i] = 0.0; }
  __syncthreads();
  const int64_t n = a.n;
  const uint16_t* so = GB_PTR(const uint16_t, a.slot_of) + (int64_t)j * n;
  const double* raw = GB_PTR(const double, a.raw) + (int64_t)GB_PTR(const int32_t, a.tree_raw)[j] * n;
  const double* y = GB_PTR(const double, a.yreg);
  const unsigned long long* st = GB_PTR(const unsigned long long, a.sel_state) + (int64_t)j * S * 4;
  const double delta = GB_PTR(const double, a.tree_delta)[j];
  const int64_t r0 = (int64_t)blockIdx.x * 1024;
  for (int u = 0; u < 4; ++u) {
    const int64_t r = r0 + u * 256 + threadIdx.x;
    if (r >= n) break;
    const int sl = so[r];
    if (sl == 0xFFFF) continue;
    const double d = (y[r] - raw[r]) - gb_key_to_double(st[4 * sl]);
    const double t = d > 0.0 ? fmin(delta, d) : (d < 0.0 ? -fmin(delta, -d) : 0.0);
    atomicAdd(&sm[sl], t);
    atomicAdd(&cn[sl], 1.0);
  }
  __syncthreads();
  double* ss = GB_PTR(double, a.slot_sum) + (int64_t)j * S * 2;
  for (int i = threadIdx.x; i < S; i += 256)
    if (cn[i] > 0.0) {
      atomicAdd(&ss[2 * i], sm[i]);
      atomicAdd(&ss[2 * i + 1], cn[i]);
    }
}

__global__ __launch_bounds__(256) void k_gb_values(GbStageArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t S = a.S;
  if (i >= a.J * S) return;
  const int j = (int)(i / S);
  const int32_t node = GB_PTR(const int32_t, a.slot_node)[i];
  double v = 0.0;
  if (node >= 0) {
    const int loss = GB_PTR(const int32_t, a.tree_loss)[j];
    if (loss == kGbAbs || loss == kGbQuant || loss == kGbHuber) {
      const double med = gb_key_to_double(GB_PTR(const unsigned long long, a.sel_state)[4 * i]);
      v = med;
      if (loss == kGbHuber) {   // med + mean of the clipped deviations (k_gb_huber_terms)
        const double* ss = GB_PTR(const double, a.slot_sum) + 2 * i;
        v = med + ss[0] / fmax(ss[1], 1.0);
      }
    } else if (loss == kGbLog || loss == kGbExp) {
      const double* ss = GB_PTR(const double, a.slot_sum) + 2 * i;
      double num = ss[0];
      const double den = ss[1];
      if (a.K > 1) num = num * (double)(a.K - 1) / (double)a.K;
      v = fabs(den) < 1e-150 ? (num == 0.0 ? 0.0 : copysign(1e150, num)) : num / den;
    } else {   // squared error: the node mean of the builder's exact sums
      const double* nv = GB_PTR(const double, a.node_val) + (int64_t)node * 3;
      v = nv[0] > 0.0 ? nv[1] / fmax(nv[0], 1e-300) : 0.0;
    }
  }
  GB_PTR(double, a.slot_val)[i] = v;
}

template <int S>
__global__ __launch_bounds__(256) void k_gb_update(GbStageArgs a) {
  __shared__ double val[S];
  __shared__ int32_t tsplit[S], tnode[S];
  const int j = blockIdx.y;
  gb_load_tree<S>(GB_PTR(const NodeRec, a.nodes), j, tsplit, tnode);
  for (int i = threadIdx.x; i < S; i += 256) val[i] = GB_PTR(const double, a.slot_val)[(int64_t)j * S + i];
  __syncthreads();
  const int64_t n = a.n;
  const uint8_t* X = GB_PTR(const uint8_t, a.Xb);
  const uint8_t* XT = GB_PTR(const uint8_t, a.XbT);
  double* raw = GB_PTR(double, a.raw) + (int64_t)GB_PTR(const int32_t, a.tree_raw)[j] * n;
  const double lr = GB_PTR(const double, a.tree_lr)[j];
  const int64_t r0 = (int64_t)blockIdx.x * 1024;
  for (int u = 0; u < 4; ++u) {
    const int64_t r = r0 + u * 256 + threadIdx.x;
    if (r >= n) continue;
    raw[r] += val[gb_walk<S>(tsplit, X, a.ld, XT, n, r)] * lr;
  }
}

__device__ __forceinline__ double gb_sigmoid(double x) { return 1.0 / (1.0 + exp(-x)); }

__global__ __launch_bounds__(256) void k_sel_delta(GbGradArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.A) return;
  const unsigned long long* st = GB_PTR(const unsigned long long, a.sel_state) + 4 * i;
  GB_PTR(double, a.fit_delta)[i] = st[3] ? gb_key_to_double(st[0]) : 0.0;
}

template <int KMAX>
__global__ __launch_bounds__(256) void k_gb_grad(GbGradArgs a) {
  const int fa = blockIdx.y;
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = a.n;
  if (r >= n) return;
  const int K = (int)a.K;
  const int loss = GB_PTR(const int32_t, a.fit_loss)[fa];
  const double* raw = GB_PTR(const double, a.raw) + (int64_t)GB_PTR(const int32_t, a.fit_raw)[fa] * n;
  double* g = GB_PTR(double, a.grad) + (int64_t)fa * K * n;
  float* t = GB_PTR(float, a.tgt) + (int64_t)fa * K * n;
  if (loss == kGbLog && K > 1) {   // softmax over the fit's K raw rows (max-shifted, like torch)
    double z[KMAX];
    double mx = -INFINITY;
    for (int k = 0; k < K && k < KMAX; ++k) { z[k] = raw[(int64_t)k * n + r]; mx = fmax(mx, z[k]); }
    double s = 0.0;
    for (int k = 0; k < K && k < KMAX; ++k) { z[k] = exp(z[k] - mx); s += z[k]; }
    const int y = GB_PTR(const int32_t, a.ycls)[r];
    for (int k = 0; k < K && k < KMAX; ++k) {
      const double v = (y == k ? 1.0 : 0.0) - z[k] / s;
      g[(int64_t)k * n + r] = v;
      t[(int64_t)k * n + r] = (float)v;
    }
    return;
  }
  const double x = raw[r];
  double v;
  if (loss == kGbLog) {
    v = (double)GB_PTR(const int32_t, a.ycls)[r] - gb_sigmoid(x);
  } else if (loss == kGbExp) {
    const double yb = (double)GB_PTR(const int32_t, a.ycls)[r];
    v = yb * exp(-x) - (1.0 - yb) * exp(x);
  } else {   // squared error and the percentile losses, from the residual
    const double diff = GB_PTR(const double, a.yreg)[r] - x;
    if (loss == kGbAbs) {
      v = diff > 0.0 ? 1.0 : (diff < 0.0 ? -1.0 : 0.0);
    } else if (loss == kGbQuant) {
      const double al = GB_PTR(const double, a.fit_alpha)[fa];
      v = diff >= 0.0 ? al : al - 1.0;
    } else if (loss == kGbHuber) {
      const double dl = GB_PTR(const double, a.fit_delta)[fa];
      v = fabs(diff) <= dl ? diff : (diff > 0.0 ? dl : (diff < 0.0 ? -dl : 0.0));
    } else {
      v = diff;
    }
  }
  g[r] = v;
  t[r] = (float)v;
}

// exponent histogram of regression targets (ops/forest_ops.py reg_exponent_counts; the
// fixed-point rule forest_common.h reg_exponents_counts): out[t][k + 160] counts target t's
// nonzero values with frexp exponent k, out[t][0] its zeros, bad[0] the non-finite values.
// One LDS histogram per workgroup, flushed with one global atomic per nonzero bin.
constexpr int kExpOffK = 160, kExpBinsK = 320;
__global__ __launch_bounds__(256) void k_exp_hist(const float* __restrict__ y, int64_t n, int64_t ystride,
                                                  unsigned long long* out, unsigned long long* bad) {
  __shared__ unsigned int h[kExpBinsK];
  __shared__ unsigned int nb;
  for (int i = threadIdx.x; i < kExpBinsK; i += 256) h[i] = 0u;
  if (threadIdx.x == 0) nb = 0u;
  __syncthreads();
  const int t = blockIdx.y;
  const float* yt = y + (int64_t)t * ystride;
  const int64_t i0 = (int64_t)blockIdx.x * 4096;
  const int64_t i1 = i0 + 4096 < n ? i0 + 4096 : n;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
    const float v = yt[i];
    if (!isfinite(v)) { atomicAdd(&nb, 1u); continue; }
    int k = 0;
    if (v != 0.0f) frexpf(v, &k);
    atomicAdd(&h[v != 0.0f ? k + kExpOffK : 0], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kExpBinsK; i += 256)
    if (h[i]) atomicAdd(&out[(int64_t)t * kExpBinsK + i], (unsigned long long)h[i]);
  if (threadIdx.x == 0 && nb) atomicAdd(bad, (unsigned long long)nb);
}

// the 8 byte passes of the (tree, leaf) percentile select (state zeroed, hist zero on entry)
template <int SV>
int leaf_select(GbStageArgs* a, dim3 grid, hipStream_t st) {
  if (!a->slot_of || !a->sel_hist || !a->sel_state || !a->tree_q || !a->yreg) return 2;
  const int64_t nseg = a->J * SV;
  k_sel_init<<<(unsigned)((nseg + 255) / 256), 256, 0, st>>>((unsigned long long*)a->sel_state, nseg);
  const dim3 gsel((unsigned)((a->n + kSelRows - 1) / kSelRows), grid.y);
  for (int shift = 56; shift >= 0; shift -= 8) {
    if (SV <= 64) k_sel_leaf<(SV <= 64 ? SV : 1)><<<gsel, 256, 0, st>>>(*a, shift);
    else k_sel_leaf<0><<<gsel, 256, 0, st>>>(*a, shift);
    k_sel_pick<<<(unsigned)nseg, 64, 0, st>>>((unsigned long long*)a->sel_state, (unsigned int*)a->sel_hist,
                                             (const double*)a->tree_q, nseg, SV, shift);
  }
  return 0;
}

}  // namespace dml

using namespace dml;

extern "C" {

// targets x [n] float32 rows at stride ystride (ystride = n for one target); out int64
// [targets][320] and bad int64 [1], zeroed by the caller
int dml_exp_hist(const float* y, int64_t n, int64_t ystride, int64_t targets, int64_t* out, int64_t* bad,
                 hipStream_t st) {
  if (n <= 0 || targets <= 0) return 0;
  if (targets > 65535) return 2;
  k_exp_hist<<<dim3((unsigned)((n + 4095) / 4096), (unsigned)targets), 256, 0, st>>>(
      y, n, ystride, (unsigned long long*)out, (unsigned long long*)bad);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_gb_sizeof_stage_args() { return (int)sizeof(GbStageArgs); }
int dml_gb_sizeof_grad_args() { return (int)sizeof(GbGradArgs); }

// leaf sums + leaf values + raw update of one stage (slot_sum / slot_node zeroed / -1 by the caller)
int dml_gb_stage(GbStageArgs* a, hipStream_t st) {
  if (a->J <= 0 || a->n <= 0) return 0;
  if (a->phase != 0) return 2;
  const dim3 grid((unsigned)((a->n + 1023) / 1024), (unsigned)a->J);
  switch (a->S) {
#define GB_CASE(SV)                                                                   \
    case SV:                                                                          \
      k_gb_leafsums<SV><<<grid, 256, 0, st>>>(*a);                                    \
      if (a->pct_any) {                                                               \
        if (leaf_select<SV>(a, grid, st)) return 2;                                   \
        k_gb_huber_terms<SV><<<grid, 256, 0, st>>>(*a);                               \
      }                                                                               \
      k_gb_values<<<(unsigned)((a->J * SV + 255) / 256), 256, 0, st>>>(*a);           \
      k_gb_update<SV><<<grid, 256, 0, st>>>(*a);                                      \
      break;
    GB_CASE(4) GB_CASE(8) GB_CASE(16) GB_CASE(32) GB_CASE(64) GB_CASE(128) GB_CASE(256) GB_CASE(512) GB_CASE(1024)
    GB_CASE(2048)
#undef GB_CASE
    default: return 2;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// one phase of a row-sharded stage (GbStageArgs::phase 1..3; the caller all-reduces between)
int dml_gb_stage_phase(GbStageArgs* a, hipStream_t st) {
  if (a->J <= 0 || a->n <= 0) return 0;
  if (a->phase < 1 || a->phase > 3) return 2;
  const dim3 grid((unsigned)((a->n + 1023) / 1024), (unsigned)a->J);
  switch (a->S) {
#define GB_CASE(SV)                                                                   \
    case SV:                                                                          \
      if (a->phase == 1) k_gb_leafsums<SV><<<grid, 256, 0, st>>>(*a);                 \
      if (a->phase == 3) k_gb_huber_terms<SV><<<grid, 256, 0, st>>>(*a);              \
      if (a->phase == 2) {                                                            \
        k_gb_values<<<(unsigned)((a->J * SV + 255) / 256), 256, 0, st>>>(*a);         \
        k_gb_update<SV><<<grid, 256, 0, st>>>(*a);                                    \
      }                                                                               \
      break;
    GB_CASE(4) GB_CASE(8) GB_CASE(16) GB_CASE(32) GB_CASE(64) GB_CASE(128) GB_CASE(256) GB_CASE(512) GB_CASE(1024)
    GB_CASE(2048)
#undef GB_CASE
    default: return 2;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// one step of the (tree, leaf) percentile select of a row-sharded stage: which = 0 clears the
// states, 1 counts this rank's byte `shift` into sel_hist (the caller then all-reduces it),
// 2 picks the byte from the summed counts (and clears them)
int dml_gb_sel_step(GbStageArgs* a, int which, int shift, hipStream_t st) {
  if (a->J <= 0) return 0;
  if (!a->slot_of || !a->sel_hist || !a->sel_state || !a->tree_q || !a->yreg) return 2;
  if (shift < 0 || shift > 56 || (shift & 7)) return 2;
  const int64_t nseg = a->J * a->S;
  if (which == 0) {
    k_sel_init<<<(unsigned)((nseg + 255) / 256), 256, 0, st>>>((unsigned long long*)a->sel_state, nseg);
  } else if (which == 1) {
    if (a->n > 0) {
      const dim3 gsel((unsigned)((a->n + kSelRows - 1) / kSelRows), (unsigned)a->J);
      if (a->S <= 64) {
        switch (a->S) {
          case 4: k_sel_leaf<4><<<gsel, 256, 0, st>>>(*a, shift); break;
          case 8: k_sel_leaf<8><<<gsel, 256, 0, st>>>(*a, shift); break;
          case 16: k_sel_leaf<16><<<gsel, 256, 0, st>>>(*a, shift); break;
          case 32: k_sel_leaf<32><<<gsel, 256, 0, st>>>(*a, shift); break;
          case 64: k_sel_leaf<64><<<gsel, 256, 0, st>>>(*a, shift); break;
          default: return 2;
        }
      } else {
        k_sel_leaf<0><<<gsel, 256, 0, st>>>(*a, shift);
      }
    }
  } else if (which == 2) {
    k_sel_pick<<<(unsigned)nseg, 64, 0, st>>>((unsigned long long*)a->sel_state, (unsigned int*)a->sel_hist,
                                             (const double*)a->tree_q, nseg, a->S, shift);
  } else {
    return 2;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// huber delta of every active fit: the alpha percentile (inverted CDF) of |y - raw| over the
// fit's training rows, into fit_delta (fits of other losses are skipped)
int dml_gb_huber_delta(GbGradArgs* a, hipStream_t st) {
  if (a->A <= 0 || a->n <= 0) return 0;
  if (!a->fit_train || !a->sel_hist || !a->sel_state || !a->fit_alpha || !a->fit_delta || !a->yreg) return 2;
  const dim3 grid((unsigned)((a->n + kSelRows - 1) / kSelRows), (unsigned)a->A);
  k_sel_init<<<(unsigned)((a->A + 255) / 256), 256, 0, st>>>((unsigned long long*)a->sel_state, a->A);
  for (int shift = 56; shift >= 0; shift -= 8) {
    k_sel_fit<<<grid, 256, 0, st>>>(*a, shift);
    k_sel_pick<<<(unsigned)a->A, 64, 0, st>>>((unsigned long long*)a->sel_state, (unsigned int*)a->sel_hist,
                                             (const double*)a->fit_alpha, a->A, 1, shift);
  }
  k_sel_delta<<<(unsigned)((a->A + 255) / 256), 256, 0, st>>>(*a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// one step of the huber-delta select of a row-sharded stage (which: 0 init, 1 count this rank's
// rows, 2 pick from the all-reduced counts, 3 write fit_delta)
int dml_gb_fit_sel_step(GbGradArgs* a, int which, int shift, hipStream_t st) {
  if (a->A <= 0) return 0;
  if (!a->fit_train || !a->sel_hist || !a->sel_state || !a->fit_alpha || !a->fit_delta || !a->yreg) return 2;
  if (shift < 0 || shift > 56 || (shift & 7)) return 2;
  if (which == 0) {
    k_sel_init<<<(unsigned)((a->A + 255) / 256), 256, 0, st>>>((unsigned long long*)a->sel_state, a->A);
  } else if (which == 1) {
    if (a->n > 0)
      k_sel_fit<<<dim3((unsigned)((a->n + kSelRows - 1) / kSelRows), (unsigned)a->A), 256, 0, st>>>(*a, shift);
  } else if (which == 2) {
    k_sel_pick<<<(unsigned)a->A, 64, 0, st>>>((unsigned long long*)a->sel_state, (unsigned int*)a->sel_hist,
                                             (const double*)a->fit_alpha, a->A, 1, shift);
  } else if (which == 3) {
    k_sel_delta<<<(unsigned)((a->A + 255) / 256), 256, 0, st>>>(*a);
  } else {
    return 2;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_gb_grad(GbGradArgs* a, hipStream_t st) {
  if (a->A <= 0 || a->n <= 0) return 0;
  if (a->K > 64) return 2;
  const dim3 grid((unsigned)((a->n + 255) / 256), (unsigned)a->A);
  if (a->K <= 8) k_gb_grad<8><<<grid, 256, 0, st>>>(*a);
  else k_gb_grad<64><<<grid, 256, 0, st>>>(*a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
