// forest_mae.hip — criterion="absolute_error" (sklearn MAE) regression trees on the GPU.
//
// sklearn grows MAE trees with per-node weighted medians (WeightedMedianCalculator);
// the reference forwards criterion="absolute_error" verbatim to RandomForestRegressor
// (aws-prod/worker/worker.py:45, :450-452).  The histogram tiers of forest.hip cannot
// evaluate it (a median is not a sum), so MAE builds run this separate level-synchronous
// builder, node for node equal to the host builder (csrc/runtime/forest_cpu.cpp):
//
//   * every tree's rows are kept in (y, row id) order: one global stable sort of the
//     targets (ops/forest_ops.py build_gpu_mae), in-bag rows compacted in that order
//     per tree (k_mae_fill), and every partition is stable -- a node's rows are always its
//     targets in ascending order, so medians are prefix-weight crossings;
//   * targets are the fixed-point yq of forest_common.h (reg_quantize), weights the
//     bootstrap counts: every abs deviation is an exact integer (mae_absdev), the split
//     gain -(al + ar) the same double on both builders;
//   * one 256-thread workgroup per open node (k_mae_level): per visited feature, a bin
//     histogram (weights, w yq, rows) gives every threshold's side totals, then thread b
//     scans the node's rows in target order and finds both sides' weighted medians for
//     threshold b (the rows stream through LDS, every thread reading the same element: an
//     LDS broadcast) -- O(256 m) per feature, no sort per candidate;
//   * accept (sklearn impurity_improvement on the MAE impurities), stable partition, the
//     children's medians / abs deviations, enqueue.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "forest_common.h"

namespace dml {
namespace mae {

constexpr int NT = 256;
constexpr int CHUNK = 1024;   // rows staged in LDS per pass step

// ctypes-facing arguments (every field 8 bytes; ops/forest_ops.py MaeArgs mirrors the order)
struct MaeArgs {
  int64_t Xb, ld, n, d;
  int64_t yreg;                 // float [n]
  int64_t roles;                // uint8 [splits][n]
  int64_t specs, T;             // TreeSpec [T] (device; min_weight_leaf set by k_mae_root)
  int64_t perm;                 // int32 [n]: row ids in (y, row id) order
  int64_t yq_e1, yq_e2;
  int64_t counts;               // int32 [T]: in-bag rows per tree (k_mae_count)
  int64_t row_off;              // int64 [T + 1]
  int64_t rows_a, rows_b;       // uint32 [rows_total] each
  int64_t nodes, vals, nabs;    // int32 [cap][2], double [cap][3], double [cap]
  int64_t pool_cap;
  int64_t open_a, open_b, open_cap;   // MaeOpen [open_cap] each
  int64_t counters;             // int32 [8]: 0 pool, 1 small open count (next), 2 overflow, 3 big open count (next)
  int64_t tree_W;               // double [T]
  int64_t n_nodes_out, levels_out, status_out;
  // nodes of >= big_rows rows: their first P visiting positions are evaluated by one
  // workgroup each (k_mae_eval), then k_mae_decide selects in visiting order
  int64_t big_a, big_b, big_cap;      // MaeOpen [big_cap] each
  int64_t res, P, big_rows;           // FeatRes [big_cap][P]
};

struct MaeOpen {
  int32_t tree, node;
  int64_t start;
  int32_t count, depth;
  uint64_t key;
  int64_t W, S;   // the node's integer sums w, w yq (node_stats)
};

// one visited feature of a node: whether it is non-constant, its best threshold (lowest bin
// of the largest gain), the gain and both sides' exact abs deviations, the left weight
struct FeatRes {
  double g;
  int64_t al, ar, wl;
  int32_t bin, nc;
};

template <typename T>
__device__ __forceinline__ T* P(int64_t v) { return reinterpret_cast<T*>(v); }

struct Ctx {
  const uint8_t* Xb;
  int64_t ld;
  int32_t n, d;
  const float* y;
  const uint8_t* roles;
  TreeSpec* specs;
  RegScale rq;
  NodeRec* nodes;
  double* vals;
  double* nabs;
  int64_t pool_cap;
  int32_t* counters;
  double* tree_W;
  int64_t open_cap, big_cap, big_rows;
};

__host__ Ctx make_ctx(const MaeArgs* a) {
  Ctx c;
  c.Xb = reinterpret_cast<const uint8_t*>(a->Xb);
  c.ld = a->ld;
  c.n = (int32_t)a->n;
  c.d = (int32_t)a->d;
  c.y = reinterpret_cast<const float*>(a->yreg);
  c.roles = reinterpret_cast<const uint8_t*>(a->roles);
  c.specs = reinterpret_cast<TreeSpec*>(a->specs);
  c.rq = reg_scale((int)a->yq_e1, (int)a->yq_e2);
  c.nodes = reinterpret_cast<NodeRec*>(a->nodes);
  c.vals = reinterpret_cast<double*>(a->vals);
  c.nabs = reinterpret_cast<double*>(a->nabs);
  c.pool_cap = a->pool_cap;
  c.counters = reinterpret_cast<int32_t*>(a->counters);
  c.tree_W = reinterpret_cast<double*>(a->tree_W);
  c.open_cap = a->open_cap;
  c.big_cap = a->big_cap;
  c.big_rows = a->big_rows;
  return c;
}

__device__ __forceinline__ bool in_bag(const Ctx& c, const TreeSpec& s, uint32_t row, uint32_t& w) {
  if (c.roles[(int64_t)s.split * c.n + row] != 1) return false;
  w = boot_weight(s, row);
  return w != 0u;
}

__device__ __forceinline__ int64_t row_yq(const Ctx& c, uint32_t row) {
  int64_t yq, y2q;
  reg_quantize(c.y[row], c.rq, yq, y2q);
  return yq;
}

// block-wide inclusive scan of one int64 per thread (256 threads; sh: >= 256 int64 scratch)
__device__ int64_t block_scan(int64_t v, int64_t* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {
    const int64_t add = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const int64_t r = sh[t];
  __syncthreads();
  return r;
}

__device__ int64_t block_sum(int64_t v, int64_t* sh) {
  const int64_t s = block_scan(v, sh);
  __shared__ int64_t tot;
  if (threadIdx.x == NT - 1) tot = s;
  __syncthreads();
  const int64_t r = tot;
  __syncthreads();
  return r;
}

// W, S, median and abs deviation of the rows [rows, rows + count) (target order): the node
// value {W, W med, ab + W med^2} into v, returns ab (forest_common.h mae_node_value)
__device__ double node_stats(const Ctx& c, const TreeSpec& s, const uint32_t* rows, int count, double* v,
                             int64_t* sh, int64_t& Wout, int64_t& Sout) {
  int64_t w_loc = 0, s_loc = 0;
  for (int i = threadIdx.x; i < count; i += NT) {
    const uint32_t r = rows[i];
    const int64_t w = (int64_t)boot_weight(s, r);
    w_loc += w;
    s_loc += w * row_yq(c, r);
  }
  const int64_t W = block_sum(w_loc, sh), S = (int64_t)(uint64_t)block_sum(s_loc, sh);
  // the first position whose prefix weight reaches W / 2 (2 prefix >= W), chunk by chunk
  __shared__ int64_t base_w, base_s;
  __shared__ int found_k;
  __shared__ int64_t f_c, f_cs;
  if (threadIdx.x == 0) { base_w = 0; base_s = 0; found_k = -1; }
  __syncthreads();
  for (int c0 = 0; c0 < count; c0 += NT) {
    const int i = c0 + (int)threadIdx.x;
    int64_t w = 0, wy = 0;
    if (i < count) {
      const uint32_t r = rows[i];
      w = (int64_t)boot_weight(s, r);
      wy = w * row_yq(c, r);
    }
    const int64_t pw = block_scan(w, sh) + base_w;
    const int64_t ps = (int64_t)((uint64_t)block_scan(wy, sh) + (uint64_t)base_s);
    // the lowest i with 2 pw >= W: exactly one thread sees its predecessor below
    const int64_t prev = pw - w;
    if (i < count && 2 * pw >= W && 2 * prev < W) { found_k = i; f_c = pw; f_cs = ps; }
    __syncthreads();
    if (threadIdx.x == NT - 1) { base_w = pw; base_s = ps; }
    __syncthreads();
    if (found_k >= 0) break;
  }
  const int k = found_k >= 0 ? found_k : 0;
  const uint32_t rk = rows[k];
  const bool tie = found_k >= 0 && 2 * f_c == W && k + 1 < count;
  const double ylo = (double)c.y[rk];
  const double yhi = tie ? (double)c.y[rows[k + 1]] : ylo;
  Wout = W;
  Sout = S;
  return mae_node_value(W, S, found_k >= 0 ? f_c : 0, found_k >= 0 ? f_cs : 0, row_yq(c, rk), ylo, yhi, tie, c.rq,
                        v);
}

__device__ bool visit(const TreeSpec& s, int count, int depth, double W, double ab) {
  return !(leaf_by_counts(s, count, depth) || leaf_by_weight(s, W) || (W > 0.0 ? ab / W : 0.0) <= kEps);
}

// next level's small (one workgroup per node) or big (one per visited feature) list
__device__ void enqueue(const Ctx& c, MaeOpen* out, MaeOpen* out_big, int tree, int node, int64_t start, int count,
                        int depth, uint64_t key, int64_t W, int64_t S) {
  const bool big = count >= c.big_rows;
  const int idx = atomicAdd(&c.counters[big ? 3 : 1], 1);
  if (idx >= (big ? c.big_cap : c.open_cap)) { atomicOr(&c.counters[2], 1); return; }
  MaeOpen o;
  o.tree = tree; o.node = node; o.start = start; o.count = count; o.depth = depth; o.key = key; o.W = W; o.S = S;
  (big ? out_big : out)[idx] = o;
}

// ---- roots ------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_mae_count(Ctx c, int32_t* counts) {
  const int t = blockIdx.y;
  const TreeSpec s = c.specs[t];
  int loc = 0;
  for (int64_t r = (int64_t)blockIdx.x * 4096 + threadIdx.x; r < (int64_t)(blockIdx.x + 1) * 4096 && r < c.n; r += NT) {
    uint32_t w;
    loc += in_bag(c, s, (uint32_t)r, w) ? 1 : 0;
  }
  __shared__ int sh[NT];
  sh[threadIdx.x] = loc;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && sh[0]) atomicAdd(&counts[t], sh[0]);
}

// tree t's in-bag rows in (y, row id) order: a stable compaction of the global order
__global__ __launch_bounds__(NT) void k_mae_fill(Ctx c, const int32_t* perm, const int64_t* row_off, uint32_t* rows) {
  const int t = blockIdx.x;
  const TreeSpec s = c.specs[t];
  __shared__ int64_t sh[NT];
  int64_t base = row_off[t];
  for (int c0 = 0; c0 < c.n; c0 += NT) {
    const int i = c0 + (int)threadIdx.x;
    uint32_t w = 0;
    const uint32_t r = i < c.n ? (uint32_t)perm[i] : 0u;
    const bool keep = i < c.n && in_bag(c, s, r, w);
    const int64_t incl = block_scan(keep ? 1 : 0, sh);
    if (keep) rows[base + incl - 1] = r;
    __shared__ int64_t tot;
    if (threadIdx.x == NT - 1) tot = incl;
    __syncthreads();
    base += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void k_mae_root(Ctx c, const int64_t* row_off, const uint32_t* rows, MaeOpen* open,
                                                 MaeOpen* open_big) {
  const int t = blockIdx.x;
  __shared__ int64_t sh[NT];
  __shared__ double v[3];
  TreeSpec s = c.specs[t];
  const int count = (int)(row_off[t + 1] - row_off[t]);
  if (threadIdx.x == 0) {
    const NodeRec leaf{-1, -1};
    c.nodes[t] = leaf;
  }
  if (count == 0) {
    if (threadIdx.x < 3) c.vals[(int64_t)t * 3 + threadIdx.x] = 0.0;
    if (threadIdx.x == 0) { c.nabs[t] = 0.0; c.tree_W[t] = 0.0; }
    return;
  }
  int64_t W, S;
  double vv[3];
  const double ab = node_stats(c, s, rows + row_off[t], count, vv, sh, W, S);
  if (threadIdx.x == 0) {
    for (int q = 0; q < 3; ++q) c.vals[(int64_t)t * 3 + q] = vv[q];
    c.nabs[t] = ab;
    c.tree_W[t] = vv[0];
    s.min_weight_leaf = s.min_weight_frac * vv[0];   // read by every later level
    c.specs[t].min_weight_leaf = s.min_weight_leaf;
    if (visit(s, count, 0, vv[0], ab)) enqueue(c, open, open_big, t, t, row_off[t], count, 0, root_key(s.seed), W, S);
  }
  (void)v;
}

// ---- one level ------------------------------------------------------------------------
struct MaeSmem {
  int64_t sh[NT];
  uint32_t hw[256], hr[256];        // per-bin weight / rows
  unsigned long long hs[256];       // per-bin sum w yq
  uint8_t cb[CHUNK], cw[CHUNK];     // staged rows: bin, weight, target
  int64_t cy[CHUNK];
  double g_b[NT];
  int64_t al_b[NT], ar_b[NT];
  int more;
  FeatRes res;
};

// feature f of the node (rows [rows, rows + cnt) in target order, sums Wn / Sn): every
// threshold's side totals from a bin histogram, then thread b scans the rows in target
// order for both sides' weighted medians; the result lands in sm.res (valid after return)
__device__ void mae_feature(const Ctx& c, const TreeSpec& s, const uint32_t* rows, int cnt, int64_t Wn, int64_t Sn,
                            int f, MaeSmem& sm) {
  const int tid = threadIdx.x;
  sm.hw[tid] = 0u; sm.hr[tid] = 0u; sm.hs[tid] = 0ull;
  __syncthreads();
  for (int i = tid; i < cnt; i += NT) {
    const uint32_t r = rows[i];
    const int b = c.Xb[(int64_t)r * c.ld + f];
    const uint32_t w = boot_weight(s, r);
    atomicAdd(&sm.hw[b], w);
    atomicAdd(&sm.hr[b], 1u);
    atomicAdd(&sm.hs[b], (unsigned long long)((int64_t)w * row_yq(c, r)));
  }
  __syncthreads();
  // thread b: prefix over bins 0..b (inclusive) -> left totals of threshold b
  const int b = tid;
  const uint32_t rb = sm.hr[b];
  const int64_t WL = block_scan((int64_t)sm.hw[b], sm.sh);
  const int64_t SL = (int64_t)(uint64_t)block_scan((int64_t)sm.hs[b], sm.sh);
  const int64_t RL = block_scan((int64_t)rb, sm.sh);
  const int64_t WR = Wn - WL, SR = (int64_t)((uint64_t)Sn - (uint64_t)SL);
  const int nrr = cnt - (int)RL;
  // the host builder's candidates: non-empty bins below 255 with rows on the right
  const bool nc_b = b < 255 && rb > 0 && nrr > 0;
  const bool cand = nc_b && (int)RL >= s.min_samples_leaf && nrr >= s.min_samples_leaf &&
                    !side_too_light(s, (double)WL, (double)WR);
  const bool nc = __syncthreads_or(nc_b ? 1 : 0) != 0;
  int64_t cwl = 0, csl = 0, cwr = 0, csr = 0;
  int64_t medl = 0, wlel = 0, slel = 0, medr = 0, wler = 0, sler = 0;
  bool fl = !cand, fr = !cand;
  for (int c0 = 0; c0 < cnt; c0 += CHUNK) {
    const int m = min(CHUNK, cnt - c0);
    if (tid == 0) sm.more = 0;
    for (int i = tid; i < m; i += NT) {
      const uint32_t r = rows[c0 + i];
      sm.cb[i] = c.Xb[(int64_t)r * c.ld + f];
      sm.cw[i] = (uint8_t)boot_weight(s, r);
      sm.cy[i] = row_yq(c, r);
    }
    __syncthreads();
    if (!(fl && fr)) {
      for (int i = 0; i < m; ++i) {
        const int64_t w = sm.cw[i], yq = sm.cy[i];
        if ((int)sm.cb[i] <= b) {
          if (!fl) {
            cwl += w; csl += w * yq;
            if (2 * cwl >= WL) { fl = true; medl = yq; wlel = cwl; slel = csl; }
          }
        } else if (!fr) {
          cwr += w; csr += w * yq;
          if (2 * cwr >= WR) { fr = true; medr = yq; wler = cwr; sler = csr; }
        }
        if (fl && fr) break;
      }
      if (!(fl && fr)) sm.more = 1;
    }
    __syncthreads();
    const int go = sm.more;
    __syncthreads();
    if (!go) break;
  }
  double g = -INFINITY;
  int64_t alq = 0, arq = 0;
  if (cand) {
    alq = mae_absdev(WL, SL, medl, wlel, slel);
    arq = mae_absdev(WR, SR, medr, wler, sler);
    g = -((double)alq + (double)arq);
  }
  sm.g_b[tid] = g; sm.al_b[tid] = alq; sm.ar_b[tid] = arq;
  __syncthreads();
  if (tid == 0) {
    // the host sweep: bins ascending, strictly greater wins (lowest bin on ties)
    double gb = -INFINITY;
    int bb = -1;
    for (int q = 0; q < 255; ++q)
      if (sm.g_b[q] > gb) { gb = sm.g_b[q]; bb = q; }
    FeatRes r;
    r.g = gb; r.bin = bb; r.nc = nc ? 1 : 0;
    r.al = bb >= 0 ? sm.al_b[bb] : 0;
    r.ar = bb >= 0 ? sm.ar_b[bb] : 0;
    int64_t wl = 0;
    for (int q = 0; q <= bb; ++q) wl += sm.hw[q];
    r.wl = wl;
    sm.res = r;
  }
  __syncthreads();
}

// the node's running selection over its visiting order (thread 0; the host loop)
struct MaeBest {
  int nonconst = 0, feat = -1, bin = -1;
  double gain = -INFINITY, al = 0.0, ar = 0.0;
  int64_t wl = 0;
};

__device__ __forceinline__ void mae_select(const Ctx& c, MaeBest& bs, const FeatRes& r, int f) {
  if (!r.nc) return;
  ++bs.nonconst;
  if (r.bin >= 0 && r.g > bs.gain) {
    bs.gain = r.g; bs.feat = f; bs.bin = r.bin;
    bs.al = (double)r.al * c.rq.i1; bs.ar = (double)r.ar * c.rq.i1; bs.wl = r.wl;
  }
}

// accept the best split (thread 0's bs), stable partition, children's medians / values,
// enqueue (all threads)
__device__ void mae_finish(const Ctx& c, const TreeSpec& s, const MaeOpen& on, const MaeBest& bs,
                           const uint32_t* rows, uint32_t* rows_next, MaeOpen* next, MaeOpen* next_big, MaeSmem& sm) {
  const int tid = threadIdx.x;
  const int cnt = on.count;
  __shared__ int sp_feat, sp_bin, sp_base;
  if (tid == 0) {
    sp_base = -1; sp_feat = bs.feat; sp_bin = bs.bin;
    if (bs.feat >= 0) {
      const double Wt = c.tree_W[on.tree];
      const double wN = (double)on.W, wL = (double)bs.wl, wR = wN - wL;
      const double imp = improvement(Wt, wN, c.nabs[on.node] / wN, wL, bs.al / wL, wR, bs.ar / wR);
      if (!(imp + kEps < (double)s.min_impurity_decrease)) {
        const int base = atomicAdd(&c.counters[0], 2);
        if ((int64_t)base + 2 > c.pool_cap) {
          atomicOr(&c.counters[2], 1);
        } else {
          const NodeRec leaf{-1, -1};
          c.nodes[base] = leaf;
          c.nodes[base + 1] = leaf;
          NodeRec rec; rec.split = pack_split(bs.feat, bs.bin); rec.left = base;
          c.nodes[on.node] = rec;
          sp_base = base;
        }
      }
    }
  }
  __syncthreads();
  const int base = sp_base;
  if (base < 0) return;
  const int feat = sp_feat, sbin = sp_bin;
  // stable partition: left rows keep their (target) order, then the right rows
  int64_t nl_total = 0;
  {
    int64_t lbase = 0, rbase = 0;
    int64_t lc = 0;
    for (int i = tid; i < cnt; i += NT) lc += (c.Xb[(int64_t)rows[i] * c.ld + feat] <= sbin) ? 1 : 0;
    nl_total = block_sum(lc, sm.sh);
    for (int c0 = 0; c0 < cnt; c0 += NT) {
      const int i = c0 + tid;
      const uint32_t r = i < cnt ? rows[i] : 0u;
      const bool left = i < cnt && c.Xb[(int64_t)r * c.ld + feat] <= sbin;
      const bool right = i < cnt && !left;
      const int64_t pl = block_scan(left ? 1 : 0, sm.sh);
      const int64_t pr = block_scan(right ? 1 : 0, sm.sh);
      if (left) rows_next[on.start + lbase + pl - 1] = r;
      if (right) rows_next[on.start + nl_total + rbase + pr - 1] = r;
      __shared__ int64_t tl, tr;
      if (tid == NT - 1) { tl = pl; tr = pr; }
      __syncthreads();
      lbase += tl; rbase += tr;
      __syncthreads();
    }
  }
  __syncthreads();
  const int nl = (int)nl_total;
  for (int side = 0; side < 2; ++side) {
    const int64_t st = on.start + (side ? nl : 0);
    const int ccount = side ? cnt - nl : nl;
    double vv[3];
    int64_t W, S;
    const double ab = node_stats(c, s, rows_next + st, ccount, vv, sm.sh, W, S);
    if (tid == 0) {
      const int node = base + side;
      for (int q = 0; q < 3; ++q) c.vals[(int64_t)node * 3 + q] = vv[q];
      c.nabs[node] = ab;
      if (visit(s, ccount, on.depth + 1, vv[0], ab))
        enqueue(c, next, next_big, on.tree, node, st, ccount, on.depth + 1, child_key(on.key, side), W, S);
    }
    __syncthreads();
  }
}

// small nodes: one workgroup per node, features one after another
__global__ __launch_bounds__(NT) void k_mae_level(Ctx c, const MaeOpen* open, MaeOpen* next, MaeOpen* next_big,
                                                  const uint32_t* rows_cur, uint32_t* rows_next) {
  const MaeOpen on = open[blockIdx.x];
  const TreeSpec s = c.specs[on.tree];
  __shared__ MaeSmem sm;
  __shared__ int nc_sh;
  const uint32_t* rows = rows_cur + on.start;
  const FeatPerm fp = feat_perm(on.key, c.d);
  MaeBest bs;
  int nonconst = 0;
  for (int pos = 0; nonconst < s.max_features && pos < c.d; ++pos) {
    const int f = feature_at(fp, pos, c.d);
    mae_feature(c, s, rows, on.count, on.W, on.S, f, sm);
    if (threadIdx.x == 0) { mae_select(c, bs, sm.res, f); nc_sh = bs.nonconst; }
    __syncthreads();
    nonconst = nc_sh;
    __syncthreads();
  }
  mae_finish(c, s, on, bs, rows, rows_next, next, next_big, sm);
}

// big nodes, step 1: one workgroup per (node, visiting position < P)
__global__ __launch_bounds__(NT) void k_mae_eval(Ctx c, const MaeOpen* big, const uint32_t* rows_cur, FeatRes* res,
                                                 int P) {
  const MaeOpen on = big[blockIdx.x];
  const TreeSpec s = c.specs[on.tree];
  const int pos = blockIdx.y;
  if (pos >= c.d) return;
  __shared__ MaeSmem sm;
  const FeatPerm fp = feat_perm(on.key, c.d);
  mae_feature(c, s, rows_cur + on.start, on.count, on.W, on.S, feature_at(fp, pos, c.d), sm);
  if (threadIdx.x == 0) res[(int64_t)blockIdx.x * P + pos] = sm.res;
}

// big nodes, step 2: selection in visiting order over the evaluated positions (further
// positions, needed only when constant features leave fewer than max_features among the
// first P, are evaluated here), then the split as for small nodes
__global__ __launch_bounds__(NT) void k_mae_decide(Ctx c, const MaeOpen* big, const FeatRes* res, int P,
                                                   MaeOpen* next, MaeOpen* next_big, const uint32_t* rows_cur,
                                                   uint32_t* rows_next) {
  const MaeOpen on = big[blockIdx.x];
  const TreeSpec s = c.specs[on.tree];
  __shared__ MaeSmem sm;
  __shared__ int nc_sh;
  const uint32_t* rows = rows_cur + on.start;
  const FeatPerm fp = feat_perm(on.key, c.d);
  MaeBest bs;
  int nonconst = 0;
  for (int pos = 0; nonconst < s.max_features && pos < c.d; ++pos) {
    const int f = feature_at(fp, pos, c.d);
    if (pos < P) {
      if (threadIdx.x == 0) mae_select(c, bs, res[(int64_t)blockIdx.x * P + pos], f);
    } else {
      mae_feature(c, s, rows, on.count, on.W, on.S, f, sm);
      if (threadIdx.x == 0) mae_select(c, bs, sm.res, f);
    }
    if (threadIdx.x == 0) nc_sh = bs.nonconst;
    __syncthreads();
    nonconst = nc_sh;
    __syncthreads();
  }
  mae_finish(c, s, on, bs, rows, rows_next, next, next_big, sm);
}

}  // namespace mae
}  // namespace dml

using namespace dml;
using namespace dml::mae;

#define MAE_OK(x) do { if ((x) != hipSuccess) return 1; } while (0)

extern "C" {

int dml_mae_sizeof_args() { return (int)sizeof(MaeArgs); }
int dml_mae_sizeof_open() { return (int)sizeof(MaeOpen); }
int dml_mae_sizeof_res() { return (int)sizeof(FeatRes); }

// in-bag rows per tree (a->counts zeroed by the caller)
int dml_mae_count(MaeArgs* a, hipStream_t st) {
  if (a->T <= 0 || a->n <= 0) return 0;
  const Ctx c = make_ctx(a);
  k_mae_count<<<dim3((unsigned)((a->n + 4095) / 4096), (unsigned)a->T), NT, 0, st>>>(c, reinterpret_cast<int32_t*>(a->counts));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// the whole build: roots, then one k_mae_level launch per level (the open count is read back
// per level); status_out 1 = node pool or open-list overflow (the caller regrows)
int dml_mae_build(MaeArgs* a, hipStream_t st) {
  a->status_out = 0;
  a->levels_out = 0;
  if (a->T <= 0) { a->n_nodes_out = 0; return 0; }
  const Ctx c = make_ctx(a);
  int32_t* counters = reinterpret_cast<int32_t*>(a->counters);
  MaeOpen* open[2] = {reinterpret_cast<MaeOpen*>(a->open_a), reinterpret_cast<MaeOpen*>(a->open_b)};
  MaeOpen* big[2] = {reinterpret_cast<MaeOpen*>(a->big_a), reinterpret_cast<MaeOpen*>(a->big_b)};
  FeatRes* res = reinterpret_cast<FeatRes*>(a->res);
  const int P = (int)a->P;
  uint32_t* rows[2] = {reinterpret_cast<uint32_t*>(a->rows_a), reinterpret_cast<uint32_t*>(a->rows_b)};
  MAE_OK(hipMemsetAsync(counters, 0, 8 * sizeof(int32_t), st));
  const int32_t pool0 = (int32_t)a->T;   // nodes [0, T) are the roots
  MAE_OK(hipMemcpyAsync(counters, &pool0, sizeof(int32_t), hipMemcpyHostToDevice, st));
  k_mae_fill<<<(unsigned)a->T, NT, 0, st>>>(c, reinterpret_cast<const int32_t*>(a->perm),
                                            reinterpret_cast<const int64_t*>(a->row_off), rows[0]);
  k_mae_root<<<(unsigned)a->T, NT, 0, st>>>(c, reinterpret_cast<const int64_t*>(a->row_off), rows[0], open[0], big[0]);
  MAE_OK(hipGetLastError());
  int cur = 0;
  int32_t h[4];
  while (true) {
    MAE_OK(hipMemcpyAsync(h, counters, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    MAE_OK(hipStreamSynchronize(st));
    if (h[2]) { a->status_out = 1; break; }
    const int n_open = h[1], n_big = h[3];
    if (n_open == 0 && n_big == 0) break;
    if (++a->levels_out > (1 << 20)) { a->status_out = 2; break; }   // a node never shrinks: cannot happen
    MAE_OK(hipMemsetAsync(counters + 1, 0, sizeof(int32_t), st));
    MAE_OK(hipMemsetAsync(counters + 3, 0, sizeof(int32_t), st));
    // a level's children are written at their parents' positions: rows of unsplit nodes are
    // not copied (nobody reads them again)
    if (n_big) {
      k_mae_eval<<<dim3((unsigned)n_big, (unsigned)P), NT, 0, st>>>(c, big[cur], rows[cur], res, P);
      k_mae_decide<<<(unsigned)n_big, NT, 0, st>>>(c, big[cur], res, P, open[1 - cur], big[1 - cur], rows[cur],
                                                   rows[1 - cur]);
    }
    if (n_open)
      k_mae_level<<<(unsigned)n_open, NT, 0, st>>>(c, open[cur], open[1 - cur], big[1 - cur], rows[cur], rows[1 - cur]);
    MAE_OK(hipGetLastError());
    cur = 1 - cur;
  }
  MAE_OK(hipMemcpyAsync(h, counters, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  MAE_OK(hipStreamSynchronize(st));
  a->n_nodes_out = h[0];
  if (h[2]) a->status_out = 1;
  return 0;
}

}  // extern "C"
