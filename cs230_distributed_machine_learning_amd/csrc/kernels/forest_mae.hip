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
  int64_t counters;             // int32 [8]: 0 pool, 1 open count (next), 2 overflow
  int64_t tree_W;               // double [T]
  int64_t n_nodes_out, levels_out, status_out;
};

struct MaeOpen {
  int32_t tree, node;
  int64_t start;
  int32_t count, depth;
  uint64_t key;
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
  int64_t open_cap;
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
                             int64_t* sh, int64_t& Wout) {
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
  return mae_node_value(W, S, found_k >= 0 ? f_c : 0, found_k >= 0 ? f_cs : 0, row_yq(c, rk), ylo, yhi, tie, c.rq,
                        v);
}

__device__ bool visit(const TreeSpec& s, int count, int depth, double W, double ab) {
  return !(leaf_by_counts(s, count, depth) || leaf_by_weight(s, W) || (W > 0.0 ? ab / W : 0.0) <= kEps);
}

__device__ void enqueue(const Ctx& c, MaeOpen* out, int tree, int node, int64_t start, int count, int depth,
                        uint64_t key) {
  const int idx = atomicAdd(&c.counters[1], 1);
  if (idx >= c.open_cap) { atomicOr(&c.counters[2], 1); return; }
  MaeOpen o;
  o.tree = tree; o.node = node; o.start = start; o.count = count; o.depth = depth; o.key = key;
  out[idx] = o;
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

__global__ __launch_bounds__(NT) void k_mae_root(Ctx c, const int64_t* row_off, const uint32_t* rows, MaeOpen* open) {
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
  int64_t W;
  double vv[3];
  const double ab = node_stats(c, s, rows + row_off[t], count, vv, sh, W);
  if (threadIdx.x == 0) {
    for (int q = 0; q < 3; ++q) c.vals[(int64_t)t * 3 + q] = vv[q];
    c.nabs[t] = ab;
    c.tree_W[t] = vv[0];
    s.min_weight_leaf = s.min_weight_frac * vv[0];   // read by every later level
    c.specs[t].min_weight_leaf = s.min_weight_leaf;
    if (visit(s, count, 0, vv[0], ab)) enqueue(c, open, t, t, row_off[t], count, 0, root_key(s.seed));
  }
  (void)v;
}

// ---- one level: one workgroup per open node ---------------------------------------------
__global__ __launch_bounds__(NT) void k_mae_level(Ctx c, const MaeOpen* open, MaeOpen* next, const uint32_t* rows_cur,
                                                  uint32_t* rows_next) {
  const MaeOpen on = open[blockIdx.x];
  const TreeSpec s = c.specs[on.tree];
  const int tid = threadIdx.x;
  const int cnt = on.count;
  const uint32_t* rows = rows_cur + on.start;
  __shared__ int64_t sh[NT];
  __shared__ uint32_t hw[256], hr[256];        // per-bin weight / rows
  __shared__ unsigned long long hs[256];       // per-bin sum w yq
  __shared__ uint8_t cb[CHUNK], cw[CHUNK];     // staged rows: bin, weight, target
  __shared__ int64_t cy[CHUNK];
  __shared__ double g_b[NT];
  __shared__ int64_t al_b[NT], ar_b[NT];
  __shared__ int more;
  // node totals (integers)
  int64_t wloc = 0, sloc = 0;
  for (int i = tid; i < cnt; i += NT) {
    const uint32_t r = rows[i];
    const int64_t w = (int64_t)boot_weight(s, r);
    wloc += w;
    sloc += w * row_yq(c, r);
  }
  const int64_t Wn = block_sum(wloc, sh), Sn = (int64_t)(uint64_t)block_sum(sloc, sh);
  const FeatPerm fp = feat_perm(on.key, c.d);
  int nonconst = 0, best_feat = -1, best_bin = -1;
  double best_gain = -INFINITY, mae_l = 0.0, mae_r = 0.0;
  int64_t best_wl = 0;
  for (int pos = 0; nonconst < s.max_features && pos < c.d; ++pos) {
    const int f = feature_at(fp, pos, c.d);
    // (1) per-bin totals
    hw[tid] = 0u; hr[tid] = 0u; hs[tid] = 0ull;
    __syncthreads();
    for (int i = tid; i < cnt; i += NT) {
      const uint32_t r = rows[i];
      const int b = c.Xb[(int64_t)r * c.ld + f];
      const uint32_t w = boot_weight(s, r);
      atomicAdd(&hw[b], w);
      atomicAdd(&hr[b], 1u);
      atomicAdd(&hs[b], (unsigned long long)((int64_t)w * row_yq(c, r)));
    }
    __syncthreads();
    // thread b: prefix over bins 0..b (inclusive) -> left totals of threshold b
    const int b = tid;
    const uint32_t rb = hr[b];
    const int64_t WL = block_scan((int64_t)hw[b], sh);
    const int64_t SL = (int64_t)(uint64_t)block_scan((int64_t)hs[b], sh);
    const int64_t RL = block_scan((int64_t)rb, sh);
    const int64_t WR = Wn - WL, SR = (int64_t)((uint64_t)Sn - (uint64_t)SL);
    const int nrr = cnt - (int)RL;
    // the host builder's candidates: non-empty bins below 255 with rows on the right
    const bool nc_b = b < 255 && rb > 0 && nrr > 0;
    bool cand = nc_b && (int)RL >= s.min_samples_leaf && nrr >= s.min_samples_leaf &&
                !side_too_light(s, (double)WL, (double)WR);
    const bool nc = __syncthreads_or(nc_b ? 1 : 0) != 0;
    // (2) medians of both sides for every candidate threshold: one scan in target order
    int64_t cwl = 0, csl = 0, cwr = 0, csr = 0;
    int64_t medl = 0, wlel = 0, slel = 0, medr = 0, wler = 0, sler = 0;
    bool fl = !cand, fr = !cand;
    for (int c0 = 0; c0 < cnt; c0 += CHUNK) {
      const int m = min(CHUNK, cnt - c0);
      if (tid == 0) more = 0;
      for (int i = tid; i < m; i += NT) {
        const uint32_t r = rows[c0 + i];
        cb[i] = c.Xb[(int64_t)r * c.ld + f];
        cw[i] = (uint8_t)boot_weight(s, r);
        cy[i] = row_yq(c, r);
      }
      __syncthreads();
      if (!(fl && fr)) {
        for (int i = 0; i < m; ++i) {
          const int64_t w = cw[i], yq = cy[i];
          if ((int)cb[i] <= b) {
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
        if (!(fl && fr)) more = 1;
      }
      __syncthreads();
      const int go = more;
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
    g_b[tid] = g; al_b[tid] = alq; ar_b[tid] = arq;
    __syncthreads();
    if (tid == 0) {
      // the host sweep: bins ascending, strictly greater wins (lowest bin on ties)
      double gb = -INFINITY;
      int bb = -1;
      for (int q = 0; q < 255; ++q)
        if (g_b[q] > gb) { gb = g_b[q]; bb = q; }
      if (nc) {
        ++nonconst;
        if (bb >= 0 && gb > best_gain) {
          best_gain = gb; best_feat = f; best_bin = bb;
          mae_l = (double)al_b[bb] * c.rq.i1; mae_r = (double)ar_b[bb] * c.rq.i1;
        }
      }
      sh[0] = nonconst;
    }
    __syncthreads();
    nonconst = (int)sh[0];
    if (tid == 0 && best_bin >= 0 && best_feat == f) {
      // the chosen threshold's left weight (prefix of hw up to best_bin)
      int64_t wl = 0;
      for (int q = 0; q <= best_bin; ++q) wl += hw[q];
      best_wl = wl;
    }
    __syncthreads();
  }
  // ---- decision (thread 0), broadcast through LDS
  __shared__ int sp_feat, sp_bin, sp_base, sp_nl;
  if (tid == 0) {
    sp_base = -1; sp_feat = best_feat; sp_bin = best_bin; sp_nl = 0;
    if (best_feat >= 0) {
      const double Wt = c.tree_W[on.tree];
      const double wN = (double)Wn, wL = (double)best_wl, wR = wN - wL;
      const double imp = improvement(Wt, wN, c.nabs[on.node] / wN, wL, mae_l / wL, wR, mae_r / wR);
      if (!(imp + kEps < (double)s.min_impurity_decrease)) {
        const int base = atomicAdd(&c.counters[0], 2);
        if ((int64_t)base + 2 > c.pool_cap) {
          atomicOr(&c.counters[2], 1);
        } else {
          const NodeRec leaf{-1, -1};
          c.nodes[base] = leaf;
          c.nodes[base + 1] = leaf;
          NodeRec rec; rec.split = pack_split(best_feat, best_bin); rec.left = base;
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
  // ---- stable partition: left rows keep their (target) order, then the right rows
  int64_t nl_total = 0;
  {
    int64_t lbase = 0, rbase = 0;
    // left count first (the right block starts after it)
    int64_t lc = 0;
    for (int i = tid; i < cnt; i += NT) lc += (c.Xb[(int64_t)rows[i] * c.ld + feat] <= sbin) ? 1 : 0;
    nl_total = block_sum(lc, sh);
    for (int c0 = 0; c0 < cnt; c0 += NT) {
      const int i = c0 + tid;
      const uint32_t r = i < cnt ? rows[i] : 0u;
      const bool left = i < cnt && c.Xb[(int64_t)r * c.ld + feat] <= sbin;
      const bool right = i < cnt && !left;
      const int64_t pl = block_scan(left ? 1 : 0, sh);
      const int64_t pr = block_scan(right ? 1 : 0, sh);
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
  // ---- children: medians, abs deviations, values; enqueue the ones worth visiting
  const int nl = (int)nl_total;
  for (int side = 0; side < 2; ++side) {
    const int64_t st = on.start + (side ? nl : 0);
    const int ccount = side ? cnt - nl : nl;
    double vv[3];
    int64_t W;
    const double ab = node_stats(c, s, rows_next + st, ccount, vv, sh, W);
    if (tid == 0) {
      const int node = base + side;
      for (int q = 0; q < 3; ++q) c.vals[(int64_t)node * 3 + q] = vv[q];
      c.nabs[node] = ab;
      if (visit(s, ccount, on.depth + 1, vv[0], ab))
        enqueue(c, next, on.tree, node, st, ccount, on.depth + 1, child_key(on.key, side));
    }
    __syncthreads();
  }
}

}  // namespace mae
}  // namespace dml

using namespace dml;
using namespace dml::mae;

#define MAE_OK(x) do { if ((x) != hipSuccess) return 1; } while (0)

extern "C" {

int dml_mae_sizeof_args() { return (int)sizeof(MaeArgs); }
int dml_mae_sizeof_open() { return (int)sizeof(MaeOpen); }

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
  uint32_t* rows[2] = {reinterpret_cast<uint32_t*>(a->rows_a), reinterpret_cast<uint32_t*>(a->rows_b)};
  MAE_OK(hipMemsetAsync(counters, 0, 8 * sizeof(int32_t), st));
  const int32_t pool0 = (int32_t)a->T;   // nodes [0, T) are the roots
  MAE_OK(hipMemcpyAsync(counters, &pool0, sizeof(int32_t), hipMemcpyHostToDevice, st));
  k_mae_fill<<<(unsigned)a->T, NT, 0, st>>>(c, reinterpret_cast<const int32_t*>(a->perm),
                                            reinterpret_cast<const int64_t*>(a->row_off), rows[0]);
  k_mae_root<<<(unsigned)a->T, NT, 0, st>>>(c, reinterpret_cast<const int64_t*>(a->row_off), rows[0], open[0]);
  MAE_OK(hipGetLastError());
  int cur = 0;
  int32_t h[4];
  while (true) {
    MAE_OK(hipMemcpyAsync(h, counters, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    MAE_OK(hipStreamSynchronize(st));
    if (h[2]) { a->status_out = 1; break; }
    const int n_open = h[1];
    if (n_open == 0) break;
    if (++a->levels_out > (1 << 20)) { a->status_out = 2; break; }   // a node never shrinks: cannot happen
    MAE_OK(hipMemsetAsync(counters + 1, 0, sizeof(int32_t), st));
    // a level's children are written at their parents' positions: rows of unsplit nodes are
    // not copied (nobody reads them again)
    k_mae_level<<<(unsigned)n_open, NT, 0, st>>>(c, open[cur], open[1 - cur], rows[cur], rows[1 - cur]);
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
