// forest_cpu.cpp — CPU random-forest builder/predictor (the plumbing/CI path).
//
// Grows exactly the trees the HIP builder (../kernels/forest.hip) grows: both take
// every random decision (bootstrap weights, per-node feature order) and every split
// score from forest_common.h, classification histograms are exact integers, and
// ties break identically (earliest feature in visit order, then lowest bin).  The GPU
// builds breadth-first with atomic node allocation; this builds depth-first with a
// local counter; `dml_cpu_forest_export` renumbers into the GPU's pool layout (tree t's
// root at index t, children in consecutive pairs) so predictions are comparable
// element-for-element.
//
// Used when no GPU is present (BASELINE config 1: the iris plumbing job) and as the
// oracle for the HIP kernels' tests.  Trees are built in parallel with OpenMP.
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <vector>
#include <algorithm>
#include "../kernels/forest_common.h"

namespace dml {

struct CpuTree {
  std::vector<NodeRec> nodes;   // local numbering, root = 0
  std::vector<double> vals;     // [nodes][VC]
};

struct CpuForest {
  int T = 0, VC = 0;
  std::vector<CpuTree> trees;
};

struct Data {
  const uint8_t* Xb; int64_t ld; int n, d, C, CH, VC, is_reg;
  const int32_t* ycls; const float* yreg; const uint8_t* roles;
  int64_t ystride;
  const double* cw;   // class-weight table [T][C] (rows of cw_mode 1 trees), or null
  const int8_t* mono; // monotonic_cst table [fits][d] (+1 / -1 / 0; binary classifiers'
                      // rows already constrain the class-0 fraction), or null
  RegScale rq;        // regression fixed point (forest_common.h)
  const int64_t* yq;  // per (target, row): rint(y 2^e1), rint(y^2 2^e2) -- computed once per build
  const int64_t* y2q;
};

struct Job { int node, start, count, depth; uint64_t key; double lo, hi; };

// Fenwick tree over the y-ranks of one node's rows: integer weights and weighted
// fixed-point targets (w yq, forest_common.h reg_quantize), so the abs deviations -- and the
// MAE split choice -- are exact integers, the same on the HIP builder (forest_mae.hip)
struct Fenwick {
  int m = 0;
  std::vector<int64_t> w, s;
  void reset(int m_) { m = m_; w.assign(m + 1, 0); s.assign(m + 1, 0); }
  void fill(const int64_t* ws, const int64_t* yq) {   // every rank present: linear build
    for (int i = 1; i <= m; ++i) { w[i] = ws[i - 1]; s[i] = ws[i - 1] * yq[i - 1]; }
    for (int i = 1; i <= m; ++i) {
      const int j = i + (i & -i);
      if (j <= m) { w[j] += w[i]; s[j] += s[i]; }
    }
  }
  void add(int r, int64_t dw, int64_t ds) {
    for (int i = r + 1; i <= m; i += i & -i) { w[i] += dw; s[i] += ds; }
  }
  // sum w |yq - median| of the set (total weight W, weighted sum S): the deviation is the
  // same for every median of the set, so take the lowest rank whose prefix reaches W/2
  int64_t absdev(int64_t W, int64_t S, const int64_t* yq) const {
    int pos = 0, step = 1;
    while (step * 2 <= m) step *= 2;
    int64_t cw = 0;
    for (; step; step >>= 1)
      if (pos + step <= m && 2 * (cw + w[pos + step]) < W) { pos += step; cw += w[pos]; }
    return mae_absdev(W, S, yq[pos], prefix_w(pos), prefix_s(pos));
  }
  int64_t prefix_w(int pos) const { int64_t r = 0; for (int i = pos + 1; i > 0; i -= i & -i) r += w[i]; return r; }
  int64_t prefix_s(int pos) const { int64_t r = 0; for (int i = pos + 1; i > 0; i -= i & -i) r += s[i]; return r; }
};

static void build_tree(const Data& D, const TreeSpec& s_in, int64_t t, CpuTree& out) {
  TreeSpec s = s_in;   // min_weight_leaf is set once the tree's total weight is known
  const uint8_t* role = D.roles + (int64_t)s.split * D.n;
  const float* Y = D.ystride ? D.yreg + (int64_t)s.target * D.ystride : D.yreg;
  const int64_t* YQ = D.is_reg ? D.yq + (D.ystride ? (int64_t)s.target * D.ystride : 0) : nullptr;
  const int64_t* Y2Q = D.is_reg ? D.y2q + (D.ystride ? (int64_t)s.target * D.ystride : 0) : nullptr;
  std::vector<uint32_t> rows, tmp;
  std::vector<uint32_t> wts;  // indexed by row id through a parallel array
  rows.reserve(D.n);
  std::vector<uint32_t> wrow(D.n, 0);
  std::vector<double> root(D.VC, 0.0);
  uint64_t rw = 0, ry = 0, ryy = 0;   // regression root sums (integer, see forest_common.h)
  for (int r = 0; r < D.n; ++r) {
    if (role[r] != 1) continue;
    const uint32_t w = boot_weight(s, (uint32_t)r);
    if (!w) continue;
    rows.push_back((uint32_t)r);
    wrow[r] = w;
    if (D.is_reg) {
      rw += w; ry += (uint64_t)((int64_t)w * YQ[r]); ryy += (uint64_t)((int64_t)w * Y2Q[r]);
    } else {
      root[D.ycls[r]] += (double)w;
    }
  }
  if (D.is_reg) { root[0] = (double)rw; root[1] = reg_s1(ry, D.rq); root[2] = reg_s2(ryy, D.rq); }
  tmp.resize(rows.size());
  // criterion="absolute_error" (sklearn MAE): node value = weighted median, impurity =
  // sum w |y - median| / W.  Node values are stored as {W, W*median, abs + W*median^2}
  // so that v1/v0 is the median (what predict reads) and mse_impurity(v) is the MAE
  // impurity (what max_leaf_nodes / ccp_alpha pruning read); the exact abs sums of the
  // nodes are kept aside for the purity and acceptance tests
  const bool mae = D.is_reg && s.criterion == kMAE;
  std::vector<double> nabs;
  std::vector<uint32_t> ord;
  std::vector<double> ys;
  std::vector<int64_t> ws, yqs;
  std::vector<int32_t> rank_of(mae ? D.n : 0);
  Fenwick fl, fr;
  auto sort_rows = [&](int start, int count) {   // node rows by (y, row id)
    ord.assign(rows.begin() + start, rows.begin() + start + count);
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return Y[a] < Y[b] || (Y[a] == Y[b] && a < b); });
    ys.resize(count); ws.resize(count); yqs.resize(count);
    for (int k = 0; k < count; ++k) {
      ys[k] = (double)Y[ord[k]]; ws[k] = (int64_t)wrow[ord[k]]; yqs[k] = YQ[ord[k]]; rank_of[ord[k]] = k;
    }
  };
  auto mae_node = [&](int start, int count, double* v) {   // sklearn WeightedMedianCalculator
    sort_rows(start, count);
    int64_t W = 0, S = 0;
    for (int k = 0; k < count; ++k) { W += ws[k]; S += ws[k] * yqs[k]; }
    int64_t c = 0, cs = 0;
    int k = 0;
    while (k < count && 2 * c < W) { c += ws[k]; cs += ws[k] * yqs[k]; ++k; }
    const int km = k > 0 ? k - 1 : 0;
    return mae_node_value(W, S, c, cs, yqs[km], ys[km], (2 * c == W && k < count) ? ys[k] : ys[km],
                          2 * c == W && k < count, D.rq, v);
  };
  if (mae && !rows.empty()) nabs.push_back(mae_node(0, (int)rows.size(), root.data()));
  // class weights multiply the (integer) class sums: root statistics here, every
  // histogram channel below -- exactly where the HIP builder applies them
  std::vector<double> cwv(D.is_reg ? 0 : D.C, 1.0);
  if (!D.is_reg && s.cw_mode != 0) {
    if (s.cw_mode == 2) balanced_weights(root.data(), D.C, cwv.data());
    else if (D.cw) for (int k = 0; k < D.C; ++k) cwv[k] = D.cw[t * D.C + k];
    for (int k = 0; k < D.C; ++k) root[k] *= cwv[k];
  }
  out.nodes.clear(); out.vals.clear();
  NodeRec leaf{-1, -1};
  out.nodes.push_back(leaf);
  out.vals.insert(out.vals.end(), root.begin(), root.end());
  double Wt = 0.0;
  if (D.is_reg) Wt = root[0];
  else for (int k = 0; k < D.C; ++k) Wt += root[k];
  s.min_weight_leaf = s.min_weight_frac * Wt;

  auto impurity_of = [&](const double* v) {
    if (D.is_reg) return mse_impurity(v[0], v[1], v[2]);
    ClsAcc a; a.init(s.criterion);
    for (int k = 0; k < D.C; ++k) a.add(v[k]);
    return cls_impurity(a, s.criterion);
  };
  // monotonic_cst (sklearn >= 1.4): a constrained feature's split must keep the children's
  // values ordered and inside the node's bounds; the children's bounds meet at the mean of
  // the two values (sklearn's middle_value rounding); every node value is clipped to its bounds once the tree is grown
  const int8_t* mono = D.mono ? D.mono + (int64_t)s.fit * D.d : nullptr;
  std::vector<double> nlo(1, -INFINITY), nhi(1, INFINITY);   // (helpers: forest_common.h)
  auto node_imp = [&](int node, const double* v) { return mae ? nabs[node] / v[0] : impurity_of(v); };
  auto visit = [&](int count, int depth, const double* v, double imp) {
    const bool pure = (D.is_reg && !mae) ? reg_pure(v, D.rq) : imp <= kEps;
    return !(leaf_by_counts(s, count, depth) || leaf_by_weight(s, vals_weight(v, D.C, D.is_reg)) || pure);
  };

  std::vector<Job> stack;
  if (!rows.empty() && visit((int)rows.size(), 0, root.data(), node_imp(0, root.data())))
    stack.push_back({0, 0, (int)rows.size(), 0, root_key(s.seed), -INFINITY, INFINITY});
  const int CH = D.CH;
  std::vector<uint32_t> hu((size_t)CH * 256);
  std::vector<uint64_t> hr((size_t)3 * 256);   // regression: (w | rows << 32), sum w yq, sum w y2q
  std::vector<double> best_left(CH), cand_left(CH);
  while (!stack.empty()) {
    Job jb = stack.back();
    stack.pop_back();
    const FeatPerm fp = feat_perm(jb.key, D.d);
    int pos = 0, nonconst = 0, best_feat = -1, best_bin = -1;
    double best_gain = -INFINITY;
    const uint32_t* nr = rows.data() + jb.start;
    double mae_l = 0.0, mae_r = 0.0;   // abs sums of the best split's sides
    double best_mid = 0.0;             // mean of the best split's two side values
    int64_t Wn = 0, Sn = 0;
    int bcnt[256];
    if (mae) {
      sort_rows(jb.start, jb.count);
      for (int k = 0; k < jb.count; ++k) { Wn += ws[k]; Sn += ws[k] * yqs[k]; }
    }
    while (nonconst < s.max_features && pos < D.d) {
      const int f = feature_at(fp, pos, D.d);
      ++pos;
      double g_best = -INFINITY;
      int b_best = -1;
      bool nc = false;
      if (mae) {
        // exact MAE sweep: rows enter the left set bin by bin; the medians and abs
        // deviations of both sides come from Fenwick trees over the node's y-ranks
        std::fill(bcnt, bcnt + 256, 0);
        for (int i = 0; i < jb.count; ++i) ++bcnt[D.Xb[(int64_t)nr[i] * D.ld + f]];
        std::vector<int> boff(257, 0);
        for (int b = 0; b < 256; ++b) boff[b + 1] = boff[b] + bcnt[b];
        std::vector<uint32_t> byb(jb.count);
        { std::vector<int> cur(boff.begin(), boff.end() - 1);
          for (int i = 0; i < jb.count; ++i) byb[cur[D.Xb[(int64_t)nr[i] * D.ld + f]]++] = nr[i]; }
        fl.reset(jb.count); fr.reset(jb.count); fr.fill(ws.data(), yqs.data());
        int64_t Wl = 0, Sl = 0;
        int nl = 0;
        for (int b = 0; b < 255; ++b) {
          if (!bcnt[b]) continue;
          for (int i = boff[b]; i < boff[b + 1]; ++i) {
            const int k = rank_of[byb[i]];
            const int64_t w = ws[k], wy = w * yqs[k];
            fl.add(k, w, wy); fr.add(k, -w, -wy);
            Wl += w; Sl += wy;
          }
          nl += bcnt[b];
          const int nrr = jb.count - nl;
          if (nrr == 0) break;
          nc = true;
          if (nl < s.min_samples_leaf || nrr < s.min_samples_leaf) continue;
          if (side_too_light(s, (double)Wl, (double)(Wn - Wl))) continue;
          const int64_t al = fl.absdev(Wl, Sl, yqs.data()), ar = fr.absdev(Wn - Wl, Sn - Sl, yqs.data());
          // the gain -(al + ar) as a double of the exact integer sum (the HIP builder's value)
          const double g = -((double)al + (double)ar);
          if (g > g_best) {
            g_best = g; b_best = b;
            if (g > best_gain) { mae_l = (double)al * D.rq.i1; mae_r = (double)ar * D.rq.i1; best_left[0] = (double)Wl; }
          }
        }
        if (nc) {
          ++nonconst;
          if (b_best >= 0 && g_best > best_gain) { best_gain = g_best; best_feat = f; best_bin = b_best; }
        }
      } else if (!D.is_reg) {
        std::fill(hu.begin(), hu.end(), 0u);
        for (int i = 0; i < jb.count; ++i) {
          const uint32_t r = nr[i];
          const int b = D.Xb[(int64_t)r * D.ld + f];
          hu[D.ycls[r] * 256 + b] += wrow[r];
          hu[D.C * 256 + b] += 1u;
        }
        for (int ch = 0; ch < CH; ++ch)
          for (int b = 1; b < 256; ++b) hu[ch * 256 + b] += hu[ch * 256 + b - 1];
        const uint32_t tot_rows = hu[D.C * 256 + 255];
        for (int b = 0; b < 255; ++b) {
          const uint32_t rl = hu[D.C * 256 + b], rr = tot_rows - rl;
          nc |= (rl > 0 && rr > 0);
          if (rl < (uint32_t)s.min_samples_leaf || rr < (uint32_t)s.min_samples_leaf) continue;
          ClsAcc L, R; L.init(s.criterion); R.init(s.criterion);
          for (int k = 0; k < D.C; ++k) {
            const double lc = (double)hu[k * 256 + b] * cwv[k], tc = (double)hu[k * 256 + 255] * cwv[k];
            L.add(lc); R.add(tc - lc);
          }
          if (side_too_light(s, L.w, R.w)) continue;
          const double l0 = (double)hu[b] * cwv[0], t0c = (double)hu[255] * cwv[0];
          const double vl = side_value(L.w, l0), vr = side_value(R.w, t0c - l0);
          if (mono && mono[f] && !mono_ok(mono[f], jb.lo, jb.hi, vl, vr)) continue;
          const double g = cls_proxy(L, R, s.criterion);
          if (g > g_best) {
            g_best = g; b_best = b;
            if (g > best_gain) best_mid = mono_mid(L.w, l0, R.w, t0c - l0);
          }
        }
        if (nc) {
          ++nonconst;
          if (b_best >= 0 && g_best > best_gain) {
            best_gain = g_best; best_feat = f; best_bin = b_best;
            for (int ch = 0; ch < CH; ++ch) best_left[ch] = (double)hu[ch * 256 + b_best] * (ch < D.C ? cwv[ch] : 1.0);
          }
        }
      } else {
        std::fill(hr.begin(), hr.end(), 0ull);
        for (int i = 0; i < jb.count; ++i) {
          const uint32_t r = nr[i];
          const int b = D.Xb[(int64_t)r * D.ld + f];
          const int64_t w = wrow[r];
          hr[b] += (uint64_t)w | (1ull << 32); hr[256 + b] += (uint64_t)(w * YQ[r]); hr[512 + b] += (uint64_t)(w * Y2Q[r]);
        }
        for (int ch = 0; ch < 3; ++ch)
          for (int b = 1; b < 256; ++b) hr[ch * 256 + b] += hr[ch * 256 + b - 1];
        const uint32_t tot_rows = (uint32_t)(hr[255] >> 32);
        for (int b = 0; b < 255; ++b) {
          const uint32_t rl = (uint32_t)(hr[b] >> 32), rr = tot_rows - rl;
          nc |= (rl > 0 && rr > 0);
          if (rl < (uint32_t)s.min_samples_leaf || rr < (uint32_t)s.min_samples_leaf) continue;
          const double l0 = reg_w(hr[b]), t0 = reg_w(hr[255]), l1 = reg_s1(hr[256 + b], D.rq),
                       t1 = reg_s1(hr[256 + 255], D.rq);
          if (side_too_light(s, l0, t0 - l0)) continue;
          const double vl = side_value(l0, l1), vr = side_value(t0 - l0, t1 - l1);
          if (mono && mono[f] && !mono_ok(mono[f], jb.lo, jb.hi, vl, vr)) continue;
          const double g = reg_proxy(s.criterion, l0, l1, t0 - l0, t1 - l1);
          if (g > g_best) {
            g_best = g; b_best = b;
            if (g > best_gain) best_mid = mono_mid(l0, l1, t0 - l0, t1 - l1);
          }
        }
        if (nc) {
          ++nonconst;
          if (b_best >= 0 && g_best > best_gain) {
            best_gain = g_best; best_feat = f; best_bin = b_best;
            const uint64_t* h = hr.data() + b_best;
            best_left[0] = reg_w(h[0]); best_left[1] = reg_s1(h[256], D.rq); best_left[2] = reg_s2(h[512], D.rq);
            best_left[3] = reg_rows(h[0]);
          }
        }
      }
    }
    if (best_feat < 0) continue;
    // accept?
    const double* pv = out.vals.data() + (size_t)jb.node * D.VC;
    double impN, impL, impR, wN, wL, wR;
    if (mae) {
      wN = pv[0]; wL = best_left[0]; wR = pv[0] - best_left[0];
      impN = nabs[jb.node] / wN; impL = mae_l / wL; impR = mae_r / wR;
    } else if (D.is_reg) {
      wN = pv[0]; wL = best_left[0]; wR = pv[0] - best_left[0];
      impN = mse_impurity(pv[0], pv[1], pv[2]);
      impL = mse_impurity(best_left[0], best_left[1], best_left[2]);
      impR = mse_impurity(pv[0] - best_left[0], pv[1] - best_left[1], pv[2] - best_left[2]);
    } else {
      ClsAcc N, L, R; N.init(s.criterion); L.init(s.criterion); R.init(s.criterion);
      for (int k = 0; k < D.C; ++k) { N.add(pv[k]); L.add(best_left[k]); R.add(pv[k] - best_left[k]); }
      wN = N.w; wL = L.w; wR = R.w;
      impN = cls_impurity(N, s.criterion); impL = cls_impurity(L, s.criterion); impR = cls_impurity(R, s.criterion);
    }
    const double imp = mae ? improvement(Wt, wN, impN, wL, impL, wR, impR)
                           : accept_improvement(s, D.is_reg != 0, pv, best_left.data(), Wt, wN, impN, wL, impL, wR, impR);
    if (imp + kEps < (double)s.min_impurity_decrease) continue;
    // split
    const int base = (int)out.nodes.size();
    out.nodes.push_back(leaf);
    out.nodes.push_back(leaf);
    out.vals.resize((size_t)(base + 2) * D.VC);
    pv = out.vals.data() + (size_t)jb.node * D.VC;
    double* lv = out.vals.data() + (size_t)base * D.VC;
    double* rv = lv + D.VC;
    if (!mae)
      for (int k = 0; k < D.VC; ++k) { lv[k] = best_left[k]; rv[k] = pv[k] - best_left[k]; }
    out.nodes[jb.node].split = pack_split(best_feat, best_bin);
    out.nodes[jb.node].left = base;
    const int nl = (int)best_left[CH - 1];
    // stable partition
    uint32_t* nrw = rows.data() + jb.start;
    int li = 0, ri = 0;
    uint32_t* tw = tmp.data();
    for (int i = 0; i < jb.count; ++i) {
      const uint32_t r = nrw[i];
      if (D.Xb[(int64_t)r * D.ld + best_feat] <= best_bin) nrw[li++] = r;
      else tw[ri++] = r;
    }
    memcpy(nrw + li, tw, (size_t)ri * 4);
    (void)nl;
    const int mc = mono ? mono[best_feat] : 0;
    double llo, lhi, rlo, rhi;
    mono_child_bounds(mc, jb.lo, jb.hi, best_mid, 0, llo, lhi);
    mono_child_bounds(mc, jb.lo, jb.hi, best_mid, 1, rlo, rhi);
    nlo.resize(base + 2); nhi.resize(base + 2);
    nlo[base] = llo; nhi[base] = lhi; nlo[base + 1] = rlo; nhi[base + 1] = rhi;
    if (mae) {
      nabs.resize(base + 2);
      nabs[base] = mae_node(jb.start, li, lv);
      nabs[base + 1] = mae_node(jb.start + li, jb.count - li, rv);
    }
    const double* lvv = out.vals.data() + (size_t)base * D.VC;
    const double* rvv = lvv + D.VC;
    // push right first so the left subtree is processed first (depth-first, left-major)
    if (visit(jb.count - li, jb.depth + 1, rvv, node_imp(base + 1, rvv)))
      stack.push_back({base + 1, jb.start + li, jb.count - li, jb.depth + 1, child_key(jb.key, 1), rlo, rhi});
    if (visit(li, jb.depth + 1, lvv, node_imp(base, lvv)))
      stack.push_back({base, jb.start, li, jb.depth + 1, child_key(jb.key, 0), llo, lhi});
  }
  if (mono)   // clip every node's value to its bounds (sklearn clip_node_value)
    for (size_t i = 0; i < out.nodes.size(); ++i) mono_clip(out.vals.data() + i * D.VC, D.is_reg, nlo[i], nhi[i]);
}

}  // namespace dml

using namespace dml;

extern "C" {

int dml_cpu_sizeof_treespec() { return (int)sizeof(TreeSpec); }

void* dml_cpu_forest_build_mono(const uint8_t* Xb, int64_t ld, int64_t n, int64_t d, const int32_t* ycls,
                                const float* yreg, int64_t n_classes, int64_t is_reg, const uint8_t* roles,
                                const TreeSpec* specs, int64_t T, int64_t ystride, const double* cw,
                                const int8_t* mono, int64_t e1, int64_t e2) {
  Data D;
  // regression: every (target, row) quantised once (forest_common.h fixed point)
  std::vector<int64_t> yq, y2q;
  D.rq = reg_scale((int)e1, (int)e2);
  D.yq = D.y2q = nullptr;
  if (is_reg) {
    int64_t targets = 1;
    if (ystride > 0)
      for (int64_t t = 0; t < T; ++t) targets = std::max<int64_t>(targets, (int64_t)specs[t].target + 1);
    const int64_t len = ystride > 0 ? (targets - 1) * ystride + n : n;
    yq.resize(len); y2q.resize(len);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < len; ++i) reg_quantize(yreg[i], D.rq, yq[i], y2q[i]);
    D.yq = yq.data(); D.y2q = y2q.data();
  }
  D.mono = mono;
  D.ystride = ystride;
  D.cw = cw;
  D.Xb = Xb; D.ld = ld; D.n = (int)n; D.d = (int)d; D.is_reg = (int)is_reg;
  D.C = is_reg ? 1 : (int)n_classes;
  D.CH = is_reg ? 4 : (int)n_classes + 1;
  D.VC = is_reg ? 3 : (int)n_classes;
  D.ycls = ycls; D.yreg = yreg; D.roles = roles;
  CpuForest* F = new CpuForest();
  F->T = (int)T;
  F->VC = D.VC;
  F->trees.resize(T);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t t = 0; t < T; ++t) build_tree(D, specs[t], t, F->trees[t]);
  return F;
}

void* dml_cpu_forest_build(const uint8_t* Xb, int64_t ld, int64_t n, int64_t d, const int32_t* ycls,
                           const float* yreg, int64_t n_classes, int64_t is_reg, const uint8_t* roles,
                           const TreeSpec* specs, int64_t T, int64_t ystride, const double* cw) {
  int e1 = 0, e2 = 0;
  if (is_reg) {   // exponents from the data (entry point of the host self-test)
    int64_t targets = 1;
    if (ystride > 0)
      for (int64_t t = 0; t < T; ++t) targets = std::max<int64_t>(targets, (int64_t)specs[t].target + 1);
    std::vector<int64_t> cnt((size_t)targets * kExpBins, 0);
    for (int64_t t = 0; t < targets; ++t)
      for (int64_t i = 0; i < n; ++i) {
        const float y = yreg[(ystride > 0 ? t * ystride : 0) + i];
        int k = 0;
        if (y != 0.0f) frexp((double)y, &k);
        cnt[(size_t)t * kExpBins + (y != 0.0f ? k + kExpOff : 0)]++;
      }
    reg_exponents_counts(cnt.data(), targets, e1, e2);
  }
  return dml_cpu_forest_build_mono(Xb, ld, n, d, ycls, yreg, n_classes, is_reg, roles, specs, T, ystride, cw,
                                   nullptr, e1, e2);
}

void dml_reg_exponents(const int64_t* cnt, int64_t targets, int32_t* out) {
  int e1, e2;
  reg_exponents_counts(cnt, targets, e1, e2);
  out[0] = e1; out[1] = e2;
}

int64_t dml_cpu_forest_num_nodes(void* h) {
  CpuForest* F = (CpuForest*)h;
  int64_t s = 0;
  for (auto& t : F->trees) s += (int64_t)t.nodes.size();
  return s;
}

// export into the GPU pool layout: root of tree t at index t, then each tree's
// non-root nodes contiguously (children pairs stay adjacent).
void dml_cpu_forest_export(void* h, NodeRec* nodes, double* vals) {
  CpuForest* F = (CpuForest*)h;
  int64_t next = F->T;
  for (int t = 0; t < F->T; ++t) {
    const CpuTree& tr = F->trees[t];
    const int64_t base = next;
    auto gidx = [&](int64_t local) { return local == 0 ? (int64_t)t : base + local - 1; };
    for (size_t i = 0; i < tr.nodes.size(); ++i) {
      NodeRec r = tr.nodes[i];
      if (r.left >= 0) r.left = (int32_t)gidx(r.left);
      const int64_t g = gidx((int64_t)i);
      nodes[g] = r;
      memcpy(vals + g * F->VC, tr.vals.data() + i * F->VC, sizeof(double) * F->VC);
    }
    next += (int64_t)tr.nodes.size() - 1;
  }
}

// leaf[t * n + row] for trees t0 .. t0+T-1 (roots at node t) over all n rows
void dml_cpu_forest_apply(const uint8_t* Xb, int64_t ld, int64_t n, const NodeRec* nodes, int32_t t0, int32_t T,
                          int32_t* leaf) {
#pragma omp parallel for collapse(2) schedule(static)
  for (int32_t t = 0; t < T; ++t)
    for (int64_t r = 0; r < n; ++r) {
      const uint8_t* xr = Xb + r * ld;
      int node = t0 + t;
      NodeRec nr = nodes[node];
      while (nr.split >= 0) {
        node = nr.left + (xr[nr.split >> 8] > (nr.split & 255) ? 1 : 0);
        nr = nodes[node];
      }
      leaf[(int64_t)t * n + r] = node;
    }
}

// max_leaf_nodes: best-first top of each limited tree (forest_common.h, the routine the
// HIP kernel k_prune_best_first runs); limit[t] <= 0 leaves tree t alone
void dml_cpu_forest_prune(NodeRec* nodes, const double* vals, int64_t VC, int32_t C, int32_t is_reg,
                          const TreeSpec* specs, const int32_t* limit, int32_t T, int32_t* leaves) {
  std::vector<FrontierEnt> heap;
  for (int32_t t = 0; t < T; ++t) {
    if (limit[t] <= 0) {
      if (leaves) leaves[t] = -1;
      continue;
    }
    heap.resize((size_t)limit[t]);
    const int n = best_first_prune(nodes, vals, VC, C, is_reg != 0, specs[t].criterion, t, limit[t], heap.data());
    if (leaves) leaves[t] = n;
  }
}

// sklearn midpoint thresholds for exactly-binned features (same two passes as predict.hip)
void dml_cpu_forest_refine(const uint8_t* Xb, int64_t ld, int64_t n, NodeRec* nodes, int64_t P, const TreeSpec* specs,
                           int32_t T, const uint8_t* roles, const float* vals, const uint8_t* exact) {
  std::vector<uint32_t> hi((size_t)P, 0xFFFFFFFFu);
  for (int32_t t = 0; t < T; ++t) {
    const TreeSpec& s = specs[t];
    for (int64_t r = 0; r < n; ++r) {
      if (roles[(int64_t)s.split * n + r] != 1 || boot_weight(s, (uint32_t)r) == 0) continue;
      const uint8_t* xr = Xb + r * ld;
      int node = t;
      NodeRec nr = nodes[node];
      while (nr.split >= 0) {
        const uint32_t b = xr[nr.split >> 8];
        if (b > (uint32_t)(nr.split & 255)) {
          if (b < hi[node]) hi[node] = b;
          node = nr.left + 1;
        } else {
          node = nr.left;
        }
        nr = nodes[node];
      }
    }
  }
  for (int64_t i = 0; i < P; ++i) {
    const NodeRec nr = nodes[i];
    if (nr.split < 0) continue;
    const int f = nr.split >> 8, blo = nr.split & 255;
    const uint32_t bhi = hi[i];
    if (!exact[f] || bhi > 255u || (int)bhi <= blo) continue;
    const float* v = vals + (int64_t)f * 256;
    double m = (double)v[blo] / 2.0 + (double)v[bhi] / 2.0;
    if (m == (double)v[bhi] || !(m == m)) m = (double)v[blo];
    int b = blo;
    while (b + 1 < (int)bhi && (double)v[b + 1] <= m) ++b;
    nodes[i].split = f * 256 + b;
  }
}

void dml_cpu_forest_free(void* h) { delete (CpuForest*)h; }

// predict rows (same accumulation order as predict.hip)
void dml_cpu_forest_predict(const uint8_t* Xb, int64_t ld, const NodeRec* nodes, const double* val, int64_t VC,
                            int64_t is_reg, int64_t C, const int32_t* fit_tree_off, const int64_t* fit_row_off,
                            const int32_t* rows, int64_t F, int32_t* out_cls, float* out_reg, float* out_proba) {
  for (int64_t f = 0; f < F; ++f) {
    const int64_t r0 = fit_row_off[f], r1 = fit_row_off[f + 1];
#pragma omp parallel for schedule(static)
    for (int64_t i = r0; i < r1; ++i) {
      const uint8_t* xr = Xb + (int64_t)rows[i] * ld;
      std::vector<float> p(is_reg ? 1 : C, 0.f);
      double acc = 0.0;
      int nt = 0;
      for (int t = fit_tree_off[f]; t < fit_tree_off[f + 1]; ++t) {
        int node = t;
        NodeRec nr = nodes[node];
        while (nr.split >= 0) {
          const int b = xr[nr.split >> 8];
          node = nr.left + (b > (nr.split & 255) ? 1 : 0);
          nr = nodes[node];
        }
        const double* v = val + (int64_t)node * VC;
        if (is_reg) {
          if (v[0] > 0.0) { acc += v[1] / v[0]; ++nt; }
        } else {
          double W = 0.0;
          for (int k = 0; k < C; ++k) W += v[k];
          if (W > 0.0) {
            const double inv = 1.0 / W;
            for (int k = 0; k < C; ++k) p[k] += (float)(v[k] * inv);
          }
        }
      }
      if (is_reg) {
        out_reg[i] = nt ? (float)(acc / nt) : 0.f;
      } else {
        int best = 0;
        float bv = p[0];
        for (int k = 1; k < C; ++k)
          if (p[k] > bv) { bv = p[k]; best = k; }
        out_cls[i] = best;
        if (out_proba) {
          const float ntf = (float)(fit_tree_off[f + 1] - fit_tree_off[f]);
          for (int k = 0; k < C; ++k) out_proba[i * C + k] = p[k] / ntf;
        }
      }
    }
  }
}

// bin X (row-major float32 [n,d]) with per-feature sorted edges [d][255] (+inf padded)
void dml_cpu_bin(const float* X, int64_t n, int64_t d, const float* edges, uint8_t* out, int64_t ld) {
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n; ++r) {
    for (int64_t f = 0; f < d; ++f) {
      const float x = X[r * d + f];
      const float* e = edges + f * 255;
      int lo = 0, hi = 255;
      while (lo < hi) {  // count of edges < x
        const int mid = (lo + hi) >> 1;
        if (e[mid] < x) lo = mid + 1; else hi = mid;
      }
      out[r * ld + f] = (uint8_t)lo;
    }
  }
}

}  // extern "C"
