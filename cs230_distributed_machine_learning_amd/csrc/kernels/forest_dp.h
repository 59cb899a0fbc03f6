// forest_dp.h — row-sharded (data-parallel) forest builder: the per-node decisions
// shared by the HIP kernels (forest_dp.hip) and the C++ twin (../runtime/forest_dp_cpu.cpp).
//
// SURVEY §2.7 / §5.8 "DP mode": every rank holds a contiguous row block of the table; the
// forest grows LEVEL-SYNCHRONOUSLY.  Each rank builds the histograms of every open node
// over its own rows, ONE all-reduce per level-round sums them over ranks (RCCL over
// xGMI), and every rank then takes the identical split decisions from the identical
// global histograms -- so every rank holds the same node pool and partitions only its
// own rows.  Nothing but histograms crosses the links; no rank ever sees another rank's
// rows.  The reference has no counterpart (its workers each re-read the whole CSV and
// fit one candidate alone, aws-prod/worker/worker.py:406-425, :315).
//
// Every decision is the one forest_cpu.cpp / forest.hip take (forest_common.h): the
// bootstrap weight of GLOBAL row r0 + r, the keyed per-node feature order (feature_at),
// the "stop after max_features non-constant features" search, first-strictly-better
// ties, the min_impurity_decrease test and the leaf rules.  Classification histograms
// are exact integers, so a row-sharded forest is the SAME forest the one-GPU builder
// grows (tests/test_forest_dp.py checks node-for-node equality of the predictions).
//
// A node's search may need several rounds: a round evaluates KR visiting positions of
// every still-searching node; a node whose KR positions held too many constant features
// continues in the next round from where it stopped.
#pragma once
#include "forest_common.h"

#if defined(__HIPCC__)
#pragma clang fp contract(off)
#endif

namespace dml {

// One open node of the current level (identical on every rank).  64 bytes.
struct DpSlot {
  uint64_t key;       // feature-order key (root_key / child_key chain)
  double best_gain;   // best proxy so far (-inf before the first candidate)
  double count;       // GLOBAL rows in the node (bagged rows, unweighted)
  int32_t node;       // pool index
  int32_t tree;       // batch tree index
  int32_t depth;
  int32_t pos;        // next visiting position
  int32_t nonconst;   // non-constant features visited so far
  int32_t best_feat;  // -1: none yet
  int32_t best_bin;
  int32_t done;       // 1: search finished
  int32_t split;      // accept(): 1 = the node splits
  int32_t child;      // children(): pool index of the left child
};

// Argument block of every DP entry point (pointers as int64, same layout in ctypes).
struct DpArgs {
  int64_t Xb, ld, n, d, r0;          // local bins [n][ld]; r0 = global id of local row 0
  int64_t ycls, yreg;                // int32 [n] | float [n] (local rows)
  int64_t C, CH, VC, is_reg;
  int64_t roles;                     // uint8 [n_splits][n] (local rows)
  int64_t specs, T;                  // TreeSpec [T]
  int64_t cw;                        // double [T][C] class weights (cls) or 0
  int64_t tree_W;                    // double [T]
  int64_t root;                      // [T][CH] root statistics (all-reduced): double (cls) |
                                     // int64 {sum w, sum w yq, sum w y2q, rows} (reg)
  int64_t wts;                       // uint8 [T][n] bootstrap weight of (tree, local row) (init only)
  // (tree, row) pairs of every open node, sorted by node
  int64_t act_row, act_tree, act_node, A;
  int64_t new_node;                  // int32 [A] partition output (-1: the pair leaves)
  // the level's open nodes
  int64_t slots, best_left, S_open;  // DpSlot [S_open]; double [S_open][CH]
  int64_t seg_start, seg_cnt;        // int64 [S_open]: the slot's pairs in act_*
  // one search round
  int64_t srch, S, KR;               // int32 [S] slot ids being searched; KR positions each
  int64_t feats;                     // int32 [S][KR] feature of each position (-1 past d)
  int64_t hist;                      // [S][KR][CH][256] uint32 (cls) | [S][KR][3][256] uint64 (reg:
                                     // w | rows << 32, sum w yq, sum w y2q -- exact, see forest_common.h)
  int64_t tile_s, tile_off, n_tiles, tile_rows;  // LDS tiles: search index, pair offset in the segment
  int64_t small_s, n_small;          // search indices of small segments (global atomics)
  int64_t lds_feats;                 // positions per LDS pass (hist tiles)
  // node pool
  int64_t nodes, vals, P;            // int32 [cap][2], double [cap][VC]; P = first free index
  int64_t child_base;                // int32 [S_open]: 2 * (#splitting slots before this one)
  int64_t next, next_open;           // DpSlot [2 * n_split], int32 [2 * n_split]
  int64_t slot_of, lvl_lo, lvl_n;    // int32 [lvl_n]: slot of node lvl_lo + i (-1 none)
  // threshold refinement
  int64_t hi, binvals, exact, P_total;
  int64_t ystride;                   // > 0: yreg is [targets][ystride], tree t regresses on row specs[t].target
  int64_t yq_e1, yq_e2;              // regression fixed point (forest_common.h), global over the ranks
};

template <typename T>
DML_HD T* dp_ptr(int64_t v) { return (T*)(uintptr_t)v; }

// 32-bit words of one searching slot's histogram block
DML_HD int64_t dp_hist_words(const DpArgs& a) { return a.is_reg ? a.KR * 3 * 256 * 2 : a.KR * a.CH * 256; }

// regression target of (tree, local row): gradient boosting gives every tree its own row
DML_HD float dp_target(const DpArgs& a, int tree, int64_t r) {
  const float* y = dp_ptr<const float>(a.yreg);
  return a.ystride ? y[(int64_t)dp_ptr<const TreeSpec>(a.specs)[tree].target * a.ystride + r] : y[r];
}

// impurity of a node's value vector
DML_HD double dp_impurity(const double* v, int C, int is_reg, int crit) {
  if (is_reg) return mse_impurity(v[0], v[1], v[2]);
  ClsAcc a;
  a.init(crit);
  for (int k = 0; k < C; ++k) a.add(v[k]);
  return cls_impurity(a, crit);
}

// the builders' "grow this node?" rule (forest_cpu.cpp visit())
DML_HD bool dp_visit(const TreeSpec& t, double count, int depth, const double* v, int C, int is_reg,
                     const RegScale& q) {
  return !(leaf_by_counts(t, (int)count, depth) || leaf_by_weight(t, vals_weight(v, C, is_reg)) ||
           (is_reg ? reg_pure(v, q) : dp_impurity(v, C, is_reg, t.criterion) <= kEps));
}

// Root of tree ``t`` from its all-reduced statistics: class weights (balanced_subsample
// from the bootstrap counts), node value, tree weight, and the first slot.
// Returns 1 when the root is an open node.
DML_HD int dp_root_one(const DpArgs& a, int t, DpSlot* slot) {
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[t];
  const int C = (int)a.C, CH = (int)a.CH, VC = (int)a.VC;
  const double* st = dp_ptr<const double>(a.root) + (int64_t)t * CH;
  double* v = dp_ptr<double>(a.vals) + (int64_t)t * VC;
  double count;
  int32_t* nd = dp_ptr<int32_t>(a.nodes) + 2 * (int64_t)t;
  nd[0] = -1;
  nd[1] = -1;
  double W = 0.0;
  if (a.is_reg) {   // exact integer sums over every rank's rows
    const RegScale q = reg_scale((int)a.yq_e1, (int)a.yq_e2);
    const uint64_t* si = dp_ptr<const uint64_t>(a.root) + (int64_t)t * CH;
    v[0] = (double)si[0]; v[1] = reg_s1(si[1], q); v[2] = reg_s2(si[2], q);
    W = v[0];
    count = (double)si[3];
  } else {
    double* cwv = a.cw ? dp_ptr<double>(a.cw) + (int64_t)t * C : nullptr;
    if (cwv && s.cw_mode == 2) balanced_weights(st, C, cwv);
    for (int k = 0; k < C; ++k) {
      v[k] = (cwv && s.cw_mode != 0) ? st[k] * cwv[k] : st[k];
      W += v[k];
    }
    count = st[CH - 1];
  }
  dp_ptr<double>(a.tree_W)[t] = W;
  dp_ptr<TreeSpec>(a.specs)[t].min_weight_leaf = s.min_weight_frac * W;   // read by every later step
  slot->key = root_key(s.seed);
  slot->best_gain = -INFINITY;
  slot->count = count;
  slot->node = t;
  slot->tree = t;
  slot->depth = 0;
  slot->pos = slot->nonconst = 0;
  slot->best_feat = slot->best_bin = -1;
  slot->done = slot->split = 0;
  slot->child = -1;
  return (count > 0.0 && dp_visit(s, count, 0, v, C, (int)a.is_reg, reg_scale((int)a.yq_e1, (int)a.yq_e2))) ? 1 : 0;
}

// class weight vector of a tree (null = all ones)
DML_HD const double* dp_cwv(const DpArgs& a, int t) {
  if (a.is_reg || !a.cw) return nullptr;
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[t];
  return s.cw_mode != 0 ? dp_ptr<const double>(a.cw) + (int64_t)t * a.C : nullptr;
}

// Evaluate the KR positions of one searching slot from its global histograms,
// continuing the feature search exactly where forest_cpu.cpp's loop would be.
// ``h``: this slot's [KR][CH][256] block; ``f``: its [KR] features.
DML_HDM void dp_eval_slot(const DpArgs& a, DpSlot& sl, double* best_left, const void* h, const int32_t* f) {
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[sl.tree];
  const int C = (int)a.C, CH = (int)a.CH, KR = (int)a.KR, d = (int)a.d;
  const double* cwv = dp_cwv(a, sl.tree);
  for (int k = 0; k < KR && !sl.done; ++k) {
    const int feat = f[k];
    if (feat < 0) {
      sl.done = 1;
      break;
    }
    sl.pos += 1;
    double g_best = -INFINITY;
    int b_best = -1;
    bool nc = false;
    if (!a.is_reg) {
      const uint32_t* hu = (const uint32_t*)h + (int64_t)k * CH * 256;
      uint32_t tot[kMaxClasses + 1], pre[kMaxClasses + 1];
      for (int ch = 0; ch < CH; ++ch) {
        uint32_t acc = 0;
        for (int b = 0; b < 256; ++b) acc += hu[ch * 256 + b];
        tot[ch] = acc;
        pre[ch] = 0;
      }
      for (int b = 0; b < 255; ++b) {
        for (int ch = 0; ch < CH; ++ch) pre[ch] += hu[ch * 256 + b];
        const uint32_t rl = pre[C], rr = tot[C] - rl;
        nc |= (rl > 0 && rr > 0);
        if (rl < (uint32_t)s.min_samples_leaf || rr < (uint32_t)s.min_samples_leaf) continue;
        ClsAcc L, R;
        L.init(s.criterion);
        R.init(s.criterion);
        for (int c = 0; c < C; ++c) {
          const double cw = cwv ? cwv[c] : 1.0;
          const double lc = (double)pre[c] * cw, tc = (double)tot[c] * cw;
          L.add(lc);
          R.add(tc - lc);
        }
        if (side_too_light(s, L.w, R.w)) continue;
        const double g = cls_proxy(L, R, s.criterion);
        if (g > g_best) {
          g_best = g;
          b_best = b;
        }
      }
      if (nc) {
        sl.nonconst += 1;
        if (b_best >= 0 && g_best > sl.best_gain) {
          sl.best_gain = g_best;
          sl.best_feat = feat;
          sl.best_bin = b_best;
          for (int ch = 0; ch < CH; ++ch) {
            uint32_t acc = 0;
            for (int b = 0; b <= b_best; ++b) acc += hu[ch * 256 + b];
            best_left[ch] = (double)acc * ((ch < C && cwv) ? cwv[ch] : 1.0);
          }
        }
      }
    } else {
      // integer prefix sums in bin order: forest_cpu.cpp's regression histogram scan
      const RegScale q = reg_scale((int)a.yq_e1, (int)a.yq_e2);
      const uint64_t* hr = (const uint64_t*)h + (int64_t)k * 3 * 256;
      uint64_t tot[3] = {0ull, 0ull, 0ull}, pre[3] = {0ull, 0ull, 0ull};
      for (int ch = 0; ch < 3; ++ch)
        for (int b = 0; b < 256; ++b) tot[ch] += hr[ch * 256 + b];
      for (int b = 0; b < 255; ++b) {
        for (int ch = 0; ch < 3; ++ch) pre[ch] += hr[ch * 256 + b];
        const uint32_t rl = (uint32_t)(pre[0] >> 32), rr = (uint32_t)(tot[0] >> 32) - rl;
        nc |= (rl > 0 && rr > 0);
        if (rl < (uint32_t)s.min_samples_leaf || rr < (uint32_t)s.min_samples_leaf) continue;
        const double l0 = reg_w(pre[0]), t0 = reg_w(tot[0]), l1 = reg_s1(pre[1], q), t1 = reg_s1(tot[1], q);
        if (side_too_light(s, l0, t0 - l0)) continue;
        const double g = reg_proxy(s.criterion, l0, l1, t0 - l0, t1 - l1);
        if (g > g_best) {
          g_best = g;
          b_best = b;
        }
      }
      if (nc) {
        sl.nonconst += 1;
        if (b_best >= 0 && g_best > sl.best_gain) {
          sl.best_gain = g_best;
          sl.best_feat = feat;
          sl.best_bin = b_best;
          uint64_t acc[3] = {0ull, 0ull, 0ull};
          for (int ch = 0; ch < 3; ++ch)
            for (int b = 0; b <= b_best; ++b) acc[ch] += hr[ch * 256 + b];
          best_left[0] = reg_w(acc[0]); best_left[1] = reg_s1(acc[1], q); best_left[2] = reg_s2(acc[2], q);
          best_left[3] = reg_rows(acc[0]);
        }
      }
    }
    if (sl.nonconst >= s.max_features || sl.pos >= d) sl.done = 1;
  }
}

// Accept or reject the slot's best split (forest_cpu.cpp "accept?").
DML_HD int dp_accept_one(const DpArgs& a, const DpSlot& sl, const double* best_left) {
  if (sl.best_feat < 0) return 0;
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[sl.tree];
  const int C = (int)a.C;
  const double* pv = dp_ptr<const double>(a.vals) + (int64_t)sl.node * a.VC;
  double impN, impL, impR, wN, wL, wR;
  if (a.is_reg) {
    wN = pv[0]; wL = best_left[0]; wR = pv[0] - best_left[0];
    impN = mse_impurity(pv[0], pv[1], pv[2]);
    impL = mse_impurity(best_left[0], best_left[1], best_left[2]);
    impR = mse_impurity(pv[0] - best_left[0], pv[1] - best_left[1], pv[2] - best_left[2]);
  } else {
    ClsAcc N, L, R;
    N.init(s.criterion); L.init(s.criterion); R.init(s.criterion);
    for (int k = 0; k < C; ++k) { N.add(pv[k]); L.add(best_left[k]); R.add(pv[k] - best_left[k]); }
    wN = N.w; wL = L.w; wR = R.w;
    impN = cls_impurity(N, s.criterion); impL = cls_impurity(L, s.criterion); impR = cls_impurity(R, s.criterion);
  }
  const double Wt = dp_ptr<const double>(a.tree_W)[sl.tree];
  const double imp = accept_improvement(s, a.is_reg != 0, pv, best_left, Wt, wN, impN, wL, impL, wR, impR);
  return (imp + kEps < (double)s.min_impurity_decrease) ? 0 : 1;
}

// Write a splitting slot's children (pool indices P + child_base[i], +1) and their
// candidate slots for the next level.
DML_HDM void dp_children_one(const DpArgs& a, int i) {
  DpSlot& sl = dp_ptr<DpSlot>(a.slots)[i];
  if (!sl.split) return;
  const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[sl.tree];
  const int C = (int)a.C, CH = (int)a.CH, VC = (int)a.VC;
  const int cb = dp_ptr<const int32_t>(a.child_base)[i];
  const int left = (int)a.P + cb;
  sl.child = left;
  int32_t* nd = dp_ptr<int32_t>(a.nodes);
  double* vals = dp_ptr<double>(a.vals);
  const double* bl = dp_ptr<const double>(a.best_left) + (int64_t)i * CH;
  nd[2 * (int64_t)sl.node] = pack_split(sl.best_feat, sl.best_bin);
  nd[2 * (int64_t)sl.node + 1] = left;
  const double* pv = vals + (int64_t)sl.node * VC;
  double* lv = vals + (int64_t)left * VC;
  double* rv = lv + VC;
  for (int k = 0; k < VC; ++k) { lv[k] = bl[k]; rv[k] = pv[k] - bl[k]; }
  const double nl = bl[CH - 1];
  DpSlot* nx = dp_ptr<DpSlot>(a.next) + cb;
  int32_t* op = dp_ptr<int32_t>(a.next_open) + cb;
  for (int side = 0; side < 2; ++side) {
    nd[2 * (int64_t)(left + side)] = -1;
    nd[2 * (int64_t)(left + side) + 1] = -1;
    DpSlot c;
    c.key = child_key(sl.key, side);
    c.best_gain = -INFINITY;
    c.count = side == 0 ? nl : sl.count - nl;
    c.node = left + side;
    c.tree = sl.tree;
    c.depth = sl.depth + 1;
    c.pos = c.nonconst = 0;
    c.best_feat = c.best_bin = -1;
    c.done = c.split = 0;
    c.child = -1;
    nx[side] = c;
    op[side] = dp_visit(s, c.count, c.depth, side == 0 ? lv : rv, C, (int)a.is_reg,
                          reg_scale((int)a.yq_e1, (int)a.yq_e2)) ? 1 : 0;
  }
}

// New node of pair ``i`` after the level's splits (-1: its node became or stayed a leaf,
// or its child is not grown further).
DML_HD int32_t dp_partition_one(const DpArgs& a, int64_t i) {
  const int32_t node = dp_ptr<const int32_t>(a.act_node)[i];
  const int64_t rel = (int64_t)node - a.lvl_lo;
  if (rel < 0 || rel >= a.lvl_n) return -1;
  const int32_t s = dp_ptr<const int32_t>(a.slot_of)[rel];
  if (s < 0) return -1;
  const DpSlot& sl = dp_ptr<const DpSlot>(a.slots)[s];
  if (!sl.split) return -1;
  const int32_t r = dp_ptr<const int32_t>(a.act_row)[i];
  const uint32_t b = dp_ptr<const uint8_t>(a.Xb)[(int64_t)r * a.ld + sl.best_feat];
  const int32_t child = sl.child + (b > (uint32_t)sl.best_bin ? 1 : 0);
  return dp_ptr<const int32_t>(a.next_open)[child - a.P] ? child : -1;
}

// Midpoint threshold of node ``i`` once the global ``hi`` (smallest bin that went right
// among the node's training rows, all-reduced MIN over ranks) is known -- the second
// pass of forest_cpu.cpp's dml_cpu_forest_refine.
DML_HD void dp_refine_one(const DpArgs& a, int64_t i) {
  int32_t* nd = dp_ptr<int32_t>(a.nodes) + 2 * i;
  if (nd[0] < 0) return;
  const int f = nd[0] >> 8, blo = nd[0] & 255;
  const uint32_t bhi = dp_ptr<const uint32_t>(a.hi)[i];
  if (!dp_ptr<const uint8_t>(a.exact)[f] || bhi > 255u || (int)bhi <= blo) return;
  const float* v = dp_ptr<const float>(a.binvals) + (int64_t)f * 256;
  double m = (double)v[blo] / 2.0 + (double)v[bhi] / 2.0;
  if (m == (double)v[bhi] || !(m == m)) m = (double)v[blo];
  int b = blo;
  while (b + 1 < (int)bhi && (double)v[b + 1] <= m) ++b;
  nd[0] = f * 256 + b;
}

}  // namespace dml
