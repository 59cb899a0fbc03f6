// forest_common.h — definitions shared by the HIP forest builder (forest.hip) and the
// C++ CPU builder (../runtime/forest_cpu.cpp).  Everything that decides the SHAPE of a
// tree lives here (RNG streams, bootstrap weights, per-node feature order, split
// scoring, leaf rules), so the two builders grow identical trees and the GPU path can
// be checked exactly against the CPU path.
//
// Semantics follow scikit-learn's BestSplitter/DepthFirstTreeBuilder as used by
// RandomForest{Classifier,Regressor} (the reference's compute delegate, called at
// aws-prod/worker/worker.py:315,326,341), re-expressed on 256-bin quantised features:
//   * leaf if depth>=max_depth, n<min_samples_split, n<2*min_samples_leaf, or pure;
//   * features are visited in a per-node random order and the search stops after
//     max_features NON-constant features (constant ones do not count);
//   * best split = max proxy improvement, first strictly-better wins (ties go to the
//     earliest visited feature, then the lowest bin);
//   * split rejected if improvement + eps < min_impurity_decrease.
// Bootstrap uses Poisson(lambda) per-row weights (lambda = max_samples fraction,
// 1.0 by default) instead of an exact multinomial draw: same expectation and
// asymptotic distribution, no per-tree index array, recomputable anywhere.
//
// Scores are computed from per-channel sums in a FIXED order with fp-contraction off
// so both builders evaluate bit-identical doubles.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DML_HD __host__ __device__ __forceinline__
#define DML_HDM __host__ __device__ __forceinline__
#else
#include <math.h>
#define DML_HD static inline
#define DML_HDM inline
#endif

namespace dml {

constexpr int kBins = 256;        // uint8 bins
constexpr int kPoisTable = 12;    // Poisson CDF thresholds kept per tree
constexpr int kMaxClasses = 64;   // classification channels supported by the builders

// kMAE (sklearn "absolute_error") is grown by the host builder only (forest_cpu.cpp):
// its split search needs per-node weighted medians, not histogram sums
// kFriedman (sklearn "friedman_mse") grows exactly like kMSE (its split proxy ranks
// candidates the same way); only the min_impurity_decrease test differs (accept_improvement)
enum Criterion : int32_t { kGini = 0, kEntropy = 1, kMSE = 2, kPoisson = 3, kMAE = 4, kFriedman = 5 };

// Per-tree build specification (POD, identical layout on host, device and ctypes).
struct TreeSpec {
  uint64_t seed;            // tree seed: bootstrap stream and root node key
  int32_t split;            // which role vector (split) the tree trains on
  int32_t fit;              // owning fit index
  int32_t max_depth;        // INT32_MAX for None
  int32_t min_samples_split;
  int32_t min_samples_leaf;
  int32_t max_features;     // k (>=1, <= n_features)
  int32_t bootstrap;        // 0 all rows, 1 Poisson(lambda) bootstrap, 2 Bernoulli subsample (p = pois_cdf[0] / 2^32)
  int32_t criterion;        // Criterion
  float min_impurity_decrease;
  int32_t target;           // row of the per-tree target matrix (ForestArgs.ystride > 0: boosting)
  uint32_t pois_cdf[kPoisTable];  // P(K<=j) * 2^32 (saturated), j = 0..11
  int32_t cw_mode;          // class weights: 0 none, 1 fixed row of the cw table (dict / "balanced"),
                            // 2 "balanced_subsample" (row computed from this tree's bootstrap counts)
  int32_t reserved;
  double min_weight_frac;   // sklearn min_weight_fraction_leaf
  double min_weight_leaf;   // = min_weight_frac x the tree's total weight; set by each builder at the root
};

// sklearn class_weight="balanced_subsample" for one tree from its root class counts
// (bootstrap-weighted): n_samples / (n_present_classes * count_k); absent classes get 1.
DML_HD void balanced_weights(const double* counts, int C, double* out) {
  double total = 0.0;
  int present = 0;
  for (int k = 0; k < C; ++k) {
    total += counts[k];
    present += counts[k] > 0.0 ? 1 : 0;
  }
  for (int k = 0; k < C; ++k) out[k] = counts[k] > 0.0 ? total / ((double)present * counts[k]) : 1.0;
}

// node record written by both builders
struct NodeRec {
  int32_t split;  // feature*256 + bin, or -1 for a leaf
  int32_t left;   // index of left child (right = left + 1), -1 for a leaf
};

DML_HD int32_t pack_split(int feat, int bin) { return feat * kBins + bin; }

// ---- RNG ------------------------------------------------------------------------
DML_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

DML_HD uint32_t hash_u32(uint64_t key, uint64_t ctr) {
  return (uint32_t)(splitmix64(key ^ splitmix64(ctr + 0x632BE59BD9B4E019ull)) >> 32);
}

// bootstrap weight of `row` for the tree (TS: TreeSpec, or any view with its fields --
// the HIP node kernels pass a register-resident NodeSpec)
// the row half of boot_weight's hash (hash_u32's inner splitmix64): the same for every
// tree, so k_count_active computes it once per row for a group of trees
DML_HD uint64_t boot_row_key(uint32_t row) {
  return splitmix64(0xB0075ull * 0x100000000ull + row + 0x632BE59BD9B4E019ull);
}

template <class TS>
DML_HD uint32_t boot_weight(const TS& t, uint32_t row) {
  if (!t.bootstrap) return 1u;
  const uint32_t u = hash_u32(t.seed, 0xB0075ull * 0x100000000ull + row);
  if (t.bootstrap == 2) return u < t.pois_cdf[0] ? 1u : 0u;
  // inverse CDF: the table is non-decreasing, so "first j with u < T[j]" = #{j : u >= T[j]}
  // (branch-free: 12 compares against wave-uniform table entries, no per-lane loop)
  uint32_t k = 0;
#pragma unroll
  for (int j = 0; j < kPoisTable; ++j) k += u >= t.pois_cdf[j] ? 1u : 0u;
  return k;
}

DML_HD uint64_t root_key(uint64_t seed) { return splitmix64(seed ^ 0x7EE5EEDull); }

DML_HD uint64_t child_key(uint64_t parent, int side) {
  return splitmix64(parent * 0x9E3779B97F4A7C15ull + 0x51ED27ull + (uint64_t)side);
}

// Per-node feature visiting order: a keyed pseudo-random permutation of [0, d) that is
// evaluated POSITION BY POSITION -- feature_at(key, k, d) is the k-th feature visited --
// so a GPU lane can compute its own position's feature with no wave-wide min-search
// (each lane of a wave takes one position; sklearn draws a random order too).  The
// permutation is a 3-round keyed bijection on [0, 2^b) (odd multiply + add, xor-shift:
// each step is invertible mod 2^b) restricted to [0, d) by cycle walking.
struct FeatPerm {
  uint32_t m1, a1, m2, a2, m3, a3, mask, sh;
};

DML_HD FeatPerm feat_perm(uint64_t node_key, int d) {
  FeatPerm p;
  int b = 1;
  while ((1 << b) < d) ++b;
  p.mask = (1u << b) - 1u;
  p.sh = (uint32_t)((b + 1) >> 1);
  const uint64_t h1 = splitmix64(node_key ^ 0xFEA7FEA7ull), h2 = splitmix64(h1);
  const uint64_t h3 = splitmix64(h2);
  p.m1 = ((uint32_t)h1 | 1u) & p.mask; p.a1 = (uint32_t)(h1 >> 32) & p.mask;
  p.m2 = ((uint32_t)h2 | 1u) & p.mask; p.a2 = (uint32_t)(h2 >> 32) & p.mask;
  p.m3 = ((uint32_t)h3 | 1u) & p.mask; p.a3 = (uint32_t)(h3 >> 32) & p.mask;
  if (p.mask == 1u) { p.m1 = p.m2 = p.m3 = 1u; }
  return p;
}

DML_HD uint32_t feat_perm_step(const FeatPerm& p, uint32_t x) {
  x = (x * p.m1 + p.a1) & p.mask;
  x ^= x >> p.sh;
  x = (x * p.m2 + p.a2) & p.mask;
  x ^= x >> p.sh;
  x = (x * p.m3 + p.a3) & p.mask;
  x ^= x >> p.sh;
  return x;
}

// k-th feature of the node's visiting order (k < d)
DML_HD int feature_at(const FeatPerm& p, int k, int d) {
  uint32_t x = feat_perm_step(p, (uint32_t)k);
  while (x >= (uint32_t)d) x = feat_perm_step(p, x);   // cycle walk: stays a permutation of [0, d)
  return (int)x;
}

// binary classification: (w class0, w class1, rows) packed in one u64 so a histogram
// update is ONE 64-bit LDS atomic.  Fields are 21/21/22 bits; a node or chunk must stay
// under kPackMaxRows rows (weights <= kPoisTable).
constexpr uint64_t kPackMask21 = (1ull << 21) - 1ull;
constexpr int kPackMaxRows = 131072;
DML_HD uint64_t pack_bin(int cls, uint32_t w) {
  return (cls == 0 ? (uint64_t)w : ((uint64_t)w << 21)) | (1ull << 42);
}

// ---- impurity from channel sums ----------------------------------------------------
#if defined(__HIPCC__)
#pragma clang fp contract(off)
#endif

// log2 for the entropy criterion, written out in IEEE +,-,*,/ (no FMA contraction in this
// header) so host and device round identically: the device libm's log2 and glibc's can
// differ by an ulp, enough to flip an entropy tie between two splits and make the HIP and
// C++ builders grow different trees.  x = m 2^e with m in [sqrt(1/2), sqrt(2));
// ln m = 2 atanh(s), s = (m-1)/(m+1), |s| < 0.1716: the series to s^21 is below 1e-18.
DML_HD double dlog2(double x) {
  int e;
#if defined(__HIP_DEVICE_COMPILE__)
  double m = ::frexp(x, &e);
#else
  double m = frexp(x, &e);
#endif
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e -= 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double s2 = s * s;
  double p = 1.0 / 21.0;
  p = p * s2 + 1.0 / 19.0;
  p = p * s2 + 1.0 / 17.0;
  p = p * s2 + 1.0 / 15.0;
  p = p * s2 + 1.0 / 13.0;
  p = p * s2 + 1.0 / 11.0;
  p = p * s2 + 1.0 / 9.0;
  p = p * s2 + 1.0 / 7.0;
  p = p * s2 + 1.0 / 5.0;
  p = p * s2 + 1.0 / 3.0;
  p = p * s2 + 1.0;
  return (double)e + (2.0 * s * p) * 1.44269504088896340736;
}

// Accumulator for one side of a classification split, fed class sums in class order.
// The entropy term (c log2 c) is only accumulated for the entropy criterion: for Gini
// it would be dead work (a double log2 per class per candidate bin).
struct ClsAcc {
  double w, sq, clogc;
  bool ent;
  DML_HDM void init(int crit) { w = 0.0; sq = 0.0; clogc = 0.0; ent = crit == kEntropy; }
  DML_HDM void add(double c) {
    w += c;
    sq += c * c;
    if (ent && c > 0.0) clogc += c * dlog2(c);
  }
};

// impurity of a node from its accumulator
DML_HD double cls_impurity(const ClsAcc& a, int crit) {
  if (a.w <= 0.0) return 0.0;
  if (crit == kEntropy) return dlog2(a.w) - a.clogc / a.w;   // -sum p log2 p
  return 1.0 - a.sq / (a.w * a.w);                           // gini
}

// proxy improvement (larger is better) ~ -(wl*imp_l + wr*imp_r) up to a constant
DML_HD double cls_proxy(const ClsAcc& l, const ClsAcc& r, int crit) {
  if (crit == kEntropy) return (l.clogc - l.w * dlog2(l.w)) + (r.clogc - r.w * dlog2(r.w));
  return (l.sq * r.w + r.sq * l.w) / (l.w * r.w);  // = l.sq/l.w + r.sq/r.w with one division
}

// ---- regression sums: exact, order-independent fixed point --------------------------
// Regression histograms (both builders, every tier) accumulate per bin, in 64-bit INTEGER
// arithmetic: sum w and the row count packed as (w | rows << 32), sum w*yq and sum w*y2q,
// with yq = rint(y 2^e1), y2q = rint(y^2 2^e2).  e1 / e2 are chosen per build (host side,
// `reg_exponents_counts`) so that no sum over a tree's rows can exceed 2^62 in magnitude.
// Integer sums are exact in ANY order: GPU atomics no longer make a regression tree
// depend on arrival order, and the C++ builder, doing the same integer sums, grows the
// identical tree (sklearn accumulates these sums in float64; the fixed-point grid is
// max|y| 2^-38 at a million rows, below fp32 y's own resolution for all but tiny y).
// Doubles are formed from the integer sums only for scoring:
//   channel 0: (double)(sum w), 1: (double)sum(w yq) 2^-e1, 2: (double)sum(w y2q) 2^-e2,
//   3: rows (regression best_left / node layout {w, wy, wyy} + rows, as before).
struct RegScale {
  double s1, s2, i1, i2;   // 2^e1, 2^e2, 2^-e1, 2^-e2
};

DML_HD RegScale reg_scale(int e1, int e2) {
  RegScale q;
  q.s1 = ldexp(1.0, e1); q.s2 = ldexp(1.0, e2);
  q.i1 = ldexp(1.0, -e1); q.i2 = ldexp(1.0, -e2);
  return q;
}

// exponents of a build from the per-target histogram of the targets' frexp exponents
// (cnt[t][k + kExpOff] rows with |y| in [2^(k-1), 2^k), bucket 0 the zeros):
// B1 = max_t sum_k c 2^k >= sum|y|, B2 likewise with 4^k >= sum y^2, summed sequentially
// in bucket order (every term exact); e1 = 61 - exponent(15 B1) so any bootstrap-weighted
// (w <= 15) sum over a tree's rows stays below 2^61, e2 the same from B2.  The y^2 grid
// follows the target's total energy, not n max|y|^2 (a node of small targets beside one
// outlier keeps its variance).  ops/forest_ops.py `reg_exponents_of_counts` is this rule.
constexpr int kExpOff = 160, kExpBins = 320;

inline void reg_exponents_counts(const int64_t* cnt, int64_t targets, int& e1, int& e2) {
  double b1 = 0.0, b2 = 0.0;
  for (int64_t t = 0; t < targets; ++t) {
    double s1 = 0.0, s2 = 0.0;
    for (int j = 1; j < kExpBins; ++j) {
      const double c = (double)cnt[t * kExpBins + j];
      s1 += c * ldexp(1.0, j - kExpOff);
      s2 += c * ldexp(1.0, 2 * (j - kExpOff));
    }
    b1 = s1 > b1 ? s1 : b1;
    b2 = s2 > b2 ? s2 : b2;
  }
  int k;
  e1 = 0; e2 = 0;
  if (b1 > 0.0) { frexp(15.0 * b1, &k); e1 = 61 - k; }
  if (b2 > 0.0) { frexp(15.0 * b2, &k); e2 = 61 - k; }
  e1 = e1 < -1000 ? -1000 : (e1 > 1000 ? 1000 : e1);
  e2 = e2 < -1000 ? -1000 : (e2 > 1000 ? 1000 : e2);
}

// round half to even, identically on host (llrint, default rounding mode) and device
DML_HD int64_t reg_round(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (int64_t)__double2ll_rn(v);
#else
  return (int64_t)llrint(v);
#endif
}

// a row's fixed-point target and squared target (y*y is exact in double: 48-bit product)
DML_HD void reg_quantize(float y, const RegScale& q, int64_t& yq, int64_t& y2q) {
  const double yd = (double)y;
  yq = reg_round(yd * q.s1);
  y2q = reg_round((yd * yd) * q.s2);
}

// ---- absolute_error (MAE) in fixed point ----------------------------------------------
// sum w |yq - med| of a set with total weight W and sum w yq S, from the median's prefix
// (wle / sle: weight and sum w yq of the ranks up to and including the median, in y order):
// med (2 wle - W) + (S - 2 sle), in modular unsigned arithmetic -- exact whenever the result
// fits (it is < 1.5 * 2^62: W |med| <= 2 sum w |yq| < 2^62 under reg_exponents_counts)
DML_HD int64_t mae_absdev(int64_t W, int64_t S, int64_t medq, int64_t wle, int64_t sle) {
  const uint64_t a = (uint64_t)medq * (uint64_t)(2 * wle - W);
  const uint64_t b = (uint64_t)S - 2ull * (uint64_t)sle;
  return (int64_t)(a + b);
}

// node value of an MAE node, {W, W med, ab + W med^2}: v1 / v0 is the median predict reads
// (sklearn's WeightedMedianCalculator: the mean of the two middle values when the prefix
// weight lands exactly on W / 2) and mse_impurity(v) the MAE impurity; ab is the exact abs
// deviation (c / cs: the prefix up to and including the lower median, medq its target).
// Both builders call this with the same integers, so their node values are identical.
DML_HD double mae_node_value(int64_t W, int64_t S, int64_t c, int64_t cs, int64_t medq, double ylo, double yhi,
                             bool tie, const RegScale& q, double* v) {
  const double med = tie ? (ylo + yhi) / 2.0 : ylo;
  const double ab = (double)mae_absdev(W, S, medq, c, cs) * q.i1;
  v[0] = (double)W; v[1] = (double)W * med; v[2] = ab + (double)W * med * med;
  return ab;
}

constexpr uint64_t kRegLo32 = 0xFFFFFFFFull;
// the double channels of integer sums (w | rows << 32, sum w yq, sum w y2q)
DML_HD double reg_w(uint64_t wr) { return (double)(wr & kRegLo32); }
DML_HD double reg_rows(uint64_t wr) { return (double)(wr >> 32); }
DML_HD double reg_s1(uint64_t v, const RegScale& q) { return (double)(int64_t)v * q.i1; }
DML_HD double reg_s2(uint64_t v, const RegScale& q) { return (double)(int64_t)v * q.i2; }

// regression: s0 = sum w, s1 = sum w*y, s2 = sum w*y^2
DML_HD double mse_impurity(double s0, double s1, double s2) {
  if (s0 <= 0.0) return 0.0;
  const double m = s1 / s0;
  return s2 / s0 - m * m;
}

DML_HD double mse_proxy(double l0, double l1, double r0, double r1) {
  return l1 * l1 / l0 + r1 * r1 / r0;
}

// regression split proxy (larger is better) from (sum w, sum wy) of both sides.
// Poisson (sklearn's criterion="poisson"): sum_l log(mean_l) + sum_r log(mean_r), -inf
// when a side's sum of y is not positive; log2 (dlog2: host/device-identical) ranks the
// same as sklearn's natural log.  Node impurities (purity, min_impurity_decrease) stay
// the squared-error ones: zero exactly when y is constant, like the Poisson deviance.
DML_HD double reg_proxy(int crit, double l0, double l1, double r0, double r1) {
  if (crit == kPoisson) {
    if (l1 <= 1e-15 || r1 <= 1e-15) return -INFINITY;
    return l1 * dlog2(l1 / l0) + r1 * dlog2(r1 / r0);
  }
  return mse_proxy(l0, l1, r0, r1);
}

// sklearn's impurity_improvement(), scaled by the node's share of the tree's weight
DML_HD double improvement(double W_tree, double W_node, double imp_node, double wl, double imp_l,
                          double wr, double imp_r) {
  return (W_node / W_tree) * (imp_node - (wr / W_node) * imp_r - (wl / W_node) * imp_l);
}

constexpr double kEps = 1e-7;  // sklearn EPSILON for purity / min_impurity_decrease tests

// regression purity.  sklearn stops at impurity <= DBL_EPSILON on float64 sums; ours is
// formed from the fixed-point sums, whose rounding bounds the impurity a constant target
// can compute: |S2/W err| <= 2^-e2 / 2, |mean err| <= 2^-e1 / 2, so |imp err| <= 2^-e2 / 2 +
// |mean| 2^-e1 + 2^-2e1 / 4, plus a few ulps of S2/W.  A node is pure below that bound:
// nodes of tiny but real variance (small targets, late boosting residuals) keep splitting
// as in sklearn, where the old absolute 1e-7 made them leaves.
constexpr double kDblEps = 2.220446049250313e-16;
DML_HD bool reg_pure(const double* v, const RegScale& q) {
  if (!(v[0] > 0.0)) return true;
  const double m = v[1] / v[0];
  const double tol = 0.5 * q.i2 + fabs(m) * q.i1 + q.i1 * q.i1 + 8.0 * kDblEps * fabs(v[2] / v[0]);
  return mse_impurity(v[0], v[1], v[2]) <= (tol > kDblEps ? tol : kDblEps);
}

// the improvement the min_impurity_decrease test reads: sklearn's impurity_improvement(),
// or for friedman_mse FriedmanMSE.impurity_improvement = (w_r s_l - w_l s_r)^2 /
// (w_l w_r W_node), which is not scaled by the tree weight.  pv / bl: the node's and the
// left side's regression sums {w, w y, ...}
template <class TS>
DML_HD double accept_improvement(const TS& s, bool is_reg, const double* pv, const double* bl, double Wt,
                                 double wN, double impN, double wL, double impL, double wR, double impR) {
  if (is_reg && s.criterion == kFriedman) {
    const double wl = bl[0], wr = pv[0] - bl[0], diff = wr * bl[1] - wl * (pv[1] - bl[1]);
    return diff * diff / (wl * wr * pv[0]);
  }
  return improvement(Wt, wN, impN, wL, impL, wR, impR);
}

// ---- monotonic_cst (sklearn >= 1.4) --------------------------------------------------
// A split on a constrained feature (m = +1 increasing, -1 decreasing; binary classifiers
// constrain the class-0 fraction, so their rows arrive negated) must keep both children's
// values inside the node's [lo, hi] and ordered; the children's bounds meet at the mean of
// the two values (sklearn's middle_value), and every node value is clipped to its bounds
// once the tree is grown.  Shared by the host builder and every HIP tier.
DML_HD double side_value(double w, double a) { return w > 0.0 ? a / w : 0.0; }

DML_HD bool mono_ok(int m, double lo, double hi, double vl, double vr) {
  return vl >= lo && vr >= lo && vl <= hi && vr <= hi && (vl - vr) * m <= 0.0;
}

// the children's bound: mean of the two side values, from (left weight, left value sum,
// right weight, right value sum)
DML_HD double mono_mid(double lw, double la, double rw, double ra) { return la / (2.0 * lw) + ra / (2.0 * rw); }

// a child's [lo, hi] from the parent's and the split's middle value
DML_HD void mono_child_bounds(int m, double lo, double hi, double mid, int side, double& clo, double& chi) {
  if (side == 0) { clo = m < 0 ? mid : lo; chi = m > 0 ? mid : hi; }
  else { clo = m > 0 ? mid : lo; chi = m < 0 ? mid : hi; }
}

// clip a grown node's value to its bounds (regression: the mean moves, the squared-error
// impurity stays; binary: the class-0 fraction is clipped, class 1 takes the rest)
DML_HD void mono_clip(double* v, int is_reg, double lo, double hi) {
  if (is_reg) {
    if (v[0] <= 0.0) return;
    const double m = v[1] / v[0];
    const double c = m < lo ? lo : (m > hi ? hi : m);
    v[2] += v[0] * (c * c - m * m);
    v[1] = v[0] * c;
  } else {
    const double W = v[0] + v[1];
    if (W <= 0.0) return;
    const double f = v[0] / W;
    const double c = f < lo ? lo : (f > hi ? hi : f);
    v[0] = W * c;
    v[1] = W * (1.0 - c);
  }
}

// leaf-by-counts rule (before any split search)
template <class TS>
DML_HD bool leaf_by_counts(const TS& t, int count, int depth) {
  return depth >= t.max_depth || count < t.min_samples_split || count < 2 * t.min_samples_leaf;
}

// min_weight_fraction_leaf (sklearn): a node lighter than 2 x min_weight_leaf is a leaf,
// and a split leaving either side lighter than min_weight_leaf is not a candidate.
// Weights include bootstrap counts and class weights (sklearn's sample weights).
template <class TS>
DML_HD bool leaf_by_weight(const TS& t, double w_node) {
  return t.min_weight_leaf > 0.0 && w_node < 2.0 * t.min_weight_leaf;
}

template <class TS>
DML_HD bool side_too_light(const TS& t, double wl, double wr) {
  return t.min_weight_leaf > 0.0 && (wl < t.min_weight_leaf || wr < t.min_weight_leaf);
}

// total weight of a node value vector (class sums | (sum w, sum wy, sum wy^2))
DML_HD double vals_weight(const double* v, int C, int is_reg) {
  if (is_reg) return v[0];
  double w = 0.0;
  for (int k = 0; k < C; ++k) w += v[k];
  return w;
}

// ---- max_leaf_nodes: best-first selection on a grown tree ---------------------------
// sklearn grows a max_leaf_nodes tree best-first (BestFirstTreeBuilder): it always
// expands the frontier node of largest impurity improvement and stops after L-1
// expansions.  Every node's split here is a function of the node alone (keyed feature
// permutation, same rows), so that tree is exactly the top of the depth-first tree this
// builder grows: replay the best-first order over the grown tree and turn the internal
// nodes still on the frontier into leaves (their stored sums are their leaf values).
// One routine for the HIP kernel (one lane per tree) and the C++ builder: same order,
// same doubles, identical trees.

DML_HD double val_impurity(const double* v, int C, bool is_reg, int crit, double& w) {
  if (is_reg) { w = v[0]; return mse_impurity(v[0], v[1], v[2]); }
  ClsAcc a;
  a.init(crit);
  for (int k = 0; k < C; ++k) a.add(v[k]);
  w = a.w;
  return cls_impurity(a, crit);
}

DML_HD double split_priority(const NodeRec* nodes, const double* vals, int64_t VC, int C, bool is_reg, int crit,
                             double Wt, int node) {
  double wN, wL, wR;
  const int l = nodes[node].left;
  const double iN = val_impurity(vals + (int64_t)node * VC, C, is_reg, crit, wN);
  const double iL = val_impurity(vals + (int64_t)l * VC, C, is_reg, crit, wL);
  const double iR = val_impurity(vals + (int64_t)(l + 1) * VC, C, is_reg, crit, wR);
  return improvement(Wt, wN, iN, wL, iL, wR, iR);
}

struct FrontierEnt {
  double pri;
  int32_t node, pad;
};

// max-heap order: larger improvement first, then the smaller node id (deterministic ties)
DML_HD bool frontier_before(const FrontierEnt& a, const FrontierEnt& b) {
  return a.pri > b.pri || (a.pri == b.pri && a.node < b.node);
}

DML_HDM void frontier_push(FrontierEnt* h, int& n, FrontierEnt e) {
  int i = n++;
  while (i > 0) {
    const int p = (i - 1) >> 1;
    if (!frontier_before(e, h[p])) break;
    h[i] = h[p];
    i = p;
  }
  h[i] = e;
}

DML_HDM FrontierEnt frontier_pop(FrontierEnt* h, int& n) {
  const FrontierEnt top = h[0];
  const FrontierEnt last = h[--n];
  int i = 0;
  for (;;) {
    const int l = 2 * i + 1;
    if (l >= n) break;
    const int m = (l + 1 < n && frontier_before(h[l + 1], h[l])) ? l + 1 : l;
    if (!frontier_before(h[m], last)) break;
    h[i] = h[m];
    i = m;
  }
  if (n > 0) h[i] = last;
  return top;
}

// Keep the best-first top of the tree rooted at ``root`` with at most L leaves.
// ``heap``: scratch for at least L entries (the frontier never holds more).
// Returns the number of leaves of the kept tree.
DML_HDM int best_first_prune(NodeRec* nodes, const double* vals, int64_t VC, int C, bool is_reg, int crit, int root,
                             int L, FrontierEnt* heap) {
  if (nodes[root].split < 0) return 1;
  double Wt;
  val_impurity(vals + (int64_t)root * VC, C, is_reg, crit, Wt);
  int n = 0, leaves = 1, budget = L - 1;
  frontier_push(heap, n, FrontierEnt{split_priority(nodes, vals, VC, C, is_reg, crit, Wt, root), root, 0});
  while (n > 0) {
    const FrontierEnt e = frontier_pop(heap, n);
    if (budget <= 0) {   // out of expansions: this frontier node stays a leaf
      nodes[e.node].split = -1;
      nodes[e.node].left = -1;
      continue;
    }
    --budget;
    ++leaves;
    const int l = nodes[e.node].left;
    for (int s = 0; s < 2; ++s)
      if (nodes[l + s].split >= 0)
        frontier_push(heap, n, FrontierEnt{split_priority(nodes, vals, VC, C, is_reg, crit, Wt, l + s), l + s, 0});
  }
  return leaves;
}

}  // namespace dml
