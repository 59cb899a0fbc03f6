// forest.hip — batched level-wise random-forest builder and predictor for CDNA4 (gfx950).
//
// Replaces the delegated scikit-learn tree builders the reference calls per task
// (aws-prod/worker/worker.py:315 `model.fit`, :326/:341 `cross_val_score` -> 5 more
// fits, :322/:336 `predict`).  Instead of one CPU fit per (candidate, fold) this builds
// EVERY tree of MANY fits (candidates x CV folds x trees) at once, breadth-first,
// against one HBM-resident binned copy of the dataset.  Folds and bootstraps are never
// materialised: a row's role (train/test) comes from a per-split uint8 vector and its
// bootstrap weight is recomputed from a counter hash (forest_common.h).
//
// Work per level is bucketed by node size so every node gets a right-sized worker:
//   * wave tier  (count <= wave_max):  one 64-lane wave per node; LDS histogram,
//     wave-scan over the 256 bins, wave-argmax, ballot-based stable partition — one
//     fused kernel, no global histogram traffic;
//   * block tier (count <= block_max): one 256-thread workgroup per node, same fused
//     pipeline with 4 waves evaluating features in parallel;
//   * large tier (count > block_max):  per (node, row-chunk) workgroups build LDS
//     histograms and flush them with ONE coalesced atomic pass into a per-node global
//     histogram; a per-node kernel scans/selects; a chunked kernel partitions.
// Histograms are integer (uint32) for classification, so results are bit-identical
// to the CPU builder whatever the atomic arrival order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <type_traits>
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "forest_common.h"
#include "wave_ops.h"

#ifndef DML_RPT_BLOCK
#define DML_RPT_BLOCK 1
#endif
#if DML_RPT_BLOCK < 1 || DML_RPT_BLOCK > 4
#error "DML_RPT_BLOCK must be 1..4"
#endif
#ifndef DML_BLOCK_NT
// threads per block-tier node of a binary-classification build: 2 waves.  With the LDS slab
// sized to the batch's max_features (10: 22 KB) 7 nodes share a CU instead of 4 at 256
// threads -- the per-node serial phases (setup, split selection, partition scan) overlap
// across more nodes (sweep build 0.988 -> 0.974 s, 0.960 s with wave_max 256;
// profiles/r6_block_nt128_sweep.txt).  Multiclass / regression builds keep 4 waves: their
// wider histogram planes (up to 96 KB of LDS) allow only 1-2 nodes per CU.
#define DML_BLOCK_NT 128
#endif
template <int MODE> constexpr int block_nt() { return MODE == 1 ? DML_BLOCK_NT : 256; }
#ifndef DML_NODES_WPE
// block tier (binary): 4 waves per SIMD = 4 workgroups per CU.  With the register-rows paths
// compiled out (DML_BLOCK_STREAM_ONLY) and the window loop's bins packed 4 per register the
// kernel fits 127 VGPRs without spills (it needed 168 at 3 waves before): sweep build
// 1.029 -> 1.008 s (profiles/r5_block_occupancy.txt)
#define DML_NODES_WPE 4
#endif
// eval_feature is called with an LDS histogram (fused node kernels) and a global one
// (large tier): inlined, each call site keeps its address space (ds_read / global_load);
// out of line, every histogram access is a flat op that also counts on lgkmcnt.
#ifndef DML_EVAL_NOINLINE
#define DML_EVAL_ATTR __attribute__((always_inline))
#else
#define DML_EVAL_ATTR
#endif
#ifndef DML_PART_U2
#define DML_PART_U2 4          // block-tier partition pass 2: row positions per thread per round
#endif
#ifndef DML_KGL_LARGE
#define DML_KGL_LARGE 16       // k_hist_large: widest feature group of the pipelined (and unit-weight) loop
#endif
#ifndef DML_KGW_LARGE
#define DML_KGW_LARGE 32       // k_hist_large: widest round of a row-window node (two 16-B pieces of the line)
#endif
#ifndef DML_PART_KEEP
#define DML_PART_KEEP 2        // block-tier partition: rounds whose row ids pass 1 keeps in registers (0/1/2: 1.018/1.014/1.009 s sweep build, r5 e6)
#endif
#ifndef DML_NODES_WPE_WAVE
#define DML_NODES_WPE_WAVE 4   // wave tier (binary): 2 / 3 / 5 / 6 measured slower (ROUND3.md)
#endif
#ifndef DML_NODES_WPE_WAVE_MAX
#define DML_NODES_WPE_WAVE_MAX 8   // wave tier (binary) occupancy cap: 8 -> 64 VGPRs (spills), lower -> more VGPRs
#endif
#ifndef DML_KGMAX_BLOCK
#define DML_KGMAX_BLOCK 16     // block tier: largest feature group with register-resident bins
#endif
#ifndef DML_BLOCK_STREAM_ONLY
#define DML_BLOCK_STREAM_ONLY 1   // block-tier nodes (> wave_max >= 256 rows) always stream their rows
#endif
#ifndef DML_NODES_WPE_REG
#define DML_NODES_WPE_REG 2   // regression node kernels: 3 histogram planes + payloads fit 256 VGPRs, no spills
#endif
#ifndef DML_NODES_WPE_MC
#define DML_NODES_WPE_MC 2    // multiclass: C+1 histogram planes; 2 waves per SIMD without spills beats 4 with
#endif
#ifndef DML_SUB_SEG_REG
#define DML_SUB_SEG_REG 1     // regression subtrees: segmented evaluation of nodes <= 32 rows
#endif
#ifndef DML_KGMAX_WAVE
#define DML_KGMAX_WAVE 4
#endif
#ifndef DML_ROW_WINDOWS
#define DML_ROW_WINDOWS 1      // block tier: whole-row dwordx4 loads for the first feature group (d <= 112)
#endif
#ifndef DML_WAVE_WIN_ROWS
#define DML_WAVE_WIN_ROWS 4    // wave tier: rows whose line windows are in flight together (1, 2 or 4; 0 = byte gathers)
#endif
#ifndef DML_GINI_PF
#define DML_GINI_PF 1          // binary Gini: fp32 pre-filter of candidate bins (eval_feature)
#endif
#ifndef DML_EVAL_PAIRS
#define DML_EVAL_PAIRS 0       // k_nodes: binary-Gini features evaluated two at a time (1 both tiers, 2 wave, 3 block; slower)
#endif
#ifndef DML_WAVE_PREFETCH
#define DML_WAVE_PREFETCH 12   // wave tier: visiting positions whose bins are gathered up front
#endif
// large-tier grids: node index fastest (1) so chunk c of EVERY large node is in flight at
// once -- at the top levels the rows behind chunk c of all trees of a fold are nearly the
// same rows, so those table lines are served from the XCD's L2 -- or chunk fastest (0)
#ifndef DML_LARGE_NODE_FAST
#define DML_LARGE_NODE_FAST 1
#endif
#if DML_LARGE_NODE_FAST
#define DML_LSLOT ((int)blockIdx.x)
#define DML_LCHUNK ((int)blockIdx.y)
#else
#define DML_LSLOT ((int)blockIdx.y)
#define DML_LCHUNK ((int)blockIdx.x)
#endif

// optional per-phase cycle accounting of the fused node kernel (-DDML_PHASE_PROF builds only)
#ifdef DML_PHASE_PROF
// [0] wave tier, [1] block tier, [2] subtree tier phases (slot 7: nodes), [3] rows per tier +
// subtree internal-node counts by evaluation path
__device__ unsigned long long g_phase[4][8];
#define PH_BEGIN uint64_t _pt = clock64(); uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PH(i) if (threadIdx.x == 0) { const uint64_t _n = clock64(); _acc[i] += _n - _pt; _pt = _n; }
#define PH_END(t) if (threadIdx.x == 0) { _acc[7] = 1; for (int _i = 0; _i < 8; ++_i) atomicAdd(&g_phase[t][_i], _acc[_i]); \
                                            atomicAdd(&g_phase[3][t], (unsigned long long)on.count); }
#define PH_CNT(i, v) if (threadIdx.x == 0) atomicAdd(&g_phase[3][i], (unsigned long long)(v));
#define PH_ARGS_DECL , uint64_t& _pt, uint64_t* _acc
#define PH_ARGS_PASS , _pt, _acc
#else
#define PH_BEGIN
#define PH(i)
#define PH_END(t)
#define PH_CNT(i, v)
#define PH_ARGS_DECL
#define PH_ARGS_PASS
#endif

namespace dml {

// an open node: its rows are rows_cur[start, start + count) -- `start` is ABSOLUTE (tree
// offset folded in at enqueue), so a node kernel's first dependent load is its rows
struct OpenNode {
  int32_t tree, node;
  int64_t start;
  int32_t count, depth;
  uint64_t key;
  int32_t pool_base;   // subtree tier: first pool slot of the subtree's reserved pairs (-1: k_subtree
                       // reserves them itself, -2: pool overflow already flagged)
  int32_t tier;        // child staging slot: the child's tier, -1 = no open child
};

// ctypes-facing argument block: every field is 8 bytes (pointers as int64).
struct ForestArgs {
  int64_t Xb, ld, n, d;
  int64_t ycls, yreg, n_classes, is_reg;
  int64_t roles, n_splits;
  int64_t specs, T;
  int64_t active_count;  // int32[T]  (count phase output)
  int64_t row_off;       // int64[T+1] device offsets (exclusive prefix of active_count)
  int64_t rows_total;
  int64_t max_active;    // max over trees of active_count
  int64_t nodes, node_val, pool_cap;  // NodeRec*, double* [pool_cap*VC]
  int64_t tree_W;        // double[T]
  int64_t workspace, workspace_bytes;
  int64_t wave_max, block_max, chunk;
  int64_t kg_wave, kg_block, kg_large;
  int64_t slack_wave;
  int64_t sub_max, sub_cache_d;
  // outputs
  int64_t n_nodes_out, status_out, levels_out, large_rounds_out;
  int64_t tier_nodes_out[4];
  int64_t ystride;       // >0: tree t regresses on yreg[specs[t].target * ystride + row] (boosting)
  int64_t XbT;           // optional feature-major copy of the bins, uint8 [d][n] (0 = none)
  int64_t cw;            // class-weight table double [T][C] (0 = no class weights in this build)
  int64_t yq_e1, yq_e2;  // regression fixed-point exponents (forest_common.h reg_exponents)
  int64_t mono;          // int8 [fits][d] monotonic_cst rows (binary classifiers negated), 0 = none
  int64_t nbound;        // double [pool_cap][2] node bounds (lo, hi) when mono != 0
  int64_t fast_crit;     // 1 + the single criterion of a build with no class weights, monotonic
                         // constraints or min_weight_fraction_leaf (node kernels specialised on it); 0 = generic
  // early predict: a host PredictArgs for the build's fits (0 = none) and a host int32[n_fits]
  // of the level after which fit f's trees are complete (its max_depth - 1); the builder
  // launches fit f's predict right after that level on its own stream, overlapping the
  // deeper fits' remaining levels, and marks the entry -2
  int64_t early_pred, fit_done_level, n_fits;
  // > 0 (binary classification, no monotonic constraints, row cache on): tier 1 holds the
  // nodes of sub_max < count <= bigsub_max (= wave_max, <= 256) and k_bigsub grows each
  // one's whole subtree on chip
  int64_t bigsub_max;
  // 1: every tree evaluates every feature (max_features == d: boosting, max_features=None)
  // -- the large tier then needs exactly ceil(d / kg_large) feature rounds per level, launched
  // without reading the "need more" flag back after each round
  int64_t all_features;
  int64_t sub_small;   // 0 < sub_small < sub_max (<= 32): subtree roots of <= sub_small rows -> tier 4
  // boosting (regression, unit weights, whole-histogram roots): uint32 [T][d][256] row counts
  // of every tree's ROOT histogram.  The root's rows are the fit's training rows at every stage
  // of an active set, so its count planes never change: root_counts_valid = 0 -> this build's
  // root level stores them, 1 -> the root level skips its count atomics and copies them in
  int64_t root_counts, root_counts_valid;
  // regression build whose every tree has unit row weights (no bootstrap: boosting): the large
  // tier's LDS histograms drop the unused half of the count plane (3 KB instead of 4 KB per
  // feature: 16 features in 48 KB, three workgroups per CU instead of two)
  int64_t large_unit;
  // unit-weight regression build whose fixed-point targets satisfy |yq| < 2^39 (ops/forest_ops.py
  // checks it from the exponent histogram) with <= 4095-row large-tier chunks: the large tier's
  // row count and w yq share ONE u64 LDS atomic, (1 << 52) + yq + 2^39 per row (kPack*)
  int64_t large_pack;
};

// 0 subtree, 1 wave, 2 block, 3 large, 4 small subtree (<= sub_small rows: the subtree kernel
// with an LDS row cache of half the size, so twice as many of them fit a CU)
constexpr int kTiers = 5;
enum CounterSlot { kCntSets = 0 /*10*/, kPool = 10, kOverflow = 11, kNeedMore = 12, kOpenOvf = 13, kNumCounters = 16 };

struct LState {
  OpenNode on;
  int32_t pos, nonconst, g, done;
  int32_t best_feat, best_bin, split, nl;
  double best_gain;
  int32_t best_pos; // visiting position of the best split's feature
  int32_t scr_n;    // positions [0, scr_n) have their bins in Ctx::bscr (round 0, <= 16 features)
  double best_mid;  // monotonic_cst: middle value of the best split
  // whole-histogram levels (Ctx::full_cur): features [0, scr_id) -- by feature id -- have their
  // bins in bscr; derive: the histogram is parent - sibling (no row pass), par / sib the
  // parent's large slot one level up and the sibling's slot at this level
  int32_t scr_id, derive, par, sib;
};

struct Ctx {
  const uint8_t* Xb;
  int64_t ld;
  int32_t n, d, C, CH, VC, is_reg;
  const int32_t* ycls;
  const float* yreg;
  const uint8_t* roles;
  const TreeSpec* specs;
  int32_t T;
  int32_t* active_count;
  const int64_t* row_off;
  uint32_t* rows_cur;
  uint32_t* rows_next;
  NodeRec* nodes;
  double* node_val;
  int64_t pool_cap;
  double* tree_W;
  OpenNode* open[2][kTiers];
  int64_t open_cap[kTiers];
  // child staging: the wave/block-tier parent at level position i writes its two children to
  // stage[2 i + side] (no atomics); k_compact buckets them into the next level's open lists
  // with one atomic per workgroup and tier -- a per-child returning atomic on one counter
  // address per tier serialised ~60 M times per bench build (+0.56 s for one extra per child)
  OpenNode* stage;
  int32_t* counters;
  int32_t* cursors;      // [T]
  LState* lstate;
  int16_t* lperm;        // [cap_large][d]
  double* lbest_left;    // [cap_large][CH]
  void* ghist;           // [cap_large][kg_large][CH][256] (u32 or f32)
  int32_t* lcursor;      // [cap_large][2]
  // whole-histogram large levels (every tree evaluates every feature and the level's
  // histograms fit the budget): each large node's histogram over ALL d features,
  // [slot][d][global planes][256], is kept for the next level, where the larger of two
  // large-tier siblings takes parent - smaller sibling instead of a pass over its rows.
  // gf_cur / gf_prev: this level's and the previous level's buffers; pinfo_cur[slot] =
  // {parent slot, sibling slot, derive?} as written by the previous level's k_split_large,
  // pinfo_next the same for the next level
  void* gf_cur;
  const void* gf_prev;
  const int4* pinfo_cur;
  int4* pinfo_next;
  int32_t full_cur, full_prev;
  int32_t root_cnt_skip;       // root level of a build with cached root counts: no count atomics
  int32_t large_compact;       // ForestArgs::large_unit (and kg_large <= DML_KGL_LARGE): 3-KB LDS slices
  int32_t fm_div;              // k_hist_large: row-window gathers for boosting nodes < n / fm_div rows (0: none)
  int32_t kg_rw;               // k_hist_large: features per round of a row-window node (multiple of 16; 0: kg_large)
  int32_t large_pack;          // ForestArgs::large_pack (with large_compact): packed count | w yq words
  uint32_t* root_counts;       // ForestArgs::root_counts (null: none)
  int64_t pi_cap;        // entries of each pinfo table
  // whole-histogram levels: every (large node, visiting position)'s split candidate, from
  // k_split_full (one wave per feature, all features of all nodes in one launch), selected in
  // visiting order by k_split_full_select: [slot][d] (+ [CH] for the left sums)
  double* fr_g;
  double* fr_mid;
  double* fr_left;
  int32_t* fr_b;
  int32_t* fr_n;
  unsigned long long* lyy;   // [cap_large] regression: sum w y2q of the best split's left rows
  int64_t large_cap;
  int32_t wave_max, block_max, chunk, kg_wave, kg_block, kg_large, slack_wave;
  int32_t sub_max, sub_cache_d;
  int32_t bigsub_max;    // > 0: tier 1 (sub_max < count <= bigsub_max) is grown by k_bigsub
  int32_t sub_small;     // 0 < sub_small < sub_max: subtree roots of <= sub_small rows go to tier 4
  int64_t ystride;
  // row words: rows_cur/rows_next hold row | bootstrap weight << rbits | class << (rbits + 4)
  // when `packed` (the weight and label travel with the row through every partition, so
  // no kernel re-gathers ycls or re-hashes the bootstrap weight); else plain row ids
  uint32_t rmask;
  int32_t rbits, packed;
  // block tier, streamed nodes: the feature group's bins of every row, 16 B per row
  // position (positions of rows_cur), written by the histogram pass so the partition
  // reads the split feature's bin with 16-B-strided coalesced loads instead of
  // re-gathering a 128-B table line per row
  uint8_t* bscr;
  // feature-major bins [d][n] (optional): the large tier's nodes hold a dense, sorted
  // share of the table's rows, so a 64-lane gather of one feature from the feature-major
  // copy touches a couple of lines instead of 64 row lines
  const uint8_t* XbT;
  // class weights (sklearn class_weight): row t of a [T][C] table multiplies tree t's
  // integer class sums wherever they become doubles (histogram scans, root and child
  // statistics); rows of balanced_subsample trees are filled by k_roots
  const double* cw;
  // regression: exact integer histogram sums of w, w yq, w y2q (forest_common.h)
  RegScale rq;
  unsigned long long* rsum;   // [T][3] integer root sums (k_fill_active -> k_roots)
  // monotonic_cst: per-fit constraint rows and every pool node's value bounds [lo, hi]
  // (forest_common.h mono_*); null when no tree of the build is constrained
  const int8_t* mono;
  double* nbound;
};

// The TreeSpec fields the kernels read, as scalars (a by-value TreeSpec would live in
// scratch memory: it embeds the Poisson table, which stays behind a pointer here).
struct NodeSpec {
  uint64_t seed;
  const uint32_t* pois_cdf;
  int32_t split, fit, max_depth, min_samples_split, min_samples_leaf, max_features, bootstrap, criterion, target,
      cw_mode;
  float min_impurity_decrease;
  double min_weight_leaf;
};
// the constraint of feature f for the tree's fit (0: unconstrained or no table)
template <int FC = -1>
__device__ __forceinline__ int mono_of(const Ctx& c, const NodeSpec& s, int f) {
  if constexpr (FC >= 0) return 0;
  return c.mono ? (int)c.mono[(int64_t)s.fit * c.d + f] : 0;
}

// children's bounds from the parent's and the chosen split (every child of a build with a
// constraint table gets bounds, unconstrained splits pass the parent's through)
template <int FC = -1>
__device__ __forceinline__ void mono_children(const Ctx& c, int node, int left, int m, double mid) {
  if (FC >= 0 || !c.nbound) return;
  const double lo = c.nbound[2 * (int64_t)node], hi = c.nbound[2 * (int64_t)node + 1];
  for (int side = 0; side < 2; ++side) {
    double clo, chi;
    mono_child_bounds(m, lo, hi, mid, side, clo, chi);
    c.nbound[2 * (int64_t)(left + side)] = clo;
    c.nbound[2 * (int64_t)(left + side) + 1] = chi;
  }
}

// Node kernels specialised on one criterion (FC >= 0): the build has no class weights, no
// monotonic constraints and no min_weight_fraction_leaf, so those branches and every other
// criterion's scoring (entropy log2 series, Poisson) compile out of the kernel (spec_of here,
// and tree_cw / mono_of / mono_children / the node-bound reads return their neutral values).
template <int FC>
__device__ __forceinline__ NodeSpec spec_of(const Ctx& c, int tree) {
  const TreeSpec& t = c.specs[tree];
  NodeSpec s;
  s.seed = t.seed; s.pois_cdf = t.pois_cdf; s.split = t.split; s.fit = t.fit; s.max_depth = t.max_depth;
  s.min_samples_split = t.min_samples_split; s.min_samples_leaf = t.min_samples_leaf;
  s.max_features = t.max_features; s.bootstrap = t.bootstrap; s.criterion = t.criterion; s.target = t.target;
  s.cw_mode = t.cw_mode; s.min_impurity_decrease = t.min_impurity_decrease; s.min_weight_leaf = t.min_weight_leaf;
  if constexpr (FC >= 0) { s.criterion = FC; s.min_weight_leaf = 0.0; }
  return s;
}

// target vector of a tree (shared y, or its own row of the boosting target matrix)
__device__ __forceinline__ const float* tree_y(const Ctx& c, const NodeSpec& s) {
  return c.ystride ? c.yreg + (int64_t)s.target * c.ystride : c.yreg;
}

__device__ __forceinline__ uint32_t word_row(const Ctx& c, uint32_t wd) { return wd & c.rmask; }

// PK: the kernel is specialised on packed row words (FC >= 0 builds are launched only then)
template <bool PK = false>
__device__ __forceinline__ uint32_t word_weight(const Ctx& c, const NodeSpec& s, uint32_t wd) {
  return (PK || c.packed) ? (wd >> c.rbits) & 15u : boot_weight(s, wd);
}

template <bool PK = false>
__device__ __forceinline__ int word_cls(const Ctx& c, uint32_t wd) {
  return (PK || c.packed) ? (int)(wd >> (c.rbits + 4)) : c.ycls[wd];
}

// class-weight row of a tree (nullptr: every weight is 1)
template <int FC = -1>
__device__ __forceinline__ const double* tree_cw(const Ctx& c, int tree) {
  if constexpr (FC >= 0) return nullptr;
  return (c.cw && c.specs[tree].cw_mode) ? c.cw + (int64_t)tree * c.C : nullptr;
}
__device__ __forceinline__ double cwk(const double* cw, int k) { return cw ? cw[k] : 1.0; }

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ int lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// ------------------------------------------------------------------------------------
// node bookkeeping
// ------------------------------------------------------------------------------------
__device__ double node_impurity(const Ctx& c, int node, int crit) {
  const double* v = c.node_val + (int64_t)node * c.VC;
  if (c.is_reg) return mse_impurity(v[0], v[1], v[2]);
  ClsAcc a;
  a.init(crit);
  for (int k = 0; k < c.C; ++k) a.add(v[k]);
  return cls_impurity(a, crit);
}

__device__ double node_weight(const Ctx& c, int node) {
  const double* v = c.node_val + (int64_t)node * c.VC;
  if (c.is_reg) return v[0];
  double w = 0.0;
  for (int k = 0; k < c.C; ++k) w += v[k];
  return w;
}

// the tier a node of `count` rows is grown by
__device__ __forceinline__ int tier_of(const Ctx& c, int count) {
  if (count <= c.sub_max) return count <= c.sub_small ? 4 : 0;
  return count <= c.wave_max ? 1 : (count <= c.block_max ? 2 : 3);
}

// decide whether a freshly created node is worth visiting; enqueue it into `set`
// (returns the node's index in the next level's large-tier list, else -1)
__device__ int enqueue_or_leaf(const Ctx& c, int tree, int node, int64_t start, int count, int depth,
                               uint64_t key, int set) {
  const NodeSpec s = spec_of<-1>(c, tree);
  if (leaf_by_counts(s, count, depth)) return -1;
  if (leaf_by_weight(s, node_weight(c, node))) return -1;
  if (c.is_reg ? reg_pure(c.node_val + (int64_t)node * c.VC, c.rq) : node_impurity(c, node, s.criterion) <= kEps)
    return -1;
  const int tier = tier_of(c, count);
  const int idx = atomicAdd(&c.counters[set * kTiers + tier], 1);
  if (idx >= c.open_cap[tier]) {
    atomicOr(&c.counters[kOpenOvf], 1);
    return -1;
  }
  OpenNode on;
  on.tree = tree; on.node = node; on.start = start; on.count = count; on.depth = depth;
  on.key = key; on.pool_base = -1; on.tier = tier;
  c.open[set][tier][idx] = on;
  return tier == 3 ? idx : -1;
}

// node pairs a subtree-tier node reserves: a subtree over cnt0 rows has at most
// cnt0 / min_samples_leaf - 1 splits, and at most 2^levels_left - 1 under max_depth
template <class TS>
__device__ __forceinline__ int subtree_max_splits(const TS& s, int cnt0, int depth) {
  int max_splits = cnt0 / max(1, s.min_samples_leaf) - 1;
  const int levels_left = s.max_depth - depth;
  if (levels_left < 30) max_splits = min(max_splits, (1 << max(0, levels_left)) - 1);
  return max(0, max_splits);
}

// allocate two children, write parent record and children stats. returns left index or -1.
__device__ int make_children(const Ctx& c, int node, int feat, int bin, const double* left_ch) {
  const int base = atomicAdd(&c.counters[kPool], 2);
  if ((int64_t)base + 2 > c.pool_cap) {
    atomicOr(&c.counters[kOverflow], 1);
    return -1;
  }
  NodeRec leaf; leaf.split = -1; leaf.left = -1;
  c.nodes[base] = leaf;
  c.nodes[base + 1] = leaf;
  const double* pv = c.node_val + (int64_t)node * c.VC;
  double* lv = c.node_val + (int64_t)base * c.VC;
  double* rv = lv + c.VC;
  for (int k = 0; k < c.VC; ++k) {
    lv[k] = left_ch[k];
    rv[k] = pv[k] - left_ch[k];
  }
  NodeRec rec; rec.split = pack_split(feat, bin); rec.left = base;
  c.nodes[node] = rec;
  return base;
}

// ------------------------------------------------------------------------------------
// histogram modes
// ------------------------------------------------------------------------------------
// MODE 0: classification, C class planes + 1 row-count plane of uint32 [CH][256]
// MODE 1: binary classification, ONE uint64 plane: (w0 | w1 << 21 | rows << 42)
// MODE 2: regression, float planes (sum w, sum wy, sum wy^2, rows) [4][256]
template <int MODE> struct HT;
template <> struct HT<0> { using T = uint32_t; };
template <> struct HT<1> { using T = unsigned long long; };
template <> struct HT<2> { using T = unsigned long long; };

// planes of one feature's histogram: MODE 1 one packed plane, MODE 2 three integer planes
// (w | rows << 32, sum w yq, sum w y2q), MODE 0 the CH class/row planes
__host__ __device__ __forceinline__ int hist_planes(int MODE, int CH) { return MODE == 1 ? 1 : (MODE == 2 ? 3 : CH); }
// the large tier's regression histograms drop the y^2 plane: a split's choice needs only
// (w | rows, w yq); the children's sum w y2q comes from the partition pass, which sees
// every row once (k_partition_large / k_large_finish) -- one u64 LDS atomic fewer per
// (row, feature) in the kernel that dominates boosting builds
__host__ __device__ __forceinline__ int large_planes(int MODE, int CH) { return MODE == 2 ? 2 : hist_planes(MODE, CH); }

// histogram payload of one row: MODE 0 cls | w << 32, MODE 1 packed u64, MODE 2 the
// row's three integer regression terms
struct RegPL {
  unsigned long long wr, wy, wyy;   // w | 1 << 32, w yq, w y2q (two's complement)
};
template <int MODE> struct PLT { using T = uint64_t; };
template <> struct PLT<2> { using T = RegPL; };

__device__ __forceinline__ RegPL reg_payload(const Ctx& c, uint32_t w, float y) {
  int64_t yq, y2q;
  reg_quantize(y, c.rq, yq, y2q);
  RegPL p;
  p.wr = (unsigned long long)w | (1ull << 32);
  p.wy = (unsigned long long)((int64_t)w * yq);
  p.wyy = (unsigned long long)((int64_t)w * y2q);
  return p;
}

template <typename CT>
__device__ __forceinline__ void scan256(CT* p, int lane) {
  CT v0 = p[4 * lane], v1 = p[4 * lane + 1], v2 = p[4 * lane + 2], v3 = p[4 * lane + 3];
  v1 += v0; v2 += v1; v3 += v2;
  CT t;
  if constexpr (sizeof(CT) == 8) t = (CT)wave::incl_scan_u64((uint64_t)v3);
  else t = wave::incl_scan<CT>(v3);
  const CT ex = wave::excl_from_incl<CT>(t);
  p[4 * lane] = v0 + ex; p[4 * lane + 1] = v1 + ex; p[4 * lane + 2] = v2 + ex; p[4 * lane + 3] = v3 + ex;
}

// channel `ch` (CH layout: classes.., rows / s0,s1,s2,rows) of cumulative bin b
template <int MODE>
__device__ __forceinline__ double hist_chan(const typename HT<MODE>::T* h, int ch, int CH, int b) {
  if constexpr (MODE == 1) {
    const unsigned long long v = h[b];
    return (double)(ch == 2 ? (v >> 42) : ((v >> (21 * ch)) & kPackMask21));
  } else {
    return (double)h[ch * 256 + b];
  }
}

// ONE wave evaluates one feature's histogram: in-place scans, best bin, non-constant
// flag, the best bin's cumulative channels (out_left[CH]); optionally zeroes the
// histogram afterwards so the next feature group needs no clearing pass.
// monotonic_cst of one evaluated feature: its constraint m (0 = none) and the node's bounds
struct MonoQ {
  int m;
  double lo, hi;
};

template <int MODE>
__device__ DML_EVAL_ATTR void eval_feature_lds(typename HT<MODE>::T* h, int C, int CH, const NodeSpec& s, int lane,
                                 double* out_gain, int* out_bin, int* out_nc, double* out_left, bool zero_after,
                                 const double* cw, MonoQ mq, double* out_mid);

// binary Gini with class weights in [2^-20, 2^20] and no monotonic constraint: the fp32
// pre-filter path of eval_feature below
__device__ __forceinline__ bool gini_pf_ok(const NodeSpec& s, double cw0, double cw1) {
  return DML_GINI_PF && s.criterion == kGini && cw0 >= 0x1p-20 && cw0 <= 0x1p20 && cw1 >= 0x1p-20 && cw1 <= 0x1p20;
}

// Binary Gini, fp32 pre-filter + fp64 re-scoring (see eval_feature), for NF features at
// once: feature f's histogram is h + f * FS * span and its outputs sit FS apart.  The NF
// scans and reductions are independent chains that the scheduler interleaves -- one wave
// evaluates a wave-tier node's features, so this chain is that tier's critical path.
// A candidate whose own bin is empty is skipped: its cumulative channels equal the previous
// bin's, which wins the tie (lowest bin), so the split chosen is unchanged; what is left is
// usually one contender per lane, re-scored in one pass.
template <int NF, int FS>
__device__ DML_EVAL_ATTR void eval_gini_pf(unsigned long long* h, int span, const NodeSpec& s, int lane,
                                           double* out_gain, int* out_bin, int* out_nc, double* out_left, int CH,
                                           bool zero_after, double cw0, double cw1) {
  uint64_t v[NF][4];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int i = 0; i < 4; ++i) v[f][i] = h[f * FS * span + 4 * lane + i];
  if (zero_after) {
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) h[f * FS * span + 4 * lane + i] = 0ull;
  }
  uint32_t nz[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    nz[f] = (v[f][0] != 0ull ? 1u : 0u) | (v[f][1] != 0ull ? 2u : 0u) | (v[f][2] != 0ull ? 4u : 0u) |
            (v[f][3] != 0ull ? 8u : 0u);
    v[f][1] += v[f][0]; v[f][2] += v[f][1]; v[f][3] += v[f][2];
  }
  uint64_t t[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) t[f] = wave::incl_scan_u64(v[f][3]);
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const uint64_t ex = wave::excl_from_incl<uint64_t>(t[f]);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[f][i] += ex;
  }
  const uint32_t mslu = (uint32_t)s.min_samples_leaf;
  const float cw0f = (float)cw0, cw1f = (float)cw1;
  const bool mwl = s.min_weight_leaf > 0.0;
  uint32_t tr[NF], t0i[NF], t1i[NF];
  float q[NF][4], qm[NF];
  bool nc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const uint64_t tv = wave::bcast<uint64_t>(t[f], 63);
    tr[f] = (uint32_t)(tv >> 42); t0i[f] = (uint32_t)(tv & kPackMask21); t1i[f] = (uint32_t)((tv >> 21) & kPackMask21);
    const double t0 = (double)t0i[f] * cw0, t1 = (double)t1i[f] * cw1;
    qm[f] = -INFINITY;
    nc[f] = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t cv = v[f][i];
      const uint32_t rl = (uint32_t)(cv >> 42), rr = tr[f] - rl;
      const uint32_t l0i = (uint32_t)(cv & kPackMask21), l1i = (uint32_t)((cv >> 21) & kPackMask21);
      nc[f] |= (rl > 0u && rr > 0u);
      bool ok = ((nz[f] >> i) & 1u) && (lane * 4 + i) != 255 && rl >= mslu && rr >= mslu;
      if (mwl) {
        const double l0 = (double)l0i * cw0, l1 = (double)l1i * cw1;
        ok = ok && !side_too_light(s, l0 + l1, (t0 - l0) + (t1 - l1));
      }
      const float a0 = (float)l0i * cw0f, a1 = (float)l1i * cw1f;
      const float r0 = (float)(t0i[f] - l0i) * cw0f, r1 = (float)(t1i[f] - l1i) * cw1f;
      const float wl = a0 + a1, wr = r0 + r1;
      const float num = (a0 * a0 + a1 * a1) * wr + (r0 * r0 + r1 * r1) * wl;
      q[f][i] = ok ? num * __builtin_amdgcn_rcpf(wl * wr) : -INFINITY;
      qm[f] = fmaxf(qm[f], q[f][i]);
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) qm[f] = wave::max_f32(qm[f], lane);
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const float thr = qm[f] - qm[f] * 0x1p-14f;
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) m |= (q[f][i] >= thr && q[f][i] != -INFINITY) ? (1u << i) : 0u;
    const double t0 = (double)t0i[f] * cw0, t1 = (double)t1i[f] * cw1;
    double best = -INFINITY;
    int bb = -1;
    while (__ballot(m != 0u) != 0ull) {
      if (m != 0u) {
        const int i = __builtin_ctz(m);
        m &= m - 1u;
        const uint64_t cv = i == 0 ? v[f][0] : i == 1 ? v[f][1] : i == 2 ? v[f][2] : v[f][3];
        const double l0 = (double)(cv & kPackMask21) * cw0, l1 = (double)((cv >> 21) & kPackMask21) * cw1;
        ClsAcc L, R;
        L.init(kGini); R.init(kGini);
        L.add(l0); L.add(l1);
        R.add(t0 - l0); R.add(t1 - l1);
        const double g = cls_proxy(L, R, kGini);
        if (g > best) { best = g; bb = lane * 4 + i; }
      }
    }
    const uint64_t cm = __ballot(bb >= 0);
    if (__popcll(cm) == 1) {
      const int src = (int)__builtin_ctzll(cm);
      best = wave::bcast<double>(best, src);
      bb = wave::bcast<int>(bb, src);
    } else {
      wave::argmax(best, bb, lane);
    }
    const bool any_nc = __ballot(nc[f]) != 0ull;
    const int src = bb >= 0 ? (bb >> 2) : 0, sel = bb >= 0 ? (bb & 3) : 0;
    const uint64_t mine = sel == 0 ? v[f][0] : sel == 1 ? v[f][1] : sel == 2 ? v[f][2] : v[f][3];
    const uint64_t cv = wave::bcast<uint64_t>(mine, src);
    if (lane == 0) {
      double* ol = out_left + f * FS * CH;
      ol[0] = bb >= 0 ? (double)(cv & kPackMask21) * cw0 : 0.0;
      ol[1] = bb >= 0 ? (double)((cv >> 21) & kPackMask21) * cw1 : 0.0;
      ol[2] = bb >= 0 ? (double)(cv >> 42) : 0.0;
      out_gain[f * FS] = best; out_bin[f * FS] = bb; out_nc[f * FS] = any_nc ? 1 : 0;
    }
  }
}

// ONE wave evaluates one feature's histogram.  Binary (MODE 1) and regression (MODE 2)
// histograms are read ONCE into registers (4 bins per lane), scanned with DPP, scored and
// arg-maxed without writing the scan back to LDS; the histogram is cleared by the same
// lanes right after the read.  Multiclass (MODE 0) keeps the LDS path (C+1 planes).
// RP: regression planes present (3, or 2 without the y^2 plane: out_left[2] is then 0)
template <int MODE, int RP = 3>
__device__ DML_EVAL_ATTR void eval_feature(typename HT<MODE>::T* h, int C, int CH, const NodeSpec& s, int lane,
                             double* out_gain, int* out_bin, int* out_nc, double* out_left, bool zero_after,
                             const double* cw = nullptr, const RegScale* rq = nullptr, MonoQ mq = MonoQ{0, 0.0, 0.0},
                             double* out_mid = nullptr) {
  if constexpr (MODE == 0) {
    eval_feature_lds<MODE>(h, C, CH, s, lane, out_gain, out_bin, out_nc, out_left, zero_after, cw, mq, out_mid);
  } else {
    using CT = typename HT<MODE>::T;
    if constexpr (MODE == 1) {
      if (mq.m == 0 && gini_pf_ok(s, cwk(cw, 0), cwk(cw, 1))) {
        eval_gini_pf<1, 1>(h, 256, s, lane, out_gain, out_bin, out_nc, out_left, CH, zero_after, cwk(cw, 0), cwk(cw, 1));
        if (out_mid && lane == 0) *out_mid = 0.0;
        return;
      }
    }
    constexpr int NP = MODE == 1 ? 1 : RP;     // planes: packed u64 | (w | rows << 32, w yq[, w y2q]) integers
    CT v[NP][4];
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) v[q][i] = h[q * 256 + 4 * lane + i];
    if (zero_after) {
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) h[q * 256 + 4 * lane + i] = (CT)0;
    }
    // in-lane prefix + wave exclusive offset -> cumulative value of bin 4*lane+i
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      v[q][1] += v[q][0]; v[q][2] += v[q][1]; v[q][3] += v[q][2];
      CT t;
      if constexpr (sizeof(CT) == 8) t = (CT)wave::incl_scan_u64((uint64_t)v[q][3]);
      else t = wave::incl_scan<CT>(v[q][3]);
      const CT ex = wave::excl_from_incl<CT>(t);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[q][i] += ex;
    }
    CT tot[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) tot[q] = wave::bcast<CT>(v[q][3], 63);
    const double msl = (double)s.min_samples_leaf;
    const double cw0 = cwk(cw, 0), cw1 = cwk(cw, 1);
    double best = -INFINITY, bmid = 0.0;
    int bb = -1;
    bool nc = false;
    double tot_rows;
    if constexpr (MODE == 1) tot_rows = (double)((uint64_t)tot[0] >> 42);
    else tot_rows = reg_rows(tot[0]);
    // binary Gini: fp32 pre-filter.  Every candidate bin is scored in fp32 (relative error
    // < 2^-19: all terms are sums and products of non-negative values), and only the bins
    // within 2^-14 of the wave's fp32 maximum -- a set that provably holds every bin whose
    // fp64 score equals the fp64 maximum -- are re-scored in fp64 with the exact formula of
    // the generic path below.  The split chosen is therefore the one the full fp64 sweep
    // (and the host builder) chooses, at ~1 fp64 score per lane instead of 4.
    bool pf = false;
    if constexpr (MODE == 1 && DML_GINI_PF)
      pf = s.criterion == kGini && mq.m == 0 && cw0 >= 0x1p-20 && cw0 <= 0x1p20 && cw1 >= 0x1p-20 && cw1 <= 0x1p20;
    if (MODE == 1 && pf) {
      const uint64_t tv = (uint64_t)tot[0];
      const uint32_t trows = (uint32_t)(tv >> 42), t0i = (uint32_t)(tv & kPackMask21),
                     t1i = (uint32_t)((tv >> 21) & kPackMask21);
      const uint32_t mslu = (uint32_t)s.min_samples_leaf;
      const float cw0f = (float)cw0, cw1f = (float)cw1;
      const double t0 = (double)t0i * cw0, t1 = (double)t1i * cw1;
      const bool mwl = s.min_weight_leaf > 0.0;
      float q[4];
      float qmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t cv = (uint64_t)v[0][i];
        const uint32_t rl = (uint32_t)(cv >> 42), rr = trows - rl;
        const uint32_t l0i = (uint32_t)(cv & kPackMask21), l1i = (uint32_t)((cv >> 21) & kPackMask21);
        nc |= (rl > 0u && rr > 0u);
        bool ok = (lane * 4 + i) != 255 && rl >= mslu && rr >= mslu;
        if (mwl) {   // the generic path's side weights, same doubles
          const double l0 = (double)l0i * cw0, l1 = (double)l1i * cw1;
          ok = ok && !side_too_light(s, l0 + l1, (t0 - l0) + (t1 - l1));
        }
        const float a0 = (float)l0i * cw0f, a1 = (float)l1i * cw1f;
        const float r0 = (float)(t0i - l0i) * cw0f, r1 = (float)(t1i - l1i) * cw1f;
        const float wl = a0 + a1, wr = r0 + r1;
        const float num = (a0 * a0 + a1 * a1) * wr + (r0 * r0 + r1 * r1) * wl;
        q[i] = ok ? num * __builtin_amdgcn_rcpf(wl * wr) : -INFINITY;
        qmax = fmaxf(qmax, q[i]);
      }
      qmax = wave::max_f32(qmax, lane);
      const float thr = qmax - qmax * 0x1p-14f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!(q[i] >= thr) || q[i] == -INFINITY) continue;
        const uint64_t cv = (uint64_t)v[0][i];
        const double l0 = (double)(cv & kPackMask21) * cw0, l1 = (double)((cv >> 21) & kPackMask21) * cw1;
        ClsAcc L, R;
        L.init(s.criterion); R.init(s.criterion);
        L.add(l0); L.add(l1);
        R.add(t0 - l0); R.add(t1 - l1);
        const double g = cls_proxy(L, R, s.criterion);
        if (g > best) { best = g; bb = lane * 4 + i; }
      }
    } else
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = lane * 4 + i;
      double rl;
      if constexpr (MODE == 1) rl = (double)((uint64_t)v[0][i] >> 42);
      else rl = reg_rows(v[0][i]);
      const double rr = tot_rows - rl;
      if (b == 255) continue;
      nc |= (rl > 0.0 && rr > 0.0);
      if (rl < msl || rr < msl) continue;
      double g, mid = 0.0;
      if constexpr (MODE == 1) {
        const uint64_t cv = (uint64_t)v[0][i], tv = (uint64_t)tot[0];
        const double l0 = (double)(cv & kPackMask21) * cw0, l1 = (double)((cv >> 21) & kPackMask21) * cw1;
        const double t0 = (double)(tv & kPackMask21) * cw0, t1 = (double)((tv >> 21) & kPackMask21) * cw1;
        ClsAcc L, R;
        L.init(s.criterion); R.init(s.criterion);
        L.add(l0); L.add(l1);
        R.add(t0 - l0); R.add(t1 - l1);
        if (side_too_light(s, L.w, R.w)) continue;
        if (mq.m) {   // monotonic_cst on the class-0 fraction (forest_cpu.cpp)
          if (!mono_ok(mq.m, mq.lo, mq.hi, side_value(L.w, l0), side_value(R.w, t0 - l0))) continue;
          mid = mono_mid(L.w, l0, R.w, t0 - l0);
        }
        g = cls_proxy(L, R, s.criterion);
      } else {   // the host builder's formula (forest_cpu.cpp), on the same integers
        const double l0 = reg_w(v[0][i]), t0 = reg_w(tot[0]), l1 = reg_s1(v[1][i], *rq), t1 = reg_s1(tot[1], *rq);
        if (side_too_light(s, l0, t0 - l0)) continue;
        if (mq.m) {
          if (!mono_ok(mq.m, mq.lo, mq.hi, side_value(l0, l1), side_value(t0 - l0, t1 - l1))) continue;
          mid = mono_mid(l0, l1, t0 - l0, t1 - l1);
        }
        g = reg_proxy(s.criterion, l0, l1, t0 - l0, t1 - l1);
      }
      if (g > best) { best = g; bb = b; bmid = mid; }
    }
    {
      // one lane holding a candidate (the usual outcome of the fp32 pre-filter): its pair
      // is the wave's argmax, no reduction needed
      const uint64_t cm = __ballot(bb >= 0);
      if (__popcll(cm) == 1) {
        const int src = (int)__builtin_ctzll(cm);
        best = wave::bcast<double>(best, src);
        bb = wave::bcast<int>(bb, src);
      } else {
        wave::argmax(best, bb, lane);
      }
    }
    const bool any_nc = __ballot(nc) != 0ull;
    // the winning bin's cumulative channels, broadcast from its owner lane
    const int src = bb >= 0 ? (bb >> 2) : 0, sel = bb >= 0 ? (bb & 3) : 0;
    if constexpr (MODE == 1) {
      uint64_t mine = (uint64_t)v[0][0];
#pragma unroll
      for (int i = 1; i < 4; ++i) if (sel == i) mine = (uint64_t)v[0][i];
      const uint64_t cv = wave::bcast<uint64_t>(mine, src);
      if (lane == 0) {
        out_left[0] = bb >= 0 ? (double)(cv & kPackMask21) * cw0 : 0.0;
        out_left[1] = bb >= 0 ? (double)((cv >> 21) & kPackMask21) * cw1 : 0.0;
        out_left[2] = bb >= 0 ? (double)(cv >> 42) : 0.0;
      }
    } else {
      uint64_t mine[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        mine[q] = v[q][0];
#pragma unroll
        for (int i = 1; i < 4; ++i) if (sel == i) mine[q] = v[q][i];
      }
      uint64_t cq[3] = {0ull, 0ull, 0ull};
#pragma unroll
      for (int q = 0; q < NP; ++q) cq[q] = wave::bcast<uint64_t>(mine[q], src);
      if (lane == 0) {   // channels {w, w y, w y^2, rows}
        out_left[0] = bb >= 0 ? reg_w(cq[0]) : 0.0;
        out_left[1] = bb >= 0 ? reg_s1(cq[1], *rq) : 0.0;
        out_left[2] = (bb >= 0 && NP == 3) ? reg_s2(cq[2], *rq) : 0.0;
        out_left[3] = bb >= 0 ? reg_rows(cq[0]) : 0.0;
      }
    }
    if (out_mid) {   // the winning bin's middle value, from its owner lane
      const double m = wave::bcast<double>(bmid, bb >= 0 ? (bb >> 2) : 0);
      if (lane == 0) *out_mid = m;
    }
    if (lane == 0) { *out_gain = best; *out_bin = bb; *out_nc = any_nc ? 1 : 0; }
  }
}

template <int MODE>
__device__ DML_EVAL_ATTR void eval_feature_lds(typename HT<MODE>::T* h, int C, int CH, const NodeSpec& s, int lane,
                                 double* out_gain, int* out_bin, int* out_nc, double* out_left, bool zero_after,
                                 const double* cw, MonoQ mq, double* out_mid) {
  using CT = typename HT<MODE>::T;
  static_assert(MODE == 0, "binary and regression histograms are evaluated in registers (eval_feature)");
  const int planes = hist_planes(MODE, CH);
  for (int ch = 0; ch < planes; ++ch) scan256<CT>(h + ch * 256, lane);
  wave_lds_sync();
  const double tot_rows = hist_chan<MODE>(h, CH - 1, CH, 255);
  const double msl = (double)s.min_samples_leaf;
  double best = -INFINITY, bmid = 0.0;
  int bb = -1;
  bool nc = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = lane * 4 + i;
    if (b == 255) break;
    const double rl = hist_chan<MODE>(h, CH - 1, CH, b);
    const double rr = tot_rows - rl;
    nc |= (rl > 0.0 && rr > 0.0);
    if (rl < msl || rr < msl) continue;
    double g, mid = 0.0;
    {
      ClsAcc L, R;
      L.init(s.criterion); R.init(s.criterion);
      double l0 = 0.0, t0 = 0.0;
      for (int k = 0; k < C; ++k) {
        const double lc = hist_chan<MODE>(h, k, CH, b) * cwk(cw, k);
        const double tc = hist_chan<MODE>(h, k, CH, 255) * cwk(cw, k);
        if (k == 0) { l0 = lc; t0 = tc; }
        L.add(lc);
        R.add(tc - lc);
      }
      if (side_too_light(s, L.w, R.w)) continue;
      if (mq.m) {   // binary monotonic_cst (class-0 fraction)
        if (!mono_ok(mq.m, mq.lo, mq.hi, side_value(L.w, l0), side_value(R.w, t0 - l0))) continue;
        mid = mono_mid(L.w, l0, R.w, t0 - l0);
      }
      g = cls_proxy(L, R, s.criterion);
    }
    if (g > best) { best = g; bb = b; bmid = mid; }
  }
  wave::argmax(best, bb, lane);
  if (out_mid) {
    const double m = wave::bcast<double>(bmid, bb >= 0 ? (bb >> 2) : 0);
    if (lane == 0) *out_mid = m;
  }
  const bool any_nc = __ballot(nc) != 0ull;
  if (lane < CH) out_left[lane] = bb >= 0 ? hist_chan<MODE>(h, lane, CH, bb) * (lane < C ? cwk(cw, lane) : 1.0) : 0.0;
  if (lane == 0) { *out_gain = best; *out_bin = bb; *out_nc = any_nc ? 1 : 0; }
  if (zero_after) {
    wave_lds_sync();
    for (int ch = 0; ch < planes; ++ch) {
      CT* p = h + ch * 256 + 4 * lane;
      p[0] = (CT)0; p[1] = (CT)0; p[2] = (CT)0; p[3] = (CT)0;
    }
  }
}

template <int MODE, int RP = 3>
__device__ __forceinline__ void hist_add_row(typename HT<MODE>::T* hist, const Ctx& c, const float* ty,
                                             const int16_t* feats, int g, uint32_t row, uint32_t w, int span) {
  const uint8_t* xr = c.Xb + (int64_t)row * c.ld;
  if constexpr (MODE == 0) {
    const int y = c.ycls[row];
    for (int j = 0; j < g; ++j) {
      const int b = xr[feats[j]];
      uint32_t* hj = hist + j * span;
      atomicAdd(&hj[y * 256 + b], w);
      atomicAdd(&hj[c.C * 256 + b], 1u);
    }
  } else if constexpr (MODE == 1) {
    const unsigned long long pv = pack_bin(c.ycls[row], w);
    for (int j = 0; j < g; ++j) atomicAdd(&hist[j * span + xr[feats[j]]], pv);
  } else {
    const RegPL p = reg_payload(c, w, ty[row]);
    for (int j = 0; j < g; ++j) {
      const int b = xr[feats[j]];
      unsigned long long* hj = hist + j * span;
      atomicAdd(&hj[b], p.wr);
      atomicAdd(&hj[256 + b], p.wy);
      if (RP == 3) atomicAdd(&hj[512 + b], p.wyy);
    }
  }
}

// serial selection over an evaluated group, in visiting order (thread 0)
__device__ void select_group(const Ctx& c, const NodeSpec& s, const int16_t* feats, int g, const double* rg,
                             const int* rb, const int* rn, const double* rleft, double* best_left, int& nonconst,
                             double& best_gain, int& best_feat, int& best_bin, int& upd_j) {
  upd_j = -1;
  for (int j = 0; j < g; ++j) {
    if (!rn[j]) continue;
    ++nonconst;
    if (rb[j] >= 0 && rg[j] > best_gain) {
      best_gain = rg[j];
      best_feat = feats[j];
      best_bin = rb[j];
      upd_j = j;
      for (int ch = 0; ch < c.CH; ++ch) best_left[ch] = rleft[j * c.CH + ch];
    }
    if (nonconst >= s.max_features) break;
  }
}

// final split decision given the best candidate; returns true if node splits
__device__ bool accept_split(const Ctx& c, const NodeSpec& s, int node, int tree, const double* best_left) {
  const double* pv = c.node_val + (int64_t)node * c.VC;
  const double Wt = c.tree_W[tree];
  double impN, impL, impR, wN, wL, wR;
  if (c.is_reg) {
    wN = pv[0]; wL = best_left[0]; wR = pv[0] - best_left[0];
    impN = mse_impurity(pv[0], pv[1], pv[2]);
    impL = mse_impurity(best_left[0], best_left[1], best_left[2]);
    impR = mse_impurity(pv[0] - best_left[0], pv[1] - best_left[1], pv[2] - best_left[2]);
  } else {
    ClsAcc N, L, R;
    N.init(s.criterion); L.init(s.criterion); R.init(s.criterion);
    for (int k = 0; k < c.C; ++k) { N.add(pv[k]); L.add(best_left[k]); R.add(pv[k] - best_left[k]); }
    wN = N.w; wL = L.w; wR = R.w;
    impN = cls_impurity(N, s.criterion); impL = cls_impurity(L, s.criterion); impR = cls_impurity(R, s.criterion);
  }
  const double imp = accept_improvement(s, c.is_reg != 0, pv, best_left, Wt, wN, impN, wL, impL, wR, impR);
  return !(imp + kEps < (double)s.min_impurity_decrease);
}

// scratch block of the fused kernel
struct Scratch {
  uint64_t last;
  double best_gain;
  double W;                 // tree weight (prefetched)
  int32_t best_feat, best_bin, nonconst, pos, first, base, nl, best_j;
  int32_t best_pos;         // visiting position of the best split's feature
  int32_t scr_n;            // streamed nodes: positions [0, scr_n) have their bins in Ctx::bscr
  int32_t wcnt[32];         // partition: [2][RPT][NW] per-wave counts
  double best_mid;          // monotonic_cst: middle value of the best split
  double lo, hi;            // monotonic_cst: this node's bounds
};

struct FusedLayout {
  size_t hist, feats, rg, rb, rn, rleft, rmid, best_left, pvs, rvs, sc, total;
};

__host__ __device__ inline FusedLayout fused_layout(int KG, int span, int elem, int CH) {
  FusedLayout L;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = (off + bytes + 15) / 16 * 16; return o; };
  L.hist = take((size_t)KG * span * elem);
  L.feats = take((size_t)KG * 2);
  L.rg = take((size_t)KG * 8);
  L.rb = take((size_t)KG * 4);
  L.rn = take((size_t)KG * 4);
  L.rleft = take((size_t)KG * CH * 8);
  L.rmid = take((size_t)KG * 8);
  L.best_left = take((size_t)CH * 8);
  L.pvs = take((size_t)CH * 8);
  L.rvs = take((size_t)CH * 8);
  L.sc = take(sizeof(Scratch));
  L.total = off;
  return L;
}

// ------------------------------------------------------------------------------------
// fused per-node kernel (wave tier NT=64, block tier NT=256)
// ------------------------------------------------------------------------------------
// accept_split / make_children / enqueue on values already held on-chip (LDS): the
// parent's channel sums and the tree weight are prefetched at kernel start, so the
// decision makes no dependent global round trips.
__device__ __forceinline__ bool accept_split_v(const Ctx& c, const NodeSpec& s, const double* pv, double Wt, const double* best_left) {
  // classification with min_impurity_decrease <= 0: the test cannot reject. The impurity
  // decrease of a Gini / entropy split is >= 0 (concave impurities) and every term of the
  // computed value is <= log2(64) in magnitude, so its rounding error is ~1e-14, far inside
  // kEps: the host builder, which evaluates the test, accepts every such split too
  if (!c.is_reg && s.min_impurity_decrease <= 0.0f) return true;
  double impN, impL, impR, wN, wL, wR;
  if (c.is_reg) {
    wN = pv[0]; wL = best_left[0]; wR = pv[0] - best_left[0];
    impN = mse_impurity(pv[0], pv[1], pv[2]);
    impL = mse_impurity(best_left[0], best_left[1], best_left[2]);
    impR = mse_impurity(pv[0] - best_left[0], pv[1] - best_left[1], pv[2] - best_left[2]);
  } else {
    ClsAcc N, L, R;
    N.init(s.criterion); L.init(s.criterion); R.init(s.criterion);
    for (int k = 0; k < c.C; ++k) { N.add(pv[k]); L.add(best_left[k]); R.add(pv[k] - best_left[k]); }
    wN = N.w; wL = L.w; wR = R.w;
    impN = cls_impurity(N, s.criterion); impL = cls_impurity(L, s.criterion); impR = cls_impurity(R, s.criterion);
  }
  const double imp = accept_improvement(s, c.is_reg != 0, pv, best_left, Wt, wN, impN, wL, impL, wR, impR);
  return !(imp + kEps < (double)s.min_impurity_decrease);
}

// "impurity > kEps" of a child's value vector; a Gini-specialised binary build decides it on
// the integer class weights (pure <=> a class is absent: a mixed node of total weight W < 2e7
// has Gini >= 2 (W - 1) / W^2 > kEps, and a pure one computes exactly 0)
template <int FC>
__device__ __forceinline__ bool impure_v(const Ctx& c, const NodeSpec& s, const double* v);

__device__ __forceinline__ double impurity_of_vals(const Ctx& c, const double* v, int crit) {
  if (c.is_reg) return mse_impurity(v[0], v[1], v[2]);
  ClsAcc a;
  a.init(crit);
  for (int k = 0; k < c.C; ++k) a.add(v[k]);
  return cls_impurity(a, crit);
}

template <int FC>
__device__ __forceinline__ bool impure_v(const Ctx& c, const NodeSpec& s, const double* v) {
  if constexpr (FC == kGini)
    if (c.C == 2) return v[0] > 0.0 && v[1] > 0.0;
  if (c.is_reg) return !reg_pure(v, c.rq);
  return impurity_of_vals(c, v, s.criterion) > kEps;
}

// a wave/block-tier child into its staging slot (k_compact enqueues it): tier -1 = leaf
template <int FC>
__device__ __forceinline__ void stage_child(const Ctx& c, const NodeSpec& s, int tree, int node, int64_t start, int count, int depth,
                            uint64_t key, int64_t slot, const double* vals) {
  int tier = -1;
  if (!leaf_by_counts(s, count, depth) && !leaf_by_weight(s, vals_weight(vals, c.C, c.is_reg)) &&
      impure_v<FC>(c, s, vals))
    tier = tier_of(c, count);
  OpenNode on;
  on.tree = tree; on.node = node; on.start = start; on.count = count; on.depth = depth;
  on.key = key; on.pool_base = -1; on.tier = tier;
  c.stage[slot] = on;
}

// histogram payload of one row (PLT above)
template <int MODE>
__device__ __forceinline__ typename PLT<MODE>::T row_payload(const Ctx& c, const float* ty, uint32_t row, uint32_t w) {
  if constexpr (MODE == 0) return (uint64_t)(uint32_t)c.ycls[row] | ((uint64_t)w << 32);
  else if constexpr (MODE == 1) return pack_bin(c.ycls[row], w);
  else return reg_payload(c, w, ty[row]);
}

template <int MODE, bool PK = false>
__device__ __forceinline__ typename PLT<MODE>::T word_payload(const Ctx& c, const NodeSpec& s, const float* ty,
                                                              uint32_t wd) {
  if (!PK && !c.packed) return row_payload<MODE>(c, ty, wd, boot_weight(s, wd));
  const uint32_t w = (wd >> c.rbits) & 15u;
  if constexpr (MODE == 0) return (uint64_t)(wd >> (c.rbits + 4)) | ((uint64_t)w << 32);
  else if constexpr (MODE == 1) return pack_bin((int)(wd >> (c.rbits + 4)), w);
  else return reg_payload(c, w, ty[wd & c.rmask]);
}

// Pipelined payloads, in two halves.  payload_fetch issues the row's payload LOAD (regression:
// its target) unconditionally -- an absent row (0xFFFFFFFF) reads row 0 -- right after the step's
// bin gathers; payload_finish turns it into the payload when the step is consumed.  The old
// single-step `valid ? word_payload(...) : PL{}` put that load under an exec mask and used its
// value at once: the compiler then waited with vmcnt(0), i.e. for the NEXT step's bin gathers
// too, which drained the software pipeline every half-iteration (k_hist_large<2> ISA: one
// vmcnt(0) per step; 75 % of its wave cycles waiting, profiles/r4_gbrt_hist_large_pmc.txt).
// Classification payloads live in the packed row word (no load); the unpacked fallback keeps
// word_payload's own loads.
struct PRaw {
  uint32_t wd;
  float y;
};

template <int MODE, bool PK = false>
__device__ __forceinline__ PRaw payload_fetch(const Ctx& c, const float* ty, uint32_t wd) {
  PRaw r;
  r.wd = wd;
  r.y = 0.0f;
  if constexpr (MODE == 2) r.y = ty[(wd != 0xFFFFFFFFu ? wd : 0u) & c.rmask];
  return r;
}

template <int MODE, bool PK = false>
__device__ __forceinline__ typename PLT<MODE>::T payload_finish(const Ctx& c, const NodeSpec& s, const float* ty,
                                                                const PRaw& r) {
  if constexpr (MODE == 2) {
    const uint32_t w = (PK || c.packed) ? (r.wd >> c.rbits) & 15u : boot_weight(s, r.wd);
    return reg_payload(c, w, r.y);
  } else {
    return word_payload<MODE, PK>(c, s, ty, r.wd);
  }
}

// large-tier regression, unit row weights: u32 row count in the slice's first KB + the w yq plane
// (wo: the w yq plane's offset in the slice -- 256, or 128 in the compact 3-KB slices)
template <int MODE>
__device__ __forceinline__ void hist_add_unit(typename HT<MODE>::T* hj, int b, const typename PLT<MODE>::T& pl,
                                              int wo) {
  if constexpr (MODE == 2) {
    atomicAdd((uint32_t*)hj + b, 1u);
    atomicAdd(&hj[wo + b], pl.wy);
  }
}

// packed LDS words of a large_pack build: one u64 atomic per (row, feature) carries the row
// count (bits 52..63, <= 4095 rows per workgroup) and the biased w yq (yq + 2^39 > 0, so the
// 52-bit field never borrows from the count; its sum over <= 4095 rows stays below 2^52)
constexpr int kPackShift = 52;
constexpr unsigned long long kPackBias = 1ull << 39;
template <int MODE>
__device__ __forceinline__ void hist_add_packed(typename HT<MODE>::T* hj, int b, const typename PLT<MODE>::T& pl,
                                                int wo) {
  if constexpr (MODE == 2) atomicAdd(&hj[wo + b], (1ull << kPackShift) + ((unsigned long long)pl.wy + kPackBias));
}
// a packed word -> (row count, w yq) in the two's-complement u64 of the regression planes
__device__ __forceinline__ uint32_t pack_count(unsigned long long v) { return (uint32_t)(v >> kPackShift); }
__device__ __forceinline__ unsigned long long pack_wy(unsigned long long v) {
  return (v & ((1ull << kPackShift) - 1)) - ((v >> kPackShift) << 39);
}

// the same with the count plane supplied elsewhere (boosting roots: ForestArgs::root_counts)
template <int MODE>
__device__ __forceinline__ void hist_add_wy(typename HT<MODE>::T* hj, int b, const typename PLT<MODE>::T& pl,
                                            int wo) {
  if constexpr (MODE == 2) atomicAdd(&hj[wo + b], pl.wy);
}

template <int MODE, int RP = 3>
__device__ __forceinline__ void hist_add(typename HT<MODE>::T* hj, const Ctx& c, int b, const typename PLT<MODE>::T& pl) {
#ifdef DML_X2_ATOMIC   // sensitivity build: every histogram atomic issued twice (the second adds 0)
  if constexpr (MODE == 1) atomicAdd(&hj[b], (unsigned long long)(pl * (uint64_t)((uint32_t)c.n >> 31)));
#endif
  if constexpr (MODE == 2) {
    atomicAdd(&hj[b], pl.wr);
    atomicAdd(&hj[256 + b], pl.wy);
    if (RP == 3) atomicAdd(&hj[512 + b], pl.wyy);
    return;
  }
  if constexpr (MODE == 0) {
    atomicAdd(&hj[(int)(uint32_t)pl * 256 + b], (uint32_t)(pl >> 32));
    atomicAdd(&hj[c.C * 256 + b], 1u);
  } else if constexpr (MODE == 1) {
    atomicAdd(&hj[b], (unsigned long long)pl);
  }
}

template <int NT, int MODE, int FC>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MODE == 2 ? DML_NODES_WPE_REG : (MODE == 0 ? DML_NODES_WPE_MC : (NT == 64 ? DML_NODES_WPE_WAVE : DML_NODES_WPE)), (MODE == 1 && NT == 64) ? DML_NODES_WPE_WAVE_MAX : 8))) void k_nodes(Ctx c, int tier, int set_cur,
                                                                                                   int pair_base, int stage_base) {
  using CT = typename HT<MODE>::T;
  constexpr bool PK = FC >= 0;   // specialised builds have packed row words
  constexpr int NW = NT / 64;
  constexpr int RPT = NT == 64 ? 4 : DML_RPT_BLOCK;   // rows per thread in registers (<= 4: packed u8 x 4)
  static_assert(RPT >= 1 && RPT <= 4, "RPT");
  static_assert(2 * RPT * (NT / 64) <= 32, "Scratch::wcnt too small for this NT x RPT");
  constexpr int KGMAX = NT == 64 ? DML_KGMAX_WAVE : DML_KGMAX_BLOCK;   // feature-group bound (register-resident bins)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  PH_BEGIN
  const OpenNode on = c.open[set_cur][tier][blockIdx.x];
  const NodeSpec s = spec_of<FC>(c, on.tree);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int d = c.d;
  const int KG = min(NT == 64 ? c.kg_wave : c.kg_block, KGMAX);
  const int slack = NT == 64 ? c.slack_wave : 0;
  const int span = hist_planes(MODE, c.CH) * 256;
  const FusedLayout FL = fused_layout(KG, span, (int)sizeof(CT), c.CH);
  CT* hist = (CT*)(smem + FL.hist);
  int16_t* feats = (int16_t*)(smem + FL.feats);
  double* rg = (double*)(smem + FL.rg);
  int* rb = (int*)(smem + FL.rb);
  int* rn = (int*)(smem + FL.rn);
  double* rleft = (double*)(smem + FL.rleft);
  double* rmid = (double*)(smem + FL.rmid);     // monotonic_cst: each feature's best middle value
  double* best_left = (double*)(smem + FL.best_left);
  double* pvs = (double*)(smem + FL.pvs);       // parent channel sums
  double* rvs = (double*)(smem + FL.rvs);       // right child channel sums
  Scratch* sc = (Scratch*)(smem + FL.sc);

  for (int i = tid; i < KG * span; i += NT) hist[i] = (CT)0;
  if (tid < c.VC) pvs[tid] = c.node_val[(int64_t)on.node * c.VC + tid];
  if (tid == 0) {
    sc->best_gain = -INFINITY; sc->best_feat = -1; sc->best_bin = -1;
    sc->nonconst = 0; sc->pos = 0; sc->first = 1; sc->last = 0; sc->best_j = -1;
    sc->best_pos = 1 << 30; sc->scr_n = 0;
    sc->W = c.tree_W[on.tree];
    sc->best_mid = 0.0;
    sc->lo = (FC < 0 && c.nbound) ? c.nbound[2 * (int64_t)on.node] : -INFINITY;
    sc->hi = (FC < 0 && c.nbound) ? c.nbound[2 * (int64_t)on.node + 1] : INFINITY;
  }
  const FeatPerm fp = feat_perm(on.key, d);   // node's feature visiting order (forest_common.h)
  const uint32_t* rows = c.rows_cur + on.start;
  const float* ty = tree_y(c, s);
  const int cnt = on.count;
  // rows (+ bootstrap weight + label payload) of a <= NT*RPT-row node stay in registers
  // for every feature group and the partition; larger nodes stream in NT*RPT chunks.
  // (block tier, DML_BLOCK_STREAM_ONLY: nodes there have > wave_max >= NT rows, so the
  // register-rows paths are compiled out of it -- their registers no longer bound its occupancy)
  const bool reg_rows = (NT > 64 && DML_BLOCK_STREAM_ONLY) ? false : cnt <= NT * RPT;
  uint32_t rrow[RPT], rbin[RPT];
  using PL = typename PLT<MODE>::T;
  PL rpl[RPT];
  PRaw rpr[RPT];
  // row ids, then the payload loads (payload_fetch: unconditional, so they stay counted in
  // flight while the bin gathers issue), then the payloads once the gathers are out
  auto load_rows = [&](int base) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int r = base + tid + NT * u;
      rrow[u] = r < cnt ? rows[r] : 0xFFFFFFFFu;
    }
  };
  auto fetch_rows = [&]() {
#pragma unroll
    for (int u = 0; u < RPT; ++u) rpr[u] = payload_fetch<MODE, PK>(c, ty, rrow[u]);
  };
  auto finish_rows = [&]() {
#pragma unroll
    for (int u = 0; u < RPT; ++u)
      rpl[u] = rrow[u] != 0xFFFFFFFFu ? payload_finish<MODE, PK>(c, s, ty, rpr[u]) : PL{};
  };
  if (reg_rows) load_rows(0);
#pragma unroll
  for (int u = 0; u < RPT; ++u) rbin[u] = 0;
  __syncthreads();
  PH(0)
  if (reg_rows) fetch_rows();
  const int k = s.max_features;
  uint32_t pk[KGMAX];   // register rows: the group's bins packed 4 x u8 per feature (live across eval)
  // wave tier, register rows: the bins of the first KPRE visiting positions are gathered
  // ONCE, all in flight together, before the first feature group -- the later groups
  // (KG histograms at a time fit LDS) then start without another gather round trip
  constexpr int KPRE = (NT == 64 && RPT == 4) ? DML_WAVE_PREFETCH : 0;
  uint32_t pre[KPRE > 0 ? KPRE : 1];
  int npre = 0;
  if constexpr (KPRE > 0) {
    if (reg_rows) {
      npre = min(KPRE, min(k + slack, d));
      if (DML_ROW_WINDOWS && DML_WAVE_WIN_ROWS > 0 && npre >= 8 && d <= 112 && (c.ld & 15) == 0 && c.ld >= 112 &&
          (((uintptr_t)c.Xb) & 15) == 0) {
        // whole row lines (7 dwordx4 loads = 7 cache-line lookups per row instead of npre byte
        // gathers), DML_WAVE_WIN_ROWS rows' lines in flight at a time, each prefetched
        // position's byte picked out by a uniform register index
        typedef uint32_t v32u __attribute__((ext_vector_type(32)));
        int fdw[KPRE], fsh[KPRE];
#pragma unroll
        for (int q = 0; q < KPRE; ++q) {
          const int f = __builtin_amdgcn_readfirstlane(q < npre ? feature_at(fp, q, d) : 0);
          fdw[q] = f >> 2;
          fsh[q] = (f & 3) * 8;
          pre[q] = 0u;
        }
        constexpr int WR = DML_WAVE_WIN_ROWS > 0 ? DML_WAVE_WIN_ROWS : 1;
#pragma unroll
        for (int u0 = 0; u0 < RPT; u0 += WR) {
          v32u w[WR];
#pragma unroll
          for (int uu = 0; uu < WR; ++uu) {
            const uint32_t r = rrow[u0 + uu];
            const uint4* xr = (const uint4*)(c.Xb + (int64_t)(r != 0xFFFFFFFFu ? (r & c.rmask) : 0u) * c.ld);
#pragma unroll
            for (int k7 = 0; k7 < 7; ++k7) {
              const uint4 qv = xr[k7];
              w[uu][4 * k7] = qv.x; w[uu][4 * k7 + 1] = qv.y; w[uu][4 * k7 + 2] = qv.z; w[uu][4 * k7 + 3] = qv.w;
            }
          }
#pragma unroll
          for (int q = 0; q < KPRE; ++q)
            if (q < npre)
#pragma unroll
              for (int uu = 0; uu < WR; ++uu) pre[q] |= ((w[uu][fdw[q]] >> fsh[q]) & 0xFFu) << (8 * (u0 + uu));
        }
      } else {
      uint32_t raw[KPRE][RPT];
      // row lines of the lane's rows (an absent row reads row 0: every load is unconditional)
      const uint8_t* xr[RPT];
#pragma unroll
      for (int u = 0; u < RPT; ++u) xr[u] = c.Xb + (int64_t)(rrow[u] != 0xFFFFFFFFu ? (rrow[u] & c.rmask) : 0u) * c.ld;
#pragma unroll
      for (int q = 0; q < KPRE; ++q) {
        const int f = __builtin_amdgcn_readfirstlane(q < npre ? feature_at(fp, q, d) : 0);
#pragma unroll
        for (int u = 0; u < RPT; ++u) raw[q][u] = q < npre ? (uint32_t)xr[u][f] : 0u;
#ifdef DML_X2_GATHER   // sensitivity build: every bin gathered twice
#pragma unroll
      for (int u = 0; u < RPT; ++u)
        raw[q][u] |= (q < npre && rrow[u] != 0xFFFFFFFFu) ? (uint32_t)c.Xb[(int64_t)(rrow[u] & c.rmask) * c.ld + f + ((uint32_t)c.n >> 31)] : 0u;
#endif
      }
#pragma unroll
      for (int q = 0; q < KPRE; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int u = 0; u < RPT; ++u) v |= raw[q][u] << (8 * u);
        pre[q] = v;
      }
      }
    }
  }
  if (reg_rows) finish_rows();
  while (true) {
    // wave-uniform loop state in SGPRs: the per-group bounds (g) are then scalar branches, not
    // exec masks (a masked load merges into a phi whose copies force vmcnt(0) waits)
    const int pos = __builtin_amdgcn_readfirstlane(sc->pos), nonconst = __builtin_amdgcn_readfirstlane(sc->nonconst);
    if (nonconst >= k || pos >= d) break;
    const int g = min(KG, min(k - nonconst + slack, d - pos));
    if (tid < g) feats[tid] = (int16_t)feature_at(fp, pos + tid, d);   // one visiting position per lane
    __syncthreads();
    PH(1)
    if (KPRE > 0 && reg_rows && pos + g <= npre) {
      // prefetched group: histogram atomics straight from the packed register bins
#pragma unroll
      for (int q = 0; q < (KPRE > 0 ? KPRE : 1); ++q) {
        if (q >= pos && q < pos + g) {
          CT* hj = hist + (q - pos) * span;
#pragma unroll
          for (int u = 0; u < RPT; ++u)
            if (rrow[u] != 0xFFFFFFFFu) hist_add<MODE>(hj, c, (int)((pre[q] >> (8 * u)) & 0xFFu), rpl[u]);
        }
      }
    } else
    if (!reg_rows && RPT == 1) {
      // large node, one row per thread per NT-row chunk, software-pipelined over chunks with
      // two register sets (A: even chunks, B: odd chunks) that swap roles without copies: per
      // chunk, the row id two chunks ahead is loaded first, then the next chunk's bins are
      // gathered, then this chunk's histogram atomics run -- so waiting for this chunk's bins
      // never waits for the next chunk's (vmcnt retires in issue order, and a register copy of
      // a pending load would force exactly that wait)
      // Every load of a chunk is issued unconditionally and their number is a compile-time G = g:
      // with a conditional or variable count the compiler cannot count outstanding loads and
      // waits for all of them (vmcnt(0)), which would drain the next chunk's gathers too.
      constexpr uint32_t INV = 0xFFFFFFFFu;
      auto run = [&](auto Gc) {
        constexpr int G = decltype(Gc)::value;
        int fj[G];
#pragma unroll
        for (int j = 0; j < G; ++j) fj[j] = __builtin_amdgcn_readfirstlane((int)feats[j < g ? j : 0]);
        auto row_at = [&](int r) -> uint32_t {
          const uint32_t v = rows[min(r, cnt - 1)];
          return r < cnt ? v : INV;
        };
        auto gather = [&](uint32_t r, uint32_t* b) {
          const uint8_t* xr = c.Xb + (int64_t)(r != INV ? (r & c.rmask) : 0u) * c.ld;
#pragma unroll
          for (int j = 0; j < G; ++j) b[j] = (uint32_t)xr[fj[j]];
#ifdef DML_X2_GATHER
#pragma unroll
          for (int j = 0; j < G; ++j) b[j] |= (uint32_t)xr[fj[j] + ((uint32_t)c.n >> 31)];
#endif
        };
        auto consume = [&](int base, bool valid, const uint32_t* b, const PRaw& pr) {
          if (NT > 64 && pos == 0 && valid) {
            uint32_t w4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < G && j < 16; ++j) w4[j >> 2] |= (j < g ? b[j] & 0xFFu : 0u) << (8 * (j & 3));
            *(uint4*)(c.bscr + (on.start + base + tid) * 16) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
          }
          if (valid) {
            const PL pl = payload_finish<MODE, PK>(c, s, ty, pr);
#pragma unroll
            for (int j = 0; j < G; ++j)
              if (j < g) hist_add<MODE>(hist + j * span, c, (int)b[j], pl);
          }
        };
        uint32_t rA = row_at(tid), rB = row_at(NT + tid);
        uint32_t bA[G], bB[G];
        gather(rA, bA);
        PRaw pA = payload_fetch<MODE, PK>(c, ty, rA), pB;
        bool vA = rA != INV, vB = false;
        for (int base = 0; base < cnt; base += 2 * NT) {
          rA = row_at(base + 2 * NT + tid);       // chunk k+2's row id
          gather(rB, bB);                         // chunk k+1's bins
          pB = payload_fetch<MODE, PK>(c, ty, rB);
          vB = rB != INV;
          consume(base, vA, bA, pA);              // chunk k
          rB = row_at(base + 3 * NT + tid);       // chunk k+3's row id
          gather(rA, bA);                         // chunk k+2's bins
          pA = payload_fetch<MODE, PK>(c, ty, rA);
          vA = rA != INV;
          consume(base + NT, vB, bB, pB);         // chunk k+1
        }
      };
      // d <= 112 on 16-B aligned rows, first group of >= 8 features: the whole row line comes
      // in as 7 dwordx4 loads (7 cache-line lookups per row instead of g >= 8 byte gathers --
      // the gathers are lookup-bound, one line per CU clock) and each feature's byte is
      // picked out of the 28 loaded dwords by a uniform register index
      auto runw = [&](auto Gc) {
        constexpr int G = decltype(Gc)::value;
        typedef uint32_t v32u __attribute__((ext_vector_type(32)));
        int fdw[G], fsh[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int f = __builtin_amdgcn_readfirstlane((int)feats[j < g ? j : 0]);
          fdw[j] = f >> 2;
          fsh[j] = (f & 3) * 8;
        }
        auto row_at = [&](int r) -> uint32_t {
          const uint32_t v = rows[min(r, cnt - 1)];
          return r < cnt ? v : INV;
        };
        auto load_win = [&](uint32_t r, v32u& w) {
          const uint4* xr = (const uint4*)(c.Xb + (int64_t)(r != INV ? (r & c.rmask) : 0u) * c.ld);
#pragma unroll
          for (int k = 0; k < 7; ++k) {
            const uint4 q = xr[k];
            w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
          }
        };
        // the group's bins stay packed 4 x u8 per register between extract and consume (the
        // layout of the row's bscr slot): 2 x ceil(G/4) registers for the two chunks in flight
        // instead of 2 x G -- the block tier's occupancy is bounded by this loop's registers
        constexpr int NPK = (G + 3) / 4;
        auto extract = [&](const v32u& w, uint32_t* b) {
#pragma unroll
          for (int q = 0; q < NPK; ++q) b[q] = 0u;
#pragma unroll
          for (int j = 0; j < G; ++j) b[j >> 2] |= (j < g ? (w[fdw[j]] >> fsh[j]) & 0xFFu : 0u) << (8 * (j & 3));
        };
        auto consume = [&](int base, bool valid, const uint32_t* b, const PRaw& pr) {
          if (NT > 64 && pos == 0 && valid)
            *(uint4*)(c.bscr + (on.start + base + tid) * 16) =
                make_uint4(b[0], NPK > 1 ? b[NPK > 1 ? 1 : 0] : 0u, NPK > 2 ? b[NPK > 2 ? 2 : 0] : 0u,
                           NPK > 3 ? b[NPK > 3 ? 3 : 0] : 0u);
          if (valid) {
            const PL pl = payload_finish<MODE, PK>(c, s, ty, pr);
#pragma unroll
            for (int j = 0; j < G; ++j)
              if (j < g) hist_add<MODE>(hist + j * span, c, (int)((b[j >> 2] >> (8 * (j & 3))) & 0xFFu), pl);
          }
        };
        v32u win;
        uint32_t bA[NPK], bB[NPK];
        uint32_t rA = row_at(tid), rB = row_at(NT + tid);
        load_win(rA, win);
        PRaw pA = payload_fetch<MODE, PK>(c, ty, rA), pB;
        extract(win, bA);
        bool vA = rA != INV, vB = false;
        for (int base = 0; base < cnt; base += 2 * NT) {
          load_win(rB, win);                      // chunk k+1's row lines
          pB = payload_fetch<MODE, PK>(c, ty, rB);
          rA = row_at(base + 2 * NT + tid);       // chunk k+2's row id
          consume(base, vA, bA, pA);              // chunk k
          extract(win, bB);
          vB = rB != INV;
          load_win(rA, win);                      // chunk k+2's row lines
          pA = payload_fetch<MODE, PK>(c, ty, rA);
          rB = row_at(base + 3 * NT + tid);       // chunk k+3's row id
          consume(base + NT, vB, bB, pB);         // chunk k+1
          extract(win, bA);
          vA = rA != INV;
        }
      };
      if (DML_ROW_WINDOWS && NT > 64 && pos == 0 && g >= 8 && d <= 112 && (c.ld & 15) == 0 && c.ld >= 112 &&
          (((uintptr_t)c.Xb) & 15) == 0) {
        switch (g) {
          case 8: runw(std::integral_constant<int, (8 < KGMAX ? 8 : KGMAX)>{}); break;
          case 9: runw(std::integral_constant<int, (9 < KGMAX ? 9 : KGMAX)>{}); break;
          case 10: runw(std::integral_constant<int, (10 < KGMAX ? 10 : KGMAX)>{}); break;
          case 11: runw(std::integral_constant<int, (11 < KGMAX ? 11 : KGMAX)>{}); break;
          case 12: runw(std::integral_constant<int, (12 < KGMAX ? 12 : KGMAX)>{}); break;
          default: runw(std::integral_constant<int, KGMAX>{}); break;
        }
      } else
      // one instantiation per group size: an extra load per row is an extra cache-line lookup,
      // and the gathers are lookup-bound (one line per CU clock)
      switch (g) {
#define DML_G_CASE(N) case N: run(std::integral_constant<int, (N < KGMAX ? N : KGMAX)>{}); break;
        DML_G_CASE(1) DML_G_CASE(2) DML_G_CASE(3) DML_G_CASE(4) DML_G_CASE(5) DML_G_CASE(6) DML_G_CASE(7)
        DML_G_CASE(8) DML_G_CASE(9) DML_G_CASE(10) DML_G_CASE(11) DML_G_CASE(12) DML_G_CASE(13) DML_G_CASE(14)
        DML_G_CASE(15)
#undef DML_G_CASE
        default: run(std::integral_constant<int, KGMAX>{}); break;
      }
    } else
    for (int base = 0; base < cnt; base += NT * RPT) {
      if (!reg_rows) { load_rows(base); fetch_rows(); }
      // all g x RPT bin loads are issued before the first histogram atomic
      uint32_t bins[KGMAX][RPT];
#pragma unroll
      for (int j = 0; j < KGMAX; ++j) {
        if (j < g) {
          const int64_t f = feats[j];
#pragma unroll
          for (int u = 0; u < RPT; ++u)
            bins[j][u] = rrow[u] != 0xFFFFFFFFu ? (uint32_t)c.Xb[(int64_t)(rrow[u] & c.rmask) * c.ld + f] : 0u;
        }
      }
      if (!reg_rows) finish_rows();
#pragma unroll
      for (int j = 0; j < KGMAX; ++j) {
        if (j < g) {
          CT* hj = hist + j * span;
#pragma unroll
          for (int u = 0; u < RPT; ++u)
            if (rrow[u] != 0xFFFFFFFFu) hist_add<MODE>(hj, c, (int)bins[j][u], rpl[u]);
        }
      }
      if (NT > 64 && !reg_rows && pos == 0) {
        // streamed block-tier node, RPT rows per thread: the first group's bins (<= 16
        // visiting positions) into each row's scratch slot, as the one-row pipeline does
#pragma unroll
        for (int u = 0; u < RPT; ++u)
          if (rrow[u] != 0xFFFFFFFFu) {
            uint32_t w4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < KGMAX && j < 16; ++j)
              if (j < g) w4[j >> 2] |= (bins[j][u] & 0xFFu) << (8 * (j & 3));
            *(uint4*)(c.bscr + (on.start + base + tid + NT * u) * 16) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
          }
      }
      if (NT == 64 && !reg_rows && pos < 16) {
        // streamed wave-tier node: this group's bins at byte (visiting position) of the slot
#pragma unroll
        for (int u = 0; u < RPT; ++u)
          if (rrow[u] != 0xFFFFFFFFu) {
            uint8_t* slot = c.bscr + (on.start + base + tid + NT * u) * 16;
#pragma unroll
            for (int j = 0; j < KGMAX; ++j)
              if (j < g && pos + j < 16) slot[pos + j] = (uint8_t)bins[j][u];
          }
      }
      if (reg_rows) {
#pragma unroll
        for (int j = 0; j < KGMAX; ++j)
        {
          uint32_t v = 0;
#pragma unroll
          for (int u = 0; u < RPT; ++u) v |= bins[j][u] << (8 * u);
          pk[j] = j < g ? v : 0u;
        }
      }
    }
    __syncthreads();
    PH(2)
    int j0 = wid;
#if !defined(DML_X2_EVAL) && DML_EVAL_PAIRS
    if constexpr (MODE == 1 && (DML_EVAL_PAIRS == 1 || (DML_EVAL_PAIRS == 2) == (NT == 64))) {
      // features j and j + NW evaluated together (two interleaved chains)
      const double* cw = tree_cw<FC>(c, on.tree);
      if (gini_pf_ok(s, cwk(cw, 0), cwk(cw, 1)))
        for (; j0 + NW < g; j0 += 2 * NW) {
          if (mono_of<FC>(c, s, feats[j0]) != 0 || mono_of<FC>(c, s, feats[j0 + NW]) != 0) break;
          eval_gini_pf<2, NW>(hist + j0 * span, span, s, lane, rg + j0, rb + j0, rn + j0, rleft + j0 * c.CH, c.CH, true,
                              cwk(cw, 0), cwk(cw, 1));
          if (lane == 0) { rmid[j0] = 0.0; rmid[j0 + NW] = 0.0; }
        }
    }
#endif
    for (int j = j0; j < g; j += NW) {
#ifdef DML_X2_EVAL   // sensitivity build: every feature evaluated twice (the first keeps the histogram)
      eval_feature<MODE>(hist + j * span, c.C, c.CH, s, lane, rg + j, rb + j, rn + j, rleft + j * c.CH, false,
                         tree_cw<FC>(c, on.tree), &c.rq, MonoQ{mono_of<FC>(c, s, feats[j]), sc->lo, sc->hi}, rmid + j);
      wave_lds_sync();
#endif
      eval_feature<MODE>(hist + j * span, c.C, c.CH, s, lane, rg + j, rb + j, rn + j, rleft + j * c.CH, true,
                         tree_cw<FC>(c, on.tree), &c.rq, MonoQ{mono_of<FC>(c, s, feats[j]), sc->lo, sc->hi}, rmid + j);
    }
    __syncthreads();
    PH(3)
    if (wid == 0) {
      // wave-parallel form of select_group(): feature j counts if it is non-constant and
      // among the first (k - nonconst) non-constant ones of the group; the first maximal
      // gain among those replaces the running best if strictly better
      const int nc0 = sc->nonconst;
      const bool isnc = lane < g && rn[lane] != 0;
      const uint64_t m = __ballot(isnc);
      const bool considered = isnc && nc0 + lane_prefix(m) + 1 <= k;
      const bool has = considered && rb[lane] >= 0;
      double gj = has ? rg[lane] : -INFINITY;
      int jj = has ? lane : 64;
      wave::argmax(gj, jj, lane);
      const bool upd = jj < 64 && gj > sc->best_gain;
      if (upd && lane < c.CH) best_left[lane] = rleft[jj * c.CH + lane];
      if (lane == 0) {
        if (upd) {
          sc->best_gain = gj; sc->best_feat = feats[jj]; sc->best_bin = rb[jj]; sc->best_pos = pos + jj;
          sc->best_mid = rmid[jj];
        }
        sc->best_j = upd ? jj : -1;
        // bscr slots: byte q of a row's 16-B slot = visiting position q (written by the
        // streamed histogram passes: the block tier's first group, the wave tier's groups)
        if (!reg_rows) sc->scr_n = NT > 64 ? (pos == 0 ? min(g, 16) : sc->scr_n) : min(16, pos + g);
        sc->nonconst = min(nc0 + __popcll(m), k);
        sc->pos = pos + g;
      }
    }
    __syncthreads();
    PH(4)
    if (reg_rows) {
      const int bj = sc->best_j;
      uint32_t sel = 0;
      if (KPRE > 0 && pos + g <= npre) {
#pragma unroll
        for (int q = 0; q < (KPRE > 0 ? KPRE : 1); ++q)
          if (q == pos + bj) sel = pre[q];
      } else {
#pragma unroll
        for (int j = 0; j < KGMAX; ++j)
          if (j == bj) sel = pk[j];
      }
      if (bj >= 0)
#pragma unroll
        for (int u = 0; u < RPT; ++u) rbin[u] = (sel >> (8 * u)) & 0xFFu;
    }
  }
  // ---- decision (on-chip values only)
  if (tid == 0) {
    // this node's child pair was reserved by the host for the whole level (no pool atomic)
    int base = pair_base + 2 * (int)blockIdx.x;
    NodeRec leaf; leaf.split = -1; leaf.left = -1;
    c.nodes[base] = leaf;
    c.nodes[base + 1] = leaf;
    if (!(sc->best_feat >= 0 && accept_split_v(c, s, pvs, sc->W, best_left))) {
      base = -1;   // the reserved pair stays as two unreferenced leaves
      c.stage[2 * (stage_base + (int64_t)blockIdx.x)].tier = -1;
      c.stage[2 * (stage_base + (int64_t)blockIdx.x) + 1].tier = -1;
    } else {
      {
        double* lv = c.node_val + (int64_t)base * c.VC;
        for (int q = 0; q < c.VC; ++q) {
          rvs[q] = pvs[q] - best_left[q];
          lv[q] = best_left[q];
          lv[c.VC + q] = rvs[q];
        }
        NodeRec rec; rec.split = pack_split(sc->best_feat, sc->best_bin); rec.left = base;
        c.nodes[on.node] = rec;
        mono_children<FC>(c, on.node, base, mono_of<FC>(c, s, sc->best_feat), sc->best_mid);
      }
    }
    sc->base = base;
    sc->nl = base >= 0 ? (int)best_left[c.CH - 1] : 0;
  }
  __syncthreads();
  PH(5)
  const int base = sc->base;
  if (base < 0) { PH_END(NT == 64 ? 0 : 1) return; }
  const int feat = sc->best_feat, bin = sc->best_bin, nl = sc->nl;
  constexpr int RT = NT > 64 ? 64 : 1;   // the right child is enqueued by another wave / lane
  if (tid == 0)
    stage_child<FC>(c, s, on.tree, base, on.start, nl, on.depth + 1, child_key(on.key, 0),
                2 * (stage_base + (int64_t)blockIdx.x), best_left);
  if (tid == RT)
    stage_child<FC>(c, s, on.tree, base + 1, on.start + nl, cnt - nl, on.depth + 1, child_key(on.key, 1),
                2 * (stage_base + (int64_t)blockIdx.x) + 1, rvs);
  // ---- stable partition
#ifdef DML_X2_PART   // sensitivity build: the (idempotent) partition pass runs twice
  for (int rep_ = 0; rep_ < 2; ++rep_) {
#endif
  if (NT > 64 && !reg_rows && cnt <= 128 * NT && (size_t)((cnt + 63) / 64) * 12 <= (size_t)KG * span * sizeof(CT)) {
    // block tier, streamed node: two passes and two barriers for the whole node (not two per
    // chunk).  Pass 1 ranks every row (split bin from the histogram pass's scratch, else
    // gathered) into one ballot word per 64-row group in LDS (the histograms are dead);
    // one block scan gives every group's left offset; pass 2 re-reads the row ids
    // (coalesced) and writes each row at its stable rank.
    uint64_t* lflag = (uint64_t*)hist;                        // [ngrp] left flags
    int* loff = (int*)(lflag + ((cnt + 63) / 64));            // [ngrp] exclusive left offsets
    const int ngrp = (cnt + 63) / 64;
    const int bjs = __builtin_amdgcn_readfirstlane((sc->best_pos < sc->scr_n) ? sc->best_pos : -1);
    const int fsplit = __builtin_amdgcn_readfirstlane(feat), bsplit = __builtin_amdgcn_readfirstlane(bin);
    constexpr int U = 4;   // positions per thread per round, all loads issued before the ballots
    // the row ids of the first KR rounds are loaded WITH the split bins and kept in registers
    // for pass 2 (which then issues no loads for them): one memory round trip less per round
    // for nodes of <= KR * U * NT rows (most block-tier nodes)
    constexpr int KR = DML_PART_KEEP;
    static_assert(DML_PART_U2 == U, "pass 2 walks the positions of pass 1");
    uint32_t rk[KR > 0 ? KR : 1][U];
#pragma unroll
    for (int q = 0; q < (KR > 0 ? KR : 1); ++q)
#pragma unroll
      for (int u = 0; u < U; ++u) rk[q][u] = 0u;
    for (int p0 = 0, q = 0; p0 < cnt; p0 += U * NT, ++q) {
      uint32_t bv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = min(p0 + u * NT + tid, cnt - 1);
        const uint32_t r = (KR > 0 || bjs < 0) ? rows[p] : 0u;
        if (bjs >= 0) {
          bv[u] = c.bscr[(on.start + p) * 16 + bjs];
        } else {
          bv[u] = c.Xb[(int64_t)(r & c.rmask) * c.ld + fsplit];
        }
#pragma unroll
        for (int qq = 0; qq < KR; ++qq)
          if (qq == q) rk[qq][u] = r;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * NT + tid;
        const uint64_t m = __ballot(p < cnt && (int)bv[u] <= bsplit);
        if (lane == 0 && p - lane < cnt) lflag[(p - lane) >> 6] = m;
      }
    }
    __syncthreads();
    // exclusive prefix of the groups' left counts (<= 2 NT groups: two per thread)
    {
      const int g0 = 2 * tid, g1 = 2 * tid + 1;
      const int c0 = g0 < ngrp ? __popcll(lflag[g0]) : 0, c1 = g1 < ngrp ? __popcll(lflag[g1]) : 0;
      const int incl = wave::incl_scan<int>(c0 + c1);
      if (lane == 63) sc->wcnt[wid] = incl;
      __syncthreads();
      int wbase = 0;
      for (int w = 0; w < wid; ++w) wbase += sc->wcnt[w];
      const int ex = wbase + incl - (c0 + c1);
      if (g0 < ngrp) loff[g0] = ex;
      if (g1 < ngrp) loff[g1] = ex + c0;
    }
    __syncthreads();
    // pass 2, U2 positions per thread per round: the row-id loads of a round are issued
    // (unconditionally, clamped) before its stores, so consecutive rounds do not each wait a
    // full memory round trip behind the previous round's store
    constexpr int U2 = DML_PART_U2;
    for (int p0 = tid, q = 0; p0 < cnt; p0 += U2 * NT, ++q) {
      uint32_t rr[U2];
      if (q < KR) {   // kept from pass 1 (uniform branch: q is the round index)
#pragma unroll
        for (int qq = 0; qq < KR; ++qq)
          if (qq == q)
#pragma unroll
            for (int u = 0; u < U2; ++u) rr[u] = rk[qq][u];
      } else {
#pragma unroll
        for (int u = 0; u < U2; ++u) rr[u] = rows[min(p0 + u * NT, cnt - 1)];
      }
#pragma unroll
      for (int u = 0; u < U2; ++u) {
        const int p = p0 + u * NT;
        if (p >= cnt) break;
        const int q = p >> 6;
        const uint64_t m = lflag[q];
        const int lft = __popcll(m & ((1ull << (p & 63)) - 1ull));
        const bool left = (m >> (p & 63)) & 1ull;
        const int l0 = loff[q];
        c.rows_next[on.start + (left ? l0 + lft : nl + (q * 64 - l0) + ((p & 63) - lft))] = rr[u];
      }
    }
  } else {
  uint32_t* out = c.rows_next + on.start;
  int baseL = 0, baseR = 0;
  // streaming (large-node) partition: the split-feature bins of the next chunk and the row
  // ids two chunks ahead are prefetched while the current chunk is ranked and written
  constexpr uint32_t INVR = 0xFFFFFFFFu;
  auto prow = [&](int r) -> uint32_t { return r < cnt ? rows[r] : INVR; };
  // the split feature's bin at row position p: from the histogram pass's scratch when the
  // final feature group (the one the scratch holds) produced the best split, else gathered
  const int bj_scr = (!reg_rows && sc->best_pos < sc->scr_n) ? sc->best_pos : -1;
  auto pbin = [&](int p, uint32_t r) -> uint32_t {
    if (r == INVR) return 0u;
    if (bj_scr >= 0) return (uint32_t)c.bscr[(on.start + p) * 16 + bj_scr];
    return (uint32_t)c.Xb[(int64_t)(r & c.rmask) * c.ld + feat];
  };
  uint32_t nrow = INVR, nbin = 0, frow = INVR;
  if (!reg_rows && RPT == 1) {
    rrow[0] = prow(tid);
    rbin[0] = pbin(tid, rrow[0]);
    nrow = prow(NT + tid);
  }
  for (int cb = 0; cb < cnt; cb += NT * RPT) {
    if (!reg_rows) {
      if constexpr (RPT == 1) {
        nbin = pbin(cb + NT + tid, nrow);
        frow = prow(cb + 2 * NT + tid);
      } else {
        load_rows(cb);
#pragma unroll
        for (int u = 0; u < RPT; ++u)
          rbin[u] = rrow[u] == 0xFFFFFFFFu ? 0u
                  : bj_scr >= 0 ? (uint32_t)c.bscr[(on.start + cb + tid + NT * u) * 16 + bj_scr]
                                : (uint32_t)c.Xb[(int64_t)(rrow[u] & c.rmask) * c.ld + feat];
      }
    }
    uint64_t ml[RPT], mr[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const bool valid = rrow[u] != 0xFFFFFFFFu;
      const bool left = valid && (int)rbin[u] <= bin;
      ml[u] = __ballot(left);
      mr[u] = __ballot(valid && !left);
    }
    int offL[RPT], offR[RPT], totL = 0, totR = 0;
    if constexpr (NW == 1) {
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        offL[u] = totL; offR[u] = totR;
        totL += __popcll(ml[u]); totR += __popcll(mr[u]);
      }
    } else {
      if (lane == 0)
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
          sc->wcnt[u * NW + wid] = __popcll(ml[u]);
          sc->wcnt[RPT * NW + u * NW + wid] = __popcll(mr[u]);
        }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        int l = 0, r = 0, lb = 0, rbb = 0;
        for (int w = 0; w < NW; ++w) {
          const int cl = sc->wcnt[u * NW + w], cr = sc->wcnt[RPT * NW + u * NW + w];
          if (w < wid) { lb += cl; rbb += cr; }
          l += cl; r += cr;
        }
        offL[u] = totL + lb; offR[u] = totR + rbb;
        totL += l; totR += r;
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const bool valid = rrow[u] != 0xFFFFFFFFu;
      if (!valid) continue;
      if ((int)rbin[u] <= bin) out[baseL + offL[u] + lane_prefix(ml[u])] = rrow[u];
      else out[nl + baseR + offR[u] + lane_prefix(mr[u])] = rrow[u];
    }
    baseL += totL; baseR += totR;
    if (!reg_rows && RPT == 1) { rrow[0] = nrow; rbin[0] = nbin; nrow = frow; }
  }
  }   // streamed block-tier / register-rows partition
#ifdef DML_X2_PART
  }
#endif
  PH(6)
  PH_END(NT == 64 ? 0 : 1)
}

// ------------------------------------------------------------------------------------
// subtree tier: one wave grows the WHOLE subtree under a node with <= 64 rows
// ------------------------------------------------------------------------------------
// Each lane owns one row (bin row cached in LDS, class/target and bootstrap weight in
// registers).  A node is a 64-bit lane mask; the subtree is walked depth-first with an
// LDS stack.  A feature is evaluated by an in-wave bitonic sort of (bin, lane) keys
// followed by wave prefix sums of the class weights — every candidate threshold is one
// lane, no 256-bin histogram is cleared, scanned or flushed.  Candidates are only the
// last lane of each run of equal bins, so the chosen split equals the CPU builder's
// (cumulative sums at "bin <= b" are the same integers).
struct SubEntry {
  uint64_t mask;
  uint64_t key;
  int32_t node, depth;
  double lo, hi;   // monotonic_cst bounds of the node
};
// the stack entry of a criterion-specialised build (FC >= 0: no monotonic_cst, so no bounds):
// 24 instead of 40 B, 1 KB less LDS per 64-row subtree wave (10.3 -> 9.3 KB at d = 100:
// 17 instead of 15 subtree waves per CU)
struct SubEntryLite {
  uint64_t mask;
  uint64_t key;
  int32_t node, depth;
};
template <int FC> using SubEntryT = typename std::conditional<(FC >= 0), SubEntryLite, SubEntry>::type;
__device__ __forceinline__ double e_lo(const SubEntry& e) { return e.lo; }
__device__ __forceinline__ double e_hi(const SubEntry& e) { return e.hi; }
__device__ __forceinline__ double e_lo(const SubEntryLite&) { return -INFINITY; }
__device__ __forceinline__ double e_hi(const SubEntryLite&) { return INFINITY; }
__device__ __forceinline__ void set_bounds(SubEntry& e, double lo, double hi) { e.lo = lo; e.hi = hi; }
__device__ __forceinline__ void set_bounds(SubEntryLite&, double, double) {}

// evaluate one feature for the rows in `mask`; lane data: bin b (valid if in mask).
template <bool REG>
__device__ __forceinline__ void sub_eval(const Ctx& c, const NodeSpec& s, uint64_t mask, int cnt, int lane, int my_bin, int my_cls,
                         float my_w, int64_t my_yq, double& gain, int& bin, bool& nonconst, const double* cw,
                         MonoQ mq, double& mid) {
  const bool act = (mask >> lane) & 1ull;
  // classification: the row's class and weight ride in the key's low bits (bin << 10 | cls << 4
  // | w), so the sorted lanes hold their rows' payload without shuffles (equal keys are
  // interchangeable rows); regression keeps (bin, lane) keys and shuffles its 64-bit targets
  const uint32_t key = !act ? 0xFFFFFFFFu
                            : (REG ? ((uint32_t)my_bin << 6) | (uint32_t)lane
                                   : ((uint32_t)my_bin << 10) | ((uint32_t)my_cls << 4) | ((uint32_t)my_w & 15u));
  const uint32_t sk = wave::bitonic64(key, lane);
  const bool valid_row = lane < cnt;
  const int b = valid_row ? (int)(sk >> (REG ? 6 : 10)) : 1024;
  const int bnext = wave::shift_down1<int>(b, lane, 1024);
  const int blast = wave::bcast<int>(b, cnt - 1);
  const int bfirst = wave::bcast<int>(b, 0);
  nonconst = bfirst != blast;
  const int lrows = lane + 1, rrows = cnt - lrows;
  const bool cand = valid_row && lane < cnt - 1 && b != bnext && lrows >= s.min_samples_leaf &&
                    rrows >= s.min_samples_leaf;
  double g = -INFINITY, mid_l = 0.0;
  bool ok = cand;   // cand and both sides at least min_weight_leaf heavy
  if constexpr (!REG) {
    const int ycls = (int)((sk >> 4) & 63u);
    const uint32_t w = valid_row ? (sk & 15u) : 0u;
    ClsAcc L, R;
    L.init(s.criterion); R.init(s.criterion);
    double l0 = 0.0, t0 = 0.0;
    if (c.C == 2) {
      // binary: ONE scan of (w | w [class 1] << 16) carries both channels (<= 64 rows weigh < 2^16)
      const uint32_t pre = wave::incl_scan<uint32_t>(w | (ycls == 1 ? w << 16 : 0u));
      const uint32_t tot = wave::bcast<uint32_t>(pre, cnt - 1);
      const uint32_t p1 = pre >> 16, p0 = (pre & 0xFFFFu) - p1, q1 = tot >> 16, q0 = (tot & 0xFFFFu) - q1;
      const double lw0 = (double)p0 * cwk(cw, 0), tw0 = (double)q0 * cwk(cw, 0);
      const double lw1 = (double)p1 * cwk(cw, 1), tw1 = (double)q1 * cwk(cw, 1);
      l0 = lw0; t0 = tw0;
      L.add(lw0); R.add(tw0 - lw0);
      L.add(lw1); R.add(tw1 - lw1);
    } else {
      for (int k = 0; k < c.C; ++k) {
        const uint32_t v = (ycls == k) ? w : 0u;
        const uint32_t pre = wave::incl_scan<uint32_t>(v);
        const uint32_t tot = wave::bcast<uint32_t>(pre, cnt - 1);
        const double lw = (double)pre * cwk(cw, k), tw = (double)tot * cwk(cw, k);
        if (k == 0) { l0 = lw; t0 = tw; }
        L.add(lw);
        R.add(tw - lw);
      }
    }
    ok = cand && !side_too_light(s, L.w, R.w);
    if (ok && mq.m) {   // monotonic_cst (class-0 fraction)
      ok = mono_ok(mq.m, mq.lo, mq.hi, side_value(L.w, l0), side_value(R.w, t0 - l0));
      mid_l = mono_mid(L.w, l0, R.w, t0 - l0);
    }
    if (ok) g = cls_proxy(L, R, s.criterion);
  } else {
    // integer prefix sums of w and w yq in (bin, lane) order: at the last lane of a bin
    // run they are the host builder's histogram prefix sums (forest_common.h)
    const int src = (int)(sk & 63u);
    const uint32_t wsh = (uint32_t)__shfl((int)(uint32_t)my_w, src);
    const uint32_t ylo = (uint32_t)__shfl((int)(uint32_t)(uint64_t)my_yq, src);
    const uint32_t yhi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)my_yq >> 32), src);
    const int64_t yq = (int64_t)(((uint64_t)yhi << 32) | ylo);
    const uint64_t w = valid_row ? (uint64_t)wsh : 0ull;
    const uint64_t wy = valid_row ? (uint64_t)((int64_t)wsh * yq) : 0ull;
    const uint64_t p0 = wave::incl_scan_u64(w), p1 = wave::incl_scan_u64(wy);
    const uint64_t t0 = wave::bcast<uint64_t>(p0, cnt - 1), t1 = wave::bcast<uint64_t>(p1, cnt - 1);
    const double l0 = (double)p0, tt0 = (double)t0, l1 = reg_s1(p1, c.rq), tt1 = reg_s1(t1, c.rq);
    ok = cand && !side_too_light(s, l0, tt0 - l0);
    if (ok && mq.m) {
      ok = mono_ok(mq.m, mq.lo, mq.hi, side_value(l0, l1), side_value(tt0 - l0, tt1 - l1));
      mid_l = mono_mid(l0, l1, tt0 - l0, tt1 - l1);
    }
    if (ok) g = reg_proxy(s.criterion, l0, l1, tt0 - l0, tt1 - l1);
  }
  int bl;
  if (!REG && s.criterion == kGini && !mq.m) {
    // Gini gains of candidates are positive doubles, whose bit patterns order like the
    // values: a u64 max, then the first lane holding it (the lowest candidate bin)
    uint64_t gb = ok ? __builtin_bit_cast(uint64_t, g) : 0ull;
    uint64_t mx = gb;
#define DML_MAXU64_STEP(M) { const uint64_t o = wave::shfl_xor<M>(mx, lane); mx = o > mx ? o : mx; }
    DML_MAXU64_STEP(32) DML_MAXU64_STEP(16) DML_MAXU64_STEP(8) DML_MAXU64_STEP(4) DML_MAXU64_STEP(2) DML_MAXU64_STEP(1)
#undef DML_MAXU64_STEP
    const uint64_t hit = __ballot(ok && gb == mx);
    bl = hit ? (int)__builtin_ctzll(hit) : 64;
    g = hit ? __builtin_bit_cast(double, mx) : -INFINITY;
  } else {
    bl = ok ? lane : 64;
    wave::argmax(g, bl, lane);
  }
  mid = wave::bcast<double>(mid_l, bl & 63);
  gain = g;
  const int bsel = wave::bcast<int>(b, bl & 63);
  bin = bl < 64 ? bsel : -1;
}

// ---- segmented evaluation of small subtree nodes (classification) -------------------
// A node with cnt <= WD rows (WD = 8/16/32) is evaluated on 64 / WD features at once: the
// wave is cut into WD-lane segments, each segment holds the node's rows compacted into
// its first cnt lanes and evaluates one feature of the node's visiting order (in-segment
// bitonic sort, segment-relative prefix sums, in-segment argmax).  The candidates, their
// scores and the tie-break (lowest bin, then visiting order) are exactly those of the
// one-feature-per-wave path, so the split found is identical -- most subtree nodes are
// tiny, and this replaces 64-lane sorts of 2-8 valid rows.
template <int WD>
__device__ __forceinline__ uint32_t bitonic_seg(uint32_t key, int j, int lane) {
#define DML_SEG_STEP(K, J)                                      \
  {                                                             \
    const uint32_t other = wave::xor32<J>(key, lane);           \
    const bool up = (K) == WD ? true : ((j & (K)) == 0);        \
    const bool lower = (j & (J)) == 0;                          \
    const uint32_t mn = key < other ? key : other;              \
    const uint32_t mx = key < other ? other : key;              \
    key = (lower == up) ? mn : mx;                              \
  }
  DML_SEG_STEP(2, 1)
  DML_SEG_STEP(4, 2) DML_SEG_STEP(4, 1)
  DML_SEG_STEP(8, 4) DML_SEG_STEP(8, 2) DML_SEG_STEP(8, 1)
  if constexpr (WD >= 16) { DML_SEG_STEP(16, 8) DML_SEG_STEP(16, 4) DML_SEG_STEP(16, 2) DML_SEG_STEP(16, 1) }
  if constexpr (WD >= 32) {
    DML_SEG_STEP(32, 16) DML_SEG_STEP(32, 8) DML_SEG_STEP(32, 4) DML_SEG_STEP(32, 2) DML_SEG_STEP(32, 1)
  }
#undef DML_SEG_STEP
  return key;
}

template <int WD>
__device__ __forceinline__ void argmax_seg(double& g, int& idx, int lane) {
#define DML_SEG_ARG(M)                                               \
  {                                                                  \
    const double og = wave::shfl_xor<M>(g, lane);                    \
    const int oi = wave::shfl_xor<M>(idx, lane);                     \
    if (og > g || (og == g && (unsigned)oi < (unsigned)idx)) {       \
      g = og;                                                        \
      idx = oi;                                                      \
    }                                                                \
  }
  if constexpr (WD >= 32) DML_SEG_ARG(16)
  if constexpr (WD >= 16) DML_SEG_ARG(8)
  DML_SEG_ARG(4) DML_SEG_ARG(2) DML_SEG_ARG(1)
#undef DML_SEG_ARG
}

// evaluates the node whose rows are the compact indices [0, cnt) (src lane of compact
// row j: `src`); updates the running (nonconst, best) in visiting order exactly like the
// per-feature loop.  xc: LDS row-bin cache (stride dp); cls_j / w_j: class and weight of
// compact row j (valid in every segment's lane j).
// Regression (REG): the key carries (bin, compact row j, w); the row's fixed-point target
// comes from segment lane j by one 64-bit shuffle, and the two integer channels (w, w yq)
// are scanned per segment -- the same integer prefix sums, hence the same doubles, as
// sub_eval's one-feature path and the host builder.
template <int WD, bool REG = false>
__device__ __forceinline__ void sub_node_seg(const Ctx& c, const NodeSpec& s, const FeatPerm& fp, int cnt, int lane, int src,
                             int cls_j, uint32_t w_j, const uint8_t* xc, int dp, int& nonconst, double& best_g,
                             int& best_f, int& best_b, const double* cw, int64_t yq_j = 0) {
  constexpr int S = 64 / WD;
  const int d = c.d;
  const int seg = lane / WD, j = lane & (WD - 1);
  const bool valid_row = j < cnt;
  // the row's class and weight ride in the low bits of its sort key (bin << 10 | cls << 4 | w):
  // after the sort every lane holds its sorted row's payload, no shuffles (rows of equal
  // keys are interchangeable: the sums at the end of a bin run are the same)
  const uint32_t pay = REG ? (((uint32_t)j << 4) | (w_j & 15u)) : (((uint32_t)cls_j << 4) | (w_j & 15u));
  // the first 64 visiting positions, one per lane, computed once for the node; a pass reads
  // its S positions' features by readlane (the cycle-walking permutation costs ~40 VALU)
  const int fo = feature_at(fp, min(lane, d - 1), d);
  for (int pos = 0; nonconst < s.max_features && pos < d; pos += S) {
    const bool has_f = pos + seg < d;
    int f = 0;
    if (pos + S <= 64) {
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const int fq = __builtin_amdgcn_readlane(fo, pos + q);
        if (seg == q) f = fq;
      }
      if (!has_f) f = 0;
    } else {
      f = has_f ? feature_at(fp, pos + seg, d) : 0;
    }
    const int my_bin = (valid_row && has_f) ? (int)xc[src * dp + f] : 0;
    const uint32_t key = valid_row ? ((uint32_t)my_bin << 10) | pay : 0xFFFFFFFFu;
    const uint32_t sk = bitonic_seg<WD>(key, j, lane);
    const int b = valid_row ? (int)(sk >> 10) : 1024;
    const int bnext = wave::shift_down1<int>(b, lane, 1024);
    const int ycls = (int)((sk >> 4) & 63u);
    const uint32_t w = valid_row ? (sk & 15u) : 0u;
    const bool cand = valid_row && j < cnt - 1 && b != bnext && j + 1 >= s.min_samples_leaf &&
                      cnt - j - 1 >= s.min_samples_leaf;
    const bool ncl = valid_row && j < cnt - 1 && b != bnext;
    double g = -INFINITY;
    if constexpr (REG) {
      const int srcl = seg * WD + (int)((sk >> 4) & 31u);
      const uint64_t yq = wave::bcast_lane<uint64_t>((uint64_t)yq_j, srcl);
      const uint64_t wv = valid_row ? (uint64_t)w : 0ull, wy = valid_row ? (uint64_t)((int64_t)w * (int64_t)yq) : 0ull;
      uint64_t p0 = wave::incl_scan_u64(wv), p1 = wave::incl_scan_u64(wy);
      uint64_t b0 = 0, b1 = 0, t0 = 0, t1 = 0;
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const uint64_t bq0 = q ? wave::bcast<uint64_t>(p0, q * WD - 1) : 0ull, bq1 = q ? wave::bcast<uint64_t>(p1, q * WD - 1) : 0ull;
        const uint64_t eq0 = wave::bcast<uint64_t>(p0, q * WD + cnt - 1), eq1 = wave::bcast<uint64_t>(p1, q * WD + cnt - 1);
        if (seg == q) { b0 = bq0; b1 = bq1; t0 = eq0 - bq0; t1 = eq1 - bq1; }
      }
      p0 -= b0; p1 -= b1;
      const double l0 = (double)p0, tt0 = (double)t0, l1 = reg_s1(p1, c.rq), tt1 = reg_s1(t1, c.rq);
      if (cand && !side_too_light(s, l0, tt0 - l0)) g = reg_proxy(s.criterion, l0, l1, tt0 - l0, tt1 - l1);
    } else {
    ClsAcc L, R;
    L.init(s.criterion); R.init(s.criterion);
    // segment-relative inclusive prefix: subtract the inclusive total of the preceding segments
    auto seg_scan = [&](uint32_t v, uint32_t& pre, uint32_t& tot) {
      pre = wave::incl_scan<uint32_t>(v);
      uint32_t base = 0;
      tot = 0;
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const uint32_t bq = q ? (uint32_t)__builtin_amdgcn_readlane((int)pre, q * WD - 1) : 0u;
        const uint32_t eq = (uint32_t)__builtin_amdgcn_readlane((int)pre, q * WD + cnt - 1);
        if (seg == q) { base = bq; tot = eq - bq; }
      }
      pre -= base;
    };
    if (c.C == 2) {
      // binary: ONE scan of (w | w [class 1] << 16) carries both channels (a node of <= 32
      // rows weighs < 2^16)
      uint32_t pre, tot;
      seg_scan(w | (ycls == 1 ? w << 16 : 0u), pre, tot);
      const uint32_t l1 = pre >> 16, l0 = (pre & 0xFFFFu) - l1, t1 = tot >> 16, t0 = (tot & 0xFFFFu) - t1;
      const double lw0 = (double)l0 * cwk(cw, 0), tw0 = (double)t0 * cwk(cw, 0);
      const double lw1 = (double)l1 * cwk(cw, 1), tw1 = (double)t1 * cwk(cw, 1);
      L.add(lw0); R.add(tw0 - lw0);
      L.add(lw1); R.add(tw1 - lw1);
    } else {
      for (int k = 0; k < c.C; ++k) {
        uint32_t pre, tot;
        seg_scan((ycls == k) ? w : 0u, pre, tot);
        const double lw = (double)pre * cwk(cw, k), tw = (double)tot * cwk(cw, k);
        L.add(lw);
        R.add(tw - lw);
      }
    }
    if (cand && !side_too_light(s, L.w, R.w)) g = cls_proxy(L, R, s.criterion);
    }
    const bool ok = g != -INFINITY;
    int bl = ok ? j : 64;
    argmax_seg<WD>(g, bl, lane);
    const int bsel = __shfl(b, seg * WD + (bl & (WD - 1)));
    const uint64_t ncm = __ballot(ncl);
    // selection over the S features in visiting order, vectorised: segment q counts when its
    // feature is non-constant and among the first (max_features - nonconst) such; the first
    // maximal gain among the counted ones replaces the running best if strictly better --
    // exactly the sequential loop's outcome
    uint32_t ncs = 0;   // bit q: segment q's feature is non-constant (and exists)
#pragma unroll
    for (int q = 0; q < S; ++q)
      if (pos + q < d && ((ncm >> (q * WD)) & (WD == 64 ? ~0ull : ((1ull << WD) - 1ull))) != 0ull) ncs |= 1u << q;
    const int room = s.max_features - nonconst;
    const bool counted = ((ncs >> seg) & 1u) && __popc(ncs & ((1u << seg) - 1u)) < room;
    double gq = (counted && bl < 64) ? g : -INFINITY;
    int qi = (counted && bl < 64) ? seg : 64;
    if constexpr (S >= 2) {
      auto step = [&](auto Mc) {
        constexpr int M = decltype(Mc)::value;
        const double og = wave::shfl_xor<M>(gq, lane);
        const int oi = wave::shfl_xor<M>(qi, lane);
        if (og > gq || (og == gq && oi < qi)) { gq = og; qi = oi; }
      };
      if constexpr (WD <= 32) step(std::integral_constant<int, 32>{});
      if constexpr (WD <= 16) step(std::integral_constant<int, 16>{});
      if constexpr (WD <= 8) step(std::integral_constant<int, 8>{});
    }
    nonconst = min(s.max_features, nonconst + __popc(ncs));
    gq = wave::bcast<double>(gq, 0);
    qi = wave::bcast<int>(qi, 0);
    if (qi < 64 && gq > best_g) {
      best_g = gq;
      best_f = feature_at(fp, pos + qi, d);
      best_b = __builtin_amdgcn_readlane(bsel, qi * WD);
    }
  }
}

// Grows the whole subtree under one node of <= 64 rows with ONE wave (k_subtree; k_bigsub
// for its small nodes): stack[0] / sstats[0..VC) hold the node on entry.  Lane `lane` holds
// one row of the node: its class / weight / fixed-point target in registers and its bins
// at xc[my_lr * dp] (IDENT: my_lr == lane).  alloc() (lane 0) hands out the next reserved
// child pair, or -1.
template <bool REG, int FC, bool IDENT, class Alloc, class E>
__device__ __forceinline__ void subtree_dfs(const Ctx& c, const NodeSpec& s, int lane, int my_lr, int my_cls, float my_w,
                                            int64_t my_yq, int64_t my_y2q, const uint8_t* xc, int dp, bool cache,
                                            const uint8_t* xg, int cnt0, E* stack, double* sstats,
                                            double* left_ch, double* right_ch, int32_t* cidx, double Wt,
                                            const double* tcw, Alloc alloc PH_ARGS_DECL) {
  const int d = c.d;
  const int VC = c.VC;
  int sp = 1;
  while (sp > 0) {
    --sp;
    const E e = stack[sp];
    const double* pv = sstats + sp * VC;
    const int cnt = __popcll(e.mask);
    int nonconst = 0, best_f = -1, best_b = -1;
    double best_g = -INFINITY, best_mid = 0.0;
    const FeatPerm fp = feat_perm(e.key, d);
    if (cache && cnt <= 32 && (FC >= 0 || !c.mono) && DML_SUB_SEG_REG + !REG > 0) {
      // compact the node's rows: compact row j <- lane of the j-th set bit of the mask
      const bool in = (e.mask >> lane) & 1ull;
      if (in) cidx[lane_prefix(e.mask)] = lane;
      wave_lds_sync();
      const int jx = cnt <= 8 ? (lane & 7) : (cnt <= 16 ? (lane & 15) : (lane & 31));
      const int src0 = jx < cnt ? cidx[jx] : 0;
      const int src = IDENT ? src0 : __shfl(my_lr, src0);   // the source lane's cached row
      const int cls_j = REG ? 0 : __shfl(my_cls, src0);
      const uint32_t w_j = (uint32_t)__shfl((int)(uint32_t)my_w, src0);
      const int64_t yq_j = REG ? (int64_t)wave::bcast_lane<uint64_t>((uint64_t)my_yq, src0) : 0;
#if defined(DML_X2_SUB) && DML_X2_SUB != 2   // sensitivity build: every segmented evaluation twice (the first into copies)
      {
        int nc2 = nonconst, bf2 = best_f, bb2 = best_b;
        double bg2 = best_g;
        if (cnt <= 8) sub_node_seg<8, REG>(c, s, fp, cnt, lane, src, cls_j, w_j, xc, dp, nc2, bg2, bf2, bb2, tcw, yq_j);
        else if (cnt <= 16) sub_node_seg<16, REG>(c, s, fp, cnt, lane, src, cls_j, w_j, xc, dp, nc2, bg2, bf2, bb2, tcw, yq_j);
        else sub_node_seg<32, REG>(c, s, fp, cnt, lane, src, cls_j, w_j, xc, dp, nc2, bg2, bf2, bb2, tcw, yq_j);
        if (bg2 == -12345.0 && bf2 == 7 && nc2 == 3) atomicOr(&c.counters[kOpenOvf], bb2);
      }
#endif
      if (cnt <= 8) sub_node_seg<8, REG>(c, s, fp, cnt, lane, src, cls_j, w_j, xc, dp, nonconst, best_g, best_f, best_b, tcw, yq_j);
      else if (cnt <= 16) sub_node_seg<16, REG>(c, s, fp, cnt, lane, src, cls_j, w_j, xc, dp, nonconst, best_g, best_f, best_b, tcw, yq_j);
      else sub_node_seg<32, REG>(c, s, fp, cnt, lane, src, cls_j, w_j, xc, dp, nonconst, best_g, best_f, best_b, tcw, yq_j);
      wave_lds_sync();   // cidx is rewritten by the next node
      PH(1)
      PH_CNT(4, 1)
      PH_CNT(5, cnt)
    } else
    for (int pos = 0; nonconst < s.max_features && pos < d; ++pos) {
      const int f = feature_at(fp, pos, d);
      const int my_bin = cache ? xc[my_lr * dp + f] : (lane < cnt0 ? xg[f] : 0);
      double g, mid;
      int bb;
      bool nc;
#if defined(DML_X2_SUB) && DML_X2_SUB != 1   // sensitivity: every one-feature evaluation twice
      sub_eval<REG>(c, s, e.mask, cnt, lane, my_bin, my_cls, my_w, my_yq, g, bb, nc, tcw,
                    MonoQ{mono_of<FC>(c, s, f), e_lo(e), e_hi(e)}, mid);
      if (g == -12345.0 && bb == 7) atomicOr(&c.counters[kOpenOvf], (int)nc);
#endif
      sub_eval<REG>(c, s, e.mask, cnt, lane, my_bin, my_cls, my_w, my_yq, g, bb, nc, tcw,
                    MonoQ{mono_of<FC>(c, s, f), e_lo(e), e_hi(e)}, mid);
      if (nc) {
        ++nonconst;
        if (bb >= 0 && g > best_g) { best_g = g; best_f = f; best_b = bb; best_mid = mid; }
      }
    }
    if (!(cache && cnt <= 32 && (FC >= 0 || !c.mono) && DML_SUB_SEG_REG + !REG > 0)) {
      PH(2)
      PH_CNT(6, 1)
      PH_CNT(7, cnt)
    }
    if (best_f < 0) continue;
    const int mybin = cache ? xc[my_lr * dp + best_f] : (lane < cnt0 ? xg[best_f] : 0);
    const bool in = (e.mask >> lane) & 1ull;
    const uint64_t lm = __ballot(in && mybin <= best_b) & e.mask;
    const uint64_t rm = e.mask & ~lm;
    // left child statistics (class weights / regression sums) by wave reductions
    if (!REG && c.C == 2) {   // binary: one packed integer sum (a <= 64-row node weighs < 2^16)
      const bool inl = (lm >> lane) & 1ull;
      const uint32_t w = (uint32_t)my_w;
      const uint32_t x = wave::sum<uint32_t>(inl ? (w | (my_cls == 1 ? w << 16 : 0u)) : 0u, lane);
      const uint32_t l1 = x >> 16, l0 = (x & 0xFFFFu) - l1;
      if (lane == 0) {
        const double v0 = (double)l0 * cwk(tcw, 0), v1 = (double)l1 * cwk(tcw, 1);
        left_ch[0] = v0; right_ch[0] = pv[0] - v0;
        left_ch[1] = v1; right_ch[1] = pv[1] - v1;
      }
    } else
    for (int k = 0; k < VC; ++k) {
      double v;
      const bool inl = (lm >> lane) & 1ull;
      if constexpr (REG) {   // integer sums (exact in any order), then the double channels
        const int64_t wi = (int64_t)my_w;
        uint64_t q = !inl ? 0ull : (uint64_t)(k == 0 ? wi : (k == 1 ? wi * my_yq : wi * my_y2q));
        q = wave::sum<uint64_t>(q, lane);
        v = k == 0 ? (double)q : (k == 1 ? reg_s1(q, c.rq) : reg_s2(q, c.rq));
      } else {
        v = (inl && my_cls == k) ? (double)my_w : 0.0;
        v = wave::sum<double>(v, lane);     // integer-valued: exact in any order
        v *= cwk(tcw, k);
      }
      if (lane == 0) { left_ch[k] = v; right_ch[k] = pv[k] - v; }
    }
    wave_lds_sync();
    int base = -1;
    if (lane == 0 && accept_split_v(c, s, pv, Wt, left_ch)) base = alloc();
    if (lane == 0 && base >= 0) {
      NodeRec leaf; leaf.split = -1; leaf.left = -1;
      c.nodes[base] = leaf;
      c.nodes[base + 1] = leaf;
      double* lv = c.node_val + (int64_t)base * VC;
      for (int q = 0; q < VC; ++q) {
        lv[q] = left_ch[q];
        lv[VC + q] = right_ch[q];
      }
      NodeRec rec; rec.split = pack_split(best_f, best_b); rec.left = base;
      c.nodes[e.node] = rec;
      mono_children<FC>(c, e.node, base, mono_of<FC>(c, s, best_f), best_mid);
    }
    base = wave::bcast<int>(base, 0);
    if (base < 0) continue;
    const int nl = __popcll(lm), nr = cnt - nl;
    // push right then left (left subtree first); leaf-by-count/purity children are not pushed.
    // The popped entry's slot `sp` is reused: compute both children's sums before writing.
    if (lane == 0) {
      const int dep = e.depth + 1;
      const bool push_r = !leaf_by_counts(s, nr, dep) && !leaf_by_weight(s, vals_weight(right_ch, c.C, c.is_reg)) &&
                          impure_v<FC>(c, s, right_ch);
      const bool push_l = !leaf_by_counts(s, nl, dep) && !leaf_by_weight(s, vals_weight(left_ch, c.C, c.is_reg)) &&
                          impure_v<FC>(c, s, left_ch);
      const int mbest = mono_of<FC>(c, s, best_f);
      if (push_r) {
        E r; r.mask = rm; r.key = child_key(e.key, 1); r.node = base + 1; r.depth = dep;
        double blo, bhi;
        mono_child_bounds(mbest, e_lo(e), e_hi(e), best_mid, 1, blo, bhi);
        set_bounds(r, blo, bhi);
        for (int q = 0; q < VC; ++q) sstats[sp * VC + q] = right_ch[q];
        stack[sp++] = r;
      }
      if (push_l) {
        E l; l.mask = lm; l.key = child_key(e.key, 0); l.node = base; l.depth = dep;
        double blo, bhi;
        mono_child_bounds(mbest, e_lo(e), e_hi(e), best_mid, 0, blo, bhi);
        set_bounds(l, blo, bhi);
        for (int q = 0; q < VC; ++q) sstats[sp * VC + q] = left_ch[q];
        stack[sp++] = l;
      }
    }
    sp = wave::bcast<int>(sp, 0);
    wave_lds_sync();
    PH(3)
  }
}

// SR: rows the LDS layout holds (64; 32 for the small-subtree tier 4, whose roots have
// <= sub_small <= 32 rows -- the DFS stack never holds more entries than the root has rows)
template <bool REG, int FC, int SR = 64>
__global__ __launch_bounds__(64) void k_subtree(Ctx c, int set_cur, int tier) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  PH_BEGIN
  const OpenNode on = c.open[set_cur][tier][blockIdx.x];
  const NodeSpec s = spec_of<FC>(c, on.tree);
  const int lane = threadIdx.x;
  const int d = c.d;
  const int VC = c.VC;
  const bool cache = c.sub_cache_d > 0;
  const int dp = c.sub_cache_d;
  // LDS: DFS stack, per-entry channel sums (no global re-reads of node stats), left
  // child sums, row-bin cache
  using E = SubEntryT<FC>;
  E* stack = (E*)smem;
  double* sstats = (double*)(stack + SR);            // [SR][VC]
  double* left_ch = sstats + SR * VC;                // [VC]
  double* right_ch = left_ch + VC;                   // [VC] (+ pad)
  uint8_t* xc = (uint8_t*)(left_ch + ((2 * VC + 1) & ~1));
  int32_t* cidx = (int32_t*)(xc + ((SR * c.sub_cache_d + 15) & ~15));   // [64] compaction map
  const int cnt0 = on.count;
  const uint32_t* rows = c.rows_cur + on.start;
  uint32_t row = 0;
  int my_cls = 0;
  float my_w = 0.f;
  int64_t my_yq = 0, my_y2q = 0;   // regression: the row's fixed-point y, y^2
  if (lane < cnt0) {
    const uint32_t wd = rows[lane];
    row = word_row(c, wd);
    my_w = (float)word_weight(c, s, wd);
    if constexpr (REG) reg_quantize(tree_y(c, s)[row], c.rq, my_yq, my_y2q);
    else my_cls = word_cls(c, wd);
  }
  const uint8_t* xg = c.Xb + (int64_t)row * c.ld;
  if (cache && lane < cnt0) {
    // the row's bins, ONE 16-B load per 16 features (a byte loop costs the vector memory
    // pipeline one address per feature per row: 100 instead of 7 at d = 100) and one
    // 4-B LDS store per 4 features (dp is a multiple of 4)
    if ((c.ld & 15) == 0 && c.ld >= ((d + 15) & ~15)) {
      const uint4* src = (const uint4*)xg;
      uint32_t* dst = (uint32_t*)(xc + lane * dp);
      const int nw = dp >> 2, nseg = (d + 15) >> 4;
      for (int q0 = 0; q0 < nseg; q0 += 8) {   // 8 loads in flight before the first store
        uint4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = q0 + i < nseg ? src[q0 + i] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int w0 = 4 * (q0 + i);
          if (w0 + 0 < nw) dst[w0 + 0] = v[i].x;
          if (w0 + 1 < nw) dst[w0 + 1] = v[i].y;
          if (w0 + 2 < nw) dst[w0 + 2] = v[i].z;
          if (w0 + 3 < nw) dst[w0 + 3] = v[i].w;
        }
      }
    } else {
      for (int j = 0; j < d; ++j) xc[lane * dp + j] = xg[j];
    }
  }
#ifdef DML_X2_SUBSETUP   // sensitivity build: the setup's dependent chain (row word -> row line) twice
  if (cache && lane < cnt0 && (c.ld & 15) == 0) {
    const uint32_t msk = (uint32_t)c.n >> 31;   // 0 at run time, unknown to the compiler
    const uint32_t wd2 = rows[lane + (int)((xc[lane * dp] & 1u) * msk)];
    const uint4* src2 = (const uint4*)(c.Xb + (int64_t)word_row(c, wd2) * c.ld);
    uint32_t* dst = (uint32_t*)(xc + lane * dp);
    for (int q = 0; q < ((d + 15) >> 4); ++q) {
      const uint4 v = src2[q];
      dst[0] |= (v.x | v.y | v.z | v.w) & msk;
    }
  }
#endif
  // a subtree over cnt0 rows has at most cnt0 - 1 splits: all its node pairs are reserved at
  // once -- by k_compact for staged nodes (on.pool_base), else with ONE pool atomic here
  // (unused pairs stay unreferenced)
  int pool_base = on.pool_base;
  const int max_splits = subtree_max_splits(s, cnt0, on.depth);
  if (lane == 0) {
    const int want = 2 * max_splits;
    if (pool_base == -1) {
      pool_base = want > 0 ? atomicAdd(&c.counters[kPool], want) : 0;
      if (want > 0 && (int64_t)pool_base + want > c.pool_cap) {
        atomicOr(&c.counters[kOverflow], 1);
        pool_base = -1;
      }
    } else if (pool_base < 0) {
      pool_base = -1;   // k_compact flagged the overflow
    }
    E e;
    e.mask = cnt0 >= 64 ? ~0ull : ((1ull << cnt0) - 1ull);
    e.key = on.key; e.node = on.node; e.depth = on.depth;
    set_bounds(e, (FC < 0 && c.nbound) ? c.nbound[2 * (int64_t)on.node] : -INFINITY,
               (FC < 0 && c.nbound) ? c.nbound[2 * (int64_t)on.node + 1] : INFINITY);
    stack[0] = e;
  }
  if (lane < VC) sstats[lane] = c.node_val[(int64_t)on.node * VC + lane];
  const double Wt = c.tree_W[on.tree];
  const double* tcw = REG ? nullptr : tree_cw<FC>(c, on.tree);
  pool_base = wave::bcast<int>(pool_base, 0);
  if (pool_base < 0) return;
  int used = 0;   // child pairs handed out (lane 0's copy counts)
  wave_lds_sync();
  PH(0)
  subtree_dfs<REG, FC, true>(c, s, lane, lane, my_cls, my_w, my_yq, my_y2q, xc, dp, cache, xg, cnt0, stack, sstats,
                             left_ch, right_ch, cidx, Wt, tcw,
                             [&]() { return used < max_splits ? pool_base + 2 * used++ : -1; } PH_ARGS_PASS);
  used = wave::bcast<int>(used, 0);
  // reserved-but-unused node pairs become well-formed (unreferenced) leaves, so any
  // pass over the whole pool sees valid records
  const NodeRec leaf{-1, -1};
  for (int i = 2 * used + lane; i < 2 * max_splits; i += 64) c.nodes[pool_base + i] = leaf;
  PH(4)
  PH_END(2)
}

// ------------------------------------------------------------------------------------
// big-subtree tier (binary classification): ONE 256-thread workgroup grows the WHOLE
// subtree under a node of <= bigsub_max (<= 256) rows
// ------------------------------------------------------------------------------------
// The node's rows are read from HBM / the Infinity Cache ONCE: their row words, then each
// row's bin line into an LDS row cache.  (The wave tier gathers every row's line again at
// each of the two or three levels above the subtree tier, and each of those nodes is a
// chain of dependent global round trips -- open node, row words, row lines -- issued while
// the level's block tier keeps the memory system saturated: the phase profile puts 41 % of
// a wave-tier node's cycles and 41 % of a subtree root's in those loads.)  Below the root
// every node lives on chip: a node is a range [start, start + cnt) of the workgroup's local
// row permutation `lp`, and the four waves are independent workers taking nodes from a
// locked LDS stack:
//   * cnt > 64:  the wave builds LDS histograms of DML_BIG_KG features at a time from the
//                cached bins (4 rows per lane), evaluates them with eval_feature -- the wave
//                and block tiers' routine: same candidates, same fp64 scores -- selects in
//                visiting order exactly as k_nodes does, partitions its range stably and
//                pushes the children;
//   * cnt <= 64: the wave grows the node's whole subtree with subtree_dfs (k_subtree's
//                sort-based / segmented evaluation), lanes mapped to the range's rows.
// Child pairs come from the subtree's reserved pool range (k_compact, or one pool atomic).
#ifndef DML_BIG_KG
#define DML_BIG_KG 2   // features per histogram group of a big node (2 KB of LDS each)
#endif
#ifndef DML_BIG_STACK
#define DML_BIG_STACK 128   // live entries: disjoint nodes of >= 2 rows of <= 256
#endif

struct BigEntry {
  uint64_t key;
  int32_t node, depth;
  int32_t start, cnt;
  double v0, v1;   // class-weight sums of the node (binary)
};

struct BigShared {
  int32_t lock, top, pending, used, pool_base, max_splits, overflow, pad;
};

// per-wave scratch: a big node's histograms + evaluation slots, or a small node's DFS state
struct BigWave {
  size_t hist, rg, rb, rn, rleft, cur, dfs_stack, dfs_stats, dfs_lr, dfs_cidx, total;
};

__host__ __device__ inline BigWave big_wave_layout() {
  BigWave L;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = (off + bytes + 15) / 16 * 16; return o; };
  // big-node view
  L.hist = take((size_t)DML_BIG_KG * 256 * 8);
  L.rg = take((size_t)DML_BIG_KG * 8);
  L.rb = take((size_t)DML_BIG_KG * 4);
  L.rn = take((size_t)DML_BIG_KG * 4);
  L.rleft = take((size_t)DML_BIG_KG * 3 * 8);
  L.cur = take(sizeof(BigEntry));
  const size_t big_end = off;
  // small-node (DFS) view, aliased onto the same bytes
  off = 0;
  L.dfs_stack = take(64 * sizeof(SubEntry));
  L.dfs_stats = take(64 * 2 * 8);
  L.dfs_lr = take(2 * 2 * 8);            // left_ch, right_ch
  L.dfs_cidx = take(64 * 4);
  L.total = off > big_end ? off : big_end;
  return L;
}

struct BigLayout {
  size_t sh, stk, rcls, rw, lp, tmp, waves, xc, total;
};

__host__ __device__ inline BigLayout big_layout(int rmax, int dp) {
  BigLayout L;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = (off + bytes + 15) / 16 * 16; return o; };
  L.sh = take(sizeof(BigShared));
  L.stk = take((size_t)DML_BIG_STACK * sizeof(BigEntry));
  L.rcls = take(256);
  L.rw = take(256);
  L.lp = take(256);
  L.tmp = take(256);
  L.waves = take(4 * big_wave_layout().total);
  L.xc = take((size_t)rmax * dp);
  L.total = off;
  return L;
}

__device__ __forceinline__ void big_lock(BigShared* sh) {
  while (atomicCAS(&sh->lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void big_unlock(BigShared* sh) {
  __threadfence_block();
  atomicExch(&sh->lock, 0);
}

template <int FC>
__global__ __launch_bounds__(256) void k_bigsub(Ctx c, int set_cur) {
  constexpr bool PK = FC >= 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const OpenNode on = c.open[set_cur][1][blockIdx.x];
  const NodeSpec s = spec_of<FC>(c, on.tree);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int d = c.d, dp = c.sub_cache_d;
  const BigLayout L = big_layout(c.bigsub_max, dp);
  const BigWave W = big_wave_layout();
  BigShared* sh = (BigShared*)(smem + L.sh);
  BigEntry* stk = (BigEntry*)(smem + L.stk);
  uint8_t* rcls = smem + L.rcls;
  uint8_t* rw = smem + L.rw;
  uint8_t* lp = smem + L.lp;
  uint8_t* tmp = smem + L.tmp;
  uint8_t* xc = smem + L.xc;
  unsigned char* wv = smem + L.waves + (size_t)wid * W.total;
  const int cnt0 = on.count;
  // ---- the node's rows, once: row word (weight, class) and the row's bin line
  if (tid < cnt0) {
    const uint32_t wd = c.rows_cur[on.start + tid];
    const uint32_t row = word_row(c, wd);
    rw[tid] = (uint8_t)word_weight<PK>(c, s, wd);
    rcls[tid] = (uint8_t)word_cls<PK>(c, wd);
    lp[tid] = (uint8_t)tid;
    const uint8_t* xg = c.Xb + (int64_t)row * c.ld;
    uint32_t* dst = (uint32_t*)(xc + tid * dp);
    const int nw = dp >> 2;
    if ((c.ld & 15) == 0 && c.ld >= ((d + 15) & ~15)) {
      const uint4* src = (const uint4*)xg;
      const int nseg = (d + 15) >> 4;
      for (int q0 = 0; q0 < nseg; q0 += 8) {   // 8 loads in flight before the first store
        uint4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = q0 + i < nseg ? src[q0 + i] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int w0 = 4 * (q0 + i);
          if (w0 + 0 < nw) dst[w0 + 0] = v[i].x;
          if (w0 + 1 < nw) dst[w0 + 1] = v[i].y;
          if (w0 + 2 < nw) dst[w0 + 2] = v[i].z;
          if (w0 + 3 < nw) dst[w0 + 3] = v[i].w;
        }
      }
    } else {
      for (int j = 0; j < d; ++j) xc[tid * dp + j] = xg[j];
    }
  }
  if (tid == 0) {
    // every pair the subtree can need, reserved at once (k_compact for staged nodes)
    int pool_base = on.pool_base;
    const int max_splits = subtree_max_splits(s, cnt0, on.depth);
    const int want = 2 * max_splits;
    if (pool_base == -1) {
      pool_base = want > 0 ? atomicAdd(&c.counters[kPool], want) : 0;
      if (want > 0 && (int64_t)pool_base + want > c.pool_cap) {
        atomicOr(&c.counters[kOverflow], 1);
        pool_base = -1;
      }
    } else if (pool_base < 0) {
      pool_base = -1;   // k_compact flagged the overflow
    }
    sh->lock = 0; sh->used = 0; sh->pool_base = pool_base; sh->max_splits = max_splits; sh->overflow = 0;
    BigEntry e;
    e.key = on.key; e.node = on.node; e.depth = on.depth; e.start = 0; e.cnt = cnt0;
    e.v0 = c.node_val[(int64_t)on.node * 2]; e.v1 = c.node_val[(int64_t)on.node * 2 + 1];
    stk[0] = e;
    sh->top = 1;
    sh->pending = 1;
  }
  __syncthreads();
  const int pool_base = sh->pool_base, max_splits = sh->max_splits;
  if (pool_base < 0) return;
  const double Wt = c.tree_W[on.tree];
  const double* tcw = tree_cw<FC>(c, on.tree);
  auto alloc = [&]() -> int {   // lane 0: next reserved child pair
    const int u = atomicAdd(&sh->used, 1);
    return u < max_splits ? pool_base + 2 * u : -1;
  };
  BigEntry* cur = (BigEntry*)(wv + W.cur);
  const int k = s.max_features;
  // ---- worker loop: take a node, grow it (big) or its whole subtree (small), push children
  for (int spins = 0;;) {
    int got = 0;
    if (lane == 0) {
      big_lock(sh);
      if (sh->top > 0) {
        *cur = stk[--sh->top];
        got = 1;
      }
      big_unlock(sh);
    }
    got = __builtin_amdgcn_readfirstlane(got);
    if (!got) {
      const int pend = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(&sh->pending, 0) : 0);
      if (pend == 0) break;
      if (++spins > (1 << 24)) {   // never expected: bounded so a bug cannot hang the GPU
        if (lane == 0) atomicOr(&c.counters[kOverflow], 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    wave_lds_sync();
    const BigEntry e = *cur;
    const int cnt = e.cnt, start = e.start;
    if (cnt <= 64) {
      // ---- small node: the whole subtree below it, one wave (k_subtree's DFS)
      SubEntry* dstack = (SubEntry*)(wv + W.dfs_stack);
      double* dstats = (double*)(wv + W.dfs_stats);
      double* left_ch = (double*)(wv + W.dfs_lr);
      double* right_ch = left_ch + 2;
      int32_t* cidx = (int32_t*)(wv + W.dfs_cidx);
      const int my_lr = lane < cnt ? (int)lp[start + lane] : 0;
      const int my_cls = lane < cnt ? (int)rcls[my_lr] : 0;
      const float my_w = lane < cnt ? (float)rw[my_lr] : 0.f;
      wave_lds_sync();   // `cur` aliases the DFS stack
      if (lane == 0) {
        SubEntry r;
        r.mask = cnt >= 64 ? ~0ull : ((1ull << cnt) - 1ull);
        r.key = e.key; r.node = e.node; r.depth = e.depth; r.lo = -INFINITY; r.hi = INFINITY;
        dstack[0] = r;
        dstats[0] = e.v0; dstats[1] = e.v1;
      }
      wave_lds_sync();
#ifdef DML_PHASE_PROF
      uint64_t _pt = clock64(); uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
      subtree_dfs<false, FC, false>(c, s, lane, my_lr, my_cls, my_w, 0, 0, xc, dp, true, nullptr, cnt, dstack, dstats,
                                    left_ch, right_ch, cidx, Wt, tcw, alloc PH_ARGS_PASS);
      if (lane == 0) atomicAdd(&sh->pending, -1);
      continue;
    }
    // ---- big node (65..256 rows): histograms from the cached bins, 4 rows per lane
    unsigned long long* hist = (unsigned long long*)(wv + W.hist);
    double* rg = (double*)(wv + W.rg);
    int* rb = (int*)(wv + W.rb);
    int* rn = (int*)(wv + W.rn);
    double* rleft = (double*)(wv + W.rleft);
    int lr[4];
    uint64_t pl[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = lane + 64 * u;
      lr[u] = p < cnt ? (int)lp[start + p] : -1;
      pl[u] = lr[u] >= 0 ? pack_bin((int)rcls[lr[u]], (uint32_t)rw[lr[u]]) : 0ull;
    }
    for (int i = lane; i < DML_BIG_KG * 256; i += 64) hist[i] = 0ull;
    wave_lds_sync();
    const FeatPerm fp = feat_perm(e.key, d);
    int pos = 0, nonconst = 0, best_feat = -1, best_bin = -1;
    double best_gain = -INFINITY, bl0 = 0.0, bl1 = 0.0;
    while (nonconst < k && pos < d) {
      const int g = min(DML_BIG_KG, min(k - nonconst, d - pos));
      int fj[DML_BIG_KG];
#pragma unroll
      for (int j = 0; j < DML_BIG_KG; ++j) fj[j] = __builtin_amdgcn_readfirstlane(j < g ? feature_at(fp, pos + j, d) : 0);
#pragma unroll
      for (int j = 0; j < DML_BIG_KG; ++j) {
        if (j >= g) continue;
        uint32_t b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = lr[u] >= 0 ? (uint32_t)xc[lr[u] * dp + fj[j]] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (lr[u] >= 0) atomicAdd(&hist[j * 256 + b[u]], (unsigned long long)pl[u]);
      }
      wave_lds_sync();
      for (int j = 0; j < g; ++j)
        eval_feature<1>(hist + j * 256, 2, 3, s, lane, rg + j, rb + j, rn + j, rleft + j * 3, true, tcw, nullptr,
                        MonoQ{0, 0.0, 0.0}, nullptr);
      wave_lds_sync();
      // select in visiting order (k_nodes' wave-parallel form of select_group)
      const bool isnc = lane < g && rn[lane] != 0;
      const uint64_t m = __ballot(isnc);
      const bool considered = isnc && nonconst + lane_prefix(m) + 1 <= k;
      const bool has = considered && rb[lane] >= 0;
      double gj = has ? rg[lane] : -INFINITY;
      int jj = has ? lane : 64;
      wave::argmax(gj, jj, lane);
      if (jj < 64 && gj > best_gain) {
        best_gain = gj;
        best_feat = fj[0];
#pragma unroll
        for (int j = 1; j < DML_BIG_KG; ++j) if (jj == j) best_feat = fj[j];
        best_bin = rb[jj];
        bl0 = rleft[jj * 3]; bl1 = rleft[jj * 3 + 1];
      }
      nonconst = min(nonconst + __popcll(m), k);
      pos += g;
    }
    // ---- decision (lane 0) on the node's sums; child pair from the reserved range
    int base = -1;
    const double best_left[3] = {bl0, bl1, 0.0};
    const double pv[2] = {e.v0, e.v1};
    if (lane == 0 && best_feat >= 0 && accept_split_v(c, s, pv, Wt, best_left)) base = alloc();
    if (lane == 0 && base >= 0) {
      NodeRec leaf; leaf.split = -1; leaf.left = -1;
      c.nodes[base] = leaf;
      c.nodes[base + 1] = leaf;
      double* lv = c.node_val + (int64_t)base * 2;
      lv[0] = bl0; lv[1] = bl1; lv[2] = e.v0 - bl0; lv[3] = e.v1 - bl1;
      NodeRec rec; rec.split = pack_split(best_feat, best_bin); rec.left = base;
      c.nodes[e.node] = rec;
    }
    base = __builtin_amdgcn_readfirstlane(base);
    int npush = 0;
    if (base >= 0) {
      // ---- stable partition of the node's range (left rows keep their order, then right)
      uint64_t ml[4], mr[4];
      int nlw = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool left = lr[u] >= 0 && (int)xc[lr[u] * dp + best_feat] <= best_bin;
        ml[u] = __ballot(left);
        mr[u] = __ballot(lr[u] >= 0 && !left);
        nlw += __popcll(ml[u]);
      }
      int offL = 0, offR = nlw;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (lr[u] >= 0) {
          const bool left = (ml[u] >> lane) & 1ull;
          tmp[start + (left ? offL + lane_prefix(ml[u]) : offR + lane_prefix(mr[u]))] = (uint8_t)lr[u];
        }
        offL += __popcll(ml[u]);
        offR += __popcll(mr[u]);
      }
      wave_lds_sync();
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (lr[u] >= 0) lp[start + lane + 64 * u] = tmp[start + lane + 64 * u];
      wave_lds_sync();
      if (lane == 0) {
        const double rv0 = e.v0 - bl0, rv1 = e.v1 - bl1;
        BigEntry ch[2];
        ch[0].key = child_key(e.key, 0); ch[0].node = base; ch[0].depth = e.depth + 1;
        ch[0].start = start; ch[0].cnt = nlw; ch[0].v0 = bl0; ch[0].v1 = bl1;
        ch[1].key = child_key(e.key, 1); ch[1].node = base + 1; ch[1].depth = e.depth + 1;
        ch[1].start = start + nlw; ch[1].cnt = cnt - nlw; ch[1].v0 = rv0; ch[1].v1 = rv1;
        bool push[2];
        for (int side = 0; side < 2; ++side) {
          const double vals[2] = {ch[side].v0, ch[side].v1};
          push[side] = !leaf_by_counts(s, ch[side].cnt, ch[side].depth) && !leaf_by_weight(s, vals[0] + vals[1]) &&
                       impure_v<FC>(c, s, vals);
        }
        npush = (int)push[0] + (int)push[1];
        if (npush) {
          big_lock(sh);
          // right first: the left child is taken next (depth-first, like the other tiers)
          for (int side = 1; side >= 0; --side) {
            if (!push[side]) continue;
            if (sh->top < DML_BIG_STACK) stk[sh->top++] = ch[side];
            else { sh->overflow = 1; atomicOr(&c.counters[kOverflow], 1); --npush; }
          }
          atomicAdd(&sh->pending, npush);
          big_unlock(sh);
        }
      }
    }
    if (lane == 0) atomicAdd(&sh->pending, -1);
  }
  __syncthreads();
  // reserved-but-unused node pairs become well-formed (unreferenced) leaves
  const int used = min(sh->used, max_splits);
  const NodeRec leaf{-1, -1};
  for (int i = 2 * used + tid; i < 2 * max_splits; i += 256) c.nodes[pool_base + i] = leaf;
}

// ------------------------------------------------------------------------------------
// large tier
// ------------------------------------------------------------------------------------
// one wave per large node: state + the first feature group of its visiting order
__global__ __launch_bounds__(64) void k_large_prep(Ctx c, int set_cur, int nL) {
  const int slot = blockIdx.x;
  const int lane = threadIdx.x;
  LState st;
  st.on = c.open[set_cur][3][slot];
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  int16_t* feats = c.lperm + (int64_t)slot * c.d;
  st.g = min(c.kg_large, min(s.max_features, c.d));
  const FeatPerm fp = feat_perm(st.on.key, c.d);
  const int nperm = c.full_cur ? c.d : st.g;   // whole-histogram level: the whole visiting order
  for (int j = lane; j < nperm; j += 64) feats[j] = (int16_t)feature_at(fp, j, c.d);
  if (lane != 0) return;
  st.pos = 0; st.nonconst = 0; st.done = 0; st.best_feat = -1; st.best_bin = -1; st.split = 0; st.nl = 0;
  st.best_gain = -INFINITY;
  st.best_mid = 0.0;
  st.best_pos = 1 << 30;
  st.scr_n = st.g <= 16 ? st.g : 0;
  st.scr_id = 0; st.derive = 0; st.par = -1; st.sib = -1;
  c.lyy[slot] = 0ull;
  if (c.full_cur) {
    // the next level's sibling table: its large nodes (<= 2 per node here) start as "no parent"
    const int4 none = make_int4(-1, -1, -1, -1);
    if (2 * slot < c.pi_cap) c.pinfo_next[2 * slot] = none;
    if (2 * slot + 1 < c.pi_cap) c.pinfo_next[2 * slot + 1] = none;
    // whole-histogram level: round r's row pass covers features [r kg, (r + 1) kg) by id, so
    // bscr holds features [0, g0) (not visiting positions); a larger sibling is derived
    st.scr_n = 0;
    const int g0 = min(c.kg_large, c.d);
    if (c.full_prev) {
      const int4 pi = c.pinfo_cur[slot];
      if (pi.x >= 0) { st.par = pi.x; st.sib = pi.y; st.derive = pi.z; }
    }
    st.scr_id = (!st.derive && g0 <= 16) ? g0 : 0;
  }
  c.lstate[slot] = st;
  c.lcursor[2 * slot] = 0;
  c.lcursor[2 * slot + 1] = 0;
}

__device__ __forceinline__ uint32_t large_bin(const Ctx& c, uint32_t wd, int f) {
  const uint32_t row = wd & c.rmask;
  return c.XbT ? (uint32_t)c.XbT[(int64_t)f * c.n + row] : (uint32_t)c.Xb[(int64_t)row * c.ld + f];
}

// fround >= 0 (whole-histogram level): the round's features are [fround kg, ...) by id and
// the histogram goes to the node's whole-feature buffer (Ctx::gf_cur); derived nodes skip
template <int MODE, bool PK>
__global__ __launch_bounds__(256) void k_hist_large(Ctx c, int fround) {
  using CT = typename HT<MODE>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int slot = DML_LSLOT;
  const LState& st = c.lstate[slot];
  // node state read once (the loop's bscr stores could alias it: a reference would reload it)
  const int st_pos = fround >= 0 ? fround : __builtin_amdgcn_readfirstlane(st.pos);
  const int64_t st_start = st.on.start;
  if (st.done || (fround >= 0 && st.derive)) return;
  const int r0 = DML_LCHUNK * c.chunk;
  if (r0 >= st.on.count) return;
  const int r1 = min(r0 + c.chunk, st.on.count);
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  // row-window node: a sparse node (under n / fm_div rows) of a unit-weight whole-feature level
  // (boosting).  Its rounds are kg_rw features wide when the host set that (fewer rounds: each
  // round re-reads one cache line per row), kg_large otherwise; a node past its last round exits
  const bool rw_node = MODE == 2 && fround >= 0 && s.bootstrap == 0 && c.fm_div > 0 && (c.ld & 15) == 0 &&
                       c.ld >= 32 && (int64_t)st.on.count * c.fm_div < (int64_t)c.n;
  const int kgr = (rw_node && c.kg_rw > 0) ? c.kg_rw : c.kg_large;
  const int f0 = fround >= 0 ? fround * kgr : 0;
  if (fround >= 0 && f0 >= c.d) return;
  const int g = fround >= 0 ? min(kgr, c.d - f0) : st.g;
  constexpr int RPL = MODE == 2 ? 2 : 3;
  const int span = large_planes(MODE, c.CH) * 256;
  // compact slices (unit-weight regression builds, host-checked): u32 counts in 128 words, then
  // the w yq plane -- LDS stride ls = 384 words per feature instead of span = 512
  const bool compact = MODE == 2 && c.large_compact != 0;
  // packed builds: one u64 word per bin (count | w yq), 2 KB per feature
  const bool packed = compact && c.large_pack != 0;
  const int ls = packed ? 256 : (compact ? 384 : span), wo = packed ? 0 : (compact ? 128 : 256);
  __shared__ int16_t feats[64];
  CT* hist = (CT*)smem;
  const int16_t* perm = c.lperm + (int64_t)slot * c.d + st.pos;
  for (int j = threadIdx.x; j < g; j += 256) feats[j] = fround >= 0 ? (int16_t)(f0 + j) : perm[j];
  for (int i = threadIdx.x; i < g * ls; i += 256) hist[i] = (CT)0;
  __syncthreads();
  const uint32_t* rows = c.rows_cur + st.on.start;
  const float* ty = tree_y(c, s);
  constexpr int KGL = DML_KGL_LARGE;
  // regression tree without bootstrap: every active row weighs 1, so the (w | rows << 32)
  // plane is a row count -- kept as u32 LDS counters (ds_add_u32: half the bytes and bank
  // pairs of the u64 add) in the first KB of each feature's 4-KB slice, widened at the flush
  constexpr int KGW = DML_KGW_LARGE;
  const bool uw = MODE == 2 && s.bootstrap == 0 && g <= (rw_node ? KGW : KGL);
  // cached root counts (boosting): the count plane is copied in by k_root_counts, so only the
  // w yq plane is accumulated (one LDS atomic per (row, feature) instead of two)
  const bool skipc = MODE == 2 && s.bootstrap == 0 && fround >= 0 && c.root_cnt_skip != 0;
  if (g <= KGL || (uw && rw_node)) {
    // ping-pong software pipeline with compile-time-counted unconditional gathers (the block
    // tier's loop in k_nodes): the row id two steps ahead and the next step's bins are in
    // flight while this step's histogram atomics run, with no vmcnt(0) drain between steps
    constexpr uint32_t INV = 0xFFFFFFFFu;
    using PL = typename PLT<MODE>::T;
    const int t0 = r0 + (int)threadIdx.x;
    // row windows (RW): a whole-histogram round reads features [f0, f0 + g) -- contiguous ids, at
    // most two aligned 16-B pieces of the row line -- so a sparse node's row-major gather is two
    // dwordx4 loads of one cache line per row (the bytes picked out by uniform register index)
    // instead of g byte loads, while a feature-major gather of a node holding 1/2^k of the rows
    // pays ~2^k / 128 line lookups per (row, feature).  Nodes under n / fm_div rows
    // (DML_LARGE_FM_DIV, opt-in; see the Ctx setup) of unit-weight whole-feature rounds (boosting)
    const bool rwin = rw_node && uw && (f0 & 15) + g <= 32;
    // feature offsets otherwise: the feature-major copy (stride n) when present, else the row line
    const bool fm = c.XbT != nullptr && !rwin;
    auto run = [&](auto Gc, auto UWc, auto RWc) __attribute__((always_inline)) {
      constexpr int G = decltype(Gc)::value;
      constexpr bool UW = decltype(UWc)::value;
      constexpr bool RW = decltype(RWc)::value;
      int64_t fo[G];
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int64_t f = __builtin_amdgcn_readfirstlane((int)feats[j < g ? j : 0]);
        fo[j] = fm ? f * c.n : f;
      }
      const uint8_t* tab = fm ? c.XbT : c.Xb;
      const int64_t rstride = fm ? 1 : c.ld;
      auto row_at = [&](int r) -> uint32_t {
        const uint32_t v = rows[min(r, r1 - 1)];
        return r < r1 ? v : INV;
      };
      // RW: the two 16-B pieces covering the round's bytes, the dword / shift of each feature
      const int q0 = __builtin_amdgcn_readfirstlane(f0 >> 4);
      const int q1 = __builtin_amdgcn_readfirstlane(min(q0 + 1, (int)(c.ld >> 4) - 1));
      int wi[G], wsh[G];
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int p = (f0 & 15) + (j < g ? j : 0);
        wi[j] = __builtin_amdgcn_readfirstlane(p >> 2);
        wsh[j] = (p & 3) * 8;
      }
      auto gather = [&](uint32_t wd, uint32_t* b) {
#ifdef DML_PROBE_NOGATHER   // timing probe only (wrong histograms): bins from the row id, no table read
#pragma unroll
        for (int j = 0; j < G; ++j) b[j] = (wd + 37u * (uint32_t)j) & 0xFFu;
#else
        if constexpr (RW) {
          typedef uint32_t v8u __attribute__((ext_vector_type(8)));
          const uint4* xr = (const uint4*)(c.Xb + (int64_t)(wd != INV ? (wd & c.rmask) : 0u) * c.ld);
          const uint4 v0 = xr[q0], v1 = xr[q1];
          v8u w;
          w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w; w[4] = v1.x; w[5] = v1.y; w[6] = v1.z; w[7] = v1.w;
#pragma unroll
          for (int j = 0; j < G; ++j) b[j] = (w[wi[j]] >> wsh[j]) & 0xFFu;
        } else {
          const uint8_t* xr = tab + (int64_t)(wd != INV ? (wd & c.rmask) : 0u) * rstride;
#pragma unroll
          for (int j = 0; j < G; ++j) b[j] = (uint32_t)xr[fo[j]];
        }
#endif
      };
      auto consume = [&](int r, bool valid, const uint32_t* b, const PRaw& pr) {
        if (!valid) return;
        if (st_pos == 0) {   // round 0: bins of visiting positions 0..15 (Ctx::bscr)
          uint32_t w4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int j = 0; j < G && j < 16; ++j) w4[j >> 2] |= (j < g ? b[j] & 0xFFu : 0u) << (8 * (j & 3));
          *(uint4*)(c.bscr + (st_start + r) * 16) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        const PL pl = payload_finish<MODE, PK>(c, s, ty, pr);
        if constexpr (MODE == 2 && UW) {
          if (skipc) {   // wave-uniform: the count plane comes from the root-count cache
#pragma unroll
            for (int j = 0; j < G; ++j)
              if (j < g) hist_add_wy<MODE>(hist + j * ls, (int)b[j], pl, wo);
          } else if (packed) {   // wave-uniform: count and w yq in one atomic
#pragma unroll
            for (int j = 0; j < G; ++j)
              if (j < g) hist_add_packed<MODE>(hist + j * ls, (int)b[j], pl, wo);
          } else {
#pragma unroll
            for (int j = 0; j < G; ++j)
              if (j < g) hist_add_unit<MODE>(hist + j * ls, (int)b[j], pl, wo);
          }
        } else {
#pragma unroll
          for (int j = 0; j < G; ++j)
            if (j < g) hist_add<MODE, RPL>(hist + j * span, c, (int)b[j], pl);
        }
      };
      uint32_t rA = row_at(t0), rB = row_at(t0 + 256);
      uint32_t bA[G], bB[G];
      gather(rA, bA);
      PRaw pA = payload_fetch<MODE, PK>(c, ty, rA), pB;
      bool vA = rA != INV, vB = false;
      for (int r = t0; r < r1; r += 512) {
        rA = row_at(r + 512);
        gather(rB, bB);
        pB = payload_fetch<MODE, PK>(c, ty, rB);
        vB = rB != INV;
        consume(r, vA, bA, pA);
        rB = row_at(r + 768);
        gather(rA, bA);
        pA = payload_fetch<MODE, PK>(c, ty, rA);
        vA = rA != INV;
        consume(r + 256, vB, bB, pB);
      }
    };
    auto rung = [&](auto UWc, auto RWc) __attribute__((always_inline)) {
      switch (g) {
#define DML_G_CASE(N) case N: run(std::integral_constant<int, N>{}, UWc, RWc); break;
        DML_G_CASE(1) DML_G_CASE(2) DML_G_CASE(3) DML_G_CASE(4) DML_G_CASE(5) DML_G_CASE(6) DML_G_CASE(7)
        DML_G_CASE(8) DML_G_CASE(9) DML_G_CASE(10) DML_G_CASE(11) DML_G_CASE(12) DML_G_CASE(13) DML_G_CASE(14)
        DML_G_CASE(15)
#undef DML_G_CASE
        default: run(std::integral_constant<int, KGL>{}, UWc, RWc); break;
      }
    };
    if constexpr (MODE == 2) {
      // row windows only where boosting runs them (unit-weight whole-feature rounds), ONE
      // instantiation (G = KGL; features past g are masked): more copies of this loop made the
      // compiler outline it (a function call per row step)
      if (uw && rwin) run(std::integral_constant<int, KGW>{}, std::true_type{}, std::true_type{});
      else if (uw) rung(std::true_type{}, std::false_type{});
      else rung(std::false_type{}, std::false_type{});
    } else {
      rung(std::false_type{}, std::false_type{});
    }
  } else if constexpr (MODE == 2) {
    // wide groups (g > KGL, e.g. boosting's whole-feature rounds of 24): per row, the bins of 8
    // features at a time from the row's line, all 8 loads issued before their atomics (the
    // visiting list is padded to a multiple of 8 with its first feature, so the loads are
    // unconditional; the atomics stop at g); the count plane is skipped when cached
    for (int j = g + threadIdx.x; j < ((g + 7) & ~7) && j < 64; j += 256) feats[j] = feats[0];
    __syncthreads();
    for (int r = r0 + threadIdx.x; r < r1; r += 256) {
      const uint32_t wd = rows[r];
      const uint32_t row = word_row(c, wd);
      const RegPL p = reg_payload(c, word_weight(c, s, wd), ty[row]);
      const uint8_t* xr = c.Xb + (int64_t)row * c.ld;
      for (int j0 = 0; j0 < g; j0 += 8) {
        uint32_t bb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) bb[u] = xr[feats[j0 + u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (j0 + u >= g) break;
          CT* hj = hist + (j0 + u) * span;
          if (!skipc) atomicAdd(&hj[bb[u]], p.wr);
          atomicAdd(&hj[256 + bb[u]], p.wy);
        }
      }
    }
  } else {
    for (int r = r0 + threadIdx.x; r < r1; r += 256) {
      const uint32_t row = rows[r];
      hist_add_row<MODE, RPL>(hist, c, ty, feats, g, word_row(c, row), word_weight(c, s, row), span);
    }
  }
  __syncthreads();
  // flush into the node's global histogram: unpacked planes [CH][256] (u32) for
  // classification, the three integer planes (u64) for regression
  const int gspan = large_planes(MODE == 1 ? 0 : MODE, c.CH) * 256;
  // per-round buffer, or the node's whole-feature buffer at the round's first feature
  const int64_t goff = fround >= 0 ? ((int64_t)slot * c.d + f0) * gspan : (int64_t)slot * c.kg_large * gspan;
  void* gbase = fround >= 0 ? c.gf_cur : c.ghist;
  if constexpr (MODE == 1) {
    uint32_t* gh = (uint32_t*)gbase + goff;
    for (int i = threadIdx.x; i < g * 256; i += 256) {
      const unsigned long long v = hist[i];
      if (!v) continue;
      const int j = i >> 8, b = i & 255;
      uint32_t* gj = gh + j * gspan;
      const uint32_t w0 = (uint32_t)(v & kPackMask21), w1 = (uint32_t)((v >> 21) & kPackMask21);
      if (w0) atomicAdd(&gj[b], w0);
      if (w1) atomicAdd(&gj[256 + b], w1);
      atomicAdd(&gj[512 + b], (uint32_t)(v >> 42));
    }
  } else {
    CT* gh = (CT*)gbase + goff;
    // whole-feature buffers of unit-weight trees keep the count plane as u32 row counts too
    // (gcnt: half the flush atomics' bytes for that plane; see whole_counts_u32)
    const bool gcnt = MODE == 2 && fround >= 0 && s.bootstrap == 0;
    for (int i = threadIdx.x; i < g * span; i += 256) {
      const int j = i / span, b = i - j * span;
      if (MODE == 2 && b < 256 && skipc) continue;   // count plane: copied from the root-count cache
      // LDS word of global element (j, b): the same index, or (compact) the w yq plane at wo;
      // packed words (not at a cached root) hold both the count and the biased w yq
      const bool pk = packed && !skipc;
      CT v = (MODE == 2 && b >= 256) ? hist[j * ls + wo + (b - 256)] : (compact ? (CT)0 : hist[i]);
      if (MODE == 2 && b >= 256 && pk) v = (CT)pack_wy((unsigned long long)v);
      if (MODE == 2 && b < 256 && (uw || gcnt)) {
        // row count of bin b: the u32 LDS counters, or rows << 32 of the (w | rows << 32) plane
        const uint32_t n1 = pk ? pack_count((unsigned long long)hist[j * ls + wo + b])
                               : (uw ? ((const uint32_t*)(hist + j * ls))[b] : (uint32_t)((uint64_t)v >> 32));
        if (gcnt) {
          if (n1) atomicAdd((uint32_t*)(gh + j * span) + b, n1);
          continue;
        }
        v = (CT)((unsigned long long)n1 | ((unsigned long long)n1 << 32));   // w = rows
      }
#ifndef DML_PROBE_NOFLUSH   // timing probe only (wrong histograms): no global flush atomics
      if (v != (CT)0) atomicAdd(&gh[i], v);
#else
      if (v == (CT)0x5A5A5A5A5A5Aull) gh[i] = v;   // keeps the LDS reads live
#endif
    }
  }
}

// boosting roots: the u32 count planes of the root histograms (gf_cur, gcnt layout: the first KB
// of each feature's count plane) <-> the per-tree cache ForestArgs::root_counts.  save = 1 stores
// a build's root counts, save = 0 copies them into a build that skipped its count atomics.
__global__ __launch_bounds__(256) void k_root_counts(Ctx c, int save) {
  const int slot = blockIdx.x, f = blockIdx.y;
  const int64_t gspan = (int64_t)large_planes(2, c.CH) * 256;
  const int tree = c.lstate[slot].on.tree;
  uint32_t* g = (uint32_t*)((unsigned long long*)c.gf_cur + ((int64_t)slot * c.d + f) * gspan);
  uint32_t* r = c.root_counts + ((int64_t)tree * c.d + f) * 256;
  const int b = threadIdx.x;
  if (save) r[b] = g[b];
  else g[b] = r[b];
}

// whole-histogram level: a derived node's histogram over all d features = its parent's
// (previous level) - its sibling's (this level's row pass), in exact integer arithmetic
// (u32 class / row counts, two's-complement u64 regression sums); MODE = global layout
template <int MODE>
__global__ __launch_bounds__(256) void k_hist_derive(Ctx c) {
  using CT = typename HT<MODE>::T;
  const int slot = blockIdx.x;
  const LState& st = c.lstate[slot];
  if (!st.derive) return;
  const int64_t per = (int64_t)c.d * large_planes(MODE, c.CH) * 256;
  CT* dst = (CT*)c.gf_cur + (int64_t)slot * per;
  const CT* par = (const CT*)c.gf_prev + (int64_t)st.par * per;
  const CT* sib = (const CT*)c.gf_cur + (int64_t)st.sib * per;
  for (int64_t i = (int64_t)blockIdx.y * 1024 + threadIdx.x; i < per && i < (int64_t)(blockIdx.y + 1) * 1024; i += 256)
    dst[i] = par[i] - sib[i];
}

__device__ void large_commit(const Ctx& c, const NodeSpec& s, LState& st, int slot, const double* best_left, int set_cur);

// whole-feature regression histogram of a unit-weight tree: bins 0..255 of the count plane are
// u32 row counts (k_hist_large's gcnt flush) in the plane's first KB; element i of the usual
// (w | rows << 32, w yq) layout.  Derivation (parent - sibling, as u64 words) stays exact on the
// packed counts: every parent bin count >= the sibling's, so no borrow crosses a u32 boundary.
__device__ __forceinline__ unsigned long long whole_counts_u32(const unsigned long long* h, int i) {
  if (i < 256) {
    const unsigned long long n1 = ((const uint32_t*)h)[i];
    return n1 | (n1 << 32);
  }
  return h[i];
}

// evaluates the node's global histogram; MODE here is the GLOBAL layout (0 or 2)
template <int MODE>
__global__ __launch_bounds__(256) void k_split_large(Ctx c, int set_cur) {
  using CT = typename HT<MODE>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int slot = blockIdx.x;
  LState& st = c.lstate[slot];
  if (st.done) return;
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  const int g = st.g, span = large_planes(MODE, c.CH) * 256;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  CT* hist = (CT*)smem;
  double* rg = (double*)(smem + (size_t)c.kg_large * span * sizeof(CT));
  int* rb = (int*)(rg + c.kg_large);
  int* rn = rb + c.kg_large;
  double* rleft = (double*)(rn + c.kg_large + (c.kg_large & 1));
  double* rmid = rleft + (int64_t)c.kg_large * c.CH;   // monotonic_cst middle values
  __shared__ int need_more;
  const int16_t* feats = c.lperm + (int64_t)slot * c.d + st.pos;
  if (c.full_cur) {   // whole-feature buffer: the group's features by id
    const CT* gf = (const CT*)c.gf_cur + (int64_t)slot * c.d * span;
    const bool gcnt = MODE == 2 && s.bootstrap == 0;
    for (int i = tid; i < g * span; i += 256) {
      const int j = i / span;
      const CT* hf = gf + (int64_t)feats[j] * span;
      if constexpr (MODE == 2) hist[i] = gcnt ? (CT)whole_counts_u32(hf, i - j * span) : hf[i - j * span];
      else hist[i] = hf[i - j * span];
    }
  } else {
    const CT* gh = (const CT*)c.ghist + (int64_t)slot * c.kg_large * span;
    for (int i = tid; i < g * span; i += 256) hist[i] = gh[i];
  }
  const double nlo = c.nbound ? c.nbound[2 * (int64_t)st.on.node] : -INFINITY;
  const double nhi = c.nbound ? c.nbound[2 * (int64_t)st.on.node + 1] : INFINITY;
  __syncthreads();
  for (int j = wid; j < g; j += 4)
    eval_feature<MODE, 2>(hist + j * span, c.C, c.CH, s, lane, rg + j, rb + j, rn + j, rleft + j * c.CH, false,
                          tree_cw(c, st.on.tree), &c.rq, MonoQ{mono_of(c, s, feats[j]), nlo, nhi}, rmid + j);
  __syncthreads();
  double* best_left = c.lbest_left + (int64_t)slot * c.CH;
  if (tid == 0) {
    int nc = st.nonconst, bf = st.best_feat, bbin = st.best_bin;
    double bg = st.best_gain;
    int uj;
    select_group(c, s, feats, g, rg, rb, rn, rleft, best_left, nc, bg, bf, bbin, uj);
    st.nonconst = nc; st.best_gain = bg; st.best_feat = bf; st.best_bin = bbin;
    if (uj >= 0) { st.best_pos = st.pos + uj; st.best_mid = rmid[uj]; }
    st.pos += g;
    need_more = (st.nonconst < s.max_features && st.pos < c.d) ? 1 : 0;
  }
  __syncthreads();
  if (need_more) {
    // extend the visiting order by the next feature group and ask the host for a round
    if (wid == 0) {
      const int g2 = min(c.kg_large, min(s.max_features - st.nonconst, c.d - st.pos));
      int16_t* perm = c.lperm + (int64_t)slot * c.d;
      const FeatPerm fp = feat_perm(st.on.key, c.d);
      for (int j = lane; j < g2; j += 64) perm[st.pos + j] = (int16_t)feature_at(fp, st.pos + j, c.d);
      if (lane == 0) {
        st.g = g2;
        atomicOr(&c.counters[kNeedMore], 1);
      }
    }
    return;
  }
  if (tid != 0) return;
  st.done = 1;
  if (c.is_reg) {
    // regression: the best candidate is partitioned first; k_large_finish adds the left
    // rows' sum w y2q (from the partition pass) and then accepts / creates / enqueues
    if (st.best_feat >= 0) { st.split = 2; st.nl = (int)best_left[c.CH - 1]; }
    return;
  }
  large_commit(c, s, st, slot, best_left, set_cur);
}

// whole-histogram level, all split candidates at once: workgroup (slot, q) evaluates visiting
// positions 4q .. 4q+3 of large node `slot`, one wave each, from the node's whole-feature
// histogram (Ctx::gf_cur).  Replaces ceil(d / kg_large) dependent k_split_large launches of nL
// workgroups each (20 workgroups on a 256-CU chip for a boosting stage of 20 trees).  The
// regression layout is evaluated straight from global memory (eval_feature reads 4 bins per
// lane); the class-plane layout is staged in LDS (eval_feature_lds scans in place).
template <int GM>
__global__ __launch_bounds__(256) void k_split_full(Ctx c) {
  using CT = typename HT<GM>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int slot = blockIdx.x;
  const LState& st = c.lstate[slot];
  if (st.done) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p = blockIdx.y * 4 + wid;
  const bool active = p < c.d;
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  const int span = large_planes(GM, c.CH) * 256;
  const int f = active ? (int)c.lperm[(int64_t)slot * c.d + p] : 0;
  CT* h = (CT*)c.gf_cur + ((int64_t)slot * c.d + f) * span;
  if constexpr (GM == 0) {
    CT* lh = (CT*)smem + (int64_t)wid * span;
    for (int i = lane; i < span && active; i += 64) lh[i] = h[i];
    h = lh;
    __syncthreads();
  } else {
    if (s.bootstrap == 0) {   // u32 count plane (whole_counts_u32) -> the evaluator's layout, in LDS
      CT* lh = (CT*)smem + (int64_t)wid * span;
      for (int i = lane; i < span && active; i += 64) lh[i] = (CT)whole_counts_u32(h, i);
      h = lh;
      __syncthreads();
    }
  }
  if (!active) return;
  const double nlo = c.nbound ? c.nbound[2 * (int64_t)st.on.node] : -INFINITY;
  const double nhi = c.nbound ? c.nbound[2 * (int64_t)st.on.node + 1] : INFINITY;
  const int64_t o = (int64_t)slot * c.d + p;
  eval_feature<GM, 2>(h, c.C, c.CH, s, lane, c.fr_g + o, c.fr_b + o, c.fr_n + o, c.fr_left + o * c.CH, false,
                      tree_cw(c, st.on.tree), &c.rq, MonoQ{mono_of(c, s, f), nlo, nhi}, c.fr_mid + o);
}

// the node's best candidate in visiting order, 64 positions per step (k_nodes' wave-parallel
// form of select_group: the same order, ties and non-constant count as the per-group rounds),
// then the k_split_large tail
template <int GM>
__global__ __launch_bounds__(64) void k_split_full_select(Ctx c, int set_cur) {
  const int slot = blockIdx.x;
  const int lane = threadIdx.x;
  LState& st = c.lstate[slot];
  if (st.done) return;
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  const int k = s.max_features;
  const int64_t o = (int64_t)slot * c.d;
  double* best_left = c.lbest_left + (int64_t)slot * c.CH;
  int nonconst = st.nonconst, best_pos = -1;
  double best_gain = st.best_gain;
  for (int q0 = 0; q0 < c.d && nonconst < k; q0 += 64) {
    const int p = q0 + lane;
    const bool isnc = p < c.d && c.fr_n[o + p] != 0;
    const uint64_t m = __ballot(isnc);
    const bool considered = isnc && nonconst + lane_prefix(m) + 1 <= k;
    const bool has = considered && c.fr_b[o + p] >= 0;
    double gj = has ? c.fr_g[o + p] : -INFINITY;
    int jj = has ? p : (1 << 30);
    wave::argmax(gj, jj, lane);
    if (jj < (1 << 30) && gj > best_gain) { best_gain = gj; best_pos = jj; }
    nonconst = min(nonconst + __popcll(m), k);
  }
  if (best_pos >= 0 && lane < c.CH) best_left[lane] = c.fr_left[(o + best_pos) * c.CH + lane];
  if (lane != 0) return;
  st.nonconst = nonconst;
  if (best_pos >= 0) {
    st.best_gain = best_gain;
    st.best_feat = c.lperm[o + best_pos];
    st.best_bin = c.fr_b[o + best_pos];
    st.best_pos = best_pos;
    st.best_mid = c.fr_mid[o + best_pos];
  }
  st.pos = c.d;
  st.done = 1;
  if (c.is_reg) {   // as k_split_large: partition first, k_large_finish accepts
    if (st.best_feat >= 0) { st.split = 2; st.nl = (int)best_left[c.CH - 1]; }
    return;
  }
  large_commit(c, s, st, slot, best_left, set_cur);
}

// accept the node's best split, create and enqueue its children (+ the next level's
// sibling table on whole-histogram levels); st.split = 1 when it splits, else 0
__device__ void large_commit(const Ctx& c, const NodeSpec& s, LState& st, int slot, const double* best_left, int set_cur) {
  int base = -1;
  if (st.best_feat >= 0 && accept_split(c, s, st.on.node, st.on.tree, best_left))
    base = make_children(c, st.on.node, st.best_feat, st.best_bin, best_left);
  if (base < 0) { st.split = 0; return; }
  mono_children(c, st.on.node, base, mono_of(c, s, st.best_feat), st.best_mid);
  st.split = 1;
  st.nl = (int)best_left[c.CH - 1];
  const int set_next = 1 - set_cur;
  const int il = enqueue_or_leaf(c, st.on.tree, base, st.on.start, st.nl, st.on.depth + 1, child_key(st.on.key, 0),
                                 set_next);
  const int ir = enqueue_or_leaf(c, st.on.tree, base + 1, st.on.start + st.nl, st.on.count - st.nl, st.on.depth + 1,
                                 child_key(st.on.key, 1), set_next);
  if (c.full_cur && il >= 0 && ir >= 0) {
    // both children are large: the next level passes over the smaller one's rows and
    // derives the larger (ties: the right child is derived)
    const int dl = st.nl > st.on.count - st.nl ? 1 : 0;
    c.pinfo_next[il] = make_int4(slot, ir, dl, 0);
    c.pinfo_next[ir] = make_int4(slot, il, 1 - dl, 0);
  }
}

__global__ __launch_bounds__(256) void k_partition_large(Ctx c) {
  // pass 1 ranks the chunk's rows (split bins prefetched one step ahead, flags kept in LDS)
  // and reserves the chunk's left/right ranges with ONE atomic pair; pass 2 writes the rows
  // at ballot/prefix offsets (no global atomics per 256 rows)
  const int slot = DML_LSLOT;
  const LState& st = c.lstate[slot];
  if (!st.split) return;
  const int r0 = DML_LCHUNK * c.chunk;
  if (r0 >= st.on.count) return;
  const int r1 = min(r0 + c.chunk, st.on.count);
  const int feat = st.best_feat, bin = st.best_bin, nl = st.nl;
  const uint32_t* rows = c.rows_cur + st.on.start;
  uint32_t* out = c.rows_next + st.on.start;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* lflag = (uint64_t*)smem;            // [chunk / 64] left-flag words (ballots)
  __shared__ int wcnt[8];
  __shared__ int tbase[2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr uint32_t INV = 0xFFFFFFFFu;
  auto row_at = [&](int r) -> uint32_t { return r < r1 ? rows[r] : INV; };
  // split bin at row position p: from the histogram pass's scratch if the final round's
  // group produced the best split (st.best_j >= 0), else gathered from the table -- its
  // feature-major copy when present (a node's rows are sorted: lanes read neighbouring bytes
  // of one feature line instead of one row line each)
  const int bj = st.scr_id > 0 ? (st.best_feat < st.scr_id ? st.best_feat : -1)
                               : (st.best_pos < st.scr_n ? st.best_pos : -1);
  const uint8_t* xfeat = c.XbT ? c.XbT + (int64_t)feat * c.n : nullptr;
  auto bin_of = [&](int p, uint32_t row) -> int {
    if (row == INV) return 0;
    if (bj >= 0) return (int)c.bscr[(st.on.start + p) * 16 + bj];
    if (xfeat) return (int)xfeat[row & c.rmask];
    return (int)c.Xb[(int64_t)(row & c.rmask) * c.ld + feat];
  };
  // regression: sum w y2q of the left rows (k_large_finish completes the left child's sums),
  // accumulated in pass 1 from targets fetched one step ahead with the split bins -- fetched
  // unconditionally (an absent row reads row 0): a target load under the left-row mask, used
  // at once, would wait for every older load (vmcnt(0)), i.e. for the prefetched steps too
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  const float* ty = c.is_reg ? tree_y(c, s) : nullptr;
  auto y_of = [&](uint32_t row) -> float { return ty ? ty[(row != INV ? row : 0u) & c.rmask] : 0.0f; };
  unsigned long long lyy = 0ull;
  int myL = 0;
  {
    uint32_t ra = row_at(r0 + tid);
    int ba = bin_of(r0 + tid, ra);
    float ya = y_of(ra);
    uint32_t rbn = row_at(r0 + tid + 256);
    for (int t0 = r0; t0 < r1; t0 += 256) {
      const int bb = bin_of(t0 + 256 + tid, rbn);
      const float yb = y_of(rbn);
      const uint32_t rc2 = row_at(t0 + 512 + tid);
      const bool left = ra != INV && ba <= bin;
      const uint64_t ml = __ballot(left);
      if (lane == 0) lflag[(t0 - r0) / 64 + wid] = ml;
      myL += left ? 1 : 0;
      if (ty && left) {
        int64_t yq, y2q;
        reg_quantize(ya, c.rq, yq, y2q);
        lyy += (unsigned long long)((int64_t)word_weight(c, s, ra) * y2q);
      }
      ra = rbn; ba = bb; ya = yb; rbn = rc2;
    }
  }
  if (ty) {   // exact integer sum: any order
    lyy = (unsigned long long)wave::sum<uint64_t>((uint64_t)lyy, lane);
    if (lane == 0 && lyy) atomicAdd(&c.lyy[slot], lyy);
  }
  // block totals -> one atomic pair for the whole chunk
  for (int m = 32; m >= 1; m >>= 1) myL += __shfl_xor(myL, m);
  if (lane == 0) wcnt[wid] = myL;
  __syncthreads();
  if (tid == 0) {
    const int totL = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    const int totR = (r1 - r0) - totL;
    tbase[0] = atomicAdd(&c.lcursor[2 * slot], totL);
    tbase[1] = atomicAdd(&c.lcursor[2 * slot + 1], totR);
  }
  __syncthreads();
  int baseL = tbase[0], baseR = tbase[1];
  // row ids of DML_PART_U2 256-row steps are loaded (clamped, unconditionally) before the
  // steps' stores: consecutive steps do not each wait a memory round trip
  constexpr int U2 = DML_PART_U2;
  uint32_t rq[U2];
  for (int t0 = r0; t0 < r1; t0 += 256) {
    const int r = t0 + tid;
    const bool valid = r < r1;
    const int uq = ((t0 - r0) >> 8) % U2;
    if (uq == 0) {
#pragma unroll
      for (int u = 0; u < U2; ++u) rq[u] = rows[min(r + 256 * u, r1 - 1)];
    }
    uint32_t row = rq[0];
#pragma unroll
    for (int u = 1; u < U2; ++u) if (uq == u) row = rq[u];
    const int wi = (t0 - r0) / 64;
    const uint64_t ml = lflag[wi + wid];
    const uint64_t vm = valid ? ~0ull : 0ull;
    const uint64_t mvalid = __ballot(valid);
    const uint64_t mr = mvalid & ~ml;
    int offL = 0, offR = 0, totL = 0, totR = 0;
    for (int w = 0; w < 4; ++w) {
      const uint64_t lw = lflag[wi + w];
      const int nvw = max(0, min(64, r1 - (t0 + 64 * w)));
      const uint64_t vw = nvw >= 64 ? ~0ull : ((1ull << nvw) - 1ull);
      const int cl = __popcll(lw), cr = __popcll(vw & ~lw);
      if (w < wid) { offL += cl; offR += cr; }
      totL += cl; totR += cr;
    }
    (void)vm;
    if (valid) {
      if ((ml >> lane) & 1ull) out[baseL + offL + lane_prefix(ml)] = row;
      else out[nl + baseR + offR + lane_prefix(mr)] = row;
    }
    baseL += totL; baseR += totR;
  }
}

// regression large nodes after the partition: the left child's sum w y2q completes the
// best split's statistics, then the split is accepted or the node stays a leaf (its
// partitioned range is then unused)
__global__ __launch_bounds__(64) void k_large_finish(Ctx c, int set_cur) {
  const int slot = blockIdx.x;
  if (threadIdx.x != 0) return;
  LState& st = c.lstate[slot];
  if (st.split != 2) return;
  const NodeSpec s = spec_of<-1>(c, st.on.tree);
  double* best_left = c.lbest_left + (int64_t)slot * c.CH;
  best_left[2] = reg_s2(c.lyy[slot], c.rq);
  large_commit(c, s, st, slot, best_left, set_cur);
}

// ------------------------------------------------------------------------------------
// tree roots: active-row count, fill, root statistics
// ------------------------------------------------------------------------------------
// A block counts 1024 rows for kCntG trees: the row half of the bootstrap hash
// (hash_u32's inner splitmix64 of the row counter) is the same for every tree, so it is
// computed once per row and group, and "weight > 0" is one compare against the smallest
// Poisson threshold instead of the whole inverse-CDF table (exactly boot_weight(...) > 0).
constexpr int kCntG = 8;
__global__ __launch_bounds__(256) void k_count_active(Ctx c, int T) {
  const int t0 = blockIdx.y * kCntG;
  const int r0 = blockIdx.x * 1024;
  uint64_t inner[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    inner[i] = boot_row_key((uint32_t)(r0 + i * 256 + threadIdx.x));
  __shared__ int red[kCntG][4];
  for (int g = 0; g < kCntG; ++g) {
    const int t = t0 + g;
    int cnt = 0;
    if (t < T) {   // block-uniform
      const NodeSpec s = spec_of<-1>(c, t);
      const uint8_t* role = c.roles + (int64_t)s.split * c.n;
      uint32_t tmin = s.pois_cdf[0];
      for (int j = 1; j < kPoisTable; ++j) tmin = min(tmin, s.pois_cdf[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + i * 256 + threadIdx.x;
        if (r < c.n && role[r] == 1) {
          bool on = true;
          if (s.bootstrap) {
            const uint32_t u = (uint32_t)(splitmix64(s.seed ^ inner[i]) >> 32);
            on = s.bootstrap == 2 ? u < s.pois_cdf[0] : u >= tmin;
          }
          cnt += on;
        }
      }
    }
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0) red[g][threadIdx.x >> 6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x < kCntG && t0 + (int)threadIdx.x < T) {
    const int g = threadIdx.x;
    const int tot = red[g][0] + red[g][1] + red[g][2] + red[g][3];
    if (tot) atomicAdd(&c.active_count[t0 + g], tot);
  }
}

template <bool REG>
__global__ __launch_bounds__(256) void k_fill_active(Ctx c) {
  const int t = blockIdx.y;
  const NodeSpec s = spec_of<-1>(c, t);
  const uint8_t* role = c.roles + (int64_t)s.split * c.n;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ int wcnt[16];
  __shared__ int base_s;
  __shared__ double acc[kMaxClasses];
  __shared__ unsigned long long racc[3];   // regression: integer sums w, w yq, w y2q
  for (int k = tid; k < kMaxClasses; k += 256) acc[k] = 0.0;
  if (tid < 3) racc[tid] = 0ull;
  const int r0 = blockIdx.x * 1024;
  uint32_t wts[4];
  bool act[4];
  int mine = 0;
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + tid * 4 + i;
    wts[i] = (r < c.n && role[r] == 1) ? boot_weight(s, (uint32_t)r) : 0u;
    act[i] = wts[i] > 0;
    mine += act[i];
  }
  // block exclusive scan of `mine` (rows stay in ascending order inside the block)
  int incl = mine;
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off);
    if (lane >= off) incl += o;
  }
  if (lane == 63) wcnt[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    int tot = 0;
    for (int w = 0; w < 4; ++w) { const int v = wcnt[w]; wcnt[8 + w] = tot; tot += v; }
    base_s = tot ? atomicAdd(&c.cursors[t], tot) : 0;
  }
  __syncthreads();
  int p = base_s + wcnt[8 + wid] + incl - mine;
  uint32_t* out = c.rows_cur + c.row_off[t];
  // root sums: per-thread integer partials, one wave reduction, ONE LDS atomic per wave and
  // channel (a per-row atomic on the same 2-3 addresses serialises every lane of the wave)
  constexpr int kCW = 8;
  uint32_t cw8[kCW] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  uint64_t rs0 = 0ull, rs1 = 0ull, rs2 = 0ull;
  for (int i = 0; i < 4; ++i) {
    if (!act[i]) continue;
    const uint32_t r = (uint32_t)(r0 + tid * 4 + i);
    uint32_t wd = r;
    if (c.packed) {
      wd |= wts[i] << c.rbits;
      if constexpr (!REG) wd |= (uint32_t)c.ycls[r] << (c.rbits + 4);
    }
    out[p++] = wd;
    if constexpr (REG) {
      const RegPL q = reg_payload(c, wts[i], tree_y(c, s)[r]);
      rs0 += (uint64_t)wts[i]; rs1 += (uint64_t)q.wy; rs2 += (uint64_t)q.wyy;
    } else {
      const int y = c.ycls[r];
      if (c.C <= kCW) {
#pragma unroll
        for (int k = 0; k < kCW; ++k) cw8[k] += (k == y) ? wts[i] : 0u;
      } else {
        atomicAdd(&acc[y], (double)wts[i]);
      }
    }
  }
  if constexpr (REG) {
    rs0 = wave::sum<uint64_t>(rs0, lane); rs1 = wave::sum<uint64_t>(rs1, lane); rs2 = wave::sum<uint64_t>(rs2, lane);
    if (lane == 0) {
      if (rs0) atomicAdd(&racc[0], (unsigned long long)rs0);
      if (rs1) atomicAdd(&racc[1], (unsigned long long)rs1);
      if (rs2) atomicAdd(&racc[2], (unsigned long long)rs2);
    }
  } else if (c.C <= kCW) {
#pragma unroll
    for (int k = 0; k < kCW; ++k) {
      if (k >= c.C) break;
      const uint32_t v = wave::sum<uint32_t>(cw8[k], lane);   // integer class weights: exact
      if (lane == 0 && v) atomicAdd(&acc[k], (double)v);
    }
  }
  __syncthreads();
  if constexpr (REG) {
    if (tid < 3 && racc[tid]) atomicAdd(&c.rsum[(int64_t)t * 3 + tid], racc[tid]);
  } else {
    for (int k = tid; k < c.VC; k += 256)
      if (acc[k] != 0.0) atomicAdd(&c.node_val[(int64_t)t * c.VC + k], acc[k]);
  }
}

__global__ void k_init_counters(Ctx c) { c.counters[kPool] = c.T; }

// per-level setup in one launch: zero the next level's open-list counters (set `set`) and,
// pool >= 0, publish the level's node-pair reservation -- replaces a memset and a host->device
// copy, i.e. two of the commands the host issues one by one while the GPU waits right after
// the level's count read-back
__global__ void k_level_setup(Ctx c, int set, int pool) {
  const int i = threadIdx.x;
  if (i < kTiers) c.counters[set * kTiers + i] = 0;
  if (i == kTiers && pool >= 0) c.counters[kPool] = pool;
}

// Buckets one level's staged wave/block-tier children into the next level's open lists.
// 1024 staging slots per workgroup; each tier's positions come from wave scans and ONE atomic
// per tier per workgroup, and the subtree tier's node pairs (subtree_max_splits) are reserved
// here the same way (one pool atomic per workgroup) and handed over in OpenNode::pool_base.
// Open-list order within a workgroup follows the staging order; across workgroups it is the
// atomics' order (node numbering was never order-independent; tree shapes are).
__global__ __launch_bounds__(256) void k_compact(Ctx c, int set, int64_t n) {
  constexpr int NQ = kTiers + 1;   // per-tier entries + subtree pool slots
  __shared__ int wtot[4][NQ];
  __shared__ int gbase[NQ];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * 1024 + tid * 4;
  OpenNode e[4];
  int want[4];
  int cnt[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) cnt[q] = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    want[u] = 0;
    e[u].tier = -1;
    if (i0 + u < n) e[u] = c.stage[i0 + u];
    const int t = e[u].tier;
    if (t < 0) continue;
    ++cnt[t];
    if (t == 0 || t == 4 || (t == 1 && c.bigsub_max > 0)) {   // whole-subtree tiers: every pair reserved here
      want[u] = 2 * subtree_max_splits(c.specs[e[u].tree], e[u].count, e[u].depth);
      cnt[kTiers] += want[u];
    }
  }
  int off[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int inc = wave::incl_scan<int>(cnt[q]);
    off[q] = inc - cnt[q];
    if (lane == 63) wtot[wid][q] = inc;
  }
  __syncthreads();
  if (tid < NQ) {
    int tot = 0;
    for (int w = 0; w < 4; ++w) {
      const int v = wtot[w][tid];
      wtot[w][tid] = tot;
      tot += v;
    }
    int* ctr = tid < kTiers ? &c.counters[set * kTiers + tid] : &c.counters[kPool];
    gbase[tid] = tot ? atomicAdd(ctr, tot) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NQ; ++q) off[q] += gbase[q] + wtot[wid][q];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = e[u].tier;
    if (t < 0) continue;
    int idx = 0;
#pragma unroll
    for (int q = 0; q < kTiers; ++q)
      if (q == t) idx = off[q]++;
    if (t == 0 || t == 4 || (t == 1 && c.bigsub_max > 0)) {
      const int pb = off[kTiers];
      off[kTiers] += want[u];
      if (want[u] > 0 && (int64_t)pb + want[u] > c.pool_cap) {
        atomicOr(&c.counters[kOverflow], 1);
        e[u].pool_base = -2;
      } else {
        e[u].pool_base = pb;
      }
    }
    if (idx >= c.open_cap[t]) {
      atomicOr(&c.counters[kOpenOvf], 1);
      continue;
    }
    c.open[set][t][idx] = e[u];
  }
}

// monotonic_cst: clip every node's value to its bounds once the trees are grown (the host
// builder clips every node of a build that has a constraint table, forest_cpu.cpp)
__global__ void k_mono_clip(Ctx c, int64_t P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  mono_clip(c.node_val + i * c.VC, c.is_reg, c.nbound[2 * i], c.nbound[2 * i + 1]);
}

__global__ void k_roots(Ctx c) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= c.T) return;
  NodeRec leaf; leaf.split = -1; leaf.left = -1;
  c.nodes[t] = leaf;
  if (c.is_reg) {   // integer root sums -> the double channels (forest_common.h)
    const unsigned long long* q = c.rsum + (int64_t)t * 3;
    double* v = c.node_val + (int64_t)t * c.VC;
    v[0] = (double)q[0]; v[1] = reg_s1(q[1], c.rq); v[2] = reg_s2(q[2], c.rq);
  }
  if (!c.is_reg && c.cw && c.specs[t].cw_mode) {
    double* row = const_cast<double*>(c.cw) + (int64_t)t * c.C;
    double* v = c.node_val + (int64_t)t * c.VC;
    if (c.specs[t].cw_mode == 2) balanced_weights(v, c.C, row);   // from this tree's bootstrap counts
    for (int k = 0; k < c.C; ++k) v[k] *= row[k];
  }
  c.tree_W[t] = node_weight(c, t);
  {   // min_weight_fraction_leaf -> absolute weight, read by every later kernel of the build
    TreeSpec& sm = const_cast<TreeSpec&>(c.specs[t]);
    sm.min_weight_leaf = sm.min_weight_frac * c.tree_W[t];
  }
  const int cnt = c.active_count[t];
  if (cnt == 0) return;
  enqueue_or_leaf(c, t, t, c.row_off[t], cnt, 0, root_key(c.specs[t].seed), 0);
}

// ------------------------------------------------------------------------------------
// host orchestration
// ------------------------------------------------------------------------------------
static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Layout {
  size_t rows_b, open[2][kTiers], stage, counters, cursors, lstate, lperm, lbest, ghist, lcursor, lyy, bscr, rsum, total;
  int64_t stage_cap;
  int64_t open_cap[kTiers], large_cap;
};

static int build_mode(const ForestArgs* a) { return a->is_reg ? 2 : (a->n_classes == 2 ? 1 : 0); }

static size_t mode_elem(int mode) { return mode == 0 ? 4 : 8; }

// bytes of one feature's large-tier GLOBAL histogram: u32 [CH][256] (classification,
// binary unpacked), u64 [3][256] (regression integer planes)
// bytes per feature of a large-tier global histogram (large_planes: no y^2 plane)
static size_t ghist_feat_bytes(int mode, int CH) { return mode == 2 ? (size_t)2 * 256 * 8 : (size_t)CH * 256 * 4; }

static Layout plan(const ForestArgs* a) {
  Layout L{};
  const int64_t R = a->rows_total, T = a->T;
  const int64_t C = a->is_reg ? 3 : a->n_classes;
  const int64_t CH = a->is_reg ? 4 : a->n_classes + 1;
  // a level's nodes hold disjoint rows: <= R / (smallest node of the tier) of each tier.
  // Subtree-tier nodes are roots or children of the previous level's wave/block/large nodes.
  L.open_cap[1] = R / (a->sub_max + 1) + T + 16;
  L.open_cap[2] = R / (a->wave_max + 1) + T + 16;
  L.open_cap[3] = R / (a->block_max + 1) + T + 16;
  L.open_cap[0] = 2 * (L.open_cap[1] + L.open_cap[2] + L.open_cap[3]) + T + 16;
  L.open_cap[4] = L.open_cap[0];
  L.large_cap = L.open_cap[3];
  L.stage_cap = 2 * (L.open_cap[1] + L.open_cap[2]);
  (void)C;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
  L.rows_b = take((size_t)R * 4);
  for (int s = 0; s < 2; ++s)
    for (int t = 0; t < kTiers; ++t) L.open[s][t] = take((size_t)L.open_cap[t] * sizeof(OpenNode));
  L.stage = take((size_t)L.stage_cap * sizeof(OpenNode));
  L.counters = take(kNumCounters * 4);
  L.cursors = take((size_t)T * 4);
  L.lstate = take((size_t)L.large_cap * sizeof(LState));
  L.lperm = take((size_t)L.large_cap * a->d * 2);
  L.lbest = take((size_t)L.large_cap * CH * 8);
  L.ghist = take((size_t)L.large_cap * a->kg_large * ghist_feat_bytes(build_mode(a), (int)CH));
  L.lcursor = take((size_t)L.large_cap * 8);
  L.lyy = take((size_t)L.large_cap * 8);
  L.bscr = take((size_t)R * 16);
  L.rsum = take((size_t)T * 3 * 8);
  L.total = off;
  return L;
}

static size_t fused_lds(const ForestArgs* a, int KG) {
  const int CH = a->is_reg ? 4 : (int)a->n_classes + 1;
  const int mode = build_mode(a);
  const int span = hist_planes(mode, CH) * 256;
  return fused_layout(KG, span, (int)mode_elem(mode), CH).total + 16;
}

static size_t sub_lds(const ForestArgs* a, int SR = 64, bool lite = false) {
  const int VC = a->is_reg ? 3 : (int)a->n_classes;
  size_t b = SR * (lite ? sizeof(SubEntryLite) : sizeof(SubEntry)) + (size_t)SR * VC * 8 + ((2 * VC + 1) & ~1) * 8;
  b += (size_t)((SR * a->sub_cache_d + 15) & ~15) + 64 * 4 + 16;   // row-bin cache + compaction map
  return b;
}

static Ctx make_ctx(const ForestArgs* a, const Layout& L) {
  Ctx c{};
  unsigned char* ws = (unsigned char*)a->workspace;
  c.Xb = (const uint8_t*)a->Xb; c.ld = a->ld; c.n = (int)a->n; c.d = (int)a->d;
  c.is_reg = (int)a->is_reg;
  c.C = c.is_reg ? 1 : (int)a->n_classes;
  c.CH = c.is_reg ? 4 : (int)a->n_classes + 1;
  c.VC = c.is_reg ? 3 : (int)a->n_classes;
  c.ycls = (const int32_t*)a->ycls; c.yreg = (const float*)a->yreg;
  c.ystride = a->ystride;
  c.roles = (const uint8_t*)a->roles; c.specs = (const TreeSpec*)a->specs; c.T = (int)a->T;
  c.active_count = (int32_t*)a->active_count; c.row_off = (const int64_t*)a->row_off;
  c.nodes = (NodeRec*)a->nodes; c.node_val = (double*)a->node_val; c.pool_cap = a->pool_cap;
  c.tree_W = (double*)a->tree_W;
  c.rows_next = (uint32_t*)(ws + L.rows_b);
  for (int s = 0; s < 2; ++s)
    for (int t = 0; t < kTiers; ++t) c.open[s][t] = (OpenNode*)(ws + L.open[s][t]);
  for (int t = 0; t < kTiers; ++t) c.open_cap[t] = L.open_cap[t];
  c.stage = (OpenNode*)(ws + L.stage);
  c.counters = (int32_t*)(ws + L.counters);
  c.cursors = (int32_t*)(ws + L.cursors);
  c.lstate = (LState*)(ws + L.lstate);
  c.lperm = (int16_t*)(ws + L.lperm);
  c.lbest_left = (double*)(ws + L.lbest);
  c.ghist = (void*)(ws + L.ghist);
  c.lcursor = (int32_t*)(ws + L.lcursor);
  c.lyy = (unsigned long long*)(ws + L.lyy);
  c.bscr = ws + L.bscr;
  c.rsum = (unsigned long long*)(ws + L.rsum);
  c.mono = (const int8_t*)a->mono;
  c.nbound = a->mono ? (double*)a->nbound : nullptr;
  c.rq = reg_scale((int)a->yq_e1, (int)a->yq_e2);
  c.XbT = (const uint8_t*)a->XbT;
  c.cw = (const double*)a->cw;
  c.large_cap = L.large_cap;
  c.wave_max = (int)a->wave_max; c.block_max = (int)a->block_max; c.chunk = (int)a->chunk;
  c.kg_wave = (int)a->kg_wave; c.kg_block = (int)a->kg_block; c.kg_large = (int)a->kg_large;
  // row windows: opt-in (DML_LARGE_FM_DIV=8: +12 % on a single config-6 job after the warmup fit,
  // but back-to-back jobs gain nothing and their histogram kernels run ~25 % longer under three
  // concurrent lanes -- the sparse levels then touch the row-major table AND the feature-major
  // copy; profiles/r6_gbrt_cfg6_row_windows.txt)
  c.fm_div = getenv("DML_LARGE_FM_DIV") ? atoi(getenv("DML_LARGE_FM_DIV")) : 0;
  // row-window rounds kg_rw features wide (DML_LARGE_KG_RW: a multiple of 16, <= 32; 0 = kg_large)
  c.kg_rw = getenv("DML_LARGE_KG_RW") ? atoi(getenv("DML_LARGE_KG_RW")) : 0;
  if (c.kg_rw < 0 || c.kg_rw > DML_KGW_LARGE || (c.kg_rw & 15) != 0 || !c.is_reg || !c.fm_div) c.kg_rw = 0;
  c.large_compact = (c.is_reg && a->large_unit && a->kg_large <= DML_KGL_LARGE && !getenv("DML_LARGE_NO_COMPACT")) ? 1 : 0;
  c.large_pack = (c.large_compact && a->large_pack && a->chunk <= 4095 && !getenv("DML_LARGE_NO_PACK")) ? 1 : 0;
  c.slack_wave = (int)a->slack_wave;
  c.sub_max = (int)a->sub_max;
  c.sub_cache_d = (int)a->sub_cache_d;
  c.bigsub_max = 0;   // set by build_impl for the builds it applies to
  c.sub_small = (a->sub_small > 0 && a->sub_small < a->sub_max && a->sub_small <= 32) ? (int)a->sub_small : 0;
  {
    int cbits = 0;
    if (!c.is_reg)
      while ((1 << cbits) < c.C) ++cbits;
    c.rbits = 28 - cbits;   // 4 weight bits (bootstrap weights <= kPoisTable = 12)
    c.packed = (a->n < ((int64_t)1 << c.rbits) - 1) && getenv("DML_ROW_WORDS_OFF") == nullptr ? 1 : 0;
    c.rmask = c.packed ? (uint32_t)((1u << c.rbits) - 1u) : 0xFFFFFFFFu;
  }
  return c;
}

static int g_last_err_line = 0;
static hipError_t g_last_err = hipSuccess;
#define HIP_OK(x)                                       \
  do {                                                  \
    hipError_t e_ = (x);                                \
    if (e_ != hipSuccess) {                             \
      g_last_err = e_; g_last_err_line = __LINE__;      \
      return 100 + (int)e_;                             \
    }                                                   \
  } while (0)

// build LANES: independent builds driven concurrently from different host threads, each on
// its own stream (boosting runs its fits in two lanes so one lane's kernels fill the GPU while
// the other's host thread waits on a level read-back).  Every host-side resource of a build --
// side streams, pinned read-back words, whole-histogram buffers, early-predict stream -- is
// per (lane, device); a thread selects its lane with dml_forest_set_lane (default 0).
constexpr int kLanes = 4;
static thread_local int t_lane = 0;

// side streams so the four node tiers of a level overlap (their tails otherwise
// serialise: a level's few large nodes leave most CUs idle while small nodes wait)
struct SideStreams {
  hipStream_t s[3] = {nullptr, nullptr, nullptr};
  hipEvent_t fork = nullptr, join[3] = {nullptr, nullptr, nullptr};
  bool ok = false;
};

static SideStreams* side_streams() {
  static SideStreams lanes[kLanes];
  SideStreams& ss = lanes[t_lane];
  if (!ss.ok) {
    bool good = hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) == hipSuccess;
    // DML_TIER_PRIO: stream priorities of the (subtree, wave, block) tier streams as 3 digits,
    // 0 = normal, 1 = high (e.g. "001": the block tier -- the level's critical path -- first)
    const char* pr = getenv("DML_TIER_PRIO");
    int lo_pr = 0, hi_pr = 0;
    if (hipDeviceGetStreamPriorityRange(&lo_pr, &hi_pr) != hipSuccess) lo_pr = hi_pr = 0;
    for (int i = 0; i < 3 && good; ++i) {
      const bool high = pr && (int)strlen(pr) > i && pr[i] == '1';
      good = hipStreamCreateWithPriority(&ss.s[i], hipStreamNonBlocking, high ? hi_pr : lo_pr) == hipSuccess &&
             hipEventCreateWithFlags(&ss.join[i], hipEventDisableTiming) == hipSuccess;
    }
    ss.ok = good;
    if (!good) return nullptr;
  }
  return &ss;
}

static hipEvent_t pred_event() {
  static hipEvent_t ev[kLanes] = {};
  hipEvent_t& e = ev[t_lane];
  if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
  return e;
}

// stream of the early per-fit predicts (forest.hip build_impl)
static hipStream_t pred_stream() {
  static hipStream_t st[kLanes] = {};
  hipStream_t& s = st[t_lane];
  if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
  return s;
}

static int32_t* pinned_counters() {
  static int32_t* pl[kLanes] = {};
  int32_t*& p = pl[t_lane];
  if (!p) {
    if (hipHostMalloc((void**)&p, 64 * sizeof(int32_t), hipHostMallocDefault) != hipSuccess) p = nullptr;
  }
  return p;
}

// whole-histogram large levels: two per-parity node-histogram buffers and two pinfo
// tables per device, grown on demand (outside the Python-sized workspace: their size
// follows the level's large-node count, known only at run time)
struct FullBufs {
  void* gf[2] = {nullptr, nullptr};
  size_t gf_bytes[2] = {0, 0};
  int4* pinfo = nullptr;   // [2][pi_cap]
  int64_t pi_cap = 0;
  void* fr = nullptr;      // k_split_full's per-(node, position) candidates
  size_t fr_bytes = 0;
};
static FullBufs g_full_bufs[kLanes][16];
static FullBufs* full_bufs(int lane = -1) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  return &g_full_bufs[lane < 0 ? t_lane : lane][dev];
}
static bool ensure_bytes(void*& p, size_t& have, size_t need) {
  if (have >= need) return true;
  if (p) { (void)hipFree(p); p = nullptr; have = 0; }
  const size_t want = need + need / 4;
  if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; return false; }
  have = want;
  return true;
}

// free the current device's whole-histogram buffers (ops/forest_ops.py _Arena.clear: another
// family needs the HBM); the next whole-histogram level allocates them again
static int release_full_bufs() {
  for (int lane = 0; lane < kLanes; ++lane) {
  FullBufs* b = full_bufs(lane);
  if (!b) return 0;
  if (b->gf[0] || b->gf[1] || b->pinfo || b->fr) {
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    for (int i = 0; i < 2; ++i) {
      if (b->gf[i]) (void)hipFree(b->gf[i]);
      b->gf[i] = nullptr;
      b->gf_bytes[i] = 0;
    }
    if (b->pinfo) (void)hipFree(b->pinfo);
    b->pinfo = nullptr;
    b->pi_cap = 0;
    if (b->fr) (void)hipFree(b->fr);
    b->fr = nullptr;
    b->fr_bytes = 0;
  }
  }
  return 0;
}

}  // namespace dml

using namespace dml;

extern "C" int dml_forest_release_scratch() { return release_full_bufs(); }
// the calling host thread's build lane (0 .. kLanes-1); returns the lane count
extern "C" int dml_forest_set_lane(int lane) {
  if (lane < 0 || lane >= kLanes) return -1;
  t_lane = lane;
  return kLanes;
}

// kernel-level test hooks (tests/test_forest_gpu.py): wave primitives vs ds_bpermute
// out layout per block of 64: [sorted | scan | xor1 | xor2 | xor4 | xor8 | xor16 | xor32 |
//                             argmax idx | shift_down1 | min]
__global__ void k_test_wave_prims(const uint32_t* in, uint32_t* out) {
  const int lane = threadIdx.x;
  const uint32_t v = in[blockIdx.x * 64 + lane];
  uint32_t* o = out + (size_t)blockIdx.x * 64 * 11;
  o[0 * 64 + lane] = wave::bitonic64(v, lane);
  o[1 * 64 + lane] = wave::incl_scan<uint32_t>(v);
  o[2 * 64 + lane] = wave::xor32<1>(v, lane);
  o[3 * 64 + lane] = wave::xor32<2>(v, lane);
  o[4 * 64 + lane] = wave::xor32<4>(v, lane);
  o[5 * 64 + lane] = wave::xor32<8>(v, lane);
  o[6 * 64 + lane] = wave::xor32<16>(v, lane);
  o[7 * 64 + lane] = wave::xor32<32>(v, lane);
  double g = (double)(v % 97u);
  int idx = lane;
  wave::argmax(g, idx, lane);
  o[8 * 64 + lane] = (uint32_t)idx;
  o[9 * 64 + lane] = (uint32_t)wave::shift_down1<int>((int)v, lane, -1);
  o[10 * 64 + lane] = (uint32_t)wave::min_u64(((uint64_t)v << 32) | (uint32_t)lane, lane);
}

struct PredictArgs;
extern "C" int dml_forest_predict_fit(const PredictArgs* a, int32_t f, hipStream_t st);

extern "C" {

int dml_forest_phase_stats(unsigned long long* out) {
#ifdef DML_PHASE_PROF
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 32) != hipSuccess) return 1;
  unsigned long long z[32] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return 1;
  return 0;
#else
  (void)out;
  return 2;
#endif
}

int dml_test_wave_prims(const uint32_t* in, uint32_t* out, int64_t nblocks, hipStream_t st) {
  k_test_wave_prims<<<(unsigned)nblocks, 64, 0, st>>>(in, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

const char* dml_forest_last_error(int* line) {
  if (line) *line = g_last_err_line;
  return hipGetErrorString(g_last_err);
}

int dml_forest_sizeof_treespec() { return (int)sizeof(TreeSpec); }
int dml_forest_sizeof_args() { return (int)sizeof(ForestArgs); }
int dml_forest_sizeof_node() { return (int)sizeof(NodeRec); }

// bytes of workspace the build needs (rows_total, d, classes, tiers must be set);
// the rows_a buffer (rows_total uint32) is carved right after it.
int64_t dml_forest_workspace_bytes(const ForestArgs* a) {
  Layout L = plan(a);
  return (int64_t)(L.total + align_up((size_t)a->rows_total * 4, 256));
}

// phase 1: count active (train & bootstrap weight > 0) rows per tree into a->active_count
int dml_forest_count(ForestArgs* a, hipStream_t st) {
  Ctx c{};
  c.n = (int)a->n; c.roles = (const uint8_t*)a->roles; c.specs = (const TreeSpec*)a->specs;
  c.active_count = (int32_t*)a->active_count;
  HIP_OK(hipMemsetAsync(c.active_count, 0, a->T * 4, st));
  dim3 grid((unsigned)((a->n + 1023) / 1024), (unsigned)((a->T + kCntG - 1) / kCntG));
  k_count_active<<<grid, 256, 0, st>>>(c, (int)a->T);
  HIP_OK(hipGetLastError());
  return 0;
}

}  // extern "C"

// level loop for one histogram mode (0 cls, 1 packed binary, 2 regression)
template <int MODE>
static int build_impl(ForestArgs* a, hipStream_t st) {
  constexpr bool REG = MODE == 2;
  constexpr int GM = MODE == 2 ? 2 : 0;  // global (large-tier) histogram layout
  // the criterion the node kernels are specialised on (gini / squared_error builds)
  constexpr int FCX = REG ? kMSE : kGini;
  Layout L = plan(a);
  if ((size_t)a->workspace_bytes < (size_t)dml_forest_workspace_bytes(a)) return 2;
  Ctx c = make_ctx(a, L);
  const bool fast = a->fast_crit == FCX + 1 && c.packed;   // PK kernels assume packed row words
  // big-subtree tier (binary): the caller sized tier 1 for it (wave_max <= bigsub_max <= 256)
  const bool big = MODE == 1 && a->bigsub_max > 0;
  if (big && (a->bigsub_max > 256 || a->wave_max > a->bigsub_max || a->sub_cache_d <= 0 || a->mono || a->n_classes != 2))
    return 12;
  if (big) c.bigsub_max = (int)a->bigsub_max;
  const size_t lds_big = big ? big_layout((int)a->bigsub_max, (int)a->sub_cache_d).total + 16 : 0;
  uint32_t* rows_a = (uint32_t*)(((unsigned char*)a->workspace) + L.total);
  c.rows_cur = rows_a;
  int32_t* h = pinned_counters();
  if (!h) return 3;
  const bool reg = REG;
  if (!reg && (a->n_classes < 1 || a->n_classes > kMaxClasses)) return 5;
  if (a->d > 32767) return 6;

  HIP_OK(hipMemsetAsync(c.counters, 0, kNumCounters * 4, st));
  HIP_OK(hipMemsetAsync(c.cursors, 0, a->T * 4, st));
  HIP_OK(hipMemsetAsync(c.node_val, 0, (size_t)a->T * c.VC * 8, st));
  if (reg) HIP_OK(hipMemsetAsync(c.rsum, 0, (size_t)a->T * 3 * 8, st));
  k_init_counters<<<1, 1, 0, st>>>(c);
  dim3 gfill((unsigned)((a->n + 1023) / 1024), (unsigned)a->T);
  if (reg) k_fill_active<true><<<gfill, 256, 0, st>>>(c);
  else k_fill_active<false><<<gfill, 256, 0, st>>>(c);
  k_roots<<<(unsigned)((a->T + 255) / 256), 256, 0, st>>>(c);
  HIP_OK(hipGetLastError());

  const size_t lds_s = sub_lds(a);
  const size_t lds_s32 = sub_lds(a, 32);
  const size_t lds_sub_f = sub_lds(a, 64, true), lds_sub32_f = sub_lds(a, 32, true);   // k_subtree<REG, FCX>
  const size_t lds_w = fused_lds(a, (int)a->kg_wave);
  const size_t lds_b = fused_lds(a, (int)std::min<int64_t>(a->kg_block, DML_KGMAX_BLOCK));   // the kernel's KG
  const int CH = c.CH;
  // k_hist_large's dynamic LDS, optionally padded (DML_LARGE_LDS_MIN bytes) to cap its
  // workgroups per CU.  No padding: once the regression payload loads stopped draining the
  // gather pipeline (payload_fetch), two and more workgroups per CU beat one (GBRT config 6
  // 13.7 -> 14.9 CV-fits/s at 8192-row chunks; the 96-KB floor used before was measured on
  // the draining loop).
  const size_t lds_hl_floor = getenv("DML_LARGE_LDS_MIN") ? (size_t)atol(getenv("DML_LARGE_LDS_MIN")) : 0;
  const size_t lds_hl = std::max<size_t>((size_t)a->kg_large *
                                             (c.large_pack ? 256 : (c.large_compact ? 384 : large_planes(MODE, CH) * 256)) *
                                             mode_elem(MODE),
                                         std::min<size_t>(lds_hl_floor, 150 * 1024));
  // levels that can hold row-window nodes (below the top two) size the LDS for kg_rw-wide rounds
  const size_t lds_hl_rw = std::max<size_t>(lds_hl, (size_t)std::max<int>(c.kg_rw, (int)a->kg_large) *
                                                        (c.large_pack ? 256 : (c.large_compact ? 384 : large_planes(MODE, CH) * 256)) *
                                                        mode_elem(MODE));
  const size_t lds_sl = (size_t)a->kg_large * ghist_feat_bytes(MODE, CH) + a->kg_large * 16 + 16 +
                        (size_t)a->kg_large * CH * 8 + (size_t)a->kg_large * 8 + 64;
  const size_t lds_max = 160 * 1024;
  if (lds_w > lds_max || lds_b > lds_max || lds_sl > lds_max || lds_s > lds_max || lds_big > lds_max) return 7;
  if (a->sub_max > 64) return 9;
  {
    const int need = (int)std::max(std::max(std::max(lds_s, lds_w), std::max(lds_b, lds_sl)),
                                   std::max(lds_big, std::max(lds_hl, lds_hl_rw)));
    static int attr_set[3] = {0, 0, 0};
    if (need > 64 * 1024 && need > attr_set[MODE]) {
      HIP_OK(hipFuncSetAttribute((const void*)k_subtree<REG, -1>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_subtree<REG, FCX>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_nodes<64, MODE, -1>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_nodes<64, MODE, FCX>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_nodes<block_nt<MODE>(), MODE, -1>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_nodes<block_nt<MODE>(), MODE, FCX>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_hist_large<MODE, false>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_hist_large<MODE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      HIP_OK(hipFuncSetAttribute((const void*)k_split_large<GM>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      if constexpr (MODE == 1) {
        HIP_OK(hipFuncSetAttribute((const void*)k_bigsub<FCX>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
        HIP_OK(hipFuncSetAttribute((const void*)k_bigsub<-1>, hipFuncAttributeMaxDynamicSharedMemorySize, need));
      }
      attr_set[MODE] = need;
    }
  }
  const unsigned nchunks = (unsigned)((a->max_active + a->chunk - 1) / a->chunk);
  int cur = 0, levels = 0, large_rounds = 0;
  int fpar = 0;             // whole-histogram buffer parity of this level
  bool prev_full = false;   // the previous level kept its large nodes' whole histograms
  int64_t peak_open = 0;   // most open nodes of any level so far (early-predict tail rule)
  for (int i = 0; i < 4; ++i) a->tier_nodes_out[i] = 0;
  while (true) {
    HIP_OK(hipMemcpyAsync(h, c.counters, kNumCounters * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (h[kOpenOvf]) { a->status_out = 4; break; }
    const int ns = h[cur * kTiers + 0], nw = h[cur * kTiers + 1], nb = h[cur * kTiers + 2], nL = h[cur * kTiers + 3];
    const int ns4 = h[cur * kTiers + 4];
    if (ns + ns4 + nw + nb + nL == 0) break;
    if (++levels > 1 << 20) return 8;
    const int64_t open_now = (int64_t)ns + ns4 + nw + nb + nL;
    peak_open = std::max(peak_open, open_now);
    int level_pool = -1;   // k_level_setup below
    // reserve the child pairs of every wave/block-tier node of this level up front (a
    // big-subtree node's pairs were reserved with its subtree's: k_compact / k_bigsub)
    const int64_t pair_w = h[kPool], pair_b = pair_w + (big ? 0 : 2LL * nw), pool_next = pair_b + 2LL * nb;
    if (pool_next > a->pool_cap) {
      // pool overflow: the caller regrows with a bigger pool -- first make the stream wait for
      // any early predict still reading this pool / writing its outputs (their buffers are
      // freed and re-carved by the retry)
      if (a->early_pred && pred_stream()) {
        HIP_OK(hipEventRecord(pred_event(), pred_stream()));
        HIP_OK(hipStreamWaitEvent(st, pred_event(), 0));
      }
      a->status_out = 1;
      return 0;
    }
    if ((big ? 0 : nw) + nb) level_pool = (int)pool_next;
    k_level_setup<<<1, 64, 0, st>>>(c, 1 - cur, level_pool);
    a->tier_nodes_out[0] += ns + ns4; a->tier_nodes_out[1] += nw; a->tier_nodes_out[2] += nb; a->tier_nodes_out[3] += nL;
    SideStreams* ss = side_streams();
    static const bool serial_tiers = getenv("DML_SERIAL_TIERS") != nullptr;   // profiling: tiers one after another
    const bool fork = !serial_tiers && ss != nullptr && ((ns + ns4 > 0) + (nw > 0) + (nb > 0) + (nL > 0)) > 1;
    hipStream_t s0 = st, s1 = st, s2 = st;
    if (fork) {
      HIP_OK(hipEventRecord(ss->fork, st));
      for (int i = 0; i < 3; ++i) HIP_OK(hipStreamWaitEvent(ss->s[i], ss->fork, 0));
      s0 = ss->s[0]; s1 = ss->s[1]; s2 = ss->s[2];
    }
    // block-tier children stage after the wave tier's (none under the big-subtree tier)
    const int stage_b = big ? 0 : nw;
    // DML_BLOCK_FIRST: launch the block tier before the subtree / wave tiers
    static const bool block_first = getenv("DML_BLOCK_FIRST") && atoi(getenv("DML_BLOCK_FIRST")) != 0;
    if (block_first && nb) {
      if (fast) k_nodes<block_nt<MODE>(), MODE, FCX><<<nb, block_nt<MODE>(), lds_b, s2>>>(c, 2, cur, (int)pair_b, stage_b);
      else k_nodes<block_nt<MODE>(), MODE, -1><<<nb, block_nt<MODE>(), lds_b, s2>>>(c, 2, cur, (int)pair_b, stage_b);
    }
    const int nb_late = block_first ? 0 : nb;
    if (fast) {
      if (ns4) k_subtree<REG, FCX, 32><<<ns4, 64, lds_sub32_f, s0>>>(c, cur, 4);
      if (ns) k_subtree<REG, FCX><<<ns, 64, lds_sub_f, s0>>>(c, cur, 0);
      if (nw) {
        if constexpr (MODE == 1) {
          if (big) k_bigsub<FCX><<<nw, 256, lds_big, s1>>>(c, cur);
          else k_nodes<64, MODE, FCX><<<nw, 64, lds_w, s1>>>(c, 1, cur, (int)pair_w, 0);
        } else {
          k_nodes<64, MODE, FCX><<<nw, 64, lds_w, s1>>>(c, 1, cur, (int)pair_w, 0);
        }
      }
      if (nb_late) k_nodes<block_nt<MODE>(), MODE, FCX><<<nb, block_nt<MODE>(), lds_b, s2>>>(c, 2, cur, (int)pair_b, stage_b);
    } else {
      if (ns4) k_subtree<REG, -1, 32><<<ns4, 64, lds_s32, s0>>>(c, cur, 4);
      if (ns) k_subtree<REG, -1><<<ns, 64, lds_s, s0>>>(c, cur, 0);
      if (nw) {
        if constexpr (MODE == 1) {
          if (big) k_bigsub<-1><<<nw, 256, lds_big, s1>>>(c, cur);
          else k_nodes<64, MODE, -1><<<nw, 64, lds_w, s1>>>(c, 1, cur, (int)pair_w, 0);
        } else {
          k_nodes<64, MODE, -1><<<nw, 64, lds_w, s1>>>(c, 1, cur, (int)pair_w, 0);
        }
      }
      if (nb_late) k_nodes<block_nt<MODE>(), MODE, -1><<<nb, block_nt<MODE>(), lds_b, s2>>>(c, 2, cur, (int)pair_b, stage_b);
    }
    // whole-histogram level: every tree evaluates every feature and the level's node
    // histograms over all d features fit the budget -> keep them, and derive the larger of
    // two large siblings at the next level from its parent's (DML_LARGE_SUB=0: off)
    const size_t full_node_b = (size_t)a->d * ghist_feat_bytes(MODE, CH);
    const bool sub_on = !getenv("DML_LARGE_SUB") || atoi(getenv("DML_LARGE_SUB")) != 0;
    const double sub_gb = getenv("DML_LARGE_SUB_GB") ? atof(getenv("DML_LARGE_SUB_GB")) : 4.0;
    bool full = sub_on && nL > 0 && a->all_features && (double)nL * full_node_b <= sub_gb * 1e9;
    FullBufs* fb = full ? full_bufs() : nullptr;
    if (full && (!fb || !ensure_bytes(fb->gf[fpar], fb->gf_bytes[fpar], (size_t)nL * full_node_b))) full = false;
    if (full && fb->pi_cap < c.large_cap) {
      void* pp = fb->pinfo;
      size_t have = (size_t)fb->pi_cap * 2 * sizeof(int4);
      if (!ensure_bytes(pp, have, (size_t)c.large_cap * 2 * sizeof(int4))) { fb->pinfo = nullptr; fb->pi_cap = 0; full = false; }
      else { fb->pinfo = (int4*)pp; fb->pi_cap = (int64_t)(have / (2 * sizeof(int4))); prev_full = false; }
    }
    // k_split_full's candidate arrays: [nL][d] gain, mid, [CH] left sums (double), bin, nc (int)
    const size_t fr_per = (size_t)a->d * (16 + 8 * (size_t)CH + 8);
    if (full && !ensure_bytes(fb->fr, fb->fr_bytes, (size_t)nL * fr_per + 64)) full = false;
    c.full_cur = full ? 1 : 0;
    c.full_prev = (full && prev_full) ? 1 : 0;
    if (full) {
      const size_t nd = (size_t)nL * a->d;
      c.fr_g = (double*)fb->fr;
      c.fr_mid = c.fr_g + nd;
      c.fr_left = c.fr_mid + nd;
      c.fr_b = (int32_t*)(c.fr_left + nd * CH);
      c.fr_n = c.fr_b + nd;
      c.gf_cur = fb->gf[fpar];
      c.gf_prev = fb->gf[1 - fpar];
      c.pinfo_cur = fb->pinfo + (int64_t)fpar * fb->pi_cap;
      c.pinfo_next = fb->pinfo + (int64_t)(1 - fpar) * fb->pi_cap;
      c.pi_cap = fb->pi_cap;
    }
    // boosting root level with a root-count cache (roots only: every open node is a large root)
    const bool root_cache = MODE == 2 && full && levels == 1 && a->root_counts && nL == (int)a->T &&
                            ns + ns4 + nw + nb == 0;
    c.root_counts = root_cache ? (uint32_t*)a->root_counts : nullptr;
    c.root_cnt_skip = root_cache && a->root_counts_valid ? 1 : 0;
    if (nL && full) {
      k_large_prep<<<nL, 64, 0, st>>>(c, cur, nL);
      const int rounds = (int)((a->d + a->kg_large - 1) / a->kg_large);
      HIP_OK(hipMemsetAsync(c.gf_cur, 0, (size_t)nL * full_node_b, st));
      if (c.root_cnt_skip) k_root_counts<<<dim3((unsigned)nL, (unsigned)a->d), 256, 0, st>>>(c, 0);
      const dim3 gh = DML_LARGE_NODE_FAST ? dim3((unsigned)nL, nchunks) : dim3(nchunks, (unsigned)nL);
      // below the top two levels a node may be a row-window node with kg_rw-wide rounds: the
      // rounds' LDS covers kg_rw features (its later rounds exit at once for such nodes)
      Ctx cr = c;
      if (levels < 3) cr.kg_rw = 0;
      const size_t lds_round = cr.kg_rw > 0 ? lds_hl_rw : lds_hl;
      for (int round = 0; round < rounds; ++round) {
        ++large_rounds;
        if (c.packed) k_hist_large<MODE, true><<<gh, 256, lds_round, st>>>(cr, round);
        else k_hist_large<MODE, false><<<gh, 256, lds_round, st>>>(cr, round);
      }
      if (root_cache && !c.root_cnt_skip) {
        k_root_counts<<<dim3((unsigned)nL, (unsigned)a->d), 256, 0, st>>>(c, 1);
        a->root_counts_valid = 1;   // in/out: the cache now holds this active set's root counts
      }
      c.root_cnt_skip = 0;
      if (c.full_prev) {
        const int64_t per = (int64_t)a->d * large_planes(GM, CH) * 256;
        k_hist_derive<GM><<<dim3((unsigned)nL, (unsigned)((per + 1023) / 1024)), 256, 0, st>>>(c);
      }
      // every candidate in one launch (class planes staged in LDS: 4 features' worth, within
      // the default 64 KB; more classes than that keep the per-group rounds)
      const size_t lds_sf = (size_t)4 * ghist_feat_bytes(GM, CH);
      if (lds_sf <= 64 * 1024) {
        k_split_full<GM><<<dim3((unsigned)nL, (unsigned)((a->d + 3) / 4)), 256, lds_sf, st>>>(c);
        k_split_full_select<GM><<<nL, 64, 0, st>>>(c, cur);
      } else {
        for (int round = 0; round < rounds; ++round) k_split_large<GM><<<nL, 256, lds_sl, st>>>(c, cur);
      }
      const dim3 gp = DML_LARGE_NODE_FAST ? dim3((unsigned)nL, nchunks) : dim3(nchunks, (unsigned)nL);
      k_partition_large<<<gp, 256, (size_t)((a->chunk + 255) / 256) * 4 * 8, st>>>(c);
      if (reg) k_large_finish<<<nL, 64, 0, st>>>(c, cur);
    } else if (nL) {
      k_large_prep<<<nL, 64, 0, st>>>(c, cur, nL);
      const int fixed_rounds = a->all_features ? (int)((a->d + a->kg_large - 1) / a->kg_large) : 0;
      for (int round = 0;; ++round) {
        ++large_rounds;
        HIP_OK(hipMemsetAsync(c.ghist, 0, (size_t)nL * a->kg_large * ghist_feat_bytes(MODE, CH), st));
        HIP_OK(hipMemsetAsync(c.counters + kNeedMore, 0, 4, st));
        const dim3 gh = DML_LARGE_NODE_FAST ? dim3((unsigned)nL, nchunks) : dim3(nchunks, (unsigned)nL);
        if (c.packed) k_hist_large<MODE, true><<<gh, 256, lds_hl, st>>>(c, -1);
        else k_hist_large<MODE, false><<<gh, 256, lds_hl, st>>>(c, -1);
        k_split_large<GM><<<nL, 256, lds_sl, st>>>(c, cur);
        if (fixed_rounds) {   // every node visits every feature: the round count is known
          if (round + 1 >= fixed_rounds) break;
          continue;
        }
        HIP_OK(hipMemcpyAsync(h + 32, c.counters + kNeedMore, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (!h[32]) break;
      }
      const dim3 gp = DML_LARGE_NODE_FAST ? dim3((unsigned)nL, nchunks) : dim3(nchunks, (unsigned)nL);
      k_partition_large<<<gp, 256, (size_t)((a->chunk + 255) / 256) * 4 * 8, st>>>(c);
      if (reg) k_large_finish<<<nL, 64, 0, st>>>(c, cur);
    }
    if (fork) {
      for (int i = 0; i < 3; ++i) {
        HIP_OK(hipEventRecord(ss->join[i], ss->s[i]));
        HIP_OK(hipStreamWaitEvent(st, ss->join[i], 0));
      }
    }
    if ((big ? 0 : nw) + nb) {   // the staged children of the wave/block tiers -> next level's open lists
      const int64_t nst = 2LL * ((big ? 0 : nw) + nb);
      k_compact<<<(unsigned)((nst + 1023) / 1024), 256, 0, st>>>(c, 1 - cur, nst);
    }
    HIP_OK(hipGetLastError());
    // fits complete after this level: predict them now -- unless the build is in its tail (few
    // open nodes left): the predicts then have little tree work to hide behind and, sharing a
    // hardware queue with a tier stream, hold up the remaining levels; such fits stay marked
    // and are predicted after the build, all in one launch (ops/forest_ops.py GpuPredict.run)
    if (a->early_pred && a->fit_done_level && open_now * 16 >= peak_open) {
      int32_t* done = (int32_t*)a->fit_done_level;
      hipStream_t ps = pred_stream();
      bool any = false;
      for (int64_t f = 0; f < a->n_fits && ps; ++f) {
        if (done[f] != levels - 1) continue;
        if (!any) {
          HIP_OK(hipEventRecord(pred_event(), st));
          HIP_OK(hipStreamWaitEvent(ps, pred_event(), 0));
          any = true;
        }
        if (dml_forest_predict_fit((const PredictArgs*)a->early_pred, (int32_t)f, ps) != 0) return 11;
        done[f] = -2;
      }
    }
    uint32_t* t = c.rows_cur; c.rows_cur = c.rows_next; c.rows_next = t;
    cur = 1 - cur;
    prev_full = full;
    fpar = 1 - fpar;
  }
  HIP_OK(hipMemcpyAsync(h, c.counters, kNumCounters * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  a->n_nodes_out = h[kPool];
  if (c.mono && c.nbound && h[kPool] > 0) {
    const int64_t P = std::min<int64_t>(h[kPool], a->pool_cap);
    k_mono_clip<<<(unsigned)((P + 255) / 256), 256, 0, st>>>(c, P);
    HIP_OK(hipGetLastError());
  }
  if (a->early_pred && pred_stream()) {   // later work on st sees the early predicts' outputs
    HIP_OK(hipEventRecord(pred_event(), pred_stream()));
    HIP_OK(hipStreamWaitEvent(st, pred_event(), 0));
  }
  a->levels_out = levels;
  a->large_rounds_out = large_rounds;
  if (a->status_out != 4) a->status_out = h[kOverflow] ? 1 : (h[kOpenOvf] ? 4 : 0);
  return 0;
}

extern "C" {

// phase 2: build every tree; status_out: 0 ok, 1 node-pool overflow, 4 open-list overflow
int dml_forest_build(ForestArgs* a, hipStream_t st) {
  switch (build_mode(a)) {
    case 1: return build_impl<1>(a, st);
    case 2: return build_impl<2>(a, st);
    default: return build_impl<0>(a, st);
  }
}

}  // extern "C"
