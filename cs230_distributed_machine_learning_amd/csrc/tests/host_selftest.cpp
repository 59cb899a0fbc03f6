// Host self-test of the C++ runtime (csrc/runtime/*.cpp), built with
// -fsanitize=address,undefined by build.build_sanitized() and run by
// tests/test_host_sanitizers.py.  The reference has no race detection or sanitizers
// (SURVEY §5.2); this covers every entry point the Python layer calls through ctypes:
// tree building (gini / entropy / mse, bootstrap on/off, depth limits), export, leaf
// apply, threshold refinement, batched predict, binning, LPT placement and chunking.
// Exit status 0 = all invariants hold and the sanitizers saw nothing.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

#include "forest_common.h"

using namespace dml;

extern "C" {
void* dml_cpu_forest_build(const uint8_t*, int64_t, int64_t, int64_t, const int32_t*, const float*, int64_t, int64_t,
                           const uint8_t*, const TreeSpec*, int64_t, int64_t, const double*);
int64_t dml_cpu_forest_num_nodes(void*);
void dml_cpu_forest_export(void*, NodeRec*, double*);
void dml_cpu_forest_apply(const uint8_t*, int64_t, int64_t, const NodeRec*, int32_t, int32_t, int32_t*);
void dml_cpu_forest_free(void*);
void dml_cpu_forest_predict(const uint8_t*, int64_t, const NodeRec*, const double*, int64_t, int64_t, int64_t,
                            const int32_t*, const int64_t*, const int32_t*, int64_t, int32_t*, float*, float*);
void dml_cpu_bin(const float*, int64_t, int64_t, const float*, uint8_t*, int64_t);
double dml_lpt_assign(const double*, const double*, int64_t, const double*, const double*, const double*, int64_t,
                      int32_t*);
int64_t dml_chunk_units(const double*, int64_t, double, int64_t, int32_t*);
}

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static uint64_t rng_state = 0x1234567ull;
static uint32_t rnd() { rng_state = splitmix64(rng_state); return (uint32_t)(rng_state >> 32); }
static float rndf() { return (rnd() >> 8) * (1.0f / 16777216.0f); }

static TreeSpec make_spec(uint64_t seed, int fit, int depth, int mss, int msl, int mf, int boot, int crit) {
  TreeSpec s{};
  s.seed = seed; s.split = 0; s.fit = fit; s.max_depth = depth; s.min_samples_split = mss;
  s.min_samples_leaf = msl; s.max_features = mf; s.bootstrap = boot; s.criterion = crit;
  s.min_impurity_decrease = 0.f; s.target = 0;
  double p = std::exp(-1.0), cdf = 0.0;   // Poisson(1)
  for (int j = 0; j < kPoisTable; ++j) {
    cdf += p; p /= (double)(j + 1);
    const double v = cdf * 4294967296.0;
    s.pois_cdf[j] = v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
  }
  return s;
}

static void forest_case(bool is_reg, int crit) {
  const int64_t n = 3000, d = 13, C = is_reg ? 1 : 3;
  std::vector<float> X(n * d);
  for (auto& v : X) v = rndf() * 2.f - 1.f;
  // edges: 255 per feature, uniform quantiles of U(-1,1), +inf padded after 200
  std::vector<float> edges(d * 255);
  for (int64_t f = 0; f < d; ++f)
    for (int k = 0; k < 255; ++k)
      edges[f * 255 + k] = k < 200 ? -1.f + 2.f * (k + 1) / 201.f : std::numeric_limits<float>::infinity();
  std::vector<uint8_t> Xb(n * d);
  dml_cpu_bin(X.data(), n, d, edges.data(), Xb.data(), d);
  for (auto b : Xb) CHECK(b <= 200);
  std::vector<int32_t> ycls(n);
  std::vector<float> yreg(n);
  for (int64_t i = 0; i < n; ++i) {
    const float s = X[i * d + 0] + 0.5f * X[i * d + 3] - X[i * d + 7];
    ycls[i] = s < -0.4f ? 0 : (s < 0.4f ? 1 : 2);
    yreg[i] = s + 0.05f * (rndf() - 0.5f);
  }
  std::vector<uint8_t> roles(n);
  for (int64_t i = 0; i < n; ++i) roles[i] = (i % 5 == 0) ? 2 : 1;   // 1 train, 2 test
  std::vector<TreeSpec> specs;
  const int T = 8;
  for (int t = 0; t < T; ++t)
    specs.push_back(make_spec(0x9e37ull * (t + 1), t / 4, t % 2 ? 6 : std::numeric_limits<int32_t>::max(),
                              2 + t % 3, 1 + t % 2, t % 3 == 0 ? (int)d : 4, t % 4 == 3 ? 0 : 1, crit));
  if (!is_reg)   // class_weight="balanced_subsample" on some trees (weights from the bootstrap counts)
    for (int t = 4; t < T; t += 5) specs[t].cw_mode = 2;
  void* h = dml_cpu_forest_build(Xb.data(), d, n, d, is_reg ? nullptr : ycls.data(), is_reg ? yreg.data() : nullptr,
                                 C, is_reg, roles.data(), specs.data(), T, 0, nullptr);
  CHECK(h != nullptr);
  const int64_t P = dml_cpu_forest_num_nodes(h);
  CHECK(P >= T);
  const int64_t VC = is_reg ? 3 : C;
  std::vector<NodeRec> nodes(P);
  std::vector<double> vals(P * VC);
  dml_cpu_forest_export(h, nodes.data(), vals.data());
  dml_cpu_forest_free(h);
  for (int64_t p = 0; p < P; ++p) {
    if (nodes[p].split >= 0) {
      CHECK(nodes[p].left > p && nodes[p].left + 1 < P);
      CHECK((nodes[p].split >> 8) < d);
    } else {
      CHECK(nodes[p].left == -1);
    }
  }
  // leaf map of every row for every tree
  std::vector<int32_t> leaf((size_t)n * T);
  dml_cpu_forest_apply(Xb.data(), d, n, nodes.data(), 0, T, leaf.data());
  for (auto l : leaf) CHECK(l >= 0 && l < P && nodes[l].split < 0);
  // batched predict of the test rows of 2 fits (trees [0,4) and [4,8))
  std::vector<int32_t> rows;
  for (int64_t i = 0; i < n; ++i)
    if (roles[i] == 2) rows.push_back((int32_t)i);
  const int64_t R = (int64_t)rows.size();
  std::vector<int32_t> rows2(rows);
  rows2.insert(rows2.end(), rows.begin(), rows.end());
  const int32_t tree_off[3] = {0, 4, 8};
  const int64_t row_off[3] = {0, R, 2 * R};
  std::vector<int32_t> out_cls(2 * R, -1);
  std::vector<float> out_reg(2 * R, 0.f), proba(2 * R * C, 0.f);
  dml_cpu_forest_predict(Xb.data(), d, nodes.data(), vals.data(), VC, is_reg, C, tree_off, row_off, rows2.data(), 2,
                         out_cls.data(), out_reg.data(), is_reg ? nullptr : proba.data());
  double hits = 0.0, se = 0.0, var = 0.0, mean = 0.0;
  for (int64_t i = 0; i < 2 * R; ++i) mean += yreg[rows2[i]];
  mean /= (double)(2 * R);
  for (int64_t i = 0; i < 2 * R; ++i) {
    const int32_t r = rows2[i];
    if (is_reg) {
      se += (out_reg[i] - yreg[r]) * (out_reg[i] - yreg[r]);
      var += (yreg[r] - mean) * (yreg[r] - mean);
    } else {
      CHECK(out_cls[i] >= 0 && out_cls[i] < C);
      float ps = 0.f;
      for (int k = 0; k < C; ++k) ps += proba[i * C + k];
      CHECK(std::fabs(ps - 1.f) < 1e-3f);
      hits += out_cls[i] == ycls[r];
    }
  }
  if (is_reg) {
    std::printf("regression r2 %.3f\n", 1.0 - se / var);
    CHECK(1.0 - se / var > 0.5);
  } else {
    std::printf("classification (criterion %d) accuracy %.3f\n", crit, hits / (2 * R));
    CHECK(hits / (2 * R) > 0.7);
  }
}

static void sched_case() {
  const int64_t n = 37, w = 5;
  std::vector<double> costs(n), mem(n), speed(w), cap(w, 0.0), load0(w, 0.0);
  for (int64_t i = 0; i < n; ++i) { costs[i] = 0.1 + rndf() * 5.0; mem[i] = 10.0 * (i % 3); }
  for (int64_t j = 0; j < w; ++j) speed[j] = 0.5 + j * 0.25;
  std::vector<int32_t> out(n, -2);
  double mk = dml_lpt_assign(costs.data(), mem.data(), n, speed.data(), cap.data(), load0.data(), w, out.data());
  double tot = 0.0;
  for (int64_t i = 0; i < n; ++i) { CHECK(out[i] >= 0 && out[i] < w); tot += costs[i]; }
  double sp = 0.0;
  for (auto s : speed) sp += s;
  CHECK(mk >= tot / sp - 1e-9);
  // a worker with too little memory never gets a unit that does not fit
  cap[0] = 5.0;
  dml_lpt_assign(costs.data(), mem.data(), n, speed.data(), cap.data(), load0.data(), w, out.data());
  double used0 = 0.0;
  for (int64_t i = 0; i < n; ++i) if (out[i] == 0) used0 += mem[i];
  CHECK(used0 <= 5.0);
  std::vector<int32_t> chunk(n);
  const int64_t nc = dml_chunk_units(costs.data(), n, 3.0, 8, chunk.data());
  CHECK(nc >= 8 && chunk[0] == 0 && chunk[n - 1] == nc - 1);
  for (int64_t i = 1; i < n; ++i) CHECK(chunk[i] == chunk[i - 1] || chunk[i] == chunk[i - 1] + 1);
  CHECK(dml_chunk_units(costs.data(), 0, 3.0, 1, chunk.data()) == 0);
}

int main() {
  forest_case(false, kGini);
  forest_case(false, kEntropy);
  forest_case(true, kMSE);
  forest_case(true, kMAE);   // integer Fenwick sweep + exact abs deviations (forest_common.h mae_absdev)
  sched_case();
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("host selftest ok\n");
  return 0;
}
