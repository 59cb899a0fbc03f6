// forest_dp_cpu.cpp — C++ twin of forest_dp.hip (row-sharded forest builder steps).
//
// Same entry point shape as the HIP library (one ``step`` switch over a DpArgs block),
// same per-node decisions (forest_dp.h), so the CPU plumbing path and the GPU path of a
// row-sharded job grow the same trees.  Histograms are built per searching node (each
// node's block is private to one OpenMP thread: no atomics, same integer sums).
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <algorithm>
#include <vector>
#include "../kernels/forest_dp.h"

namespace dml {

static void dp_weights(const DpArgs& a) {
#pragma omp parallel for schedule(static)
  for (int64_t idx = 0; idx < a.T * a.n; ++idx) {
    const int t = (int)(idx / a.n);
    const int64_t r = idx - (int64_t)t * a.n;
    const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[t];
    const uint8_t role = dp_ptr<const uint8_t>(a.roles)[(int64_t)s.split * a.n + r];
    const uint32_t w = role == 1 ? boot_weight(s, (uint32_t)(a.r0 + r)) : 0u;
    dp_ptr<uint8_t>(a.wts)[idx] = (uint8_t)(w > 255u ? 255u : w);
  }
}

static void dp_root_stats(const DpArgs& a) {
  const int CH = (int)a.CH;
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < a.T; ++t) {
    const uint8_t* w8 = dp_ptr<const uint8_t>(a.wts) + t * a.n;
    double* out = dp_ptr<double>(a.root) + t * CH;
    if (!a.is_reg) {
      std::vector<uint64_t> cnt(CH, 0);
      for (int64_t r = 0; r < a.n; ++r) {
        if (!w8[r]) continue;
        cnt[dp_ptr<const int32_t>(a.ycls)[r]] += w8[r];
        cnt[CH - 1] += 1;
      }
      for (int c = 0; c < CH; ++c) out[c] += (double)cnt[c];
    } else {   // exact integer sums {w, w yq, w y2q, rows} (forest_common.h)
      const RegScale q = reg_scale((int)a.yq_e1, (int)a.yq_e2);
      uint64_t acc[4] = {0ull, 0ull, 0ull, 0ull};
      for (int64_t r = 0; r < a.n; ++r) {
        if (!w8[r]) continue;
        int64_t yq, y2q;
        reg_quantize(dp_target(a, (int)t, r), q, yq, y2q);
        const int64_t w = w8[r];
        acc[0] += (uint64_t)w; acc[1] += (uint64_t)(w * yq); acc[2] += (uint64_t)(w * y2q); acc[3] += 1ull;
      }
      uint64_t* outi = dp_ptr<uint64_t>(a.root) + t * CH;
      for (int c = 0; c < 4; ++c) outi[c] += acc[c];
    }
  }
}

static void dp_hist(const DpArgs& a) {
  const int CH = (int)a.CH, C = (int)a.C, KR = (int)a.KR;
  const uint8_t* Xb = dp_ptr<const uint8_t>(a.Xb);
  const TreeSpec* specs = dp_ptr<const TreeSpec>(a.specs);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t s = 0; s < a.S; ++s) {
    const int slot = dp_ptr<const int32_t>(a.srch)[s];
    const int64_t seg0 = dp_ptr<const int64_t>(a.seg_start)[slot], cnt = dp_ptr<const int64_t>(a.seg_cnt)[slot];
    const int32_t* fs = dp_ptr<const int32_t>(a.feats) + s * KR;
    uint32_t* hu = dp_ptr<uint32_t>(a.hist) + s * dp_hist_words(a);
    uint64_t* hr = (uint64_t*)hu;
    const RegScale q = reg_scale((int)a.yq_e1, (int)a.yq_e2);
    for (int64_t i = 0; i < cnt; ++i) {
      const int64_t p = seg0 + i;
      const int32_t r = dp_ptr<const int32_t>(a.act_row)[p];
      const int t = dp_ptr<const int32_t>(a.act_tree)[p];
      const uint32_t w = boot_weight(specs[t], (uint32_t)(a.r0 + r));
      const uint8_t* xr = Xb + (int64_t)r * a.ld;
      if (!a.is_reg) {
        const int y = dp_ptr<const int32_t>(a.ycls)[r];
        for (int k = 0; k < KR && fs[k] >= 0; ++k) {
          const int b = xr[fs[k]];
          hu[(k * CH + y) * 256 + b] += w;
          hu[(k * CH + C) * 256 + b] += 1u;
        }
      } else {
        int64_t yq, y2q;
        reg_quantize(dp_target(a, t, r), q, yq, y2q);
        const uint64_t wr = (uint64_t)w | (1ull << 32), wy = (uint64_t)((int64_t)w * yq), wyy = (uint64_t)((int64_t)w * y2q);
        for (int k = 0; k < KR && fs[k] >= 0; ++k) {
          uint64_t* h = hr + (k * 3) * 256 + xr[fs[k]];
          h[0] += wr; h[256] += wy; h[512] += wyy;
        }
      }
    }
  }
}

static void dp_refine_hi(const DpArgs& a) {
  const NodeRec* nodes = dp_ptr<const NodeRec>(a.nodes);
  uint32_t* hi = dp_ptr<uint32_t>(a.hi);
  for (int64_t t = 0; t < a.T; ++t) {
    const TreeSpec& s = dp_ptr<const TreeSpec>(a.specs)[t];
    for (int64_t r = 0; r < a.n; ++r) {
      if (dp_ptr<const uint8_t>(a.roles)[(int64_t)s.split * a.n + r] != 1 ||
          boot_weight(s, (uint32_t)(a.r0 + r)) == 0)
        continue;
      const uint8_t* xr = dp_ptr<const uint8_t>(a.Xb) + r * a.ld;
      int node = (int)t;
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
}

}  // namespace dml

using namespace dml;

extern "C" {

int dml_cpu_dp_sizeof_args() { return (int)sizeof(DpArgs); }
int dml_cpu_dp_sizeof_slot() { return (int)sizeof(DpSlot); }

int dml_cpu_dp_step(const DpArgs* ap, int step) {
  const DpArgs& a = *ap;
  switch (step) {
    case 0: dp_weights(a); break;
    case 1: dp_root_stats(a); break;
    case 2:
      for (int64_t t = 0; t < a.T; ++t) {
        DpSlot sl;
        dp_ptr<int32_t>(a.next_open)[t] = dp_root_one(a, (int)t, &sl);
        dp_ptr<DpSlot>(a.next)[t] = sl;
      }
      break;
    case 3:
#pragma omp parallel for schedule(static)
      for (int64_t idx = 0; idx < a.S * a.KR; ++idx) {
        const int64_t s = idx / a.KR, k = idx - s * a.KR;
        const DpSlot& sl = dp_ptr<const DpSlot>(a.slots)[dp_ptr<const int32_t>(a.srch)[s]];
        const int p = sl.pos + (int)k;
        dp_ptr<int32_t>(a.feats)[idx] = p < a.d ? feature_at(feat_perm(sl.key, (int)a.d), p, (int)a.d) : -1;
      }
      break;
    case 4: dp_hist(a); break;
    case 5:
#pragma omp parallel for schedule(dynamic, 16)
      for (int64_t s = 0; s < a.S; ++s) {
        const int slot = dp_ptr<const int32_t>(a.srch)[s];
        DpSlot& sl = dp_ptr<DpSlot>(a.slots)[slot];
        dp_eval_slot(a, sl, dp_ptr<double>(a.best_left) + (int64_t)slot * a.CH,
                     dp_ptr<const uint32_t>(a.hist) + s * dp_hist_words(a), dp_ptr<const int32_t>(a.feats) + s * a.KR);
      }
      break;
    case 6:
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < a.S_open; ++i) {
        DpSlot& sl = dp_ptr<DpSlot>(a.slots)[i];
        sl.split = dp_accept_one(a, sl, dp_ptr<const double>(a.best_left) + i * a.CH);
      }
      break;
    case 7:
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < a.S_open; ++i) dp_children_one(a, (int)i);
      break;
    case 8:
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < a.A; ++i) dp_ptr<int32_t>(a.new_node)[i] = dp_partition_one(a, i);
      break;
    case 9: dp_refine_hi(a); break;
    case 10:
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < a.P_total; ++i) dp_refine_one(a, i);
      break;
    default:
      return 1;
  }
  return 0;
}

}  // extern "C"
