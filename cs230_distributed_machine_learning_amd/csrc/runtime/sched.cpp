// sched.cpp — placement core of the scheduler (native).
//
// The reference scheduler (aws-prod/scheduler/scheduler_service.py:173-191) picks, per
// incoming task, the worker minimising load/speed + estimate/speed among workers whose
// reserved memory fits, with a learned runtime estimate.  This is the batch form of the
// same rule: Longest-Processing-Time-first list scheduling over workers with speed
// factors and memory capacities — a 4/3-approximation of the optimal makespan for
// identical workers — plus the reference's "reserve memory" feasibility test.
// Units that fit on no worker are reported (-1) and HELD by the caller rather than
// dropped (reference defect D14).
#include <stdint.h>
#include <algorithm>
#include <numeric>
#include <vector>

extern "C" {

// costs[n] (seconds at speed 1), mem[n] (MB, may be 0), speed[w] (>0), cap[w] (MB, 0 = unlimited),
// load0[w] initial queued seconds (speed-scaled).  out_worker[n] = assigned worker or -1.
// Returns the predicted makespan (seconds).
double dml_lpt_assign(const double* costs, const double* mem, int64_t n, const double* speed, const double* cap,
                      const double* load0, int64_t w, int32_t* out_worker) {
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return costs[a] > costs[b]; });
  std::vector<double> finish(w), used(w, 0.0);
  for (int64_t j = 0; j < w; ++j) finish[j] = load0 ? load0[j] : 0.0;
  for (int64_t i : order) {
    int64_t best = -1;
    double best_t = 0.0;
    for (int64_t j = 0; j < w; ++j) {
      if (speed[j] <= 0.0) continue;
      if (cap && cap[j] > 0.0 && mem && used[j] + mem[i] > cap[j]) continue;
      const double t = finish[j] + costs[i] / speed[j];
      if (best < 0 || t < best_t) { best = j; best_t = t; }
    }
    out_worker[i] = (int32_t)best;
    if (best >= 0) {
      finish[best] = best_t;
      if (mem) used[best] += mem[i];
    }
  }
  double mk = 0.0;
  for (int64_t j = 0; j < w; ++j) mk = std::max(mk, finish[j]);
  return mk;
}

// Split an LPT-ordered list of unit costs into chunks of ~target seconds each while
// keeping at least `min_chunks` chunks (progress granularity for streaming status).
// out_chunk[n] = chunk id in processing order; returns the number of chunks.
int64_t dml_chunk_units(const double* costs, int64_t n, double target, int64_t min_chunks, int32_t* out_chunk) {
  double total = 0.0;
  for (int64_t i = 0; i < n; ++i) total += costs[i];
  if (min_chunks > 0 && total / (double)min_chunks < target) target = total / (double)min_chunks;
  int64_t c = 0;
  double acc = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    if (acc > 0.0 && acc + costs[i] > target) { ++c; acc = 0.0; }
    out_chunk[i] = (int32_t)c;
    acc += costs[i];
  }
  return n ? c + 1 : 0;
}

}  // extern "C"
