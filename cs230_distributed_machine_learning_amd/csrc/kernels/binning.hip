// binning.hip — K1: quantise a resident float32 table into uint8 bins (row-major).
//
// The reference re-parses the full CSV per task (aws-prod/worker/worker.py:406-425)
// and lets sklearn sort raw floats per node.  Here the table is quantised ONCE per
// dataset per GPU: bin(x) = #{edges < x} over <=255 sorted per-feature edges (+inf
// padded), so "x <= edge[b]" <=> "bin <= b" and every tree/fit/candidate reuses the
// same 1-byte-per-cell copy (1M x 100 = 100 MB, resident in HBM / Infinity Cache).
//
// One thread per cell, consecutive threads on consecutive cells of a row-major row
// (coalesced 4-B loads, 1-B stores); the edge table of a feature is 1 KiB and stays
// L1/L2-resident, so the 8-step branch-free lower_bound is latency-hidden by
// occupancy.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_bin(const float* __restrict__ X, int64_t n, int64_t d,
                                             const float* __restrict__ edges, uint8_t* __restrict__ out,
                                             int64_t ld) {
  const int64_t total = n * d;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / d, f = i - r * d;
    const float x = X[i];
    const float* e = edges + f * 255;
    // branch-free lower_bound over 255 (+1 virtual) entries
    int lo = 0;
#pragma unroll
    for (int step = 128; step >= 1; step >>= 1) {
      const int probe = lo + step - 1;
      if (probe < 255 && e[probe] < x) lo += step;
    }
    out[r * ld + f] = (uint8_t)lo;
  }
}

extern "C" int dml_bin(const float* X, int64_t n, int64_t d, const float* edges, uint8_t* out, int64_t ld,
                       hipStream_t st) {
  const int64_t total = n * d;
  if (total <= 0) return 0;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 256 * 64) blocks = 256 * 64;
  k_bin<<<(unsigned)blocks, 256, 0, st>>>(X, n, d, edges, out, ld);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
