// linear.hip — K7/K8 epilogue for batched logistic regression (many fits per pass).
//
// The reference fits LogisticRegression one candidate x one fold at a time on CPU
// (aws-prod/worker/worker.py:39 whitelist, :315/:326 fit + cross_val_score).  Here every
// (candidate, fold) of a job is one block of columns of ONE weight matrix, so the
// forward product Z = X W_all and the gradient product G = X^T R are plain GEMMs over
// all fits at once (hipBLASLt), and this kernel is the fused row-wise middle:
//   link (sigmoid / softmax / one-vs-rest sigmoid), fold masking, per-fit loss, and the
//   residual R = (P - Y) * role_mask * scale — one read of Z, one write of R.
// Thread t handles (row = t / F, fit = t % F): consecutive lanes read consecutive
// column groups of the same Z row (coalesced).  Per-fit losses are reduced in LDS
// (double) and flushed with one atomic per fit per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

constexpr int kMaxFitsLds = 2048;

__device__ __forceinline__ float softplus(float x) {  // log(1 + exp(x)), stable
  return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
}

__device__ __forceinline__ float sigmoidf(float x) {
  return x >= 0.f ? 1.f / (1.f + expf(-x)) : expf(x) / (1.f + expf(x));
}

__global__ __launch_bounds__(256) void k_lr_link_grad(const float* __restrict__ Z, int64_t n, int64_t M,
                                                      const int32_t* __restrict__ y, const uint8_t* __restrict__ roles,
                                                      const int32_t* __restrict__ col0, const int32_t* __restrict__ K,
                                                      const int32_t* __restrict__ kind,
                                                      const int32_t* __restrict__ split,
                                                      const float* __restrict__ scale, int64_t F,
                                                      const float* __restrict__ cw, int64_t cwC,
                                                      float* __restrict__ R, double* __restrict__ loss) {
  __shared__ double acc[kMaxFitsLds];
  const bool use_lds = F <= kMaxFitsLds;
  if (use_lds)
    for (int i = threadIdx.x; i < F; i += 256) acc[i] = 0.0;
  __syncthreads();
  const int64_t total = n * F;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t row = t / F;
    const int f = (int)(t - row * F);
    const int c0 = col0[f], k = K[f];
    const float* z = Z + row * M + c0;
    float* r = R + row * M + c0;
    const bool train = roles[(int64_t)split[f] * n + row] == 1;
    if (!train) {
      for (int j = 0; j < k; ++j) r[j] = 0.f;
      continue;
    }
    const int yi = y[row];
    const float s = cw ? scale[f] * cw[(int64_t)f * cwC + yi] : scale[f];   // class weights scale the row
    float l = 0.f;
    if (kind[f] == 1) {  // multinomial softmax over k columns
      float m = z[0];
      for (int j = 1; j < k; ++j) m = fmaxf(m, z[j]);
      float se = 0.f;
      for (int j = 0; j < k; ++j) se += expf(z[j] - m);
      const float lse = m + logf(se);
      for (int j = 0; j < k; ++j) r[j] = (expf(z[j] - lse) - (j == yi ? 1.f : 0.f)) * s;
      l = lse - z[yi];
    } else {  // kind 0: one sigmoid column with target (y == 1); kind 2: column j target (y == j)
      for (int j = 0; j < k; ++j) {
        const float tgt = (kind[f] == 0) ? (yi == 1 ? 1.f : 0.f) : (yi == j ? 1.f : 0.f);
        const float zj = z[j];
        r[j] = (sigmoidf(zj) - tgt) * s;
        l += softplus(tgt > 0.5f ? -zj : zj);
      }
    }
    if (use_lds) atomicAdd(&acc[f], (double)(l * s));
    else atomicAdd(&loss[f], (double)(l * s));
  }
  __syncthreads();
  if (use_lds)
    for (int i = threadIdx.x; i < F; i += 256)
      if (acc[i] != 0.0) atomicAdd(&loss[i], acc[i]);
}

// row-wise prediction: argmax class (softmax/ovr) or sign (binary) for each fit's rows
__global__ __launch_bounds__(256) void k_lr_predict(const float* __restrict__ Z, int64_t M,
                                                    const int32_t* __restrict__ rows, const int64_t* __restrict__ row_off,
                                                    const int32_t* __restrict__ col0, const int32_t* __restrict__ K,
                                                    const int32_t* __restrict__ kind, int64_t F, int32_t* __restrict__ out) {
  const int f = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = row_off[f], nr = row_off[f + 1] - r0;
  if (i >= nr) return;
  const float* z = Z + (int64_t)rows[r0 + i] * M + col0[f];
  int best = 0;
  if (kind[f] == 0) {
    best = z[0] > 0.f ? 1 : 0;
  } else {
    float bv = z[0];
    for (int j = 1; j < K[f]; ++j)
      if (z[j] > bv) { bv = z[j]; best = j; }
  }
  out[r0 + i] = best;
}

}  // namespace

extern "C" {

int dml_lr_link_grad(const float* Z, int64_t n, int64_t M, const int32_t* y, const uint8_t* roles,
                     const int32_t* col0, const int32_t* K, const int32_t* kind, const int32_t* split,
                     const float* scale, int64_t F, const float* cw, int64_t cwC, float* R, double* loss,
                     hipStream_t st) {
  if (n <= 0 || F <= 0) return 0;
  if (hipMemsetAsync(loss, 0, F * sizeof(double), st) != hipSuccess) return 1;
  int64_t blocks = (n * F + 255) / 256;
  if (blocks > 256 * 32) blocks = 256 * 32;
  k_lr_link_grad<<<(unsigned)blocks, 256, 0, st>>>(Z, n, M, y, roles, col0, K, kind, split, scale, F, cw, cwC, R,
                                                   loss);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_lr_predict(const float* Z, int64_t M, const int32_t* rows, const int64_t* row_off, int64_t max_rows,
                   const int32_t* col0, const int32_t* K, const int32_t* kind, int64_t F, int32_t* out,
                   hipStream_t st) {
  if (F <= 0 || max_rows <= 0) return 0;
  dim3 grid((unsigned)((max_rows + 255) / 256), (unsigned)F);
  k_lr_predict<<<grid, 256, 0, st>>>(Z, M, rows, row_off, col0, K, kind, F, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
