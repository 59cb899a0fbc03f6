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

// ---- LinearRegression: every split's normal-equation moments in one pass over X ------
// For split s the moments of z_r = [x_r - c_x, 1, y_r - c_y] over its train rows:
//   M_s = sum_{r : roles[s][r] == TRAIN} z_r z_r^T        ((d+2) x (d+2), float64)
// which hold the count, the shifted sums, X^T X, X^T y and y^T y.  The shift c (the
// column means over all rows, host-computed) keeps the centring on the host accurate:
// each split's mean is close to c, so M_s - n_s dm dm^T loses nothing to cancellation.
// Tiles: v_mfma_f64_16x16x4_f64 (exact f64 products and sums; lane l feeds row
// (l>>4) of a 4-row step: A = z[row][16 ti + (l&15)] masked by the split's role,
// B = z[row][16 tj + (l&15)]); one workgroup per (row chunk, upper-triangle tile pair),
// all splits at once (the z loads are shared), 4 waves over the chunk reduced through
// LDS f64 atomics, then one global f64 atomic per tile entry per workgroup.
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double zval(const float* __restrict__ X, int64_t ld, const float* __restrict__ y,
                                       const double* __restrict__ shift, int64_t d, int64_t r, int c) {
  if (c < d) return (double)X[r * ld + c] - shift[c];
  if (c == d) return 1.0;
  if (c == d + 1) return y ? (double)y[r] - shift[d] : 0.0;
  return 0.0;
}

template <int S>
__global__ __launch_bounds__(256) void k_split_moments(const float* __restrict__ X, int64_t ld,
                                                       const float* __restrict__ y, const double* __restrict__ shift,
                                                       const uint8_t* __restrict__ roles, int64_t n, int64_t d,
                                                       int tiles, int64_t rows_per_wg, double* __restrict__ out,
                                                       int64_t Dp) {
  __shared__ double red[S * 4 * 64];
  // upper-triangle tile pair of this workgroup
  int pair = blockIdx.y, ti = 0;
  while (pair >= tiles - ti) { pair -= tiles - ti; ++ti; }
  const int tj = ti + pair;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < S * 4 * 64; i += 256) red[i] = 0.0;
  const int64_t per_wave = rows_per_wg / 4;
  const int64_t r_begin = (int64_t)blockIdx.x * rows_per_wg + wave * per_wave;
  const int64_t r_end = min(n, r_begin + per_wave);
  const int ca = ti * 16 + (lane & 15), cb = tj * 16 + (lane & 15);
  f64x4 acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 4) {
    const int64_t r = r0 + (lane >> 4);
    const bool live = r < r_end;
    const double a = live ? zval(X, ld, y, shift, d, r, ca) : 0.0;
    const double b = live ? zval(X, ld, y, shift, d, r, cb) : 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double am = (live && roles[(int64_t)s * n + r] == 1) ? a : 0.0;
      acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(am, b, acc[s], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int g = 0; g < 4; ++g) atomicAdd(&red[(s * 4 + g) * 64 + lane], acc[s][g]);
  __syncthreads();
  // C/D map of 16x16x4 f64: column lane & 15, row (lane >> 4) + 4 g
  for (int i = threadIdx.x; i < S * 4 * 64; i += 256) {
    const int s = i / 256, g = (i / 64) & 3, l = i & 63;
    const double v = red[i];
    if (v != 0.0) {
      const int64_t row = ti * 16 + (l >> 4) + 4 * g, col = tj * 16 + (l & 15);
      atomicAdd(&out[((int64_t)s * Dp + row) * Dp + col], v);
    }
  }
}

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

// out: [S][Dp][Dp] float64 zeroed, Dp = roundup(d + 2, 16); only tiles with ti <= tj are
// written (the host mirrors them).  y may be null (column d+1 = 0).  S <= 8 per launch.
int dml_split_moments(const float* X, int64_t ld, const float* y, const double* shift, const uint8_t* roles,
                      int64_t n, int64_t d, int32_t S, double* out, int64_t Dp, hipStream_t st) {
  if (n <= 0 || S <= 0) return 0;
  if (S > 8 || Dp % 16 || Dp < d + 2) return 2;
  const int tiles = (int)(Dp / 16);
  const int64_t rows_per_wg = 4096;
  dim3 grid((unsigned)((n + rows_per_wg - 1) / rows_per_wg), (unsigned)(tiles * (tiles + 1) / 2));
  switch (S) {
#define DML_MOM(k) case k: k_split_moments<k><<<grid, 256, 0, st>>>(X, ld, y, shift, roles, n, d, tiles, rows_per_wg, out, Dp); break;
    DML_MOM(1) DML_MOM(2) DML_MOM(3) DML_MOM(4) DML_MOM(5) DML_MOM(6) DML_MOM(7) DML_MOM(8)
#undef DML_MOM
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
