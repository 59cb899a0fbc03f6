// svm.hip — batched SMO for kernel SVMs: one workgroup per dual problem, all problems
// of a job (candidates x CV folds x one-vs-one class pairs / epsilon-SVR) in one launch.
//
// Reference: SVC / SVR are whitelisted estimators (aws-prod/worker/worker.py:40,47) fitted
// by libsvm (sklearn svm/_libsvm, C++ SMO) once per (candidate, fold) on CPU.  This
// kernel runs the SAME dual algorithm — libsvm's Solver: second-order working-set
// selection (WSS3, Fan et al. 2005), analytic two-variable update with box clipping,
// gradient maintenance G += Q_i da_i + Q_j da_j, stopping when
// max_{I_up} -yG + max_{I_low} yG < eps — so it converges to libsvm's solution (same
// tie rules: the later index wins, as libsvm's >= / <= scans do).  Shrinking is a
// libsvm speed heuristic that does not change the optimum and is not used.
//
// Mapping (gfx950): a 256-thread workgroup owns one problem; per SMO iteration it makes
// two kernel-column passes over the problem's rows (feature-major rows -> coalesced) and
// two fused reduce/update sweeps over its variables, with wave64 DPP-free shuffles and an
// LDS combine across the 4 waves.  State (alpha, G) lives in HBM, so the host can run
// the solver in bounded chunks of iterations (no long-running kernels) and resume.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

constexpr int NT = 256;
constexpr int kMaxLdsD = 2048;   // query rows up to this many features are staged in LDS
constexpr double kTau = 1e-12;
constexpr double kInf = 1e300;

enum { KLIN = 0, KPOLY = 1, KRBF = 2, KSIG = 3 };

// host-shared problem record: every field 8 bytes
struct SvmProb {
  int64_t xoff;      // feature-major rows of this problem's rowset: X[xoff + f * nrows + r]
  int64_t roff;      // per-row arrays (qd): qd[roff + r]
  int64_t nrows;     // rows in the rowset
  int64_t L;         // dual variables (nrows for SVC, 2 nrows for epsilon-SVR)
  int64_t voff;      // per-variable arrays: y, C, alpha, G at [voff, voff + L)
  int64_t koff;      // kernel-column scratch: 2 * nrows floats at koff
  int64_t kernel, degree;
  double gamma, coef0, eps;
  int64_t max_iter;  // total iteration budget
  int64_t iters;     // in/out: iterations done so far
  int64_t status;    // in/out: 0 running, 1 optimal, 2 iteration limit
  int64_t svr;       // 1: variable t uses row t mod nrows
};

__device__ __forceinline__ float kfun(int kernel, double gamma, double coef0, int degree, float acc) {
  switch (kernel) {
    case KRBF: return (float)exp(-gamma * (double)acc);
    case KPOLY: {
      const double b = gamma * (double)acc + coef0;
      double r = 1.0;
      for (int i = 0; i < degree; ++i) r *= b;
      return (float)r;
    }
    case KSIG: return (float)tanh(gamma * (double)acc + coef0);
    default: return acc;
  }
}

struct Cand {
  double v;
  int idx;
};

// better(a, b): a replaces b.  MAX=true: larger value, ties -> larger index.
template <bool MAX>
__device__ __forceinline__ bool better(double av, int ai, double bv, int bi) {
  if (ai < 0) return false;
  if (bi < 0) return true;
  if (MAX) return av > bv || (av == bv && ai > bi);
  return av < bv || (av == bv && ai > bi);
}

template <bool MAX>
__device__ Cand block_reduce(Cand c, Cand* red) {
  for (int m = 32; m >= 1; m >>= 1) {
    const double ov = __shfl_xor(c.v, m);
    const int oi = __shfl_xor(c.idx, m);
    if (better<MAX>(ov, oi, c.v, c.idx)) { c.v = ov; c.idx = oi; }
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wid] = c;
  __syncthreads();
  Cand r = red[0];
  for (int w = 1; w < NT / 64; ++w)
    if (better<MAX>(red[w].v, red[w].idx, r.v, r.idx)) r = red[w];
  __syncthreads();
  return r;
}

__device__ double block_max(double v, double* red) {
  for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m));
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  double r = red[0];
  for (int w = 1; w < NT / 64; ++w) r = fmax(r, red[w]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ bool is_upper(double a, double c) { return a >= c; }
__device__ __forceinline__ bool is_lower(double a) { return a <= 0.0; }

// kernel column of rowset row `src` against all rows -> col[r]
__device__ void kernel_column(const SvmProb& p, const float* __restrict__ X, int64_t d, int64_t src, float* xs,
                              float* __restrict__ col) {
  const bool lds = d <= kMaxLdsD;
  const float* base = X + p.xoff;
  if (lds) {
    for (int64_t f = threadIdx.x; f < d; f += NT) xs[f] = base[f * p.nrows + src];
    __syncthreads();
  }
  const int kernel = (int)p.kernel;
  for (int64_t r = threadIdx.x; r < p.nrows; r += NT) {
    float acc = 0.f;
    if (kernel == KRBF) {
      for (int64_t f = 0; f < d; ++f) {
        const float a = lds ? xs[f] : base[f * p.nrows + src];
        const float t = a - base[f * p.nrows + r];
        acc = __builtin_fmaf(t, t, acc);
      }
    } else {
      for (int64_t f = 0; f < d; ++f) {
        const float a = lds ? xs[f] : base[f * p.nrows + src];
        acc = __builtin_fmaf(a, base[f * p.nrows + r], acc);
      }
    }
    col[r] = kfun(kernel, p.gamma, p.coef0, (int)p.degree, acc);
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void k_smo(const float* __restrict__ X, int64_t d, SvmProb* probs,
                                            const float* __restrict__ yv, const double* __restrict__ Cv,
                                            const float* __restrict__ qd, double* __restrict__ alpha,
                                            double* __restrict__ G, float* __restrict__ kbuf, int64_t chunk) {
  SvmProb& P = probs[blockIdx.x];
  if (P.status != 0) return;
  __shared__ float xs[kMaxLdsD];
  __shared__ Cand red[NT / 64];
  __shared__ double redd[NT / 64];
  __shared__ double upd[2];
  const SvmProb p = P;
  const int64_t L = p.L, nr = p.nrows;
  const float* y = yv + p.voff;
  const double* C = Cv + p.voff;
  double* a = alpha + p.voff;
  double* g = G + p.voff;
  float* Ki = kbuf + p.koff;
  float* Kj = Ki + nr;
  const float* QD = qd + p.roff;
  auto rowof = [&](int64_t t) { return (p.svr && t >= nr) ? t - nr : t; };

  int64_t it = p.iters;
  int status = 0;
  const int64_t stop_at = min(p.max_iter, it + chunk);
  // select i over I_up: max -y_t G_t (ties -> larger t)
  Cand ci{-kInf, -1};
  for (int64_t t = threadIdx.x; t < L; t += NT) {
    const double yt = y[t];
    const bool up = yt > 0 ? !is_upper(a[t], C[t]) : !is_lower(a[t]);
    if (up) {
      const double v = -yt * g[t];
      if (better<true>(v, (int)t, ci.v, ci.idx)) { ci.v = v; ci.idx = (int)t; }
    }
  }
  while (true) {
    if (it >= stop_at) { status = it >= p.max_iter ? 2 : 0; break; }
    const Cand bi = block_reduce<true>(ci, red);
    const int i = bi.idx;
    if (i < 0) { status = 1; break; }
    const double Gmax = bi.v;
    const double yi = y[i];
    const int64_t ri = rowof(i);
    kernel_column(p, X, d, ri, xs, Ki);
    // select j over I_low with the second-order gain; Gmax2 = max_{I_low} y_t G_t
    Cand cj{kInf, -1};
    double gmax2 = -kInf;
    const double QDi = QD[ri];
    for (int64_t t = threadIdx.x; t < L; t += NT) {
      const double yt = y[t];
      const int64_t rt = rowof(t);
      const double kit = (double)Ki[rt];
      if (yt > 0) {
        if (!is_lower(a[t])) {
          const double gd = Gmax + g[t];
          gmax2 = fmax(gmax2, g[t]);
          if (gd > 0) {
            double qc = QDi + QD[rt] - 2.0 * yi * (yi * yt * kit);
            const double od = qc > 0 ? -(gd * gd) / qc : -(gd * gd) / kTau;
            if (better<false>(od, (int)t, cj.v, cj.idx)) { cj.v = od; cj.idx = (int)t; }
          }
        }
      } else {
        if (!is_upper(a[t], C[t])) {
          const double gd = Gmax - g[t];
          gmax2 = fmax(gmax2, -g[t]);
          if (gd > 0) {
            double qc = QDi + QD[rt] + 2.0 * yi * (yi * yt * kit);
            const double od = qc > 0 ? -(gd * gd) / qc : -(gd * gd) / kTau;
            if (better<false>(od, (int)t, cj.v, cj.idx)) { cj.v = od; cj.idx = (int)t; }
          }
        }
      }
    }
    const Cand bj = block_reduce<false>(cj, red);
    const double Gmax2 = block_max(gmax2, redd);
    if (Gmax + Gmax2 < p.eps || bj.idx < 0) { status = 1; break; }
    const int j = bj.idx;
    const double yj = y[j];
    const int64_t rj = rowof(j);
    kernel_column(p, X, d, rj, xs, Kj);
    if (threadIdx.x == 0) {
      // libsvm Solver::Solve two-variable update (Q_ij = y_i y_j K_ij)
      const double Ci = C[i], Cj = C[j];
      const double Qij = yi * yj * (double)Ki[rj];
      const double QDj = QD[rj];
      const double oai = a[i], oaj = a[j];
      double ai = oai, aj = oaj;
      if (yi != yj) {
        double qc = QDi + QDj + 2.0 * Qij;
        if (qc <= 0) qc = kTau;
        const double delta = (-g[i] - g[j]) / qc;
        const double diff = ai - aj;
        ai += delta; aj += delta;
        if (diff > 0) { if (aj < 0) { aj = 0; ai = diff; } }
        else { if (ai < 0) { ai = 0; aj = -diff; } }
        if (diff > Ci - Cj) { if (ai > Ci) { ai = Ci; aj = Ci - diff; } }
        else { if (aj > Cj) { aj = Cj; ai = Cj + diff; } }
      } else {
        double qc = QDi + QDj - 2.0 * Qij;
        if (qc <= 0) qc = kTau;
        const double delta = (g[i] - g[j]) / qc;
        const double sum = ai + aj;
        ai -= delta; aj += delta;
        if (sum > Ci) { if (ai > Ci) { ai = Ci; aj = sum - Ci; } }
        else { if (aj < 0) { aj = 0; ai = sum; } }
        if (sum > Cj) { if (aj > Cj) { aj = Cj; ai = sum - Cj; } }
        else { if (ai < 0) { ai = 0; aj = sum; } }
      }
      a[i] = ai; a[j] = aj;
      upd[0] = ai - oai; upd[1] = aj - oaj;
    }
    __syncthreads();
    const double dai = upd[0], daj = upd[1];
    // gradient update fused with the next iteration's i-selection
    ci = Cand{-kInf, -1};
    for (int64_t t = threadIdx.x; t < L; t += NT) {
      const double yt = y[t];
      const int64_t rt = rowof(t);
      const double gt = g[t] + yt * (yi * (double)Ki[rt] * dai + yj * (double)Kj[rt] * daj);
      g[t] = gt;
      const bool up = yt > 0 ? !is_upper(a[t], C[t]) : !is_lower(a[t]);
      if (up) {
        const double v = -yt * gt;
        if (better<true>(v, (int)t, ci.v, ci.idx)) { ci.v = v; ci.idx = (int)t; }
      }
    }
    ++it;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    P.iters = it;
    P.status = status;
  }
}

}  // namespace

extern "C" {

int dml_svm_sizeof_prob() { return (int)sizeof(SvmProb); }

// X: concatenated feature-major rowsets; probs: device array of SvmProb (iters/status updated).
int dml_svm_smo(const float* X, int64_t d, void* probs, int64_t nprob, const float* y, const double* C,
                const float* qd, double* alpha, double* G, float* kbuf, int64_t chunk, hipStream_t st) {
  if (nprob <= 0) return 0;
  k_smo<<<(unsigned)nprob, NT, 0, st>>>(X, d, (SvmProb*)probs, y, C, qd, alpha, G, kbuf, chunk);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
