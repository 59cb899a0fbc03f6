// svm_cpu.cpp — the batched SMO solver of svm.hip on the host (no-GPU path and oracle).
//
// Same dual algorithm as libsvm's Solver (what sklearn SVC/SVR run per fit, reference
// aws-prod/worker/worker.py:40,47): WSS3 second-order working-set selection, analytic
// two-variable update, gradient maintenance, eps stopping rule, later index wins ties.
// Problems are independent and run in parallel with OpenMP.
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

namespace {

constexpr double kTau = 1e-12;
constexpr double kInf = 1e300;
enum { KLIN = 0, KPOLY = 1, KRBF = 2, KSIG = 3 };

struct SvmProb {
  int64_t xoff, roff, nrows, L, voff, koff, kernel, degree;
  double gamma, coef0, eps;
  int64_t max_iter, iters, status, svr;
  int64_t coff, moff;   // GPU split solver only (svm.hip)
};

float kfun(int kernel, double gamma, double coef0, int degree, float acc) {
  switch (kernel) {
    case KRBF: return (float)std::exp(-gamma * (double)acc);
    case KPOLY: {
      const double b = gamma * (double)acc + coef0;
      double r = 1.0;
      for (int i = 0; i < degree; ++i) r *= b;
      return (float)r;
    }
    case KSIG: return (float)std::tanh(gamma * (double)acc + coef0);
    default: return acc;
  }
}

void column(const SvmProb& p, const float* X, int64_t d, int64_t src, float* col) {
  const float* base = X + p.xoff;
  for (int64_t r = 0; r < p.nrows; ++r) {
    float acc = 0.f;
    if (p.kernel == KRBF) {
      for (int64_t f = 0; f < d; ++f) {
        const float t = base[f * p.nrows + src] - base[f * p.nrows + r];
        acc = std::fma(t, t, acc);
      }
    } else {
      for (int64_t f = 0; f < d; ++f) acc = std::fma(base[f * p.nrows + src], base[f * p.nrows + r], acc);
    }
    col[r] = kfun((int)p.kernel, p.gamma, p.coef0, (int)p.degree, acc);
  }
}

void solve(SvmProb& p, const float* X, int64_t d, const float* yv, const double* Cv, const float* qd, double* alpha,
           double* G) {
  const int64_t L = p.L, nr = p.nrows;
  const float* y = yv + p.voff;
  const double* C = Cv + p.voff;
  double* a = alpha + p.voff;
  double* g = G + p.voff;
  const float* QD = qd + p.roff;
  std::vector<float> Ki(nr), Kj(nr);
  auto rowof = [&](int64_t t) { return (p.svr && t >= nr) ? t - nr : t; };
  int64_t it = p.iters;
  int status = 2;
  while (it < p.max_iter) {
    double Gmax = -kInf;
    int64_t i = -1;
    for (int64_t t = 0; t < L; ++t) {
      const bool up = y[t] > 0 ? a[t] < C[t] : a[t] > 0;
      if (up && -y[t] * g[t] >= Gmax) { Gmax = -y[t] * g[t]; i = t; }
    }
    if (i < 0) { status = 1; break; }
    const double yi = y[i];
    const int64_t ri = rowof(i);
    column(p, X, d, ri, Ki.data());
    double Gmax2 = -kInf, odmin = kInf;
    int64_t j = -1;
    const double QDi = QD[ri];
    for (int64_t t = 0; t < L; ++t) {
      const double yt = y[t];
      const int64_t rt = rowof(t);
      const double kit = Ki[rt];
      if (yt > 0) {
        if (a[t] > 0) {
          const double gd = Gmax + g[t];
          if (g[t] >= Gmax2) Gmax2 = g[t];
          if (gd > 0) {
            const double qc = QDi + QD[rt] - 2.0 * yi * (yi * yt * kit);
            const double od = qc > 0 ? -(gd * gd) / qc : -(gd * gd) / kTau;
            if (od <= odmin) { odmin = od; j = t; }
          }
        }
      } else {
        if (a[t] < C[t]) {
          const double gd = Gmax - g[t];
          if (-g[t] >= Gmax2) Gmax2 = -g[t];
          if (gd > 0) {
            const double qc = QDi + QD[rt] + 2.0 * yi * (yi * yt * kit);
            const double od = qc > 0 ? -(gd * gd) / qc : -(gd * gd) / kTau;
            if (od <= odmin) { odmin = od; j = t; }
          }
        }
      }
    }
    if (Gmax + Gmax2 < p.eps || j < 0) { status = 1; break; }
    const double yj = y[j];
    const int64_t rj = rowof(j);
    column(p, X, d, rj, Kj.data());
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
    const double dai = ai - oai, daj = aj - oaj;
    for (int64_t t = 0; t < L; ++t) {
      const int64_t rt = rowof(t);
      g[t] += y[t] * (yi * (double)Ki[rt] * dai + yj * (double)Kj[rt] * daj);
    }
    ++it;
  }
  p.iters = it;
  p.status = status;
}

}  // namespace

extern "C" {

int dml_cpu_svm_sizeof_prob() { return (int)sizeof(SvmProb); }

void dml_cpu_svm_smo(const float* X, int64_t d, void* probs, int64_t nprob, const float* y, const double* C,
                     const float* qd, double* alpha, double* G) {
  SvmProb* P = (SvmProb*)probs;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t k = 0; k < nprob; ++k)
    if (P[k].status == 0) solve(P[k], X, d, y, C, qd, alpha, G);
}

}  // extern "C"
