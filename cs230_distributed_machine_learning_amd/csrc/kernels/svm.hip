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

#include "wave_ops.h"

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
  int64_t coff;      // split solver: kernel-column cache, S * nrows floats at coff
  int64_t moff;      // split solver: per-workgroup cache maps, B * (nrows + 2 S) ints at moff
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
  const int lane = threadIdx.x & 63;
#define SVM_BR(M) { const double ov = dml::wave::shfl_xor<M>(c.v, lane); const int oi = dml::wave::shfl_xor<M>(c.idx, lane); \
                    if (better<MAX>(ov, oi, c.v, c.idx)) { c.v = ov; c.idx = oi; } }
  SVM_BR(32) SVM_BR(16) SVM_BR(8) SVM_BR(4) SVM_BR(2) SVM_BR(1)
#undef SVM_BR
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
  const int lane = threadIdx.x & 63;
  v = fmax(v, dml::wave::shfl_xor<32>(v, lane)); v = fmax(v, dml::wave::shfl_xor<16>(v, lane));
  v = fmax(v, dml::wave::shfl_xor<8>(v, lane)); v = fmax(v, dml::wave::shfl_xor<4>(v, lane));
  v = fmax(v, dml::wave::shfl_xor<2>(v, lane)); v = fmax(v, dml::wave::shfl_xor<1>(v, lane));
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

// ======================================================================================
// Split SMO: B workgroups per dual problem + an LRU kernel-column cache in HBM.
//
// One workgroup per problem leaves most of the 256 CUs idle (a job has tens of problems)
// and recomputes two kernel columns per iteration.  Here workgroup w of problem p owns
// the row slice [r0, r1) (and, for epsilon-SVR, the variables of those rows): the
// selection sweeps, the kernel-column slices and the gradient update are slice-local, and
// per SMO iteration the B workgroups exchange only two small records (the slice's best i
// candidate with its G / alpha; the best j candidate with its G / alpha and max y G).
// Each record word is a 64-bit agent-scope atomic carrying (sequence tag << 32 | 32
// payload bits), so a reader spins until every word of a record shows the current tag:
// no grid barrier, no cache-wide fences.  Every workgroup then reduces the B records in
// the same order and runs the same two-variable update, so all of them take identical
// decisions (libsvm's selection, update and stopping rules, as k_smo).
//
// Kernel columns go through an LRU cache of S columns per problem (libsvm's Kernel
// cache, here S * nrows floats in HBM): the slot map (row -> slot) and the slot stamps
// are replicated per workgroup -- every replica sees the same i/j sequence, so all make
// the same hit/miss/victim decisions with no shared writes -- and each workgroup fills or
// reads only its own slice of a slot.
//
// Co-residency: a record spin needs all B workgroups of its problem running; the host
// keeps the grid within the occupancy bound (checked in dml_svm_smo_split) and every spin
// gives up after kSpinLimit polls (status 3: the host reports an error, no hang).
constexpr int kRecW = 12;                 // 64-bit words per record
constexpr int kMaxB = 21;                 // workgroups per problem (B * kRecW <= NT: records read in one round;
                                          // 39 measured slower, 12.5 vs 11.4 s: longer exchanges)
constexpr int kMaxSlots = 1 << 16;        // cache slots per problem
constexpr uint64_t kSpinLimit = 1ull << 22;  // ~5 s of polling: a stuck peer ends the launch, not the GPU
constexpr int kTagN = 4096;               // LDS row -> slot tags in front of the cache map (power of two)
// kSweepU: variables per thread per sweep step.  The wide variant (8: a slice of <= 2048
// rows is ONE step, one memory round trip per sweep) holds more registers (one wave per
// SIMD), so the host uses it only when few problems remain (the long tail of a search:
// the last large-C problems); 4 keeps two waves per SIMD for the crowded early launches.

__device__ __forceinline__ void rec_put(uint64_t* w, uint32_t tag, uint32_t payload) {
  __hip_atomic_store(w, ((uint64_t)tag << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lo32(double v) { return (uint32_t)__builtin_bit_cast(uint64_t, v); }
__device__ __forceinline__ uint32_t hi32(double v) { return (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32); }
__device__ __forceinline__ double mkd(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

struct SplitCtx {
  int B, w, S;
  int64_t r0, r1;
};

// a working-set candidate with the values its exchange record carries (G, alpha, C, y, QD,
// K(i, t)): the lane that found it already holds them, so the record needs no global load
// after the block reduction
struct CandP {
  double v;
  int idx;
  double g, a, c;
  float y, q, k;
};

// the block's best candidate: a wave butterfly over (value, index, source lane) only -- the
// winning lane then stores its whole record -- and, fused into the same pass (one pair of
// barriers), the block max of `mx` (the j sweep's max over I_low of y G)
template <bool MAX>
__device__ CandP block_reduce_p(CandP c, CandP* red, double& mx, double* redd) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double v = c.v;
  int idx = c.idx, src = lane;
  // butterfly steps on DPP / permlane (VALU), not ds_bpermute (an LDS round trip per step)
#define SVM_BRP(M) { const double ov = dml::wave::shfl_xor<M>(v, lane); \
                     const int oi = dml::wave::shfl_xor<M>(idx, lane), os = dml::wave::shfl_xor<M>(src, lane); \
                     if (better<MAX>(ov, oi, v, idx)) { v = ov; idx = oi; src = os; } \
                     mx = fmax(mx, dml::wave::shfl_xor<M>(mx, lane)); }
  SVM_BRP(32) SVM_BRP(16) SVM_BRP(8) SVM_BRP(4) SVM_BRP(2) SVM_BRP(1)
#undef SVM_BRP
  if (lane == src) red[wid] = c;        // the wave's winner (src is wave-uniform after the butterfly)
  if (lane == 0) redd[wid] = mx;
  __syncthreads();
  CandP r = red[0];
  double m2 = redd[0];
  for (int w = 1; w < NT / 64; ++w) {
    if (better<MAX>(red[w].v, red[w].idx, r.v, r.idx)) r = red[w];
    m2 = fmax(m2, redd[w]);
  }
  __syncthreads();
  mx = m2;
  return r;
}

// publish this workgroup's record (payload words v[0..n)) and gather all B records of the
// exchange into pay[B][kRecW]; returns false if a spin gave up
__device__ bool exchange(uint64_t* rec, const SplitCtx& sc, uint32_t seq, const uint32_t* v, int n,
                         uint32_t* pay, int* abort_flag) {
  uint64_t* mine = rec + ((int64_t)(seq & 1) * sc.B + sc.w) * kRecW;
  if (threadIdx.x < n) rec_put(mine + threadIdx.x, seq, v[threadIdx.x]);
  const int total = sc.B * kRecW;
  for (int q = threadIdx.x; q < total; q += NT) {
    if ((q % kRecW) >= n) continue;
    const uint64_t* src = rec + (int64_t)(seq & 1) * sc.B * kRecW + q;
    uint64_t x;
    uint64_t spins = 0;
    while (true) {
      x = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)(x >> 32) == seq) break;
      if (++spins > kSpinLimit) { *abort_flag = 1; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    pay[q] = (uint32_t)x;
  }
  __syncthreads();
  return *abort_flag == 0;
}

// the winning record of an exchange (wave 0: lane q holds record q, a butterfly argmax with
// the `better` order -- a strict total order on (value, index) pairs, so the same record the
// sequential scan picks), and for MAX = false the max over all records of the double at
// words [7, 8] (Gmax2).  Every thread then reads only the winner's words (one LDS broadcast
// each) instead of scanning all B records itself.
template <bool MAX>
__device__ void pick_record(const uint32_t* pay, int B, int* s_win, double* s_g2) {
  if (threadIdx.x < 64) {
    const int q = threadIdx.x;
    const uint32_t* r = pay + q * kRecW;
    double v = q < B ? mkd(r[0], r[1]) : 0.0;
    int idx = q < B ? (int)r[2] : -1;
    int who = q;
    double g2 = (!MAX && q < B) ? mkd(r[7], r[8]) : -kInf;
#define SVM_PR(M) { const double ov = dml::wave::shfl_xor<M>(v, q); \
                    const int oi = dml::wave::shfl_xor<M>(idx, q), ow = dml::wave::shfl_xor<M>(who, q); \
                    if (better<MAX>(ov, oi, v, idx)) { v = ov; idx = oi; who = ow; } \
                    if (!MAX) g2 = fmax(g2, dml::wave::shfl_xor<M>(g2, q)); }
    SVM_PR(32) SVM_PR(16) SVM_PR(8) SVM_PR(4) SVM_PR(2) SVM_PR(1)
#undef SVM_PR
    if (q == 0) {
      *s_win = idx >= 0 ? who : -1;
      if (!MAX) *s_g2 = g2;
    }
  }
  __syncthreads();
}

// kernel value of rowset rows (a, b) -- the same arithmetic as kernel_column's entry
__device__ float kernel_pair(const SvmProb& p, const float* X, int64_t d, int64_t a, int64_t b) {
  const float* base = X + p.xoff;
  float acc = 0.f;
  if (p.kernel == KRBF) {
    for (int64_t f = 0; f < d; ++f) {
      const float t = base[f * p.nrows + a] - base[f * p.nrows + b];
      acc = __builtin_fmaf(t, t, acc);
    }
  } else {
    for (int64_t f = 0; f < d; ++f) acc = __builtin_fmaf(base[f * p.nrows + a], base[f * p.nrows + b], acc);
  }
  return kfun((int)p.kernel, p.gamma, p.coef0, (int)p.degree, acc);
}

// column of rowset row `src`, rows [r0, r1) only.  Each thread carries 4 rows (stride NT)
// through an unrolled feature loop so 4 x 4 independent loads are in flight (a one-row
// fma chain waits out one memory latency per feature); the per-row arithmetic (feature
// order, fmaf chain) is kernel_column's.
__device__ void column_slice(const SvmProb& p, const float* __restrict__ X, int64_t d, int64_t src, float* xs,
                             float* __restrict__ col, int64_t r0, int64_t r1) {
  const bool lds = d <= kMaxLdsD;
  const float* base = X + p.xoff;
  if (lds) {
    for (int64_t f = threadIdx.x; f < d; f += NT) xs[f] = base[f * p.nrows + src];
    __syncthreads();
  }
  const int kernel = (int)p.kernel;
  const int64_t nr = p.nrows;
  for (int64_t rb = r0 + threadIdx.x; rb < r1; rb += 4 * NT) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t rr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rr[k] = min(rb + k * NT, r1 - 1);   // clamped: the tail recomputes a valid row
    // features in blocks of kColF: the block's 4 x kColF loads are all issued before its
    // first FMA (a cache miss is a memory round trip per BLOCK of features, not per 4);
    // the FMA order per row is unchanged (f ascending), so every entry is the same float
    constexpr int kColF = 16;
    for (int64_t f0 = 0; f0 < d; f0 += kColF) {
      float xv[kColF][4];
#pragma unroll
      for (int q = 0; q < kColF; ++q) {
        const int64_t f = min(f0 + q, d - 1);
        const float* xf = base + f * nr;
#pragma unroll
        for (int k = 0; k < 4; ++k) xv[q][k] = xf[rr[k]];
      }
#pragma unroll
      for (int q = 0; q < kColF; ++q) {
        if (f0 + q >= d) break;
        const int64_t f = f0 + q;
        const float a = lds ? xs[f] : base[f * nr + src];
        if (kernel == KRBF) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float t = a - xv[q][k];
            acc[k] = __builtin_fmaf(t, t, acc[k]);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] = __builtin_fmaf(a, xv[q][k], acc[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (rb + k * NT < r1) col[rb + k * NT] = kfun(kernel, p.gamma, p.coef0, (int)p.degree, acc[k]);
  }
  __syncthreads();
}

// LRU-style lookup of the column of `row` in this workgroup's replica of the cache map;
// fills the slice on a miss.  Victim: the least recently used of 256 slots sampled by a
// hash of the tick (all slots when S <= 256, i.e. exact LRU) -- O(1) per miss for any S
// and the same choice in every replica.  Returns the slot's column base.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// The workgroup's replica of the map is fronted by an LDS tag array (kTagN direct-mapped
// row -> slot entries, kept exact: set on every lookup, cleared when a slot's old row is
// evicted), so a hit on a recently used row costs one LDS read instead of a global round
// trip and two barriers (SMO revisits a small working set: ~90 % of the lookups hit).
__device__ float* cache_column(const SvmProb& p, const float* X, int64_t d, float* kc, int32_t* slot_of,
                               int32_t* row_of, uint32_t* stamp, uint32_t tick, int64_t row, const SplitCtx& sc,
                               float* xs, int* s_slot, int* s_red, int32_t* tag_row, int32_t* tag_slot,
                               int* s_miss) {
  const int h = (int)(row & (kTagN - 1));
  if (tag_row[h] == (int32_t)row) {   // uniform: every thread reads the same LDS word
    const int slot = tag_slot[h];
    if (threadIdx.x == 0) stamp[slot] = tick;
    return kc + p.coff + (int64_t)slot * p.nrows;
  }
  int slot = __builtin_amdgcn_readfirstlane(slot_of[row]);   // the same word in every lane
  const bool hit = slot >= 0;
  __syncthreads();   // every thread has read the tag before thread 0 rewrites it
  if (hit) {
    if (threadIdx.x == 0) { tag_row[h] = (int32_t)row; tag_slot[h] = slot; stamp[slot] = tick; }
    return kc + p.coff + (int64_t)slot * p.nrows;
  }
  {
    const uint32_t cand = sc.S <= NT ? (uint32_t)threadIdx.x : mix32(tick * 2654435761U + threadIdx.x) % (uint32_t)sc.S;
    uint64_t best = cand < (uint32_t)sc.S ? (((uint64_t)stamp[cand] << 32) | cand) : ~0ull;
    for (int m = 32; m >= 1; m >>= 1) {
      const uint64_t o = __shfl_xor(best, m);
      best = o < best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) reinterpret_cast<uint64_t*>(s_red)[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t bb = reinterpret_cast<uint64_t*>(s_red)[0];
      for (int q = 1; q < NT / 64; ++q) {
        const uint64_t o = reinterpret_cast<uint64_t*>(s_red)[q];
        bb = o < bb ? o : bb;
      }
      const int v = (int)(uint32_t)bb;
      const int old = row_of[v];
      if (old >= 0) {
        slot_of[old] = -1;
        if (tag_row[old & (kTagN - 1)] == old) tag_row[old & (kTagN - 1)] = -1;
      }
      slot_of[row] = v;
      row_of[v] = (int32_t)row;
      tag_row[h] = (int32_t)row;
      tag_slot[h] = v;
      *s_slot = v;
      ++*s_miss;   // (profiling)
    }
    __syncthreads();
    slot = *s_slot;
  }
  if (threadIdx.x == 0) stamp[slot] = tick;
  float* col = kc + p.coff + (int64_t)slot * p.nrows;
  column_slice(p, X, d, row, xs, col, sc.r0, sc.r1);
  __syncthreads();
  return col;
}

template <int kSweepU>
__global__ __launch_bounds__(NT) void k_smo_split(const float* __restrict__ X, int64_t d, const SvmProb* probs,
                                                  int B, int S, const float* __restrict__ yv,
                                                  const double* __restrict__ Cv, const float* __restrict__ qd,
                                                  double* __restrict__ alpha, double* __restrict__ G,
                                                  float* __restrict__ kc, int32_t* __restrict__ meta,
                                                  uint64_t* __restrict__ recs, int64_t* __restrict__ out_state,
                                                  int64_t chunk, int64_t* __restrict__ prof) {
  // prof (optional, workgroup 0 only): wall-clock ticks per phase + cache misses
  int64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tph = wall_clock64();
  const bool do_prof = prof != nullptr && blockIdx.x == 0;
#define SVM_PH(k) if (do_prof) { const uint64_t t_ = wall_clock64(); ph[k] += (int64_t)(t_ - tph); tph = t_; }
  const int pid = blockIdx.x / B;
  const SvmProb p = probs[pid];
  if (p.status != 0) return;
  __shared__ float xs[kMaxLdsD];
  __shared__ CandP red[NT / 64];
  __shared__ double redd[NT / 64];
  __shared__ uint32_t pay[kMaxB * kRecW];
  __shared__ int s_slot, s_abort;
  __shared__ uint32_t vals[kRecW];
  __shared__ int s_red[2 * (NT / 64)];
  __shared__ int32_t tag_row[kTagN], tag_slot[kTagN];
  __shared__ int s_miss, s_win;
  __shared__ double s_g2;
  for (int q = threadIdx.x; q < kTagN; q += NT) tag_row[q] = -1;
  if (threadIdx.x == 0) s_miss = 0;
  SplitCtx sc;
  sc.B = B;
  sc.w = blockIdx.x - pid * B;
  sc.S = S;
  const int64_t nr = p.nrows, L = p.L;
  sc.r0 = nr * sc.w / B;
  sc.r1 = nr * (sc.w + 1) / B;
  const float* y = yv + p.voff;
  const double* C = Cv + p.voff;
  double* a = alpha + p.voff;
  double* g = G + p.voff;
  const float* QD = qd + p.roff;
  uint64_t* rec = recs + (int64_t)pid * 2 * B * kRecW;
  int32_t* my_meta = meta + p.moff + (int64_t)sc.w * (nr + 2 * S);
  int32_t* slot_of = my_meta;                 // [nr]
  int32_t* row_of = my_meta + nr;             // [S]
  uint32_t* stamp = reinterpret_cast<uint32_t*>(my_meta + nr + S);   // [S]
  if (threadIdx.x == 0) s_abort = 0;
  __syncthreads();
  auto rowof = [&](int64_t t) { return (p.svr && t >= nr) ? t - nr : t; };
  const int nseg = p.svr ? 2 : 1;             // this slice's variables: [r0,r1) (+ nr for SVR)
  // wide variant, one-segment slice of <= kSweepU * NT variables: the slice's y, alpha, C, G and
  // QD stay in registers for the whole launch (thread tid owns variables r0 + tid + k NT), so
  // each sweep loads only its kernel-column entries; G / alpha go back to memory at the end
  constexpr int RU = kSweepU == 8 ? 8 : 1;
  const bool regst = kSweepU == 8 && nseg == 1 && sc.r1 - sc.r0 <= (int64_t)kSweepU * NT;
  float rs_y[RU], rs_q[RU], rs_ki[RU];
  double rs_a[RU], rs_C[RU], rs_g[RU];
  if constexpr (kSweepU == 8) {
    if (regst) {
#pragma unroll
      for (int k = 0; k < RU; ++k) {
        const int64_t t = min(sc.r0 + threadIdx.x + k * NT, sc.r1 - 1);
        rs_y[k] = y[t]; rs_a[k] = a[t]; rs_C[k] = C[t]; rs_g[k] = g[t]; rs_q[k] = QD[t]; rs_ki[k] = 0.f;
      }
    }
  }

  int64_t it = p.iters;
  int status = 0;
  uint32_t seq = 0;
  const int64_t stop_at = min(p.max_iter, it + chunk);
  auto local_i = [&]() {
    CandP ci{-kInf, -1, 0.0, 0.0, 0.0, 0.f, 0.f, 0.f};
    if constexpr (kSweepU == 8) {
      if (regst) {
#pragma unroll
        for (int k = 0; k < RU; ++k) {
          const int64_t t = sc.r0 + threadIdx.x + k * NT;
          if (t >= sc.r1) break;
          const bool up = rs_y[k] > 0 ? !is_upper(rs_a[k], rs_C[k]) : !is_lower(rs_a[k]);
          if (up) {
            const double v = -(double)rs_y[k] * rs_g[k];
            if (better<true>(v, (int)t, ci.v, ci.idx))
              ci = CandP{v, (int)t, rs_g[k], rs_a[k], rs_C[k], rs_y[k], rs_q[k], 0.f};
          }
        }
        return ci;
      }
    }
    for (int sgi = 0; sgi < nseg; ++sgi)
      for (int64_t t = sc.r0 + sgi * nr + threadIdx.x; t < sc.r1 + sgi * nr; t += NT) {
        const double yt = y[t], at = a[t], Ct = C[t], gt = g[t];
        const bool up = yt > 0 ? !is_upper(at, Ct) : !is_lower(at);
        if (up) {
          const double v = -yt * gt;
          if (better<true>(v, (int)t, ci.v, ci.idx))
            ci = CandP{v, (int)t, gt, at, Ct, (float)yt, QD[rowof(t)], 0.f};
        }
      }
    return ci;
  };
  CandP ci = local_i();
  while (true) {
    if (it >= stop_at) { status = it >= p.max_iter ? 2 : 0; break; }
    // ---- exchange 1: i = argmax over I_up of -y G (with G_i, alpha_i) ----
    double unused_mx = -kInf;
    const CandP bi_l = block_reduce_p<true>(ci, red, unused_mx, redd);
    if (threadIdx.x == 0) {
      // the candidate's own per-variable values travel with it (G, alpha, y, QD, C: no
      // dependent loads, here or by the other workgroups once the winner is known)
      const int t = bi_l.idx;
      vals[0] = lo32(bi_l.v); vals[1] = hi32(bi_l.v); vals[2] = (uint32_t)t;
      vals[3] = lo32(bi_l.g); vals[4] = hi32(bi_l.g); vals[5] = lo32(bi_l.a); vals[6] = hi32(bi_l.a);
      vals[7] = __float_as_uint(bi_l.y); vals[8] = __float_as_uint(bi_l.q);
      vals[9] = lo32(bi_l.c); vals[10] = hi32(bi_l.c);
    }
    __syncthreads();
    SVM_PH(0)
    if (!exchange(rec, sc, ++seq, vals, 11, pay, &s_abort)) { status = 3; break; }
    SVM_PH(1)
    double Gmax = -kInf, gi = 0.0, ai_old = 0.0, Ci = 0.0;
    float yi_f = 0.f, QDi_f = 0.f;
    int i = -1;
    pick_record<true>(pay, B, &s_win, &s_g2);
    if (s_win >= 0) {
      const uint32_t* r = pay + s_win * kRecW;
      Gmax = mkd(r[0], r[1]); i = (int)r[2]; gi = mkd(r[3], r[4]); ai_old = mkd(r[5], r[6]);
      yi_f = __uint_as_float(r[7]); QDi_f = __uint_as_float(r[8]); Ci = mkd(r[9], r[10]);
    }
    __syncthreads();
    if (i < 0) { status = 1; break; }
    const double yi = yi_f;
    const int64_t ri = rowof(i);
    const uint32_t tick = (uint32_t)(2 * (it + 1));
    const float* Ki = cache_column(p, X, d, kc, slot_of, row_of, stamp, tick, ri, sc, xs, &s_slot, s_red, tag_row,
                                   tag_slot, &s_miss);
    SVM_PH(2)
    // ---- local j candidates (second-order gain) + max over I_low of y G ----
    // 4 variables per thread per step, every load issued before any use (latency-bound
    // sweep); selection ties break by index, so the visiting order does not matter
    CandP cj{kInf, -1, 0.0, 0.0, 0.0, 0.f, 0.f, 0.f};
    double gmax2 = -kInf;
    const double QDi = QDi_f;
    // one j candidate: the same selection arithmetic for both state layouts
    auto j_cand = [&](int64_t t, double yt, double at, double Ct, double gt, float qt, float kt) {
      if (yt > 0) {
        if (!is_lower(at)) {
          const double gd = Gmax + gt;
          gmax2 = fmax(gmax2, gt);
          if (gd > 0) {
            double qc = QDi + (double)qt - 2.0 * yi * (yi * yt * (double)kt);
            const double od = qc > 0 ? -(gd * gd) / qc : -(gd * gd) / kTau;
            if (better<false>(od, (int)t, cj.v, cj.idx)) cj = CandP{od, (int)t, gt, at, Ct, (float)yt, qt, kt};
          }
        }
      } else {
        if (!is_upper(at, Ct)) {
          const double gd = Gmax - gt;
          gmax2 = fmax(gmax2, -gt);
          if (gd > 0) {
            double qc = QDi + (double)qt + 2.0 * yi * (yi * yt * (double)kt);
            const double od = qc > 0 ? -(gd * gd) / qc : -(gd * gd) / kTau;
            if (better<false>(od, (int)t, cj.v, cj.idx)) cj = CandP{od, (int)t, gt, at, Ct, (float)yt, qt, kt};
          }
        }
      }
    };
    bool swept = false;
    if constexpr (kSweepU == 8) {
      if (regst) {   // registers hold the slice: only column i's entries are loaded
#pragma unroll
        for (int k = 0; k < RU; ++k) rs_ki[k] = Ki[min(sc.r0 + threadIdx.x + k * NT, sc.r1 - 1)];
#pragma unroll
        for (int k = 0; k < RU; ++k) {
          const int64_t t = sc.r0 + threadIdx.x + k * NT;
          if (t >= sc.r1) break;
          j_cand(t, (double)rs_y[k], rs_a[k], rs_C[k], rs_g[k], rs_q[k], rs_ki[k]);
        }
        swept = true;
      }
    }
    for (int sgi = 0; sgi < nseg && !swept; ++sgi) {
      const int64_t lo = sc.r0 + sgi * nr, hi = sc.r1 + sgi * nr;
      for (int64_t tb = lo + threadIdx.x; tb < hi; tb += kSweepU * NT) {
        float yk[kSweepU], kk[kSweepU], qk[kSweepU];
        double ak[kSweepU], Ck[kSweepU], gk[kSweepU];
#pragma unroll
        for (int k = 0; k < kSweepU; ++k) {
          const int64_t t = min(tb + k * NT, hi - 1);
          const int64_t rt = rowof(t);
          yk[k] = y[t]; ak[k] = a[t]; Ck[k] = C[t]; gk[k] = g[t]; kk[k] = Ki[rt]; qk[k] = QD[rt];
        }
#pragma unroll
        for (int k = 0; k < kSweepU; ++k) {
          const int64_t t = tb + k * NT;
          if (t >= hi) break;
          j_cand(t, (double)yk[k], ak[k], Ck[k], gk[k], qk[k], kk[k]);
        }
      }
    }
    double gm2_l = gmax2;
    const CandP bj_l = block_reduce_p<false>(cj, red, gm2_l, redd);
    if (threadIdx.x == 0) {
      // K(i, j) of the slice's j comes from the slice of column i it just filled: the entry
      // kernel_pair would recompute with the same arithmetic (every workgroup takes it from
      // the winning record, no workgroup recomputes it)
      const int t = bj_l.idx;
      vals[0] = lo32(bj_l.v); vals[1] = hi32(bj_l.v); vals[2] = (uint32_t)t;
      vals[3] = lo32(bj_l.g); vals[4] = hi32(bj_l.g); vals[5] = lo32(bj_l.a); vals[6] = hi32(bj_l.a);
      vals[7] = lo32(gm2_l); vals[8] = hi32(gm2_l); vals[9] = __float_as_uint(bj_l.k);
      vals[10] = __float_as_uint(bj_l.y); vals[11] = __float_as_uint(bj_l.q);
    }
    __syncthreads();
    SVM_PH(3)
    // ---- exchange 2 ----
    if (!exchange(rec, sc, ++seq, vals, 12, pay, &s_abort)) { status = 3; break; }
    SVM_PH(4)
    double bjv = kInf, gj = 0.0, aj_old = 0.0, Gmax2 = -kInf;
    float kij = 0.f, yj_f = 0.f, QDj_f = 0.f;
    int j = -1;
    pick_record<false>(pay, B, &s_win, &s_g2);
    Gmax2 = s_g2;
    if (s_win >= 0) {
      const uint32_t* r = pay + s_win * kRecW;
      bjv = mkd(r[0], r[1]); j = (int)r[2]; gj = mkd(r[3], r[4]); aj_old = mkd(r[5], r[6]);
      kij = __uint_as_float(r[9]); yj_f = __uint_as_float(r[10]); QDj_f = __uint_as_float(r[11]);
    }
    __syncthreads();
    if (Gmax + Gmax2 < p.eps || j < 0) { status = 1; break; }
    const double Cj = C[j];   // issued before the cache lookup, used by the update
    const double yj = yj_f;
    const int64_t rj = rowof(j);
    const float* Kj = cache_column(p, X, d, kc, slot_of, row_of, stamp, tick + 1, rj, sc, xs, &s_slot, s_red, tag_row,
                                   tag_slot, &s_miss);
    SVM_PH(5)
    // ---- two-variable update: every workgroup computes the same values ----
    const double Qij = yi * yj * (double)kij;
    const double QDj = QDj_f;
    double ai = ai_old, aj = aj_old;
    if (yi != yj) {
      double qc = QDi + QDj + 2.0 * Qij;
      if (qc <= 0) qc = kTau;
      const double delta = (-gi - gj) / qc;
      const double diff = ai - aj;
      ai += delta; aj += delta;
      if (diff > 0) { if (aj < 0) { aj = 0; ai = diff; } }
      else { if (ai < 0) { ai = 0; aj = -diff; } }
      if (diff > Ci - Cj) { if (ai > Ci) { ai = Ci; aj = Ci - diff; } }
      else { if (aj > Cj) { aj = Cj; ai = Cj + diff; } }
    } else {
      double qc = QDi + QDj - 2.0 * Qij;
      if (qc <= 0) qc = kTau;
      const double delta = (gi - gj) / qc;
      const double sum = ai + aj;
      ai -= delta; aj += delta;
      if (sum > Ci) { if (ai > Ci) { ai = Ci; aj = sum - Ci; } }
      else { if (aj < 0) { aj = 0; ai = sum; } }
      if (sum > Cj) { if (aj > Cj) { aj = Cj; ai = sum - Cj; } }
      else { if (ai < 0) { ai = 0; aj = sum; } }
    }
    const double dai = ai - ai_old, daj = aj - aj_old;
    auto owns = [&](int t) { const int64_t r = rowof(t); return r >= sc.r0 && r < sc.r1; };
    if (threadIdx.x == 0) {
      if (owns(i)) a[i] = ai;
      if (owns(j)) a[j] = aj;
    }
    __syncthreads();
    // gradient update of this slice fused with its next i candidates (4 per thread per step)
    ci = CandP{-kInf, -1, 0.0, 0.0, 0.0, 0.f, 0.f, 0.f};
    bool updated = false;
    if constexpr (kSweepU == 8) {
      if (regst) {   // column i's entries are still in registers from the j sweep
        float kjr[RU];
#pragma unroll
        for (int k = 0; k < RU; ++k) kjr[k] = Kj[min(sc.r0 + threadIdx.x + k * NT, sc.r1 - 1)];
#pragma unroll
        for (int k = 0; k < RU; ++k) {
          const int64_t t = sc.r0 + threadIdx.x + k * NT;
          if (t >= sc.r1) break;
          if (t == i) rs_a[k] = ai;
          if (t == j) rs_a[k] = aj;
          const double yt = rs_y[k];
          const double gt = rs_g[k] + yt * (yi * (double)rs_ki[k] * dai + yj * (double)kjr[k] * daj);
          rs_g[k] = gt;
          const bool up = yt > 0 ? !is_upper(rs_a[k], rs_C[k]) : !is_lower(rs_a[k]);
          if (up) {
            const double v = -yt * gt;
            if (better<true>(v, (int)t, ci.v, ci.idx)) ci = CandP{v, (int)t, gt, rs_a[k], rs_C[k], rs_y[k], rs_q[k], 0.f};
          }
        }
        updated = true;
      }
    }
    for (int sgi = 0; sgi < nseg && !updated; ++sgi) {
      const int64_t lo = sc.r0 + sgi * nr, hi = sc.r1 + sgi * nr;
      for (int64_t tb = lo + threadIdx.x; tb < hi; tb += kSweepU * NT) {
        float yk[kSweepU], kik[kSweepU], kjk[kSweepU], qk[kSweepU];
        double ak[kSweepU], Ck[kSweepU], gk[kSweepU];
#pragma unroll
        for (int k = 0; k < kSweepU; ++k) {
          const int64_t t = min(tb + k * NT, hi - 1);
          const int64_t rt = rowof(t);
          yk[k] = y[t]; ak[k] = a[t]; Ck[k] = C[t]; gk[k] = g[t]; kik[k] = Ki[rt]; kjk[k] = Kj[rt]; qk[k] = QD[rt];
        }
#pragma unroll
        for (int k = 0; k < kSweepU; ++k) {
          const int64_t t = tb + k * NT;
          if (t >= hi) break;
          const double yt = yk[k];
          const double gt = gk[k] + yt * (yi * (double)kik[k] * dai + yj * (double)kjk[k] * daj);
          g[t] = gt;
          const bool up = yt > 0 ? !is_upper(ak[k], Ck[k]) : !is_lower(ak[k]);
          if (up) {
            const double v = -yt * gt;
            if (better<true>(v, (int)t, ci.v, ci.idx)) ci = CandP{v, (int)t, gt, ak[k], Ck[k], yk[k], qk[k], 0.f};
          }
        }
      }
    }
    ++it;
    __syncthreads();
    SVM_PH(6)
  }
#undef SVM_PH
  if constexpr (kSweepU == 8) {
    if (regst) {   // the slice's G and alpha back to memory (the host resumes or finishes from them)
#pragma unroll
      for (int k = 0; k < RU; ++k) {
        const int64_t t = sc.r0 + threadIdx.x + k * NT;
        if (t < sc.r1) { g[t] = rs_g[k]; a[t] = rs_a[k]; }
      }
    }
  }
  if (do_prof && threadIdx.x == 0) {
    ph[7] = s_miss;
    for (int k = 0; k < 8; ++k) prof[k] += ph[k];
  }
  if (threadIdx.x == 0 && sc.w == 0) {
    out_state[2 * pid] = it;
    out_state[2 * pid + 1] = status;
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

// Split solver: probs (device, read-only) x B workgroups each; S cache slots per problem
// (2 <= S <= 1024); kc: cache columns (coff per problem); meta: per-problem per-workgroup
// maps (moff; slot_of = -1, row_of = -1, stamp = 0 initially); recs: nprob * 2 * B * kRecW
// zeroed words; out_state: [nprob][2] (iterations, status) written by workgroup 0.
// wide: the 8-variables-per-step sweep variant (see kSweepU above)
int dml_svm_smo_split(const float* X, int64_t d, const void* probs, int64_t nprob, int32_t B, int32_t S,
                      const float* y, const double* C, const float* qd, double* alpha, double* G, float* kc,
                      int32_t* meta, uint64_t* recs, int64_t* out_state, int64_t chunk, int64_t* prof,
                      int32_t wide, hipStream_t st) {
  if (nprob <= 0) return 0;
  if (B < 1 || B > kMaxB || S < 2 || S > kMaxSlots) return 2;
  if (B > 1) {   // every workgroup of the grid must be resident at once (record spins)
    int per_cu = 0, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 3;
    const hipError_t oe = wide ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_smo_split<8>, NT, 0)
                               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_smo_split<4>, NT, 0);
    if (oe != hipSuccess) return 3;
    if ((int64_t)nprob * B > (int64_t)per_cu * prop.multiProcessorCount / 2) return 4;
  }
  if (wide)
    k_smo_split<8><<<(unsigned)(nprob * B), NT, 0, st>>>(X, d, (const SvmProb*)probs, B, S, y, C, qd, alpha, G, kc,
                                                          meta, recs, out_state, chunk, prof);
  else
    k_smo_split<4><<<(unsigned)(nprob * B), NT, 0, st>>>(X, d, (const SvmProb*)probs, B, S, y, C, qd, alpha, G, kc,
                                                          meta, recs, out_state, chunk, prof);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// workgroups the host may launch at once (narrow variant; *wide_resident: the wide one's)
int dml_svm_split_limits(int32_t* max_b, int32_t* max_slots, int32_t* wide_resident) {
  *max_b = kMaxB;
  *max_slots = kMaxSlots;
  int per_cu = 0, per_cu_w = 0, dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_smo_split<4>, NT, 0) != hipSuccess) return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_w, k_smo_split<8>, NT, 0) != hipSuccess) return -1;
  if (wide_resident) *wide_resident = per_cu_w * prop.multiProcessorCount / 2;
  return per_cu * prop.multiProcessorCount / 2;
}

}  // extern "C"
