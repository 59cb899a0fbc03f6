// lr_mfma.hip — logistic-regression objective on the matrix cores (K7/K8, MFMA).
//
// Reference: LogisticRegression is fitted one (candidate, fold) at a time by sklearn on
// CPU (aws-prod/worker/worker.py:39 whitelist; :315 fit, :326/:341 cross_val_score).
// Here every fit of a batch is a block of columns of ONE weight matrix and one objective
// evaluation of the whole batch is two GEMM-shaped passes on MFMA:
//
//   forward  Z = X W + b         A = X    [n x d]   B^T = W^T [M x d]
//            -> fused epilogue: link (sigmoid / softmax / OvR), fold mask, class weights,
//               per-fit loss, residual R = (P - Y) * s written TRANSPOSED (R^T [M x n])
//   gradient G^T = R^T X         A = R^T  [M x n]   B^T = X^T [d+1 x n]  (split-K over n;
//               X^T carries a row of ones, so the intercept gradient falls out of the GEMM)
//
// Numerics: fp32-equivalent "bf16x3".  Every fp32 operand is stored as hi = bf16(v) and
// lo = bf16(v - hi) (|v - hi - lo| <= 2^-16 |v|) and a product is hi*hi + hi*lo + lo*hi,
// accumulated in fp32 by v_mfma_f32_16x16x32_bf16: three bf16 MFMAs per product run at
// 2.5 PF / 3 vs the 157 TF of the exact fp32 MFMA (no xf32 on gfx950), with a relative
// error of ~1e-5 per dot product — far below the L-BFGS tolerances (1e-4 on max|grad|).
//
// Tiling (CDNA4, wave64): 256-thread workgroups own a 128 x 128 output tile; each wave a
// 64 x 64 quadrant = 4 x 4 MFMA 16x16 tiles (16 fp32x4 accumulators).  K advances 32 at a
// time through a double-buffered LDS stage (A hi/lo + B hi/lo, 64 KB), one barrier per
// k-step, the next stage's global loads in flight while the current one is multiplied.
// LDS rows are 64 B with the 16-B chunk index XOR-swizzled by bit 2 of the row, which makes
// the ds_read_b128 fragment reads conflict-free under CDNA4's 4x16-lane b128 grouping.
// Every operand lives in HBM in a K-TILED layout, element (row, k) at
// ((k / 32) * rows + row) * 32 + k % 32: one stage of one operand part (128 rows x 32 k) is
// ONE contiguous 8-KB block.  (Row-major operands cost 2-3x here: a stage touched 128 rows
// 64 B each, for R^T / X^T rows megabytes apart — measured 12.6 -> ~4 ms on the gradient.)
// Block ids are remapped XCD-aware (id % 8 = XCD): the column tiles of one row group (and,
// in the gradient, every tile of one K slice) share an XCD, so X / R^T panels are fetched
// from HBM once per XCD L2, not once per column tile.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#ifndef LRM_PASSES
#define LRM_PASSES 3   // A/B instrumentation: 1 = hi*hi only, 0 = no MFMA (never in production)
#endif
#ifndef LRM_DMA_HALF
#define LRM_DMA_HALF 0   // A/B instrumentation: 1 = half of the k-steps stage operands (never in production)
#endif
#ifndef LRM_EPI_PROBE
#define LRM_EPI_PROBE 0   // A/B instrumentation: 1 = fwd3 epilogue without the link math (never in production)
#endif

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int THREADS = 256;
constexpr int PART = BM * BK;              // bf16 elements of one operand part of one stage
constexpr int STAGE = 4 * PART;            // A hi, A lo, B hi, B lo
constexpr int STAGE_BYTES = 2 * STAGE * 2; // two stages: 64 KB (also holds the fp32 Z tile)
constexpr int LACC_BYTES = 2 * BN * 8;     // per-column loss partials (double)

// ctypes-facing argument blocks (every field 8 bytes)
struct FwdArgs {
  int64_t xh, xl, xrows;         // X hi/lo, K-tiled over xrows (= row_tiles*BM) rows, Kp deep
  int64_t wh, wl;                // W^T hi/lo, K-tiled over col_tiles*BN rows, Kp deep
  int64_t n, Kp, row_tiles, col_tiles, row_groups;
  int64_t bias;                  // float [col_tiles*BN]
  int64_t col_fit;               // int32 [col_tiles*BN]: fit owning the column, -1 = padding
  int64_t fit_col0, fit_k, fit_kind, fit_split;   // int32 [F] (fit_col0 in padded columns)
  int64_t scale;                 // float [F]
  int64_t cw, cwC;               // float [F x cwC] class weights (0 = none)
  int64_t y, roles;              // int32 [n], uint8 [S x n]
  int64_t rh, rl, kr;            // R^T hi/lo, K-tiled over col_tiles*BN rows, kr (= xrows) deep
  int64_t loss;                  // double [F] (accumulated; caller zeroes)
  int64_t lpart;                 // v3: double [row_tiles x col_tiles*BN] per-item column loss partials
  int64_t col_info;              // v3: int32 [Mp] kind << 28 | split << 16 | positive class (-1: padding)
  int64_t col_scale;             // v3: float [Mp] the column's fit's loss scale
  int64_t n_splits;              // v3: role rows of `roles`
  int64_t softmax_any;           // v3: 1 if any fit is multinomial (Z tile through LDS)
  int64_t row_base;              // v3 row chunks: first (256-row) tile of the chunk; R^T rows are local
  int64_t live;                  // v3 (nullable): int32 [1 + col_tiles] = n_live, then the column tiles
                                 // holding a still-active fit (the others are skipped: their R^T and
                                 // loss partials keep stale values the solver never reads)
  int64_t w_zero;                // v3: 1 if every weight is 0 (logits = bias; the GEMM is skipped)
  // v3 fold-grouped rows (nullable): the operand rows are permuted so that each split's rows
  // without a training role form whole row tiles; an item whose column tile belongs to ONE
  // split (ct_split[ct] >= 0) and whose row tile holds no training row of it
  // (rt_skip[split * rt_stride + rt] != 0) skips its GEMM: its logits only ever meet a zero
  // loss scale, so the epilogue writes exact zeros to R^T and the loss partials
  int64_t ct_split;              // int32 [col_tiles]: the split of every fit column of the tile, -1 mixed
  int64_t rt_skip;               // uint8 [n_splits x rt_stride]
  int64_t rt_stride;             // row tiles of the whole operand (xrows / 256)
};

struct GradArgs {
  int64_t rh, rl, unused;        // R^T hi/lo, K-tiled over m_tiles*BM rows, Kp deep
  int64_t xth, xtl;              // X^T hi/lo (+ ones row), K-tiled over n_tiles*BN rows, Kp deep
  int64_t m_tiles, n_tiles, Kp;  // Kp = rows of the dataset, padded
  int64_t S, Kc;                 // K slices (multiple of 8) and slice length (multiple of BK)
  int64_t out;                   // float [S x m_tiles*BM x n_tiles*BN] partial G^T slabs
  int64_t bk_off;                // v3 row chunks: the chunk's first data row (B = X^T's k offset)
  int64_t slab0;                 // v3 row chunks: first output slab of this chunk
  int64_t mlive;                 // v3 (nullable): int32 per m tile, 0 = no active fit (workgroups exit)
  int64_t kskip;                 // v3 (nullable): int32 [m_tiles x S]: the slice holds no training row of
                                 // the m tile's split (fold-grouped rows): the slab is written as zeros
};

struct Operands {
  const uint16_t* ah;
  const uint16_t* al;
  int64_t arows;   // rows of the K-tiled A operand (k-block stride = arows * 32)
  const uint16_t* bh;
  const uint16_t* bl;
  int64_t brows;
  int64_t bk_off;  // B's k index = A's + bk_off (v3 gradient over a row chunk; multiple of 32)
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }

// operands arrive as integers (ctypes argument blocks): pin them to the GLOBAL address
// space, otherwise hipcc emits flat loads, which also count on lgkmcnt and make every
// LDS-fragment wait drain the next stage's prefetch
typedef const __attribute__((address_space(1))) u32x4* gvec;
typedef __attribute__((address_space(1))) u32x4* gvec_w;
#define GPTR(T, v) ((T*)(__attribute__((address_space(1))) T*)(uintptr_t)(v))

__device__ __forceinline__ u32x4 gload(const uint16_t* p) { return *(gvec)(uintptr_t)p; }

// global -> registers: each of the 4 parts is one contiguous 8-KB block (128 rows x 32 k,
// K-tiled layout): chunk q (16 B) = row q / 4, k chunk q % 4
__device__ __forceinline__ void load_stage(const Operands& op, int64_t row0, int64_t col0, int64_t k0, u32x4 (&r)[8],
                                           int tid) {
  const int64_t ab = ((k0 >> 5) * op.arows + row0) * BK, bb = ((k0 >> 5) * op.brows + col0) * BK;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + i * THREADS;
    r[0 + i] = gload(op.ah + ab + q * 8);
    r[2 + i] = gload(op.al + ab + q * 8);
    r[4 + i] = gload(op.bh + bb + q * 8);
    r[6 + i] = gload(op.bl + bb + q * 8);
  }
}

__device__ __forceinline__ void store_stage(uint16_t* st, const u32x4 (&r)[8], int tid) {
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + i * THREADS;
      const int row = q >> 2, c = q & 3;
      *(u32x4*)(st + p * PART + row * BK + swz(row, c) * 8) = r[p * 2 + i];
    }
}

// direct global -> LDS staging (global_load_lds_dwordx4, CDNA4): no staging registers, no
// ds_write pass.  One wave-instruction fills 64 consecutive 16-B LDS slots (base + 16*lane);
// the XOR swizzle is applied on the SOURCE side: the lane owning LDS slot p = 4*row + pc
// fetches chunk pc ^ f(row) of that row, all inside the same contiguous 1 KB of HBM.
__device__ __forceinline__ void glds_stage(const Operands& op, int64_t row0, int64_t col0, int64_t k0, uint16_t* st,
                                           int tid) {
  const int64_t ab = ((k0 >> 5) * op.arows + row0) * BK, bb = ((k0 >> 5) * op.brows + col0) * BK;
  const int w = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int slot0 = (w * 2 + i) * 64;          // first LDS slot of this wave-instruction
    const int p = slot0 + lane, row = p >> 2;
    const int src = row * 4 + swz(row, p & 3);   // swz is an involution
    const uint16_t* srcs[4] = {op.ah + ab, op.al + ab, op.bh + bb, op.bl + bb};
#pragma unroll
    for (int part = 0; part < 4; ++part)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(uintptr_t)(srcs[part] + src * 8),
                                       (__attribute__((address_space(3))) void*)(st + part * PART + slot0 * 8), 16, 0,
                                       0);
  }
}

__device__ __forceinline__ bf16x8 frag(const uint16_t* part, int row, int chunk) {
  return __builtin_bit_cast(bf16x8, *(const u32x4*)(part + row * BK + swz(row, chunk) * 8));
}

// one 32-deep k-step of the wave's 64 x 64 quadrant: 16 tiles x 3 bf16 MFMAs
__device__ __forceinline__ void mma_stage(const uint16_t* st, f32x4 (&acc)[4][4], int wm, int wn, int lane) {
  const int r = lane & 15, g = lane >> 4;
  bf16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int arow = wm * 64 + i * 16 + r;
    const int brow = wn * 64 + i * 16 + r;
    ah[i] = frag(st + 0 * PART, arow, g);
    al[i] = frag(st + 1 * PART, arow, g);
    bh[i] = frag(st + 2 * PART, brow, g);
    bl[i] = frag(st + 3 * PART, brow, g);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#if LRM_PASSES >= 3
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#endif
#if LRM_PASSES >= 1
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#else
      acc[i][j][0] += (float)ah[i][0] * (float)bh[j][0] + (float)al[i][1] * (float)bl[j][1];
#endif
    }
}

// C[row0:+128, col0:+128] = sum_{k in [kb, ke)} A[row, k] * B^T[col, k]  (bf16x3)
// Ends with a barrier (the staging LDS is free afterwards).  kb >= ke gives zeros.
__device__ __forceinline__ void gemm_tile(const Operands& op, int64_t row0, int64_t col0, int64_t kb, int64_t ke,
                                          uint16_t* smem, f32x4 (&acc)[4][4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (kb >= ke) return;
  const int lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
#ifndef LRM_REGSTAGE
  glds_stage(op, row0, col0, kb, smem, tid);
  __syncthreads();
  int cur = 0;
  for (int64_t k = kb; k < ke; k += BK) {
    if (k + BK < ke) glds_stage(op, row0, col0, k + BK, smem + (cur ^ 1) * STAGE, tid);
    mma_stage(smem + cur * STAGE, acc, wm, wn, lane);
#ifdef LRM_SCHED_FENCE
    // A/B only: every MFMA of the step ahead of the barrier (the scheduler otherwise hoists the
    // barrier to just after the last fragment read) -- measured slower: fwd 228 -> 245 ms,
    // grad 135 -> 188 ms at 10M x 1000 x 2560 (profiles/r5_lr_ab.txt)
    __builtin_amdgcn_sched_barrier(0);
#endif
    __syncthreads();   // drains this wave's LDS-DMA (vmcnt(0)) and publishes the stage
    cur ^= 1;
  }
#else   // register staging (A/B reference)
  u32x4 r[8];
  load_stage(op, row0, col0, kb, r, tid);
  store_stage(smem, r, tid);
  __syncthreads();
  int cur = 0;
  for (int64_t k = kb; k < ke; k += BK) {
    const bool more = k + BK < ke;
#ifndef LRM_NOLOAD
    if (more) load_stage(op, row0, col0, k + BK, r, tid);
#endif
    mma_stage(smem + cur * STAGE, acc, wm, wn, lane);
#ifndef LRM_NOSTORE
    if (more) store_stage(smem + (cur ^ 1) * STAGE, r, tid);
#endif
    __syncthreads();
    cur ^= 1;
  }
#endif
}

__device__ __forceinline__ void put_hilo(uint16_t* hp, uint16_t* lp, float v) {
  const __bf16 h = (__bf16)v;
  const __bf16 l = (__bf16)(v - (float)h);
  *hp = __builtin_bit_cast(uint16_t, h);
  *lp = __builtin_bit_cast(uint16_t, l);
}

// 8 fp32 values -> 8 packed bf16 hi + 8 packed bf16 lo (one 16-B store each)
__device__ __forceinline__ void split8(const float (&v)[8], u32x4& hv, u32x4& lv) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const __bf16 h0 = (__bf16)v[2 * q], h1 = (__bf16)v[2 * q + 1];
    const __bf16 l0 = (__bf16)(v[2 * q] - (float)h0), l1 = (__bf16)(v[2 * q + 1] - (float)h1);
    hv[q] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    lv[q] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
  }
}

// Z tile element (row, col) at zs[row * BN + (col ^ (bit 2 of row) << 4)]: the accumulator
// writes (32 lanes = two rows 4 apart x 16 columns) hit 32 distinct banks and the
// epilogue's reads (64 consecutive columns of one row) 64 distinct banks.
__device__ __forceinline__ int zidx(int row, int col) { return row * BN + (col ^ (((row >> 2) & 1) << 4)); }

constexpr int YS_BYTES = BM * 4;   // the tile's labels, staged once per tile

__global__ __launch_bounds__(THREADS, 2) void k_lr_fwd(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[STAGE_BYTES + LACC_BYTES + YS_BYTES];
  uint16_t* smem = reinterpret_cast<uint16_t*>(smem_raw);
  float* zs = reinterpret_cast<float*>(smem_raw);
  double* lacc = reinterpret_cast<double*>(smem_raw + STAGE_BYTES);
  int32_t* ys = reinterpret_cast<int32_t*>(smem_raw + STAGE_BYTES + LACC_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  // XCD-aware decomposition: the column tiles of one row group run on one XCD
  const int64_t b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int64_t ct = local % a.col_tiles;
  const int64_t rg = (local / a.col_tiles) * 8 + xcd;
  if (rg >= a.row_groups) return;   // grid-uniform (host sizes the grid exactly)

  const auto col_fit = GPTR(const int32_t, a.col_fit);
  const auto bias = GPTR(const float, a.bias);
  const auto y = GPTR(const int32_t, a.y);
  const auto roles = GPTR(const uint8_t, a.roles);
  const Operands op{reinterpret_cast<const uint16_t*>(a.xh), reinterpret_cast<const uint16_t*>(a.xl), a.xrows,
                    reinterpret_cast<const uint16_t*>(a.wh), reinterpret_cast<const uint16_t*>(a.wl),
                    a.col_tiles * BN};
  const int64_t Mp = a.col_tiles * BN;
  const int64_t col0 = ct * BN;
  const int wm = w >> 1, wn = w & 1;

  // epilogue mapping: thread = (column c of the tile, 64-row half rh); the lead column of a
  // fit owns the fit's k columns for its rows.  Everything about the fit is tile-invariant.
  const int c = tid & (BN - 1), rh = tid >> 7;
  const int f = col_fit[col0 + c];
  const bool lead = f >= 0 && reinterpret_cast<const int32_t*>(a.fit_col0)[f] == col0 + c;
  int k = 0, kind = 0;
  int64_t role_off = 0;
  float s0 = 0.f;
  const float* cwf = nullptr;
  if (lead) {
    k = reinterpret_cast<const int32_t*>(a.fit_k)[f];
    kind = reinterpret_cast<const int32_t*>(a.fit_kind)[f];
    role_off = (int64_t)reinterpret_cast<const int32_t*>(a.fit_split)[f] * a.n;
    s0 = reinterpret_cast<const float*>(a.scale)[f];
    if (a.cw) cwf = GPTR(const float, a.cw) + (int64_t)f * a.cwC;
  }
  // R^T is K-tiled too: (column, row) at ((row / 32) * Mp + column) * 32 + row % 32
  const auto RH = GPTR(uint16_t, a.rh) + (col0 + c) * BK;
  const auto RL = GPTR(uint16_t, a.rl) + (col0 + c) * BK;
  double lossacc = 0.0;

  for (int64_t rt = rg; rt < a.row_tiles; rt += a.row_groups) {
    const int64_t row0 = rt * BM;
    f32x4 acc[4][4];
    gemm_tile(op, row0, col0, 0, a.Kp, smem, acc, tid);
    // accumulators (+ bias) -> fp32 Z tile in the (now free) staging LDS; labels -> LDS
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + (lane & 15);
        const float bv = bias[col0 + col];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + e;
          zs[zidx(row, col)] = acc[i][j][e] + bv;
        }
      }
    if (tid < BM) ys[tid] = row0 + tid < a.n ? y[row0 + tid] : 0;
    __syncthreads();
    if (lead) {
      float lsum = 0.f;
      for (int rr = 0; rr < 64; rr += 8) {
        const int lr0 = rh * 64 + rr;
        const int64_t g0 = row0 + lr0;
        float sc[8];
        int yv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int64_t g = g0 + e;
          yv[e] = ys[lr0 + e];
          const bool tr = g < a.n && roles[role_off + g] == 1;
          sc[e] = tr ? (cwf ? s0 * cwf[yv[e]] : s0) : 0.f;   // 0 also zeroes R of held-out rows
        }
        if (kind == 1) {   // multinomial softmax over k columns
          float lse[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float m = zs[zidx(lr0 + e, c)];
            for (int j = 1; j < k; ++j) m = fmaxf(m, zs[zidx(lr0 + e, c + j)]);
            float se = 0.f;
            for (int j = 0; j < k; ++j) se += __expf(zs[zidx(lr0 + e, c + j)] - m);
            lse[e] = m + __logf(se);
            lsum += sc[e] * (lse[e] - zs[zidx(lr0 + e, c + yv[e])]);
          }
          for (int j = 0; j < k; ++j) {
            float r[8];
#pragma unroll
            for (int e = 0; e < 8; ++e)
              r[e] = (__expf(zs[zidx(lr0 + e, c + j)] - lse[e]) - (yv[e] == j ? 1.f : 0.f)) * sc[e];
            u32x4 hv, lv;
            split8(r, hv, lv);
            const int64_t off = ((g0 >> 5) * Mp + j) * BK + (g0 & (BK - 1));
            *(gvec_w)(RH + off) = hv;
            *(gvec_w)(RL + off) = lv;
          }
        } else {           // 0: one sigmoid column (target y == 1); 2: OvR column j (target y == j)
          for (int j = 0; j < k; ++j) {
            float r[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float z = zs[zidx(lr0 + e, c + j)];
              const bool pos = kind == 0 ? yv[e] == 1 : yv[e] == j;
              const float ex = __expf(-fabsf(z));                    // one exp, one log, one rcp
              const float inv = __builtin_amdgcn_rcpf(1.f + ex);
              const float p = z >= 0.f ? inv : ex * inv;             // sigmoid(z)
              const float t = pos ? -z : z;                          // loss = softplus(t), |t| = |z|
              lsum += sc[e] * (fmaxf(t, 0.f) + __logf(1.f + ex));
              r[e] = (p - (pos ? 1.f : 0.f)) * sc[e];
            }
            u32x4 hv, lv;
            split8(r, hv, lv);
            const int64_t off = ((g0 >> 5) * Mp + j) * BK + (g0 & (BK - 1));
            *(gvec_w)(RH + off) = hv;
            *(gvec_w)(RL + off) = lv;
          }
        }
      }
      lossacc += (double)lsum;
    }
    __syncthreads();   // Z tile / label reads done before the next tile's staging writes
  }
  // the two row halves of a column combine in LDS; one atomic per fit per workgroup
  if (rh == 1) lacc[c] = lossacc;
  __syncthreads();
  if (rh == 0 && lead) {
    const double v = lossacc + lacc[c];
    if (v != 0.0) atomicAdd(reinterpret_cast<double*>(a.loss) + f, v);
  }
}

__global__ __launch_bounds__(THREADS, 2) void k_lr_grad(GradArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[STAGE_BYTES];
  uint16_t* smem = reinterpret_cast<uint16_t*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // every output tile of one K slice runs on one XCD (shared R^T / X^T panels in its L2)
  const int64_t b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int64_t tiles = a.m_tiles * a.n_tiles;
  const int64_t tile = local % tiles;
  const int64_t s = (local / tiles) * 8 + xcd;
  if (s >= a.S) return;
  const int64_t mt = tile / a.n_tiles, nt = tile % a.n_tiles;
  const int64_t kb = s * a.Kc;
  const int64_t ke = kb + a.Kc < a.Kp ? kb + a.Kc : a.Kp;
  const Operands op{reinterpret_cast<const uint16_t*>(a.rh), reinterpret_cast<const uint16_t*>(a.rl),
                    a.m_tiles * BM, reinterpret_cast<const uint16_t*>(a.xth), reinterpret_cast<const uint16_t*>(a.xtl),
                    a.n_tiles * BN};
  f32x4 acc[4][4];
  gemm_tile(op, mt * BM, nt * BN, kb, ke, smem, acc, tid);
  const int64_t ldo = a.n_tiles * BN;
  const auto out = GPTR(float, a.out) + s * (a.m_tiles * BM) * ldo;
  const int wm = w >> 1, wn = w & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t col = nt * BN + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = mt * BM + wm * 64 + i * 16 + (lane >> 4) * 4 + e;
        out[row * ldo + col] = acc[i][j][e];
      }
    }
}

// fp32 [rows x cols] (row-major, ld) -> bf16 hi/lo in the K-tiled operand layout with
// `drows` operand rows: not transposed, operand (row r, k c); transposed, operand
// (row c, k r).  One-time operand preparation per dataset (destinations pre-zeroed).
// blockIdx.x walks 64-row tiles (rows can be ~10M), blockIdx.y 64-column tiles.
__global__ __launch_bounds__(256) void k_split_hilo(const float* __restrict__ src, int64_t rows, int64_t cols,
                                                     int64_t ld, uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                                     int64_t drows, int transpose, const int64_t* __restrict__ perm) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    // operand row r holds source row perm[r] (fold-grouped rows; identity without perm)
    tile[i][tx] = (r < rows && c < cols) ? src[(perm ? perm[r] : r) * ld + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    if (!transpose) {
      const int64_t r = r0 + i, c = c0 + tx;
      const int64_t o = ((c >> 5) * drows + r) * BK + (c & (BK - 1));
      if (r < rows && c < cols) put_hilo(hi + o, lo + o, tile[i][tx]);
    } else {   // destination [cols x rows]
      const int64_t r = r0 + tx, c = c0 + i;
      const int64_t o = ((r >> 5) * drows + c) * BK + (r & (BK - 1));
      if (r < rows && c < cols) put_hilo(hi + o, lo + o, tile[tx][i]);
    }
  }
}


// ---- v3: 256 x 128 output tiles, 8 waves, 3-stage LDS-DMA ring, one workgroup per CU ----------
// The 2-stage kernels above leave a stage's DMA latency covered by ONE step of MFMAs (and two
// workgroups per CU at 64 KB of staging each); the forward's W^T operand (all fits' columns,
// 10 MB at 2560 fits) does not stay in an XCD's 4 MB L2, so its misses outlast that cover.  Here
// a stage is loaded TWO steps ahead (3 buffers x 48 KB), the barrier waits with a counted
// vmcnt (the newest stage stays in flight across it), and a 256-row tile halves the forward's
// W^T traffic per row.  The forward walks a static round-robin of (row tile, column tile) items
// per XCD (row tiles rt % 8 == XCD, so a row tile's 20-odd column items share that XCD's L2);
// each item writes its per-column loss partials to lpart (summed over row tiles by the host).
namespace v3 {
constexpr int WMW = 4, WNW = 2;
constexpr int TM = 64 * WMW, TN = 64 * WNW;             // 256 x 128
constexpr int NT = 64 * WMW * WNW;                      // 512 threads
constexpr int NST = 3;
constexpr int APART = TM * BK, BPART = TN * BK;         // bf16 elements of one part of one stage
constexpr int STG = 2 * APART + 2 * BPART;
constexpr int STG_BYTES = NST * STG * 2;                // 144 KB
constexpr int A_INSTR = APART * 2 / 1024;               // 1-KiB wave-instructions per A part
constexpr int B_INSTR = BPART * 2 / 1024;
constexpr int STAGE_INSTR = 2 * A_INSTR + 2 * B_INSTR;
constexpr int PER_WAVE = STAGE_INSTR / (NT / 64);       // LDS-DMA instructions per wave per stage
static_assert(STAGE_INSTR % (NT / 64) == 0, "stage must split evenly over the waves");
static_assert(TM * TN * 4 + 4 * TN * 8 + TM * 4 <= STG_BYTES, "epilogue scratch must fit the staging LDS");
}  // namespace v3

// counted wait for this wave's LDS-DMA + its LDS reads, then the workgroup barrier.  Inline asm
// (not __syncthreads, whose fence drains vmcnt(0)): the newest stage stays in flight.
template <int N>
__device__ __forceinline__ void v3_wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ __forceinline__ void v3_glds_piece(const uint16_t* src, uint16_t* dst, int slot0, int lane) {
  const int p = slot0 + lane, row = p >> 2;
  const int srci = row * 4 + swz(row, p & 3);   // swizzle on the source side (swz is an involution)
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(uintptr_t)(src + srci * 8),
                                   (__attribute__((address_space(3))) void*)(dst + slot0 * 8), 16, 0, 0);
}

// one stage = 48 one-KiB pieces; wave w fetches pieces 2w, 2w+1 of A hi and of A lo and piece w
// of B hi and of B lo (6 per wave, parts fixed at compile time, w wave-uniform)
__device__ __forceinline__ void v3_glds_stage(const Operands& op, int64_t row0, int64_t col0, int64_t k0,
                                              uint16_t* st, int w, int lane) {
  using namespace v3;
  static_assert(A_INSTR == 2 * (NT / 64) && B_INSTR == NT / 64, "piece split assumes 8 waves, 256 x 128");
  const int64_t ab = ((k0 >> 5) * op.arows + row0) * BK, bb = (((k0 + op.bk_off) >> 5) * op.brows + col0) * BK;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    v3_glds_piece(op.ah + ab, st, (2 * w + h) * 64, lane);
    v3_glds_piece(op.al + ab, st + APART, (2 * w + h) * 64, lane);
  }
  v3_glds_piece(op.bh + bb, st + 2 * APART, w * 64, lane);
  v3_glds_piece(op.bl + bb, st + 2 * APART + BPART, w * 64, lane);
}

__device__ __forceinline__ void v3_mma(const uint16_t* st, f32x4 (&acc)[4][4], int wm, int wn, int lane) {
  using namespace v3;
  const int r = lane & 15, g = lane >> 4;
  bf16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int arow = wm * 64 + i * 16 + r;
    const int brow = wn * 64 + i * 16 + r;
    ah[i] = frag(st, arow, g);
    al[i] = frag(st + APART, arow, g);
    bh[i] = frag(st + 2 * APART, brow, g);
    bl[i] = frag(st + 2 * APART + BPART, brow, g);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#if LRM_PASSES >= 3
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#endif
#if LRM_PASSES >= 1
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#else   // probe: keep the fragment reads live without the matrix cores
      acc[i][j][0] += (float)ah[i][0] + (float)al[i][1] + (float)bh[j][2] + (float)bl[j][3];
#endif
    }
}

// C[row0:+256, col0:+128] over k in [kb, ke) (bf16x3); every wave owns a 64 x 64 quadrant.
// Ends with a barrier after every DMA has landed (the staging LDS is free afterwards).
__device__ __forceinline__ void v3_gemm(const Operands& op, int64_t row0, int64_t col0, int64_t kb, int64_t ke,
                                        uint16_t* smem, f32x4 (&acc)[4][4], int tid) {
  using namespace v3;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (ke - kb) / BK;
  if (nk <= 0) return;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), wm = w >> 1, wn = w & 1;
  v3_glds_stage(op, row0, col0, kb, smem, w, lane);
  if (nk > 1) v3_glds_stage(op, row0, col0, kb + BK, smem + STG, w, lane);
  int cur = 0;   // buffer of step t (t % 3)
  for (int64_t t = 0; t < nk; ++t) {
    // stage t landed (stage t+1 may stay in flight); every wave is done with step t-1's buffer
    if (t + 1 < nk) v3_wait_barrier<PER_WAVE>();
    else v3_wait_barrier<0>();
    const int nxt = cur == 0 ? 2 : cur - 1;   // (t + 2) % 3 == (t - 1) % 3
#if LRM_DMA_HALF   // timing probe only (wrong results): the ring is refilled every other k-step
    if (t + 2 < nk && (t & 1) == 0) v3_glds_stage(op, row0, col0, kb + (t + 2) * BK, smem + nxt * STG, w, lane);
#else
    if (t + 2 < nk) v3_glds_stage(op, row0, col0, kb + (t + 2) * BK, smem + nxt * STG, w, lane);
#endif
    v3_mma(smem + cur * STG, acc, wm, wn, lane);
    cur = cur == 2 ? 0 : cur + 1;
  }
  v3_wait_barrier<0>();
}

constexpr int V3_ROLE_ROWS = 8;   // role rows staged per item in LDS (cv <= 7 + holdout; more: read from HBM)

__global__ __launch_bounds__(v3::NT, 1) void k_lr_fwd3(FwdArgs a) {
  using namespace v3;
  // staging ring + (past it) the item's labels and role rows: loaded at the item's start (in
  // flight under its GEMM), stored once the GEMM has drained.  ONE LDS object: with separate
  // __shared__ arrays the compiler's wait pass makes every fragment read wait vmcnt(0)
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[STG_BYTES + TM * 4 + V3_ROLE_ROWS * TM];
  int32_t* eps_y = reinterpret_cast<int32_t*>(smem_raw + STG_BYTES);
  uint8_t* eps_r = smem_raw + STG_BYTES + TM * 4;
  uint16_t* smem = reinterpret_cast<uint16_t*>(smem_raw);
  float* zs = reinterpret_cast<float*>(smem_raw);                              // Z tile (softmax batches)
  double* lq = reinterpret_cast<double*>(smem_raw + TM * TN * 4);              // [4][TN] partials
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int64_t b = blockIdx.x, xcd = b & 7, slot = b >> 3, slots = gridDim.x >> 3;
  // row tiles of this launch: [row_base, row_base + row_tiles) of X; R^T (and its K-tiled
  // layout) covers only the launch's rows (local row index = global - row_base * TM)
  const int64_t rt_here = a.row_tiles > xcd ? (a.row_tiles - xcd + 7) / 8 : 0;
  const auto live = a.live ? GPTR(const int32_t, a.live) : nullptr;
  const int64_t n_ct = live ? __builtin_amdgcn_readfirstlane(live[0]) : a.col_tiles;   // live column tiles
  const int64_t items = rt_here * n_ct;
  const int64_t rbase = a.row_base * TM;
  const auto col_fit = GPTR(const int32_t, a.col_fit);
  const auto bias = GPTR(const float, a.bias);
  const auto y = GPTR(const int32_t, a.y);
  const auto roles = GPTR(const uint8_t, a.roles);
  const auto lpart = GPTR(double, a.lpart);
  const auto cinfo_g = GPTR(const int32_t, a.col_info);
  const auto cscale_g = GPTR(const float, a.col_scale);
  const auto cwt = a.cw ? GPTR(const float, a.cw) : nullptr;
  const Operands op{reinterpret_cast<const uint16_t*>(a.xh), reinterpret_cast<const uint16_t*>(a.xl), a.xrows,
                    reinterpret_cast<const uint16_t*>(a.wh), reinterpret_cast<const uint16_t*>(a.wl),
                    a.col_tiles * TN};
  const int64_t Mp = a.col_tiles * TN;
  const bool softmax = a.softmax_any != 0;
  const int S = (int)a.n_splits;
  const bool stage_roles = S <= V3_ROLE_ROWS;
  const bool w_zero = a.w_zero != 0;
  const int nchunk = stage_roles ? S * (TM / 4) : 0;   // 4-row role chunks of the item (<= NT)
  static_assert(V3_ROLE_ROWS * (TM / 4) <= NT, "one role chunk per thread");
  for (int64_t it = slot; it < items; it += slots) {
    const int64_t rtl = xcd + 8 * (it / n_ct);
    const int64_t ct = live ? __builtin_amdgcn_readfirstlane(live[1 + it % n_ct]) : it % n_ct;
    const int64_t rt = a.row_base + rtl;               // global row tile
    const int64_t row0 = rt * TM, col0 = ct * TN;
    // fold-grouped rows: no training row of this column tile's split in the row tile
    bool skip_gemm = false;
    if (a.ct_split) {
      const int cs = __builtin_amdgcn_readfirstlane(GPTR(const int32_t, a.ct_split)[ct]);
      if (cs >= 0) skip_gemm = GPTR(const uint8_t, a.rt_skip)[(int64_t)cs * a.rt_stride + rt] != 0;
    }
    // ---- item prologue: epilogue operands in flight under the GEMM.  Every load is
    // unconditional (clamped address, value selected after the GEMM): a load under a branch
    // merges into a phi whose copy waits vmcnt(0) -- i.e. would drain the GEMM's DMA ring
    const int ty = tid & (TM - 1);
    const int32_t ypre = y[min(row0 + ty, (int64_t)a.n - 1)];
    uint32_t rpre = 0;
    {
      const int chk = tid < nchunk ? tid : 0, sp = chk / (TM / 4), r4 = (chk % (TM / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        rpre |= (uint32_t)roles[(int64_t)sp * a.n + min(row0 + r4 + e, (int64_t)a.n - 1)] << (8 * e);
    }
    int32_t cinfo[4], cfit[4];
    float cscale[4], cbias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gc = col0 + wn * 64 + j * 16 + (lane & 15);
      cinfo[j] = cinfo_g[gc];
      cscale[j] = cscale_g[gc];
      cbias[j] = bias[gc];
      cfit[j] = col_fit[gc];
    }
    f32x4 acc[4][4];
    if (w_zero || skip_gemm) {   // W = 0 (the solver's first evaluation): Z = bias, no GEMM; or no training row
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
      v3_gemm(op, row0, col0, 0, a.Kp, smem, acc, tid);
    }
    if (tid < TM) eps_y[tid] = row0 + tid < a.n ? ypre : 0;
    if (tid < nchunk) {   // rows past n read as role 0 (held out)
      const int r4 = (tid % (TM / 4)) * 4;
      uint32_t v = rpre;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (row0 + r4 + e >= a.n) v &= ~(0xFFu << (8 * e));
      *reinterpret_cast<uint32_t*>(eps_r + tid * 4) = v;
    }
    __syncthreads();
    auto role_at = [&](int sp, int lrow) -> int {
      if (stage_roles) return eps_r[sp * TM + lrow];
      const int64_t g = row0 + lrow;
      return g < a.n ? (int)roles[(int64_t)sp * a.n + g] : 0;
    };
    if (!softmax) {
      // ---- register epilogue: every column is an independent sigmoid (binary / OvR)
      float lsum[4] = {0.f, 0.f, 0.f, 0.f};
      // the lane's 4 x 4 rows: labels as one 16-B LDS read per row quad (not one per element)
      int4 yq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) yq[i] = *reinterpret_cast<const int4*>(eps_y + wm * 64 + i * 16 + (lane >> 4) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ci = cinfo[j];
        if (ci < 0) continue;                                 // padding column: R stays 0
        const int kind = ci >> 28, sp = (ci >> 16) & 0xFFF, tgt = ci & 0xFFFF;
        const int64_t gc = col0 + wn * 64 + j * 16 + (lane & 15);
        const auto RH = GPTR(uint16_t, a.rh) + gc * BK;
        const auto RL = GPTR(uint16_t, a.rl) + gc * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int lr0 = wm * 64 + i * 16 + (lane >> 4) * 4;
          // the quad's 4 role bytes in one 4-B LDS read (staged rows; else per element)
          const uint32_t rq4 = stage_roles ? *reinterpret_cast<const uint32_t*>(eps_r + sp * TM + lr0) : 0u;
          float r[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int lrow = lr0 + e;
            const int yv = e == 0 ? yq[i].x : e == 1 ? yq[i].y : e == 2 ? yq[i].z : yq[i].w;
            const int rl = stage_roles ? (int)((rq4 >> (8 * e)) & 0xFFu) : role_at(sp, lrow);
            const bool tr = row0 + lrow < a.n && rl == 1;
            const float sc = tr ? (cwt ? cscale[j] * cwt[(int64_t)cfit[j] * a.cwC + yv] : cscale[j]) : 0.f;
            const float z = acc[i][j][e] + cbias[j];
            const bool pos = kind == 0 ? yv == 1 : yv == tgt;
#if LRM_EPI_PROBE   // timing probe only (wrong results): the link math replaced by one multiply
            lsum[j] += sc * z;
            r[e] = (z - (pos ? 1.f : 0.f)) * sc;
#else
            const float ex = __expf(-fabsf(z));                    // one exp, one log, one rcp
            const float inv = __builtin_amdgcn_rcpf(1.f + ex);
            const float p = z >= 0.f ? inv : ex * inv;
            const float t = pos ? -z : z;
            lsum[j] += sc * (fmaxf(t, 0.f) + __logf(1.f + ex));
            r[e] = (p - (pos ? 1.f : 0.f)) * sc;
#endif
          }
          u32x2 hv, lv;
          {
            const __bf16 h0 = (__bf16)r[0], h1 = (__bf16)r[1], h2 = (__bf16)r[2], h3 = (__bf16)r[3];
            const __bf16 l0 = (__bf16)(r[0] - (float)h0), l1 = (__bf16)(r[1] - (float)h1);
            const __bf16 l2 = (__bf16)(r[2] - (float)h2), l3 = (__bf16)(r[3] - (float)h3);
            hv.x = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
            hv.y = (uint32_t)__builtin_bit_cast(uint16_t, h2) | ((uint32_t)__builtin_bit_cast(uint16_t, h3) << 16);
            lv.x = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
            lv.y = (uint32_t)__builtin_bit_cast(uint16_t, l2) | ((uint32_t)__builtin_bit_cast(uint16_t, l3) << 16);
          }
          const int64_t g0 = row0 - rbase + lr0;   // local row; 4 consecutive rows inside one 32-row K block
          const int64_t off = (g0 >> 5) * Mp * BK + (g0 & (BK - 1));
          *(__attribute__((address_space(1))) u32x2*)(RH + off) = hv;
          *(__attribute__((address_space(1))) u32x2*)(RL + off) = lv;
        }
      }
      // column sums: the 4 lanes of a column (lane >> 4), then the 4 row-waves (wm) in LDS
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double v = (double)lsum[j];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (lane < 16) lq[wm * TN + wn * 64 + j * 16 + lane] = v;
      }
    } else {
      // ---- multinomial batches: Z tile through LDS, the lead column of a fit owns its k columns
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = wn * 64 + j * 16 + (lane & 15);
          const float bv = bias[col0 + col];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + e;
            zs[zidx(row, col)] = acc[i][j][e] + bv;
          }
        }
      __syncthreads();
      const int c = tid & (TN - 1), rq = tid >> 7;
      const int f = col_fit[col0 + c];
      const bool lead = f >= 0 && reinterpret_cast<const int32_t*>(a.fit_col0)[f] == col0 + c;
      double lossq = 0.0;
      if (lead) {
        const int k = reinterpret_cast<const int32_t*>(a.fit_k)[f];
        const int kind = reinterpret_cast<const int32_t*>(a.fit_kind)[f];
        const int sp = reinterpret_cast<const int32_t*>(a.fit_split)[f];
        const float s0 = reinterpret_cast<const float*>(a.scale)[f];
        const float* cwf = a.cw ? GPTR(const float, a.cw) + (int64_t)f * a.cwC : nullptr;
        const auto RH = GPTR(uint16_t, a.rh) + (col0 + c) * BK;
        const auto RL = GPTR(uint16_t, a.rl) + (col0 + c) * BK;
        float lsumq = 0.f;
        for (int rr = 0; rr < 64; rr += 8) {
          const int lr0 = rq * 64 + rr;
          const int64_t g0 = row0 - rbase + lr0;   // local row of the R^T chunk
          float sc[8];
          int yv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            yv[e] = eps_y[lr0 + e];
            const bool tr = row0 + lr0 + e < a.n && role_at(sp, lr0 + e) == 1;
            sc[e] = tr ? (cwf ? s0 * cwf[yv[e]] : s0) : 0.f;
          }
          if (kind == 1) {
            float lse[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float m = zs[zidx(lr0 + e, c)];
              for (int jj = 1; jj < k; ++jj) m = fmaxf(m, zs[zidx(lr0 + e, c + jj)]);
              float se = 0.f;
              for (int jj = 0; jj < k; ++jj) se += __expf(zs[zidx(lr0 + e, c + jj)] - m);
              lse[e] = m + __logf(se);
              lsumq += sc[e] * (lse[e] - zs[zidx(lr0 + e, c + yv[e])]);
            }
            for (int jj = 0; jj < k; ++jj) {
              float r[8];
#pragma unroll
              for (int e = 0; e < 8; ++e)
                r[e] = (__expf(zs[zidx(lr0 + e, c + jj)] - lse[e]) - (yv[e] == jj ? 1.f : 0.f)) * sc[e];
              u32x4 hv, lv;
              split8(r, hv, lv);
              const int64_t off = ((g0 >> 5) * Mp + jj) * BK + (g0 & (BK - 1));
              *(gvec_w)(RH + off) = hv;
              *(gvec_w)(RL + off) = lv;
            }
          } else {
            for (int jj = 0; jj < k; ++jj) {
              float r[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float z = zs[zidx(lr0 + e, c + jj)];
                const bool pos = kind == 0 ? yv[e] == 1 : yv[e] == jj;
                const float ex = __expf(-fabsf(z));
                const float inv = __builtin_amdgcn_rcpf(1.f + ex);
                const float p = z >= 0.f ? inv : ex * inv;
                const float t = pos ? -z : z;
                lsumq += sc[e] * (fmaxf(t, 0.f) + __logf(1.f + ex));
                r[e] = (p - (pos ? 1.f : 0.f)) * sc[e];
              }
              u32x4 hv, lv;
              split8(r, hv, lv);
              const int64_t off = ((g0 >> 5) * Mp + jj) * BK + (g0 & (BK - 1));
              *(gvec_w)(RH + off) = hv;
              *(gvec_w)(RL + off) = lv;
            }
          }
        }
        lossq = (double)lsumq;
      }
      lq[rq * TN + c] = lossq;
    }
    __syncthreads();
    if (tid < TN) lpart[rt * Mp + col0 + tid] = lq[tid] + lq[TN + tid] + lq[2 * TN + tid] + lq[3 * TN + tid];
    __syncthreads();   // Z tile / labels / partials read before the next item's staging writes
  }
}

__global__ __launch_bounds__(v3::NT, 1) void k_lr_grad3(GradArgs a) {
  using namespace v3;
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[STG_BYTES];
  uint16_t* smem = reinterpret_cast<uint16_t*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int64_t b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int64_t tiles = a.m_tiles * a.n_tiles;
  const int64_t tile = local % tiles;
  const int64_t s = (local / tiles) * 8 + xcd;
  if (s >= a.S) return;   // workgroup-uniform, before any barrier
  const int64_t mt = tile / a.n_tiles, nt = tile % a.n_tiles;
  if (a.mlive && GPTR(const int32_t, a.mlive)[mt] == 0) return;   // every fit of the m tile has stopped
  const int64_t kb = s * a.Kc;
  const int64_t ke = kb + a.Kc < a.Kp ? kb + a.Kc : a.Kp;
  if (a.kskip && GPTR(const int32_t, a.kskip)[mt * a.S + s] != 0) {
    // fold-grouped rows: the slice holds no training row of the m tile's split (R^T is 0 there)
    const int64_t ldo = a.n_tiles * TN;
    const auto out = GPTR(float, a.out) + (a.slab0 + s) * (a.m_tiles * TM) * ldo;
    const int64_t col = nt * TN + (tid & (TN - 1));
    for (int64_t row = mt * TM + (tid >> 7); row < (mt + 1) * TM; row += NT / TN) out[row * ldo + col] = 0.f;
    return;
  }
  const Operands op{reinterpret_cast<const uint16_t*>(a.rh), reinterpret_cast<const uint16_t*>(a.rl),
                    a.m_tiles * TM, reinterpret_cast<const uint16_t*>(a.xth), reinterpret_cast<const uint16_t*>(a.xtl),
                    a.n_tiles * TN, a.bk_off};
  f32x4 acc[4][4];
  v3_gemm(op, mt * TM, nt * TN, kb, ke, smem, acc, tid);
  const int64_t ldo = a.n_tiles * TN;
  const auto out = GPTR(float, a.out) + (a.slab0 + s) * (a.m_tiles * TM) * ldo;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t col = nt * TN + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = mt * TM + wm * 64 + i * 16 + (lane >> 4) * 4 + e;
        out[row * ldo + col] = acc[i][j][e];
      }
    }
}

}  // namespace

extern "C" {

int dml_lr_mfma_tile() { return BM; }

int dml_lr_mfma_fwd(const FwdArgs* a, hipStream_t st) {
  if (a->row_tiles <= 0 || a->col_tiles <= 0) return 0;
  if (a->Kp % BK || a->row_groups % 8 || a->row_groups <= 0) return 2;
  if (a->xrows != a->row_tiles * BM || a->kr != a->xrows) return 2;
  const int64_t blocks = a->col_tiles * a->row_groups;
  if (blocks > 0x7fffffff) return 2;
  k_lr_fwd<<<(unsigned)blocks, THREADS, 0, st>>>(*a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_lr_mfma_grad(const GradArgs* a, hipStream_t st) {
  if (a->m_tiles <= 0 || a->n_tiles <= 0) return 0;
  if (a->Kp % BK || a->Kc % BK || a->S % 8 || a->S <= 0 || a->S * a->Kc < a->Kp) return 2;
  const int64_t blocks = a->m_tiles * a->n_tiles * a->S;
  if (blocks > 0x7fffffff) return 2;
  k_lr_grad<<<(unsigned)blocks, THREADS, 0, st>>>(*a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_split_hilo(const float* src, int64_t rows, int64_t cols, int64_t ld, uint16_t* hi, uint16_t* lo,
                   int64_t drows, int32_t transpose, const int64_t* perm, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return 0;
  dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((cols + 63) / 64));
  if (grid.y > 65535) return 2;
  k_split_hilo<<<grid, 256, 0, st>>>(src, rows, cols, ld, hi, lo, drows, transpose, perm);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// v3 (256 x 128 tiles, 3-stage ring): the row tile of X (forward) / of R^T (gradient)
int dml_lr_v3_row_tile() { return v3::TM; }

int dml_lr_mfma_fwd3(const FwdArgs* a, hipStream_t st) {
  if (a->row_tiles <= 0 || a->col_tiles <= 0) return 0;
  if (a->Kp % BK || a->row_groups % 8 || a->row_groups <= 0 || !a->lpart || a->n_splits <= 0) return 2;
  if (!a->col_info || !a->col_scale) return 2;
  if (a->row_base < 0 || (a->row_base + a->row_tiles) * v3::TM > a->xrows || a->kr != a->row_tiles * v3::TM) return 2;
  if (a->ct_split && (!a->rt_skip || a->rt_stride * v3::TM != a->xrows)) return 2;
  if (a->row_groups > 0x7fffffff) return 2;
  k_lr_fwd3<<<(unsigned)a->row_groups, v3::NT, 0, st>>>(*a);   // row_groups = workgroups (persistent)
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_lr_mfma_grad3(const GradArgs* a, hipStream_t st) {
  if (a->m_tiles <= 0 || a->n_tiles <= 0) return 0;
  if (a->Kp % BK || a->Kc % BK || a->S % 8 || a->S <= 0 || a->S * a->Kc < a->Kp) return 2;
  if (a->bk_off % BK || a->bk_off < 0 || a->slab0 < 0) return 2;
  const int64_t blocks = a->m_tiles * a->n_tiles * a->S;
  if (blocks > 0x7fffffff) return 2;
  k_lr_grad3<<<(unsigned)blocks, v3::NT, 0, st>>>(*a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dml_lr_sizeof_fwd_args() { return (int)sizeof(FwdArgs); }
int dml_lr_sizeof_grad_args() { return (int)sizeof(GradArgs); }

}  // extern "C"
