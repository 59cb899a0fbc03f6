// Micro-benchmark: histogram of G random features per row over a node-sorted row list,
// (A) one byte gather per (row, feature) vs (B) whole rows staged into LDS with coalesced
// 16-B loads, features read from LDS.  1M x 128-B binned table (the headline's Xb).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int LD = 128;
constexpr int G = 10;

__device__ __forceinline__ int feat_of(int blk, int j) { return (int)((blk * 2654435761u + j * 40503u) % 100u); }

// A: one thread per row, G byte gathers, LDS u64 atomics
__global__ __launch_bounds__(256) void kA(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  __shared__ unsigned long long h[G * 256];
  for (int i = threadIdx.x; i < G * 256; i += 256) h[i] = 0;
  __syncthreads();
  int f[G];
  for (int j = 0; j < G; ++j) f[j] = feat_of(blockIdx.x, j);
  const uint32_t* rr = rows + (size_t)blockIdx.x * chunk;
  for (int r = threadIdx.x; r < chunk; r += 256) {
    const uint32_t row = rr[r];
    const uint8_t* x = Xb + (size_t)row * LD;
    uint32_t b[G];
#pragma unroll
    for (int j = 0; j < G; ++j) b[j] = x[f[j]];
#pragma unroll
    for (int j = 0; j < G; ++j) atomicAdd(&h[j * 256 + b[j]], 1ull + (row & 1));
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < G * 256; i += 256) s += h[i] * (i + 1);
  if (threadIdx.x < 64) atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), s);
}

// B: 256 rows per tile staged into LDS (stride SB bytes), 8 lanes x 16 B per row
template <int SB>
__global__ __launch_bounds__(256) void kB(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  __shared__ unsigned long long h[G * 256];
  __shared__ __attribute__((aligned(16))) uint8_t tile[256 * SB];
  for (int i = threadIdx.x; i < G * 256; i += 256) h[i] = 0;
  int f[G];
  for (int j = 0; j < G; ++j) f[j] = feat_of(blockIdx.x, j);
  const uint32_t* rr = rows + (size_t)blockIdx.x * chunk;
  const int seg = threadIdx.x & 7;
  for (int base = 0; base < chunk; base += 256) {
    __syncthreads();
    // 8 passes of 32 rows: thread t loads segment t%8 of row base + pass*32 + t/8
    uint4 v[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int lr = p * 32 + (threadIdx.x >> 3);
      const uint32_t row = rr[base + lr];
      v[p] = *(const uint4*)(Xb + (size_t)row * LD + seg * 16);
    }
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int lr = p * 32 + (threadIdx.x >> 3);
      uint8_t* dst = tile + lr * SB + seg * 16;
      if constexpr (SB % 16 == 0) *(uint4*)dst = v[p];
      else { uint32_t* d = (uint32_t*)dst; d[0] = v[p].x; d[1] = v[p].y; d[2] = v[p].z; d[3] = v[p].w; }
    }
    __syncthreads();
    const uint32_t row = rr[base + threadIdx.x];
    const uint8_t* x = tile + threadIdx.x * SB;
    uint32_t b[G];
#pragma unroll
    for (int j = 0; j < G; ++j) b[j] = x[f[j]];
#pragma unroll
    for (int j = 0; j < G; ++j) atomicAdd(&h[j * 256 + b[j]], 1ull + (row & 1));
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < G * 256; i += 256) s += h[i] * (i + 1);
  if (threadIdx.x < 64) atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), s);
}


// B2: as B, register double-buffer: tile t+1's 16-B loads are in flight while tile t is
// read from LDS and histogrammed
template <int SB>
__global__ __launch_bounds__(256) void kB2(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  __shared__ unsigned long long h[G * 256];
  __shared__ __attribute__((aligned(16))) uint8_t tile[256 * SB];
  for (int i = threadIdx.x; i < G * 256; i += 256) h[i] = 0;
  int f[G];
  for (int j = 0; j < G; ++j) f[j] = feat_of(blockIdx.x, j);
  const uint32_t* rr = rows + (size_t)blockIdx.x * chunk;
  const int seg = threadIdx.x & 7;
  uint4 v[8];
  uint32_t rid[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) rid[p] = rr[p * 32 + (threadIdx.x >> 3)];
#pragma unroll
  for (int p = 0; p < 8; ++p) v[p] = *(const uint4*)(Xb + (size_t)rid[p] * LD + seg * 16);
  for (int base = 0; base < chunk; base += 256) {
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int lr = p * 32 + (threadIdx.x >> 3);
      uint8_t* dst = tile + lr * SB + seg * 16;
      if constexpr (SB % 16 == 0) *(uint4*)dst = v[p];
      else { uint32_t* d = (uint32_t*)dst; d[0] = v[p].x; d[1] = v[p].y; d[2] = v[p].z; d[3] = v[p].w; }
    }
    const uint32_t row = rr[base + threadIdx.x];
    if (base + 256 < chunk) {
#pragma unroll
      for (int p = 0; p < 8; ++p) rid[p] = rr[base + 256 + p * 32 + (threadIdx.x >> 3)];
#pragma unroll
      for (int p = 0; p < 8; ++p) v[p] = *(const uint4*)(Xb + (size_t)rid[p] * LD + seg * 16);
    }
    __syncthreads();
    const uint8_t* x = tile + threadIdx.x * SB;
    uint32_t b[G];
#pragma unroll
    for (int j = 0; j < G; ++j) b[j] = x[f[j]];
#pragma unroll
    for (int j = 0; j < G; ++j) atomicAdd(&h[j * 256 + b[j]], 1ull + (row & 1));
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < G * 256; i += 256) s += h[i] * (i + 1);
  if (threadIdx.x < 64) atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), s);
}

// C: gather version without histogram atomics (pure gather cost: xor-reduce the bins)
__global__ __launch_bounds__(256) void kC(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  int f[G];
  for (int j = 0; j < G; ++j) f[j] = feat_of(blockIdx.x, j);
  const uint32_t* rr = rows + (size_t)blockIdx.x * chunk;
  unsigned long long acc = 0;
  for (int r = threadIdx.x; r < chunk; r += 256) {
    const uint32_t row = rr[r];
    const uint8_t* x = Xb + (size_t)row * LD;
    uint32_t b[G];
#pragma unroll
    for (int j = 0; j < G; ++j) b[j] = x[f[j]];
#pragma unroll
    for (int j = 0; j < G; ++j) acc += b[j] * (j + 1);
  }
  atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), acc);
}

// D: atomics only (bins from a hash, no table reads): LDS histogram atomic cost
__global__ __launch_bounds__(256) void kD(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  __shared__ unsigned long long h[G * 256];
  for (int i = threadIdx.x; i < G * 256; i += 256) h[i] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < chunk; r += 256) {
    const uint32_t x = (uint32_t)(blockIdx.x * 0x9E3779B9u + r * 0x85EBCA6Bu);
#pragma unroll
    for (int j = 0; j < G; ++j) atomicAdd(&h[j * 256 + ((x >> (j * 3)) & 255)], 1ull);
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < G * 256; i += 256) s += h[i] * (i + 1);
  if (threadIdx.x < 64) atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), s);
}

// E: the G features' distinct 16-B segments gathered with dwordx4 loads (one per segment
// per row), bytes extracted in registers
__global__ __launch_bounds__(256) void kE(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  __shared__ unsigned long long h[G * 256];
  for (int i = threadIdx.x; i < G * 256; i += 256) h[i] = 0;
  __syncthreads();
  int f[G];
  for (int j = 0; j < G; ++j) f[j] = feat_of(blockIdx.x, j);
  // segment mask (uniform)
  uint32_t segmask = 0;
  for (int j = 0; j < G; ++j) segmask |= 1u << (f[j] >> 4);
  const uint32_t* rr = rows + (size_t)blockIdx.x * chunk;
  for (int r = threadIdx.x; r < chunk; r += 256) {
    const uint32_t row = rr[r];
    const uint8_t* x = Xb + (size_t)row * LD;
    uint4 seg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) if (segmask & (1u << k)) seg[k] = *(const uint4*)(x + 16 * k); else seg[k] = make_uint4(0,0,0,0);
    uint32_t b[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int k = f[j] >> 4, w = (f[j] >> 2) & 3, sh = (f[j] & 3) * 8;
      uint32_t v = 0;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) if (kk == k) v = w == 0 ? seg[kk].x : w == 1 ? seg[kk].y : w == 2 ? seg[kk].z : seg[kk].w;
      b[j] = (v >> sh) & 255u;
    }
#pragma unroll
    for (int j = 0; j < G; ++j) atomicAdd(&h[j * 256 + b[j]], 1ull + (row & 1));
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < G * 256; i += 256) s += h[i] * (i + 1);
  if (threadIdx.x < 64) atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), s);
}
// F: as A but 2-row software pipeline (next row's 10 bins in flight during this row's atomics)
__global__ __launch_bounds__(256) void kF(const uint8_t* Xb, const uint32_t* rows, int chunk, unsigned long long* out) {
  __shared__ unsigned long long h[G * 256];
  for (int i = threadIdx.x; i < G * 256; i += 256) h[i] = 0;
  __syncthreads();
  int f[G];
  for (int j = 0; j < G; ++j) f[j] = feat_of(blockIdx.x, j);
  const uint32_t* rr = rows + (size_t)blockIdx.x * chunk;
  uint32_t ra = threadIdx.x < chunk ? rr[threadIdx.x] : 0;
  uint32_t b0[G];
#pragma unroll
  for (int j = 0; j < G; ++j) b0[j] = Xb[(size_t)ra * LD + f[j]];
  for (int r = threadIdx.x; r < chunk; r += 256) {
    const bool more = r + 256 < chunk;
    const uint32_t rb = more ? rr[r + 256] : 0;
    uint32_t b1[G];
#pragma unroll
    for (int j = 0; j < G; ++j) b1[j] = more ? Xb[(size_t)rb * LD + f[j]] : 0u;
#pragma unroll
    for (int j = 0; j < G; ++j) atomicAdd(&h[j * 256 + b0[j]], 1ull + (ra & 1));
    ra = rb;
#pragma unroll
    for (int j = 0; j < G; ++j) b0[j] = b1[j];
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < G * 256; i += 256) s += h[i] * (i + 1);
  if (threadIdx.x < 64) atomicAdd(out + 8 + (blockIdx.x & 1023) * 8 + ((threadIdx.x & 7)), s);
}

int main(int argc, char** argv) {
  const int n = 1000000;
  const int chunk = argc > 1 ? atoi(argv[1]) : 1024;       // rows per block (= node size)
  const long total = argc > 2 ? atol(argv[2]) : 16000000;  // row visits
  const int nblk = (int)(total / chunk);
  std::vector<uint8_t> hx((size_t)n * LD);
  std::mt19937 g(1);
  for (auto& b : hx) b = (uint8_t)g();
  std::vector<uint32_t> hr((size_t)nblk * chunk);
  for (int b = 0; b < nblk; ++b) {
    for (int i = 0; i < chunk; ++i) hr[(size_t)b * chunk + i] = g() % n;
    std::sort(hr.begin() + (size_t)b * chunk, hr.begin() + (size_t)(b + 1) * chunk);
  }
  uint8_t* Xb; uint32_t* rows; unsigned long long* out;
  CHECK(hipMalloc(&Xb, hx.size())); CHECK(hipMalloc(&rows, hr.size() * 4)); CHECK(hipMalloc(&out, 10 * 8200 * 8));
  CHECK(hipMemcpy(Xb, hx.data(), hx.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, int slot) {
    for (int it = 0; it < 2; ++it) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int it = 0; it < reps; ++it) launch();
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    std::vector<unsigned long long> h(8200); CHECK(hipMemcpy(h.data(), out + (size_t)slot * 8200, 8200 * 8, hipMemcpyDeviceToHost));
    unsigned long long cs = 0; for (auto x : h) cs += x;
    printf("%-12s chunk %6d: %8.3f ms  %7.2f G row-visits/s  check %llu\n", name, chunk, ms, total / ms / 1e6, cs / 7);
  };
  CHECK(hipMemset(out, 0, 10 * 8200 * 8));
  run("gather", [&] { kA<<<nblk, 256>>>(Xb, rows, chunk, out + 0 * 8200); }, 0);
  run("seg16", [&] { kE<<<nblk, 256>>>(Xb, rows, chunk, out + 8 * 8200); }, 8);
  run("gather_pipe", [&] { kF<<<nblk, 256>>>(Xb, rows, chunk, out + 9 * 8200); }, 9);
  run("stage132", [&] { kB<132><<<nblk, 256>>>(Xb, rows, chunk, out + 1 * 8200); }, 1);
  run("stage144", [&] { kB<144><<<nblk, 256>>>(Xb, rows, chunk, out + 2 * 8200); }, 2);
  run("stage128", [&] { kB<128><<<nblk, 256>>>(Xb, rows, chunk, out + 3 * 8200); }, 3);
  run("stage2_132", [&] { kB2<132><<<nblk, 256>>>(Xb, rows, chunk, out + 4 * 8200); }, 4);
  run("stage2_144", [&] { kB2<144><<<nblk, 256>>>(Xb, rows, chunk, out + 5 * 8200); }, 5);
  run("gather_only", [&] { kC<<<nblk, 256>>>(Xb, rows, chunk, out + 6 * 8200); }, 6);
  run("atomics_only", [&] { kD<<<nblk, 256>>>(Xb, rows, chunk, out + 7 * 8200); }, 7);
  return 0;
}
