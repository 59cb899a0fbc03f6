// Row-gather microbenchmark: per-lane row windows vs cooperative (lane-linear) row loads.
//
// Question: the forest builder's block / wave tiers read, per row visit, the row's 112-B bin
// line as 7 dwordx4 loads issued by ONE lane (64 rows per wave-instruction: 64 cache-line
// lookups per instruction).  Loading the same rows cooperatively (7 lanes per row, 9 rows
// per wave-instruction, ~16 lines) costs ~4x fewer lookups, but the bytes then sit in the
// wrong lanes and go through LDS.  Which wins once the histogram atomics are counted?
//
//   A  per-lane windows   : 7 x global_load_dwordx4 per lane-row, bytes by uniform register index
//   B  cooperative + LDS  : global_load_lds_dwordx4 (lane-linear image, 7 per 64 rows),
//                           then each lane reads its row's G bytes with ds_read_u8
//   C  cooperative regs   : global_load_dwordx4 in the same lane-linear order + ds_write_b128
//
// Each row visit adds G = 10 bins into a per-workgroup LDS histogram (G x 256 u32), as the
// block tier does.  Table: N rows x 112 B, random row ids.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/micro_coop_gather.bin scripts/micro_coop_gather.hip
//   (run the binary on the GPU box: ./scripts/micro_coop_gather.bin [rows] [visits] [row pitch])
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int LD = 112;      // row bytes
constexpr int G = 10;        // features per row visit
constexpr int NT = 256;      // threads per workgroup
constexpr int ROWS_PER_WAVE_STEP = 64;

struct Feats { int f[G]; };

template <bool ATOM>
__global__ __launch_bounds__(NT) void k_perlane(const uint8_t* __restrict__ X, const uint32_t* __restrict__ idx,
                                                int64_t nvis, int per_wg, Feats fs, uint32_t* out, int pitch) {
  __shared__ uint32_t hist[G * 256];
  for (int i = threadIdx.x; i < G * 256; i += NT) hist[i] = 0;
  __syncthreads();
  typedef uint32_t v32u __attribute__((ext_vector_type(32)));
  int fdw[G], fsh[G];
#pragma unroll
  for (int j = 0; j < G; ++j) { fdw[j] = fs.f[j] >> 2; fsh[j] = (fs.f[j] & 3) * 8; }
  const int64_t b0 = (int64_t)blockIdx.x * per_wg;
  const int64_t b1 = b0 + per_wg < nvis ? b0 + per_wg : nvis;
  uint32_t acc = 0;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += NT) {
    const uint32_t r = idx[i];
    const uint4* xr = (const uint4*)(X + (int64_t)r * pitch);
    v32u w;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const uint4 q = xr[k];
      w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t b = (w[fdw[j]] >> fsh[j]) & 0xFFu;
      if (ATOM) atomicAdd(&hist[j * 256 + b], 1u);
      else acc += b * (j + 1);
    }
  }
  if (!ATOM) atomicAdd(&out[G * 256], acc);
  __syncthreads();
  for (int i = threadIdx.x; i < G * 256; i += NT) atomicAdd(&out[i], hist[i]);
}

// cooperative: the wave's 64 rows of a step land in LDS as a lane-linear 64 x 112-B image
// (7 KiB), chunk q = k*64 + lane -> row q / 7, window q % 7
template <bool GLDS, int NB, bool ATOM>
__global__ __launch_bounds__(NT) void k_coop(const uint8_t* __restrict__ X, const uint32_t* __restrict__ idx,
                                             int64_t nvis, int per_wg, Feats fs, uint32_t* out, int pitch) {
  __shared__ uint32_t hist[G * 256];
  __shared__ __attribute__((aligned(16))) uint8_t img[NT / 64][NB][64 * LD];
  for (int i = threadIdx.x; i < G * 256; i += NT) hist[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * per_wg;
  const int64_t b1 = b0 + per_wg < nvis ? b0 + per_wg : nvis;
  // each wave takes consecutive 64-visit steps of the workgroup's range
  const int64_t nsteps = (b1 - b0 + 63) / 64;
  // row ids of a step's 7 chunks first (clamped, no branches), then the 7 row loads: a
  // row load waiting on its id must not also wait on older row loads
  auto ids = [&](int64_t step, uint32_t* r) {
    const int64_t base = b0 + step * 64;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int q = k * 64 + lane;
      const int64_t vi = base + q / 7;
      r[k] = idx[vi < b1 ? vi : b1 - 1];
    }
  };
  auto stage = [&](const uint32_t* r, int buf) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int q = k * 64 + lane;
      const int win = q - (q / 7) * 7;
      const uint8_t* src = X + (int64_t)r[k] * pitch + win * 16;
      uint8_t* dst = &img[wv][buf][k * 1024];
      if constexpr (GLDS) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      } else {
        const uint4 v = *(const uint4*)src;
        *(uint4*)(dst + lane * 16) = v;
      }
    }
  };
  int buf = 0;
  uint32_t acc = 0;
  int64_t s = wv;
  uint32_t rid[7];
  if (NB == 2 && s < nsteps) { ids(s, rid); stage(rid, 0); }
  for (; s < nsteps; s += NT / 64) {
    if constexpr (NB == 1) {
      ids(s, rid);
      stage(rid, 0);
      __builtin_amdgcn_s_waitcnt(GLDS ? 0x0F70 : 0xC07F);
    } else {
      const int64_t sn = s + NT / 64;
      if (sn < nsteps) {
        ids(sn, rid);                       // waits (in order) for this step's rows too
        stage(rid, buf ^ 1);
        if constexpr (GLDS) __builtin_amdgcn_s_waitcnt(0x0F77);   // vmcnt(7): this step's rows landed
      } else if constexpr (GLDS) {
        __builtin_amdgcn_s_waitcnt(0x0F70);                        // vmcnt(0)
      }
      if constexpr (!GLDS) __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0): ds_writes done
    }
    __builtin_amdgcn_wave_barrier();
    const int64_t vi = b0 + s * 64 + lane;
    const uint8_t* row = &img[wv][buf][lane * LD];
    uint32_t bv[G];
#pragma unroll
    for (int j = 0; j < G; ++j) bv[j] = row[fs.f[j]];
    if (vi < b1) {
#pragma unroll
      for (int j = 0; j < G; ++j) {
        if (ATOM) atomicAdd(&hist[j * 256 + bv[j]], 1u);
        else acc += bv[j] * (j + 1);
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (NB == 2) buf ^= 1;
  }
  if (!ATOM) atomicAdd(&out[G * 256], acc);
  __syncthreads();
  for (int i = threadIdx.x; i < G * 256; i += NT) atomicAdd(&out[i], hist[i]);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int64_t nvis = argc > 2 ? atoll(argv[2]) : 64 << 20;
  const int pitch = argc > 3 ? atoi(argv[3]) : LD;
  std::vector<uint8_t> hX((size_t)n * pitch);
  uint64_t z = 88172645463325252ull;
  auto rnd = [&]() { z ^= z << 13; z ^= z >> 7; z ^= z << 17; return z; };
  for (auto& b : hX) b = (uint8_t)rnd();
  std::vector<uint32_t> hI(nvis);
  for (auto& v : hI) v = (uint32_t)(rnd() % (uint64_t)n);
  Feats fs;
  const int fl[G] = {3, 17, 22, 38, 41, 57, 70, 84, 91, 99};
  for (int j = 0; j < G; ++j) fs.f[j] = fl[j];
  // host reference histogram
  std::vector<uint32_t> ref(G * 256, 0);
  for (int64_t i = 0; i < nvis; ++i)
    for (int j = 0; j < G; ++j) ref[j * 256 + hX[(size_t)hI[i] * pitch + fs.f[j]]]++;
  uint8_t* X; uint32_t *I, *out;
  CK(hipMalloc(&X, hX.size())); CK(hipMalloc(&I, nvis * 4)); CK(hipMalloc(&out, (G * 256 + 1) * 4));
  CK(hipMemcpy(X, hX.data(), hX.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(I, hI.data(), nvis * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int per_wg = 4096;
  const int nwg = (int)((nvis + per_wg - 1) / per_wg);
  const char* names[5] = {"A per-lane windows", "B coop glds x2", "C coop regs x2", "B1 coop glds x1", "C1 coop regs x1"};
  uint64_t ref_acc = 0;
  for (int64_t i = 0; i < nvis; ++i)
    for (int j = 0; j < G; ++j) ref_acc += (uint64_t)hX[(size_t)hI[i] * pitch + fs.f[j]] * (j + 1);
  for (int atom = 1; atom >= 0; --atom)
  for (int v = 0; v < 5; ++v) {
    float best = 1e30f;
    bool ok = true;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemset(out, 0, (G * 256 + 1) * 4));
      CK(hipEventRecord(e0));
#define L(K) K<<<nwg, NT>>>(X, I, nvis, per_wg, fs, out, pitch)
      if (atom) {
        if (v == 0) L(k_perlane<true>); else if (v == 1) L((k_coop<true, 2, true>)); else if (v == 2) L((k_coop<false, 2, true>));
        else if (v == 3) L((k_coop<true, 1, true>)); else L((k_coop<false, 1, true>));
      } else {
        if (v == 0) L(k_perlane<false>); else if (v == 1) L((k_coop<true, 2, false>)); else if (v == 2) L((k_coop<false, 2, false>));
        else if (v == 3) L((k_coop<true, 1, false>)); else L((k_coop<false, 1, false>));
      }
#undef L
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
      std::vector<uint32_t> h(G * 256 + 1);
      CK(hipMemcpy(h.data(), out, (G * 256 + 1) * 4, hipMemcpyDeviceToHost));
      if (atom) ok = ok && std::equal(ref.begin(), ref.end(), h.begin());
      else ok = ok && h[G * 256] == (uint32_t)ref_acc;
    }
    printf("%s %-22s %8.3f ms  %7.2f G row-visits/s  %s\n", atom ? "hist " : "xor  ", names[v], best,
           nvis / (best * 1e-3) / 1e9, ok ? "ok" : "MISMATCH");
  }
  return 0;
}
