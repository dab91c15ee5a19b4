// Standalone flash-attention lab: flash2 (attention2.hip) vs v1 (attention.hip) timing on random inputs,
// a numerics spot check of flash2 against a naive fp32 GPU reference, timing ablations (no softmax / no
// MFMA in the loop) and per-segment s_memtime stamps of one workgroup.
//
//   bash tools/gemm_lab/build.sh && ./tools/gemm_lab/bin/attn_lab
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels/launchers.h"

namespace shai {
void launch_flash2_exp(const AttnArgs& a, int exp, hipStream_t s);
void flash2_read_stamps(unsigned long long* host);
}  // namespace shai
using shai::bf16_t;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__device__ __forceinline__ float bf(bf16_t x) { return __uint_as_float((uint32_t)x << 16); }

__global__ void fill(bf16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    // approximately N(0, 1): sum of 4 uniforms, rescaled
    float u = 0.f;
    for (int r = 0; r < 4; ++r) { u += (h & 0xff) / 255.f; h >>= 8; }
    __bf16 b = (__bf16)((u - 2.f) * 1.7320508f);
    p[i] = __builtin_bit_cast(bf16_t, b);
  }
}

// reference for the first `rows` queries of (b = 0, h = 0): one thread per query row
__global__ void ref_rows(const bf16_t* q, const bf16_t* k, const bf16_t* v, float* out, int S, int H, int D, int rows,
                         float scale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  float m = -1e30f, l = 0.f;
  float acc[128];
  for (int d = 0; d < D; ++d) acc[d] = 0.f;
  for (int j = 0; j < S; ++j) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += bf(q[(long)i * H * D + d]) * bf(k[(long)j * H * D + d]);
    s *= scale;
    const float mn = fmaxf(m, s), a = expf(m - mn), p = expf(s - mn);
    l = l * a + p;
    for (int d = 0; d < D; ++d) acc[d] = acc[d] * a + p * bf(v[(long)j * H * D + d]);
    m = mn;
  }
  for (int d = 0; d < D; ++d) out[i * D + d] = acc[d] / l;
}

int main() {
  struct Case { int B, H, S, D; };
  const Case cases[] = {{8, 5, 4096, 64}, {64, 5, 4096, 64}, {8, 10, 1024, 64}, {64, 10, 1024, 64}, {1, 24, 4608, 128}, {4, 32, 2048, 128}};
  setenv("SHAI_FLASH_V1", "1", 1);  // launch_flash_attn -> v1 kernel
  setenv("SHAI_FLASH64_DMA", "0", 1);  // launch_flash64 -> the register-staged kernel (the DMA one is its own row)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Case& c : cases) {
    const long n = (long)c.B * c.S * c.H * c.D;
    bf16_t *q, *k, *v, *o;
    CK(hipMalloc(&q, n * 2)); CK(hipMalloc(&k, n * 2)); CK(hipMalloc(&v, n * 2)); CK(hipMalloc(&o, n * 2));
    fill<<<2048, 256>>>(q, n, 1); fill<<<2048, 256>>>(k, n, 2); fill<<<2048, 256>>>(v, n, 3);
    shai::AttnArgs a{};
    a.q = q; a.k = k; a.v = v; a.o = o;
    a.B = c.B; a.Sq = c.S; a.Skv = c.S; a.Hq = c.H; a.Hkv = c.H; a.D = c.D;
    const long ts = (long)c.H * c.D, bs = ts * c.S;
    a.q_bs = a.k_bs = a.v_bs = a.o_bs = bs;
    a.q_ts = a.k_ts = a.v_ts = a.o_ts = ts;
    a.scale = 1.f / sqrtf((float)c.D);
    const double flop = 4.0 * c.B * c.H * (double)c.S * c.S * c.D;
    printf("== B%d H%d S%d d%d\n", c.B, c.H, c.S, c.D);
    // numerics spot check (flash2 production variant)
    {
      const int rows = 64;
      float* ref;
      CK(hipMalloc(&ref, rows * c.D * 4));
      ref_rows<<<1, 64>>>(q, k, v, ref, c.S, c.H, c.D, rows, a.scale);
      CK(hipDeviceSynchronize());
      for (int kv = 0; kv < (c.D == 64 ? 3 : 1); ++kv) {
      if (c.D == 64) {
        if (kv == 0) shai::launch_flash64(a, 0);  // production d64 kernel
        else if (kv == 2) shai::launch_flash64_x2(a, 0);
        else shai::launch_flash64_dma(a, 0);
      } else shai::launch_flash2_exp(a, 0, 0);
      CK(hipDeviceSynchronize());
      std::vector<float> hr(rows * c.D);
      std::vector<bf16_t> ho(rows * ts);
      CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ho.data(), o, ho.size() * 2, hipMemcpyDeviceToHost));
      double err = 0, mx = 0;
      for (int i = 0; i < rows; ++i)
        for (int d = 0; d < c.D; ++d) {
          uint32_t u = (uint32_t)ho[(long)i * ts + d] << 16;
          float f;
          memcpy(&f, &u, 4);
          err = fmax(err, fabs(f - hr[i * c.D + d]));
          mx = fmax(mx, fabs(hr[i * c.D + d]));
        }
      printf("  %s max_abs_err %.4f (max |ref| %.3f) %s\n", c.D == 64 ? (kv == 0 ? "flash64" : kv == 1 ? "f64dma" : "f64x2") : "flash2", err, mx, err < 0.02 * mx + 0.01 ? "OK" : "MISMATCH");
      }
      CK(hipFree(ref));
    }
    struct V { const char* name; int exp; };  // exp < 0: v1
    const V vars[] = {{"v1", -1}, {"flash2", 0}, {"flash64", -2}, {"f64dma", -3}, {"f64x2", -5}};
    constexpr int NV = sizeof(vars) / sizeof(vars[0]);
    float best[NV];
    for (int vi = 0; vi < NV; ++vi) best[vi] = 1e30f;
    for (int r = 0; r < 5; ++r)
      for (int vi = 0; vi < NV; ++vi) {
        if (vars[vi].exp <= -3 && c.D != 64) continue;
        auto run = [&]() {
          if (vars[vi].exp == -2) { if (c.D == 64) shai::launch_flash64(a, 0); }
          else if (vars[vi].exp == -3) shai::launch_flash64_dma(a, 0);
          else if (vars[vi].exp == -5) shai::launch_flash64_x2(a, 0);
          else if (vars[vi].exp < 0) shai::launch_flash_attn(a, 0);
          else shai::launch_flash2_exp(a, vars[vi].exp, 0);
        };
        run();
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < 10; ++it) run();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best[vi] = fminf(best[vi], ms / 10);
      }
    for (int vi = 0; vi < NV; ++vi)
      if (best[vi] < 1e29f)
        printf("  %-13s %8.1f us  %7.1f TF/s\n", vars[vi].name, best[vi] * 1e3, flop / (best[vi] * 1e-3) / 1e12);
    // stamps: 4 per tile per wave (M start, M end, V start, V end); print mean durations over tiles 2..nt-2
    for (int exp : {4, 12}) {
      shai::launch_flash2_exp(a, exp, 0);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> st(2 * 2048);
      shai::flash2_read_stamps(st.data());
      const int nt = (c.S + 63) / 64;
      for (int g = 0; g < 2; ++g) {
        double mseg = 0, mbar = 0, vseg = 0, vbar = 0;
        int cnt = 0;
        for (int t = 2; t + 2 < nt && 4 * t + 4 < 2048; ++t, ++cnt) {
          const unsigned long long* s = &st[g * 2048 + 4 * t];
          mseg += (double)(s[1] - s[0]);
          mbar += (double)(s[2] - s[1]);
          vseg += (double)(s[3] - s[2]);
          vbar += (double)(s[4] - s[3]);
        }
        printf("  stamps exp%d group %d: M-seg %.0f, wait %.0f, V-seg %.0f, wait %.0f cycles (mean of %d tiles)\n",
               exp, g, mseg / cnt, mbar / cnt, vseg / cnt, vbar / cnt, cnt);
      }
    }
    CK(hipFree(q)); CK(hipFree(k)); CK(hipFree(v)); CK(hipFree(o));
  }
  return 0;
}
