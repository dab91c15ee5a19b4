// Decode-GEMM lab (M = 64 activation rows, bf16 W [N, K]): where does the skinny kernel's time go?
// A stripped copy of the skinny kernel's streaming skeleton (gemv.hip: 64-row W tile, 4 waves, LDS-DMA ring,
// one barrier per 64-deep K step) with the pieces switchable at compile time --
//   W   : the weight tile DMA only (the HBM stream at this geometry)
//   WX  : + the 64-row activation tile DMA (what every workgroup re-stages from L2)
//   WXM : + fragment reads and the MFMAs (the production inner loop, partial sums written out)
// -- against the production kernel (launch_skinny_kg) on the Mistral-7B shapes, weights rotated over enough copies
// to stream HBM.  Build and run on the box:  hipcc ... decode_lab.cpp gemv.o (tools/gemm_lab/build_decode.sh).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels/launchers.h"

using shai::bf16_t;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

typedef __bf16 bf16x8l __attribute__((ext_vector_type(8)));
typedef float f16l __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lab_lds_void;

__global__ void fill_kernel(bf16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float f = ((h & 0xffffff) / 16777216.0f * 2.f - 1.f) * 0.02f;
    p[i] = __builtin_bit_cast(bf16_t, (__bf16)f);
  }
}

__device__ __forceinline__ int swz(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3); }

template <int PER, int N>
__device__ __forceinline__ void wait_upto(int pending) {
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (pending >= N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N * PER) : "memory");
    else wait_upto<PER, N - 1>(pending);
  }
}

// MODE 0 = W, 1 = WX, 2 = WXM.  STAGES-deep ring of (W 64x64 [+ X 64x64]) tiles.
template <int MODE, int STAGES, bool NT>
__global__ void __launch_bounds__(256) sk_lab(const bf16_t* __restrict__ W, const bf16_t* __restrict__ X, int N, int K,
                                              int kg_steps, float* __restrict__ out) {
  constexpr bool DX = MODE >= 1, DM = MODE >= 2;
  constexpr int W_EL = 64 * 64, X_EL = DX ? 64 * 64 : 0, ST = W_EL + X_EL, PER = 2 + (DX ? 2 : 0);
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * 64, kg = blockIdx.y;
  const int ksteps = K / 64, t0 = kg * kg_steps, nk = max(0, min(ksteps, t0 + kg_steps) - t0);
  const __amdgpu_buffer_rsrc_t rW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(W), (short)0, (int)min((long)N * K * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t rX =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X), (short)0, 64 * K * 2, 0x00020000);
  const int lrow = lane >> 3, lpos = lane & 7;
  int wr[2], wc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    wr[j] = (w * 2 + j) * 8 + lrow;
    wc[j] = lpos ^ ((wr[j] >> 1) & 7);
  }
  const int xr = w * 8 + lrow, xc = lpos ^ ((xr >> 1) & 7);
  auto stage = [&](int buf, int step) {
    bf16_t* sw = sm + buf * ST;
    const int k0 = (t0 + step) * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t off = (uint32_t)(((long)(n0 + wr[j]) * K + k0 + wc[j] * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lab_lds_void*)(sw + (w * 2 + j) * 8 * 64), 16, off, 0, 0, NT ? 2 : 0);
    }
    if constexpr (DX) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t off = (uint32_t)(((long)(xr + 32 * j) * K + k0 + xc * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lab_lds_void*)(sw + W_EL + (32 * j + w * 8) * 64), 16, off, 0, 0, 0);
      }
    }
  };
  f16l acc[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[h][j][i] = 0.f;
  const int fr = lane & 31, fh = lane >> 5, ch = 2 * w + fh;
  float sink = 0.f;
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < nk) stage(i, i);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    wait_upto<PER, STAGES - 2>(min(STAGES - 2, nk - 1 - kt));
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nk) stage(buf == 0 ? STAGES - 1 : buf - 1, kt + STAGES - 1);
    const bf16_t* sw = sm + buf * ST;
    if constexpr (DM) {
      const bf16x8l w0 = *reinterpret_cast<const bf16x8l*>(sw + swz(fr, ch));
      const bf16x8l w1 = *reinterpret_cast<const bf16x8l*>(sw + swz(32 + fr, ch));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8l xf = *reinterpret_cast<const bf16x8l*>(sw + W_EL + swz(32 * j + fr, ch));
        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, xf, acc[0][j], 0, 0, 0);
        acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, xf, acc[1][j], 0, 0, 0);
      }
    } else {
      sink += (float)sw[lane];  // one LDS read per step so the loop is not empty
    }
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = sink;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) s += acc[h][j][i];
  out[((long)blockIdx.y * gridDim.x + blockIdx.x) * 256 + tid] = s;
}

template <int MODE, int STAGES, bool NT>
void run_lab(const bf16_t* W, const bf16_t* X, int N, int K, int kg, float* out, hipStream_t s) {
  const int ksteps = K / 64, kgs = (ksteps + kg - 1) / kg;
  const size_t lds = (size_t)STAGES * (64 * 64 + (MODE >= 1 ? 64 * 64 : 0)) * 2;
  sk_lab<MODE, STAGES, NT><<<dim3(N / 64, kg), 256, lds, s>>>(W, X, N, K, kgs, out);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  struct Shape { const char* name; int N, K; };
  const Shape shapes[] = {{"qkv 6144x4096", 6144, 4096}, {"o 4096x4096", 4096, 4096},
                          {"gate_up 28672x4096", 28672, 4096}, {"down 4096x14336", 4096, 14336}};
  const int M = 64;
  bf16_t* X;
  CK(hipMalloc(&X, (size_t)M * 14336 * 2));
  fill_kernel<<<1024, 256>>>(X, (long)M * 14336, 7);
  float* out;
  CK(hipMalloc(&out, (size_t)64 << 20));
  float* ws;
  CK(hipMalloc(&ws, (size_t)256 << 20));
  bf16_t* C;
  CK(hipMalloc(&C, (size_t)M * 28672 * 2));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    const long wbytes = (long)sh.N * sh.K * 2;
    const int ncopy = (int)std::max(2L, std::min(16L, (768L << 20) / wbytes + 1));
    std::vector<bf16_t*> Ws(ncopy);
    for (int i = 0; i < ncopy; ++i) {
      CK(hipMalloc(&Ws[i], wbytes));
      fill_kernel<<<2048, 256>>>(Ws[i], (long)sh.N * sh.K, 11 + i);
    }
    CK(hipDeviceSynchronize());
    auto timeit = [&](auto&& fn) {
      for (int i = 0; i < 4; ++i) fn(Ws[i % ncopy]);
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) fn(Ws[i % ncopy]);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1000.f / iters;
    };
    printf("== %s (%.1f MB of weights, %d copies)\n", sh.name, wbytes / 1e6, ncopy);
    for (int kg : {1, 2, 4, 8}) {
      if ((sh.K / 64) / kg < 4) continue;
      const float tw = timeit([&](const bf16_t* W) { run_lab<0, 4, true>(W, X, sh.N, sh.K, kg, out, st); });
      const float tw6 = timeit([&](const bf16_t* W) { run_lab<0, 8, true>(W, X, sh.N, sh.K, kg, out, st); });
      const float twx = timeit([&](const bf16_t* W) { run_lab<1, 4, true>(W, X, sh.N, sh.K, kg, out, st); });
      const float twxm = timeit([&](const bf16_t* W) { run_lab<2, 4, true>(W, X, sh.N, sh.K, kg, out, st); });
      shai::GemmArgs g{};
      g.A = X;
      g.M = M;
      g.K = sh.K;
      g.N = sh.N;
      g.lda = sh.K;
      g.ldw = sh.K;
      g.C = C;
      g.ldc = sh.N;
      g.batch = 1;
      g.alpha = 1.f;
      g.res_alpha = 1.f;
      const float tp = timeit([&](const bf16_t* W) {
        g.W = W;
        shai::launch_skinny_kg(g, ws, kg, st, true, true);
      });
      // production kernel, split-K partial slabs only (no fixup, no fold launch): loop + cross-wave LDS reduction +
      // fp32 partial stores
      const float tpp = kg > 1 ? timeit([&](const bf16_t* W) {
        g.W = W;
        shai::launch_skinny_kg(g, ws, kg, st, false, false);
      }) : 0.f;
      // production kernel with a separate fold launch
      const float tpf = kg > 1 ? timeit([&](const bf16_t* W) {
        g.W = W;
        shai::launch_skinny_kg(g, ws, kg, st, false, true);
      }) : 0.f;
      auto tb = [&](float us) { return wbytes / (us * 1e-6) / 1e12; };
      printf("kg %2d (%4d WGs): W-only %6.1f us %.2f TB/s | W 8-stage %6.1f us %.2f | W+X %6.1f us %.2f | W+X+MFMA %6.1f us "
             "%.2f | production fixup %6.1f us %.2f | partials only %6.1f | + fold launch %6.1f\n",
             kg, sh.N / 64 * kg, tw, tb(tw), tw6, tb(tw6), twx, tb(twx), twxm, tb(twxm), tp, tb(tp), tpp, tpf);
    }
    for (bf16_t* p : Ws) CK(hipFree(p));
  }
  return 0;
}
