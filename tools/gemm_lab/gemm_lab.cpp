// Standalone GEMM / implicit-GEMM conv lab: numerics of the hand-written kernels against a naive fp32
// GPU reference, then interleaved timing rounds (guide rule 24) of v4 (gemm_8ph.hip) vs v5 (gemm_w4.hip) vs v6
// (gemm_8ph.hip) on random [-1, 1) bf16 operands.  No torch: builds in seconds with hipcc.
//
//   bash tools/gemm_lab/build.sh && ./build/gemm_lab [--quick]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels/launchers.h"

namespace shai {
void launch_gemm4(const GemmArgs& a, float* ws, int splits, int bn, hipStream_t s, bool persist);
bool gemm4_supported(const GemmArgs& a);
void launch_gemm4_var(const GemmArgs& a, int var, int bn, hipStream_t s);
bool gemm_w4_supported(const GemmArgs& a);
void launch_gemm_w4(const GemmArgs& a, int bn, hipStream_t s);
bool gemm_ws_supported(const GemmArgs& a);
void launch_gemm_ws(const GemmArgs& a, hipStream_t s);
void gemm_ws_set_ablation(int a);
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

__global__ void fill_kernel(bf16_t* p, long n, uint32_t seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = ((h & 0xffffff) / 16777216.0f * 2.f - 1.f) * scale;
    __bf16 b = (__bf16)f;
    p[i] = __builtin_bit_cast(bf16_t, b);
  }
}

// naive reference: C[m, n] = sum_k A[m, k] W[n, k] (+ bias) (+ residual) in fp32
__global__ void ref_gemm(const bf16_t* A, const bf16_t* W, const bf16_t* bias, const bf16_t* R, float* C, int M, int N,
                         int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf(A[(long)m * K + k]) * bf(W[(long)n * K + k]);
  if (bias) s += bf(bias[n]);
  if (R) s += bf(R[(long)m * N + n]);
  C[(long)m * N + n] = s;
}

// naive NHWC conv reference (3x3 / 1x1, stride, pad, optional nearest-2x upsample)
__global__ void ref_conv(const bf16_t* X, const bf16_t* W, float* C, int Nimg, int H, int Wd, int Cin, int OH, int OW,
                         int Cout, int KH, int KW, int stride, int pad, int ups) {
  const int co = blockIdx.x * blockDim.x + threadIdx.x;
  const long m = blockIdx.y;
  if (co >= Cout) return;
  const int n = (int)(m / (OH * OW)), rem = (int)(m % (OH * OW)), oh = rem / OW, ow = rem % OW;
  float s = 0.f;
  for (int kh = 0; kh < KH; ++kh)
    for (int kw = 0; kw < KW; ++kw) {
      int ih, iw;
      if (ups) {
        const int uh = oh - pad + kh, uw = ow - pad + kw;
        if (uh < 0 || uh >= 2 * H || uw < 0 || uw >= 2 * Wd) continue;
        ih = uh >> 1; iw = uw >> 1;
      } else {
        ih = oh * stride - pad + kh; iw = ow * stride - pad + kw;
        if (ih < 0 || ih >= H || iw < 0 || iw >= Wd) continue;
      }
      const bf16_t* x = X + (((long)n * H + ih) * Wd + iw) * Cin;
      const bf16_t* w = W + (long)co * KH * KW * Cin + (kh * KW + kw) * Cin;
      for (int c = 0; c < Cin; ++c) s += bf(x[c]) * bf(w[c]);
    }
  C[m * Cout + co] = s;
}

// GLU reference in place of the fp32 product: out[m, c] = h[m, 2c] * gelu(h[m, 2c + 1]) (erf GELU)
__global__ void ref_glu(const float* H, float* O, long M, int N) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= M * (N / 2)) return;
  const long m = i / (N / 2);
  const int c = (int)(i % (N / 2));
  const float a = H[m * N + 2 * c], g = H[m * N + 2 * c + 1];
  O[i] = a * 0.5f * g * (1.f + erff(g * 0.70710678f));
}

__global__ void err_kernel(const bf16_t* C, const float* R, long n, float* out) {
  float e = 0.f, r = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    e = fmaxf(e, fabsf(bf(C[i]) - R[i]));
    r = fmaxf(r, fabsf(R[i]));
  }
  atomicMax((int*)&out[0], __float_as_int(e));
  atomicMax((int*)&out[1], __float_as_int(r));
}

struct Problem {
  std::string name;
  int M, N, K;            // plain GEMM (conv: M = N*OH*OW, K = KH*KW*Cin)
  int conv = 0, Nimg = 0, H = 0, Wd = 0, Cin = 0, KH = 1, stride = 1, pad = 0, ups = 0;
  bool bias = false, res = false, glu = false;
  bool lnf = false;  // folded LayerNorm with (mean, rstd) = (0, 1) and zero column sums: same product, fold path timed
};

static Problem gemm(const char* nm, int M, int N, int K, bool bias = false, bool res = false) {
  Problem p;
  p.name = nm; p.M = M; p.N = N; p.K = K; p.bias = bias; p.res = res;
  return p;
}
static Problem geglu(const char* nm, int M, int N, int K) {
  Problem p = gemm(nm, M, N, K, true);
  p.glu = true;
  return p;
}
static Problem ln(Problem p) {
  p.lnf = true;
  p.name += "_ln";
  return p;
}
static Problem conv(const char* nm, int Nimg, int H, int Cin, int Cout, int KH, int ups = 0) {
  Problem p;
  p.name = nm; p.conv = 1; p.Nimg = Nimg; p.H = H; p.Wd = H; p.Cin = Cin; p.KH = KH; p.pad = KH / 2; p.ups = ups;
  const int oh = ups ? 2 * H : H;
  p.M = Nimg * oh * oh; p.N = Cout; p.K = KH * KH * Cin;
  return p;
}

static shai::GemmArgs make_args(const Problem& P, bf16_t* A, bf16_t* W, bf16_t* C, bf16_t* bias, bf16_t* R) {
  shai::GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.A = A; g.W = W; g.C = C; g.bias = P.bias ? bias : nullptr; g.residual = P.res ? R : nullptr;
  g.M = P.M; g.N = P.N; g.K = P.K;
  g.lda = P.conv ? P.Cin : P.K; g.ldw = P.K; g.ldc = P.glu ? P.N / 2 : P.N; g.ldr = g.ldc;
  if (P.glu) { g.glu = 1; g.act = 2; }  // ACT_GELU (erf)
  g.batch = 1; g.rows_per_bias2d = 1; g.alpha = 1.f; g.res_alpha = 1.f; g.rows_per_gate = 1;
  if (P.conv) {
    g.conv = 1; g.Nimg = P.Nimg; g.H = P.H; g.Wd = P.Wd; g.Cin = P.Cin; g.KH = P.KH; g.KW = P.KH;
    g.stride = P.stride; g.pad = P.pad; g.upsample = P.ups;
    g.OH = P.ups ? 2 * P.H : P.H; g.OW = P.ups ? 2 * P.Wd : P.Wd;
  }
  return g;
}

int main(int argc, char** argv) {
  const bool quick = argc > 1 && !strcmp(argv[1], "--quick");
  const bool plain_only = argc > 2 && !strcmp(argv[2], "--plain");
  std::vector<Problem> probs = {
      gemm("sq4096", 4096, 4096, 4096),
      gemm("sq8192", 8192, 8192, 8192),
      gemm("ragged", 1000, 1000, 1000, true, true),
      gemm("flux_ff_up", 4608, 12288, 3072, true),
      gemm("flux_ff_dn", 4608, 3072, 12288, false, true),
      gemm("sd_ff_up", 262144 / 4, 2560, 320, true),
      geglu("sd_geglu64", 262144, 2560, 320),
      geglu("sd_geglu32", 65536, 5120, 640),
      geglu("sd_geglu16", 16384, 10240, 1280),
      gemm("sd_qkv", 262144, 960, 320),
      gemm("sd_proj_res", 262144, 320, 320, true, true),
      gemm("sd_ff_dn_res", 65536, 640, 2560, true, true),
      gemm("llm_pf_qkv", 8192, 6144, 4096),
      gemm("ws_ragged_res", 1000, 640, 320, true, true),
      geglu("ws_ragged_glu", 1000, 960, 320),
      gemm("sd_q320", 262144, 320, 320, true),
      ln(geglu("sd_geglu64", 262144, 2560, 320)),
      ln(gemm("sd_qkv", 262144, 960, 320)),
      conv("unet64_320", 64, 64, 320, 320, 3),
      conv("unet32_640", 64, 32, 640, 640, 3),
      conv("unet16_1280", 64, 16, 1280, 1280, 3),
      conv("unet64_640to320", 64, 64, 640, 320, 3),
      conv("unet_up32_1280", 64, 16, 1280, 1280, 3, 1),
      conv("vae256_256", 4, 256, 256, 256, 3),
      gemm("sd_geglu32_plain", 65536, 5120, 640),
      gemm("sd_geglu16_plain", 16384, 10240, 1280),
  };
  if (quick) probs.resize(3);
  if (argc > 1 && !strcmp(argv[1], "--ws")) {  // the low-K problems of the W-stationary kernel only
    std::vector<Problem> q;
    for (auto& P : probs)
      if (!P.conv && P.K == 320) q.push_back(P);
    probs = q;
  }
  if (argc > 1 && !strcmp(argv[1], "--glu")) {  // GEGLU problems beside the plain GEMM of the same shape
    std::vector<Problem> q;
    for (auto& P : probs)
      if (!P.conv && !P.lnf && P.name.rfind("sd_geglu", 0) == 0) q.push_back(P);
    probs = q;
  }
  if (plain_only) {
    std::vector<Problem> q;
    for (auto& P : probs)
      if (!P.conv) q.push_back(P);
    probs = q;
  }
  size_t maxA = 0, maxW = 0, maxC = 0;
  for (auto& P : probs) {
    const size_t a = P.conv ? (size_t)P.Nimg * P.H * P.Wd * P.Cin : (size_t)P.M * P.K;
    maxA = std::max(maxA, a);
    maxW = std::max(maxW, (size_t)P.N * P.K);
    maxC = std::max(maxC, (size_t)P.M * P.N);
  }
  bf16_t *A, *W, *C, *bias, *R;
  float *ref, *err, *ws, *mr, *cols;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&W, maxW * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&R, maxC * 2));
  CK(hipMalloc(&bias, 65536 * 2));
  CK(hipMalloc(&ref, maxC * 6));  // GLU problems keep the product and the GLU output
  CK(hipMalloc(&err, 8));
  CK(hipMalloc(&ws, 64));
  {
    size_t maxM = 0;
    for (auto& P : probs) maxM = std::max(maxM, (size_t)P.M);
    std::vector<float> h(2 * maxM);
    for (size_t i = 0; i < maxM; ++i) { h[2 * i] = 0.f; h[2 * i + 1] = 1.f; }
    CK(hipMalloc(&mr, 2 * maxM * 4));
    CK(hipMemcpy(mr, h.data(), 2 * maxM * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&cols, 65536 * 4));
    CK(hipMemset(cols, 0, 65536 * 4));
  }
  fill_kernel<<<4096, 256>>>(A, maxA, 1u, 1.f);
  fill_kernel<<<4096, 256>>>(W, maxW, 2u, 1.f);
  fill_kernel<<<4096, 256>>>(R, maxC, 3u, 1.f);
  fill_kernel<<<64, 256>>>(bias, 65536, 4u, 1.f);
  CK(hipDeviceSynchronize());
  hipStream_t s = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  struct Var {
    const char* name;
    int kind;  // 0: v3 256 4-stage, 1: v3 256 2-stage, 2: v3 320 2-stage, 10+v: v4 schedule variant v
  };
  const Var vars[] = {{"v4_256w", 30}, {"v4_256pwn", 70}, {"v4_320w", 130}, {"v4_320pwn", 170}, {"w4_256", 5}, {"w4_320", 6},
                      {"ws_320", 7}, {"ws_nost", 107}, {"ws_nomfma", 207}, {"ws_nodma", 407}, {"ws_dmaonly", 307}};
  constexpr int NV = sizeof(vars) / sizeof(vars[0]);
  auto run = [&](const Var& v, const shai::GemmArgs& g) {
    switch (v.kind) {
      case 5: shai::launch_gemm_w4(g, 256, s); break;
      case 6: shai::launch_gemm_w4(g, 320, s); break;
      case 7: case 107: case 207: case 307: case 407:
        shai::gemm_ws_set_ablation(v.kind / 100);
        shai::launch_gemm_ws(g, s);
        shai::gemm_ws_set_ablation(0);
        break;
      default: shai::launch_gemm4_var(g, v.kind % 100 - 10, v.kind >= 100 ? 320 : 256, s); break;
    }
  };

  for (auto& P : probs) {
    shai::GemmArgs g = make_args(P, A, W, C, bias, R);
    if (P.lnf) {
      g.row_mr = mr;
      g.col_s = cols;
    }
    // reference
    if (P.conv) {
      ref_conv<<<dim3((P.N + 127) / 128, P.M), 128>>>(A, W, ref, P.Nimg, P.H, P.Wd, P.Cin, g.OH, g.OW, P.N, P.KH, P.KH,
                                                      1, P.pad, P.ups);
    } else {
      ref_gemm<<<dim3((P.N + 127) / 128, P.M), 128>>>(A, W, P.bias ? bias : nullptr, P.res ? R : nullptr, ref, P.M,
                                                      P.N, P.K);
    }
    if (P.glu) {  // ref holds the M x N product; the GLU output (M x N/2) goes behind it
      const long no = (long)P.M * (P.N / 2);
      ref_glu<<<(unsigned)((no + 255) / 256), 256>>>(ref, ref + (long)P.M * P.N, P.M, P.N);
    }
    CK(hipDeviceSynchronize());
    const float* refc = P.glu ? ref + (long)P.M * P.N : ref;
    const long nout = P.glu ? (long)P.M * (P.N / 2) : (long)P.M * P.N;
    const double flop = 2.0 * P.M * P.N * P.K;
    printf("== %s M=%d N=%d K=%d%s\n", P.name.c_str(), P.M, P.N, P.K, P.conv ? " (conv)" : "");
    std::vector<float> best(NV, 1e30f);
    for (int vi = 0; vi < NV; ++vi) {
      if (vars[vi].kind >= 10 && vars[vi].kind % 100 != 7 && !shai::gemm4_supported(g)) continue;
      if ((vars[vi].kind == 5 || vars[vi].kind == 6) && !shai::gemm_w4_supported(g)) continue;
      if (vars[vi].kind % 100 == 7 && !shai::gemm_ws_supported(g)) continue;
      if (vars[vi].kind > 100 && vars[vi].kind % 100 == 7) continue;  // ablations: timing only
      CK(hipMemset(C, 0, (size_t)P.M * P.N * 2));
      CK(hipMemset(err, 0, 8));
      run(vars[vi], g);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      err_kernel<<<1024, 256>>>(C, refc, nout, err);
      float he[2];
      CK(hipMemcpy(he, err, 8, hipMemcpyDeviceToHost));
      const float tol = 0.02f * he[1] + 0.05f;
      printf("  %-10s max_abs_err=%.4f (max |ref| %.2f) %s\n", vars[vi].name, he[0], he[1],
             he[0] <= tol ? "OK" : "MISMATCH");
    }
    const int rounds = quick ? 2 : 5, iters = 10;
    for (int r = 0; r < rounds; ++r) {
      for (int vi = 0; vi < NV; ++vi) {
        if (vars[vi].kind >= 10 && vars[vi].kind % 100 != 7 && !shai::gemm4_supported(g)) continue;
        if ((vars[vi].kind == 5 || vars[vi].kind == 6) && !shai::gemm_w4_supported(g)) continue;
        if (vars[vi].kind % 100 == 7 && !shai::gemm_ws_supported(g)) continue;
        run(vars[vi], g);
        CK(hipEventRecord(e0, s));
        for (int it = 0; it < iters; ++it) run(vars[vi], g);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best[vi] = std::min(best[vi], ms / iters);
      }
    }
    for (int vi = 0; vi < NV; ++vi) {
      if (best[vi] > 1e29f) continue;
      printf("  %-10s %9.1f us  %7.1f TF/s\n", vars[vi].name, best[vi] * 1e3, flop / (best[vi] * 1e-3) / 1e12);
    }
    fflush(stdout);
  }
  return 0;
}
