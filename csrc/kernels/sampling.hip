// Fused temperature / top-k / top-p / multinomial sampling, one workgroup per
// sequence (the reference relies on Neuron on-device sampling with
// global_topk 64, cova/mllama-32-11b-vllm-trn1-config.yaml:19-22, and on vLLM's
// sampler with temperature 0.7 / top-k 50 / top-p 0.9, app/vllm_model_api.py:24).
//
// Replaces the topk -> softmax -> cumsum -> mask -> multinomial -> gather chain
// (six launches and a [B, V] fp32 copy) with one kernel:
//   1. exact K-th largest logit by 4-pass byte radix select over order-preserving
//      uint32 keys (wave-private LDS histograms, row re-read from L2 each pass);
//   2. gather exactly K candidates (of the keys equal to the K-th, the lowest indices) into LDS;
//   3. bitonic sort of the candidates (descending value, ascending index: deterministic);
//   4. p_i = exp((l_i - l_0) / T), inclusive block scan, nucleus cut at top_p
//      (keep i while the mass BEFORE i is <= top_p of the total -- the same rule
//      as the torch reference path), draw with a host-supplied uniform.
// Temperature <= 0 rows are greedy (K = 1).  Same distribution as
// shai_amd.engines.llm.sample(); the uniforms come from the engine's generator.
#include "common.h"
#include "launchers.h"

namespace shai {

constexpr int SMP_T = 1024;          // threads per row
constexpr int SMP_MAXK = 1024;       // candidates kept in LDS
constexpr int SMP_WAVES = SMP_T / 64;

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <bool BF16>
__device__ __forceinline__ float smp_load(const void* row, int i) {
  if constexpr (BF16) return bf2f(reinterpret_cast<const bf16_t*>(row)[i]);
  else return reinterpret_cast<const float*>(row)[i];
}

template <bool BF16>
__global__ void __launch_bounds__(SMP_T) sample_kernel(const void* __restrict__ logits, long ld, int V,
                                                       const float* __restrict__ temps, const int* __restrict__ topk,
                                                       const float* __restrict__ topp,
                                                       const float* __restrict__ uniforms, int* __restrict__ out) {
  // 4 histogram copies per wave (by lane & 3): logits crowd into a few exponent bins, and same-address LDS
  // atomics of one wave instruction serialise -- the copies cut the worst case from 64-way to 16-way
  __shared__ uint32_t hist[SMP_WAVES][4][256];
  __shared__ uint32_t tot[256];
  __shared__ float cval[SMP_MAXK];
  __shared__ int cidx[SMP_MAXK];
  __shared__ float scan[SMP_MAXK];
  __shared__ uint32_t s_prefix, s_k, s_cnt, s_eq;
  const int row = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const char* base = reinterpret_cast<const char*>(logits) + (long)row * ld * (BF16 ? 2 : 4);
  const float T = temps[row];
  int K = topk[row];
  if (T <= 0.f) K = 1;
  if (K <= 0 || K > V) K = V;
  K = min(K, SMP_MAXK);

  // ---- 1. radix select: key threshold with count(key > thr) < K <= count(key >= thr)
  if (tid == 0) {
    s_prefix = 0;
    s_k = K;
  }
  uint32_t mask = 0;
  // bf16 logits: the low 16 bits of a key are fixed by its sign, so the top two digits already fix the threshold
  for (int pass = 3; pass >= (BF16 ? 2 : 0); --pass) {
    for (int i = tid; i < SMP_WAVES * 4 * 256; i += SMP_T) (&hist[0][0][0])[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    const int sh = 8 * pass;
    for (int i = tid; i < V; i += SMP_T) {
      const uint32_t key = f2key(smp_load<BF16>(base, i));
      if ((key & mask) == prefix) atomicAdd(&hist[w][lane & 3][(key >> sh) & 255], 1u);
    }
    __syncthreads();
    if (tid < 256) {
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < SMP_WAVES; ++q) s += (hist[q][0][tid] + hist[q][1][tid]) + (hist[q][2][tid] + hist[q][3][tid]);
      tot[tid] = s;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t k = s_k, above = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (above + tot[b] >= k) break;
        above += tot[b];
      }
      s_k = k - above;
      s_prefix = prefix | ((uint32_t)b << sh);
      s_eq = tot[b];  // after the last pass: how many elements equal the threshold key
    }
    mask |= 255u << sh;
    __syncthreads();
  }
  uint32_t thr = s_prefix;
  // (bf16: a negative value's key has its low 16 bits all ones, a positive value's all zeros)
  if (BF16 && !(thr & 0x80000000u)) thr |= 0xFFFFu;
  const uint32_t ties = s_k;  // how many elements equal to thr to keep
  // ---- 2. gather exactly K candidates: every key above the threshold, and of the keys equal to it the
  // `ties` with the lowest vocabulary indices (deterministic; when every equal key is kept no ordering is
  // needed, otherwise every wave counts the equal keys of its row chunk, then ranks them in index order)
  const bool all_ties = s_eq <= ties;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for (int i = tid; i < V; i += SMP_T) {
    const float v = smp_load<BF16>(base, i);
    const uint32_t key = f2key(v);
    if (key > thr || (all_ties && key == thr)) {
      const uint32_t slot = atomicAdd(&s_cnt, 1u);
      if (slot < (uint32_t)SMP_MAXK) {
        cval[slot] = v;
        cidx[slot] = i;
      }
    }
  }
  __syncthreads();
  if (!all_ties) {  // ordered selection of the `ties` lowest-index equal keys: wave w owns chunk w of the row
    __shared__ uint32_t tie_cnt[SMP_WAVES];
    const int C = ((V + SMP_WAVES - 1) / SMP_WAVES + 63) & ~63;
    const int c0 = w * C, c1 = min(V, c0 + C);
    uint32_t mine = 0;
    for (int i0 = c0; i0 < c1; i0 += 64) {
      const int i = i0 + lane;
      mine += __popcll(__ballot(i < c1 && f2key(smp_load<BF16>(base, i)) == thr));
    }
    if (lane == 0) tie_cnt[w] = mine;
    __syncthreads();
    uint32_t rank0 = 0;
    for (int q = 0; q < w; ++q) rank0 += tie_cnt[q];
    const uint32_t above = s_cnt;
    for (int i0 = c0; i0 < c1 && rank0 < ties; i0 += 64) {
      const int i = i0 + lane;
      const float v = i < c1 ? smp_load<BF16>(base, i) : 0.f;
      const bool eq = i < c1 && f2key(v) == thr;
      const unsigned long long bal = __ballot(eq);
      const uint32_t rank = rank0 + __popcll(bal & ((1ull << lane) - 1ull));
      if (eq && rank < ties && above + rank < (uint32_t)SMP_MAXK) {
        cval[above + rank] = v;
        cidx[above + rank] = i;
      }
      rank0 += __popcll(bal);
    }
    __syncthreads();
    if (tid == 0) s_cnt = above + ties;
  }
  __syncthreads();
  const int n = min((int)s_cnt, SMP_MAXK);
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = tid; i < P; i += SMP_T)
    if (i >= n) {
      cval[i] = -INFINITY;
      cidx[i] = -1;
    }
  __syncthreads();
  // ---- 3. bitonic sort, descending by value, ties by ascending index (a total order: the result does not
  // depend on the gather's slot order)
  for (int k2 = 2; k2 <= P; k2 <<= 1) {
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += SMP_T) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool desc = (i & k2) == 0;
          const float a = cval[i], b = cval[ixj];
          const int ia = cidx[i], ib = cidx[ixj];
          // "b ranks before a": larger value, or equal value and smaller index (padding: -inf, index -1)
          const bool b_first = b > a || (b == a && (unsigned)ib < (unsigned)ia);
          const bool a_first = a > b || (a == b && (unsigned)ia < (unsigned)ib);
          if (desc ? b_first : a_first) {
            cval[i] = b;
            cval[ixj] = a;
            const int t = cidx[i];
            cidx[i] = cidx[ixj];
            cidx[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  if (T <= 0.f || n == 1) {
    if (tid == 0) out[row] = cidx[0];
    return;
  }
  // ---- 4. probabilities, inclusive scan, nucleus cut, draw
  const float inv_t = 1.f / T, l0 = cval[0];
  const float p = tid < n ? __expf((cval[tid] - l0) * inv_t) : 0.f;
  // block inclusive scan (wave scan + wave totals)
  float x = p;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __shared__ float wsum[SMP_WAVES];
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (tid < 64) {
    float s = tid < SMP_WAVES ? wsum[tid] : 0.f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (tid < SMP_WAVES) wsum[tid] = s;
  }
  __syncthreads();
  const float incl = x + (w > 0 ? wsum[w - 1] : 0.f);
  if (tid < SMP_MAXK) scan[tid] = incl;
  __syncthreads();
  const float total = scan[n - 1];
  const float cut = topp[row] * total;
  // kept prefix length L: number of i with (mass before i) <= cut  (always >= 1)
  __shared__ int s_L;
  if (tid == 0) s_L = 0;
  __syncthreads();
  if (tid < n && incl - p <= cut) atomicAdd(&s_L, 1);
  __syncthreads();
  const int L = max(1, s_L);
  const float target = uniforms[row] * scan[L - 1];
  __shared__ int s_pick;
  if (tid == 0) s_pick = 0;
  __syncthreads();
  if (tid < L - 1 && scan[tid] <= target) atomicAdd(&s_pick, 1);
  __syncthreads();
  if (tid == 0) out[row] = cidx[min(s_pick, L - 1)];
}

void launch_sample(const void* logits, bool bf16, long ld, int B, int V, const float* temps, const int* top_k,
                   const float* top_p, const float* uniforms, int* out, hipStream_t s) {
  if (bf16) sample_kernel<true><<<B, SMP_T, 0, s>>>(logits, ld, V, temps, top_k, top_p, uniforms, out);
  else sample_kernel<false><<<B, SMP_T, 0, s>>>(logits, ld, V, temps, top_k, top_p, uniforms, out);
}

}  // namespace shai
