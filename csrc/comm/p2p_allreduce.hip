// All-reduce over xGMI peer memory for tensor-parallel messages: a one-shot kernel for small,
// latency-bound ones (LLM decode: [B, 4096] bf16 after o_proj / down_proj, a few KB to ~1 MB) and a
// two-shot reduce-scatter + all-gather kernel (p2p_two_shot, below) for mid-size ones (Flux / prefill).
//
// RCCL's ring/tree all-reduce pays several link latencies per call; on a fully
// connected 8x MI355X node every GPU can instead READ every peer's buffer
// directly over its own xGMI link.  Each rank exposes one uncached device buffer
// through a HIP IPC handle (exchanged once over torch.distributed); per call:
//   1. every workgroup copies its slice of the local input into the local buffer,
//   2. cross-GPU start barrier per workgroup (system-scope flag stores into each
//      peer's signal area, spin on the local one -- epochs count calls, so the
//      flags never need resetting and the kernel is HIP-graph replay safe),
//   3. it sums the same slice from all `world` buffers (fp32 accumulate) into the
//      output, 4. an end barrier so nobody overwrites a slice a peer still reads.
// The buffer is allocated uncached (hipDeviceMallocUncached) and every read of a
// PEER's buffer is a system-coherent buffer load (sc0 sc1), so peer data is never
// served stale from a cache whatever the importer's IPC mapping type.  Spins are
// bounded: a missing peer ends the call with the error flag set -- in the device
// signal area AND in a host-mapped word the engine polls after every step without a
// device sync (shai_p2p_error) -- instead of hanging the GPU.
//
// p2p_all_gather (below) reuses the same buffers and barriers: rank-major
// concatenation of every rank's shard (vocab-parallel logits).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "kernels/common.h"  // SHAI_DASSERT (device debug flavour)

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;

struct Layout {  // signal area at the start of each rank's buffer
  // flags[phase][block][src_rank] = epoch written by src_rank
  uint32_t flags[2][kMaxBlocks][kMaxRanks];
  uint32_t epoch[kMaxBlocks];  // local per-block call counter
  uint32_t error;
  uint32_t pad[63];
};
constexpr size_t kDataOff = (sizeof(Layout) + 4095) & ~size_t(4095);

struct Peers {
  char* base[kMaxRanks];
  uint32_t* host_err;        // host-mapped (pinned) error word
  unsigned long long spin_ticks;  // barrier timeout in wall-clock ticks (constant-rate counter)
};

// cache-policy bits of a vector memory instruction (gfx94x/gfx950): sc0 = 1, nt = 2, sc1 = 16; sc0|sc1 = system
// scope -- a peer's bytes come over xGMI from its HBM, never from a (possibly stale) local cache line
constexpr int kSysCoherent = 1 | 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t peer_rsrc(const char* base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0,
                                           (int)(bytes > 0x7fffffffu ? 0x7fffffffu : bytes), 0x00020000);
}

// 16 bytes at uint4 index i of the buffer behind rsrc (i * 16 < 2 GiB)
__device__ __forceinline__ uint4 peer_load16(__amdgpu_buffer_rsrc_t r, long i) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, kSysCoherent));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void barrier_phase(const Peers& P, Layout* me, int phase, int rank, int world,
                                              uint32_t epoch) {
  const int b = blockIdx.x, t = threadIdx.x;
  if (t < world) {
    Layout* peer = reinterpret_cast<Layout*>(P.base[t]);
    __hip_atomic_store(&peer->flags[phase][b][rank], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(&me->flags[phase][b][t], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (wall_clock64() - t0 > P.spin_ticks) {
        __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (P.host_err) __hip_atomic_store(P.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// Fused output stage of a row-parallel layer on the reduced row-major [rows, ncols] bf16 message:
//   out = residual + gate[row / rows_per_gate] * (sum + bias)
// bias (per column, added once after the reduction), gate (AdaLN-Zero: one row of ncols per image, row stride
// gate_ld8 16-B groups) and residual ([rows, ncols], may be the output itself) are each optional.  16-B group i
// holds columns (8 i) % ncols .. + 7 of row i / (ncols / 8) (ncols % 8 == 0).
struct Epi {
  const uint4* bias;      // [ncols] bf16 or nullptr
  const uint4* residual;  // [rows, ncols] bf16 or nullptr
  int ncols8;             // ncols / 8
  const uint4* gate = nullptr;
  int gate_ld8 = 0;
  int rows_per_gate = 1;
  int row0 = 0;           // first message row's index in the gate's row space (a row slab of a larger output)
};

__device__ __forceinline__ void add_bf16x8(float acc[8], uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    acc[2 * e] += __uint_as_float(w[e] << 16);
    acc[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
  }
}

__device__ __forceinline__ void apply_epi(const Epi& E, long i, float acc[8]) {
  const int row = (int)i / E.ncols8, c8 = (int)i - row * E.ncols8;  // i < 2^31: the slot is <= 16 MiB
  if (E.bias) add_bf16x8(acc, E.bias[c8]);
  if (E.gate) {
    const uint4 g = E.gate[(long)((E.row0 + row) / E.rows_per_gate) * E.gate_ld8 + c8];
    const uint32_t w[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] *= __uint_as_float(w[e] << 16);
      acc[2 * e + 1] *= __uint_as_float(w[e] & 0xffff0000u);
    }
  }
  if (E.residual) add_bf16x8(acc, E.residual[i]);
}

__device__ __forceinline__ uint4 pack_bf16x8(const float acc[8]);

// STAGED: the input already sits in this rank's slot A (the row-parallel GEMM wrote its partial there), so the
// copy of step 1 is skipped; the slot is never rewritten before every peer is past this call's end barrier.
// off: byte offset of the message inside every rank's slot (a row slab of a staged output; 0 otherwise).
template <bool STAGED>
__global__ void __launch_bounds__(512) p2p_one_shot(Peers P, int rank, int world, const uint4* in,
                                                    uint4* out, long n16, Epi E, size_t off) {
  __shared__ uint32_t s_epoch;
  // debug build: rank / world within the peer table, this block's epoch slot inside the signal area
  SHAI_DASSERT(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world && blockIdx.x < (unsigned)kMaxBlocks);
  Layout* me = reinterpret_cast<Layout*>(P.base[rank]);
  if (threadIdx.x == 0) {
    const uint32_t e = me->epoch[blockIdx.x] + 1;
    me->epoch[blockIdx.x] = e;
    s_epoch = e;
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  uint4* mine = reinterpret_cast<uint4*>(P.base[rank] + kDataOff + off);
  const long stride = (long)gridDim.x * blockDim.x;
  if (!STAGED) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) mine[i] = in[i];
    __threadfence_system();
  }
  __syncthreads();
  barrier_phase(P, me, 0, rank, world, epoch);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < world; ++r) {
      const uint4 v = r == rank ? mine[i] : peer_load16(peer_rsrc(P.base[r] + kDataOff + off, n16 * 16), i);
      add_bf16x8(acc, v);
    }
    apply_epi(E, i, acc);
    out[i] = pack_bf16x8(acc);
  }
  __syncthreads();
  barrier_phase(P, me, 1, rank, world, epoch);
}

__device__ __forceinline__ uint4 pack_bf16x8(const float acc[8]) {
  uint32_t o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // round-to-nearest-even to bf16
    uint32_t lo = __float_as_uint(acc[2 * e]), hi = __float_as_uint(acc[2 * e + 1]);
    lo = (lo + 0x7fffu + ((lo >> 16) & 1u)) >> 16;
    hi = (hi + 0x7fffu + ((hi >> 16) & 1u)) >> 16;
    o[e] = lo | (hi << 16);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Two-shot (reduce-scatter + all-gather) all-reduce for mid-size messages (Flux / prefill row-parallel
// outputs, 256 KiB - 16 MiB: the default routing in parallel/comm.py).  The message is cut into `world` segments; rank r owns segment r.
//   phase 0: copy the input into the local staging slot A (only the positions this block will hand out),
//   barrier, phase 1: sum segment r over every rank's slot A (world-1 remote reads of M/world each, all xGMI
//   links busy at once) into the local slot B, barrier, phase 2: gather every segment s from rank s's slot B
//   into the output.  Per rank (world-1)/world * M crosses the links twice, vs 2 (world-1)/world * M through
//   ONE link per direction for a single ring.  Block b of every rank touches the same positions in every
//   phase, so the per-block flag barriers order all the hand-offs (no grid-wide barrier); the next call's
//   first barrier protects slot B from being overwritten while a peer still gathers it.
// STAGED as for the one-shot kernel (no phase-0 copy); the fused epilogue (bias, residual) is applied by the
// segment's owner in phase 1, so every element gets it exactly once and phase 2 gathers final values.
template <bool STAGED>
__global__ void __launch_bounds__(512) p2p_two_shot(Peers P, int rank, int world, const uint4* in, uint4* out,
                                                    long n16, size_t slot_bytes, Epi E, size_t off) {
  __shared__ uint32_t s_epoch;
  // debug build: rank / world within the peer table, this block's epoch slot inside the signal area
  SHAI_DASSERT(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world && blockIdx.x < (unsigned)kMaxBlocks);
  Layout* me = reinterpret_cast<Layout*>(P.base[rank]);
  if (threadIdx.x == 0) {
    const uint32_t e = me->epoch[blockIdx.x] + 1;
    me->epoch[blockIdx.x] = e;
    s_epoch = e;
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const long seg = (n16 + world - 1) / world;
  const long stride = (long)gridDim.x * blockDim.x;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  SHAI_DASSERT(off % 16 == 0 && off + (size_t)n16 * 16 <= slot_bytes);  // the message (slab) stays in slot A / B
  uint4* slotA = reinterpret_cast<uint4*>(P.base[rank] + kDataOff + off);
  uint4* slotB = reinterpret_cast<uint4*>(P.base[rank] + kDataOff + slot_bytes + off);
  if (!STAGED) {
    for (int s = 0; s < world; ++s) {
      const long beg = s * seg, end = min(n16, beg + seg);
      for (long i = beg + t0; i < end; i += stride) slotA[i] = in[i];
    }
    __threadfence_system();
  }
  __syncthreads();
  barrier_phase(P, me, 0, rank, world, epoch);
  {
    const long beg = rank * seg, end = min(n16, beg + seg);
    for (long i = beg + t0; i < end; i += stride) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int r = 0; r < world; ++r) {
        const int src = (rank + r) % world;  // stagger the peers so the links are loaded evenly
        const uint4 v = src == rank ? slotA[i] : peer_load16(peer_rsrc(P.base[src] + kDataOff + off, n16 * 16), i);
        add_bf16x8(acc, v);
      }
      apply_epi(E, i, acc);
      slotB[i] = pack_bf16x8(acc);
    }
  }
  __threadfence_system();
  __syncthreads();
  barrier_phase(P, me, 1, rank, world, epoch);
  for (int r = 0; r < world; ++r) {
    const int s = (rank + r) % world;
    const long beg = s * seg, end = min(n16, beg + seg);
    if (s == rank) {
      for (long i = beg + t0; i < end; i += stride) out[i] = slotB[i];
    } else {
      const __amdgpu_buffer_rsrc_t rb = peer_rsrc(P.base[s] + kDataOff + slot_bytes + off, n16 * 16);
      for (long i = beg + t0; i < end; i += stride) out[i] = peer_load16(rb, i);
    }
  }
}

// All-gather: out[r * n16 + i] = rank r's in[i] (rank-major concatenation), one shot.  Each rank stages its
// shard in slot A, start barrier, every rank reads every peer's shard over its xGMI link, end barrier (a
// peer may still be reading our slot A until then).
__global__ void __launch_bounds__(512) p2p_all_gather(Peers P, int rank, int world, const uint4* in, uint4* out,
                                                      long n16) {
  __shared__ uint32_t s_epoch;
  // debug build: rank / world within the peer table, this block's epoch slot inside the signal area
  SHAI_DASSERT(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world && blockIdx.x < (unsigned)kMaxBlocks);
  Layout* me = reinterpret_cast<Layout*>(P.base[rank]);
  if (threadIdx.x == 0) {
    const uint32_t e = me->epoch[blockIdx.x] + 1;
    me->epoch[blockIdx.x] = e;
    s_epoch = e;
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  uint4* mine = reinterpret_cast<uint4*>(P.base[rank] + kDataOff);
  const long stride = (long)gridDim.x * blockDim.x;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long i = t0; i < n16; i += stride) {
    const uint4 v = in[i];
    mine[i] = v;
    out[(long)rank * n16 + i] = v;
  }
  __threadfence_system();
  __syncthreads();
  barrier_phase(P, me, 0, rank, world, epoch);
  for (int r = 1; r < world; ++r) {
    const int s = (rank + r) % world;
    const __amdgpu_buffer_rsrc_t rb = peer_rsrc(P.base[s] + kDataOff, n16 * 16);
    for (long i = t0; i < n16; i += stride) out[(long)s * n16 + i] = peer_load16(rb, i);
  }
  __syncthreads();
  barrier_phase(P, me, 1, rank, world, epoch);
}

struct Ctx {
  int rank, world, device;
  int max_blocks;  // grid cap (identical on every rank): ranks sharing one GPU must all fit on it at once
  size_t max_bytes;
  char* local;
  uint32_t* host_err;  // pinned, mapped into the device address space (Peers::host_err)
  Peers peers;
  bool opened[kMaxRanks];
  long long launches[5];  // one-shot, two-shot, staged one-shot, staged two-shot, all-gather (host-side count)
};

}  // namespace

extern "C" {

// Returns nullptr on failure.  handle_out receives the 64-byte hipIpcMemHandle_t.
void* shai_p2p_create(int rank, int world, size_t max_bytes, char* handle_out) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return nullptr;
  Ctx* c = new Ctx();
  c->rank = rank;
  c->world = world;
  c->max_bytes = max_bytes;
  c->max_blocks = kMaxBlocks;
  (void)hipGetDevice(&c->device);
  // signal area | slot A (staging, both algorithms) | slot B (two-shot reduced segments)
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&c->local), kDataOff + 2 * max_bytes,
                            hipDeviceMallocUncached) != hipSuccess) {
    delete c;
    return nullptr;
  }
  (void)hipMemset(c->local, 0, kDataOff);
  (void)hipDeviceSynchronize();
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, c->local) != hipSuccess) {
    (void)hipFree(c->local);
    delete c;
    return nullptr;
  }
  memcpy(handle_out, &h, sizeof(h));
  memset(&c->peers, 0, sizeof(c->peers));
  c->peers.base[rank] = c->local;
  {  // barrier timeout: SHAI_P2P_TIMEOUT_S seconds (default 20) of the constant-rate wall clock
    int khz = 100000;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device);
    const char* e = getenv("SHAI_P2P_TIMEOUT_S");
    const double secs = e ? atof(e) : 20.0;
    c->peers.spin_ticks = (unsigned long long)(secs * 1000.0 * (khz > 0 ? khz : 100000));
  }
  c->host_err = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&c->host_err), sizeof(uint32_t),
                    hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    *c->host_err = 0;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, c->host_err, 0) == hipSuccess) c->peers.host_err = static_cast<uint32_t*>(dp);
  }
  return c;
}

int shai_p2p_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// Cap every kernel's grid at n workgroups (1..256); must be called identically on every rank.
void shai_p2p_set_max_blocks(void* ctx, int n) {
  Ctx* c = static_cast<Ctx*>(ctx);
  c->max_blocks = n < 1 ? 1 : (n > kMaxBlocks ? kMaxBlocks : n);
}

// handles: world consecutive 64-byte handles (own entry ignored).  0 on success.
int shai_p2p_open(void* ctx, const char* handles) {
  Ctx* c = static_cast<Ctx*>(ctx);
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, handles + (size_t)r * sizeof(h), sizeof(h));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -1 - r;
    c->peers.base[r] = static_cast<char*>(p);
    c->opened[r] = true;
  }
  return 0;
}

// bf16 sum of `bytes` (multiple of 16, <= max_bytes) from in into out (may alias) on stream.
int shai_p2p_allreduce_bf16(void* ctx, const void* in, void* out, size_t bytes, hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (bytes % 16 != 0 || bytes > c->max_bytes) return -1;
  const long n16 = (long)(bytes / 16);
  int blocks = (int)((n16 + 511) / 512);
  if (blocks > c->max_blocks) blocks = c->max_blocks;
  if (blocks < 1) blocks = 1;
  // every rank must use the same grid: it is a function of bytes only
  hipLaunchKernelGGL(p2p_one_shot<false>, dim3(blocks), dim3(512), 0, stream, c->peers, c->rank, c->world,
                     static_cast<const uint4*>(in), static_cast<uint4*>(out), n16, Epi{nullptr, nullptr, 1}, (size_t)0);
  ++c->launches[0];
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Two-shot (reduce-scatter + all-gather) bf16 sum for mid-size messages; same contract as above.
int shai_p2p_allreduce2_bf16(void* ctx, const void* in, void* out, size_t bytes, hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (bytes % 16 != 0 || bytes > c->max_bytes) return -1;
  const long n16 = (long)(bytes / 16);
  const long per_rank = (n16 + c->world - 1) / c->world;
  int blocks = (int)((per_rank + 511) / 512);
  if (blocks > c->max_blocks) blocks = c->max_blocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(p2p_two_shot<false>, dim3(blocks), dim3(512), 0, stream, c->peers, c->rank, c->world,
                     static_cast<const uint4*>(in), static_cast<uint4*>(out), n16, c->max_bytes,
                     Epi{nullptr, nullptr, 1}, (size_t)0);
  ++c->launches[1];
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// This rank's staging slot (slot A): a row-parallel GEMM writes its partial product straight into it and
// shai_p2p_allreduce_staged reduces from there (no staging copy).  Returns the device pointer; *bytes = capacity.
void* shai_p2p_staging(void* ctx, size_t* bytes) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (bytes) *bytes = c->max_bytes;
  return c->local + kDataOff;
}

// out[rows, ncols] = residual + gate[(row0 + row) / rows_per_gate] * (sum over ranks of every rank's staged
// partial + bias) for the `bytes` = rows * ncols * 2 message at byte offset `slot_off` of slot A (a row slab of a
// larger staged output: a row-parallel GEMM split into slabs reduces slab i while slab i + 1 is computed; every
// slab is its own collective, issued in the same order on every rank).  bias / residual / gate optional, gate row
// stride gate_ld elements; out may be the residual itself; bf16, fp32 accumulation.  two_shot selects
// reduce-scatter + all-gather (mid-size messages) over one-shot.  Every rank must pass the same bytes / ncols /
// slot_off / two_shot.  0 on success.
int shai_p2p_allreduce_staged_at(void* ctx, void* out, size_t bytes, int ncols, const void* bias,
                                 const void* residual, const void* gate, int gate_ld, int rows_per_gate, int row0,
                                 size_t slot_off, int two_shot, hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (bytes % 16 != 0 || slot_off % 16 != 0 || slot_off + bytes > c->max_bytes || ncols <= 0 || ncols % 8 != 0 ||
      (bytes / 2) % ncols != 0 || row0 < 0)
    return -1;
  if ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(residual) |
       reinterpret_cast<uintptr_t>(gate)) & 15)
    return -3;
  if (gate && (gate_ld % 8 != 0 || gate_ld < ncols || rows_per_gate < 1)) return -4;
  const long n16 = (long)(bytes / 16);
  Epi E{static_cast<const uint4*>(bias), static_cast<const uint4*>(residual), ncols / 8};
  E.gate = static_cast<const uint4*>(gate);
  E.gate_ld8 = gate_ld / 8;
  E.rows_per_gate = rows_per_gate;
  E.row0 = row0;
  const uint4* in = reinterpret_cast<const uint4*>(c->local + kDataOff + slot_off);
  int blocks;
  if (two_shot) {
    blocks = (int)(((n16 + c->world - 1) / c->world + 511) / 512);
  } else {
    blocks = (int)((n16 + 511) / 512);
  }
  if (blocks > c->max_blocks) blocks = c->max_blocks;
  if (blocks < 1) blocks = 1;
  if (two_shot) {
    hipLaunchKernelGGL(p2p_two_shot<true>, dim3(blocks), dim3(512), 0, stream, c->peers, c->rank, c->world, in,
                       static_cast<uint4*>(out), n16, c->max_bytes, E, slot_off);
    ++c->launches[3];
  } else {
    hipLaunchKernelGGL(p2p_one_shot<true>, dim3(blocks), dim3(512), 0, stream, c->peers, c->rank, c->world, in,
                       static_cast<uint4*>(out), n16, E, slot_off);
    ++c->launches[2];
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The whole message at the start of slot A (row0 = 0).
int shai_p2p_allreduce_staged(void* ctx, void* out, size_t bytes, int ncols, const void* bias, const void* residual,
                              const void* gate, int gate_ld, int rows_per_gate, int two_shot, hipStream_t stream) {
  return shai_p2p_allreduce_staged_at(ctx, out, bytes, ncols, bias, residual, gate, gate_ld, rows_per_gate, 0, 0,
                                      two_shot, stream);
}

// Host-side launch counts (captured launches count once): [one-shot, two-shot, staged one-shot, staged two-shot,
// all-gather].
void shai_p2p_launch_counts(void* ctx, long long* out5) {
  Ctx* c = static_cast<Ctx*>(ctx);
  for (int i = 0; i < 5; ++i) out5[i] = c->launches[i];
}

// Rank-major all-gather of `bytes` (multiple of 16, <= max_bytes) per rank: out holds world * bytes.
int shai_p2p_allgather(void* ctx, const void* in, void* out, size_t bytes, hipStream_t stream) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (bytes % 16 != 0 || bytes > c->max_bytes) return -1;
  const long n16 = (long)(bytes / 16);
  int blocks = (int)((n16 + 511) / 512);
  if (blocks > c->max_blocks) blocks = c->max_blocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(p2p_all_gather, dim3(blocks), dim3(512), 0, stream, c->peers, c->rank, c->world,
                     static_cast<const uint4*>(in), static_cast<uint4*>(out), n16);
  ++c->launches[4];
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// 1 if any spin timed out since creation (a peer did not arrive).  Reads the host-mapped word: no device
// synchronisation, cheap enough to poll after every engine step (falls back to a device read without it).
int shai_p2p_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c->host_err) return (int)__atomic_load_n(c->host_err, __ATOMIC_ACQUIRE);
  uint32_t e = 0;
  (void)hipMemcpy(&e, c->local + offsetof(Layout, error), 4, hipMemcpyDeviceToHost);
  return (int)e;
}

void shai_p2p_destroy(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return;
  for (int r = 0; r < c->world; ++r)
    if (c->opened[r]) (void)hipIpcCloseMemHandle(c->peers.base[r]);
  (void)hipFree(c->local);
  if (c->host_err) (void)hipHostFree(c->host_err);
  delete c;
}

}  // extern "C"
