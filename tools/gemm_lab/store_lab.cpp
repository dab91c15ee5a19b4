// Store-path lab: bytes/s of 16-B-per-lane global stores by the shape one wave-instruction covers (a GEMM epilogue
// writes 16 rows x 64 B per instruction; a staged epilogue could write whole 128-B lines or 1 KB contiguous).
//   hipcc --offload-arch=gfx950 -O3 tools/gemm_lab/store_lab.cpp -o tools/gemm_lab/bin/store_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// MODE 0: 16 rows x 64 B (lane: row = lane & 15, 16 B at (lane >> 4) * 16), row stride ld bytes
// MODE 1: 8 rows x 128 B (row = lane >> 3, 16 B at (lane & 7) * 16)
// MODE 2: 1 KB contiguous (lane * 16)
// MODE 3: 4 rows x 256 B
template <int MODE, bool BUF>
__global__ void __launch_bounds__(256) st_kernel(char* out, long ld, int iters, long bytes) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long wave = (long)blockIdx.x * (blockDim.x >> 6) + w;
  const long nwaves = (long)gridDim.x * (blockDim.x >> 6);
  uint4 v = make_uint4(lane, w, blockIdx.x, 7);
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
  for (int it = 0; it < iters; ++it) {
    const long blk = wave + nwaves * it;  // one 1 KB block per instruction
    long off;
    if (MODE == 0) off = (blk / 10) * 16 * ld + (blk % 10) * 64 + (lane & 15) * ld + (lane >> 4) * 16;
    else if (MODE == 1) off = (blk / 5) * 8 * ld + (blk % 5) * 128 + (lane >> 3) * ld + (lane & 7) * 16;
    else if (MODE == 2) off = blk * 1024 + lane * 16;
    else off = (blk / 2) * 4 * ld + (blk % 2) * 256 + (lane >> 4) * ld + (lane & 15) * 16;
    off %= bytes;
    if (BUF) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, (int)off, 0, 0);
    else *reinterpret_cast<uint4*>(out + off) = v;
    v.w += 1;
  }
}

int main() {
  const long ld = 640;  // bytes per row (320 bf16 columns)
  const long bytes = 1L << 30;
  char* out;
  CK(hipMalloc(&out, bytes + 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"16rows x 64B", "8rows x 128B", "1KB contiguous", "4rows x 256B"};
  for (int wpc : {4, 8}) {
    for (int mode = 0; mode < 4; ++mode) {
      for (int buf = 0; buf < 2; ++buf) {
        const int blocks = 256, threads = 64 * wpc;
        const int iters = (int)((bytes / 1024) / (blocks * wpc));
        auto run = [&]() {
          switch (mode * 2 + buf) {
            case 0: st_kernel<0, false><<<blocks, threads>>>(out, ld, iters, bytes); break;
            case 1: st_kernel<0, true><<<blocks, threads>>>(out, ld, iters, bytes); break;
            case 2: st_kernel<1, false><<<blocks, threads>>>(out, ld, iters, bytes); break;
            case 3: st_kernel<1, true><<<blocks, threads>>>(out, ld, iters, bytes); break;
            case 4: st_kernel<2, false><<<blocks, threads>>>(out, ld, iters, bytes); break;
            case 5: st_kernel<2, true><<<blocks, threads>>>(out, ld, iters, bytes); break;
            case 6: st_kernel<3, false><<<blocks, threads>>>(out, ld, iters, bytes); break;
            default: st_kernel<3, true><<<blocks, threads>>>(out, ld, iters, bytes); break;
          }
        };
        run();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
          CK(hipEventRecord(e0));
          run();
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        printf("waves/CU %d  %-16s %s  %7.2f TB/s\n", wpc, names[mode], buf ? "buffer" : "global", bytes / (best * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
