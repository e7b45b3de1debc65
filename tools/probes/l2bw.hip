// Probe: per-CU fill rate from L2 (or HBM) into LDS by LDS-DMA, and into VGPRs by global loads,
// as a function of waves per CU and loads in flight per wave. Every block streams its own slice
// of a buffer (footprint F bytes, re-read R times); the time is one launch over 256 x BPC blocks.
// Output: one line per case, GB/s chip-wide and per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __attribute__((address_space(3))) void lds_void_t;

template <int DEPTH>
__global__ void dma_k(const char* x, int slice, int reps, unsigned* sink) {
  __shared__ __attribute__((aligned(1024))) char sm[64 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const char* base = x + (size_t)blockIdx.x * slice;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, slice, 0x00020000);
  const int per = slice / 1024;                 // 1 KB pieces in the slice
  char* dst = sm + (wave % 16) * 4096;
  int p = wave;
  for (int it = 0; it < reps; ++it) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(dst + (d & 3) * 1024), 16, p * 1024 + lane * 16, 0, 0, 0);
      p += nw;
      if (p >= per) p -= per;
    }
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(DEPTH) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0 && sm[0] == 123) sink[0] = 1;
}

template <int DEPTH>
__global__ void vgpr_k(const char* x, int slice, int reps, unsigned* sink) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const char* base = x + (size_t)blockIdx.x * slice;
  const int per = slice / 1024;
  int p = wave;
  u4 acc = {0, 0, 0, 0};
  for (int it = 0; it < reps; ++it) {
    u4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      v[d] = *reinterpret_cast<const u4*>(base + (size_t)p * 1024 + lane * 16);
      p += nw;
      if (p >= per) p -= per;
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) acc ^= v[d];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = acc[0];
}

int main(int argc, char** argv) {
  char* x; unsigned* sink;
  const size_t big = (size_t)512 << 20;
  hipMalloc(&x, big); hipMalloc(&sink, 64);
  hipMemset(x, 1, big);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  struct Case { const char* name; int kind, depth, threads, bpc; size_t slice; };
  // slice per block: 8 KB x 256 x bpc blocks = 2-4 MB footprint (L2-resident after the first pass);
  // 1 MB slices = 256 MB+ footprint (HBM / Infinity Cache).
  for (size_t slice : {(size_t)8 << 10, (size_t)64 << 10, (size_t)1 << 20}) {
    for (int kind = 0; kind < 2; ++kind)
      for (int threads : {256, 512})
        for (int bpc : {1, 2})
          for (int depth : {4, 8, 16}) {
            const int nb = 256 * bpc;
            if ((size_t)nb * slice > big) continue;
            const long bytes_per_rep = (long)nb * (threads / 64) * depth * 1024;
            const int reps = (int)(((size_t)2 << 30) / bytes_per_rep);
            auto launch = [&]() {
              if (kind == 0) {
                if (depth == 4) dma_k<4><<<nb, threads>>>(x, (int)slice, reps, sink);
                else if (depth == 8) dma_k<8><<<nb, threads>>>(x, (int)slice, reps, sink);
                else dma_k<16><<<nb, threads>>>(x, (int)slice, reps, sink);
              } else {
                if (depth == 4) vgpr_k<4><<<nb, threads>>>(x, (int)slice, reps, sink);
                else if (depth == 8) vgpr_k<8><<<nb, threads>>>(x, (int)slice, reps, sink);
                else vgpr_k<16><<<nb, threads>>>(x, (int)slice, reps, sink);
              }
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double gb = (double)bytes_per_rep * reps / 1e9;
            printf("%-4s slice %7zu KB  thr %3d  blk/CU %d  depth %2d : %8.1f GB/s chip  %6.1f GB/s per CU  (%.2f ms)\n",
                   kind ? "vgpr" : "dma", slice >> 10, threads, bpc, depth, gb / (ms * 1e-3), gb / (ms * 1e-3) / 256, ms);
          }
  }
  return 0;
}
