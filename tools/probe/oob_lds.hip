// Probe: what an out-of-range raw-buffer LDS-DMA load leaves in LDS (zero, or untouched),
// and whether soffset takes part in the range check. Prints one line per case.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void_t;
__global__ void k(const char* x, unsigned* y, int nbytes, unsigned vo_bad, int so) {
  __shared__ __attribute__((aligned(16))) unsigned sm[4 * 256];
  for (int i = threadIdx.x; i < 4 * 256; i += 64) sm[i] = 0xDEADBEEFu;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, nbytes, 0x00020000);
  const unsigned lane = threadIdx.x;
  // case 0: valid offsets; case 1: lane-odd voffset out of range; case 2: valid voffset + soffset past the end;
  // case 3: voffset 0x80000000 on all lanes.
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(sm + 0 * 256), 16, lane * 16, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(sm + 1 * 256), 16, (lane & 1) ? vo_bad : lane * 16, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(sm + 2 * 256), 16, lane * 16, so, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(sm + 3 * 256), 16, 0x80000000u, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * 256; i += 64) y[i] = sm[i];
}
int main() {
  const int n = 1024;   // 64 lanes x 16 B
  char* x; unsigned* y;
  hipMalloc(&x, 1 << 20); hipMalloc(&y, 4 * 256 * 4);
  unsigned h[1 << 18];
  for (int i = 0; i < (1 << 18); ++i) h[i] = 0x11110000u + i;
  hipMemcpy(x, h, 1 << 20, hipMemcpyHostToDevice);
  k<<<1, 64>>>(x, y, n, 0x80000000u, 512);
  unsigned o[4 * 256];
  if (hipMemcpy(o, y, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess) { printf("fail\n"); return 1; }
  for (int c = 0; c < 4; ++c) {
    int zero = 0, dead = 0, good = 0, other = 0;
    for (int i = 0; i < 256; ++i) {
      const unsigned v = o[c * 256 + i];
      if (v == 0) ++zero; else if (v == 0xDEADBEEFu) ++dead; else if (v == 0x11110000u + i) ++good; else ++other;
    }
    printf("case %d: zero %d untouched %d in-range-data %d other %d (first words %08x %08x %08x %08x | lane1 %08x)\n", c, zero, dead, good, other,
           o[c * 256], o[c * 256 + 1], o[c * 256 + 2], o[c * 256 + 3], o[c * 256 + 4]);
  }
  return 0;
}
