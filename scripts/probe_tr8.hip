// Probe of the gfx950 transposing LDS read ds_read_b64_tr_b8 (the 8-bit sibling of the
// ds_read_b64_tr_b16 the wgrad kernel uses): which LDS bytes land in which lane / byte.
// Round-3 groundwork for an fp8 weight-gradient kernel (docs/ROUND2.md, open levers).
//
//   hipcc --offload-arch=gfx950 -O2 scripts/probe_tr8.hip -o build/probe_tr8 && build/probe_tr8
//
// One wave, 512 B of LDS filled with a known pattern.  Two address patterns: lane * 8 (linear)
// and (lane % 8) * 64 + (lane / 8) * 8 (a column walk over 64-byte rows).  The byte at LDS offset
// o holds (o & 255) in pass 0 and (o >> 8) in pass 1, so each result byte names its source offset
// exactly.  Output: for each pattern and lane, the source offsets of result bytes 0..7.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef int v2i __attribute__((ext_vector_type(2)));

__global__ void probe(uint32_t* out, int pass, int pattern) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[512];
  const int lane = threadIdx.x;
  for (int i = lane; i < 512; i += 64) lds[i] = (unsigned char)(pass == 0 ? (i & 255) : (i >> 8));
  __syncthreads();
  const int off = pattern == 0 ? lane * 8 : (lane % 8) * 64 + (lane / 8) * 8;
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (__attribute__((address_space(3))) v2i*)(reinterpret_cast<uintptr_t>(lds + off)));
  out[lane * 2 + 0] = (uint32_t)r.x;
  out[lane * 2 + 1] = (uint32_t)r.y;
}

int main() {
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 128 * sizeof(uint32_t)) != hipSuccess) return 1;
  uint32_t h[2][128];
  for (int pattern = 0; pattern < 2; ++pattern) {
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, pass, pattern);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      if (hipMemcpy(h[pass], d, sizeof(h[pass]), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    }
    printf("pattern %d (%s): lane: source LDS byte offsets of result bytes 0..7\n", pattern,
           pattern == 0 ? "addr = lane*8" : "addr = (lane%8)*64 + (lane/8)*8");
    for (int lane = 0; lane < 64; ++lane) {
      printf("%2d:", lane);
      for (int b = 0; b < 8; ++b) {
        const uint32_t lo = (h[0][lane * 2 + b / 4] >> (8 * (b % 4))) & 255u;
        const uint32_t hi = (h[1][lane * 2 + b / 4] >> (8 * (b % 4))) & 255u;
        printf(" %3u", hi * 256 + lo);
      }
      printf("\n");
    }
  }
  (void)hipFree(d);
  return 0;
}
