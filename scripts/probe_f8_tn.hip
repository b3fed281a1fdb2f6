// Weight-gradient-shaped fp8 MFMA fragment built with ds_read_b64_tr_b8 (profiles/r2_tr_b8_probe.md):
// D[16 kout][16 chan] = sum over 128 pixels of dy[p][kout] (e5m2) * x[p][chan] (e4m3), both tiles
// stored in LDS row-major by pixel (16 bytes per pixel row), on ONE
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales.  Checked against a host fp32 reference.
// Round-3 groundwork for an fp8 wgrad kernel (docs/ROUND2.md).
//
//   hipcc --offload-arch=gfx950 -O2 scripts/probe_f8_tn.hip -o build/probe_f8_tn && build/probe_f8_tn
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// operand fragment of lane l: 32 k-bytes (pixels 32*(l>>4) .. +31) of column l & 15, as four
// transposing reads; in read r, lane 2k'+h of its 16-lane group points at pixel row
// 32*(l>>4) + 8r + k', bytes 8h .. 8h+7
__device__ v8i frag_tr8(const unsigned char* tile, int lane) {
  const int g = lane >> 4, i = lane & 15, kk = i >> 1, h = i & 1;
  v8i f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const unsigned char* p = tile + (32 * g + 8 * r + kk) * 16 + 8 * h;
    v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
        (__attribute__((address_space(3))) v2i*)(reinterpret_cast<uintptr_t>(p)));
    f[2 * r] = v.x;
    f[2 * r + 1] = v.y;
  }
  return f;
}

__global__ void f8_tn(const unsigned char* dy, const unsigned char* x, float* d) {
  __shared__ __attribute__((aligned(16))) unsigned char sdy[128 * 16], sx[128 * 16];
  const int lane = threadIdx.x;
  for (int i = lane; i < 128 * 16; i += 64) { sdy[i] = dy[i]; sx[i] = x[i]; }
  __syncthreads();
  const v8i a = frag_tr8(sdy, lane);  // rows of D: kout
  const v8i b = frag_tr8(sx, lane);   // columns of D: channels
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  // A in e5m2 (cbsz 1), B in e4m3 (blgp 0), unit E8M0 scales (the encoding tests/test_fp8_gpu.py pins)
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 1, 0, 0, 0, 0, 0);
#pragma unroll
  for (int e = 0; e < 4; ++e) d[(4 * (lane >> 4) + e) * 16 + (lane & 15)] = acc[e];
}

static float dec(unsigned char v, int ebits) {  // OCP e4m3fn (ebits 4) / e5m2 (ebits 5), finite
  const int mbits = 7 - ebits, bias = ebits == 4 ? 7 : 15;
  const int s = v >> 7, e = (v >> mbits) & ((1 << ebits) - 1), m = v & ((1 << mbits) - 1);
  const float f = e == 0 ? std::ldexp((float)m, 1 - bias - mbits)
                         : std::ldexp(1.f + (float)m / (float)(1 << mbits), e - bias);
  return s ? -f : f;
}

static unsigned char rnd(int ebits) {  // finite, modest magnitude
  for (;;) {
    const unsigned char v = (unsigned char)(std::rand() & 255);
    const int e = (v >> (7 - ebits)) & ((1 << ebits) - 1);
    if (ebits == 4 && (v & 0x7f) == 0x7f) continue;            // e4m3fn NaN
    if (ebits == 5 && e == 31) continue;                        // e5m2 inf / NaN
    if (std::fabs(dec(v, ebits)) > 64.f) continue;
    return v;
  }
}

int main() {
  std::srand(7);
  unsigned char hdy[128 * 16], hx[128 * 16];
  for (int i = 0; i < 128 * 16; ++i) { hdy[i] = rnd(5); hx[i] = rnd(4); }
  unsigned char *ddy, *dx;
  float* dd;
  if (hipMalloc(&ddy, sizeof(hdy)) || hipMalloc(&dx, sizeof(hx)) || hipMalloc(&dd, 256 * sizeof(float))) return 1;
  if (hipMemcpy(ddy, hdy, sizeof(hdy), hipMemcpyHostToDevice) || hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice))
    return 2;
  hipLaunchKernelGGL(f8_tn, dim3(1), dim3(64), 0, 0, ddy, dx, dd);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  float hd[256];
  if (hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost)) return 4;
  double maxrel = 0.0, ref_norm = 0.0, err_norm = 0.0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double ref = 0.0;
      for (int p = 0; p < 128; ++p) ref += (double)dec(hdy[p * 16 + r], 5) * (double)dec(hx[p * 16 + c], 4);
      const double err = std::fabs(hd[r * 16 + c] - ref);
      ref_norm += ref * ref;
      err_norm += err * err;
      maxrel = std::fmax(maxrel, err / (std::fabs(ref) + 1e-3));
    }
  const double rel = std::sqrt(err_norm / (ref_norm + 1e-30));
  // a wrong lane / byte layout gives rel_l2 ~ 1; fp32 accumulation of 128 exact products of up
  // to ~3e4 against a double reference leaves ~1e-5..1e-4
  printf("fp8 TN fragment via ds_read_b64_tr_b8 + mfma_scale 16x16x128: rel_l2 %.3e max_rel %.3e -> %s\n",
         rel, maxrel, rel < 1e-3 ? "PASS" : "FAIL");
  printf("D[0][0..3] = %g %g %g %g\n", hd[0], hd[1], hd[2], hd[3]);
  (void)hipFree(ddy); (void)hipFree(dx); (void)hipFree(dd);
  return rel < 1e-3 ? 0 : 5;
}
