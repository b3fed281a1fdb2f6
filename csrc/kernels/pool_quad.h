// Max-pool (3x3 / s2 / p1) gradient gather in quad form, shared by the stem's fused BN/pool
// backward passes (bn_act.hip) and the fused stem weight gradient (stem.hip).
#pragma once
#include "common.h"

namespace pdt {

// Quad form of the max-pool gradient gather: input pixels (2a+dh, 2b+dw) of quad (n, a, b) are
// covered only by the pooled windows W00 = (a, b), W01 = (a, b+1), W10 = (a+1, b), W11 = (a+1, b+1),
// at fixed window positions: (0,0) <- W00@4; (0,1) <- W00@5 + W01@3; (1,0) <- W00@7 + W10@1;
// (1,1) <- W00@8 + W01@6 + W10@2 + W11@0.  Four (argmax, gradient) loads serve four pixels,
// branch-free; windows past the pooled edge get argmax 0xff (never matches).  Quads and pooled
// outputs coincide one to one (Ho = ceil(H/2) for k3/s2/p1).
struct PoolQuad { f8 g[4]; };  // g[dh*2 + dw]

// combine step of the gather on already-loaded (argmax, gradient) pairs of the four windows
__device__ __forceinline__ PoolQuad pool_grad_quad_regs(const uint2 (&id)[4], const f8 (&gw)[4]) {
  PoolQuad q;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t s[4];
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) s[wi] = ((j < 4 ? id[wi].x : id[wi].y) >> (8 * (j & 3))) & 0xffu;
    const float g00 = gw[0].v[j], g01 = gw[1].v[j], g10 = gw[2].v[j], g11 = gw[3].v[j];
    q.g[0].v[j] = s[0] == 4u ? g00 : 0.f;
    q.g[1].v[j] = (s[0] == 5u ? g00 : 0.f) + (s[1] == 3u ? g01 : 0.f);
    q.g[2].v[j] = (s[0] == 7u ? g00 : 0.f) + (s[2] == 1u ? g10 : 0.f);
    q.g[3].v[j] = ((s[0] == 8u ? g00 : 0.f) + (s[1] == 6u ? g01 : 0.f)) +
                  ((s[2] == 2u ? g10 : 0.f) + (s[3] == 0u ? g11 : 0.f));
  }
  return q;
}

__device__ __forceinline__ PoolQuad pool_grad_quad(const uint4* __restrict__ dp, const uint2* __restrict__ idx,
                                                   int n, int a, int b, int c8, int C8, int Ho, int Wo) {
  uint2 id[4];
  f8 gw[4];
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    const int ho = a + (wi >> 1), wo = b + (wi & 1);
    if (ho < Ho && wo < Wo) {
      const int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * C8 + c8;
      id[wi] = idx[o];
      gw[wi] = unpack8(dp[o]);
    } else {
      id[wi] = make_uint2(0xffffffffu, 0xffffffffu);
#pragma unroll
      for (int j = 0; j < 8; ++j) gw[wi].v[j] = 0.f;
    }
  }
  return pool_grad_quad_regs(id, gw);
}

// (n, a, b) of quad / pooled-output index qd (32-bit math; the host bounds the sizes)
__device__ __forceinline__ void quad_coords(uint32_t qd, int Ho, int Wo, int& n, int& a, int& b) {
  const uint32_t q2 = qd / (uint32_t)Wo;
  b = (int)(qd - q2 * (uint32_t)Wo);
  const uint32_t nn = q2 / (uint32_t)Ho;
  a = (int)(q2 - nn * (uint32_t)Ho);
  n = (int)nn;
}

}  // namespace pdt
