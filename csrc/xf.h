// BN + ReLU transform applied to a conv's activation operand in LDS (csrc/conv.hip forward,
// csrc/conv_wgrad.hip weight gradient): the BN output never exists in memory.
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"
#include "tbamd.h"

namespace tbamd {

// BatchNorm + ReLU applied to the B (activation) operand as it lands in LDS: x -> max(x * scale[c]
// + shift[c], 0) in place, by the lane that staged the 16-B chunk, between its DMA wait and the
// barrier that publishes the tile; zero-page chunks (padded taps, pixels past the end) stay zero.
// The BN output is then never written: its consumer conv reads the BN input (bn1 -> conv2,
// bn2 -> conv3 of a bottleneck; VERDICT r3 item 1 "fold BN-apply into the conv operand read").
struct XfArgs {
  const float* scale;
  const float* shift;
};

// 8 bf16 values (one 16-B LDS chunk) -> max(v * sc + sh, 0), the arithmetic of norm_bn.hip bn_apply_k
__device__ __forceinline__ uint4 xf_chunk(uint4 v, const float (&sc)[8], const float (&sh)[8]) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = fmaxf(__builtin_fmaf(bf2f((uint16_t)(w[e] & 0xffff)), sc[2 * e], sh[2 * e]), 0.f);
    const float hi = fmaxf(__builtin_fmaf(bf2f((uint16_t)(w[e] >> 16)), sc[2 * e + 1], sh[2 * e + 1]), 0.f);
    w[e] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void xf_load(const XfArgs& xf, int c0, float (&sc)[8], float (&sh)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(xf.scale + c0);
  const float4 b = *reinterpret_cast<const float4*>(xf.scale + c0 + 4);
  const float4 c = *reinterpret_cast<const float4*>(xf.shift + c0);
  const float4 d = *reinterpret_cast<const float4*>(xf.shift + c0 + 4);
  sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
  sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w; sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
}

// the tiled forward keeps the coefficients of all input channels in LDS (C <= kXfMaxC, tbamd.h):
// scale at [0, kXfMaxC), shift at [kXfMaxC, 2 kXfMaxC) floats

__device__ __forceinline__ void xf_stage(const XfArgs& xf, int C, uint4* dst, int tid) {
  float4* d = reinterpret_cast<float4*>(dst);
  for (int i = tid; i < C / 4; i += 256) {
    d[i] = reinterpret_cast<const float4*>(xf.scale)[i];
    d[kXfMaxC / 4 + i] = reinterpret_cast<const float4*>(xf.shift)[i];
  }
}

__device__ __forceinline__ void xf_lds(const uint4* src, int c0, float (&sc)[8], float (&sh)[8]) {
  const float4* s = reinterpret_cast<const float4*>(src);
  const float4 a = s[c0 / 4], b = s[c0 / 4 + 1];
  const float4 c = s[kXfMaxC / 4 + c0 / 4], d = s[kXfMaxC / 4 + c0 / 4 + 1];
  sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
  sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w; sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
}

}  // namespace tbamd
