// Max-pool backward as a GATHER, shared by pool.hip (maxpool_bwd_gather_k) and the fused
// pool + BatchNorm backward of norm_bn.hip (bn_bwd_partial_k / bn_bwd_apply_k with POOL): the
// gradient reaching input pixel (n, h, w), channels c0..c0+7, is the sum of the pooled gradients
// of the <= ceil(k/s)^2 windows covering it whose 1-byte argmax is this tap.  Fused into the BN
// backward, the full-resolution pool-input gradient (112x112x64 per image for the ResNet stem)
// is never written or read back.
#pragma once
#include "common.h"

namespace tbamd {

struct PoolSrc {
  const void* dy;      // pooled gradient [N][P][Q][C]
  const uint8_t* idx;  // window argmax (tap r*k + u) per pooled element
  int H, W, C, P, Q, k, s, pad;
};

template <int DT>
__device__ __forceinline__ void pool_gather8(const PoolSrc& g, int n, int h, int w, int c0, float acc[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  // windows p with p*s - pad <= h <= p*s - pad + k - 1
  const int hp = h + g.pad, wp = w + g.pad;
  const int p_lo = hp - (g.k - 1) <= 0 ? 0 : (hp - (g.k - 1) + g.s - 1) / g.s;
  const int p_hi = min(hp / g.s, g.P - 1);
  const int q_lo = wp - (g.k - 1) <= 0 ? 0 : (wp - (g.k - 1) + g.s - 1) / g.s;
  const int q_hi = min(wp / g.s, g.Q - 1);
  const storage_t<DT>* dy = (const storage_t<DT>*)g.dy;
  const int64_t nb = (int64_t)n * g.P;
  if (g.k <= 2 * g.s) {
    // at most 2 x 2 windows (the 3x3/2 stem pool): all 4 argmax + gradient loads issued before
    // any is used (clamped addresses for the missing windows, masked out below)
    uint2 iv[4];
    float v[4][8];
    int tap[4];
    const int pc = min(p_lo, g.P - 1), qc = min(q_lo, g.Q - 1);  // (uncovered trailing pixels: p_lo = P)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p_lo + (j >> 1), q = q_lo + (j & 1);
      const bool ok = p <= p_hi && q <= q_hi;
      tap[j] = ok ? (hp - p * g.s) * g.k + (wp - q * g.s) : -1;
      const int64_t o = ((nb + (ok ? p : pc)) * g.Q + (ok ? q : qc)) * g.C + c0;
      iv[j] = *reinterpret_cast<const uint2*>(g.idx + o);
      load_vec<DT, 8>(dy + o, v[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t a = ((i < 4 ? iv[j].x : iv[j].y) >> (8 * (i & 3))) & 0xffu;
        if ((int)a == tap[j]) acc[i] += v[j][i];
      }
    return;
  }
  for (int p = p_lo; p <= p_hi; ++p) {
    for (int q = q_lo; q <= q_hi; ++q) {
      const int tap = (hp - p * g.s) * g.k + (wp - q * g.s);
      const int64_t o = ((nb + p) * g.Q + q) * g.C + c0;
      const uint2 iv = *reinterpret_cast<const uint2*>(g.idx + o);
      float v[8];
      load_vec<DT, 8>(dy + o, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t a = ((i < 4 ? iv.x : iv.y) >> (8 * (i & 3))) & 0xffu;
        if ((int)a == tap) acc[i] += v[i];
      }
    }
  }
}

// the pool-input gradient of BN row r (= (n * H + h) * W + w), 8 channels from c0
template <int DT>
__device__ __forceinline__ void pool_gather_row(const PoolSrc& g, int64_t r, int c0, float acc[8]) {
  const uint32_t ur = (uint32_t)r;
  const uint32_t t = ur / (uint32_t)g.W;
  const int w = (int)(ur - t * (uint32_t)g.W);
  const uint32_t n = t / (uint32_t)g.H;
  const int h = (int)(t - n * (uint32_t)g.H);
  pool_gather8<DT>(g, (int)n, h, w, c0, acc);
}

}  // namespace tbamd
