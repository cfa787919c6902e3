// Fused BatchNorm-apply + activation + max-pool (NHWC) and its gather backward.
//
// ResNet's stem is conv7x7/2 -> BN -> ReLU -> maxpool3x3/2: the unfused chain
// writes the 112x112x64 post-ReLU tensor and reads it straight back (and the
// ATen NHWC max-pool backward scatters through 64-bit indices).  Here the
// forward reads the conv output once, applies the per-channel affine + act in
// registers, and writes only the pooled tensor plus a 1-byte window argmax per
// output element.  The backward is a GATHER (no atomics): every input pixel
// visits the <= ceil(k/s)^2 windows covering it and sums the output grads whose
// argmax is its tap; the result feeds the BN backward (which recomputes the
// ReLU mask from x).  8 channels (16 B) per thread.
//
// Reference parity: torchvision resnet stem (nn.MaxPool2d(3, 2, 1)) used by the
// reference's examples/img_cls/resnet.py.
#include "common.h"
#include "tbamd.h"
#include "pool_gather.h"

namespace tbamd {

namespace {

struct PoolGeom {
  int N, H, W, C, P, Q, k, s, pad;
};

template <int DT, int ACT>
__global__ __launch_bounds__(256) void bn_act_maxpool_fwd_k(const storage_t<DT>* __restrict__ x,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, float slope,
                                                            storage_t<DT>* __restrict__ y,
                                                            uint8_t* __restrict__ idx, PoolGeom g) {
  const int CV = g.C / 8;
  const int64_t total = (int64_t)g.N * g.P * g.Q * CV;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  int64_t pix = t / CV;
  const int q = (int)(pix % g.Q);
  pix /= g.Q;
  const int p = (int)(pix % g.P);
  const int n = (int)(pix / g.P);
  const int c0 = cv * 8;
  float sc[8], sf[8], best[8];
  int arg[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[c0 + i];
    sf[i] = shift[c0 + i];
    best[i] = -INFINITY;
    arg[i] = 0;
  }
  const int h0 = p * g.s - g.pad, w0 = q * g.s - g.pad;
  for (int r = 0; r < g.k; ++r) {
    const int h = h0 + r;
    if ((unsigned)h >= (unsigned)g.H) continue;
    for (int u = 0; u < g.k; ++u) {
      const int w = w0 + u;
      if ((unsigned)w >= (unsigned)g.W) continue;
      float v[8];
      load_vec<DT, 8>(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + c0, v);
      const int tap = r * g.k + u;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        // same fma as the BN apply kernels, so the backward's ReLU mask matches
        const float z = act_fwd<ACT>(__builtin_fmaf(v[i], sc[i], sf[i]), slope);
        if (z > best[i]) {
          best[i] = z;
          arg[i] = tap;
        }
      }
    }
  }
  store_vec<DT, 8>(y + t * 8, best);
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    lo |= (uint32_t)arg[i] << (8 * i);
    hi |= (uint32_t)arg[i + 4] << (8 * i);
  }
  *reinterpret_cast<uint2*>(idx + t * 8) = make_uint2(lo, hi);
}

template <int DT>
__global__ __launch_bounds__(256) void maxpool_bwd_gather_k(const storage_t<DT>* __restrict__ dy,
                                                            const uint8_t* __restrict__ idx,
                                                            storage_t<DT>* __restrict__ dx, PoolGeom g) {
  const int CV = g.C / 8;
  const int64_t total = (int64_t)g.N * g.H * g.W * CV;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  int64_t pix = t / CV;
  const int w = (int)(pix % g.W);
  pix /= g.W;
  const int h = (int)(pix % g.H);
  const int n = (int)(pix / g.H);
  const PoolSrc ps{dy, idx, g.H, g.W, g.C, g.P, g.Q, g.k, g.s, g.pad};
  float acc[8];
  pool_gather8<DT>(ps, n, h, w, cv * 8, acc);
  store_vec<DT, 8>(dx + t * 8, acc);
}

}  // namespace

void bn_act_maxpool_fwd(int dt, const void* x, const float* scale, const float* shift, int act, float slope, int N,
                        int H, int W, int C, int k, int s, int pad, void* y, uint8_t* idx, hipStream_t st) {
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  PoolGeom g{N, H, W, C, P, Q, k, s, pad};
  const int64_t total = (int64_t)N * P * Q * (C / 8);
  if (total == 0) return;
  TBAMD_DISPATCH_DT(dt, DT, {
    using T = storage_t<DT>;
    TBAMD_DISPATCH_ACT(act, ACT, {
      bn_act_maxpool_fwd_k<DT, ACT><<<cdiv(total, 256), 256, 0, st>>>((const T*)x, scale, shift, slope, (T*)y, idx,
                                                                     g);
    });
  });
}

void maxpool_bwd(int dt, const void* dy, const uint8_t* idx, int N, int H, int W, int C, int k, int s, int pad,
                 void* dx, hipStream_t st) {
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  PoolGeom g{N, H, W, C, P, Q, k, s, pad};
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (total == 0) return;
  TBAMD_DISPATCH_DT(dt, DT, {
    using T = storage_t<DT>;
    maxpool_bwd_gather_k<DT><<<cdiv(total, 256), 256, 0, st>>>((const T*)dy, idx, (T*)dx, g);
  });
}

// ---------------------------------------------------------------- global average pool
// Classifier head pooling (reference resnet.py:111-112 AdaptiveAvgPool2d(1) -> flatten ->
// Linear) on NHWC activations: one thread per (image, 8 channels), 16-B
// loads down the HW positions, f32 sums -> y [N][C].  The backward writes the broadcast
// dy / HW straight in NHWC order with 16-B stores (no expand + layout copy).
template <int DT>
__global__ __launch_bounds__(256) void gap_fwd_k(const storage_t<DT>* __restrict__ x, int N, int HW, int C,
                                                 storage_t<DT>* __restrict__ y) {
  const int C8 = C / 8;
  const int64_t total = (int64_t)N * C8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int n = (int)(i / C8), c = (int)(i % C8) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const storage_t<DT>* p = x + (int64_t)n * HW * C + c;
    for (int h = 0; h < HW; ++h) {
      float v[8];
      Vec8<DT>::load(p + (int64_t)h * C, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
    const float inv = 1.f / HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    Vec8<DT>::store(y + (int64_t)n * C + c, acc);
  }
}

template <int DT>
__global__ __launch_bounds__(256) void gap_bwd_k(const storage_t<DT>* __restrict__ dy, int N, int HW, int C,
                                                 storage_t<DT>* __restrict__ dx) {
  const int C8 = C / 8;
  const int64_t total = (int64_t)N * HW * C8;
  const float inv = 1.f / HW;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C8) * 8;
    const int64_t pix = i / C8;
    const int n = (int)(pix / HW);
    float v[8];
    Vec8<DT>::load(dy + (int64_t)n * C + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= inv;
    Vec8<DT>::store(dx + pix * C + c, v);
  }
}

void global_avgpool_fwd(int dt, const void* x, int N, int HW, int C, void* y, hipStream_t st) {
  const int64_t total = (int64_t)N * (C / 8);
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  TBAMD_DISPATCH_DT(dt, DT, {
    gap_fwd_k<DT><<<(int)g, 256, 0, st>>>((const storage_t<DT>*)x, N, HW, C, (storage_t<DT>*)y);
  });
}

void global_avgpool_bwd(int dt, const void* dy, int N, int HW, int C, void* dx, hipStream_t st) {
  const int64_t total = (int64_t)N * HW * (C / 8);
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  TBAMD_DISPATCH_DT(dt, DT, {
    gap_bwd_k<DT><<<(int)g, 256, 0, st>>>((const storage_t<DT>*)dy, N, HW, C, (storage_t<DT>*)dx);
  });
}

}  // namespace tbamd
