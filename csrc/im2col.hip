// Explicit im2col / col2im for the conv shapes the implicit-GEMM kernels do not cover well:
// 3-channel image convs with 9x9 / 4x4 windows (StyleNet input layer, DCGAN discriminator
// input and generator output) and big-channel convs over a handful of pixels (VGG-19 at batch 1,
// 512 channels at 16x16 / 32x32).  The product then runs on the native GEMM engine
// (csrc/gemm.hip / gemm8.hip), so these layers no longer fall back to MIOpen (reference: the
// cuDNN calls behind StyleNet / VGG / DCGAN convs).
//
//   im2col: col[m][k], m = (n, p, q) output pixel, k = (r, s, c) tap-major, row length KP
//           (RSC rounded up to 8, zero tail) -- the GEMM's K operand layout.  The input is read
//           through the virtual tensor pad(upsample_nearest(x, up), pad, zero | reflect), so the
//           StyleNet / AdaIN reflect-pad + upsample chains need no materialised intermediate.
//   col2im: dx[n][h][w][c] = sum over the taps (r, s) whose window position lands on (h, w) of
//           col[(n, p, q)][(r, s, c)] (+ bias[c]) -- a GATHER per output element (no atomics,
//           deterministic): the input gradient of a conv, and the forward of a transposed conv.
#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

struct ColGeom {
  int N, H, W, C;  // source tensor (NHWC)
  int R, S, P, Q;  // window and output grid
  int st, pad, upsh, reflect, KP;
};

__device__ __forceinline__ int virt(int v, int n, bool reflect) {
  if (reflect) return v < 0 ? -v : (v >= n ? 2 * n - 2 - v : v);
  return v;
}

__global__ __launch_bounds__(256) void im2col_k(const uint16_t* __restrict__ x, uint16_t* __restrict__ col,
                                                ColGeom g) {
  const int RSC = g.R * g.S * g.C;
  const int kch = g.KP / 8;
  const int64_t total = (int64_t)g.N * g.P * g.Q * kch;
  const int Hv = g.H << g.upsh, Wv = g.W << g.upsh;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / kch;
    const int k0 = (int)(e % kch) * 8;
    const int q = (int)(m % g.Q);
    const int64_t t = m / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    uint16_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + i;
      uint16_t o = 0;
      if (k < RSC) {
        const int c = k % g.C, rs = k / g.C;
        const int r = rs / g.S, s = rs % g.S;
        const int vh = virt(p * g.st - g.pad + r, Hv, g.reflect), vw = virt(q * g.st - g.pad + s, Wv, g.reflect);
        if ((unsigned)vh < (unsigned)Hv && (unsigned)vw < (unsigned)Wv) {
          const int64_t src = (((int64_t)n * g.H + (vh >> g.upsh)) * g.W + (vw >> g.upsh)) * g.C + c;
          if (TB_BOUNDS_OK(src < (int64_t)g.N * g.H * g.W * g.C, kBndAnySrc)) o = x[src];
        }
      }
      v[i] = o;
    }
    uint4 w;
    w.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
    w.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
    w.z = (uint32_t)v[4] | ((uint32_t)v[5] << 16);
    w.w = (uint32_t)v[6] | ((uint32_t)v[7] << 16);
    *reinterpret_cast<uint4*>(col + m * g.KP + k0) = w;
  }
}

// dx (the conv INPUT grid, H x W x C) from col over the output grid P x Q; zero padding, no upsampling
__global__ __launch_bounds__(256) void col2im_k(const uint16_t* __restrict__ col, uint16_t* __restrict__ dx,
                                                const uint16_t* __restrict__ bias, ColGeom g) {
  const int64_t total = (int64_t)g.N * g.H * g.W * g.C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % g.C);
    int64_t t = e / g.C;
    const int w = (int)(t % g.W);
    t /= g.W;
    const int h = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc = bias ? bf2f(bias[c]) : 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hp = h + g.pad - r;
      if (hp < 0 || hp % g.st) continue;
      const int p = hp / g.st;
      if (p >= g.P) continue;
      for (int s = 0; s < g.S; ++s) {
        const int wq = w + g.pad - s;
        if (wq < 0 || wq % g.st) continue;
        const int q = wq / g.st;
        if (q >= g.Q) continue;
        const int64_t m = ((int64_t)n * g.P + p) * g.Q + q;
        acc += bf2f(col[m * g.KP + (r * g.S + s) * g.C + c]);
      }
    }
    dx[e] = f2bf(acc);
  }
}

int grid_for(int64_t work) {
  int64_t gs = (work + 255) / 256;
  if (gs > 16384) gs = 16384;
  return gs < 1 ? 1 : (int)gs;
}

}  // namespace

void im2col_nhwc(const void* x, void* col, int N, int H, int W, int C, int R, int S, int P, int Q, int stride,
                 int pad, int up, int reflect, int KP, hipStream_t st) {
  const ColGeom g{N, H, W, C, R, S, P, Q, stride, pad, up == 4 ? 2 : (up == 2 ? 1 : 0), reflect ? 1 : 0, KP};
  const int64_t work = (int64_t)N * P * Q * (KP / 8);
  hipLaunchKernelGGL(im2col_k, dim3(grid_for(work)), dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)col, g);
}

void col2im_nhwc(const void* col, void* dx, const void* bias, int N, int H, int W, int C, int R, int S, int P, int Q,
                 int stride, int pad, int KP, hipStream_t st) {
  const ColGeom g{N, H, W, C, R, S, P, Q, stride, pad, 0, 0, KP};
  const int64_t work = (int64_t)N * H * W * C;
  hipLaunchKernelGGL(col2im_k, dim3(grid_for(work)), dim3(256), 0, st, (const uint16_t*)col, (uint16_t*)dx,
                     (const uint16_t*)bias, g);
}

}  // namespace tbamd
