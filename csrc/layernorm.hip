// Row LayerNorm (+ optional residual add producing the new residual stream)
// for gfx950: one wave per row, the row held in registers (two-pass exact
// variance), 16-B vector loads; backward reduces dgamma/dbeta per workgroup
// into [nblk][C] partials merged by a second kernel (deterministic).
//
// Needed by the ViT-B/16 north-star config (BASELINE.json config 5); the
// reference has no transformer.
#include "common.h"
#include "tbamd.h"

namespace tbamd {

constexpr int kLnWaves = 4;  // rows per workgroup

template <int DT, int VPL>
__global__ __launch_bounds__(64 * kLnWaves) void ln_fwd_k(const storage_t<DT>* __restrict__ x,
                                                          const storage_t<DT>* __restrict__ res,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, int64_t M, int C,
                                                          float eps, storage_t<DT>* __restrict__ y,
                                                          storage_t<DT>* __restrict__ xsum,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = C / 8;
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nv) {
      Vec8<DT>::load(x + row * C + vi * 8, v[i]);
      if (res) {
        float r[8];
        Vec8<DT>::load(res + row * C + vi * 8, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[i][k] += r[k];
        Vec8<DT>::store(xsum + row * C + vi * 8, v[i]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[i][k];
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[i][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nv) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = vi * 8 + k;
        o[k] = (v[i][k] - mean) * rstd * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
      }
      Vec8<DT>::store(y + row * C + vi * 8, o);
    }
  }
}

template <int DT, int VPL>
__global__ __launch_bounds__(64 * kLnWaves) void ln_bwd_k(const storage_t<DT>* __restrict__ dy,
                                                          const storage_t<DT>* __restrict__ x,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in, int64_t M, int C,
                                                          int rows_per_blk, storage_t<DT>* __restrict__ dx,
                                                          float* __restrict__ pdg, float* __restrict__ pdb) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = C / 8;
  float ag[VPL][8], ab[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[i][k] = ab[i][k] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  for (int64_t row = r0 + wv; row < r0 + rows_per_blk && row < M; row += kLnWaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[VPL][8], gd[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv) {
        float xv[8], dv[8];
        Vec8<DT>::load(x + row * C + vi * 8, xv);
        Vec8<DT>::load(dy + row * C + vi * 8, dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int c = vi * 8 + k;
          xh[i][k] = (xv[k] - mean) * rstd;
          gd[i][k] = dv[k] * (gamma ? gamma[c] : 1.f);
          s1 += gd[i][k];
          s2 += gd[i][k] * xh[i][k];
          ag[i][k] += dv[k] * xh[i][k];
          ab[i][k] += dv[k];
        }
      }
    }
    s1 = wave_sum(s1) / (float)C;
    s2 = wave_sum(s2) / (float)C;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nv) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (gd[i][k] - s1 - xh[i][k] * s2);
        Vec8<DT>::store(dx + row * C + vi * 8, o);
      }
    }
  }
  // reduce the 4 waves' column partials through LDS, write [blk][C]
  __shared__ float red[kLnWaves][2][VPL * 512];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[wv][0][vi * 8 + k] = ag[i][k];
        red[wv][1][vi * 8 + k] = ab[i][k];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 64 * kLnWaves) {
    float g = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < kLnWaves; ++w) {
      g += red[w][0][c];
      b += red[w][1][c];
    }
    pdg[(int64_t)blockIdx.x * C + c] = g;
    pdb[(int64_t)blockIdx.x * C + c] = b;
  }
}

// column sums of two [nblk][C] partial arrays: one workgroup per 64 columns,
// 16 row-groups per workgroup (each strides the rows), f64 accumulation, then a
// fixed-order LDS merge (deterministic).  Was one thread per column: 3
// workgroups for C = 768 and a 1024-long dependent loop each (0.23 ms/call).
constexpr int kColRG = 16;
__global__ __launch_bounds__(64 * kColRG) void col_sum2_k(const float* __restrict__ a, const float* __restrict__ b,
                                                          int nblk, int C, float* __restrict__ oa,
                                                          float* __restrict__ ob) {
  __shared__ double red[2][kColRG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  double sa = 0.0, sb = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int i = ty; i < nblk; i += kColRG) {
      sa += a[(int64_t)i * C + c];
      sb += b[(int64_t)i * C + c];
    }
  }
  red[0][ty][tx] = sa;
  red[1][ty][tx] = sb;
  __syncthreads();
  if (ty == 0 && c < C) {
    double ta = 0.0, tb = 0.0;
    for (int r = 0; r < kColRG; ++r) {
      ta += red[0][r][tx];
      tb += red[1][r][tx];
    }
    if (oa) oa[c] = (float)ta;
    if (ob) ob[c] = (float)tb;
  }
}

static int ln_vpl(int C) { return C <= 512 ? 1 : C <= 1024 ? 2 : C <= 2048 ? 4 : 8; }

int ln_bwd_blocks(int64_t M) {
  int64_t b = (M + 31) / 32;  // >= 32 rows per workgroup
  if (b > 1024) b = 1024;
  return (int)(b < 1 ? 1 : b);
}

template <int DT, int V>
static void ln_fwd_launch(const void* x, const void* res, const float* gamma, const float* beta, int64_t M, int C,
                          float eps, void* y, void* xsum, float* mean, float* rstd, hipStream_t st) {
  using T = storage_t<DT>;
  ln_fwd_k<DT, V><<<cdiv(M, kLnWaves), 64 * kLnWaves, 0, st>>>((const T*)x, (const T*)res, gamma, beta, M, C, eps,
                                                              (T*)y, (T*)xsum, mean, rstd);
}

template <int DT, int V>
static void ln_bwd_launch(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                          int64_t M, int C, int rpb, void* dx, float* pdg, float* pdb, int nblk, hipStream_t st) {
  using T = storage_t<DT>;
  ln_bwd_k<DT, V><<<nblk, 64 * kLnWaves, 0, st>>>((const T*)dy, (const T*)x, gamma, mean, rstd, M, C, rpb, (T*)dx,
                                                 pdg, pdb);
}

void ln_forward(int dt, const void* x, const void* res, const float* gamma, const float* beta, int64_t M, int C,
                float eps, void* y, void* xsum, float* mean, float* rstd, hipStream_t st) {
  const int v = ln_vpl(C);
  TBAMD_DISPATCH_DT(dt, DT, {
    if (v == 1) ln_fwd_launch<DT, 1>(x, res, gamma, beta, M, C, eps, y, xsum, mean, rstd, st);
    else if (v == 2) ln_fwd_launch<DT, 2>(x, res, gamma, beta, M, C, eps, y, xsum, mean, rstd, st);
    else if (v == 4) ln_fwd_launch<DT, 4>(x, res, gamma, beta, M, C, eps, y, xsum, mean, rstd, st);
    else ln_fwd_launch<DT, 8>(x, res, gamma, beta, M, C, eps, y, xsum, mean, rstd, st);
  });
}

void ln_backward(int dt, const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                 int64_t M, int C, void* dx, float* pdg, float* pdb, int nblk, float* dgamma, float* dbeta,
                 hipStream_t st) {
  const int rpb = (int)((M + nblk - 1) / nblk);
  const int v = ln_vpl(C);
  TBAMD_DISPATCH_DT(dt, DT, {
    if (v == 1) ln_bwd_launch<DT, 1>(dy, x, gamma, mean, rstd, M, C, rpb, dx, pdg, pdb, nblk, st);
    else if (v == 2) ln_bwd_launch<DT, 2>(dy, x, gamma, mean, rstd, M, C, rpb, dx, pdg, pdb, nblk, st);
    else if (v == 4) ln_bwd_launch<DT, 4>(dy, x, gamma, mean, rstd, M, C, rpb, dx, pdg, pdb, nblk, st);
    else ln_bwd_launch<DT, 8>(dy, x, gamma, mean, rstd, M, C, rpb, dx, pdg, pdb, nblk, st);
  });
  col_sum2_k<<<cdiv(C, 64), 64 * kColRG, 0, st>>>(pdg, pdb, nblk, C, dgamma, dbeta);
}

}  // namespace tbamd
