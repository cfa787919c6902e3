// Small fused loss / resampling kernels for the style-transfer and MNIST
// generative examples.
//
// Reference call sites:
//   K19 total variation    examples/img_stt/online/online.py:66-69, offline.py:31-34
//   K20 per-(n,c) mean/std examples/img_stt/adain/adain.py:55-63
//   K21 BCE-with-logits, KL examples/img_gen/vae/vae.py:72-75,112
//   K22 hinge relu(m ± D)  examples/img_gen/gan/gan.py:104,107
//   K16 ReflectionPad2d    online.py:46, adain.py:36 (Conv lambda)
//   K17 Upsample(x2)       online.py:48, adain.py:38 (DeconvIN)
//   standalone activations (LeakyReLU(0.2) after the bias-only DCGAN discriminator input conv;
//   any nn.ReLU / GELU / SiLU / LeakyReLU nativize cannot fuse into a producer)
//
// Every scalar loss is a two-level deterministic reduction: a persistent grid
// writes one f32 partial per workgroup, a single workgroup folds them in f64.
// Backward kernels read the upstream gradient from device memory (no host
// sync, hipGraph-capturable).  Layout-generic kernels take the element stride
// of the spatial axes, so NCHW and channels_last tensors run the same code.
#include <algorithm>

#include "common.h"
#include "tbamd.h"

namespace tbamd {

namespace {

constexpr int kNT = 256;

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

__device__ __forceinline__ void write_partial(float acc, float* part) {
  __shared__ float red[kNT / 64];
  const float s = block_sum<kNT>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// out[0] = scale * Σ part (f64 fold, fixed order)
__global__ __launch_bounds__(kNT) void fold_k(const float* __restrict__ part, int n, float scale,
                                              float* __restrict__ out) {
  __shared__ double red[kNT / 64];
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += kNT) a += part[i];
  a = wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)((red[0] + red[1] + red[2] + red[3]) * (double)scale);
}

int reduce_grid(int64_t total) { return std::max(1, std::min(1024, cdiv(total, kNT * 8))); }

// ------------------------------------------------------------ total variation
// element idx has column w = (idx / inner) % W and row h = (idx / (inner·W)) % H;
// horizontal neighbour at +inner, vertical at +inner·W (inner = 1 NCHW, C NHWC)
template <int DT>
__global__ __launch_bounds__(kNT) void tv_fwd_k(const storage_t<DT>* __restrict__ x, int64_t total, int H, int W,
                                                int inner, float* __restrict__ part) {
  float acc = 0.f;
  const int64_t sh = (int64_t)inner * W;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int64_t q = i / inner;
    const int w = (int)(q % W);
    const int h = (int)((q / W) % H);
    const float v = Elem<DT>::ld(x, i);
    if (w < W - 1) acc += fabsf(v - Elem<DT>::ld(x, i + inner));
    if (h < H - 1) acc += fabsf(v - Elem<DT>::ld(x, i + sh));
  }
  write_partial(acc, part);
}

template <int DT>
__global__ __launch_bounds__(kNT) void tv_bwd_k(const storage_t<DT>* __restrict__ x, const float* __restrict__ gout,
                                                int64_t total, int H, int W, int inner,
                                                storage_t<DT>* __restrict__ dx) {
  const float g = gout[0];
  const int64_t sh = (int64_t)inner * W;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int64_t q = i / inner;
    const int w = (int)(q % W);
    const int h = (int)((q / W) % H);
    const float v = Elem<DT>::ld(x, i);
    float d = 0.f;
    if (w < W - 1) d += sgnf(v - Elem<DT>::ld(x, i + inner));
    if (w > 0) d -= sgnf(Elem<DT>::ld(x, i - inner) - v);
    if (h < H - 1) d += sgnf(v - Elem<DT>::ld(x, i + sh));
    if (h > 0) d -= sgnf(Elem<DT>::ld(x, i - sh) - v);
    Elem<DT>::st(dx, i, d * g);
  }
}

// ------------------------------------------------------------------ hinge
// loss = mean(relu(margin + sign·x))
template <int DT>
__global__ __launch_bounds__(kNT) void hinge_fwd_k(const storage_t<DT>* __restrict__ x, int64_t n, float margin,
                                                   float sign, float* __restrict__ part) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT)
    acc += fmaxf(margin + sign * Elem<DT>::ld(x, i), 0.f);
  write_partial(acc, part);
}

template <int DT>
__global__ __launch_bounds__(kNT) void hinge_bwd_k(const storage_t<DT>* __restrict__ x, const float* __restrict__ gout,
                                                   int64_t n, float margin, float sign,
                                                   storage_t<DT>* __restrict__ dx) {
  const float g = gout[0] * sign / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT)
    Elem<DT>::st(dx, i, (margin + sign * Elem<DT>::ld(x, i)) > 0.f ? g : 0.f);
}

// ------------------------------------------------------- BCE with logits
// loss = mean(max(x,0) - x·y + log1p(exp(-|x|))), dx = (σ(x) - y)·g/n
template <int DT>
__global__ __launch_bounds__(kNT) void bce_fwd_k(const storage_t<DT>* __restrict__ x, const storage_t<DT>* __restrict__ y,
                                                 int64_t n, float* __restrict__ part) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
    const float v = Elem<DT>::ld(x, i), t = Elem<DT>::ld(y, i);
    acc += fmaxf(v, 0.f) - v * t + log1pf(__expf(-fabsf(v)));
  }
  write_partial(acc, part);
}

template <int DT>
__global__ __launch_bounds__(kNT) void bce_bwd_k(const storage_t<DT>* __restrict__ x, const storage_t<DT>* __restrict__ y,
                                                 const float* __restrict__ gout, int64_t n,
                                                 storage_t<DT>* __restrict__ dx) {
  const float g = gout[0] / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
    const float v = Elem<DT>::ld(x, i);
    Elem<DT>::st(dx, i, (1.f / (1.f + __expf(-v)) - Elem<DT>::ld(y, i)) * g);
  }
}

// ---------------------------------------------------- Gaussian KL (VAE)
// loss = mean_rows(-0.5 Σ_d (1 + lv - mu² - e^lv)); rows = B
template <int DT>
__global__ __launch_bounds__(kNT) void kld_fwd_k(const storage_t<DT>* __restrict__ mu, const storage_t<DT>* __restrict__ lv,
                                                 int64_t n, float* __restrict__ part) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
    const float m = Elem<DT>::ld(mu, i), l = Elem<DT>::ld(lv, i);
    acc += -0.5f * (1.f + l - m * m - __expf(l));
  }
  write_partial(acc, part);
}

template <int DT>
__global__ __launch_bounds__(kNT) void kld_bwd_k(const storage_t<DT>* __restrict__ mu, const storage_t<DT>* __restrict__ lv,
                                                 const float* __restrict__ gout, int64_t n, int64_t rows,
                                                 storage_t<DT>* __restrict__ dmu, storage_t<DT>* __restrict__ dlv) {
  const float g = gout[0] / (float)rows;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
    Elem<DT>::st(dmu, i, g * Elem<DT>::ld(mu, i));
    Elem<DT>::st(dlv, i, g * 0.5f * (__expf(Elem<DT>::ld(lv, i)) - 1.f));
  }
}

// ------------------------------------------------- per-(n, c) mean / std
// element (n, c, s) at n·sN + c·sC + s·sS.  Workgroup = (n, tile of CT
// channels); lane layout cl = tid % CT over channels (coalesced for NHWC with
// CT = 64), sl = tid / CT over the S spatial positions.  Two passes (mean,
// then Σ(x-mean)²) keep the unbiased variance exact for large means.
template <int DT, int CT>
__global__ __launch_bounds__(kNT) void mustd_fwd_k(const storage_t<DT>* __restrict__ x, int C, int64_t S,
                                                   int64_t sN, int64_t sC, int64_t sS, float eps,
                                                   float* __restrict__ mean, float* __restrict__ std) {
  constexpr int SG = kNT / CT;
  __shared__ float red[SG][CT];
  const int cl = threadIdx.x % CT, sl = threadIdx.x / CT;
  const int n = blockIdx.y;
  const int c = blockIdx.x * CT + cl;
  const bool ok = c < C;
  const storage_t<DT>* p = x + (int64_t)n * sN + (int64_t)(ok ? c : 0) * sC;
  float a = 0.f;
  if (ok)
    for (int64_t s = sl; s < S; s += SG) a += Elem<DT>::ld(p, s * sS);
  red[sl][cl] = a;
  __syncthreads();
  if (CT == 1) {
    // SG = 256 partials of one channel: tree over the workgroup
    float v = wave_sum(threadIdx.x < SG ? red[threadIdx.x][0] : 0.f);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][0] = v;
    __syncthreads();
    if (threadIdx.x == 0) red[0][0] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
  } else if (sl == 0) {
    float t = 0.f;
    for (int j = 0; j < SG; ++j) t += red[j][cl];
    red[0][cl] = t;
  }
  __syncthreads();
  const float m = red[0][CT == 1 ? 0 : cl] / (float)S;
  __syncthreads();
  float q = 0.f;
  if (ok)
    for (int64_t s = sl; s < S; s += SG) {
      const float d = Elem<DT>::ld(p, s * sS) - m;
      q += d * d;
    }
  red[sl][cl] = q;
  __syncthreads();
  if (CT == 1) {
    float v = wave_sum(threadIdx.x < SG ? red[threadIdx.x][0] : 0.f);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][0] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float t = red[0][0] + red[1][0] + red[2][0] + red[3][0];
      mean[(int64_t)n * C + c] = m;
      std[(int64_t)n * C + c] = sqrtf(t / (float)(S > 1 ? S - 1 : 1) + eps);
    }
  } else if (sl == 0 && ok) {
    float t = 0.f;
    for (int j = 0; j < SG; ++j) t += red[j][cl];
    mean[(int64_t)n * C + c] = m;
    std[(int64_t)n * C + c] = sqrtf(t / (float)(S > 1 ? S - 1 : 1) + eps);
  }
}

// NHWC (channels_last) statistics split over spatial chunks.  The one-workgroup-per-
// (sample, 64 channels) kernel above walks all S pixels with 4 pixel groups -- 32 workgroups
// and 16 K dependent loads per thread for AdaIN's relu1_2 features [32, 64, 256, 256]
// (3 ms a call).  Here a grid of (chunk, channel block, sample) workgroups each reduce one
// chunk of >= 256 pixels with VEC-wide loads (16 B per lane for 16-bit types when C % 8 == 0),
// as sums of (x - x[n, pixel 0, c]) and their squares (the shift keeps the one-pass variance
// well conditioned); a finalize merges the chunks per (n, c) in f64, in a fixed order.
template <int DT, int VEC>
__global__ __launch_bounds__(kNT) void mustd_part_nhwc_k(const storage_t<DT>* __restrict__ x, int C, int64_t S,
                                                         int64_t chunk, float* __restrict__ part) {
  constexpr int LP = 64 / VEC, PG = kNT / LP;  // lanes per pixel (64 channels), pixel groups
  __shared__ float red[2][PG][64];
  const int lc = threadIdx.x % LP, pg = threadIdx.x / LP;
  const int n = blockIdx.z, cblk = blockIdx.y, ck = blockIdx.x;
  const int c0 = cblk * 64 + lc * VEC;
  const bool ok = c0 < C;  // C % VEC == 0 when VEC > 1
  const storage_t<DT>* xn = x + (int64_t)n * S * C;
  float sh[VEC], sa[VEC], sq[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) sh[e] = sa[e] = sq[e] = 0.f;
  if (ok) {
    load_vec<DT, VEC>(xn + c0, sh);
    const int64_t p0 = (int64_t)ck * chunk, p1 = min(S, p0 + chunk);
#pragma unroll 4
    for (int64_t p = p0 + pg; p < p1; p += PG) {
      float v[VEC];
      load_vec<DT, VEC>(xn + p * C + c0, v);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float d = v[e] - sh[e];
        sa[e] += d;
        sq[e] = __builtin_fmaf(d, d, sq[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    red[0][pg][lc * VEC + e] = sa[e];
    red[1][pg][lc * VEC + e] = sq[e];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = cblk * 64 + threadIdx.x;
    float a = 0.f, q = 0.f;
#pragma unroll 8
    for (int j = 0; j < PG; ++j) {
      a += red[0][j][threadIdx.x];
      q += red[1][j][threadIdx.x];
    }
    if (c < C) {
      float* o = part + (((int64_t)n * gridDim.x + ck) * 2) * C;
      o[c] = a;
      o[C + c] = q;
    }
  }
}

template <int DT>
__global__ __launch_bounds__(kNT) void mustd_fin_nhwc_k(const storage_t<DT>* __restrict__ x, const float* __restrict__ part,
                                                        int N, int C, int64_t S, int nck, float eps,
                                                        float* __restrict__ mean, float* __restrict__ std) {
  const int i = blockIdx.x * kNT + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  double a = 0.0, q = 0.0;
  for (int k = 0; k < nck; ++k) {
    const float* o = part + (((int64_t)n * nck + k) * 2) * C;
    a += (double)o[c];
    q += (double)o[C + c];
  }
  const double md = a / (double)S;
  double var = (q - a * md) / (double)(S > 1 ? S - 1 : 1);
  if (var < 0.0) var = 0.0;
  mean[i] = (float)((double)Elem<DT>::ld(x + (int64_t)n * S * C, c) + md);
  std[i] = (float)sqrt(var + (double)eps);
}

// dx = dmu/S + dstd·(x - mu)/((S-1)·std) over the same (n, c, s) addressing;
// `cmod`/`cdivn` decode (n, c) from the flat index: c = (i / cdivn) % C, n = i / (C·S)
template <int DT>
__global__ __launch_bounds__(kNT) void mustd_bwd_k(const storage_t<DT>* __restrict__ x, const float* __restrict__ mean,
                                                   const float* __restrict__ std, const float* __restrict__ dmean,
                                                   const float* __restrict__ dstd, int64_t total, int C, int64_t S,
                                                   int64_t cdivn, storage_t<DT>* __restrict__ dx) {
  const float inv_s = 1.f / (float)S, inv_s1 = 1.f / (float)(S > 1 ? S - 1 : 1);
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int64_t n = i / ((int64_t)C * S);
    const int c = (int)((i / cdivn) % C);
    const int64_t j = n * C + c;
    const float v = Elem<DT>::ld(x, i);
    Elem<DT>::st(dx, i, dmean[j] * inv_s + dstd[j] * (v - mean[j]) * inv_s1 / std[j]);
  }
}

// NHWC backward, C % 8 == 0: per-(n, c) affine coefficients dx = a + b x first (a tiny
// kernel), then one 16-B-vector pass over x (the flat-index kernel above spends two 64-bit
// divisions and four coefficient loads per element)
__global__ __launch_bounds__(kNT) void mustd_coef_k(const float* __restrict__ mean, const float* __restrict__ std,
                                                    const float* __restrict__ dmean, const float* __restrict__ dstd,
                                                    int NC, int64_t S, float* __restrict__ coef) {
  const int i = blockIdx.x * kNT + threadIdx.x;
  if (i >= NC) return;
  const float inv_s = 1.f / (float)S, inv_s1 = 1.f / (float)(S > 1 ? S - 1 : 1);
  const float bq = dstd[i] * inv_s1 / std[i];
  coef[i] = dmean[i] * inv_s - bq * mean[i];
  coef[NC + i] = bq;
}

template <int DT>
__global__ __launch_bounds__(kNT) void mustd_bwd_nhwc_k(const storage_t<DT>* __restrict__ x,
                                                        const float* __restrict__ coef, int NC, int C, int64_t S,
                                                        int64_t n8, storage_t<DT>* __restrict__ dx) {
  const int64_t SC = S * C;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kNT) {
    const int64_t e0 = i * 8;
    const int n = (int)(e0 / SC);
    const int c0 = (int)(e0 % C);
    const float* ca = coef + (int64_t)n * C + c0;
    float v[8];
    load_vec<DT, 8>(x + e0, v);
    const float4 a0 = *reinterpret_cast<const float4*>(ca), a1 = *reinterpret_cast<const float4*>(ca + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(ca + NC), b1 = *reinterpret_cast<const float4*>(ca + NC + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = __builtin_fmaf(bv[e], v[e], av[e]);
    store_vec<DT, 8>(dx + e0, v);
  }
}

// ---------------------------------------------- NHWC reflection padding
__device__ __forceinline__ int reflect(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

// y [N][Ho][Wo][C] <- x [N][H][W][C]; one thread per output element, channel fastest
template <int DT>
__global__ __launch_bounds__(kNT) void rpad_fwd_k(const storage_t<DT>* __restrict__ x, int N, int H, int W, int C,
                                                  int pt, int pl, int Ho, int Wo, storage_t<DT>* __restrict__ y) {
  const int64_t total = (int64_t)N * Ho * Wo * C;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int ow = (int)(q % Wo);
    q /= Wo;
    const int oh = (int)(q % Ho);
    const int64_t n = q / Ho;
    const int ih = reflect(oh - pt, H), iw = reflect(ow - pl, W);
    Elem<DT>::st(y, i, Elem<DT>::ld(x, ((n * H + ih) * W + iw) * C + c));
  }
}

// gather form of the backward (deterministic, no atomics): input row i
// receives output rows o with reflect(o - p) == i: o = i + p always, o = p - i
// when 1 <= i <= p (top mirror), o = p + 2(H-1) - i when H-1-pb <= i <= H-2
__device__ __forceinline__ int rpad_sources(int i, int n, int p, int pe, int* o) {
  int k = 0;
  o[k++] = i + p;
  if (i >= 1 && i <= p) o[k++] = p - i;
  if (i <= n - 2 && i >= n - 1 - pe) o[k++] = p + 2 * (n - 1) - i;
  return k;
}

template <int DT>
__global__ __launch_bounds__(kNT) void rpad_bwd_k(const storage_t<DT>* __restrict__ dy, int N, int H, int W, int C,
                                                  int pt, int pb, int pl, int pr, int Ho, int Wo,
                                                  storage_t<DT>* __restrict__ dx) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int iw = (int)(q % W);
    q /= W;
    const int ih = (int)(q % H);
    const int64_t n = q / H;
    int rh[3], rw[3];
    const int nh = rpad_sources(ih, H, pt, pb, rh), nw = rpad_sources(iw, W, pl, pr, rw);
    float a = 0.f;
    for (int u = 0; u < nh; ++u)
      for (int v = 0; v < nw; ++v) a += Elem<DT>::ld(dy, ((n * Ho + rh[u]) * Wo + rw[v]) * C + c);
    Elem<DT>::st(dx, i, a);
  }
}

// ----------------------------------------- NHWC nearest upsample (integer factor)
template <int DT>
__global__ __launch_bounds__(kNT) void up_fwd_k(const storage_t<DT>* __restrict__ x, int N, int H, int W, int C, int f,
                                                storage_t<DT>* __restrict__ y) {
  const int Ho = H * f, Wo = W * f;
  const int64_t total = (int64_t)N * Ho * Wo * C;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int ow = (int)(q % Wo);
    q /= Wo;
    const int oh = (int)(q % Ho);
    const int64_t n = q / Ho;
    Elem<DT>::st(y, i, Elem<DT>::ld(x, ((n * H + oh / f) * W + ow / f) * C + c));
  }
}

template <int DT>
__global__ __launch_bounds__(kNT) void up_bwd_k(const storage_t<DT>* __restrict__ dy, int N, int H, int W, int C, int f,
                                                storage_t<DT>* __restrict__ dx) {
  const int Ho = H * f, Wo = W * f;
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int c = (int)(i % C);
    int64_t q = i / C;
    const int iw = (int)(q % W);
    q /= W;
    const int ih = (int)(q % H);
    const int64_t n = q / H;
    float a = 0.f;
    for (int u = 0; u < f; ++u)
      for (int v = 0; v < f; ++v) a += Elem<DT>::ld(dy, ((n * Ho + ih * f + u) * Wo + iw * f + v) * C + c);
    Elem<DT>::st(dx, i, a);
  }
}

int ew_grid(int64_t total) { return std::max(1, std::min(8192, cdiv(total, kNT * 4))); }

// y = act(x), dx = dy * act'(x): 8 elements (16 B for 16-bit types) per lane per step,
// grid-stride; same device functions as the fused BN / GEMM epilogues
template <int DT, int ACT>
__global__ __launch_bounds__(kNT) void act_fwd_k(const storage_t<DT>* __restrict__ x, storage_t<DT>* __restrict__ y,
                                                int64_t n8, float slope) {
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kNT) {
    float v[8];
    load_vec<DT, 8>(x + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = act_fwd<ACT>(v[e], slope);
    store_vec<DT, 8>(y + i * 8, v);
  }
}

template <int DT, int ACT>
__global__ __launch_bounds__(kNT) void act_bwd_k(const storage_t<DT>* __restrict__ x,
                                                const storage_t<DT>* __restrict__ dy, storage_t<DT>* __restrict__ dx,
                                                int64_t n8, float slope) {
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kNT) {
    float v[8], g[8];
    load_vec<DT, 8>(x + i * 8, v);
    load_vec<DT, 8>(dy + i * 8, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= act_bwd<ACT>(v[e], slope);
    store_vec<DT, 8>(dx + i * 8, g);
  }
}

}  // namespace

int aux_partials() { return 1024; }

void tv_forward(int dt, const void* x, int64_t total, int H, int W, int inner, float* part, float* out,
                hipStream_t st) {
  const int g = reduce_grid(total);
  TBAMD_DISPATCH_DT(dt, DT, { tv_fwd_k<DT><<<g, kNT, 0, st>>>((const storage_t<DT>*)x, total, H, W, inner, part); });
  fold_k<<<1, kNT, 0, st>>>(part, g, 1.f, out);
}

void tv_backward(int dt, const void* x, const float* gout, int64_t total, int H, int W, int inner, void* dx,
                 hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    tv_bwd_k<DT><<<ew_grid(total), kNT, 0, st>>>((const storage_t<DT>*)x, gout, total, H, W, inner,
                                                 (storage_t<DT>*)dx);
  });
}

void hinge_forward(int dt, const void* x, int64_t n, float margin, float sign, float* part, float* out,
                   hipStream_t st) {
  const int g = reduce_grid(n);
  TBAMD_DISPATCH_DT(dt, DT, { hinge_fwd_k<DT><<<g, kNT, 0, st>>>((const storage_t<DT>*)x, n, margin, sign, part); });
  fold_k<<<1, kNT, 0, st>>>(part, g, 1.f / (float)n, out);
}

void hinge_backward(int dt, const void* x, const float* gout, int64_t n, float margin, float sign, void* dx,
                    hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    hinge_bwd_k<DT><<<ew_grid(n), kNT, 0, st>>>((const storage_t<DT>*)x, gout, n, margin, sign,
                                                (storage_t<DT>*)dx);
  });
}

void bce_logits_forward(int dt, const void* x, const void* y, int64_t n, float* part, float* out, hipStream_t st) {
  const int g = reduce_grid(n);
  TBAMD_DISPATCH_DT(dt, DT, {
    bce_fwd_k<DT><<<g, kNT, 0, st>>>((const storage_t<DT>*)x, (const storage_t<DT>*)y, n, part);
  });
  fold_k<<<1, kNT, 0, st>>>(part, g, 1.f / (float)n, out);
}

void bce_logits_backward(int dt, const void* x, const void* y, const float* gout, int64_t n, void* dx,
                         hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    bce_bwd_k<DT><<<ew_grid(n), kNT, 0, st>>>((const storage_t<DT>*)x, (const storage_t<DT>*)y, gout, n,
                                              (storage_t<DT>*)dx);
  });
}

void kld_forward(int dt, const void* mu, const void* lv, int64_t n, int64_t rows, float* part, float* out,
                 hipStream_t st) {
  const int g = reduce_grid(n);
  TBAMD_DISPATCH_DT(dt, DT, {
    kld_fwd_k<DT><<<g, kNT, 0, st>>>((const storage_t<DT>*)mu, (const storage_t<DT>*)lv, n, part);
  });
  fold_k<<<1, kNT, 0, st>>>(part, g, 1.f / (float)rows, out);
}

void kld_backward(int dt, const void* mu, const void* lv, const float* gout, int64_t n, int64_t rows, void* dmu,
                  void* dlv, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    kld_bwd_k<DT><<<ew_grid(n), kNT, 0, st>>>((const storage_t<DT>*)mu, (const storage_t<DT>*)lv, gout, n, rows,
                                              (storage_t<DT>*)dmu, (storage_t<DT>*)dlv);
  });
}

int64_t mean_std_workspace(int N, int C, int64_t S, bool channels_last) {
  if (!channels_last) return 0;
  const int64_t wgs = (int64_t)N * cdiv(C, 64);
  int64_t nck = std::max<int64_t>(1, std::min<int64_t>(cdiv(2048, wgs), cdiv(S, 256)));
  const int64_t chunk = cdiv(S, nck);
  nck = cdiv(S, chunk);
  return (int64_t)N * nck * 2 * C;
}

void mean_std_forward(int dt, const void* x, int N, int C, int64_t S, bool channels_last, float eps, float* mean,
                      float* std, hipStream_t st, float* ws) {
  const int64_t sN = (int64_t)C * S;
  TBAMD_DISPATCH_DT(dt, DT, {
    if (channels_last && ws != nullptr) {
      const int64_t wgs = (int64_t)N * cdiv(C, 64);
      int64_t nck = std::max<int64_t>(1, std::min<int64_t>(cdiv(2048, wgs), cdiv(S, 256)));
      const int64_t chunk = cdiv(S, nck);
      nck = cdiv(S, chunk);
      const dim3 grid((unsigned)nck, cdiv(C, 64), N);
      if (C % 8 == 0)
        mustd_part_nhwc_k<DT, 8><<<grid, kNT, 0, st>>>((const storage_t<DT>*)x, C, S, chunk, ws);
      else
        mustd_part_nhwc_k<DT, 1><<<grid, kNT, 0, st>>>((const storage_t<DT>*)x, C, S, chunk, ws);
      mustd_fin_nhwc_k<DT><<<cdiv(N * C, kNT), kNT, 0, st>>>((const storage_t<DT>*)x, ws, N, C, S, (int)nck, eps,
                                                            mean, std);
    } else if (channels_last) {
      dim3 grid(cdiv(C, 64), N);
      mustd_fwd_k<DT, 64><<<grid, kNT, 0, st>>>((const storage_t<DT>*)x, C, S, sN, 1, C, eps, mean, std);
    } else {
      dim3 grid(C, N);
      mustd_fwd_k<DT, 1><<<grid, kNT, 0, st>>>((const storage_t<DT>*)x, C, S, sN, S, 1, eps, mean, std);
    }
  });
}

void mean_std_backward(int dt, const void* x, const float* mean, const float* std, const float* dmean,
                       const float* dstd, int N, int C, int64_t S, bool channels_last, void* dx, hipStream_t st,
                       float* coef) {
  const int64_t total = (int64_t)N * C * S;
  if (channels_last && coef != nullptr && C % 8 == 0) {
    const int NC = N * C;
    mustd_coef_k<<<cdiv(NC, kNT), kNT, 0, st>>>(mean, std, dmean, dstd, NC, S, coef);
    const int64_t n8 = total / 8;
    int64_t grid = (n8 + kNT - 1) / kNT;
    if (grid > 16384) grid = 16384;
    TBAMD_DISPATCH_DT(dt, DT, {
      mustd_bwd_nhwc_k<DT><<<(int)grid, kNT, 0, st>>>((const storage_t<DT>*)x, coef, NC, C, S, n8,
                                                      (storage_t<DT>*)dx);
    });
    return;
  }
  TBAMD_DISPATCH_DT(dt, DT, {
    mustd_bwd_k<DT><<<ew_grid(total), kNT, 0, st>>>((const storage_t<DT>*)x, mean, std, dmean, dstd, total, C, S,
                                                    channels_last ? 1 : S, (storage_t<DT>*)dx);
  });
}

void reflect_pad_forward(int dt, const void* x, int N, int H, int W, int C, int pt, int pb, int pl, int pr,
                         void* y, hipStream_t st) {
  const int Ho = H + pt + pb, Wo = W + pl + pr;
  TBAMD_DISPATCH_DT(dt, DT, {
    rpad_fwd_k<DT><<<ew_grid((int64_t)N * Ho * Wo * C), kNT, 0, st>>>((const storage_t<DT>*)x, N, H, W, C, pt, pl,
                                                                       Ho, Wo, (storage_t<DT>*)y);
  });
}

void reflect_pad_backward(int dt, const void* dy, int N, int H, int W, int C, int pt, int pb, int pl, int pr,
                          void* dx, hipStream_t st) {
  const int Ho = H + pt + pb, Wo = W + pl + pr;
  TBAMD_DISPATCH_DT(dt, DT, {
    rpad_bwd_k<DT><<<ew_grid((int64_t)N * H * W * C), kNT, 0, st>>>((const storage_t<DT>*)dy, N, H, W, C, pt, pb,
                                                                     pl, pr, Ho, Wo, (storage_t<DT>*)dx);
  });
}

void upsample_nearest_forward(int dt, const void* x, int N, int H, int W, int C, int f, void* y, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    up_fwd_k<DT><<<ew_grid((int64_t)N * H * W * C * f * f), kNT, 0, st>>>((const storage_t<DT>*)x, N, H, W, C, f,
                                                                           (storage_t<DT>*)y);
  });
}

void upsample_nearest_backward(int dt, const void* dy, int N, int H, int W, int C, int f, void* dx,
                               hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    up_bwd_k<DT><<<ew_grid((int64_t)N * H * W * C), kNT, 0, st>>>((const storage_t<DT>*)dy, N, H, W, C, f,
                                                                   (storage_t<DT>*)dx);
  });
}

static int act_grid(int64_t n8) {
  const int64_t g = (n8 + kNT - 1) / kNT;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}

void act_forward(int dt, int act, const void* x, void* y, int64_t n, float slope, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, AV, {
      act_fwd_k<DT, AV><<<act_grid(n8), kNT, 0, st>>>((const storage_t<DT>*)x, (storage_t<DT>*)y, n8, slope);
    });
  });
}

void act_backward(int dt, int act, const void* x, const void* dy, void* dx, int64_t n, float slope, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, AV, {
      act_bwd_k<DT, AV><<<act_grid(n8), kNT, 0, st>>>((const storage_t<DT>*)x, (const storage_t<DT>*)dy,
                                                      (storage_t<DT>*)dx, n8, slope);
    });
  });
}

}  // namespace tbamd
