// Generic NHWC convolution on gfx950 MFMA for the shapes the 64-channel
// implicit-GEMM kernels (conv.hip / conv_wgrad.hip) do not take:
//
//   * any channel counts (LeNet 1->6->16, StyleNet / AdaIN 3 / 32 channels,
//     9x9 taps), any kernel size and stride;
//   * fp32 activations at reference precision (examples/img_stt/*.yml run fp32)
//     on the exact-f32 MFMA v_mfma_f32_16x16x4_f32, bf16 on v_mfma_f32_16x16x32_bf16;
//   * ReflectionPad2d and nearest Upsample(xU) FOLDED into the input addressing
//     (reference online.py:46-48, adain.py:36-38: Conv = pad + conv, DeconvIN =
//     upsample + pad + conv): no padded / upsampled tensor is ever written.
//
// The input is read through a virtual grid  xv = pad(upsample(dilate(x)))  (upsample
// factor U, or dilation D for input gradients, zero or reflect padding):
//
//   forward   y[n,p,q,k]   = b[k] + sum_{r,s,c} xv[n, p*st - pad + r, q*st - pad + s, c] w[k,r,s,c]
//   wgrad     dW[k,r,s,c]  = sum_{n,p,q} dy[n,p,q,k] xv[n, p*st - pad + r, q*st - pad + s, c]
//   dgrad     the forward kernel on dy dilated by st, zero pad R-1, flipped weights,
//             gives dL/dxv on the padded virtual grid; conv_any_fold sums it back
//             onto x (the reflect mirror images and the U x U upsampled copies of
//             every input pixel).
//
// Implicit GEMM with register-staged operands (arbitrary C forbids the 16-B
// direct-to-LDS loads of conv.hip): 64-pixel x BM-channel tiles, 32-deep reduction
// chunks, one 256-thread workgroup per tile, the next chunk's gathers in flight
// while the current chunk is multiplied.  Reference: SURVEY.md §2.3.1 K1/K2/K3,
// K16, K17.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// fp32 operands as an unevaluated sum hi + lo of two bf16 (hi = RNE(v), lo = RNE(v - hi)):
// a product is hi_a hi_b + hi_a lo_b + lo_a hi_b on the bf16 MFMA (the lo_a lo_b term and lo's
// own rounding are below 2^-16 relative), three v_mfma_f32_16x16x32_bf16 per 32-deep step in
// place of eight v_mfma_f32_16x16x4_f32 -- ~1e-5 relative error, finer than the TF32 that
// cuDNN applies to the reference's fp32 convolutions by default (torch allow_tf32)
__device__ __forceinline__ void split8(const float* v, bf16x8_t& hi, bf16x8_t& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    hi[e] = h;
    lo[e] = (__bf16)(v[e] - (float)h);
  }
}

__device__ __forceinline__ f32x4_t mfma_split(const bf16x8_t& ah, const bf16x8_t& al, const bf16x8_t& bh,
                                              const bf16x8_t& bl, f32x4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);  // small terms first
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// fp32 convs: split-bf16 MFMA (default) or the exact-f32 MFMA (conv_any_set_f32_split(false))
bool g_f32_split = true;

constexpr int kCA_BN = 64;   // pixels per tile
constexpr int kCA_KC = 32;   // reduction chunk
constexpr int kCA_T = 256;

struct AnyGeom {
  int N, H, W, C;       // real input
  int K, R, S;          // out channels, taps
  int P, Q;             // output grid
  int st, pad;          // stride, padding of the virtual grid
  int up, dil;          // upsample factor (>= 1) or input dilation (>= 1); not both > 1
  int reflect;          // reflect padding (else zero)
  int Hv, Wv;           // virtual (upsampled / dilated, unpadded) input size
  int Pp, Qp;           // per-phase output grid ceil(P / dil) x ceil(Q / dil) (dil > 1)
};

// Stride-phase decomposition of a dilated input (the input gradient of a strided conv,
// transposed convs): output pixels of one parity class (p % D, q % D) = (a, b) only meet
// the taps r = r0 + D r' with r0 = (pad - a) mod D, which read the REAL input row
// (a - pad + r0) / D + p' + r'  (p = a + D p').  A tile holds pixels of one class, so the
// reduction runs over ceil((R - r0) / D) x ceil((S - s0) / D) x C instead of R x S x C:
// no gathers or MFMAs are spent on the dilation zeros (4x less work at stride 2).
struct PhaseTile {
  int a, b, r0, s0, nr, ns;
};

__device__ __forceinline__ PhaseTile phase_of(const AnyGeom& g, int ph) {
  PhaseTile t;
  t.a = ph / g.dil;
  t.b = ph - t.a * g.dil;
  t.r0 = ((g.pad - t.a) % g.dil + g.dil) % g.dil;
  t.s0 = ((g.pad - t.b) % g.dil + g.dil) % g.dil;
  t.nr = t.r0 < g.R ? (g.R - t.r0 + g.dil - 1) / g.dil : 0;
  t.ns = t.s0 < g.S ? (g.S - t.s0 + g.dil - 1) / g.dil : 0;
  return t;
}

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 4) return p[i];
  else return bf2f(p[i]);
}

// element of the virtual input at padded-relative coordinate (hv, wv) (may be < 0 or >= Hv)
template <typename T>
__device__ __forceinline__ float xv_at(const T* __restrict__ x, const AnyGeom& g, int n, int hv, int wv, int c) {
  if (g.reflect) {
    hv = hv < 0 ? -hv : (hv >= g.Hv ? 2 * g.Hv - 2 - hv : hv);
    wv = wv < 0 ? -wv : (wv >= g.Wv ? 2 * g.Wv - 2 - wv : wv);
  } else if ((unsigned)hv >= (unsigned)g.Hv || (unsigned)wv >= (unsigned)g.Wv) {
    return 0.f;
  }
  int h = hv, w = wv;  // (uniform branches: no integer division on the plain path)
  if (g.dil > 1) {
    if (hv % g.dil != 0 || wv % g.dil != 0) return 0.f;
    h = hv / g.dil;
    w = wv / g.dil;
  } else if (g.up > 1) {
    h = hv / g.up;
    w = wv / g.up;
  }
  const int64_t i = (((int64_t)n * g.H + h) * g.W + w) * g.C + c;
  if (!TB_BOUNDS_OK(i >= 0 && i < (int64_t)g.N * g.H * g.W * g.C, kBndAnySrc)) return 0.f;
  return ldf(x, i);
}

template <typename T>
__device__ __forceinline__ T to_t(float v) {
  if constexpr (sizeof(T) == 4) return v;
  else return f2bf(v);
}

// 8 consecutive reduction indices kk0 .. kk0+7 ((r, s, c), c fastest) of one pixel
template <typename T>
__device__ __forceinline__ void gather8(const T* __restrict__ x, const AnyGeom& g, int n, int hv0, int wv0,
                                        int kk0, int Kred, float* v) {
  int rs = kk0 / g.C, c = kk0 - rs * g.C;
  int r = rs / g.S, s = rs - r * g.S;
  if ((g.C & 7) == 0) {  // the 8 values are one tap's contiguous channels (kk0 % 8 == 0): vector load
    if (kk0 >= Kred) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      return;
    }
    int hv = hv0 + r, wv = wv0 + s;
    bool ok = true;
    if (g.reflect) {
      hv = hv < 0 ? -hv : (hv >= g.Hv ? 2 * g.Hv - 2 - hv : hv);
      wv = wv < 0 ? -wv : (wv >= g.Wv ? 2 * g.Wv - 2 - wv : wv);
    } else {
      ok = (unsigned)hv < (unsigned)g.Hv && (unsigned)wv < (unsigned)g.Wv;
    }
    int h = hv, w = wv;
    if (ok) {
      if (g.dil > 1) {
        ok = hv % g.dil == 0 && wv % g.dil == 0;
        h = hv / g.dil;
        w = wv / g.dil;
      } else if (g.up > 1) {
        h = hv / g.up;
        w = wv / g.up;
      }
    }
    if (!ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      return;
    }
    const int64_t i0 = (((int64_t)n * g.H + h) * g.W + w) * g.C + c;
    if (!TB_BOUNDS_OK(i0 >= 0 && i0 + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndAnySrc)) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      return;
    }
    const T* p = x + i0;
    if constexpr (sizeof(T) == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const uint4 a = *reinterpret_cast<const uint4*>(p);
      const uint32_t u[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = bf2f((uint16_t)(u[e] & 0xffff));
        v[2 * e + 1] = bf2f((uint16_t)(u[e] >> 16));
      }
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = (kk0 + e < Kred) ? xv_at(x, g, n, hv0 + r, wv0 + s, c) : 0.f;
    if (++c == g.C) {
      c = 0;
      if (++s == g.S) {
        s = 0;
        ++r;
      }
    }
  }
}

// phase-mode gather: 8 consecutive reduction indices (r', s', c) of one pixel whose tap
// (0, 0) reads real input (hb, wb); taps outside the input are the zero padding
template <typename T>
__device__ __forceinline__ void gather8_ph(const T* __restrict__ x, const AnyGeom& g, int n, int hb, int wb, int ns,
                                           int kk0, int Kred, float* v) {
  int rs = kk0 / g.C, c = kk0 - rs * g.C;
  int r = rs / ns, s = rs - r * ns;
  const int64_t nb = (int64_t)n * g.H;
  if ((g.C & 7) == 0) {
    const int h = hb + r, w = wb + s;
    if (kk0 >= Kred || (unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      return;
    }
    const int64_t i0 = ((nb + h) * g.W + w) * g.C + c;
    if (!TB_BOUNDS_OK(i0 >= 0 && i0 + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndAnySrc)) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      return;
    }
    const T* p = x + i0;
    if constexpr (sizeof(T) == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const uint4 a = *reinterpret_cast<const uint4*>(p);
      const uint32_t u[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = bf2f((uint16_t)(u[e] & 0xffff));
        v[2 * e + 1] = bf2f((uint16_t)(u[e] >> 16));
      }
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int h = hb + r, w = wb + s;
    float val = 0.f;
    if (kk0 + e < Kred && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W) {
      const int64_t i = ((nb + h) * g.W + w) * g.C + c;
      if (TB_BOUNDS_OK(i >= 0 && i < (int64_t)g.N * g.H * g.W * g.C, kBndAnySrc)) val = ldf(x, i);
    }
    v[e] = val;
    if (++c == g.C) {
      c = 0;
      if (++s == ns) {
        s = 0;
        ++r;
      }
    }
  }
}

// ---------------------------------------------------------------- forward
// LDS tiles [rows][KC + 8] of T (the +8 pad staggers the fragment rows over banks).
// PH: stride-phase mode (g.dil > 1, zero padding, no upsampling), see PhaseTile.
// NB: 64-pixel blocks per tile (each wave multiplies NB 16-pixel fragments): narrow
// outputs (K <= 16 / 32) take 256 / 128 pixels per tile so a barrier pair and the
// weight chunk are shared by NB x as many MFMAs and gathers.
template <typename T, int BM, int NB, bool PH, bool SPLIT = false>
__global__ __launch_bounds__(kCA_T) void conv_any_fwd_k(const T* __restrict__ x, const T* __restrict__ w,
                                                        const T* __restrict__ bias, T* __restrict__ y, AnyGeom g) {
  constexpr int LD = kCA_KC + 8;
  constexpr int TM = BM / 16;
  constexpr int BN = kCA_BN * NB;
  constexpr int AE = BM * kCA_KC / kCA_T;  // weight elements per thread per chunk
  constexpr int CL = BM + 8;               // row pitch of the staged [BN][BM] output tile
  constexpr int SMEM = (BM + BN) * LD > BN * CL ? (BM + BN) * LD : BN * CL;
  __shared__ __attribute__((aligned(16))) T smem[SMEM];  // operand tiles As | Bs, reused by the epilogue's output staging
  T (*As)[LD] = reinterpret_cast<T (*)[LD]>(smem);
  T (*Bs)[LD] = reinterpret_cast<T (*)[LD]>(smem + BM * LD);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntm = (g.K + BM - 1) / BM;
  const int tm = blockIdx.x % ntm;
  int64_t tile = blockIdx.x / ntm;
  const int m0 = tm * BM;
  const int Kfull = g.R * g.S * g.C;  // weight row length
  PhaseTile ph{0, 0, 0, 0, g.R, g.S};
  int64_t NPIX = (int64_t)g.N * g.P * g.Q;  // pixels of this tile's class
  if constexpr (PH) {
    NPIX = (int64_t)g.N * g.Pp * g.Qp;
    const int64_t tpp = (NPIX + BN - 1) / BN;
    const int c = (int)(tile / tpp);
    tile -= (int64_t)c * tpp;
    ph = phase_of(g, c);
  }
  const int64_t pix0 = tile * BN;
  const int Kred = ph.nr * ph.ns * g.C;
  const int nchunks = (Kred + kCA_KC - 1) / kCA_KC;

  // pixel index of the class -> (n, output row/col, real-input origin of tap (0, 0)); false if outside
  auto decode = [&](int64_t pix, int& n, int& p, int& q, int& h0, int& w0) -> bool {
    if (pix >= NPIX) return false;
    if constexpr (PH) {
      const int qq = (int)(pix % g.Qp);
      const int64_t t = pix / g.Qp;
      const int pp = (int)(t % g.Pp);
      n = (int)(t / g.Pp);
      p = ph.a + g.dil * pp;
      q = ph.b + g.dil * qq;
      h0 = (ph.a - g.pad + ph.r0) / g.dil + pp;  // exact: a - pad + r0 == 0 (mod dil)
      w0 = (ph.b - g.pad + ph.s0) / g.dil + qq;
      return p < g.P && q < g.Q;
    } else {
      q = (int)(pix % g.Q);
      const int64_t t = pix / g.Q;
      p = (int)(t % g.P);
      n = (int)(t / g.P);
      h0 = p * g.st - g.pad;
      w0 = q * g.st - g.pad;
      return true;
    }
  };

  // this thread's B-tile pixels (bp + 64 j) and reduction sub-range
  const int bp = tid >> 2, bk = (tid & 3) * 8;
  int n[NB], hv0[NB], wv0[NB];
  bool pv[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    int pp_, qq_;
    n[j] = hv0[j] = wv0[j] = 0;
    pv[j] = decode(pix0 + bp + kCA_BN * j, n[j], pp_, qq_, hv0[j], wv0[j]);
  }
  // this thread's weight column (tid % 32 for every AE element: 256 % KC == 0)
  const int acol = tid % kCA_KC;
  float bv[NB][8], av[AE];
  auto load = [&](int ch) {
    const int kk0 = ch * kCA_KC;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (pv[j]) {
        if constexpr (PH) gather8_ph(x, g, n[j], hv0[j], wv0[j], ph.ns, kk0 + bk, Kred, bv[j]);
        else gather8(x, g, n[j], hv0[j], wv0[j], kk0 + bk, Kred, bv[j]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[j][e] = 0.f;
      }
    }
    const int kk = kk0 + acol;
    int woff = kk;
    if constexpr (PH) {  // (r', s', c) of the class -> the full weight row's (r0 + D r', s0 + D s', c)
      const int rs = kk / g.C, c = kk - rs * g.C;
      const int r = rs / ph.ns, s = rs - r * ph.ns;
      woff = ((ph.r0 + g.dil * r) * g.S + ph.s0 + g.dil * s) * g.C + c;
    }
#pragma unroll
    for (int i = 0; i < AE; ++i) {
      const int k = m0 + (tid + kCA_T * i) / kCA_KC;
      av[i] = (k < g.K && kk < Kred) ? ldf(w, (int64_t)k * Kfull + woff) : 0.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = bp + kCA_BN * j;
      if constexpr (sizeof(T) == 2) {  // one 16-B LDS store for the 8 gathered values
        uint32_t u[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = (uint32_t)f2bf(bv[j][2 * e]) | ((uint32_t)f2bf(bv[j][2 * e + 1]) << 16);
        *reinterpret_cast<uint4*>(&Bs[row][bk]) = make_uint4(u[0], u[1], u[2], u[3]);
      } else {
        *reinterpret_cast<float4*>(&Bs[row][bk]) = make_float4(bv[j][0], bv[j][1], bv[j][2], bv[j][3]);
        *reinterpret_cast<float4*>(&Bs[row][bk + 4]) = make_float4(bv[j][4], bv[j][5], bv[j][6], bv[j][7]);
      }
    }
#pragma unroll
    for (int i = 0; i < AE; ++i) {
      const int e = tid + kCA_T * i;
      As[e / kCA_KC][e % kCA_KC] = to_t<T>(av[i]);
    }
  };

  f32x4_t acc[NB][TM];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  load(0);
  for (int ch = 0; ch < nchunks; ++ch) {
    __syncthreads();  // previous chunk's fragments read
    store();
    __syncthreads();
    if (ch + 1 < nchunks) load(ch + 1);  // next chunk's gathers in flight during the MFMAs
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = kCA_BN * j + wave * 16 + fr;  // this lane's pixel row of the B tile
      if constexpr (sizeof(T) == 2) {
        const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(&Bs[col][fq * 8]);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&As[i * 16 + fr][fq * 8]);
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j][i], 0, 0, 0);
        }
      } else {
        // the 8 MFMAs of a chunk take k = 8 fq + e (a permutation of the reduction, the same
        // for both operands): each lane's operands are 8 contiguous floats, two 16-B LDS reads
        const float4 b0 = *reinterpret_cast<const float4*>(&Bs[col][fq * 8]);
        const float4 b1 = *reinterpret_cast<const float4*>(&Bs[col][fq * 8 + 4]);
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        bf16x8_t bh, bl;
        if constexpr (SPLIT) split8(bb, bh, bl);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float4 a0 = *reinterpret_cast<const float4*>(&As[i * 16 + fr][fq * 8]);
          const float4 a1 = *reinterpret_cast<const float4*>(&As[i * 16 + fr][fq * 8 + 4]);
          const float aa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
          if constexpr (SPLIT) {  // lane's 8 values are k = 8 fq + e: the bf16 MFMA's own layout
            bf16x8_t ah, al;
            split8(aa, ah, al);
            acc[j][i] = mfma_split(ah, al, bh, bl, acc[j][i]);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa[e], bb[e], acc[j][i], 0, 0, 0);
          }
        }
      }
    }
  }
  // lane holds channels m0 + 16 i + 4 fq + (0..3) of pixel pix0 + 64 j + 16 wave + fr
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  if ((g.K & 7) == 0) {
    // staged through LDS (the B tile's space) so every lane stores 16 contiguous bytes of
    // an output row: the 2-byte scattered stores of the direct path ran at ~0.5 TB/s
    T (*Cst)[CL] = reinterpret_cast<T (*)[CL]>(smem);
    __syncthreads();  // last chunk's fragments read
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kl = i * 16 + fq * 4 + e;
          float v = acc[j][i][e];
          if (bias && m0 + kl < g.K) v += ldf(bias, m0 + kl);
          Cst[kCA_BN * j + wave * 16 + fr][kl] = to_t<T>(v);
        }
    __syncthreads();
    constexpr int VE = 16 / sizeof(T);  // elements per 16-B vector
    constexpr int VPR = BM / VE;        // vectors per staged row
    for (int v = tid; v < BN * VPR; v += kCA_T) {
      const int row = v / VPR, kl = (v - row * VPR) * VE;
      if (m0 + kl >= g.K) continue;  // (K % 8 == 0: a vector is all in or all out)
      int on, op_, oq, oh, ow;
      if (!decode(pix0 + row, on, op_, oq, oh, ow)) continue;
      const int64_t o = (((int64_t)on * g.P + op_) * g.Q + oq) * g.K + m0 + kl;
      if (TB_BOUNDS_OK(o + VE <= NPQ * g.K, kBndAnyDst))
        *reinterpret_cast<uint4*>(y + o) = *reinterpret_cast<const uint4*>(&Cst[row][kl]);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    int on, op_, oq, oh, ow;
    if (!decode(pix0 + kCA_BN * j + wave * 16 + fr, on, op_, oq, oh, ow)) continue;
    const int64_t op = ((int64_t)on * g.P + op_) * g.Q + oq;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = m0 + i * 16 + fq * 4 + e;
        if (k >= g.K) continue;
        float v = acc[j][i][e];
        if (bias) v += ldf(bias, k);
        if (TB_BOUNDS_OK(op * g.K + k < NPQ * g.K, kBndAnyDst)) y[op * g.K + k] = to_t<T>(v);
      }
    }
  }
}

// ---------------------------------------------------------------- weight gradient
// dW[k][kk] (f32 partials per pixel split): A = dy^T [k][pix], B = xv^T [kk][pix], reduction
// over pixels in stages of kWU x 32 (kWU MFMA k-steps per barrier pair, kWU gathers per
// thread in flight); LDS tiles are written transposed so fragment rows are contiguous
constexpr int kWU = 4;
template <typename T, int BM, bool SPLIT = false>
__global__ __launch_bounds__(kCA_T) void conv_any_wgrad_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                          float* __restrict__ part, AnyGeom g, int64_t pix_per) {
  constexpr int KP = kCA_KC * kWU;  // pixels per stage
  constexpr int LD = KP + 8;
  constexpr int TM = BM / 16;
  constexpr int BNK = 64;  // reduction-index (r, s, c) columns per tile
  __shared__ T As[BM][LD];   // [k][pix]
  __shared__ T Bs[BNK][LD];  // [kk][pix]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int Kred = g.R * g.S * g.C;
  const int ntm = (g.K + BM - 1) / BM;
  const int tm = blockIdx.x % ntm, tn = blockIdx.x / ntm;
  const int m0 = tm * BM, kk0 = tn * BNK;
  const int64_t pb = (int64_t)blockIdx.y * pix_per;
  const int64_t pe = min(NPQ, pb + pix_per);

  // B staging: thread -> pixels (tid & 31) + 32 u, 8 consecutive kk at kk0 + (tid >> 5) * 8
  const int sp = tid & 31, skk = (tid >> 5) * 8;
  // A staging: the same pixels, BM/8 consecutive channels at (tid >> 5) * (BM / 8)
  constexpr int AK = BM / 8;
  const int sak = (tid >> 5) * AK;
  const bool avec = sizeof(T) == 2 && AK == 8 && (g.K & 7) == 0 && m0 + sak + 8 <= g.K;  // one 16-B dy load
  float bv[kWU][8], av[kWU][AK];
  auto load = [&](int64_t p0) {
#pragma unroll
    for (int u = 0; u < kWU; ++u) {
      const int64_t pix = p0 + u * kCA_KC + sp;
      if (pix < pe) {
        const int q = (int)(pix % g.Q);
        const int64_t t = pix / g.Q;
        const int p = (int)(t % g.P), n = (int)(t / g.P);
        gather8(x, g, n, p * g.st - g.pad, q * g.st - g.pad, kk0 + skk, Kred, bv[u]);
        if (avec) {
          const uint4 v = *reinterpret_cast<const uint4*>(dy + pix * g.K + m0 + sak);
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            av[u][2 * e] = bf2f((uint16_t)(w4[e] & 0xffff));
            av[u][2 * e + 1] = bf2f((uint16_t)(w4[e] >> 16));
          }
        } else {
#pragma unroll
          for (int e = 0; e < AK; ++e) {
            const int k = m0 + sak + e;
            av[u][e] = k < g.K ? ldf(dy, pix * g.K + k) : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[u][e] = 0.f;
#pragma unroll
        for (int e = 0; e < AK; ++e) av[u][e] = 0.f;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < kWU; ++u) {
#pragma unroll
      for (int e = 0; e < 8; ++e) Bs[skk + e][u * kCA_KC + sp] = to_t<T>(bv[u][e]);
#pragma unroll
      for (int e = 0; e < AK; ++e) As[sak + e][u * kCA_KC + sp] = to_t<T>(av[u][e]);
    }
  };
  f32x4_t acc[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  if (pb < pe) load(pb);
  for (int64_t p0 = pb; p0 < pe; p0 += KP) {
    __syncthreads();
    store();
    __syncthreads();
    if (p0 + KP < pe) load(p0 + KP);
    const int col = wave * 16 + fr;  // kk row of the B tile
#pragma unroll
    for (int u = 0; u < kWU; ++u) {
      const int pc = u * kCA_KC + fq * 8;
      if constexpr (sizeof(T) == 2) {
        const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(&Bs[col][pc]);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&As[i * 16 + fr][pc]);
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
        }
      } else {
        // the 8 MFMAs of a 32-pixel step take k = 8 fq + j (a permutation of the reduction,
        // the same for both operands): each lane's operands are 8 contiguous floats
        const float4 b0 = *reinterpret_cast<const float4*>(&Bs[col][pc]);
        const float4 b1 = *reinterpret_cast<const float4*>(&Bs[col][pc + 4]);
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        bf16x8_t bh, bl;
        if constexpr (SPLIT) split8(bb, bh, bl);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float4 a0 = *reinterpret_cast<const float4*>(&As[i * 16 + fr][pc]);
          const float4 a1 = *reinterpret_cast<const float4*>(&As[i * 16 + fr][pc + 4]);
          const float aa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
          if constexpr (SPLIT) {
            bf16x8_t ah, al;
            split8(aa, ah, al);
            acc[i] = mfma_split(ah, al, bh, bl, acc[i]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa[j], bb[j], acc[i], 0, 0, 0);
          }
        }
      }
    }
  }
  const int kk = kk0 + wave * 16 + fr;
  if (kk >= Kred) return;
  float* pp = part + (int64_t)blockIdx.y * g.K * Kred;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = m0 + i * 16 + fq * 4 + e;
      if (k < g.K) pp[(int64_t)k * Kred + kk] = acc[i][e];
    }
}

// sum the [splits][n] partials: 64 columns x 16 split groups per workgroup, merged through
// LDS in a fixed order (deterministic).  One thread per column walking all splits serially
// was latency-bound: ~120 us for a 64 x 48 dW over 512 splits.
constexpr int kWrG = 16;
template <typename T>
__global__ __launch_bounds__(64 * kWrG) void conv_any_wreduce_k(const float* __restrict__ part, int splits, int64_t n,
                                                                T* __restrict__ out) {
  __shared__ float red[kWrG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + tx;
  float s = 0.f;
  if (i < n) {
#pragma unroll 4
    for (int j = ty; j < splits; j += kWrG) s += part[(int64_t)j * n + i];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < kWrG; ++r) t += red[r][tx];
    out[i] = to_t<T>(t);
  }
}

// ---------------------------------------------------------------- input-gradient fold
// dx[n, h, w, c] = sum of dXp over the padded-virtual positions that read x[n, h, w, c]:
// virtual rows hv in [h*U, h*U + U) (upsample), each at padded row hv + pad and, with
// reflect padding, at its mirror images pad - hv (1 <= hv <= pad) and
// pad + 2 (Hv - 1) - hv (Hv - 1 - pad <= hv <= Hv - 2); rows beyond the dgrad grid Hg
// received no gradient
template <typename T, int V>
__global__ __launch_bounds__(256) void conv_any_fold_k(const T* __restrict__ dxp, int Hg, int Wg, AnyGeom g,
                                                       T* __restrict__ dx) {
  // V consecutive channels per thread (V = 8: 16-B bf16 / 2 x 16-B f32 vectors when C % 8 == 0)
  const int CV = g.C / V;
  const int64_t total = (int64_t)g.N * g.H * g.W * CV;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % CV) * V;
    int64_t t = i / CV;
    const int w = (int)(t % g.W);
    t /= g.W;
    const int h = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float s[V];
#pragma unroll
    for (int e = 0; e < V; ++e) s[e] = 0.f;
    for (int uy = 0; uy < g.up; ++uy) {
      const int hv = h * g.up + uy;
      int rows[3], nr = 0;
      rows[nr++] = hv + g.pad;
      if (g.reflect) {
        if (hv >= 1 && hv <= g.pad) rows[nr++] = g.pad - hv;
        if (hv <= g.Hv - 2 && hv >= g.Hv - 1 - g.pad) rows[nr++] = g.pad + 2 * (g.Hv - 1) - hv;
      }
      for (int ux = 0; ux < g.up; ++ux) {
        const int wv = w * g.up + ux;
        int cols[3], nc = 0;
        cols[nc++] = wv + g.pad;
        if (g.reflect) {
          if (wv >= 1 && wv <= g.pad) cols[nc++] = g.pad - wv;
          if (wv <= g.Wv - 2 && wv >= g.Wv - 1 - g.pad) cols[nc++] = g.pad + 2 * (g.Wv - 1) - wv;
        }
        for (int a = 0; a < nr; ++a) {
          if (rows[a] >= Hg) continue;
          for (int b = 0; b < nc; ++b) {
            if (cols[b] >= Wg) continue;
            const int64_t o = (((int64_t)n * Hg + rows[a]) * Wg + cols[b]) * g.C + c;
            if constexpr (V == 8 && sizeof(T) == 2) {
              const uint4 u = *reinterpret_cast<const uint4*>(dxp + o);
              const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                s[2 * e] += bf2f((uint16_t)(uu[e] & 0xffff));
                s[2 * e + 1] += bf2f((uint16_t)(uu[e] >> 16));
              }
            } else {
#pragma unroll
              for (int e = 0; e < V; ++e) s[e] += ldf(dxp, o + e);
            }
          }
        }
      }
    }
    const int64_t od = (((int64_t)n * g.H + h) * g.W + w) * g.C + c;
    if constexpr (V == 8 && sizeof(T) == 2) {
      uint32_t u[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) u[e] = (uint32_t)f2bf(s[2 * e]) | ((uint32_t)f2bf(s[2 * e + 1]) << 16);
      *reinterpret_cast<uint4*>(dx + od) = make_uint4(u[0], u[1], u[2], u[3]);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) dx[od + e] = to_t<T>(s[e]);
    }
  }
}

template <typename T>
void launch_fwd(const void* x, const void* w, const void* b, void* y, const AnyGeom& g, hipStream_t st) {
  const bool ph = g.dil > 1 && g.st == 1 && !g.reflect && g.up == 1;  // (every dgrad-as-forward)
  const int64_t npix = ph ? (int64_t)g.N * g.Pp * g.Qp : (int64_t)g.N * g.P * g.Q;
  const int nph = ph ? g.dil * g.dil : 1;
  auto go = [&](auto bm, auto nb) {
    constexpr int BM = decltype(bm)::value, NB = decltype(nb)::value;
    const int64_t ntn = ((npix + kCA_BN * NB - 1) / (kCA_BN * NB)) * nph;
    const int64_t grid = ((g.K + BM - 1) / BM) * ntn;
    const bool split = std::is_same<T, float>::value && g_f32_split;
    if (ph && split)
      conv_any_fwd_k<T, BM, NB, true, true>
          <<<(unsigned)grid, kCA_T, 0, st>>>((const T*)x, (const T*)w, (const T*)b, (T*)y, g);
    else if (ph)
      conv_any_fwd_k<T, BM, NB, true>
          <<<(unsigned)grid, kCA_T, 0, st>>>((const T*)x, (const T*)w, (const T*)b, (T*)y, g);
    else if (split)
      conv_any_fwd_k<T, BM, NB, false, true>
          <<<(unsigned)grid, kCA_T, 0, st>>>((const T*)x, (const T*)w, (const T*)b, (T*)y, g);
    else
      conv_any_fwd_k<T, BM, NB, false>
          <<<(unsigned)grid, kCA_T, 0, st>>>((const T*)x, (const T*)w, (const T*)b, (T*)y, g);
  };
  // narrow outputs take wider pixel tiles while there are >= 1024 of them (4 per CU)
  auto enough = [&](int nb) { return (npix + kCA_BN * nb - 1) / (kCA_BN * nb) * nph >= 1024; };
  using std::integral_constant;
  if (g.K <= 16) {
    if (enough(4)) go(integral_constant<int, 16>{}, integral_constant<int, 4>{});
    else go(integral_constant<int, 16>{}, integral_constant<int, 1>{});
  } else if (g.K <= 32) {
    if (enough(2)) go(integral_constant<int, 32>{}, integral_constant<int, 2>{});
    else go(integral_constant<int, 32>{}, integral_constant<int, 1>{});
  } else {
    go(integral_constant<int, 64>{}, integral_constant<int, 1>{});
  }
}

template <typename T>
void launch_wgrad(const void* x, const void* dy, float* part, int splits, void* dw, const AnyGeom& g,
                  hipStream_t st) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int Kred = g.R * g.S * g.C;
  int64_t per = (NPQ + splits - 1) / splits;
  per = (per + kCA_KC * kWU - 1) / (kCA_KC * kWU) * (kCA_KC * kWU);
  auto go = [&](auto bm) {
    constexpr int BM = decltype(bm)::value;
    const dim3 grid((unsigned)(((g.K + BM - 1) / BM) * ((Kred + 63) / 64)), (unsigned)splits);
    if (std::is_same<T, float>::value && g_f32_split)
      conv_any_wgrad_k<T, BM, true><<<grid, kCA_T, 0, st>>>((const T*)x, (const T*)dy, part, g, per);
    else
      conv_any_wgrad_k<T, BM><<<grid, kCA_T, 0, st>>>((const T*)x, (const T*)dy, part, g, per);
  };
  if (g.K <= 16) go(std::integral_constant<int, 16>{});
  else if (g.K <= 32) go(std::integral_constant<int, 32>{});
  else go(std::integral_constant<int, 64>{});
  const int64_t n = (int64_t)g.K * Kred;
  conv_any_wreduce_k<T><<<(unsigned)((n + 63) / 64), 64 * kWrG, 0, st>>>(part, splits, n, (T*)dw);
}

// debug-build plumbing probe: one guarded read with index `i` of an n-element buffer
__global__ void bounds_probe_k(const float* __restrict__ x, int64_t n, int64_t i, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = TB_BOUNDS_OK(i >= 0 && i < n, kBndAnySrc) ? x[i] : -1.f;
}

}  // namespace

void conv_any_set_f32_split(bool on) { g_f32_split = on; }
bool conv_any_f32_split() { return g_f32_split; }

void bounds_probe(const float* x, int64_t n, int64_t i, float* out, hipStream_t st) {
  bounds_probe_k<<<1, 64, 0, st>>>(x, n, i, out);
}

static AnyGeom any_geom(const ConvAnyShape& s) {
  AnyGeom g{s.N, s.H, s.W, s.C, s.K, s.R, s.S, s.P, s.Q, s.stride, s.pad, s.up, s.dil, s.reflect, 0, 0, 0, 0};
  g.Hv = s.dil > 1 ? (s.H - 1) * s.dil + 1 : s.H * s.up;
  g.Wv = s.dil > 1 ? (s.W - 1) * s.dil + 1 : s.W * s.up;
  g.Pp = (s.P + s.dil - 1) / s.dil;
  g.Qp = (s.Q + s.dil - 1) / s.dil;
  return g;
}

void conv_any_fwd(int f32, const void* x, const void* w, const void* bias, void* y, const ConvAnyShape& s,
                  hipStream_t st) {
  const AnyGeom g = any_geom(s);
  if ((int64_t)g.N * g.P * g.Q == 0 || g.K == 0) return;
  if (f32) launch_fwd<float>(x, w, bias, y, g, st);
  else launch_fwd<uint16_t>(x, w, bias, y, g, st);
}

int conv_any_wgrad_splits(const ConvAnyShape& s) {
  const int64_t NPQ = (int64_t)s.N * s.P * s.Q;
  const int64_t tiles = (int64_t)((s.K + 63) / 64) * ((s.R * s.S * s.C + 63) / 64);
  int64_t sp = (1024 + tiles - 1) / tiles;             // ~4 workgroups per CU
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, NPQ / 512));  // >= 4 stages per split
  return (int)std::max<int64_t>(1, std::min<int64_t>(sp, 512));
}

void conv_any_wgrad(int f32, const void* x, const void* dy, float* part, int splits, void* dw,
                    const ConvAnyShape& s, hipStream_t st) {
  const AnyGeom g = any_geom(s);
  if (f32) launch_wgrad<float>(x, dy, part, splits, dw, g, st);
  else launch_wgrad<uint16_t>(x, dy, part, splits, dw, g, st);
}

void conv_any_fold(int f32, const void* dxp, int Hg, int Wg, void* dx, const ConvAnyShape& s, hipStream_t st) {
  const AnyGeom g = any_geom(s);
  const bool v8 = g.C % 8 == 0;
  const int64_t total = (int64_t)g.N * g.H * g.W * (v8 ? g.C / 8 : g.C);
  if (total == 0) return;
  int64_t gs = (total + 255) / 256;
  if (gs > 8192) gs = 8192;
  auto go = [&](auto tv, auto vv) {
    using T = decltype(tv);
    constexpr int V = decltype(vv)::value;
    conv_any_fold_k<T, V><<<(unsigned)gs, 256, 0, st>>>((const T*)dxp, Hg, Wg, g, (T*)dx);
  };
  if (f32) {
    if (v8) go(float{}, std::integral_constant<int, 8>{});
    else go(float{}, std::integral_constant<int, 1>{});
  } else {
    if (v8) go(uint16_t{}, std::integral_constant<int, 8>{});
    else go(uint16_t{}, std::integral_constant<int, 1>{});
  }
}

}  // namespace tbamd
