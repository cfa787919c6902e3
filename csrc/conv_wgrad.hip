// Weight gradient of the NHWC convolution on gfx950 MFMA.
//
//   dW[k][r][s][c] = sum_{n,p,q} dY[n,p,q,k] * X[n, p*st-pad+r, q*st-pad+s, c]
//
// is a GEMM with M = K (out channels), N = R*S*C (weight columns, the
// channels_last weight layout) and a reduction over every output pixel
// (N*P*Q — 800k for ResNet-50's first stage at batch 256).  Both operands are
// stored with the REDUCTION dimension strided (dY rows are pixels holding K
// contiguous channels, X rows are pixels holding C contiguous channels), so
// the tiles are staged pixel-major into LDS with direct-to-LDS loads and the
// MFMA operands are produced by gfx950's transposing LDS read
// (ds_read_b64_tr_b16, cdna_hip_programming.md §5.5 T10): 4 pixel rows x 16
// channels per 16-lane group, delivered column-major.
//
// LDS image: [64 pixel rows][BM or BN bf16], 32-byte slots XOR-swizzled by a
// row function chosen so each 32-lane half of a transposing read (rows
// 8g+q and 8(g+1)+q, q = 0..3) hits 8 distinct 32-byte bank slots:
//   256-B rows: slot ^= (row & 3) | ((row >> 3) & 1) << 2
//   128-B rows: slot ^= ((row >> 1) & 1) | ((row >> 3) & 1) << 1   (2 rows per bank window)
// The direct-to-LDS loads are lane-linear in LDS, so the global source of each
// lane is pre-swizzled instead (rule 21).
//
// The reduction is split over `splits` pixel ranges (enough workgroups to fill
// 256 CUs even when M x N is one tile); partial f32 tiles are summed by a
// second, deterministic kernel that also rounds to bf16.  Workgroups of one
// pixel range are placed on one XCD so its L2 serves the dY/X rows that all
// the (k, rsc) tiles of that range re-read.
//
// Reference parity: the conv weight gradients of every example model
// (cuDNN wgrad behind torch.nn.Conv2d in the reference).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "tbamd.h"
#include "xf.h"

namespace tbamd {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

__device__ __attribute__((aligned(64))) uint4 g_wgrad_zero_page[16];

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// exact unsigned division by a runtime constant for n < 2^31
struct FastDiv {
  uint32_t mul;
  uint32_t shift;
  uint32_t d;
};

static FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{(uint32_t)m, l, d};
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.mul) + n) >> f.shift;
}

struct WgradGeom {
  int N, H, W, C, K, R, S, P, Q, st, pad;
  int ncol;        // R*S*C
  int npq;         // N*P*Q (< 2^31)
  int pix_split;   // pixels per split (multiple of 64)
  int splits;
  FastDiv fq, fp;  // divide by Q, by P
  // VIRT kernels only: x is read through pad(upsample_nearest(x, 2^upsh)), zero or reflect
  int upsh, reflect, Hv, Wv;
};

// swizzled 16-byte chunk of a row: ROWB = bytes per LDS row (64, 128 or 256).  64-B rows
// (32-channel dY tiles of narrow-output convs): rows r and r+4 share a bank window, so the
// 32-B slot flips with bit 3 of the row -- rows 8g+q of the two 16-lane groups of a half differ
template <int ROWB>
__device__ __forceinline__ int wz(int row) {
  if constexpr (ROWB == 256) return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  else if constexpr (ROWB == 128) return ((((row >> 1) & 1) | (((row >> 3) & 1) << 1))) << 1;
  else return ((row >> 3) & 1) << 1;
}

// transposed fragment read: lane (g = l>>4, q = (l>>2)&3, p = l&3) supplies row
// 8g + q (+4 for the second half) of the k-step and columns cb + 4p .. cb + 4p + 3
template <int ROWB>
__device__ __forceinline__ bf16x8_t tr_frag(const char* base, int ks, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lc = (cb >> 3) + (p >> 1);
  const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
  const int o0 = r0 * ROWB + ((lc ^ wz<ROWB>(r0)) << 4) + ((p & 1) << 3);
  const int o1 = r1 * ROWB + ((lc ^ wz<ROWB>(r1)) << 4) + ((p & 1) << 3);
  const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + o0));
  const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + o1));
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  const s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

constexpr int kWgThreads = 256;
// pixels per k-iteration.  One LDS stage, no prefetch ring: a 2-stage glds ring (-2.2 % on the
// ResNet-50 step) and 128-pixel k-tiles (-1 %) both made the step slower -- a faster weight gradient
// takes more of the bandwidth the compute stream's chain needs (profiles/r05_wgrad); removed.
constexpr int kWgBK = 64;

// XF: x is the INPUT of a BatchNorm + ReLU whose output the conv consumed (csrc/xf.h): each lane
// applies the transform to its own staged X chunks (8 channels, the same for all of its passes)
template <int BM, int BN, bool FINAL, int OCC = 2, bool STEM = false, bool VIRT = false, bool XF = false>
__global__ __launch_bounds__(kWgThreads, OCC) void conv_wgrad_k(const uint16_t* __restrict__ dy,
                                                              const uint16_t* __restrict__ x,
                                                              float* __restrict__ part,
                                                              uint16_t* __restrict__ dw, WgradGeom g,
                                                              XfArgs xf = XfArgs{}) {
  static_assert(!XF || (!STEM && !VIRT), "XF: plain weight gradient");
  constexpr int BK = kWgBK;
  constexpr int ROWA = BM * 2, ROWB = BN * 2;  // bytes per LDS row
  constexpr int CPA = BM / 8, CPB = BN / 8;    // 16-B chunks per row
  constexpr int A_PASSES = BK * CPA / kWgThreads, B_PASSES = BK * CPB / kWgThreads;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int STAGE = BK * (ROWA + ROWB);  // bytes
  __shared__ __attribute__((aligned(16))) char lds[STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntm = g.K / BM, ntn = g.ncol / BN, ntiles = ntm * ntn;
  const int nwg = ntiles * g.splits;
  int bid = blockIdx.x;
  {
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  const int split = bid / ntiles, tile = bid - split * ntiles;
  const int tile_m = tile % ntm, tile_n = tile / ntm;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int pb = split * g.pix_split;
  const int pe = min(pb + g.pix_split, g.npq);
  const int KT = (pe - pb + BK - 1) / BK;

  // per-pass lane geometry (fixed for the whole kernel: the row of a lane and
  // therefore its column chunk never change, only the pixel advances)
  const uint16_t* asrc[A_PASSES];
  int arow[A_PASSES];
#pragma unroll
  for (int i = 0; i < A_PASSES; ++i) {
    const int row = i * (kWgThreads / CPA) + wave * (64 / CPA) + lane / CPA;
    const int lc = (lane % CPA) ^ wz<ROWA>(row);
    arow[i] = row;
    asrc[i] = dy + m0 + lc * 8;
  }
  int brow[B_PASSES], bdr[B_PASSES], bds[B_PASSES], bc[B_PASSES];
#pragma unroll
  for (int i = 0; i < B_PASSES; ++i) {
    const int row = i * (kWgThreads / CPB) + wave * (64 / CPB) + lane / CPB;
    const int lc = (lane % CPB) ^ wz<ROWB>(row);
    const int col = n0 + lc * 8;  // weight column (r, s, c) of this chunk
    const int c = col % g.C, rs = col / g.C;
    brow[i] = row;
    bdr[i] = rs / g.S - g.pad;
    bds[i] = rs % g.S - g.pad;
    bc[i] = c;
    if constexpr (STEM) {  // packed column r*32 + s*4 + c: chunk = window row r, pixels s, s+1, 4 ch each
      bdr[i] = col >> 5;
      bds[i] = (col & 31) >> 2;
      bc[i] = 0;
    }
  }

  const void* zpage = pin_sgpr(g_wgrad_zero_page);
  uint32_t bvalid = 0u;  // XF: which of this lane's X chunks of the staged k-tile hold real pixels
  float xsc[XF ? 8 : 1], xsh[XF ? 8 : 1];
  if constexpr (XF) {
    float sc8[8], sh8[8];
    xf_load(xf, bc[0], sc8, sh8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xsc[e] = sc8[e];
      xsh[e] = sh8[e];
    }
  }
  auto issue = [&](int kt, int buf) {
    char* A = lds + buf * STAGE;
    char* B = A + BK * ROWA;
    const int p0 = pb + kt * BK;
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      const int pix = p0 + arow[i];
      const void* src = pix < pe ? (const void*)(asrc[i] + (int64_t)pix * g.K) : zpage;
      glds16(src, A + (i * kWgThreads + wave * 64) * 16);
    }
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      const int pix = p0 + brow[i];
      const void* src = zpage;
      if (pix < pe) {
        const uint32_t t = fdiv((uint32_t)pix, g.fq);
        const int q = pix - (int)t * g.Q;
        const uint32_t n = fdiv(t, g.fp);
        const int p = (int)t - (int)n * g.P;
        const int h = p * g.st + bdr[i], w = q * g.st + bds[i];
        if constexpr (STEM) {  // pre-padded image: always in bounds (conv.hip stem_dims)
          src = x + (((int64_t)n * g.H + h) * g.W + w) * 4;
        } else if constexpr (VIRT) {  // padded-virtual (h, w): mirror or zero, then the upsampled source
          const int vh = g.reflect ? (h < 0 ? -h : (h >= g.Hv ? 2 * g.Hv - 2 - h : h)) : h;
          const int vw = g.reflect ? (w < 0 ? -w : (w >= g.Wv ? 2 * g.Wv - 2 - w : w)) : w;
          if ((unsigned)vh < (unsigned)g.Hv && (unsigned)vw < (unsigned)g.Wv)
            src = x + (((int64_t)n * g.H + (vh >> g.upsh)) * g.W + (vw >> g.upsh)) * g.C + bc[i];
        } else if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W) {
          src = x + (((int64_t)n * g.H + h) * g.W + w) * g.C + bc[i];
        }
      }
      glds16(src, B + (i * kWgThreads + wave * 64) * 16);
      if constexpr (XF) {
        if (i == 0) bvalid = 0u;
        bvalid |= (uint32_t)(src != zpage) << i;
      }
    }
  };
  auto xform = [&](int buf) {
    if constexpr (XF) {
      char* B = lds + buf * STAGE + BK * ROWA;
      float sc8[8], sh8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc8[e] = xsc[e];
        sh8[e] = xsh[e];
      }
#pragma unroll
      for (int i = 0; i < B_PASSES; ++i) {
        if (!((bvalid >> i) & 1u)) continue;
        uint4* p = reinterpret_cast<uint4*>(B + (i * kWgThreads + wave * 64) * 16) + lane;
        *p = xf_chunk(*p, sc8, sh8);
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // single LDS buffer: more resident workgroups instead of prefetch depth
  for (int kt = 0; kt < KT; ++kt) {
    issue(kt, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    xform(0);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_frag<ROWA>(lds, ks, wm * WM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tr_frag<ROWB>(lds + BK * ROWA, ks, wn * WN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // D[m][n]: lane holds rows (lane>>4)*4 + e, column lane & 15
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wm * WM + i * 16 + fq * 4 + e;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + fr;
        if constexpr (FINAL) dw[(int64_t)m * g.ncol + n] = f2bf(acc[i][j][e]);
        else part[((int64_t)split * g.K + m) * g.ncol + n] = acc[i][j][e];
      }
    }
}

// dw = bf16(sum over splits of part).  A workgroup owns 64 consecutive
// outputs (16 float4 columns) and spreads the splits over 16 lanes per column,
// so even a 64x64 weight with hundreds of splits keeps thousands of loads in
// flight; the 16 lane sums are merged in a fixed order (deterministic).
constexpr int kRedCols = 16, kRedLanes = 16;
template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce_k(const float* __restrict__ part, int splits, int64_t total,
                                                      OutT* __restrict__ dw) {
  __shared__ float4 red[kRedLanes][kRedCols];
  const int tx = threadIdx.x % kRedCols, ty = threadIdx.x / kRedCols;
  const int64_t i4 = ((int64_t)blockIdx.x * kRedCols + tx) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < total) {
    int k = ty;
#pragma unroll 1
    for (; k + 3 * kRedLanes < splits; k += 4 * kRedLanes) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(part + (int64_t)(k + u * kRedLanes) * total + i4);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s.x += v[u].x;
        s.y += v[u].y;
        s.z += v[u].z;
        s.w += v[u].w;
      }
    }
    for (; k < splits; k += kRedLanes) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)k * total + i4);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && i4 < total) {
    for (int j = 1; j < kRedLanes; ++j) {
      const float4 v = red[j][tx];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<float4*>(dw + i4) = s;
    } else {
      const uint32_t lo = (uint32_t)f2bf(s.x) | ((uint32_t)f2bf(s.y) << 16);
      const uint32_t hi = (uint32_t)f2bf(s.z) | ((uint32_t)f2bf(s.w) << 16);
      *reinterpret_cast<uint2*>(dw + i4) = make_uint2(lo, hi);
    }
  }
}

// f32 -> (hi, lo) bf16 pair, hi = RNE(v), lo = RNE(v - hi): hi*a + hi*b-style products of the pairs
// carry ~16 mantissa bits (the split-bf16 scheme of csrc/conv_any.hip's fp32 path)
__global__ __launch_bounds__(256) void split_bf16_k(const float* __restrict__ v, int64_t n4, uint16_t* __restrict__ hi,
                                                    uint16_t* __restrict__ lo) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 a = reinterpret_cast<const float4*>(v)[i];
    const float f[4] = {a.x, a.y, a.z, a.w};
    uint16_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      h[e] = f2bf(f[e]);
      l[e] = f2bf(f[e] - bf2f(h[e]));
    }
    reinterpret_cast<uint2*>(hi)[i] = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
    reinterpret_cast<uint2*>(lo)[i] = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
  }
}

// tuning override (0 = default: 2 workgroups/CU).  Occupancy 2 instead of 3: the weight gradients
// share the chip with the compute stream's input-gradient / BatchNorm chain, and skipping them
// outright makes the ResNet-50 step 20 % faster (diagnostic, gpurun_out/r5_22) -- fewer resident
// weight-gradient workgroups per CU leave that chain more room: +1.0-1.6 % on the step
// (scripts/r5/gpu23-25.sh, profiles/r05_wgrad/)
int g_wgrad_occ = 0;

template <int BM, int BN, int OCC>
void launch_wgrad_s(const uint16_t* dy, const uint16_t* x, float* part, uint16_t* dw, const WgradGeom& g,
                    hipStream_t st) {
  const int nwg = (g.K / BM) * (g.ncol / BN) * g.splits;
  if (g.splits == 1)
    conv_wgrad_k<BM, BN, true, OCC><<<nwg, kWgThreads, 0, st>>>(dy, x, part, dw, g);
  else
    conv_wgrad_k<BM, BN, false, OCC><<<nwg, kWgThreads, 0, st>>>(dy, x, part, dw, g);
}

template <int BM, int BN>
void launch_wgrad(const uint16_t* dy, const uint16_t* x, float* part, uint16_t* dw, const WgradGeom& g,
                  hipStream_t st) {
  switch (g_wgrad_occ) {
    case 3: launch_wgrad_s<BM, BN, 3>(dy, x, part, dw, g, st); break;
    case 4: launch_wgrad_s<BM, BN, 4>(dy, x, part, dw, g, st); break;
    default: launch_wgrad_s<BM, BN, 2>(dy, x, part, dw, g, st);
  }
}

WgradGeom plan_wgrad(int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad) {
  WgradGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.P = P, g.Q = Q, g.st = stride, g.pad = pad;
  g.ncol = R * S * C;
  g.npq = N * P * Q;
  const int BM = K % 128 == 0 ? 128 : (K % 64 == 0 ? 64 : 32);
  const int BN = g.ncol % 128 == 0 ? 128 : 64;
  const int64_t tiles = (int64_t)(K / BM) * (g.ncol / BN);
  const int bk = kWgBK;
  const int64_t kiters = (g.npq + bk - 1) / bk;
  // about one full wave of resident workgroups (single-stage kernels: 3-4 per CU);
  // TBAMD_WGRAD_WAVES=f scales it (A/B: fewer splits = less split-K partial traffic for the
  // reduce, fewer workgroups beside the compute stream's kernels)
  static const double waves = [] {
    const char* e = getenv("TBAMD_WGRAD_WAVES");
    const double v = e ? atof(e) : 1.0;
    return v > 0.0 && v <= 8.0 ? v : 1.0;
  }();
  const int64_t target = (int64_t)(((BM == 128 && BN == 128) ? 768 : 1024) * waves);
  int64_t splits = (target + tiles - 1) / tiles;
  splits = std::min<int64_t>(splits, std::max<int64_t>(g.npq / 1024, 1));  // >= 1024 pixels each
  // partials <= TBAMD_WGRAD_CAP_MB (32) MiB: the split-K slabs are written and read back once each
  static const int64_t cap_mb = [] {
    const char* e = getenv("TBAMD_WGRAD_CAP_MB");
    const int64_t v = e ? atoll(e) : 32;
    return v >= 1 && v <= 1024 ? v : 32;
  }();
  const int64_t cap = (cap_mb << 20) / ((int64_t)K * g.ncol * 4);
  splits = std::max<int64_t>(1, std::min(splits, std::max<int64_t>(cap, 1)));
  const int64_t per = ((kiters + splits - 1) / splits) * bk;
  g.pix_split = (int)per;
  g.splits = (int)((g.npq + per - 1) / per);
  g.fq = make_fastdiv((uint32_t)Q);
  g.fp = make_fastdiv((uint32_t)P);
  return g;
}

}  // namespace

// stem weight gradient [K][256] (packed like the forward's weights) from dy [N*P*Q][K] and
// the pre-padded image [N][Hp][Wp][4]: columns are (window row r, tap s, channel c)
int64_t conv_stem_wgrad_workspace(int N, int Hp, int Wp, int K, int P, int Q) {
  const WgradGeom g = plan_wgrad(N, Hp, Wp, 4, K, 8, 8, P, Q, 2, 0);
  return g.splits > 1 ? (int64_t)g.splits * K * g.ncol : 0;
}

void conv_stem_wgrad(const void* dy, const void* xp, void* dwp, float* workspace, int N, int Hp, int Wp, int K,
                     int P, int Q, hipStream_t st) {
  const WgradGeom g = plan_wgrad(N, Hp, Wp, 4, K, 8, 8, P, Q, 2, 0);
  const uint16_t* d = (const uint16_t*)dy;
  const uint16_t* xx = (const uint16_t*)xp;
  uint16_t* o = (uint16_t*)dwp;
  const int nwg = (K / (K % 128 == 0 ? 128 : 64)) * (g.ncol / 128) * g.splits;
  if (K % 128 == 0) {
    if (g.splits == 1) conv_wgrad_k<128, 128, true, 3, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g);
    else conv_wgrad_k<128, 128, false, 3, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g);
  } else {
    if (g.splits == 1) conv_wgrad_k<64, 128, true, 3, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g);
    else conv_wgrad_k<64, 128, false, 3, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g);
  }
  if (g.splits > 1) {
    const int64_t total = (int64_t)K * g.ncol;
    wgrad_reduce_k<uint16_t><<<cdiv(total, 4 * kRedCols), kRedCols * kRedLanes, 0, st>>>(workspace, g.splits, total, o);
  }
}

// weight gradient of a conv over pad(upsample_nearest(x, up), pad, reflect|zero), up = 1, 2, 4
void conv_wgrad_virtual(const void* dy, const void* x, void* dw, float* workspace, int N, int H, int W, int C, int K,
                        int R, int S, int P, int Q, int stride, int pad, int up, int reflect, hipStream_t st) {
  WgradGeom g = plan_wgrad(N, H, W, C, K, R, S, P, Q, stride, pad);
  g.upsh = up == 4 ? 2 : (up == 2 ? 1 : 0);
  g.reflect = reflect ? 1 : 0;
  g.Hv = H * up;
  g.Wv = W * up;
  const uint16_t* d = (const uint16_t*)dy;
  const uint16_t* xx = (const uint16_t*)x;
  uint16_t* o = (uint16_t*)dw;
  auto go = [&](auto bm, auto bn) {
    constexpr int BM = decltype(bm)::value, BN = decltype(bn)::value;
    const int nwg = (g.K / BM) * (g.ncol / BN) * g.splits;
    if (g.splits == 1)
      conv_wgrad_k<BM, BN, true, 3, false, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g);
    else
      conv_wgrad_k<BM, BN, false, 3, false, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g);
  };
  using std::integral_constant;
  const bool bm128 = K % 128 == 0, bn128 = g.ncol % 128 == 0;
  if (K % 64 != 0) go(integral_constant<int, 32>{}, integral_constant<int, 64>{});  // K = 32, 96, ...
  else if (bm128 && bn128) go(integral_constant<int, 128>{}, integral_constant<int, 128>{});
  else if (bm128) go(integral_constant<int, 128>{}, integral_constant<int, 64>{});
  else if (bn128) go(integral_constant<int, 64>{}, integral_constant<int, 128>{});
  else go(integral_constant<int, 64>{}, integral_constant<int, 64>{});
  if (g.splits > 1) {
    const int64_t total = (int64_t)K * g.ncol;
    wgrad_reduce_k<uint16_t><<<cdiv(total, 4 * kRedCols), kRedCols * kRedLanes, 0, st>>>(workspace, g.splits, total, o);
  }
}

// weight gradient of a conv over relu(x * scale + shift) (per channel of x), the transform applied
// to the staged X tiles (csrc/xf.h): single stage, 2 workgroups/CU (3 with TBAMD_WGRAD_OCC=3)
void conv_wgrad_xf(const void* dy, const void* x, void* dw, float* workspace, const float* scale, const float* shift,
                   int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad,
                   hipStream_t st) {
  const WgradGeom g = plan_wgrad(N, H, W, C, K, R, S, P, Q, stride, pad);
  const XfArgs xf{scale, shift};
  const uint16_t* d = (const uint16_t*)dy;
  const uint16_t* xx = (const uint16_t*)x;
  uint16_t* o = (uint16_t*)dw;
  auto go = [&](auto bm, auto bn) {
    constexpr int BM = decltype(bm)::value, BN = decltype(bn)::value;
    const int nwg = (g.K / BM) * (g.ncol / BN) * g.splits;
    if (g_wgrad_occ == 3) {
      if (g.splits == 1)
        conv_wgrad_k<BM, BN, true, 3, false, false, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g, xf);
      else
        conv_wgrad_k<BM, BN, false, 3, false, false, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g, xf);
    } else if (g.splits == 1) {
      conv_wgrad_k<BM, BN, true, 2, false, false, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g, xf);
    } else {
      conv_wgrad_k<BM, BN, false, 2, false, false, true><<<nwg, kWgThreads, 0, st>>>(d, xx, workspace, o, g, xf);
    }
  };
  using std::integral_constant;
  const bool bm128 = K % 128 == 0, bn128 = g.ncol % 128 == 0;
  if (bm128 && bn128) go(integral_constant<int, 128>{}, integral_constant<int, 128>{});
  else if (bm128) go(integral_constant<int, 128>{}, integral_constant<int, 64>{});
  else if (bn128) go(integral_constant<int, 64>{}, integral_constant<int, 128>{});
  else go(integral_constant<int, 64>{}, integral_constant<int, 64>{});
  if (g.splits > 1) {
    const int64_t total = (int64_t)K * g.ncol;
    wgrad_reduce_k<uint16_t><<<cdiv(total, 4 * kRedCols), kRedCols * kRedLanes, 0, st>>>(workspace, g.splits, total, o);
  }
}

void conv_wgrad_set_occupancy(int o) { g_wgrad_occ = o; }

// fp32 weight gradient on the bf16 MFMA kernel: dy and x are split into bf16 (hi, lo) pairs and
// dW = dyh.xh + dyh.xl + dyl.xh (three passes of conv_wgrad_k into one f32 partial workspace of
// 3 x splits slabs, reduced in a fixed order to f32).  Shapes with C % 64 == K % 64 == 0, any
// stride, optionally over the virtual input pad(upsample(x)) (up = 1, 2, 4; reflect or zero).
// The reference's fp32 style-transfer convs (examples/img_stt/*.yml fp16: false) run there.
int64_t conv_wgrad_split32_workspace(int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride,
                                     int pad) {
  const WgradGeom g = plan_wgrad(N, H, W, C, K, R, S, P, Q, stride, pad);
  return 3ll * g.splits * K * g.ncol;  // floats
}

void conv_wgrad_split32(const float* dy, const float* x, float* dw, uint16_t* dyh, uint16_t* dyl, uint16_t* xh,
                        uint16_t* xl, float* part, int N, int H, int W, int C, int K, int R, int S, int P, int Q,
                        int stride, int pad, int up, int reflect, hipStream_t st) {
  const int64_t ndy = (int64_t)N * P * Q * K, nx = (int64_t)N * H * W * C;
  auto grid4 = [](int64_t n4) { return (int)std::min<int64_t>((n4 + 255) / 256, 8192); };
  split_bf16_k<<<grid4(ndy / 4), 256, 0, st>>>(dy, ndy / 4, dyh, dyl);
  split_bf16_k<<<grid4(nx / 4), 256, 0, st>>>(x, nx / 4, xh, xl);
  WgradGeom g = plan_wgrad(N, H, W, C, K, R, S, P, Q, stride, pad);
  const bool virt = up != 1 || reflect;
  g.upsh = up == 4 ? 2 : (up == 2 ? 1 : 0);
  g.reflect = reflect ? 1 : 0;
  g.Hv = H * up;
  g.Wv = W * up;
  const int64_t slab = (int64_t)g.splits * K * g.ncol;
  const uint16_t* A[3] = {dyh, dyh, dyl};
  const uint16_t* B[3] = {xh, xl, xh};
  auto go = [&](auto bm, auto bn) {
    constexpr int BM = decltype(bm)::value, BN = decltype(bn)::value;
    const int nwg = (g.K / BM) * (g.ncol / BN) * g.splits;
    for (int t = 0; t < 3; ++t) {
      if (virt)
        conv_wgrad_k<BM, BN, false, 3, false, true><<<nwg, kWgThreads, 0, st>>>(A[t], B[t], part + t * slab, nullptr, g);
      else
        conv_wgrad_k<BM, BN, false, 3><<<nwg, kWgThreads, 0, st>>>(A[t], B[t], part + t * slab, nullptr, g);
    }
  };
  using std::integral_constant;
  const bool bm128 = K % 128 == 0, bn128 = g.ncol % 128 == 0;
  if (bm128 && bn128) go(integral_constant<int, 128>{}, integral_constant<int, 128>{});
  else if (bm128) go(integral_constant<int, 128>{}, integral_constant<int, 64>{});
  else if (bn128) go(integral_constant<int, 64>{}, integral_constant<int, 128>{});
  else go(integral_constant<int, 64>{}, integral_constant<int, 64>{});
  const int64_t total = (int64_t)K * g.ncol;
  wgrad_reduce_k<float><<<cdiv(total, 4 * kRedCols), kRedCols * kRedLanes, 0, st>>>(part, 3 * g.splits, total, dw);
}

void split_bf16(const float* v, int64_t n, uint16_t* hi, uint16_t* lo, hipStream_t st) {
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  split_bf16_k<<<(int)std::min<int64_t>((n4 + 255) / 256, 8192), 256, 0, st>>>(v, n4, hi, lo);
}

int conv_wgrad_supported(int C, int K, int64_t NPQ) {
  return C % 64 == 0 && K % 64 == 0 && NPQ < (1ll << 31);
}

int64_t conv_wgrad_workspace(int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad) {
  const WgradGeom g = plan_wgrad(N, H, W, C, K, R, S, P, Q, stride, pad);
  return g.splits > 1 ? (int64_t)g.splits * K * g.ncol : 0;  // floats
}

void conv_wgrad(const void* dy, const void* x, void* dw, float* workspace, int N, int H, int W, int C, int K, int R,
                int S, int P, int Q, int stride, int pad, hipStream_t st) {
  const WgradGeom g = plan_wgrad(N, H, W, C, K, R, S, P, Q, stride, pad);
  const uint16_t* d = (const uint16_t*)dy;
  const uint16_t* xx = (const uint16_t*)x;
  uint16_t* o = (uint16_t*)dw;
  const bool bm128 = K % 128 == 0, bn128 = g.ncol % 128 == 0;
  if (bm128 && bn128) launch_wgrad<128, 128>(d, xx, workspace, o, g, st);
  else if (bm128) launch_wgrad<128, 64>(d, xx, workspace, o, g, st);
  else if (bn128) launch_wgrad<64, 128>(d, xx, workspace, o, g, st);
  else launch_wgrad<64, 64>(d, xx, workspace, o, g, st);
  if (g.splits > 1) {
    const int64_t total = (int64_t)K * g.ncol;  // multiple of 4096
    wgrad_reduce_k<uint16_t><<<cdiv(total, 4 * kRedCols), kRedCols * kRedLanes, 0, st>>>(workspace, g.splits, total, o);
  }
}

}  // namespace tbamd
