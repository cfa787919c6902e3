// Implicit-GEMM NHWC convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
// Reference: every conv of the examples goes through cuDNN (torchvision
// ResNet / VGG, StyleNet, AdaIN decoder).  Here:
//
//   y[n,p,q,k] = sum_{r,s,c} x[n, p*st-pad+r, q*st-pad+s, c] * w[k,r,s,c]
//
// is computed as D[k][pixel] = W[k][(r,s,c)] . Xcol[(r,s,c)][pixel] so that
// BOTH MFMA operands are read 16 B at a time along the reduction dimension
// (weights are [K][R][S][C], activations NHWC), and each lane's 4 accumulator
// rows are 4 consecutive output channels of one pixel (8-B NHWC stores).
//
// Tiling: BM (out channels) x BN (pixels) x BK=64 per workgroup, 4 waves in a
// 2x2 grid, each wave (BM/2)x(BN/2) as 16x16 MFMA tiles.  Operands are staged
// global -> LDS directly (global_load_lds, 16 B per lane, double buffered —
// single buffered for reductions of <= 2 k-tiles — one barrier per k-tile;
// the next tile's loads are in flight while the current one is multiplied).
// Out-of-image taps read a zero page instead of being masked.
// LDS rows are 128 B with the 16-B chunk index XOR-swizzled by (row>>1)&7, which
// makes every ds_read_b128 lane group conflict-free (4 cycles) — see
// cdna_hip_programming.md §5.5 T2.  Workgroups are remapped so the BM-tiles
// that share a pixel tile run on the same XCD (shared L2 for the activations).
//
// The epilogue optionally adds a bias, applies ReLU, and emits per-workgroup
// per-channel (sum, sum of squares) of the bf16 outputs: the BatchNorm
// statistics pass is fused into the conv (the BN kernels then skip one full
// read of the activation).
//
// Requirements (checked by the host): C % 64 == 0, K % BM == 0, bf16 data.
// dgrad of a stride-1 conv is the same kernel on dY with flipped/transposed
// weights (see ops/conv.py).
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "tbamd.h"
#include "xf.h"

namespace tbamd {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

struct ConvGeom {
  int N, H, W, C, K, R, S, P, Q, st, pad;
  // VIRT kernels only: the input is read through xv = pad(upsample_nearest(x, 2^upsh)),
  // zero or reflect padding (StyleNet / AdaIN ReflectionPad + Upsample + Conv, K16/K17)
  int upsh, reflect, Hv, Wv;
};

constexpr int kConvBK = 64;
constexpr int kStemKT = 4;  // stem reduction: 8 rows x 32 (7 taps x 4 ch, padded) = 256 = 4 k-tiles
constexpr int kConvThreads = 256;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// zero source for padded taps: out-of-image pixels are copied from here by the
// direct-to-LDS loads, so the staging path needs no per-lane select
__device__ __attribute__((aligned(64))) uint4 g_conv_zero_page[16];

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ uint32_t add_bf16x2(uint32_t a, uint32_t b) {
  const float lo = bf2f((uint16_t)(a & 0xffff)) + bf2f((uint16_t)(b & 0xffff));
  const float hi = bf2f((uint16_t)(a >> 16)) + bf2f((uint16_t)(b >> 16));
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// ADD: y = conv(x) + addend (same layout as y) — used by dgrad to fold in the
// gradient of a residual branch that shares the conv's input; ADD == 2 masks
// the addend with one bit per element ([pixel][K/8] bytes: a ReLU mask the BN
// forward saved, so that branch's gradient dy * mask is never materialised)
// BNB (dgrad only): the output dX is the upstream gradient of a BatchNorm(+act)
// whose input xb / coefficients are given; the epilogue also emits that BN's
// backward partial sums per pixel tile, [ntn][2][K] = (sum dz, sum dz*(xb-mean)),
// with dz = dX * act'(z): BNB 1 = ReLU mask recomputed as fma(xb,scale,shift) > 0,
// 2 = ReLU mask from saved bits, 3 = no activation.  The BN backward then
// skips its own partial pass over (dX, xb).
struct BnBwdEpi {
  const uint16_t* xb;
  const float* scale;
  const float* shift;
  const float* mean;
  const uint8_t* bits;
  float* part;
};

// GXF (1x1 stride-1 dgrad only): the dgrad's input is NOT the materialised BN input gradient but
// the BN OUTPUT gradient g of the BatchNorm(+ReLU) that consumed this conv's output; the BN
// backward apply  dX = ka[c] * act'(z) * g + c0[c] + c1[c] * xb  (xb: the BN input, i.e. this
// conv's forward output) runs on the operand as it lands in LDS (the lane that staged the 16-B
// chunk transforms it between its DMA wait and the barrier).  GXF 1: ReLU mask recomputed as
// fma(xb, scale, shift) > 0; 2: mask from the BN's saved bits ([pixel][C/8] bytes).  ``out``
// (optional): the workgroups of the first output-channel tile also store the transformed chunk,
// the materialised dX the weight gradient reads.  The BN backward then runs no apply pass.
struct GxfArgs {
  const uint16_t* xb;
  const uint8_t* bits;
  const float* scale;
  const float* shift;
  const float* coef;  // [3][C] = ka, c0, c1 (norm_bn.hip BwdFin)
  uint16_t* out;
};

// Stride-2 dgrad, one output parity class (a, b) per launch (sub-pixel decomposition):
// dX[n, 2i+a, 2j+b, c] = sum over the taps (r, s) with r = a + pad (mod 2), s = b + pad (mod 2)
// of dY[n, i + dr, j + ds, :] . W[:, r, s, c],  dr = (a + pad - r) / 2, ds = (b + pad - s) / 2.
// Every tap of the kernel is used by exactly one class: no work on the zeros a stride-1
// conv over the zero-dilated dY would multiply.
struct S2Cls {
  int a, b, ntap, st;  // (a, b): the class's output phase; st: the conv stride (2 or 3)
  int dr[16], ds[16], wrs[16];  // input offsets and flipped-weight tap index per class tap
  int H, W;                     // dX spatial dims (the output of this dgrad)
  int tile_base;                // first BN-partial row of this class (BNB: rows of all classes stacked)
};

// The stride^2 phase classes of one stride-2 or stride-3 dgrad in ONE launch (workgroups of class
// k are [wg_start[k], wg_start[k+1]) of the XCD-remapped grid): the small late layers (DCGAN 4x4
// and 8x8 maps, ResNet stage 4) fill 64-256 workgroups per class, a quarter of the chip each.
// (9 classes: the whole set stays inside the 4 KiB kernel-argument segment.)
constexpr int kS2MaxCls = 9;
struct S2Set {
  int ncls;
  int wg_start[kS2MaxCls + 1];
  ConvGeom g[kS2MaxCls];
  S2Cls c[kS2MaxCls];
};

// reflect a padded-virtual coordinate into [0, Hv) (zero padding: left as is, the caller's
// bounds test sends it to the zero page)
__device__ __forceinline__ int p_virt_h(int v, const ConvGeom& g) {
  return g.reflect ? (v < 0 ? -v : (v >= g.Hv ? 2 * g.Hv - 2 - v : v)) : v;
}
__device__ __forceinline__ int p_virt_w(int v, const ConvGeom& g) {
  return g.reflect ? (v < 0 ? -v : (v >= g.Wv ? 2 * g.Wv - 2 - v : v)) : v;
}

template <int BM, int BN, bool STATS, bool BIAS, bool RELU, int STAGES, int ADD, int OCC = 2, int BNB = 0,
          bool STEM = false, bool S2D = false, bool VIRT = false, int PRIO = 3, int GXF = 0>
__global__ __launch_bounds__(kConvThreads, OCC) void conv_fwd_k(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ w,
                                                              uint16_t* __restrict__ y,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ stats,
                                                              const uint16_t* __restrict__ addend,
                                                              const uint8_t* __restrict__ amask, ConvGeom g_in,
                                                              BnBwdEpi bnb = BnBwdEpi{},
                                                              std::conditional_t<S2D, S2Set, S2Cls> s2arg = {},
                                                              GxfArgs gxa = GxfArgs{}) {
  static_assert(!S2D || (ADD == 0 && !STATS && !STEM), "S2D: dgrad epilogue (optionally BN partials) only");
  static_assert(!VIRT || (!S2D && !STEM), "VIRT: plain forward addressing only");
  static_assert(GXF == 0 || (STAGES == 1 && !S2D && !STEM && !VIRT && !STATS),
                "GXF: single-stage 1x1 dgrad addressing only (host: R = S = 1, stride 1, pad 0)");
  constexpr int BK = kConvBK;
  constexpr int A_PASSES = BM / 32, B_PASSES = BN / 32;
  constexpr int WM = BM / 2, WN = BN / 2;  // per-wave tile
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int STAGE = (BM + BN) * BK / 8;  // uint4 per stage
  // ONE shared array (staging x2, reused for the epilogue tile): see the
  // "second __shared__ object" trap in cdna_hip_programming.md §5
  // STAGES == 1 (short reductions, e.g. 1x1 convs with C <= 128): half the LDS,
  // twice the resident workgroups, which is what hides latency there
  constexpr int OUT_U4 = BN * BM / 8 + (STATS ? BM : 0);  // epilogue tile + stats scratch
  constexpr int LDS_U4 = STAGES * STAGE > OUT_U4 ? STAGES * STAGE : OUT_U4;
  __shared__ __attribute__((aligned(16))) uint4 lds[LDS_U4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  ConvGeom g = g_in;
  // XCD-aware remap: blocks b and b+8 share an XCD; give each XCD a contiguous
  // range of tile ids so the channel tiles of one pixel tile share its L2.
  int bid = blockIdx.x;
  int kcls = 0;
  if constexpr (S2D) {
    // merged parity classes: class by RAW block id (each class range starts at a multiple of 8,
    // so dispatch spreads every class over all 8 XCDs -- a 1x1 stride-2 dgrad has one class
    // with work and three zero-fill classes), then the usual XCD remap within the class
    while (kcls + 1 < s2arg.ncls && bid >= s2arg.wg_start[kcls + 1]) ++kcls;
    bid -= s2arg.wg_start[kcls];
    g = s2arg.g[kcls];
  }
  // the class descriptor stays in the kernel-argument segment (its tap tables are indexed
  // per k-tile: a private copy would live in scratch)
  const S2Cls& cls = [&]() -> const S2Cls& {
    if constexpr (S2D) return s2arg.c[kcls];
    else return s2arg;
  }();
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int ntm = g.K / BM;
  const int ntn = (int)((NPQ + BN - 1) / BN);
  {
    const int nwg = ntm * ntn;
    if constexpr (S2D) {
      if (bid >= nwg) return;  // padding block of a class range (whole workgroup: uniform exit)
    }
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  const int tile_m = bid % ntm;
  const int tile_n = bid / ntm;
  const int m0 = tile_m * BM;
  const int64_t n0 = (int64_t)tile_n * BN;

  const int Kred = g.R * g.S * g.C;
  const int cblocks = g.C / BK;
  // STEM: 8 rows x 32 packed (tap, channel) values = 4 k-tiles of 64 (see conv_stem_fwd)
  const int KT = STEM ? kStemKT : (S2D ? cls.ntap * cblocks : g.R * g.S * cblocks);
  // lane -> (row within the wave's 8-row slab, LDS slot); the global source
  // chunk is pre-swizzled so the linear LDS image is XOR-swizzled (rule 21)
  const int lrow = wave * 8 + (lane >> 3);
  const int slot = lane & 7;

  int64_t pix_base[B_PASSES];
  int pix_h[B_PASSES], pix_w[B_PASSES], pix_n[B_PASSES];
#pragma unroll
  for (int i = 0; i < B_PASSES; ++i) {
    const int64_t pix = n0 + lrow + 32 * i;
    const bool ok = pix < NPQ;
    const int64_t pp = ok ? pix : 0;
    const int q = (int)(pp % g.Q);
    const int64_t t = pp / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    pix_n[i] = ok ? n : -1;
    pix_h[i] = ok ? p * g.st - g.pad : -(1 << 20);  // invalid rows never pass the bounds test
    pix_w[i] = q * g.st - g.pad;
    pix_base[i] = (((int64_t)n * g.H + pix_h[i]) * g.W + pix_w[i]) * g.C;
    if constexpr (STEM) pix_base[i] = ok ? (((int64_t)n * g.H + p * g.st) * g.W + q * g.st) * g.C : 0;
  }
  // the A passes' sources differ by the uniform 32 * Kred (the swizzle of rows lrow + 32 i is
  // lrow's): one per-lane pointer instead of A_PASSES (VGPRs for the main loop's fragments)
  const uint16_t* wsrc0 = w + (int64_t)(m0 + lrow) * Kred + (slot ^ swz(lrow, 0)) * 8;
  const int64_t wpass = (int64_t)32 * Kred;

  const int cbl = STEM ? 1 : cblocks;  // (STEM has C = 4 < BK: no channel blocks)
  const void* zpage = pin_sgpr(g_conv_zero_page);
  // GXF: this lane's BN-input chunks / mask bytes of the tile in flight, issued with the tile's DMA
  // and used after its wait (1x1 addressing: every B pass of a lane holds the same logical channel
  // chunk).  The per-channel coefficients [ka | c0 | c1 (| scale | shift)] x C floats sit in the
  // dynamic LDS region behind the staging array, copied once per workgroup: held in registers
  // across the wait they spilled (the single-stage kernel is compiled for 4 workgroups / CU).
  uint4 gx_v[GXF ? B_PASSES : 1];
  uint32_t gx_m[GXF == 2 ? B_PASSES : 1];
  extern __shared__ __attribute__((aligned(16))) float gx_lds[];
  auto issue = [&](int kt, int buf) {
    const int rs = kt / cbl, cb = kt - rs * cbl;
    int r = rs / g.S, s = rs - r * g.S;
    int wofs = kt * BK;
    if constexpr (S2D) {  // class tap rs: input offset (dr, ds), weights of tap wrs
      r = cls.dr[rs];
      s = cls.ds[rs];
      wofs = (cls.wrs[rs] * cbl + cb) * BK;
    }
    uint4* A = lds + buf * STAGE;
    uint4* B = A + BM * BK / 8;
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      const uint16_t* wsrc = wsrc0 + i * wpass;
      const bool wok = TB_BOUNDS_OK(wsrc + wofs + 8 <= w + (int64_t)g.K * Kred, kBndConvW);
      glds16(wok ? (const void*)(wsrc + wofs) : zpage, A + (32 * i + wave * 8) * 8);
    }
    if constexpr (STEM) {
      // k-tile kt = image rows 2kt, 2kt+1 of the window; each row is one
      // contiguous 64-B run of the pre-padded 4-channel image (8 pixels x 4 ch)
#pragma unroll
      for (int i = 0; i < B_PASSES; ++i) {
        const int row = lrow + 32 * i;
        const int lc = slot ^ swz(row, 0);
        const int64_t off = (int64_t)(2 * kt + (lc >> 2)) * g.W * g.C + (lc & 3) * 8;
        const void* src = pix_h[i] >= 0 ? (const void*)(x + pix_base[i] + off) : zpage;
        glds16(src, B + (32 * i + wave * 8) * 8);
      }
    } else if constexpr (VIRT) {
      // padded-virtual coordinates -> mirror (reflect) or zero page, then the upsampled
      // source pixel (>> upsh): the padded / upsampled tensor is never written
#pragma unroll
      for (int i = 0; i < B_PASSES; ++i) {
        const int row = lrow + 32 * i;
        int vh = p_virt_h(pix_h[i] + r, g), vw = p_virt_w(pix_w[i] + s, g);
        bool ok = pix_n[i] >= 0 && (unsigned)vh < (unsigned)g.Hv && (unsigned)vw < (unsigned)g.Wv;
        const int64_t off = (((int64_t)(ok ? pix_n[i] : 0) * g.H + (vh >> g.upsh)) * g.W + (vw >> g.upsh)) * g.C +
                            cb * BK + (slot ^ swz(row, 0)) * 8;
        ok = ok && TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc);
        glds16(ok ? (const void*)(x + off) : zpage, B + (32 * i + wave * 8) * 8);
      }
    } else {
    const int64_t tap = ((int64_t)r * g.W + s) * g.C + cb * BK;
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      const int row = lrow + 32 * i;
      const int ih = pix_h[i] + r, iw = pix_w[i] + s;
      bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const int64_t off = pix_base[i] + tap + (slot ^ swz(row, 0)) * 8;
      ok = ok && TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc);
      const void* src = ok ? (const void*)(x + off) : zpage;
      glds16(src, B + (32 * i + wave * 8) * 8);
      if constexpr (GXF != 0) {
        // the BN input at the same [pixel][channel] offset (1x1: the dgrad input's own layout);
        // the mask byte of those 8 channels is [pixel][C/8] = off / 8
        gx_v[i] = ok ? *reinterpret_cast<const uint4*>(gxa.xb + off) : make_uint4(0u, 0u, 0u, 0u);
        if constexpr (GXF == 2) gx_m[i] = ok ? (uint32_t)gxa.bits[off >> 3] : 0u;
      }
    }
    }
  };
  // GXF: the coefficient rows into the dynamic LDS region (visible after the next barrier)
  auto gxf_stage_coef = [&]() {
    if constexpr (GXF != 0) {
      const int C4 = g.C >> 2;
      float4* d = reinterpret_cast<float4*>(gx_lds);
      const float4* cf = reinterpret_cast<const float4*>(gxa.coef);
      for (int i = tid; i < 3 * C4; i += kConvThreads) d[i] = cf[i];
      if constexpr (GXF == 1) {
        const float4* sc = reinterpret_cast<const float4*>(gxa.scale);
        const float4* sf = reinterpret_cast<const float4*>(gxa.shift);
        for (int i = tid; i < C4; i += kConvThreads) {
          d[3 * C4 + i] = sc[i];
          d[4 * C4 + i] = sf[i];
        }
      }
    }
  };
  // GXF: dX = ka * act'(z) * g + c0 + c1 * xb on this lane's landed chunks of k-tile kt, in place
  // (norm_bn.hip bn_bwd_apply_k's arithmetic); tail pixels keep the zero page's zeros
  auto gxf_apply = [&](int kt) {
    if constexpr (GXF != 0) {
      uint4* B = lds + BM * BK / 8;
      const int c0 = kt * BK + (slot ^ swz(lrow, 0)) * 8;
      float ka[8], k0[8], k1[8], sc[8], sf[8];
      auto ld8 = [&](int row, float (&v)[8]) {
        const float4 a = *reinterpret_cast<const float4*>(gx_lds + row * g.C + c0);
        const float4 b = *reinterpret_cast<const float4*>(gx_lds + row * g.C + c0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      };
      ld8(0, ka);
      ld8(1, k0);
      ld8(2, k1);
      if constexpr (GXF == 1) {
        ld8(3, sc);
        ld8(4, sf);
      }
      const bool wr = gxa.out != nullptr && tile_m == 0;
#pragma unroll
      for (int i = 0; i < B_PASSES; ++i) {
        if (pix_n[i] < 0) continue;
        uint4* p = B + (32 * i + lrow) * 8 + slot;
        const uint4 gv = *p, xv = gx_v[i];
        const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w}, xw[4] = {xv.x, xv.y, xv.z, xv.w};
        uint32_t ow[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float d[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = 2 * e + h;
            const float xf = bf2f((uint16_t)(xw[e] >> (16 * h)));
            const float gf = bf2f((uint16_t)(gw[e] >> (16 * h)));
            bool keep;
            if constexpr (GXF == 1) keep = __builtin_fmaf(xf, sc[k], sf[k]) > 0.f;
            else keep = (gx_m[i] >> k) & 1u;
            const float dz = keep ? gf : 0.f;
            d[h] = ka[k] * dz + k0[k] + k1[k] * xf;
          }
          ow[e] = (uint32_t)f2bf(d[0]) | ((uint32_t)f2bf(d[1]) << 16);
        }
        const uint4 o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        *p = o;
        if (wr) *reinterpret_cast<uint4*>(gxa.out + pix_base[i] + c0) = o;
      }
    }
  };
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int cur) {
    const uint4* A = lds + cur * STAGE;
    const uint4* B = A + BM * BK / 8;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[TM], bfr[TN];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8_t, A[row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + fr;
        bfr[j] = __builtin_bit_cast(bf16x8_t, B[row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (STAGES >= 2) {
    // Ring of STAGES LDS buffers, STAGES-1 tiles in flight: one raw barrier per
    // k-tile and a COUNTED vmcnt (never 0 in steady state), so the prefetch
    // stays in flight across the barrier (cdna_hip_programming.md §5,
    // "Pipelining across barriers").  LPT = direct-to-LDS loads per lane per tile.
    constexpr int LPT = A_PASSES + B_PASSES;
#pragma unroll
    for (int t = 0; t < STAGES - 1; ++t)
      if (t < KT) issue(t, t);
    int cur = 0, nxt = STAGES - 1;
    for (int kt = 0; kt < KT; ++kt) {
      if (kt + STAGES - 2 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((STAGES - 2) * LPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // tile kt landed for every wave; buffer nxt is free
      asm volatile("" ::: "memory");
      if (kt + STAGES - 1 < KT) issue(kt + STAGES - 1, nxt);
      compute(cur);
      cur = cur + 1 == STAGES ? 0 : cur + 1;
      nxt = nxt + 1 == STAGES ? 0 : nxt + 1;
    }
    __syncthreads();  // last tile read by every wave before the epilogue reuses LDS
  } else {
  issue(0, 0);
  if constexpr (GXF != 0) {
    gxf_stage_coef();  // (its loads overlap the first tile's)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // coefficients visible to every lane
    gxf_apply(0);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = 0;
    const uint4* A = lds + cur * STAGE;
    const uint4* B = A + BM * BK / 8;
    // PRIO: the wave in its LDS-read + MFMA phase wins issue arbitration over the SIMD's other
    // waves (their staging / address work fills the gaps): s_setprio 3 measured -2.8 % on the 22
    // ResNet-50 forward shapes, +0.4 % on the whole step from the plain forward alone
    // (profiles/r02_convstudy/setprio.jsonl)
    if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[TM], bfr[TN];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + fr;
        af[i] = __builtin_bit_cast(bf16x8_t, A[row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + fr;
        bfr[j] = __builtin_bit_cast(bf16x8_t, B[row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < KT) {
      __syncthreads();  // every wave is done reading the single stage
      issue(kt + 1, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (GXF != 0) {
      if (kt + 1 < KT) gxf_apply(kt + 1);
    }
    __syncthreads();
  }
  }

  // ---- epilogue: bias/ReLU/bf16 in registers -> swizzled LDS tile [BN][BM]
  // -> 16-B coalesced row stores (each pixel's BM channels are contiguous)
  constexpr int CPR = BM / 8;  // 16-B chunks per pixel row of the output tile
  uint16_t* ot = reinterpret_cast<uint16_t*>(lds);
  float ssum[TM][4], ssq[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) ssum[i][e] = ssq[i][e] = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wm * WM + i * 16 + fq * 4;  // local out channel (multiple of 4)
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (BIAS) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bias[m0 + cl + e];
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int pl = wn * WN + j * 16 + fr;  // local pixel
      const bool pv = n0 + pl < NPQ;
      uint16_t hv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[i][j][e] + bv[e];
        if constexpr (RELU) v = fmaxf(v, 0.f);
        hv[e] = f2bf(v);
        if constexpr (STATS) {
          if (pv) {
            const float vr = bf2f(hv[e]);
            ssum[i][e] += vr;
            ssq[i][e] += vr * vr;
          }
        }
      }
      const int chunk = (cl >> 3) ^ (pl & (CPR - 1));
      *reinterpret_cast<uint2*>(ot + pl * BM + chunk * 8 + (cl & 7)) =
          make_uint2((uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16));
    }
  }
  __syncthreads();
  // BN-backward partials: a thread's 16-B chunk ck (8 channels) is fixed across
  // its rows (kConvThreads % CPR == 0)
  float bsc[8], bsf[8], bmu[8], bdb[8], bdg[8];
  if constexpr (BNB != 0) {
    const int c0 = m0 + (tid % CPR) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bmu[e] = bnb.mean[c0 + e];
      if constexpr (BNB == 1) {
        bsc[e] = bnb.scale[c0 + e];
        bsf[e] = bnb.shift[c0 + e];
      }
      bdb[e] = bdg[e] = 0.f;
    }
  }
  // The epilogue's global reads (residual addend + its mask, the BN input xb + its mask) are
  // issued for PB rows at once, before the first of them is needed: issued one row at a time
  // behind that row's store they were PB dependent HBM round trips per workgroup (the compiler
  // cannot move a load of xb above a store to y), which made the BN-backward dgrads of stage 1
  // run at 3-3.7 TB/s.
  constexpr int IT = BN * CPR / kConvThreads;
  constexpr int PB = IT < 4 ? IT : 4;
  constexpr bool PRE = ADD != 0 || BNB != 0;
  uint4 pre_a[PRE ? PB : 1], pre_x[PRE ? PB : 1];
  uint32_t pre_am[PRE ? PB : 1], pre_xm[PRE ? PB : 1];
#pragma unroll
  for (int it0 = 0; it0 < IT; it0 += PB) {
  if constexpr (PRE) {
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int idx = (it0 + u) * kConvThreads + tid;
      const int pl = idx / CPR, ck = idx % CPR;
      const int64_t pix = n0 + pl < NPQ ? n0 + pl : NPQ - 1;  // (rows past NPQ: a valid address, unused)
      if constexpr (ADD != 0) {
        pre_a[u] = *reinterpret_cast<const uint4*>(addend + pix * g.K + m0 + ck * 8);
        if constexpr (ADD == 2) pre_am[u] = amask[pix * (g.K / 8) + (m0 >> 3) + ck];
      }
      if constexpr (BNB != 0) {
        int64_t opix = pix;
        if constexpr (S2D) {
          const int j = (int)(pix % g.Q);
          const int64_t t = pix / g.Q;
          const int i = (int)(t % g.P);
          const int64_t n = t / g.P;
          opix = (n * cls.H + cls.st * i + cls.a) * cls.W + cls.st * j + cls.b;
        }
        pre_x[u] = *reinterpret_cast<const uint4*>(bnb.xb + opix * g.K + m0 + ck * 8);
        if constexpr (BNB == 2) pre_xm[u] = bnb.bits[opix * (g.K / 8) + (m0 >> 3) + ck];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < PB; ++u) {
    const int it = it0 + u;
    const int idx = it * kConvThreads + tid;
    const int pl = idx / CPR, ck = idx % CPR;
    const int64_t pix = n0 + pl;
    if (pix < NPQ) {
      uint4 v = *reinterpret_cast<const uint4*>(ot + pl * BM + ((ck ^ (pl & (CPR - 1))) * 8));
      if constexpr (ADD != 0) {
        uint4 a = pre_a[u];
        if constexpr (ADD == 2) {
          const uint32_t bits = pre_am[u];
          const auto keep = [&](uint32_t u, int i) {
            return (((bits >> i) & 1u) ? 0x0000ffffu : 0u) & u | ((((bits >> (i + 1)) & 1u) ? 0xffff0000u : 0u) & u);
          };
          a = make_uint4(keep(a.x, 0), keep(a.y, 2), keep(a.z, 4), keep(a.w, 6));
        }
        v = make_uint4(add_bf16x2(v.x, a.x), add_bf16x2(v.y, a.y), add_bf16x2(v.z, a.z), add_bf16x2(v.w, a.w));
      }
      int64_t opix = pix;
      if constexpr (S2D) {  // class pixel (n, i, j) -> dX pixel (n, st i + a, st j + b)
        const int j = (int)(pix % g.Q);
        const int64_t t = pix / g.Q;
        const int i = (int)(t % g.P);
        const int64_t n = t / g.P;
        opix = (n * cls.H + cls.st * i + cls.a) * cls.W + cls.st * j + cls.b;
      }
      const int64_t ylim = S2D ? (int64_t)g.N * cls.H * cls.W * g.K : NPQ * g.K;
      if (TB_BOUNDS_OK(opix * g.K + m0 + ck * 8 + 8 <= ylim, kBndConvDst))
        *reinterpret_cast<uint4*>(y + opix * g.K + m0 + ck * 8) = v;
      if constexpr (BNB != 0) {
        const uint4 xq = pre_x[u];
        const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, xw[4] = {xq.x, xq.y, xq.z, xq.w};
        uint32_t bits = 0xffu;
        if constexpr (BNB == 2) bits = pre_xm[u];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dv = bf2f((uint16_t)(vw[e >> 1] >> (16 * (e & 1))));
          const float xv = bf2f((uint16_t)(xw[e >> 1] >> (16 * (e & 1))));
          bool keep = true;
          if constexpr (BNB == 1) keep = __builtin_fmaf(xv, bsc[e], bsf[e]) > 0.f;
          if constexpr (BNB == 2) keep = (bits >> e) & 1u;
          const float dz = keep ? dv : 0.f;
          bdb[e] += dz;
          bdg[e] += dz * (xv - bmu[e]);
        }
      }
    }
  }
  }
  if constexpr (BNB != 0) {
    // reduce the kConvThreads / CPR rows of each chunk through LDS (the output
    // tile has been fully read: barrier first), one partial row per pixel tile
    // first across the rows a wave holds (lanes l, l + CPR, ... share a chunk: shuffles), then
    // the four waves through LDS: every thread busy, no serial walk over the rows
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bdb[e] += __shfl_xor(bdb[e], o, 64);
        bdg[e] += __shfl_xor(bdg[e], o, 64);
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);  // [4 waves][2][BM]
    if (lane < CPR) {
      const int c8 = lane * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * BM + c8 + e] = bdb[e];
        red[(wave * 2 + 1) * BM + c8 + e] = bdg[e];
      }
    }
    __syncthreads();
    const int64_t prow = (int64_t)tile_n + (S2D ? cls.tile_base : 0);
    for (int q = tid; q < 2 * BM; q += kConvThreads) {
      const int kind = q / BM, cl = q - kind * BM;
      const float s = (red[(0 * 2 + kind) * BM + cl] + red[(1 * 2 + kind) * BM + cl]) +
                      (red[(2 * 2 + kind) * BM + cl] + red[(3 * 2 + kind) * BM + cl]);
      bnb.part[(prow * 2 + kind) * g.K + m0 + cl] = s;
    }
  }
  if constexpr (STATS) {
    // reduce over the 16 lanes sharing a channel quad, then over the two
    // waves (wn) sharing the channel rows, through the (now free) LDS tail
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ssum[i][e] += __shfl_xor(ssum[i][e], o, 64);
          ssq[i][e] += __shfl_xor(ssq[i][e], o, 64);
        }
      }
    // [2 (wn)][2][BM] floats, disjoint from the BN x BM bf16 output tile
    float* red = reinterpret_cast<float*>(lds + BN * BM / 8);
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int cl = wm * WM + i * 16 + fq * 4 + e;
          red[(wn * 2 + 0) * BM + cl] = ssum[i][e];
          red[(wn * 2 + 1) * BM + cl] = ssq[i][e];
        }
    }
    __syncthreads();
    for (int cl = tid; cl < BM; cl += kConvThreads) {
      float* s0 = &stats[((int64_t)tile_n * 2 + 0) * g.K + m0 + cl];
      float* s1 = &stats[((int64_t)tile_n * 2 + 1) * g.K + m0 + cl];
      *s0 = red[0 * BM + cl] + red[2 * BM + cl];
      *s1 = red[1 * BM + cl] + red[3 * BM + cl];
    }
  }
}

static bool conv_big_pix(int64_t NPQ, int K);

// fp32 convolution as split-bf16 MFMA (the reference precision of the style-transfer examples):
// x = xh + xl, w = wh + wl (bf16 pairs, RNE), y = wh.xh + wh.xl + wl.xh accumulated in f32 --
// three v_mfma_f32_16x16x32_bf16 per fragment pair instead of eight 16x16x4 f32 MFMAs.  The
// implicit-GEMM structure of conv_fwd_k (same tiles, XOR-swizzled LDS, zero page for padded
// taps, XCD remap), single LDS stage holding both the hi and the lo tiles, f32 output with an
// optional bias / ReLU epilogue straight from the accumulators (16-B stores of 4 channels).
// The stride-1 input gradient is the same kernel on dy with the flipped, transposed weight.
//
// Few output pixels (VGG-19 at batch 1: 16² / 32² maps of 512 channels -> 16-64 tiles for 256 CUs)
// split the reduction over blockIdx.y (PART): each split writes its raw f32 partial tile to
// y + split * NPQ * K, and split_part_reduce_k sums the partials in a fixed order (deterministic)
// and applies the bias / ReLU.
//
// LO = false: plain bf16 operands (xl / wl unused, one MFMA per fragment pair) -- the few-pixel
// bf16 forward (VGG-19 perceptual loss at batch 1) on the same split-reduction path.
template <int BM, int BN, bool BIAS, bool RELU, bool PART = false, bool LO = true>
__global__ __launch_bounds__(kConvThreads, 2) void conv_fwd_split_k(const uint16_t* __restrict__ xh,
                                                                    const uint16_t* __restrict__ xl,
                                                                    const uint16_t* __restrict__ wh,
                                                                    const uint16_t* __restrict__ wl,
                                                                    float* __restrict__ y,
                                                                    const float* __restrict__ bias, ConvGeom g) {
  constexpr int BK = kConvBK;
  constexpr int A_PASSES = BM / 32, B_PASSES = BN / 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int STAGE = (BM + BN) * BK / 8;  // uint4 per operand set (hi or lo)
  __shared__ __attribute__((aligned(16))) uint4 lds[(LO ? 2 : 1) * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int ntm = g.K / BM;
  const int ntn = (int)((NPQ + BN - 1) / BN);
  int bid = blockIdx.x;
  {
    const int nwg = ntm * ntn;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  const int tile_m = bid % ntm, tile_n = bid / ntm;
  const int m0 = tile_m * BM;
  const int64_t n0 = (int64_t)tile_n * BN;
  const int Kred = g.R * g.S * g.C;
  const int cblocks = g.C / BK;
  const int KT = g.R * g.S * cblocks;
  // reduction steps of this workgroup: all of them, or split blockIdx.y of gridDim.y
  const int kt_lo = PART ? (int)((int64_t)blockIdx.y * KT / gridDim.y) : 0;
  const int kt_hi = PART ? (int)((int64_t)(blockIdx.y + 1) * KT / gridDim.y) : KT;
  if (PART) y += (int64_t)blockIdx.y * NPQ * g.K;
  const int lrow = wave * 8 + (lane >> 3);
  const int slot = lane & 7;

  int64_t pix_base[B_PASSES];
  int pix_h[B_PASSES], pix_w[B_PASSES];
#pragma unroll
  for (int i = 0; i < B_PASSES; ++i) {
    const int64_t pix = n0 + lrow + 32 * i;
    const bool ok = pix < NPQ;
    const int64_t pp = ok ? pix : 0;
    const int q = (int)(pp % g.Q);
    const int64_t t = pp / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    pix_h[i] = ok ? p * g.st - g.pad : -(1 << 20);
    pix_w[i] = q * g.st - g.pad;
    pix_base[i] = (((int64_t)n * g.H + pix_h[i]) * g.W + pix_w[i]) * g.C;
  }
  int64_t woff[A_PASSES];
#pragma unroll
  for (int i = 0; i < A_PASSES; ++i) {
    const int row = lrow + 32 * i;
    woff[i] = (int64_t)(m0 + row) * Kred + (slot ^ swz(row, 0)) * 8;
  }
  const void* zpage = pin_sgpr(g_conv_zero_page);
  auto issue = [&](int kt) {
    const int rs = kt / cblocks, cb = kt - rs * cblocks;
    const int r = rs / g.S, s = rs - r * g.S;
    const int wofs = kt * BK;
#pragma unroll
    for (int hl = 0; hl < (LO ? 2 : 1); ++hl) {
      uint4* A = lds + hl * STAGE;
      uint4* B = A + BM * BK / 8;
      const uint16_t* wsrc = hl ? wl : wh;
      const uint16_t* xsrc = hl ? xl : xh;
#pragma unroll
      for (int i = 0; i < A_PASSES; ++i) glds16(wsrc + woff[i] + wofs, A + (32 * i + wave * 8) * 8);
      const int64_t tap = ((int64_t)r * g.W + s) * g.C + cb * BK;
#pragma unroll
      for (int i = 0; i < B_PASSES; ++i) {
        const int row = lrow + 32 * i;
        const int ih = pix_h[i] + r, iw = pix_w[i] + s;
        bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const int64_t off = pix_base[i] + tap + (slot ^ swz(row, 0)) * 8;
        ok = ok && TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc);
        glds16(ok ? (const void*)(xsrc + off) : zpage, B + (32 * i + wave * 8) * 8);
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;

  issue(kt_lo);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = kt_lo; kt < kt_hi; ++kt) {
    __builtin_amdgcn_s_setprio(3);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int ch = ks * 4 + fq;
      bf16x8_t ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + fr;
        ah[i] = __builtin_bit_cast(bf16x8_t, lds[row * 8 + swz(row, ch)]);
        if constexpr (LO) al[i] = __builtin_bit_cast(bf16x8_t, lds[(LO ? STAGE : 0) + row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + fr;
        bh[j] = __builtin_bit_cast(bf16x8_t, lds[BM * BK / 8 + row * 8 + swz(row, ch)]);
        if constexpr (LO)
          bl[j] = __builtin_bit_cast(bf16x8_t, lds[(LO ? STAGE : 0) + BM * BK / 8 + row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (LO) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < kt_hi) {
      __syncthreads();
      issue(kt + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wm * WM + i * 16 + fq * 4;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (BIAS && !PART) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bias[m0 + cl + e];
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t pix = n0 + wn * WN + j * 16 + fr;
      if (pix >= NPQ) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bv[e];
        if constexpr (RELU && !PART) v[e] = fmaxf(v[e], 0.f);
      }
      if (TB_BOUNDS_OK(pix * g.K + m0 + cl + 4 <= NPQ * g.K, kBndConvDst))
        *reinterpret_cast<float4*>(y + pix * g.K + m0 + cl) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// y[i] = act(sum_s part[s][i] + bias[i % K]), float4 per lane, the splits summed in order
// (OT = float: the split-bf16 fp32 output; OT = uint16_t: a bf16 output, 4 channels per 8-B store)
template <bool BIAS, bool RELU, typename OT = float>
__global__ __launch_bounds__(256) void split_part_reduce_k(const float* __restrict__ part, int ns, int64_t n4,
                                                           int K, const float* __restrict__ bias,
                                                           OT* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = reinterpret_cast<const float4*>(part)[i];
    for (int s = 1; s < ns; ++s) {
      const float4 u = reinterpret_cast<const float4*>(part)[s * n4 + i];
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    if constexpr (BIAS) {
      const int k = (int)((i * 4) % K);
      v.x += bias[k]; v.y += bias[k + 1]; v.z += bias[k + 2]; v.w += bias[k + 3];
    }
    if constexpr (RELU) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    if constexpr (sizeof(OT) == 2)
      reinterpret_cast<uint2*>(y)[i] = make_uint2((uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16),
                                                  (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16));
    else
      reinterpret_cast<float4*>(y)[i] = v;
  }
}

template <int BM, int BN>
static void launch_split(const uint16_t* xh, const uint16_t* xl, const uint16_t* wh, const uint16_t* wl, float* y,
                         const float* bias, bool relu, const ConvGeom& g, hipStream_t st, float* part = nullptr,
                         int ns = 1) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  if (ns > 1) {
    const dim3 grid((g.K / BM) * (int)((NPQ + BN - 1) / BN), ns);
    conv_fwd_split_k<BM, BN, false, false, true><<<grid, kConvThreads, 0, st>>>(xh, xl, wh, wl, part, nullptr, g);
    const int64_t n4 = NPQ * g.K / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    if (bias) {
      if (relu) split_part_reduce_k<true, true><<<blocks, 256, 0, st>>>(part, ns, n4, g.K, bias, y);
      else split_part_reduce_k<true, false><<<blocks, 256, 0, st>>>(part, ns, n4, g.K, bias, y);
    } else {
      if (relu) split_part_reduce_k<false, true><<<blocks, 256, 0, st>>>(part, ns, n4, g.K, bias, y);
      else split_part_reduce_k<false, false><<<blocks, 256, 0, st>>>(part, ns, n4, g.K, bias, y);
    }
    return;
  }
  const dim3 grid((g.K / BM) * (int)((NPQ + BN - 1) / BN));
  if (bias) {
    if (relu) conv_fwd_split_k<BM, BN, true, true><<<grid, kConvThreads, 0, st>>>(xh, xl, wh, wl, y, bias, g);
    else conv_fwd_split_k<BM, BN, true, false><<<grid, kConvThreads, 0, st>>>(xh, xl, wh, wl, y, bias, g);
  } else {
    if (relu) conv_fwd_split_k<BM, BN, false, true><<<grid, kConvThreads, 0, st>>>(xh, xl, wh, wl, y, bias, g);
    else conv_fwd_split_k<BM, BN, false, false><<<grid, kConvThreads, 0, st>>>(xh, xl, wh, wl, y, bias, g);
  }
}

// x (hi, lo) [N][H][W][C], w (hi, lo) [K][R][S][C] bf16, y [N][P][Q][K] f32; C % 64 == K % 64 == 0
// reduction splits for few-pixel shapes (1 = none): enough workgroups for two per CU, each split
// at least 4 reduction steps of 64 channels
int conv_fwd_split32_ksplit(int N, int C, int K, int R, int S, int P, int Q) {
  const int64_t NPQ = (int64_t)N * P * Q;
  if (K % 128 != 0 || conv_big_pix(NPQ, K)) return 1;
  const int64_t tiles = (K / 128) * ((NPQ + 63) / 64);
  if (tiles >= 256) return 1;
  const int KT = R * S * (C / kConvBK);
  int ns = (int)std::min<int64_t>((512 + tiles - 1) / tiles, KT / 4);
  return ns < 2 ? 1 : std::min(ns, 32);
}

void conv_fwd_split32(const void* xh, const void* xl, const void* wh, const void* wl, float* y, const float* bias,
                      bool relu, int N, int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad,
                      hipStream_t st, float* part) {
  const ConvGeom g{N, H, W, C, K, R, S, P, Q, stride, pad};
  const bool bigpix = conv_big_pix((int64_t)N * P * Q, K);
  const uint16_t *a = (const uint16_t*)xh, *b = (const uint16_t*)xl, *c = (const uint16_t*)wh,
                 *d = (const uint16_t*)wl;
  const int ns = part ? conv_fwd_split32_ksplit(N, C, K, R, S, P, Q) : 1;
  if (ns > 1) {  // K % 128 == 0, few pixels
    launch_split<128, 64>(a, b, c, d, y, bias, relu, g, st, part, ns);
    return;
  }
  if (K % 128 == 0) {
    if (bigpix) launch_split<128, 128>(a, b, c, d, y, bias, relu, g, st);
    else launch_split<128, 64>(a, b, c, d, y, bias, relu, g, st);
  } else {
    if (bigpix) launch_split<64, 128>(a, b, c, d, y, bias, relu, g, st);
    else launch_split<64, 64>(a, b, c, d, y, bias, relu, g, st);
  }
}

// bf16 forward of a few-pixel conv (N*P*Q small, K % 128 == 0): the reduction split over
// blockIdx.y into f32 partials `part` [ns][NPQ][K], summed in split order with bias / ReLU into bf16 y
int conv_fwd_splitk_bf16_ksplit(int N, int C, int K, int R, int S, int P, int Q) {
  return conv_fwd_split32_ksplit(N, C, K, R, S, P, Q);
}

void conv_fwd_splitk_bf16(const void* x, const void* w, void* y, const float* bias, bool relu, int N, int H, int W,
                          int C, int K, int R, int S, int P, int Q, int stride, int pad, float* part, int ns,
                          hipStream_t st) {
  const ConvGeom g{N, H, W, C, K, R, S, P, Q, stride, pad};
  const int64_t NPQ = (int64_t)N * P * Q;
  const uint16_t *xb = (const uint16_t*)x, *wb = (const uint16_t*)w;
  const dim3 grid((K / 128) * (int)((NPQ + 63) / 64), ns);
  conv_fwd_split_k<128, 64, false, false, true, false><<<grid, kConvThreads, 0, st>>>(xb, xb, wb, wb, part, nullptr, g);
  const int64_t n4 = NPQ * K / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
  uint16_t* yb = (uint16_t*)y;
  if (bias) {
    if (relu) split_part_reduce_k<true, true, uint16_t><<<blocks, 256, 0, st>>>(part, ns, n4, K, bias, yb);
    else split_part_reduce_k<true, false, uint16_t><<<blocks, 256, 0, st>>>(part, ns, n4, K, bias, yb);
  } else {
    if (relu) split_part_reduce_k<false, true, uint16_t><<<blocks, 256, 0, st>>>(part, ns, n4, K, bias, yb);
    else split_part_reduce_k<false, false, uint16_t><<<blocks, 256, 0, st>>>(part, ns, n4, K, bias, yb);
  }
}

// weights [K][R][S][C] -> [C][R][S][K] with the taps flipped (dgrad of stride-1 conv)
__global__ void flip_transpose_w_k(const uint16_t* __restrict__ w, int K, int R, int S, int C,
                                   uint16_t* __restrict__ wt) {
  const int64_t total = (int64_t)K * R * S * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int s = (int)(t % S);
    t /= S;
    const int r = (int)(t % R);
    const int k = (int)(t / R);
    wt[(((int64_t)c * R + (R - 1 - r)) * S + (S - 1 - s)) * K + k] = w[i];
  }
}

// ---------------------------------------------------------------------------
int conv_fwd_supported(int C, int K) { return (C % kConvBK == 0) && (K % 64 == 0); }

// pixel tile: 128 when that still gives >= ~2 workgroups per CU, else 64
static bool conv_big_pix(int64_t NPQ, int K) {
  const int64_t ntm = K % 128 == 0 ? K / 128 : K / 64;
  return (NPQ / 128) * ntm >= 512;
}

// ---------------------------------------------------------------- persistent 1x1 forward
// A 1x1 stride-1 conv with a short reduction (C = 64 / 128 input channels: the expanding c3 /
// downsample convs of ResNet stages 1-2, 64 -> 256 and 128 -> 512) is a stream: per 128-pixel tile
// it reads 16-32 KiB and writes 32 KiB per 128 output channels, for 1-2 MFMA k-steps.  One
// workgroup per tile (conv_fwd_k) spends most of its life waiting for its single load and its
// stores: 3-3.5 TB/s measured (profiles/r04_*).  Here a workgroup owns one 128-channel tile, keeps
// its weights in REGISTERS (the MFMA A fragments, loaded once), and walks a strided stream of
// pixel tiles: the next tile's activations are in flight (direct-to-LDS, double buffered) while
// the current one is multiplied and its bf16 output leaves through an LDS staging tile in 16-B
// rows.  The BatchNorm statistics accumulate in registers over the whole stream and leave once:
// one partial row per stream (rows = conv_fwd_stats_rows), not one per pixel tile.
// Workgroups b and b + 8 share an XCD: the channel tiles of one stream are placed on one XCD so
// they read each activation tile through the same L2.
template <int CI, int BN, bool STATS, bool XF = false>
__global__ __launch_bounds__(kConvThreads, 2) void conv1x1_fwd_k(const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ w,
                                                               uint16_t* __restrict__ y, float* __restrict__ stats,
                                                               int64_t NPQ, int K, int nstreams,
                                                               XfArgs xf = XfArgs{}) {
  constexpr int BM = 128, KS = CI / 64, TM = 4, TN = BN / 32;  // waves 2 (ch) x 2 (px): 64 x BN/2 each
  constexpr int BT = KS * BN * 64 / 8;  // uint4 per activation tile (KS slabs of [BN][64])
  constexpr int OUT = BN * BM / 8;      // uint4 of the bf16 output staging tile [BN][BM]
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * BT + OUT + BM / 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fq = lane >> 4;
  const int ntm = K / BM;
  const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
  const int tile_m = j % ntm;
  const int s = (j / ntm) * 8 + xcd;  // this workgroup's stream (host: grid = ntm * nstreams, nstreams % 8 == 0)
  const int m0 = tile_m * BM;
  const int64_t ntn = (NPQ + BN - 1) / BN;

  // weights -> registers once: lane holds A[m0 + wm*64 + i*16 + fr][ks*64 + kk*32 + fq*8 .. +7]
  bf16x8_t af[TM][KS * 2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int q = 0; q < KS * 2; ++q)
      af[i][q] = __builtin_bit_cast(
          bf16x8_t, *reinterpret_cast<const uint4*>(w + (int64_t)(m0 + wm * 64 + i * 16 + fr) * CI + q * 32 + fq * 8));

  const int lrow = wave * 8 + (lane >> 3), slot = lane & 7;
  const void* zpage = pin_sgpr(g_conv_zero_page);
  // stage pixel tile t into buffer buf: 4 passes of 32 rows, KS slabs of 64 channels (glds, XOR-swizzled)
  auto issue = [&](int64_t t, int buf) {
    uint4* B = lds + buf * BT;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < BN / 32; ++i) {
        const int row = lrow + 32 * i;
        const int64_t pix = t * BN + row;
        const void* src =
            pix < NPQ ? (const void*)(x + pix * CI + ks * 64 + (slot ^ swz(row, 0)) * 8) : zpage;
        glds16(src, B + ks * BN * 8 + (32 * i + wave * 8) * 8);
      }
  };
  constexpr int LPT = KS * (BN / 32);  // direct-to-LDS loads per lane per tile
  constexpr int NST = BN * BM / 8 / kConvThreads;  // 16-B output stores per lane per tile
  // XF: the BN + ReLU of the input applied to this lane's staged chunks (channels ks*64 + its slot)
  float xsc[XF ? KS : 1][8], xsh[XF ? KS : 1][8];
  if constexpr (XF) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) xf_load(xf, ks * 64 + (slot ^ swz(lrow, 0)) * 8, xsc[ks], xsh[ks]);
  }

  float ssum[TM][4], ssq[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) ssum[i][e] = ssq[i][e] = 0.f;

  uint16_t* ot = reinterpret_cast<uint16_t*>(lds + 2 * BT);
  int64_t t = s;
  if (t < ntn) issue(t, 0);
  int cur = 0;
  bool first = true;
  for (; t < ntn; t += nstreams, cur ^= 1) {
    // this tile's loads landed (for this lane: the NST stores issued after them may still fly)
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    first = false;
    if constexpr (XF) {  // this lane's chunks of tile t (pixels past the end stay zero)
      uint4* Bt = lds + cur * BT;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < BN / 32; ++i) {
          if (t * BN + lrow + 32 * i >= NPQ) continue;
          uint4* p = Bt + ks * BN * 8 + (32 * i + wave * 8) * 8 + lane;
          *p = xf_chunk(*p, xsc[ks], xsh[ks]);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every lane's loads landed; the staging tile was read out
    asm volatile("" ::: "memory");
    if (t + nstreams < ntn) issue(t + nstreams, cur ^ 1);
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) acc[i][jn] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const uint4* B = lds + cur * BT;
#pragma unroll
    for (int q = 0; q < KS * 2; ++q) {
      const int ks = q >> 1, ch = (q & 1) * 4 + fq;
      bf16x8_t bfr[TN];
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) {
        const int row = wn * (BN / 2) + jn * 16 + fr;
        bfr[jn] = __builtin_bit_cast(bf16x8_t, B[ks * BN * 8 + row * 8 + swz(row, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jn = 0; jn < TN; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][q], bfr[jn], acc[i][jn], 0, 0, 0);
    }
    // epilogue: bf16 -> staging [BN][BM] (16-B chunk XOR-swizzled by pixel), statistics in registers
    const int64_t n0 = t * BN;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cl = wm * 64 + i * 16 + fq * 4;
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) {
        const int pl = wn * (BN / 2) + jn * 16 + fr;
        uint16_t hv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hv[e] = f2bf(acc[i][jn][e]);
          if constexpr (STATS) {
            if (n0 + pl < NPQ) {
              const float vr = bf2f(hv[e]);
              ssum[i][e] += vr;
              ssq[i][e] += vr * vr;
            }
          }
        }
        const int chunk = (cl >> 3) ^ (pl & 15);
        *reinterpret_cast<uint2*>(ot + pl * BM + chunk * 8 + (cl & 7)) =
            make_uint2((uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int it = 0; it < NST; ++it) {
      const int idx = it * kConvThreads + tid;
      const int pl = idx >> 4, ck = idx & 15;
      const uint4 v = *reinterpret_cast<const uint4*>(ot + pl * BM + ((ck ^ (pl & 15)) * 8));
      const int64_t pix = n0 + pl;
      // (rows past NPQ: stored to the last valid row's own slot -- never: skipped)
      if (pix < NPQ) *reinterpret_cast<uint4*>(y + pix * K + m0 + ck * 8) = v;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  if constexpr (STATS) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ssum[i][e] += __shfl_xor(ssum[i][e], o, 64);
          ssq[i][e] += __shfl_xor(ssq[i][e], o, 64);
        }
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);  // [2 (wn)][2][BM]
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int cl = wm * 64 + i * 16 + fq * 4 + e;
          red[(wn * 2 + 0) * BM + cl] = ssum[i][e];
          red[(wn * 2 + 1) * BM + cl] = ssq[i][e];
        }
    }
    __syncthreads();
    if (tid < BM) {
      float* s0 = &stats[((int64_t)s * 2 + 0) * K + m0 + tid];
      float* s1 = &stats[((int64_t)s * 2 + 1) * K + m0 + tid];
      *s0 = red[0 * BM + tid] + red[2 * BM + tid];
      *s1 = red[1 * BM + tid] + red[3 * BM + tid];
    }
  }
}

static bool g_conv1x1p = [] {
  const char* e = getenv("TBAMD_CONV1X1P");
  return !(e && e[0] == '0');
}();
void conv_set_persistent_1x1(bool on) { g_conv1x1p = on; }  // (A/B and tests; conv_fwd_stats_rows follows it)

// the persistent 1x1 kernel takes this forward (plain or statistics epilogue only)
static bool conv1x1p_eligible(int C, int K, int R, int S, int stride, int pad, int64_t NPQ) {
  return g_conv1x1p && R == 1 && S == 1 && stride == 1 && pad == 0 && (C == 64 || C == 128) && K % 128 == 0 &&
         NPQ >= (int64_t)128 * 256;
}

// streams per channel tile: two workgroups per CU over the whole chip, a multiple of 8, at most
// one stream per pixel tile
static int conv1x1p_bn(int C) { return C == 64 ? 128 : 64; }  // (C = 128: 64-pixel tiles keep 2 workgroups/CU)
static int conv1x1p_streams(int64_t NPQ, int K, int C) {
  const int ntm = K / 128, bn = conv1x1p_bn(C);
  int ns = (512 / ntm) & ~7;
  const int64_t ntn = (NPQ + bn - 1) / bn;
  if (ns > ntn) ns = (int)(ntn & ~(int64_t)7);
  return ns < 8 ? 8 : ns;
}

// the big-tile kernel takes this forward (conv_big.hip; with the heuristic mode the persistent 1x1
// keeps its shapes)
static int big_for(int64_t NPQ, int C, int K, int R, int S, int stride, int pad) {
  const int code = conv_big_choice(NPQ, C, K, R, S, stride, pad);
  if (code && conv_big_mode_now() == 1 && conv1x1p_eligible(C, K, R, S, stride, pad, NPQ)) return 0;
  return code;
}

// the 128x128 / persistent-1x1 kernels' statistics rows (the BN-in-operand forward, conv_fwd_xf,
// path always runs them)
int conv_fwd_stats_rows_tiled(int64_t NPQ, int C, int K, int R, int S, int stride, int pad) {
  if (conv1x1p_eligible(C, K, R, S, stride, pad, NPQ)) return conv1x1p_streams(NPQ, K, C);
  return conv_fwd_pixel_tiles(NPQ, K);
}

int conv_fwd_stats_rows(int64_t NPQ, int C, int K, int R, int S, int stride, int pad) {
  if (const int big = big_for(NPQ, C, K, R, S, stride, pad)) {
    const int bn = conv_big_pixel_tile(big);
    return (int)((NPQ + bn - 1) / bn);
  }
  return conv_fwd_stats_rows_tiled(NPQ, C, K, R, S, stride, pad);
}

int conv_fwd_bnb_rows(int64_t NPQ, int C, int K, int R, int S, int stride, int pad) {
  if (const int big = conv_big_choice(NPQ, C, K, R, S, stride, pad)) {
    const int bn = conv_big_pixel_tile(big);
    return (int)((NPQ + bn - 1) / bn);
  }
  return conv_fwd_pixel_tiles(NPQ, K);
}

int conv_fwd_pixel_tiles(int64_t NPQ, int K) {
  const int BN = conv_big_pix(NPQ, K) ? 128 : 64;
  return (int)((NPQ + BN - 1) / BN);
}

// pipeline depth override for tuning experiments (0 = heuristic)
static int g_conv_stages = [] {  // (TBAMD_CONV_STAGES: the same override from the environment, for A/B runs)
  const char* e = getenv("TBAMD_CONV_STAGES");
  return e ? atoi(e) : 0;
}();
static int g_conv_occ = 0;  // min workgroups per CU the single-stage kernel is compiled for (0 = 4)
void conv_set_stages(int s) { g_conv_stages = s; }
void conv_set_occupancy(int o) { g_conv_occ = o; }

template <int BM, int BN, bool STATS, bool BIAS, bool RELU, int ADD = 0, int BNB = 0>
static void launch_conv(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias, float* stats,
                        const uint16_t* addend, const uint8_t* amask, const ConvGeom& g, hipStream_t st,
                        const BnBwdEpi& bnb = BnBwdEpi{}) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int ntn = (int)((NPQ + BN - 1) / BN);
  const int ntm = g.K / BM;
  const dim3 grid(ntm * ntn);
  if constexpr (ADD != 0 || BNB != 0) {
    // dgrad epilogues: single stage, 4 workgroups/CU by default; TBAMD_CONV_EPI_STAGES=2|3 pipelines
    // the k-loop instead (A/B for the long-reduction 1x1 input gradients, e.g. 256 -> 64)
    static const int epi_stages = [] {
      const char* e = getenv("TBAMD_CONV_EPI_STAGES");
      return e ? atoi(e) : 1;
    }();
    if (epi_stages == 2)
      conv_fwd_k<BM, BN, STATS, BIAS, RELU, 2, ADD, 2, BNB>
          <<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
    else if (epi_stages == 3)
      conv_fwd_k<BM, BN, STATS, BIAS, RELU, 3, ADD, 2, BNB>
          <<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
    else
      conv_fwd_k<BM, BN, STATS, BIAS, RELU, 1, ADD, 4, BNB>
          <<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
  } else {
    int stages = g_conv_stages;
    if (stages == 0) stages = 1;  // measured: occupancy beats pipeline depth here (profiles/r01_conv)
    switch (stages) {
      case 1:
        // single LDS stage compiled for 4 workgroups/CU (<= 128 VGPRs): the
        // measured optimum (profiles/r01_conv/tune_*.jsonl)
        if (g_conv_occ == 2)
          conv_fwd_k<BM, BN, STATS, BIAS, RELU, 1, ADD, 2><<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
        else if (g_conv_occ == 3)
          conv_fwd_k<BM, BN, STATS, BIAS, RELU, 1, ADD, 3><<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
        else
          conv_fwd_k<BM, BN, STATS, BIAS, RELU, 1, ADD, 4><<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
        break;
      case 3:
        conv_fwd_k<BM, BN, STATS, BIAS, RELU, 3, ADD><<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
        break;
      case 4:
        conv_fwd_k<BM, BN, STATS, BIAS, RELU, 4, ADD><<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
        break;
      default:
        conv_fwd_k<BM, BN, STATS, BIAS, RELU, 2, ADD><<<grid, kConvThreads, 0, st>>>(x, w, y, bias, stats, addend, amask, g, bnb, S2Cls{});
    }
  }
}

template <int BM, int BN, int ADD>
static void dispatch_bnb(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* addend,
                         const uint8_t* amask, int bnb_mode, const BnBwdEpi& bnb, const ConvGeom& g,
                         hipStream_t st) {
  switch (bnb_mode) {
    case 1: launch_conv<BM, BN, false, false, false, ADD, 1>(x, w, y, nullptr, nullptr, addend, amask, g, st, bnb); break;
    case 2: launch_conv<BM, BN, false, false, false, ADD, 2>(x, w, y, nullptr, nullptr, addend, amask, g, st, bnb); break;
    default: launch_conv<BM, BN, false, false, false, ADD, 3>(x, w, y, nullptr, nullptr, addend, amask, g, st, bnb);
  }
}

template <int BM, int BN>
static void dispatch_epi(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias, float* stats,
                         const uint16_t* addend, const uint8_t* amask, bool relu, const ConvGeom& g,
                         hipStream_t st, int bnb_mode = 0, const BnBwdEpi& bnb = BnBwdEpi{}) {
  if (bnb_mode != 0) {
    if (addend && amask) dispatch_bnb<BM, BN, 2>(x, w, y, addend, amask, bnb_mode, bnb, g, st);
    else if (addend) dispatch_bnb<BM, BN, 1>(x, w, y, addend, nullptr, bnb_mode, bnb, g, st);
    else dispatch_bnb<BM, BN, 0>(x, w, y, nullptr, nullptr, bnb_mode, bnb, g, st);
  } else if (addend) {
    if (amask) launch_conv<BM, BN, false, false, false, 2>(x, w, y, nullptr, nullptr, addend, amask, g, st);
    else launch_conv<BM, BN, false, false, false, 1>(x, w, y, nullptr, nullptr, addend, nullptr, g, st);
  } else if (stats) {
    if (bias) launch_conv<BM, BN, true, true, false>(x, w, y, bias, stats, nullptr, nullptr, g, st, bnb);
    else launch_conv<BM, BN, true, false, false>(x, w, y, bias, stats, nullptr, nullptr, g, st, bnb);
  } else if (bias) {
    if (relu) launch_conv<BM, BN, false, true, true>(x, w, y, bias, stats, nullptr, nullptr, g, st);
    else launch_conv<BM, BN, false, true, false>(x, w, y, bias, stats, nullptr, nullptr, g, st);
  } else {
    if (relu) launch_conv<BM, BN, false, false, true>(x, w, y, bias, stats, nullptr, nullptr, g, st);
    else launch_conv<BM, BN, false, false, false>(x, w, y, bias, stats, nullptr, nullptr, g, st);
  }
}

// GXF 1x1 input gradient (see GxfArgs): single stage, 4 workgroups/CU like the other dgrad epilogues
template <int BM, int BN, int ADD, int BNB, int GXF>
static void launch_gxf(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* addend,
                       const uint8_t* amask, const ConvGeom& g, hipStream_t st, const BnBwdEpi& bnb,
                       const GxfArgs& gxa) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const dim3 grid((g.K / BM) * (int)((NPQ + BN - 1) / BN));
  const size_t coef_bytes = (size_t)(GXF == 1 ? 5 : 3) * g.C * sizeof(float);
  conv_fwd_k<BM, BN, false, false, false, 1, ADD, 4, BNB, false, false, false, 3, GXF>
      <<<grid, kConvThreads, coef_bytes, st>>>(x, w, y, nullptr, nullptr, addend, amask, g, bnb, S2Cls{}, gxa);
}

template <int BM, int BN>
static bool dispatch_gxf(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* addend,
                         const uint8_t* amask, const ConvGeom& g, hipStream_t st, int bnb_mode, const BnBwdEpi& bnb,
                         int gxf, const GxfArgs& gxa) {
  const int add = addend ? (amask ? 2 : 1) : 0;
  // the combinations a bottleneck produces: conv3's dgrad under the block-output BN (GXF 2, bn2's
  // partials), conv1's dgrad under bn1 (GXF 1; the residual gradient added, masked or not, and the
  // previous block's output-BN partials or none)
  if (gxf == 2 && add == 0 && bnb_mode == 1) launch_gxf<BM, BN, 0, 1, 2>(x, w, y, addend, amask, g, st, bnb, gxa);
  else if (gxf == 1 && add == 2 && bnb_mode == 2) launch_gxf<BM, BN, 2, 2, 1>(x, w, y, addend, amask, g, st, bnb, gxa);
  else if (gxf == 1 && add == 1 && bnb_mode == 2) launch_gxf<BM, BN, 1, 2, 1>(x, w, y, addend, amask, g, st, bnb, gxa);
  else if (gxf == 1 && add == 1 && bnb_mode == 0) launch_gxf<BM, BN, 1, 0, 1>(x, w, y, addend, amask, g, st, bnb, gxa);
  else return false;
  return true;
}

bool conv_dgrad_gxf_supported(int gxf, int add, int bnb_mode) {
  return (gxf == 2 && add == 0 && bnb_mode == 1) || (gxf == 1 && add == 2 && bnb_mode == 2) ||
         (gxf == 1 && add == 1 && (bnb_mode == 2 || bnb_mode == 0));
}

int conv_gxf_bnb_rows(int64_t NPQ, int K) {
  (void)K;
  return (int)((NPQ + 63) / 64);  // conv_dgrad_gxf's 64-pixel tiles
}

void conv_dgrad_gxf(const void* x, const void* w, void* y, const void* addend, const uint8_t* amask, int N, int H,
                    int W, int C, int K, hipStream_t st, int bnb_mode, const void* bnb_x, const float* bnb_scale,
                    const float* bnb_shift, const float* bnb_mean, const uint8_t* bnb_bits, float* bnb_part, int gxf,
                    const void* gx_x, const uint8_t* gx_bits, const float* gx_scale, const float* gx_shift,
                    const float* gx_coef, void* gx_out) {
  const BnBwdEpi bnb{(const uint16_t*)bnb_x, bnb_scale, bnb_shift, bnb_mean, bnb_bits, bnb_part};
  const GxfArgs gxa{(const uint16_t*)gx_x, gx_bits, gx_scale, gx_shift, gx_coef, (uint16_t*)gx_out};
  const ConvGeom g{N, H, W, C, K, 1, 1, H, W, 1, 0};
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  const uint16_t* aa = (const uint16_t*)addend;
  bool ok;
  // (64-pixel tiles only: the 128-pixel ones have no VGPRs left for the staged BN input and spill)
  if (K % 128 == 0) ok = dispatch_gxf<128, 64>(xx, ww, yy, aa, amask, g, st, bnb_mode, bnb, gxf, gxa);
  else ok = dispatch_gxf<64, 64>(xx, ww, yy, aa, amask, g, st, bnb_mode, bnb, gxf, gxa);
  if (!ok) throw std::runtime_error("conv_dgrad_gxf: unsupported (gxf, addend, bnb_mode) combination");
}

// stats (optional): [conv_fwd_stats_rows][2][K] raw per-tile (or per-stream) sums of the bf16 output
void conv_fwd(const void* x, const void* w, void* y, const float* bias, float* stats, const void* addend,
              const uint8_t* amask, bool relu, int N, int H, int W, int C, int K, int R, int S, int P, int Q,
              int stride, int pad, hipStream_t st, int bnb_mode, const void* bnb_x, const float* bnb_scale,
              const float* bnb_shift, const float* bnb_mean, const uint8_t* bnb_bits, float* bnb_part) {
  const BnBwdEpi bnb{(const uint16_t*)bnb_x, bnb_scale, bnb_shift, bnb_mean, bnb_bits, bnb_part};
  ConvGeom g{N, H, W, C, K, R, S, P, Q, stride, pad};
  const int64_t NPQ = (int64_t)N * P * Q;
  {
    const int big = bnb_mode != 0 || addend ? conv_big_choice(NPQ, C, K, R, S, stride, pad)
                                            : big_for(NPQ, C, K, R, S, stride, pad);
    if (big) {
      conv_big_fwd(x, w, y, bias, stats, addend, amask, relu, N, H, W, C, K, R, S, P, Q, stride, pad, st, bnb_mode,
                   bnb_x, bnb_scale, bnb_shift, bnb_mean, bnb_bits, bnb_part, big);
      return;
    }
  }

  const bool bigpix = conv_big_pix(NPQ, K);
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  const uint16_t* aa = (const uint16_t*)addend;
  if (!bias && !relu && !addend && bnb_mode == 0 && conv1x1p_eligible(C, K, R, S, stride, pad, NPQ)) {
    const int ns = conv1x1p_streams(NPQ, K, C);
    const dim3 grid((K / 128) * ns);
    if (C == 64) {
      if (stats) conv1x1_fwd_k<64, 128, true><<<grid, kConvThreads, 0, st>>>(xx, ww, yy, stats, NPQ, K, ns);
      else conv1x1_fwd_k<64, 128, false><<<grid, kConvThreads, 0, st>>>(xx, ww, yy, nullptr, NPQ, K, ns);
    } else {
      if (stats) conv1x1_fwd_k<128, 64, true><<<grid, kConvThreads, 0, st>>>(xx, ww, yy, stats, NPQ, K, ns);
      else conv1x1_fwd_k<128, 64, false><<<grid, kConvThreads, 0, st>>>(xx, ww, yy, nullptr, NPQ, K, ns);
    }
    return;
  }
  if (K % 128 == 0) {
    if (bigpix) dispatch_epi<128, 128>(xx, ww, yy, bias, stats, aa, amask, relu, g, st, bnb_mode, bnb);
    else dispatch_epi<128, 64>(xx, ww, yy, bias, stats, aa, amask, relu, g, st, bnb_mode, bnb);
  } else {
    if (bigpix) dispatch_epi<64, 128>(xx, ww, yy, bias, stats, aa, amask, relu, g, st, bnb_mode, bnb);
    else dispatch_epi<64, 64>(xx, ww, yy, bias, stats, aa, amask, relu, g, st, bnb_mode, bnb);
  }
}

// the BN-in-operand forward runs where the persistent 1x1 kernel does: its few long-lived
// workgroups stage the coefficients once and the transform is off the critical path.  (On the tiled
// kernels it was -3.4 % on the ResNet-50 step -- the per-k-tile transform sat on the single-stage
// critical path, profiles/r04_xf -- and that variant was removed.)
bool conv_fwd_xf_supported(int64_t NPQ, int C, int K, int R, int S, int stride, int pad) {
  return conv1x1p_eligible(C, K, R, S, stride, pad, NPQ);
}

// forward conv of relu(bn(x)) with the BN + ReLU applied to the activation operand in LDS (XfArgs):
// statistics epilogue when `stats` (same rows as conv_fwd), no bias / relu / addend
template <bool STATS>
static void launch_xf(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const ConvGeom& g,
                      const XfArgs& xf, hipStream_t st) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  if (conv1x1p_eligible(g.C, g.K, g.R, g.S, g.st, g.pad, NPQ)) {
    const int ns = conv1x1p_streams(NPQ, g.K, g.C);
    const dim3 grid((g.K / 128) * ns);
    if (g.C == 64)
      conv1x1_fwd_k<64, 128, STATS, true><<<grid, kConvThreads, 0, st>>>(x, w, y, stats, NPQ, g.K, ns, xf);
    else
      conv1x1_fwd_k<128, 64, STATS, true><<<grid, kConvThreads, 0, st>>>(x, w, y, stats, NPQ, g.K, ns, xf);
    return;
  }
  throw std::runtime_error("conv2d_fwd_xf: the BN-in-operand forward runs on the persistent 1x1 kernel only "
                           "(C = 64 / 128, 1x1 stride 1, enough pixels: conv_fwd_xf_supported)");
}

void conv_fwd_xf(const void* x, const void* w, void* y, float* stats, const float* scale, const float* shift, int N,
                 int H, int W, int C, int K, int R, int S, int P, int Q, int stride, int pad, hipStream_t st) {
  const ConvGeom g{N, H, W, C, K, R, S, P, Q, stride, pad};
  const XfArgs xf{scale, shift};
  if (stats) launch_xf<true>((const uint16_t*)x, (const uint16_t*)w, (uint16_t*)y, stats, g, xf, st);
  else launch_xf<false>((const uint16_t*)x, (const uint16_t*)w, (uint16_t*)y, nullptr, g, xf, st);
}

// conv over the virtual input pad(upsample_nearest(x, up), pad, reflect|zero) (up = 1, 2, 4):
// the plain forward kernel with VIRT addressing (bias optional, no other epilogue)
template <int BM, int BN>
static void launch_virt(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias, const ConvGeom& g,
                        hipStream_t st) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const dim3 grid((g.K / BM) * (int)((NPQ + BN - 1) / BN));
  if (bias)
    conv_fwd_k<BM, BN, false, true, false, 1, 0, 4, 0, false, false, true>
        <<<grid, kConvThreads, 0, st>>>(x, w, y, bias, nullptr, nullptr, nullptr, g);
  else
    conv_fwd_k<BM, BN, false, false, false, 1, 0, 4, 0, false, false, true>
        <<<grid, kConvThreads, 0, st>>>(x, w, y, nullptr, nullptr, nullptr, nullptr, g);
}

void conv_fwd_virtual(const void* x, const void* w, void* y, const float* bias, int N, int H, int W, int C, int K,
                      int R, int S, int P, int Q, int stride, int pad, int up, int reflect, hipStream_t st) {
  ConvGeom g{N, H, W, C, K, R, S, P, Q, stride, pad, up == 4 ? 2 : (up == 2 ? 1 : 0), reflect ? 1 : 0, H * up, W * up};
  const int64_t NPQ = (int64_t)N * P * Q;
  const bool bigpix = conv_big_pix(NPQ, K);
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  if (K % 128 == 0) {
    if (bigpix) launch_virt<128, 128>(xx, ww, yy, bias, g, st);
    else launch_virt<128, 64>(xx, ww, yy, bias, g, st);
  } else {
    if (bigpix) launch_virt<64, 128>(xx, ww, yy, bias, g, st);
    else launch_virt<64, 64>(xx, ww, yy, bias, g, st);
  }
}

// ---------------------------------------------------------------- 7x7/2 stem
// The ResNet stem (C = 3, 7x7, stride 2, pad 3) does not fit the C % 64 == 0
// channel-block loader.  The image is re-laid once per step as [N][2P+6][2Q+6][4]
// (zero border, 4th channel zero); then for output pixel (p, q) and window row r
// the 7 taps x 4 channels are 28 contiguous values starting at padded pixel
// (2p + r, 2q), read as a 64-B run (the 4 trailing values belong to the next
// pixel and meet zero weights).  The reduction is 8 rows (row 7 has zero
// weights) x 32 = 256 = 4 k-tiles of 64: the same MFMA main loop, LDS image and
// BN-statistics epilogue as every other conv, no per-tap bounds test.
__global__ __launch_bounds__(256) void stem_pad_k(const uint16_t* __restrict__ x, uint16_t* __restrict__ xp, int N,
                                                  int H, int W, int Hp, int Wp, int pad) {
  const int64_t total = (int64_t)N * Hp * Wp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int w = (int)(i % Wp);
    const int64_t t = i / Wp;
    const int h = (int)(t % Hp);
    const int n = (int)(t / Hp);
    const int ih = h - pad, iw = w - pad;
    uint32_t lo = 0, hi = 0;
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
      const uint16_t* s = x + (((int64_t)n * H + ih) * W + iw) * 3;
      lo = (uint32_t)s[0] | ((uint32_t)s[1] << 16);
      hi = (uint32_t)s[2];
    }
    *reinterpret_cast<uint2*>(xp + i * 4) = make_uint2(lo, hi);
  }
}

// padded image [N][2P+6][2Q+6][4]: every window row / 8-pixel run of every output pixel is
// in bounds (row 2p + 7 and column 2q + 7 are read against zero weights), rows 16-B aligned
static void stem_dims(int H, int W, int& P, int& Q, int& Hp, int& Wp) {
  P = (H - 1) / 2 + 1;
  Q = (W - 1) / 2 + 1;
  Hp = 2 * P + 6;
  Wp = 2 * Q + 6;
}

int64_t conv_stem_workspace(int N, int H, int W) {
  int P, Q, Hp, Wp;
  stem_dims(H, W, P, Q, Hp, Wp);
  return (int64_t)N * Hp * Wp * 4;
}

template <int BM, int BN, bool STATS>
static void launch_stem(const uint16_t* xp, const uint16_t* wp, uint16_t* y, float* stats, const ConvGeom& g,
                        hipStream_t st) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const dim3 grid((g.K / BM) * (int)((NPQ + BN - 1) / BN));
  conv_fwd_k<BM, BN, STATS, false, false, 1, 0, 4, 0, true>
      <<<grid, kConvThreads, 0, st>>>(xp, wp, y, nullptr, stats, nullptr, nullptr, g);
}

void conv_stem_pad(const void* x, void* xp, int N, int H, int W, hipStream_t st) {
  int P, Q, Hp, Wp;
  stem_dims(H, W, P, Q, Hp, Wp);
  const int64_t tot = (int64_t)N * Hp * Wp;
  int64_t gs = (tot + 255) / 256;
  if (gs > 8192) gs = 8192;
  stem_pad_k<<<(int)gs, 256, 0, st>>>((const uint16_t*)x, (uint16_t*)xp, N, H, W, Hp, Wp, 3);
}

void stem_geometry(int H, int W, int* P, int* Q, int* Hp, int* Wp) { stem_dims(H, W, *P, *Q, *Hp, *Wp); }

void conv_stem_fwd(const void* xp, const void* wp, void* y, float* stats, int N, int H, int W, int K,
                   hipStream_t st) {
  int P, Q, Hp, Wp;
  stem_dims(H, W, P, Q, Hp, Wp);
  // padded geometry: C = 4, R = S = 8 so that Kred = R * S * C = 256 (the packed weight row)
  const ConvGeom g{N, Hp, Wp, 4, K, 8, 8, P, Q, 2, 0};
  const bool bigpix = conv_big_pix((int64_t)N * P * Q, K);
  const uint16_t* xx = (const uint16_t*)xp;
  const uint16_t* ww = (const uint16_t*)wp;
  uint16_t* yy = (uint16_t*)y;
#define TB_STEM(BM_, BN_)                                               \
  do {                                                                  \
    if (stats) launch_stem<BM_, BN_, true>(xx, ww, yy, stats, g, st);   \
    else launch_stem<BM_, BN_, false>(xx, ww, yy, nullptr, g, st);      \
  } while (0)
  if (K % 128 == 0) {
    if (bigpix) TB_STEM(128, 128);
    else TB_STEM(128, 64);
  } else {
    if (bigpix) TB_STEM(64, 128);
    else TB_STEM(64, 64);
  }
#undef TB_STEM
}

// ------------------------------------------------------- stride-2 dgrad (classes)
template <int BM, int BN, int BNB>
static void launch_s2_b(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, const S2Set& set,
                        const BnBwdEpi& bnb, hipStream_t st) {
  const int nwg = set.wg_start[set.ncls];
  if (nwg == 0) return;
  conv_fwd_k<BM, BN, false, false, false, 1, 0, 4, BNB, false, true>
      <<<nwg, kConvThreads, 0, st>>>(dy, wt, dx, nullptr, nullptr, nullptr, nullptr, set.g[0], bnb, set);
}

template <int BM, int BN>
static void launch_s2(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, const S2Set& set, int bnb_mode,
                      const BnBwdEpi& bnb, hipStream_t st) {
  switch (bnb_mode) {
    case 1: launch_s2_b<BM, BN, 1>(dy, wt, dx, set, bnb, st); break;
    case 2: launch_s2_b<BM, BN, 2>(dy, wt, dx, set, bnb, st); break;
    case 3: launch_s2_b<BM, BN, 3>(dy, wt, dx, set, bnb, st); break;
    default: launch_s2_b<BM, BN, 0>(dy, wt, dx, set, bnb, st);
  }
}

// one pixel-tile width for all classes of a merged launch (the largest class decides)
static int s2_bn(int N, int H, int W, int Cf, int st) {
  return conv_big_pix((int64_t)N * ((H + st - 1) / st) * ((W + st - 1) / st), Cf) ? 128 : 64;
}

// BN-partial rows written by conv_dgrad_s2 (the per-class pixel tiles stacked)
int conv_dgrad_s2_tiles(int N, int H, int W, int Cf, int st) {
  const int BN = s2_bn(N, H, W, Cf, st);
  int t = 0;
  for (int a = 0; a < st; ++a)
    for (int b = 0; b < st; ++b) {
      const int64_t NPQ = (int64_t)N * ((H - a + st - 1) / st) * ((W - b + st - 1) / st);
      t += (int)((NPQ + BN - 1) / BN);
    }
  return t;
}

// the phase decomposition takes this strided input gradient: stride 2 or 3, at most 16 taps per
// class (ceil(R / st) * ceil(S / st): up to 8x8 at stride 2, 12x12 at stride 3)
bool conv_dgrad_s2_supported(int R, int S, int st) {
  return (st == 2 || st == 3) && ((R + st - 1) / st) * ((S + st - 1) / st) <= 16;
}

// dy [N, P, Q, Kf] (Kf = forward output channels), wt = conv_flip_transpose_weight(w) [Cf][R][S][Kf],
// dx [N, H, W, Cf]; stride cs (2 or 3), padding pad.  Output phase (a, b) of dX (rows cs*i + a,
// columns cs*j + b) is a stride-1 conv of dY with the taps r = a + pad (mod cs), s = b + pad (mod cs)
// at input offset ((a + pad - r) / cs, (b + pad - s) / cs): cs^2 implicit-GEMM classes, one launch.
void conv_dgrad_s2(const void* dy, const void* wt, void* dx, int N, int P, int Q, int Kf, int Cf, int R, int S,
                   int pad, int H, int W, hipStream_t st, int bnb_mode, const void* bnb_x, const float* bnb_scale,
                   const float* bnb_shift, const float* bnb_mean, const uint8_t* bnb_bits, float* bnb_part,
                   int cs) {
  if (!conv_dgrad_s2_supported(R, S, cs)) throw std::runtime_error("conv_dgrad_s2: stride 2 / 3, <= 16 taps per class");
  const BnBwdEpi bnb{(const uint16_t*)bnb_x, bnb_scale, bnb_shift, bnb_mean, bnb_bits, bnb_part};
  const int BN = s2_bn(N, H, W, Cf, cs);
  const int BM = Cf % 128 == 0 ? 128 : 64;
  S2Set set{};
  int tile_base = 0;
  auto phase = [cs](int v) { return ((v % cs) + cs) % cs; };
  for (int a = 0; a < cs; ++a)
    for (int b = 0; b < cs; ++b) {
      S2Cls c{};
      c.a = a;
      c.b = b;
      c.st = cs;
      c.H = H;
      c.W = W;
      c.ntap = 0;
      for (int r = 0; r < R; ++r) {
        if (phase(a + pad - r) != 0) continue;
        for (int s = 0; s < S; ++s) {
          if (phase(b + pad - s) != 0) continue;
          c.dr[c.ntap] = (a + pad - r) / cs;  // (exact: a + pad - r is a multiple of cs)
          c.ds[c.ntap] = (b + pad - s) / cs;
          c.wrs[c.ntap] = (R - 1 - r) * S + (S - 1 - s);  // flipped weight layout
          ++c.ntap;
        }
      }
      // class output grid: rows cs*i + a < H, columns cs*j + b < W; "input" = dY (P x Q, Kf channels)
      const int Hc = (H - a + cs - 1) / cs, Wc = (W - b + cs - 1) / cs;
      const ConvGeom g{N, P, Q, Kf, Cf, R, S, Hc, Wc, 1, 0};
      const int64_t NPQ = (int64_t)N * Hc * Wc;
      const int ntiles = (int)((NPQ + BN - 1) / BN);
      c.tile_base = tile_base;
      tile_base += ntiles;
      if (NPQ == 0) continue;
      set.g[set.ncls] = g;
      set.c[set.ncls] = c;
      set.wg_start[set.ncls + 1] = set.wg_start[set.ncls] + ((Cf / BM) * ntiles + 7) / 8 * 8;
      ++set.ncls;
    }
  if (set.ncls == 0) return;
  const uint16_t* d = (const uint16_t*)dy;
  const uint16_t* w = (const uint16_t*)wt;
  uint16_t* o = (uint16_t*)dx;
  if (BM == 128) {
    if (BN == 128) launch_s2<128, 128>(d, w, o, set, bnb_mode, bnb, st);
    else launch_s2<128, 64>(d, w, o, set, bnb_mode, bnb, st);
  } else {
    if (BN == 128) launch_s2<64, 128>(d, w, o, set, bnb_mode, bnb, st);
    else launch_s2<64, 64>(d, w, o, set, bnb_mode, bnb, st);
  }
}

// Many weights in ONE launch (the flipped copies of every trainable conv of a model
// are refreshed once per optimizer step instead of once per conv per backward).
// The weight [K][R][S][C] is a [K][RSC] matrix; its flipped transpose is [RSC'][K]
// with row rsc = (r, s, c) -> c*R*S + (R-1-r)*S + (S-1-s).  One workgroup moves one
// 64 x 64 tile through LDS: 16-B coalesced reads along RSC, 16-B coalesced writes
// along K (K % 64 == 0 and C % 64 == 0: every native conv).
// table rows (int64): [src, dst, K, R, S, C, 0, 0]; chunks: (tensor, tile id).
struct FlipChunk {
  int32_t t;
  int32_t pad;
  int64_t tile, unused;
};

__global__ __launch_bounds__(256) void flip_transpose_mt_k(const FlipChunk* __restrict__ chunks,
                                                           const int64_t* __restrict__ table) {
  __shared__ uint16_t tl[64][72];  // [k][rsc] (+8 pad: the column gathers spread over banks)
  const FlipChunk ck = chunks[blockIdx.x];
  const int64_t* row = table + (int64_t)ck.t * 8;
  const uint16_t* w = reinterpret_cast<const uint16_t*>(row[0]);
  uint16_t* wt = reinterpret_cast<uint16_t*>(row[1]);
  const int K = (int)row[2], R = (int)row[3], S = (int)row[4], C = (int)row[5];
  const int64_t RSC = (int64_t)R * S * C;
  const int ntc = (int)(RSC / 64);
  const int kt = (int)(ck.tile / ntc), ct = (int)(ck.tile % ntc);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i, r = e >> 3, c8 = e & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(w + (int64_t)(kt * 64 + r) * RSC + ct * 64 + c8 * 8);
    *reinterpret_cast<uint4*>(&tl[r][c8 * 8]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i, cc = e >> 3, k8 = e & 7;
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = (uint32_t)tl[k8 * 8 + 2 * j][cc] | ((uint32_t)tl[k8 * 8 + 2 * j + 1][cc] << 16);
    const int64_t rsc = (int64_t)ct * 64 + cc;
    const int c = (int)(rsc % C);
    const int rs = (int)(rsc / C);
    const int r = rs / S, s = rs - r * S;
    const int64_t drow = ((int64_t)c * R + (R - 1 - r)) * S + (S - 1 - s);
    *reinterpret_cast<uint4*>(wt + drow * K + kt * 64 + k8 * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void conv_flip_transpose_weights_mt(const void* chunks, int nchunks, const int64_t* table, hipStream_t st) {
  if (nchunks > 0)
    flip_transpose_mt_k<<<nchunks, 256, 0, st>>>(reinterpret_cast<const FlipChunk*>(chunks), table);
}

void conv_flip_transpose_weight(const void* w, int K, int R, int S, int C, void* wt, hipStream_t st) {
  const int64_t total = (int64_t)K * R * S * C;
  int64_t gs = (total + 255) / 256;
  if (gs > 4096) gs = 4096;
  flip_transpose_w_k<<<(int)gs, 256, 0, st>>>((const uint16_t*)w, K, R, S, C, (uint16_t*)wt);
}

}  // namespace tbamd
