// Narrow-output convolution (K <= 16 output channels) on gfx950 MFMA.
//
// The last layer of the style-transfer decoders maps 64 (AdaIN) or 32 (StyleNet)
// channels to an RGB image through a 9x9 window behind a reflection pad
// (reference examples/img_stt/adain/adain.py:51, online/online.py:57).  As an
// implicit GEMM that is M = 3 output channels against a 5184-deep reduction: the
// channel-tiled kernels (conv.hip, conv_any.hip) and MIOpen spend their time
// re-gathering the 81 taps of every pixel from L2 for three useful output rows
// (4.3 ms fwd for AdaIN's b32 @256 on MIOpen, 15 TF/s).
//
// Here one workgroup owns a 16 x 16 output tile of one image and stages its halo
// -- (16 + R - 1) x (16 + S - 1) virtual pixels x C channels, reflect / zero padding
// and nearest upsampling resolved while staging -- ONCE in LDS with direct-to-LDS
// loads; all R*S taps then read it from LDS:
//
//   D[k][pix] += W[k][tap][c0..c0+31] . halo[pix + tap][c0..c0+31]     (v_mfma_f32_16x16x32_bf16)
//
// with the (zero-padded to 16) output channels as the MFMA rows and 16 consecutive
// output pixels of one tile row as its columns.  Each wave owns 4 tile rows (4
// accumulators); the weight fragment of a tap is shared by those 4 MFMAs and
// prefetched one tap ahead from global memory (the whole padded weight is 166 KB,
// L2-resident).  Halo pixel rows are 16-B chunk-swizzled (chunk ^ (p & 7) for 64
// channels, chunk ^ ((p >> 1) & 3) for 32), which keeps every ds_read_b128 lane group
// on 16 distinct bank slots for any tap offset (scripted search, see
// profiles/r02_narrow/README.md).
#include <algorithm>

#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

constexpr int kNT = 256;           // threads (4 waves)
constexpr int kTH = 16, kTW = 16;  // output tile
constexpr int kMaxTap = 9;         // R, S <= 9
constexpr int kHaloPix = (kTH + kMaxTap - 1) * (kTW + kMaxTap - 1);  // 576

__device__ __attribute__((aligned(64))) uint4 g_narrow_zero[16];

struct NarrowGeom {
  int N, H, W, C, K, R, S, P, Q, pad, upsh, reflect, Hv, Wv;
  int HR, HC;            // halo rows / cols
  int tiles_h, tiles_w;  // output tiles per image
  // output placement: pixel (p, q) -> (p * ys + ya, q * ys + yb) of a YH x YW map (a stride
  // phase of a transposed conv; 1, 0, 0, P, Q for a plain conv); padw: left padding
  int ys, ya, yb, YH, YW, padw;
};

template <int NCH>
__device__ __forceinline__ int hswz(int p, int c) {
  if constexpr (NCH == 8) return c ^ (p & 7);
  else return c ^ ((p >> 1) & 3);
}

// padded virtual coordinate -> unpadded virtual coordinate in [0, lim), or -1 (zero padding)
__device__ __forceinline__ int vmap(int v, int lim, int reflect) {
  if (reflect) v = v < 0 ? -v : (v >= lim ? 2 * lim - 2 - v : v);
  return (unsigned)v < (unsigned)lim ? v : -1;
}

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

template <int NCH>
__global__ __launch_bounds__(kNT, 2) void conv_narrow_fwd_k(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ w16,
                                                            const float* __restrict__ bias,
                                                            uint16_t* __restrict__ y, NarrowGeom g) {
  constexpr int SLOTS = (kHaloPix * NCH + kNT - 1) / kNT * kNT;
  __shared__ __attribute__((aligned(16))) uint4 halo[SLOTS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_img = g.tiles_h * g.tiles_w;
  const int n = blockIdx.x / per_img, rem = blockIdx.x - n * per_img;
  const int th = rem / g.tiles_w;
  const int oh0 = th * kTH, ow0 = (rem - th * g.tiles_w) * kTW;

  // ---- stage the halo: LDS slot s = p * NCH + pc holds logical chunk hswz(p, pc) of
  // halo pixel p (the XOR is its own inverse); lane-linear slots, pre-swizzled sources
  const void* zpage = pin_sgpr(g_narrow_zero);
  const int total = g.HR * g.HC * NCH;
  const int64_t img = (int64_t)n * g.H * g.W;
  for (int base = wave * 64; base < total; base += kNT) {
    const int sl = base + lane;
    const void* src = zpage;
    if (sl < total) {
      const int p = sl / NCH, pc = sl - p * NCH;
      const int hr = p / g.HC, hc = p - hr * g.HC;
      const int vh = vmap(oh0 - g.pad + hr, g.Hv, g.reflect), vw = vmap(ow0 - g.padw + hc, g.Wv, g.reflect);
      if (vh >= 0 && vw >= 0) {
        const int64_t off = (img + (int64_t)(vh >> g.upsh) * g.W + (vw >> g.upsh)) * g.C + hswz<NCH>(p, pc) * 8;
        if (TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc)) src = x + off;
      }
    }
    glds16(src, halo + base);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- taps: 4 accumulators per wave (tile rows 4w .. 4w+3), A = weights of out channel
  // (lane & 15), k chunk (lane >> 4); B = 16 pixels of one tile row at the tap offset
  const int fr = lane & 15, fq = lane >> 4;
  const int RS = g.R * g.S;
  const uint16_t* wl = w16 + (int64_t)fr * RS * g.C + fq * 8;
  constexpr int KC = NCH / 4;  // 32-deep k chunks per tap
  f32x4_t acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t an[KC];
#pragma unroll
  for (int cc = 0; cc < KC; ++cc) an[cc] = *reinterpret_cast<const bf16x8_t*>(wl + cc * 32);
  int r = 0, s = 0;
  for (int tap = 0; tap < RS; ++tap) {
    bf16x8_t a[KC];
#pragma unroll
    for (int cc = 0; cc < KC; ++cc) a[cc] = an[cc];
    if (tap + 1 < RS) {
#pragma unroll
      for (int cc = 0; cc < KC; ++cc)
        an[cc] = *reinterpret_cast<const bf16x8_t*>(wl + (int64_t)(tap + 1) * g.C + cc * 32);
    }
    const int prow = (wave * 4 + r) * g.HC + s + fr;  // halo pixel of (tile row 4w, col fr) at this tap
#pragma unroll
    for (int cc = 0; cc < KC; ++cc) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = prow + i * g.HC;
        const bf16x8_t b = __builtin_bit_cast(bf16x8_t, halo[p * NCH + hswz<NCH>(p, cc * 4 + fq)]);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cc], b, acc[i], 0, 0, 0);
      }
    }
    if (++s == g.S) {
      s = 0;
      ++r;
    }
  }

  // ---- epilogue: lane holds out channels 4*fq + e of pixel column fr
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oh = oh0 + wave * 4 + i, ow = ow0 + fr;
    if (oh >= g.P || ow >= g.Q) continue;
    uint16_t* yo = y + (((int64_t)n * g.YH + oh * g.ys + g.ya) * g.YW + ow * g.ys + g.yb) * g.K;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = fq * 4 + e;
      if (k < g.K) yo[k] = f2bf(acc[i][e] + (bias ? bias[k] : 0.f));
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Weight gradient of the same convolution:
//
//   dW[k][r][s][c] = sum_{n,p,q} dy[n,p,q,k] * xv[n, p - pad + r, q - pad + s, c]
//
// D[k][c] (16 padded output channels x 16 input channels) += A[k][32 pixels] . B[32 pixels][c]
// per MFMA, the reduction running over output pixels.  A workgroup owns one 16-channel block
// of C and a contiguous range of 16 x 16 pixel tiles (split-K over pixels); per tile it stages
// the 16-channel halo (direct-to-LDS) and the tile's dy TRANSPOSED to [16 k][256 pixels]
// (zero rows past K), so the A fragment is one 16-B LDS read and the B fragment the
// transposing ds_read_b64_tr_b16 pair of conv_wgrad.hip over the halo rows of the tap.  The
// R*S taps are dealt to the 4 waves (<= kWTap accumulators each); partial sums go to
// part[split][16][R*S][C] in f32 and are summed over the splits by the host wrapper.
constexpr int kWTap = 21;  // taps per wave: 4 waves x 21 >= 81

// 32-B halo pixel slot: pixels p and p + 8 (rows j and j + 8 of one transposing read) are
// 256 B apart in a linear image, i.e. on the same banks; XOR-ing bit 2 with bit 3 puts the
// 8 pixels {b..b+3, b+8..b+11} a 32-lane half reads on 8 distinct 32-B bank groups for
// every b (an involution within each aligned group of 16 pixels)
__device__ __forceinline__ int wsw(int p) { return p ^ (((p >> 3) & 1) << 2); }

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

__global__ __launch_bounds__(kNT, 2) void conv_narrow_wgrad_k(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ dy,
                                                              float* __restrict__ part, NarrowGeom g,
                                                              int tiles_per_split) {
  __shared__ __attribute__((aligned(16))) uint4 halo[(kHaloPix * 2 + kNT - 1) / kNT * kNT];  // [pix][16 ch]
  // [k][tile pixel], rows padded by 16 B so the 16 A-fragment rows fall on distinct bank slots
  __shared__ __attribute__((aligned(16))) uint16_t dyt[16][kTH * kTW + 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = blockIdx.x % (g.C / 16), split = blockIdx.x / (g.C / 16);
  const int per_img = g.tiles_h * g.tiles_w;
  const int ntiles = g.N * per_img;
  const int t0 = split * tiles_per_split, t1 = min(ntiles, t0 + tiles_per_split);
  const int RS = g.R * g.S;
  const int tap0 = wave * kWTap;  // this wave's taps: [tap0, min(RS, tap0 + kWTap))
  const void* zpage = pin_sgpr(g_narrow_zero);
  const int g4 = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int fr = lane & 15;

  f32x4_t acc[kWTap];
#pragma unroll
  for (int j = 0; j < kWTap; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int t = t0; t < t1; ++t) {
    const int n = t / per_img, rem = t - n * per_img;
    const int th = rem / g.tiles_w;
    const int oh0 = th * kTH, ow0 = (rem - th * g.tiles_w) * kTW;
    // halo of the 16-channel block: 32-B pixel slot wsw(p), two 16-B chunks each (whole
    // groups of 16 pixels: wsw permutes within them)
    const int hpix = g.HR * g.HC;
    const int total = (hpix + 15) / 16 * 32;
    const int64_t img = (int64_t)n * g.H * g.W;
    for (int base = wave * 64; base < total; base += kNT) {
      const int sl = base + lane;
      const void* src = zpage;
      const int p = wsw(sl >> 1), ch = sl & 1;
      if (p < hpix) {
        const int hr = p / g.HC, hc = p - hr * g.HC;
        const int vh = vmap(oh0 - g.pad + hr, g.Hv, g.reflect), vw = vmap(ow0 - g.padw + hc, g.Wv, g.reflect);
        if (vh >= 0 && vw >= 0) {
          const int64_t off = (img + (int64_t)(vh >> g.upsh) * g.W + (vw >> g.upsh)) * g.C + cb * 16 + ch * 8;
          if (TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc)) src = x + off;
        }
      }
      glds16(src, halo + base);
    }
    // dy tile transposed (one thread per tile pixel; K <= 16 values, zero past K / outside)
    {
      const int oh = oh0 + (tid >> 4), ow = ow0 + (tid & 15);
      const bool ok = oh < g.P && ow < g.Q;
      const uint16_t* dp = dy + (((int64_t)n * g.P + (ok ? oh : 0)) * g.Q + (ok ? ow : 0)) * g.K;
#pragma unroll
      for (int k = 0; k < 16; ++k) dyt[k][tid] = (ok && k < g.K) ? dp[k] : (uint16_t)0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* hb = reinterpret_cast<const char*>(halo);
#pragma unroll 1
    for (int ks = 0; ks < kTH * kTW / 32; ++ks) {
      // A: dy^T rows k = fr, pixels 32 ks + 8 g4 .. +7
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&dyt[fr][ks * 32 + g4 * 8]);
      // rows j0 = 8 g4 + q4 and j0 + 4 of this 32-pixel step: tile row 2 ks + (j >> 4), col j & 15
      const int j0 = 8 * g4 + q4, j1 = j0 + 4;
      const int hp0 = (2 * ks + (j0 >> 4)) * g.HC + (j0 & 15);
      const int hp1 = (2 * ks + (j1 >> 4)) * g.HC + (j1 & 15);
#pragma unroll
      for (int j = 0; j < kWTap; ++j) {
        const int tap = tap0 + j;
        if (tap < RS) {
          const int r = tap / g.S, s = tap - r * g.S;
          const int sh = r * g.HC + s;
          const s16x4_t v0 =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(hb + wsw(hp0 + sh) * 32 + p4 * 8));
          const s16x4_t v1 =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(hb + wsw(hp1 + sh) * 32 + p4 * 8));
          typedef short s16x8_t __attribute__((ext_vector_type(8)));
          const s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8_t, v), acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // halo / dyt reused by the next tile
  }
  // D[k][c]: lane holds k = 4 g4 + e, channel column fr of the block
#pragma unroll
  for (int j = 0; j < kWTap; ++j) {
    const int tap = tap0 + j;
    if (tap >= RS) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * g4 + e;
      part[(((int64_t)split * 16 + k) * RS + tap) * g.C + cb * 16 + fr] = acc[j][e];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Tiny-input-channel forward (C*R*S <= 256: the RGB input convs -- VGG 3->64 3x3, DCGAN
// discriminator 3->64 4x4/2, StyleNet 3->32 9x9, LeNet 1->6 5x5).  The whole (r, s, c)
// reduction of an output pixel is at most 8 MFMA k-steps, so the im2col row is gathered
// straight into the B fragment (8 values per lane per k-step, the input is a few MB and stays
// in L1/L2), the packed weights [K][32*KT] are the A fragments, and each wave produces 64
// pixels x up to 64 output channels (16 accumulators).  The kernel is output-write bound
// (64 channels per 3 input channels); the channel-tiled kernels reach 0.6 TB/s on these
// shapes.  Reflect / zero padding resolved per gathered tap; optional bias and ReLU epilogue.
struct TinyGeom {
  int N, H, W, C, K, R, S, P, Q, st, pad, reflect, kred;
};

template <int KT, bool RELU>
__global__ __launch_bounds__(kNT) void conv_tinyc_fwd_k(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wp,
                                                        const int* __restrict__ tab, const float* __restrict__ bias,
                                                        uint16_t* __restrict__ y, TinyGeom g) {
  __shared__ int ltab[32 * KT];  // flattened reduction index -> (dr | ds << 8 | c << 16), -1 past kred
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 32 * KT; i += kNT) ltab[i] = i < g.kred ? tab[i] : -1;
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int kb0 = blockIdx.y * 64;                 // first output channel of this workgroup
  const int nkb = min(4, (g.K - kb0) / 16);        // 16-channel row blocks (K % 16 == 0)
  const int64_t pix0 = (int64_t)blockIdx.x * 256 + wave * 64;
  // the 4 pixels (one per 16-pixel block) this lane gathers
  int ih0[4], iw0[4];
  const uint16_t* img[4];
  bool pv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t pix = pix0 + 16 * j + fr;
    pv[j] = pix < NPQ;
    const int64_t pp = pv[j] ? pix : 0;
    const int q = (int)(pp % g.Q);
    const int64_t t = pp / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    ih0[j] = p * g.st - g.pad;
    iw0[j] = q * g.st - g.pad;
    img[j] = x + (int64_t)n * g.H * g.W * g.C;
  }
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    bf16x8_t a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = kb0 + 16 * i + fr;
      a[i] = i < nkb ? *reinterpret_cast<const bf16x8_t*>(wp + (int64_t)m * (32 * KT) + 32 * t + 8 * fq)
                     : bf16x8_t{};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint16_t v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int code = ltab[32 * t + 8 * fq + e];
        uint16_t val = 0;
        if (code >= 0 && pv[j]) {
          int h = ih0[j] + (code & 0xff), w = iw0[j] + ((code >> 8) & 0xff);
          const int c = code >> 16;
          if (g.reflect) {
            h = h < 0 ? -h : (h >= g.H ? 2 * g.H - 2 - h : h);
            w = w < 0 ? -w : (w >= g.W ? 2 * g.W - 2 - w : w);
          }
          if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
            val = img[j][((int64_t)h * g.W + w) * g.C + c];
        }
        v[e] = val;
      }
      const uint4 u = make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                                 (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16));
      const bf16x8_t b = __builtin_bit_cast(bf16x8_t, u);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nkb) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
    }
  }
  // D[ch][pix]: lane holds channels 16 i + 4 fq + e of pixel 16 j + fr -> one 8-B store
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= nkb) continue;
    const int c0 = kb0 + 16 * i + 4 * fq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bias[c0 + e];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t pix = pix0 + 16 * j + fr;
      if (pix >= NPQ) continue;
      uint16_t hv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[i][j][e] + bv[e];
        if constexpr (RELU) v = fmaxf(v, 0.f);
        hv[e] = f2bf(v);
      }
      *reinterpret_cast<uint2*>(y + pix * g.K + c0) =
          make_uint2((uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16));
    }
  }
}

// fp32 variant (the reference precision of the style-transfer examples: StyleNet's 9x9 3->32
// input conv): the gathered fp32 im2col values are split in registers into bf16 (hi, lo) =
// (RNE(v), RNE(v - hi)), the packed weights come as a (hi, lo) pair, and each k-step runs
// wh.xh + wh.xl + wl.xh on three MFMAs; f32 output (16-B stores of 4 channels).
template <int KT, bool RELU>
__global__ __launch_bounds__(kNT) void conv_tiny32_fwd_k(const float* __restrict__ x, const uint16_t* __restrict__ wph,
                                                         const uint16_t* __restrict__ wpl, const int* __restrict__ tab,
                                                         const float* __restrict__ bias, float* __restrict__ y,
                                                         TinyGeom g) {
  __shared__ int ltab[32 * KT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 32 * KT; i += kNT) ltab[i] = i < g.kred ? tab[i] : -1;
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int kb0 = blockIdx.y * 64;
  const int nkb = min(4, (g.K - kb0) / 16);
  const int64_t pix0 = (int64_t)blockIdx.x * 256 + wave * 64;
  int ih0[4], iw0[4];
  const float* img[4];
  bool pv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t pix = pix0 + 16 * j + fr;
    pv[j] = pix < NPQ;
    const int64_t pp = pv[j] ? pix : 0;
    const int q = (int)(pp % g.Q);
    const int64_t t = pp / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    ih0[j] = p * g.st - g.pad;
    iw0[j] = q * g.st - g.pad;
    img[j] = x + (int64_t)n * g.H * g.W * g.C;
  }
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    bf16x8_t ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t o = (int64_t)(kb0 + 16 * i + fr) * (32 * KT) + 32 * t + 8 * fq;
      ah[i] = i < nkb ? *reinterpret_cast<const bf16x8_t*>(wph + o) : bf16x8_t{};
      al[i] = i < nkb ? *reinterpret_cast<const bf16x8_t*>(wpl + o) : bf16x8_t{};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        uint32_t hp = 0, lp = 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int code = ltab[32 * t + 8 * fq + 2 * e2 + half];
          float val = 0.f;
          if (code >= 0 && pv[j]) {
            int h = ih0[j] + (code & 0xff), w = iw0[j] + ((code >> 8) & 0xff);
            const int c = code >> 16;
            if (g.reflect) {
              h = h < 0 ? -h : (h >= g.H ? 2 * g.H - 2 - h : h);
              w = w < 0 ? -w : (w >= g.W ? 2 * g.W - 2 - w : w);
            }
            if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W) val = img[j][((int64_t)h * g.W + w) * g.C + c];
          }
          const uint16_t hi = f2bf(val);
          const uint16_t lo = f2bf(val - bf2f(hi));
          hp |= (uint32_t)hi << (16 * half);
          lp |= (uint32_t)lo << (16 * half);
        }
        hw[e2] = hp;
        lw[e2] = lp;
      }
      const bf16x8_t bh = __builtin_bit_cast(bf16x8_t, make_uint4(hw[0], hw[1], hw[2], hw[3]));
      const bf16x8_t bl = __builtin_bit_cast(bf16x8_t, make_uint4(lw[0], lw[1], lw[2], lw[3]));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nkb) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][j], 0, 0, 0);
        }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= nkb) continue;
    const int c0 = kb0 + 16 * i + 4 * fq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bias[c0 + e];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t pix = pix0 + 16 * j + fr;
      if (pix >= NPQ) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bv[e];
        if constexpr (RELU) v[e] = fmaxf(v[e], 0.f);
      }
      *reinterpret_cast<float4*>(y + pix * g.K + c0) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// fp32 narrow forward (the RGB heads and 3-channel input gradients at the reference precision):
// the halo tile is staged from the fp32 input one 32-channel group at a time, split on the way
// into bf16 hi / lo halos in LDS (2 x 36 KB), and every tap runs wh.xh + wh.xl + wl.xh on three
// MFMAs per fragment pair -- no separate split pass, one halo read; f32 output + bias.
template <int NG>  // 32-channel groups (C = 32 * NG)
__global__ __launch_bounds__(kNT, 2) void conv_narrow32_fwd_k(const float* __restrict__ x,
                                                              const uint16_t* __restrict__ w16h,
                                                              const uint16_t* __restrict__ w16l,
                                                              const float* __restrict__ bias, float* __restrict__ y,
                                                              NarrowGeom g) {
  constexpr int NCH = 4;  // 16-B chunks (8 channels) per halo pixel and group
  __shared__ __attribute__((aligned(16))) uint4 hh[kHaloPix * NCH];
  __shared__ __attribute__((aligned(16))) uint4 hl[kHaloPix * NCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_img = g.tiles_h * g.tiles_w;
  const int n = blockIdx.x / per_img, rem = blockIdx.x - n * per_img;
  const int th = rem / g.tiles_w;
  const int oh0 = th * kTH, ow0 = (rem - th * g.tiles_w) * kTW;
  const int total = g.HR * g.HC * NCH;
  const int64_t img = (int64_t)n * g.H * g.W;
  const int fr = lane & 15, fq = lane >> 4;
  const int RS = g.R * g.S;
  f32x4_t acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int grp = 0; grp < NG; ++grp) {
    if (grp) __syncthreads();  // every wave is done with the previous group's halos
    for (int sl = tid; sl < total; sl += kNT) {
      const int p = sl / NCH, pc = sl - p * NCH;
      const int hr = p / g.HC, hc = p - hr * g.HC;
      const int vh = vmap(oh0 - g.pad + hr, g.Hv, g.reflect), vw = vmap(ow0 - g.padw + hc, g.Wv, g.reflect);
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (vh >= 0 && vw >= 0) {
        const int64_t off =
            (img + (int64_t)(vh >> g.upsh) * g.W + (vw >> g.upsh)) * g.C + grp * 32 + hswz<NCH>(p, pc) * 8;
        if (TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc)) {
          v0 = *reinterpret_cast<const float4*>(x + off);
          v1 = *reinterpret_cast<const float4*>(x + off + 4);
        }
      }
      const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      uint32_t h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint16_t h0 = f2bf(f[2 * e]), h1 = f2bf(f[2 * e + 1]);
        const uint16_t l0 = f2bf(f[2 * e] - bf2f(h0)), l1 = f2bf(f[2 * e + 1] - bf2f(h1));
        h[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        l[e] = (uint32_t)l0 | ((uint32_t)l1 << 16);
      }
      hh[sl] = make_uint4(h[0], h[1], h[2], h[3]);
      hl[sl] = make_uint4(l[0], l[1], l[2], l[3]);
    }
    __syncthreads();
    const int64_t wo = (int64_t)fr * RS * g.C + grp * 32 + fq * 8;
    bf16x8_t nh = *reinterpret_cast<const bf16x8_t*>(w16h + wo);
    bf16x8_t nl = *reinterpret_cast<const bf16x8_t*>(w16l + wo);
    int r = 0, s = 0;
    for (int tap = 0; tap < RS; ++tap) {
      const bf16x8_t ah = nh, al = nl;
      if (tap + 1 < RS) {
        nh = *reinterpret_cast<const bf16x8_t*>(w16h + wo + (int64_t)(tap + 1) * g.C);
        nl = *reinterpret_cast<const bf16x8_t*>(w16l + wo + (int64_t)(tap + 1) * g.C);
      }
      const int prow = (wave * 4 + r) * g.HC + s + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = prow + i * g.HC;
        const int ix = p * NCH + hswz<NCH>(p, fq);
        const bf16x8_t bh = __builtin_bit_cast(bf16x8_t, hh[ix]);
        const bf16x8_t bl = __builtin_bit_cast(bf16x8_t, hl[ix]);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[i], 0, 0, 0);
      }
      if (++s == g.S) {
        s = 0;
        ++r;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oh = oh0 + wave * 4 + i, ow = ow0 + fr;
    if (oh >= g.P || ow >= g.Q) continue;
    float* yo = y + (((int64_t)n * g.YH + oh * g.ys + g.ya) * g.YW + ow * g.ys + g.yb) * g.K;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = fq * 4 + e;
      if (k < g.K) yo[k] = acc[i][e] + (bias ? bias[k] : 0.f);
    }
  }
}

// Stride-1 tiny-channel forward from an LDS halo tile (C <= 4: StyleNet's 9x9 3->32 input conv,
// VGG 3->64): conv_tinyc_fwd_k gathers every im2col value from L1/L2 (R*S*C scalar loads per
// output pixel) and is gather bound.  Here a workgroup owns a 16 x 16 output tile, stages its
// (16+R-1) x (16+S-1) halo once -- 4 channels per pixel (zero past C), reflect / zero padding
// resolved, fp32 split into bf16 hi / lo on the way -- and the reduction runs in (tap, 4-channel)
// order, so a lane's 8-deep B fragment is two 8-B LDS reads (two adjacent taps of its pixel).
// Weights [K][32*KT] packed in that order (KT = ceil(R*S/8)); bf16 runs one MFMA per pair, fp32
// three (wh.xh + wh.xl + wl.xh).
template <bool F32, bool RELU>
__global__ __launch_bounds__(kNT) void conv_tinyhalo_fwd_k(const void* __restrict__ x_, const uint16_t* __restrict__ wph,
                                                           const uint16_t* __restrict__ wpl,
                                                           const float* __restrict__ bias, void* __restrict__ y_,
                                                           NarrowGeom g, int KT) {
  __shared__ __attribute__((aligned(16))) uint2 hh[kHaloPix];
  __shared__ __attribute__((aligned(16))) uint2 hl[F32 ? kHaloPix : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_img = g.tiles_h * g.tiles_w;
  const int n = blockIdx.x / per_img, rem = blockIdx.x - n * per_img;
  const int th = rem / g.tiles_w;
  const int oh0 = th * kTH, ow0 = (rem - th * g.tiles_w) * kTW;
  const int64_t img = (int64_t)n * g.H * g.W;
  for (int p = tid; p < g.HR * g.HC; p += kNT) {
    const int hr = p / g.HC, hc = p - hr * g.HC;
    const int vh = vmap(oh0 - g.pad + hr, g.H, g.reflect), vw = vmap(ow0 - g.pad + hc, g.W, g.reflect);
    float f[4] = {0.f, 0.f, 0.f, 0.f};
    if (vh >= 0 && vw >= 0) {
      const int64_t off = (img + (int64_t)vh * g.W + vw) * g.C;
      for (int c = 0; c < g.C; ++c) {
        if constexpr (F32) f[c] = static_cast<const float*>(x_)[off + c];
        else f[c] = bf2f(static_cast<const uint16_t*>(x_)[off + c]);
      }
    }
    uint16_t h[4], l[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      h[c] = f2bf(f[c]);
      l[c] = f2bf(f[c] - bf2f(h[c]));
    }
    hh[p] = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
    if constexpr (F32) hl[p] = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
  }
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  const int kb0 = blockIdx.y * 64;
  const int nkb = min(4, (g.K - kb0) / 16);
  const int RS = g.R * g.S;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < KT; ++t) {
    bf16x8_t ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t o = (int64_t)(kb0 + 16 * i + fr) * (32 * KT) + 32 * t + 8 * fq;
      ah[i] = i < nkb ? *reinterpret_cast<const bf16x8_t*>(wph + o) : bf16x8_t{};
      if constexpr (F32) al[i] = i < nkb ? *reinterpret_cast<const bf16x8_t*>(wpl + o) : bf16x8_t{};
    }
    // this lane's two taps (zero weights past R*S: read tap 0 there)
    int tap0 = 8 * t + 2 * fq, tap1 = tap0 + 1;
    tap0 = tap0 < RS ? tap0 : 0;
    tap1 = tap1 < RS ? tap1 : 0;
    const int r0 = tap0 / g.S, s0 = tap0 - r0 * g.S, r1 = tap1 / g.S, s1 = tap1 - r1 * g.S;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wave * 4 + j;
      const int p0 = (row + r0) * g.HC + fr + s0, p1 = (row + r1) * g.HC + fr + s1;
      const uint2 u0 = hh[p0], u1 = hh[p1];
      const bf16x8_t bh = __builtin_bit_cast(bf16x8_t, make_uint4(u0.x, u0.y, u1.x, u1.y));
      if constexpr (F32) {
        const uint2 v0 = hl[p0], v1 = hl[p1];
        const bf16x8_t bl = __builtin_bit_cast(bf16x8_t, make_uint4(v0.x, v0.y, v1.x, v1.y));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < nkb) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < nkb) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][j], 0, 0, 0);
      }
    }
  }
  // D[ch][pix]: lane holds channels 16 i + 4 fq + e of tile pixel (row wave*4 + j, col fr)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= nkb) continue;
    const int c0 = kb0 + 16 * i + 4 * fq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bias[c0 + e];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oh = oh0 + wave * 4 + j, ow = ow0 + fr;
      if (oh >= g.P || ow >= g.Q) continue;
      const int64_t yi = (((int64_t)n * g.P + oh) * g.Q + ow) * g.K + c0;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bv[e];
        if constexpr (RELU) v[e] = fmaxf(v[e], 0.f);
      }
      if constexpr (F32) {
        *reinterpret_cast<float4*>(static_cast<float*>(y_) + yi) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(y_) + yi) =
            make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                       (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
      }
    }
  }
}

// Weight gradient of the same stride-1 tiny-channel convolution (StyleNet's 9x9 3->32 input conv):
//
//   dW[k][tap][c] = sum_pix dy[pix][k] * halo[pix + tap][c]     (c < 4, zero past C)
//
// as D[k][idx = 4 tap + c] += dyᵀ[k][32 pixels] . im2col[32 pixels][idx] on MFMA.  A workgroup walks
// 16 x 16 output tiles (blockIdx.x, + gridDim.x, ...); per tile it stages the input halo (as the
// forward) and dy TRANSPOSED to [k][pixel] (rows padded to 264 for conflict-free A reads), then
// each wave accumulates its share of the idx column tiles (j = wave + 4 jj) over the tile's 256
// pixels; B (8 pixels of one tile row at the tap's offset, one channel) is gathered from the halo.
// fp32: x and dy split into bf16 hi / lo while staging, three MFMAs per pair.  Partial sums go to
// part[block][K][16 * NJ] in f32 and tinyhalo_wgrad_reduce_k sums them in block order.
constexpr int kDyT = 264;  // dyᵀ row stride (u16)

template <bool F32>
__global__ __launch_bounds__(kNT, 2) void conv_tinyhalo_wgrad_k(const void* __restrict__ x_, const void* __restrict__ dy_,
                                                                float* __restrict__ part, NarrowGeom g, int ntiles,
                                                                int NJ) {
  __shared__ __attribute__((aligned(16))) uint2 hh[kHaloPix];
  __shared__ __attribute__((aligned(16))) uint2 hl[F32 ? kHaloPix : 1];
  __shared__ __attribute__((aligned(16))) uint16_t dth[64 * kDyT];
  __shared__ __attribute__((aligned(16))) uint16_t dtl[F32 ? 64 * kDyT : 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int KT16 = g.K / 16, RS = g.R * g.S;
  const int per_img = g.tiles_h * g.tiles_w;
  f32x4_t acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) acc[i][jj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint16_t* hh16 = reinterpret_cast<const uint16_t*>(hh);
  const uint16_t* hl16 = reinterpret_cast<const uint16_t*>(hl);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / per_img, rem = t - n * per_img;
    const int th = rem / g.tiles_w;
    const int oh0 = th * kTH, ow0 = (rem - th * g.tiles_w) * kTW;
    const int64_t img = (int64_t)n * g.H * g.W;
    __syncthreads();  // every wave is done with the previous tile
    for (int p = tid; p < g.HR * g.HC; p += kNT) {
      const int hr = p / g.HC, hc = p - hr * g.HC;
      const int vh = vmap(oh0 - g.pad + hr, g.H, g.reflect), vw = vmap(ow0 - g.pad + hc, g.W, g.reflect);
      float f[4] = {0.f, 0.f, 0.f, 0.f};
      if (vh >= 0 && vw >= 0) {
        const int64_t off = (img + (int64_t)vh * g.W + vw) * g.C;
        for (int c = 0; c < g.C; ++c) {
          if constexpr (F32) f[c] = static_cast<const float*>(x_)[off + c];
          else f[c] = bf2f(static_cast<const uint16_t*>(x_)[off + c]);
        }
      }
      uint16_t h[4], l[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        h[c] = f2bf(f[c]);
        l[c] = f2bf(f[c] - bf2f(h[c]));
      }
      hh[p] = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
      if constexpr (F32) hl[p] = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
    }
    // dy tile -> dyᵀ[k][pixel] (zero outside the output)
    const int cg8 = g.K / 8;
    for (int e = tid; e < 256 * cg8; e += kNT) {
      const int pix = e / cg8, cg = e - pix * cg8;
      const int oh = oh0 + (pix >> 4), ow = ow0 + (pix & 15);
      float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (oh < g.P && ow < g.Q) {
        const int64_t off = (((int64_t)n * g.P + oh) * g.Q + ow) * g.K + cg * 8;
        if constexpr (F32) {
          const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(dy_) + off);
          const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(dy_) + off + 4);
          f[0] = a.x, f[1] = a.y, f[2] = a.z, f[3] = a.w, f[4] = b.x, f[5] = b.y, f[6] = b.z, f[7] = b.w;
        } else {
          const uint4 u = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(dy_) + off);
          const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f[2 * q] = bf2f((uint16_t)(w[q] & 0xffff));
            f[2 * q + 1] = bf2f((uint16_t)(w[q] >> 16));
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint16_t hv = f2bf(f[q]);
        dth[(cg * 8 + q) * kDyT + pix] = hv;
        if constexpr (F32) dtl[(cg * 8 + q) * kDyT + pix] = f2bf(f[q] - bf2f(hv));
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int ps = 0; ps < 8; ++ps) {
      const int p0 = 32 * ps + 8 * fq;            // this lane's 8 tile pixels (one tile row)
      const int pr = p0 >> 4, pc0 = p0 & 15;
      bf16x8_t ah[4], al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < KT16) {
          ah[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(dth + (16 * i + fr) * kDyT + p0));
          if constexpr (F32)
            al[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(dtl + (16 * i + fr) * kDyT + p0));
        }
      }
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) {
        const int j = wave + 4 * jj;
        if (j >= NJ) continue;
        const int idx = 16 * j + fr, tap = idx >> 2, c = idx & 3;
        const bool ok = tap < RS;
        const int r = ok ? tap / g.S : 0, s = ok ? tap - (tap / g.S) * g.S : 0;
        const int hb = ((pr + r) * g.HC + pc0 + s) * 4 + c;
        uint32_t bw[4], lw[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bw[q] = ok ? ((uint32_t)hh16[hb + 8 * q] | ((uint32_t)hh16[hb + 8 * q + 4] << 16)) : 0u;
          if constexpr (F32) lw[q] = ok ? ((uint32_t)hl16[hb + 8 * q] | ((uint32_t)hl16[hb + 8 * q + 4] << 16)) : 0u;
        }
        const bf16x8_t bh = __builtin_bit_cast(bf16x8_t, make_uint4(bw[0], bw[1], bw[2], bw[3]));
        if constexpr (F32) {
          const bf16x8_t bl = __builtin_bit_cast(bf16x8_t, make_uint4(lw[0], lw[1], lw[2], lw[3]));
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < KT16) {
              acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][jj], 0, 0, 0);
              acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][jj], 0, 0, 0);
              acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][jj], 0, 0, 0);
            }
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < KT16) acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][jj], 0, 0, 0);
        }
      }
    }
  }
  // D[k][idx]: lane holds k = 16 i + 4 fq + e, idx = 16 j + fr
  float* pb = part + (int64_t)blockIdx.x * g.K * (16 * NJ);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= KT16) continue;
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int j = wave + 4 * jj;
      if (j >= NJ) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) pb[(int64_t)(16 * i + 4 * fq + e) * (16 * NJ) + 16 * j + fr] = acc[i][jj][e];
    }
  }
}

// dW [K][R][S][C] (fp32 or bf16) = sum over blocks of part[b][k][4 tap + c], in block order
template <bool F32OUT>
__global__ __launch_bounds__(256) void tinyhalo_wgrad_reduce_k(const float* __restrict__ part, int nb, int K, int RS,
                                                               int C, int NJ, void* __restrict__ dw) {
  const int total = K * RS * C;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < total; o += gridDim.x * 256) {
    const int c = o % C, t = o / C, tap = t % RS, k = t / RS;
    const int64_t col = (int64_t)k * (16 * NJ) + 4 * tap + c;
    float v = 0.f;
    for (int b = 0; b < nb; ++b) v += part[(int64_t)b * K * (16 * NJ) + col];
    if constexpr (F32OUT) static_cast<float*>(dw)[o] = v;
    else static_cast<uint16_t*>(dw)[o] = f2bf(v);
  }
}

}  // namespace

int conv_tinyhalo_wgrad_blocks(int N, int H, int W, int R, int S, int pad) {
  const int P = H + 2 * pad - R + 1, Q = W + 2 * pad - S + 1;
  const int ntiles = N * cdiv(P, kTH) * cdiv(Q, kTW);
  return ntiles < 512 ? ntiles : 512;
}

int conv_tinyhalo_wgrad_cols(int R, int S) { return cdiv(R * S * 4, 16); }

// dW of conv_tinyhalo_fwd's convolution: x [N][H][W][C], dy [N][P][Q][K] (fp32 or bf16), K % 16 == 0,
// K <= 64; part holds blocks * K * 16 * cols floats; dw [K][R][S][C] in x's dtype
void conv_tinyhalo_wgrad(bool f32, const void* x, const void* dy, float* part, void* dw, int N, int H, int W, int C,
                         int K, int R, int S, int pad, int reflect, hipStream_t st) {
  NarrowGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.pad = pad, g.padw = pad;
  g.upsh = 0, g.reflect = reflect ? 1 : 0, g.Hv = H, g.Wv = W;
  g.P = H + 2 * pad - R + 1, g.Q = W + 2 * pad - S + 1;
  g.HR = kTH + R - 1, g.HC = kTW + S - 1;
  g.tiles_h = cdiv(g.P, kTH), g.tiles_w = cdiv(g.Q, kTW);
  g.ys = 1, g.ya = g.yb = 0, g.YH = g.P, g.YW = g.Q;
  const int ntiles = N * g.tiles_h * g.tiles_w;
  if (ntiles <= 0) return;
  const int nb = conv_tinyhalo_wgrad_blocks(N, H, W, R, S, pad), NJ = conv_tinyhalo_wgrad_cols(R, S);
  if (f32) conv_tinyhalo_wgrad_k<true><<<nb, kNT, 0, st>>>(x, dy, part, g, ntiles, NJ);
  else conv_tinyhalo_wgrad_k<false><<<nb, kNT, 0, st>>>(x, dy, part, g, ntiles, NJ);
  const int total = K * R * S * C;
  const int rb = cdiv(total, 256) < 1024 ? cdiv(total, 256) : 1024;
  if (f32) tinyhalo_wgrad_reduce_k<true><<<rb, 256, 0, st>>>(part, nb, K, R * S, C, NJ, dw);
  else tinyhalo_wgrad_reduce_k<false><<<rb, 256, 0, st>>>(part, nb, K, R * S, C, NJ, dw);
}

int conv_tinyhalo_supported(int C, int K, int R, int S, int stride, int up) {
  return C >= 1 && C <= 4 && K % 16 == 0 && K >= 16 && R <= kMaxTap && S <= kMaxTap && stride == 1 && up == 1;
}

// x [N][H][W][C] (fp32 or bf16), (wph, wpl) [K][32*KT] packed in (tap, 4-channel) order (wpl fp32 only),
// y [N][P][Q][K] (fp32 or bf16); stride 1, zero or reflect padding
void conv_tinyhalo_fwd(bool f32, const void* x, const void* wph, const void* wpl, const float* bias, void* y, int N,
                       int H, int W, int C, int K, int R, int S, int pad, int reflect, bool relu, hipStream_t st) {
  NarrowGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.pad = pad, g.padw = pad;
  g.upsh = 0, g.reflect = reflect ? 1 : 0, g.Hv = H, g.Wv = W;
  g.P = H + 2 * pad - R + 1, g.Q = W + 2 * pad - S + 1;
  g.HR = kTH + R - 1, g.HC = kTW + S - 1;
  g.tiles_h = cdiv(g.P, kTH), g.tiles_w = cdiv(g.Q, kTW);
  g.ys = 1, g.ya = g.yb = 0, g.YH = g.P, g.YW = g.Q;
  const int KT = cdiv(R * S, 8);
  const dim3 grid(N * g.tiles_h * g.tiles_w, cdiv(K, 64));
  if (grid.x == 0) return;
  const uint16_t *wh = (const uint16_t*)wph, *wl = (const uint16_t*)wpl;
  if (f32) {
    if (relu) conv_tinyhalo_fwd_k<true, true><<<grid, kNT, 0, st>>>(x, wh, wl, bias, y, g, KT);
    else conv_tinyhalo_fwd_k<true, false><<<grid, kNT, 0, st>>>(x, wh, wl, bias, y, g, KT);
  } else {
    if (relu) conv_tinyhalo_fwd_k<false, true><<<grid, kNT, 0, st>>>(x, wh, wl, bias, y, g, KT);
    else conv_tinyhalo_fwd_k<false, false><<<grid, kNT, 0, st>>>(x, wh, wl, bias, y, g, KT);
  }
}

// fp32 x [N][H][W][C], (wph, wpl) [K][32*KT] packed bf16 split pair, y f32 [N][P][Q][K]
void conv_tiny32_fwd(const float* x, const void* wph, const void* wpl, const int* tab, const float* bias, float* y,
                     int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int reflect, bool relu,
                     hipStream_t st) {
  TinyGeom g{N, H, W, C, K, R, S, 0, 0, stride, pad, reflect ? 1 : 0, C * R * S};
  g.P = (H + 2 * pad - R) / stride + 1;
  g.Q = (W + 2 * pad - S) / stride + 1;
  const int64_t NPQ = (int64_t)N * g.P * g.Q;
  if (NPQ <= 0) return;
  const int KT = cdiv(g.kred, 32);
  const dim3 grid((unsigned)cdiv(NPQ, 256), cdiv(K, 64));
  const uint16_t* wh = (const uint16_t*)wph;
  const uint16_t* wl = (const uint16_t*)wpl;
#define TB_TINY32(KT_)                                                                                 \
  case KT_:                                                                                            \
    if (relu) conv_tiny32_fwd_k<KT_, true><<<grid, kNT, 0, st>>>(x, wh, wl, tab, bias, y, g);         \
    else conv_tiny32_fwd_k<KT_, false><<<grid, kNT, 0, st>>>(x, wh, wl, tab, bias, y, g);             \
    break;
  switch (KT) {
    TB_TINY32(1)
    TB_TINY32(2)
    TB_TINY32(3)
    TB_TINY32(4)
    TB_TINY32(5)
    TB_TINY32(6)
    TB_TINY32(7)
    TB_TINY32(8)
    default: break;
  }
#undef TB_TINY32
}

// One stride phase (a, b) of a transposed convolution as a narrow forward: output pixels
// (m * st + a, n * st + b) of y [N][YH][YW][K] read the R' x S' input window starting at
// (m - pad_h, n - pad_w) (zero padding) with the phase's weights w16 [16][R'][S'][C].
void conv_narrow_fwd_phase(const void* x, const void* w16, const float* bias, void* y, int N, int H, int W, int C,
                           int K, int R, int S, int pad_h, int pad_w, int P, int Q, int st, int a, int b, int YH,
                           int YW, hipStream_t st_) {
  NarrowGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.pad = pad_h, g.padw = pad_w;
  g.upsh = 0, g.reflect = 0, g.Hv = H, g.Wv = W, g.P = P, g.Q = Q;
  g.HR = kTH + R - 1, g.HC = kTW + S - 1;
  g.tiles_h = cdiv(P, kTH), g.tiles_w = cdiv(Q, kTW);
  g.ys = st, g.ya = a, g.yb = b, g.YH = YH, g.YW = YW;
  const int grid = N * g.tiles_h * g.tiles_w;
  if (grid == 0) return;
  if (C == 64)
    conv_narrow_fwd_k<8><<<grid, kNT, 0, st_>>>((const uint16_t*)x, (const uint16_t*)w16, bias, (uint16_t*)y, g);
  else
    conv_narrow_fwd_k<4><<<grid, kNT, 0, st_>>>((const uint16_t*)x, (const uint16_t*)w16, bias, (uint16_t*)y, g);
}

int conv_tinyc_supported(int C, int K, int R, int S) { return C * R * S <= 256 && K % 16 == 0 && K >= 16; }

// x [N][H][W][C], wp [K][32*KT] packed (r, s, c)-major reduction rows (zero tail), tab [kred] codes
// r | s << 8 | c << 16, y [N][P][Q][K]; zero or reflect padding
void conv_tinyc_fwd(const void* x, const void* wp, const int* tab, const float* bias, void* y, int N, int H, int W,
                    int C, int K, int R, int S, int stride, int pad, int reflect, bool relu, hipStream_t st) {
  TinyGeom g{N, H, W, C, K, R, S, 0, 0, stride, pad, reflect ? 1 : 0, C * R * S};
  g.P = (H + 2 * pad - R) / stride + 1;
  g.Q = (W + 2 * pad - S) / stride + 1;
  const int64_t NPQ = (int64_t)N * g.P * g.Q;
  if (NPQ <= 0) return;
  const int KT = cdiv(g.kred, 32);
  const dim3 grid((unsigned)cdiv(NPQ, 256), cdiv(K, 64));
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)wp;
  uint16_t* yy = (uint16_t*)y;
#define TB_TINY(KT_)                                                                                        \
  case KT_:                                                                                                 \
    if (relu) conv_tinyc_fwd_k<KT_, true><<<grid, kNT, 0, st>>>(xx, ww, tab, bias, yy, g);                \
    else conv_tinyc_fwd_k<KT_, false><<<grid, kNT, 0, st>>>(xx, ww, tab, bias, yy, g);                    \
    break;
  switch (KT) {
    TB_TINY(1)
    TB_TINY(2)
    TB_TINY(3)
    TB_TINY(4)
    TB_TINY(5)
    TB_TINY(6)
    TB_TINY(7)
    default:
      TB_TINY(8)
  }
#undef TB_TINY
}

void conv_narrow_fwd32(const float* x, const void* w16h, const void* w16l, const float* bias, float* y, int N, int H,
                       int W, int C, int K, int R, int S, int pad, int up, int reflect, hipStream_t st) {
  NarrowGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.pad = pad;
  g.upsh = up == 4 ? 2 : (up == 2 ? 1 : 0);
  g.reflect = reflect ? 1 : 0;
  g.Hv = H * up, g.Wv = W * up;
  g.P = g.Hv + 2 * pad - R + 1, g.Q = g.Wv + 2 * pad - S + 1;
  g.HR = kTH + R - 1, g.HC = kTW + S - 1;
  g.tiles_h = cdiv(g.P, kTH), g.tiles_w = cdiv(g.Q, kTW);
  g.ys = 1, g.ya = g.yb = 0, g.YH = g.P, g.YW = g.Q, g.padw = pad;
  const int grid = N * g.tiles_h * g.tiles_w;
  if (grid == 0) return;
  const uint16_t *wh = (const uint16_t*)w16h, *wl = (const uint16_t*)w16l;
  if (C == 64) conv_narrow32_fwd_k<2><<<grid, kNT, 0, st>>>(x, wh, wl, bias, y, g);
  else conv_narrow32_fwd_k<1><<<grid, kNT, 0, st>>>(x, wh, wl, bias, y, g);
}

int conv_narrow_supported(int C, int K, int R, int S, int stride, int up) {
  return (C == 32 || C == 64) && K >= 1 && K <= 16 && R <= kMaxTap && S <= kMaxTap && stride == 1 &&
         (up == 1 || up == 2 || up == 4);
}

// x [N][H][W][C] bf16, w16 [16][R][S][C] bf16 (rows >= K zero), bias f32 [K] or null,
// y [N][P][Q][K] bf16; the input is read through pad(upsample_nearest(x, up), pad, reflect|zero)
void conv_narrow_fwd(const void* x, const void* w16, const float* bias, void* y, int N, int H, int W, int C, int K,
                     int R, int S, int pad, int up, int reflect, hipStream_t st) {
  NarrowGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.pad = pad;
  g.upsh = up == 4 ? 2 : (up == 2 ? 1 : 0);
  g.reflect = reflect ? 1 : 0;
  g.Hv = H * up, g.Wv = W * up;
  g.P = g.Hv + 2 * pad - R + 1, g.Q = g.Wv + 2 * pad - S + 1;
  g.HR = kTH + R - 1, g.HC = kTW + S - 1;
  g.tiles_h = cdiv(g.P, kTH), g.tiles_w = cdiv(g.Q, kTW);
  g.ys = 1, g.ya = g.yb = 0, g.YH = g.P, g.YW = g.Q, g.padw = pad;
  const int grid = N * g.tiles_h * g.tiles_w;
  if (grid == 0) return;
  if (C == 64)
    conv_narrow_fwd_k<8><<<grid, kNT, 0, st>>>((const uint16_t*)x, (const uint16_t*)w16, bias, (uint16_t*)y, g);
  else
    conv_narrow_fwd_k<4><<<grid, kNT, 0, st>>>((const uint16_t*)x, (const uint16_t*)w16, bias, (uint16_t*)y, g);
}

// dW partials for conv_narrow_fwd's convolution: part [splits][16][R*S][C] f32 (summed over the
// splits and rows >= K dropped by the caller).  Returns nothing; see conv_narrow_wgrad_splits.
int conv_narrow_wgrad_splits(int N, int H, int W, int C, int R, int S, int pad, int up) {
  const int P = H * up + 2 * pad - R + 1, Q = W * up + 2 * pad - S + 1;
  const int ntiles = N * cdiv(P, kTH) * cdiv(Q, kTW);
  // ~2 resident workgroups per CU across the C / 16 channel blocks, >= 4 tiles each
  int splits = cdiv(512, C / 16);
  splits = std::min(splits, std::max(1, ntiles / 4));
  const int per = cdiv(ntiles, splits);
  return cdiv(ntiles, per);
}

void conv_narrow_wgrad(const void* x, const void* dy, float* part, int splits, int N, int H, int W, int C, int K,
                       int R, int S, int pad, int up, int reflect, hipStream_t st) {
  NarrowGeom g{};
  g.N = N, g.H = H, g.W = W, g.C = C, g.K = K, g.R = R, g.S = S, g.pad = pad;
  g.upsh = up == 4 ? 2 : (up == 2 ? 1 : 0);
  g.reflect = reflect ? 1 : 0;
  g.Hv = H * up, g.Wv = W * up;
  g.P = g.Hv + 2 * pad - R + 1, g.Q = g.Wv + 2 * pad - S + 1;
  g.HR = kTH + R - 1, g.HC = kTW + S - 1;
  g.tiles_h = cdiv(g.P, kTH), g.tiles_w = cdiv(g.Q, kTW);
  g.ys = 1, g.ya = g.yb = 0, g.YH = g.P, g.YW = g.Q, g.padw = pad;
  const int ntiles = N * g.tiles_h * g.tiles_w;
  const int per = cdiv(ntiles, splits);
  conv_narrow_wgrad_k<<<splits * (C / 16), kNT, 0, st>>>((const uint16_t*)x, (const uint16_t*)dy, part, g, per);
}

}  // namespace tbamd
