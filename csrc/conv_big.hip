// Big-tile implicit-GEMM NHWC convolution for gfx950: one 8-wave workgroup per CU.
//
// Reference: every conv of the examples goes through cuDNN (torchvision ResNet, resnet.py:44-68,111;
// SURVEY.md §2.3.1 K1/K2).  The round-1..4 kernel (conv.hip conv_fwd_k) runs 128x128 tiles with 4
// waves and 2-4 workgroups per CU: every workgroup pulls 32 KiB of operands per 2.1 MFLOP through L2
// and waits on each k-tile's loads with a single LDS stage (19-24 % MFMA busy on the ResNet-50
// step, profiles/r04_pmc).  Here:
//
//   * a BN (256 or 128) pixel x BM (64 / 128 / 256) channel tile per workgroup, 8 waves (512
//     threads, 2 per SIMD), one workgroup per CU: 25-50 % fewer L2 bytes per FLOP than 128x128;
//   * a ring of STAGES LDS buffers filled by direct-to-LDS loads (global_load_lds, 16 B per lane)
//     with STAGES-1 k-tiles in flight ACROSS the one raw barrier per k-tile: a counted vmcnt,
//     never 0 inside the loop (cdna_hip_programming.md §5 "Pipelining across barriers");
//   * MFMA v_mfma_f32_16x16x32_bf16 (MF = 16) or v_mfma_f32_32x32x16_bf16 (MF = 32) on the same
//     LDS image (128-B rows, 16-B chunks XOR-swizzled by (row >> 1) & 7: conflict-free
//     ds_read_b128 for both fragment shapes);
//   * the same fused epilogues as conv_fwd_k, computed from the bf16 output tile staged in LDS
//     (so they are independent of the MFMA shape): bias / ReLU, BatchNorm statistics (STATS), a
//     residual addend optionally masked by saved ReLU bits (ADD 1 / 2), and the BN-backward
//     partials of the BN whose output gradient this dgrad is (BNB 1 / 2 / 3).
//
//   y[n,p,q,k] = sum_{r,s,c} x[n, p*st-pad+r, q*st-pad+s, c] * w[k,r,s,c]
//   D[k][pixel] = W[k][(r,s,c)] . Xcol[(r,s,c)][pixel]  (A = weights, B = activations)
//
// Requirements (host-checked): C % 64 == 0, K % BM == 0, bf16.  A stride-1 input gradient is the
// same kernel on dY with flipped / transposed weights (ops/conv.py).
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int kBK = 64;
constexpr int kThreads = 512;

struct BigGeom {
  int N, H, W, C, K, R, S, P, Q, st, pad;
};

struct BigEpi {
  const float* bias;
  float* stats;            // STATS: [ntn][2][K] raw (sum, sum of squares) of the bf16 outputs
  const uint16_t* addend;  // ADD: y += addend (ADD 2: masked by amask bits)
  const uint8_t* amask;
  const uint16_t* xb;      // BNB: the BN input (pre-BN activations), [NPQ][K]
  const float* scale;      // BNB 1: ReLU mask recomputed as fma(xb, scale, shift) > 0
  const float* shift;
  const float* mean;       // BNB: batch mean of xb
  const uint8_t* bits;     // BNB 2: saved ReLU bits
  float* part;             // BNB: [ntn][2][K] = (sum dz, sum dz * (xb - mean))
};

__device__ __forceinline__ int bswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// zero source for out-of-image taps and rows past the last pixel: the direct-to-LDS loads copy
// from here instead of being masked (no per-lane select on the staging path)
__device__ __attribute__((aligned(64))) uint4 g_big_zero_page[16];

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

template <int BM, int BN, int MF, int STAGES, bool STATS, bool BIAS, bool RELU, int ADD, int BNB>
__global__ __launch_bounds__(kThreads, 2) void conv_big_k(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ y, BigGeom g, BigEpi e) {
  static_assert(BM == 64 || BM == 128 || BM == 256, "BM");
  static_assert(BN == 128 || BN == 256, "BN");
  static_assert(MF == 16 || MF == 32, "MFMA shape");
  static_assert(!(STATS && (ADD || BNB)), "STATS is a forward epilogue; ADD / BNB are dgrad epilogues");
  constexpr int BK = kBK;
  // wave grid: BM / 64 waves along the channels, the rest along the pixels
  constexpr int WGM = BM / 64, WGN = 8 / WGM;
  constexpr int WM = 64, WN = BN / WGN;
  static_assert(WN >= MF && WN % MF == 0, "wave tile");
  constexpr int TM = WM / MF, TN = WN / MF;
  constexpr int A_PASSES = BM / 64, B_PASSES = BN / 64;  // 8 waves x 8 rows = 64 rows per pass
  constexpr int LPT = A_PASSES + B_PASSES;               // direct-to-LDS loads per lane per k-tile
  constexpr int STAGE_U4 = (BM + BN) * BK / 8;
  constexpr int OUT_U4 = BN * BM / 8;                     // epilogue: bf16 tile [BN][BM]
  constexpr int RED_F = 8 * 2 * BM;                       // epilogue: [8 waves][2][BM] floats
  constexpr int LDS_U4 = STAGES * STAGE_U4 > OUT_U4 + RED_F / 4 ? STAGES * STAGE_U4 : OUT_U4 + RED_F / 4;
  static_assert(LDS_U4 * 16 <= 160 * 1024, "LDS");
  // ONE shared array (staging ring, then the epilogue tile): see the second-__shared__-object trap,
  // cdna_hip_programming.md §5
  __shared__ __attribute__((aligned(16))) uint4 lds[LDS_U4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const int ntm = g.K / BM;
  const int ntn = (int)((NPQ + BN - 1) / BN);
  int bid = blockIdx.x;
  {
    // XCD-aware remap (bijective for any grid): blocks b and b+8 share an XCD, so each XCD gets a
    // contiguous range of tile ids -- the channel tiles of one pixel tile share its L2
    const int nwg = ntm * ntn;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  const int tile_m = bid % ntm;
  const int tile_n = bid / ntm;
  const int m0 = tile_m * BM;
  const int64_t n0 = (int64_t)tile_n * BN;

  const int Kred = g.R * g.S * g.C;
  const int cblocks = g.C / BK;
  const int KT = g.R * g.S * cblocks;
  const int lrow = wave * 8 + (lane >> 3);  // row within a 64-row pass
  const int slot = lane & 7;

  int64_t pix_base[B_PASSES];
  int pix_h[B_PASSES], pix_w[B_PASSES];
#pragma unroll
  for (int i = 0; i < B_PASSES; ++i) {
    const int64_t pix = n0 + lrow + 64 * i;
    const bool ok = pix < NPQ;
    const int64_t pp = ok ? pix : 0;
    const int q = (int)(pp % g.Q);
    const int64_t t = pp / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    pix_h[i] = ok ? p * g.st - g.pad : -(1 << 20);  // rows past NPQ never pass the bounds test
    pix_w[i] = q * g.st - g.pad;
    pix_base[i] = (((int64_t)n * g.H + pix_h[i]) * g.W + pix_w[i]) * g.C + (slot ^ bswz(lrow, 0)) * 8;
  }
  // A passes: rows lrow + 64 i share lrow's swizzle (64 % 16 == 0): one pointer, uniform pass stride
  const uint16_t* wsrc0 = w + (int64_t)(m0 + lrow) * Kred + (slot ^ bswz(lrow, 0)) * 8;
  const int64_t wpass = (int64_t)64 * Kred;
  const void* zpage = pin_sgpr(g_big_zero_page);

  auto issue = [&](int kt, int buf) {
    const int rs = kt / cblocks, cb = kt - rs * cblocks;
    const int r = rs / g.S, s = rs - r * g.S;
    uint4* A = lds + buf * STAGE_U4;
    uint4* B = A + BM * BK / 8;
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      const uint16_t* src = wsrc0 + i * wpass + kt * BK;
      const bool wok = TB_BOUNDS_OK(src + 8 <= w + (int64_t)g.K * Kred, kBndConvW);
      glds16(wok ? (const void*)src : zpage, A + (64 * i + wave * 8) * 8);
    }
    const int64_t tap = ((int64_t)r * g.W + s) * g.C + cb * BK;
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      const int ih = pix_h[i] + r, iw = pix_w[i] + s;
      bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const int64_t off = pix_base[i] + tap;
      ok = ok && TB_BOUNDS_OK(off >= 0 && off + 8 <= (int64_t)g.N * g.H * g.W * g.C, kBndConvSrc);
      glds16(ok ? (const void*)(x + off) : zpage, B + (64 * i + wave * 8) * 8);
    }
  };

  // accumulators: TM x TN MFMA tiles of MF x MF
  using acc_t = std::conditional_t<MF == 16, f32x4_t, f32x16_t>;
  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = acc_t{};

  auto compute = [&](int buf) {
    const uint4* A = lds + buf * STAGE_U4;
    const uint4* B = A + BM * BK / 8;
    if constexpr (MF == 16) {
      const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8_t af[TM], bfr[TN];
        const int ch = ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 16 + fr;
          af[i] = __builtin_bit_cast(bf16x8_t, A[row * 8 + bswz(row, ch)]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + j * 16 + fr;
          bfr[j] = __builtin_bit_cast(bf16x8_t, B[row * 8 + bswz(row, ch)]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        bf16x8_t af[TM], bfr[TN];
        const int ch = kk * 2 + fh;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 32 + fr;
          af[i] = __builtin_bit_cast(bf16x8_t, A[row * 8 + bswz(row, ch)]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + j * 32 + fr;
          bfr[j] = __builtin_bit_cast(bf16x8_t, B[row * 8 + bswz(row, ch)]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // ---- main loop: ring of STAGES buffers, STAGES-1 k-tiles in flight, ONE raw barrier per k-tile.
  // Iteration kt: wait for this lane's loads of tile kt (a COUNTED vmcnt leaves the younger tiles in
  // flight), barrier (every wave's tile-kt DMA has landed; every wave finished reading tile kt-1,
  // whose buffer is the one refilled next), issue tile kt+STAGES-1, multiply tile kt.
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < KT) issue(t, t);
  int cur = 0, nxt = STAGES - 1;
  for (int kt = 0; kt < KT; ++kt) {
    if constexpr (STAGES == 3) {
      if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (STAGES == 4) {
      if (kt + 2 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPT) : "memory");
      else if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + STAGES - 1 < KT) issue(kt + STAGES - 1, nxt);
    compute(cur);
    cur = cur + 1 == STAGES ? 0 : cur + 1;
    nxt = nxt + 1 == STAGES ? 0 : nxt + 1;
  }
  __syncthreads();  // every wave is done with the ring before the epilogue reuses it

  // ---- epilogue 1: accumulators (+ bias, ReLU) -> bf16 -> LDS tile [BN pixels][BM channels],
  // 16-B chunk index XOR-swizzled by the pixel row (conflict-free row reads below)
  constexpr int CPR = BM / 8;  // 16-B chunks per pixel row
  uint16_t* ot = reinterpret_cast<uint16_t*>(lds);
  auto put4 = [&](int cl, int pl, float v0, float v1, float v2, float v3) {
    float v[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (BIAS) v[q] += e.bias[m0 + cl + q];
      if constexpr (RELU) v[q] = fmaxf(v[q], 0.f);
    }
    const int chunk = (cl >> 3) ^ (pl & (CPR - 1));
    *reinterpret_cast<uint2*>(ot + pl * BM + chunk * 8 + (cl & 7)) =
        make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                   (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
  };
  if constexpr (MF == 16) {
    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        put4(wm * WM + i * 16 + fq * 4, wn * WN + j * 16 + fr, acc[i][j][0], acc[i][j][1], acc[i][j][2],
             acc[i][j][3]);
  } else {
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          put4(wm * WM + i * 32 + 8 * gq + 4 * fh, wn * WN + j * 32 + fr, acc[i][j][4 * gq + 0],
               acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
  }
  __syncthreads();

  // ---- epilogue 2: 16-B row stores; a thread's chunk ck (8 channels) is fixed across its rows
  // (kThreads % CPR == 0), so it accumulates the STATS sums / BN-backward partials of those 8
  // channels over its rows in registers
  const int ck = tid % CPR;
  constexpr bool SUMS = STATS || BNB != 0;
  float s0[8], s1[8];
  float bsc[8], bsf[8], bmu[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s0[q] = s1[q] = 0.f;
  if constexpr (BNB != 0) {
    const int c0 = m0 + ck * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      bmu[q] = e.mean[c0 + q];
      if constexpr (BNB == 1) {
        bsc[q] = e.scale[c0 + q];
        bsf[q] = e.shift[c0 + q];
      }
    }
  }
  constexpr int IT = BN * CPR / kThreads;
  constexpr int PB = IT < 4 ? IT : 4;  // the epilogue's global reads are issued PB rows ahead
  constexpr bool PRE = ADD != 0 || BNB != 0;
  uint4 pre_a[PRE ? PB : 1], pre_x[PRE ? PB : 1];
  uint32_t pre_am[PRE ? PB : 1], pre_xm[PRE ? PB : 1];
#pragma unroll
  for (int it0 = 0; it0 < IT; it0 += PB) {
    if constexpr (PRE) {
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int idx = (it0 + u) * kThreads + tid;
        const int pl = idx / CPR;
        const int64_t pix = n0 + pl < NPQ ? n0 + pl : NPQ - 1;  // (rows past NPQ: a valid address, unused)
        if constexpr (ADD != 0) {
          pre_a[u] = *reinterpret_cast<const uint4*>(e.addend + pix * g.K + m0 + ck * 8);
          if constexpr (ADD == 2) pre_am[u] = e.amask[pix * (g.K / 8) + (m0 >> 3) + ck];
        }
        if constexpr (BNB != 0) {
          pre_x[u] = *reinterpret_cast<const uint4*>(e.xb + pix * g.K + m0 + ck * 8);
          if constexpr (BNB == 2) pre_xm[u] = e.bits[pix * (g.K / 8) + (m0 >> 3) + ck];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int idx = (it0 + u) * kThreads + tid;
      const int pl = idx / CPR;
      const int64_t pix = n0 + pl;
      if (pix < NPQ) {
        uint4 v = *reinterpret_cast<const uint4*>(ot + pl * BM + ((ck ^ (pl & (CPR - 1))) * 8));
        if constexpr (ADD != 0) {
          uint4 a = pre_a[u];
          if constexpr (ADD == 2) {
            const uint32_t bits = pre_am[u];
            const auto keep = [&](uint32_t wv, int i) {
              return ((((bits >> i) & 1u) ? 0x0000ffffu : 0u) & wv) |
                     ((((bits >> (i + 1)) & 1u) ? 0xffff0000u : 0u) & wv);
            };
            a = make_uint4(keep(a.x, 0), keep(a.y, 2), keep(a.z, 4), keep(a.w, 6));
          }
          v = make_uint4(add_bf16x2(v.x, a.x), add_bf16x2(v.y, a.y), add_bf16x2(v.z, a.z), add_bf16x2(v.w, a.w));
        }
        if (TB_BOUNDS_OK(pix * g.K + m0 + ck * 8 + 8 <= NPQ * g.K, kBndConvDst))
          *reinterpret_cast<uint4*>(y + pix * g.K + m0 + ck * 8) = v;
        const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
        if constexpr (STATS) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float vr = bf2f((uint16_t)(vw[q >> 1] >> (16 * (q & 1))));
            s0[q] += vr;
            s1[q] += vr * vr;
          }
        }
        if constexpr (BNB != 0) {
          const uint4 xq = pre_x[u];
          const uint32_t xw[4] = {xq.x, xq.y, xq.z, xq.w};
          uint32_t bits = 0xffu;
          if constexpr (BNB == 2) bits = pre_xm[u];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float dv = bf2f((uint16_t)(vw[q >> 1] >> (16 * (q & 1))));
            const float xv = bf2f((uint16_t)(xw[q >> 1] >> (16 * (q & 1))));
            bool keep = true;
            if constexpr (BNB == 1) keep = __builtin_fmaf(xv, bsc[q], bsf[q]) > 0.f;
            if constexpr (BNB == 2) keep = (bits >> q) & 1u;
            const float dz = keep ? dv : 0.f;
            s0[q] += dz;
            s1[q] += dz * (xv - bmu[q]);
          }
        }
      }
    }
  }
  if constexpr (SUMS) {
    // reduce the rows of each chunk: lanes l, l + CPR, ... of a wave share a chunk (shuffles),
    // then the 8 waves through LDS (after the output tile; every thread busy, no serial walk)
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s0[q] += __shfl_xor(s0[q], o, 64);
        s1[q] += __shfl_xor(s1[q], o, 64);
      }
    float* red = reinterpret_cast<float*>(lds + OUT_U4);  // [8 waves][2][BM]
    if (lane < CPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wave * 2 + 0) * BM + lane * 8 + q] = s0[q];
        red[(wave * 2 + 1) * BM + lane * 8 + q] = s1[q];
      }
    }
    __syncthreads();
    float* dst = STATS ? e.stats : e.part;
    for (int qi = tid; qi < 2 * BM; qi += kThreads) {
      const int kind = qi / BM, cl = qi - kind * BM;
      float s = 0.f;
#pragma unroll
      for (int wv = 0; wv < 8; ++wv) s += red[(wv * 2 + kind) * BM + cl];
      dst[((int64_t)tile_n * 2 + kind) * g.K + m0 + cl] = s;
    }
  }
}

// per-shape mode: 0 = the 128x128 kernels (conv.hip); otherwise a packed tile choice
// (set by conv_set_big / TBAMD_CONV_BIG, and by the route table through conv_big_choice)
int g_big_mode = [] {
  const char* s = getenv("TBAMD_CONV_BIG");
  return s ? atoi(s) : 0;
}();

template <int BM, int BN, int MF, int STAGES>
void launch(const uint16_t* x, const uint16_t* w, uint16_t* y, const BigGeom& g, const BigEpi& e, bool relu,
            int bnb_mode, hipStream_t st) {
  const int64_t NPQ = (int64_t)g.N * g.P * g.Q;
  const dim3 grid((g.K / BM) * (int)((NPQ + BN - 1) / BN));
  const dim3 block(kThreads);
#define TB_BIG(ST_, BI_, RE_, AD_, BB_) \
  conv_big_k<BM, BN, MF, STAGES, ST_, BI_, RE_, AD_, BB_><<<grid, block, 0, st>>>(x, w, y, g, e)
  if (bnb_mode != 0) {
    if (e.addend && e.amask) {
      if (bnb_mode == 1) TB_BIG(false, false, false, 2, 1);
      else if (bnb_mode == 2) TB_BIG(false, false, false, 2, 2);
      else TB_BIG(false, false, false, 2, 3);
    } else if (e.addend) {
      if (bnb_mode == 1) TB_BIG(false, false, false, 1, 1);
      else if (bnb_mode == 2) TB_BIG(false, false, false, 1, 2);
      else TB_BIG(false, false, false, 1, 3);
    } else {
      if (bnb_mode == 1) TB_BIG(false, false, false, 0, 1);
      else if (bnb_mode == 2) TB_BIG(false, false, false, 0, 2);
      else TB_BIG(false, false, false, 0, 3);
    }
  } else if (e.addend) {
    if (e.amask) TB_BIG(false, false, false, 2, 0);
    else TB_BIG(false, false, false, 1, 0);
  } else if (e.stats) {
    if (e.bias) TB_BIG(true, true, false, 0, 0);
    else TB_BIG(true, false, false, 0, 0);
  } else if (e.bias) {
    if (relu) TB_BIG(false, true, true, 0, 0);
    else TB_BIG(false, true, false, 0, 0);
  } else {
    if (relu) TB_BIG(false, false, true, 0, 0);
    else TB_BIG(false, false, false, 0, 0);
  }
#undef TB_BIG
}

}  // namespace

// Tile choice encoding (conv_big_choice): 0 = not this kernel; else BM | BN << 12 | (MF == 32) << 24 |
// STAGES << 28 (BM, BN < 4096; STAGES < 8)
int conv_big_encode(int bm, int bn, int mf, int stages) {
  return bm | (bn << 12) | ((mf == 32 ? 1 : 0) << 24) | (stages << 28);
}
static void big_decode(int code, int& bm, int& bn, int& mf, int& stages) {
  bm = code & 0xfff;
  bn = (code >> 12) & 0xfff;
  mf = ((code >> 24) & 1) ? 32 : 16;
  stages = (code >> 28) & 0x7;
}

void conv_set_big(int mode) { g_big_mode = mode; }
int conv_get_big() { return g_big_mode; }

// per-call choice (the conv route candidates "big*" of ops/conv.py: conv2d_fwd(big=code) sets it
// for the duration of one call, host thread-local); -1 = follow the global mode
static thread_local int g_big_call = -1;
void conv_big_set_call(int code) { g_big_call = code; }
int conv_big_mode_now() { return g_big_call >= 0 ? g_big_call : g_big_mode; }

// the instantiated configurations (conv_big_fwd's list)
static bool big_instantiated(int bm, int bn, int mf, int stages) {
  const int c = conv_big_encode(bm, bn, mf, stages);
  static const int list[] = {conv_big_encode(128, 256, 16, 2), conv_big_encode(128, 256, 16, 3),
                             conv_big_encode(128, 256, 32, 3), conv_big_encode(128, 128, 16, 4),
                             conv_big_encode(64, 256, 16, 3),  conv_big_encode(64, 256, 32, 3),
                             conv_big_encode(256, 256, 16, 2), conv_big_encode(256, 128, 16, 3),
                             conv_big_encode(256, 256, 32, 2), conv_big_encode(256, 128, 32, 3),
                             conv_big_encode(128, 128, 32, 4)};
  for (int v : list)
    if (v == c) return true;
  return false;
}

// which big-tile configuration (if any) conv_fwd uses for this shape: the global override first
// (TBAMD_CONV_BIG / conv_set_big: 0 off, 1 = the default heuristic, or an encoded choice); every
// configuration needs C % 64 == 0, K % BM == 0 and must be instantiated.
int conv_big_choice(int64_t NPQ, int C, int K, int R, int S, int stride, int pad) {
  (void)R; (void)S; (void)stride; (void)pad;
  int code = conv_big_mode_now();
  if (code == 0 || C % kBK != 0 || NPQ <= 0) return 0;
  if (code == 1) {
    // default heuristic: the widest channel tile the layer has, 256-pixel tiles while that
    // still gives >= 256 workgroups (one per CU), 16x16x32 MFMA, 3 stages
    const int bm = K % 128 == 0 ? 128 : 64;
    const int bn = (NPQ / 256) * (K / bm) >= 256 || bm == 64 ? 256 : 128;
    code = conv_big_encode(bm, bn, 16, bn == 256 ? 3 : 4);
  }
  int bm, bn, mf, stages;
  big_decode(code, bm, bn, mf, stages);
  if (bm == 0 || K % bm != 0 || !big_instantiated(bm, bn, mf, stages)) return 0;
  return code;
}

int conv_big_pixel_tile(int code) { return (code >> 12) & 0xfff; }

void conv_big_fwd(const void* x, const void* w, void* y, const float* bias, float* stats, const void* addend,
                  const uint8_t* amask, bool relu, int N, int H, int W, int C, int K, int R, int S, int P, int Q,
                  int stride, int pad, hipStream_t st, int bnb_mode, const void* bnb_x, const float* bnb_scale,
                  const float* bnb_shift, const float* bnb_mean, const uint8_t* bnb_bits, float* bnb_part,
                  int code) {
  const BigGeom g{N, H, W, C, K, R, S, P, Q, stride, pad};
  const BigEpi e{bias, stats, (const uint16_t*)addend, amask, (const uint16_t*)bnb_x, bnb_scale, bnb_shift,
                 bnb_mean, bnb_bits, bnb_part};
  int bm, bn, mf, stages;
  big_decode(code, bm, bn, mf, stages);
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  // the instantiated set (big_instantiated)
#define TB_GO(BM_, BN_, MF_, S_)                                                      \
  if (bm == BM_ && bn == BN_ && mf == MF_ && stages == S_) {                         \
    launch<BM_, BN_, MF_, S_>(xx, ww, yy, g, e, relu, bnb_mode, st);                 \
    const hipError_t err = hipGetLastError();                                        \
    if (err != hipSuccess)                                                           \
      throw std::runtime_error(std::string("conv_big_fwd launch: ") + hipGetErrorString(err)); \
    return;                                                                          \
  }
  TB_GO(128, 256, 16, 2) TB_GO(128, 256, 16, 3) TB_GO(128, 256, 32, 3) TB_GO(128, 128, 16, 4)
  TB_GO(64, 256, 16, 3) TB_GO(64, 256, 32, 3) TB_GO(256, 256, 16, 2) TB_GO(256, 128, 16, 3)
  TB_GO(256, 256, 32, 2) TB_GO(256, 128, 32, 3) TB_GO(128, 128, 32, 4)
#undef TB_GO
  throw std::runtime_error("conv_big_fwd: tile configuration " + std::to_string(code) + " is not instantiated");
}

}  // namespace tbamd
