// Dense bf16 GEMM engine on gfx950 MFMA (v_mfma_f32_16x16x32_bf16), 512-thread
// workgroups, for Linear layers and 1x1 convolutions:
//
//   Y[p][q] = epi( sum_k X[p][k] * W(q, k) )         p < P (rows: tokens / pixels)
//                                                     q < Q (out features, contiguous in Y)
//   W(q, k) = W[q][k]   (TW = false: nn.Linear weight [out][in] / 1x1 conv weight [K][C])
//   W(q, k) = W[k][q]   (TW = true:  the same weight read transposed — input gradient
//                                    dX = dY . W without materialising W^T)
//
// Reference: every Linear of the examples (GAN/VAE MLPs, LeNet head, ResNet FC,
// ViT) runs through cuBLAS; here it is one kernel
// family with fused epilogues (bias, exact GELU saving the pre-activation,
// residual add).
//
// Orientation: the MFMA computes D[q][p] (W rows as the A operand, X rows as
// the B operand), so each lane's 4 accumulator rows are 4 CONSECUTIVE output
// features of one row p: 8-byte contiguous bf16 stores, per-lane bias quads.
//
// Tiling: BP x BQ output tile per workgroup, BK = 64, 8 waves in a WPxWQ grid.
// Both operands are staged global -> LDS by direct-to-LDS loads (16 B per lane,
// 1 KiB per wave instruction), double buffered: the loads of k-tile t+1 are
// issued before the MFMAs of tile t and retired by the one vmcnt(0) + barrier
// per k-tile (cdna_hip_programming.md §5.5 T3+T4 "minimum 2-phase").
// LDS rows are 128 B.  Row-read tiles ([rows][64 k], read with ds_read_b128)
// XOR the 16-B chunk by (row>>1)&7; transposed tiles ([64 k][64 cols], read
// with ds_read_b64_tr_b16) XOR it by ((row>>1)&1 | (row>>3)&1<<1)<<1, which
// keeps both the b128 row reads and the natural-k-order transposed reads of a
// 32-lane half on 32 distinct bank pairs.  The swizzle is applied to the
// GLOBAL source address (the LDS image is lane-linear; rule 21).  Workgroups
// are remapped so one XCD runs contiguous tile ids (q fastest: the Q tiles of
// one X panel share that XCD's L2).
//
// Tails: P and Q arbitrary (out-of-range rows read a zero page, their outputs
// are not stored), K % 8 == 0 (chunks past K read zeros).
#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
typedef __attribute__((address_space(3))) i16x4_t lds_i16x4_t;

constexpr int kGemmThreads = 512;
constexpr int kBK = 64;

__device__ __attribute__((aligned(64))) uint4 g_gemm_zero[64];  // 1 KiB of zeros

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ int swz_r(int row) { return (row >> 1) & 7; }                          // row-read tiles
__device__ __forceinline__ int swz_t(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }  // transposed

// epilogue codes
enum : int { kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiBiasRes = 3, kEpiRes = 4 };

struct GemmArgs {
  const uint16_t* X;    // [P][K] (row stride ldx)
  const uint16_t* W;    // TW ? [K][Q] : [Q][K]
  uint16_t* Y;          // [P][Q] (row stride ldy)
  const uint16_t* bias; // [Q] bf16
  const uint16_t* res;  // [P][Q] residual (row stride ldy)
  uint16_t* Z;          // [P][Q] pre-activation (GELU epilogue), may be null
  int P, Q, K;
  int64_t ldx, ldy;
};

__device__ __forceinline__ float gelu_exact(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }

template <int BP, int BQ, int WP, bool TW, int EPI>
__global__ __launch_bounds__(kGemmThreads, 1) void gemm_k(GemmArgs a) {
  constexpr int WQ = 8 / WP;
  constexpr int PW = BP / WP, QW = BQ / WQ;  // per-wave tile
  constexpr int TP = PW / 16, TQ = QW / 16;
  static_assert(TP >= 1 && TQ >= 1 && BQ % 64 == 0 && BP % 64 == 0, "tile");
  constexpr int W_U4 = BQ * kBK / 8, X_U4 = BP * kBK / 8;
  constexpr int STAGE = W_U4 + X_U4;          // uint4 per stage
  constexpr int NI = (BP + BQ) / 64;          // glds instructions per wave per stage
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wp = wave / WQ, wq = wave % WQ;
  const int ntp = (a.P + BP - 1) / BP, ntq = (a.Q + BQ - 1) / BQ;
  const int nwg = ntp * ntq;
  int bid = blockIdx.x;
  {
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  const int tq = bid % ntq, tp = bid / ntq;
  const int p0 = tp * BP, q0 = tq * BQ;
  const int KT = (a.K + kBK - 1) / kBK;

  // ---- per-lane staging sources (NI wave-instructions of 8 rows x 128 B)
  // instruction i of wave w covers combined rows 8*(w + 8 j) .. +7 ([W rows | X rows])
  const uint16_t* src[NI];
  int kofs[NI];   // element offset of this lane's chunk along k (row-read) or 0
  int64_t kstr[NI];  // per-k-tile advance (elements)
  bool kchk[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int crow = 8 * (wave + 8 * j) + (lane >> 3);  // combined row
    const int pos = lane & 7;
    if (crow < BQ) {
      if constexpr (!TW) {
        const int row = crow, q = q0 + row;
        const int ch = pos ^ swz_r(row);
        src[j] = q < a.Q ? a.W + (int64_t)q * a.K + ch * 8 : nullptr;
        kofs[j] = ch * 8;
        kstr[j] = kBK;
        kchk[j] = true;
      } else {
        // subtile st = crow / 64 covers columns q0 + 64 st .. +63; row = k within the tile
        const int st = crow >> 6, row = crow & 63;
        const int ch = pos ^ swz_t(row);
        const int q = q0 + 64 * st + ch * 8;
        src[j] = q < a.Q ? a.W + (int64_t)row * a.Q + q : nullptr;  // + k0 * Q per tile
        kofs[j] = row;  // the k of this row
        kstr[j] = (int64_t)kBK * a.Q;
        kchk[j] = true;
      }
    } else {
      const int row = crow - BQ, p = p0 + row;
      const int ch = pos ^ swz_r(row);
      src[j] = p < a.P ? a.X + (int64_t)p * a.ldx + ch * 8 : nullptr;
      kofs[j] = ch * 8;
      kstr[j] = kBK;
      kchk[j] = true;
    }
  }

  auto issue = [&](int kt, int buf) {
    uint4* base = lds + buf * STAGE;
    const int k0 = kt * kBK;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const bool ok = src[j] != nullptr && (k0 + kofs[j] < a.K);
      const void* s = ok ? (const void*)(src[j] + (int64_t)kt * kstr[j]) : (const void*)g_gemm_zero;
      glds16(s, base + (wave + 8 * j) * 64);
    }
  };

  f32x4_t acc[TQ][TP];
#pragma unroll
  for (int i = 0; i < TQ; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  auto compute = [&](int buf) {
    const uint4* Wt = lds + buf * STAGE;
    const uint4* Xt = Wt + W_U4;
#pragma unroll
    for (int ks = 0; ks < kBK / 32; ++ks) {
      bf16x8_t af[TQ], bf[TP];
#pragma unroll
      for (int i = 0; i < TQ; ++i) {
        const int qr = wq * QW + 16 * i;  // first out feature of this 16-block (tile-local)
        if constexpr (!TW) {
          const int row = qr + fr, ch = ks * 4 + fg;
          af[i] = __builtin_bit_cast(bf16x8_t, Wt[row * 8 + (ch ^ swz_r(row))]);
        } else {
          // transposed: lane -> column qr + fr, k = 32 ks + 8 fg + (0..7)
          const int st = qr >> 6, c = (qr & 63) + 4 * (fr & 3);  // lane 4qq+pp supplies (row qq, col 4pp)
          const int r0 = 32 * ks + 8 * fg + (fr >> 2);
          const char* tb = reinterpret_cast<const char*>(Wt + st * 512);
          const int ch = c >> 3, b8 = (c & 4) ? 8 : 0;
          const char* a0 = tb + r0 * 128 + ((ch ^ swz_t(r0)) << 4) + b8;
          const char* a1 = tb + (r0 + 4) * 128 + ((ch ^ swz_t(r0 + 4)) << 4) + b8;
          const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a0);
          const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a1);
          const i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8_t, v);
        }
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int row = wp * PW + 16 * j + fr, ch = ks * 4 + fg;
        bf[j] = __builtin_bit_cast(bf16x8_t, Xt[row * 8 + (ch ^ swz_r(row))]);
      }
#pragma unroll
      for (int i = 0; i < TQ; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  // ---- main loop: prefetch t+1 while multiplying t; one drain + barrier per k-tile
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) issue(kt + 1, cur ^ 1);
    compute(cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds q = q0 + wq*QW + 16 i + 4 fg + (0..3), p = p0 + wp*PW + 16 j + fr
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const int q = q0 + wq * QW + 16 * i + 4 * fg;
    if (q >= a.Q) continue;  // Q % 4 == 0 is required by the host
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == kEpiBias || EPI == kEpiBiasGelu || EPI == kEpiBiasRes) {
      const uint2 b2 = *reinterpret_cast<const uint2*>(a.bias + q);
      bv[0] = bf2f((uint16_t)(b2.x & 0xffff));
      bv[1] = bf2f((uint16_t)(b2.x >> 16));
      bv[2] = bf2f((uint16_t)(b2.y & 0xffff));
      bv[3] = bf2f((uint16_t)(b2.y >> 16));
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int p = p0 + wp * PW + 16 * j + fr;
      if (p >= a.P) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
      const int64_t o = (int64_t)p * a.ldy + q;
      if constexpr (EPI == kEpiBiasRes || EPI == kEpiRes) {
        const uint2 r2 = *reinterpret_cast<const uint2*>(a.res + o);
        v[0] += bf2f((uint16_t)(r2.x & 0xffff));
        v[1] += bf2f((uint16_t)(r2.x >> 16));
        v[2] += bf2f((uint16_t)(r2.y & 0xffff));
        v[3] += bf2f((uint16_t)(r2.y >> 16));
      }
      if constexpr (EPI == kEpiBiasGelu) {
        uint16_t zb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          zb[e] = f2bf(v[e]);
          v[e] = gelu_exact(bf2f(zb[e]));  // GELU of the stored pre-activation (backward recomputes from z)
        }
        if (a.Z)
          *reinterpret_cast<uint2*>(a.Z + o) = make_uint2((uint32_t)zb[0] | ((uint32_t)zb[1] << 16),
                                                          (uint32_t)zb[2] | ((uint32_t)zb[3] << 16));
      }
      *reinterpret_cast<uint2*>(a.Y + o) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                      (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
    }
  }
}

template <int BP, int BQ, int WP, bool TW>
void launch_epi(const GemmArgs& a, int epi, hipStream_t st) {
  const int nwg = ((a.P + BP - 1) / BP) * ((a.Q + BQ - 1) / BQ);
  switch (epi) {
    case kEpiBias: gemm_k<BP, BQ, WP, TW, kEpiBias><<<nwg, kGemmThreads, 0, st>>>(a); break;
    case kEpiBiasGelu: gemm_k<BP, BQ, WP, TW, kEpiBiasGelu><<<nwg, kGemmThreads, 0, st>>>(a); break;
    case kEpiBiasRes: gemm_k<BP, BQ, WP, TW, kEpiBiasRes><<<nwg, kGemmThreads, 0, st>>>(a); break;
    case kEpiRes: gemm_k<BP, BQ, WP, TW, kEpiRes><<<nwg, kGemmThreads, 0, st>>>(a); break;
    default: gemm_k<BP, BQ, WP, TW, kEpiNone><<<nwg, kGemmThreads, 0, st>>>(a);
  }
}

// tile configurations (index = host-visible "tile" id)
//   0: 256 x 256 (waves 2P x 4Q, 128 x 64 per wave)
//   1: 256 x 128 (4 x 2, 64 x 64)
//   2: 128 x 256 (2 x 4, 64 x 64)
//   3: 128 x 128 (4 x 2, 32 x 64)
//   4: 256 x  64 (4 x 2, 64 x 32)
//   5: 128 x  64 (8 x 1, 16 x 64)
template <bool TW>
void launch_tile(const GemmArgs& a, int tile, int epi, hipStream_t st) {
  switch (tile) {
    case 0: launch_epi<256, 256, 2, TW>(a, epi, st); break;
    case 1: launch_epi<256, 128, 4, TW>(a, epi, st); break;
    case 2: launch_epi<128, 256, 2, TW>(a, epi, st); break;
    case 3: launch_epi<128, 128, 4, TW>(a, epi, st); break;
    case 4: launch_epi<256, 64, 4, TW>(a, epi, st); break;
    default: launch_epi<128, 64, 8, TW>(a, epi, st);
  }
}

constexpr int kTileP[6] = {256, 256, 128, 128, 256, 128};
constexpr int kTileQ[6] = {256, 128, 256, 128, 64, 64};

}  // namespace

int gemm_num_tiles() { return 6; }

// heuristic tile: the fewest partial waves of workgroups over the 256 CUs,
// larger tiles preferred on ties (more MFMA per staged byte)
int gemm_pick_tile(int P, int Q, int K) {
  int best = 3;
  double best_cost = 1e30;
  for (int t = 0; t < 6; ++t) {
    if (kTileQ[t] > 64 && Q <= kTileQ[t] / 2) continue;  // mostly empty Q tiles
    const int64_t nwg = (int64_t)((P + kTileP[t] - 1) / kTileP[t]) * ((Q + kTileQ[t] - 1) / kTileQ[t]);
    const double waves = (double)((nwg + 255) / 256);
    // time ~ waves x per-tile work; per-tile work ~ BP*BQ / efficiency(tile)
    const double eff = (kTileP[t] * kTileQ[t] >= 256 * 128) ? 1.0 : (kTileP[t] * kTileQ[t] >= 128 * 128 ? 0.85 : 0.7);
    const double cost = waves * kTileP[t] * kTileQ[t] / eff;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = t;
    }
  }
  (void)K;
  return best;
}

// Y = epi(X W^T) (tw = 0) or epi(X W) (tw = 1); see the file header
void gemm_bf16(const void* X, int64_t ldx, const void* W, bool tw, void* Y, int64_t ldy, const void* bias,
               const void* res, void* Z, int P, int Q, int K, int epi, int tile, hipStream_t st) {
  if (P <= 0 || Q <= 0) return;
  GemmArgs a{(const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, (const uint16_t*)bias, (const uint16_t*)res,
             (uint16_t*)Z, P, Q, K, ldx, ldy};
  if (tile < 0 || tile >= 6) tile = gemm_pick_tile(P, Q, K);
  if (tw) launch_tile<true>(a, tile, epi, st);
  else launch_tile<false>(a, tile, epi, st);
}

}  // namespace tbamd
