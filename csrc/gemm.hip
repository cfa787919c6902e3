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
enum : int { kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiBiasRes = 3, kEpiRes = 4, kEpiF32 = 5,
             kEpiBiasRelu = 6, kEpiRelu = 7 };

struct GemmArgs {
  const uint16_t* X;    // [P][K] (row stride ldx)
  const uint16_t* W;    // TW ? [K][Q] : [Q][K]
  uint16_t* Y;          // [P][Q] (row stride ldy)
  const uint16_t* bias; // [Q] bf16
  const uint16_t* res;  // [P][Q] residual (row stride ldy)
  uint16_t* Z;          // [P][Q] pre-activation (GELU epilogue), may be null
  float* part;          // split-K f32 partials [S][P][Q] (kEpiF32)
  int P, Q, K;
  int64_t ldx, ldy;
};

__device__ __forceinline__ float gelu_exact(float z) { return gelu_f(z); }

template <int BP, int BQ, int WP, bool TX, bool TW, int EPI, int NS = 2>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_k(GemmArgs a) {
  constexpr int WQ = 8 / WP;
  constexpr int PW = BP / WP, QW = BQ / WQ;  // per-wave tile
  constexpr int TP = PW / 16, TQ = QW / 16;
  static_assert(TP >= 1 && TQ >= 1 && BQ % 64 == 0 && BP % 64 == 0, "tile");
  constexpr int W_U4 = BQ * kBK / 8, X_U4 = BP * kBK / 8;
  constexpr int STAGE = W_U4 + X_U4;          // uint4 per stage
  constexpr int NI = (BP + BQ) / 64;          // glds instructions per wave per stage
  __shared__ __attribute__((aligned(16))) uint4 lds[(NS == 12 ? 2 : NS) * STAGE];

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
  // split-K (EPI == kEpiF32): blockIdx.y owns k-tiles [kt0, kt1)
  const int kts = (KT + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * kts;
  const int kt1 = min(KT, kt0 + kts);

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
    } else if constexpr (!TX) {
      const int row = crow - BQ, p = p0 + row;
      const int ch = pos ^ swz_r(row);
      src[j] = p < a.P ? a.X + (int64_t)p * a.ldx + ch * 8 : nullptr;
      kofs[j] = ch * 8;
      kstr[j] = kBK;
      kchk[j] = true;
    } else {
      // X stored [K][P] (ldx = row stride): subtiles of 64 columns, rows = k
      const int xrow = crow - BQ, st = xrow >> 6, row = xrow & 63;
      const int ch = pos ^ swz_t(row);
      const int p = p0 + 64 * st + ch * 8;
      src[j] = p < a.P ? a.X + (int64_t)row * a.ldx + p : nullptr;
      kofs[j] = row;
      kstr[j] = (int64_t)kBK * a.ldx;
      kchk[j] = true;
    }
  }

  const void* zpage = pin_sgpr(g_gemm_zero);
  auto issue = [&](int kt, int buf) {
    uint4* base = lds + buf * STAGE;
    const int k0 = kt * kBK;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      bool ok = src[j] != nullptr && (k0 + kofs[j] < a.K);
      // extent of the operand this instruction reads: X [P][ldx] or [K][ldx], W [Q][K] or [K][Q]
      ok = ok && TB_BOUNDS_OK(src[j] + (int64_t)kt * kstr[j] + 8 <=
                                  (j * 8 * 8 + wave * 8 < BQ ? a.W + (int64_t)a.Q * a.K
                                                             : a.X + (TX ? (int64_t)a.K : (int64_t)a.P) * a.ldx),
                              kBndGemmSrc);
      const void* s = ok ? (const void*)(src[j] + (int64_t)kt * kstr[j]) : zpage;
      glds16(s, base + (wave + 8 * j) * 64);
    }
  };

  f32x4_t acc[TQ][TP];
#pragma unroll
  for (int i = 0; i < TQ; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // transposed operand fragment: tile = [64 k][64 cols] subtiles (128-B rows, swz_t);
  // lane -> column cl (tile-local, 16-aligned block + fr), k = 32 ks + 8 fg + (0..7)
  auto tr_read = [&](const uint4* tile, int cblk, int ks) -> bf16x8_t {
    const int st = cblk >> 6, c = (cblk & 63) + 4 * (fr & 3);  // lane 4qq+pp supplies (row qq, col 4pp)
    const int r0 = 32 * ks + 8 * fg + (fr >> 2);
    const char* tb = reinterpret_cast<const char*>(tile + st * 512);
    const int ch = c >> 3, b8 = (c & 4) ? 8 : 0;
    const char* a0 = tb + r0 * 128 + ((ch ^ swz_t(r0)) << 4) + b8;
    const char* a1 = tb + (r0 + 4) * 128 + ((ch ^ swz_t(r0 + 4)) << 4) + b8;
    const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a0);
    const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a1);
    const i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  };
  // fragments of one 32-deep half (ks) of the k-tile in LDS buffer buf
  auto frags = [&](int buf, int ks, bf16x8_t (&af)[TQ], bf16x8_t (&bf)[TP]) {
    const uint4* Wt = lds + buf * STAGE;
    const uint4* Xt = Wt + W_U4;
#pragma unroll
    for (int i = 0; i < TQ; ++i) {
      const int qr = wq * QW + 16 * i;
      if constexpr (!TW) {
        const int row = qr + fr, ch = ks * 4 + fg;
        af[i] = __builtin_bit_cast(bf16x8_t, Wt[row * 8 + (ch ^ swz_r(row))]);
      } else {
        af[i] = tr_read(Wt, qr, ks);
      }
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      if constexpr (!TX) {
        const int row = wp * PW + 16 * j + fr, ch = ks * 4 + fg;
        bf[j] = __builtin_bit_cast(bf16x8_t, Xt[row * 8 + (ch ^ swz_r(row))]);
      } else {
        bf[j] = tr_read(Xt, wp * PW + 16 * j, ks);
      }
    }
  };
  auto mma = [&](const bf16x8_t (&af)[TQ], const bf16x8_t (&bf)[TP]) {
#pragma unroll
    for (int i = 0; i < TQ; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
  };
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
          af[i] = tr_read(Wt, qr, ks);
        }
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        if constexpr (!TX) {
          const int row = wp * PW + 16 * j + fr, ch = ks * 4 + fg;
          bf[j] = __builtin_bit_cast(bf16x8_t, Xt[row * 8 + (ch ^ swz_r(row))]);
        } else {
          bf[j] = tr_read(Xt, wp * PW + 16 * j, ks);
        }
      }
#pragma unroll
      for (int i = 0; i < TQ; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  // ---- main loop: prefetch t+1 while multiplying t; one drain + barrier per k-tile
  if constexpr (NS == 12) {
    // split-half schedule: the barrier sits BETWEEN the two 32-deep halves, and
    // each half's LDS fragment reads are issued while the previous half's MFMAs
    // run, so no wave starts a k-tile with exposed ds_read latency
    //   iter kt: issue glds(kt+1) | read F1(kt) | MFMA F0(kt) | vmcnt(0) lgkm(0) barrier
    //            | read F0(kt+1) | MFMA F1(kt)
    bf16x8_t a0[TQ], b0[TP], a1[TQ], b1[TP];
    if (kt0 < kt1) issue(kt0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt0 < kt1) frags(0, 0, a0, b0);
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) issue(kt + 1, cur ^ 1);
      frags(cur, 1, a1, b1);
      mma(a0, b0);
      // every wave's reads of buffer cur are complete and tile kt+1 has landed
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (more) frags(cur ^ 1, 0, a0, b0);
      mma(a1, b1);
    }
    __syncthreads();
  } else if constexpr (NS == 2) {
    if (kt0 < kt1) issue(kt0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      if (kt + 1 < kt1) issue(kt + 1, cur ^ 1);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // NS-deep ring: NS-1 k-tiles in flight; a COUNTED vmcnt retires the oldest and one raw
    // s_barrier per k-tile publishes it (a __syncthreads() would drain every LDS-DMA:
    // cdna_hip_programming.md §5 "Pipelining across barriers")
#pragma unroll
    for (int t = 0; t < NS - 1; ++t)
      if (kt0 + t < kt1) issue(kt0 + t, t);
    int cur = 0, nxt = NS - 1;
    for (int kt = kt0; kt < kt1; ++kt) {
      if (kt + NS - 2 < kt1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // tile kt landed for every wave; buffer nxt is free
      asm volatile("" ::: "memory");
      if (kt + NS - 1 < kt1) issue(kt + NS - 1, nxt);
      __builtin_amdgcn_s_setprio(1);
      compute(cur);
      __builtin_amdgcn_s_setprio(0);
      cur = cur + 1 == NS ? 0 : cur + 1;
      nxt = nxt + 1 == NS ? 0 : nxt + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (EPI == kEpiF32) {
    // split-K partial: f32 slab blockIdx.y of [S][P][Q]
    float* part = a.part + (int64_t)blockIdx.y * a.P * a.Q;
#pragma unroll
    for (int i = 0; i < TQ; ++i) {
      const int q = q0 + wq * QW + 16 * i + 4 * fg;
      if (q >= a.Q) continue;
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int p = p0 + wp * PW + 16 * j + fr;
        if (p >= a.P) continue;
        *reinterpret_cast<float4*>(part + (int64_t)p * a.Q + q) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }

  // ---- epilogue: lane holds q = q0 + wq*QW + 16 i + 4 fg + (0..3), p = p0 + wp*PW + 16 j + fr
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const int q = q0 + wq * QW + 16 * i + 4 * fg;
    if (q >= a.Q) continue;  // Q % 4 == 0 is required by the host
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == kEpiBias || EPI == kEpiBiasGelu || EPI == kEpiBiasRes ||
                    EPI == kEpiBiasRelu) {
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
      if constexpr (EPI == kEpiBiasRelu || EPI == kEpiRelu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          *reinterpret_cast<uint2*>(a.Y + o) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                      (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
    }
  }
}

template <int BP, int BQ, int WP, bool TX, bool TW, int NS>
void launch_epi(const GemmArgs& a, int epi, int splits, hipStream_t st) {
  const int nwg = ((a.P + BP - 1) / BP) * ((a.Q + BQ - 1) / BQ);
  const dim3 grid(nwg, epi == kEpiF32 ? splits : 1);
  switch (epi) {
    case kEpiBias: gemm_k<BP, BQ, WP, TX, TW, kEpiBias, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    case kEpiBiasGelu: gemm_k<BP, BQ, WP, TX, TW, kEpiBiasGelu, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    case kEpiBiasRes: gemm_k<BP, BQ, WP, TX, TW, kEpiBiasRes, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    case kEpiRes: gemm_k<BP, BQ, WP, TX, TW, kEpiRes, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    case kEpiF32: gemm_k<BP, BQ, WP, TX, TW, kEpiF32, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    case kEpiBiasRelu: gemm_k<BP, BQ, WP, TX, TW, kEpiBiasRelu, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    case kEpiRelu: gemm_k<BP, BQ, WP, TX, TW, kEpiRelu, NS><<<grid, kGemmThreads, 0, st>>>(a); break;
    default: gemm_k<BP, BQ, WP, TX, TW, kEpiNone, NS><<<grid, kGemmThreads, 0, st>>>(a);
  }
}

// tile configurations (index = host-visible "tile" id)
//   0: 256 x 256 (waves 2P x 4Q, 128 x 64 per wave), 2 LDS stages (128 KiB)
//   1: 256 x 128 (4 x 2, 64 x 64), 2 stages      6: same, 3-stage ring (144 KiB)
//   2: 128 x 256 (2 x 4, 64 x 64), 2 stages      7: same, 3-stage ring
//   3: 128 x 128 (4 x 2, 32 x 64), 2 stages      8: same, 3-stage ring (96 KiB)
//   4: 256 x  64 (4 x 2, 64 x 32), 2 stages      9: same, 3-stage ring
//   5: 128 x  64 (8 x 1, 16 x 64), 2 stages
//   10-15: tiles 0-5 with the split-half schedule (barrier between the k-halves)
template <bool TX, bool TW>
void launch_tile(const GemmArgs& a, int tile, int epi, int splits, hipStream_t st) {
  switch (tile) {
    case 0: launch_epi<256, 256, 2, TX, TW, 2>(a, epi, splits, st); break;
    case 1: launch_epi<256, 128, 4, TX, TW, 2>(a, epi, splits, st); break;
    case 2: launch_epi<128, 256, 2, TX, TW, 2>(a, epi, splits, st); break;
    case 3: launch_epi<128, 128, 4, TX, TW, 2>(a, epi, splits, st); break;
    case 4: launch_epi<256, 64, 4, TX, TW, 2>(a, epi, splits, st); break;
    case 6: launch_epi<256, 128, 4, TX, TW, 3>(a, epi, splits, st); break;
    case 7: launch_epi<128, 256, 2, TX, TW, 3>(a, epi, splits, st); break;
    case 8: launch_epi<128, 128, 4, TX, TW, 3>(a, epi, splits, st); break;
    case 9: launch_epi<256, 64, 4, TX, TW, 3>(a, epi, splits, st); break;
    case 10: launch_epi<256, 256, 2, TX, TW, 12>(a, epi, splits, st); break;
    case 11: launch_epi<256, 128, 4, TX, TW, 12>(a, epi, splits, st); break;
    case 12: launch_epi<128, 256, 2, TX, TW, 12>(a, epi, splits, st); break;
    case 13: launch_epi<128, 128, 4, TX, TW, 12>(a, epi, splits, st); break;
    case 14: launch_epi<256, 64, 4, TX, TW, 12>(a, epi, splits, st); break;
    case 15: launch_epi<128, 64, 8, TX, TW, 12>(a, epi, splits, st); break;
    default: launch_epi<128, 64, 8, TX, TW, 2>(a, epi, splits, st);
  }
}

// split-K combine: out[p][q] (bf16, row stride ldo) = sum_s part[s][p][q]; 8 outputs per thread
__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ part, int S, int P, int Q,
                                                       uint16_t* __restrict__ out, int64_t ldo) {
  const int64_t n8 = (int64_t)P * Q / 8;
  const int64_t PQ = (int64_t)P * Q;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      const float4 a0 = *reinterpret_cast<const float4*>(part + s * PQ + 8 * i);
      const float4 a1 = *reinterpret_cast<const float4*>(part + s * PQ + 8 * i + 4);
      v[0] += a0.x; v[1] += a0.y; v[2] += a0.z; v[3] += a0.w;
      v[4] += a1.x; v[5] += a1.y; v[6] += a1.z; v[7] += a1.w;
    }
    const int64_t e = 8 * i;
    const int p = (int)(e / Q), q = (int)(e % Q);
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(out + (int64_t)p * ldo + q) = o;
  }
}

constexpr int kNumTiles = 16;
constexpr int kTileP[kNumTiles] = {256, 256, 128, 128, 256, 128, 256, 128, 128, 256, 256, 256, 128, 128, 256, 128};
constexpr int kTileQ[kNumTiles] = {256, 128, 256, 128, 64, 64, 128, 256, 128, 64, 256, 128, 256, 128, 64, 64};

}  // namespace

// tile id kTile8 = the 8-phase 256x256 kernel of csrc/gemm8.hip (NT products with K % 64 == 0;
// other orientations / split-K fall back to tile 10, the same tile with the split-half schedule)
constexpr int kTile8 = kNumTiles;
// tile ids kTile8 + 1 / + 2: the 8-phase kernel over the rows that fill whole rounds of the 256 CUs,
// the remaining rows on the 128 x 128 tile (2-stage / 3-stage ring) -- a 256 x 256 grid one tile
// row past a whole round (ViT's N = 768 products: 297 tiles) would otherwise run a second round at
// 16 % occupancy
constexpr int kTile8Tail = kNumTiles + 1;
int gemm_num_tiles() { return kNumTiles + 3; }

// rows of the whole-round part of a tile-8 grid (0: no such split helps)
static int gemm8_bulk_rows(int P, int Q) {
  const int ntq = (Q + 255) / 256, ntp = (P + 255) / 256;
  const int total = ntp * ntq, full = (total / 256) * 256;
  if (full == 0 || full == total) return 0;
  const int pb = (full / ntq) * 256;
  return pb >= P ? 0 : pb;
}
static int tile_p(int t) { return kTileP[t]; }
static int tile_q(int t) { return kTileQ[t]; }

// heuristic tile: the fewest partial waves of workgroups over the 256 CUs,
// larger tiles preferred on ties (more MFMA per staged byte)
int gemm_pick_tile(int P, int Q, int K) {
  int best = 3;
  double best_cost = 1e30;
  for (int t = 0; t < 6; ++t) {  // (the 3-stage variants are picked by the autotuner only)
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

// Y = epi(X W^T) (tw = 0) or epi(X W) (tw = 1); tx = 1: X stored [K][P] (Y = X^T ...).
// splits > 1 (epilogue none only): f32 partials in `part` ([splits][P][Q]) + a combine pass.
void gemm_bf16(const void* X, int64_t ldx, bool tx, const void* W, bool tw, void* Y, int64_t ldy, const void* bias,
               const void* res, void* Z, int P, int Q, int K, int epi, int tile, int splits, float* part,
               hipStream_t st) {
  if (P <= 0 || Q <= 0) return;
  GemmArgs a{(const uint16_t*)X, (const uint16_t*)W, (uint16_t*)Y, (const uint16_t*)bias, (const uint16_t*)res,
             (uint16_t*)Z, part, P, Q, K, ldx, ldy};
  if (tile < 0 || tile >= gemm_num_tiles()) tile = gemm_pick_tile(P, Q, K);
  if (tile >= kTile8Tail) {
    const int pb = gemm8_bulk_rows(P, Q);
    const bool nt = !tw && epi != kEpiF32 && gemm8_supported(P, Q, K, ldx);
    const bool nn = tw && epi == kEpiNone && gemm8_nn_supported(P, Q, K, ldx);
    if (pb > 0 && !tx && (nt || nn)) {
      const int tt = tile == kTile8Tail ? 3 : 8;
      gemm_bf16(X, ldx, false, W, tw, Y, ldy, bias, res, Z, pb, Q, K, epi, kTile8, 1, nullptr, st);
      const int64_t ro = (int64_t)pb * ldy;
      gemm_bf16((const uint16_t*)X + (int64_t)pb * ldx, ldx, false, W, tw, (uint16_t*)Y + ro, ldy, bias,
                res ? (const uint16_t*)res + ro : nullptr, Z ? (uint16_t*)Z + ro : nullptr, P - pb, Q, K, epi, tt, 1,
                nullptr, st);
      return;
    }
    tile = kTile8;  // (no whole-round split for this shape / orientation: the plain 8-phase grid)
  }
  if (tile == kTile8) {
    // NT / NN: the 8-phase kernel (whole k per tile)
    if (!tx && !tw && epi != kEpiF32 && gemm8_supported(P, Q, K, ldx)) {
      gemm8_bf16(X, ldx, W, Y, ldy, bias, res, Z, P, Q, K, epi, st);
      return;
    }
    if (!tx && tw && epi == kEpiNone && gemm8_nn_supported(P, Q, K, ldx)) {
      gemm8_nn_bf16(X, ldx, W, Y, ldy, nullptr, nullptr, P, Q, K, st);
      return;
    }
    if (tx && tw && epi == kEpiNone && ldy == Q && gemm8_tn_supported(P, Q, K, ldx)) {
      // weight gradient: the 8-phase schedule on transposing LDS reads, split-K partials
      const int s = gemm8_tn_splits(K / kBK, splits);
      gemm8_tn_bf16(X, ldx, W, Y, ldy, P, Q, K, s, part, st);
      if (s > 1) {
        const int64_t n8 = (int64_t)P * Q / 8;
        int64_t gs = (n8 + 255) / 256;
        if (gs > 2048) gs = 2048;
        splitk_reduce_k<<<(int)gs, 256, 0, st>>>(part, s, P, Q, (uint16_t*)Y, ldy);
      }
      return;
    }
    tile = 10;
  }
  const int e = splits > 1 ? (int)kEpiF32 : epi;
  if (tx) {
    if (tw) launch_tile<true, true>(a, tile, e, splits, st);
    else launch_tile<true, false>(a, tile, e, splits, st);
  } else {
    if (tw) launch_tile<false, true>(a, tile, e, splits, st);
    else launch_tile<false, false>(a, tile, e, splits, st);
  }
  if (splits > 1) {
    const int64_t n8 = (int64_t)P * Q / 8;
    int64_t gs = (n8 + 255) / 256;
    if (gs > 2048) gs = 2048;
    splitk_reduce_k<<<(int)gs, 256, 0, st>>>(part, splits, P, Q, (uint16_t*)Y, ldy);
  }
}

// split count for a split-K GEMM: enough workgroups to cover the CUs twice, each
// split >= 8 k-tiles
int gemm_pick_splits(int P, int Q, int K, int tile) {
  if (tile < 0 || tile >= gemm_num_tiles()) tile = gemm_pick_tile(P, Q, K);
  if (tile >= kTile8) tile = 10;
  const int64_t nwg = (int64_t)((P + tile_p(tile) - 1) / tile_p(tile)) * ((Q + tile_q(tile) - 1) / tile_q(tile));
  const int KT = (K + kBK - 1) / kBK;
  int s = (int)((512 + nwg - 1) / nwg);
  if (s > KT / 8) s = KT / 8;
  return s < 1 ? 1 : s;
}

}  // namespace tbamd
