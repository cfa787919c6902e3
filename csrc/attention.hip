// Fused multi-head attention (flash style) on gfx950 MFMA, head dim 64, bf16.
//
// Not in the reference (it has no attention model); this is
// K26 of SURVEY.md §2.3.1 for the ViT-B/16 north-star config: softmax(QKᵀ·s)·V
// forward and its backward without materialising the N x N scores.
//
// All products are v_mfma_f32_16x16x32_bf16 with the "swapped" orientation
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"):
//
//   forward   Sᵀ[key][q] = K·Qᵀ         -> each lane owns ONE query column, so the
//             online-softmax row statistics are per-lane scalars, and the
//             accumulator is already the B operand of
//             Oᵀ[d][q] += Vᵀ·Pᵀ          (Vᵀ fragments via ds_read_b64_tr_b16)
//   dQ pass   Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ, dSᵀ = Pᵀ∘(dPᵀ-δ), dQᵀ += Kᵀ·dSᵀ
//   dK/dV     S = Q·Kᵀ, dP = dO·Vᵀ (key on the lane), dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS
//
// dQ and dK/dV are two kernels (the dQ pass recomputes S and dP) so no float
// atomics are needed and every gradient is written exactly once, deterministic.
// K/V (or Q/dO) tiles of 64 rows x 128 B are staged global->LDS with direct
// LDS loads (global_load_lds, 16 B per lane), double buffered; the 16-B chunk
// of row r sits at chunk ^ (((r>>1)&3)<<1), which keeps both the ds_read_b128
// row reads of the 16x16x32 operand and the transposed ds_read_b64_tr_b16
// reads conflict-free (scripts/lds_banks.py checks the bank map).  Rows past N
// come from a zero page (keys are masked to -inf, queries are not stored).
// Workgroups are remapped so that the blocks of one (batch, head) run on the
// same XCD and share its L2 for K/V (or Q/dO).
#include <type_traits>

#include "common.h"
#include "mfma_tile.h"
#include "tbamd.h"

namespace tbamd {
namespace {

constexpr int kBlk = 128;           // queries (fwd, dQ) or keys (dK/dV) per workgroup: 4 waves x 32
constexpr float kLog2e = 1.4426950408889634f;

// XCD-aware block order: consecutive logical ids (the blocks of one (b, h)) on one XCD
__device__ __forceinline__ void block_coords(int nblk, int H, int& x, int& h, int& b) {
  const int nwg = gridDim.x;
  const int id = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = id % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + id / 8;
  x = lid % nblk;
  const int bh = lid / nblk;
  h = bh % H;
  b = bh / H;
}

__device__ __forceinline__ const uint16_t* head(const uint16_t* p, const int64_t* s, int b, int h) {
  return p + b * s[0] + h * s[1];
}

// ------------------------------------------------------------------ forward
// normalised Oᵀ -> O rows and the log-sum-exp of each query (the backward's softmax statistics)
__device__ __forceinline__ void fwd_store(const AttnArgs& a, int b, int h, int q0, const f32x4_t (&acc)[4][2],
                                          const float (&m)[2], const float (&l)[2], int fr, int fg) {
  const int N = a.N;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float lt = l[qt];
    lt += __shfl_xor(lt, 16);
    lt += __shfl_xor(lt, 32);
    const int qi = q0 + 16 * qt + fr;
    if (qi < N) {
      const float inv = 1.f / lt;
      uint16_t* op = a.o + b * a.so[0] + h * a.so[1] + qi * a.so[2] + 4 * fg;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) st4(op + 16 * dt, acc[dt][qt], inv);
      if (fg == 0) a.lse[((int64_t)b * a.H + h) * N + qi] = (m[qt] + log2f(lt)) * 0.6931471805599453f;
    }
  }
}

// One 64-key tile of the forward for a wave's 32 queries: Sᵀ = K·Qᵀ, online softmax (running max m,
// lane-partial row sum l), Oᵀ += Vᵀ·Pᵀ.  Kt / Vt: the swizzled LDS tiles of keys t*64 .. +63.
// EDGE: the tile holds keys past N (the last tile when N % 64 != 0): only there are the key mask
// and the sub-tile skips compiled in.  exp2: the bare v_exp_f32 (__builtin_amdgcn_exp2f; exp2f adds a
// range reduction for denormal results -- an ldexp, two selects and an add per score).
template <bool EDGE>
__device__ __forceinline__ void fwd_tile(const uint4* Kt, const uint4* Vt, int t, int N, int nqt, float c,
                                         const bf16x8_t (&qf)[2][2], f32x4_t (&acc)[4][2], float (&m)[2],
                                         float (&l)[2], int fr, int fg) {
  // valid keys in this tile: 16-key sub-tiles (and 32-key PV steps) past N are skipped
  // (N = 197 -> the last tile holds 5 keys: 13 sub-tiles of 16 computed instead of 16)
  const int nvk = EDGE ? N - t * kTile : kTile;
  f32x4_t s[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) s[mt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      if (16 * mt >= nvk) continue;
      const bf16x8_t kf = row_frag(Kt, 16 * mt + fr, 4 * ks + fg);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        if (qt < nqt) s[mt][qt] = mfma(kf, qf[qt][ks], s[mt][qt]);
    }
  const int key0 = t * kTile + 4 * fg;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    if (qt >= nqt) continue;
    // the max runs on the raw scores (c > 0: max(s * c) = c * max(s)) and the scale folds into the
    // exponent's fma: one VALU op per score fewer than scaling every score first
    float mx = -INFINITY;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (EDGE) {
          if (key0 + 16 * mt + i >= N) s[mt][qt][i] = -INFINITY;
        }
        mx = fmaxf(mx, s[mt][qt][i]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m[qt], mx * c);
    const float alpha = __builtin_amdgcn_exp2f(m[qt] - mn);
    m[qt] = mn;
    float ls = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[mt][qt][i], c, -mn));
        s[mt][qt][i] = p;
        ls += p;
      }
    l[qt] = l[qt] * alpha + ls;  // lane-partial; summed over the 4 lane groups at the end
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt][qt] *= alpha;
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (32 * ks >= nvk) continue;
    bf16x8_t pf[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) pf[qt] = pack_frag(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8_t vf = tr_frag(Vt, 32 * ks, dt, fr, fg);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        if (qt < nqt) acc[dt][qt] = mfma(vf, pf[qt], acc[dt][qt]);
    }
  }
}

__global__ __launch_bounds__(256, 2) void attn_fwd_k(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * 2 * kTileU4];  // [buf][K | V] = 32 KiB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int N = a.N;
  int xb, h, b;
  block_coords((N + kBlk - 1) / kBlk, a.H, xb, h, b);
  const uint16_t* qp = head(a.q, a.sq, b, h);
  const uint16_t* kp = head(a.k, a.sk, b, h);
  const uint16_t* vp = head(a.v, a.sv, b, h);
  const int q0 = xb * kBlk + wave * 32;
  const bool wave_live = q0 < N;
  // the last wave of a head may hold <= 16 queries (N = 197: queries 192..196): its second
  // 16-query sub-tile is skipped (wave-uniform) in every product and in the softmax
  const int nqt = q0 + 16 < N ? 2 : 1;
  const float c = a.scale * kLog2e;

  // Qᵀ as the B operand: lane holds Q[q0 + 16qt + fr][32ks + 8fg .. +7]
  bf16x8_t qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0 + 16 * qt + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = qi < N ? ld_frag(qp + qi * a.sq[2] + 32 * ks + 8 * fg) : bf16x8_t{};
  }
  f32x4_t acc[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) acc[dt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

  const int nt = (N + kTile - 1) / kTile;
  stage_tile(lds, kp, a.sk[2], 0, N, wave, lane);
  stage_tile(lds + kTileU4, vp, a.sv[2], 0, N, wave, lane);
  auto next = [&](int t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile t landed; every wave is done with the other buffer
    if (t + 1 < nt) {
      uint4* Kn = lds + ((t + 1) & 1) * 2 * kTileU4;
      stage_tile(Kn, kp, a.sk[2], (t + 1) * kTile, N, wave, lane);
      stage_tile(Kn + kTileU4, vp, a.sv[2], (t + 1) * kTile, N, wave, lane);
    }
  };
  // full tiles unmasked, the edge tile peeled, the query sub-tile count a constant (as the head
  // kernel); a wave with no query only helps stage tiles
  const int nfull = N / kTile;
  auto run = [&](auto nq) {
    constexpr int NQ = decltype(nq)::value;
    for (int t = 0; t < nfull; ++t) {
      next(t);
      const uint4* Kt = lds + (t & 1) * 2 * kTileU4;
      if (wave_live) fwd_tile<false>(Kt, Kt + kTileU4, t, N, NQ, c, qf, acc, m, l, fr, fg);
    }
    if (nfull < nt) {
      next(nfull);
      const uint4* Kt = lds + (nfull & 1) * 2 * kTileU4;
      if (wave_live) fwd_tile<true>(Kt, Kt + kTileU4, nfull, N, NQ, c, qf, acc, m, l, fr, fg);
    }
  };
  if (nqt == 2) run(std::integral_constant<int, 2>{});
  else run(std::integral_constant<int, 1>{});
  fwd_store(a, b, h, q0, acc, m, l, fr, fg);
}

// Whole-head forward (N <= 256, the ViT-B/16 197 tokens): ONE workgroup of 8 waves per (batch, head)
// stages the head's K and V whole (waves 0-3 the K tiles, 4-7 the V tiles: 64 KiB) with one wait and
// one barrier, then every wave runs its 32 queries over all keys from LDS with no further barrier.
// The two 128-query workgroups of attn_fwd_k each staged K / V and paid a vmcnt(0) + barrier per
// 64-key tile (64.5 us per ViT-B layer at 11 % MFMA busy, profiles/r05_vit/pmc_table_before_tnfill.txt).
constexpr int kHeadWaves = 8, kHeadTiles = 4;
__global__ __launch_bounds__(512, 2) void attn_fwd_head_k(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * kHeadTiles * kTileU4];  // [K tiles | V tiles]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int N = a.N;
  const int h = (int)(blockIdx.x % a.H), b = (int)(blockIdx.x / a.H);
  const uint16_t* qp = head(a.q, a.sq, b, h);
  const uint16_t* kp = head(a.k, a.sk, b, h);
  const uint16_t* vp = head(a.v, a.sv, b, h);
  const int nt = (N + kTile - 1) / kTile;  // <= kHeadTiles (host check)
  {
    const bool kv = wave >= 4;
    uint4* base = lds + (kv ? kHeadTiles * kTileU4 : 0);
    const uint16_t* src = kv ? vp : kp;
    const int64_t rs = kv ? a.sv[2] : a.sk[2];
    for (int t = 0; t < nt; ++t) stage_tile(base + t * kTileU4, src, rs, t * kTile, N, wave & 3, lane);
  }
  const int q0 = wave * 32;
  const bool wave_live = q0 < N;
  const int nqt = q0 + 16 < N ? 2 : 1;
  const float c = a.scale * kLog2e;
  bf16x8_t qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0 + 16 * qt + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = qi < N ? ld_frag(qp + qi * a.sq[2] + 32 * ks + 8 * fg) : bf16x8_t{};
  }
  f32x4_t acc[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) acc[dt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every K / V tile of the head landed (the only barrier)
  if (!wave_live) return;
  // full tiles unmasked, then the edge tile (peeled: a branch between two bodies inside the loop
  // cost 168 VGPRs, one workgroup per CU)
  // (the query sub-tile count stays a runtime value here: as a constant, two loop copies took 130
  // VGPRs -- 128 forced -- and measured 92 vs 89 us per call, r5_43)
  const int nfull = N / kTile;
  for (int t = 0; t < nfull; ++t)
    fwd_tile<false>(lds + t * kTileU4, lds + (kHeadTiles + t) * kTileU4, t, N, nqt, c, qf, acc, m, l, fr, fg);
  if (nfull < nt)
    fwd_tile<true>(lds + nfull * kTileU4, lds + (kHeadTiles + nfull) * kTileU4, nfull, N, nqt, c, qf, acc, m, l, fr,
                   fg);
  fwd_store(a, b, h, q0, acc, m, l, fr, fg);
}

// ------------------------------------------------- backward: dQ (+ delta)
// A wave's 32 queries: Q / dO fragments (B operands), delta = rowsum(dO * O) (written for the dK/dV
// pass) and the log2-domain log-sum-exp
struct DqRows {
  bf16x8_t qf[2][2], df[2][2];
  float lse2[2], delta[2];
};

__device__ __forceinline__ void dq_rows(const AttnArgs& a, int b, int h, int q0, int fr, int fg, DqRows& r) {
  const int N = a.N;
  const uint16_t* qp = head(a.q, a.sq, b, h);
  const uint16_t* op = head(a.o, a.so, b, h);
  const uint16_t* dop = head(a.dout, a.sdo, b, h);
  const int64_t bh = (int64_t)b * a.H + h;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0 + 16 * qt + fr;
    const bool ok = qi < N;
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      r.qf[qt][ks] = ok ? ld_frag(qp + qi * a.sq[2] + 32 * ks + 8 * fg) : bf16x8_t{};
      r.df[qt][ks] = ok ? ld_frag(dop + qi * a.sdo[2] + 32 * ks + 8 * fg) : bf16x8_t{};
      const bf16x8_t of = ok ? ld_frag(op + qi * a.so[2] + 32 * ks + 8 * fg) : bf16x8_t{};
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += (float)r.df[qt][ks][j] * (float)of[j];
    }
    dsum += __shfl_xor(dsum, 16);
    dsum += __shfl_xor(dsum, 32);
    r.delta[qt] = dsum;
    r.lse2[qt] = ok ? a.lse[bh * N + qi] * kLog2e : 0.f;
    if (ok && fg == 0) a.delta[bh * N + qi] = dsum;
  }
}

// One 64-key tile of the dQ pass: Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ, dSᵀ = Pᵀ∘(dPᵀ-δ), dQᵀ += Kᵀ·dSᵀ
template <bool EDGE>
__device__ __forceinline__ void dq_tile(const uint4* Kt, const uint4* Vt, int t, int N, int nqt, float c,
                                        const DqRows& r, f32x4_t (&acc)[4][2], int fr, int fg) {
  const int nvk = EDGE ? N - t * kTile : kTile;  // valid keys in the tile
  f32x4_t s[4][2], dp[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      s[mt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dp[mt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      if (16 * mt >= nvk) continue;
      const bf16x8_t kf = row_frag(Kt, 16 * mt + fr, 4 * ks + fg);
      const bf16x8_t vf = row_frag(Vt, 16 * mt + fr, 4 * ks + fg);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        if (qt >= nqt) continue;
        s[mt][qt] = mfma(kf, r.qf[qt][ks], s[mt][qt]);
        dp[mt][qt] = mfma(vf, r.df[qt][ks], dp[mt][qt]);
      }
    }
  const int key0 = t * kTile + 4 * fg;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p =
            !EDGE || key0 + 16 * mt + i < N ? __builtin_amdgcn_exp2f(s[mt][qt][i] * c - r.lse2[qt]) : 0.f;
        s[mt][qt][i] = p * (dp[mt][qt][i] - r.delta[qt]);  // dS (in units of the scaled scores)
      }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (32 * ks >= nvk) continue;
    bf16x8_t sf[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) sf[qt] = pack_frag(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8_t kf = tr_frag(Kt, 32 * ks, dt, fr, fg);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        if (qt < nqt) acc[dt][qt] = mfma(kf, sf[qt], acc[dt][qt]);
    }
  }
}

__device__ __forceinline__ void dq_store(const AttnArgs& a, int b, int h, int q0, const f32x4_t (&acc)[4][2],
                                         int fr, int fg) {
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0 + 16 * qt + fr;
    if (qi < a.N) {
      uint16_t* p = a.dq + b * a.sdq[0] + h * a.sdq[1] + qi * a.sdq[2] + 4 * fg;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) st4(p + 16 * dt, acc[dt][qt], a.scale);
    }
  }
}

// 3 waves per SIMD (154 VGPRs): three 4-wave workgroups per CU.  (A whole-head dQ -- one 8-wave
// workgroup per (batch, head), K / V staged once, as attn_fwd_head_k -- measured 174 vs 165 us per
// ViT-B call and was removed, profiles/r05_vit.)
__global__ __launch_bounds__(256, 3) void attn_bwd_dq_k(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * 2 * kTileU4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int N = a.N;
  int xb, h, b;
  block_coords((N + kBlk - 1) / kBlk, a.H, xb, h, b);
  const uint16_t* kp = head(a.k, a.sk, b, h);
  const uint16_t* vp = head(a.v, a.sv, b, h);
  const int q0 = xb * kBlk + wave * 32;
  const bool wave_live = q0 < N;
  const int nqt = q0 + 16 < N ? 2 : 1;  // (as the forward)
  const float c = a.scale * kLog2e;
  DqRows r;
  dq_rows(a, b, h, q0, fr, fg, r);
  f32x4_t acc[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) acc[dt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nt = (N + kTile - 1) / kTile;
  stage_tile(lds, kp, a.sk[2], 0, N, wave, lane);
  stage_tile(lds + kTileU4, vp, a.sv[2], 0, N, wave, lane);
  // tile t landed (every wave is done with the other buffer) -> stage tile t + 1 into it
  auto next = [&](int t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < nt) {
      uint4* Kn = lds + ((t + 1) & 1) * 2 * kTileU4;
      stage_tile(Kn, kp, a.sk[2], (t + 1) * kTile, N, wave, lane);
      stage_tile(Kn + kTileU4, vp, a.sv[2], (t + 1) * kTile, N, wave, lane);
    }
  };
  // full tiles unmasked, the edge tile peeled (one body per loop keeps the VGPR count down)
  const int nfull = N / kTile;
  // the query sub-tile count as a constant: the waves of one workgroup may run different copies of
  // the loop, which pass the same barriers in the same order
  auto run = [&](auto nq) {
    constexpr int NQ = decltype(nq)::value;
    for (int t = 0; t < nfull; ++t) {
      next(t);
      const uint4* Kt = lds + (t & 1) * 2 * kTileU4;
      if (wave_live) dq_tile<false>(Kt, Kt + kTileU4, t, N, NQ, c, r, acc, fr, fg);
    }
    if (nfull < nt) {
      next(nfull);
      const uint4* Kt = lds + (nfull & 1) * 2 * kTileU4;
      if (wave_live) dq_tile<true>(Kt, Kt + kTileU4, nfull, N, NQ, c, r, acc, fr, fg);
    }
  };
  if (nqt == 2) run(std::integral_constant<int, 2>{});
  else run(std::integral_constant<int, 1>{});
  dq_store(a, b, h, q0, acc, fr, fg);
}

// ---------------------------------------------- backward: dK and dV
// A wave's 32 keys: K / V fragments as B operands (lane holds K[k0 + 16kt + fr][32ks + 8fg .. +7])
struct KvRows {
  bf16x8_t kf[2][2], vf[2][2];
};

__device__ __forceinline__ void kv_rows(const AttnArgs& a, int b, int h, int k0, int fr, int fg, KvRows& r) {
  const int N = a.N;
  const uint16_t* kp = head(a.k, a.sk, b, h);
  const uint16_t* vp = head(a.v, a.sv, b, h);
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int ki = k0 + 16 * kt + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      r.kf[kt][ks] = ki < N ? ld_frag(kp + ki * a.sk[2] + 32 * ks + 8 * fg) : bf16x8_t{};
      r.vf[kt][ks] = ki < N ? ld_frag(vp + ki * a.sv[2] + 32 * ks + 8 * fg) : bf16x8_t{};
    }
  }
}

// One 64-query tile: S = Q·Kᵀ, dP = dO·Vᵀ (key on the lane), dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS.
// lse_t / del_t: the tile's 64 log2-domain log-sum-exps (+inf past N) and deltas in LDS.
template <bool EDGE>
__device__ __forceinline__ void dkdv_tile(const uint4* Qt, const uint4* Dt, const float* lse_t, const float* del_t,
                                          int t, int N, int nkt, float c, const KvRows& r, f32x4_t (&dv)[4][2],
                                          f32x4_t (&dk)[4][2], int fr, int fg) {
  const int nvq = EDGE ? N - t * kTile : kTile;  // valid queries in the tile
  f32x4_t s[4][2], dp[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[mt][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dp[mt][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  // S[q][key] = Q·Kᵀ, dP = dO·Vᵀ: lane holds rows q = 16mt + 4fg + i, column key = 16kt + fr
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      if (16 * mt >= nvq) continue;
      const bf16x8_t qa = row_frag(Qt, 16 * mt + fr, 4 * ks + fg);
      const bf16x8_t da = row_frag(Dt, 16 * mt + fr, 4 * ks + fg);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (kt >= nkt) continue;
        s[mt][kt] = mfma(qa, r.kf[kt][ks], s[mt][kt]);
        dp[mt][kt] = mfma(da, r.vf[kt][ks], dp[mt][kt]);
      }
    }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const float4 l4 = *reinterpret_cast<const float4*>(lse_t + 16 * mt + 4 * fg);
    const float4 d4 = *reinterpret_cast<const float4*>(del_t + 16 * mt + 4 * fg);
    const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dl[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(s[mt][kt][i] * c - lv[i]);
        s[mt][kt][i] = p;
        dp[mt][kt][i] = p * (dp[mt][kt][i] - dl[i]);
      }
  }
  // dVᵀ[d][key] += dOᵀ·P, dKᵀ[d][key] += Qᵀ·dS (sum over the tile's 64 queries)
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (32 * ks >= nvq) continue;
    bf16x8_t pf[2], sf[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      pf[kt] = pack_frag(s[2 * ks][kt], s[2 * ks + 1][kt]);
      sf[kt] = pack_frag(dp[2 * ks][kt], dp[2 * ks + 1][kt]);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8_t oa = tr_frag(Dt, 32 * ks, dt, fr, fg);
      const bf16x8_t qa = tr_frag(Qt, 32 * ks, dt, fr, fg);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (kt >= nkt) continue;
        dv[dt][kt] = mfma(oa, pf[kt], dv[dt][kt]);
        dk[dt][kt] = mfma(qa, sf[kt], dk[dt][kt]);
      }
    }
  }
}

__device__ __forceinline__ void dkdv_store(const AttnArgs& a, int b, int h, int k0, const f32x4_t (&dk)[4][2],
                                           const f32x4_t (&dv)[4][2], int fr, int fg) {
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int ki = k0 + 16 * kt + fr;
    if (ki < a.N) {
      uint16_t* pk = a.dk + b * a.sdk[0] + h * a.sdk[1] + ki * a.sdk[2] + 4 * fg;
      uint16_t* pv = a.dv + b * a.sdv[0] + h * a.sdv[1] + ki * a.sdv[2] + 4 * fg;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        st4(pk + 16 * dt, dk[dt][kt], a.scale);
        st4(pv + 16 * dt, dv[dt][kt], 1.f);
      }
    }
  }
}

__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_k(AttnArgs a) {
  // [buf][Q | dO] tiles, then [buf][lse2 | delta] x 64 floats
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * 2 * kTileU4 + 2 * 2 * kTile / 4];
  float* rowc = reinterpret_cast<float*>(lds + 2 * 2 * kTileU4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int N = a.N;
  int xb, h, b;
  block_coords((N + kBlk - 1) / kBlk, a.H, xb, h, b);
  const uint16_t* qp = head(a.q, a.sq, b, h);
  const uint16_t* dop = head(a.dout, a.sdo, b, h);
  const int64_t bh = (int64_t)b * a.H + h;
  const int k0 = xb * kBlk + wave * 32;
  const bool wave_live = k0 < N;
  const int nkt = k0 + 16 < N ? 2 : 1;  // the last wave's second 16-key sub-tile may be empty
  const float c = a.scale * kLog2e;
  KvRows r;
  kv_rows(a, b, h, k0, fr, fg, r);
  f32x4_t dv[4][2], dk[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      dv[dt][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dk[dt][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }

  auto issue = [&](int t, int buf) {
    uint4* Qn = lds + buf * 2 * kTileU4;
    stage_tile(Qn, qp, a.sq[2], t * kTile, N, wave, lane);
    stage_tile(Qn + kTileU4, dop, a.sdo[2], t * kTile, N, wave, lane);
    if (tid < 2 * kTile) {
      const int rr = tid & (kTile - 1), qi = t * kTile + rr;
      float v;
      if (tid < kTile) v = qi < N ? a.lse[bh * N + qi] * kLog2e : INFINITY;  // P = 0 for absent queries
      else v = qi < N ? a.delta[bh * N + qi] : 0.f;
      rowc[buf * 2 * kTile + tid] = v;
    }
  };

  const int nt = (N + kTile - 1) / kTile;
  issue(0, 0);
  auto next = [&](int t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < nt) issue(t + 1, (t & 1) ^ 1);
  };
  // full tiles unmasked, the edge tile peeled
  const int nfull = N / kTile;
  for (int t = 0; t < nfull; ++t) {
    next(t);
    const uint4* Qt = lds + (t & 1) * 2 * kTileU4;
    const float* lse_t = rowc + (t & 1) * 2 * kTile;
    if (wave_live) dkdv_tile<false>(Qt, Qt + kTileU4, lse_t, lse_t + kTile, t, N, nkt, c, r, dv, dk, fr, fg);
  }
  if (nfull < nt) {
    next(nfull);
    const uint4* Qt = lds + (nfull & 1) * 2 * kTileU4;
    const float* lse_t = rowc + (nfull & 1) * 2 * kTile;
    if (wave_live) dkdv_tile<true>(Qt, Qt + kTileU4, lse_t, lse_t + kTile, nfull, N, nkt, c, r, dv, dk, fr, fg);
  }
  dkdv_store(a, b, h, k0, dk, dv, fr, fg);
}

// Whole-head dK/dV (N <= 256): one 8-wave workgroup per (batch, head) stages the head's Q and dO
// whole (waves 0-3 Q, 4-7 dO) and its log-sum-exps / deltas (kHeadTiles x 64 each) behind one wait
// and one barrier; each wave then runs its 32 keys over every query tile from LDS
__global__ __launch_bounds__(512, 2) void attn_bwd_dkdv_head_k(AttnArgs a) {
  constexpr int kRows = kHeadTiles * kTile;
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * kHeadTiles * kTileU4 + 2 * kRows / 4];
  float* rowc = reinterpret_cast<float*>(lds + 2 * kHeadTiles * kTileU4);  // [lse2 | delta] x kRows
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int N = a.N;
  const int h = (int)(blockIdx.x % a.H), b = (int)(blockIdx.x / a.H);
  const int64_t bh = (int64_t)b * a.H + h;
  const int nt = (N + kTile - 1) / kTile;  // <= kHeadTiles (host check)
  {
    const bool dq = wave >= 4;
    uint4* base = lds + (dq ? kHeadTiles * kTileU4 : 0);
    const uint16_t* src = dq ? head(a.dout, a.sdo, b, h) : head(a.q, a.sq, b, h);
    const int64_t rs = dq ? a.sdo[2] : a.sq[2];
    for (int t = 0; t < nt; ++t) stage_tile(base + t * kTileU4, src, rs, t * kTile, N, wave & 3, lane);
  }
  {
    const int qi = tid & (kRows - 1);
    float v;
    if (tid < kRows) v = qi < N ? a.lse[bh * N + qi] * kLog2e : INFINITY;  // P = 0 for absent queries
    else v = qi < N ? a.delta[bh * N + qi] : 0.f;
    rowc[tid] = v;
  }
  const int k0 = wave * 32;
  const bool wave_live = k0 < N;
  const int nkt = k0 + 16 < N ? 2 : 1;
  const float c = a.scale * kLog2e;
  KvRows r;
  kv_rows(a, b, h, k0, fr, fg, r);
  f32x4_t dv[4][2], dk[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      dv[dt][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dk[dt][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every Q / dO tile and row constant of the head landed (the only barrier)
  if (!wave_live) return;
  const int nfull = N / kTile;
  auto run = [&](auto nk) {  // the key sub-tile count as a constant (as the head forward)
    constexpr int NK = decltype(nk)::value;
    for (int t = 0; t < nfull; ++t)
      dkdv_tile<false>(lds + t * kTileU4, lds + (kHeadTiles + t) * kTileU4, rowc + t * kTile,
                       rowc + kRows + t * kTile, t, N, NK, c, r, dv, dk, fr, fg);
    if (nfull < nt)
      dkdv_tile<true>(lds + nfull * kTileU4, lds + (kHeadTiles + nfull) * kTileU4, rowc + nfull * kTile,
                      rowc + kRows + nfull * kTile, nfull, N, NK, c, r, dv, dk, fr, fg);
  };
  if (nkt == 2) run(std::integral_constant<int, 2>{});
  else run(std::integral_constant<int, 1>{});
  dkdv_store(a, b, h, k0, dk, dv, fr, fg);
}

}  // namespace

int attn_supported(int D) { return D == 64; }

// Whole-head (one workgroup per (batch, head)) forward and dK/dV for N <= 256, measured fastest on
// ViT-B/16 (profiles/r05_vit); TBAMD_ATTN_HEAD is a bit mask (1 forward, 4 dK/dV; default 5) for
// A/B, 0 = the 128-row workgroups everywhere
static int g_attn_head = [] {
  const char* e = getenv("TBAMD_ATTN_HEAD");
  return e ? atoi(e) & 5 : 5;
}();

int attn_set_head_mask(int mask) {
  const int old = g_attn_head;
  if (mask >= 0) g_attn_head = mask & 5;
  return old;
}

void attn_fwd(const AttnArgs& a, hipStream_t st) {
  if ((g_attn_head & 1) && a.N <= kHeadTiles * kTile) {
    hipLaunchKernelGGL(attn_fwd_head_k, dim3(a.H * a.B), dim3(kHeadWaves * 64), 0, st, a);
    return;
  }
  const int nblk = (a.N + kBlk - 1) / kBlk;
  hipLaunchKernelGGL(attn_fwd_k, dim3(nblk * a.H * a.B), dim3(256), 0, st, a);
}

void attn_bwd(const AttnArgs& a, hipStream_t st) {
  const bool fits = a.N <= kHeadTiles * kTile;
  const int nblk = (a.N + kBlk - 1) / kBlk;
  // dQ pass first: it also writes delta = rowsum(dO * O), which the dK/dV pass reads
  hipLaunchKernelGGL(attn_bwd_dq_k, dim3(nblk * a.H * a.B), dim3(256), 0, st, a);
  if ((g_attn_head & 4) && fits)
    hipLaunchKernelGGL(attn_bwd_dkdv_head_k, dim3(a.H * a.B), dim3(kHeadWaves * 64), 0, st, a);
  else
    hipLaunchKernelGGL(attn_bwd_dkdv_k, dim3(nblk * a.H * a.B), dim3(256), 0, st, a);
}

}  // namespace tbamd
