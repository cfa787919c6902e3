// Gram matrix G[b] = F_bᵀ F_b · scale of NHWC features (SYRK on MFMA), K18 of
// SURVEY.md §2.3.1 — the style losses of examples/img_stt (reference:
// online.py:60-63 per-sample bmm, offline.py:25-28 whole-image matmul).
//
// F_b is [HW][C] (channels_last rows).  Only the upper-triangle BT x BT output
// tiles are computed; the reduction over HW is split across workgroups
// (split-K) so that a 64-channel Gram over 512² pixels still fills the chip,
// and each split writes an f32 partial tile; a second kernel sums the splits in
// a fixed order (deterministic), scales, and mirrors the lower triangle.
//
// Both MFMA operands are COLUMNS of a staged [64 pixels][64 channels] tile
// (A[i][p] = F[p][i], B[p][j] = F[p][j]), read with ds_read_b64_tr_b16 through
// mfma_tile.h's tr_frag; A and B use the same pixel permutation, so the
// product sums over pixels exactly.  Tiles are staged with direct global->LDS
// loads, double buffered, one barrier per 64-pixel step.
#include "common.h"
#include "mfma_tile.h"
#include "tbamd.h"

namespace tbamd {
namespace {

// upper-triangle tile pair index -> (ti, tj), ti <= tj
__device__ __forceinline__ void tile_pair(int tp, int nt, int& ti, int& tj) {
  ti = 0;
  int rem = tp;
  while (rem >= nt - ti) {
    rem -= nt - ti;
    ++ti;
  }
  tj = ti + rem;
}

template <int BT>
__global__ __launch_bounds__(256, 2) void gram_partial_k(const uint16_t* __restrict__ f, float* __restrict__ part,
                                                         int C, int64_t HW, int nt, int ntp, int nsplit,
                                                         int64_t pix_per_split) {
  constexpr int SL = BT / 64;        // 64-channel slices per operand tile
  constexpr int STAGE = 2 * SL * kTileU4;  // A slices then B slices
  constexpr int TW = BT / 32;        // 16x16 MFMA tiles per wave side (wave tile BT/2)
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;

  const int s = blockIdx.x % nsplit;
  const int tp = (blockIdx.x / nsplit) % ntp;
  const int b = blockIdx.x / (nsplit * ntp);
  int ti, tj;
  tile_pair(tp, nt, ti, tj);
  const bool diag = ti == tj;
  const int64_t p0 = s * pix_per_split;
  const int64_t p1 = p0 + pix_per_split < HW ? p0 + pix_per_split : HW;
  const uint16_t* fb = f + (int64_t)b * HW * C;
  const int nst = (int)((p1 - p0 + kTile - 1) / kTile);
  // stage_tile takes int row indices relative to the split start
  const int lim = (int)(p1 - p0);
  const uint16_t* fa = fb + p0 * C + ti * BT;
  const uint16_t* fbb = fb + p0 * C + tj * BT;

  auto issue = [&](int st, int buf) {
    uint4* A = lds + buf * STAGE;
#pragma unroll
    for (int sl = 0; sl < SL; ++sl) {
      stage_tile(A + sl * kTileU4, fa + sl * 64, C, st * kTile, lim, wave, lane);
      if (!diag) stage_tile(A + (SL + sl) * kTileU4, fbb + sl * 64, C, st * kTile, lim, wave, lane);
    }
  };

  f32x4_t acc[TW][TW];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nst > 0) issue(0, 0);
  for (int st = 0; st < nst; ++st) {
    const uint4* A = lds + (st & 1) * STAGE;
    const uint4* Bt = diag ? A : A + SL * kTileU4;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (st + 1 < nst) issue(st + 1, (st + 1) & 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[TW], bfr[TW];
#pragma unroll
      for (int i = 0; i < TW; ++i) {
        const int ca = wm * (BT / 2) + 16 * i;  // channel offset inside the A tile
        af[i] = tr_frag(A + (ca >> 6) * kTileU4, 32 * ks, (ca & 63) >> 4, fr, fg);
        const int cb = wn * (BT / 2) + 16 * i;
        bfr[i] = tr_frag(Bt + (cb >> 6) * kTileU4, 32 * ks, (cb & 63) >> 4, fr, fg);
      }
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TW; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    }
  }
  // partial tile [BT][BT] f32: lane holds rows 16i + 4fg + r, column 16j + fr
  float* out = part + (((int64_t)b * ntp + tp) * nsplit + s) * BT * BT;
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BT / 2) + 16 * i + 4 * fg + r;
        const int col = wn * (BT / 2) + 16 * j + fr;
        out[row * BT + col] = acc[i][j][r];
      }
}

// sum the splits (fixed order), scale, mirror: out [B][C][C] f32.  Works in
// tile space so the split partials are read along their contiguous rows: a
// workgroup owns 16 consecutive elements of one tile and spreads the splits
// over 16 lane groups (a 64x64 Gram of a 512x512 image has ~1000 splits; one
// thread per output walking them serially took 0.24 ms), merged through LDS in
// a fixed order.
constexpr int kGrQ = 16, kGrS = 16;
template <int BT>
__global__ __launch_bounds__(kGrQ * kGrS) void gram_reduce_k(const float* __restrict__ part, float* __restrict__ out,
                                                            int C, int nt, int ntp, int nsplit, float scale) {
  __shared__ float red[kGrS][kGrQ];
  const int tx = threadIdx.x % kGrQ, ty = threadIdx.x / kGrQ;
  constexpr int per_tile = BT * BT / kGrQ;
  const int64_t bt = blockIdx.x / per_tile;  // b * ntp + tp
  const int q = (int)(blockIdx.x % per_tile) * kGrQ + tx;
  const float* p = part + bt * nsplit * (int64_t)(BT * BT) + q;
  float acc = 0.f;
#pragma unroll 8
  for (int s = ty; s < nsplit; s += kGrS) acc += p[(int64_t)s * BT * BT];
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < kGrS; ++r) t += red[r][tx];
    t *= scale;
    const int b = (int)(bt / ntp);
    int tp = (int)(bt % ntp), ti = 0;
    while (tp >= nt - ti) {  // upper-triangle tile index -> (ti, tj)
      tp -= nt - ti;
      ++ti;
    }
    const int tj = ti + tp;
    const int i = ti * BT + q / BT, j = tj * BT + q % BT;
    float* o = out + (int64_t)b * C * C;
    o[(int64_t)i * C + j] = t;
    if (ti != tj) o[(int64_t)j * C + i] = t;
  }
}

// backward prologue: sym[b] = bf16((dG[b] + dG[b]^T) * scale), the symmetric operand of the
// input-gradient GEMM dF_b = F_b sym_b (one pass over the [B][C][C] f32 gradient)
__global__ __launch_bounds__(256) void gram_sym_k(const float* __restrict__ dg, uint16_t* __restrict__ sym, int B,
                                                  int C, float scale) {
  const int64_t total = (int64_t)B * C * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t b = e / ((int64_t)C * C);
    const int r = (int)(e % ((int64_t)C * C));
    const int i = r / C, j = r % C;
    const float* g = dg + b * C * C;
    sym[e] = f2bf((g[(int64_t)i * C + j] + g[(int64_t)j * C + i]) * scale);
  }
}

}  // namespace

void gram_sym(const float* dg, void* sym, int B, int C, float scale, hipStream_t st) {
  const int64_t total = (int64_t)B * C * C;
  int64_t gs = (total + 255) / 256;
  if (gs > 4096) gs = 4096;
  if (gs > 0) hipLaunchKernelGGL(gram_sym_k, dim3((unsigned)gs), dim3(256), 0, st, dg, (uint16_t*)sym, B, C, scale);
}

int gram_tile(int C) { return C % 128 == 0 ? 128 : (C % 64 == 0 ? 64 : 0); }

int gram_splits(int B, int C, int64_t HW) {
  const int BT = gram_tile(C);
  const int nt = C / BT, ntp = nt * (nt + 1) / 2;
  const int64_t steps = (HW + kTile - 1) / kTile;
  // ~512 workgroups (2 per CU), at least 4 pixel steps per split
  int64_t ns = (512 + (int64_t)B * ntp - 1) / ((int64_t)B * ntp);
  const int64_t maxs = (steps + 3) / 4;
  if (ns > maxs) ns = maxs;
  return ns < 1 ? 1 : (int)ns;
}

int64_t gram_workspace(int B, int C, int64_t HW) {
  const int BT = gram_tile(C);
  const int nt = C / BT, ntp = nt * (nt + 1) / 2;
  return (int64_t)B * ntp * gram_splits(B, C, HW) * BT * BT;
}

void gram(const void* f, int B, int64_t HW, int C, float scale, float* workspace, float* out, hipStream_t st) {
  const int BT = gram_tile(C);
  const int nt = C / BT, ntp = nt * (nt + 1) / 2;
  const int ns = gram_splits(B, C, HW);
  const int64_t steps = (HW + kTile - 1) / kTile;
  const int64_t pps = (steps + ns - 1) / ns * kTile;
  const dim3 grid((unsigned)((int64_t)B * ntp * ns));
  const dim3 rgrid((unsigned)((int64_t)B * ntp * (BT * BT / kGrQ)));
  if (BT == 128) {
    hipLaunchKernelGGL(gram_partial_k<128>, grid, dim3(256), 0, st, (const uint16_t*)f, workspace, C, HW, nt, ntp, ns,
                       pps);
    hipLaunchKernelGGL(gram_reduce_k<128>, rgrid, dim3(kGrQ * kGrS), 0, st, workspace, out, C, nt, ntp, ns, scale);
  } else {
    hipLaunchKernelGGL(gram_partial_k<64>, grid, dim3(256), 0, st, (const uint16_t*)f, workspace, C, HW, nt, ntp, ns,
                       pps);
    hipLaunchKernelGGL(gram_reduce_k<64>, rgrid, dim3(kGrQ * kGrS), 0, st, workspace, out, C, nt, ntp, ns, scale);
  }
}

}  // namespace tbamd
