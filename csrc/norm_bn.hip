// Fused NHWC BatchNorm (+ residual add + activation) for gfx950.
//
// Replaces the reference's cuDNN BatchNorm2d -> ReLU -> residual add chain
// (torchvision ResNet used at
// /root/reference/examples/img_cls/resnet/resnet.py:111) with four kernels:
//
//   forward :  stats_partial  ->  stats_finalize (+ running-stat update)  ->  apply
//   backward:  bwd_partial (also emits d_residual)  ->  bwd_finalize  ->  bwd_apply
//
// The activation tensor is viewed as [M, C] (M = N*H*W, channels innermost).
// Every pass streams 16 B per lane (8 channels); per-channel reductions are
// shifted sums in f32 per workgroup, merged in f64 by the finalize kernels,
// so the result is deterministic (no float atomics).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <stdexcept>

#include "common.h"
#include "tbamd.h"

namespace tbamd {

constexpr int kBnThreads = 256;
constexpr int kGroupsPerTile = 64;  // channel groups (of VEC channels) per workgroup tile

struct BnGeom {
  int G;    // channel groups = C / VEC
  int GT;   // groups per tile = min(G, 64)
  int rpp;  // rows per pass = 256 / GT
};
__host__ __device__ inline BnGeom bn_geom(int C, int VEC) {
  BnGeom g;
  g.G = C / VEC;
  g.GT = g.G < kGroupsPerTile ? g.G : kGroupsPerTile;
  g.rpp = kBnThreads / g.GT;
  return g;
}

// ---------------------------------------------------------------------------
// forward statistics: per workgroup shifted sums  S = Σ(x - s), Q = Σ(x - s)^2
// shift s = x[0, c] keeps the f32 sums well conditioned when |mean| >> std.
// grid = (nblk, ceil(G / 64)); partials laid out [nblk][C].
template <int DT, int VEC>
__global__ __launch_bounds__(kBnThreads) void bn_stats_partial_k(
    const storage_t<DT>* __restrict__ x, int64_t M, int C, int64_t rows_per_blk,
    float* __restrict__ psum, float* __restrict__ psq) {
  const BnGeom g = bn_geom(C, VEC);
  // blockIdx.z = sample (GroupNorm / InstanceNorm statistics); BN uses one "sample"
  x += (int64_t)blockIdx.z * M * C;
  psum += (int64_t)blockIdx.z * gridDim.x * C;
  psq += (int64_t)blockIdx.z * gridDim.x * C;
  const int tid = threadIdx.x;
  const int gl = tid % g.GT, rl = tid / g.GT;
  const int grp = blockIdx.y * kGroupsPerTile + gl;
  const bool active = rl < g.rpp && gl < g.GT && grp < g.G;
  __shared__ float sm_s[kBnThreads * VEC];
  __shared__ float sm_q[kBnThreads * VEC];
  float s[VEC], q[VEC], sh[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) s[i] = q[i] = 0.f;
  if (active) {
    const int c0 = grp * VEC;
    load_vec<DT, VEC>(x + c0, sh);
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
    int64_t r1 = r0 + rows_per_blk;
    if (r1 > M) r1 = M;
    int64_t r = r0 + rl;
    // 4 rows in flight per lane
    for (; r + 3 * g.rpp < r1; r += 4 * g.rpp) {
      float v0[VEC], v1[VEC], v2[VEC], v3[VEC];
      load_vec<DT, VEC>(x + r * C + c0, v0);
      load_vec<DT, VEC>(x + (r + g.rpp) * C + c0, v1);
      load_vec<DT, VEC>(x + (r + 2 * g.rpp) * C + c0, v2);
      load_vec<DT, VEC>(x + (r + 3 * g.rpp) * C + c0, v3);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float d0 = v0[i] - sh[i], d1 = v1[i] - sh[i], d2 = v2[i] - sh[i], d3 = v3[i] - sh[i];
        s[i] += (d0 + d1) + (d2 + d3);
        q[i] += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    }
    for (; r < r1; r += g.rpp) {
      float v[VEC];
      load_vec<DT, VEC>(x + r * C + c0, v);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float d = v[i] - sh[i];
        s[i] += d;
        q[i] += d * d;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    sm_s[tid * VEC + i] = s[i];
    sm_q[tid * VEC + i] = q[i];
  }
  __syncthreads();
  // (group, element) pairs of this tile: GT * VEC <= 512; two per thread.
  const int npairs = g.GT * VEC;
  for (int p = tid; p < npairs; p += kBnThreads) {
    const int pg = p / VEC, pe = p % VEC;
    const int cgrp = blockIdx.y * kGroupsPerTile + pg;
    if (cgrp >= g.G) continue;
    float ts = 0.f, tq = 0.f;
    for (int rr = 0; rr < g.rpp; ++rr) {
      const int t = rr * g.GT + pg;
      ts += sm_s[t * VEC + pe];
      tq += sm_q[t * VEC + pe];
    }
    const int c = cgrp * VEC + pe;
    psum[(int64_t)blockIdx.x * C + c] = ts;
    psq[(int64_t)blockIdx.x * C + c] = tq;
  }
}

// ---------------------------------------------------------------------------
// Column-sum finalize shared by the BN statistics / backward reductions.
//
// Input: two [nrows][C] float partial arrays (row stride `rs` floats) written
// by a partial-sum pass (BN stats, BN backward, or the conv epilogue with one
// row per pixel tile — 6272 rows for ResNet-50's first stage).  A grid of
// ceil(C/64) x NSL workgroups sums NSL row slices in f64 (64 channels x 4 row
// groups per workgroup, coalesced 256-B rows); the LAST workgroup of each
// channel block (device-scope atomic ticket) merges the NSL slice sums in a
// fixed order — deterministic — and runs the per-channel epilogue `fin`.  One
// launch, and every CU participates even for C = 64.  The tickets reset
// themselves at the end of each launch; every HIP stream gets its own ticket
// row (kColsumStreamSlots rows, assigned on first use by colsum_stream_slot), so
// launches on two streams — comm/compute overlap, two models on two streams —
// never share a counter.  Launches on ONE stream are serialised by the stream.
constexpr int kColsumStreamSlots = 32;
constexpr int kColsumTickets = 4096;  // channel blocks of 64: C <= 262144
__device__ unsigned g_colsum_ticket[kColsumStreamSlots][kColsumTickets];

// host: stream -> ticket row (a small open table).  Once kColsumStreamSlots distinct streams have
// a row, a new stream gets -1 and its launches take the single-phase path (one workgroup per
// channel block, no tickets): slower, but two streams never share arrival counters.
static int colsum_stream_slot(hipStream_t st) {
  static std::mutex mu;
  static hipStream_t streams[kColsumStreamSlots];
  static int used = 0;
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < used; ++i)
    if (streams[i] == st) return i;
  if (used == kColsumStreamSlots) return -1;
  streams[used] = st;
  return used++;
}

constexpr int kColsumRowGroups = 4;

// Slab publish of the in-launch reductions below.  WT (default): every slab word is stored
// write-through (an agent-scope relaxed atomic store = global_store sc1), the storing waves drain
// (vmcnt 0) and one lane adds the ticket -- no release fence.  The fence it replaces
// (buffer_wbl2 sc1) writes back EVERY dirty line of the XCD's L2, i.e. the megabytes of
// activations the conv in front of this finalize just stored (cdna_hip_programming.md §5
// "In-launch split-K reduction", sc1 form; §6 Guideline 16 R1).  The reducer keeps its
// agent-scope acquire and reads the slabs with plain loads.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void slab_store_wt(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
static const bool g_colsum_wt = [] {
  const char* e = getenv("TBAMD_COLSUM_WT");
  return !(e && e[0] == '0');
}();

template <class Fin, bool WT = true>
__global__ __launch_bounds__(256) void colsum_fin_k(const float* __restrict__ pa, const float* __restrict__ pb,
                                                    int64_t rs, int nrows, int C, int rows_per_sl,
                                                    double* __restrict__ ws, Fin fin, int slot) {
  unsigned* ticket = g_colsum_ticket[slot];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * rows_per_sl;
  const int r1 = min(r0 + rows_per_sl, nrows);
  double a = 0.0, b = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int r = r0 + ty; r < r1; r += kColsumRowGroups) {
      a += (double)pa[(int64_t)r * rs + c];
      b += (double)pb[(int64_t)r * rs + c];
    }
  }
  __shared__ double sm[2][kColsumRowGroups][64];
  __shared__ bool last;
  sm[0][ty][tx] = a;
  sm[1][ty][tx] = b;
  __syncthreads();
  if (ty == 0) {
#pragma unroll
    for (int i = 1; i < kColsumRowGroups; ++i) {
      a += sm[0][i][tx];
      b += sm[1][i][tx];
    }
  }
  if (gridDim.y == 1) {
    if (ty == 0 && c < C) fin(c, a, b);
    return;
  }
  if (ty == 0 && c < C) {
    if constexpr (WT) {
      slab_store_wt(&ws[((int64_t)blockIdx.y * 2 + 0) * C + c], a);
      slab_store_wt(&ws[((int64_t)blockIdx.y * 2 + 1) * C + c], b);
    } else {
      ws[((int64_t)blockIdx.y * 2 + 0) * C + c] = a;
      ws[((int64_t)blockIdx.y * 2 + 1) * C + c] = b;
    }
  }
  // publish the slab (cdna_hip_programming.md §5 "in-launch split-K reduction"):
  // drain stores -> barrier -> (plain stores: one agent-scope release) -> ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add(&ticket[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  // reducer: all 256 threads read the slabs (slice sl -> row group sl % 4),
  // merged in a fixed order -> deterministic
  a = b = 0.0;
  if (c < C) {
    for (int sl = ty; sl < (int)gridDim.y; sl += kColsumRowGroups) {
      a += ws[((int64_t)sl * 2 + 0) * C + c];
      b += ws[((int64_t)sl * 2 + 1) * C + c];
    }
  }
  sm[0][ty][tx] = a;
  sm[1][ty][tx] = b;
  __syncthreads();
  if (ty == 0 && c < C) {
#pragma unroll
    for (int i = 1; i < kColsumRowGroups; ++i) {
      a += sm[0][i][tx];
      b += sm[1][i][tx];
    }
    fin(c, a, b);
  }
  if (threadIdx.x == 0) ticket[blockIdx.x] = 0u;
}

// Vectorised variant for C % 4 == 0 and 16-B aligned rows (every conv-epilogue statistics
// array and dgrad BN-partial array): 16 lanes x float4 cover the 64 channels of the block and
// 16 row groups stride the slice, so a slice of ~100 rows is ~6 float4 pairs per lane, all in
// flight at once (the scalar kernel above walks 25 dependent-latency rounds for the same
// slice).  Same fixed summation order per channel -> deterministic; same ticket protocol.
template <class Fin, bool WT = true>
__global__ __launch_bounds__(256) void colsum_fin4_k(const float* __restrict__ pa, const float* __restrict__ pb,
                                                     int64_t rs, int nrows, int C, int rows_per_sl,
                                                     double* __restrict__ ws, Fin fin, int slot) {
  unsigned* ticket = g_colsum_ticket[slot];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + tx * 4;
  const int r0 = blockIdx.y * rows_per_sl;
  const int r1 = min(r0 + rows_per_sl, nrows);
  double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
  if (c0 < C) {
#pragma unroll 4
    for (int r = r0 + ty; r < r1; r += 16) {
      const float4 va = *reinterpret_cast<const float4*>(pa + (int64_t)r * rs + c0);
      const float4 vb = *reinterpret_cast<const float4*>(pb + (int64_t)r * rs + c0);
      a[0] += (double)va.x;
      a[1] += (double)va.y;
      a[2] += (double)va.z;
      a[3] += (double)va.w;
      b[0] += (double)vb.x;
      b[1] += (double)vb.y;
      b[2] += (double)vb.z;
      b[3] += (double)vb.w;
    }
  }
  // the 16 row groups: the 4 of a wave (lanes tx, tx + 16, tx + 32, tx + 48) by shuffles, then the
  // 4 waves through LDS laid out [wave][kind][e][tx] -- lane-consecutive doubles on both the
  // 16-lane stores and the 64-channel reads (the [ty][channel] layout this replaces put the 16
  // lanes of a store 32 B apart: 32 % bank conflicts)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] += __shfl_xor(a[e], 16);
    a[e] += __shfl_xor(a[e], 32);
    b[e] += __shfl_xor(b[e], 16);
    b[e] += __shfl_xor(b[e], 32);
  }
  __shared__ double sm[4][2][4][16];
  __shared__ double sm2[2][4][64];  // (the reducer's [g4][channel] sums, below)
  __shared__ bool last;
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sm[wv][0][e][tx] = a[e];
      sm[wv][1][e][tx] = b[e];
    }
  }
  __syncthreads();
  const int cl = threadIdx.x & 63, c = blockIdx.x * 64 + cl;
  double sa = 0.0, sb = 0.0;
  if (threadIdx.x < 64) {
    // channel cl = 4 tx + e
    const int e = cl & 3, t = cl >> 2;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sa += sm[w][0][e][t];
      sb += sm[w][1][e][t];
    }
  }
  if (gridDim.y == 1) {
    if (threadIdx.x < 64 && c < C) fin(c, sa, sb);
    return;
  }
  if (threadIdx.x < 64 && c < C) {
    if constexpr (WT) {
      slab_store_wt(&ws[((int64_t)blockIdx.y * 2 + 0) * C + c], sa);
      slab_store_wt(&ws[((int64_t)blockIdx.y * 2 + 1) * C + c], sb);
    } else {
      ws[((int64_t)blockIdx.y * 2 + 0) * C + c] = sa;
      ws[((int64_t)blockIdx.y * 2 + 1) * C + c] = sb;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add(&ticket[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  // reducer: slices strided over 4 row groups (tid >> 6), merged in a fixed order
  const int g4 = threadIdx.x >> 6;
  sa = sb = 0.0;
  if (c < C) {
#pragma unroll 8
    for (int sl = g4; sl < (int)gridDim.y; sl += 4) {
      sa += ws[((int64_t)sl * 2 + 0) * C + c];
      sb += ws[((int64_t)sl * 2 + 1) * C + c];
    }
  }
  sm2[0][g4][cl] = sa;
  sm2[1][g4][cl] = sb;
  __syncthreads();
  if (threadIdx.x < 64 && c < C) {
    sa = sm2[0][0][cl] + sm2[0][1][cl] + sm2[0][2][cl] + sm2[0][3][cl];
    sb = sm2[1][0][cl] + sm2[1][1][cl] + sm2[1][2][cl] + sm2[1][3][cl];
    fin(c, sa, sb);
  }
  if (threadIdx.x == 0) ticket[blockIdx.x] = 0u;
}

// f64 workspace (doubles) colsum_fin_k needs for nrows partial rows of C channels
// slice count: >= `min_rows` partial rows per workgroup, at most `max_sl` workgroups per
// 64-channel block (TBAMD_COLSUM="min_rows,max_sl" overrides the defaults for tuning)
static int colsum_slices(int nrows) {
  // 32 / 128: +0.3-0.4 % on the ResNet-50 step over 64 / 64 (profiles/r05_colsum)
  static int min_rows = -1, max_sl = 128;
  if (min_rows < 0) {
    min_rows = 32;
    if (const char* e = getenv("TBAMD_COLSUM")) {
      int a = 0, b = 0;
      if (sscanf(e, "%d,%d", &a, &b) == 2 && a > 0 && b > 0 && b <= 1024) {
        min_rows = a;
        max_sl = b;
      }
    }
  }
  int nsl = cdiv(nrows, min_rows);
  return nsl < 1 ? 1 : (nsl > max_sl ? max_sl : nsl);
}

int64_t colsum_workspace(int nrows, int C) { return (int64_t)colsum_slices(nrows) * 2 * C; }

// A/B switch for the finalize kernel (TBAMD_COLSUM_SCALAR=1: scalar colsum_fin_k everywhere)
static const bool g_colsum_scalar = [] {
  const char* e = getenv("TBAMD_COLSUM_SCALAR");
  return e && e[0] == '1';
}();

template <class Fin>
static void launch_colsum_fin(const float* pa, const float* pb, int64_t rs, int nrows, int C, double* ws, Fin fin,
                              hipStream_t st) {
  int nsl = colsum_slices(nrows);
  int slot = nsl > 1 ? colsum_stream_slot(st) : 0;
  if (slot < 0) nsl = 1, slot = 0;  // out of ticket rows: single phase (see colsum_stream_slot)
  const int rps = cdiv(nrows, nsl);
  const bool vec = C % 4 == 0 && rs % 4 == 0 && ((uintptr_t)pa & 15) == 0 && ((uintptr_t)pb & 15) == 0;
  const dim3 grid(cdiv(C, 64), nsl);
  if (vec && !g_colsum_scalar) {
    if (g_colsum_wt) colsum_fin4_k<Fin, true><<<grid, 256, 0, st>>>(pa, pb, rs, nrows, C, rps, ws, fin, slot);
    else colsum_fin4_k<Fin, false><<<grid, 256, 0, st>>>(pa, pb, rs, nrows, C, rps, ws, fin, slot);
  } else {
    if (g_colsum_wt) colsum_fin_k<Fin, true><<<grid, 256, 0, st>>>(pa, pb, rs, nrows, C, rps, ws, fin, slot);
    else colsum_fin_k<Fin, false><<<grid, 256, 0, st>>>(pa, pb, rs, nrows, C, rps, ws, fin, slot);
  }
}

// training statistics -> mean / invstd (saved for backward), fused affine
// scale / shift, running stats (unbiased variance, torch semantics) and the
// num_batches_tracked counter.  (s, q) are sums of (x - shift) and its square.
template <int DT>
struct StatsFin {
  int64_t M;
  const storage_t<DT>* shift_x;  // row 0 of x: per-channel shift of the partial sums (nullptr: raw sums)
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  int64_t* nbt;
  float momentum, eps;
  float *mean_out, *invstd_out, *scale_out, *shift_out;
  __device__ void operator()(int c, double s, double q) const {
    const double md = s / (double)M;
    double var = q / (double)M - md * md;
    if (var < 0.0) var = 0.0;
    const float mean = (float)((shift_x ? (double)Elem<DT>::ld(shift_x, c) : 0.0) + md);
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    mean_out[c] = mean;
    invstd_out[c] = invstd;
    const float gm = gamma ? gamma[c] : 1.f;
    const float bt = beta ? beta[c] : 0.f;
    const float sc = gm * invstd;
    scale_out[c] = sc;
    shift_out[c] = bt - mean * sc;
    if (running_mean) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
    }
    if (nbt && c == 0) *nbt += 1;
  }
};

// eval-mode coefficients from running stats
__global__ void bn_eval_coeffs_k(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                 const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                 float* mean_out, float* invstd_out, float* scale_out, float* shift_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rv[c] + eps);
  const float gm = gamma ? gamma[c] : 1.f;
  const float bt = beta ? beta[c] : 0.f;
  mean_out[c] = rm[c];
  invstd_out[c] = invstd;
  scale_out[c] = gm * invstd;
  shift_out[c] = bt - rm[c] * gm * invstd;
}

// ---------------------------------------------------------------------------
// forward apply: y = act(x * scale[c] + shift[c] (+ res)).
// Row-tiled like the reductions: each lane owns VEC fixed channels, keeps
// their scale/shift in registers and walks rows (no per-element index math).
// MASK (VEC == 8): also write one bit per element, (y > 0), as a byte per
// 8-channel group ([M][C/8]) — the backward then reads 1/16 of y's bytes.
// RESAFF (RES, VEC == 8): the residual is itself the INPUT of a BatchNorm without activation (a
// bottleneck's downsample branch, ops/norm.py lazy affine residual): res * rsc[c] + rsh[c] is added,
// so that BN's output is never written.
template <int DT, int VEC, int ACT, bool RES, bool MASK = false, bool RESAFF = false>
__global__ __launch_bounds__(kBnThreads) void bn_apply_k(const storage_t<DT>* __restrict__ x,
                                                         const storage_t<DT>* __restrict__ res,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int64_t M, int C,
                                                         int64_t rows_per_blk, float slope,
                                                         storage_t<DT>* __restrict__ y,
                                                         uint8_t* __restrict__ mask = nullptr,
                                                         const float* __restrict__ rsc = nullptr,
                                                         const float* __restrict__ rsh = nullptr, int rev = 0) {
  static_assert(!MASK || VEC == 8, "mask bits need 8-channel groups");
  static_assert(!RESAFF || (RES && VEC == 8), "affine residual: 8-channel groups");
  const BnGeom g = bn_geom(C, VEC);
  {
    const int64_t zo = (int64_t)blockIdx.z * M * C;
    x += zo;
    y += zo;
    if constexpr (RES) res += zo;
    if constexpr (MASK) mask += (int64_t)blockIdx.z * M * (C / 8);
    scale += (int64_t)blockIdx.z * C;
    shift += (int64_t)blockIdx.z * C;
  }
  const int tid = threadIdx.x;
  const int gl = tid % g.GT, rl = tid / g.GT;
  const int grp = blockIdx.y * kGroupsPerTile + gl;
  if (rl >= g.rpp || grp >= g.G) return;
  const int c0 = grp * VEC;
  float sc[VEC], sf[VEC], rc[RESAFF ? VEC : 1], rf[RESAFF ? VEC : 1];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    sc[i] = scale[c0 + i];
    sf[i] = shift[c0 + i];
  }
  if constexpr (RESAFF) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      rc[i] = rsc[c0 + i];
      rf[i] = rsh[c0 + i];
    }
  }
  // rev: the first-dispatched workgroups take the LAST rows -- the lines the producer wrote last are
  // the ones still in the memory-side cache (g_bn_rev, TBAMD_BN_REVERSE)
  const int64_t r0 = (int64_t)(rev ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x) * rows_per_blk;
  int64_t r1 = r0 + rows_per_blk;
  if (r1 > M) r1 = M;
  int64_t r = r0 + rl;
  for (; r + g.rpp < r1; r += 2 * g.rpp) {
    const int64_t o0 = r * C + c0, o1 = (r + g.rpp) * C + c0;
    float v0[VEC], v1[VEC], q0[VEC], q1[VEC];
    load_vec<DT, VEC>(x + o0, v0);
    load_vec<DT, VEC>(x + o1, v1);
    if constexpr (RES) {
      load_vec<DT, VEC>(res + o0, q0);
      load_vec<DT, VEC>(res + o1, q1);
    }
    if constexpr (RESAFF) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        q0[i] = __builtin_fmaf(q0[i], rc[i], rf[i]);
        q1[i] = __builtin_fmaf(q1[i], rc[i], rf[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float z0 = __builtin_fmaf(v0[i], sc[i], sf[i]), z1 = __builtin_fmaf(v1[i], sc[i], sf[i]);
      if constexpr (RES) {
        z0 += q0[i];
        z1 += q1[i];
      }
      v0[i] = act_fwd<ACT>(z0, slope);
      v1[i] = act_fwd<ACT>(z1, slope);
    }
    store_vec<DT, VEC>(y + o0, v0);
    store_vec<DT, VEC>(y + o1, v1);
    if constexpr (MASK) {
      uint32_t b0 = 0, b1 = 0;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        b0 |= (uint32_t)(v0[i] > 0.f) << i;
        b1 |= (uint32_t)(v1[i] > 0.f) << i;
      }
      mask[r * (C / 8) + grp] = (uint8_t)b0;
      mask[(r + g.rpp) * (C / 8) + grp] = (uint8_t)b1;
    }
  }
  if (r < r1) {
    const int64_t o0 = r * C + c0;
    float v0[VEC], q0[VEC];
    load_vec<DT, VEC>(x + o0, v0);
    if constexpr (RES) load_vec<DT, VEC>(res + o0, q0);
    if constexpr (RESAFF) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) q0[i] = __builtin_fmaf(q0[i], rc[i], rf[i]);
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float z0 = __builtin_fmaf(v0[i], sc[i], sf[i]);
      if constexpr (RES) z0 += q0[i];
      v0[i] = act_fwd<ACT>(z0, slope);
    }
    store_vec<DT, VEC>(y + o0, v0);
    if constexpr (MASK) {
      uint32_t b0 = 0;
#pragma unroll
      for (int i = 0; i < VEC; ++i) b0 |= (uint32_t)(v0[i] > 0.f) << i;
      mask[r * (C / 8) + grp] = (uint8_t)b0;
    }
  }
}

// ---------------------------------------------------------------------------
// backward partial sums: Σ dz and Σ dz * (x - mean), per workgroup.
// dz = dy * act'(z); the ReLU mask is recomputed from x (fma identical to the
// forward) unless a residual was added (then it comes from the saved output y);
// other activations recompute z from x (+ res).  Optionally writes dres = dz.
// MASKIN (RES + ReLU, VEC == 8): the ReLU mask comes from the forward's bit
// mask instead of y, and the residual gradient dy*mask is NOT written (its
// consumer applies the mask itself).
template <int DT, int VEC, int ACT, bool RES, bool MASKIN = false>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_partial_k(
    const storage_t<DT>* __restrict__ dy, const storage_t<DT>* __restrict__ y,
    const storage_t<DT>* __restrict__ x, const storage_t<DT>* __restrict__ res,
    const float* __restrict__ mean, const float* __restrict__ scale, const float* __restrict__ shift,
    int64_t M, int C, int64_t rows_per_blk, float slope, storage_t<DT>* __restrict__ dres,
    float* __restrict__ pdb, float* __restrict__ pdg, const uint8_t* __restrict__ maskin = nullptr) {
  const BnGeom g = bn_geom(C, VEC);
  {
    if constexpr (MASKIN) maskin += (int64_t)blockIdx.z * M * (C / 8);
    const int64_t zo = (int64_t)blockIdx.z * M * C;
    dy += zo;
    y += zo;
    x += zo;
    if constexpr (RES) {
      res += zo;
      dres += zo;
    }
    mean += (int64_t)blockIdx.z * C;
    scale += (int64_t)blockIdx.z * C;
    shift += (int64_t)blockIdx.z * C;
    pdb += (int64_t)blockIdx.z * gridDim.x * C;
    pdg += (int64_t)blockIdx.z * gridDim.x * C;
  }
  const int tid = threadIdx.x;
  const int gl = tid % g.GT, rl = tid / g.GT;
  const int grp = blockIdx.y * kGroupsPerTile + gl;
  const bool active = rl < g.rpp && gl < g.GT && grp < g.G;
  __shared__ float sm_a[kBnThreads * VEC];
  __shared__ float sm_b[kBnThreads * VEC];
  float sdb[VEC], sdg[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) sdb[i] = sdg[i] = 0.f;
  if (active) {
    const int c0 = grp * VEC;
    float mu[VEC], sc[VEC], sf[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      mu[i] = mean[c0 + i];
      sc[i] = scale[c0 + i];
      sf[i] = shift[c0 + i];
    }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
    int64_t r1 = r0 + rows_per_blk;
    if (r1 > M) r1 = M;
    for (int64_t r = r0 + rl; r < r1; r += g.rpp) {
      const int64_t off = r * C + c0;
      float vdy[VEC], vx[VEC], dz[VEC];
      load_vec<DT, VEC>(dy + off, vdy);
      load_vec<DT, VEC>(x + off, vx);
      if constexpr (MASKIN) {
        const uint32_t bits = maskin[r * (C / 8) + grp];
#pragma unroll
        for (int i = 0; i < VEC; ++i) dz[i] = (bits >> i) & 1u ? vdy[i] : 0.f;
      } else if constexpr (ACT == kActReLU && RES) {
        float vy[VEC];
        load_vec<DT, VEC>(y + off, vy);
#pragma unroll
        for (int i = 0; i < VEC; ++i) dz[i] = vy[i] > 0.f ? vdy[i] : 0.f;
      } else if constexpr (ACT == kActReLU) {
        // mask recomputed from x with the forward's exact fma: saves a read of y
#pragma unroll
        for (int i = 0; i < VEC; ++i) dz[i] = __builtin_fmaf(vx[i], sc[i], sf[i]) > 0.f ? vdy[i] : 0.f;
      } else if constexpr (ACT == kActNone) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) dz[i] = vdy[i];
      } else {
        float vr[VEC];
        if constexpr (RES) load_vec<DT, VEC>(res + off, vr);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          float z = __builtin_fmaf(vx[i], sc[i], sf[i]);
          if constexpr (RES) z += vr[i];
          dz[i] = vdy[i] * act_bwd<ACT>(z, slope);
        }
      }
      if constexpr (RES && !MASKIN) store_vec<DT, VEC>(dres + off, dz);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        sdb[i] += dz[i];
        sdg[i] += dz[i] * (vx[i] - mu[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    sm_a[tid * VEC + i] = sdb[i];
    sm_b[tid * VEC + i] = sdg[i];
  }
  __syncthreads();
  const int npairs = g.GT * VEC;
  for (int p = tid; p < npairs; p += kBnThreads) {
    const int pg = p / VEC, pe = p % VEC;
    const int cgrp = blockIdx.y * kGroupsPerTile + pg;
    if (cgrp >= g.G) continue;
    float ta = 0.f, tb = 0.f;
    for (int rr = 0; rr < g.rpp; ++rr) {
      const int t = rr * g.GT + pg;
      ta += sm_a[t * VEC + pe];
      tb += sm_b[t * VEC + pe];
    }
    const int c = cgrp * VEC + pe;
    pdb[(int64_t)blockIdx.x * C + c] = ta;
    pdg[(int64_t)blockIdx.x * C + c] = tb;
  }
}

// backward finalize: dbeta, dgamma and the dx coefficients  dx = a*dz + c0 + c1*x
struct BwdFin {
  int64_t M;
  const float *gamma, *mean, *invstd;
  int training;
  float *dgamma, *dbeta, *coef;
  int C;
  __device__ void operator()(int c, double a, double b) const {
    const double is = invstd[c];
    const double db = a;
    const double dg = b * is;
    if (dgamma) dgamma[c] = (float)dg;
    if (dbeta) dbeta[c] = (float)db;
    const double gm = gamma ? gamma[c] : 1.0;
    const double ka = gm * is;
    double c1 = 0.0, c0 = 0.0;
    if (training) {
      c1 = -ka * is * dg / (double)M;
      c0 = -ka * db / (double)M - c1 * (double)mean[c];
    }
    coef[c] = (float)ka;
    coef[C + c] = (float)c0;
    coef[2 * C + c] = (float)c1;
  }
};

// backward apply: dx = a*dz + c0 + c1*x (dz recomputed, or read from dres).
// Row-tiled; per-channel coefficients live in registers.
template <int DT, int VEC, int ACT, bool RES, bool DZ_GIVEN, bool MASKIN = false>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_apply_k(
    const storage_t<DT>* __restrict__ dy, const storage_t<DT>* __restrict__ y,
    const storage_t<DT>* __restrict__ x, const storage_t<DT>* __restrict__ res,
    const storage_t<DT>* __restrict__ dzin, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, int64_t M, int C,
    int64_t rows_per_blk, float slope, storage_t<DT>* __restrict__ dx,
    const uint8_t* __restrict__ maskin = nullptr, storage_t<DT>* __restrict__ dzout = nullptr, int rev = 0) {
  // dzout (MASKIN only): also write dz = dy * mask, the residual branch's gradient
  const BnGeom g = bn_geom(C, VEC);
  {
    if constexpr (MASKIN) maskin += (int64_t)blockIdx.z * M * (C / 8);
    const int64_t zo = (int64_t)blockIdx.z * M * C;
    dy += zo;
    y += zo;
    x += zo;
    dx += zo;
    if constexpr (RES) res += zo;
    if constexpr (DZ_GIVEN) dzin += zo;
    coef += (int64_t)blockIdx.z * 3 * C;
    scale += (int64_t)blockIdx.z * C;
    shift += (int64_t)blockIdx.z * C;
  }
  const int tid = threadIdx.x;
  const int gl = tid % g.GT, rl = tid / g.GT;
  const int grp = blockIdx.y * kGroupsPerTile + gl;
  if (rl >= g.rpp || grp >= g.G) return;
  const int c0 = grp * VEC;
  float ka[VEC], k0[VEC], k1[VEC], sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    ka[i] = coef[c0 + i];
    k0[i] = coef[C + c0 + i];
    k1[i] = coef[2 * C + c0 + i];
    if constexpr (!DZ_GIVEN && ACT != kActNone && !(ACT == kActReLU && RES)) {
      sc[i] = scale[c0 + i];
      sf[i] = shift[c0 + i];
    }
  }
  const int64_t r0 = (int64_t)(rev ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x) * rows_per_blk;
  int64_t r1 = r0 + rows_per_blk;
  if (r1 > M) r1 = M;
  for (int64_t r = r0 + rl; r < r1; r += g.rpp) {
    const int64_t e = r * C + c0;
    float vx[VEC], dz[VEC];
    load_vec<DT, VEC>(x + e, vx);
    if constexpr (MASKIN) {
      float vdy[VEC];
      load_vec<DT, VEC>(dy + e, vdy);
      const uint32_t bits = maskin[r * (C / 8) + grp];
#pragma unroll
      for (int k = 0; k < VEC; ++k) dz[k] = (bits >> k) & 1u ? vdy[k] : 0.f;
      if (dzout) store_vec<DT, VEC>(dzout + (int64_t)blockIdx.z * M * C + e, dz);
    } else if constexpr (DZ_GIVEN) {
      load_vec<DT, VEC>(dzin + e, dz);
    } else {
      float vdy[VEC];
      load_vec<DT, VEC>(dy + e, vdy);
      if constexpr (ACT == kActReLU && RES) {
        float vy[VEC];
        load_vec<DT, VEC>(y + e, vy);
#pragma unroll
        for (int k = 0; k < VEC; ++k) dz[k] = vy[k] > 0.f ? vdy[k] : 0.f;
      } else if constexpr (ACT == kActReLU) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) dz[k] = __builtin_fmaf(vx[k], sc[k], sf[k]) > 0.f ? vdy[k] : 0.f;
      } else if constexpr (ACT == kActNone) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) dz[k] = vdy[k];
      } else {
        float vr[VEC];
        if constexpr (RES) load_vec<DT, VEC>(res + e, vr);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          float z = __builtin_fmaf(vx[k], sc[k], sf[k]);
          if constexpr (RES) z += vr[k];
          dz[k] = vdy[k] * act_bwd<ACT>(z, slope);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) dz[k] = ka[k] * dz[k] + k0[k] + k1[k] * vx[k];
    store_vec<DT, VEC>(dx + e, dz);
  }
}

// The block-output BN's backward apply (ReLU after a residual add, saved mask bits) when the residual
// is a bottleneck's downsample branch: while forming dz = dy * mask it also accumulates that branch
// BN's backward partial sums (sum dz, sum dz * (xds - mean_ds)) -- dz is exactly the branch BN's
// output gradient -- into pds [gridDim.x][2][C] (fixed-order LDS reduction, deterministic).  The
// branch BN's backward then finalises from pds instead of re-reading (dy, xds) in a partial pass
// (ops/norm.py ResidualGradLink carrier).
template <int DT>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_apply_dsp_k(
    const storage_t<DT>* __restrict__ dy, const storage_t<DT>* __restrict__ x, const float* __restrict__ coef,
    int64_t M, int C, int64_t rows_per_blk, storage_t<DT>* __restrict__ dx, const uint8_t* __restrict__ maskin,
    const storage_t<DT>* __restrict__ xds, const float* __restrict__ mean_ds, float* __restrict__ pds) {
  constexpr int VEC = 8;
  const BnGeom g = bn_geom(C, VEC);
  const int tid = threadIdx.x;
  const int gl = tid % g.GT, rl = tid / g.GT;
  const int grp = blockIdx.y * kGroupsPerTile + gl;
  const bool active = rl < g.rpp && grp < g.G;
  __shared__ float sm_a[kBnThreads * VEC];
  __shared__ float sm_b[kBnThreads * VEC];
  float sdb[VEC], sdg[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) sdb[i] = sdg[i] = 0.f;
  if (active) {
    const int c0 = grp * VEC;
    float ka[VEC], k0[VEC], k1[VEC], mu[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      ka[i] = coef[c0 + i];
      k0[i] = coef[C + c0 + i];
      k1[i] = coef[2 * C + c0 + i];
      mu[i] = mean_ds[c0 + i];
    }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
    int64_t r1 = r0 + rows_per_blk;
    if (r1 > M) r1 = M;
    for (int64_t r = r0 + rl; r < r1; r += g.rpp) {
      const int64_t e = r * C + c0;
      float vx[VEC], vdy[VEC], vd[VEC], dz[VEC];
      load_vec<DT, VEC>(x + e, vx);
      load_vec<DT, VEC>(dy + e, vdy);
      load_vec<DT, VEC>(xds + e, vd);
      const uint32_t bits = maskin[r * (C / 8) + grp];
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        dz[k] = (bits >> k) & 1u ? vdy[k] : 0.f;
        sdb[k] += dz[k];
        sdg[k] += dz[k] * (vd[k] - mu[k]);
        dz[k] = ka[k] * dz[k] + k0[k] + k1[k] * vx[k];
      }
      store_vec<DT, VEC>(dx + e, dz);
    }
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    sm_a[tid * VEC + i] = sdb[i];
    sm_b[tid * VEC + i] = sdg[i];
  }
  __syncthreads();
  const int npairs = g.GT * VEC;
  for (int p = tid; p < npairs; p += kBnThreads) {
    const int pg = p / VEC, pe = p % VEC;
    const int cgrp = blockIdx.y * kGroupsPerTile + pg;
    if (cgrp >= g.G) continue;
    float ta = 0.f, tb = 0.f;
    for (int rr = 0; rr < g.rpp; ++rr) {
      const int t = rr * g.GT + pg;
      ta += sm_a[t * VEC + pe];
      tb += sm_b[t * VEC + pe];
    }
    const int c = cgrp * VEC + pe;
    pds[((int64_t)blockIdx.x * 2 + 0) * C + c] = ta;
    pds[((int64_t)blockIdx.x * 2 + 1) * C + c] = tb;
  }
}

// ---------------------------------------------------------------------------
// GroupNorm / InstanceNorm finalizers (per (sample, group) statistics).
// Partials are per channel (shifted by x[n, 0, c]); merged in f64 per group.
// One workgroup per (n, g).  Outputs are expanded per (n, c) so the streaming
// apply / backward kernels above serve both BN and GN.
__global__ __launch_bounds__(256) void gn_stats_finalize_k(
    const float* __restrict__ psum, const float* __restrict__ psq, const float* __restrict__ shift_src_f,
    int nblk, int64_t HW, int C, int G, const float* __restrict__ gamma, const float* __restrict__ beta,
    float eps, float* __restrict__ mean_out, float* __restrict__ invstd_out, float* __restrict__ scale_out,
    float* __restrict__ shift_out) {
  const int n = blockIdx.x / G, gi = blockIdx.x % G;
  const int Cg = C / G;
  const int c0 = gi * Cg;
  __shared__ double red[2][256];
  double sm = 0.0, sq = 0.0;
  // each thread: a subset of (channel, partial) pairs; converts shifted sums to raw moments
  for (int t = threadIdx.x; t < Cg * nblk; t += 256) {
    const int cc = c0 + t % Cg, b = t / Cg;
    const int64_t o = ((int64_t)n * nblk + b) * C + cc;
    const double S = psum[o], Q = psq[o];
    const double sh = shift_src_f[(int64_t)n * C + cc];
    // Σx = S + cnt*sh ; Σx² = Q + 2 sh S + cnt sh² ; cnt added once per channel below
    sm += S;
    sq += Q + 2.0 * sh * S;
  }
  // per-channel shift terms (cnt = HW rows per channel)
  for (int cc = threadIdx.x; cc < Cg; cc += 256) {
    const double sh = shift_src_f[(int64_t)n * C + c0 + cc];
    sm += (double)HW * sh;
    sq += (double)HW * sh * sh;
  }
  red[0][threadIdx.x] = sm;
  red[1][threadIdx.x] = sq;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  const double cnt = (double)HW * Cg;
  const double mean = red[0][0] / cnt;
  double var = red[1][0] / cnt - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int cc = threadIdx.x; cc < Cg; cc += 256) {
    const int c = c0 + cc;
    const int64_t o = (int64_t)n * C + c;
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    mean_out[o] = (float)mean;
    invstd_out[o] = invstd;
    scale_out[o] = gm * invstd;
    shift_out[o] = bt - (float)mean * gm * invstd;
  }
}

// backward: per (n, g) -> dx coefficients; per (n, c) -> dgamma/dbeta contributions
__global__ __launch_bounds__(256) void gn_bwd_finalize_k(
    const float* __restrict__ pdb, const float* __restrict__ pdg, int nblk, int64_t HW, int C, int G,
    const float* __restrict__ gamma, const float* __restrict__ mean_e, const float* __restrict__ invstd_e,
    float* __restrict__ coef, float* __restrict__ dg_nc, float* __restrict__ db_nc) {
  const int n = blockIdx.x / G, gi = blockIdx.x % G;
  const int Cg = C / G;
  const int c0 = gi * Cg;
  __shared__ double red[2][256];
  const double is = invstd_e[(int64_t)n * C + c0];
  const double mu = mean_e[(int64_t)n * C + c0];
  double s1 = 0.0, s2 = 0.0;
  for (int cc = threadIdx.x; cc < Cg; cc += 256) {
    const int c = c0 + cc;
    double A = 0.0, Bv = 0.0;
    for (int b = 0; b < nblk; ++b) {
      const int64_t o = ((int64_t)n * nblk + b) * C + c;
      A += pdb[o];
      Bv += pdg[o];
    }
    const double gm = gamma ? gamma[c] : 1.0;
    s1 += gm * A;
    s2 += gm * Bv * is;
    db_nc[(int64_t)n * C + c] = (float)A;
    dg_nc[(int64_t)n * C + c] = (float)(Bv * is);
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  const double cnt = (double)HW * Cg;
  const double S1 = red[0][0], S2 = red[1][0];
  const double k1 = -is * is * S2 / cnt;
  const double k0 = -is * S1 / cnt - k1 * mu;
  for (int cc = threadIdx.x; cc < Cg; cc += 256) {
    const int c = c0 + cc;
    const double gm = gamma ? gamma[c] : 1.0;
    float* cf = coef + (int64_t)n * 3 * C;
    cf[c] = (float)(is * gm);
    cf[C + c] = (float)k0;
    cf[2 * C + c] = (float)k1;
  }
}

__global__ void sum_over_samples_k(const float* __restrict__ v, int N, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C || !out) return;
  double s = 0.0;
  for (int n = 0; n < N; ++n) s += v[(int64_t)n * C + c];
  out[c] = (float)s;
}

// first-row values as f32 (the per-channel shift of each sample's partial sums)
template <int DT>
__global__ void gather_row0_k(const storage_t<DT>* __restrict__ x, int64_t HW, int C, int N,
                              float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * C) return;
  const int64_t n = i / C, c = i % C;
  out[i] = Elem<DT>::ld(x, n * HW * C + c);
}

// ---------------------------------------------------------------------------
// host launchers

static int bn_nblk(int64_t M, int C, int VEC, int ytiles, int S) {
  // ~2 workgroups per CU in total, but at least 4 passes of rows each
  const BnGeom g = bn_geom(C, VEC);
  int64_t target = 512 / ((int64_t)ytiles * S);
  if (target < 1) target = 1;
  int64_t max_blk = (M + g.rpp * 4 - 1) / (g.rpp * 4);
  if (max_blk < 1) max_blk = 1;
  return (int)(target < max_blk ? target : max_blk);
}

int bn_partial_blocks(int64_t M, int C) { return norm_partial_blocks(M, C, 1); }

int norm_partial_blocks(int64_t M, int C, int S) {
  const int VEC = (C % 8 == 0) ? 8 : 1;
  const BnGeom g = bn_geom(C, VEC);
  const int ytiles = cdiv(g.G, kGroupsPerTile);
  return bn_nblk(M, C, VEC, ytiles, S);
}

// elementwise passes: up to `g_apply_wg` workgroups in total, each at least `g_apply_minpass` row
// passes -- many short-lived workgroups.  A 2-read / 1-write bf16 stream runs 5.1 TB/s as 2048
// long-lived chunked workgroups and 6.0 TB/s as a full grid of one-vector threads
// (scripts/tools/membw_probe.hip).  16384 vs 2048: ResNet-50 +1.7 %, ResNet-101 +3 %; the uncapped
// grid (131072) gave ResNet-50 the same but cost ResNet-101 3-6 % (profiles/r06_bnwg/).  With the
// last-written-first order (g_bn_rev) 32768 beats 16384 by +0.2 % on ResNet-50 in 6 of 7 pairs
// (profiles/r06_bnwg/cap32k_ab.txt).
// TBAMD_BN_APPLY_WG / _MINPASS: A/B runs.
static const int g_apply_wg = [] {
  const char* e = getenv("TBAMD_BN_APPLY_WG");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : 32768;
}();
static const int g_apply_minpass = [] {
  const char* e = getenv("TBAMD_BN_APPLY_MINPASS");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : 2;
}();
// the apply passes walk their rows last-written-first: the first-dispatched workgroups take the rows
// the producing kernel stored LAST, which are the lines still in the memory-side cache (a 411 MB
// stage-1 tensor does not fit; its tail does).  +0.2-1.0 % on ResNet-50 in 6 of 6 alternated pairs,
// +1-7 % on ResNet-101 (profiles/r06_bnwg/reverse_ab.txt).  TBAMD_BN_REVERSE=0: first-row-first.
static const int g_bn_rev = [] {
  const char* e = getenv("TBAMD_BN_REVERSE");
  return e && e[0] == '0' ? 0 : 1;
}();
static int bn_apply_blocks(int64_t M, int C, int VEC, int ytiles, int S) {
  const BnGeom g = bn_geom(C, VEC);
  int64_t target = g_apply_wg / ((int64_t)ytiles * S);
  if (target < 1) target = 1;
  const int64_t rows_min = (int64_t)g.rpp * g_apply_minpass;
  int64_t max_blk = (M + rows_min - 1) / rows_min;
  if (max_blk < 1) max_blk = 1;
  return (int)(target < max_blk ? target : max_blk);
}

// the downsample-partials apply keeps ~8 workgroups per CU: each workgroup also writes a partial row
static int bn_dsp_blocks(int64_t M, int C, int ytiles) {
  const BnGeom g = bn_geom(C, 8);
  int64_t target = 2048 / (int64_t)ytiles;
  if (target < 1) target = 1;
  int64_t max_blk = (M + g.rpp * 2 - 1) / (g.rpp * 2);
  if (max_blk < 1) max_blk = 1;
  return (int)(target < max_blk ? target : max_blk);
}

template <int DT>
static void launch_stats_partial(const void* x, int S, int64_t M, int C, int nblk, float* psum, float* psq,
                                 hipStream_t st) {
  using T = storage_t<DT>;
  const bool vec = (C % 8 == 0);
  const BnGeom g = bn_geom(C, vec ? 8 : 1);
  dim3 grid(nblk, cdiv(g.G, kGroupsPerTile), S);
  const int64_t rpb = (M + nblk - 1) / nblk;
  if (vec)
    bn_stats_partial_k<DT, 8><<<grid, kBnThreads, 0, st>>>((const T*)x, M, C, rpb, psum, psq);
  else
    bn_stats_partial_k<DT, 1><<<grid, kBnThreads, 0, st>>>((const T*)x, M, C, rpb, psum, psq);
}

void bn_forward_train(int dt, const void* x, int64_t M, int C, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                      float* psum, float* psq, int nblk, double* fin_ws, float* mean, float* invstd, float* scale,
                      float* shift, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    using T = storage_t<DT>;
    launch_stats_partial<DT>(x, 1, M, C, nblk, psum, psq, st);
    StatsFin<DT> fin{M, (const T*)x, gamma, beta, running_mean, running_var, nbt, momentum, eps,
                     mean, invstd, scale, shift};
    launch_colsum_fin(psum, psq, C, nblk, C, fin_ws, fin, st);
  });
}

void bn_finalize_from_conv(const float* part, int nblk, int64_t M, int C, const float* gamma, const float* beta,
                           float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                           double* fin_ws, float* mean, float* invstd, float* scale, float* shift, hipStream_t st) {
  // conv epilogue partials: [nblk][2][C] raw sums of the bf16 outputs
  StatsFin<kF32> fin{M, nullptr, gamma, beta, running_mean, running_var, nbt, momentum, eps,
                     mean, invstd, scale, shift};
  launch_colsum_fin(part, part + C, 2 * (int64_t)C, nblk, C, fin_ws, fin, st);
}

void gn_forward_stats(int dt, const void* x, int N, int64_t HW, int C, int G, const float* gamma,
                      const float* beta, float eps, float* psum, float* psq, float* row0, int nblk, float* mean,
                      float* invstd, float* scale, float* shift, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    using T = storage_t<DT>;
    launch_stats_partial<DT>(x, N, HW, C, nblk, psum, psq, st);
    gather_row0_k<DT><<<cdiv((int64_t)N * C, 256), 256, 0, st>>>((const T*)x, HW, C, N, row0);
    gn_stats_finalize_k<<<N * G, 256, 0, st>>>(psum, psq, row0, nblk, HW, C, G, gamma, beta, eps, mean,
                                               invstd, scale, shift);
  });
}

void bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                    float eps, float* mean, float* invstd, float* scale, float* shift, hipStream_t st) {
  bn_eval_coeffs_k<<<cdiv(C, 256), 256, 0, st>>>(C, gamma, beta, rm, rv, eps, mean, invstd, scale, shift);
}

template <int DT, int ACT>
static void bn_apply_t(const void* x, const void* res, const float* scale, const float* shift, int S,
                       int64_t M, int C, float slope, void* y, uint8_t* mask, hipStream_t st,
                       const float* rsc = nullptr, const float* rsh = nullptr) {
  using T = storage_t<DT>;
  const bool vec = (C % 8 == 0);
  const int VECv = vec ? 8 : 1;
  const BnGeom g = bn_geom(C, VECv);
  const int ytiles = cdiv(g.G, kGroupsPerTile);
  const int nblk = bn_apply_blocks(M, C, VECv, ytiles, S);
  const int64_t rpb = (M + nblk - 1) / nblk;
  dim3 grid(nblk, ytiles, S);
  if (rsc) {  // affine residual (ReLU after the add, mask kept: the bottleneck output BN)
    if constexpr (ACT == kActReLU) {
      if (mask && vec && res) {
        bn_apply_k<DT, 8, ACT, true, true, true><<<grid, kBnThreads, 0, st>>>(
            (const T*)x, (const T*)res, scale, shift, M, C, rpb, slope, (T*)y, mask, rsc, rsh, g_bn_rev);
        return;
      }
    }
    throw std::runtime_error("bn_apply: an affine residual needs ReLU, a mask, C % 8 == 0");
  }
  if constexpr (ACT == kActReLU) {
    if (mask && vec && res) {
      bn_apply_k<DT, 8, ACT, true, true><<<grid, kBnThreads, 0, st>>>((const T*)x, (const T*)res, scale, shift, M,
                                                                    C, rpb, slope, (T*)y, mask, nullptr, nullptr,
                                                                    g_bn_rev);
      return;
    }
  }
  if (vec) {
    if (res)
      bn_apply_k<DT, 8, ACT, true><<<grid, kBnThreads, 0, st>>>((const T*)x, (const T*)res, scale, shift, M, C,
                                                              rpb, slope, (T*)y, nullptr, nullptr, nullptr, g_bn_rev);
    else
      bn_apply_k<DT, 8, ACT, false><<<grid, kBnThreads, 0, st>>>((const T*)x, nullptr, scale, shift, M, C, rpb,
                                                               slope, (T*)y, nullptr, nullptr, nullptr, g_bn_rev);
  } else {
    if (res)
      bn_apply_k<DT, 1, ACT, true><<<grid, kBnThreads, 0, st>>>((const T*)x, (const T*)res, scale, shift, M, C,
                                                              rpb, slope, (T*)y);
    else
      bn_apply_k<DT, 1, ACT, false><<<grid, kBnThreads, 0, st>>>((const T*)x, nullptr, scale, shift, M, C, rpb,
                                                               slope, (T*)y);
  }
}

void bn_apply(int dt, const void* x, const void* res, const float* scale, const float* shift, int64_t M,
              int C, int act, float slope, void* y, uint8_t* mask, hipStream_t st, const float* rsc,
              const float* rsh) {
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, {
      bn_apply_t<DT, ACT>(x, res, scale, shift, 1, M, C, slope, y, mask, st, rsc, rsh);
    });
  });
}

void norm_apply(int dt, const void* x, const void* res, const float* scale, const float* shift, int S,
                int64_t M, int C, int act, float slope, void* y, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, { bn_apply_t<DT, ACT>(x, res, scale, shift, S, M, C, slope, y, nullptr, st); });
  });
}

template <int DT, int ACT>
static void launch_bwd_partial(const void* dy, const void* y, const void* x, const void* res, int S, int64_t M,
                               int C, float slope, const float* mean, const float* scale, const float* shift,
                               int nblk, float* pdb, float* pdg, void* dres, const uint8_t* maskin,
                               hipStream_t st) {
  using T = storage_t<DT>;
  const bool vec = (C % 8 == 0);
  const BnGeom g = bn_geom(C, vec ? 8 : 1);
  dim3 grid(nblk, cdiv(g.G, kGroupsPerTile), S);
  const int64_t rpb = (M + nblk - 1) / nblk;
  const T *tdy = (const T*)dy, *ty = (const T*)y, *tx = (const T*)x, *tres = (const T*)res;
  // (ACT none + maskin: dy is the unmasked gradient of a residual whose ReLU mask lives downstream)
  if constexpr (ACT == kActReLU || ACT == kActNone) {
    if (maskin && vec) {
      bn_bwd_partial_k<DT, 8, ACT, true, true><<<grid, kBnThreads, 0, st>>>(
          tdy, ty, tx, tres, mean, scale, shift, M, C, rpb, slope, nullptr, pdb, pdg, maskin);
      return;
    }
  }
  if (vec) {
    if (dres)
      bn_bwd_partial_k<DT, 8, ACT, true><<<grid, kBnThreads, 0, st>>>(tdy, ty, tx, tres, mean, scale, shift, M, C,
                                                                     rpb, slope, (T*)dres, pdb, pdg);
    else
      bn_bwd_partial_k<DT, 8, ACT, false><<<grid, kBnThreads, 0, st>>>(tdy, ty, tx, tres, mean, scale, shift, M, C,
                                                                      rpb, slope, nullptr, pdb, pdg);
  } else {
    if (dres)
      bn_bwd_partial_k<DT, 1, ACT, true><<<grid, kBnThreads, 0, st>>>(tdy, ty, tx, tres, mean, scale, shift, M, C,
                                                                     rpb, slope, (T*)dres, pdb, pdg);
    else
      bn_bwd_partial_k<DT, 1, ACT, false><<<grid, kBnThreads, 0, st>>>(tdy, ty, tx, tres, mean, scale, shift, M, C,
                                                                      rpb, slope, nullptr, pdb, pdg);
  }
}

template <int DT, int ACT>
static void launch_bwd_apply(const void* dy, const void* y, const void* x, const void* res, const void* dres,
                             int S, int64_t M, int C, float slope, const float* scale, const float* shift,
                             const float* coef, void* dx, const uint8_t* maskin, hipStream_t st,
                             void* dzout = nullptr) {
  using T = storage_t<DT>;
  const bool vec = (C % 8 == 0);
  const int VECv = vec ? 8 : 1;
  const BnGeom g = bn_geom(C, VECv);
  const int ytiles = cdiv(g.G, kGroupsPerTile);
  const int nab = bn_apply_blocks(M, C, VECv, ytiles, S);
  const int64_t rpb = (M + nab - 1) / nab;
  dim3 agrid(nab, ytiles, S);
  const T *tdy = (const T*)dy, *ty = (const T*)y, *tx = (const T*)x, *tres = (const T*)res;
  if constexpr (ACT == kActReLU || ACT == kActNone) {
    if (maskin && vec) {
      tb_launch_ev(bn_bwd_apply_k<DT, 8, ACT, true, false, true>, agrid, dim3(kBnThreads), 0, st,
                   tdy, ty, tx, tres, nullptr, scale, shift, coef, M, C, rpb, slope, (T*)dx, maskin, (T*)dzout,
                   g_bn_rev);
      return;
    }
  }
  if (vec) {
    if (dres)
      tb_launch_ev(bn_bwd_apply_k<DT, 8, ACT, true, true>, agrid, dim3(kBnThreads), 0, st,
                   tdy, ty, tx, tres, (const T*)dres, scale, shift, coef, M, C, rpb, slope, (T*)dx, nullptr, nullptr,
                   g_bn_rev);
    else
      tb_launch_ev(bn_bwd_apply_k<DT, 8, ACT, false, false>, agrid, dim3(kBnThreads), 0, st,
                   tdy, ty, tx, tres, nullptr, scale, shift, coef, M, C, rpb, slope, (T*)dx, nullptr, nullptr,
                   g_bn_rev);
  } else {
    if (dres)
      tb_launch_ev(bn_bwd_apply_k<DT, 1, ACT, true, true>, agrid, dim3(kBnThreads), 0, st,
                   tdy, ty, tx, tres, (const T*)dres, scale, shift, coef, M, C, rpb, slope, (T*)dx, nullptr, nullptr, 0);
    else
      tb_launch_ev(bn_bwd_apply_k<DT, 1, ACT, false, false>, agrid, dim3(kBnThreads), 0, st,
                   tdy, ty, tx, tres, nullptr, scale, shift, coef, M, C, rpb, slope, (T*)dx, nullptr, nullptr, 0);
  }
}

void bn_backward(int dt, const void* dy, const void* y, const void* x, const void* res, int64_t M, int C,
                 int act, float slope, const float* gamma, const float* mean, const float* invstd,
                 const float* scale, const float* shift, int training, float* pdb, float* pdg, int nblk,
                 double* fin_ws, float* coef, float* dgamma, float* dbeta, void* dres, void* dx,
                 const uint8_t* maskin, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, {
      launch_bwd_partial<DT, ACT>(dy, y, x, res, 1, M, C, slope, mean, scale, shift, nblk, pdb, pdg,
                                  maskin ? nullptr : dres, maskin, st);
      BwdFin fin{M, gamma, mean, invstd, training, dgamma, dbeta, coef, C};
      launch_colsum_fin(pdb, pdg, C, nblk, C, fin_ws, fin, st);
      launch_bwd_apply<DT, ACT>(dy, y, x, res, maskin ? nullptr : dres, 1, M, C, slope, scale, shift, coef, dx,
                                maskin, st);
    });
  });
}

// ---------------------------------------------------------------------------
// BN backward of maxpool3x3/2/pad1(act(BN(x))) (the ResNet stem) straight from the POOLED
// gradient.  A thread owns a 2 x 2 input-pixel block x 8 channels: the only windows covering it
// are (m, j), (m, j+1), (m+1, j), (m+1, j+1) of the pooled grid, so 4 argmax + 4 gradient loads
// give the pool-input gradient dA of all 4 pixels (a per-pixel gather reads 9 window slots for
// the same 4 pixels), and the full-resolution dA is never written or read back.  Taps (r*3 + u):
//   (2m, 2j) <- (m,j):4      (2m, 2j+1) <- (m,j):5 + (m,j+1):3
//   (2m+1, 2j) <- (m,j):7 + (m+1,j):1      (2m+1, 2j+1) <- (m,j):8 + (m,j+1):6 + (m+1,j):2 + (m+1,j+1):0
// H, W even (P = H/2, Q = W/2); 256 / (C/8) blocks in flight per workgroup.
struct StemPoolGeom {
  int N, H, W, C, G, lanes;  // G = C / 8 channel groups; lanes = kBnThreads / G
  int64_t blocks;            // N * (H/2) * (W/2)
  int64_t per_wg;            // blocks per workgroup
};

template <int DT>
__device__ __forceinline__ void stem_pool_da(const storage_t<DT>* __restrict__ dyp, const uint8_t* __restrict__ idx,
                                             const StemPoolGeom& g, int64_t b, int c0, float da[4][8],
                                             int64_t& xo) {
  const int Q = g.W >> 1, P = g.H >> 1;
  const int j = (int)(b % Q);
  const int64_t t = b / Q;
  const int m = (int)(t % P);
  const int n = (int)(t / P);
  xo = (((int64_t)n * g.H + 2 * m) * g.W + 2 * j) * g.C + c0;  // pixel (2m, 2j)
  const bool okq = j + 1 < Q, okp = m + 1 < P;
  const int64_t o00 = (((int64_t)n * P + m) * Q + j) * g.C + c0;
  const int64_t o01 = okq ? o00 + g.C : o00;
  const int64_t o10 = okp ? o00 + (int64_t)Q * g.C : o00;
  const int64_t o11 = okp && okq ? o00 + (int64_t)(Q + 1) * g.C : o00;
  const uint2 i00 = *reinterpret_cast<const uint2*>(idx + o00), i01 = *reinterpret_cast<const uint2*>(idx + o01);
  const uint2 i10 = *reinterpret_cast<const uint2*>(idx + o10), i11 = *reinterpret_cast<const uint2*>(idx + o11);
  float v00[8], v01[8], v10[8], v11[8];
  load_vec<DT, 8>(dyp + o00, v00);
  load_vec<DT, 8>(dyp + o01, v01);
  load_vec<DT, 8>(dyp + o10, v10);
  load_vec<DT, 8>(dyp + o11, v11);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int sh = 8 * (i & 3);
    const uint32_t a00 = ((i < 4 ? i00.x : i00.y) >> sh) & 0xffu;
    const uint32_t a01 = okq ? ((i < 4 ? i01.x : i01.y) >> sh) & 0xffu : 0xffu;
    const uint32_t a10 = okp ? ((i < 4 ? i10.x : i10.y) >> sh) & 0xffu : 0xffu;
    const uint32_t a11 = okp && okq ? ((i < 4 ? i11.x : i11.y) >> sh) & 0xffu : 0xffu;
    da[0][i] = a00 == 4u ? v00[i] : 0.f;
    da[1][i] = (a00 == 5u ? v00[i] : 0.f) + (a01 == 3u ? v01[i] : 0.f);
    da[2][i] = (a00 == 7u ? v00[i] : 0.f) + (a10 == 1u ? v10[i] : 0.f);
    da[3][i] = ((a00 == 8u ? v00[i] : 0.f) + (a01 == 6u ? v01[i] : 0.f)) +
               ((a10 == 2u ? v10[i] : 0.f) + (a11 == 0u ? v11[i] : 0.f));
  }
}

template <int DT, int ACT>
__global__ __launch_bounds__(kBnThreads) void stem_pool_bn_bwd_partial_k(
    const storage_t<DT>* __restrict__ dyp, const uint8_t* __restrict__ idx, const storage_t<DT>* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ scale, const float* __restrict__ shift, StemPoolGeom g,
    float slope, float* __restrict__ pdb, float* __restrict__ pdg) {
  const int tid = threadIdx.x, gq = tid % g.G, bl = tid / g.G;
  const int c0 = gq * 8;
  float mu[8], sc[8], sf[8], sdb[8], sdg[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = mean[c0 + i];
    sc[i] = scale[c0 + i];
    sf[i] = shift[c0 + i];
    sdb[i] = sdg[i] = 0.f;
  }
  const int64_t b0 = (int64_t)blockIdx.x * g.per_wg;
  const int64_t b1 = min(b0 + g.per_wg, g.blocks);
  if (bl < g.lanes) {
    for (int64_t b = b0 + bl; b < b1; b += g.lanes) {
      float da[4][8];
      int64_t xo;
      stem_pool_da<DT>(dyp, idx, g, b, c0, da, xo);
      float vx[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) load_vec<DT, 8>(x + xo + ((q >> 1) * (int64_t)g.W + (q & 1)) * g.C, vx[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float z = __builtin_fmaf(vx[q][i], sc[i], sf[i]);
          float dz;
          if constexpr (ACT == kActReLU) dz = z > 0.f ? da[q][i] : 0.f;
          else dz = da[q][i] * act_bwd<ACT>(z, slope);
          sdb[i] += dz;
          sdg[i] += dz * (vx[q][i] - mu[i]);
        }
    }
  }
  // [lane][C] layout (tid * 8 + i = bl * C + c0 + i): 16-B stores, channel-consecutive reads
  __shared__ float4 sm_a[kBnThreads * 2];
  __shared__ float4 sm_b[kBnThreads * 2];
  sm_a[2 * tid] = make_float4(sdb[0], sdb[1], sdb[2], sdb[3]);
  sm_a[2 * tid + 1] = make_float4(sdb[4], sdb[5], sdb[6], sdb[7]);
  sm_b[2 * tid] = make_float4(sdg[0], sdg[1], sdg[2], sdg[3]);
  sm_b[2 * tid + 1] = make_float4(sdg[4], sdg[5], sdg[6], sdg[7]);
  __syncthreads();
  const float* fa = reinterpret_cast<const float*>(sm_a);
  const float* fb = reinterpret_cast<const float*>(sm_b);
  for (int p = tid; p < g.C; p += kBnThreads) {
    float ta = 0.f, tb = 0.f;
    for (int l = 0; l < g.lanes; ++l) {
      ta += fa[l * g.C + p];
      tb += fb[l * g.C + p];
    }
    pdb[(int64_t)blockIdx.x * g.C + p] = ta;
    pdg[(int64_t)blockIdx.x * g.C + p] = tb;
  }
}

template <int DT, int ACT>
__global__ __launch_bounds__(kBnThreads) void stem_pool_bn_bwd_apply_k(
    const storage_t<DT>* __restrict__ dyp, const uint8_t* __restrict__ idx, const storage_t<DT>* __restrict__ x,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ coef, StemPoolGeom g,
    float slope, storage_t<DT>* __restrict__ dx) {
  const int tid = threadIdx.x, gq = tid % g.G, bl = tid / g.G;
  if (bl >= g.lanes) return;
  const int c0 = gq * 8;
  float ka[8], k0[8], k1[8], sc[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ka[i] = coef[c0 + i];
    k0[i] = coef[g.C + c0 + i];
    k1[i] = coef[2 * g.C + c0 + i];
    sc[i] = scale[c0 + i];
    sf[i] = shift[c0 + i];
  }
  const int64_t b0 = (int64_t)blockIdx.x * g.per_wg;
  const int64_t b1 = min(b0 + g.per_wg, g.blocks);
  for (int64_t b = b0 + bl; b < b1; b += g.lanes) {
    float da[4][8];
    int64_t xo;
    stem_pool_da<DT>(dyp, idx, g, b, c0, da, xo);
    float vx[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) load_vec<DT, 8>(x + xo + ((q >> 1) * (int64_t)g.W + (q & 1)) * g.C, vx[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float z = __builtin_fmaf(vx[q][i], sc[i], sf[i]);
        float dz;
        if constexpr (ACT == kActReLU) dz = z > 0.f ? da[q][i] : 0.f;
        else dz = da[q][i] * act_bwd<ACT>(z, slope);
        o[i] = ka[i] * dz + k0[i] + k1[i] * vx[q][i];
      }
      store_vec<DT, 8>(dx + xo + ((q >> 1) * (int64_t)g.W + (q & 1)) * g.C, o);
    }
  }
}

// whether bn_backward_pool takes this shape (else: the gather kernel + bn_backward)
bool bn_backward_pool_ok(int H, int W, int C, int k, int s, int pad) {
  const int G = C / 8;
  return k == 3 && s == 2 && pad == 1 && H % 2 == 0 && W % 2 == 0 && C % 8 == 0 && G <= kBnThreads &&
         kBnThreads % G == 0;
}

int bn_backward_pool_blocks(int N, int H, int W, int C) {
  const int64_t blocks = (int64_t)N * (H / 2) * (W / 2);
  const int lanes = kBnThreads / (C / 8);
  // ~4 passes of the workgroup's lanes per workgroup, at most 2048 workgroups (the partial rows)
  int64_t nwg = (blocks + 4 * lanes - 1) / (4 * lanes);
  return (int)std::max<int64_t>(1, std::min<int64_t>(nwg, 2048));
}

void bn_backward_pool(int dt, const void* dyp, const uint8_t* idx, const void* x, int N, int H, int W, int C, int k,
                      int s, int pad, int act, float slope, const float* gamma, const float* mean,
                      const float* invstd, const float* scale, const float* shift, int training, float* pdb,
                      float* pdg, int nblk, double* fin_ws, float* coef, float* dgamma, float* dbeta, void* dx,
                      hipStream_t st) {
  (void)k; (void)s; (void)pad;  // (bn_backward_pool_ok: 3x3/2, pad 1)
  StemPoolGeom g{N, H, W, C, C / 8, kBnThreads / (C / 8), (int64_t)N * (H / 2) * (W / 2), 0};
  g.per_wg = (g.blocks + nblk - 1) / nblk;
  const int64_t M = (int64_t)N * H * W;
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, {
      using T = storage_t<DT>;
      stem_pool_bn_bwd_partial_k<DT, ACT><<<nblk, kBnThreads, 0, st>>>((const T*)dyp, idx, (const T*)x, mean, scale,
                                                                       shift, g, slope, pdb, pdg);
      BwdFin fin{M, gamma, mean, invstd, training, dgamma, dbeta, coef, C};
      launch_colsum_fin(pdb, pdg, C, nblk, C, fin_ws, fin, st);
      StemPoolGeom ga = g;
      const int64_t nab = std::min<int64_t>((g.blocks + g.lanes - 1) / g.lanes, 8192);
      ga.per_wg = (g.blocks + nab - 1) / nab;
      tb_launch_ev(stem_pool_bn_bwd_apply_k<DT, ACT>, dim3((unsigned)nab), dim3(kBnThreads), 0, st, (const T*)dyp,
                   idx, (const T*)x, scale, shift, (const float*)coef, ga, slope, (T*)dx);
    });
  });
}

// BN backward when the partial sums came from the dgrad epilogue that produced
// dy (conv.hip BNB): part [nrows][2][C] = (sum dz, sum dz*(x-mean))
// rows of the downsample-branch partials bn_backward_from_partials writes (its apply grid's x extent)
int bn_bwd_dsp_rows(int64_t M, int C) {
  const BnGeom g = bn_geom(C, 8);
  return bn_dsp_blocks(M, C, cdiv(g.G, kGroupsPerTile));
}

void bn_backward_from_partials(int dt, const void* dy, const void* y, const void* x, int64_t M, int C, int act,
                               float slope, const float* gamma, const float* mean, const float* invstd,
                               const float* scale, const float* shift, int training, const float* part, int nrows,
                               double* fin_ws, float* coef, float* dgamma, float* dbeta, void* dx,
                               const uint8_t* maskin, hipStream_t st, void* dres, const void* xds,
                               const float* mean_ds, float* pds) {
  BwdFin fin{M, gamma, mean, invstd, training, dgamma, dbeta, coef, C};
  launch_colsum_fin(part, part + C, 2 * (int64_t)C, nrows, C, fin_ws, fin, st);
  if (xds) {  // ReLU-after-residual with mask bits, the residual a downsample branch (see the kernel)
    if (!(maskin && act == kActReLU && C % 8 == 0 && !dres))
      throw std::runtime_error("bn_backward_from_partials: downsample partials need the ReLU mask, C % 8 == 0");
    const BnGeom g = bn_geom(C, 8);
    const int ytiles = cdiv(g.G, kGroupsPerTile);
    const int nab = bn_dsp_blocks(M, C, ytiles);
    const int64_t rpb = (M + nab - 1) / nab;
    TBAMD_DISPATCH_DT(dt, DT, {
      using T = storage_t<DT>;
      tb_launch_ev(bn_bwd_apply_dsp_k<DT>, dim3(nab, ytiles, 1), dim3(kBnThreads), 0, st, (const T*)dy,
                   (const T*)x, (const float*)coef, M, C, rpb, (T*)dx, maskin, (const T*)xds, mean_ds, pds);
    });
    return;
  }
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, {
      launch_bwd_apply<DT, ACT>(dy, y, x, nullptr, nullptr, 1, M, C, slope, scale, shift, coef, dx, maskin, st,
                                dres);
    });
  });
}

// deferred BN backward (conv.hip GXF): the finalize alone -- dgamma, dbeta and the dx coefficients
// [3][C] -- from the consumer dgrad's partial sums; the apply then runs in the next conv's dgrad
// operand staging (or bn_backward_apply_coef when that conv cannot take it)
void bn_backward_coef(const float* part, int nrows, int64_t M, int C, const float* gamma, const float* mean,
                      const float* invstd, int training, double* fin_ws, float* coef, float* dgamma, float* dbeta,
                      hipStream_t st) {
  BwdFin fin{M, gamma, mean, invstd, training, dgamma, dbeta, coef, C};
  launch_colsum_fin(part, part + C, 2 * (int64_t)C, nrows, C, fin_ws, fin, st);
}

void bn_backward_apply_coef(int dt, const void* dy, const void* x, int64_t M, int C, int act, float slope,
                            const float* scale, const float* shift, const float* coef, void* dx,
                            const uint8_t* maskin, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, {
      launch_bwd_apply<DT, ACT>(dy, x, x, nullptr, nullptr, 1, M, C, slope, scale, shift, coef, dx, maskin, st);
    });
  });
}

void gn_backward(int dt, const void* dy, const void* y, const void* x, const void* res, int N, int64_t HW, int C,
                 int G, int act, float slope, const float* gamma, const float* mean, const float* invstd,
                 const float* scale, const float* shift, float* pdb, float* pdg, int nblk, float* coef,
                 float* dg_nc, float* db_nc, float* dgamma, float* dbeta, void* dres, void* dx, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DT, {
    TBAMD_DISPATCH_ACT(act, ACT, {
      launch_bwd_partial<DT, ACT>(dy, y, x, res, N, HW, C, slope, mean, scale, shift, nblk, pdb, pdg, dres, nullptr,
                                  st);
      gn_bwd_finalize_k<<<N * G, 256, 0, st>>>(pdb, pdg, nblk, HW, C, G, gamma, mean, invstd, coef, dg_nc, db_nc);
      sum_over_samples_k<<<cdiv(C, 256), 256, 0, st>>>(dg_nc, N, C, dgamma);
      sum_over_samples_k<<<cdiv(C, 256), 256, 0, st>>>(db_nc, N, C, dbeta);
      launch_bwd_apply<DT, ACT>(dy, y, x, res, dres, N, HW, C, slope, scale, shift, coef, dx, nullptr, st);
    });
  });
}

// ---------------------------------------------------------------------------
// completion-event pool for the side-stream hand-off (tb_launch_ev): events are created once
// (timing disabled) and cycled; a wait captures an event's state when it is enqueued, so an
// event may be re-armed as soon as its wait was issued
namespace {
constexpr int kStopEvents = 64;
hipEvent_t g_stop_events[kStopEvents];
int64_t g_stop_next = 0;
}  // namespace

int64_t stop_event_arm() {
  const int64_t id = g_stop_next++ % kStopEvents;
  if (!g_stop_events[id]) (void)hipEventCreateWithFlags(&g_stop_events[id], hipEventDisableTiming);
  armed_stop_event() = g_stop_events[id];
  return id;
}

bool stop_event_disarm() {
  const bool fired = armed_stop_event() == nullptr;
  armed_stop_event() = nullptr;
  return fired;
}

void stream_wait_stop_event(hipStream_t st, int64_t id) {
  (void)hipStreamWaitEvent(st, g_stop_events[id % kStopEvents], 0);
}

}  // namespace tbamd
