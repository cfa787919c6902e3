// Row LayerNorm (+ optional residual add producing the new residual stream)
// for gfx950: one wave per row, the row held in registers (two-pass exact
// variance), 16-B vector loads; backward reduces dgamma/dbeta per workgroup
// into [nblk][C] partials merged by a second kernel (deterministic).
//
// Needed by the ViT-B/16 north-star config (BASELINE.json config 5); the
// reference has no transformer.
#include "common.h"
#include "tbamd.h"

namespace tbamd {

constexpr int kLnWaves = 4;  // waves per workgroup
constexpr int kLnMaxR = 8;   // rows per wave-iteration (upper bound)

// Row-group layout shared by forward and backward.  A wave processes R rows per
// iteration; the R*C/8 16-byte chunks of the group are dealt round-robin to the
// 64 lanes (chunk j -> lane j % 64, slot j / 64), so for C = 768 (96 chunks per
// row) R = 2 gives every lane exactly 3 chunks instead of leaving half the wave
// idle on a 1.5-chunk row.  The (row-in-group, column) of each slot is the same
// in every iteration, so gamma/beta are loaded once per wave and the wave then
// strides over row groups (persistent grid, several 16-B loads in flight per
// lane).  Per-row statistics are segmented wave reductions (one per row slot).
struct LnSlot {
  int r;     // row within the group
  int vi;    // 8-wide column chunk
  bool on;   // slot holds a chunk
};

template <int NCH>
__device__ __forceinline__ void ln_layout(int lane, int nv, int R, LnSlot (&sl)[NCH]) {
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int j = lane + 64 * i;
    sl[i].on = j < R * nv;
    sl[i].r = sl[i].on ? j / nv : 0;
    sl[i].vi = sl[i].on ? j - sl[i].r * nv : 0;
  }
}

// per-row wave sums of per-slot partials: out[rr] = sum over lanes/slots with r == rr
template <int NCH, int RB>
__device__ __forceinline__ void ln_row_sums(const float (&part)[NCH], const LnSlot (&sl)[NCH], int R,
                                            float (&out)[RB]) {
#pragma unroll
  for (int rr = 0; rr < RB; ++rr) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) t += (sl[i].on && sl[i].r == rr) ? part[i] : 0.f;
    out[rr] = rr < R ? wave_sum(t) : 0.f;
  }
}

// v[r] for a per-lane r, as a masked sum: a select chain gets folded back into a
// dynamically indexed private array (scratch memory) by the optimizer
template <int RB>
__device__ __forceinline__ float ln_pick(const float (&v)[RB], int r) {
  float o = 0.f;
#pragma unroll
  for (int rr = 0; rr < RB; ++rr) o += r == rr ? v[rr] : 0.f;
  return o;
}

__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// 8 elements kept in their storage format between load and use (4 VGPRs for
// 16-bit types instead of 8 floats): the prefetch buffers of the backward
template <int DT> struct Raw8 {
  uint4 a;
  __device__ __forceinline__ void load(const uint16_t* p) { a = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void unpack(float (&v)[8]) const {
    Vec8<DT>::load(reinterpret_cast<const uint16_t*>(&a), v);
  }
};
template <> struct Raw8<kF32> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void unpack(float (&v)[8]) const {
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};

// RM: rows per group fixed at compile time (1/2/4/8), or 0 = runtime R <= kLnMaxR
template <int DT, int NCH, int RM>
__global__ __launch_bounds__(64 * kLnWaves) void ln_fwd_k(const storage_t<DT>* __restrict__ x,
                                                          const storage_t<DT>* __restrict__ res,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, int64_t M, int C, int Rrt,
                                                          float eps, storage_t<DT>* __restrict__ y,
                                                          storage_t<DT>* __restrict__ xsum,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int RB = RM ? RM : kLnMaxR;
  const int R = RM ? RM : Rrt;
  const int lane = threadIdx.x & 63;
  const int nv = C / 8;
  LnSlot sl[NCH];
  ln_layout<NCH>(lane, nv, R, sl);
  // gamma/beta stay in registers only for narrow layouts (occupancy); wider ones
  // re-read them from L1 (the same 2*C floats for every wave)
  constexpr bool kCache = NCH <= 2;
  float g[kCache ? NCH : 1][8], b[kCache ? NCH : 1][8];
  if constexpr (kCache) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[i][k] = 1.f;
        b[i][k] = 0.f;
      }
      if (sl[i].on && gamma) load8f(gamma + sl[i].vi * 8, g[i]);
      if (sl[i].on && beta) load8f(beta + sl[i].vi * 8, b[i]);
    }
  }
  const int64_t ngroups = (M + R - 1) / R;
  const int64_t stride = (int64_t)gridDim.x * kLnWaves;
  const int64_t gfirst = (int64_t)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  // software pipeline (as in the backward): the next group's x / residual are in
  // flight while this group is reduced and written
  constexpr bool kPrefetch = NCH <= 3;
  Raw8<DT> xc[NCH], rc[NCH];
  auto load_group = [&](int64_t gq, Raw8<DT> (&xs)[NCH], Raw8<DT> (&rs)[NCH]) {
    const int64_t q0 = gq * R;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (gq < ngroups && sl[i].on && q0 + sl[i].r < M) {
        const int64_t off = (q0 + sl[i].r) * C + sl[i].vi * 8;
        xs[i].load(x + off);
        if (res) rs[i].load(res + off);
      }
    }
  };
  if constexpr (kPrefetch) load_group(gfirst, xc, rc);
  for (int64_t grp = gfirst; grp < ngroups; grp += stride) {
    const int64_t r0 = grp * R;
    Raw8<DT> xn[kPrefetch ? NCH : 1], rn[kPrefetch ? NCH : 1];
    if constexpr (kPrefetch) load_group(grp + stride, xn, rn);
    else load_group(grp, xc, rc);
    float v[NCH][8];
    bool ok[NCH];
    float part[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      ok[i] = sl[i].on && r0 + sl[i].r < M;
      const int64_t off = (r0 + sl[i].r) * C + sl[i].vi * 8;
      part[i] = 0.f;
      if (ok[i]) {
        xc[i].unpack(v[i]);
        if (res) {
          float rv[8];
          rc[i].unpack(rv);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[i][k] += rv[k];
          Vec8<DT>::store(xsum + off, v[i]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) part[i] += v[i][k];
      }
    }
    float mean[RB], rstd[RB];
    ln_row_sums<NCH, RB>(part, sl, R, mean);
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) mean[rr] *= 1.f / (float)C;
    float mu[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      mu[i] = ln_pick<RB>(mean, sl[i].r);
      part[i] = 0.f;
      if (ok[i]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = v[i][k] - mu[i];
          part[i] += d * d;
        }
      }
    }
    ln_row_sums<NCH, RB>(part, sl, R, rstd);
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) rstd[rr] = rsqrtf(rstd[rr] * (1.f / (float)C) + eps);
    if (lane < R && r0 + lane < M) {
      mean_out[r0 + lane] = ln_pick<RB>(mean, lane);
      rstd_out[r0 + lane] = ln_pick<RB>(rstd, lane);
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (ok[i]) {
        const float rs = ln_pick<RB>(rstd, sl[i].r);
        float gg[8], bb[8];
        if constexpr (kCache) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            gg[k] = g[i][k];
            bb[k] = b[i][k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            gg[k] = 1.f;
            bb[k] = 0.f;
          }
          if (gamma) load8f(gamma + sl[i].vi * 8, gg);
          if (beta) load8f(beta + sl[i].vi * 8, bb);
        }
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (v[i][k] - mu[i]) * rs * gg[k] + bb[k];
        Vec8<DT>::store(y + (r0 + sl[i].r) * C + sl[i].vi * 8, o);
      }
    }
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        xc[i] = xn[i];
        rc[i] = rn[i];
      }
    }
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)) [+ dadd]; per-workgroup
// column partials of dgamma = sum dy*xhat and dbeta = sum dy, merged into
// [blk][C] in a fixed order (waves in turn, row slots in turn): deterministic.
template <int DT, int NCH, int RM>
__global__ __launch_bounds__(64 * kLnWaves) void ln_bwd_k(const storage_t<DT>* __restrict__ dy,
                                                          const storage_t<DT>* __restrict__ x,
                                                          const storage_t<DT>* __restrict__ dadd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in, int64_t M, int C, int Rrt,
                                                          int64_t groups_per_blk, storage_t<DT>* __restrict__ dx,
                                                          float* __restrict__ pdg, float* __restrict__ pdb) {
  constexpr bool kCacheG = NCH <= 2;
  constexpr int RB = RM ? RM : kLnMaxR;
  const int R = RM ? RM : Rrt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = C / 8;
  LnSlot sl[NCH];
  ln_layout<NCH>(lane, nv, R, sl);
  float gc[kCacheG ? NCH : 1][8];
  if constexpr (kCacheG) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) gc[i][k] = 1.f;
      if (sl[i].on && gamma) load8f(gamma + sl[i].vi * 8, gc[i]);
    }
  }
  float ag[NCH][8], ab[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[i][k] = ab[i][k] = 0.f;
  const int64_t ngroups = (M + R - 1) / R;
  const int64_t g0 = (int64_t)blockIdx.x * groups_per_blk;
  const int64_t g1 = g0 + groups_per_blk < ngroups ? g0 + groups_per_blk : ngroups;
  // software pipeline: the next group's x / dy are in flight while this group
  // is reduced and written (the VGPR budget allows 2 waves per SIMD, so each
  // wave keeps two groups of loads outstanding instead of one)
  // (wide layouts: no prefetch, the registers are not there)
  constexpr bool kPrefetch = NCH <= 3;
  // the residual-stream gradient dadd is fetched with x / dy (one group ahead) rather than
  // after the row reductions, where its latency sat between the sums and the dx store
  Raw8<DT> xc[NCH], dc[NCH], ac[NCH];
  auto load_group = [&](int64_t gq, Raw8<DT> (&xs)[NCH], Raw8<DT> (&ds)[NCH], Raw8<DT> (&as)[NCH]) {
    const int64_t q0 = gq * R;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (gq < g1 && sl[i].on && q0 + sl[i].r < M) {
        const int64_t off = (q0 + sl[i].r) * C + sl[i].vi * 8;
        xs[i].load(x + off);
        ds[i].load(dy + off);
        if (dadd) as[i].load(dadd + off);
      }
    }
  };
  if constexpr (kPrefetch) load_group(g0 + wv, xc, dc, ac);
  for (int64_t grp = g0 + wv; grp < g1; grp += kLnWaves) {
    const int64_t r0 = grp * R;
    Raw8<DT> xn[kPrefetch ? NCH : 1], dn[kPrefetch ? NCH : 1], an[kPrefetch ? NCH : 1];
    if constexpr (kPrefetch) load_group(grp + kLnWaves, xn, dn, an);
    else load_group(grp, xc, dc, ac);
    float xh[NCH][8], gd[NCH][8];
    bool ok[NCH];
    float p1[NCH], p2[NCH];
    float mrow[RB], rrow[RB];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      const bool in = rr < R && r0 + rr < M;
      mrow[rr] = in ? mean_in[r0 + rr] : 0.f;
      rrow[rr] = in ? rstd_in[r0 + rr] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      ok[i] = sl[i].on && r0 + sl[i].r < M;
      p1[i] = p2[i] = 0.f;
      if (ok[i]) {
        const float mu = ln_pick<RB>(mrow, sl[i].r), rs = ln_pick<RB>(rrow, sl[i].r);
        float gg[8];
        if constexpr (kCacheG) {
#pragma unroll
          for (int k = 0; k < 8; ++k) gg[k] = gc[i][k];
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) gg[k] = 1.f;
          if (gamma) load8f(gamma + sl[i].vi * 8, gg);
        }
        float xv[8], dvv[8];
        xc[i].unpack(xv);
        dc[i].unpack(dvv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dv = dvv[k];
          xh[i][k] = (xv[k] - mu) * rs;
          gd[i][k] = dv * gg[k];
          p1[i] += gd[i][k];
          p2[i] += gd[i][k] * xh[i][k];
          ag[i][k] += dv * xh[i][k];
          ab[i][k] += dv;
        }
      }
    }
    float s1[RB], s2[RB];
    ln_row_sums<NCH, RB>(p1, sl, R, s1);
    ln_row_sums<NCH, RB>(p2, sl, R, s2);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (ok[i]) {
        const int64_t off = (r0 + sl[i].r) * C + sl[i].vi * 8;
        const float a1 = ln_pick<RB>(s1, sl[i].r) * (1.f / (float)C);
        const float a2 = ln_pick<RB>(s2, sl[i].r) * (1.f / (float)C);
        const float rs = ln_pick<RB>(rrow, sl[i].r);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rs * (gd[i][k] - a1 - xh[i][k] * a2);
        if (dadd) {
          float av[8];
          ac[i].unpack(av);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += av[k];
        }
        Vec8<DT>::store(dx + off, o);
      }
    }
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        xc[i] = xn[i];
        dc[i] = dn[i];
        ac[i] = an[i];
      }
    }
  }
  // fixed-order merge: the 4 waves add their per-slot partials in turn into a
  // [NCH][64 lanes][8] image (every lane owns its slots, so no two lanes touch
  // one word), then column c gathers its R row slots (chunk r*nv + c/8)
  __shared__ float red[2][8 * 64 * 8];
  for (int w = 0; w < kLnWaves; ++w) {
    if (wv == w) {
#pragma unroll
      for (int i = 0; i < NCH; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int a = (i * 64 + lane) * 8 + k;
          red[0][a] = (w ? red[0][a] : 0.f) + ag[i][k];
          red[1][a] = (w ? red[1][a] : 0.f) + ab[i][k];
        }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < C; c += 64 * kLnWaves) {
    float tg = 0.f, tb = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      const int a = (rr * nv + (c >> 3)) * 8 + (c & 7);
      tg += red[0][a];
      tb += red[1][a];
    }
    pdg[(int64_t)blockIdx.x * C + c] = tg;
    pdb[(int64_t)blockIdx.x * C + c] = tb;
  }
}

// column sums of two [nblk][C] partial arrays: one workgroup per 64 columns,
// 16 row-groups per workgroup (each strides the rows), f64 accumulation, then a
// fixed-order LDS merge (deterministic).  Was one thread per column: 3
// workgroups for C = 768 and a 1024-long dependent loop each (0.23 ms/call).
constexpr int kColRG = 16;
__global__ __launch_bounds__(64 * kColRG) void col_sum2_k(const float* __restrict__ a, const float* __restrict__ b,
                                                          int nblk, int C, float* __restrict__ oa,
                                                          float* __restrict__ ob) {
  __shared__ double red[2][kColRG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  double sa = 0.0, sb = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int i = ty; i < nblk; i += kColRG) {
      sa += a[(int64_t)i * C + c];
      sb += b[(int64_t)i * C + c];
    }
  }
  red[0][ty][tx] = sa;
  red[1][ty][tx] = sb;
  __syncthreads();
  if (ty == 0 && c < C) {
    double ta = 0.0, tb = 0.0;
    for (int r = 0; r < kColRG; ++r) {
      ta += red[0][r][tx];
      tb += red[1][r][tx];
    }
    if (oa) oa[c] = (float)ta;
    if (ob) ob[c] = (float)tb;
  }
}

// (R rows per wave-iteration, NCH 16-B chunks per lane): smallest R whose
// R*C/8 chunks tile the 64 lanes exactly with >= 2 chunks per lane (<= 8); else
// one row per iteration with ceil(C/512) chunks.
static void ln_shape(int C, int& R, int& nch) {
  const int nv = C / 8;
  for (int r = 1; r <= kLnMaxR; ++r) {
    if ((r * nv) % 64 == 0 && r * nv / 64 >= 2 && r * nv / 64 <= 8) {
      R = r;
      nch = r * nv / 64;
      return;
    }
  }
  R = 1;
  nch = (nv + 63) / 64;
}

int ln_bwd_blocks(int64_t M) {
  int64_t b = (M + 15) / 16;  // >= 16 rows per workgroup
  if (b > 512) b = 512;       // one resident round at 2 workgroups per CU
  return (int)(b < 1 ? 1 : b);
}

// (R, NCH) pairs with a compile-time row count (ViT-Ti/S/B/L/H widths 192..1280,
// 1536..4096); anything else runs the runtime-R kernel
#define TBAMD_LN_SHAPES(L)                                          \
  if (R == 2 && nch == 3) L(3, 2);        /* C = 768  */             \
  else if (R == 4 && nch == 3) L(3, 4);   /* C = 384  */             \
  else if (R == 8 && nch == 3) L(3, 8);   /* C = 192  */             \
  else if (R == 2 && nch == 2) L(2, 2);   /* C = 512  */             \
  else if (R == 4 && nch == 2) L(2, 4);   /* C = 256  */             \
  else if (R == 1 && nch == 2) L(2, 1);   /* C = 1024 */             \
  else if (R == 2 && nch == 5) L(5, 2);   /* C = 1280 */             \
  else if (R == 1 && nch == 3) L(3, 1);   /* C = 1536 */             \
  else if (R == 1 && nch == 4) L(4, 1);   /* C = 2048 */             \
  else if (R == 1 && nch == 6) L(6, 1);   /* C = 3072 */             \
  else if (R == 1 && nch == 8) L(8, 1);   /* C = 4096 */             \
  else if (nch == 1) L(1, 0);                                        \
  else if (nch == 2) L(2, 0);                                        \
  else if (nch == 3) L(3, 0);                                        \
  else if (nch == 4) L(4, 0);                                        \
  else if (nch == 5) L(5, 0);                                        \
  else if (nch == 6) L(6, 0);                                        \
  else if (nch == 7) L(7, 0);                                        \
  else L(8, 0)

#define TB_LNF(NCH_, RM_)                                                                                   \
  ln_fwd_k<DT, NCH_, RM_><<<(int)nblk, 64 * kLnWaves, 0, st>>>((const T*)x, (const T*)res, gamma, beta, M, C, R, \
                                                               eps, (T*)y, (T*)xsum, mean, rstd)
#define TB_LNB(NCH_, RM_)                                                                                    \
  ln_bwd_k<DT, NCH_, RM_><<<nblk, 64 * kLnWaves, 0, st>>>((const T*)dy, (const T*)x, (const T*)dadd, gamma, mean, \
                                                          rstd, M, C, R, gpb, (T*)dx, pdg, pdb)

void ln_forward(int dt, const void* x, const void* res, const float* gamma, const float* beta, int64_t M, int C,
                float eps, void* y, void* xsum, float* mean, float* rstd, hipStream_t st) {
  int R, nch;
  ln_shape(C, R, nch);
  const int64_t ngroups = (M + R - 1) / R;
  int64_t nblk = (ngroups + kLnWaves - 1) / kLnWaves;
  if (nblk > 2048) nblk = 2048;  // persistent: 8192 waves stride over the row groups
  TBAMD_DISPATCH_DT(dt, DT, {
    using T = storage_t<DT>;
    TBAMD_LN_SHAPES(TB_LNF);
  });
}

void ln_backward(int dt, const void* dy, const void* x, const void* dadd, const float* gamma, const float* mean,
                 const float* rstd, int64_t M, int C, void* dx, float* pdg, float* pdb, int nblk, float* dgamma,
                 float* dbeta, hipStream_t st) {
  int R, nch;
  ln_shape(C, R, nch);
  const int64_t ngroups = (M + R - 1) / R;
  const int64_t gpb = (ngroups + nblk - 1) / nblk;
  TBAMD_DISPATCH_DT(dt, DT, {
    using T = storage_t<DT>;
    TBAMD_LN_SHAPES(TB_LNB);
  });
  col_sum2_k<<<cdiv(C, 64), 64 * kColRG, 0, st>>>(pdg, pdb, nblk, C, dgamma, dbeta);
}

#undef TB_LNF
#undef TB_LNB
#undef TBAMD_LN_SHAPES

}  // namespace tbamd
