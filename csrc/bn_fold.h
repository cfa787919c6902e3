// BatchNorm statistics finalized inside the conv that produces them.
//
// A conv whose epilogue emits BN partial sums (one [2][K] row per pixel tile or per stream,
// csrc/conv.hip STATS) used to hand them to a separate finalize launch (csrc/norm_bn.hip
// colsum_fin4_k: ~8 us per BatchNorm, latency-bound, 53 per ResNet-50 forward).  Folded, the
// reduction runs in the conv's own tail, in two levels of arrival tickets:
//
//   * the rows are cut into groups of `group` rows per channel tile; the workgroup that
//     arrives LAST in its group (agent-scope ticket) sums the group's rows (fixed order) into
//     a level-1 row of doubles -- every group but the last one finishes while other
//     workgroups of the conv are still computing;
//   * the last level-1 arrival of the channel tile sums the level-1 rows (fixed order) and
//     writes mean / invstd / scale / shift, the running statistics and the batch counter,
//     exactly as norm_bn.hip StatsFin does.
//
// Publication follows the in-launch split reduction of cdna_hip_programming.md §5 (the
// write-through form of norm_bn.hip colsum_fin4_k): rows are stored write-through
// (agent-scope relaxed atomic stores = global_store sc1), the storing waves drain, one lane
// takes the ticket, the last arrival acquires at agent scope and reads with plain loads.
// Counters return to zero before the launch ends (the last arrival of each counter resets it).
// Summation order is fixed -> deterministic run to run.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace tbamd {

struct BnFold {
  unsigned* tick;  // [ntm][ngroups + 1] arrival counters (nullptr: not folded)
  double* l1;      // [ngroups][2][K] level-1 sums (ngroups > 1)
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float* coeff;  // forward: [4][K] mean, invstd, scale, shift; backward: [3][K] coef (norm_bn.hip BwdFin)
  int64_t M;     // rows of the BN input (N*P*Q)
  float momentum, eps;
  int rows, group, ngroups, K;
  // backward (bwd = 1): the partials are (sum dz, sum dz (x - mean)) of a dgrad BNB epilogue
  int bwd, training;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
};

// level-1 group size for `rows` partial rows: >= 64 rows a group, at most 256 groups
inline int bn_fold_group(int rows) {
  int g = 64;
  if ((rows + g - 1) / g > 256) g = (rows + 255) / 256;
  return g;
}
inline int bn_fold_ngroups(int rows) {
  const int g = bn_fold_group(rows);
  return (rows + g - 1) / g;
}

#if defined(__HIPCC__)
__device__ __forceinline__ void fold_st_f32(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fold_st_f64(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every thread of the workgroup: true in the workgroup whose arrival at *tk is number
// expect_last + 1 (its earlier vector stores are drained first; it acquires at agent scope)
__device__ __forceinline__ bool fold_arrive(unsigned* tk, unsigned expect_last, volatile int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expect_last;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

__device__ __forceinline__ void fold_reset(unsigned* tk) {
  __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// backward partials -> dgamma, dbeta and the apply coefficients (norm_bn.hip BwdFin)
__device__ __forceinline__ void bn_fold_fin_bwd(const BnFold& f, int c, double a, double b) {
  const double is = f.invstd[c];
  const double db = a;
  const double dg = b * is;
  if (f.dgamma) f.dgamma[c] = (float)dg;
  if (f.dbeta) f.dbeta[c] = (float)db;
  const double gm = f.gamma ? f.gamma[c] : 1.0;
  const double ka = gm * is;
  double c1 = 0.0, c0 = 0.0;
  if (f.training) {
    c1 = -ka * is * dg / (double)f.M;
    c0 = -ka * db / (double)f.M - c1 * (double)f.mean[c];
  }
  f.coeff[c] = (float)ka;
  f.coeff[f.K + c] = (float)c0;
  f.coeff[2 * f.K + c] = (float)c1;
}

// training statistics -> coefficients, running statistics, counter (norm_bn.hip StatsFin)
__device__ __forceinline__ void bn_fold_fin(const BnFold& f, int c, double s, double q) {
  if (f.bwd) {
    bn_fold_fin_bwd(f, c, s, q);
    return;
  }
  const double md = s / (double)f.M;
  double var = q / (double)f.M - md * md;
  if (var < 0.0) var = 0.0;
  const float mean = (float)md;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float gm = f.gamma ? f.gamma[c] : 1.f;
  const float bt = f.beta ? f.beta[c] : 0.f;
  const float sc = gm * invstd;
  f.coeff[c] = mean;
  f.coeff[f.K + c] = invstd;
  f.coeff[2 * f.K + c] = sc;
  f.coeff[3 * f.K + c] = bt - mean * sc;
  if (f.rmean) {
    const double unb = f.M > 1 ? var * (double)f.M / (double)(f.M - 1) : var;
    f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * mean;
    f.rvar[c] = (float)((1.0 - f.momentum) * f.rvar[c] + f.momentum * unb);
  }
  if (f.nbt && c == 0) *f.nbt += 1;
}

// Tail of a 256-thread workgroup that has just stored (write-through) its partial row `row`
// ([2][BM] at channel m0 of stats [rows][2][K]) for channel tile tile_m.  scratch: >= 4 KiB + 4 B
// of LDS no thread still reads.
template <int BM>
__device__ __forceinline__ void bn_fold_tail(const BnFold& f, const float* stats, int tile_m, int row, int m0,
                                             void* scratch) {
  constexpr int NT = 256, P = 2 * BM, RT = NT / P;
  static_assert(NT % P == 0, "pairs per workgroup");
  double* sm = reinterpret_cast<double*>(scratch);  // [NT]
  double* sm2 = sm + NT;                             // [P]
  volatile int* flag = reinterpret_cast<volatile int*>(sm2 + P);
  const int tid = threadIdx.x;
  const int ng = f.ngroups;
  const int grp = row / f.group;
  const int g0 = grp * f.group, g1 = min(g0 + f.group, f.rows);
  unsigned* tk = f.tick + (int64_t)tile_m * (ng + 1);
  if (!fold_arrive(tk + grp, (unsigned)(g1 - g0 - 1), flag)) return;
  const int pr = tid % P, sub = tid / P;
  const int kind = pr / BM, cl = pr - kind * BM;
  double a = 0.0;
  for (int r = g0 + sub; r < g1; r += RT) a += (double)stats[((int64_t)r * 2 + kind) * f.K + m0 + cl];
  sm[tid] = a;
  __syncthreads();
  double v = 0.0;
  if (tid < P) {
#pragma unroll
    for (int k = 0; k < RT; ++k) v += sm[k * P + tid];
  }
  if (tid == 0) fold_reset(tk + grp);
  if (ng > 1) {
    if (tid < P) fold_st_f64(&f.l1[((int64_t)grp * 2 + kind) * f.K + m0 + cl], v);
    if (!fold_arrive(tk + ng, (unsigned)(ng - 1), flag)) return;
    double b = 0.0;
    for (int q = sub; q < ng; q += RT) b += f.l1[((int64_t)q * 2 + kind) * f.K + m0 + cl];
    sm[tid] = b;
    __syncthreads();
    v = 0.0;
    if (tid < P) {
#pragma unroll
      for (int k = 0; k < RT; ++k) v += sm[k * P + tid];
    }
    if (tid == 0) fold_reset(tk + ng);
  }
  if (tid < P) sm2[tid] = v;
  __syncthreads();
  if (tid < BM) bn_fold_fin(f, m0 + tid, sm2[tid], sm2[BM + tid]);
}
#endif

}  // namespace tbamd
