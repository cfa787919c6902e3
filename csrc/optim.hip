// Multi-tensor fused optimizers for gfx950: AdamW (+ EMA), SGD (momentum /
// nesterov / dampening / coupled weight decay), global-L2 grad norm with the
// clip coefficient computed on device, and AMP unscale/inf-skip folded in.
//
// Reference behaviour: torch.optim.AdamW / SGD built by OptimizerConfig.make
// (/root/reference/torchbooster/config.py:418-438) and stepped by utils.step
// (/root/reference/torchbooster/utils.py:237-252) after clip_grad_norm_.
// SURVEY.md §2.3.1 K11-K14.
//
// Every kernel walks a chunk table: chunk b covers elements
// [start, start+len) of tensor `tidx`; per-tensor pointers live in a device
// table so one launch covers every parameter of the model (161 tensors for
// ResNet-50).  Scalars that change per step without a host round-trip (clip
// coefficient, AMP inverse scale, found-inf flag) are read from device memory.
#include "common.h"
#include "tbamd.h"

namespace tbamd {

constexpr int kOptThreads = 256;

struct ChunkDesc {
  int32_t tidx;
  int32_t pad;
  int64_t start;
  int64_t len;
};

// per-tensor pointer slots in the table (int64 each)
enum Slot : int { kP = 0, kG = 1, kM = 2, kV = 3, kPM = 4, kEMA = 5, kVMAX = 6, kNumSlots = 8 };

// Combined gradient multiplier: clip coefficient * AMP inverse scale.
__device__ __forceinline__ float grad_mult(const float* clip_coef, const float* inv_scale) {
  float m = 1.f;
  if (clip_coef) m *= *clip_coef;
  if (inv_scale) m *= *inv_scale;
  return m;
}

template <int PDT, int GDT, bool MASTER, bool EMA, bool AMS>
__global__ __launch_bounds__(kOptThreads) void adamw_mt_k(const ChunkDesc* __restrict__ chunks,
                                                           const int64_t* __restrict__ table, float lr,
                                                           float beta1, float beta2, float eps, float wd,
                                                           float bc1, float bc2_sqrt, float ema_decay,
                                                           const float* clip_coef, const float* inv_scale,
                                                           const float* found_inf, const float* hyper) {
  if (found_inf && *found_inf != 0.f) return;
  if (hyper) {  // hipGraph replay: step-dependent scalars live in device memory
    lr = hyper[0];
    bc1 = hyper[1];
    bc2_sqrt = hyper[2];
  }
  const ChunkDesc cd = chunks[blockIdx.x];
  const int64_t* slots = table + (int64_t)cd.tidx * kNumSlots;
  // with a master copy, p is the f32 master and pm the model-dtype param
  float* p = reinterpret_cast<float*>(slots[kP]);
  storage_t<PDT>* pm = reinterpret_cast<storage_t<PDT>*>(slots[kPM]);
  const storage_t<GDT>* g = reinterpret_cast<const storage_t<GDT>*>(slots[kG]);
  float* m = reinterpret_cast<float*>(slots[kM]);
  float* v = reinterpret_cast<float*>(slots[kV]);
  float* ema = reinterpret_cast<float*>(slots[kEMA]);
  float* vmax = reinterpret_cast<float*>(slots[kVMAX]);
  const float gm = grad_mult(clip_coef, inv_scale);
  const float step_size = lr / bc1;
  const float decay = 1.f - lr * wd;
  for (int64_t i = cd.start + threadIdx.x; i < cd.start + cd.len; i += kOptThreads) {
    float pv;
    if constexpr (MASTER) pv = p[i];
    else pv = Elem<PDT>::ld(pm, i);
    const float gv = Elem<GDT>::ld(g, i) * gm;
    float mv = m[i], vv = v[i];
    mv = beta1 * mv + (1.f - beta1) * gv;
    vv = beta2 * vv + (1.f - beta2) * gv * gv;
    m[i] = mv;
    v[i] = vv;
    float den;
    if constexpr (AMS) {
      const float vm = fmaxf(vmax[i], vv);
      vmax[i] = vm;
      den = sqrtf(vm) / bc2_sqrt + eps;
    } else {
      den = sqrtf(vv) / bc2_sqrt + eps;
    }
    pv = pv * decay - step_size * mv / den;
    if constexpr (MASTER) {
      p[i] = pv;
      Elem<PDT>::st(pm, i, pv);
    } else {
      Elem<PDT>::st(pm, i, pv);
    }
    if constexpr (EMA) ema[i] = ema_decay * ema[i] + (1.f - ema_decay) * pv;
  }
}

template <int PDT, int GDT, bool MASTER, bool MOM, bool NESTEROV>
__global__ __launch_bounds__(kOptThreads) void sgd_mt_k(const ChunkDesc* __restrict__ chunks,
                                                         const int64_t* __restrict__ table, float lr,
                                                         float momentum, float dampening, float wd,
                                                         int first_step, const float* clip_coef,
                                                         const float* inv_scale, const float* found_inf,
                                                         const float* hyper) {
  if (found_inf && *found_inf != 0.f) return;
  if (hyper) lr = hyper[0];  // hipGraph replay: lr from device memory
  const ChunkDesc cd = chunks[blockIdx.x];
  const int64_t* slots = table + (int64_t)cd.tidx * kNumSlots;
  float* p = reinterpret_cast<float*>(slots[kP]);
  storage_t<PDT>* pm = reinterpret_cast<storage_t<PDT>*>(slots[kPM]);
  const storage_t<GDT>* g = reinterpret_cast<const storage_t<GDT>*>(slots[kG]);
  float* buf = reinterpret_cast<float*>(slots[kM]);
  const float gm = grad_mult(clip_coef, inv_scale);
  for (int64_t i = cd.start + threadIdx.x; i < cd.start + cd.len; i += kOptThreads) {
    float pv;
    if constexpr (MASTER) pv = p[i];
    else pv = Elem<PDT>::ld(pm, i);
    float d = Elem<GDT>::ld(g, i) * gm + wd * pv;
    if constexpr (MOM) {
      float b = first_step ? d : momentum * buf[i] + (1.f - dampening) * d;
      buf[i] = b;
      d = NESTEROV ? d + momentum * b : b;
    }
    pv -= lr * d;
    if constexpr (MASTER) p[i] = pv;
    Elem<PDT>::st(pm, i, pv);
  }
}

// Σ g^2 per chunk (f32 partial per chunk, deterministic)
template <int GDT>
__global__ __launch_bounds__(kOptThreads) void sumsq_mt_k(const ChunkDesc* __restrict__ chunks,
                                                           const int64_t* __restrict__ table,
                                                           float* __restrict__ partial) {
  __shared__ float red[kOptThreads / 64];
  const ChunkDesc cd = chunks[blockIdx.x];
  const storage_t<GDT>* g =
      reinterpret_cast<const storage_t<GDT>*>(table[(int64_t)cd.tidx * kNumSlots + kG]);
  float s = 0.f;
  // 16-B vector body (chunk starts are multiples of the chunk size, tensors are
  // 256-B aligned in their flat stores / buckets), scalar tail
  const int64_t end = cd.start + cd.len;
  const int64_t vend = cd.start + (cd.len & ~(int64_t)7);
  const bool vec_ok = (reinterpret_cast<uintptr_t>(g + cd.start) & 15) == 0;
  int64_t i0 = cd.start;
  if (vec_ok) {
    for (int64_t i = cd.start + 8 * (int64_t)threadIdx.x; i < vend; i += 8 * kOptThreads) {
      float v[8];
      load_vec<GDT, 8>(g + i, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[e] * v[e];
    }
    i0 = vend;
  }
  for (int64_t i = i0 + threadIdx.x; i < end; i += kOptThreads) {
    const float v = Elem<GDT>::ld(g, i);
    s += v * v;
  }
  s = block_sum<kOptThreads>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// norm finalize: out[0] = total norm, out[1] = clip coef (1 if max_norm <= 0),
// out[2] = 1 if non-finite.  Optional inv_scale multiplies the norm first
// (norm of unscaled grads) — matches scaler.unscale_ + clip_grad_norm_.
__global__ __launch_bounds__(256) void norm_finalize_k(const float* __restrict__ partial, int n,
                                                       float max_norm, const float* inv_scale,
                                                       float* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += (double)partial[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = red[0] + red[1] + red[2] + red[3];
    double nrm = sqrt(t);
    if (inv_scale) nrm *= (double)(*inv_scale);
    const float fn = (float)nrm;
    out[0] = fn;
    float coef = 1.f;
    if (max_norm > 0.f) {
      coef = (float)((double)max_norm / (nrm + 1e-6));
      if (coef > 1.f) coef = 1.f;
      if (!isfinite(fn)) coef = fn;  // torch multiplies grads by a nan/inf coefficient too
    }
    out[1] = coef;
    out[2] = isfinite(fn) ? 0.f : 1.f;
  }
}

// g *= s (in place), s on device (used for standalone clip_grad_norm_)
template <int GDT>
__global__ __launch_bounds__(kOptThreads) void scale_mt_k(const ChunkDesc* __restrict__ chunks,
                                                           const int64_t* __restrict__ table,
                                                           const float* __restrict__ s) {
  const ChunkDesc cd = chunks[blockIdx.x];
  storage_t<GDT>* g = reinterpret_cast<storage_t<GDT>*>(table[(int64_t)cd.tidx * kNumSlots + kG]);
  const float f = *s;
  if (f == 1.f) return;
  for (int64_t i = cd.start + threadIdx.x; i < cd.start + cd.len; i += kOptThreads)
    Elem<GDT>::st(g, i, Elem<GDT>::ld(g, i) * f);
}

// ---------------------------------------------------------------------------
void adamw_mt(int pdt, int gdt, bool master, bool ema, bool amsgrad, const void* chunks, int nchunks,
              const int64_t* table, float lr, float beta1, float beta2, float eps, float wd, float bc1,
              float bc2_sqrt, float ema_decay, const float* clip_coef, const float* inv_scale,
              const float* found_inf, hipStream_t st, const float* hyper) {
  if (nchunks == 0) return;
  const ChunkDesc* cd = reinterpret_cast<const ChunkDesc*>(chunks);
#define TB_ADAM(M_, E_, A_)                                                                         \
  adamw_mt_k<PDT, GDT, M_, E_, A_><<<nchunks, kOptThreads, 0, st>>>(cd, table, lr, beta1, beta2, eps, \
                                                                     wd, bc1, bc2_sqrt, ema_decay,   \
                                                                     clip_coef, inv_scale, found_inf, hyper)
  TBAMD_DISPATCH_DT(pdt, PDT, {
    TBAMD_DISPATCH_DT(gdt, GDT, {
      if (master) {
        if (ema) { if (amsgrad) TB_ADAM(true, true, true); else TB_ADAM(true, true, false); }
        else { if (amsgrad) TB_ADAM(true, false, true); else TB_ADAM(true, false, false); }
      } else {
        if (ema) { if (amsgrad) TB_ADAM(false, true, true); else TB_ADAM(false, true, false); }
        else { if (amsgrad) TB_ADAM(false, false, true); else TB_ADAM(false, false, false); }
      }
    });
  });
#undef TB_ADAM
}

void sgd_mt(int pdt, int gdt, bool master, float momentum, float dampening, bool nesterov, float wd,
            float lr, int first_step, const void* chunks, int nchunks, const int64_t* table,
            const float* clip_coef, const float* inv_scale, const float* found_inf, hipStream_t st,
            const float* hyper) {
  if (nchunks == 0) return;
  const ChunkDesc* cd = reinterpret_cast<const ChunkDesc*>(chunks);
#define TB_SGD(M_, MO_, N_)                                                                        \
  sgd_mt_k<PDT, GDT, M_, MO_, N_><<<nchunks, kOptThreads, 0, st>>>(cd, table, lr, momentum, dampening, \
                                                                    wd, first_step, clip_coef,       \
                                                                    inv_scale, found_inf, hyper)
  const bool mom = momentum != 0.f;
  TBAMD_DISPATCH_DT(pdt, PDT, {
    TBAMD_DISPATCH_DT(gdt, GDT, {
      if (master) {
        if (mom) { if (nesterov) TB_SGD(true, true, true); else TB_SGD(true, true, false); }
        else TB_SGD(true, false, false);
      } else {
        if (mom) { if (nesterov) TB_SGD(false, true, true); else TB_SGD(false, true, false); }
        else TB_SGD(false, false, false);
      }
    });
  });
#undef TB_SGD
}

void grad_norm_mt(int gdt, const void* chunks, int nchunks, const int64_t* table, float max_norm,
                  const float* inv_scale, float* partial, float* out3, hipStream_t st) {
  const ChunkDesc* cd = reinterpret_cast<const ChunkDesc*>(chunks);
  if (nchunks > 0) {
    TBAMD_DISPATCH_DT(gdt, GDT, {
      sumsq_mt_k<GDT><<<nchunks, kOptThreads, 0, st>>>(cd, table, partial);
    });
  }
  norm_finalize_k<<<1, 256, 0, st>>>(partial, nchunks, max_norm, inv_scale, out3);
}

void grad_norm_multi(int ngroups, const int* gdts, const void* const* chunks, const int* nchunks,
                     const int64_t* const* tables, float max_norm, const float* inv_scale, float* partial,
                     float* out3, hipStream_t st) {
  int off = 0;
  for (int i = 0; i < ngroups; ++i) {
    if (nchunks[i] > 0) {
      const ChunkDesc* cd = reinterpret_cast<const ChunkDesc*>(chunks[i]);
      TBAMD_DISPATCH_DT(gdts[i], GDT, {
        sumsq_mt_k<GDT><<<nchunks[i], kOptThreads, 0, st>>>(cd, tables[i], partial + off);
      });
    }
    off += nchunks[i];
  }
  norm_finalize_k<<<1, 256, 0, st>>>(partial, off, max_norm, inv_scale, out3);
}

void scale_mt(int gdt, const void* chunks, int nchunks, const int64_t* table, const float* s,
              hipStream_t st) {
  if (nchunks == 0) return;
  const ChunkDesc* cd = reinterpret_cast<const ChunkDesc*>(chunks);
  TBAMD_DISPATCH_DT(gdt, GDT, { scale_mt_k<GDT><<<nchunks, kOptThreads, 0, st>>>(cd, table, s); });
}

}  // namespace tbamd
