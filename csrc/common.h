// Shared device helpers for the torchbooster_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel file:
//   * wave = 64 lanes; every block size is a multiple of 64.
//   * bf16 is carried as raw 16-bit payload (uint16_t) in memory; arithmetic is
//     fp32.  f32 -> bf16 uses the compiler cast, which lowers to
//     v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950.
//   * memory-bound kernels move 16 B per lane (8 x bf16 or 4 x f32).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tbamd.h"

namespace tbamd {

// ---- bounds-checked debug build: `python -m torchbooster_amd._build
// --bounds` compiles every kernel with -DTBAMD_BOUNDS into _C_bounds.so.  Guarded
// accesses then test their index against the tensor extent the kernel derives from
// its shape arguments; a violation sets a bit in a per-file device flag (a vector
// atomic) and the access is redirected (zero page / skipped store) instead of
// faulting.  The host reads and clears every file's flag after each native op
// (ops/_ext.py, TBAMD_BOUNDS=1) and raises naming the op.  Normal builds: the
// guards are the constant `true` and cost nothing.
void bounds_register_reader(unsigned (*reader)());
#ifdef TBAMD_BOUNDS
namespace bounds {
static __device__ unsigned g_flag;
static unsigned read_and_clear() {
  unsigned v = 0, z = 0;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_flag), sizeof(v));
  if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_flag), &z, sizeof(z));
  return v;
}
struct Registrar {
  Registrar() { bounds_register_reader(&read_and_clear); }
};
static Registrar g_registrar;
__device__ __forceinline__ bool ok(bool cond, unsigned code) {
  if (!cond) atomicOr(&g_flag, code);
  return cond;
}
}  // namespace bounds
#define TB_BOUNDS_OK(cond, code) (::tbamd::bounds::ok((cond), (code)))
#else
#define TB_BOUNDS_OK(cond, code) true
#endif
// violation codes (bit per kernel family)
enum : unsigned {
  kBndConvSrc = 1u << 0, kBndConvW = 1u << 1, kBndConvDst = 1u << 2, kBndGemmSrc = 1u << 3,
  kBndGemmDst = 1u << 4, kBndAnySrc = 1u << 5, kBndAnyDst = 1u << 6, kBndWgradSrc = 1u << 7,
};

// Materialise a global's address once, in SGPRs, before a loop: without this hipcc
// re-loads the address from the GOT inside the loop body (an s_load whose
// s_waitcnt lgkmcnt(0) also drains every LDS read in flight).
__device__ __forceinline__ const void* pin_sgpr(const void* p) {
  asm volatile("" : "+s"(p));
  return p;
}

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float h2f(uint16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// Element load/store for the three storage types; T is the storage type tag.
template <int DT> struct Elem;
template <> struct Elem<kF32> {
  using T = float;
  __device__ __forceinline__ static float ld(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void st(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elem<kBF16> {
  using T = uint16_t;
  __device__ __forceinline__ static float ld(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
  __device__ __forceinline__ static void st(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
};
template <> struct Elem<kF16> {
  using T = uint16_t;
  __device__ __forceinline__ static float ld(const uint16_t* p, int64_t i) { return h2f(p[i]); }
  __device__ __forceinline__ static void st(uint16_t* p, int64_t i, float v) { p[i] = f2h(v); }
};

// 8-wide vector load/store: 16 B for 16-bit types, 32 B (2 x dwordx4) for f32.
template <int DT> struct Vec8;
template <> struct Vec8<kBF16> {
  __device__ __forceinline__ static void load(const uint16_t* p, float (&v)[8]) {
    uint4 r = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<kF16> {
  __device__ __forceinline__ static void load(const uint16_t* p, float (&v)[8]) {
    uint4 r = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = h2f((uint16_t)(w[i] & 0xffff));
      v[2 * i + 1] = h2f((uint16_t)(w[i] >> 16));
    }
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2h(v[2 * i]) | ((uint32_t)f2h(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<kF32> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <int DT> using storage_t = typename Elem<DT>::T;

// VEC consecutive elements <-> f32 registers (16-B accesses when VEC == 8)
template <int DT, int VEC>
__device__ __forceinline__ void load_vec(const storage_t<DT>* p, float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    Vec8<DT>::load(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[i] = Elem<DT>::ld(p, i);
  }
}
template <int DT, int VEC>
__device__ __forceinline__ void store_vec(storage_t<DT>* p, const float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    Vec8<DT>::store(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) Elem<DT>::st(p, i, v[i]);
  }
}


// Full-wave (64-lane) reductions via DPP-backed shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x < NT / 64) r = red[threadIdx.x];
  if (wid == 0) r = wave_sum(r);
  if (threadIdx.x == 0) red[0] = r;
  __syncthreads();
  r = red[0];
  __syncthreads();
  return r;
}

// Activation codes shared by fused epilogues.
enum Act : int { kActNone = 0, kActReLU = 1, kActGELU = 2, kActSiLU = 3, kActLeaky = 4 };

// erf(x / sqrt 2) and exp(-x^2 / 2) sharing ONE exponential (Abramowitz & Stegun 7.1.26:
// |error| <= 1.5e-7, below the rounding of a bf16 or f32 GELU output), ~12 instructions
// against the ~30 (with branches) of erff — GELU sits in GEMM / norm epilogues over
// whole activations (ViT MLP: 77 M elements per layer).
__device__ __forceinline__ void erf_sqrt2_gauss(float x, float& erfv, float& gauss) {
  const float ax = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  gauss = __expf(-0.5f * x * x);
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  erfv = copysignf(1.f - poly * gauss, x);
}
__device__ __forceinline__ float gelu_f(float x) {
  // exact (erf) GELU, matching torch.nn.GELU() default
  float e, g;
  erf_sqrt2_gauss(x, e, g);
  return 0.5f * x * (1.f + e);
}
__device__ __forceinline__ float gelu_grad(float x) {
  float e, g;
  erf_sqrt2_gauss(x, e, g);
  return 0.5f * (1.f + e) + x * 0.3989422804014327f * g;
}
__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = 1.f / (1.f + __expf(-x));
  return s * (1.f + x * (1.f - s));
}

template <int ACT>
__device__ __forceinline__ float act_fwd(float z, float slope) {
  if constexpr (ACT == kActReLU) return fmaxf(z, 0.f);
  else if constexpr (ACT == kActGELU) return gelu_f(z);
  else if constexpr (ACT == kActSiLU) return silu_f(z);
  else if constexpr (ACT == kActLeaky) return z > 0.f ? z : z * slope;
  else return z;
}
// derivative of act at pre-activation z
template <int ACT>
__device__ __forceinline__ float act_bwd(float z, float slope) {
  if constexpr (ACT == kActReLU) return z > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == kActGELU) return gelu_grad(z);
  else if constexpr (ACT == kActSiLU) return silu_grad(z);
  else if constexpr (ACT == kActLeaky) return z > 0.f ? 1.f : slope;
  else return 1.f;
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// ---- completion-event hand-off to a second stream (ops/streams.py).  The host arms an event;
// the next launch made through tb_launch_ev records it as the kernel's OWN completion (the
// hipExtLaunchKernelGGL stop event) instead of a separate marker packet behind the kernel:
// hipEventRecord + a side-stream wait costs the producing queue 4.6 us after a 26 us kernel,
// the stop event 0.75 us (profiles/r03_fork/fork_cost.jsonl).
inline hipEvent_t& armed_stop_event() {
  static thread_local hipEvent_t ev = nullptr;
  return ev;
}
template <typename... KArgs, typename... Args>
inline void tb_launch_ev(void (*k)(KArgs...), dim3 grid, dim3 block, uint32_t shm, hipStream_t st, Args... args) {
  hipEvent_t& slot = armed_stop_event();
  const hipEvent_t ev = slot;
  slot = nullptr;
  hipExtLaunchKernelGGL(k, grid, block, shm, st, nullptr, ev, 0u, static_cast<KArgs>(args)...);
}

}  // namespace tbamd

#define TBAMD_DISPATCH_DT(dt, DTV, ...)                         \
  switch (dt) {                                                 \
    case tbamd::kF32: { constexpr int DTV = tbamd::kF32; __VA_ARGS__; } break;   \
    case tbamd::kBF16: { constexpr int DTV = tbamd::kBF16; __VA_ARGS__; } break; \
    case tbamd::kF16: { constexpr int DTV = tbamd::kF16; __VA_ARGS__; } break;   \
    default: break;                                             \
  }

#define TBAMD_DISPATCH_ACT(a, AV, ...)                            \
  switch (a) {                                                    \
    case tbamd::kActNone: { constexpr int AV = tbamd::kActNone; __VA_ARGS__; } break; \
    case tbamd::kActReLU: { constexpr int AV = tbamd::kActReLU; __VA_ARGS__; } break; \
    case tbamd::kActGELU: { constexpr int AV = tbamd::kActGELU; __VA_ARGS__; } break; \
    case tbamd::kActSiLU: { constexpr int AV = tbamd::kActSiLU; __VA_ARGS__; } break; \
    case tbamd::kActLeaky: { constexpr int AV = tbamd::kActLeaky; __VA_ARGS__; } break; \
    default: break;                                               \
  }
