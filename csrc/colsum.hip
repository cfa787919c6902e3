// Column sums of row-major [M, C] activations (bias gradients of Linear layers)
// and the fused GELU backward + bias-gradient pass of a Linear -> GELU pair.
//
// Reference: every nn.Linear with bias of the examples (lenet.py:33-35,
// gan.py:35-48, vae.py:37-56) and the ViT MLP (north-star config 5); the bias
// gradient is Σ_rows dY.  ATen runs it as a generic reduction (≈1 TB/s on
// [25216, 768] bf16); here a workgroup owns a 512-column strip of a row range —
// one wave per 1-KiB row segment, 4 rows in flight per workgroup and 4 per wave —
// and writes one f32 partial row, which a second tiny kernel sums in a fixed order
// (deterministic) into the output dtype.
//
// gelu_bwd_colsum: dZ = dY * GELU'(Z) written in bf16/f32 AND the column sums of
// dZ (the fc1 bias gradient) from the same registers — one pass instead of two.
#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {


// the value as stored in DT (bit-identical to re-reading what was written)
template <int DT>
__device__ __forceinline__ float stored_as(float v) {
  if constexpr (DT == kBF16) return bf2f(f2bf(v));
  else if constexpr (DT == kF16) return h2f(f2h(v));
  else return v;
}

// A wave streams one row segment of 512 columns (64 lanes x 16 B = 1 KiB
// contiguous per load instruction) and the 4 waves of a workgroup take every 4th
// row of the split; the 4 partial rows are merged through LDS in a fixed order.
// (Was 8 lanes per 128-B row segment: eight 128-B pieces per wave instruction,
// ~3.7 TB/s on the fused GELU pass.)
constexpr int kCsCols = 512;
template <int DT, bool GELU>
__global__ __launch_bounds__(256) void colsum_partial_k(const storage_t<DT>* __restrict__ dy,
                                                        const storage_t<DT>* __restrict__ z,
                                                        storage_t<DT>* __restrict__ dz, int64_t M, int C,
                                                        int64_t rows_per_split, float* __restrict__ part) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c0 = blockIdx.x * kCsCols + lane * 8;
  const int split = blockIdx.y;
  const int64_t r0 = split * rows_per_split;
  int64_t r1 = r0 + rows_per_split;
  if (r1 > M) r1 = M;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
#pragma unroll 4
    for (int64_t r = r0 + wv; r < r1; r += 4) {
      float v[8];
      load_vec<DT, 8>(dy + r * C + c0, v);
      if constexpr (GELU) {
        float zv[8];
        load_vec<DT, 8>(z + r * C + c0, zv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_grad(zv[e]);
        store_vec<DT, 8>(dz + r * C + c0, v);
        // the bias gradient sums the values as stored (what the weight GEMMs see)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = stored_as<DT>(v[e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
  __shared__ float red[4][kCsCols];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[wv][lane * 8 + e] = acc[e];
  __syncthreads();
  for (int c = tid; c < kCsCols; c += 256) {
    const int cc = blockIdx.x * kCsCols + c;
    if (cc < C) part[(int64_t)split * C + cc] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// sum the [nsplit][C] partials: 64 columns x 16 split groups per workgroup, merged
// through LDS in a fixed order (one thread walking hundreds of splits serially
// was 80 us for C = 768)
constexpr int kFinRG = 16;
template <int DT>
__global__ __launch_bounds__(64 * kFinRG) void colsum_final_k(const float* __restrict__ part, int nsplit, int C,
                                                              storage_t<DT>* __restrict__ out) {
  __shared__ float red[kFinRG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int i = ty; i < nsplit; i += kFinRG) s += part[(int64_t)i * C + c];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < kFinRG; ++r) t += red[r][tx];
    Elem<DT>::st(out, c, t);
  }
}

}  // namespace

// y = GELU(z) (exact erf form, the same device function as the fused epilogues and the
// backward) over a contiguous tensor: 8 elements (16 B for 16-bit types) per lane per step,
// grid-stride.  The ViT fc1 forward when the GEMM itself runs on hipBLASLt (bias epilogue):
// replaces ATen's GeluCUDAKernel, so the steady-state ViT forward has no ATen compute kernel.
template <int DT>
__global__ __launch_bounds__(256) void gelu_fwd_k(const storage_t<DT>* __restrict__ z, storage_t<DT>* __restrict__ y,
                                                  int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load_vec<DT, 8>(z + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
    store_vec<DT, 8>(y + i * 8, v);
  }
}

void gelu_forward(int dt, const void* z, void* y, int64_t n, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  int64_t grid = (n8 + 255) / 256;
  if (grid > 8192) grid = 8192;
  TBAMD_DISPATCH_DT(dt, DT, {
    gelu_fwd_k<DT><<<(int)grid, 256, 0, st>>>((const storage_t<DT>*)z, (storage_t<DT>*)y, n8);
  });
}

void colsum_finalize(int dt, const float* part, int nsplit, int C, void* out, hipStream_t st) {
  TBAMD_DISPATCH_DT(dt, DTV, {
    colsum_final_k<DTV><<<(C + 63) / 64, 64 * kFinRG, 0, st>>>(part, nsplit, C, (storage_t<DTV>*)out);
  });
}

int colsum_splits(int64_t M, int C) {
  const int64_t cb = (C + kCsCols - 1) / kCsCols;
  int64_t s = (1024 + cb - 1) / cb;  // ~1024 workgroups (4 per CU)
  const int64_t maxs = (M + 31) / 32;  // >= 32 rows (8 per wave) per split
  if (s > maxs) s = maxs;
  if (s > 512) s = 512;
  return s < 1 ? 1 : (int)s;
}

void colsum(int dt, const void* dy, const void* z, void* dz, int64_t M, int C, float* part, void* out,
            hipStream_t st) {
  const int ns = colsum_splits(M, C);
  const int64_t rps = (M + ns - 1) / ns;
  const dim3 grid((C + kCsCols - 1) / kCsCols, ns);
  TBAMD_DISPATCH_DT(dt, DTV, {
    using T = storage_t<DTV>;
    if (z)
      colsum_partial_k<DTV, true><<<grid, 256, 0, st>>>((const T*)dy, (const T*)z, (T*)dz, M, C, rps, part);
    else
      colsum_partial_k<DTV, false><<<grid, 256, 0, st>>>((const T*)dy, nullptr, nullptr, M, C, rps, part);
    colsum_final_k<DTV><<<(C + 63) / 64, 64 * kFinRG, 0, st>>>(part, ns, C, (T*)out);
  });
}

}  // namespace tbamd
