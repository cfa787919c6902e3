// Column sums of row-major [M, C] activations (bias gradients of Linear layers)
// and the fused GELU backward + bias-gradient pass of a Linear -> GELU pair.
//
// Reference: every nn.Linear with bias of the examples (lenet.py:33-35,
// gan.py:35-48, vae.py:37-56) and the ViT MLP (north-star config 5); the bias
// gradient is Σ_rows dY.  ATen runs it as a generic reduction (≈1 TB/s on
// [25216, 768] bf16); here a workgroup owns a 64-column strip of a row range —
// 8 lanes cover one 128-B row segment, 32 rows in flight per workgroup — and
// writes one f32 partial row, which a second tiny kernel sums in a fixed order
// (deterministic) into the output dtype.
//
// gelu_bwd_colsum: dZ = dY * GELU'(Z) written in bf16/f32 AND the column sums of
// dZ (the fc1 bias gradient) from the same registers — one pass instead of two.
#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

constexpr int kCsRows = 32;  // row lanes per workgroup (x 8 column chunks = 256 threads)

template <int DT, bool GELU>
__global__ __launch_bounds__(256) void colsum_partial_k(const storage_t<DT>* __restrict__ dy,
                                                        const storage_t<DT>* __restrict__ z,
                                                        storage_t<DT>* __restrict__ dz, int64_t M, int C,
                                                        int64_t rows_per_split, float* __restrict__ part) {
  const int tid = threadIdx.x;
  const int ch = tid & 7, rl = tid >> 3;
  const int c0 = blockIdx.x * 64 + ch * 8;
  const int split = blockIdx.y;
  const int64_t r0 = split * rows_per_split;
  int64_t r1 = r0 + rows_per_split;
  if (r1 > M) r1 = M;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    for (int64_t r = r0 + rl; r < r1; r += kCsRows) {
      float v[8];
      load_vec<DT, 8>(dy + r * C + c0, v);
      if constexpr (GELU) {
        float zv[8];
        load_vec<DT, 8>(z + r * C + c0, zv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_grad(zv[e]);
        store_vec<DT, 8>(dz + r * C + c0, v);
        // the bias gradient sums the values as stored (what the weight GEMMs see)
        load_vec<DT, 8>(dz + r * C + c0, v);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
  __shared__ float red[kCsRows][64 + 1];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][ch * 8 + e] = acc[e];
  __syncthreads();
  if (tid < 64) {
    const int c = blockIdx.x * 64 + tid;
    float s = 0.f;
    for (int r = 0; r < kCsRows; ++r) s += red[r][tid];
    if (c < C) part[(int64_t)split * C + c] = s;
  }
}

template <int DT>
__global__ __launch_bounds__(256) void colsum_final_k(const float* __restrict__ part, int nsplit, int C,
                                                      storage_t<DT>* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int i = 0; i < nsplit; ++i) s += part[(int64_t)i * C + c];
  Elem<DT>::st(out, c, s);
}

}  // namespace

int colsum_splits(int64_t M, int C) {
  const int64_t cb = (C + 63) / 64;
  int64_t s = (512 + cb - 1) / cb;  // ~512 workgroups
  const int64_t maxs = (M + kCsRows - 1) / kCsRows;
  if (s > maxs) s = maxs;
  if (s > 256) s = 256;
  return s < 1 ? 1 : (int)s;
}

void colsum(int dt, const void* dy, const void* z, void* dz, int64_t M, int C, float* part, void* out,
            hipStream_t st) {
  const int ns = colsum_splits(M, C);
  const int64_t rps = (M + ns - 1) / ns;
  const dim3 grid((C + 63) / 64, ns);
  TBAMD_DISPATCH_DT(dt, DTV, {
    using T = storage_t<DTV>;
    if (z)
      colsum_partial_k<DTV, true><<<grid, 256, 0, st>>>((const T*)dy, (const T*)z, (T*)dz, M, C, rps, part);
    else
      colsum_partial_k<DTV, false><<<grid, 256, 0, st>>>((const T*)dy, nullptr, nullptr, M, C, rps, part);
    colsum_final_k<DTV><<<(C + 255) / 256, 256, 0, st>>>(part, ns, C, (T*)out);
  });
}

}  // namespace tbamd
