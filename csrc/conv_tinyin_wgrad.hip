// Weight gradient of a 4x4 / stride-2 / pad-1 conv whose INPUT has 3 channels and whose output has
// 64 (bf16, NHWC) -- and, with the roles swapped, of the 64 -> 3 transposed conv that mirrors it:
//
//   dW[k][r][s][c] = sum_{n,p,q} G[n][p][q][k] * T[n][2p + r - 1][2q + s - 1][c]
//
//   * DCGAN discriminator input conv: T = the RGB image, G = dY of the 64-channel output
//     (ref examples/img_gen/gan/gan.py D);
//   * DCGAN generator output transposed conv (64 -> 3, 4x4 / 2): T = dY of the RGB output,
//     G = the 64-channel input X (ConvTranspose2d weight [in = 64][out = 3][4][4], same physical
//     [k][r][s][c] layout under channels_last) -- the one shape the route tuner still sent to
//     MIOpen (0.059 vs 0.111 ms for the generic kernel).
//
// A GEMM with M = 64 (k), N = 48 (r, s, c), reduced over every output pixel (N * P * Q, half a
// million for DCGAN b128): far too narrow for the channel-tiled wgrad kernels, and MIOpen's
// solvers read the 3-channel operand with 6-byte pixel strides.  Here a workgroup walks output
// rows (n, p): the 64 x 64 G row is staged TRANSPOSED into LDS ([k][q], so the reduction index q
// is contiguous: plain ds_read_b128 fragments), the 48 x 64 im2col slice of T is gathered once per
// row into LDS the same way ([(r, s, c)][q]), and 4 waves (one 16-row k tile each, 3 N tiles)
// run 2 k-steps of v_mfma_f32_16x16x32_bf16 per row.  Rows are split over workgroups; each writes
// its 64 x 48 f32 partial, and a second pass sums them in workgroup order (deterministic).
#include "common.h"
#include "tbamd.h"

namespace tbamd {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kTK = 64, kTC = 3, kTR = 4, kTN = kTR * kTR * kTC;  // 48 (r, s, c) columns
constexpr int kTQ = 64;                                            // output pixels per row
constexpr int kTStride = kTQ + 8;                                  // LDS row pitch (bf16): 144 B

__global__ __launch_bounds__(256) void wgrad_tinyin_k(const uint16_t* __restrict__ T, const uint16_t* __restrict__ G,
                                                      float* __restrict__ part, int N, int P, int H, int W,
                                                      int rows_per_wg) {
  __shared__ __attribute__((aligned(16))) uint16_t gt[kTK * kTStride];  // G row transposed [k][q]
  __shared__ __attribute__((aligned(16))) uint16_t dt[kTN * kTStride];  // T im2col slice [(r,s,c)][q]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nrows = N * P;
  const int row0 = blockIdx.x * rows_per_wg;
  const int row1 = min(row0 + rows_per_wg, nrows);
  f32x4_t acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // software pipeline: row + 1's G chunks and T values are loaded into registers while row's
  // fragments are multiplied (the LDS images are rewritten only after the closing barrier)
  const int tq = tid & 63, tr = tid >> 6;
  uint4 gv[2];
  uint16_t tv[kTR * kTC];
  auto load = [&](int row) {
    const int n = row / P, p = row - n * P;
    const uint16_t* grow = G + (int64_t)row * kTQ * kTK;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int ch = it * 256 + tid;
      gv[it] = *reinterpret_cast<const uint4*>(grow + (ch >> 3) * kTK + (ch & 7) * 8);
    }
    const int y = 2 * p + tr - 1;
    const bool yok = (unsigned)y < (unsigned)H;
    const uint16_t* trow = T + ((int64_t)n * H + (yok ? y : 0)) * W * kTC;
#pragma unroll
    for (int s = 0; s < kTR; ++s) {
      const int x = 2 * tq + s - 1;
      const bool ok = yok && (unsigned)x < (unsigned)W;
#pragma unroll
      for (int c = 0; c < kTC; ++c) tv[s * kTC + c] = ok ? trow[x * kTC + c] : (uint16_t)0;
    }
  };
  if (row0 < row1) load(row0);
  for (int row = row0; row < row1; ++row) {
    // G row transposed into [k][q]; thread (q, r)'s T values into [(r, s, c)][q]
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int ch = it * 256 + tid, q = ch >> 3, k0 = (ch & 7) * 8;
      const uint32_t w4[4] = {gv[it].x, gv[it].y, gv[it].z, gv[it].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gt[(k0 + 2 * e) * kTStride + q] = (uint16_t)(w4[e] & 0xffffu);
        gt[(k0 + 2 * e + 1) * kTStride + q] = (uint16_t)(w4[e] >> 16);
      }
    }
#pragma unroll
    for (int i = 0; i < kTR * kTC; ++i) dt[(tr * kTR * kTC + i) * kTStride + tq] = tv[i];
    __syncthreads();
    if (row + 1 < row1) load(row + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8_t af =
          __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(gt + (wave * 16 + fr) * kTStride + ks * 32 + fq * 8));
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const bf16x8_t bf =
            __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(dt + (j * 16 + fr) * kTStride + ks * 32 + fq * 8));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave read gt / dt before the next row rewrites them
  }
  // partial [wg][k][n]: lane (fr, fq) holds C[k = 16 wave + 4 fq + e][n = 16 j + fr]
  float* out = part + (int64_t)blockIdx.x * kTK * kTN;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) out[(wave * 16 + fq * 4 + e) * kTN + j * 16 + fr] = acc[j][e];
}

// dW (bf16) = sum over the partials in a fixed order: a block owns 16 outputs; 16 thread groups
// sum interleaved partials (8 loads in flight each), combined in group order through LDS
__global__ __launch_bounds__(256) void wgrad_tinyin_reduce_k(const float* __restrict__ part, int nparts,
                                                             uint16_t* __restrict__ dw) {
  __shared__ float red[16][16];
  const int o = blockIdx.x * 16 + (threadIdx.x & 15), g = threadIdx.x >> 4;
  float s = 0.f;
  int w = g;
#pragma unroll 1
  for (; w + 7 * 16 < nparts; w += 8 * 16) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(w + u * 16) * kTK * kTN + o];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; w < nparts; w += 16) s += part[(int64_t)w * kTK * kTN + o];
  red[g][threadIdx.x & 15] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
    dw[o] = f2bf(t);
  }
}

}  // namespace

bool wgrad_tinyin_supported(int C, int K, int R, int S, int stride, int pad, int P, int Q, int H, int W) {
  return C == kTC && K == kTK && R == kTR && S == kTR && stride == 2 && pad == 1 && Q == kTQ && H == 2 * P &&
         W == 2 * Q;
}

// ~1024 workgroups (4 per CU, 8 output rows each at DCGAN b128), at least 4 rows each
int wgrad_tinyin_parts(int N, int P) {
  const int rows = N * P;
  const int rpw = rows >= 1024 * 4 ? cdiv(rows, 1024) : 4;
  return cdiv(rows, rpw);
}

void wgrad_tinyin(const void* T, const void* G, void* dw, float* part, int N, int P, int H, int W, hipStream_t st) {
  const int rows = N * P;
  const int nparts = wgrad_tinyin_parts(N, P);
  const int rpw = cdiv(rows, nparts);
  wgrad_tinyin_k<<<nparts, 256, 0, st>>>((const uint16_t*)T, (const uint16_t*)G, part, N, P, H, W, rpw);
  wgrad_tinyin_reduce_k<<<kTK * kTN / 16, 256, 0, st>>>(part, nparts, (uint16_t*)dw);
}

}  // namespace tbamd
