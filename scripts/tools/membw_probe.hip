// Streaming-bandwidth probe for the BN passes' access pattern (gfx950): how close to HBM peak can a
// 2-read / 1-write bf16 stream get, and which load/store form gets there?  Standalone (no torch):
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/membw scripts/tools/membw_probe.hip && /tmp/membw
// Variants: the grid-stride 16-B loop the BN kernels use (U rows in flight per lane), with plain or
// non-temporal stores / loads, and a persistent grid (one wave set per CU) vs an oversubscribed one.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(uint4 r, uint4* p) {
  const u32x4 v = {r.x, r.y, r.z, r.w};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

__device__ __forceinline__ uint4 addbf(uint4 a, uint4 b) {
  // bf16 pairs: a + b (round to nearest even), enough arithmetic to be a realistic stream
  uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w}, o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float lo = __uint_as_float(aw[e] << 16) + __uint_as_float(bw[e] << 16);
    float hi = __uint_as_float(aw[e] & 0xffff0000u) + __uint_as_float(bw[e] & 0xffff0000u);
    uint32_t l = __float_as_uint(lo), h = __float_as_uint(hi);
    l = (l + 0x7fffu + ((l >> 16) & 1u)) >> 16;
    h = (h + 0x7fffu + ((h >> 16) & 1u)) & 0xffff0000u;
    o[e] = l | h;
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int U, bool NTS, bool NTL>
__global__ __launch_bounds__(256) void add_k(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                             uint4* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
    uint4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n) {
        if constexpr (NTL) {
          va[u] = ld_nt(a + i);
          vb[u] = ld_nt(b + i);
        } else {
          va[u] = a[i];
          vb[u] = b[i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n) {
        const uint4 r = addbf(va[u], vb[u]);
        if constexpr (NTS) st_nt(r, y + i);
        else y[i] = r;
      }
    }
  }
}

// each block a contiguous chunk (the BN apply kernels' row tiling: rows_per_blk rows per block)
template <bool NTS>
__global__ __launch_bounds__(256) void add_chunk_k(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                   uint4* __restrict__ y, int64_t n, int64_t per_blk) {
  const int64_t s0 = (int64_t)blockIdx.x * per_blk;
  const int64_t s1 = s0 + per_blk < n ? s0 + per_blk : n;
  for (int64_t i = s0 + threadIdx.x; i < s1; i += 256) {
    const uint4 r = addbf(a[i], b[i]);
    if constexpr (NTS) st_nt(r, y + i);
    else y[i] = r;
  }
}

// full grid, U vectors per thread 256 apart inside the block's contiguous 256*U span
template <int U>
__global__ __launch_bounds__(256) void add_span_k(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                  uint4* __restrict__ y, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  uint4 va[U], vb[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n) {
      va[u] = a[base + u * 256];
      vb[u] = b[base + u * 256];
    }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n) y[base + u * 256] = addbf(va[u], vb[u]);
}

template <class F>
static void timeit(const char* name, int blocks, int64_t n, F launch) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CHECK(hipEventRecord(e0));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = 3.0 * (double)n * 16.0 * reps;
  printf("%-28s blocks %6d  %7.3f ms/pass  %6.2f TB/s\n", name, blocks, ms / reps, bytes / (ms * 1e-3) / 1e12);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

template <int U, bool NTS, bool NTL>
static void run(const char* name, const uint4* a, const uint4* b, uint4* y, int64_t n, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) add_k<U, NTS, NTL><<<blocks, 256>>>(a, b, y, n);
  CHECK(hipEventRecord(e0));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) add_k<U, NTS, NTL><<<blocks, 256>>>(a, b, y, n);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = 3.0 * (double)n * 16.0 * reps;
  printf("%-28s blocks %6d  %7.3f ms/pass  %6.2f TB/s\n", name, blocks, ms / reps, bytes / (ms * 1e-3) / 1e12);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main() {
  const int64_t elems = 205520896;  // a ResNet-50 stage-1 256-channel activation at b256 (bf16)
  const int64_t n = elems / 8;      // 16-B vectors
  uint4 *a, *b, *y;
  CHECK(hipMalloc(&a, n * 16));
  CHECK(hipMalloc(&b, n * 16));
  CHECK(hipMalloc(&y, n * 16));
  CHECK(hipMemset(a, 0x3c, n * 16));
  CHECK(hipMemset(b, 0x3d, n * 16));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("device %s, %d CUs, tensor %.1f MB x 3 streams\n", p.name, cus, n * 16 / 1e6);
  for (int occ : {4, 8, 16}) {
    const int blocks = cus * occ;
    char nm[64];
    snprintf(nm, sizeof nm, "U1 plain occ%d", occ);
    run<1, false, false>(nm, a, b, y, n, blocks);
    snprintf(nm, sizeof nm, "U2 plain occ%d", occ);
    run<2, false, false>(nm, a, b, y, n, blocks);
    snprintf(nm, sizeof nm, "U4 plain occ%d", occ);
    run<4, false, false>(nm, a, b, y, n, blocks);
    snprintf(nm, sizeof nm, "U2 nt-store occ%d", occ);
    run<2, true, false>(nm, a, b, y, n, blocks);
    snprintf(nm, sizeof nm, "U4 nt-store occ%d", occ);
    run<4, true, false>(nm, a, b, y, n, blocks);
    snprintf(nm, sizeof nm, "U4 nt-load+store occ%d", occ);
    run<4, true, true>(nm, a, b, y, n, blocks);
  }
  // oversubscribed: one element per thread (the ATen-style grid)
  run<1, false, false>("U1 plain full grid", a, b, y, n, (int)((n + 255) / 256));
  run<1, true, false>("U1 nt-store full grid", a, b, y, n, (int)((n + 255) / 256));
  for (int nb : {1024, 2048, 4096, 8192, 16384}) {
    const int64_t per = (n + nb - 1) / nb;
    char nm[64];
    snprintf(nm, sizeof nm, "chunked plain %d", nb);
    timeit(nm, nb, n, [&] { add_chunk_k<false><<<nb, 256>>>(a, b, y, n, per); });
    snprintf(nm, sizeof nm, "chunked nt-store %d", nb);
    timeit(nm, nb, n, [&] { add_chunk_k<true><<<nb, 256>>>(a, b, y, n, per); });
  }
  {
    int nb2 = (int)((n + 511) / 512), nb4 = (int)((n + 1023) / 1024), nb8 = (int)((n + 2047) / 2048);
    timeit("span U2 full grid", nb2, n, [&] { add_span_k<2><<<nb2, 256>>>(a, b, y, n); });
    timeit("span U4 full grid", nb4, n, [&] { add_span_k<4><<<nb4, 256>>>(a, b, y, n); });
    timeit("span U8 full grid", nb8, n, [&] { add_span_k<8><<<nb8, 256>>>(a, b, y, n); });
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(y));
  return 0;
}
