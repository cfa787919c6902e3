// Device-side input pipeline kernel: uint8 NHWC images -> normalised bf16/f32
// NHWC (channels_last) with fused random crop + horizontal flip.
//
// The reference normalises on the CPU in DataLoader workers
// (T.ToTensor + T.Normalize, /root/reference/examples/img_cls/resnet/resnet.py:96-103)
// and ships f32 tensors over PCIe (25 MB/iter at b2048, 154 MB at ResNet-50 b256).
// Here the host ships raw uint8 (4x fewer bytes) through pinned buffers and this
// kernel does crop/flip/normalise on the device.
#include "common.h"
#include "tbamd.h"

namespace tbamd {

// one thread per output pixel (all C channels); C <= 4
template <int ODT>
__global__ __launch_bounds__(256) void u8_crop_flip_norm_k(
    const uint8_t* __restrict__ in, int N, int Hi, int Wi, int C, int Ho, int Wo,
    const int32_t* __restrict__ offs, const uint8_t* __restrict__ flip, const float* __restrict__ mean,
    const float* __restrict__ inv_std, storage_t<ODT>* __restrict__ out) {
  const int64_t total = (int64_t)N * Ho * Wo;
  float m[4], s[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    m[c] = c < C ? mean[c] : 0.f;
    s[c] = c < C ? inv_std[c] : 1.f;
  }
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % Wo);
    const int64_t t = p / Wo;
    const int y = (int)(t % Ho);
    const int n = (int)(t / Ho);
    int oy = 0, ox = 0;
    if (offs) {
      oy = offs[2 * n];
      ox = offs[2 * n + 1];
    }
    const int sx = (flip && flip[n]) ? (Wo - 1 - x) : x;
    int iy = y + oy, ix = sx + ox;
    // reflect padding for crops that reach outside (RandomCrop(padding, reflect))
    if (iy < 0) iy = -iy;
    if (iy >= Hi) iy = 2 * Hi - 2 - iy;
    if (ix < 0) ix = -ix;
    if (ix >= Wi) ix = 2 * Wi - 2 - ix;
    const uint8_t* src = in + (((int64_t)n * Hi + iy) * Wi + ix) * C;
    storage_t<ODT>* dst = out + p * C;
    for (int c = 0; c < C; ++c) Elem<ODT>::st(dst, c, ((float)src[c] * (1.f / 255.f) - m[c]) * s[c]);
  }
}

void u8_crop_flip_normalize(int odt, const uint8_t* in, int N, int Hi, int Wi, int C, int Ho, int Wo,
                            const int32_t* offs, const uint8_t* flip, const float* mean, const float* inv_std,
                            void* out, hipStream_t st) {
  const int64_t total = (int64_t)N * Ho * Wo;
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  TBAMD_DISPATCH_DT(odt, ODT, {
    u8_crop_flip_norm_k<ODT><<<(int)g, 256, 0, st>>>(in, N, Hi, Wi, C, Ho, Wo, offs, flip, mean, inv_std,
                                                     (storage_t<ODT>*)out);
  });
}

}  // namespace tbamd
