// Fused softmax cross-entropy (+ label smoothing, ignore_index, class weights
// omitted) with the batch accuracy as a side output, for gfx950.
//
// Reference call sites: cross_entropy(..., label_smoothing=0.1) and
// metrics.accuracy in the img_cls examples
// (/root/reference/examples/img_cls/resnet/resnet.py:61-62,
//  /root/reference/torchbooster/metrics.py:11-27).  SURVEY.md §2.3.1 K9/K10.
//
// forward : one wave per row -> row max, log-sum-exp, Σx, x[label], argmax;
//           per-row loss / lse / correct are written, then a single-block
//           finalize produces mean loss and accuracy (deterministic).
// backward: dlogits = (softmax - (1-ε)·onehot - ε/K) · gout / n_valid.
#include "common.h"
#include "tbamd.h"

namespace tbamd {

template <int DT>
__global__ __launch_bounds__(256) void ce_fwd_k(const storage_t<DT>* __restrict__ logits,
                                                const int64_t* __restrict__ labels, int64_t N, int K,
                                                float smoothing, int64_t ignore_index,
                                                float* __restrict__ row_loss, float* __restrict__ row_lse,
                                                float* __restrict__ row_ok) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const storage_t<DT>* x = logits + row * K;
  float mx = -INFINITY;
  int amx = 0;
  for (int k = lane; k < K; k += 64) {
    const float v = Elem<DT>::ld(x, k);
    if (v > mx) { mx = v; amx = k; }
  }
  // wave argmax (first index wins ties, like torch.argmax)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amx, o, 64);
    if (om > mx || (om == mx && oa < amx)) { mx = om; amx = oa; }
  }
  float se = 0.f, sx = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float v = Elem<DT>::ld(x, k);
    se += __expf(v - mx);
    sx += v;
  }
  se = wave_sum(se);
  sx = wave_sum(sx);
  if (lane == 0) {
    const float lse = mx + __logf(se);
    const int64_t y = labels[row];
    row_lse[row] = lse;
    if (y == ignore_index) {
      row_loss[row] = 0.f;
      row_ok[row] = -1.f;  // marks ignored row
    } else {
      const float xy = Elem<DT>::ld(x, y);
      const float nll = lse - xy;
      const float smooth = lse - sx / (float)K;
      row_loss[row] = (1.f - smoothing) * nll + smoothing * smooth;
      row_ok[row] = (amx == (int)y) ? 1.f : 0.f;
    }
  }
}

// out[0] = mean loss over valid rows, out[1] = correct / N (accuracy over all
// rows, as metrics.accuracy divides by logits.size(0)), out[2] = n_valid
__global__ __launch_bounds__(256) void ce_finalize_k(const float* __restrict__ row_loss,
                                                     const float* __restrict__ row_ok, int64_t N,
                                                     float* __restrict__ out) {
  __shared__ double red[3][4];
  double l = 0.0, c = 0.0, nv = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += 256) {
    const float ok = row_ok[i];
    l += row_loss[i];
    if (ok >= 0.f) { nv += 1.0; c += ok; }
  }
  l = wave_sum_d(l);
  c = wave_sum_d(c);
  nv = wave_sum_d(nv);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = l;
    red[1][threadIdx.x >> 6] = c;
    red[2][threadIdx.x >> 6] = nv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double L = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const double Cc = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const double V = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    out[0] = V > 0 ? (float)(L / V) : NAN;
    out[1] = (float)(Cc / (double)N);
    out[2] = (float)V;
  }
}

template <int DT>
__global__ __launch_bounds__(256) void ce_bwd_k(const storage_t<DT>* __restrict__ logits,
                                                const int64_t* __restrict__ labels,
                                                const float* __restrict__ row_lse,
                                                const float* __restrict__ gout, const float* __restrict__ stats,
                                                int64_t N, int K, float smoothing, int64_t ignore_index,
                                                storage_t<DT>* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t y = labels[row];
  const storage_t<DT>* x = logits + row * K;
  storage_t<DT>* dx = dlogits + row * K;
  if (y == ignore_index) {
    for (int k = lane; k < K; k += 64) Elem<DT>::st(dx, k, 0.f);
    return;
  }
  const float g = gout[0] / stats[2];
  const float lse = row_lse[row];
  const float off = smoothing / (float)K;
  for (int k = lane; k < K; k += 64) {
    const float p = __expf(Elem<DT>::ld(x, k) - lse);
    float d = p - off;
    if (k == (int)y) d -= (1.f - smoothing);
    Elem<DT>::st(dx, k, d * g);
  }
}

void ce_forward(int dt, const void* logits, const int64_t* labels, int64_t N, int K, float smoothing,
                int64_t ignore_index, float* row_loss, float* row_lse, float* row_ok, float* out3,
                hipStream_t st) {
  const int grid = cdiv(N, 4);
  TBAMD_DISPATCH_DT(dt, DT, {
    if (N > 0)
      ce_fwd_k<DT><<<grid, 256, 0, st>>>((const storage_t<DT>*)logits, labels, N, K, smoothing,
                                         ignore_index, row_loss, row_lse, row_ok);
  });
  ce_finalize_k<<<1, 256, 0, st>>>(row_loss, row_ok, N, out3);
}

void ce_backward(int dt, const void* logits, const int64_t* labels, const float* row_lse, const float* gout,
                 const float* stats3, int64_t N, int K, float smoothing, int64_t ignore_index,
                 void* dlogits, hipStream_t st) {
  const int grid = cdiv(N, 4);
  TBAMD_DISPATCH_DT(dt, DT, {
    if (N > 0)
      ce_bwd_k<DT><<<grid, 256, 0, st>>>((const storage_t<DT>*)logits, labels, row_lse, gout, stats3, N,
                                         K, smoothing, ignore_index, (storage_t<DT>*)dlogits);
  });
}

}  // namespace tbamd
