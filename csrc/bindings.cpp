// Python bindings for the torchbooster_amd native library (_C).
//
// Tensors are validated here (device, dtype, contiguity, 16-B alignment for
// the vectorised paths), workspaces come from the PyTorch caching allocator,
// and every launch goes onto the caller's current HIP stream, so all ops are
// hipGraph-capturable.
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "tbamd.h"
#include "runtime.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dt_code(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return tbamd::kF32;
    case at::kBFloat16: return tbamd::kBF16;
    case at::kHalf: return tbamd::kF16;
    default: TORCH_CHECK(false, "torchbooster_amd: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "torchbooster_amd: ", name, " must be a GPU tensor");
}

const float* fptr(const optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "expected contiguous f32 tensor");
  return t->data_ptr<float>();
}
float* fptr_mut(const optional<Tensor>& t) { return const_cast<float*>(fptr(t)); }

// [M, C] view requirement: contiguous, and 16-B aligned for the 8-wide path.
Tensor as_rows(const Tensor& t) {
  Tensor c = t.contiguous();
  if (reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 != 0) c = c.clone();
  return c;
}

// ---------------------------------------------------------------- BatchNorm
// ReLU-after-residual bit mask [M, C/8] (uint8) when requested and applicable
static Tensor make_mask(const Tensor& x, const Tensor& res, int64_t act, bool want) {
  if (!want || !res.defined() || act != 1 || x.size(1) % 8 != 0) return Tensor();
  return at::empty({x.size(0), x.size(1) / 8}, x.options().dtype(at::kByte));
}

static int64_t* nbt_ptr(const optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() == 1 && t->is_cuda(), "num_batches_tracked: int64 scalar");
  return t->data_ptr<int64_t>();
}

std::vector<Tensor> bn_forward(const Tensor& x_, const optional<Tensor>& weight,
                               const optional<Tensor>& bias, const optional<Tensor>& running_mean,
                               const optional<Tensor>& running_var, bool training, double momentum,
                               double eps, const optional<Tensor>& residual, int64_t act, double slope,
                               const optional<Tensor>& num_batches_tracked, bool want_mask) {
  check_cuda(x_, "x");
  TORCH_CHECK(x_.dim() == 2, "bn_forward expects [M, C]");
  const at::DeviceGuard guard(x_.device());
  Tensor x = as_rows(x_);
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  Tensor scale = at::empty({C}, fopt), shift = at::empty({C}, fopt);
  auto st = cur_stream();
  Tensor wf, bf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  const float* g = wf.defined() ? wf.data_ptr<float>() : nullptr;
  const float* b = bf.defined() ? bf.data_ptr<float>() : nullptr;
  if (training) {
    TORCH_CHECK(M > 0, "bn_forward: empty batch in training mode");
    const int nblk = tbamd::bn_partial_blocks(M, C);
    Tensor ws = at::empty({2, (int64_t)nblk, C}, fopt);
    Tensor fws = at::empty({tbamd::colsum_workspace(nblk, C)}, x.options().dtype(at::kDouble));
    tbamd::bn_forward_train(dt_code(x), x.data_ptr(), M, C, g, b, fptr_mut(running_mean),
                            fptr_mut(running_var), nbt_ptr(num_batches_tracked), (float)momentum, (float)eps,
                            ws[0].data_ptr<float>(), ws[1].data_ptr<float>(), nblk, fws.data_ptr<double>(),
                            mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                            shift.data_ptr<float>(), st);
  } else {
    TORCH_CHECK(running_mean.has_value() && running_var.has_value(), "eval BN needs running stats");
    tbamd::bn_eval_coeffs(C, g, b, fptr(running_mean), fptr(running_var), (float)eps, mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(), st);
  }
  Tensor res;
  if (residual.has_value() && residual->defined()) {
    res = as_rows(*residual);
    TORCH_CHECK(res.sizes() == x.sizes() && res.scalar_type() == x.scalar_type(), "residual mismatch");
  }
  Tensor y = at::empty_like(x);
  Tensor mask = make_mask(x, res, act, want_mask);
  if (M > 0)
    tbamd::bn_apply(dt_code(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr,
                    scale.data_ptr<float>(), shift.data_ptr<float>(), M, C, (int)act, (float)slope,
                    y.data_ptr(), mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, st);
  return {y, mean, invstd, scale, shift, mask};
}

std::vector<Tensor> bn_backward(const Tensor& dy_, const Tensor& y_, const Tensor& x_,
                                const optional<Tensor>& residual, const optional<Tensor>& weight,
                                const Tensor& mean, const Tensor& invstd, const Tensor& scale,
                                const Tensor& shift, bool training, int64_t act, double slope,
                                bool need_dres, const optional<Tensor>& dgamma_out,
                                const optional<Tensor>& dbeta_out, const optional<Tensor>& mask) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor x = as_rows(x_);
  Tensor dy = as_rows(dy_.to(x.scalar_type()));
  Tensor y = as_rows(y_);
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor res;
  if (residual.has_value() && residual->defined()) res = as_rows(*residual);
  Tensor wf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  const int nblk = tbamd::bn_partial_blocks(M, C);
  Tensor ws = at::empty({2, (int64_t)nblk, C}, fopt);
  Tensor fws = at::empty({tbamd::colsum_workspace(nblk, C)}, x.options().dtype(at::kDouble));
  Tensor coef = at::empty({3, C}, fopt);
  auto out_or_new = [&](const optional<Tensor>& o) {
    if (o.has_value() && o->defined()) {  // zero-copy gradient slot
      TORCH_CHECK(o->scalar_type() == at::kFloat && o->numel() == C && o->is_contiguous(), "bn_backward: out");
      return *o;
    }
    return at::empty({C}, fopt);
  };
  Tensor dgamma = out_or_new(dgamma_out), dbeta = out_or_new(dbeta_out);
  Tensor dx = at::empty_like(x);
  const uint8_t* maskin = nullptr;
  if (mask.has_value() && mask->defined()) {
    // act 1: this BN's own ReLU-after-residual mask; act 0: dy is a carrier whose mask comes from the
    // block-output BN downstream (ops/norm.py ResidualGradLink carrier: the downsample branch's BN)
    TORCH_CHECK((act == 1 || act == 0) && C % 8 == 0 && mask->numel() == M * (C / 8) &&
                    mask->scalar_type() == at::kByte,
                "bn_backward: mask needs ReLU or no activation, C % 8 == 0 and [M, C/8] bytes");
    maskin = mask->data_ptr<uint8_t>();
    need_dres = false;  // the residual's consumer applies the mask to dy itself
  }
  Tensor dres;
  if (need_dres) dres = at::empty_like(x);
  if (M > 0)
    tbamd::bn_backward(dt_code(x), dy.data_ptr(), y.data_ptr(), x.data_ptr(),
                       res.defined() ? res.data_ptr() : nullptr, M, C, (int)act, (float)slope,
                       wf.defined() ? wf.data_ptr<float>() : nullptr, mean.data_ptr<float>(),
                       invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                       training ? 1 : 0, ws[0].data_ptr<float>(), ws[1].data_ptr<float>(), nblk,
                       fws.data_ptr<double>(), coef.data_ptr<float>(), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                       need_dres ? dres.data_ptr() : nullptr, dx.data_ptr(), maskin, cur_stream());
  else {
    dgamma.zero_();
    dbeta.zero_();
  }
  return {dx, dgamma, dbeta, dres};
}

// BN backward whose partial sums were emitted by the dgrad epilogue (conv2d_fwd bnb_mode)
std::vector<Tensor> bn_backward_from_partials(const Tensor& dy_, const Tensor& x_, const Tensor& part,
                                              const optional<Tensor>& weight, const Tensor& mean,
                                              const Tensor& invstd, const Tensor& scale, const Tensor& shift,
                                              bool training, int64_t act, double slope,
                                              const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out,
                                              const optional<Tensor>& mask, bool want_dres,
                                              const optional<Tensor>& ds_x, const optional<Tensor>& ds_mean) {
  // want_dres (ReLU-after-residual with saved mask bits): also returns dres = dy * mask
  // ds_x / ds_mean (the residual is a downsample branch: its BN input rows and batch mean): also
  // returns that BN's backward partials [rows][2][C] from this apply pass (ops/norm.py carrier)
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor x = as_rows(x_);
  Tensor dy = as_rows(dy_.to(x.scalar_type()));
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(part.dim() == 3 && part.size(1) == 2 && part.size(2) == C, "bn_backward_from_partials: part");
  auto fopt = x.options().dtype(at::kFloat);
  Tensor wf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  auto out_or_new = [&](const optional<Tensor>& o) {
    if (o.has_value() && o->defined()) {
      TORCH_CHECK(o->scalar_type() == at::kFloat && o->numel() == C && o->is_contiguous(), "bn_backward: out");
      return *o;
    }
    return at::empty({C}, fopt);
  };
  Tensor dgamma = out_or_new(dgamma_out), dbeta = out_or_new(dbeta_out);
  Tensor coef = at::empty({3, C}, fopt);
  Tensor fws = at::empty({tbamd::colsum_workspace((int)part.size(0), C)}, x.options().dtype(at::kDouble));
  const uint8_t* maskin = nullptr;
  if (mask.has_value() && mask->defined()) maskin = mask->data_ptr<uint8_t>();
  Tensor dx = at::empty_like(x);
  Tensor dres;
  if (want_dres) {
    TORCH_CHECK(maskin != nullptr && act == 1 && C % 8 == 0, "bn_backward_from_partials: dres needs the ReLU mask");
    dres = at::empty_like(x);
  }
  Tensor dsx, dsp;
  if (ds_x.has_value() && ds_x->defined()) {
    dsx = as_rows(*ds_x);
    TORCH_CHECK(dsx.scalar_type() == x.scalar_type() && dsx.size(0) == M && dsx.size(1) == C && maskin &&
                    act == 1 && C % 8 == 0 && !want_dres && ds_mean.has_value() && ds_mean->defined() &&
                    ds_mean->scalar_type() == at::kFloat && ds_mean->numel() == C && ds_mean->is_contiguous(),
                "bn_backward_from_partials: downsample partials need rows like x, f32 [C] mean, the ReLU mask");
    dsp = at::empty({tbamd::bn_bwd_dsp_rows(M, C), 2, C}, fopt);
  }
  tbamd::bn_backward_from_partials(dt_code(x), dy.data_ptr(), x.data_ptr(), x.data_ptr(), M, C, (int)act,
                                   (float)slope, wf.defined() ? wf.data_ptr<float>() : nullptr,
                                   mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                                   shift.data_ptr<float>(), training ? 1 : 0, part.data_ptr<float>(),
                                   (int)part.size(0), fws.data_ptr<double>(), coef.data_ptr<float>(),
                                   dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), dx.data_ptr(), maskin,
                                   cur_stream(), dres.defined() ? dres.data_ptr() : nullptr,
                                   dsx.defined() ? dsx.data_ptr() : nullptr,
                                   dsx.defined() ? ds_mean->data_ptr<float>() : nullptr,
                                   dsx.defined() ? dsp.data_ptr<float>() : nullptr);
  return {dx, dgamma, dbeta, dres, dsp};
}

// ------------------------------------------------------ GroupNorm / InstanceNorm
// x: [N*HW, C] rows (NHWC), statistics per (sample, group)
std::vector<Tensor> gn_forward(const Tensor& x_, int64_t N, int64_t G, const optional<Tensor>& weight,
                               const optional<Tensor>& bias, double eps, const optional<Tensor>& residual,
                               int64_t act, double slope) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = as_rows(x_);
  const int C = (int)x.size(1);
  TORCH_CHECK(N > 0 && x.size(0) % N == 0, "gn_forward: rows not divisible by N");
  TORCH_CHECK(G > 0 && C % G == 0, "gn_forward: C % G != 0");
  const int64_t HW = x.size(0) / N;
  auto fopt = x.options().dtype(at::kFloat);
  Tensor wf, bf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  Tensor coeff = at::empty({4, N, C}, fopt);  // mean, invstd, scale, shift (per n, c)
  const int nblk = tbamd::norm_partial_blocks(HW, C, (int)N);
  Tensor ws = at::empty({2, N, (int64_t)nblk, C}, fopt);
  Tensor row0 = at::empty({N, C}, fopt);
  auto st = cur_stream();
  tbamd::gn_forward_stats(dt_code(x), x.data_ptr(), (int)N, HW, C, (int)G, wf.defined() ? wf.data_ptr<float>() : nullptr,
                          bf.defined() ? bf.data_ptr<float>() : nullptr, (float)eps, ws[0].data_ptr<float>(),
                          ws[1].data_ptr<float>(), row0.data_ptr<float>(), nblk, coeff[0].data_ptr<float>(),
                          coeff[1].data_ptr<float>(), coeff[2].data_ptr<float>(), coeff[3].data_ptr<float>(), st);
  Tensor res;
  if (residual.has_value() && residual->defined()) res = as_rows(*residual);
  Tensor y = at::empty_like(x);
  tbamd::norm_apply(dt_code(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, coeff[2].data_ptr<float>(),
                    coeff[3].data_ptr<float>(), (int)N, HW, C, (int)act, (float)slope, y.data_ptr(), st);
  return {y, coeff};
}

// zero-copy gradient slot of an affine norm parameter ([C] f32 contiguous) or a new tensor
static Tensor slot_or_new(const optional<Tensor>& o, int64_t C, const at::TensorOptions& fopt, const char* what) {
  if (o.has_value() && o->defined()) {
    TORCH_CHECK(o->scalar_type() == at::kFloat && o->numel() == C && o->is_contiguous(), what, ": gradient slot");
    return *o;
  }
  return at::empty({C}, fopt);
}

std::vector<Tensor> gn_backward(const Tensor& dy_, const Tensor& y_, const Tensor& x_, const optional<Tensor>& residual,
                                const optional<Tensor>& weight, const Tensor& coeff, int64_t N, int64_t G, int64_t act,
                                double slope, bool need_dres, const optional<Tensor>& dgamma_out,
                                const optional<Tensor>& dbeta_out) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor x = as_rows(x_);
  Tensor dy = as_rows(dy_.to(x.scalar_type()));
  Tensor y = as_rows(y_);
  const int C = (int)x.size(1);
  const int64_t HW = x.size(0) / N;
  auto fopt = x.options().dtype(at::kFloat);
  Tensor res;
  if (residual.has_value() && residual->defined()) res = as_rows(*residual);
  Tensor wf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  const int nblk = tbamd::norm_partial_blocks(HW, C, (int)N);
  Tensor ws = at::empty({2, N, (int64_t)nblk, C}, fopt);
  Tensor coef = at::empty({N, 3, C}, fopt);
  Tensor nc = at::empty({2, N, C}, fopt);
  Tensor dgamma = slot_or_new(dgamma_out, C, fopt, "gn_backward"), dbeta = slot_or_new(dbeta_out, C, fopt, "gn_backward");
  Tensor dx = at::empty_like(x);
  Tensor dres;
  if (need_dres) dres = at::empty_like(x);
  tbamd::gn_backward(dt_code(x), dy.data_ptr(), y.data_ptr(), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr,
                     (int)N, HW, C, (int)G, (int)act, (float)slope, wf.defined() ? wf.data_ptr<float>() : nullptr,
                     coeff[0].data_ptr<float>(), coeff[1].data_ptr<float>(), coeff[2].data_ptr<float>(),
                     coeff[3].data_ptr<float>(), ws[0].data_ptr<float>(), ws[1].data_ptr<float>(), nblk,
                     coef.data_ptr<float>(), nc[0].data_ptr<float>(), nc[1].data_ptr<float>(),
                     dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), need_dres ? dres.data_ptr() : nullptr,
                     dx.data_ptr(), cur_stream());
  return {dx, dgamma, dbeta, dres};
}

// --------------------------------------------------------------- LayerNorm
// returns {y, xsum (x + residual, or undefined), mean, rstd}
std::vector<Tensor> ln_forward(const Tensor& x_, const optional<Tensor>& residual, const optional<Tensor>& weight,
                               const optional<Tensor>& bias, double eps) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = as_rows(x_);
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0 && C <= 4096, "ln_forward: C % 8 == 0 and C <= 4096");
  Tensor res, xsum;
  if (residual.has_value() && residual->defined()) {
    res = as_rows(residual->to(x.scalar_type()));
    xsum = at::empty_like(x);
  }
  Tensor wf, bf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  auto fopt = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({M}, fopt), rstd = at::empty({M}, fopt);
  Tensor y = at::empty_like(x);
  if (M > 0)
    tbamd::ln_forward(dt_code(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr,
                      wf.defined() ? wf.data_ptr<float>() : nullptr, bf.defined() ? bf.data_ptr<float>() : nullptr, M,
                      C, (float)eps, y.data_ptr(), xsum.defined() ? xsum.data_ptr() : nullptr, mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), cur_stream());
  return {y, xsum, mean, rstd};
}

// dadd (optional, same shape as x): added to dx in the kernel (residual-stream gradient)
std::vector<Tensor> ln_backward(const Tensor& dy_, const Tensor& x_, const optional<Tensor>& weight,
                                const Tensor& mean, const Tensor& rstd, const optional<Tensor>& dadd_,
                                const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor x = as_rows(x_);
  Tensor dy = as_rows(dy_.to(x.scalar_type()));
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  Tensor wf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  auto fopt = x.options().dtype(at::kFloat);
  const int nblk = tbamd::ln_bwd_blocks(M);
  Tensor ws = at::empty({2, (int64_t)nblk, C}, fopt);
  Tensor dg = slot_or_new(dgamma_out, C, fopt, "ln_backward"), db = slot_or_new(dbeta_out, C, fopt, "ln_backward");
  Tensor dx = at::empty_like(x);
  Tensor dadd;
  if (dadd_.has_value() && dadd_->defined()) {
    dadd = as_rows(dadd_->to(x.scalar_type()));
    TORCH_CHECK(dadd.size(0) == M && dadd.size(1) == C, "ln_backward: dadd shape");
  }
  if (M > 0)
    tbamd::ln_backward(dt_code(x), dy.data_ptr(), x.data_ptr(), dadd.defined() ? dadd.data_ptr() : nullptr,
                       wf.defined() ? wf.data_ptr<float>() : nullptr,
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), M, C, dx.data_ptr(), ws[0].data_ptr<float>(),
                       ws[1].data_ptr<float>(), nblk, dg.data_ptr<float>(), db.data_ptr<float>(), cur_stream());
  else {
    dg.zero_();
    db.zero_();
  }
  return {dx, dg, db};
}

// ----------------------------------------------------------- cross entropy
std::vector<Tensor> ce_forward(const Tensor& logits_, const Tensor& labels_, double smoothing,
                               int64_t ignore_index) {
  check_cuda(logits_, "logits");
  const at::DeviceGuard guard(logits_.device());
  TORCH_CHECK(logits_.dim() == 2, "ce_forward expects [N, K] logits");
  Tensor logits = logits_.contiguous();
  Tensor labels = labels_.to(at::kLong).contiguous();
  const int64_t N = logits.size(0);
  const int K = (int)logits.size(1);
  auto fopt = logits.options().dtype(at::kFloat);
  Tensor rows = at::empty({3, N}, fopt);
  Tensor out = at::empty({3}, fopt);
  tbamd::ce_forward(dt_code(logits), logits.data_ptr(), labels.data_ptr<int64_t>(), N, K, (float)smoothing,
                    ignore_index, rows[0].data_ptr<float>(), rows[1].data_ptr<float>(),
                    rows[2].data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return {out, rows[1]};
}

Tensor ce_backward(const Tensor& logits_, const Tensor& labels_, const Tensor& row_lse, const Tensor& gout,
                   const Tensor& stats, double smoothing, int64_t ignore_index) {
  const at::DeviceGuard guard(logits_.device());
  Tensor logits = logits_.contiguous();
  Tensor labels = labels_.to(at::kLong).contiguous();
  Tensor g = gout.to(at::kFloat).contiguous();
  Tensor dl = at::empty_like(logits);
  tbamd::ce_backward(dt_code(logits), logits.data_ptr(), labels.data_ptr<int64_t>(),
                     row_lse.data_ptr<float>(), g.data_ptr<float>(), stats.data_ptr<float>(),
                     logits.size(0), (int)logits.size(1), (float)smoothing, ignore_index, dl.data_ptr(),
                     cur_stream());
  return dl;
}

// ------------------------------------------- small fused losses / resampling
static Tensor aux_part(const Tensor& like) {
  return at::empty({tbamd::aux_partials()}, like.options().dtype(at::kFloat));
}
static Tensor f32_scalar(const Tensor& g) { return g.to(at::kFloat).reshape({1}).contiguous(); }

// x: 4-D, NCHW-contiguous or channels_last
Tensor tv_forward(const Tensor& x_) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.dim() == 4, "total_variation expects [N, C, H, W]");
  const bool cl = !x_.is_contiguous() && x_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor x = cl ? x_ : x_.contiguous();
  Tensor out = at::empty({}, x.options().dtype(at::kFloat));
  tbamd::tv_forward(dt_code(x), x.data_ptr(), x.numel(), (int)x.size(2), (int)x.size(3), cl ? (int)x.size(1) : 1,
                    aux_part(x).data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

Tensor tv_backward(const Tensor& x_, const Tensor& gout) {
  const at::DeviceGuard guard(x_.device());
  const bool cl = !x_.is_contiguous() && x_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor x = cl ? x_ : x_.contiguous();
  Tensor dx = at::empty_like(x);
  Tensor g = f32_scalar(gout);
  tbamd::tv_backward(dt_code(x), x.data_ptr(), g.data_ptr<float>(), x.numel(), (int)x.size(2), (int)x.size(3),
                     cl ? (int)x.size(1) : 1, dx.data_ptr(), cur_stream());
  return dx;
}

// y = act(x) / dx = dy * act'(x) on the storage of x (any layout the two share; numel % 8 == 0)
Tensor act_fwd(const Tensor& x_, int64_t act, double slope) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  const bool cl = x_.dim() == 4 && !x_.is_contiguous() && x_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor x = cl ? x_ : x_.contiguous();
  TORCH_CHECK(x.numel() % 8 == 0, "act_fwd: numel must be a multiple of 8");
  Tensor y = at::empty_like(x);
  tbamd::act_forward(dt_code(x), (int)act, x.data_ptr(), y.data_ptr(), x.numel(), (float)slope, cur_stream());
  return y;
}

Tensor act_bwd(const Tensor& x_, const Tensor& dy_, int64_t act, double slope) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  const bool cl = x_.dim() == 4 && !x_.is_contiguous() && x_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor x = cl ? x_ : x_.contiguous();
  Tensor dy = cl ? dy_.contiguous(at::MemoryFormat::ChannelsLast) : dy_.contiguous();
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides() && dy.scalar_type() == x.scalar_type(),
              "act_bwd: dy must match x");
  Tensor dx = at::empty_like(x);
  tbamd::act_backward(dt_code(x), (int)act, x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), (float)slope,
                      cur_stream());
  return dx;
}

Tensor hinge_forward(const Tensor& x_, double margin, double sign) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous();
  Tensor out = at::empty({}, x.options().dtype(at::kFloat));
  tbamd::hinge_forward(dt_code(x), x.data_ptr(), x.numel(), (float)margin, (float)sign,
                       aux_part(x).data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

Tensor hinge_backward(const Tensor& x_, const Tensor& gout, double margin, double sign) {
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous();
  Tensor dx = at::empty_like(x);
  Tensor g = f32_scalar(gout);
  tbamd::hinge_backward(dt_code(x), x.data_ptr(), g.data_ptr<float>(), x.numel(), (float)margin, (float)sign,
                        dx.data_ptr(), cur_stream());
  return dx;
}

Tensor bce_logits_forward(const Tensor& x_, const Tensor& y_) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.numel() == y_.numel(), "bce_with_logits: input and target sizes differ");
  Tensor x = x_.contiguous();
  Tensor y = y_.to(x.scalar_type()).contiguous();
  Tensor out = at::empty({}, x.options().dtype(at::kFloat));
  tbamd::bce_logits_forward(dt_code(x), x.data_ptr(), y.data_ptr(), x.numel(), aux_part(x).data_ptr<float>(),
                            out.data_ptr<float>(), cur_stream());
  return out;
}

Tensor bce_logits_backward(const Tensor& x_, const Tensor& y_, const Tensor& gout) {
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous();
  Tensor y = y_.to(x.scalar_type()).contiguous();
  Tensor dx = at::empty_like(x);
  Tensor g = f32_scalar(gout);
  tbamd::bce_logits_backward(dt_code(x), x.data_ptr(), y.data_ptr(), g.data_ptr<float>(), x.numel(),
                             dx.data_ptr(), cur_stream());
  return dx;
}

Tensor kld_forward(const Tensor& mu_, const Tensor& lv_) {
  check_cuda(mu_, "mu");
  const at::DeviceGuard guard(mu_.device());
  TORCH_CHECK(mu_.sizes() == lv_.sizes() && mu_.dim() == 2, "kld expects matching [B, D] mu / log_var");
  Tensor mu = mu_.contiguous();
  Tensor lv = lv_.to(mu.scalar_type()).contiguous();
  Tensor out = at::empty({}, mu.options().dtype(at::kFloat));
  tbamd::kld_forward(dt_code(mu), mu.data_ptr(), lv.data_ptr(), mu.numel(), mu.size(0),
                     aux_part(mu).data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

std::vector<Tensor> kld_backward(const Tensor& mu_, const Tensor& lv_, const Tensor& gout) {
  const at::DeviceGuard guard(mu_.device());
  Tensor mu = mu_.contiguous();
  Tensor lv = lv_.to(mu.scalar_type()).contiguous();
  Tensor dmu = at::empty_like(mu), dlv = at::empty_like(lv);
  Tensor g = f32_scalar(gout);
  tbamd::kld_backward(dt_code(mu), mu.data_ptr(), lv.data_ptr(), g.data_ptr<float>(), mu.numel(), mu.size(0),
                      dmu.data_ptr(), dlv.data_ptr(), cur_stream());
  return {dmu, dlv};
}

// x [N, C, H, W] (NCHW-contiguous or channels_last) -> f32 mean, unbiased std+eps: [N, C]
std::vector<Tensor> mean_std_forward(const Tensor& x_, double eps) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.dim() == 4, "mean_std expects [N, C, H, W]");
  const bool cl = !x_.is_contiguous() && x_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor x = cl ? x_ : x_.contiguous();
  const int N = (int)x.size(0), C = (int)x.size(1);
  const int64_t S = x.size(2) * x.size(3);
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({N, C}, fo), sd = at::empty({N, C}, fo);
  const int64_t wsz = tbamd::mean_std_workspace(N, C, S, cl);
  Tensor ws = wsz > 0 ? at::empty({wsz}, fo) : Tensor();
  if (x.numel() > 0)
    tbamd::mean_std_forward(dt_code(x), x.data_ptr(), N, C, S, cl, (float)eps, mean.data_ptr<float>(),
                            sd.data_ptr<float>(), cur_stream(), wsz > 0 ? ws.data_ptr<float>() : nullptr);
  return {mean, sd};
}

Tensor mean_std_backward(const Tensor& x_, const Tensor& mean, const Tensor& sd, const Tensor& dmean_,
                         const Tensor& dstd_) {
  const at::DeviceGuard guard(x_.device());
  const bool cl = !x_.is_contiguous() && x_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor x = cl ? x_ : x_.contiguous();
  Tensor dmean = dmean_.to(at::kFloat).contiguous(), dstd = dstd_.to(at::kFloat).contiguous();
  Tensor dx = at::empty_like(x);
  Tensor coef = at::empty({2 * x.size(0) * x.size(1)}, mean.options());
  if (x.numel() > 0)
    tbamd::mean_std_backward(dt_code(x), x.data_ptr(), mean.data_ptr<float>(), sd.data_ptr<float>(),
                             dmean.data_ptr<float>(), dstd.data_ptr<float>(), (int)x.size(0), (int)x.size(1),
                             x.size(2) * x.size(3), cl, dx.data_ptr(), cur_stream(), coef.data_ptr<float>());
  return dx;
}

// NHWC-only (channels_last) resampling; returns a channels_last [N, C, Ho, Wo] tensor
static Tensor nhwc_in(const Tensor& x) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "expected a channels_last [N, C, H, W] tensor");
  return x;
}

Tensor reflect_pad_forward(const Tensor& x_, int64_t pl, int64_t pr, int64_t pt, int64_t pb) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = nhwc_in(x_);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(pt < H && pb < H && pl < W && pr < W && pl >= 0 && pr >= 0 && pt >= 0 && pb >= 0,
              "reflection padding must be smaller than the input size");
  Tensor y = at::empty({N, C, H + pt + pb, W + pl + pr}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (y.numel() > 0)
    tbamd::reflect_pad_forward(dt_code(x), x.data_ptr(), N, H, W, C, (int)pt, (int)pb, (int)pl, (int)pr,
                               y.data_ptr(), cur_stream());
  return y;
}

Tensor reflect_pad_backward(const Tensor& dy_, int64_t H, int64_t W, int64_t pl, int64_t pr, int64_t pt,
                            int64_t pb) {
  const at::DeviceGuard guard(dy_.device());
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (dx.numel() > 0)
    tbamd::reflect_pad_backward(dt_code(dy), dy.data_ptr(), N, (int)H, (int)W, C, (int)pt, (int)pb, (int)pl,
                                (int)pr, dx.data_ptr(), cur_stream());
  return dx;
}

Tensor upsample_nearest_forward(const Tensor& x_, int64_t f) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = nhwc_in(x_);
  TORCH_CHECK(f >= 1, "upsample factor must be >= 1");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  Tensor y = at::empty({N, C, H * f, W * f}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (y.numel() > 0)
    tbamd::upsample_nearest_forward(dt_code(x), x.data_ptr(), N, H, W, C, (int)f, y.data_ptr(), cur_stream());
  return y;
}

Tensor upsample_nearest_backward(const Tensor& dy_, int64_t f) {
  const at::DeviceGuard guard(dy_.device());
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)dy.size(0), C = (int)dy.size(1), H = (int)(dy.size(2) / f), W = (int)(dy.size(3) / f);
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (dx.numel() > 0)
    tbamd::upsample_nearest_backward(dt_code(dy), dy.data_ptr(), N, H, W, C, (int)f, dx.data_ptr(),
                                     cur_stream());
  return dx;
}

// -------------------------------------------------------------- optimizers
void adamw_mt(const Tensor& chunks, int64_t nchunks, const Tensor& table, int64_t pdt, int64_t gdt,
              bool master, bool ema, bool amsgrad, double lr, double beta1, double beta2, double eps,
              double wd, double bc1, double bc2_sqrt, double ema_decay, const optional<Tensor>& clip_coef,
              const optional<Tensor>& inv_scale, const optional<Tensor>& found_inf,
              const optional<Tensor>& hyper) {
  const at::DeviceGuard guard(table.device());
  tbamd::adamw_mt((int)pdt, (int)gdt, master, ema, amsgrad, chunks.data_ptr(), (int)nchunks,
                  table.data_ptr<int64_t>(), (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd,
                  (float)bc1, (float)bc2_sqrt, (float)ema_decay, fptr(clip_coef), fptr(inv_scale),
                  fptr(found_inf), cur_stream(), fptr(hyper));
}

void sgd_mt(const Tensor& chunks, int64_t nchunks, const Tensor& table, int64_t pdt, int64_t gdt,
            bool master, double momentum, double dampening, bool nesterov, double wd, double lr,
            bool first_step, const optional<Tensor>& clip_coef, const optional<Tensor>& inv_scale,
            const optional<Tensor>& found_inf, const optional<Tensor>& hyper) {
  const at::DeviceGuard guard(table.device());
  tbamd::sgd_mt((int)pdt, (int)gdt, master, (float)momentum, (float)dampening, nesterov, (float)wd,
                (float)lr, first_step ? 1 : 0, chunks.data_ptr(), (int)nchunks, table.data_ptr<int64_t>(),
                fptr(clip_coef), fptr(inv_scale), fptr(found_inf), cur_stream(), fptr(hyper));
}

// returns [norm, clip_coef, nonfinite]
Tensor grad_norm_mt(const Tensor& chunks, int64_t nchunks, const Tensor& table, int64_t gdt,
                    double max_norm, const optional<Tensor>& inv_scale, const Tensor& partial) {
  const at::DeviceGuard guard(table.device());
  Tensor out = at::empty({3}, table.options().dtype(at::kFloat));
  tbamd::grad_norm_mt((int)gdt, chunks.data_ptr(), (int)nchunks, table.data_ptr<int64_t>(),
                      (float)max_norm, fptr(inv_scale), partial.data_ptr<float>(), out.data_ptr<float>(),
                      cur_stream());
  return out;
}

Tensor grad_norm_multi(const std::vector<Tensor>& chunks, const std::vector<int64_t>& nchunks,
                       const std::vector<Tensor>& tables, const std::vector<int64_t>& gdts, double max_norm,
                       const optional<Tensor>& inv_scale) {
  TORCH_CHECK(!tables.empty() && chunks.size() == tables.size() && nchunks.size() == tables.size() &&
                  gdts.size() == tables.size(), "grad_norm_multi: list sizes");
  const at::DeviceGuard guard(tables[0].device());
  const int ng = (int)tables.size();
  std::vector<const void*> cp(ng);
  std::vector<const int64_t*> tp(ng);
  std::vector<int> nc(ng), gd(ng);
  int64_t total = 0;
  for (int i = 0; i < ng; ++i) {
    cp[i] = chunks[i].data_ptr();
    tp[i] = tables[i].data_ptr<int64_t>();
    nc[i] = (int)nchunks[i];
    gd[i] = (int)gdts[i];
    total += nchunks[i];
  }
  Tensor partial = at::empty({std::max<int64_t>(total, 1)}, tables[0].options().dtype(at::kFloat));
  Tensor out = at::empty({3}, tables[0].options().dtype(at::kFloat));
  tbamd::grad_norm_multi(ng, gd.data(), cp.data(), nc.data(), tp.data(), (float)max_norm, fptr(inv_scale),
                         partial.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

void scale_mt(const Tensor& chunks, int64_t nchunks, const Tensor& table, int64_t gdt, const Tensor& s) {
  const at::DeviceGuard guard(table.device());
  tbamd::scale_mt((int)gdt, chunks.data_ptr(), (int)nchunks, table.data_ptr<int64_t>(),
                  s.data_ptr<float>(), cur_stream());
}

// -------------------------------------------------------------------- conv
// x: [N, C, H, W] logical, channels_last memory; w: [K, C, R, S] logical,
// channels_last memory ([K][R][S][C]).  Returns y [N, K, P, Q] channels_last
// and, if want_stats, per-pixel-tile (sum, sumsq) partials [ntiles, 2, K].
// ResNet stem on the native kernels (see tbamd.h): pad -> xp, forward from xp + packed
// weights wp [K, 256] -> {y [N, K, P, Q] channels_last, stats [tiles, 2, K] or undefined},
// weight gradient from dy + xp -> packed [K, 256]
Tensor conv2d_stem_pad(const Tensor& x_) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && x_.dim() == 4 && x_.size(1) == 3, "conv2d_stem_pad: bf16 [N,3,H,W]");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3);
  int P, Q, Hp, Wp;
  tbamd::stem_geometry(H, W, &P, &Q, &Hp, &Wp);
  Tensor xp = at::empty({N, Hp, Wp, 4}, x.options());
  if (N > 0) tbamd::conv_stem_pad(x.data_ptr(), xp.data_ptr(), N, H, W, cur_stream());
  return xp;
}

std::vector<Tensor> conv2d_stem_fwd(const Tensor& xp, const Tensor& wp_, int64_t H, int64_t W, bool want_stats) {
  check_cuda(xp, "xp");
  const at::DeviceGuard guard(xp.device());
  int P, Q, Hp, Wp;
  tbamd::stem_geometry((int)H, (int)W, &P, &Q, &Hp, &Wp);
  TORCH_CHECK(xp.scalar_type() == at::kBFloat16 && xp.dim() == 4 && xp.size(1) == Hp && xp.size(2) == Wp &&
                  xp.size(3) == 4 && xp.is_contiguous(), "conv2d_stem_fwd: xp from conv2d_stem_pad");
  TORCH_CHECK(wp_.scalar_type() == at::kBFloat16 && wp_.dim() == 2 && wp_.size(1) == 256 && wp_.size(0) % 64 == 0,
              "conv2d_stem_fwd: wp [K % 64 == 0, 256] bf16");
  Tensor wp = wp_.contiguous();
  const int N = (int)xp.size(0), K = (int)wp.size(0);
  Tensor y = at::empty({N, K, P, Q}, xp.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t NPQ = (int64_t)N * P * Q;
  Tensor stats;
  if (want_stats) stats = at::empty({tbamd::conv_fwd_pixel_tiles(NPQ, K), 2, K}, xp.options().dtype(at::kFloat));
  if (NPQ > 0)
    tbamd::conv_stem_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), want_stats ? stats.data_ptr<float>() : nullptr,
                         N, (int)H, (int)W, K, cur_stream());
  return {y, stats};
}

Tensor conv2d_stem_wgrad(const Tensor& dy_, const Tensor& xp, int64_t H, int64_t W) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  int P, Q, Hp, Wp;
  tbamd::stem_geometry((int)H, (int)W, &P, &Q, &Hp, &Wp);
  TORCH_CHECK(xp.dim() == 4 && xp.size(1) == Hp && xp.size(2) == Wp && xp.size(3) == 4 && xp.is_contiguous(),
              "conv2d_stem_wgrad: xp from conv2d_stem_pad");
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.size(0) == xp.size(0) && dy.size(2) == P && dy.size(3) == Q &&
                  dy.size(1) % 64 == 0, "conv2d_stem_wgrad: dy [N, K % 64, P, Q] bf16");
  const int N = (int)dy.size(0), K = (int)dy.size(1);
  Tensor dwp = at::empty({K, 256}, dy.options());
  const int64_t ws = tbamd::conv_stem_wgrad_workspace(N, Hp, Wp, K, P, Q);
  Tensor work;
  if (ws > 0) work = at::empty({ws}, dy.options().dtype(at::kFloat));
  if ((int64_t)N * P * Q == 0) return dwp.zero_();
  tbamd::conv_stem_wgrad(dy.data_ptr(), xp.data_ptr(), dwp.data_ptr(), ws > 0 ? work.data_ptr<float>() : nullptr, N,
                         Hp, Wp, K, P, Q, cur_stream());
  return dwp;
}

// input gradient of a stride-2 conv: dy [N, Kf, P, Q], wt = conv_flip_weight(w) [Cf, R, S, Kf]
// (channels_last bf16) -> dx [N, Cf, H, W] channels_last (4 parity-class launches)
std::vector<Tensor> conv2d_dgrad_s2(const Tensor& dy_, const Tensor& wt_, int64_t R, int64_t S, int64_t pad,
                                    int64_t H, int64_t W, int64_t bnb_mode, const optional<Tensor>& bnb_x,
                                    const optional<Tensor>& bnb_scale, const optional<Tensor>& bnb_shift,
                                    const optional<Tensor>& bnb_mean, const optional<Tensor>& bnb_bits,
                                    int64_t stride) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  TORCH_CHECK(dy_.scalar_type() == at::kBFloat16 && wt_.scalar_type() == at::kBFloat16, "conv2d_dgrad_s2: bf16 only");
  const int cs = (int)stride;
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor wt = wt_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)dy.size(0), Kf = (int)dy.size(1), P = (int)dy.size(2), Q = (int)dy.size(3);
  const int Cf = (int)wt.size(0);
  TORCH_CHECK(wt.dim() == 4 && wt.size(1) == Kf && wt.size(2) == R && wt.size(3) == S,
              "conv2d_dgrad_s2: wt must be the flip-transposed [Cf, Kf, R, S] weight");
  TORCH_CHECK(tbamd::conv_fwd_supported(Kf, Cf) && tbamd::conv_dgrad_s2_supported((int)R, (int)S, cs),
              "conv2d_dgrad_s2: channels % 64, stride 2 or 3, <= 16 taps per phase class");
  TORCH_CHECK(pad >= 0 && P == (H + 2 * pad - R) / cs + 1 && Q == (W + 2 * pad - S) / cs + 1,
              "conv2d_dgrad_s2: geometry");
  Tensor dx = at::empty({N, Cf, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t NHW = (int64_t)N * H * W;
  Tensor part;
  const void* bx = nullptr;
  const float *bsc = nullptr, *bsf = nullptr, *bmu = nullptr;
  const uint8_t* bbits = nullptr;
  if (bnb_mode != 0) {
    TORCH_CHECK(bnb_mode >= 1 && bnb_mode <= 3 && bnb_x.has_value() && bnb_x->numel() == NHW * Cf &&
                    bnb_x->scalar_type() == at::kBFloat16 && bnb_mean.has_value() && bnb_mean->numel() == Cf,
                "conv2d_dgrad_s2: bnb_x [N*H*W, Cf] bf16 and bnb_mean [Cf] required");
    bx = bnb_x->data_ptr();
    bmu = bnb_mean->data_ptr<float>();
    if (bnb_mode == 1) {
      TORCH_CHECK(bnb_scale.has_value() && bnb_shift.has_value(), "conv2d_dgrad_s2: bnb scale/shift");
      bsc = bnb_scale->data_ptr<float>();
      bsf = bnb_shift->data_ptr<float>();
    }
    if (bnb_mode == 2) {
      TORCH_CHECK(bnb_bits.has_value() && bnb_bits->numel() == NHW * (Cf / 8), "conv2d_dgrad_s2: bnb_bits");
      bbits = bnb_bits->data_ptr<uint8_t>();
    }
    part = at::empty({tbamd::conv_dgrad_s2_tiles(N, (int)H, (int)W, Cf, cs), 2, Cf}, dy.options().dtype(at::kFloat));
  }
  if (NHW > 0)
    tbamd::conv_dgrad_s2(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), N, P, Q, Kf, Cf, (int)R, (int)S, (int)pad,
                         (int)H, (int)W, cur_stream(), (int)bnb_mode, bx, bsc, bsf, bmu, bbits,
                         part.defined() ? part.data_ptr<float>() : nullptr, cs);
  return {dx, part};
}

std::vector<Tensor> conv2d_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride,
                               int64_t pad, bool relu, bool want_stats, const optional<Tensor>& addend,
                               const optional<Tensor>& addend_mask, int64_t bnb_mode, const optional<Tensor>& bnb_x,
                               const optional<Tensor>& bnb_scale, const optional<Tensor>& bnb_shift,
                               const optional<Tensor>& bnb_mean, const optional<Tensor>& bnb_bits, int64_t big) {
  check_cuda(x_, "x");
  // big >= 0: this call's big-tile choice (0 = the 128x128 kernels), restored on every exit
  struct BigScope {
    explicit BigScope(int64_t c) { if (c >= 0) tbamd::conv_big_set_call((int)c); }
    ~BigScope() { tbamd::conv_big_set_call(-1); }
  } big_scope(big);
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16, "conv2d_fwd: bf16 only");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && x_.size(1) == w_.size(1), "conv2d_fwd: shape");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor w = w_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w.size(0), R = (int)w.size(2), S = (int)w.size(3);
  TORCH_CHECK(tbamd::conv_fwd_supported(C, K), "conv2d_fwd: needs C % 64 == 0 and K % 64 == 0");
  const int P = (H + 2 * (int)pad - R) / (int)stride + 1, Q = (W + 2 * (int)pad - S) / (int)stride + 1;
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor bf;
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  Tensor stats;
  const int64_t NPQ = (int64_t)N * P * Q;
  if (want_stats)
    stats = at::empty({tbamd::conv_fwd_stats_rows(NPQ, C, K, R, S, (int)stride, (int)pad), 2, K},
                      x.options().dtype(at::kFloat));
  Tensor add;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(!want_stats && !bf.defined() && !relu, "conv2d_fwd: addend excludes bias / relu / stats");
    TORCH_CHECK(addend->sizes() == y.sizes() && addend->scalar_type() == at::kBFloat16, "conv2d_fwd: addend shape");
    add = addend->contiguous(at::MemoryFormat::ChannelsLast);
  }
  const uint8_t* amask = nullptr;
  if (addend_mask.has_value() && addend_mask->defined()) {
    TORCH_CHECK(add.defined() && addend_mask->scalar_type() == at::kByte && addend_mask->numel() == NPQ * (K / 8),
                "conv2d_fwd: addend_mask must be [N*P*Q, K/8] bytes");
    amask = addend_mask->data_ptr<uint8_t>();
  }
  // BN-backward partial sums of the BN whose output gradient y is (dgrad use)
  Tensor part;
  const void* bx = nullptr;
  const float *bsc = nullptr, *bsf = nullptr, *bmu = nullptr;
  const uint8_t* bbits = nullptr;
  if (bnb_mode != 0) {
    TORCH_CHECK(bnb_mode >= 1 && bnb_mode <= 3 && !want_stats && !bf.defined() && !relu, "conv2d_fwd: bnb_mode");
    TORCH_CHECK(bnb_x.has_value() && bnb_x->numel() == NPQ * K && bnb_x->scalar_type() == at::kBFloat16 &&
                    bnb_mean.has_value() && bnb_mean->numel() == K,
                "conv2d_fwd: bnb_x [N*P*Q, K] bf16 and bnb_mean [K] required");
    bx = bnb_x->data_ptr();
    bmu = bnb_mean->data_ptr<float>();
    if (bnb_mode == 1) {
      TORCH_CHECK(bnb_scale.has_value() && bnb_shift.has_value(), "conv2d_fwd: bnb scale/shift");
      bsc = bnb_scale->data_ptr<float>();
      bsf = bnb_shift->data_ptr<float>();
    }
    if (bnb_mode == 2) {
      TORCH_CHECK(bnb_bits.has_value() && bnb_bits->numel() == NPQ * (K / 8), "conv2d_fwd: bnb_bits");
      bbits = bnb_bits->data_ptr<uint8_t>();
    }
    part = at::empty({tbamd::conv_fwd_bnb_rows(NPQ, C, K, R, S, (int)stride, (int)pad), 2, K},
                     x.options().dtype(at::kFloat));
  }
  if (NPQ > 0)
    tbamd::conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), bf.defined() ? bf.data_ptr<float>() : nullptr,
                    want_stats ? stats.data_ptr<float>() : nullptr, add.defined() ? add.data_ptr() : nullptr, amask, relu, N,
                    H, W, C, K, R, S, P, Q, (int)stride, (int)pad, cur_stream(), (int)bnb_mode, bx, bsc, bsf, bmu,
                    bbits, part.defined() ? part.data_ptr<float>() : nullptr);
  return {y, bnb_mode != 0 ? part : stats};
}

// 1x1 stride-1 input gradient whose operand is a deferred BN backward apply (conv.hip GxfArgs):
// g = the BN output gradient [N, C, H, W] (C = the conv's output channels), wt the flipped /
// transposed weight [K, C, 1, 1] (K = the conv's input channels), gx_x the BN input (the conv's
// forward output, g's shape), gx_coef [3, C] from bn_backward_coef, gxf 1 (ReLU mask recomputed
// from gx_scale / gx_shift) or 2 (gx_bits [N*H*W, C/8]).  Returns [dx, bnb partials (or empty),
// dz (the materialised BN input gradient when want_dz, else empty)].
std::vector<Tensor> conv2d_dgrad_gxf(const Tensor& g_, const Tensor& wt_, const optional<Tensor>& addend,
                                     const optional<Tensor>& addend_mask, int64_t bnb_mode,
                                     const optional<Tensor>& bnb_x, const optional<Tensor>& bnb_scale,
                                     const optional<Tensor>& bnb_shift, const optional<Tensor>& bnb_mean,
                                     const optional<Tensor>& bnb_bits, int64_t gxf, const Tensor& gx_x_,
                                     const optional<Tensor>& gx_bits, const optional<Tensor>& gx_scale,
                                     const optional<Tensor>& gx_shift, const Tensor& gx_coef, bool want_dz) {
  check_cuda(g_, "g");
  const at::DeviceGuard guard(g_.device());
  TORCH_CHECK(g_.scalar_type() == at::kBFloat16 && wt_.scalar_type() == at::kBFloat16 &&
                  gx_x_.scalar_type() == at::kBFloat16, "conv2d_dgrad_gxf: bf16 only");
  TORCH_CHECK(g_.dim() == 4 && wt_.dim() == 4 && wt_.size(1) == g_.size(1) && wt_.size(2) == 1 && wt_.size(3) == 1,
              "conv2d_dgrad_gxf: 1x1 weight [K, C, 1, 1] over g [N, C, H, W]");
  TORCH_CHECK(gx_x_.sizes() == g_.sizes(), "conv2d_dgrad_gxf: gx_x must have g's shape");
  Tensor g = g_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor wt = wt_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor gx_x = gx_x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)g.size(0), C = (int)g.size(1), H = (int)g.size(2), W = (int)g.size(3);
  const int K = (int)wt.size(0);
  const int64_t NPQ = (int64_t)N * H * W;
  TORCH_CHECK(tbamd::conv_fwd_supported(C, K), "conv2d_dgrad_gxf: needs C % 64 == 0 and K % 64 == 0");
  TORCH_CHECK(gx_coef.scalar_type() == at::kFloat && gx_coef.is_contiguous() && gx_coef.numel() == 3 * C,
              "conv2d_dgrad_gxf: gx_coef [3, C] f32");
  const uint8_t* gbits = nullptr;
  const float *gsc = nullptr, *gsf = nullptr;
  if (gxf == 2) {
    TORCH_CHECK(gx_bits.has_value() && gx_bits->scalar_type() == at::kByte && gx_bits->numel() == NPQ * (C / 8),
                "conv2d_dgrad_gxf: gx_bits [N*H*W, C/8] bytes");
    gbits = gx_bits->data_ptr<uint8_t>();
  } else {
    TORCH_CHECK(gxf == 1 && gx_scale.has_value() && gx_shift.has_value() && gx_scale->numel() == C &&
                    gx_shift->numel() == C && gx_scale->scalar_type() == at::kFloat &&
                    gx_shift->scalar_type() == at::kFloat && gx_scale->is_contiguous() && gx_shift->is_contiguous(),
                "conv2d_dgrad_gxf: gxf 1 needs f32 [C] scale / shift");
    gsc = gx_scale->data_ptr<float>();
    gsf = gx_shift->data_ptr<float>();
  }
  Tensor y = at::empty({N, K, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor add;
  const uint8_t* amask = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->sizes() == y.sizes() && addend->scalar_type() == at::kBFloat16, "conv2d_dgrad_gxf: addend");
    add = addend->contiguous(at::MemoryFormat::ChannelsLast);
    if (addend_mask.has_value() && addend_mask->defined()) {
      TORCH_CHECK(addend_mask->scalar_type() == at::kByte && addend_mask->numel() == NPQ * (K / 8),
                  "conv2d_dgrad_gxf: addend_mask [N*H*W, K/8] bytes");
      amask = addend_mask->data_ptr<uint8_t>();
    }
  }
  const int add_code = add.defined() ? (amask ? 2 : 1) : 0;
  TORCH_CHECK(tbamd::conv_dgrad_gxf_supported((int)gxf, add_code, (int)bnb_mode),
              "conv2d_dgrad_gxf: unsupported (gxf, addend, bnb_mode) combination");
  Tensor part;
  const void* bx = nullptr;
  const float *bsc = nullptr, *bsf = nullptr, *bmu = nullptr;
  const uint8_t* bbits = nullptr;
  if (bnb_mode != 0) {
    TORCH_CHECK(bnb_x.has_value() && bnb_x->numel() == NPQ * K && bnb_x->scalar_type() == at::kBFloat16 &&
                    bnb_mean.has_value() && bnb_mean->numel() == K,
                "conv2d_dgrad_gxf: bnb_x [N*H*W, K] bf16 and bnb_mean [K] required");
    bx = bnb_x->data_ptr();
    bmu = bnb_mean->data_ptr<float>();
    if (bnb_mode == 1) {
      TORCH_CHECK(bnb_scale.has_value() && bnb_shift.has_value(), "conv2d_dgrad_gxf: bnb scale/shift");
      bsc = bnb_scale->data_ptr<float>();
      bsf = bnb_shift->data_ptr<float>();
    }
    if (bnb_mode == 2) {
      TORCH_CHECK(bnb_bits.has_value() && bnb_bits->numel() == NPQ * (K / 8), "conv2d_dgrad_gxf: bnb_bits");
      bbits = bnb_bits->data_ptr<uint8_t>();
    }
    part = at::empty({tbamd::conv_gxf_bnb_rows(NPQ, K), 2, K}, g.options().dtype(at::kFloat));
  }
  Tensor dz;
  if (want_dz) dz = at::empty_like(g);
  if (NPQ > 0)
    tbamd::conv_dgrad_gxf(g.data_ptr(), wt.data_ptr(), y.data_ptr(), add.defined() ? add.data_ptr() : nullptr, amask,
                          N, H, W, C, K, cur_stream(), (int)bnb_mode, bx, bsc, bsf, bmu, bbits,
                          part.defined() ? part.data_ptr<float>() : nullptr, (int)gxf, gx_x.data_ptr(), gbits, gsc,
                          gsf, gx_coef.data_ptr<float>(), dz.defined() ? dz.data_ptr() : nullptr);
  return {y, part, dz};
}

bool conv_dgrad_gxf_supported(int64_t gxf, int64_t add, int64_t bnb_mode) {
  return tbamd::conv_dgrad_gxf_supported((int)gxf, (int)add, (int)bnb_mode);
}

// deferred BN backward: the finalize only (coef [3, C], dgamma, dbeta) from the dgrad partials
std::vector<Tensor> bn_backward_coef(const Tensor& part, const optional<Tensor>& weight, const Tensor& mean,
                                     const Tensor& invstd, int64_t M, bool training,
                                     const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out) {
  check_cuda(part, "part");
  const at::DeviceGuard guard(part.device());
  TORCH_CHECK(part.dim() == 3 && part.size(1) == 2 && part.scalar_type() == at::kFloat && part.is_contiguous(),
              "bn_backward_coef: part [rows, 2, C] f32");
  const int C = (int)part.size(2);
  auto fopt = part.options();
  Tensor wf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  auto out_or_new = [&](const optional<Tensor>& o) {
    if (o.has_value() && o->defined()) {
      TORCH_CHECK(o->scalar_type() == at::kFloat && o->numel() == C && o->is_contiguous(), "bn_backward_coef: out");
      return *o;
    }
    return at::empty({C}, fopt);
  };
  Tensor dgamma = out_or_new(dgamma_out), dbeta = out_or_new(dbeta_out);
  Tensor coef = at::empty({3, C}, fopt);
  Tensor fws = at::empty({tbamd::colsum_workspace((int)part.size(0), C)}, fopt.dtype(at::kDouble));
  tbamd::bn_backward_coef(part.data_ptr<float>(), (int)part.size(0), M, C, wf.defined() ? wf.data_ptr<float>() : nullptr,
                          mean.data_ptr<float>(), invstd.data_ptr<float>(), training ? 1 : 0, fws.data_ptr<double>(),
                          coef.data_ptr<float>(), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), cur_stream());
  return {coef, dgamma, dbeta};
}

// the deferred apply when the consumer conv cannot take it: dx = ka * act'(z) * dy + c0 + c1 * x
Tensor bn_backward_apply_coef(const Tensor& dy_, const Tensor& x_, const Tensor& coef, const Tensor& scale,
                              const Tensor& shift, int64_t act, double slope, const optional<Tensor>& mask) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  TORCH_CHECK(dy_.dim() == 2 && x_.dim() == 2, "bn_backward_apply_coef: [M, C] rows");
  Tensor x = as_rows(x_);
  Tensor dy = as_rows(dy_.to(x.scalar_type()));
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(dy.size(0) == M && dy.size(1) == C && coef.numel() == 3 * C && coef.scalar_type() == at::kFloat &&
                  coef.is_contiguous(), "bn_backward_apply_coef: shapes");
  const uint8_t* maskin = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->numel() == M * (C / 8) && C % 8 == 0, "bn_backward_apply_coef: mask");
    maskin = mask->data_ptr<uint8_t>();
  }
  Tensor dx = at::empty_like(x);
  tbamd::bn_backward_apply_coef(dt_code(x), dy.data_ptr(), x.data_ptr(), M, C, (int)act, (float)slope,
                                scale.data_ptr<float>(), shift.data_ptr<float>(), coef.data_ptr<float>(),
                                dx.data_ptr(), maskin, cur_stream());
  return dx;
}

// BN apply (+ residual, activation, optional 1-bit ReLU mask) with coefficients computed
// elsewhere: coeff [4, C] = mean, invstd, scale, shift.  Returns [y, mask].
std::vector<Tensor> bn_apply_coeff(const Tensor& x_, const Tensor& coeff, const optional<Tensor>& residual,
                                   int64_t act, double slope, bool want_mask) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = as_rows(x_);
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(coeff.dim() == 2 && coeff.size(0) == 4 && coeff.size(1) == C && coeff.scalar_type() == at::kFloat &&
                  coeff.is_contiguous(),
              "bn_apply_coeff: coeff [4, C] f32");
  Tensor res;
  if (residual.has_value() && residual->defined()) res = as_rows(*residual);
  Tensor y = at::empty_like(x);
  Tensor mask = make_mask(x, res, act, want_mask);
  tbamd::bn_apply(dt_code(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, coeff[2].data_ptr<float>(),
                  coeff[3].data_ptr<float>(), M, C, (int)act, (float)slope, y.data_ptr(),
                  mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {y, mask};
}

// y = conv(relu(x * scale + shift), w) with the BN + ReLU applied in the kernel's operand staging
// (csrc/xf.h): returns [y, stats] (stats: the BN partial rows of y, as conv2d_fwd want_stats)
std::vector<Tensor> conv2d_fwd_xf(const Tensor& x_, const Tensor& w_, const Tensor& scale, const Tensor& shift,
                                  int64_t stride, int64_t pad, bool want_stats) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16, "conv2d_fwd_xf: bf16 only");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor w = w_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w.size(0), R = (int)w.size(2), S = (int)w.size(3);
  TORCH_CHECK(w.size(1) == C && tbamd::conv_fwd_supported(C, K), "conv2d_fwd_xf: needs C % 64 == 0 and K % 64 == 0");
  TORCH_CHECK(C <= tbamd::kXfMaxC, "conv2d_fwd_xf: at most ", tbamd::kXfMaxC, " input channels (coefficients in LDS)");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == C &&
                  shift.numel() == C && scale.is_contiguous() && shift.is_contiguous(),
              "conv2d_fwd_xf: scale / shift [C] f32");
  const int P = (H + 2 * (int)pad - R) / (int)stride + 1, Q = (W + 2 * (int)pad - S) / (int)stride + 1;
  const int64_t NPQ = (int64_t)N * P * Q;
  TORCH_CHECK(tbamd::conv_fwd_xf_supported(NPQ, C, K, R, S, (int)stride, (int)pad),
              "conv2d_fwd_xf: the persistent 1x1 shapes only (C = 64 / 128, 1x1 stride 1, K % 128, enough pixels)");
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor stats;
  if (want_stats)
    stats = at::empty({tbamd::conv_fwd_stats_rows_tiled(NPQ, C, K, R, S, (int)stride, (int)pad), 2, K},
                      x.options().dtype(at::kFloat));
  if (NPQ > 0)
    tbamd::conv_fwd_xf(x.data_ptr(), w.data_ptr(), y.data_ptr(), want_stats ? stats.data_ptr<float>() : nullptr,
                       scale.data_ptr<float>(), shift.data_ptr<float>(), N, H, W, C, K, R, S, P, Q, (int)stride,
                       (int)pad, cur_stream());
  return {y, stats};
}

// dW of conv(relu(x * scale + shift), w) (the transform in the X staging); out: optional slot
// dW [K = 64, C = 3, 4, 4] (channels_last) of a 4x4 / 2 / pad-1 conv: T = its 3-channel input
// [N, 3, H, W], G = the gradient of its 64-channel output [N, 64, H/2, W/2] (both NHWC bf16).  The
// 64 -> 3 transposed conv's weight gradient is the same call with T = dY and G = its input.
Tensor conv2d_wgrad_tinyin(const Tensor& T_, const Tensor& G_) {
  check_cuda(T_, "T");
  check_cuda(G_, "G");
  const at::DeviceGuard guard(T_.device());
  TORCH_CHECK(T_.scalar_type() == at::kBFloat16 && G_.scalar_type() == at::kBFloat16, "conv2d_wgrad_tinyin: bf16");
  TORCH_CHECK(T_.dim() == 4 && G_.dim() == 4 && T_.size(0) == G_.size(0), "conv2d_wgrad_tinyin: NCHW shapes");
  Tensor T = T_.contiguous(at::MemoryFormat::ChannelsLast), G = G_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)T.size(0), C = (int)T.size(1), H = (int)T.size(2), W = (int)T.size(3);
  const int K = (int)G.size(1), P = (int)G.size(2), Q = (int)G.size(3);
  TORCH_CHECK(tbamd::wgrad_tinyin_supported(C, K, 4, 4, 2, 1, P, Q, H, W),
              "conv2d_wgrad_tinyin: needs C = 3, K = 64, Q = 64, H = 2P, W = 2Q");
  Tensor part = at::empty({(int64_t)tbamd::wgrad_tinyin_parts(N, P) * K * 48}, T.options().dtype(at::kFloat));
  Tensor dw = at::empty({K, C, 4, 4}, T.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::wgrad_tinyin(T.data_ptr(), G.data_ptr(), dw.data_ptr(), part.data_ptr<float>(), N, P, H, W, cur_stream());
  return dw;
}

Tensor conv2d_wgrad_xf(const Tensor& dy_, const Tensor& x_, const Tensor& scale, const Tensor& shift, int64_t R,
                       int64_t S, int64_t stride, int64_t pad, const optional<Tensor>& out) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && dy_.scalar_type() == at::kBFloat16, "conv2d_wgrad_xf: bf16 only");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  TORCH_CHECK(tbamd::conv_wgrad_supported(C, K, (int64_t)N * dy.size(2) * dy.size(3)), "conv2d_wgrad_xf: shape");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == C &&
                  shift.numel() == C && scale.is_contiguous() && shift.is_contiguous(),
              "conv2d_wgrad_xf: scale / shift [C] f32");
  const int P = (int)dy.size(2), Q = (int)dy.size(3);
  TORCH_CHECK(P == (H + 2 * (int)pad - (int)R) / (int)stride + 1 && Q == (W + 2 * (int)pad - (int)S) / (int)stride + 1,
              "conv2d_wgrad_xf: dy shape");
  Tensor dw;
  if (out.has_value() && out->defined()) {
    dw = *out;
    TORCH_CHECK(dw.scalar_type() == at::kBFloat16 && dw.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dw.size(0) == K && dw.size(1) == C && dw.size(2) == R && dw.size(3) == S,
                "conv2d_wgrad_xf: out must be a channels_last bf16 [K, C, R, S] tensor");
  } else {
    dw = at::empty({K, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  const int64_t ws = tbamd::conv_wgrad_workspace(N, H, W, C, K, (int)R, (int)S, P, Q, (int)stride, (int)pad);
  Tensor work;
  if (ws > 0) work = at::empty({ws}, x.options().dtype(at::kFloat));
  tbamd::conv_wgrad_xf(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws > 0 ? work.data_ptr<float>() : nullptr,
                       scale.data_ptr<float>(), shift.data_ptr<float>(), N, H, W, C, K, (int)R, (int)S, P, Q,
                       (int)stride, (int)pad, cur_stream());
  return dw;
}

// w [K, C, R, S] (channels_last) -> flipped transpose [C, K, R, S] (channels_last)
Tensor conv_flip_weight(const Tensor& w_) {
  const at::DeviceGuard guard(w_.device());
  Tensor w = w_.contiguous(at::MemoryFormat::ChannelsLast);
  const int K = (int)w.size(0), C = (int)w.size(1), R = (int)w.size(2), S = (int)w.size(3);
  Tensor wt = at::empty({C, K, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_flip_transpose_weight(w.data_ptr(), K, R, S, C, wt.data_ptr(), cur_stream());
  return wt;
}

// several flipped copies in one launch: chunks int32x2+int64x2 rows (tensor, pad, start, len)
// as an int64 [n, 3] tensor (first column packs tensor index), table int64 [T, 8]
void conv_flip_weights_mt(const Tensor& chunks, int64_t nchunks, const Tensor& table) {
  const at::DeviceGuard guard(table.device());
  TORCH_CHECK(table.scalar_type() == at::kLong && chunks.scalar_type() == at::kLong, "conv_flip_weights_mt: int64 tables");
  tbamd::conv_flip_transpose_weights_mt(chunks.data_ptr(), (int)nchunks, table.data_ptr<int64_t>(), cur_stream());
}

// dW [K, C, R, S] (channels_last) of y = conv(x, w): dy [N, K, P, Q] and x
// [N, C, H, W] channels_last bf16
Tensor conv2d_wgrad(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t stride, int64_t pad,
                    const optional<Tensor>& out) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && dy_.scalar_type() == at::kBFloat16, "conv2d_wgrad: bf16 only");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)dy.size(1), P = (int)dy.size(2), Q = (int)dy.size(3);
  TORCH_CHECK(dy.size(0) == N && P == (H + 2 * (int)pad - (int)R) / (int)stride + 1 &&
                  Q == (W + 2 * (int)pad - (int)S) / (int)stride + 1,
              "conv2d_wgrad: dy shape does not match x / kernel / stride / pad");
  const int64_t NPQ = (int64_t)N * P * Q;
  TORCH_CHECK(tbamd::conv_wgrad_supported(C, K, NPQ), "conv2d_wgrad: needs C % 64 == 0 and K % 64 == 0");
  Tensor dw;
  if (out.has_value() && out->defined()) {  // e.g. a zero-copy gradient slot
    dw = *out;
    TORCH_CHECK(dw.sizes() == at::IntArrayRef({K, C, R, S}) && dw.scalar_type() == at::kBFloat16 &&
                    dw.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv2d_wgrad: out must be a channels_last bf16 [K, C, R, S] tensor");
  } else {
    dw = at::empty({K, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  if (NPQ == 0) return dw.zero_();
  const int64_t ws = tbamd::conv_wgrad_workspace(N, H, W, C, K, (int)R, (int)S, P, Q, (int)stride, (int)pad);
  Tensor work;
  if (ws > 0) work = at::empty({ws}, x.options().dtype(at::kFloat));
  tbamd::conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws > 0 ? work.data_ptr<float>() : nullptr, N, H, W,
                    C, K, (int)R, (int)S, P, Q, (int)stride, (int)pad, cur_stream());
  return dw;
}

// BN forward when the statistics come from the conv epilogue
std::vector<Tensor> bn_forward_from_stats(const Tensor& x_, const Tensor& stats, const optional<Tensor>& weight,
                                          const optional<Tensor>& bias, const optional<Tensor>& running_mean,
                                          const optional<Tensor>& running_var, double momentum, double eps,
                                          const optional<Tensor>& residual, int64_t act, double slope,
                                          const optional<Tensor>& num_batches_tracked, bool want_mask,
                                          const optional<Tensor>& res_scale, const optional<Tensor>& res_shift) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = as_rows(x_);
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(stats.dim() == 3 && stats.size(1) == 2 && stats.size(2) == C, "bn_forward_from_stats: stats shape");
  // res_scale / res_shift: the residual is the input of a BN without activation (its coefficients),
  // added as res * res_scale + res_shift (the bottleneck downsample branch, ops/norm.py)
  const bool resaff = res_scale.has_value() && res_scale->defined();
  if (resaff)
    TORCH_CHECK(res_shift.has_value() && res_shift->defined() && res_scale->scalar_type() == at::kFloat &&
                    res_shift->scalar_type() == at::kFloat && res_scale->is_contiguous() && res_shift->is_contiguous() &&
                    res_scale->numel() == C && res_shift->numel() == C && want_mask && act == 1 && C % 8 == 0 &&
                    residual.has_value() && residual->defined(),
                "bn_forward_from_stats: an affine residual needs f32 [C] scale / shift, ReLU, a mask, C % 8 == 0");
  auto fopt = x.options().dtype(at::kFloat);
  Tensor coeff = at::empty({4, C}, fopt);
  Tensor fws = at::empty({tbamd::colsum_workspace((int)stats.size(0), C)}, x.options().dtype(at::kDouble));
  Tensor wf, bf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  auto st = cur_stream();
  tbamd::bn_finalize_from_conv(stats.data_ptr<float>(), (int)stats.size(0), M, C,
                               wf.defined() ? wf.data_ptr<float>() : nullptr, bf.defined() ? bf.data_ptr<float>() : nullptr,
                               fptr_mut(running_mean), fptr_mut(running_var), nbt_ptr(num_batches_tracked),
                               (float)momentum, (float)eps, fws.data_ptr<double>(), coeff[0].data_ptr<float>(), coeff[1].data_ptr<float>(), coeff[2].data_ptr<float>(),
                               coeff[3].data_ptr<float>(), st);
  Tensor res;
  if (residual.has_value() && residual->defined()) res = as_rows(*residual);
  Tensor y = at::empty_like(x);
  Tensor mask = make_mask(x, res, act, want_mask);
  tbamd::bn_apply(dt_code(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, coeff[2].data_ptr<float>(),
                  coeff[3].data_ptr<float>(), M, C, (int)act, (float)slope, y.data_ptr(),
                  mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, st,
                  resaff ? res_scale->data_ptr<float>() : nullptr, resaff ? res_shift->data_ptr<float>() : nullptr);
  return {y, coeff[0], coeff[1], coeff[2], coeff[3], mask};
}

// ------------------------------------------------ BN statistics + fused max-pool
// Statistics only (training: from the conv-epilogue partials `stats` when
// given, else a partial pass over x; eval: running stats) -> [mean, invstd,
// scale, shift].  x: [M, C] rows.
std::vector<Tensor> bn_stats(const Tensor& x_, const optional<Tensor>& stats, const optional<Tensor>& weight,
                             const optional<Tensor>& bias, const optional<Tensor>& running_mean,
                             const optional<Tensor>& running_var, bool training, double momentum, double eps,
                             const optional<Tensor>& num_batches_tracked) {
  check_cuda(x_, "x");
  TORCH_CHECK(x_.dim() == 2, "bn_stats expects [M, C]");
  const at::DeviceGuard guard(x_.device());
  Tensor x = as_rows(x_);
  const int64_t M = x.size(0);
  const int C = (int)x.size(1);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor coeff = at::empty({4, C}, fopt);
  Tensor wf, bf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  const float* g = wf.defined() ? wf.data_ptr<float>() : nullptr;
  const float* b = bf.defined() ? bf.data_ptr<float>() : nullptr;
  float *mean = coeff[0].data_ptr<float>(), *invstd = coeff[1].data_ptr<float>();
  float *scale = coeff[2].data_ptr<float>(), *shift = coeff[3].data_ptr<float>();
  auto st = cur_stream();
  if (!training) {
    TORCH_CHECK(running_mean.has_value() && running_var.has_value(), "eval BN needs running stats");
    tbamd::bn_eval_coeffs(C, g, b, fptr(running_mean), fptr(running_var), (float)eps, mean, invstd, scale, shift,
                          st);
  } else if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->dim() == 3 && stats->size(1) == 2 && stats->size(2) == C, "bn_stats: stats shape");
    Tensor fws = at::empty({tbamd::colsum_workspace((int)stats->size(0), C)}, x.options().dtype(at::kDouble));
    tbamd::bn_finalize_from_conv(stats->data_ptr<float>(), (int)stats->size(0), M, C, g, b, fptr_mut(running_mean),
                                 fptr_mut(running_var), nbt_ptr(num_batches_tracked), (float)momentum, (float)eps,
                                 fws.data_ptr<double>(), mean, invstd, scale, shift, st);
  } else {
    TORCH_CHECK(M > 0, "bn_stats: empty batch in training mode");
    const int nblk = tbamd::bn_partial_blocks(M, C);
    Tensor ws = at::empty({2, (int64_t)nblk, C}, fopt);
    Tensor fws = at::empty({tbamd::colsum_workspace(nblk, C)}, x.options().dtype(at::kDouble));
    tbamd::bn_forward_train(dt_code(x), x.data_ptr(), M, C, g, b, fptr_mut(running_mean), fptr_mut(running_var),
                            nbt_ptr(num_batches_tracked), (float)momentum, (float)eps, ws[0].data_ptr<float>(),
                            ws[1].data_ptr<float>(), nblk, fws.data_ptr<double>(), mean, invstd, scale, shift, st);
  }
  return {coeff[0], coeff[1], coeff[2], coeff[3]};
}

// y = maxpool(act(x * scale + shift)) for NHWC x [N, C, H, W] (channels_last);
// returns [y, argmax uint8 (same shape as y)]
std::vector<Tensor> bn_act_maxpool(const Tensor& x_, const Tensor& scale, const Tensor& shift, int64_t act,
                                   double slope, int64_t k, int64_t s, int64_t pad) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.dim() == 4 && x_.size(1) % 8 == 0, "bn_act_maxpool: NCHW with C % 8 == 0");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int P = (H + 2 * (int)pad - (int)k) / (int)s + 1, Q = (W + 2 * (int)pad - (int)k) / (int)s + 1;
  TORCH_CHECK(P > 0 && Q > 0 && k <= 16 && pad < k, "bn_act_maxpool: bad window");
  Tensor y = at::empty({N, C, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor idx = at::empty({N, C, P, Q}, x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::bn_act_maxpool_fwd(dt_code(x), x.data_ptr(), scale.data_ptr<float>(), shift.data_ptr<float>(), (int)act,
                            (float)slope, N, H, W, C, (int)k, (int)s, (int)pad, y.data_ptr(),
                            idx.data_ptr<uint8_t>(), cur_stream());
  return {y, idx};
}

// input gradient of the max-pool from the saved argmax (gather, no atomics)
Tensor maxpool_backward(const Tensor& dy_, const Tensor& idx, int64_t H, int64_t W, int64_t k, int64_t s,
                        int64_t pad) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_backward: idx");
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::maxpool_bwd(dt_code(dy), dy.data_ptr(), idx.data_ptr<uint8_t>(), N, (int)H, (int)W, C, (int)k, (int)s,
                     (int)pad, dx.data_ptr(), cur_stream());
  return dx;
}

// BN backward of maxpool(act(BN(x))) from the POOLED gradient (csrc/pool_gather.h): the pool
// input's gradient is gathered inside the BN partial / apply passes, never materialised.
// x: the BN input rows [N*H*W, C]; returns (dx rows, dgamma, dbeta)
std::vector<Tensor> bn_backward_pool(const Tensor& dy_, const Tensor& idx, const Tensor& x_, int64_t N, int64_t H,
                                     int64_t W, int64_t k, int64_t s, int64_t pad, const optional<Tensor>& weight,
                                     const Tensor& mean, const Tensor& invstd, const Tensor& scale,
                                     const Tensor& shift, bool training, int64_t act, double slope,
                                     const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor x = as_rows(x_);
  Tensor dy = dy_.to(x.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  const int C = (int)x.size(1);
  const int64_t M = x.size(0);
  const int P = (int)((H + 2 * pad - k) / s + 1), Q = (int)((W + 2 * pad - k) / s + 1);
  TORCH_CHECK(C % 8 == 0 && M == N * H * W && dy.dim() == 4 && dy.size(0) == N && dy.size(1) == C &&
                  dy.size(2) == P && dy.size(3) == Q,
              "bn_backward_pool: shapes");
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == at::kByte &&
                  idx.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_backward_pool: idx");
  TORCH_CHECK(tbamd::bn_backward_pool_ok((int)H, (int)W, C, (int)k, (int)s, (int)pad), "bn_backward_pool: shape "
              "(3x3/2 pad 1, even H and W, C/8 channel groups dividing 256)");
  auto fopt = x.options().dtype(at::kFloat);
  Tensor wf;
  if (weight.has_value() && weight->defined()) wf = weight->to(at::kFloat).contiguous();
  const int nblk = tbamd::bn_backward_pool_blocks((int)N, (int)H, (int)W, C);
  Tensor ws = at::empty({2, (int64_t)nblk, C}, fopt);
  Tensor fws = at::empty({tbamd::colsum_workspace(nblk, C)}, x.options().dtype(at::kDouble));
  Tensor coef = at::empty({3, C}, fopt);
  auto out_or_new = [&](const optional<Tensor>& o) {
    if (o.has_value() && o->defined()) {
      TORCH_CHECK(o->scalar_type() == at::kFloat && o->numel() == C && o->is_contiguous(), "bn_backward_pool: out");
      return *o;
    }
    return at::empty({C}, fopt);
  };
  Tensor dgamma = out_or_new(dgamma_out), dbeta = out_or_new(dbeta_out);
  Tensor dx = at::empty_like(x);
  if (M > 0)
    tbamd::bn_backward_pool(dt_code(x), dy.data_ptr(), idx.data_ptr<uint8_t>(), x.data_ptr(), (int)N, (int)H, (int)W,
                            C, (int)k, (int)s, (int)pad, (int)act, (float)slope,
                            wf.defined() ? wf.data_ptr<float>() : nullptr, mean.data_ptr<float>(),
                            invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                            training ? 1 : 0, ws[0].data_ptr<float>(), ws[1].data_ptr<float>(), nblk,
                            fws.data_ptr<double>(), coef.data_ptr<float>(), dgamma.data_ptr<float>(),
                            dbeta.data_ptr<float>(), dx.data_ptr(), cur_stream());
  return {dx, dgamma, dbeta};
}

// ----------------------------------------------------------- input pipeline
// in: uint8 [N, Hi, Wi, C] on the GPU -> [N, C, Ho, Wo] (channels_last memory)
Tensor u8_crop_flip_normalize(const Tensor& in_, int64_t Ho, int64_t Wo, const optional<Tensor>& offs,
                              const optional<Tensor>& flip, const Tensor& mean, const Tensor& inv_std,
                              at::ScalarType out_dtype) {
  check_cuda(in_, "images");
  const at::DeviceGuard guard(in_.device());
  TORCH_CHECK(in_.scalar_type() == at::kByte && in_.dim() == 4, "expected uint8 [N, H, W, C]");
  Tensor in = in_.contiguous();
  const int N = (int)in.size(0), Hi = (int)in.size(1), Wi = (int)in.size(2), C = (int)in.size(3);
  TORCH_CHECK(C >= 1 && C <= 4, "1..4 channels supported");
  Tensor m = mean.to(in.device(), at::kFloat).contiguous();
  Tensor is = inv_std.to(in.device(), at::kFloat).contiguous();
  TORCH_CHECK(m.numel() == C && is.numel() == C, "mean/std size");
  Tensor o, f;
  if (offs.has_value() && offs->defined()) {
    o = offs->to(in.device(), at::kInt).contiguous();
    TORCH_CHECK(o.numel() == 2 * N, "offsets must be [N, 2]");
  }
  if (flip.has_value() && flip->defined()) {
    f = flip->to(in.device(), at::kByte).contiguous();
    TORCH_CHECK(f.numel() == N, "flip must be [N]");
  }
  Tensor out = at::empty({N, Ho, Wo, C}, in.options().dtype(out_dtype));
  Tensor probe = out;
  tbamd::u8_crop_flip_normalize(dt_code(probe), in.data_ptr<uint8_t>(), N, Hi, Wi, C, (int)Ho, (int)Wo,
                                o.defined() ? o.data_ptr<int32_t>() : nullptr,
                                f.defined() ? f.data_ptr<uint8_t>() : nullptr, m.data_ptr<float>(),
                                is.data_ptr<float>(), out.data_ptr(), cur_stream());
  return out.permute({0, 3, 1, 2});
}

// images uint8 [Nsrc, Hi, Wi, C] (device); src int32 [B] rows (optional: 0..B-1); params f32 [B, 8]
// (see csrc/data.hip augment_u8_k) -> [B, C, Ho, Wo] channels_last
Tensor augment_u8(const Tensor& in_, const optional<Tensor>& src, int64_t Ho, int64_t Wo, const Tensor& params,
                  const Tensor& mean, const Tensor& inv_std, at::ScalarType out_dtype, bool crop_only) {
  check_cuda(in_, "images");
  const at::DeviceGuard guard(in_.device());
  TORCH_CHECK(in_.scalar_type() == at::kByte && in_.dim() == 4, "augment_u8: expected uint8 [N, H, W, C]");
  Tensor in = in_.contiguous();
  const int Hi = (int)in.size(1), Wi = (int)in.size(2), C = (int)in.size(3);
  TORCH_CHECK(crop_only || Ho * Wo * C <= tbamd::augment_max_bytes(),
              "augment_u8: rotation / RandAugment need the image in LDS (", tbamd::augment_max_bytes(),
              " B); larger images support crop + flip only");
  TORCH_CHECK(params.dim() == 2 && params.size(1) == 8, "augment_u8: params must be [B, 8]");
  const int B = (int)params.size(0);
  Tensor pr = params.to(in.device(), at::kFloat).contiguous();
  Tensor sr;
  if (src.has_value() && src->defined()) {
    sr = src->to(in.device(), at::kInt).contiguous();
    TORCH_CHECK(sr.numel() == B, "augment_u8: src must be [B]");
  } else {
    TORCH_CHECK(in.size(0) == B, "augment_u8: without src the batch is the image tensor");
  }
  Tensor m = mean.to(in.device(), at::kFloat).contiguous();
  Tensor is = inv_std.to(in.device(), at::kFloat).contiguous();
  TORCH_CHECK(m.numel() == C && is.numel() == C, "augment_u8: mean/std size");
  Tensor out = at::empty({B, Ho, Wo, C}, in.options().dtype(out_dtype));
  (crop_only ? tbamd::crop_flip_u8 : tbamd::augment_u8)(
      dt_code(out), in.data_ptr<uint8_t>(), sr.defined() ? sr.data_ptr<int32_t>() : nullptr, B, Hi, Wi, C, (int)Ho,
      (int)Wo, pr.data_ptr<float>(), m.data_ptr<float>(), is.data_ptr<float>(), out.data_ptr(), cur_stream());
  return out.permute({0, 3, 1, 2});
}

// ---------------------------------------------------------------- generic convolution
// x [N, C, H, W], w [K, C, R, S] (bf16 or f32, any layout), virtual input
// reflect-or-zero-pad(upsample_nearest(x, up)); NHWC (channels_last) outputs
static tbamd::ConvAnyShape any_shape(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
                                     int64_t stride, int64_t pad, int64_t up, int64_t dil, bool reflect) {
  const int64_t Hv = dil > 1 ? (H - 1) * dil + 1 : H * up, Wv = dil > 1 ? (W - 1) * dil + 1 : W * up;
  TORCH_CHECK(!reflect || (pad < Hv && pad < Wv), "conv_any: reflect padding must be smaller than the input");
  const int64_t P = (Hv + 2 * pad - R) / stride + 1, Q = (Wv + 2 * pad - S) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0 && stride >= 1 && up >= 1 && dil >= 1, "conv_any: bad geometry");
  return tbamd::ConvAnyShape{(int)N, (int)H, (int)W, (int)C, (int)K, (int)R, (int)S, (int)P, (int)Q,
                             (int)stride, (int)pad, (int)up, (int)dil, reflect ? 1 : 0};
}

static int any_f32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "conv_any: ", name,
              " must be f32 or bf16");
  return t.scalar_type() == at::kFloat ? 1 : 0;
}

Tensor conv_any_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride, int64_t pad,
                    int64_t up, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  const int f32 = any_f32(x_, "x");
  TORCH_CHECK(w_.scalar_type() == x_.scalar_type(), "conv_any: x and w dtypes differ");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor w = w_.permute({0, 2, 3, 1}).contiguous();  // [K][R][S][C]
  const auto sh = any_shape(x.size(0), x.size(1), x.size(2), x.size(3), w_.size(0), w_.size(2), w_.size(3),
                            stride, pad, up, 1, reflect);
  TORCH_CHECK(w_.size(1) == x.size(1), "conv_any: channel mismatch");
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(x.scalar_type()).contiguous();
  Tensor y = at::empty({sh.N, sh.K, sh.P, sh.Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_any_fwd(f32, x.data_ptr(), w.data_ptr(), b.defined() ? b.data_ptr() : nullptr, y.data_ptr(), sh,
                      cur_stream());
  return y;
}

// y = conv2d(pad(upsample_nearest(x, up), pad, reflect|zero), w, bias), stride 1, for K <= 16
// output channels (the RGB heads of the style-transfer decoders): halo-tile kernel
Tensor conv_narrow_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t pad, int64_t up,
                       bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16, "conv_narrow_fwd: bf16 only");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && w_.size(1) == x_.size(1), "conv_narrow_fwd: shape");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w_.size(0), R = (int)w_.size(2), S = (int)w_.size(3);
  TORCH_CHECK(tbamd::conv_narrow_supported(C, K, R, S, 1, (int)up), "conv_narrow_fwd: unsupported shape");
  TORCH_CHECK(!reflect || (pad < H * up && pad < W * up), "conv_narrow_fwd: reflect pad must be < input size");
  const int P = (int)(H * up + 2 * pad - R + 1), Q = (int)(W * up + 2 * pad - S + 1);
  TORCH_CHECK(P > 0 && Q > 0, "conv_narrow_fwd: empty output");
  Tensor w16 = at::zeros({16, R, S, C}, w_.options().memory_format(at::MemoryFormat::Contiguous));
  w16.narrow(0, 0, K).copy_(w_.permute({0, 2, 3, 1}));
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_narrow_fwd(x.data_ptr(), w16.data_ptr(), b.defined() ? b.data_ptr<float>() : nullptr, y.data_ptr(), N,
                         H, W, C, K, R, S, (int)pad, (int)up, reflect ? 1 : 0, cur_stream());
  return y;
}

// fp32 conv_narrow_fwd (the reference precision of the style-transfer examples): the halo-tile kernel
// splitting the fp32 halo into bf16 hi / lo in LDS, three MFMAs per pair (csrc/conv_narrow.hip conv_narrow_fwd32)
Tensor conv_narrow_fwd_split32(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t pad,
                               int64_t up, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kFloat && w_.scalar_type() == at::kFloat, "conv_narrow_fwd_split32: fp32 only");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && w_.size(1) == x_.size(1), "conv_narrow_fwd_split32: shape");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w_.size(0), R = (int)w_.size(2), S = (int)w_.size(3);
  TORCH_CHECK(tbamd::conv_narrow_supported(C, K, R, S, 1, (int)up) && x.numel() % 4 == 0,
              "conv_narrow_fwd_split32: unsupported shape");
  TORCH_CHECK(!reflect || (pad < H * up && pad < W * up), "conv_narrow_fwd_split32: reflect pad must be < input size");
  const int P = (int)(H * up + 2 * pad - R + 1), Q = (int)(W * up + 2 * pad - S + 1);
  TORCH_CHECK(P > 0 && Q > 0, "conv_narrow_fwd_split32: empty output");
  Tensor w16 = at::zeros({16, R, S, C}, w_.options().memory_format(at::MemoryFormat::Contiguous));
  w16.narrow(0, 0, K).copy_(w_.permute({0, 2, 3, 1}));
  Tensor w16h = w16.to(at::kBFloat16);
  Tensor w16l = (w16 - w16h.to(at::kFloat)).to(at::kBFloat16);
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_narrow_fwd32(x.data_ptr<float>(), w16h.data_ptr(), w16l.data_ptr(),
                           b.defined() ? b.data_ptr<float>() : nullptr, y.data_ptr<float>(), N, H, W, C, K, R, S,
                           (int)pad, (int)up, reflect ? 1 : 0, cur_stream());
  return y;
}

// y = conv_transpose2d(x, w, bias, stride, pad) for <= 16 output channels (the DCGAN generator's
// RGB head): st x st stride phases, each a narrow halo-tile forward with that phase's taps
Tensor conv_narrow_transpose_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride,
                                 int64_t pad) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16,
              "conv_narrow_transpose_fwd: bf16 only");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && w_.size(0) == x_.size(1) && w_.size(2) == w_.size(3),
              "conv_narrow_transpose_fwd: x [N, Ci, H, W], w [Ci, Co, R, R]");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w_.size(1), R = (int)w_.size(2), st = (int)stride, p = (int)pad;
  const int Ho = (H - 1) * st - 2 * p + R, Wo = (W - 1) * st - 2 * p + R;
  TORCH_CHECK(st >= 1 && Ho > 0 && Wo > 0, "conv_narrow_transpose_fwd: geometry");
  auto floordiv = [](int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); };
  auto ceildiv = [&](int a, int b) { return -floordiv(-a, b); };
  Tensor wt = w_.permute({1, 2, 3, 0});  // [Co][R][S][Ci]
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  Tensor y = at::empty({N, K, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  struct Ph { int dmax, taps, n; std::vector<int64_t> k; };
  auto phase = [&](int a, int n_out) {
    Ph ph{};
    ph.dmax = floordiv(R - 1 - a - p, st);
    const int dmin = ceildiv(-a - p, st);
    ph.taps = ph.dmax - dmin + 1;
    ph.n = n_out > a ? (n_out - a + st - 1) / st : 0;
    for (int r = 0; r < ph.taps; ++r) ph.k.push_back(st * (ph.dmax - r) + a + p);
    return ph;
  };
  for (int a = 0; a < st; ++a) {
    const Ph pa = phase(a, Ho);
    TORCH_CHECK(pa.taps >= 1 && pa.taps <= 9, "conv_narrow_transpose_fwd: phase taps");
    for (int bb = 0; bb < st; ++bb) {
      const Ph pb = phase(bb, Wo);
      TORCH_CHECK(pb.taps >= 1 && pb.taps <= 9, "conv_narrow_transpose_fwd: phase taps");
      TORCH_CHECK(tbamd::conv_narrow_supported(C, K, pa.taps, pb.taps, 1, 1), "conv_narrow_transpose_fwd: shape");
      if (pa.n == 0 || pb.n == 0) continue;
      // the phase's taps are ky = st * (dmax - r') + a + p: a stride-st slice of the kernel,
      // reversed (no index tensors, no host-to-device copies)
      const int64_t ky0 = pa.k.back(), kx0 = pb.k.back();
      Tensor sel = wt.slice(1, ky0, pa.k.front() + 1, st).slice(2, kx0, pb.k.front() + 1, st).flip({1, 2});
      Tensor w16 = at::zeros({16, pa.taps, pb.taps, C}, w_.options().memory_format(at::MemoryFormat::Contiguous));
      w16.narrow(0, 0, K).copy_(sel);
      tbamd::conv_narrow_fwd_phase(x.data_ptr(), w16.data_ptr(), b.defined() ? b.data_ptr<float>() : nullptr,
                                   y.data_ptr(), N, H, W, C, K, pa.taps, pb.taps, pa.dmax, pb.dmax, pa.n, pb.n, st, a,
                                   bb, Ho, Wo, cur_stream());
    }
  }
  return y;
}

static Tensor tiny_tab(const Tensor& x, int C, int R, int S);

// y = conv2d(pad(x), w, bias, stride) (+ ReLU) for C*R*S <= 256 input taps (RGB / grey input convs):
// the im2col row is gathered straight into the MFMA operand (csrc/conv_narrow.hip conv_tinyc_fwd)
Tensor conv_tinyc_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride, int64_t pad,
                      bool reflect, bool relu) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16, "conv_tinyc_fwd: bf16 only");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && w_.size(1) == x_.size(1), "conv_tinyc_fwd: shape");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w_.size(0), R = (int)w_.size(2), S = (int)w_.size(3);
  TORCH_CHECK(tbamd::conv_tinyc_supported(C, K, R, S) && stride >= 1, "conv_tinyc_fwd: unsupported shape");
  TORCH_CHECK(!reflect || (pad < H && pad < W), "conv_tinyc_fwd: reflect pad must be < input size");
  const int P = (int)((H + 2 * pad - R) / stride + 1), Q = (int)((W + 2 * pad - S) / stride + 1);
  TORCH_CHECK(P > 0 && Q > 0, "conv_tinyc_fwd: empty output");
  const int kred = C * R * S, KT = (kred + 31) / 32;
  Tensor wp = at::zeros({K, 32 * KT}, w_.options().memory_format(at::MemoryFormat::Contiguous));
  wp.narrow(1, 0, kred).copy_(w_.permute({0, 2, 3, 1}).reshape({K, kred}));
  Tensor tab = tiny_tab(x, C, R, S);
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_tinyc_fwd(x.data_ptr(), wp.data_ptr(), tab.data_ptr<int32_t>(), b.defined() ? b.data_ptr<float>() : nullptr,
                        y.data_ptr(), N, H, W, C, K, R, S, (int)stride, (int)pad, reflect ? 1 : 0, relu, cur_stream());
  return y;
}

// fp32 y = conv2d(pad(x), w, bias, stride) (+ ReLU) for C*R*S <= 256 input taps as split-bf16 MFMA (the
// im2col values split in registers, the packed weights as a hi / lo pair; csrc/conv_narrow.hip conv_tiny32_fwd)
Tensor conv_tiny32_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride, int64_t pad,
                       bool reflect, bool relu) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kFloat && w_.scalar_type() == at::kFloat, "conv_tiny32_fwd: fp32 only");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && w_.size(1) == x_.size(1), "conv_tiny32_fwd: shape");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w_.size(0), R = (int)w_.size(2), S = (int)w_.size(3);
  TORCH_CHECK(tbamd::conv_tinyc_supported(C, K, R, S) && stride >= 1, "conv_tiny32_fwd: unsupported shape");
  TORCH_CHECK(!reflect || (pad < H && pad < W), "conv_tiny32_fwd: reflect pad must be < input size");
  const int P = (int)((H + 2 * pad - R) / stride + 1), Q = (int)((W + 2 * pad - S) / stride + 1);
  TORCH_CHECK(P > 0 && Q > 0, "conv_tiny32_fwd: empty output");
  const int kred = C * R * S, KT = (kred + 31) / 32;
  Tensor wf = at::zeros({K, 32 * KT}, w_.options().memory_format(at::MemoryFormat::Contiguous));
  wf.narrow(1, 0, kred).copy_(w_.permute({0, 2, 3, 1}).reshape({K, kred}));
  Tensor wph = wf.to(at::kBFloat16);
  Tensor wpl = (wf - wph.to(at::kFloat)).to(at::kBFloat16);
  Tensor tab = tiny_tab(x, C, R, S);
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_tiny32_fwd(x.data_ptr<float>(), wph.data_ptr(), wpl.data_ptr(), tab.data_ptr<int32_t>(),
                         b.defined() ? b.data_ptr<float>() : nullptr, y.data_ptr<float>(), N, H, W, C, K, R, S,
                         (int)stride, (int)pad, reflect ? 1 : 0, relu, cur_stream());
  return y;
}

// stride-1 conv with C <= 4 input channels from an LDS halo tile (csrc/conv_narrow.hip conv_tinyhalo_fwd):
// bf16, or fp32 as split-bf16 (x split while staging, weights packed as a hi / lo pair)
Tensor conv_tinyhalo_fwd(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t pad, bool reflect,
                         bool relu) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  const bool f32 = x_.scalar_type() == at::kFloat;
  TORCH_CHECK((f32 || x_.scalar_type() == at::kBFloat16) && w_.scalar_type() == x_.scalar_type(),
              "conv_tinyhalo_fwd: fp32 or bf16");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && w_.size(1) == x_.size(1), "conv_tinyhalo_fwd: shape");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w_.size(0), R = (int)w_.size(2), S = (int)w_.size(3);
  TORCH_CHECK(tbamd::conv_tinyhalo_supported(C, K, R, S, 1, 1), "conv_tinyhalo_fwd: unsupported shape");
  TORCH_CHECK(!reflect || (pad < H && pad < W), "conv_tinyhalo_fwd: reflect pad must be < input size");
  const int P = (int)(H + 2 * pad - R + 1), Q = (int)(W + 2 * pad - S + 1);
  TORCH_CHECK(P > 0 && Q > 0, "conv_tinyhalo_fwd: empty output");
  const int KT = (R * S + 7) / 8;
  // [K][R*S][4] (channels past C zero) -> [K][32*KT] (taps past R*S zero)
  Tensor wf = at::zeros({K, 8 * KT, 4}, w_.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous));
  wf.narrow(1, 0, R * S).narrow(2, 0, C).copy_(w_.permute({0, 2, 3, 1}).reshape({K, R * S, C}));
  wf = wf.view({K, 32 * KT});
  Tensor wph = wf.to(at::kBFloat16);
  Tensor wpl = f32 ? (wf - wph.to(at::kFloat)).to(at::kBFloat16) : wph;
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_tinyhalo_fwd(f32, x.data_ptr(), wph.data_ptr(), wpl.data_ptr(), b.defined() ? b.data_ptr<float>() : nullptr,
                           y.data_ptr(), N, H, W, C, K, R, S, (int)pad, reflect ? 1 : 0, relu, cur_stream());
  return y;
}

// dW [K, C, R, S] (channels_last) of conv_tinyhalo_fwd's convolution (csrc/conv_narrow.hip conv_tinyhalo_wgrad)
Tensor conv_tinyhalo_wgrad(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t pad, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  const bool f32 = x_.scalar_type() == at::kFloat;
  TORCH_CHECK((f32 || x_.scalar_type() == at::kBFloat16) && dy_.scalar_type() == x_.scalar_type(),
              "conv_tinyhalo_wgrad: fp32 or bf16");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  TORCH_CHECK(tbamd::conv_tinyhalo_supported(C, K, (int)R, (int)S, 1, 1) && K <= 64, "conv_tinyhalo_wgrad: shape");
  TORCH_CHECK(!reflect || (pad < H && pad < W), "conv_tinyhalo_wgrad: reflect pad must be < input size");
  const int P = (int)(H + 2 * pad - R + 1), Q = (int)(W + 2 * pad - S + 1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == P && dy.size(3) == Q, "conv_tinyhalo_wgrad: dy shape");
  const int nb = tbamd::conv_tinyhalo_wgrad_blocks(N, H, W, (int)R, (int)S, (int)pad);
  const int NJ = tbamd::conv_tinyhalo_wgrad_cols((int)R, (int)S);
  Tensor part = at::empty({(int64_t)nb * K * 16 * NJ}, x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous));
  Tensor dw = at::empty({K, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_tinyhalo_wgrad(f32, x.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), dw.data_ptr(), N, H, W, C, K,
                             (int)R, (int)S, (int)pad, reflect ? 1 : 0, cur_stream());
  return dw;
}

// reduction index -> (r | s << 8 | c << 16) of the tiny-channel kernels, cached per (device, C, R, S)
static Tensor tiny_tab(const Tensor& x, int C, int R, int S) {
  const int kred = C * R * S;
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int>, Tensor> tabs;
  Tensor tab;
  {
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple((int)x.get_device(), C, R, S);
    auto it = tabs.find(key);
    if (it == tabs.end()) {
      std::vector<int32_t> h(kred);
      for (int k = 0; k < kred; ++k) {
        const int c = k % C, rs = k / C;
        h[k] = (rs / S) | ((rs % S) << 8) | (c << 16);
      }
      Tensor t = at::empty({kred}, at::TensorOptions().dtype(at::kInt));
      std::memcpy(t.data_ptr<int32_t>(), h.data(), sizeof(int32_t) * kred);
      it = tabs.emplace(key, t.to(x.device())).first;
    }
    tab = it->second;
  }
  return tab;
}

// dW [K, C, R, S] (channels_last) of conv_narrow_fwd's convolution: split-K partials over pixel
// fp32 narrow-output weight gradient (the style decoders' 9x9 RGB heads at the reference
// precision): dy and x split into bf16 (hi, lo) pairs, dW = dyh.xh + dyh.xl + dyl.xh as three
// halo-tile kernel runs into one f32 partial workspace, summed in f32
Tensor conv_narrow_wgrad_split32(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t pad, int64_t up,
                                 bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kFloat && dy_.scalar_type() == at::kFloat, "conv_narrow_wgrad_split32: fp32");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  TORCH_CHECK(tbamd::conv_narrow_supported(C, K, (int)R, (int)S, 1, (int)up), "conv_narrow_wgrad_split32: shape");
  TORCH_CHECK(!reflect || (pad < H * up && pad < W * up), "conv_narrow_wgrad_split32: reflect pad");
  TORCH_CHECK(x.numel() % 4 == 0 && dy.numel() % 4 == 0, "conv_narrow_wgrad_split32: numel % 4");
  const int P = (int)(H * up + 2 * pad - R + 1), Q = (int)(W * up + 2 * pad - S + 1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == P && dy.size(3) == Q, "conv_narrow_wgrad_split32: dy shape");
  auto bf = x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast);
  Tensor xh = at::empty_like(x, bf), xl = at::empty_like(x, bf), dyh = at::empty_like(dy, bf), dyl = at::empty_like(dy, bf);
  tbamd::split_bf16(x.data_ptr<float>(), x.numel(), (uint16_t*)xh.data_ptr(), (uint16_t*)xl.data_ptr(), cur_stream());
  tbamd::split_bf16(dy.data_ptr<float>(), dy.numel(), (uint16_t*)dyh.data_ptr(), (uint16_t*)dyl.data_ptr(),
                    cur_stream());
  const int splits = tbamd::conv_narrow_wgrad_splits(N, H, W, C, (int)R, (int)S, (int)pad, (int)up);
  Tensor part = at::empty({3 * splits, 16, R * S, C}, x.options().dtype(at::kFloat));
  const Tensor* xs[3] = {&xh, &xl, &xh};
  const Tensor* ds[3] = {&dyh, &dyh, &dyl};
  for (int t = 0; t < 3; ++t)
    tbamd::conv_narrow_wgrad(xs[t]->data_ptr(), ds[t]->data_ptr(), part.data_ptr<float>() + (int64_t)t * splits * 16 * R * S * C,
                             splits, N, H, W, C, K, (int)R, (int)S, (int)pad, (int)up, reflect ? 1 : 0, cur_stream());
  return part.narrow(1, 0, K).sum(0).view({K, R, S, C}).permute({0, 3, 1, 2});
}

// tiles [splits][16][R*S][C] f32 from the halo-tile kernel, summed here
Tensor conv_narrow_wgrad(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t pad, int64_t up,
                         bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kBFloat16 && dy_.scalar_type() == at::kBFloat16, "conv_narrow_wgrad: bf16 only");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  TORCH_CHECK(tbamd::conv_narrow_supported(C, K, (int)R, (int)S, 1, (int)up), "conv_narrow_wgrad: unsupported shape");
  TORCH_CHECK(!reflect || (pad < H * up && pad < W * up), "conv_narrow_wgrad: reflect pad must be < input size");
  const int P = (int)(H * up + 2 * pad - R + 1), Q = (int)(W * up + 2 * pad - S + 1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == P && dy.size(3) == Q, "conv_narrow_wgrad: dy shape");
  const int splits = tbamd::conv_narrow_wgrad_splits(N, H, W, C, (int)R, (int)S, (int)pad, (int)up);
  Tensor part = at::empty({splits, 16, R * S, C}, x.options().dtype(at::kFloat));
  tbamd::conv_narrow_wgrad(x.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), splits, N, H, W, C, K, (int)R,
                           (int)S, (int)pad, (int)up, reflect ? 1 : 0, cur_stream());
  Tensor dw = part.narrow(1, 0, K).sum(0).view({K, R, S, C}).permute({0, 3, 1, 2});
  return dw.to(at::kBFloat16);
}

// dW [K, C, R, S] (channels_last) for y = conv_any_fwd(x, w, stride, pad, up, reflect)
Tensor conv_any_wgrad(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t stride, int64_t pad,
                      int64_t up, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  const int f32 = any_f32(x_, "x");
  TORCH_CHECK(dy_.scalar_type() == x_.scalar_type(), "conv_any: x and dy dtypes differ");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const auto sh = any_shape(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(1), R, S, stride, pad, up, 1,
                            reflect);
  TORCH_CHECK(dy.size(2) == sh.P && dy.size(3) == sh.Q && dy.size(0) == sh.N, "conv_any_wgrad: dy shape");
  const int splits = tbamd::conv_any_wgrad_splits(sh);
  Tensor part = at::empty({(int64_t)splits * sh.K * R * S * sh.C}, x.options().dtype(at::kFloat));
  Tensor dw = at::empty({sh.K, sh.C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_any_wgrad(f32, x.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), splits, dw.data_ptr(), sh,
                        cur_stream());
  return dw;
}

// dX [N, C, H, W] (channels_last) for y = conv_any_fwd(x, w, stride, pad, up, reflect): the
// forward kernel on dy dilated by the stride with flipped weights (stride-phase tiles: only
// the taps that meet real dy pixels).  Zero padding without upsampling writes dX directly
// (output grid H x W, padding R-1-pad); reflect / upsampled inputs go through the padded
// virtual grid and the fold.  `wt`: the flipped transpose [C][R][S][K] when the caller
// keeps one cached (ops/conv.py _flipped), else built here.
Tensor conv_any_dgrad(const Tensor& dy_, const Tensor& w_, int64_t H, int64_t W, int64_t stride, int64_t pad,
                      int64_t up, bool reflect, const optional<Tensor>& wt_) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  const int f32 = any_f32(dy_, "dy");
  TORCH_CHECK(w_.scalar_type() == dy_.scalar_type(), "conv_any: dy and w dtypes differ");
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t K = w_.size(0), C = w_.size(1), R = w_.size(2), S = w_.size(3);
  const auto fwd = any_shape(dy.size(0), C, H, W, K, R, S, stride, pad, up, 1, reflect);
  TORCH_CHECK(dy.size(1) == K && dy.size(2) == fwd.P && dy.size(3) == fwd.Q, "conv_any_dgrad: dy shape");
  // flipped transpose as a [C][R][S][K] conv weight (out channels C, in channels K)
  Tensor wt;
  if (wt_.has_value() && wt_->defined()) {
    wt = wt_->permute({0, 2, 3, 1});
    TORCH_CHECK(wt.is_contiguous() && wt.size(0) == C && wt.size(1) == R && wt.size(2) == S && wt.size(3) == K &&
                    wt.scalar_type() == w_.scalar_type(),
                "conv_any_dgrad: wt must be the channels_last [C, K, R, S] flipped transpose");
  } else {
    wt = w_.flip({2, 3}).permute({1, 2, 3, 0}).contiguous();
  }
  if (!reflect && up == 1 && pad <= R - 1 && pad <= S - 1) {
    auto g = any_shape(dy.size(0), K, fwd.P, fwd.Q, C, R, S, 1, R - 1 - pad, 1, stride, false);
    TORCH_CHECK(g.P <= H && g.Q <= W, "conv_any_dgrad: internal geometry");
    g.P = (int)H;  // rows / cols no tap reaches get zero gradient (the padding reads)
    g.Q = (int)W;
    Tensor dx = at::empty({fwd.N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
    tbamd::conv_any_fwd(f32, dy.data_ptr(), wt.data_ptr(), nullptr, dx.data_ptr(), g, cur_stream());
    return dx;
  }
  const int64_t Hg = (int64_t)(fwd.P - 1) * stride + R, Wg = (int64_t)(fwd.Q - 1) * stride + S;
  auto g = any_shape(dy.size(0), K, fwd.P, fwd.Q, C, R, S, 1, R - 1, 1, stride, false);
  TORCH_CHECK(g.P == Hg && g.Q == Wg, "conv_any_dgrad: internal geometry");
  Tensor dxp = at::empty({g.N, Hg, Wg, C}, dy.options().memory_format(at::MemoryFormat::Contiguous));
  // wt is already [Cout=C][R][S][Cin=K]: pass it as the packed weight (conv_any_fwd reads [K][R][S][C])
  tbamd::conv_any_fwd(f32, dy.data_ptr(), wt.data_ptr(), nullptr, dxp.data_ptr(), g, cur_stream());
  Tensor dx = at::empty({fwd.N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_any_fold(f32, dxp.data_ptr(), (int)Hg, (int)Wg, dx.data_ptr(), fwd, cur_stream());
  return dx;
}

// ---------------------------------------------------------------- virtual-input 64-channel convs
// y = conv2d(pad(upsample_nearest(x, up), pad, reflect|zero), w, bias, stride) on the implicit-GEMM
// kernels (bf16, C % 64 == K % 64 == 0, up in {1, 2, 4}): the padded / upsampled input is never
// written (StyleNet residual blocks, AdaIN decoder)
static void virt_check(const Tensor& x, const Tensor& w, int64_t up, int64_t pad, bool reflect, const char* who) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, who, ": bf16 only");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && x.size(1) == w.size(1), who, ": shape");
  TORCH_CHECK(tbamd::conv_fwd_supported((int)x.size(1), (int)w.size(0)), who, ": needs C % 64 == 0 and K % 64 == 0");
  TORCH_CHECK(up == 1 || up == 2 || up == 4, who, ": up must be 1, 2 or 4");
  TORCH_CHECK(!reflect || (pad < x.size(2) * up && pad < x.size(3) * up), who, ": reflect pad must be < input size");
}

Tensor conv2d_fwd_virtual(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride,
                          int64_t pad, int64_t up, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  virt_check(x_, w_, up, pad, reflect, "conv2d_fwd_virtual");
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor w = w_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w.size(0), R = (int)w.size(2), S = (int)w.size(3);
  const int P = (H * (int)up + 2 * (int)pad - R) / (int)stride + 1, Q = (W * (int)up + 2 * (int)pad - S) / (int)stride + 1;
  TORCH_CHECK(P > 0 && Q > 0, "conv2d_fwd_virtual: empty output");
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor bf;
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  tbamd::conv_fwd_virtual(x.data_ptr(), w.data_ptr(), y.data_ptr(), bf.defined() ? bf.data_ptr<float>() : nullptr, N,
                          H, W, C, K, R, S, P, Q, (int)stride, (int)pad, (int)up, reflect ? 1 : 0, cur_stream());
  return y;
}

// dW [K, C, R, S] (channels_last) of conv2d_fwd_virtual
// (hi, lo) bf16 pair of an f32 tensor, same sizes and strides (the layout of t is kept)
std::vector<Tensor> split_bf16(const Tensor& t_) {
  check_cuda(t_, "t");
  const at::DeviceGuard guard(t_.device());
  TORCH_CHECK(t_.scalar_type() == at::kFloat, "split_bf16: fp32");
  const bool cl = t_.dim() == 4 && !t_.is_contiguous() && t_.is_contiguous(at::MemoryFormat::ChannelsLast);
  Tensor t = cl ? t_ : t_.contiguous();
  TORCH_CHECK(t.numel() % 4 == 0, "split_bf16: numel % 4");
  Tensor hi = at::empty_like(t, t.options().dtype(at::kBFloat16));
  Tensor lo = at::empty_like(t, t.options().dtype(at::kBFloat16));
  tbamd::split_bf16(t.data_ptr<float>(), t.numel(), (uint16_t*)hi.data_ptr(), (uint16_t*)lo.data_ptr(), cur_stream());
  return {hi, lo};
}

// y = conv2d(x, w) (+ bias, ReLU) in fp32 from split-bf16 operands (csrc/conv.hip conv_fwd_split_k):
// xh/xl [N, C, H, W] channels_last, wh/wl [K, C, R, S] channels_last bf16, C % 64 == K % 64 == 0
Tensor conv2d_fwd_split32(const Tensor& xh, const Tensor& xl, const Tensor& wh, const Tensor& wl,
                          const optional<Tensor>& bias, int64_t stride, int64_t pad, bool relu) {
  check_cuda(xh, "xh");
  const at::DeviceGuard guard(xh.device());
  for (const Tensor* t : {&xh, &xl, &wh, &wl})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv2d_fwd_split32: bf16 channels_last operands");
  const int N = (int)xh.size(0), C = (int)xh.size(1), H = (int)xh.size(2), W = (int)xh.size(3);
  const int K = (int)wh.size(0), R = (int)wh.size(2), S = (int)wh.size(3);
  TORCH_CHECK(wh.size(1) == C && C % 64 == 0 && K % 64 == 0 && xl.sizes() == xh.sizes() && wl.sizes() == wh.sizes(),
              "conv2d_fwd_split32: shapes");
  const int P = (H + 2 * (int)pad - R) / (int)stride + 1, Q = (W + 2 * (int)pad - S) / (int)stride + 1;
  Tensor y = at::empty({N, K, P, Q}, xh.options().dtype(at::kFloat).memory_format(at::MemoryFormat::ChannelsLast));
  Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b.numel() == K, "conv2d_fwd_split32: bias");
  }
  const int ns = tbamd::conv_fwd_split32_ksplit(N, C, K, R, S, P, Q);
  Tensor part;  // few output pixels: the reduction is split over workgroups (f32 partials)
  if (ns > 1) part = at::empty({(int64_t)ns * N * P * Q * K}, y.options().memory_format(at::MemoryFormat::Contiguous));
  tbamd::conv_fwd_split32(xh.data_ptr(), xl.data_ptr(), wh.data_ptr(), wl.data_ptr(), y.data_ptr<float>(),
                          b.defined() ? b.data_ptr<float>() : nullptr, relu, N, H, W, C, K, R, S, P, Q, (int)stride,
                          (int)pad, cur_stream(), ns > 1 ? part.data_ptr<float>() : nullptr);
  return y;
}

// bf16 forward of a few-pixel conv with the reduction split over workgroups (csrc/conv.hip
// conv_fwd_splitk_bf16): VGG-19 512-channel maps at batch 1; C % 64 == 0, K % 128 == 0
Tensor conv2d_fwd_splitk(const Tensor& x_, const Tensor& w_, const optional<Tensor>& bias, int64_t stride, int64_t pad,
                         bool relu) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast), w = w_.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv2d_fwd_splitk: bf16");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w.size(0), R = (int)w.size(2), S = (int)w.size(3);
  TORCH_CHECK(w.size(1) == C && C % 64 == 0 && K % 128 == 0 && stride >= 1 && pad >= 0, "conv2d_fwd_splitk: shapes");
  const int P = (H + 2 * (int)pad - R) / (int)stride + 1, Q = (W + 2 * (int)pad - S) / (int)stride + 1;
  TORCH_CHECK(P > 0 && Q > 0, "conv2d_fwd_splitk: empty output");
  Tensor y = at::empty({N, K, P, Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b.numel() == K, "conv2d_fwd_splitk: bias");
  }
  const int ns = std::max(1, tbamd::conv_fwd_splitk_bf16_ksplit(N, C, K, R, S, P, Q));
  Tensor part = at::empty({(int64_t)ns * N * P * Q * K}, x.options().dtype(at::kFloat));
  tbamd::conv_fwd_splitk_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), b.defined() ? b.data_ptr<float>() : nullptr,
                              relu, N, H, W, C, K, R, S, P, Q, (int)stride, (int)pad, part.data_ptr<float>(), ns,
                              cur_stream());
  return y;
}

// fp32 dW [K, C, R, S] (channels_last) of a conv over pad(upsample(x)) on the bf16 MFMA weight-gradient
// kernel with split-bf16 operands (csrc/conv_wgrad.hip conv_wgrad_split32); C % 64 == K % 64 == 0
Tensor conv2d_wgrad_split32(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t stride, int64_t pad,
                            int64_t up, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  TORCH_CHECK(dy.scalar_type() == at::kFloat && x.scalar_type() == at::kFloat, "conv2d_wgrad_split32: fp32");
  TORCH_CHECK(C % 64 == 0 && K % 64 == 0 && (up == 1 || up == 2 || up == 4), "conv2d_wgrad_split32: channels / up");
  const int P = (H * (int)up + 2 * (int)pad - (int)R) / (int)stride + 1;
  const int Q = (W * (int)up + 2 * (int)pad - (int)S) / (int)stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == P && dy.size(3) == Q, "conv2d_wgrad_split32: dy shape");
  TORCH_CHECK((int64_t)N * P * Q < (1ll << 31), "conv2d_wgrad_split32: too many output pixels");
  Tensor dw = at::empty({K, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto bf = x.options().dtype(at::kBFloat16);
  Tensor dyh = at::empty({dy.numel()}, bf), dyl = at::empty({dy.numel()}, bf);
  Tensor xh = at::empty({x.numel()}, bf), xl = at::empty({x.numel()}, bf);
  Tensor work = at::empty({tbamd::conv_wgrad_split32_workspace(N, H, W, C, K, (int)R, (int)S, P, Q, (int)stride,
                                                               (int)pad)}, x.options());
  tbamd::conv_wgrad_split32(dy.data_ptr<float>(), x.data_ptr<float>(), dw.data_ptr<float>(),
                            (uint16_t*)dyh.data_ptr(), (uint16_t*)dyl.data_ptr(), (uint16_t*)xh.data_ptr(),
                            (uint16_t*)xl.data_ptr(), work.data_ptr<float>(), N, H, W, C, K, (int)R, (int)S, P, Q,
                            (int)stride, (int)pad, (int)up, reflect ? 1 : 0, cur_stream());
  return dw;
}

Tensor conv2d_wgrad_virtual(const Tensor& dy_, const Tensor& x_, int64_t R, int64_t S, int64_t stride, int64_t pad,
                            int64_t up, bool reflect) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "conv2d_wgrad_virtual: bf16");
  TORCH_CHECK(C % 64 == 0 && K % 32 == 0 && (up == 1 || up == 2 || up == 4), "conv2d_wgrad_virtual: channels / up");
  const int P = (H * (int)up + 2 * (int)pad - (int)R) / (int)stride + 1;
  const int Q = (W * (int)up + 2 * (int)pad - (int)S) / (int)stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == P && dy.size(3) == Q, "conv2d_wgrad_virtual: dy shape");
  Tensor dw = at::empty({K, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t ws = tbamd::conv_wgrad_workspace(N, H, W, C, K, (int)R, (int)S, P, Q, (int)stride, (int)pad);
  Tensor work;
  if (ws > 0) work = at::empty({ws}, x.options().dtype(at::kFloat));
  tbamd::conv_wgrad_virtual(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws > 0 ? work.data_ptr<float>() : nullptr,
                            N, H, W, C, K, (int)R, (int)S, P, Q, (int)stride, (int)pad, (int)up, reflect ? 1 : 0,
                            cur_stream());
  return dw;
}

// dX [N, C, H, W] of conv2d_fwd_virtual: the gradient on the padded virtual grid from the
// 64-channel dgrad kernels (stride 1: flipped-weight forward with padding R-1; stride 2: the
// four parity classes), folded back onto x (reflect mirror images, upsampled copies)
// wt = conv_flip_weight(w) [C, K, R, S] channels_last
Tensor conv2d_dgrad_virtual(const Tensor& dy_, const Tensor& wt_, int64_t H, int64_t W, int64_t stride, int64_t pad,
                            int64_t up, bool reflect) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor dy = dy_.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor wt = wt_.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && wt.scalar_type() == at::kBFloat16, "conv2d_dgrad_virtual: bf16");
  const int N = (int)dy.size(0), K = (int)dy.size(1), P = (int)dy.size(2), Q = (int)dy.size(3);
  const int C = (int)wt.size(0), R = (int)wt.size(2), S = (int)wt.size(3);
  TORCH_CHECK(wt.size(1) == K && tbamd::conv_fwd_supported(K, C), "conv2d_dgrad_virtual: wt [C, K, R, S], % 64");
  TORCH_CHECK(stride == 1 || (stride == 2 && tbamd::conv_dgrad_s2_supported(R, S, 2)),
              "conv2d_dgrad_virtual: stride 1, or 2 with <= 16 taps per phase class");
  const int Hp = (int)(H * up + 2 * pad), Wp = (int)(W * up + 2 * pad);
  TORCH_CHECK(P == (Hp - R) / (int)stride + 1 && Q == (Wp - S) / (int)stride + 1, "conv2d_dgrad_virtual: geometry");
  Tensor dxp = at::empty({N, C, Hp, Wp}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (stride == 1) {
    TORCH_CHECK(R == S, "conv2d_dgrad_virtual: square taps");
    tbamd::conv_fwd(dy.data_ptr(), wt.data_ptr(), dxp.data_ptr(), nullptr, nullptr, nullptr, nullptr, false, N, P, Q, K,
                    C, R, S, Hp, Wp, 1, R - 1, cur_stream());
  } else {
    tbamd::conv_dgrad_s2(dy.data_ptr(), wt.data_ptr(), dxp.data_ptr(), N, P, Q, K, C, R, S, 0, Hp, Wp, cur_stream());
  }
  const tbamd::ConvAnyShape fwd{N, (int)H, (int)W, C, K, R, S, P, Q, (int)stride, (int)pad, (int)up, 1, reflect ? 1 : 0};
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::conv_any_fold(0, dxp.data_ptr(), Hp, Wp, dx.data_ptr(), fwd, cur_stream());
  return dx;
}

// ---------------------------------------------------------------- global average pool (K7)
// x [N, C, H, W] channels_last (C % 8 == 0) -> [N, C]
Tensor global_avgpool(const Tensor& x_) {
  check_cuda(x_, "x");
  const at::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), C = (int)x.size(1), HW = (int)(x.size(2) * x.size(3));
  TORCH_CHECK(C % 8 == 0, "global_avgpool: C % 8 == 0");
  Tensor y = at::empty({N, C}, x.options());
  tbamd::global_avgpool_fwd(dt_code(x), x.data_ptr(), N, HW, C, y.data_ptr(), cur_stream());
  return y;
}

// dy [N, C] -> dx [N, C, H, W] channels_last = dy / (H W) broadcast
Tensor global_avgpool_backward(const Tensor& dy_, int64_t H, int64_t W) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  Tensor dy = dy_.contiguous();
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  TORCH_CHECK(C % 8 == 0, "global_avgpool_backward: C % 8 == 0");
  Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::global_avgpool_bwd(dt_code(dy), dy.data_ptr(), N, (int)(H * W), C, dx.data_ptr(), cur_stream());
  return dx;
}

// ---------------------------------------------------------------- attention
// q, k, v (and dq, dk, dv, o, dout): [B, H, N, 64] bf16 views with a unit
// head-dim stride and 16-B aligned rows (any batch/head/token strides, so the
// packed qkv projection output is consumed and the packed dqkv written in place)
static void attn_view(const Tensor& t, const char* name, int64_t B, int64_t H, int64_t N, const uint16_t** p,
                      int64_t* s) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.dim() == 4, "attention: ", name, " must be bf16 [B, H, N, D]");
  TORCH_CHECK(t.size(0) == B && t.size(1) == H && t.size(2) == N && t.size(3) == 64 && t.stride(3) == 1,
              "attention: ", name, " shape/stride mismatch (head dim 64, unit stride)");
  for (int i = 0; i < 3; ++i) {
    TORCH_CHECK(t.stride(i) % 8 == 0 || t.size(i) == 1, "attention: ", name, " strides must be multiples of 8");
    s[i] = t.stride(i);
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "attention: ", name, " not 16-B aligned");
  *p = reinterpret_cast<const uint16_t*>(t.data_ptr());
}

// -> (o [B, N, H, 64] contiguous, lse [B, H, N] f32)
std::vector<Tensor> attn_forward(const Tensor& q, const Tensor& k, const Tensor& v, double scale) {
  const at::DeviceGuard guard(q.device());
  const int64_t B = q.size(0), H = q.size(1), N = q.size(2);
  TORCH_CHECK(N >= 1 && B * H * ((N + 127) / 128) < (int64_t)INT32_MAX, "attention: bad size");
  tbamd::AttnArgs a{};
  attn_view(q, "q", B, H, N, &a.q, a.sq);
  attn_view(k, "k", B, H, N, &a.k, a.sk);
  attn_view(v, "v", B, H, N, &a.v, a.sv);
  Tensor o = at::empty({B, N, H, 64}, q.options());
  Tensor lse = at::empty({B, H, N}, q.options().dtype(at::kFloat));
  Tensor ov = o.permute({0, 2, 1, 3});
  const uint16_t* op;
  attn_view(ov, "o", B, H, N, &op, a.so);
  a.o = const_cast<uint16_t*>(op);
  a.lse = lse.data_ptr<float>();
  a.B = (int)B, a.H = (int)H, a.N = (int)N, a.scale = (float)scale;
  tbamd::attn_fwd(a, cur_stream());
  return {o, lse};
}

// writes dq, dk, dv (views, e.g. slices of one packed dqkv buffer)
void attn_backward(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& dout,
                   const Tensor& lse, double scale, const Tensor& dq, const Tensor& dk, const Tensor& dv) {
  const at::DeviceGuard guard(q.device());
  const int64_t B = q.size(0), H = q.size(1), N = q.size(2);
  tbamd::AttnArgs a{};
  attn_view(q, "q", B, H, N, &a.q, a.sq);
  attn_view(k, "k", B, H, N, &a.k, a.sk);
  attn_view(v, "v", B, H, N, &a.v, a.sv);
  const uint16_t* p;
  attn_view(o, "o", B, H, N, &p, a.so);
  a.o = const_cast<uint16_t*>(p);
  attn_view(dout, "dout", B, H, N, &a.dout, a.sdo);
  attn_view(dq, "dq", B, H, N, &p, a.sdq);
  a.dq = const_cast<uint16_t*>(p);
  attn_view(dk, "dk", B, H, N, &p, a.sdk);
  a.dk = const_cast<uint16_t*>(p);
  attn_view(dv, "dv", B, H, N, &p, a.sdv);
  a.dv = const_cast<uint16_t*>(p);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * N, "attention: lse");
  Tensor delta = at::empty({B, H, N}, lse.options());
  a.lse = lse.data_ptr<float>();
  a.delta = delta.data_ptr<float>();
  a.B = (int)B, a.H = (int)H, a.N = (int)N, a.scale = (float)scale;
  tbamd::attn_bwd(a, cur_stream());
}

// ------------------------------------------------------------ Gram matrix
// f: [B, C, H, W] bf16 channels_last (NHWC memory) -> [B, C, C] f32 = F_b^T F_b * scale
// x: bf16 [N, C, H, W] channels_last -> col [N*P*Q, KP] (KP = RSC rounded up to 8)
Tensor im2col(const Tensor& x, int64_t R, int64_t S, int64_t P, int64_t Q, int64_t stride, int64_t pad, int64_t up,
              bool reflect) {
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "im2col: expected bf16 channels_last [N, C, H, W]");
  TORCH_CHECK(up == 1 || up == 2 || up == 4, "im2col: upsample 1, 2 or 4");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t KP = (R * S * C + 7) / 8 * 8;
  Tensor col = at::empty({N * P * Q, KP}, x.options().memory_format(at::MemoryFormat::Contiguous));
  tbamd::im2col_nhwc(x.data_ptr(), col.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)R, (int)S, (int)P, (int)Q,
                     (int)stride, (int)pad, (int)up, reflect ? 1 : 0, (int)KP, cur_stream());
  return col;
}

// col [N*P*Q, KP] -> dx bf16 [N, C, H, W] channels_last (gather; + bias[C] when given)
Tensor col2im(const Tensor& col, int64_t N, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S, int64_t P,
              int64_t Q, int64_t stride, int64_t pad, const c10::optional<Tensor>& bias) {
  TORCH_CHECK(col.is_cuda() && col.dtype() == at::kBFloat16 && col.dim() == 2 && col.is_contiguous(),
              "col2im: expected contiguous bf16 [M, KP]");
  const int64_t KP = col.size(1);
  TORCH_CHECK(col.size(0) == N * P * Q && KP >= R * S * C, "col2im: col shape");
  Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(at::kBFloat16).contiguous();
    TORCH_CHECK(b.numel() == C, "col2im: bias size");
  }
  Tensor dx = at::empty({N, C, H, W}, col.options().memory_format(at::MemoryFormat::ChannelsLast));
  tbamd::col2im_nhwc(col.data_ptr(), dx.data_ptr(), b.defined() ? b.data_ptr() : nullptr, (int)N, (int)H, (int)W,
                     (int)C, (int)R, (int)S, (int)P, (int)Q, (int)stride, (int)pad, (int)KP, cur_stream());
  return dx;
}

// [B][C][C] f32 gradient of the Gram -> bf16 (dG + dG^T) * scale
Tensor gram_sym(const Tensor& dg, double scale) {
  TORCH_CHECK(dg.is_cuda() && dg.dtype() == at::kFloat && dg.dim() == 3 && dg.size(1) == dg.size(2),
              "gram_sym: expected f32 [B, C, C]");
  Tensor d = dg.contiguous();
  Tensor out = at::empty(d.sizes(), d.options().dtype(at::kBFloat16));
  tbamd::gram_sym(d.data_ptr<float>(), out.data_ptr(), (int)d.size(0), (int)d.size(1), (float)scale, cur_stream());
  return out;
}

Tensor gram_forward(const Tensor& f, double scale) {
  check_cuda(f, "features");
  const at::DeviceGuard guard(f.device());
  TORCH_CHECK(f.scalar_type() == at::kBFloat16 && f.dim() == 4 && f.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gram: expected bf16 channels_last [B, C, H, W]");
  const int B = (int)f.size(0), C = (int)f.size(1);
  const int64_t HW = f.size(2) * f.size(3);
  TORCH_CHECK(tbamd::gram_tile(C) > 0, "gram: C must be a multiple of 64");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(f.data_ptr()) % 16 == 0, "gram: features not 16-B aligned");
  Tensor ws = at::empty({tbamd::gram_workspace(B, C, HW)}, f.options().dtype(at::kFloat));
  Tensor out = at::empty({B, C, C}, f.options().dtype(at::kFloat));
  tbamd::gram(f.data_ptr(), B, HW, C, (float)scale, ws.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

// --------------------------------------------- bias gradients / GELU backward
static Tensor colsum_out(const Tensor& dy, const optional<Tensor>& out) {
  const int64_t C = dy.size(1);
  if (out.has_value() && out->defined()) {  // zero-copy gradient slot
    TORCH_CHECK(out->numel() == C && out->is_contiguous() && out->scalar_type() == dy.scalar_type(),
                "colsum: out must be a contiguous [C] tensor of dy's dtype");
    return *out;
  }
  return at::empty({C}, dy.options());
}

// dy: [M, C] -> [C] column sums (the bias gradient), in dy's dtype
Tensor colsum(const Tensor& dy_, const optional<Tensor>& out) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  TORCH_CHECK(dy_.dim() == 2 && dy_.size(1) % 8 == 0, "colsum: expected [M, C] with C % 8 == 0");
  Tensor dy = as_rows(dy_);
  const int64_t M = dy.size(0);
  const int C = (int)dy.size(1);
  Tensor o = colsum_out(dy, out);
  Tensor part = at::empty({(int64_t)tbamd::colsum_splits(M, C) * C}, dy.options().dtype(at::kFloat));
  tbamd::colsum(dt_code(dy), dy.data_ptr(), nullptr, nullptr, M, C, part.data_ptr<float>(), o.data_ptr(),
                cur_stream());
  return o;
}

// (dz = dy * GELU'(z), column sums of dz)
// y = GELU(z) (exact erf) on a contiguous tensor with numel % 8 == 0
Tensor gelu_fwd(const Tensor& z_) {
  check_cuda(z_, "z");
  const at::DeviceGuard guard(z_.device());
  Tensor z = z_.contiguous();
  TORCH_CHECK(z.numel() % 8 == 0, "gelu_fwd: numel must be a multiple of 8");
  Tensor y = at::empty_like(z);
  tbamd::gelu_forward(dt_code(z), z.data_ptr(), y.data_ptr(), z.numel(), cur_stream());
  return y;
}

std::vector<Tensor> gelu_bwd_colsum(const Tensor& dy_, const Tensor& z_, const optional<Tensor>& out) {
  check_cuda(dy_, "dy");
  const at::DeviceGuard guard(dy_.device());
  TORCH_CHECK(dy_.dim() == 2 && dy_.size(1) % 8 == 0 && z_.sizes() == dy_.sizes(),
              "gelu_bwd_colsum: expected matching [M, C] with C % 8 == 0");
  Tensor z = as_rows(z_);
  Tensor dy = as_rows(dy_.to(z.scalar_type()));
  const int64_t M = dy.size(0);
  const int C = (int)dy.size(1);
  Tensor dz = at::empty_like(dy);
  Tensor o = colsum_out(dy, out);
  Tensor part = at::empty({(int64_t)tbamd::colsum_splits(M, C) * C}, dy.options().dtype(at::kFloat));
  tbamd::colsum(dt_code(dy), dy.data_ptr(), z.data_ptr(), dz.data_ptr(), M, C, part.data_ptr<float>(), o.data_ptr(),
                cur_stream());
  return {dz, o};
}

// dZ = (dy @ w) * GELU'(z) and db = column sums of dZ, in one 8-phase NN GEMM (csrc/gemm8.hip):
// the input gradient of a Linear whose input was GELU(z) fused with that GELU's backward and the
// preceding Linear's bias gradient (ViT MLP fc2 -> fc1).  dy [P][K], w [K][Q], z [P][Q] bf16.
std::vector<Tensor> gemm_nn_gelu_bwd(const Tensor& dy, const Tensor& w_, const Tensor& z_, const optional<Tensor>& db_out,
                                     const optional<Tensor>& wt = {});

// ---------------------------------------------------------------- dense GEMM
static void check_rows_bf16(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "gemm: ", name, " must be bf16");
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 8 == 0, "gemm: ", name,
              " must be a 2-D row-major view with a row stride multiple of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "gemm: ", name, " must be 16-B aligned");
}

// y = epi(x @ w^T) (tw false, w [Q][K]) or epi(x @ w) (tw true, w [K][Q]); x [P][K], or
// x [K][P] with tx (y = x^T @ ...).  splits > 1: split-K with f32 partials (no epilogue);
// splits = 0: automatic split count (no epilogue only).
std::vector<Tensor> gemm(const Tensor& x, const Tensor& w, bool tw, const optional<Tensor>& bias,
                         const optional<Tensor>& residual, int64_t epi, bool want_z, int64_t tile,
                         const optional<Tensor>& out, bool tx, int64_t splits) {
  check_rows_bf16(x, "x");
  const at::DeviceGuard guard(x.device());
  Tensor wc = w.contiguous();
  check_rows_bf16(wc, "w");
  const int64_t P = tx ? x.size(1) : x.size(0), K = tx ? x.size(0) : x.size(1);
  const int64_t Q = tw ? wc.size(1) : wc.size(0);
  TORCH_CHECK((tw ? wc.size(0) : wc.size(1)) == K, "gemm: inner dimensions differ");
  // row-read operands move k in 16-B chunks; transposed ones move whole k rows
  TORCH_CHECK(Q % 8 == 0 && ((tx && tw) || K % 8 == 0), "gemm: Q (and K unless both operands are transposed) "
              "must be multiples of 8");
  TORCH_CHECK(!tx || P % 8 == 0, "gemm: P must be a multiple of 8 with a transposed x");
  TORCH_CHECK(P < (1ll << 31) && Q < (1ll << 31) && K < (1ll << 31), "gemm: dims too large");
  Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    check_rows_bf16(y, "out");
    TORCH_CHECK(y.size(0) == P && y.size(1) == Q, "gemm: out shape");
  } else {
    y = at::empty({P, Q}, x.options());
  }
  const void* bp = nullptr;
  Tensor bc;
  if (bias.has_value() && bias->defined()) {
    bc = bias->to(at::kBFloat16).contiguous();
    TORCH_CHECK(bc.numel() == Q, "gemm: bias size");
    bp = bc.data_ptr();
  }
  const void* rp = nullptr;
  Tensor rc;
  if (residual.has_value() && residual->defined()) {
    rc = residual->to(at::kBFloat16).contiguous();
    TORCH_CHECK(rc.dim() == 2 && rc.size(0) == P && rc.size(1) == Q && y.stride(0) == Q, "gemm: residual shape");
    rp = rc.data_ptr();
  }
  TORCH_CHECK(!((epi == 1 || epi == 2 || epi == 3 || epi == 6) && bp == nullptr), "gemm: epilogue needs a bias");
  TORCH_CHECK(!((epi == 3 || epi == 4) && rp == nullptr), "gemm: epilogue needs a residual");
  int t = (int)tile;
  if (t < 0 || t >= tbamd::gemm_num_tiles()) t = tbamd::gemm_pick_tile((int)P, (int)Q, (int)K);
  int s = (int)splits;
  if (s == 0) s = epi == 0 ? tbamd::gemm_pick_splits((int)P, (int)Q, (int)K, t) : 1;
  if (t >= 16 && !tx) s = 1;  // the 8-phase NT / NN kernel (and its whole-round + tail split) runs whole-k tiles
  TORCH_CHECK(s == 1 || epi == 0, "gemm: split-K has no epilogue");
  Tensor part;
  if (s > 1) {
    part = at::empty({(int64_t)s * P * Q}, x.options().dtype(at::kFloat));
  }
  Tensor z;
  if (epi == 2 && want_z) z = at::empty({P, Q}, x.options());
  tbamd::gemm_bf16(x.data_ptr(), x.stride(0), tx, wc.data_ptr(), tw, y.data_ptr(), y.stride(0), bp, rp,
                   z.defined() ? z.data_ptr() : nullptr, (int)P, (int)Q, (int)K, (int)epi, t, s,
                   part.defined() ? part.data_ptr<float>() : nullptr, cur_stream());
  if (z.defined()) return {y, z};
  return {y};
}

std::vector<Tensor> gemm_nn_gelu_bwd(const Tensor& dy, const Tensor& w_, const Tensor& z_,
                                     const optional<Tensor>& db_out, const optional<Tensor>& wt_) {
  check_rows_bf16(dy, "dy");
  const at::DeviceGuard guard(dy.device());
  Tensor w = w_.contiguous();
  Tensor z = z_.contiguous();
  check_rows_bf16(w, "w");
  check_rows_bf16(z, "z");
  const int64_t P = dy.size(0), K = dy.size(1), Q = w.size(1);
  TORCH_CHECK(w.size(0) == K && z.size(0) == P && z.size(1) == Q, "gemm_nn_gelu_bwd: shapes");
  TORCH_CHECK(tbamd::gemm8_nn_supported((int)P, (int)Q, (int)K, dy.stride(0)),
              "gemm_nn_gelu_bwd: needs K % 64 == 0 and Q % 8 == 0");
  Tensor y = at::empty({P, Q}, dy.options());
  const int ntp = (int)((P + 255) / 256);
  Tensor part = at::empty({(int64_t)ntp * Q}, dy.options().dtype(at::kFloat));
  Tensor db;
  if (db_out.has_value() && db_out->defined()) {
    db = *db_out;
    TORCH_CHECK(db.is_contiguous() && db.numel() == Q, "gemm_nn_gelu_bwd: db_out");
  } else {
    db = at::empty({Q}, dy.options());
  }
  if (wt_.has_value() && wt_->defined()) {  // wt = wᵀ [Q][K]: the NT kernel (row-read operands)
    const Tensor& wt = *wt_;
    check_rows_bf16(wt, "wt");
    TORCH_CHECK(wt.is_contiguous() && wt.size(0) == Q && wt.size(1) == K, "gemm_nn_gelu_bwd: wt must be w^T");
    tbamd::gemm8_nt_gelu_bwd_bf16(dy.data_ptr(), dy.stride(0), wt.data_ptr(), y.data_ptr(), Q, z.data_ptr(),
                                  part.data_ptr<float>(), (int)P, (int)Q, (int)K, cur_stream());
  } else {
    tbamd::gemm8_nn_bf16(dy.data_ptr(), dy.stride(0), w.data_ptr(), y.data_ptr(), Q, z.data_ptr(),
                         part.data_ptr<float>(), (int)P, (int)Q, (int)K, cur_stream());
  }
  tbamd::colsum_finalize(dt_code(db), part.data_ptr<float>(), ntp, (int)Q, db.data_ptr(), cur_stream());
  return {y, db};
}

}  // namespace

void register_runtime(pybind11::module& m);

// ---- bounds-checked debug build: every kernel file registers a reader of its flag
static std::vector<unsigned (*)()>& bounds_readers() {
  static std::vector<unsigned (*)()> r;
  return r;
}
namespace tbamd {
void bounds_register_reader(unsigned (*reader)()) { bounds_readers().push_back(reader); }
}  // namespace tbamd

// OR of every kernel file's violation bits since the last call (0 in normal builds)
static int64_t bounds_check() {
  unsigned v = 0;
  for (auto* r : bounds_readers()) v |= r();
  return (int64_t)v;
}

static bool bounds_enabled() {
#ifdef TBAMD_BOUNDS
  return true;
#else
  return false;
#endif
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("bounds_check", &bounds_check, "OR of the bounds-violation bits since the last call (debug build)");
  m.def("bounds_enabled", &bounds_enabled);
  // x[i] through one guarded device read (normal build: unchecked; bounds build: -1 + flag when i >= numel)
  m.def("bounds_probe", [](const Tensor& x, int64_t i) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "bounds_probe: f32 cuda tensor");
    Tensor out = at::empty({1}, x.options());
    // (the probe is only ever called with i inside the allocation's first page in tests)
    tbamd::bounds_probe(x.data_ptr<float>(), x.numel(), i, out.data_ptr<float>(), cur_stream());
    return out;
  });
  m.doc() = "torchbooster_amd native library (gfx950 HIP kernels + C++ runtime)";
  m.def("bn_forward", &bn_forward, py::arg("x"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("training"), py::arg("momentum"), py::arg("eps"), py::arg("residual"),
        py::arg("act"), py::arg("slope"), py::arg("num_batches_tracked") = py::none(),
        py::arg("want_mask") = false);
  m.def("bn_backward", &bn_backward, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("residual"),
        py::arg("weight"), py::arg("mean"), py::arg("invstd"), py::arg("scale"), py::arg("shift"),
        py::arg("training"), py::arg("act"), py::arg("slope"), py::arg("need_dres"),
        py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(), py::arg("mask") = py::none());
  m.def("conv2d_dgrad_gxf", &conv2d_dgrad_gxf, py::arg("g"), py::arg("wt"), py::arg("addend"),
        py::arg("addend_mask"), py::arg("bnb_mode"), py::arg("bnb_x"), py::arg("bnb_scale"), py::arg("bnb_shift"),
        py::arg("bnb_mean"), py::arg("bnb_bits"), py::arg("gxf"), py::arg("gx_x"), py::arg("gx_bits"),
        py::arg("gx_scale"), py::arg("gx_shift"), py::arg("gx_coef"), py::arg("want_dz"));
  m.def("conv_dgrad_gxf_supported", &conv_dgrad_gxf_supported);
  m.def("bn_backward_coef", &bn_backward_coef, py::arg("part"), py::arg("weight"), py::arg("mean"),
        py::arg("invstd"), py::arg("M"), py::arg("training"), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none());
  m.def("bn_backward_apply_coef", &bn_backward_apply_coef, py::arg("dy"), py::arg("x"), py::arg("coef"),
        py::arg("scale"), py::arg("shift"), py::arg("act"), py::arg("slope"), py::arg("mask") = py::none());
  m.def("gn_forward", &gn_forward);
  m.def("ln_forward", &ln_forward);
  m.def("ln_backward", &ln_backward, py::arg("dy"), py::arg("x"), py::arg("weight"), py::arg("mean"),
        py::arg("rstd"), py::arg("dadd") = py::none(), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none());
  m.def("conv2d_fwd", &conv2d_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"), py::arg("pad"),
        py::arg("relu"), py::arg("want_stats"), py::arg("addend") = py::none(), py::arg("addend_mask") = py::none(),
        py::arg("bnb_mode") = 0, py::arg("bnb_x") = py::none(), py::arg("bnb_scale") = py::none(),
        py::arg("bnb_shift") = py::none(), py::arg("bnb_mean") = py::none(), py::arg("bnb_bits") = py::none(),
        py::arg("big") = -1);
  m.def("bn_apply_coeff", &bn_apply_coeff, py::arg("x"), py::arg("coeff"), py::arg("residual") = py::none(),
        py::arg("act") = 1, py::arg("slope") = 0.01, py::arg("want_mask") = false);
  m.def("conv_fwd_xf_supported", &tbamd::conv_fwd_xf_supported);
  m.def("conv2d_fwd_xf", &conv2d_fwd_xf, py::arg("x"), py::arg("w"), py::arg("scale"), py::arg("shift"),
        py::arg("stride"), py::arg("pad"), py::arg("want_stats") = true);
  m.def("conv2d_wgrad_tinyin", &conv2d_wgrad_tinyin, py::arg("T"), py::arg("G"));
  m.def("conv2d_wgrad_xf", &conv2d_wgrad_xf, py::arg("dy"), py::arg("x"), py::arg("scale"), py::arg("shift"),
        py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("out") = py::none());
  m.def("conv_flip_weight", &conv_flip_weight);
  m.def("conv_set_stages", &tbamd::conv_set_stages);
  m.def("conv_set_big", &tbamd::conv_set_big);
  m.def("conv_get_big", &tbamd::conv_get_big);
  m.def("conv_big_encode", &tbamd::conv_big_encode);
  m.def("conv_big_choice", &tbamd::conv_big_choice);
  m.def("conv_set_persistent_1x1", &tbamd::conv_set_persistent_1x1);
  m.def("conv_set_occupancy", &tbamd::conv_set_occupancy);
  m.def("conv_wgrad_set_occupancy", &tbamd::conv_wgrad_set_occupancy);
  m.def("bn_stats", &bn_stats);
  m.def("bn_backward_from_partials", &bn_backward_from_partials, py::arg("dy"), py::arg("x"), py::arg("part"),
        py::arg("weight"), py::arg("mean"), py::arg("invstd"), py::arg("scale"), py::arg("shift"),
        py::arg("training"), py::arg("act"), py::arg("slope"), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none(), py::arg("mask") = py::none(), py::arg("want_dres") = false,
        py::arg("ds_x") = py::none(), py::arg("ds_mean") = py::none());
  m.def("bn_act_maxpool", &bn_act_maxpool);
  m.def("maxpool_backward", &maxpool_backward);
  m.def("bn_backward_pool", &bn_backward_pool, py::arg("dy"), py::arg("idx"), py::arg("x"), py::arg("N"),
        py::arg("H"), py::arg("W"), py::arg("k"), py::arg("s"), py::arg("pad"), py::arg("weight"), py::arg("mean"),
        py::arg("invstd"), py::arg("scale"), py::arg("shift"), py::arg("training"), py::arg("act"),
        py::arg("slope"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none());
  m.def("bn_backward_pool_ok", &tbamd::bn_backward_pool_ok);
  m.def("conv_flip_weights_mt", &conv_flip_weights_mt, py::arg("chunks"), py::arg("nchunks"), py::arg("table"));
  m.def("gemm_nn_gelu_bwd", &gemm_nn_gelu_bwd, py::arg("dy"), py::arg("w"), py::arg("z"),
        py::arg("db_out") = py::none(), py::arg("wt") = py::none());
  m.def("stop_event_arm", &tbamd::stop_event_arm);
  m.def("stop_event_disarm", &tbamd::stop_event_disarm);
  m.def("stream_wait_stop_event", [](int64_t stream, int64_t id) {
    tbamd::stream_wait_stop_event(reinterpret_cast<hipStream_t>(stream), id);
  });
  // a non-blocking stream at an explicit HIP priority (torch's pool only hands out priorities
  // <= 0; the backward side stream is created at the LOWEST priority so the caller's stream --
  // the input-gradient chain -- dispatches ahead of it without the caller changing streams).
  // Returns (stream handle, least priority, greatest priority); the stream lives for the process.
  m.def("stream_create_priority", [](int device, int priority) {
    int least = 0, greatest = 0, prev = 0;
    TORCH_CHECK(hipGetDevice(&prev) == hipSuccess && hipSetDevice(device) == hipSuccess, "hipSetDevice failed");
    TORCH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess, "stream priority range");
    hipStream_t s = nullptr;
    const hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
    (void)hipSetDevice(prev);
    TORCH_CHECK(e == hipSuccess, "hipStreamCreateWithPriority: ", hipGetErrorString(e));
    return py::make_tuple(reinterpret_cast<int64_t>(s), least, greatest);
  });
  m.def("augment_u8", &augment_u8, py::arg("images"), py::arg("src"), py::arg("Ho"), py::arg("Wo"),
        py::arg("params"), py::arg("mean"), py::arg("inv_std"), py::arg("out_dtype"), py::arg("crop_only") = false);
  m.def("conv_narrow_transpose_fwd", &conv_narrow_transpose_fwd, py::arg("x"), py::arg("w"), py::arg("bias"),
        py::arg("stride"), py::arg("pad"));
  m.def("conv_narrow_fwd_split32", &conv_narrow_fwd_split32, py::arg("x"), py::arg("w"), py::arg("bias"),
        py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv_tinyhalo_wgrad", &conv_tinyhalo_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"),
        py::arg("pad"), py::arg("reflect") = false);
  m.def("conv_tinyhalo_fwd", &conv_tinyhalo_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("pad"),
        py::arg("reflect") = false, py::arg("relu") = false);
  m.def("conv_tiny32_fwd", &conv_tiny32_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"),
        py::arg("pad"), py::arg("reflect") = false, py::arg("relu") = false);
  m.def("conv_tinyc_fwd", &conv_tinyc_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"),
        py::arg("pad"), py::arg("reflect") = false, py::arg("relu") = false);
  m.def("conv_narrow_wgrad", &conv_narrow_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"),
        py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv_narrow_fwd", &conv_narrow_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("pad"),
        py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv_any_set_f32_split", &tbamd::conv_any_set_f32_split, py::arg("on"),
        "fp32 generic convs: split-bf16 MFMA (true, default) or exact-f32 MFMA (false)");
  m.def("conv_any_f32_split", &tbamd::conv_any_f32_split);
  m.def("conv_any_fwd", &conv_any_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"),
        py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv_any_wgrad", &conv_any_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv_any_dgrad", &conv_any_dgrad, py::arg("dy"), py::arg("w"), py::arg("H"), py::arg("W"),
        py::arg("stride"), py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false, py::arg("wt") = py::none());
  m.def("conv2d_fwd_virtual", &conv2d_fwd_virtual, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"),
        py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv2d_wgrad_virtual", &conv2d_wgrad_virtual, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("conv2d_dgrad_virtual", &conv2d_dgrad_virtual, py::arg("dy"), py::arg("wt"), py::arg("H"), py::arg("W"),
        py::arg("stride"), py::arg("pad"), py::arg("up") = 1, py::arg("reflect") = false);
  m.def("global_avgpool", &global_avgpool);
  m.def("global_avgpool_backward", &global_avgpool_backward);
  m.def("gemm", &gemm, py::arg("x"), py::arg("w"), py::arg("tw") = false, py::arg("bias") = py::none(),
        py::arg("residual") = py::none(), py::arg("epi") = 0, py::arg("want_z") = false, py::arg("tile") = -1,
        py::arg("out") = py::none(), py::arg("tx") = false, py::arg("splits") = 1);
  m.def("gemm_pick_splits", &tbamd::gemm_pick_splits);
  m.def("gemm8_set_stagger", &tbamd::gemm8_set_stagger);
  m.def("gemm_pick_tile", &tbamd::gemm_pick_tile);
  m.def("gemm_num_tiles", &tbamd::gemm_num_tiles);
  m.def("conv2d_wgrad", &conv2d_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("out") = py::none());
  m.def("bn_forward_from_stats", &bn_forward_from_stats, py::arg("x"), py::arg("stats"), py::arg("weight"),
        py::arg("bias"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("residual"), py::arg("act"), py::arg("slope"), py::arg("num_batches_tracked") = py::none(),
        py::arg("want_mask") = false, py::arg("res_scale") = py::none(), py::arg("res_shift") = py::none());
  m.def("gn_backward", &gn_backward, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("residual"),
        py::arg("weight"), py::arg("coeff"), py::arg("N"), py::arg("G"), py::arg("act"), py::arg("slope"),
        py::arg("need_dres"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none());
  m.def("ce_forward", &ce_forward);
  m.def("ce_backward", &ce_backward);
  m.def("adamw_mt", &adamw_mt, py::arg("chunks"), py::arg("nchunks"), py::arg("table"), py::arg("pdt"),
        py::arg("gdt"), py::arg("master"), py::arg("ema"), py::arg("amsgrad"), py::arg("lr"), py::arg("beta1"),
        py::arg("beta2"), py::arg("eps"), py::arg("wd"), py::arg("bc1"), py::arg("bc2_sqrt"), py::arg("ema_decay"),
        py::arg("clip_coef"), py::arg("inv_scale"), py::arg("found_inf"), py::arg("hyper") = py::none());
  m.def("sgd_mt", &sgd_mt, py::arg("chunks"), py::arg("nchunks"), py::arg("table"), py::arg("pdt"), py::arg("gdt"),
        py::arg("master"), py::arg("momentum"), py::arg("dampening"), py::arg("nesterov"), py::arg("wd"),
        py::arg("lr"), py::arg("first_step"), py::arg("clip_coef"), py::arg("inv_scale"), py::arg("found_inf"),
        py::arg("hyper") = py::none());
  m.def("grad_norm_mt", &grad_norm_mt);
  m.def("grad_norm_multi", &grad_norm_multi);
  m.def("conv2d_stem_pad", &conv2d_stem_pad);
  m.def("conv2d_dgrad_s2", &conv2d_dgrad_s2, py::arg("dy"), py::arg("wt"), py::arg("R"), py::arg("S"), py::arg("pad"),
        py::arg("H"), py::arg("W"), py::arg("bnb_mode") = 0, py::arg("bnb_x") = py::none(),
        py::arg("bnb_scale") = py::none(), py::arg("bnb_shift") = py::none(), py::arg("bnb_mean") = py::none(),
        py::arg("bnb_bits") = py::none(), py::arg("stride") = 2);
  m.def("conv_dgrad_s2_supported", &tbamd::conv_dgrad_s2_supported);
  m.def("conv2d_stem_fwd", &conv2d_stem_fwd);
  m.def("conv2d_stem_wgrad", &conv2d_stem_wgrad);
  m.def("scale_mt", &scale_mt);
  m.def("u8_crop_flip_normalize", &u8_crop_flip_normalize);
  m.def("attn_forward", &attn_forward);
  m.def("attn_backward", &attn_backward);
  m.def("attn_set_head_mask", [](int64_t m) { return (int64_t)tbamd::attn_set_head_mask((int)m); });
  m.def("gram_forward", &gram_forward);
  m.def("gram_sym", &gram_sym);
  m.def("im2col", &im2col);
  m.def("col2im", &col2im, py::arg("col"), py::arg("N"), py::arg("C"), py::arg("H"), py::arg("W"), py::arg("R"),
        py::arg("S"), py::arg("P"), py::arg("Q"), py::arg("stride"), py::arg("pad"), py::arg("bias") = py::none());
  m.def("colsum", &colsum, py::arg("dy"), py::arg("out") = py::none());
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd_colsum", &gelu_bwd_colsum, py::arg("dy"), py::arg("z"), py::arg("out") = py::none());
  m.def("tv_forward", &tv_forward);
  m.def("tv_backward", &tv_backward);
  m.def("conv2d_wgrad_split32", &conv2d_wgrad_split32);
  m.def("conv_narrow_wgrad_split32", &conv_narrow_wgrad_split32);
  m.def("split_bf16", &split_bf16);
  m.def("conv2d_fwd_splitk", &conv2d_fwd_splitk, py::arg("x"), py::arg("w"), py::arg("bias") = py::none(),
        py::arg("stride") = 1, py::arg("pad") = 0, py::arg("relu") = false);
  m.def("conv_fwd_splitk_ksplit", [](int64_t N, int64_t C, int64_t K, int64_t R, int64_t S, int64_t P, int64_t Q) {
    return tbamd::conv_fwd_splitk_bf16_ksplit((int)N, (int)C, (int)K, (int)R, (int)S, (int)P, (int)Q);
  });
  m.def("conv2d_fwd_split32", &conv2d_fwd_split32, py::arg("xh"), py::arg("xl"), py::arg("wh"), py::arg("wl"),
        py::arg("bias") = py::none(), py::arg("stride") = 1, py::arg("pad") = 0, py::arg("relu") = false);
  m.def("act_fwd", &act_fwd, py::arg("x"), py::arg("act"), py::arg("slope") = 0.01);
  m.def("act_bwd", &act_bwd, py::arg("x"), py::arg("dy"), py::arg("act"), py::arg("slope") = 0.01);
  m.def("hinge_forward", &hinge_forward);
  m.def("hinge_backward", &hinge_backward);
  m.def("bce_logits_forward", &bce_logits_forward);
  m.def("bce_logits_backward", &bce_logits_backward);
  m.def("kld_forward", &kld_forward);
  m.def("kld_backward", &kld_backward);
  m.def("mean_std_forward", &mean_std_forward);
  m.def("mean_std_backward", &mean_std_backward);
  m.def("reflect_pad_forward", &reflect_pad_forward);
  m.def("reflect_pad_backward", &reflect_pad_backward);
  m.def("upsample_nearest_forward", &upsample_nearest_forward);
  m.def("upsample_nearest_backward", &upsample_nearest_backward);
  register_runtime(m);
  // one-shot all-reduce over IPC-mapped peer buffers (csrc/oneshot.hip)
  py::class_<tbamd::OneShotComm>(m, "OneShotComm")
      .def(py::init<int, int, int64_t, int64_t, double>(), py::arg("rank"), py::arg("world"),
           py::arg("capacity_bytes") = (int64_t)2 << 20, py::arg("chunk_bytes") = (int64_t)64 << 10,
           py::arg("timeout_s") = 600.0)
      .def("handles", [](const tbamd::OneShotComm& c) { return py::bytes(c.handles()); })
      .def("open",
           [](tbamd::OneShotComm& c, std::vector<py::bytes> all) {
             std::vector<std::string> v;
             for (auto& b : all) v.emplace_back(std::string(b));
             c.open(v);
           })
      .def("allreduce",
           [](tbamd::OneShotComm& c, const Tensor& in, Tensor& out, double scale) {
             TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(),
                         "oneshot allreduce: contiguous device tensors");
             TORCH_CHECK(in.numel() == out.numel() && in.scalar_type() == out.scalar_type(),
                         "oneshot allreduce: in / out mismatch");
             const at::DeviceGuard guard(in.device());
             c.allreduce(in.data_ptr(), out.data_ptr(), in.numel(), dt_code(in), (float)scale, cur_stream());
           },
           py::arg("input"), py::arg("output"), py::arg("scale") = 1.0)
      .def("error", &tbamd::OneShotComm::error)
      .def_property_readonly("capacity", &tbamd::OneShotComm::capacity);
}
