// PyTorch custom-op registration for the gfx950 kernels: torch.ops.alphago_amd.*
// All ops write into caller-provided buffers (no allocation inside), run on the
// current HIP stream and are therefore safe to capture in HIP graphs.
#include "ops_conv.h"

namespace {

using namespace agk_ops;

// x: (B, HPi, HPi, Cin) bf16; w: (T, Cout, Cin) bf16; y: (B, HPo, HPo, Cout) bf16
void conv_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, const c10::optional<Tensor>& mask,
              const Tensor& y, int64_t K, int64_t S, int64_t Pin, int64_t Po, int64_t mode,
              const c10::optional<Tensor>& mbits, int64_t tile) {
  check_dev("conv_fwd", x, w, bias, mask, y, mbits);
  // production tilings only: 0 = automatic, or a fixed 64 / 128 / 256 / 384-pixel tile (385: 384 with the
  // LDS-DMA issue spread through the MFMAs; 386 / 387: 385 / 384 with the chunk-outer K order)
  TORCH_CHECK(tile == 0 || tile == 36 || tile == 37 || tile == 40 || tile == 64 || tile == 128 || tile == 256 ||
                  tile == 384 || tile == 385 || tile == 386 || tile == 387,
              "conv_fwd tile ", tile, " is not a production tiling (0, 36, 37, 40, 64, 128, 256, 384-387); kernel-lab "
              "variants are in torch.ops.alphago_amd_lab (alphago_amd.ops.lab())");
  conv_fwd_impl(x, w, bias, mask, y, K, S, Pin, Po, mode, mbits, (int)tile);
}

// one draw per board from probs ** beta (probs: (B, NP) f32, has: (B,) bool / uint8, out: (B,) int64)
void sample_moves(const Tensor& probs, const Tensor& has, const Tensor& out, double beta, int64_t seed) {
  check_dev("sample_moves", probs, has, out);
  CHECK_F32(probs); CHECK_CONTIG(probs); CHECK_CONTIG(has); CHECK_CONTIG(out);
  TORCH_CHECK(probs.dim() == 2 && probs.size(1) <= 512, "probs (B, NP <= 512)");
  // has: (B,) any-sensible flags, or the (B, NP) uint8 sensible-move mask (the kernel takes the row's any)
  const bool mask2d = has.dim() == 2;
  TORCH_CHECK((has.scalar_type() == at::kBool || has.scalar_type() == at::kByte) &&
                  (mask2d ? (has.size(0) == probs.size(0) && has.size(1) == probs.size(1)) : has.numel() == probs.size(0)),
              "has: (B,) bool / uint8, or the (B, NP) uint8 mask");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() == probs.size(0), "out: (B,) int64");
  agk::SampleArgs a{};
  a.probs = probs.data_ptr<float>();
  a.has = mask2d ? nullptr : reinterpret_cast<const uint8_t*>(has.data_ptr());
  a.legal = mask2d ? reinterpret_cast<const uint8_t*>(has.data_ptr()) : nullptr;
  a.out = out.data_ptr<int64_t>();
  a.B = (int)probs.size(0); a.NP = (int)probs.size(1);
  a.beta = (float)beta;
  a.seed = (uint64_t)seed;
  agk::launch_sample_moves(a, cur_stream());
  launch_check("sample_moves");
}

// Small batches: the 32-pixel tile with the K loop split over nsplit workgroups per tile (tile 38) into
// ws (>= nsplit * M * Cout fp32), then one finishing pass (bias + ReLU + bitmask, or the bitmask dgrad)
void conv_fwd_splitk(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, const Tensor& y, int64_t K,
                     int64_t S, int64_t Pin, int64_t Po, int64_t mode, const c10::optional<Tensor>& mbits,
                     const Tensor& ws, int64_t nsplit) {
  check_dev("conv_fwd_splitk", x, w, bias, y, mbits, ws);
  conv_fwd_impl(x, w, bias, c10::nullopt, y, K, S, Pin, Po, mode, mbits, 38, nullptr, -1, c10::nullopt, c10::nullopt,
                c10::nullopt, 0, ws, (int)nsplit);
}

// slab: (nsplit, T, Cout, Cin) f32; dbslab: (nsplit, Cout) f32
void conv_wgrad(const Tensor& x, const Tensor& dz, const Tensor& slab, const Tensor& dbslab, int64_t K, int64_t S,
                int64_t Pin, int64_t Po, int64_t cin_real, int64_t variant) {
  check_dev("conv_wgrad", x, dz, slab, dbslab);
  // the per-tap / tap-merged kernel only; the round-4 variants (9 LDS ring, 10-13 first-layer re-cuts) and
  // the older lab variants run from torch.ops.alphago_amd_lab
  TORCH_CHECK(variant == 0 || variant == agk::kWgradSmall, "conv_wgrad variant ", variant,
              " is a kernel-lab variant (alphago_amd.ops.lab())");
  conv_wgrad_impl(x, dz, slab, dbslab, K, S, Pin, Po, cin_real, (int)variant);
}

// bitmask dgrad that also writes an e5m2 copy of dx (x *scale) and folds max |dx| into amax slots
void conv_dgrad_bits_bf8(const Tensor& dz, const Tensor& wd, const Tensor& dx, const Tensor& mbits, const Tensor& dx8,
                         const Tensor& scale, const c10::optional<Tensor>& amax, int64_t K, int64_t S, int64_t tile) {
  check_dev("conv_dgrad_bits_bf8", dz, wd, dx, mbits, dx8, scale, amax);
  TORCH_CHECK(tile == 0 || tile == 64 || tile == 128 || tile == 256 || (tile >= 384 && tile <= 387),
              "conv_dgrad_bits_bf8: production tile codes only");
  conv_fwd_impl(dz, wd, c10::nullopt, c10::nullopt, dx, K, S, 1, 1, agk::MODE_MASKBITS, mbits, (int)tile, nullptr, -1,
                dx8, scale, amax);
}

void conv_wgrad_fp8(const Tensor& x8, const Tensor& dz8, const Tensor& slab, const Tensor& dbslab,
                    const Tensor& xscale, const Tensor& gscale, const Tensor& gmul, int64_t K, int64_t S, int64_t Pin,
                    int64_t Po, const c10::optional<Tensor>& amax) {
  conv_wgrad_fp8_impl(x8, dz8, slab, dbslab, xscale, gscale, gmul, K, S, Pin, Po, amax);
}

int64_t wgrad_fp8_stage_px() { return agk::wgrad_fp8_stage_pixels(); }

bool wgrad_direct_supported_op(int64_t cout, int64_t cin, int64_t cin_real, int64_t K) {
  return agk::wgrad_direct_supported((int)cout, (int)cin, (int)cin_real, (int)K);
}

// split-free wgrad (kWgradDirect): grad_w (Cout_real, Cin_real, K, K) f32 = beta * grad_w + scale * dW,
// grad_b likewise; no slab, no reduce
void conv_wgrad_direct(const Tensor& x, const Tensor& dz, const Tensor& grad_w, const c10::optional<Tensor>& grad_b,
                       int64_t K, int64_t S, int64_t Pin, int64_t Po, double scale, double beta, int64_t ksub) {
  check_dev("conv_wgrad_direct", x, dz, grad_w, grad_b);
  CHECK_BF16(x); CHECK_BF16(dz); CHECK_F32(grad_w); CHECK_CONTIG(x); CHECK_CONTIG(dz); CHECK_CONTIG(grad_w);
  TORCH_CHECK(x.dim() == 4 && dz.dim() == 4 && dz.size(0) == x.size(0), "x, dz: (B, HP, HP, C) with the same B");
  TORCH_CHECK(x.size(2) == x.size(1) && dz.size(2) == dz.size(1), "x, dz: square padded boards");
  TORCH_CHECK(x.numel() < (1ll << 31) && dz.numel() < (1ll << 31), "tensor too large for int32 offsets");
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3), HPo = dz.size(1), Cout = dz.size(3);
  TORCH_CHECK(HPi == S + 2 * Pin && HPo == S + 2 * Po && Po >= 1 && Pin >= K / 2, "geometry mismatch");
  TORCH_CHECK(grad_w.dim() == 4 && grad_w.size(2) == K && grad_w.size(3) == K && grad_w.size(0) <= Cout &&
                  grad_w.size(1) <= Cin, "grad_w: OIHW (Cout_real <= Cout, Cin_real <= Cin, K, K)");
  TORCH_CHECK(agk::wgrad_direct_supported((int)Cout, (int)Cin, (int)grad_w.size(1), (int)K),
              "conv_wgrad_direct: Cout % 32 == 0 and Cin a multiple of 48 / 32 (or 64 with <= 48 real planes)");
  TORCH_CHECK(ksub == 1 || ksub == 2 || ksub == 4 || ksub == 8, "conv_wgrad_direct: ksub 1 / 2 / 4 / 8");
  if (grad_b.has_value()) {
    CHECK_F32(*grad_b);
    TORCH_CHECK(grad_b->numel() == grad_w.size(0), "grad_b: (Cout_real,)");
  }
  agk::ConvWgradArgs a{};
  a.x_elems = x.numel();
  a.dz_elems = dz.numel();
  a.x = bfp(x); a.dz = bfp(dz);
  a.M = (int)(B * S * S); a.S = (int)S; a.Cin = (int)Cin; a.Cout = (int)Cout; a.K = (int)K; a.T = (int)(K * K);
  a.HPi = (int)HPi; a.offi = (int)(Pin - K / 2); a.HPo = (int)HPo; a.Po = (int)Po;
  a.cin_real = (int)grad_w.size(1);
  a.cout_real = (int)grad_w.size(0);
  a.nsplit = 1;
  a.ksteps_per_split = (a.M + 31) / 32;  // >= the stage count at any ksub: the whole pixel range
  a.grad_w = grad_w.data_ptr<float>();
  a.grad_b = grad_b.has_value() ? grad_b->data_ptr<float>() : nullptr;
  a.scale = (float)scale; a.beta = (float)beta;
  agk::launch_conv_wgrad_direct(a, (int)ksub, cur_stream());
  launch_check("conv_wgrad_direct");
}

static agk::WgradReduceArgs reduce_args(const Tensor& slab, const Tensor& dbslab, const Tensor& grad_w,
                                        const c10::optional<Tensor>& grad_b, double scale, double beta) {
  check_dev("conv_wgrad_reduce", slab, dbslab, grad_w, grad_b);
  CHECK_F32(slab); CHECK_F32(grad_w); CHECK_CONTIG(grad_w); CHECK_CONTIG(slab); CHECK_CONTIG(dbslab);
  TORCH_CHECK(slab.dim() == 4 && dbslab.dim() == 2 && dbslab.size(0) == slab.size(0) && dbslab.size(1) == slab.size(2),
              "slab (nsplit, T, Cout, Cin), dbslab (nsplit, Cout)");
  const int64_t nsplit = slab.size(0), T = slab.size(1), Cout = slab.size(2), Cin = slab.size(3);
  TORCH_CHECK(grad_w.dim() == 4 && grad_w.size(2) * grad_w.size(3) == T, "grad_w must be OIHW");
  TORCH_CHECK(Cin % 4 == 0, "slab channels must be a multiple of 4 (16-byte split reads)");
  if (grad_b.has_value()) {
    CHECK_F32(*grad_b);
    TORCH_CHECK(grad_b->numel() == grad_w.size(0), "grad_b: (Cout_real,)");
  }
  agk::WgradReduceArgs a{};
  a.slab = slab.data_ptr<float>();
  a.dbias_slab = dbslab.data_ptr<float>();
  a.grad_w = grad_w.data_ptr<float>();
  a.grad_b = grad_b.has_value() ? grad_b->data_ptr<float>() : nullptr;
  a.T = (int)T; a.Cout = (int)Cout; a.Cin = (int)Cin;
  a.Cout_real = (int)grad_w.size(0); a.Cin_real = (int)grad_w.size(1);
  TORCH_CHECK(a.Cout_real <= Cout && a.Cin_real <= Cin, "grad_w larger than padded slab");
  a.nsplit = (int)nsplit;
  a.scale = (float)scale; a.beta = (float)beta;
  return a;
}

void conv_wgrad_reduce(const Tensor& slab, const Tensor& dbslab, const Tensor& grad_w, const c10::optional<Tensor>& grad_b,
                       double scale, double beta) {
  agk::launch_wgrad_reduce(reduce_args(slab, dbslab, grad_w, grad_b, scale, beta), cur_stream());
  launch_check("conv_wgrad_reduce");
}

// every listed layer's split-K reduce in one launch (same summation order as conv_wgrad_reduce)
void conv_wgrad_reduce_multi(const std::vector<Tensor>& slabs, const std::vector<Tensor>& dbslabs,
                             const std::vector<Tensor>& grad_ws, const std::vector<Tensor>& grad_bs, double scale,
                             double beta) {
  TORCH_CHECK(slabs.size() == dbslabs.size() && slabs.size() == grad_ws.size() && slabs.size() == grad_bs.size(),
              "conv_wgrad_reduce_multi: one slab, dbias slab, grad_w and grad_b per layer");
  TORCH_CHECK((int)slabs.size() <= agk::kMaxReduceJobs, "conv_wgrad_reduce_multi: at most ", agk::kMaxReduceJobs,
              " layers");
  std::vector<agk::WgradReduceArgs> jobs;
  for (size_t i = 0; i < slabs.size(); ++i)
    jobs.push_back(reduce_args(slabs[i], dbslabs[i], grad_ws[i], grad_bs[i], scale, beta));
  agk::launch_wgrad_reduce_multi(jobs, cur_stream());
  launch_check("conv_wgrad_reduce_multi");
}

void policy_head(const Tensor& y, const Tensor& w, const Tensor& b, const c10::optional<Tensor>& target,
                 const c10::optional<Tensor>& legal, const c10::optional<Tensor>& weight, const c10::optional<Tensor>& dz, const c10::optional<Tensor>& loss,
                 const c10::optional<Tensor>& correct, const c10::optional<Tensor>& dhead,
                 const c10::optional<Tensor>& probs, int64_t S, double grad_scale, double temperature, int64_t loss_kind) {
  check_dev("policy_head", y, w, b, target, legal, weight, dz, loss, correct, dhead, probs);
  CHECK_BF16(y); CHECK_CONTIG(y); CHECK_F32(w); CHECK_F32(b);
  const int64_t B = y.size(0), C = y.size(3);
  TORCH_CHECK(y.size(1) == S + 2, "head input must have pad 1");
  TORCH_CHECK(C % 8 == 0 && C <= 256, "head channels must be a multiple of 8 and <= 256");
  TORCH_CHECK(S * S <= 361, "board too large (the head holds at most 19 x 19)");
  agk::PolicyHeadArgs a{};
  a.y = bfp(y);
  a.w = w.data_ptr<float>();
  a.b = b.data_ptr<float>();
  a.B = (int)B; a.S = (int)S; a.C = (int)C; a.C_real = (int)w.numel();
  a.grad_scale = (float)grad_scale;
  a.inv_temp = (float)(1.0 / temperature);
  TORCH_CHECK(loss_kind == 0 || loss_kind == 1, "loss_kind must be 0 (CE) or 1 (reference BCE)");
  a.loss_kind = (int)loss_kind;
  const bool train = target.has_value();
  if (train) {
    TORCH_CHECK(dz && loss && correct && dhead, "training head needs dz, loss, correct, dhead");
    TORCH_CHECK(target->scalar_type() == at::kInt, "target must be int32");
    TORCH_CHECK(dz->sizes() == y.sizes(), "dz must match y");
    TORCH_CHECK(dhead->numel() >= B * (a.C_real + 1), "dhead too small");
    a.target = target->data_ptr<int>();
    a.dz = bfp_mut(*dz);
    a.loss = loss->data_ptr<float>();
    a.correct = correct->data_ptr<float>();
    a.dhead = dhead->data_ptr<float>();
  }
  if (weight.has_value()) {
    CHECK_F32(*weight);
    TORCH_CHECK(weight->numel() == B, "weight must be (B,)");
    a.weight = weight->data_ptr<float>();
  }
  if (legal.has_value()) {
    TORCH_CHECK(legal->scalar_type() == at::kByte && legal->numel() == B * S * S, "legal must be uint8 (B, S*S)");
    a.legal = legal->data_ptr<uint8_t>();
  }
  if (probs.has_value()) {
    CHECK_F32(*probs);
    TORCH_CHECK(probs->numel() == B * S * S, "probs must be (B, S*S)");
    a.probs = probs->data_ptr<float>();
  }
  if (B == 0) return;
  agk::launch_policy_head(a, train, cur_stream());
  launch_check("policy_head");
}

// z: (B, S*S) f32 <- y (B, S+2, S+2, C) bf16 . w + b
void head_logits(const Tensor& y, const Tensor& w, const Tensor& b, const Tensor& z, int64_t S) {
  check_dev("head_logits", y, w, b, z);
  CHECK_BF16(y); CHECK_CONTIG(y); CHECK_F32(w); CHECK_F32(b); CHECK_F32(z); CHECK_CONTIG(z);
  const int64_t B = y.size(0), C = y.size(3);
  TORCH_CHECK(y.size(1) == S + 2 && C % 8 == 0 && C <= 256 && w.numel() <= C && S * S <= 368, "head geometry");
  TORCH_CHECK(z.numel() == B * S * S, "z must be (B, S*S)");
  agk::PolicyHeadArgs a{};
  a.y = bfp(y); a.w = w.data_ptr<float>(); a.b = b.data_ptr<float>(); a.probs = z.data_ptr<float>();
  a.B = (int)B; a.S = (int)S; a.C = (int)C; a.C_real = (int)w.numel();
  if (B == 0) return;
  agk::launch_head_logits(a, cur_stream());
  launch_check("head_logits");
}

// dz (B, S+2, S+2, C) bf16 <- ReLU'(y) * dlogits x w;  dhead (B, C_real+1) partials
// grad[n] = sum_b dhead[b][n]; sums = {sum_b loss[b], sum_b correct[b]} (fixed order, one launch)
void head_grad_sums(const Tensor& dhead, const Tensor& loss, const Tensor& correct, const Tensor& grad,
                    const Tensor& sums) {
  check_dev("head_grad_sums", dhead, loss, correct, grad, sums);
  CHECK_F32(dhead); CHECK_F32(loss); CHECK_F32(correct); CHECK_F32(grad); CHECK_F32(sums);
  CHECK_CONTIG(dhead); CHECK_CONTIG(loss); CHECK_CONTIG(correct); CHECK_CONTIG(grad); CHECK_CONTIG(sums);
  TORCH_CHECK(dhead.dim() == 2 && loss.numel() == dhead.size(0) && correct.numel() == dhead.size(0) &&
                  grad.numel() == dhead.size(1) && sums.numel() >= 2,
              "head_grad_sums: dhead (B, N), loss/correct (B), grad (N), sums (2)");
  if (dhead.size(0) == 0) return;
  agk::launch_head_grad_sums(dhead.data_ptr<float>(), (int)dhead.size(0), (int)dhead.size(1), loss.data_ptr<float>(),
                             correct.data_ptr<float>(), grad.data_ptr<float>(), sums.data_ptr<float>(), cur_stream());
  launch_check("head_grad_sums");
}

void head_backward(const Tensor& y, const Tensor& w, const Tensor& dlogits, const Tensor& dz, const Tensor& dhead,
                   int64_t S, const c10::optional<Tensor>& dz8, const c10::optional<Tensor>& dz8_scale,
                   const c10::optional<Tensor>& dz8_amax) {
  check_dev("head_backward", y, w, dlogits, dz, dhead, dz8, dz8_scale, dz8_amax);
  CHECK_BF16(y); CHECK_CONTIG(y); CHECK_F32(w); CHECK_F32(dlogits); CHECK_CONTIG(dlogits);
  CHECK_BF16(dz); CHECK_CONTIG(dz); CHECK_F32(dhead);
  const int64_t B = y.size(0), C = y.size(3);
  TORCH_CHECK(y.size(1) == S + 2 && C % 8 == 0 && C <= 256 && w.numel() <= C && S * S <= 368, "head geometry");
  TORCH_CHECK(dz.sizes() == y.sizes() && dlogits.numel() == B * S * S && dhead.numel() >= B * (w.numel() + 1), "shapes");
  agk::PolicyHeadArgs a{};
  a.y = bfp(y); a.w = w.data_ptr<float>(); a.dz = bfp_mut(dz); a.dhead = dhead.data_ptr<float>();
  a.B = (int)B; a.S = (int)S; a.C = (int)C; a.C_real = (int)w.numel();
  if (dz8.has_value()) {  // e5m2 dY instead of the bf16 dz (dz is not written)
    TORCH_CHECK(dz8_scale.has_value() && dz8_amax.has_value(), "head_backward: dz8 needs dz8_scale and dz8_amax");
    TORCH_CHECK(dz8->scalar_type() == at::kByte && dz8->sizes() == y.sizes() && dz8->is_contiguous(),
                "head_backward: dz8 uint8 of y's shape");
    CHECK_F32(*dz8_scale);
    TORCH_CHECK(dz8_amax->scalar_type() == at::kInt && dz8_amax->numel() >= agk::kFp8AmaxSlots &&
                    dz8_amax->is_contiguous(), "head_backward: dz8_amax int32[64]");
    a.dz8 = dz8->data_ptr<uint8_t>();
    a.dz8_scale = dz8_scale->data_ptr<float>();
    a.dz8_amax = (unsigned*)dz8_amax->data_ptr<int>();
  }
  if (B == 0) return;
  agk::launch_head_backward(a, dlogits.data_ptr<float>(), cur_stream());
  launch_check("head_backward");
}

void value_out(const Tensor& h, const Tensor& w2, const Tensor& b2, const c10::optional<Tensor>& target,
               const c10::optional<Tensor>& weight, const Tensor& v, const c10::optional<Tensor>& loss,
               const c10::optional<Tensor>& correct, const c10::optional<Tensor>& dh, const c10::optional<Tensor>& dout,
               double grad_scale) {
  check_dev("value_out", h, w2, b2, target, weight, v, loss, correct, dh, dout);
  CHECK_F32(h); CHECK_CONTIG(h); CHECK_F32(w2); CHECK_F32(b2); CHECK_F32(v);
  TORCH_CHECK(h.dim() == 2, "h must be (B, D)");
  const int64_t B = h.size(0), D = h.size(1);
  TORCH_CHECK(w2.numel() == D && v.numel() == B, "shapes");
  agk::ValueOutArgs a{};
  a.h = h.data_ptr<float>(); a.w2 = w2.data_ptr<float>(); a.b2 = b2.data_ptr<float>(); a.v = v.data_ptr<float>();
  a.B = (int)B; a.D = (int)D; a.grad_scale = (float)grad_scale;
  if (target.has_value()) {
    TORCH_CHECK(loss && correct && dh && dout, "training needs loss, correct, dh, dout");
    CHECK_F32(*target);
    TORCH_CHECK(target->numel() == B && dh->numel() == B * D && dout->numel() >= B * (D + 1), "shapes");
    a.target = target->data_ptr<float>();
    a.loss = loss->data_ptr<float>(); a.correct = correct->data_ptr<float>();
    a.dh = dh->data_ptr<float>(); a.dout = dout->data_ptr<float>();
  }
  if (weight.has_value()) {
    CHECK_F32(*weight);
    TORCH_CHECK(weight->numel() == B, "weight must be (B,)");
    a.weight = weight->data_ptr<float>();
  }
  if (B == 0) return;
  agk::launch_value_out(a, cur_stream());
  launch_check("value_out");
}

void pack_input(const Tensor& planes, const c10::optional<Tensor>& sym, const c10::optional<Tensor>& target,
                const c10::optional<Tensor>& target_out, const Tensor& out, int64_t P,
                const c10::optional<Tensor>& rows, const c10::optional<Tensor>& out8) {
  check_dev("pack_input", planes, sym, target, target_out, out, rows, out8);
  TORCH_CHECK(planes.scalar_type() == at::kByte && planes.is_contiguous() && planes.dim() == 4, "planes: uint8 (B,C,S,S)");
  CHECK_BF16(out); CHECK_CONTIG(out);
  const int64_t C = planes.size(1), S = planes.size(2);
  const int64_t B = rows.has_value() ? rows->numel() : planes.size(0);
  if (rows.has_value())
    TORCH_CHECK(rows->scalar_type() == at::kLong && rows->is_contiguous(), "rows: contiguous int64 (B,)");
  TORCH_CHECK(out.size(0) == B && out.size(1) == S + 2 * P && out.size(3) >= C && out.size(3) % 8 == 0, "bad out");
  if (sym.has_value()) TORCH_CHECK(sym->scalar_type() == at::kInt && sym->numel() == B, "sym: int32 (B,)");
  if (target.has_value()) TORCH_CHECK(target->scalar_type() == at::kInt && target->numel() == B, "target: int32 (B,)");
  agk::PackInputArgs a{};
  a.planes = planes.data_ptr<uint8_t>();
  a.rows = rows.has_value() ? rows->data_ptr<int64_t>() : nullptr;
  if (out8.has_value())
    TORCH_CHECK(out8->scalar_type() == at::kByte && out8->sizes() == out.sizes() && out8->is_contiguous(),
                "pack_input: out8 uint8 of out's shape");
  a.out8 = out8.has_value() ? out8->data_ptr<uint8_t>() : nullptr;
  a.npool = planes.size(0);
  a.sym = sym.has_value() ? sym->data_ptr<int>() : nullptr;
  a.target = target.has_value() ? target->data_ptr<int>() : nullptr;
  a.target_out = target_out.has_value() ? target_out->data_ptr<int>() : nullptr;
  TORCH_CHECK(!a.target_out || a.target, "target_out needs target");
  a.out = bfp_mut(out);
  a.B = (int)B; a.S = (int)S; a.Creal = (int)C; a.Cp = (int)out.size(3); a.P = (int)P;
  if (B == 0) return;
  agk::launch_pack_input(a, cur_stream());
  launch_check("pack_input");
}

// ws: list of OIHW fp32; wf: list of (T, Coutp, Cinp) bf16; wd: list (possibly empty entries skipped)
void pack_weights(at::TensorList ws, at::TensorList wf, at::TensorList wd) {
  check_dev("pack_weights", ws, wf, wd);
  TORCH_CHECK(ws.size() == wf.size() && (wd.size() == 0 || wd.size() == ws.size()), "list sizes");
  size_t i = 0;
  while (i < ws.size()) {
    agk::PackWeightsArgs a{};
    a.nlayers = 0;
    for (; i < ws.size() && a.nlayers < agk::kMaxPackLayers; ++i) {
      const Tensor& w = ws[i];
      CHECK_F32(w); CHECK_CONTIG(w); CHECK_BF16(wf[i]);
      agk::PackLayer& L = a.layers[a.nlayers++];
      L.w = w.data_ptr<float>();
      L.Cout_real = (int)w.size(0); L.Cin_real = (int)w.size(1); L.K = (int)w.size(2);
      L.wf = bfp_mut(wf[i]);
      L.Cout_p = (int)wf[i].size(1); L.Cin_p = (int)wf[i].size(2);
      // K*K taps, or K*K + 1 with a trailing all-zero tap (Cin % 64 == 32; never written here), or the
      // packed-tap first-layer layout (conv_fwd_pk): ceil(K*K*cpt / 8) steps of 64, cpt = ceil(Cin / 8)
      const int T = L.K * L.K, cpt = (L.Cin_real + 7) / 8;
      L.pk_cpt = (wf[i].size(0) != T && wf[i].size(0) != T + 1 && L.Cin_p == 64 && L.Cin_real <= 64 &&
                  wf[i].size(0) == (T * cpt + 7) / 8) ? cpt : 0;
      TORCH_CHECK((wf[i].size(0) == T || wf[i].size(0) == T + 1 || L.pk_cpt > 0) && L.Cout_p >= L.Cout_real &&
                  L.Cin_p >= L.Cin_real, "bad wf");
      L.wd = nullptr;
      TORCH_CHECK(L.pk_cpt == 0 || !(wd.size() && wd[i].numel() > 0), "packed-tap layout: no dgrad copy");
      if (wd.size() && wd[i].numel() > 0) {
        CHECK_BF16(wd[i]);
        TORCH_CHECK(wd[i].size(1) == L.Cin_p && wd[i].size(2) == L.Cout_p, "bad wd");
        L.wd = bfp_mut(wd[i]);
      }
    }
    agk::launch_pack_weights(a, cur_stream());
    launch_check("pack_weights");
  }
}

// board: (B, S*S) int8; ages: (B, S*S) uint8; meta: (B, 2) int32; fids: feature ids
// (engine numbering) with their plane counts; every output optional.
void featurize(const Tensor& board, const Tensor& ages, const Tensor& meta, const c10::optional<Tensor>& ladder,
               at::IntArrayRef fids, at::IntArrayRef fplanes, const c10::optional<Tensor>& planes,
               const c10::optional<Tensor>& nhwc, const c10::optional<Tensor>& sensible,
               const c10::optional<Tensor>& legal, const c10::optional<Tensor>& overflow, int64_t S, int64_t P) {
  check_dev("featurize", board, ages, meta, ladder, planes, nhwc, sensible, legal, overflow);
  TORCH_CHECK(board.scalar_type() == at::kChar && board.is_contiguous() && board.dim() == 2, "board: int8 (B, S*S)");
  TORCH_CHECK(ages.scalar_type() == at::kByte && ages.is_contiguous() && ages.sizes() == board.sizes(), "ages: uint8 (B, S*S)");
  TORCH_CHECK(meta.scalar_type() == at::kInt && meta.is_contiguous() && meta.dim() == 2 && meta.size(1) == 2, "meta: int32 (B, 2)");
  TORCH_CHECK(S >= 2 && S <= 19 && board.size(1) == S * S, "board size");
  TORCH_CHECK(fids.size() == fplanes.size() && (int)fids.size() <= agk::kFzMaxFeatures, "feature list");
  CHECK_DEV(board); CHECK_DEV(ages); CHECK_DEV(meta);
  const int64_t B = board.size(0), NP = S * S;
  TORCH_CHECK(meta.size(0) == B, "meta rows");
  agk::FeaturizeArgs a{};
  a.board = board.data_ptr<int8_t>();
  a.ages = ages.data_ptr<uint8_t>();
  a.meta = meta.data_ptr<int>();
  a.B = (int)B; a.S = (int)S; a.P = (int)P; a.nf = (int)fids.size();
  int np = 0;
  for (size_t i = 0; i < fids.size(); ++i) {
    TORCH_CHECK(fids[i] >= 0 && fids[i] < 13 && fplanes[i] >= 1 && fplanes[i] <= 8, "bad feature");
    a.fids[i] = (int)fids[i];
    a.fplanes[i] = (int)fplanes[i];
    for (int k = 0; k < fplanes[i]; ++k, ++np) {
      TORCH_CHECK(np < agk::kFzMaxChannels, "too many planes");
      a.chan_feat[np] = (uint8_t)fids[i];
      a.chan_plane[np] = (uint8_t)k;
    }
    a.need_eye |= (fids[i] == 9);
  }
  a.nplanes = np;
  if (sensible.has_value()) a.need_eye = 1;
  if (ladder.has_value()) {
    TORCH_CHECK(ladder->scalar_type() == at::kByte && ladder->is_contiguous() && ladder->sizes() == board.sizes(), "ladder");
    a.ladder = ladder->data_ptr<uint8_t>();
  }
  if (planes.has_value()) {
    TORCH_CHECK(planes->scalar_type() == at::kByte && planes->is_contiguous() && planes->numel() == B * np * NP, "planes");
    a.planes = planes->data_ptr<uint8_t>();
  }
  if (nhwc.has_value()) {
    CHECK_BF16(*nhwc); CHECK_CONTIG(*nhwc);
    TORCH_CHECK(nhwc->dim() == 4 && nhwc->size(0) == B && nhwc->size(1) == S + 2 * P && nhwc->size(2) == S + 2 * P &&
                nhwc->size(3) >= np && nhwc->size(3) % 8 == 0 && nhwc->size(3) <= agk::kFzMaxChannels, "nhwc");
    a.nhwc = bfp_mut(*nhwc);
    a.Cp = (int)nhwc->size(3);
  }
  if (sensible.has_value()) {
    TORCH_CHECK(sensible->scalar_type() == at::kByte && sensible->is_contiguous() && sensible->numel() == B * NP, "sensible");
    a.sensible = sensible->data_ptr<uint8_t>();
  }
  if (legal.has_value()) {
    TORCH_CHECK(legal->scalar_type() == at::kByte && legal->is_contiguous() && legal->numel() == B * NP, "legal");
    a.legal = legal->data_ptr<uint8_t>();
  }
  if (overflow.has_value()) {
    TORCH_CHECK(overflow->scalar_type() == at::kInt && overflow->is_contiguous() && overflow->numel() == B, "overflow");
    a.overflow = overflow->data_ptr<int>();
  }
  if (B == 0) return;
  agk::launch_featurize(a, cur_stream());
  launch_check("featurize");
}

// x: (B, HPi, HPi, Cin) uint8 (e4m3); w: (nch, Cout, 64) uint8; scales int32[2]; out_scale f32[1]
void conv_fwd_fp8(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& scales, const Tensor& out_scale,
                  const c10::optional<Tensor>& amax, const c10::optional<Tensor>& y_bf16,
                  const c10::optional<Tensor>& y_fp8, int64_t K, int64_t S, int64_t Pin, int64_t Po,
                  const c10::optional<Tensor>& mbits, const c10::optional<Tensor>& sr_seed) {
  check_dev("conv_fwd_fp8", x, w, bias, scales, out_scale, amax, y_bf16, y_fp8, mbits, sr_seed);
  conv_fwd_fp8_impl(x, w, bias, scales, out_scale, amax, y_bf16, y_fp8, K, S, Pin, Po, 0, c10::nullopt, mbits,
                    sr_seed);
}

// fp8 dgrad: dx = conv(dz (e5m2, scales[0]), flipped/transposed e4m3 weights (scales[1])) masked
// by mask > 0; y_bf16 always, y_fp8 (e5m2, times out_scale) optional; amax = max |dx|
void conv_dgrad_fp8(const Tensor& dz8, const Tensor& w, const Tensor& mask, const Tensor& scales,
                    const Tensor& out_scale, const c10::optional<Tensor>& amax, const Tensor& y_bf16,
                    const c10::optional<Tensor>& y_fp8, int64_t K, int64_t S) {
  check_dev("conv_dgrad_fp8", dz8, w, mask, scales, out_scale, amax, y_bf16, y_fp8);
  conv_fwd_fp8_impl(dz8, w, out_scale, scales, out_scale, amax, y_bf16, y_fp8, K, S, 1, 1, 0, mask);
}

void conv_dgrad_fp8_bits(const Tensor& dz8, const Tensor& w8t, const Tensor& mbits, const Tensor& scales,
                         const Tensor& out_scale, const c10::optional<Tensor>& amax, const c10::optional<Tensor>& y_bf16,
                         const c10::optional<Tensor>& y_fp8, int64_t K, int64_t S) {
  conv_dgrad_fp8_bits_impl(dz8, w8t, mbits, scales, out_scale, amax, y_bf16, y_fp8, K, S);
}

void conv_dgrad_fp8_bf16(const Tensor& dz, const Tensor& w8t, const Tensor& mbits, const Tensor& scales,
                         const Tensor& in_scale, const c10::optional<Tensor>& amax, const Tensor& dx, int64_t K,
                         int64_t S) {
  conv_dgrad_fp8_bf16_impl(dz, w8t, mbits, scales, in_scale, amax, dx, K, S);
}

// every fp8 weight pack of a repack in one launch: job i packs ws[i] into outs[i] with the device
// scale scales[layer[i]] (forward layout, or transposed + flipped for the dgrad when transposed[i])
void pack_weights_fp8_multi(at::TensorList ws, at::TensorList outs, const Tensor& scales, at::IntArrayRef layer,
                            at::IntArrayRef transposed) {
  check_dev("pack_weights_fp8_multi", ws, outs, scales);
  const int n = (int)ws.size();
  TORCH_CHECK(n == (int)outs.size() && n == (int)layer.size() && n == (int)transposed.size() &&
                  n <= agk::kMaxFp8PackJobs, "pack_weights_fp8_multi: matching lists of at most 48 jobs");
  TORCH_CHECK(scales.scalar_type() == at::kFloat && scales.is_contiguous(), "scales f32");
  agk::Fp8PackArgs a{};
  a.n = n;
  for (int i = 0; i < n; ++i) {
    const Tensor& w = ws[i];
    const Tensor& o = outs[i];
    CHECK_F32(w); CHECK_CONTIG(w); CHECK_CONTIG(o);
    TORCH_CHECK(w.dim() == 4 && w.size(2) == w.size(3), "w OIHW");
    TORCH_CHECK(o.scalar_type() == at::kByte && o.dim() == 3 && (o.size(2) == 64 || o.size(2) == 32),
                "out (nch, rows_p, 64 or 32) uint8");
    TORCH_CHECK(layer[i] >= 0 && layer[i] < scales.numel(), "layer index");
    const int K = (int)w.size(2);
    const bool tr = transposed[i] != 0;
    const int rows_p = (int)o.size(1), nch = (int)o.size(0);
    agk::Fp8PackJob& j = a.jobs[i];
    j.w = w.data_ptr<float>();
    j.out = o.data_ptr<uint8_t>();
    j.scale = scales.data_ptr<float>() + layer[i];
    j.Cout_real = (int)w.size(0);
    j.Cin_real = (int)w.size(1);
    j.K = K;
    j.Cout_p = rows_p;
    // channel chunks per tap: the packed chunk count covers K*K taps (nch rounded up to even)
    const int cw = (int)o.size(2);
    j.Cin_p = (int)(((int64_t)(tr ? w.size(0) : w.size(1)) + cw - 1) / cw * cw);
    TORCH_CHECK(cw == 64 || j.Cin_p == 160, "32-channel chunks: 160-channel reductions only");
    TORCH_CHECK(nch >= K * K * (j.Cin_p / cw) && nch % (128 / cw) == 0, "out has too few chunks for the weights");
    j.nch = nch;
    j.cw = cw;
    j.transposed = tr ? 1 : 0;
  }
  agk::launch_pack_weights_fp8_multi(a, cur_stream());
  launch_check("pack_weights_fp8_multi");
}

// max |x| of a bf16 tensor into the fp8 amax slots (float bits, atomicMax per slot)
void absmax_bf16(const Tensor& x, const Tensor& amax, const Tensor& scale_any) {
  check_dev("absmax_bf16", x, amax, scale_any);
  CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "absmax_bf16: numel % 8 == 0 and a 16-byte aligned tensor");
  TORCH_CHECK(amax.scalar_type() == at::kInt && amax.numel() >= agk::kFp8AmaxSlots, "amax int32[64]");
  agk::launch_quantize_bf8_dev(bfp(x), nullptr, x.numel(), scale_any.data_ptr<float>(),
                               reinterpret_cast<unsigned*>(amax.data_ptr<int>()), cur_stream());
  launch_check("absmax_bf16");
}

void fp8_grad_scales(const Tensor& amax, const Tensor& gscales8, const Tensor& gosc, int64_t margin) {
  check_dev("fp8_grad_scales", amax, gscales8, gosc);
  TORCH_CHECK(amax.scalar_type() == at::kInt && gscales8.scalar_type() == at::kInt && gosc.scalar_type() == at::kFloat,
              "dtypes");
  const int L = (int)(amax.numel() / agk::kFp8AmaxSlots);
  TORCH_CHECK(amax.numel() % agk::kFp8AmaxSlots == 0 && L <= 64 && gscales8.numel() >= 2 * L && gosc.numel() >= L,
              "sizes (amax is (L, 64))");
  agk::launch_fp8_grad_scales(reinterpret_cast<unsigned*>(amax.data_ptr<int>()), gscales8.data_ptr<int>(),
                              gosc.data_ptr<float>(), L, (int)margin, cur_stream());
  launch_check("fp8_grad_scales");
}

// e5m2 (or, e4m3 = true, e4m3) quantisation with a device scale; amax (int32[64], float bits)
// accumulates max |x|
static void quantize_dev(const Tensor& x, const Tensor& y, const Tensor& scale, const Tensor& amax, bool e4m3);
void quantize_bf8(const Tensor& x, const Tensor& y, const Tensor& scale, const Tensor& amax) {
  quantize_dev(x, y, scale, amax, false);
}
void quantize_fp8_dev(const Tensor& x, const Tensor& y, const Tensor& scale, const Tensor& amax) {
  quantize_dev(x, y, scale, amax, true);
}
static void quantize_dev(const Tensor& x, const Tensor& y, const Tensor& scale, const Tensor& amax, bool e4m3) {
  check_dev("quantize_bf8", x, y, scale, amax);
  CHECK_BF16(x); CHECK_CONTIG(x); CHECK_DEV(x);
  TORCH_CHECK(y.scalar_type() == at::kByte && y.is_contiguous() && y.numel() == x.numel() && x.numel() % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0,
              "quantize_bf8: y uint8 of x's size, numel % 8 == 0, 16-byte aligned x");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && amax.scalar_type() == at::kInt &&
                  amax.numel() >= agk::kFp8AmaxSlots, "scale f32[1], amax int32[64]");
  agk::launch_quantize_bf8_dev(bfp(x), y.data_ptr<uint8_t>(), x.numel(), scale.data_ptr<float>(),
                               reinterpret_cast<unsigned*>(amax.data_ptr<int>()), cur_stream(), e4m3);
  launch_check(e4m3 ? "quantize_fp8_dev" : "quantize_bf8");
}

void pack_weights_fp8(const Tensor& w, const Tensor& out, double scale, const c10::optional<Tensor>& scale_dev,
                      bool transposed) {
  check_dev("pack_weights_fp8", w, out, scale_dev);
  CHECK_F32(w); CHECK_CONTIG(w);
  TORCH_CHECK(out.scalar_type() == at::kByte && out.is_contiguous() && out.dim() == 3 &&
                  (out.size(2) == 64 || out.size(2) == 32), "out (nch, rows_p, 64 or 32) uint8");
  const int K = (int)w.size(2);
  const int nch = (int)out.size(0), Cout_p = (int)out.size(1), cw = (int)out.size(2);
  // chunked extent: input channels, or output channels for the transposed (dgrad) packing
  const int Cin_p = ((int)w.size(transposed ? 0 : 1) + cw - 1) / cw * cw;
  TORCH_CHECK(cw == 64 || Cin_p == 160, "32-channel chunks: 160-channel reductions only");
  TORCH_CHECK(nch % (128 / cw) == 0 && nch >= K * K * (Cin_p / cw) && Cout_p >= w.size(transposed ? 1 : 0),
              "packed geometry");
  const float* sd = nullptr;
  if (scale_dev.has_value()) {
    CHECK_F32(*scale_dev);
    sd = scale_dev->data_ptr<float>();
  }
  agk::launch_pack_weights_fp8(w.data_ptr<float>(), out.data_ptr<uint8_t>(), (int)w.size(0), (int)w.size(1), K, Cout_p,
                               Cin_p, nch, (float)scale, sd, transposed ? 1 : 0, cw, cur_stream());
  launch_check("pack_weights_fp8");
}

// per-layer weight scales (device-side, no host sync)
void fp8_weight_scales(at::TensorList ws, const Tensor& wscale, const Tensor& scales8) {
  check_dev("fp8_weight_scales", ws, wscale, scales8);
  TORCH_CHECK((int)ws.size() <= agk::kMaxPackLayers, "too many layers");
  TORCH_CHECK(wscale.scalar_type() == at::kFloat && scales8.scalar_type() == at::kInt, "dtypes");
  TORCH_CHECK(wscale.numel() >= (int64_t)ws.size() && scales8.numel() >= 2 * (int64_t)ws.size(), "sizes");
  agk::Fp8WeightScalesArgs a{};
  for (size_t i = 0; i < ws.size(); ++i) {
    CHECK_F32(ws[i]); CHECK_CONTIG(ws[i]);
    a.w[i] = ws[i].data_ptr<float>();
    a.n[i] = (int)ws[i].numel();
  }
  a.wscale = wscale.data_ptr<float>();
  a.scales8 = scales8.data_ptr<int>();
  if (ws.empty()) return;
  agk::launch_fp8_weight_scales(a, (int)ws.size(), cur_stream());
  launch_check("fp8_weight_scales");
}

void fp8_act_scales(const Tensor& amax, const Tensor& scales8, const Tensor& osc, int64_t margin, int64_t max_drop) {
  check_dev("fp8_act_scales", amax, scales8, osc);
  TORCH_CHECK(amax.scalar_type() == at::kInt && scales8.scalar_type() == at::kInt && osc.scalar_type() == at::kFloat, "dtypes");
  const int L = (int)(amax.numel() / agk::kFp8AmaxSlots);
  TORCH_CHECK(amax.numel() % agk::kFp8AmaxSlots == 0 && L <= 64 && scales8.numel() >= 2 * L && osc.numel() >= L,
              "sizes (amax is (L, 64))");
  agk::launch_fp8_act_scales(reinterpret_cast<unsigned*>(amax.data_ptr<int>()), scales8.data_ptr<int>(),
                             osc.data_ptr<float>(), L, (int)margin, (int)max_drop, cur_stream());
  launch_check("fp8_act_scales");
}

void quantize_fp8(const Tensor& x, const Tensor& y, double scale) {
  check_dev("quantize_fp8", x, y);
  CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(y.scalar_type() == at::kByte && y.is_contiguous() && y.numel() == x.numel() && x.numel() % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0,
              "quantize_bf8: y uint8 of x's size, numel % 8 == 0, 16-byte aligned x");
  agk::launch_quantize_fp8(bfp(x), y.data_ptr<uint8_t>(), x.numel(), (float)scale, cur_stream());
  launch_check("quantize_fp8");
}

int64_t wgrad_tap_group(int64_t cout, int64_t cin, int64_t K) {
  return agk::wgrad_tap_group((int)cout, (int)cin, (int)K, 0);
}

// {taps per workgroup, workgroups per split, resident workgroups per CU, threads per workgroup} of the
// production wgrad
// src: standard (T, Cout, Cin) bf16 packs; dst: same-shape tensors receiving the weight-stationary order
// (conv_fwd tile 40 reads it; T = K*K or K*K + 1)
void ws_pack(at::TensorList src, at::TensorList dst) {
  check_dev("ws_pack", src, dst);
  TORCH_CHECK(src.size() == dst.size(), "ws_pack: list sizes");
  std::vector<agk::WsPackJob> jobs;
  for (size_t i = 0; i < src.size(); ++i) {
    CHECK_BF16(src[i]); CHECK_BF16(dst[i]); CHECK_CONTIG(src[i]); CHECK_CONTIG(dst[i]);
    TORCH_CHECK(src[i].dim() == 3 && src[i].sizes() == dst[i].sizes(), "ws_pack: (T, Cout, Cin) pairs of one shape");
    const int T = (int)src[i].size(0);
    int K = 1;
    while ((K + 1) * (K + 1) <= T) ++K;
    agk::WsPackJob j{};
    j.src = reinterpret_cast<const __bf16*>(src[i].data_ptr());
    j.dst = reinterpret_cast<__bf16*>(dst[i].data_ptr());
    j.Cout = (int)src[i].size(1);
    j.Cin = (int)src[i].size(2);
    j.K = K;
    jobs.push_back(j);
  }
  if (jobs.empty()) return;
  agk::launch_ws_pack(jobs, cur_stream());
  launch_check("ws_pack");
}

bool conv_ws_supported(int64_t cout, int64_t cin, int64_t K) {
  return agk::conv_ws_supported((int)cout, (int)cin, (int)K);
}

std::vector<int64_t> wgrad_plan(int64_t cout, int64_t cin, int64_t cin_real, int64_t K, int64_t variant) {
  int o[4];
  agk::wgrad_plan((int)cout, (int)cin, (int)(cin_real > 0 && cin_real < cin ? cin_real : cin), (int)K, (int)variant, o);
  return {o[0], o[1], o[2], o[3]};
}

void comm_proxy(const Tensor& src, const Tensor& dst, int64_t channels, double wire_us) {
  check_dev("comm_proxy", src, dst);
  TORCH_CHECK(src.scalar_type() == at::kFloat && dst.scalar_type() == at::kFloat && src.is_contiguous() &&
                  dst.is_contiguous() && dst.numel() >= src.numel() && src.numel() % 4 == 0,
              "comm_proxy: contiguous f32, dst >= src, numel % 4 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "comm_proxy: 16-byte aligned buffers");
  agk::launch_comm_proxy(src.data_ptr<float>(), dst.data_ptr<float>(), src.numel(), (int)channels, wire_us, cur_stream());
  launch_check("comm_proxy");
}

void sgd_update(const Tensor& p, const Tensor& g, double lr, double gscale) {
  check_dev("sgd_update", p, g);
  CHECK_F32(p); CHECK_F32(g); CHECK_CONTIG(p); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel(), "size mismatch");
  agk::launch_sgd(p.data_ptr<float>(), g.data_ptr<float>(), p.numel(), (float)lr, (float)gscale, cur_stream());
  launch_check("sgd_update");
}

void sgd_update_sched(const Tensor& p, const Tensor& g, const Tensor& sched, double gscale) {
  check_dev("sgd_update_sched", p, g, sched);
  CHECK_F32(p); CHECK_F32(g); CHECK_CONTIG(p); CHECK_CONTIG(g); CHECK_DEV(sched);
  TORCH_CHECK(p.numel() == g.numel(), "size mismatch");
  TORCH_CHECK(sched.scalar_type() == at::kDouble && sched.numel() == 4 && sched.is_contiguous(),
              "sched must be float64[4] {lr0, decay, iterations, lr}");
  agk::launch_sgd_sched(p.data_ptr<float>(), g.data_ptr<float>(), p.numel(), sched.data_ptr<double>(), (float)gscale,
                        cur_stream());
  launch_check("sgd_update_sched");
}

// Fused SGD + bf16 packs (pack.hip sgd_pack_kernel): conv layer i's OIHW weights live at flat offset
// w_meta[4i] with (Cout_real, Cin_real, K) = w_meta[4i+1 .. 4i+3]; wf[i] / wd[i] (wd empty: none) as
// pack_weights; plain SGD over (range_off, range_len); lr from ``sched`` (advanced) when given.
// opt: 0 SGD, 1 SGD + momentum (m1 = velocity), 2 Adam (m1, m2 = moments; an 8-entry sched carries its
// bias correction); hyper = {momentum, beta_1, beta_2, epsilon, nesterov}.
void sgd_pack(const Tensor& p, const Tensor& g, double lr, const c10::optional<Tensor>& sched, double gscale,
              at::IntArrayRef w_meta, at::TensorList wf, at::TensorList wd, at::IntArrayRef range_off,
              at::IntArrayRef range_len, int64_t opt, const c10::optional<Tensor>& m1,
              const c10::optional<Tensor>& m2, at::ArrayRef<double> hyper) {
  check_dev("sgd_pack", p, g, sched, wf, wd);
  check_dev("sgd_pack", p, m1, m2);
  TORCH_CHECK(opt >= 0 && opt <= 2, "sgd_pack: opt 0 (SGD), 1 (momentum) or 2 (Adam)");
  TORCH_CHECK(hyper.size() == 5, "sgd_pack: hyper = {momentum, beta_1, beta_2, epsilon, nesterov}");
  if (opt >= 1) {
    TORCH_CHECK(m1.has_value() && m1->scalar_type() == at::kFloat && m1->is_contiguous() &&
                m1->numel() == p.numel(), "sgd_pack: m1 must be a contiguous fp32 buffer like p");
  }
  if (opt == 2) {
    TORCH_CHECK(m2.has_value() && m2->scalar_type() == at::kFloat && m2->is_contiguous() &&
                m2->numel() == p.numel(), "sgd_pack: m2 must be a contiguous fp32 buffer like p");
  }
  CHECK_F32(p); CHECK_F32(g); CHECK_CONTIG(p); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel(), "sgd_pack: p and g sizes differ");
  const int nl = (int)wf.size();
  TORCH_CHECK(nl <= agk::kMaxPackLayers && (int)w_meta.size() == 4 * nl && (wd.size() == 0 || (int)wd.size() == nl),
              "sgd_pack: per-layer lists");
  TORCH_CHECK(range_off.size() == range_len.size() && (int)range_off.size() <= agk::kSgdPackMaxRanges, "sgd_pack: ranges");
  agk::SgdPackArgs a{};
  a.p = p.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.lr = (float)lr;
  a.gscale = (float)gscale;
  if (sched.has_value()) {
    TORCH_CHECK(sched->scalar_type() == at::kDouble && sched->is_contiguous() &&
                (sched->numel() == 4 || sched->numel() == 8),
                "sched must be float64[4] {lr0, decay, iterations, lr} or [8] (+ {beta_1, beta_2, opt, 0})");
    TORCH_CHECK(opt != 2 || sched->numel() == 8, "sgd_pack: Adam needs the 8-entry schedule");
    a.sched = sched->data_ptr<double>();
  }
  a.opt = (int)opt;
  a.m1 = opt >= 1 ? m1->data_ptr<float>() : nullptr;
  a.m2 = opt == 2 ? m2->data_ptr<float>() : nullptr;
  a.mom = (float)hyper[0];
  a.b1 = (float)hyper[1];
  a.b2 = (float)hyper[2];
  a.eps = (float)hyper[3];
  a.nesterov = hyper[4] != 0.0;
  a.nlayers = nl;
  for (int i = 0; i < nl; ++i) {
    agk::SgdPackLayer& L = a.layers[i];
    L.off = w_meta[4 * i];
    L.Cout_real = (int)w_meta[4 * i + 1]; L.Cin_real = (int)w_meta[4 * i + 2]; L.K = (int)w_meta[4 * i + 3];
    CHECK_BF16(wf[i]); CHECK_CONTIG(wf[i]);
    L.wf = bfp_mut(wf[i]);
    L.Cout_p = (int)wf[i].size(1); L.Cin_p = (int)wf[i].size(2);
    const int T = L.K * L.K, cpt = (L.Cin_real + 7) / 8;
    TORCH_CHECK(L.K == 1 || L.K == 3 || L.K == 5, "sgd_pack: 1x1, 3x3 and 5x5 kernels only");
    TORCH_CHECK(L.off >= 0 && L.off + (int64_t)L.Cout_real * L.Cin_real * T <= p.numel(), "sgd_pack: weight range");
    L.pk_cpt = (wf[i].size(0) != T && wf[i].size(0) != T + 1 && L.Cin_p == 64 && L.Cin_real <= 64 &&
                wf[i].size(0) == (T * cpt + 7) / 8) ? cpt : 0;
    TORCH_CHECK((wf[i].size(0) == T || wf[i].size(0) == T + 1 || L.pk_cpt > 0) && L.Cout_p >= L.Cout_real &&
                L.Cin_p >= L.Cin_real, "sgd_pack: bad wf");
    L.wd = nullptr;
    if (wd.size() && wd[i].numel() > 0) {
      CHECK_BF16(wd[i]); CHECK_CONTIG(wd[i]);
      TORCH_CHECK(L.pk_cpt == 0 && wd[i].size(1) == L.Cin_p && wd[i].size(2) == L.Cout_p, "sgd_pack: bad wd");
      L.wd = bfp_mut(wd[i]);
    }
  }
  a.nranges = (int)range_off.size();
  for (int r = 0; r < a.nranges; ++r) {
    TORCH_CHECK(range_off[r] >= 0 && range_len[r] >= 0 && range_off[r] + range_len[r] <= p.numel(), "sgd_pack: range");
    a.range_off[r] = range_off[r];
    a.range_len[r] = (int)range_len[r];
  }
  agk::launch_sgd_pack(a, cur_stream());
  launch_check("sgd_pack");
}

// C = beta*C + op(A) op(B) (+ bias); op(X) = X or X^T (no copies of transposed operands)
void dense_f32(const Tensor& A, const Tensor& B, const c10::optional<Tensor>& bias, const Tensor& C, bool transA,
               bool transB, double beta) {
  check_dev("dense_f32", A, B, bias, C);
  CHECK_F32(A); CHECK_F32(B); CHECK_F32(C); CHECK_DEV(A); CHECK_DEV(B); CHECK_DEV(C);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "2-D operands");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "row-major operands (unit column stride)");
  const int64_t M = transA ? A.size(1) : A.size(0), K = transA ? A.size(0) : A.size(1);
  const int64_t KB = transB ? B.size(1) : B.size(0), N = transB ? B.size(0) : B.size(1);
  TORCH_CHECK(K == KB, "inner dimensions differ: ", K, " vs ", KB);
  TORCH_CHECK(C.size(0) == M && C.size(1) == N, "C must be (", M, ", ", N, ")");
  agk::DenseArgs a{};
  a.A = A.data_ptr<float>(); a.B = B.data_ptr<float>(); a.C = C.data_ptr<float>();
  if (bias.has_value()) {
    CHECK_F32(*bias);
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "bias must be (N,)");
    a.bias = bias->data_ptr<float>();
  }
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.lda = (int)A.stride(0); a.ldb = (int)B.stride(0); a.ldc = (int)C.stride(0);
  a.beta = (float)beta;
  if (M == 0 || N == 0) return;
  a.splits = agk::dense_splits((int)M, (int)N, (int)K);
  Tensor ws;
  if (a.splits > 1) {
    ws = at::empty({(int64_t)a.splits * M * N}, C.options());
    a.ws = ws.data_ptr<float>();
  }
  agk::launch_dense_f32(a, transA, transB, cur_stream());
  launch_check("dense_f32");
}

// A deliberately invalid launch (2048 threads per block, above the 1024
// limit): the runtime rejects it, launch_check turns that into a Python
// RuntimeError -- the test of the error path every op shares.
void selftest_bad_launch() {
  agk::launch_invalid_config_probe(cur_stream());
  launch_check("selftest_bad_launch");
}

#ifdef AGK_DEBUG
// Debug build only: conv_fwd told that x holds half its real elements, so the
// kernel's bounds checks see "out-of-range" staging offsets (the accesses are
// redirected, the real buffer is never overrun) -- exercises the device check
// -> RuntimeError path end to end.
void debug_conv_fwd_understated(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& y, int64_t K,
                                int64_t S, int64_t Pin, int64_t Po) {
  check_dev("debug_conv_fwd_understated", x, w, bias, y);
  conv_fwd_impl(x, w, bias, c10::nullopt, y, K, S, Pin, Po, agk::MODE_BIAS_RELU, c10::nullopt, 0, nullptr,
                x.numel() / 2);
}
#endif

}  // namespace

TORCH_LIBRARY(alphago_amd, m) {
  m.def(
      "conv_fwd(Tensor x, Tensor w, Tensor? bias, Tensor? mask, Tensor(a!) y, int K, int S, int Pin, int Po, int mode, "
      "Tensor(b!)? mbits=None, int tile=0) -> ()");
  m.def(
      "conv_fwd_splitk(Tensor x, Tensor w, Tensor? bias, Tensor(a!) y, int K, int S, int Pin, int Po, int mode, "
      "Tensor(b!)? mbits, Tensor(c!) ws, int nsplit) -> ()");
  m.def("sample_moves(Tensor probs, Tensor has, Tensor(a!) out, float beta, int seed) -> ()");
  m.def("conv_wgrad(Tensor x, Tensor dz, Tensor(a!) slab, Tensor(b!) dbslab, int K, int S, int Pin, int Po, int cin_real=0, int variant=0) -> ()");
  m.def("conv_wgrad_reduce(Tensor slab, Tensor dbslab, Tensor(a!) grad_w, Tensor(b!)? grad_b, float scale, float beta) -> ()");
  m.def("conv_wgrad_reduce_multi(Tensor[] slabs, Tensor[] dbslabs, Tensor(a!)[] grad_ws, Tensor(b!)[] grad_bs, "
        "float scale, float beta) -> ()");
  m.def("conv_wgrad_direct(Tensor x, Tensor dz, Tensor(a!) grad_w, Tensor(b!)? grad_b, int K, int S, int Pin, int Po, "
        "float scale=1.0, float beta=0.0, int ksub=4) -> ()");
  m.def("wgrad_direct_supported(int cout, int cin, int cin_real, int K) -> bool", &wgrad_direct_supported_op);
  m.def("conv_dgrad_bits_bf8(Tensor dz, Tensor wd, Tensor(a!) dx, Tensor mbits, Tensor(b!) dx8, Tensor scale, "
        "Tensor(c!)? amax, int K, int S, int tile=0) -> ()");
  m.def("conv_wgrad_fp8(Tensor x8, Tensor dz8, Tensor(a!) slab, Tensor(b!) dbslab, Tensor xscale, Tensor gscale, "
        "Tensor gmul, int K, int S, int Pin, int Po, Tensor(c!)? amax=None) -> ()");
  m.def("wgrad_fp8_stage_px() -> int", &wgrad_fp8_stage_px);
  m.def(
      "policy_head(Tensor y, Tensor w, Tensor b, Tensor? target, Tensor? legal, Tensor? weight, Tensor(a!)? dz, Tensor(b!)? loss, "
      "Tensor(c!)? correct, Tensor(d!)? dhead, Tensor(e!)? probs, int S, float grad_scale, float temperature, "
      "int loss_kind=0) -> ()");
  m.def("head_logits(Tensor y, Tensor w, Tensor b, Tensor(a!) z, int S) -> ()");
  m.def("head_backward(Tensor y, Tensor w, Tensor dlogits, Tensor(a!) dz, Tensor(b!) dhead, int S, "
        "Tensor(c!)? dz8=None, Tensor? dz8_scale=None, Tensor(d!)? dz8_amax=None) -> ()");
  m.def("head_grad_sums(Tensor dhead, Tensor loss, Tensor correct, Tensor(a!) grad, Tensor(b!) sums) -> ()");
  m.def(
      "value_out(Tensor h, Tensor w2, Tensor b2, Tensor? target, Tensor? weight, Tensor(a!) v, Tensor(b!)? loss, "
      "Tensor(c!)? correct, Tensor(d!)? dh, Tensor(e!)? dout, float grad_scale) -> ()");
  m.def("pack_input(Tensor planes, Tensor? sym, Tensor? target, Tensor(a!)? target_out, Tensor(b!) out, int P, "
        "Tensor? rows=None, Tensor(c!)? out8=None) -> ()");
  m.def("pack_weights(Tensor[] ws, Tensor(a!)[] wf, Tensor(b!)[] wd) -> ()");
  m.def("sgd_update(Tensor(a!) p, Tensor g, float lr, float gscale) -> ()");
  m.def("comm_proxy(Tensor src, Tensor(a!) dst, int channels, float wire_us) -> ()");
  m.def("sgd_update_sched(Tensor(a!) p, Tensor g, Tensor(b!) sched, float gscale) -> ()");
  m.def("sgd_pack(Tensor(a!) p, Tensor g, float lr, Tensor(b!)? sched, float gscale, int[] w_meta, Tensor(c!)[] wf, "
        "Tensor(d!)[] wd, int[] range_off, int[] range_len, int opt, Tensor(e!)? m1, Tensor(f!)? m2, float[] hyper) -> ()");
  m.def("dense_f32(Tensor A, Tensor B, Tensor? bias, Tensor(a!) C, bool transA, bool transB, float beta) -> ()");
  // budget: node visits per capture / escape read; 4096 = lb::kLadderVisits (ladder_bb.h)
  m.def(
      "featurize(Tensor board, Tensor ages, Tensor meta, Tensor? ladder, int[] fids, int[] fplanes, Tensor(a!)? planes, "
      "Tensor(b!)? nhwc, Tensor(c!)? sensible, Tensor(d!)? legal, Tensor(e!)? overflow, int S, int P) -> ()");
  m.def(
      "conv_fwd_fp8(Tensor x, Tensor w, Tensor bias, Tensor scales, Tensor out_scale, Tensor(a!)? amax, "
      "Tensor(b!)? y_bf16, Tensor(c!)? y_fp8, int K, int S, int Pin, int Po, Tensor(d!)? mbits=None, "
      "Tensor? sr_seed=None) -> ()");
  m.def("pack_weights_fp8(Tensor w, Tensor(a!) out, float scale, Tensor? scale_dev, bool transposed=False) -> ()");
  m.def("pack_weights_fp8_multi(Tensor[] ws, Tensor(a!)[] outs, Tensor scales, int[] layer, int[] transposed) -> ()");
  m.def("absmax_bf16(Tensor x, Tensor(a!) amax, Tensor scale_any) -> ()");
  m.def("conv_dgrad_fp8_bf16(Tensor dz, Tensor w8t, Tensor mbits, Tensor scales, Tensor in_scale, Tensor(a!)? amax, "
        "Tensor(b!) dx, int K, int S) -> ()");
  m.def("conv_dgrad_fp8_bits(Tensor dz8, Tensor w8t, Tensor mbits, Tensor scales, Tensor out_scale, Tensor(a!)? amax, "
        "Tensor(b!)? y_bf16, Tensor(c!)? y_fp8, int K, int S) -> ()");
  m.def("conv_dgrad_fp8(Tensor dz8, Tensor w, Tensor mask, Tensor scales, Tensor out_scale, Tensor(a!)? amax, "
        "Tensor(b!) y_bf16, Tensor(c!)? y_fp8, int K, int S) -> ()");
  m.def("fp8_grad_scales(Tensor(a!) amax, Tensor(b!) gscales8, Tensor(c!) gosc, int margin) -> ()");
  m.def("quantize_bf8(Tensor x, Tensor(a!) y, Tensor scale, Tensor(b!) amax) -> ()");
  m.def("quantize_fp8_dev(Tensor x, Tensor(a!) y, Tensor scale, Tensor(b!) amax) -> ()");
  m.def("fp8_weight_scales(Tensor[] ws, Tensor(a!) wscale, Tensor(b!) scales8) -> ()");
  m.def("fp8_act_scales(Tensor(a!) amax, Tensor(b!) scales8, Tensor(c!) osc, int margin, int max_drop=0) -> ()");
  m.def("quantize_fp8(Tensor x, Tensor(a!) y, float scale) -> ()");
  m.def("wgrad_tap_group(int cout, int cin, int K) -> int", &wgrad_tap_group);
  m.def("wgrad_plan(int cout, int cin, int cin_real, int K, int variant=0) -> int[]", &wgrad_plan);
  m.def("conv_ws_supported(int cout, int cin, int K) -> bool", &conv_ws_supported);
  m.def("ws_pack(Tensor[] src, Tensor(a!)[] dst) -> ()");
  m.def("selftest_bad_launch() -> ()", &selftest_bad_launch);
  m.def("is_debug_build() -> bool", []() -> bool {
#ifdef AGK_DEBUG
    return true;
#else
    return false;
#endif
  });
#ifdef AGK_DEBUG
  m.def("debug_conv_fwd_understated(Tensor x, Tensor w, Tensor bias, Tensor(a!) y, int K, int S, int Pin, int Po) -> ()");
#endif
}

TORCH_LIBRARY_IMPL(alphago_amd, CUDA, m) {
  m.impl("conv_fwd", &conv_fwd);
  m.impl("sgd_pack", &sgd_pack);
  m.impl("conv_fwd_splitk", &conv_fwd_splitk);
  m.impl("sample_moves", &sample_moves);
  m.impl("conv_wgrad", &conv_wgrad);
  m.impl("conv_wgrad_reduce", &conv_wgrad_reduce);
  m.impl("conv_wgrad_direct", &conv_wgrad_direct);
  m.impl("conv_wgrad_reduce_multi", &conv_wgrad_reduce_multi);
  m.impl("conv_dgrad_bits_bf8", &conv_dgrad_bits_bf8);
  m.impl("conv_wgrad_fp8", &conv_wgrad_fp8);
  m.impl("policy_head", &policy_head);
  m.impl("pack_input", &pack_input);
  m.impl("head_logits", &head_logits);
  m.impl("head_backward", &head_backward);
  m.impl("value_out", &value_out);
  m.impl("pack_weights", &pack_weights);
  m.impl("ws_pack", &ws_pack);
  m.impl("sgd_update", &sgd_update);
  m.impl("comm_proxy", &comm_proxy);
  m.impl("sgd_update_sched", &sgd_update_sched);
  m.impl("dense_f32", &dense_f32);
#ifdef AGK_DEBUG
  m.impl("debug_conv_fwd_understated", &debug_conv_fwd_understated);
#endif
  m.impl("featurize", &featurize);
  m.impl("conv_fwd_fp8", &conv_fwd_fp8);
  m.impl("pack_weights_fp8", &pack_weights_fp8);
  m.impl("conv_dgrad_fp8", &conv_dgrad_fp8);
  m.impl("conv_dgrad_fp8_bf16", &conv_dgrad_fp8_bf16);
  m.impl("conv_dgrad_fp8_bits", &conv_dgrad_fp8_bits);
  m.impl("pack_weights_fp8_multi", &pack_weights_fp8_multi);
  m.impl("absmax_bf16", &absmax_bf16);
  m.impl("fp8_grad_scales", &fp8_grad_scales);
  m.impl("quantize_bf8", &quantize_bf8);
  m.impl("quantize_fp8_dev", &quantize_fp8_dev);
  m.impl("head_grad_sums", &head_grad_sums);
  m.impl("fp8_weight_scales", &fp8_weight_scales);
  m.impl("fp8_act_scales", &fp8_act_scales);
  m.impl("quantize_fp8", &quantize_fp8);
}
