// PyTorch custom-op registration for the gfx950 kernels: torch.ops.alphago_amd.*
// All ops write into caller-provided buffers (no allocation inside), run on the
// current HIP stream and are therefore safe to capture in HIP graphs.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a device tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")

const __bf16* bfp(const Tensor& t) { return reinterpret_cast<const __bf16*>(t.data_ptr()); }
__bf16* bfp_mut(const Tensor& t) { return reinterpret_cast<__bf16*>(t.data_ptr()); }

// x: (B, HPi, HPi, Cin) bf16; w: (T, Cout, Cin) bf16; y: (B, HPo, HPo, Cout) bf16
void conv_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, const c10::optional<Tensor>& mask,
              const Tensor& y, int64_t K, int64_t S, int64_t Pin, int64_t Po, int64_t mode,
              const c10::optional<Tensor>& mbits) {
  CHECK_DEV(x); CHECK_DEV(w); CHECK_DEV(y);
  CHECK_CONTIG(x); CHECK_CONTIG(w); CHECK_CONTIG(y);
  CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && w.dim() == 3, "bad ranks");
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3);
  const int64_t HPo = y.size(1), Cout = y.size(3);
  TORCH_CHECK(x.size(2) == HPi && y.size(2) == HPo && y.size(0) == B, "bad spatial dims");
  TORCH_CHECK(w.size(0) == K * K && w.size(1) == Cout && w.size(2) == Cin, "w must be (K*K, Cout, Cin)");
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0, "channels must be multiples of 64");
  TORCH_CHECK(Pin >= K / 2 && HPi == S + 2 * Pin && HPo == S + 2 * Po, "padding/geometry mismatch");
  TORCH_CHECK(B * HPi * HPi * Cin < (1ll << 31) && B * HPo * HPo * Cout < (1ll << 31), "tensor too large for int32 offsets");
  agk::ConvFwdArgs a{};
  a.x = bfp(x);
  a.w = bfp(w);
  a.y = bfp_mut(y);
  a.M = (int)(B * S * S);
  a.S = (int)S; a.Cin = (int)Cin; a.Cout = (int)Cout; a.K = (int)K;
  a.HPi = (int)HPi; a.offi = (int)(Pin - K / 2); a.HPo = (int)HPo; a.Po = (int)Po;
  if (mode == agk::MODE_BIAS_RELU) {
    TORCH_CHECK(bias.has_value(), "bias required");
    CHECK_F32(*bias); CHECK_DEV(*bias);
    TORCH_CHECK(bias->numel() >= Cout, "bias too small");
    a.bias = bias->data_ptr<float>();
  } else if (mode == agk::MODE_MASK) {
    TORCH_CHECK(mask.has_value(), "mask required");
    CHECK_BF16(*mask); CHECK_CONTIG(*mask);
    TORCH_CHECK(mask->sizes() == y.sizes(), "mask must match y");
    a.mask = bfp(*mask);
  }
  if (mbits.has_value()) {
    TORCH_CHECK(mbits->scalar_type() == at::kInt && mbits->is_contiguous(), "mbits int32");
    const int64_t words = (Cout % 192 == 0 ? Cout / 192 : Cout % 128 == 0 ? Cout / 128 : Cout / 64) * 8;
    TORCH_CHECK(mbits->numel() >= B * HPo * HPo * words, "mbits too small: need B*HPo*HPo*words");
    TORCH_CHECK(mode == agk::MODE_BIAS_RELU || mode == agk::MODE_MASKBITS, "mbits with modes 0 (write) / 3 (read)");
    if (mode == agk::MODE_BIAS_RELU) a.mbits_out = reinterpret_cast<uint32_t*>(mbits->data_ptr<int>());
    else a.mbits_in = reinterpret_cast<const uint32_t*>(mbits->data_ptr<int>());
  }
  TORCH_CHECK(mode != agk::MODE_MASKBITS || a.mbits_in, "mode 3 needs mbits");
  if (a.M == 0) return;
  agk::launch_conv_fwd(a, (int)mode, cur_stream());
}

// slab: (nsplit, T, Cout, Cin) f32; dbslab: (nsplit, Cout) f32
void conv_wgrad(const Tensor& x, const Tensor& dz, const Tensor& slab, const Tensor& dbslab, int64_t K, int64_t S,
                int64_t Pin, int64_t Po, int64_t cin_real) {
  CHECK_DEV(x); CHECK_DEV(dz); CHECK_DEV(slab); CHECK_DEV(dbslab);
  CHECK_BF16(x); CHECK_BF16(dz); CHECK_F32(slab); CHECK_F32(dbslab);
  CHECK_CONTIG(x); CHECK_CONTIG(dz); CHECK_CONTIG(slab); CHECK_CONTIG(dbslab);
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3);
  const int64_t HPo = dz.size(1), Cout = dz.size(3);
  const int64_t nsplit = slab.size(0);
  TORCH_CHECK(slab.dim() == 4 && slab.size(1) == K * K && slab.size(2) == Cout && slab.size(3) == Cin, "bad slab");
  TORCH_CHECK(dbslab.size(0) == nsplit && dbslab.size(1) == Cout, "bad dbias slab");
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0, "channels must be multiples of 64");
  TORCH_CHECK(HPi == S + 2 * Pin && HPo == S + 2 * Po && Po >= 1 && Pin >= K / 2, "geometry mismatch");
  agk::ConvWgradArgs a{};
  a.x = bfp(x); a.dz = bfp(dz);
  a.slab = slab.data_ptr<float>();
  a.dbias_slab = dbslab.data_ptr<float>();
  a.M = (int)(B * S * S); a.S = (int)S; a.Cin = (int)Cin; a.Cout = (int)Cout; a.K = (int)K; a.T = (int)(K * K);
  a.HPi = (int)HPi; a.offi = (int)(Pin - K / 2); a.HPo = (int)HPo; a.Po = (int)Po;
  a.cin_real = (cin_real > 0 && cin_real < Cin) ? (int)cin_real : (int)Cin;
  const int sp = agk::wgrad_stage_pixels();
  const int nks = (a.M + sp - 1) / sp;
  a.nsplit = (int)nsplit;
  a.ksteps_per_split = (nks + a.nsplit - 1) / a.nsplit;
  agk::launch_conv_wgrad(a, cur_stream());
}

void conv_wgrad_reduce(const Tensor& slab, const Tensor& dbslab, const Tensor& grad_w, const c10::optional<Tensor>& grad_b,
                       double scale, double beta) {
  CHECK_F32(slab); CHECK_F32(grad_w); CHECK_CONTIG(grad_w);
  const int64_t nsplit = slab.size(0), T = slab.size(1), Cout = slab.size(2), Cin = slab.size(3);
  TORCH_CHECK(grad_w.dim() == 4 && grad_w.size(2) * grad_w.size(3) == T, "grad_w must be OIHW");
  TORCH_CHECK(Cin % 4 == 0, "slab channels must be a multiple of 4 (16-byte split reads)");
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
  agk::launch_wgrad_reduce(a, cur_stream());
}

void policy_head(const Tensor& y, const Tensor& w, const Tensor& b, const c10::optional<Tensor>& target,
                 const c10::optional<Tensor>& legal, const c10::optional<Tensor>& weight, const c10::optional<Tensor>& dz, const c10::optional<Tensor>& loss,
                 const c10::optional<Tensor>& correct, const c10::optional<Tensor>& dhead,
                 const c10::optional<Tensor>& probs, int64_t S, double grad_scale, double temperature, int64_t loss_kind) {
  CHECK_BF16(y); CHECK_CONTIG(y); CHECK_F32(w); CHECK_F32(b);
  const int64_t B = y.size(0), C = y.size(3);
  TORCH_CHECK(y.size(1) == S + 2, "head input must have pad 1");
  TORCH_CHECK(C % 8 == 0 && C <= 256, "head channels must be a multiple of 8 and <= 256");
  TORCH_CHECK(S * S <= 368, "board too large");
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
}

// z: (B, S*S) f32 <- y (B, S+2, S+2, C) bf16 . w + b
void head_logits(const Tensor& y, const Tensor& w, const Tensor& b, const Tensor& z, int64_t S) {
  CHECK_BF16(y); CHECK_CONTIG(y); CHECK_F32(w); CHECK_F32(b); CHECK_F32(z); CHECK_CONTIG(z);
  const int64_t B = y.size(0), C = y.size(3);
  TORCH_CHECK(y.size(1) == S + 2 && C % 8 == 0 && C <= 256 && w.numel() <= C && S * S <= 368, "head geometry");
  TORCH_CHECK(z.numel() == B * S * S, "z must be (B, S*S)");
  agk::PolicyHeadArgs a{};
  a.y = bfp(y); a.w = w.data_ptr<float>(); a.b = b.data_ptr<float>(); a.probs = z.data_ptr<float>();
  a.B = (int)B; a.S = (int)S; a.C = (int)C; a.C_real = (int)w.numel();
  if (B == 0) return;
  agk::launch_head_logits(a, cur_stream());
}

// dz (B, S+2, S+2, C) bf16 <- ReLU'(y) * dlogits x w;  dhead (B, C_real+1) partials
void head_backward(const Tensor& y, const Tensor& w, const Tensor& dlogits, const Tensor& dz, const Tensor& dhead,
                   int64_t S) {
  CHECK_BF16(y); CHECK_CONTIG(y); CHECK_F32(w); CHECK_F32(dlogits); CHECK_CONTIG(dlogits);
  CHECK_BF16(dz); CHECK_CONTIG(dz); CHECK_F32(dhead);
  const int64_t B = y.size(0), C = y.size(3);
  TORCH_CHECK(y.size(1) == S + 2 && C % 8 == 0 && C <= 256 && w.numel() <= C && S * S <= 368, "head geometry");
  TORCH_CHECK(dz.sizes() == y.sizes() && dlogits.numel() == B * S * S && dhead.numel() >= B * (w.numel() + 1), "shapes");
  agk::PolicyHeadArgs a{};
  a.y = bfp(y); a.w = w.data_ptr<float>(); a.dz = bfp_mut(dz); a.dhead = dhead.data_ptr<float>();
  a.B = (int)B; a.S = (int)S; a.C = (int)C; a.C_real = (int)w.numel();
  if (B == 0) return;
  agk::launch_head_backward(a, dlogits.data_ptr<float>(), cur_stream());
}

void value_out(const Tensor& h, const Tensor& w2, const Tensor& b2, const c10::optional<Tensor>& target,
               const c10::optional<Tensor>& weight, const Tensor& v, const c10::optional<Tensor>& loss,
               const c10::optional<Tensor>& correct, const c10::optional<Tensor>& dh, const c10::optional<Tensor>& dout,
               double grad_scale) {
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
}

void pack_input(const Tensor& planes, const c10::optional<Tensor>& sym, const c10::optional<Tensor>& target,
                const c10::optional<Tensor>& target_out, const Tensor& out, int64_t P) {
  TORCH_CHECK(planes.scalar_type() == at::kByte && planes.is_contiguous() && planes.dim() == 4, "planes: uint8 (B,C,S,S)");
  CHECK_BF16(out); CHECK_CONTIG(out);
  const int64_t B = planes.size(0), C = planes.size(1), S = planes.size(2);
  TORCH_CHECK(out.size(0) == B && out.size(1) == S + 2 * P && out.size(3) >= C && out.size(3) % 8 == 0, "bad out");
  agk::PackInputArgs a{};
  a.planes = planes.data_ptr<uint8_t>();
  a.sym = sym.has_value() ? sym->data_ptr<int>() : nullptr;
  a.target = target.has_value() ? target->data_ptr<int>() : nullptr;
  a.target_out = target_out.has_value() ? target_out->data_ptr<int>() : nullptr;
  TORCH_CHECK(!a.target_out || a.target, "target_out needs target");
  a.out = bfp_mut(out);
  a.B = (int)B; a.S = (int)S; a.Creal = (int)C; a.Cp = (int)out.size(3); a.P = (int)P;
  if (B == 0) return;
  agk::launch_pack_input(a, cur_stream());
}

// ws: list of OIHW fp32; wf: list of (T, Coutp, Cinp) bf16; wd: list (possibly empty entries skipped)
void pack_weights(at::TensorList ws, at::TensorList wf, at::TensorList wd) {
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
      TORCH_CHECK(wf[i].size(0) == L.K * L.K && L.Cout_p >= L.Cout_real && L.Cin_p >= L.Cin_real, "bad wf");
      L.wd = nullptr;
      if (wd.size() && wd[i].numel() > 0) {
        CHECK_BF16(wd[i]);
        TORCH_CHECK(wd[i].size(1) == L.Cin_p && wd[i].size(2) == L.Cout_p, "bad wd");
        L.wd = bfp_mut(wd[i]);
      }
    }
    agk::launch_pack_weights(a, cur_stream());
  }
}

// board: (B, S*S) int8; ages: (B, S*S) uint8; meta: (B, 2) int32; fids: feature ids
// (engine numbering) with their plane counts; every output optional.
void featurize(const Tensor& board, const Tensor& ages, const Tensor& meta, const c10::optional<Tensor>& ladder,
               at::IntArrayRef fids, at::IntArrayRef fplanes, const c10::optional<Tensor>& planes,
               const c10::optional<Tensor>& nhwc, const c10::optional<Tensor>& sensible,
               const c10::optional<Tensor>& legal, const c10::optional<Tensor>& overflow, int64_t S, int64_t P) {
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
}

// x: (B, HPi, HPi, Cin) uint8 (e4m3); w: (nch, Cout, 64) uint8; scales int32[2]; out_scale f32[1]
void conv_fwd_fp8(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& scales, const Tensor& out_scale,
                  const c10::optional<Tensor>& amax, const c10::optional<Tensor>& y_bf16,
                  const c10::optional<Tensor>& y_fp8, int64_t K, int64_t S, int64_t Pin, int64_t Po) {
  CHECK_DEV(x); CHECK_DEV(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.scalar_type() == at::kByte && w.scalar_type() == at::kByte, "fp8 tensors are stored as uint8");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 3 && w.size(2) == 64, "x (B,HP,HP,C), w (nch, Cout, 64)");
  TORCH_CHECK(scales.scalar_type() == at::kInt && scales.numel() >= 2 && out_scale.scalar_type() == at::kFloat, "scales");
  CHECK_F32(bias);
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3), nch = w.size(0), Cout = w.size(1);
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0 && nch % 2 == 0 && nch >= K * K * (Cin / 64), "channel geometry");
  TORCH_CHECK(Pin >= K / 2 && HPi == S + 2 * Pin, "padding/geometry mismatch");
  TORCH_CHECK(y_bf16.has_value() || y_fp8.has_value(), "need an output");
  agk::ConvFp8Args a{};
  a.x = x.data_ptr<uint8_t>(); a.w = w.data_ptr<uint8_t>(); a.bias = bias.data_ptr<float>();
  a.scales = scales.data_ptr<int>(); a.out_scale = out_scale.data_ptr<float>();
  const int64_t HPo = S + 2 * Po;
  if (y_bf16.has_value()) {
    CHECK_BF16(*y_bf16); CHECK_CONTIG(*y_bf16);
    TORCH_CHECK(y_bf16->size(0) == B && y_bf16->size(1) == HPo && y_bf16->size(3) == Cout, "y_bf16 shape");
    a.y_bf16 = bfp_mut(*y_bf16);
  }
  if (y_fp8.has_value()) {
    TORCH_CHECK(y_fp8->scalar_type() == at::kByte && y_fp8->is_contiguous(), "y_fp8 uint8");
    TORCH_CHECK(y_fp8->size(0) == B && y_fp8->size(1) == HPo && y_fp8->size(3) == Cout, "y_fp8 shape");
    a.y_fp8 = y_fp8->data_ptr<uint8_t>();
  }
  if (amax.has_value()) {
    TORCH_CHECK(amax->scalar_type() == at::kInt && amax->numel() >= agk::kFp8AmaxSlots,
                "amax int32[64] (float bits, per-workgroup slots)");
    a.amax = reinterpret_cast<unsigned*>(amax->data_ptr<int>());
  }
  a.M = (int)(B * S * S); a.S = (int)S; a.Cin = (int)Cin; a.Cout = (int)Cout; a.K = (int)K;
  a.HPi = (int)HPi; a.offi = (int)(Pin - K / 2); a.HPo = (int)HPo; a.Po = (int)Po; a.nch = (int)nch;
  TORCH_CHECK(B * HPi * HPi * Cin < (1ll << 31), "tensor too large for int32 offsets");
  if (a.M == 0) return;
  agk::launch_conv_fwd_fp8(a, cur_stream());
}

void pack_weights_fp8(const Tensor& w, const Tensor& out, double scale, const c10::optional<Tensor>& scale_dev) {
  CHECK_F32(w); CHECK_CONTIG(w);
  TORCH_CHECK(out.scalar_type() == at::kByte && out.is_contiguous() && out.dim() == 3 && out.size(2) == 64, "out");
  const int K = (int)w.size(2);
  const int nch = (int)out.size(0), Cout_p = (int)out.size(1);
  const int Cin_p = ((int)w.size(1) + 63) / 64 * 64;
  TORCH_CHECK(nch % 2 == 0 && nch >= K * K * (Cin_p / 64) && Cout_p >= w.size(0), "packed geometry");
  const float* sd = nullptr;
  if (scale_dev.has_value()) {
    CHECK_F32(*scale_dev);
    sd = scale_dev->data_ptr<float>();
  }
  agk::launch_pack_weights_fp8(w.data_ptr<float>(), out.data_ptr<uint8_t>(), (int)w.size(0), (int)w.size(1), K, Cout_p,
                               Cin_p, nch, (float)scale, sd, cur_stream());
}

// per-layer weight scales (device-side, no host sync)
void fp8_weight_scales(at::TensorList ws, const Tensor& wscale, const Tensor& scales8) {
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
}

void fp8_act_scales(const Tensor& amax, const Tensor& scales8, const Tensor& osc, int64_t margin) {
  TORCH_CHECK(amax.scalar_type() == at::kInt && scales8.scalar_type() == at::kInt && osc.scalar_type() == at::kFloat, "dtypes");
  const int L = (int)(amax.numel() / agk::kFp8AmaxSlots);
  TORCH_CHECK(amax.numel() % agk::kFp8AmaxSlots == 0 && L <= 64 && scales8.numel() >= 2 * L && osc.numel() >= L,
              "sizes (amax is (L, 64))");
  agk::launch_fp8_act_scales(reinterpret_cast<unsigned*>(amax.data_ptr<int>()), scales8.data_ptr<int>(),
                             osc.data_ptr<float>(), L, (int)margin, cur_stream());
}

void quantize_fp8(const Tensor& x, const Tensor& y, double scale) {
  CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(y.scalar_type() == at::kByte && y.is_contiguous() && y.numel() == x.numel() && x.numel() % 4 == 0, "y");
  agk::launch_quantize_fp8(bfp(x), y.data_ptr<uint8_t>(), x.numel(), (float)scale, cur_stream());
}

void set_conv_tile(int64_t bm) { agk::set_conv_fwd_tile((int)bm); }
// diagnostic: per-wave segment cycle sums of the ping-pong forward, 8 uint64 per wave
void set_conv_debug(const c10::optional<Tensor>& buf) {
  if (buf.has_value()) {
    CHECK_DEV(*buf);
    TORCH_CHECK(buf->scalar_type() == at::kLong && buf->is_contiguous(), "int64 buffer");
    agk::set_conv_debug(reinterpret_cast<unsigned long long*>(buf->data_ptr<int64_t>()));
  } else {
    agk::set_conv_debug(nullptr);
  }
}
void set_wgrad_variant(int64_t v) { agk::set_wgrad_variant((int)v); }
void set_fp8_variant(int64_t v) { agk::set_fp8_variant((int)v); }
int64_t wgrad_tap_group(int64_t cout, int64_t cin, int64_t K) { return agk::wgrad_tap_group((int)cout, (int)cin, (int)K); }

void sgd_update(const Tensor& p, const Tensor& g, double lr, double gscale) {
  CHECK_F32(p); CHECK_F32(g); CHECK_CONTIG(p); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel(), "size mismatch");
  agk::launch_sgd(p.data_ptr<float>(), g.data_ptr<float>(), p.numel(), (float)lr, (float)gscale, cur_stream());
}

}  // namespace

TORCH_LIBRARY(alphago_amd, m) {
  m.def(
      "conv_fwd(Tensor x, Tensor w, Tensor? bias, Tensor? mask, Tensor(a!) y, int K, int S, int Pin, int Po, int mode, "
      "Tensor(b!)? mbits=None) -> ()");
  m.def("conv_wgrad(Tensor x, Tensor dz, Tensor(a!) slab, Tensor(b!) dbslab, int K, int S, int Pin, int Po, int cin_real=0) -> ()");
  m.def("conv_wgrad_reduce(Tensor slab, Tensor dbslab, Tensor(a!) grad_w, Tensor(b!)? grad_b, float scale, float beta) -> ()");
  m.def(
      "policy_head(Tensor y, Tensor w, Tensor b, Tensor? target, Tensor? legal, Tensor? weight, Tensor(a!)? dz, Tensor(b!)? loss, "
      "Tensor(c!)? correct, Tensor(d!)? dhead, Tensor(e!)? probs, int S, float grad_scale, float temperature, "
      "int loss_kind=0) -> ()");
  m.def("head_logits(Tensor y, Tensor w, Tensor b, Tensor(a!) z, int S) -> ()");
  m.def("head_backward(Tensor y, Tensor w, Tensor dlogits, Tensor(a!) dz, Tensor(b!) dhead, int S) -> ()");
  m.def(
      "value_out(Tensor h, Tensor w2, Tensor b2, Tensor? target, Tensor? weight, Tensor(a!) v, Tensor(b!)? loss, "
      "Tensor(c!)? correct, Tensor(d!)? dh, Tensor(e!)? dout, float grad_scale) -> ()");
  m.def("pack_input(Tensor planes, Tensor? sym, Tensor? target, Tensor(a!)? target_out, Tensor(b!) out, int P) -> ()");
  m.def("pack_weights(Tensor[] ws, Tensor(a!)[] wf, Tensor(b!)[] wd) -> ()");
  m.def("sgd_update(Tensor(a!) p, Tensor g, float lr, float gscale) -> ()");
  m.def(
      "featurize(Tensor board, Tensor ages, Tensor meta, Tensor? ladder, int[] fids, int[] fplanes, Tensor(a!)? planes, "
      "Tensor(b!)? nhwc, Tensor(c!)? sensible, Tensor(d!)? legal, Tensor(e!)? overflow, int S, int P) -> ()");
  m.def(
      "conv_fwd_fp8(Tensor x, Tensor w, Tensor bias, Tensor scales, Tensor out_scale, Tensor(a!)? amax, "
      "Tensor(b!)? y_bf16, Tensor(c!)? y_fp8, int K, int S, int Pin, int Po) -> ()");
  m.def("pack_weights_fp8(Tensor w, Tensor(a!) out, float scale, Tensor? scale_dev) -> ()");
  m.def("fp8_weight_scales(Tensor[] ws, Tensor(a!) wscale, Tensor(b!) scales8) -> ()");
  m.def("fp8_act_scales(Tensor(a!) amax, Tensor(b!) scales8, Tensor(c!) osc, int margin) -> ()");
  m.def("quantize_fp8(Tensor x, Tensor(a!) y, float scale) -> ()");
  m.def("set_conv_tile(int bm) -> ()", &set_conv_tile);
  m.def("set_conv_debug(Tensor? buf) -> ()", &set_conv_debug);
  m.def("set_wgrad_variant(int v) -> ()", &set_wgrad_variant);
  m.def("set_fp8_variant(int v) -> ()", &set_fp8_variant);
  m.def("wgrad_tap_group(int cout, int cin, int K) -> int", &wgrad_tap_group);
}

TORCH_LIBRARY_IMPL(alphago_amd, CUDA, m) {
  m.impl("conv_fwd", &conv_fwd);
  m.impl("conv_wgrad", &conv_wgrad);
  m.impl("conv_wgrad_reduce", &conv_wgrad_reduce);
  m.impl("policy_head", &policy_head);
  m.impl("pack_input", &pack_input);
  m.impl("head_logits", &head_logits);
  m.impl("head_backward", &head_backward);
  m.impl("value_out", &value_out);
  m.impl("pack_weights", &pack_weights);
  m.impl("sgd_update", &sgd_update);
  m.impl("featurize", &featurize);
  m.impl("conv_fwd_fp8", &conv_fwd_fp8);
  m.impl("pack_weights_fp8", &pack_weights_fp8);
  m.impl("fp8_weight_scales", &fp8_weight_scales);
  m.impl("fp8_act_scales", &fp8_act_scales);
  m.impl("quantize_fp8", &quantize_fp8);
}
