// Tensor -> kernel-argument marshalling of the conv ops, shared by the
// production op library (ops.cpp, torch.ops.alphago_amd) and the kernel-lab
// library (ops_lab.cpp, torch.ops.alphago_amd_lab).  Every launch is followed
// by launch_check(): a launch the runtime rejects raises a Python error; in a
// debug build (AGK_DEBUG) the op also synchronises and raises on any device
// bounds-check failure recorded by the kernels.
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <string>

#include "kernels.h"

namespace agk_ops {

using at::Tensor;

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a device tensor")

// Every tensor argument of an op must live on the current GPU: a host pointer (or another
// device's memory) handed to a kernel faults the device (an illegal access can take the
// whole card down), so the ops refuse it on the host first.  check_dev("op", a, b, ...)
// accepts tensors, optional tensors and tensor lists.
inline void check_dev_one(const char* op, c10::DeviceIndex dev, const Tensor& t) {
  TORCH_CHECK(!t.defined() || t.is_cuda(), op, ": tensor argument on ", t.device(), ", expected a GPU tensor");
  TORCH_CHECK(!t.defined() || t.get_device() == dev, op, ": tensor argument on ", t.device(),
              " but the current device is ", static_cast<int>(dev), " (kernels launch on the current device)");
}
inline void check_dev_one(const char* op, c10::DeviceIndex dev, const c10::optional<Tensor>& t) {
  if (t.has_value()) check_dev_one(op, dev, *t);
}
inline void check_dev_one(const char* op, c10::DeviceIndex dev, at::TensorList l) {
  for (const Tensor& t : l) check_dev_one(op, dev, t);
}
template <typename... Ts>
inline void check_dev(const char* op, const Ts&... ts) {
  const c10::DeviceIndex dev = c10::hip::current_device();
  (check_dev_one(op, dev, ts), ...);
}

#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")

inline const __bf16* bfp(const Tensor& t) { return reinterpret_cast<const __bf16*>(t.data_ptr()); }
inline __bf16* bfp_mut(const Tensor& t) { return reinterpret_cast<__bf16*>(t.data_ptr()); }

// Raise if the last launch on this thread failed (bad configuration, missing
// code object, ...); with AGK_DEBUG also wait for the kernel and raise on a
// recorded device bounds violation.
inline void launch_check(const char* op) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, op, ": kernel launch failed: ", hipGetErrorString(e));
#ifdef AGK_DEBUG
  const unsigned code = agk::debug_error_fetch_and_clear(cur_stream());
  TORCH_CHECK(code == 0, op, ": device bounds check failed (debug build), code 0x", std::to_string(code));
#endif
}

inline void conv_fwd_impl(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                          const c10::optional<Tensor>& mask, const Tensor& y, int64_t K, int64_t S, int64_t Pin,
                          int64_t Po, int64_t mode, const c10::optional<Tensor>& mbits, int tile,
                          unsigned long long* dbg = nullptr, long long x_elems_override = -1,
                          const c10::optional<Tensor>& y_bf8 = c10::nullopt,
                          const c10::optional<Tensor>& bf8_scale = c10::nullopt,
                          const c10::optional<Tensor>& bf8_amax = c10::nullopt, int pk_cpt = 0,
                          const c10::optional<Tensor>& sk_ws = c10::nullopt, int sk_nsplit = 0) {
  check_dev("conv_fwd_impl", x, w, bias, mask, y, mbits, y_bf8, bf8_scale, bf8_amax, sk_ws);
  CHECK_DEV(x); CHECK_DEV(w); CHECK_DEV(y);
  CHECK_CONTIG(x); CHECK_CONTIG(w); CHECK_CONTIG(y);
  CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && w.dim() == 3, "bad ranks");
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3);
  const int64_t HPo = y.size(1), Cout = y.size(3);
  TORCH_CHECK(x.size(2) == HPi && y.size(2) == HPo && y.size(0) == B, "bad spatial dims");
  // Cin % 64 == 32 (straddled K-steps, 160-wide tile only): one extra all-zero weight tap
  const int64_t taps = pk_cpt > 0 ? (K * K * pk_cpt + 7) / 8 : K * K + (Cin % 64 == 32 ? 1 : 0);
  TORCH_CHECK(w.size(0) == taps && w.size(1) == Cout && w.size(2) == Cin,
              "w must be (K*K, Cout, Cin), or (K*K + 1, Cout, Cin) when Cin % 64 == 32, or the packed-tap layout "
              "(ceil(K*K*cpt/8), Cout, 64)");
  TORCH_CHECK(pk_cpt == 0 || (Cin == 64 && mode == agk::MODE_BIAS_RELU && pk_cpt >= 4 && pk_cpt <= 8),
              "packed-tap forward: 64-channel input, bias + ReLU, 32 < cin_real <= 64");
  TORCH_CHECK((Cout % 64 == 0 && Cin % 64 == 0) || (Cout == 160 && (Cin % 64 == 0 || Cin == 160)),
              "channels must be multiples of 64, or Cout 160 with Cin 160 / a multiple of 64");
  TORCH_CHECK(Pin >= K / 2 && HPi == S + 2 * Pin && HPo == S + 2 * Po, "padding/geometry mismatch");
  TORCH_CHECK(B * HPi * HPi * Cin < (1ll << 31) && B * HPo * HPo * Cout < (1ll << 31), "tensor too large for int32 offsets");
  agk::ConvFwdArgs a{};
  a.tile = tile;
  a.dbg = dbg;
  a.x_elems = x_elems_override >= 0 ? x_elems_override : x.numel();
  a.w_elems = w.numel();
  a.y_elems = y.numel();
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
    CHECK_DEV(*mbits);
    TORCH_CHECK(mbits->scalar_type() == at::kInt && mbits->is_contiguous(), "mbits int32");
    const int64_t words = (Cout == 160 ? 1 : Cout % 192 == 0 ? Cout / 192 : Cout % 128 == 0 ? Cout / 128 : Cout / 64) * 8;
    TORCH_CHECK(mbits->numel() >= B * HPo * HPo * words, "mbits too small: need B*HPo*HPo*words");
    TORCH_CHECK(mode == agk::MODE_BIAS_RELU || mode == agk::MODE_MASKBITS, "mbits with modes 0 (write) / 3 (read)");
    if (mode == agk::MODE_BIAS_RELU) a.mbits_out = reinterpret_cast<uint32_t*>(mbits->data_ptr<int>());
    else a.mbits_in = reinterpret_cast<const uint32_t*>(mbits->data_ptr<int>());
  }
  TORCH_CHECK(mode != agk::MODE_MASKBITS || a.mbits_in, "mode 3 needs mbits");
  if (y_bf8.has_value()) {  // dgrad's e5m2 copy (y * bf8_scale) and max |y|, for the fp8 wgrad
    TORCH_CHECK(mode == agk::MODE_MASKBITS, "y_bf8: bitmask dgrad (mode 3) only");
    CHECK_DEV(*y_bf8);
    TORCH_CHECK(y_bf8->scalar_type() == at::kByte && y_bf8->is_contiguous() && y_bf8->sizes() == y.sizes(),
                "y_bf8: uint8 with y's shape");
    TORCH_CHECK(bf8_scale.has_value() && bf8_scale->scalar_type() == at::kFloat && bf8_scale->numel() >= 1,
                "y_bf8 needs a device fp32 scale");
    a.y_bf8 = y_bf8->data_ptr<uint8_t>();
    a.bf8_scale = bf8_scale->data_ptr<float>();
    if (bf8_amax.has_value()) {
      TORCH_CHECK(bf8_amax->scalar_type() == at::kInt && bf8_amax->numel() >= agk::kFp8AmaxSlots &&
                      bf8_amax->is_contiguous(), "bf8_amax: int32[64]");
      a.bf8_amax = reinterpret_cast<unsigned*>(bf8_amax->data_ptr<int>());
    }
  }
  if (sk_ws.has_value()) {  // split-K (tile 38): fp32 partials [nsplit][M][Cout]
    CHECK_F32(*sk_ws); CHECK_CONTIG(*sk_ws);
    TORCH_CHECK(tile == 38 && sk_nsplit >= 1 && sk_nsplit <= 64, "split-K: tile 38, 1 <= nsplit <= 64");
    // any width the conv takes (line 88): 64 / 128 / 192-wide tiles, or the 160-wide value tile
    TORCH_CHECK(mode != agk::MODE_MASK && !y_bf8.has_value(), "split-K: modes 0, 2, 3 without an e5m2 copy");
    TORCH_CHECK(sk_ws->numel() >= (int64_t)sk_nsplit * a.M * Cout, "split-K workspace too small: nsplit*M*Cout");
    a.sk_ws = sk_ws->data_ptr<float>();
    a.sk_nsplit = sk_nsplit;
  } else {
    TORCH_CHECK(tile != 38, "tile 38 (split-K) needs a workspace: conv_fwd_splitk");
  }
  if (a.M == 0) return;
#ifdef AGK_KERNEL_LAB
  if (pk_cpt > 0) agk::launch_conv_fwd_pk(a, pk_cpt, cur_stream());
  else agk::launch_conv_fwd(a, (int)mode, cur_stream());
#else
  TORCH_CHECK(pk_cpt <= 0, "conv_fwd: the packed-tap first layer is a kernel-lab variant");
  agk::launch_conv_fwd(a, (int)mode, cur_stream());
#endif
  launch_check("conv_fwd");
}

// slab: (nsplit, T, Cout, Cin) f32; dbslab: (nsplit, Cout) f32
inline void conv_wgrad_impl(const Tensor& x, const Tensor& dz, const Tensor& slab, const Tensor& dbslab, int64_t K,
                            int64_t S, int64_t Pin, int64_t Po, int64_t cin_real, int variant) {
  check_dev("conv_wgrad_impl", x, dz, slab, dbslab);
  CHECK_DEV(x); CHECK_DEV(dz); CHECK_DEV(slab); CHECK_DEV(dbslab);
  CHECK_BF16(x); CHECK_BF16(dz); CHECK_F32(slab); CHECK_F32(dbslab);
  CHECK_CONTIG(x); CHECK_CONTIG(dz); CHECK_CONTIG(slab); CHECK_CONTIG(dbslab);
  TORCH_CHECK(x.dim() == 4 && dz.dim() == 4 && dz.size(0) == x.size(0), "x, dz: (B, HP, HP, C) with the same B");
  TORCH_CHECK(x.size(2) == x.size(1) && dz.size(2) == dz.size(1), "x, dz: square padded boards");
  TORCH_CHECK(x.numel() < (1ll << 31) && dz.numel() < (1ll << 31), "tensor too large for int32 offsets");
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3);
  const int64_t HPo = dz.size(1), Cout = dz.size(3);
  const int64_t nsplit = slab.size(0);
  TORCH_CHECK(slab.dim() == 4 && slab.size(1) == K * K && slab.size(2) == Cout && slab.size(3) == Cin, "bad slab");
  TORCH_CHECK(dbslab.size(0) == nsplit && dbslab.size(1) == Cout, "bad dbias slab");
  TORCH_CHECK((Cin % 64 == 0 && Cout % 64 == 0) || (Cout == 160 && (Cin == 160 || Cin % 64 == 0)),
              "channels must be multiples of 64, or Cout 160 with Cin 160 / a multiple of 64");
  TORCH_CHECK(HPi == S + 2 * Pin && HPo == S + 2 * Po && Po >= 1 && Pin >= K / 2, "geometry mismatch");
  agk::ConvWgradArgs a{};
  a.variant = variant;
  a.x_elems = x.numel();
  a.dz_elems = dz.numel();
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
  launch_check("conv_wgrad");
}

// fp8 wgrad: x8 e4m3 (B, HPi, HPi, Cin) uint8, dz8 e5m2 (B, HPo, HPo, Cout) uint8, slabs as conv_wgrad_impl
inline void conv_wgrad_fp8_impl(const Tensor& x8, const Tensor& dz8, const Tensor& slab, const Tensor& dbslab,
                                const Tensor& xscale, const Tensor& gscale, const Tensor& gmul, int64_t K, int64_t S,
                                int64_t Pin, int64_t Po, const c10::optional<Tensor>& amax = c10::nullopt,
                                int probe = 0) {
  check_dev("conv_wgrad_fp8", x8, dz8, slab, dbslab, xscale, gscale, gmul, amax);
  TORCH_CHECK(x8.scalar_type() == at::kByte && dz8.scalar_type() == at::kByte, "x8 / dz8: uint8 (e4m3 / e5m2)");
  CHECK_F32(slab); CHECK_F32(dbslab);
  CHECK_CONTIG(x8); CHECK_CONTIG(dz8); CHECK_CONTIG(slab); CHECK_CONTIG(dbslab);
  TORCH_CHECK(xscale.scalar_type() == at::kInt && gscale.scalar_type() == at::kInt && gmul.scalar_type() == at::kFloat &&
                  xscale.numel() >= 1 && gscale.numel() >= 1 && gmul.numel() >= 1,
              "scales: int32 E8M0 exponents, fp32 gradient multiplier");
  TORCH_CHECK(x8.dim() == 4 && dz8.dim() == 4 && dz8.size(0) == x8.size(0), "x8, dz8: (B, HP, HP, C) with the same B");
  TORCH_CHECK(x8.numel() < (1ll << 31) && dz8.numel() < (1ll << 31), "tensor too large for int32 offsets");
  const int64_t B = x8.size(0), HPi = x8.size(1), Cin = x8.size(3);
  const int64_t HPo = dz8.size(1), Cout = dz8.size(3);
  TORCH_CHECK(agk::wgrad_fp8_supported((int)Cout, (int)Cin, (int)K), "conv_wgrad_fp8: 160 -> 160 3x3 layers only");
  TORCH_CHECK(HPi == S + 2 * Pin && HPo == S + 2 * Po && Po >= 1 && Pin >= K / 2, "geometry mismatch");
  const int64_t nsplit = slab.size(0);
  TORCH_CHECK(slab.dim() == 4 && slab.size(1) == K * K && slab.size(2) == Cout && slab.size(3) == Cin, "bad slab");
  TORCH_CHECK(dbslab.size(0) == nsplit && dbslab.size(1) == Cout, "bad dbias slab");
  agk::ConvWgradFp8Args a{};
  a.x8 = x8.data_ptr<uint8_t>();
  a.dz8 = dz8.data_ptr<uint8_t>();
  a.slab = slab.data_ptr<float>();
  a.dbias_slab = dbslab.data_ptr<float>();
  a.xscale = xscale.data_ptr<int>();
  a.gscale = gscale.data_ptr<int>();
  a.gmul = gmul.data_ptr<float>();
  if (amax.has_value()) {
    TORCH_CHECK(amax->scalar_type() == at::kInt && amax->numel() >= agk::kFp8AmaxSlots && amax->is_contiguous(),
                "amax: int32[64]");
    a.amax = reinterpret_cast<unsigned*>(amax->data_ptr<int>());
  }
  a.M = (int)(B * S * S); a.S = (int)S; a.Cin = (int)Cin; a.Cout = (int)Cout; a.K = (int)K; a.T = (int)(K * K);
  a.HPi = (int)HPi; a.offi = (int)(Pin - K / 2); a.HPo = (int)HPo; a.Po = (int)Po;
  const int sp = agk::wgrad_fp8_stage_pixels();
  const int nks = (a.M + sp - 1) / sp;
  a.nsplit = (int)nsplit;
  a.ksteps_per_split = (nks + a.nsplit - 1) / a.nsplit;
  a.probe = probe;
  if (a.M == 0) return;
  agk::launch_conv_wgrad_fp8(a, cur_stream());
  launch_check("conv_wgrad_fp8");
}

// packed fp8 weights (nch, rows, cw): cw = 64, or 32 for 160-channel reductions (32-channel chunks, no
// zero half); nch covers K*K taps of ceil(C / cw) chunks and is a multiple of the chunks per 128-K step
inline int fp8_check_chunks(const Tensor& w, int64_t K, int64_t C, const char* what) {
  const int64_t cw = w.size(2);
  TORCH_CHECK(cw == 64 || (cw == 32 && C == 160), what, ": packed chunk width 64, or 32 for 160 channels");
  const int64_t nch = w.size(0);
  TORCH_CHECK(nch % (128 / cw) == 0 && nch >= K * K * ((C + cw - 1) / cw), what, ": too few packed chunks");
  return (int)cw;
}

inline void conv_fwd_fp8_impl(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& scales,
                              const Tensor& out_scale, const c10::optional<Tensor>& amax,
                              const c10::optional<Tensor>& y_bf16, const c10::optional<Tensor>& y_fp8, int64_t K,
                              int64_t S, int64_t Pin, int64_t Po, int variant,
                              const c10::optional<Tensor>& dgrad_mask = c10::nullopt,
                              const c10::optional<Tensor>& mbits = c10::nullopt,
                              const c10::optional<Tensor>& sr_seed = c10::nullopt) {
  check_dev("conv_fwd_fp8_impl", x, w, bias, scales, out_scale, amax, y_bf16, y_fp8, dgrad_mask, mbits, sr_seed);
  // dgrad_mask given: fp8 dgrad (x = e5m2 gradients, w = transposed e4m3 weights, output masked
  // by dgrad_mask > 0, no bias, e5m2 y_fp8)
  CHECK_DEV(x); CHECK_DEV(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.scalar_type() == at::kByte && w.scalar_type() == at::kByte, "fp8 tensors are stored as uint8");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 3, "x (B,HP,HP,C), w (nch, Cout, cw)");
  TORCH_CHECK(scales.scalar_type() == at::kInt && scales.numel() >= 2 && out_scale.scalar_type() == at::kFloat, "scales");
  if (!dgrad_mask.has_value()) CHECK_F32(bias);
  const int64_t B = x.size(0), HPi = x.size(1), Cin = x.size(3), nch = w.size(0), Cout = w.size(1);
  TORCH_CHECK((Cin % 64 == 0 || Cin == 160) && (Cout % 64 == 0 || Cout == 160), "channel geometry (multiples of 64, or 160)");
  const int cw = fp8_check_chunks(w, K, Cin, "conv_fwd_fp8");
  TORCH_CHECK(Pin >= K / 2 && HPi == S + 2 * Pin, "padding/geometry mismatch");
  TORCH_CHECK(y_bf16.has_value() || y_fp8.has_value(), "need an output");
  agk::ConvFp8Args a{};
  a.variant = variant;
  a.x = x.data_ptr<uint8_t>(); a.w = w.data_ptr<uint8_t>();
  a.bias = dgrad_mask.has_value() ? nullptr : bias.data_ptr<float>();
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
  a.HPi = (int)HPi; a.offi = (int)(Pin - K / 2); a.HPo = (int)HPo; a.Po = (int)Po; a.nch = (int)nch; a.cw = cw;
  if (dgrad_mask.has_value()) {
    CHECK_DEV(*dgrad_mask); CHECK_BF16(*dgrad_mask); CHECK_CONTIG(*dgrad_mask);
    TORCH_CHECK(y_bf16.has_value() && dgrad_mask->sizes() == y_bf16->sizes(), "dgrad: mask must match y_bf16");
    TORCH_CHECK(variant == 0, "dgrad: production kernel only");
    a.dgrad = 1;
    a.mask = bfp(*dgrad_mask);
  }
  if (sr_seed.has_value()) {
    TORCH_CHECK(!dgrad_mask.has_value() && variant == 0 && sr_seed->scalar_type() == at::kInt &&
                    sr_seed->numel() >= 1, "sr_seed: int32 device scalar, production forward only");
    a.sr_seed = sr_seed->data_ptr<int>();
  }
  if (mbits.has_value()) {
    TORCH_CHECK(!dgrad_mask.has_value() && (variant == 0 || variant == 6 || variant == 7 || variant > 100),
                "mbits: the production forward, its lab tilings 6 / 7 or a lab probe");
    CHECK_DEV(*mbits);
    TORCH_CHECK(mbits->scalar_type() == at::kInt && mbits->is_contiguous(), "mbits int32");
    const int64_t words = (Cout == 160 ? 1 : Cout % 192 == 0 ? Cout / 192 : Cout % 128 == 0 ? Cout / 128 : Cout / 64) * 8;
    TORCH_CHECK(mbits->numel() >= B * HPo * HPo * words, "mbits too small: need B*HPo*HPo*words");
    a.mbits_out = reinterpret_cast<uint32_t*>(mbits->data_ptr<int>());
  }
  TORCH_CHECK(B * HPi * HPi * Cin < (1ll << 31), "tensor too large for int32 offsets");
  if (a.M == 0) return;
  agk::launch_conv_fwd_fp8(a, cur_stream());
  launch_check("conv_fwd_fp8");
}

// fp8 dgrad of the fp8-wgrad value step: dz8 e5m2 (B, HP, HP, 160) (MFMA scale scales[0]), w8t the
// transposed flipped e4m3 weights (scales[1]), ReLU' from the forward's bitmask; outputs y_fp8 (e5m2 of
// dx * out_scale[0]) and/or y_bf16; amax (optional) accumulates max |dx|
inline void conv_dgrad_fp8_bits_impl(const Tensor& dz8, const Tensor& w8t, const Tensor& mbits, const Tensor& scales,
                                     const Tensor& out_scale, const c10::optional<Tensor>& amax,
                                     const c10::optional<Tensor>& y_bf16, const c10::optional<Tensor>& y_fp8,
                                     int64_t K, int64_t S) {
  check_dev("conv_dgrad_fp8_bits", dz8, w8t, mbits, scales, out_scale, amax, y_bf16, y_fp8);
  CHECK_DEV(dz8); CHECK_DEV(w8t); CHECK_DEV(mbits); CHECK_CONTIG(dz8); CHECK_CONTIG(w8t); CHECK_CONTIG(mbits);
  TORCH_CHECK(dz8.scalar_type() == at::kByte && w8t.scalar_type() == at::kByte, "fp8 tensors are stored as uint8");
  TORCH_CHECK(dz8.dim() == 4 && w8t.dim() == 3 && dz8.size(3) == 160 && w8t.size(1) == 160,
              "dz8 (B, HP, HP, 160), w8t (nch, 160, cw)");
  const int cw = fp8_check_chunks(w8t, K, 160, "conv_dgrad_fp8_bits");
  TORCH_CHECK(scales.scalar_type() == at::kInt && scales.numel() >= 2 && out_scale.scalar_type() == at::kFloat &&
                  out_scale.numel() >= 1, "scales int32[2], out_scale f32[1]");
  TORCH_CHECK(mbits.scalar_type() == at::kInt, "mbits int32");
  TORCH_CHECK(y_bf16.has_value() || y_fp8.has_value(), "need an output");
  const int64_t B = dz8.size(0), HP = dz8.size(1), nch = w8t.size(0);
  TORCH_CHECK(HP == S + 2 && dz8.size(2) == HP, "geometry (pad 1, 160 channels)");
  TORCH_CHECK(mbits.numel() >= B * HP * HP * 8, "mbits too small: need B*HP*HP*8 words");
  agk::ConvFp8Args a{};
  a.x = dz8.data_ptr<uint8_t>(); a.w = w8t.data_ptr<uint8_t>();
  a.scales = scales.data_ptr<int>(); a.out_scale = out_scale.data_ptr<float>();
  if (y_bf16.has_value()) {
    CHECK_BF16(*y_bf16); CHECK_CONTIG(*y_bf16);
    TORCH_CHECK(y_bf16->sizes() == dz8.sizes(), "y_bf16 shape");
    a.y_bf16 = bfp_mut(*y_bf16);
  }
  if (y_fp8.has_value()) {
    TORCH_CHECK(y_fp8->scalar_type() == at::kByte && y_fp8->is_contiguous() && y_fp8->sizes() == dz8.sizes(),
                "y_fp8 uint8, shape of dz8");
    a.y_fp8 = y_fp8->data_ptr<uint8_t>();
  }
  if (amax.has_value()) {
    TORCH_CHECK(amax->scalar_type() == at::kInt && amax->numel() >= agk::kFp8AmaxSlots, "amax int32[64]");
    a.amax = reinterpret_cast<unsigned*>(amax->data_ptr<int>());
  }
  a.M = (int)(B * S * S); a.S = (int)S; a.Cin = 160; a.Cout = 160; a.K = (int)K;
  a.HPi = (int)HP; a.offi = (int)(1 - K / 2); a.HPo = (int)HP; a.Po = 1; a.nch = (int)nch; a.cw = cw;
  a.dgrad = 1;
  a.mbits_in = reinterpret_cast<const uint32_t*>(mbits.data_ptr<int>());
  TORCH_CHECK(B * HP * HP * 160 < (1ll << 31), "tensor too large for int32 offsets");
  if (a.M == 0) return;
  agk::launch_conv_fwd_fp8(a, cur_stream());
  launch_check("conv_dgrad_fp8_bits");
}

// fp8 dgrad from the bf16 gradient: dz (B, HP, HP, Cg) bf16 padded NHWC is converted to e5m2 in
// the kernel's registers (multiplier *in_scale, MFMA scale scales[0]); w8t: transposed flipped e4m3
// weights (scales[1]); ReLU' from the forward's bitmask; dx bf16; amax accumulates max |dx|
inline void conv_dgrad_fp8_bf16_impl(const Tensor& dz, const Tensor& w8t, const Tensor& mbits, const Tensor& scales,
                                     const Tensor& in_scale, const c10::optional<Tensor>& amax, const Tensor& dx,
                                     int64_t K, int64_t S) {
  check_dev("conv_dgrad_fp8_bf16", dz, w8t, mbits, scales, in_scale, amax, dx);
  CHECK_DEV(dz); CHECK_DEV(w8t); CHECK_DEV(mbits); CHECK_DEV(dx);
  CHECK_BF16(dz); CHECK_CONTIG(dz); CHECK_BF16(dx); CHECK_CONTIG(dx); CHECK_CONTIG(w8t);
  TORCH_CHECK(dz.dim() == 4 && dz.size(2) == dz.size(1) && dz.size(1) == S + 2, "dz (B, S+2, S+2, C) with pad 1");
  TORCH_CHECK(w8t.scalar_type() == at::kByte && w8t.dim() == 3, "w8t (nch, Cout, cw) e4m3");
  TORCH_CHECK(scales.scalar_type() == at::kInt && scales.numel() >= 2, "scales int32[2] (E8M0)");
  TORCH_CHECK(in_scale.scalar_type() == at::kFloat && in_scale.numel() >= 1, "in_scale f32[1]");
  TORCH_CHECK(mbits.scalar_type() == at::kInt && mbits.is_contiguous(), "mbits int32");
  const int64_t B = dz.size(0), HP = dz.size(1), Cg = dz.size(3), nch = w8t.size(0), Cout = w8t.size(1);
  TORCH_CHECK((Cg % 64 == 0 || Cg == 160) && (Cout % 64 == 0 || Cout == 160), "channel geometry (multiples of 64, or 160)");
  const int cw = fp8_check_chunks(w8t, K, Cg, "conv_dgrad_fp8_bf16");
  TORCH_CHECK(dx.size(0) == B && dx.size(1) == HP && dx.size(2) == HP && dx.size(3) == Cout, "dx shape");
  const int64_t words = (Cout == 160 ? 1 : Cout % 192 == 0 ? Cout / 192 : Cout % 128 == 0 ? Cout / 128 : Cout / 64) * 8;
  TORCH_CHECK(mbits.numel() >= B * HP * HP * words, "mbits too small: need B*HPo*HPo*words");
  TORCH_CHECK(dz.numel() < (1ll << 30) && dx.numel() < (1ll << 31), "tensor too large for int32 offsets");
  agk::ConvFp8Args a{};
  a.x = reinterpret_cast<const uint8_t*>(dz.data_ptr());
  a.w = w8t.data_ptr<uint8_t>();
  a.scales = scales.data_ptr<int>();
  a.out_scale = in_scale.data_ptr<float>();  // unused by this form; a valid device pointer
  a.in_scale = in_scale.data_ptr<float>();
  a.y_bf16 = bfp_mut(dx);
  a.mbits_in = reinterpret_cast<const uint32_t*>(mbits.data_ptr<int>());
  if (amax.has_value()) {
    TORCH_CHECK(amax->scalar_type() == at::kInt && amax->numel() >= agk::kFp8AmaxSlots, "amax int32[64]");
    a.amax = reinterpret_cast<unsigned*>(amax->data_ptr<int>());
  }
  a.dgrad_bf16 = 1;
  a.M = (int)(B * S * S); a.S = (int)S; a.Cin = (int)Cg; a.Cout = (int)Cout; a.K = (int)K;
  a.HPi = (int)HP; a.offi = 0; a.HPo = (int)HP; a.Po = 1; a.nch = (int)nch; a.cw = cw;
  if (a.M == 0) return;
  agk::launch_conv_fwd_fp8(a, cur_stream());
  launch_check("conv_dgrad_fp8_bf16");
}

}  // namespace agk_ops
