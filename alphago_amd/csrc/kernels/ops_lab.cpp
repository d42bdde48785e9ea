// Kernel-lab op library (torch.ops.alphago_amd_lab.*), built separately from
// the production library (python -m alphago_amd._build lab): the forward-conv
// tilings of conv_fwd_variants.hip and the other non-default tile codes, the
// wgrad and fp8 variants, and the segment-cycle stamp buffer of the ping-pong
// kernels.  Compiled with -DAGK_KERNEL_LAB and the kernel namespaces renamed
// (agk -> agk_lab) so it loads next to the production library.  Every choice
// is an explicit argument; nothing here is process-global.
#include "ops_conv.h"

namespace {

using namespace agk_ops;

void conv_fwd_lab(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                  const c10::optional<Tensor>& mask, const Tensor& y, int64_t K, int64_t S, int64_t Pin, int64_t Po,
                  int64_t mode, const c10::optional<Tensor>& mbits, int64_t tile,
                  const c10::optional<Tensor>& stamps) {
  check_dev("conv_fwd_lab", x, w, bias, mask, y, mbits, stamps);
  unsigned long long* dbg = nullptr;
  if (stamps.has_value()) {
    CHECK_DEV(*stamps);
    TORCH_CHECK(stamps->scalar_type() == at::kLong && stamps->is_contiguous(), "int64 stamp buffer");
    dbg = reinterpret_cast<unsigned long long*>(stamps->data_ptr<int64_t>());
  }
  conv_fwd_impl(x, w, bias, mask, y, K, S, Pin, Po, mode, mbits, (int)tile, dbg);
}

void conv_wgrad_lab(const Tensor& x, const Tensor& dz, const Tensor& slab, const Tensor& dbslab, int64_t K, int64_t S,
                    int64_t Pin, int64_t Po, int64_t cin_real, int64_t variant) {
  check_dev("conv_wgrad_lab", x, dz, slab, dbslab);
  conv_wgrad_impl(x, dz, slab, dbslab, K, S, Pin, Po, cin_real, (int)variant);
}

// First layer on the packed-tap K loop (conv_fwd_pk_kernel; production until round 4, measured equal):
// only the cin_real real input channels of the 64-channel padded input are multiplied; w in the
// packed-tap layout (pack_weights detects it)
void conv_fwd_pk_lab(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& y, int64_t K, int64_t S,
                     int64_t Pin, int64_t Po, int64_t cin_real, const c10::optional<Tensor>& mbits) {
  check_dev("conv_fwd_pk", x, w, bias, y, mbits);
  TORCH_CHECK(cin_real > 32 && cin_real <= 64, "conv_fwd_pk: 32 < cin_real <= 64");
  conv_fwd_impl(x, w, bias, c10::nullopt, y, K, S, Pin, Po, agk::MODE_BIAS_RELU, mbits, 0, nullptr, -1, c10::nullopt,
                c10::nullopt, c10::nullopt, (int)((cin_real + 7) / 8));
}

void conv_fwd_fp8_lab(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& scales,
                      const Tensor& out_scale, const c10::optional<Tensor>& amax,
                      const c10::optional<Tensor>& y_bf16, const c10::optional<Tensor>& y_fp8, int64_t K, int64_t S,
                      int64_t Pin, int64_t Po, int64_t variant, const c10::optional<Tensor>& mbits) {
  check_dev("conv_fwd_fp8_lab", x, w, bias, scales, out_scale, amax, y_bf16, y_fp8, mbits);
  conv_fwd_fp8_impl(x, w, bias, scales, out_scale, amax, y_bf16, y_fp8, K, S, Pin, Po, (int)variant, c10::nullopt,
                    mbits);
}

void conv_wgrad_fp8_lab(const Tensor& x8, const Tensor& dz8, const Tensor& slab, const Tensor& dbslab,
                        const Tensor& xscale, const Tensor& gscale, const Tensor& gmul, int64_t K, int64_t S,
                        int64_t Pin, int64_t Po, const c10::optional<Tensor>& amax, int64_t probe) {
  conv_wgrad_fp8_impl(x8, dz8, slab, dbslab, xscale, gscale, gmul, K, S, Pin, Po, amax, (int)probe);
}

int64_t wgrad_tap_group_lab(int64_t cout, int64_t cin, int64_t K, int64_t variant) {
  return agk::wgrad_tap_group((int)cout, (int)cin, (int)K, (int)variant);
}

std::vector<int64_t> wgrad_plan_lab(int64_t cout, int64_t cin, int64_t cin_real, int64_t K, int64_t variant) {
  int o[4];
  agk::wgrad_plan((int)cout, (int)cin, (int)(cin_real > 0 && cin_real < cin ? cin_real : cin), (int)K, (int)variant, o);
  return {o[0], o[1], o[2], o[3]};
}

void bf8_convert_probe(const Tensor& x, const Tensor& y, double scale, int64_t mode) {
  check_dev("bf8_convert_probe", x, y);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kByte && x.numel() == y.numel() &&
                  x.numel() % 2 == 0 && x.is_contiguous() && y.is_contiguous(), "bf16 -> uint8, even size");
  agk::launch_bf8_convert_probe(reinterpret_cast<const __bf16*>(x.data_ptr()), y.data_ptr<uint8_t>(), x.numel(),
                                (float)scale, (int)mode, cur_stream());
  launch_check("bf8_convert_probe");
}

void wino_fwd(const Tensor& x, const Tensor& u, const c10::optional<Tensor>& bias, const Tensor& y, int64_t S) {
  check_dev("wino_fwd", x, u, bias, y);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && u.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16,
              "wino_fwd: bf16 x, u, y");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(1) == S + 2 && x.size(2) == S + 2 && y.size(1) == S + 2 &&
                  y.size(2) == S + 2 && y.size(0) == x.size(0) && x.is_contiguous() && y.is_contiguous(),
              "wino_fwd: padded NHWC x, y with one-pixel borders");
  const int Cin = (int)x.size(3), Cout = (int)y.size(3);
  TORCH_CHECK(u.is_contiguous() && u.numel() == 16LL * Cin * Cout, "wino_fwd: packed weights 16 x Cin x Cout");
  TORCH_CHECK(x.numel() < (1LL << 31) && y.numel() < (1LL << 31), "wino_fwd: int32 offsets");
  if (bias.has_value())
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "wino_fwd: fp32 bias");
  agk::WinoArgs a{};
  a.x = reinterpret_cast<const __bf16*>(x.data_ptr());
  a.u = reinterpret_cast<const __bf16*>(u.data_ptr());
  a.bias = bias.has_value() ? bias->data_ptr<float>() : nullptr;
  a.y = reinterpret_cast<__bf16*>(y.data_ptr());
  a.S = (int)S;
  a.Cin = Cin;
  a.Cout = Cout;
  a.TS = (int)((S + 1) / 2);
  a.ntiles = (int)(x.size(0) * a.TS * a.TS);
  agk::launch_wino_fwd(a, cur_stream());
  launch_check("wino_fwd");
}

void tr8_probe(const Tensor& lds_init, const Tensor& addr, const Tensor& out) {
  check_dev("tr8_probe", lds_init, addr, out);
  TORCH_CHECK(lds_init.scalar_type() == at::kByte && lds_init.numel() <= 4096 && addr.scalar_type() == at::kInt &&
                  addr.numel() == 64 && out.scalar_type() == at::kLong && out.numel() == 64,
              "tr8_probe: <= 4096 LDS bytes, 64 int32 addresses, 64 int64 outputs");
  auto ac = addr.cpu();
  for (int i = 0; i < 64; ++i)
    TORCH_CHECK(ac[i].item<int>() >= 0 && ac[i].item<int>() + 8 <= 4096 && ac[i].item<int>() % 8 == 0,
                "tr8_probe: 8-byte aligned addresses inside the 4 KB LDS block");
  agk::launch_tr8_probe(lds_init.data_ptr<uint8_t>(), (int)lds_init.numel(), addr.data_ptr<int>(),
                        reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), cur_stream());
  launch_check("tr8_probe");
}

// GPU ladder reader (ladder.hip, kernel lab: 16x slower than the host reader, profiles/r2_gpu_ladders.md).
// Ladder planes from the compact board encoding: out (B, S*S) uint8, bit 0 =
// ladder capture, bit 1 = ladder escape (the encoder's CPU ladder bits).
void ladder_planes(const Tensor& board, const Tensor& meta, const Tensor& out, int64_t S, int64_t budget) {
  check_dev("ladder_planes", board, meta, out);
  CHECK_DEV(board); CHECK_DEV(meta); CHECK_DEV(out);
  TORCH_CHECK(board.scalar_type() == at::kChar && board.dim() == 2 && board.size(1) == S * S && board.is_contiguous(),
              "board int8 (B, S*S)");
  TORCH_CHECK(meta.scalar_type() == at::kInt && meta.size(0) == board.size(0) && meta.is_contiguous(), "meta int32 (B, 2)");
  TORCH_CHECK(out.scalar_type() == at::kByte && out.sizes() == board.sizes() && out.is_contiguous(), "out uint8 (B, S*S)");
  TORCH_CHECK(S >= 2 && S <= 19, "board size 2..19");
  const int64_t B = board.size(0);
  if (B == 0) return;
  auto i32 = board.options().dtype(at::kInt);
  Tensor boards = at::empty({B, (int64_t)sizeof(agk::LadderBoard)}, board.options().dtype(at::kByte));
  Tensor counts = at::empty({B + 1}, i32);  // [B] = search task counter
  agk::LadderArgs a{};
  a.board = board.data_ptr<int8_t>();
  a.meta = meta.data_ptr<int32_t>();
  a.boards = reinterpret_cast<agk::LadderBoard*>(boards.data_ptr<uint8_t>());
  a.counts = counts.data_ptr<int32_t>();
  a.out = out.data_ptr<uint8_t>();
  a.B = (int)B;
  a.S = (int)S;
  TORCH_CHECK(budget > 0, "ladder budget must be positive");
  a.budget = (int)budget;
  a.counter = a.counts + B;
  out.zero_();
  counts.zero_();
  agk::launch_ladder_prep(a, cur_stream());
  launch_check("ladder_prep");
  Tensor c = counts.narrow(0, 0, B);
  Tensor offsets = (at::cumsum(c, 0, at::kInt) - c).contiguous();
  a.offsets = offsets.data_ptr<int32_t>();
  const int threads = (int)std::min<int64_t>(16384, B * 32);
  Tensor frames = at::empty({(int64_t)threads * (int64_t)agk::ladder_frame_bytes()}, board.options().dtype(at::kByte));
  a.frames = frames.data_ptr<uint8_t>();
  agk::launch_ladder_search(a, threads, cur_stream());
  launch_check("ladder_search");
}

}  // namespace

TORCH_LIBRARY(alphago_amd_lab, m) {
  m.def(
      "conv_fwd(Tensor x, Tensor w, Tensor? bias, Tensor? mask, Tensor(a!) y, int K, int S, int Pin, int Po, int mode, "
      "Tensor(b!)? mbits, int tile, Tensor(c!)? stamps=None) -> ()");
  m.def("conv_wgrad(Tensor x, Tensor dz, Tensor(a!) slab, Tensor(b!) dbslab, int K, int S, int Pin, int Po, "
        "int cin_real, int variant) -> ()");
  m.def(
      "conv_fwd_fp8(Tensor x, Tensor w, Tensor bias, Tensor scales, Tensor out_scale, Tensor(a!)? amax, "
      "Tensor(b!)? y_bf16, Tensor(c!)? y_fp8, int K, int S, int Pin, int Po, int variant, Tensor(d!)? mbits=None) -> ()");
  m.def(
      "conv_wgrad_fp8(Tensor x8, Tensor dz8, Tensor(a!) slab, Tensor(b!) dbslab, Tensor xscale, Tensor gscale, "
      "Tensor gmul, int K, int S, int Pin, int Po, Tensor(c!)? amax, int probe) -> ()");
  m.def(
      "conv_fwd_pk(Tensor x, Tensor w, Tensor bias, Tensor(a!) y, int K, int S, int Pin, int Po, int cin_real, "
      "Tensor(b!)? mbits=None) -> ()");
  m.def("wgrad_tap_group(int cout, int cin, int K, int variant) -> int", &wgrad_tap_group_lab);
  m.def("wgrad_plan(int cout, int cin, int cin_real, int K, int variant) -> int[]", &wgrad_plan_lab);
  m.def("bf8_convert_probe(Tensor x, Tensor(a!) y, float scale, int mode) -> ()");
  m.def("wino_fwd(Tensor x, Tensor u, Tensor? bias, Tensor(a!) y, int S) -> ()");
  m.def("tr8_probe(Tensor lds_init, Tensor addr, Tensor(a!) out) -> ()");
  m.def("ladder_planes(Tensor board, Tensor meta, Tensor(a!) out, int S, int budget=4096) -> ()");
}

TORCH_LIBRARY_IMPL(alphago_amd_lab, CUDA, m) {
  m.impl("bf8_convert_probe", &bf8_convert_probe);
  m.impl("wino_fwd", &wino_fwd);
  m.impl("tr8_probe", &tr8_probe);
  m.impl("conv_fwd", &conv_fwd_lab);
  m.impl("conv_wgrad", &conv_wgrad_lab);
  m.impl("conv_fwd_fp8", &conv_fwd_fp8_lab);
  m.impl("conv_wgrad_fp8", &conv_wgrad_fp8_lab);
  m.impl("conv_fwd_pk", &conv_fwd_pk_lab);
  m.impl("ladder_planes", &ladder_planes);
}
