// Kernel argument structs and host launchers (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "common.h"

namespace agk {

enum { MODE_BIAS_RELU = 0, MODE_MASK = 1, MODE_NONE = 2, MODE_MASKBITS = 3 };

struct ConvFwdArgs {
  const __bf16* x;     // padded NHWC input
  const __bf16* w;     // packed [T][Cout][Cin]
  const float* bias;   // [Cout]           (MODE_BIAS_RELU)
  const __bf16* mask;  // layout of y      (MODE_MASK: keep where mask > 0)
  __bf16* y;           // padded NHWC output (interior written, borders untouched)
  uint32_t* mbits_out;       // MODE_BIAS_RELU: optional ReLU'(y) bitmask, (Cout/BN)*8 words per padded pixel
  const uint32_t* mbits_in;  // MODE_MASKBITS: the bitmask written by the layer's forward
  int M, S, Cin, Cout, K;
  int HPi, offi;       // input padded side, (input pad - K/2)
  int HPo, Po;         // output padded side and pad
  FastDiv divSS, divS; // filled by the launcher
  int tile;            // 0 = automatic; 128/256/384 fixed tiles; other codes: kernel-lab build only
  unsigned long long* dbg;  // kernel lab: diagnostic segment-cycle stamps, else null
  long long x_elems, w_elems, y_elems;  // tensor extents (debug-build bounds checks)
  // MODE_MASKBITS (dgrad) only, optional: an e5m2 copy of the output (y * *bf8_scale) for the fp8
  // wgrad, and max |y| folded into 64 amax slots (the next step's delayed gradient scale)
  uint8_t* y_bf8;
  const float* bf8_scale;
  unsigned* bf8_amax;
  // split-K (tile code 38, small batches): fp32 partial sums [sk_nsplit][M][Cout], finished by
  // conv_splitk_finish_kernel (bias + ReLU + bitmask, or the bitmask of dgrad)
  float* sk_ws;
  int sk_nsplit;
};

struct ConvWgradArgs {
  const __bf16* x;     // layer input (padded NHWC, Cin)
  const __bf16* dz;    // gradient at the layer's pre-activation output (padded NHWC, Cout, zero borders)
  float* slab;         // [nsplit][T][Cout][Cin]
  float* dbias_slab;   // [nsplit][Cout]
  int M, S, Cin, Cout, K, T;
  int HPi, offi, HPo, Po;
  int ksteps_per_split, nsplit;
  int cin_real;        // real input channels (<= Cin); the zero padding above it is skipped when possible
  FastDiv divSS, divS; // filled by the launcher
  int variant;         // 0 = production per-tap kernel; 5 = one-kernel-row wgrad (conv_wgrad_row.hip);
                       // 1-4 kernel-lab build only
  long long x_elems, dz_elems;  // tensor extents (debug-build bounds checks)
  int xcd_group;       // filled by the launcher: 1 = the kernel-row workgroups of a split share an XCD
  // split-free plan (kWgradDirect, nsplit 1): the tile is written straight into the OIHW fp32 gradient
  // grad_w[n][c][t] = beta * grad_w + scale * sum (n < cout_real, c < cin_real) and the bias into
  // grad_b -- no slab, no reduce launch.  grad_w == nullptr: the split slab as above.
  float* grad_w;
  float* grad_b;
  float scale, beta;
  int cout_real;
};

// fp8 wgrad (conv_wgrad_fp8.hip): e5m2 dZ x e4m3 X on the block-scaled MFMA, same slab as the bf16 wgrad
struct ConvWgradFp8Args {
  const uint8_t* x8;   // e4m3 layer input (padded NHWC, Cin), quantised with multiplier 2^ex
  const uint8_t* dz8;  // e5m2 output gradient (padded NHWC, Cout, zero borders), multiplier 2^eg
  float* slab;         // [nsplit][T][Cout][Cin]
  float* dbias_slab;   // [nsplit][Cout]
  const int* xscale;   // device E8M0 exponent 127 - ex
  const int* gscale;   // device E8M0 exponent 127 - eg
  const float* gmul;   // device 2^eg (the bias sums undo it)
  unsigned* amax;      // optional: max |dZ| (float bits, 64 slots) from the tap-0 workgroups' e5m2 bytes
  int M, S, Cin, Cout, K, T;
  int HPi, offi, HPo, Po;
  int ksteps_per_split, nsplit;  // in 128-pixel steps
  FastDiv divSS, divS;           // filled by the launcher
  int probe;                     // kernel-lab timing probe (0 = production)
};
int wgrad_fp8_supported(int Cout, int Cin, int K);
int wgrad_fp8_stage_pixels();
void launch_conv_wgrad_fp8(const ConvWgradFp8Args& a, hipStream_t st);

struct WgradReduceArgs {
  const float* slab;
  const float* dbias_slab;
  float* grad_w;  // OIHW fp32 [Cout_real][Cin_real][K][K]
  float* grad_b;  // [Cout_real] or null
  int T, Cout, Cin, Cout_real, Cin_real, nsplit;
  float scale, beta;  // grad = beta*grad + scale*sum
};
constexpr int kMaxReduceJobs = 16;
struct WgradReduceMultiArgs {
  WgradReduceArgs job[kMaxReduceJobs];
  int first[kMaxReduceJobs], nblk[kMaxReduceJobs];
  int n;
};

struct PolicyHeadArgs {
  const __bf16* y;     // padded NHWC (HP = S+2, P = 1, C)
  const float* w;      // [C_real]
  const float* b;      // [1]
  const int* target;   // [B] flat move index or -1 (no loss)
  const uint8_t* legal;  // [B][S*S] or null (inference renormalisation)
  const float* weight;   // [B] per-board gradient weight (REINFORCE reward) or null
  __bf16* dz;          // padded NHWC grad (training) or null
  float* loss;         // [B]
  float* correct;      // [B]
  float* dhead;        // [B][C_real + 1] per-board partials of dW_head, db_head
  float* probs;        // [B][S*S] or null
  uint8_t* dz8;        // head_backward only: dY as e5m2 (dz8 = e5m2(bf16(dY) * dz8_scale[0])) instead of
  const float* dz8_scale;  // the bf16 dz, for an fp8 trunk backward; max |bf16(dY)| into dz8_amax
  unsigned* dz8_amax;  // [kFp8AmaxSlots] float bits (the quantize_bf8 contract)
  int B, S, C, C_real;
  float grad_scale;    // d(mean loss)/d(logit) scale = 1/global_batch
  float inv_temp;
  int loss_kind;       // 0 = categorical CE (SL / REINFORCE), 1 = reference RL binary CE on the softmax
};

struct ValueOutArgs {
  const float* h;       // [B][D] dense-1 output
  const float* w2;      // [D]
  const float* b2;      // [1]
  const float* target;  // [B] in [-1, 1] or null (inference)
  const float* weight;  // [B] or null
  float* v;             // [B]
  float* loss;          // [B]
  float* correct;       // [B]
  float* dh;            // [B][D]
  float* dout;          // [B][D + 1] per-board partials of [dw2 | db2]
  int B, D;
  float grad_scale;
};

struct PackInputArgs {
  const uint8_t* planes;  // [B][Creal][S][S], or [npool][Creal][S][S] with rows
  const int64_t* rows;    // [B] pool row of each board or null (board b = planes[b]); rows outside
                          // [0, npool) pack an all-zero board (no out-of-bounds read)
  int64_t npool;
  const int* sym;         // [B] in 0..7 or null (identity)
  const int* target;      // [B] or null
  int* target_out;        // [B] or null
  __bf16* out;            // padded NHWC [B][S+2P][S+2P][Cp]
  uint8_t* out8;          // the same planes as e4m3 (scale 1: exact for 0/1, saturating at 448) or null
  int B, S, Creal, Cp, P;
};

constexpr int kMaxPackLayers = 24;
struct PackLayer {
  const float* w;  // OIHW fp32 [Cout_real][Cin_real][K][K]
  __bf16* wf;      // [T][Cout_p][Cin_p]; pk_cpt > 0: [ceil(T * pk_cpt / 8)][Cout_p][64] (conv_fwd_pk_kernel)
  __bf16* wd;      // [T][Cin_p][Cout_p] flipped (dgrad) or null
  int Cout_real, Cin_real, Cout_p, Cin_p, K;
  int pk_cpt;      // packed-tap first layer: 8-channel chunks per tap, else 0
};
struct PackWeightsArgs {
  PackLayer layers[kMaxPackLayers];
  int nlayers;
};

constexpr int kFzMaxFeatures = 16;
constexpr int kFzMaxChannels = 64;
struct FeaturizeArgs {
  const int8_t* board;    // [B][S*S] in {-1,0,1}
  const uint8_t* ages;    // [B][S*S] turns_since plane or 255
  const int* meta;        // [B][2] {ko or -1, player to move}
  const uint8_t* ladder;  // [B][S*S] bit0 capture, bit1 escape; or null
  uint8_t* planes;        // [B][nplanes][S][S] or null
  __bf16* nhwc;           // [B][S+2P][S+2P][Cp] or null
  uint8_t* sensible;      // [B][S*S] or null
  uint8_t* legal;         // [B][S*S] or null
  int* overflow;          // [B] or null (set to 1 when the eye DFS overflowed)
  int B, S, P, Cp, nf, nplanes, need_eye;
  int fids[kFzMaxFeatures];
  int fplanes[kFzMaxFeatures];
  uint8_t chan_feat[kFzMaxChannels];
  uint8_t chan_plane[kFzMaxChannels];
};

constexpr int kFp8AmaxSlots = 64;  // per-layer amax accumulators (spread atomics)

struct ConvFp8Args {
  const uint8_t* x;         // padded NHWC e4m3 [B][HPi][HPi][Cin], Cin % 64 == 0
  const uint8_t* w;         // e4m3 [nch][Cout][64], chunk q = tap * (Cin/64) + c, nch even (zero tail)
  const float* bias;        // [Cout]
  const int* scales;        // [2] E8M0 exponents for the MFMA: {activations, weights} (127 = 2^0)
  const float* out_scale;   // [1] multiplier applied before the e4m3 output conversion
  __bf16* y_bf16;           // optional padded NHWC bf16 output
  uint8_t* y_fp8;           // optional padded NHWC e4m3 output
  unsigned* amax;           // optional running max of the ReLU output (float bits), kFp8AmaxSlots slots
  int M, S, Cin, Cout, K;
  int HPi, offi, HPo, Po;
  int nch;                  // packed chunks (cw channels each; a K-step holds 128 / cw chunks)
  int cw;                   // chunk width: 64, or 32 for 160-channel operands packed in 32-channel chunks
  FastDiv divSS, divS;      // filled by the launcher
  FastDiv divCC, divK;      // chunks per tap, kernel width (launcher)
  int variant;              // 0 = production (pixel operand from L2, 48 px/wave); lab: 1, 3, 4 other tilings,
                            // 5 = LDS-staged operands
  // dgrad mode (production kernel only): x holds e5m2 gradients, w the transposed/flipped e4m3
  // weights; the epilogue masks by mask > 0 (the forward's bf16 activation), takes no bias,
  // tracks max |dx| and writes bf16 and/or e5m2 (out_scale) outputs
  int dgrad;
  const __bf16* mask;
  // forward, production kernel: optional ReLU'(y) bitmask in conv_fwd_kernel's layout
  // (ConvEpilogue: (Cout/BN)*8 words per padded pixel) so the bf16 dgrad can run MODE_MASKBITS
  uint32_t* mbits_out;
  // dgrad with a bf16 gradient operand (dgrad_bf16): x is the bf16 dZ (padded NHWC, Cin channels),
  // converted to e5m2 in registers as it is loaded (multiplier *in_scale); the ReLU' mask comes from
  // the forward's bitmask (mbits_in, conv_fwd_kernel's layout); bf16 output only
  int dgrad_bf16;
  const float* in_scale;
  const uint32_t* mbits_in;
  // forward, optional: stochastic rounding of the e4m3 output (v_cvt_sr_fp8_f32), random bits hashed
  // from (pixel, channel, *sr_seed); the trainer advances the device seed every step
  const int* sr_seed;
};

// Kernel choices are explicit launch arguments (ConvFwdArgs::tile,
// ConvWgradArgs::variant, ConvFp8Args::variant): no process-global state.
void launch_conv_fwd(const ConvFwdArgs& a, int mode, hipStream_t st);
// packed-tap first-layer forward (bias + ReLU, optional bitmask): cpt 8-channel chunks per tap
void launch_conv_fwd_pk(const ConvFwdArgs& a, int cpt, hipStream_t st);
void launch_conv_wgrad(const ConvWgradArgs& a, hipStream_t st);
// split-free wgrad (kWgradDirect): a.grad_w / grad_b / scale / beta / cout_real set; ksub 4 / 8 / 12
void launch_conv_wgrad_direct(const ConvWgradArgs& a, int ksub, hipStream_t st);
bool wgrad_direct_supported(int Cout, int Cin, int cin_real, int K);
// weight-stationary small-batch conv (conv_ws.hip, tile code 40): modes 0 / 2 / 3; target_wgs <= 0: 256
void launch_conv_ws(const ConvFwdArgs& a, int mode, int target_wgs, hipStream_t st, int probe = 0);
// conv_wgrad's small-batch plan (64 x 64 tap-merged tiles; ops.wgrad_config picks it)
constexpr int kWgradSmall = 14;
// split-free small-batch plan: 32 x 48 (or 32 x 32) per-tap tiles, each workgroup owns the whole pixel
// range and writes the OIHW gradient itself (ConvWgradArgs::grad_w; conv_wgrad_direct)
constexpr int kWgradDirect = 15;
// weight-stationary order of standard (tap, Cout, Cin) bf16 packs (conv_ws.hip; tile 40 reads it)
struct WsPackJob {
  const __bf16* src;
  __bf16* dst;
  int Cout, Cin, K;
  int nblk, kw, bn, nwv, ws, slices;  // filled by launch_ws_pack
};
constexpr int kMaxWsPackJobs = 32;
struct WsPackArgs {
  WsPackJob job[kMaxWsPackJobs];
  int n;
};
void launch_ws_pack(const std::vector<WsPackJob>& jobs, hipStream_t st);
bool conv_ws_supported(int Cout, int Cin, int K);
int wgrad_stage_pixels();  // pixels per wgrad pipeline stage (units of ksteps_per_split)
int wgrad_tap_group(int Cout, int Cin, int K, int variant);  // taps per wgrad workgroup (tap-merged 64-wide c tiles)
// one-kernel-row wgrad (conv_wgrad_row.hip): geometry code (0 = not applicable), grid per split, launch
int wgrad_row_code(int Cout, int Cin, int cin_real, int K);
int wgrad_row_wgs_per_split(int code, int Cout, int Cin, int cin_real, int K);
void wgrad_row_launch(int code, const ConvWgradArgs& a, hipStream_t st);
// launch plan of the wgrad that launch_conv_wgrad runs for this variant:
// {taps per workgroup, workgroups per split, resident workgroups per CU}
void wgrad_plan(int Cout, int Cin, int cin_real, int K, int variant, int out[4]);
// a launch the runtime must reject (block of 2048 threads): tests the error path
void launch_invalid_config_probe(hipStream_t st);
#ifdef AGK_DEBUG
// debug build: waits for the stream, returns and clears the bounds-violation
// code recorded by the conv kernels (0 = none)
unsigned debug_error_fetch_and_clear(hipStream_t st);
#endif
void launch_wgrad_reduce(const WgradReduceArgs& a, hipStream_t st);
void launch_wgrad_reduce_multi(const std::vector<WgradReduceArgs>& jobs, hipStream_t st);
void launch_policy_head(const PolicyHeadArgs& a, bool train, hipStream_t st);
void launch_head_logits(const PolicyHeadArgs& a, hipStream_t st);
void launch_head_backward(const PolicyHeadArgs& a, const float* dlogits, hipStream_t st);
void launch_value_out(const ValueOutArgs& a, hipStream_t st);

// fused move sampling (sample.hip): out[b] = a draw from probs[b]**beta, -1 where has[b] == 0
struct SampleArgs {
  const float* probs;    // [B][NP]
  const uint8_t* has;    // [B] any sensible move, or null: then
  const uint8_t* legal;  // [B][NP] sensible-move mask, "has" = any nonzero entry of the row
  int64_t* out;          // [B]
  int B, NP;
  float beta;
  uint64_t seed;
};
void launch_sample_moves(const SampleArgs& a, hipStream_t st);
void launch_head_grad_sums(const float* dhead, int B, int N, const float* loss, const float* correct, float* grad,
                           float* sums, hipStream_t st);
void launch_pack_input(const PackInputArgs& a, hipStream_t st);
void launch_pack_weights(const PackWeightsArgs& a, hipStream_t st);
void launch_featurize(const FeaturizeArgs& a, hipStream_t st);
void launch_conv_fwd_fp8(const ConvFp8Args& a, hipStream_t st);
void launch_pack_weights_fp8(const float* w, uint8_t* out, int Cout_real, int Cin_real, int K, int Cout_p, int Cin_p,
                             int nch, float scale, const float* scale_dev, int transposed, int cw, hipStream_t st);
struct Fp8WeightScalesArgs {
  const float* w[kMaxPackLayers];
  int n[kMaxPackLayers];
  float* wscale;  // [L]
  int* scales8;   // [L][2]
};
void launch_fp8_weight_scales(const Fp8WeightScalesArgs& a, int L, hipStream_t st);
// every fp8 weight pack of a repack (forward and transposed dgrad packs of all layers) in one launch
constexpr int kMaxFp8PackJobs = 48;
struct Fp8PackJob {
  const float* w;         // OIHW fp32
  uint8_t* out;           // [nch][rows_p][64] e4m3
  const float* scale;     // device scale (one float)
  int Cout_real, Cin_real, K, Cout_p, Cin_p, nch, transposed;
  int cw;                 // chunk width (channels per chunk): 64, or 32 for the 160-channel value layers
};
struct Fp8PackArgs {
  Fp8PackJob jobs[kMaxFp8PackJobs];
  int n;
};
void launch_pack_weights_fp8_multi(const Fp8PackArgs& a, hipStream_t st);
void launch_fp8_act_scales(unsigned* amax, int* scales8, float* osc, int L, int margin, int max_drop, hipStream_t st);
void launch_fp8_grad_scales(unsigned* amax, int* gscales8, float* gosc, int L, int margin, hipStream_t st);
void launch_quantize_bf8_dev(const __bf16* x, uint8_t* y, long n, const float* scale, unsigned* amax, hipStream_t st,
                             bool e4m3 = false);
void launch_quantize_fp8(const __bf16* x, uint8_t* y, long n, float scale, hipStream_t st);
#ifdef AGK_KERNEL_LAB
void launch_bf8_convert_probe(const __bf16* x, uint8_t* y, long n, float scale, int mode, hipStream_t st);
#endif
void launch_sgd(float* p, const float* g, int64_t n, float lr, float gscale, hipStream_t st);

// fused SGD + bf16 weight packs (pack.hip sgd_pack_kernel)
constexpr int kSgdPackMaxTaps = 25;
constexpr int kSgdPackMaxRanges = 64;
struct SgdPackLayer {
  int64_t off;     // OIHW fp32 weights at p + off (and their gradient at g + off)
  __bf16* wf;      // forward pack [T][Cout_p][Cin_p], or the packed-tap layout when pk_cpt > 0
  __bf16* wd;      // transposed dgrad pack [T][Cin_p][Cout_p] (taps flipped) or null
  int Cout_real, Cin_real, Cout_p, Cin_p, K, pk_cpt;
};
struct SgdPackArgs {
  float* p;
  const float* g;
  float lr, gscale;
  double* sched;   // device Keras schedule {lr0, decay, iterations, lr} (advanced first) or null: lr
  SgdPackLayer layers[kMaxPackLayers];
  int nlayers;
  int64_t range_off[kSgdPackMaxRanges];
  int range_len[kSgdPackMaxRanges];
  int nranges;
  // optimizer (Keras 1.0 SGD / Adam semantics): 0 = SGD (p -= lr g), 1 = SGD with momentum
  // (v = mom v - lr g; p += v, or p += mom v - lr g with nesterov), 2 = Adam (m1, m2 = first and second
  // moments; the bias-corrected step lr_t comes from the device schedule or the host).  m1 / m2 are flat
  // fp32 buffers parallel to p.
  int opt;
  float* m1;
  float* m2;
  float mom, b1, b2, eps;
  int nesterov;
};
void launch_sgd_pack(const SgdPackArgs& a, hipStream_t st);
// RCCL all-reduce stand-in (comm_proxy.hip): channels workgroups copy n floats and hold their CUs wire_us
void launch_comm_proxy(const float* src, float* dst, long n, int channels, double wire_us, hipStream_t st);

// fp32 dense layer GEMM (value head): C[M][N] = beta*C + A.B (+ bias[n]);
// A is [M][K] (lda) or, transposed, [K][M]; B is [K][N] (ldb) or [N][K]
struct DenseArgs {
  const float* A;
  const float* B;
  const float* bias;  // [N] or null
  float* C;
  int M, N, K, lda, ldb, ldc;
  float beta;
  int splits;  // split-K factor (dense_splits); > 1 needs ws of splits*M*N floats
  int kchunk;  // set by the launcher
  float* ws;
};
int dense_splits(int M, int N, int K);

// GPU ladder planes (ladder.hip; search code ../engine/ladder_bb.h)
struct LadderBoard {
  uint64_t black[6], white[6], cand[6];
  int ko, me;
};
struct LadderArgs {
  const int8_t* board;     // [B][S*S] +1 black, -1 white, 0 empty
  const int32_t* meta;     // [B][2] {ko point or -1, player to move}
  LadderBoard* boards;     // [B] prep output
  int32_t* counts;         // [B] candidate points per board
  const int32_t* offsets;  // [B] exclusive prefix sum of counts
  int32_t* counter;        // zeroed task counter of the search kernel
  void* frames;            // search threads x ladder_frame_bytes() (frame stacks)
  int budget;              // node visits per capture / escape read (lb::kLadderVisits)
  uint8_t* out;            // [B][S*S] zeroed; bit 0 = ladder capture, bit 1 = ladder escape
  int B, S;
};
size_t ladder_frame_bytes();
void launch_ladder_prep(const LadderArgs& a, hipStream_t st);
void launch_ladder_search(const LadderArgs& a, int threads, hipStream_t st);
void launch_dense_f32(const DenseArgs& a, bool transA, bool transB, hipStream_t st);
// device-side schedule (graph-capturable): sched = {lr0, decay, iterations, lr_current} f64
void launch_sgd_sched(float* p, const float* g, int64_t n, double* sched, float gscale, hipStream_t st);

// ---- kernel lab: Winograd F(2x2, 3x3) forward (winograd.hip), bias + ReLU, padded NHWC bf16
struct WinoArgs {
  const __bf16* x;    // padded NHWC input (HP = S + 2), Cin channels
  const __bf16* u;    // transformed weights, packed [16 xi][Cin/32][Cout/16][64 lanes][8]
  const float* bias;  // [Cout] or null
  __bf16* y;          // padded NHWC output (HP = S + 2), Cout channels
  int S, Cin, Cout, ntiles, TS;  // TS = (S + 1) / 2 tiles per row; ntiles = B * TS * TS
};
void launch_wino_fwd(const WinoArgs& a, hipStream_t st);

// kernel lab: ds_read_b64_tr_b8 lane-mapping probe (lab_probes.hip)
void launch_tr8_probe(const uint8_t* lds_init, int nbytes, const int* addr, unsigned long long* out, hipStream_t st);

}  // namespace agk
