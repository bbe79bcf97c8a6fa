// ghost_amd — host-side description of one implicit-GEMM convolution launch.
//
// One kernel template covers every contraction on the AEI_Net path:
//   * Conv2d 4x4/s2/p1 + BN(eval) + LeakyReLU   (AEI_Net.py:19-24)
//   * ConvTranspose2d 4x4/s2/p1 + BN + LReLU    (AEI_Net.py:27-41) as four 2x2 sub-pixel phases
//   * Conv2d 3x3/p1 (+ residual, + tanh)        (AADLayer.py:64,71,79; AEI_Net.py:139)
//   * 1x1 convs on z_attr with the fused AADLayer epilogue (AADLayer.py:20-38)
//   * the z_id GEMMs (generator.up1 ConvT k2 on a 1x1 input, every fc1/fc2)
// GEMM view: M = output pixels (NHWC rows), N = output channels, K = taps x Cin.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ghost {

enum ConvKind { CONV_FWD = 0, CONV_T4S2 = 1 };
enum Epilogue { EPI_STD = 0, EPI_AAD = 1 };

struct ConvDesc {
  int ti = 0, to = 0;               // GhostDType of input/weights and of the output
  // input activation, NHWC with channel stride ldx (pointer already at the channel offset)
  const void* x = nullptr;
  int B = 0, Hi = 0, Wi = 0, Cin = 0, ldx = 0;
  // packed weights: [npar][Npad][Kpad], K index = (ty*ntx + tx)*Cin + c
  const void* w = nullptr;
  int N = 0, Npad = 0, Kpad = 0;
  int kind = CONV_FWD;
  int kh = 1, kw = 1, stride = 1, pad = 0;
  // output NHWC (channel stride ldy, pointer at the channel offset); spatial size derived
  void* y = nullptr;
  int ldy = 0;
  // standard epilogue: v = acc*scale[n] + shift[n]; v = v>0 ? v : v*slope; v += res; tanh
  // (res_first moves the residual before the activation)
  const float* scale = nullptr;
  const float* shift = nullptr;
  float slope = 1.0f;
  const void* res = nullptr;         // same dtype as the output
  int ldres = 0;
  int tanh_out = 0;
  int res_first = 0;                 // 1: v = act(acc*scale + shift + res)  (ResNet Bottleneck, resnet.py:74-76)
  const float* prelu = nullptr;      // per-channel negative slope (nn.PReLU), overrides `slope`
  // optional second output y2 = v*scale2 + shift2 (the BatchNorm that opens the next IBasicBlock)
  void* y2 = nullptr;
  int ldy2 = 0;
  const float* scale2 = nullptr;
  const float* shift2 = nullptr;
  uint8_t* u8 = nullptr;             // optional BGR uint8 NHWC copy of a 3-channel output (faceshifter_run.py:20-21)
  // AAD epilogue (epi == EPI_AAD): output channel c pairs weight columns (gamma, beta)
  int epi = EPI_STD;
  const void* hin = nullptr;  int ldh = 0;   // h_in, same dtype as output
  const float* stat = nullptr;               // [B][C][2] = mean, rstd of h_in
  const float* idgb = nullptr;  int id_ld = 0;  // per-sample gamma_id (at c) / beta_id (at C + c)
  const float* mask = nullptr;               // [B*H*W] sigmoid mask
  int C_aad = 0;
  int force_split = 0;                       // >0: override the split-K heuristic (tests)
  int min_wgs = 0;                           // split K while the grid has fewer tiles (0 = 256)
  // optional InstanceNorm partials of the (bf16-rounded) output, written by the kernels that support
  // it (conv3x3_pp_takes): per (sample, tile, wave, channel) the mean and centred sum of squares of
  // 64 pixels; in_stats_from_tiles() merges them in fp64 into [B][C][2] mean / rstd
  float* in_part = nullptr;
  // optional arrival counters (zero on entry, left zero): a split-K GEMM whose partial tiles are small enough
  // reduces them in the last of each tile's workgroups to finish instead of a second kernel (same sums, same
  // order, same bytes).  Needs one word per (tile, phase); launches on one stream may share the words.
  unsigned* sem = nullptr;
  int nsem = 0;
};

// bytes of fp32 split-K workspace the launch may use
size_t conv_workspace_bytes(const ConvDesc& d);
// returns 0 on success, else a hipError_t / -1 (bad descriptor)
int conv_launch(const ConvDesc& d, void* ws, size_t ws_bytes, hipStream_t stream);

}  // namespace ghost
