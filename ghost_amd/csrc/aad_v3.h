// ghost_amd — register-epilogue AADLayer kernel for the 64/128-channel stages (bf16).
#pragma once
#include <hip/hip_runtime.h>

namespace ghost {

struct AadV3Desc {
  int dt = 1;                                        // storage type: GHOST_BF16 (1) or GHOST_F16 (2)
  const void* za = nullptr;  int lda = 0, Ca = 0;   // z_attr NHWC
  const void* hin = nullptr; int ldh = 0;           // h_in NHWC (shared by the L layers)
  // up_H > 0: h_in = upsample2x(hin) (bilinear x2, align_corners) with hin the [B, up_H, up_W]
  // source, sampled on the fly (values rounded to bf16 as upsample2x stores them)
  int up_H = 0, up_W = 0;
  const float* stat = nullptr;                       // [B][C][2] mean, rstd of h_in
  int B = 0, HW = 0, C = 0, L = 1, id_ld = 0;
  float slope = 0.f;
  // per layer (L <= 2): permuted weights [C/64][128][Ca], biases [C/64][128], conv_h, id table, output
  const void* w3[2] = {nullptr, nullptr};
  const float* b3[2] = {nullptr, nullptr};
  const float* wh[2] = {nullptr, nullptr};
  const float* bh[2] = {nullptr, nullptr};
  const float* idgb[2] = {nullptr, nullptr};
  void* out[2] = {nullptr, nullptr};
  int ldo[2] = {0, 0};
  // tap partials (C = 64 only): a layer with zw[l] set writes, instead of its 64 channels, its share of
  // the 3x3 conv to 3 channels that is its only consumer, per-tap sums Z_t[o] = sum_c zw[l][t*3 + o][c] *
  // out_c (t = ky*3 + kx) pre-summed along 8-column row segments (tap_rows.h: 15 fp16 per pixel; zw: bf16
  // rows of stride zwld, the narrow layout's K slice of this layer's channels); out[l] is then that buffer,
  // zr_image(HW) fp16 per sample, and the image width must be a multiple of 8
  const void* zw[2] = {nullptr, nullptr};
  int zwld = 0;
  // in-kernel clock of the launch (profiling; v4 / v5): aad_v3_clock_words(d) words of per-workgroup start
  // and per-wave end stamps
  unsigned long long* tclk = nullptr;
  int* version_out = nullptr;   // set to the kernel generation that ran (3, 4 or 5)
};

// the 3x3 / pad 1 conv to 3 channels from two tap-partial buffers (AADBlk8's output conv over
// cat(h, x'), AADLayer.py:71,79): y = tanh(sum_t (zh + zx)[p + off_t][t*3 + o]) -> bf16 y (ldy) + BGR uint8
int tap_sum3x3(int dt, const void* zh, const void* zx, int B, int H, int W, void* y, int ldy, uint8_t* u8,
               hipStream_t s);

int aad_v3_clock_words(const AadV3Desc& d);
bool aad_v3_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo);
int aad_v3(const AadV3Desc& d, hipStream_t s);

}  // namespace ghost
