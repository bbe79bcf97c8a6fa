// ghost_amd — AADBlk8's tail (two AADLayers + ReLU + the fused 128 -> 3 output conv + tanh/uint8).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ghost {

struct AadTailDesc {
  const void* za = nullptr; int lda = 0, Ca = 0;     // z_attr8 NHWC
  // layer 0: the last add_blocks AADLayer (input x), layer 1: the last_add_block AADLayer (input m);
  // up_H/up_W > 0: that input is the x2 upsample of the [B, up_H, up_W] tensor hin[l]
  const void* hin[2] = {nullptr, nullptr};
  int ldh[2] = {0, 0};
  int up_H[2] = {0, 0}, up_W[2] = {0, 0};
  const float* stat[2] = {nullptr, nullptr};
  const void* w3[2] = {nullptr, nullptr};
  const float* b3[2] = {nullptr, nullptr};
  const float* wh[2] = {nullptr, nullptr};
  const float* bh[2] = {nullptr, nullptr};
  const float* idgb[2] = {nullptr, nullptr};
  int id_ld = 0;
  const void* wn = nullptr;                           // [32][128] (pack_conv3x3_narrow of the cat weight)
  void* y = nullptr;                                  // [B, H, W, 3] bf16
  uint8_t* u8 = nullptr;
  int B = 0, H = 0, W = 0, tanh_out = 0;
};

bool aad_tail_supported(int dt, int H, int W, int Ca, int lda, int ldh0, int ldh1);
int aad_tail(const AadTailDesc& d, hipStream_t s);

}  // namespace ghost
