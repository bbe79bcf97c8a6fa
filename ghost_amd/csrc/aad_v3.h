// ghost_amd — register-epilogue AADLayer kernel for the 64/128-channel stages (bf16).
#pragma once
#include <hip/hip_runtime.h>

namespace ghost {

struct AadV3Desc {
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
};

bool aad_v3_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo);
int aad_v3(const AadV3Desc& d, hipStream_t s);

}  // namespace ghost
