// ghost_amd — AADLayer kernel for the wide stages (bf16, C in {256, 512, 1024}, Ca <= 512):
// one workgroup per (pixel block, 64-channel tile), weights in the pack_aad_v3 layout.
#pragma once
#include <hip/hip_runtime.h>

namespace ghost {

struct AadWideDesc {
  const void* za = nullptr;  int lda = 0, Ca = 0;
  const void* hin = nullptr; int ldh = 0;
  const float* stat = nullptr;                 // [B][C][2] mean, rstd of h_in
  int B = 0, HW = 0, C = 0, id_ld = 0;
  float slope = 0.f;
  const void* w3 = nullptr;                    // [C/64][128][Ca] permuted (pack.py pack_aad_v3)
  const float* b3 = nullptr;                   // [C/64][128]
  const float* wh = nullptr;                   // conv_h weight [C]
  const float* bh = nullptr;                   // conv_h bias [1]
  const float* idgb = nullptr;                 // [B][id_ld]: gamma_id at c, beta_id at C + c
  const float* mask = nullptr;                 // [B*HW] sigmoid mask of this layer (aad_mask)
  void* out = nullptr;       int ldo = 0;
  int dt = 1;                                  // storage type: GHOST_BF16 (1) or GHOST_F16 (2)
};

bool aad_wide_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo);
int aad_wide(const AadWideDesc& d, hipStream_t s);

}  // namespace ghost
