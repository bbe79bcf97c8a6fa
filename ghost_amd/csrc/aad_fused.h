// ghost_amd — fused AADLayer kernel for layers with enough pixels to fill the chip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace ghost {

// true when aad_fused can run this layer (C % 64 == 0, HW % 64 == 0, >= 512 workgroups)
bool aad_fused_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo);

// AADLayer + following activation (slope 0 = ReLU, 1 = none).  w: [2C rounded to 128][Kpad]
// gamma/beta rows interleaved per 16 channels, gbb the matching fp32 biases; stat [B][C][2]
// (mean, rstd of h_in); idgb rows of id_ld floats with gamma_id at c and beta_id at C + c.
int aad_fused(int dt, const void* za, int lda, int Ca, const void* w, int Kpad, const float* gbb, const void* hin,
              int ldh, const float* stat, const float* wh, const float* bh, const float* idgb, int id_ld, void* out,
              int ldo, int B, int HW, int C, float slope, hipStream_t s);

}  // namespace ghost
