// ghost_amd — 3x3 / pad 1 convolution to <= 3 output channels (the generator's RGB output).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ghost {

bool conv3x3_narrow_supported(int dt, int H, int W, int Cin, int ldx, int NO);
// w_narrow: [32][Kpad] with row n = tap*NO + o (tap = ky*3 + kx), K = input channel (zero rows >= 9*NO)
// zadd (optional, bf16 path): [B*H*W][32] fp16 tap partials Z[p][tap*NO + o] of further input channels that a
// producer already contracted (aad_v3.h), added to this conv's own partials before the 3x3 gather
int conv3x3_narrow(int dt, const void* x, int B, int H, int W, int Cin, int ldx, const void* w_narrow, int Kpad, int NO,
                   const void* res, int ldres, int tanh_out, void* y, int ldy, uint8_t* u8, hipStream_t s,
                   const void* zadd = nullptr);

}  // namespace ghost
