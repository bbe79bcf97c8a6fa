// ghost_amd — direct (VALU) kernel for the encoder's Conv2d(3, 32, 4, s2, p1) + BN + LReLU.
#pragma once
#include <hip/hip_runtime.h>

#include "conv_igemm.h"

namespace ghost {

bool conv_first_supported(const ConvDesc& d);
size_t conv_first_workspace_bytes();
int conv_first(const ConvDesc& d, void* ws, size_t ws_bytes, hipStream_t s);

// ArcFace stem: Conv2d(3, 64, 3, s1, p1) on the 4-channel bf16 input + BN/PReLU + second BN'd output (MFMA)
bool conv_stem3x3_supported(const ConvDesc& d);
int conv_stem3x3(const ConvDesc& d, hipStream_t s);

}  // namespace ghost
