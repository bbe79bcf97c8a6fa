// ghost_amd — direct (VALU) kernel for the encoder's Conv2d(3, 32, 4, s2, p1) + BN + LReLU.
#pragma once
#include <hip/hip_runtime.h>

#include "conv_igemm.h"

namespace ghost {

bool conv_first_supported(const ConvDesc& d);
size_t conv_first_workspace_bytes();
int conv_first(const ConvDesc& d, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace ghost
