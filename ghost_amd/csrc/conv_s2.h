// ghost_amd — the attribute encoder's Conv2d 4x4/s2/p1 + BN(eval) + LeakyReLU (AEI_Net.py:19-24) for
// Cin % 32 == 0 (conv2..conv4 of MLAttrEncoder, AEI_Net.py:48-53) as an LDS input-patch MFMA kernel.
#pragma once
#include <hip/hip_runtime.h>

#include "conv_igemm.h"

namespace ghost {

bool conv4x4s2_patch_supported(const ConvDesc& d);
int conv4x4s2_patch(const ConvDesc& d, hipStream_t s);

}  // namespace ghost
