// ghost_amd — the attribute encoder's Conv2d 4x4/s2/p1 + BN(eval) + LeakyReLU (AEI_Net.py:19-24) for
// Cin % 32 == 0 (conv2..conv4 of MLAttrEncoder, AEI_Net.py:48-53) as an LDS input-patch MFMA kernel; the same
// kernel at 3x3/s2/p1 for IResNet (ArcFace).
#pragma once
#include <hip/hip_runtime.h>

#include "conv_igemm.h"

namespace ghost {

bool conv4x4s2_patch_supported(const ConvDesc& d);
// IResNet's 3x3/s2/p1 convs (IBasicBlock epilogue: BN, PReLU, residual, second output)
bool conv3x3s2_patch_supported(const ConvDesc& d);
// either form (d.kh = 4 or 3)
int conv_s2_patch(const ConvDesc& d, hipStream_t s);

}  // namespace ghost
