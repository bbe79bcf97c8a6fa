// ghost_amd — halo-tiled 3x3/s1/p1 convolution (bf16, Cin % 32 == 0, N % 64 == 0).
#pragma once
#include <hip/hip_runtime.h>

#include "conv_igemm.h"

namespace ghost {

// true when conv3x3_halo takes this descriptor (3x3/s1/p1, bf16, standard epilogue without the
// uint8 copy, H % 16 == 0, W % 32 == 0, K ordered (channel block, tap, channel) as pack.py packs it)
bool conv3x3_halo_supported(const ConvDesc& d);
int conv3x3_halo(const ConvDesc& d, hipStream_t s);

}  // namespace ghost
