// ghost_amd — halo-tiled 3x3/s1/p1 convolution (bf16, Cin % 32 == 0, N % 64 == 0).
#pragma once
#include <hip/hip_runtime.h>

#include "conv_igemm.h"

namespace ghost {

// true when conv3x3_halo takes this descriptor (3x3/s1/p1, bf16, standard epilogue without the
// uint8 copy — PReLU / residual-first / second BN'd output allowed —, K ordered (channel block, tap,
// channel) as pack.py packs it, and either exact 16 x 32 tiles or 16 x 16 tiles that overhang the
// image by at most a quarter of their pixels)
bool conv3x3_halo_supported(const ConvDesc& d);
// true when conv3x3_halo runs the persistent 16 x 32 kernel for d, which can also emit InstanceNorm
// partials of its output (d.in_part): count of partial records per (sample, channel) in *nrec
// (the persistent 16 x 16 form for overhanging tiles / the IBasicBlock epilogue writes no partials)
bool conv3x3_pp_takes(const ConvDesc& d, int* nrec);
int conv3x3_halo(const ConvDesc& d, hipStream_t s);

// ConvTranspose2d 4x4/s2/p1 on 8 x 16 input tiles (bf16, Cin % 32 == 0, N % 64 == 0 or N == 32,
// H % 8 == 0, W % 16 == 0; weights as pack.py pack_convT4x4 lays them out)
bool convT_halo_supported(const ConvDesc& d);
int convT_halo(const ConvDesc& d, hipStream_t s);

}  // namespace ghost
