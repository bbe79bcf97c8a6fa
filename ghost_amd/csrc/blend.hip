// ghost_amd — paste-back of swapped crops into full frames on the GPU.
//
// get_final_video (utils/inference/video_processing.py:218-227), per identity j and frame i:
//   mat_rev = kornia.invert_affine_transform(tfm);  swap_t = warp_affine(swap, mat_rev, size);
//   mask_t = warp_affine(mask, mat_rev, size);      frame = uint8(mask_t*swap_t + (1-mask_t)*frame)
// kornia 0.5.4 warp_affine = normalised-coordinate affine_grid + grid_sample(bilinear, zeros,
// align_corners=True): in pixel units the destination pixel (x, y) samples the crop at
// inv(mat_rev) (x, y, 1) = tfm (x, y, 1), so the kernel maps every frame pixel through tfm directly.
// Pixels whose sample position has all four taps outside the crop get mask_t = 0 and keep the
// frame value exactly (the reference's (1-0)*frame + 0*0), so they are skipped without a write.
//
// HBM-bound: per frame at most the crop's footprint is read twice (frame, crop) and written once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ghost_amd.h"
#include "ghost_common.h"

namespace ghost {
int set_last_error(int rc, const char* msg);
}

namespace {

struct BlendArgs {
  uint8_t* frames; long fstride; int H, W;
  const uint8_t* swaps; long sstride; int Hs, Ws;
  const float* masks; long mstride;
  const float* mats;      // [F][6] crop <- frame (the tfm of crop_frames_and_get_transforms)
  const int32_t* valid;   // [F] or null
};

__global__ void __launch_bounds__(256) blend_kernel(const BlendArgs a) {
  const int f = blockIdx.y;
  if (a.valid && !a.valid[f]) return;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)a.H * a.W) return;
  const int y = (int)(p / a.W), x = (int)(p - (long)y * a.W);
  const float* m = a.mats + f * 6;
  const float ix = fmaf(m[0], (float)x, fmaf(m[1], (float)y, m[2]));
  const float iy = fmaf(m[3], (float)x, fmaf(m[4], (float)y, m[5]));
  if (!(ix > -1.f && ix < (float)a.Ws && iy > -1.f && iy < (float)a.Hs)) return;   // every tap outside
  // grid_sampler_2d bilinear (zeros padding): corner weights as PyTorch forms them
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const float nw = (fx + 1.f - ix) * (fy + 1.f - iy), ne = (ix - fx) * (fy + 1.f - iy);
  const float sw = (fx + 1.f - ix) * (iy - fy), se = (ix - fx) * (iy - fy);
  const int tx[4] = {x0, x0 + 1, x0, x0 + 1}, ty[4] = {y0, y0, y0 + 1, y0 + 1};
  const float tw[4] = {nw, ne, sw, se};
  const uint8_t* sw8 = a.swaps + f * a.sstride;
  const float* mk = a.masks + f * a.mstride;
  float ms = 0.f, sv[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (tx[t] < 0 || tx[t] >= a.Ws || ty[t] < 0 || ty[t] >= a.Hs) continue;
    const long o = (long)ty[t] * a.Ws + tx[t];
    ms += mk[o] * tw[t];
#pragma unroll
    for (int c = 0; c < 3; ++c) sv[c] += (float)sw8[o * 3 + c] * tw[t];
  }
  uint8_t* fr = a.frames + f * a.fstride + p * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = ms * sv[c] + (1.f - ms) * (float)fr[c];
    fr[c] = (uint8_t)(int)fminf(fmaxf(v, 0.f), 255.f);   // .type(torch.uint8) of a value in [0, 255]
  }
}

}  // namespace

extern "C" int ghost_blend_swaps_u8(uint8_t* frames, int64_t frame_stride, int F, int H, int W, const uint8_t* swaps,
                                    int64_t swap_stride, int Hs, int Ws, const float* masks, int64_t mask_stride,
                                    const float* mats, const int32_t* valid, void* stream) {
  if (!frames || !swaps || !masks || !mats) return ghost::set_last_error(GHOST_EINVAL, "ghost_blend_swaps_u8: null argument");
  if (F <= 0 || H <= 0 || W <= 0 || Hs <= 0 || Ws <= 0 || frame_stride < (int64_t)H * W * 3 ||
      swap_stride < (int64_t)Hs * Ws * 3 || mask_stride < (int64_t)Hs * Ws || F > 65535)
    return ghost::set_last_error(GHOST_EINVAL, "ghost_blend_swaps_u8: bad sizes");
  BlendArgs a{frames, (long)frame_stride, H, W, swaps, (long)swap_stride, Hs, Ws, masks, (long)mask_stride, mats, valid};
  dim3 grid((unsigned)(((long)H * W + 255) / 256), (unsigned)F);
  hipLaunchKernelGGL(blend_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  const int rc = (int)hipGetLastError();
  return rc ? ghost::set_last_error(rc, "ghost_blend_swaps_u8 launch failed") : 0;
}
