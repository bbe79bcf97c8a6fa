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
// Also here: the cv2.resize of the swap to the crop size that precedes the warp in the video path, and the
// image path's cv2 warpAffine composite (get_final_image), both restated from OpenCV's fixed-point algorithms.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ghost_amd.h"
#include "ghost_common.h"

namespace ghost {
int set_last_error(int rc, const char* msg);
}

namespace {

// One rounding per operation, never fused: HIP's __fmul_rn / __dadd_rn ... are plain operators compiled with the
// translation unit's contraction mode, so after inlining the compiler fuses a*b + c into an FMA.  These carry no
// contract flag (the pragma applies to the operations written in their bodies).
__device__ __forceinline__ float f_mul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float f_add(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float f_sub(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}
__device__ __forceinline__ double d_mul(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double d_add(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ double d_sub(double a, double b) {
#pragma clang fp contract(off)
  return a - b;
}

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

// cv2.resize(src, (Wd, Hd)) INTER_LINEAR on uint8 3-channel images (video_processing.py:212: the 256x256 swap
// to the 224x224 crop size), OpenCV's fixed point (resize.cpp): per axis the source index and two 11-bit
// weights, fx = (float)((d + 0.5) * scale - 0.5), clamped at the borders; horizontal pass in int, vertical
// pass as the vector VResizeLinear: (((D0 >> 4) * b0 >> 16) + ((D1 >> 4) * b1 >> 16) + 2) >> 2.  Integer
// arithmetic throughout: bit-exact against oracle/blend_ref.resize_linear_u8.
struct RzTap {
  int s0, s1, w0, w1;
};
__device__ RzTap rz_tap(int d, int src_n, int dst_n) {
  const double scale = 1.0 / ((double)dst_n / (double)src_n);
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  int s0 = (int)floorf(f);
  f = f_sub(f, (float)s0);
  if (s0 < 0) { f = 0.f; s0 = 0; }
  if (s0 >= src_n - 1) { f = 0.f; s0 = src_n - 1; }
  RzTap t;
  t.s0 = s0;
  t.s1 = min(s0 + 1, src_n - 1);
  t.w0 = (int)rintf(f_mul(f_sub(1.f, f), 2048.f));
  t.w1 = (int)rintf(f_mul(f, 2048.f));
  return t;
}

__global__ void __launch_bounds__(256) resize_u8_linear_kernel(const uint8_t* __restrict__ src, long sstride, int Hs,
                                                               int Ws, uint8_t* __restrict__ dst, long dstride, int Hd,
                                                               int Wd) {
  const int f = blockIdx.y;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)Hd * Wd) return;
  const int dy = (int)(p / Wd), dx = (int)(p - (long)dy * Wd);
  const RzTap tx = rz_tap(dx, Ws, Wd), ty = rz_tap(dy, Hs, Hd);
  const uint8_t* sb = src + f * sstride;
  const uint8_t* r0 = sb + (long)ty.s0 * Ws * 3;
  const uint8_t* r1 = sb + (long)ty.s1 * Ws * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int D0 = (int)r0[tx.s0 * 3 + c] * tx.w0 + (int)r0[tx.s1 * 3 + c] * tx.w1;
    const int D1 = (int)r1[tx.s0 * 3 + c] * tx.w0 + (int)r1[tx.s1 * 3 + c] * tx.w1;
    int v = ((((D0 >> 4) * ty.w0) >> 16) + (((D1 >> 4) * ty.w1) >> 16) + 2) >> 2;
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    dst[f * dstride + p * 3 + c] = (uint8_t)v;
  }
}

// get_final_image (image_processing.py:51-76): the full frame, and per identity j in order a 224x224 uint8 swap
// warped by cv2.warpAffine(swap, invertAffineTransform(tfm), BORDER_REPLICATE) and its mask warped with the
// default constant 0 border, composited as final = mask_t*swap_t + (1-mask_t)*final, one uint8 cast at the end.
// The mask is face_mask_static's ``mask/255`` (masks.py:83-85): a float64 array, so cv2 warps it with float table
// weights and double accumulation (remapBilinear<Cast<double,double>, float>) and numpy composites in float64:
// all of that in double here (one rounding per operation, no FMA, numpy's order).  warpAffine's fixed point (imgwarp.cpp):
// the map A (the double inverse of the given matrix, host-side) sampled at X = (rint((A1 y + A2) 1024) + 16 +
// rint(A0 x 1024)) >> 5: pixel X >> 5, sub-pixel X & 31; bilinear weights from the 32 x 32 grid (15-bit integers
// for uint8 with (sum + 2^14) >> 15, floats for the mask).
struct CvWarp {
  int sx, sy;            // top-left source pixel
  float wx1, wy1;        // sub-pixel weights (multiples of 1/32)
};
__device__ CvWarp cv_warp_pos(const double* A, int x, int y) {
  const long adelta = __double2ll_rn(d_mul(d_mul(A[0], (double)x), 1024.0));
  const long bdelta = __double2ll_rn(d_mul(d_mul(A[3], (double)x), 1024.0));
  const long X0 = __double2ll_rn(d_mul(d_add(d_mul(A[1], (double)y), A[2]), 1024.0)) + 16;
  const long Y0 = __double2ll_rn(d_mul(d_add(d_mul(A[4], (double)y), A[5]), 1024.0)) + 16;
  const long X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
  CvWarp w;
  w.sx = (int)(X >> 5);
  w.sy = (int)(Y >> 5);
  w.wx1 = (float)(X & 31) * (1.f / 32.f);
  w.wy1 = (float)(Y & 31) * (1.f / 32.f);
  return w;
}

struct ImageBlendArgs {
  uint8_t* frame; int H, W;
  const uint8_t* swaps; long sstride;   // [J][224][224][3]
  const double* masks; long mstride;    // [J][224][224] float64 (mask/255)
  const double* maps;                   // [J][6] warpAffine's effective dst -> src map
  int J, S;
};

__global__ void __launch_bounds__(256) blend_image_kernel(const ImageBlendArgs a) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)a.H * a.W) return;
  const int y = (int)(p / a.W), x = (int)(p - (long)y * a.W);
  uint8_t* fr = a.frame + p * 3;
  double fin[3] = {(double)fr[0], (double)fr[1], (double)fr[2]};
  const int S = a.S;
  for (int j = 0; j < a.J; ++j) {
    const CvWarp w = cv_warp_pos(a.maps + j * 6, x, y);
    const float wx[2] = {f_sub(1.f, w.wx1), w.wx1}, wy[2] = {f_sub(1.f, w.wy1), w.wy1};
    const uint8_t* sw = a.swaps + j * a.sstride;
    const double* mk = a.masks + j * a.mstride;
    int acc[3] = {0, 0, 0};
    double ms = 0.0;
    bool any = false;
#pragma unroll
    for (int ky = 0; ky < 2; ++ky)
#pragma unroll
      for (int kx = 0; kx < 2; ++kx) {
        const float wf = f_mul(wy[ky], wx[kx]);          // the float interpolation table entry
        const int wi = (int)rintf(f_mul(wf, 32768.f));
        const int tx = w.sx + kx, ty = w.sy + ky;
        const bool in = tx >= 0 && tx < S && ty >= 0 && ty < S;
        any |= in;
        const int cx = min(max(tx, 0), S - 1), cy = min(max(ty, 0), S - 1);   // BORDER_REPLICATE
        const long o = (long)cy * S + cx;
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += (int)sw[o * 3 + c] * wi;
        ms = d_add(ms, d_mul(in ? mk[o] : 0.0, (double)wf));          // constant 0 border
      }
    const double mt = any ? ms : 0.0;
    const double omt = d_sub(1.0, mt);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      int v = (acc[c] + (1 << 14)) >> 15;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      fin[c] = d_add(d_mul(mt, (double)v), d_mul(omt, fin[c]));
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) fr[c] = (uint8_t)(int)fin[c];   // np.array(final, dtype='uint8')
}

}  // namespace

extern "C" int ghost_resize_u8_linear(const uint8_t* src, int64_t src_stride, int F, int Hs, int Ws, uint8_t* dst,
                                      int64_t dst_stride, int Hd, int Wd, void* stream) {
  if (!src || !dst) return ghost::set_last_error(GHOST_EINVAL, "ghost_resize_u8_linear: null argument");
  if (F <= 0 || F > 65535 || Hs <= 0 || Ws <= 0 || Hd <= 0 || Wd <= 0 || src_stride < (int64_t)Hs * Ws * 3 ||
      dst_stride < (int64_t)Hd * Wd * 3)
    return ghost::set_last_error(GHOST_EINVAL, "ghost_resize_u8_linear: bad sizes");
  dim3 grid((unsigned)(((long)Hd * Wd + 255) / 256), (unsigned)F);
  hipLaunchKernelGGL(resize_u8_linear_kernel, grid, dim3(256), 0, (hipStream_t)stream, src, (long)src_stride, Hs, Ws,
                     dst, (long)dst_stride, Hd, Wd);
  const int rc = (int)hipGetLastError();
  return rc ? ghost::set_last_error(rc, "ghost_resize_u8_linear launch failed") : 0;
}

extern "C" int ghost_blend_image_u8(uint8_t* frame, int H, int W, const uint8_t* swaps, int64_t swap_stride, int J,
                                    int S, const double* masks, int64_t mask_stride, const double* maps, void* stream) {
  if (!frame || (J > 0 && (!swaps || !masks || !maps)))
    return ghost::set_last_error(GHOST_EINVAL, "ghost_blend_image_u8: null argument");
  if (H <= 0 || W <= 0 || J < 0 || S <= 0 || (J > 0 && (swap_stride < (int64_t)S * S * 3 || mask_stride < (int64_t)S * S)))
    return ghost::set_last_error(GHOST_EINVAL, "ghost_blend_image_u8: bad sizes");
  if (J == 0) return 0;
  ImageBlendArgs a{frame, H, W, swaps, (long)swap_stride, masks, (long)mask_stride, maps, J, S};
  dim3 grid((unsigned)(((long)H * W + 255) / 256));
  hipLaunchKernelGGL(blend_image_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  const int rc = (int)hipGetLastError();
  return rc ? ghost::set_last_error(rc, "ghost_blend_image_u8 launch failed") : 0;
}

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
