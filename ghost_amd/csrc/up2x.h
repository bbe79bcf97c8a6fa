// ghost_amd — bilinear x2 (align_corners=True) sample of an NHWC source, shared by the
// upsample kernel, the InstanceNorm statistics of a virtual upsampled tensor and the AAD
// kernel that reads its h_in through the upsample (AEI_Net.py:125-137).
//
// Same arithmetic as PyTorch's upsample_bilinear2d: src = dst * scale with the product
// rounded to fp32 (the empty asm keeps hipcc from re-forming scale*dst - floor as one FMA),
// lambda = src - floor(src), value = l0y*(l0x*v00 + l1x*v01) + l1y*(l0x*v10 + l1x*v11) (up2x_mix).
#pragma once
#include "ghost_common.h"

namespace ghost {

struct Up2xSrc {
  int H, W;        // source grid (output is 2H x 2W)
  float sh, sw;    // (H-1)/(2H-1), (W-1)/(2W-1), rounded once on the host
};

inline Up2xSrc up2x_src(int H, int W) {
  Up2xSrc u;
  u.H = H;
  u.W = W;
  u.sh = H > 0 ? (float)(H - 1) / (float)(2 * H - 1) : 0.f;
  u.sw = W > 0 ? (float)(W - 1) / (float)(2 * W - 1) : 0.f;
  return u;
}

struct Up2xTap {
  int o00, o01, o10, o11;   // pixel offsets inside the sample (multiply by ld)
  float ly0, ly1, lx0, lx1;
};

GHOST_DEV Up2xTap up2x_tap(const Up2xSrc& u, int oy, int ox) {
  float ry = u.sh * (float)oy, rx = u.sw * (float)ox;
  asm volatile("" : "+v"(ry), "+v"(rx));
  const int y0 = (int)ry, x0 = (int)rx;
  const int y1 = y0 + (y0 < u.H - 1 ? 1 : 0), x1 = x0 + (x0 < u.W - 1 ? 1 : 0);
  Up2xTap t;
  t.ly1 = ry - (float)y0;
  t.ly0 = 1.f - t.ly1;
  t.lx1 = rx - (float)x0;
  t.lx0 = 1.f - t.lx1;
  t.o00 = y0 * u.W + x0;
  t.o01 = y0 * u.W + x1;
  t.o10 = y1 * u.W + x0;
  t.o11 = y1 * u.W + x1;
  return t;
}

// the bilinear mix with its FMA contraction spelled out, so that every kernel that samples the
// upsample (the upsample kernel, statistics, AAD reads) rounds to the same value
GHOST_DEV float up2x_mix(float ly0, float ly1, float lx0, float lx1, float v00, float v01, float v10, float v11) {
  const float top = fmaf(lx0, v00, lx1 * v01);
  const float bot = fmaf(lx0, v10, lx1 * v11);
  return fmaf(ly0, top, ly1 * bot);
}

// VEC (16-byte) channels at `xc` (sample base + channel offset) of output pixel t, in fp32
template <typename T>
GHOST_DEV void up2x_load16_f(const T* xc, int ld, const Up2xTap& t, float* o) {
  constexpr int VEC = Vec16<T>::N;
  float v00[VEC], v01[VEC], v10[VEC], v11[VEC];
  load16_f(xc + (long)t.o00 * ld, v00);
  load16_f(xc + (long)t.o01 * ld, v01);
  load16_f(xc + (long)t.o10 * ld, v10);
  load16_f(xc + (long)t.o11 * ld, v11);
#pragma unroll
  for (int e = 0; e < VEC; ++e)
    o[e] = up2x_mix(t.ly0, t.ly1, t.lx0, t.lx1, v00[e], v01[e], v10[e], v11[e]);
}

}  // namespace ghost
