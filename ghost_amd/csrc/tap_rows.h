// ghost_amd — AADBlk8's tap partials in row-summed form (the 3x3 conv to 3 channels whose inputs the
// AADLayers in front of it contract in their epilogue; aad_v3.h, GHOST_AEI_OPT_TAP_PARTIALS).
//
// A producer holds, for each of its pixels s, the 27 per-tap values Z_{dy,dx}[o](s) = sum_c w[o][c][dy][dx] x_c(s)
// (MFMA rows 16 o + 4 dy + dx, so a lane (pixel, dy) owns the three dx of each o).  Output (y, x) needs
//   sum_dy sum_dx Z_{dy,dx}(y + dy - 1, x + dx - 1),
// so the producer pre-sums along the row inside each 8-column segment (one DPP shift each way):
//   R_dy(s) = Z_{dy,0}(s - 1) + Z_{dy,1}(s) + Z_{dy,2}(s + 1)     (neighbours outside the segment left out)
// and exports the two terms that cross the segment's ends:
//   E_left(seg)  = Z_{dy,2}(first column)    -> output column first - 1
//   E_right(seg) = Z_{dy,0}(last column)     -> output column last + 1
// All fp16.  Per image: the R region, [HW][dy = 3][4] (the 4th value 0), then the E region,
// [HW / 8][side = 2][dy = 3][4]: 15 fp16 = 30 bytes per pixel, against 64 for the per-tap record it replaces
// (27 values in 32 fp16).  Segments never straddle image rows (W % 8 == 0).
#pragma once
#include "ghost_common.h"

namespace ghost {

constexpr int kZrR = 12;   // fp16 per pixel in the R region
constexpr int kZrE = 24;   // fp16 per 8-pixel segment in the E region
constexpr int kZrPerPixel = kZrR + kZrE / 8;   // 15 fp16 per pixel

GHOST_DEV long zr_image(int HW) { return (long)HW * kZrPerPixel; }   // fp16 per image

// the consumer side: the partial sums of one image's buffer z that land on output pixel (y, x), added to s
GHOST_DEV void zr_gather(const _Float16* __restrict__ z, int H, int W, int y, int x, float (&s)[3]) {
  typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
  const _Float16* __restrict__ e = z + (long)H * W * kZrR;
  const bool last = (x & 7) == 7 && x + 1 < W, first = (x & 7) == 0 && x > 0;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = y + dy - 1;
    if (yy < 0 || yy >= H) continue;
    const long ps = (long)yy * W + x;
    const f16x4 r = *reinterpret_cast<const f16x4*>(z + ps * kZrR + dy * 4);
    f16x4 c = {0, 0, 0, 0};
    if (last) c = *reinterpret_cast<const f16x4*>(e + ((ps + 1) >> 3) * kZrE + dy * 4);           // next segment's E_left
    if (first) c = *reinterpret_cast<const f16x4*>(e + ((ps - 1) >> 3) * kZrE + 12 + dy * 4);     // previous one's E_right
#pragma unroll
    for (int o = 0; o < 3; ++o) s[o] += (float)r[o] + (float)c[o];
  }
}

}  // namespace ghost
