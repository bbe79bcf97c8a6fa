// ghost_amd — face masks for the paste-back on the GPU (utils/inference/masks.py).
//
// face_mask_static(swap, landmarks, landmarks_tgt, params) per frame (masks.py:38-86):
//   expand_eyebrows (masks.py:5-20), get_mask = cv2.fillConvexPoly(zeros, cv2.convexHull(landmarks), 255)
//   (masks.py:23-35), erode_and_blur = cv2.erode / cv2.dilate with a k x k box, zero border of 2*sigmaY,
//   cv2.GaussianBlur(mask, (0, 0), sigmaX, sigmaY) (masks.py:89-107), returned as mask / 255.
// Host side (ghost_mask_polygons, C++ on the CPU, microseconds per frame): the eyebrow expansion on int32
// landmarks and the convex hull of the 106 points (Andrew's monotone chain; collinear points dropped).
// Device side, one launch per step for a whole batch of frames:
//   mask_raster_kernel  one workgroup per frame, the H x W byte mask in LDS: every polygon edge drawn with the
//                       8-connected Bresenham of cv2.line (LineIterator, left to right, clipLine), the scanline
//                       spans of FillConvexPoly (two vertex chains from the topmost vertex, 16.16 fixed point:
//                       one thread per chain produces every row's edge x, then all threads fill), the box erode /
//                       dilate as two separable min / max passes between two LDS planes, the border fade;
//   mask_blur_kernel    separable Gaussian (cv2.getGaussianKernel taps for ksize = cvRound(6 sigma + 1) | 1,
//                       BORDER_REFLECT_101), rows then columns, fp32 products and sums in tap order without FMA
//                       contraction (the restatement's arithmetic), one cvRound to uint8, / 255 as float.
// OpenCV restated from its published 4.x algorithms (drawing.cpp FillConvexPoly / Line / clipLine,
// morph.cpp, smooth.cpp); cv2 is absent here, so the masks are pinned to oracle/mask_ref.py only (parity
// unpinned; OpenCV's 8-bit Gaussian runs in fixed point and can differ from the fp32 evaluation by ~1 LSB).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#include "ghost_amd.h"
#include "ghost_common.h"

namespace ghost {
int set_last_error(int rc, const char* msg);
}

namespace {

constexpr int kMaxV = 128;          // hull vertices per frame (the hull of 106 landmarks has at most 106)
constexpr int kMaxHW = 224 * 256;   // LDS plane: H * W <= 57 344 bytes (the 224 x 224 resized swap)
constexpr int kMaxRows = 256;
constexpr int XY_SHIFT = 16;
constexpr long XY_ONE = 1L << XY_SHIFT;

struct RasterArgs {
  const int32_t* poly;   // [F][kMaxV][2] (x, y)
  const int32_t* nv;     // [F]
  const int32_t* params; // [F][3] erode, sigmaX, sigmaY
  int H, W;
  uint8_t* out;          // [F][H][W]
};

// C integer division, truncation toward zero (int64 operands)
__device__ __forceinline__ long tdiv(long a, long b) {
  const long q = (a < 0 ? -a : a) / (b < 0 ? -b : b);
  return ((a < 0) == (b < 0)) ? q : -q;
}

// cv2 clipLine (drawing.cpp) on integer endpoints
__device__ bool clip_line(int W, int H, long& x1, long& y1, long& x2, long& y2) {
  const long right = W - 1, bottom = H - 1;
  auto code = [&](long x, long y) { return (x < 0) + (x > right) * 2 + (y < 0) * 4 + (y > bottom) * 8; };
  int c1 = code(x1, y1), c2 = code(x2, y2);
  if ((c1 & c2) == 0 && (c1 | c2) != 0) {
    long a;
    if (c1 & 12) {
      a = c1 < 8 ? 0 : bottom;
      x1 += (long)((double)(a - y1) * (double)(x2 - x1) / (double)(y2 - y1));
      y1 = a;
      c1 = (x1 < 0) + (x1 > right) * 2;
    }
    if (c2 & 12) {
      a = c2 < 8 ? 0 : bottom;
      x2 += (long)((double)(a - y2) * (double)(x2 - x1) / (double)(y2 - y1));
      y2 = a;
      c2 = (x2 < 0) + (x2 > right) * 2;
    }
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
      if (c1) {
        a = c1 == 1 ? 0 : right;
        y1 += (long)((double)(a - x1) * (double)(y2 - y1) / (double)(x2 - x1));
        x1 = a;
        c1 = 0;
      }
      if (c2) {
        a = c2 == 1 ? 0 : right;
        y2 += (long)((double)(a - x2) * (double)(y2 - y1) / (double)(x2 - x1));
        x2 = a;
        c2 = 0;
      }
    }
  }
  return (c1 | c2) == 0;
}

// cv2.line LINE_8 into the LDS plane (LineIterator, left to right)
__device__ void draw_line(uint8_t* img, int W, int H, long x1, long y1, long x2, long y2) {
  if (!(x1 >= 0 && x1 < W && y1 >= 0 && y1 < H && x2 >= 0 && x2 < W && y2 >= 0 && y2 < H))
    if (!clip_line(W, H, x1, y1, x2, y2)) return;
  if (x2 < x1) {
    long t = x1; x1 = x2; x2 = t;
    t = y1; y1 = y2; y2 = t;
  }
  const long dx = x2 - x1;
  long dy = y2 - y1;
  const long sy = dy < 0 ? -1 : 1;
  dy = dy < 0 ? -dy : dy;
  const bool maj_x = !(dy > dx);
  const long M = maj_x ? dx : dy, m = maj_x ? dy : dx;
  long err = M - 2 * m, x = x1, y = y1;
  for (long k = 0; k <= M; ++k) {
    img[y * W + x] = 255;
    if (err < 0) {
      err += 2 * M - 2 * m;
      x += 1;
      y += sy;
    } else {
      err -= 2 * m;
      if (maj_x) x += 1; else y += sy;
    }
  }
}

__global__ void __launch_bounds__(256) mask_raster_kernel(const RasterArgs a) {
  __shared__ uint8_t img[kMaxHW];
  __shared__ uint8_t tmp[kMaxHW];
  __shared__ int xs[2][kMaxRows];   // per row: the two chains' rounded span ends (INT_MIN: no fill)
  __shared__ int s_ymin, s_ymax;
  const int f = blockIdx.x, tid = threadIdx.x, H = a.H, W = a.W, HW = H * W;
  const int32_t* P = a.poly + (long)f * kMaxV * 2;
  const int n = a.nv[f];
  for (int i = tid; i < HW; i += 256) img[i] = 0;
  __syncthreads();
  // polygon edges (FillConvexPoly draws every edge v[i-1] -> v[i] with Line): one thread per edge; threads that
  // write the same pixel write the same value
  for (int i = tid; i < n; i += 256) {
    const int j = i == 0 ? n - 1 : i - 1;
    draw_line(img, W, H, P[2 * j], P[2 * j + 1], P[2 * i], P[2 * i + 1]);
  }
  // the two chains' x per row, each walked by one thread exactly as FillConvexPoly's scanline loop (both
  // chains start at the first vertex of minimal y; the shared edge budget is n)
  if (tid == 0) {
    int imin = 0;
    long ymin = P[1], ymax = P[1], xmin = P[0], xmax = P[0];
    for (int i = 0; i < n; ++i) {
      const long px = P[2 * i], py = P[2 * i + 1];
      if (py < ymin) { ymin = py; imin = i; }
      ymax = py > ymax ? py : ymax;
      xmax = px > xmax ? px : xmax;
      xmin = px < xmin ? px : xmin;
    }
    if (n < 3 || xmax < 0 || ymax < 0 || xmin >= W || ymin >= H) {
      s_ymin = 0;
      s_ymax = -1;
    } else {
      ymax = ymax < H - 1 ? ymax : H - 1;
      long ex[2] = {-XY_ONE, -XY_ONE}, edx[2] = {0, 0};
      int eidx[2] = {imin, imin}, edi[2] = {1, n - 1};
      long eye[2] = {ymin, ymin};
      int edges = n;
      long y = ymin;
      int last = (int)ymin - 1;
      for (;;) {
        for (int c = 0; c < 2; ++c) {
          if (y >= eye[c]) {
            int idx0 = eidx[c], idx = idx0 + edi[c];
            if (idx >= n) idx -= n;
            for (;;) {
              if (!(edges-- > 0)) break;
              const long ty = P[2 * idx + 1];
              if (ty > y) {
                const long xs0 = (long)P[2 * idx0] << XY_SHIFT, xe = (long)P[2 * idx] << XY_SHIFT;
                eye[c] = ty;
                edx[c] = tdiv((xe - xs0) * 2 + (ty - y), 2 * (ty - y));
                ex[c] = xs0;
                eidx[c] = idx;
                break;
              }
              idx0 = idx;
              idx += edi[c];
              if (idx >= n) idx -= n;
            }
          }
        }
        if (edges < 0) break;
        if (y >= 0) {
          const int l = ex[0] > ex[1] ? 1 : 0;
          xs[0][y] = (int)((ex[l] + (XY_ONE >> 1)) >> XY_SHIFT);
          xs[1][y] = (int)((ex[1 - l] + (XY_ONE >> 1)) >> XY_SHIFT);
          last = (int)y;
        }
        ex[0] += edx[0];
        ex[1] += edx[1];
        if (++y > ymax) break;
      }
      s_ymin = ymin > 0 ? (int)ymin : 0;
      s_ymax = last;
    }
  }
  __syncthreads();
  for (int y = s_ymin + tid; y <= s_ymax; y += 256) {
    int x1 = xs[0][y], x2 = xs[1][y];
    if (x2 >= 0 && x1 < W) {
      x1 = x1 < 0 ? 0 : x1;
      x2 = x2 >= W ? W - 1 : x2;
      for (int x = x1; x <= x2; ++x) img[y * W + x] = 255;
    }
  }
  __syncthreads();
  // erode (k = erode > 0) or dilate (k = -erode): window [p - k/2, p - k/2 + k - 1] per axis, pixels outside the
  // image ignored; columns first into tmp, then rows back into img
  const int erode = a.params[f * 3], sy = a.params[f * 3 + 2];
  const bool dil = erode <= 0;
  const int k = erode > 0 ? erode : -erode, an = k / 2;
  for (int i = tid; i < HW; i += 256) {
    const int y = i / W, x = i - y * W;
    int v = dil ? 0 : 255;
    for (int d = 0; d < k; ++d) {
      const int yy = y - an + d;
      if (yy < 0 || yy >= H) continue;
      const int t = img[yy * W + x];
      v = dil ? (t > v ? t : v) : (t < v ? t : v);
    }
    tmp[i] = (uint8_t)v;
  }
  __syncthreads();
  const int c = 2 * sy;
  uint8_t* o = a.out + (long)f * HW;
  for (int i = tid; i < HW; i += 256) {
    const int y = i / W, x = i - y * W;
    int v = dil ? 0 : 255;
    for (int d = 0; d < k; ++d) {
      const int xx = x - an + d;
      if (xx < 0 || xx >= W) continue;
      const int t = tmp[y * W + xx];
      v = dil ? (t > v ? t : v) : (t < v ? t : v);
    }
    // fade_to_border (masks.py:99-104): rows / columns [0, c) and [n - c, n) cleared (numpy's [-c:] with c > 0)
    if (c > 0 && (y < c || y >= H - c || x < c || x >= W - c)) v = 0;
    o[i] = (uint8_t)v;
  }
}

struct BlurArgs {
  const uint8_t* in;     // [F][H][W]
  const int32_t* params; // [F][3]
  int H, W;
  float* tmp;            // [F][H][W] row-filtered
  float* out;            // [F][H][W] mask / 255
  long out_stride;
};

constexpr int kMaxTaps = 256;

// cv2.getGaussianKernel(n, sigma) normalised in double, stored as float; n = cvRound(6 sigma + 1) | 1
__device__ int gauss_taps(int sigma, float* k) {
  const double s = (double)sigma, sc = -0.5 / (s * s);
  const int n = ((int)floor(s * 6.0 + 1.0 + 0.5)) | 1;
  if (n > kMaxTaps) return 0;
  double sum = 0.0;
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    sum += exp(sc * x * x);
  }
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    k[i] = (float)(exp(sc * x * x) / sum);
  }
  return n;
}

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  const int p = 2 * (n - 1);
  i = i < 0 ? -i : i;
  i %= p;
  return i >= n ? p - i : i;
}

// pass 0: rows (x taps, sigmaX) uint8 -> fp32 tmp; pass 1: columns (y taps, sigmaY) tmp -> rint -> / 255
template <int PASS>
__global__ void __launch_bounds__(256) mask_blur_kernel(const BlurArgs a) {
  __shared__ float k[kMaxTaps];
  __shared__ int s_n;
  const int f = blockIdx.y, tid = threadIdx.x, H = a.H, W = a.W;
  if (tid == 0) s_n = gauss_taps(a.params[f * 3 + (PASS == 0 ? 1 : 2)], k);
  __syncthreads();
  const int n = s_n, r = n / 2;
  const long base = (long)f * H * W;
  for (int i = blockIdx.x * 256 + tid; i < H * W; i += gridDim.x * 256) {
    const int y = i / W, x = i - y * W;
    float acc = 0.f;
    for (int t = 0; t < n; ++t) {
      float v;
      if (PASS == 0) v = (float)a.in[base + (long)y * W + reflect101(x - r + t, W)];
      else v = a.tmp[base + (long)reflect101(y - r + t, H) * W + x];
      acc = __fadd_rn(acc, __fmul_rn(k[t], v));
    }
    if (PASS == 0) {
      a.tmp[base + i] = acc;
    } else {
      float q = rintf(acc);
      q = q < 0.f ? 0.f : (q > 255.f ? 255.f : q);
      a.out[(long)f * a.out_stride + i] = (float)((double)q / 255.0);
    }
  }
}

}  // namespace

// ---- host: eyebrow expansion + convex hull (masks.py:5-35) ----
extern "C" int ghost_mask_polygons(const float* landmarks, int F, int npts, const int32_t* params, int32_t* poly,
                                   int32_t* nv) {
  if (!landmarks || !params || !poly || !nv || F < 0 || npts != 106)
    return ghost::set_last_error(GHOST_EINVAL, "ghost_mask_polygons: bad arguments (106 landmarks per frame)");
  static const int bl[5] = {35, 41, 40, 42, 39}, br[5] = {89, 95, 94, 96, 93};
  static const int tl[5] = {43, 48, 49, 51, 50}, tr[5] = {102, 103, 104, 105, 101};
  std::vector<std::pair<long, long>> p(npts), hull;
  for (int f = 0; f < F; ++f) {
    const float* L = landmarks + (long)f * npts * 2;
    const int erode = params[f * 3];
    const double mod = erode == 15 ? 2.7 : erode == -5 ? 0.5 : 2.0;
    std::vector<int32_t> li(2 * npts);
    for (int i = 0; i < 2 * npts; ++i) li[i] = (int32_t)L[i];   // np.array(lmrks, dtype=np.int32): truncation
    std::vector<int32_t> lo = li;
    for (int s = 0; s < 5; ++s)
      for (int c = 0; c < 2; ++c) {
        const int32_t topl = li[2 * tl[s] + c], botl = li[2 * bl[s] + c];
        const int32_t topr = li[2 * tr[s] + c], botr = li[2 * br[s] + c];
        lo[2 * tl[s] + c] = (int32_t)((double)topl + mod * 0.5 * (double)(topl - botl));
        lo[2 * tr[s] + c] = (int32_t)((double)topr + mod * 0.5 * (double)(topr - botr));
      }
    for (int i = 0; i < npts; ++i) p[i] = {lo[2 * i], lo[2 * i + 1]};
    std::vector<std::pair<long, long>> q = p;
    std::sort(q.begin(), q.end());
    q.erase(std::unique(q.begin(), q.end()), q.end());
    hull.clear();
    if (q.size() <= 2) {
      hull = q;
    } else {
      auto cross = [](const std::pair<long, long>& o, const std::pair<long, long>& a2, const std::pair<long, long>& b) {
        return (a2.first - o.first) * (b.second - o.second) - (a2.second - o.second) * (b.first - o.first);
      };
      std::vector<std::pair<long, long>> lower, upper;
      for (auto& pt : q) {
        while (lower.size() >= 2 && cross(lower[lower.size() - 2], lower.back(), pt) <= 0) lower.pop_back();
        lower.push_back(pt);
      }
      for (auto it = q.rbegin(); it != q.rend(); ++it) {
        while (upper.size() >= 2 && cross(upper[upper.size() - 2], upper.back(), *it) <= 0) upper.pop_back();
        upper.push_back(*it);
      }
      hull.assign(lower.begin(), lower.end() - 1);
      hull.insert(hull.end(), upper.begin(), upper.end() - 1);
    }
    if ((int)hull.size() > kMaxV) return ghost::set_last_error(GHOST_EINVAL, "ghost_mask_polygons: hull too large");
    nv[f] = (int32_t)hull.size();
    for (size_t i = 0; i < hull.size(); ++i) {
      poly[((long)f * kMaxV + i) * 2] = (int32_t)hull[i].first;
      poly[((long)f * kMaxV + i) * 2 + 1] = (int32_t)hull[i].second;
    }
  }
  return 0;
}

extern "C" int64_t ghost_face_masks_workspace_bytes(int F, int H, int W) {
  return (int64_t)F * H * W * (1 + 4) + 256;
}

// ---- device: raster + erode + fade + blur for F frames ----
extern "C" int ghost_face_masks(const int32_t* poly, const int32_t* nv, const int32_t* params, int F, int H, int W,
                                float* masks, int64_t mask_stride, void* ws, int64_t ws_bytes, void* stream) {
  if (!poly || !nv || !params || !masks || !ws) return ghost::set_last_error(GHOST_EINVAL, "ghost_face_masks: null argument");
  if (F <= 0 || H <= 0 || W <= 0 || H * W > kMaxHW || H > kMaxRows || mask_stride < (int64_t)H * W)
    return ghost::set_last_error(GHOST_EINVAL, "ghost_face_masks: bad sizes (H*W <= 57344, H <= 256)");
  if (ws_bytes < ghost_face_masks_workspace_bytes(F, H, W))
    return ghost::set_last_error(GHOST_ENOWS, "ghost_face_masks: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  uint8_t* u8 = (uint8_t*)ws;
  float* tmp = (float*)((((uintptr_t)ws + (size_t)F * H * W) + 255) & ~(uintptr_t)255);
  RasterArgs r{poly, nv, params, H, W, u8};
  hipLaunchKernelGGL(mask_raster_kernel, dim3((unsigned)F), dim3(256), 0, s, r);
  BlurArgs b{u8, params, H, W, tmp, masks, (long)mask_stride};
  const dim3 grid((unsigned)((H * W + 256 * 8 - 1) / (256 * 8)), (unsigned)F);
  hipLaunchKernelGGL(mask_blur_kernel<0>, grid, dim3(256), 0, s, b);
  hipLaunchKernelGGL(mask_blur_kernel<1>, grid, dim3(256), 0, s, b);
  const int rc = (int)hipGetLastError();
  return rc ? ghost::set_last_error(rc, "ghost_face_masks launch failed") : 0;
}
