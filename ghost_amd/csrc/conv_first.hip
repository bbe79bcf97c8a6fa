// ghost_amd — the encoder's first layer: Conv2d(3, 32, 4, s2, p1) + BN(eval) + LeakyReLU(0.1)
// (AEI_Net.py:19-24, MLAttrEncoder.conv1).
//
// K = 48 (16 taps x 3 channels) is far too shallow for a matrix-core GEMM and a 3-channel NHWC
// row is not a 16-byte vector, so the implicit GEMM spends its time on scalar gathers.  Here one
// thread owns one output pixel and all output channels: 48 input values (L1-resident: 2x2
// overlap between neighbouring outputs), 48 x N FMAs against weights that are uniform across
// the wave (fp32, scalar loads, no LDS traffic), then the BN/LReLU epilogue and 16-byte stores.
// bf16 weights are first widened to fp32 [N][48] in the caller's workspace (a 1.5 K-element
// kernel), so the FMA loop never converts a weight.
#include "conv_first.h"
#include "ghost_common.h"

namespace ghost {

struct FirstArgs {
  const void* x;
  const float* w;     // fp32 [N][48], K = (ky*4 + kx)*3 + c
  void* y;
  const float* scale;
  const float* shift;
  int Hi, Wi, ldx, Ho, Wo, Kpad, ldy;
  float slope;
  long M;
};

template <typename T, int N>
__global__ void __launch_bounds__(256) conv_first_kernel(const FirstArgs a) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  if (m >= a.M) return;
  const int hw = a.Ho * a.Wo;
  const int b = (int)(m / hw);
  const int r = (int)(m - (long)b * hw);
  const int oy = r / a.Wo, ox = r - oy * a.Wo;
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x) + (long)b * a.Hi * a.Wi * a.ldx;
  const float* __restrict__ w = a.w;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    const int iy = 2 * oy - 1 + ky;
    const bool oky = iy >= 0 && iy < a.Hi;
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) {
      const int ix = 2 * ox - 1 + kx;
      const bool ok = oky && ix >= 0 && ix < a.Wi;
      const T* px = x + ((long)(ok ? iy : 0) * a.Wi + (ok ? ix : 0)) * a.ldx;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = ok ? to_f(px[c]) : 0.f;
        const int k = (ky * 4 + kx) * 3 + c;
#pragma unroll
        for (int n = 0; n < N; ++n) acc[n] = fmaf(v, w[n * 48 + k], acc[n]);
      }
    }
  }
  T* y = reinterpret_cast<T*>(a.y) + m * a.ldy;
#pragma unroll
  for (int n0 = 0; n0 < N; n0 += Vec16<T>::N) {
    float o[Vec16<T>::N];
#pragma unroll
    for (int e = 0; e < Vec16<T>::N; ++e) {
      const int n = n0 + e;
      float v = acc[n];
      if (a.scale) v *= a.scale[n];
      if (a.shift) v += a.shift[n];
      o[e] = v > 0.f ? v : v * a.slope;
    }
    store16_f(y + n0, o);
  }
}

// bf16 with a 4-channel input (RGB + zero, 8-byte pixels): K = 4 rows x (4 taps x 4 channels) =
// 64 = two MFMA k-steps; a lane's 8 K values are two horizontally adjacent input pixels, so a
// 16-pixel B fragment is gathered with two 8-byte loads per lane and k-step (no im2col).
// Weights are the A operand (rows = output channels): lanes then hold 4 channels of one pixel.
struct FirstMfmaArgs {
  const void* x;      // [B][Hi][Wi][4]
  const void* w;      // packed [Npad][Kpad], K = (ky*4 + kx)*3 + c
  void* y;
  const float* scale;
  const float* shift;
  int Hi, Wi, Ho, Wo, Kpad, ldy;
  float slope;
  long M;
};

// each wave walks kFirstChunks runs of 64 output pixels: the weight fragments (32 gathered T per
// lane) and the BN scale/shift are set up once per wave, not once per 64 pixels (measured 81 us at
// 256x256, B = 64, with one run per wave: 1.2 TB/s for a 100 MB HBM kernel)
constexpr int kFirstChunks = 4;

template <typename T>
__global__ void __launch_bounds__(256) conv_first_mfma_kernel(const FirstMfmaArgs a) {
  const T* __restrict__ aw = reinterpret_cast<const T*>(a.w);
  const int lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wave * kFirstChunks * 64 >= a.M) return;
  // A fragments: channel rows n = 16j + lr, K = 32s + 8lq + e -> (ky, kx, c4) = (K/16, K/4 % 4, K % 4)
  v8_t<T> wf[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      T e8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = s * 32 + lq * 8 + e, ky = k >> 4, kx = (k >> 2) & 3, c4 = k & 3;
        e8[e] = c4 < 3 ? aw[(long)(j * 16 + lr) * a.Kpad + (ky * 4 + kx) * 3 + c4] : (T)0.f;
      }
      __builtin_memcpy(&wf[j][s], e8, 16);
    }
  float sc[2][4], sh[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = j * 16 + lq * 4 + r;
      sc[j][r] = a.scale ? a.scale[n] : 1.f;
      sh[j][r] = a.shift ? a.shift[n] : 0.f;
    }
  const int hw = a.Ho * a.Wo;
  for (int ch = 0; ch < kFirstChunks; ++ch) {
  const long m0 = (wave * kFirstChunks + ch) * 64;   // 64 pixels of one output row
  if (m0 >= a.M) break;
  const int b = (int)(m0 / hw);
  const int r0 = (int)(m0 - (long)b * hw);
  const int oy = r0 / a.Wo, ox0 = r0 - oy * a.Wo;
  const T* xb = reinterpret_cast<const T*>(a.x) + (long)b * a.Hi * a.Wi * 4;
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ox = ox0 + i * 16 + lr;
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ky = 2 * s + (lq >> 1), half = lq & 1;
      const int iy = 2 * oy - 1 + ky, ix = 2 * ox - 1 + 2 * half;   // pixels ix, ix + 1
      uint2 p0 = {0u, 0u}, p1 = {0u, 0u};
      if (iy >= 0 && iy < a.Hi) {
        const T* row = xb + (long)iy * a.Wi * 4;
        if (ix >= 0) p0 = *reinterpret_cast<const uint2*>(row + ix * 4);
        if (ix + 1 < a.Wi) p1 = *reinterpret_cast<const uint2*>(row + (ix + 1) * 4);
      }
      const u32x4 raw = {p0.x, p0.y, p1.x, p1.y};
      v8_t<T> bfrag;
      __builtin_memcpy(&bfrag, &raw, 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j][i] = mfma16x16x32<T>(wf[j][s], bfrag, acc[j][i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long m = m0 + i * 16 + lr;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = j * 16 + lq * 4;
      uint2 o;
      T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = fmaf(acc[j][i][r], sc[j][r], sh[j][r]);
        oe[r] = (T)(v > 0.f ? v : v * a.slope);
      }
      *reinterpret_cast<uint2*>(reinterpret_cast<T*>(a.y) + m * a.ldy + n) = o;
    }
  }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) first_weights_kernel(const T* __restrict__ w, int Kpad, int N, float* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < N * 48) out[i] = to_f(w[(long)(i / 48) * Kpad + i % 48]);
}

bool conv_first_supported(const ConvDesc& d) {
  return d.kind == CONV_FWD && d.kh == 4 && d.kw == 4 && d.stride == 2 && d.pad == 1 && d.Cin == 3 &&
         d.N == 32 && d.ti == d.to && (is16(d.ti) || d.ti == GHOST_F32) && d.epi == EPI_STD && !d.res && !d.prelu && !d.y2 &&
         !d.tanh_out && !d.u8 && d.ldy % (d.to == GHOST_F32 ? 4 : 8) == 0 && (uintptr_t)d.y % 16 == 0 &&
         d.Kpad >= 48 && !d.force_split;
}

size_t conv_first_workspace_bytes() { return 32 * 48 * sizeof(float); }

int conv_first(const ConvDesc& d, void* ws, size_t ws_bytes, hipStream_t s) {
  if (!conv_first_supported(d)) return -1;
  const int Ho = (d.Hi + 2 - 4) / 2 + 1, Wo = (d.Wi + 2 - 4) / 2 + 1;
  if (is16(d.ti) && d.ldx == 4 && Wo % 64 == 0 && d.ldy % 4 == 0 && (uintptr_t)d.x % 8 == 0) {
    FirstMfmaArgs m{};
    m.x = d.x; m.w = d.w; m.y = d.y; m.scale = d.scale; m.shift = d.shift;
    m.Hi = d.Hi; m.Wi = d.Wi; m.Ho = Ho; m.Wo = Wo; m.Kpad = d.Kpad; m.ldy = d.ldy; m.slope = d.slope;
    m.M = (long)d.B * Ho * Wo;
    const dim3 g((unsigned)(((m.M / 64 + kFirstChunks - 1) / kFirstChunks + 3) / 4));
    if (d.ti == GHOST_BF16)
      hipLaunchKernelGGL(conv_first_mfma_kernel<bf16>, g, dim3(256), 0, s, m);
    else
      hipLaunchKernelGGL(conv_first_mfma_kernel<_Float16>, g, dim3(256), 0, s, m);
    return (int)hipGetLastError();
  }
  if (!ws || ws_bytes < conv_first_workspace_bytes() || (uintptr_t)ws % 16) return -1;
  float* wf = reinterpret_cast<float*>(ws);
  if (d.ti == GHOST_BF16)
    hipLaunchKernelGGL(first_weights_kernel<bf16>, dim3(6), dim3(256), 0, s, (const bf16*)d.w, d.Kpad, 32, wf);
  else if (d.ti == GHOST_F16)
    hipLaunchKernelGGL(first_weights_kernel<_Float16>, dim3(6), dim3(256), 0, s, (const _Float16*)d.w, d.Kpad, 32, wf);
  else
    hipLaunchKernelGGL(first_weights_kernel<float>, dim3(6), dim3(256), 0, s, (const float*)d.w, d.Kpad, 32, wf);
  FirstArgs a{};
  a.x = d.x; a.w = wf; a.y = d.y; a.scale = d.scale; a.shift = d.shift;
  a.Hi = d.Hi; a.Wi = d.Wi; a.ldx = d.ldx;
  a.Ho = (d.Hi + 2 - 4) / 2 + 1;
  a.Wo = (d.Wi + 2 - 4) / 2 + 1;
  a.Kpad = d.Kpad; a.ldy = d.ldy; a.slope = d.slope;
  a.M = (long)d.B * a.Ho * a.Wo;
  dim3 grid((unsigned)((a.M + 255) / 256));
  if (d.ti == GHOST_BF16)
    hipLaunchKernelGGL((conv_first_kernel<bf16, 32>), grid, dim3(256), 0, s, a);
  else if (d.ti == GHOST_F16)
    hipLaunchKernelGGL((conv_first_kernel<_Float16, 32>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv_first_kernel<float, 32>), grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// ArcFace stem: Conv2d(3, 64, 3, s1, p1) + BN + PReLU (+ the next block's BN as a second output),
// on the same 4-channel (RGB + zero) input layout (arc_runtime.hip: stem).  K = 9 taps x 4 channels
// = 36, two MFMA k-steps (taps 8s + 2lq, +1 per lane; taps >= 9 are zero): a lane's 8 K values are
// two taps of one output pixel, gathered as two 8-byte pixel loads.  The implicit GEMM takes this
// shape on its scalar-gather path (Cin = 3): 127 us at B = 64 for 12 MB read + 206 MB written.
// ---------------------------------------------------------------------------
struct StemArgs {
  const bf16* x;      // [B][H][W][4]
  const bf16* w;      // packed [Npad][Kpad], K = (ky*3 + kx)*3 + c
  bf16* y;
  bf16* y2;
  const float* scale;
  const float* shift;
  const float* prelu;
  const float* scale2;
  const float* shift2;
  int H, W, Kpad, ldy, ldy2;
  float slope;
  int M;
};

constexpr int kStemChunks = 4;

__global__ void __launch_bounds__(256) conv_stem3x3_kernel(const StemArgs a) {
  const int lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  // the 64 x 27 weights and the five per-channel tables, staged once per workgroup (the per-lane
  // gathers of the fragments below then hit LDS, not 64 scattered global loads per lane)
  __shared__ bf16 s_w[64 * 28];
  __shared__ float s_t[5][64];
  for (int i = threadIdx.x; i < 64 * 28; i += 256) {
    const int n = i / 28, k = i - n * 28;
    s_w[i] = k < 27 ? a.w[(long)n * a.Kpad + k] : (bf16)0.f;
  }
  if (threadIdx.x < 64) {
    const int n = threadIdx.x;
    s_t[0][n] = a.scale ? a.scale[n] : 1.f;
    s_t[1][n] = a.shift ? a.shift[n] : 0.f;
    s_t[2][n] = a.prelu ? a.prelu[n] : a.slope;
    s_t[3][n] = a.y2 ? a.scale2[n] : 0.f;
    s_t[4][n] = a.y2 ? a.shift2[n] : 0.f;
  }
  __syncthreads();
  if (wave * kStemChunks * 64 >= a.M) return;
  // A fragments: rows n = 16j + lr; K = 32s + 8lq + e -> tap = 8s + 2lq + (e >> 2), c = e & 3
  bf16x8 wf[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16 e8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int tap = 8 * s + 2 * lq + (e >> 2), c = e & 3;
        e8[e] = (tap < 9 && c < 3) ? s_w[(j * 16 + lr) * 28 + tap * 3 + c] : (bf16)0.f;
      }
      __builtin_memcpy(&wf[j][s], e8, 16);
    }
  // this lane's 4 channels of each j: n = 16j + 4lq + r
  float sc[4][4], sh[4][4], pr[4][4], sc2[4][4], sh2[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = j * 16 + lq * 4 + r;
      sc[j][r] = s_t[0][n];
      sh[j][r] = s_t[1][n];
      pr[j][r] = s_t[2][n];
      sc2[j][r] = s_t[3][n];
      sh2[j][r] = s_t[4][n];
    }
  // 32-bit pixel indices (M < 2^31, checked on the host): a 64-bit division per lane and fragment
  // cost more than the MFMAs
  const int hw = a.H * a.W;
  for (int ch = 0; ch < kStemChunks; ++ch) {
    const int m0 = (int)((wave * kStemChunks + ch) * 64);
    if (m0 >= a.M) break;
    const int b0 = m0 / hw, rb = m0 - b0 * hw;       // a 64-pixel chunk spans at most two samples
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + i * 16 + lr;                // this lane's B-fragment pixel
      const bool mok = m < a.M;
      int r0 = rb + i * 16 + lr, b = b0;
      if (r0 >= hw) { r0 -= hw; ++b; }
      const int oy = r0 / a.W, ox = r0 - oy * a.W;
      const bf16* xb = a.x + (long)b * hw * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint2 p[2] = {{0u, 0u}, {0u, 0u}};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tap = 8 * s + 2 * lq + h;
          const int iy = oy + tap / 3 - 1, ix = ox + tap % 3 - 1;
          if (mok && tap < 9 && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
            p[h] = *reinterpret_cast<const uint2*>(xb + ((long)iy * a.W + ix) * 4);
        }
        const u32x4 raw = {p[0].x, p[0].y, p[1].x, p[1].y};
        bf16x8 bfrag;
        __builtin_memcpy(&bfrag, &raw, 16);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], bfrag, acc[j][i], 0, 0, 0);
      }
    }
    // epilogue (conv_igemm.hip epi_std / store_std order): v = acc*scale + shift, PReLU, y = v,
    // y2 = v*scale2 + shift2; lane holds channels 16j + 4lq + r of pixel m0 + 16i + lr
    // (measured: staging the tile through LDS for whole-row stores is slower, 95 vs 88 us)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + i * 16 + lr;
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = j * 16 + lq * 4;
        uint2 o, o2;
        bf16* oe = reinterpret_cast<bf16*>(&o);
        bf16* oe2 = reinterpret_cast<bf16*>(&o2);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = fmaf(acc[j][i][r], sc[j][r], sh[j][r]);
          v = v > 0.f ? v : v * pr[j][r];
          oe[r] = (bf16)v;
          oe2[r] = (bf16)(v * sc2[j][r] + sh2[j][r]);
        }
        *reinterpret_cast<uint2*>(a.y + (long)m * a.ldy + n) = o;
        if (a.y2) *reinterpret_cast<uint2*>(a.y2 + (long)m * a.ldy2 + n) = o2;
      }
    }
  }
}

bool conv_stem3x3_supported(const ConvDesc& d) {
  return d.kind == CONV_FWD && d.kh == 3 && d.kw == 3 && d.stride == 1 && d.pad == 1 && d.Cin == 3 && d.ldx == 4 &&
         d.N == 64 && d.ti == GHOST_BF16 && d.to == GHOST_BF16 && d.epi == EPI_STD && !d.res && !d.res_first &&
         !d.tanh_out && !d.u8 && !d.force_split && d.Kpad >= 27 && d.Npad >= 64 && d.ldy % 4 == 0 &&
         (uintptr_t)d.x % 8 == 0 && (uintptr_t)d.y % 8 == 0 && (long)d.B * d.Hi * d.Wi < (1L << 30) &&
         (!d.y2 || (d.scale2 && d.shift2 && d.ldy2 % 4 == 0 && (uintptr_t)d.y2 % 8 == 0));
}

int conv_stem3x3(const ConvDesc& d, hipStream_t s) {
  if (!conv_stem3x3_supported(d)) return -1;
  StemArgs a{};
  a.x = (const bf16*)d.x; a.w = (const bf16*)d.w; a.y = (bf16*)d.y; a.y2 = (bf16*)d.y2;
  a.scale = d.scale; a.shift = d.shift; a.prelu = d.prelu; a.scale2 = d.scale2; a.shift2 = d.shift2;
  a.H = d.Hi; a.W = d.Wi; a.Kpad = d.Kpad; a.ldy = d.ldy; a.ldy2 = d.ldy2; a.slope = d.slope;
  a.M = d.B * d.Hi * d.Wi;
  const long waves = ((long)(a.M + 63) / 64 + kStemChunks - 1) / kStemChunks;
  hipLaunchKernelGGL(conv_stem3x3_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace ghost
