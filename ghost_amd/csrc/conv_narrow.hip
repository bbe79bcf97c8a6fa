// ghost_amd — 3x3 convolution to <= 3 output channels (the generator's last conv,
// AADBlk8 64->3 / fused cat 128->3, AADLayer.py:64,71 + tanh of AEI_Net.py:139).
//
// A GEMM with N = 3 wastes 13/16 of every MFMA column and re-reads each input pixel for
// all nine taps.  Instead each workgroup takes an 8 x 32 output tile and its 10 x 34 halo:
//   Z[p][t*NO + o] = sum_c x[p][c] * w[o][c][t]          (t = tap; 9*NO <= 32 columns; MFMA)
//   out[q][o]      = sum_t Z[q + off_t][t*NO + o]         (LDS gather, fp32)
// so every input pixel is read ~1.33 times (halo) and the MFMA work shrinks 4.5x.
// Epilogue: optional residual, tanh, and the BGR uint8 copy of faceshifter_run.py:20-21.
#include "conv_narrow.h"
#include "ghost_common.h"
#include "tap_rows.h"

namespace ghost {

namespace {
constexpr int TH = 8, TW = 32;               // output tile
constexpr int HH = TH + 2, HW_ = TW + 2;     // halo tile
constexpr int HP = HH * HW_;                 // 340 halo pixels
constexpr int NRT = (HP + 15) / 16;          // 22 row tiles of 16 pixels
constexpr int ZLD = 33;                      // padded LDS row (32 columns)
}  // namespace

struct NarrowArgs {
  const void* x;
  const void* w;          // [32][Kpad]: column n = t*NO + o, K = input channel
  const void* res;
  void* y;
  uint8_t* u8;
  const _Float16* zadd;   // optional tap partials of other input channels (tap_rows.h), added to the sums
  int H, W, Cin, ldx, Kpad, ldy, ldres, NO, tanh_out;
};

template <typename T, int CIN>
__global__ void __launch_bounds__(256) conv3x3_narrow_kernel(const NarrowArgs a) {
  __shared__ float Z[NRT * 16 * ZLD];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int tiles_x = a.W / TW, tiles_y = a.H / TH;
  const int b = blockIdx.x / (tiles_x * tiles_y);
  const int r = blockIdx.x - b * tiles_x * tiles_y;
  const int y0 = (r / tiles_x) * TH, x0 = (r % tiles_x) * TW;
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);
  const long img = (long)b * a.H * a.W;

  if constexpr (CIN > 0) {
    // 16-bit storage, Cin known: the weight fragments stay in registers and each lane issues the loads of
    // two row tiles (2 * CIN/32 x 16 B) before their MFMAs, so the HBM latency overlaps
    v8_t<T> wf0[CIN / 32], wf1[CIN / 32];
#pragma unroll
    for (int k = 0; k < CIN / 32; ++k) {
      const u32x4 b0 = *reinterpret_cast<const u32x4*>(w + (long)lr * a.Kpad + k * 32 + lq * 8);
      const u32x4 b1 = *reinterpret_cast<const u32x4*>(w + (long)(16 + lr) * a.Kpad + k * 32 + lq * 8);
      __builtin_memcpy(&wf0[k], &b0, 16);
      __builtin_memcpy(&wf1[k], &b1, 16);
    }
    for (int rt = wid; rt < NRT; rt += 8) {
      u32x4 av[2][CIN / 32];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = (rt + 4 * u) * 16 + lr;
        const int hy = p / HW_, hx = p - hy * HW_;
        const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
        const bool ok = rt + 4 * u < NRT && p < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const T* xp = x + (img + (long)(ok ? iy : 0) * a.W + (ok ? ix : 0)) * a.ldx + lq * 8;
#pragma unroll
        for (int k = 0; k < CIN / 32; ++k)
          av[u][k] = ok ? *reinterpret_cast<const u32x4*>(xp + k * 32) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (rt + 4 * u >= NRT) break;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < CIN / 32; ++k) {
          v8_t<T> af;
          __builtin_memcpy(&af, &av[u][k], 16);
          acc0 = mfma16x16x32<T>(af, wf0[k], acc0);
          acc1 = mfma16x16x32<T>(af, wf1[k], acc1);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = (rt + 4 * u) * 16 + lq * 4 + i;
          Z[row * ZLD + lr] = acc0[i];
          Z[row * ZLD + 16 + lr] = acc1[i];
        }
      }
    }
  } else {
    for (int rt = wid; rt < NRT; rt += 4) {
      // this lane's halo pixel (A row) for the tile
      const int p = rt * 16 + lr;
      const int hy = p / HW_, hx = p - hy * HW_;
      const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
      const bool ok = p < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const T* xp = x + (img + (long)(ok ? iy : 0) * a.W + (ok ? ix : 0)) * a.ldx;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (sizeof(T) == 2) {
        for (int k0 = 0; k0 < a.Cin; k0 += 32) {
          u32x4 av = ok ? *reinterpret_cast<const u32x4*>(xp + k0 + lq * 8) : u32x4{0u, 0u, 0u, 0u};
          const u32x4 b0 = *reinterpret_cast<const u32x4*>(w + (long)lr * a.Kpad + k0 + lq * 8);
          const u32x4 b1 = *reinterpret_cast<const u32x4*>(w + (long)(16 + lr) * a.Kpad + k0 + lq * 8);
          v8_t<T> af, bf0, bf1;
          __builtin_memcpy(&af, &av, 16);
          __builtin_memcpy(&bf0, &b0, 16);
          __builtin_memcpy(&bf1, &b1, 16);
          acc0 = mfma16x16x32<T>(af, bf0, acc0);
          acc1 = mfma16x16x32<T>(af, bf1, acc1);
        }
      } else {
        for (int k0 = 0; k0 < a.Cin; k0 += 16) {
          const f32x4 av = ok ? *reinterpret_cast<const f32x4*>(xp + k0 + lq * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
          const f32x4 b0 = *reinterpret_cast<const f32x4*>(w + (long)lr * a.Kpad + k0 + lq * 4);
          const f32x4 b1 = *reinterpret_cast<const f32x4*>(w + (long)(16 + lr) * a.Kpad + k0 + lq * 4);
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], b0[e], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], b1[e], acc1, 0, 0, 0);
          }
        }
      }
      // C layout: column = lane&15, rows (lane>>4)*4 + i
  #pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rt * 16 + lq * 4 + i;
        Z[row * ZLD + lr] = acc0[i];
        Z[row * ZLD + 16 + lr] = acc1[i];
      }
    }
  }
  __syncthreads();
  // gather: one output pixel per thread
  const int oy = tid / TW, ox = tid - oy * TW;
  const long q = img + (long)(y0 + oy) * a.W + (x0 + ox);
  // tap partials of the channels a producer already contracted (AADBlk8's h path; row sums, tap_rows.h)
  float zs[3] = {0.f, 0.f, 0.f};
  if (a.zadd) zr_gather(a.zadd + (long)b * zr_image(a.H * a.W), a.H, a.W, y0 + oy, x0 + ox, zs);
  for (int o = 0; o < a.NO; ++o) {
    float s = 0.f;
#pragma unroll
    for (int ty = 0; ty < 3; ++ty)
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) s += Z[((oy + ty) * HW_ + ox + tx) * ZLD + (ty * 3 + tx) * a.NO + o];
    s += zs[o < 3 ? o : 0];
    if (a.res) s += to_f(reinterpret_cast<const T*>(a.res)[q * a.ldres + o]);
    if (a.tanh_out) s = tanhf(s);
    reinterpret_cast<T*>(a.y)[q * a.ldy + o] = from_f<T>(s);
    if (a.u8) {
      const float t = (s * 0.5f + 0.5f) * 255.0f;   // faceshifter_run.py:20-21
      a.u8[q * 3 + (2 - o)] = (uint8_t)(int)t;
    }
  }
}

bool conv3x3_narrow_supported(int dt, int H, int W, int Cin, int ldx, int NO) {
  const int vec = dt == GHOST_F32 ? 4 : 8;
  return NO >= 1 && NO <= 3 && H % TH == 0 && W % TW == 0 && Cin % 32 == 0 && ldx % vec == 0;
}

int conv3x3_narrow(int dt, const void* x, int B, int H, int W, int Cin, int ldx, const void* w_narrow, int Kpad, int NO,
                   const void* res, int ldres, int tanh_out, void* y, int ldy, uint8_t* u8, hipStream_t s,
                   const void* zadd) {
  if (!conv3x3_narrow_supported(dt, H, W, Cin, ldx, NO) || (uintptr_t)x % 16 || (uintptr_t)w_narrow % 16) return -1;
  if (zadd && ((uintptr_t)zadd % 16 || NO != 3 || W % 8)) return -1;
  NarrowArgs a{x, w_narrow, res, y, u8, (const _Float16*)zadd, H, W, Cin, ldx, Kpad, ldy, ldres, NO, tanh_out};
  dim3 grid((unsigned)(B * (H / TH) * (W / TW)));
#define GHOST_NARROW(T)                                                   \
  if (Cin == 128)                                                         \
    hipLaunchKernelGGL((conv3x3_narrow_kernel<T, 128>), grid, dim3(256), 0, s, a); \
  else if (Cin == 64)                                                     \
    hipLaunchKernelGGL((conv3x3_narrow_kernel<T, 64>), grid, dim3(256), 0, s, a);  \
  else                                                                    \
    hipLaunchKernelGGL((conv3x3_narrow_kernel<T, 0>), grid, dim3(256), 0, s, a);
  if (dt == GHOST_BF16) {
    GHOST_NARROW(bf16)
  } else if (dt == GHOST_F16) {
    GHOST_NARROW(_Float16)
  } else if (dt == GHOST_F32)
    hipLaunchKernelGGL((conv3x3_narrow_kernel<float, 0>), grid, dim3(256), 0, s, a);
  else
    return -1;
#undef GHOST_NARROW
  return (int)hipGetLastError();
}

}  // namespace ghost
