// ghost_amd — Conv2d 4x4/s2/p1 + BN(eval) + LeakyReLU for Cin % 32 == 0 (MLAttrEncoder conv2..conv4,
// AEI_Net.py:19-24,48-53) on gfx950.
//
// Why not the implicit GEMM: a 4x4/s2 conv reads every input pixel for 4 output pixels (16 taps over a
// stride-2 grid), so the im2col rows the GEMM gathers move 4x the input through L2 in 64-byte pieces, and
// with N = 64..256 the weight tile is re-streamed per 128 output pixels: conv2..conv4 ran at 0.11-0.15 of
// the bf16 MFMA peak, L2-bound (88 / 56 / 54 us at B = 64).
//
// Here a workgroup (4 waves) owns an 8 x 16 output tile and 64 output channels.  Per 32-channel block it
// DMAs the tile's 18 x 34 input patch into LDS once (LDS-DMA, border pixels from a zero line), split by
// column parity into two planes so that the 16 output columns of one tap read 16 consecutive 64-byte pixel
// slots (conflict-free with the slot-indexed chunk swizzle); the weights stream through a double buffer in
// K steps of one kernel row (4 taps x 32 channels x 64 rows = 16 KB, row-swizzled).  Each wave owns two
// output rows: per tap 2 patch fragments + 4 weight fragments feed 8 v_mfma_f32_16x16x32_bf16 in the
// transposed form (rows = output channels), so a lane ends with 4 consecutive channels of one pixel and the
// BN + LeakyReLU epilogue stores 8 bytes per (pixel, 4 channels).
//
// The same plan with K = 3 serves IResNet's 3x3/s2/p1 convs (the conv2 of each layer's first IBasicBlock,
// arc_runtime.hip; arcface_torch iresnet.py): a 17 x 33 patch per 8 x 16 output tile, K steps of one kernel
// row (3 taps x 32 channels), and the IBasicBlock epilogue (BN, optional PReLU, the downsampled residual,
// the next block's BatchNorm as a second output), tiles overhanging the 56 / 28 / 14 output images masked.
// On the implicit GEMM these ran at 160 TF/s (B = 128: 185 us for 29.6 GFLOP at 112 -> 56).
#include <hip/hip_runtime.h>

#include "conv_s2.h"
#include "ghost_common.h"

namespace ghost {
namespace {

constexpr int TH = 8, TW = 16;                    // output tile: 8 rows x 16 columns
constexpr int PJ = TW + 1;                        // 17 pixels per column-parity plane row (34 / 33 columns)
constexpr int BN = 64;                            // output channels per workgroup
constexpr int W_BYTES = BN * 256;                 // one K step: 64 rows x 16 chunk positions of 16 bytes
template <int K>
struct S2Geo {
  static constexpr int PR = 2 * TH + K - 2;                    // patch rows: 18 (K = 4), 17 (K = 3)
  static constexpr int PSLOTS = PR * 2 * PJ;                   // pixel slots of 64 bytes (32 channels)
  static constexpr int P_INSTR = (PSLOTS * 4 + 63) / 64;       // LDS-DMA wave instructions per patch
  static constexpr int P_BYTES = P_INSTR * 1024;               // (the last instruction's tail lands in padding)
  static constexpr int WCH = 4 * K;                            // weight chunks per row and K step (K taps x 32)
};

__device__ __attribute__((aligned(16))) unsigned int s2_zero_line[16] = {0};

struct S2Args {
  const void* x;
  const void* w;
  void* y;
  const float* scale;
  const float* shift;
  int Hi, Wi, ldx, Ho, Wo, ldy, Kpad, ncb, tiles_x, tiles_per_img;
  float slope;
  // K = 3 (IBasicBlock) epilogue: per-channel PReLU slope, residual (before the activation when res_first),
  // second output y2 = v * scale2 + shift2
  const float* prelu;
  const void* res;
  int ldres, res_first;
  void* y2;
  int ldy2;
  const float* scale2;
  const float* shift2;
};

template <int N>
GHOST_DEV void s2_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename T, int K>
__global__ void __launch_bounds__(256) conv_s2_patch_kernel(const S2Args a) {
  using Geo = S2Geo<K>;
  constexpr int PSLOTS = Geo::PSLOTS, P_INSTR = Geo::P_INSTR;
  __shared__ __attribute__((aligned(1024))) unsigned char s_p[Geo::P_BYTES];
  __shared__ __attribute__((aligned(1024))) unsigned char s_w[2 * W_BYTES];
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, lr = lane & 15,
            lq = lane >> 4;
  // neighbouring tiles share patch rows: keep them on one XCD's L2
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int b = tile / a.tiles_per_img, t = tile - b * a.tiles_per_img;
  const int tyi = t / a.tiles_x, txi = t - tyi * a.tiles_x;
  const int oy0 = tyi * TH, ox0 = txi * TW;
  const int n0 = blockIdx.y * BN;
  const T* __restrict__ xb = reinterpret_cast<const T*>(a.x) + (long)b * a.Hi * a.Wi * a.ldx;
  const int iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;

  // patch of channel block cb: slot = (patch row * 2 + column parity) * 17 + column / 2; the 16-byte chunk
  // kc of a slot is stored at position kc ^ ((slot >> 2) & 3)
  auto issue_patch = [&](int cb) {
#if defined(__HIP_DEVICE_COMPILE__)
    for (int i = wid; i < P_INSTR; i += 4) {
      const int slot = i * 16 + (lane >> 2), pos = lane & 3;
      const void* src = s2_zero_line;
      if (slot < PSLOTS) {
        const int pr = slot / (2 * PJ), rem = slot - pr * (2 * PJ);
        const int q = rem >= PJ ? 1 : 0, j = rem - q * PJ;
        const int iy = iy0 + pr, ix = ix0 + 2 * j + q;
        const int kc = pos ^ ((slot >> 2) & 3);
        if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi) src = xb + ((long)iy * a.Wi + ix) * a.ldx + cb * 32 + kc * 8;
      }
      __builtin_amdgcn_global_load_lds(src, s_p + i * 1024, 16, 0, 0);
    }
#endif
  };
  // weights of K step s = (cb, kernel row ky): row n holds taps (ky, 0..K-1) x 32 channels = 4K chunks, chunk c
  // stored at position c ^ (n & 15) of a 16-position row; four 1 KB instructions per wave (K = 3: the lanes whose
  // chunk would be 12..15 idle, so no row reads past its K step)
  auto issue_w = [&](int s, int buf) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int cb = s / K, ky = s - cb * K;
    const T* wsrc = reinterpret_cast<const T*>(a.w) + (long)n0 * a.Kpad + (cb * K * K + ky * K) * 32;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = wid * 4 + k;
      const int n = i * 4 + (lane >> 4), p = lane & 15, c = p ^ (n & 15);   // lane -> position p, chunk c
      if (K == 4 || c < Geo::WCH)
        __builtin_amdgcn_global_load_lds(wsrc + (long)n * a.Kpad + c * 8, s_w + buf * W_BYTES + i * 1024, 16, 0, 0);
    }
#endif
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int S = a.ncb * K;
  issue_patch(0);
  issue_w(0, 0);
  for (int s = 0; s < S; ++s) {
    const bool more = s + 1 < S;
    if (more) {
      issue_w(s + 1, (s + 1) & 1);   // its buffer was last read in step s - 1 (behind the barrier below)
      s2_wait_vmcnt<4>();            // everything but the 4 instructions just issued
    } else {
      s2_wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int ky = s % K;
    const unsigned char* wb = s_w + (s & 1) * W_BYTES;
#pragma unroll
    for (int tx = 0; tx < K; ++tx) {
      v8_t<T> wf[4], pf[2];
#pragma unroll
      for (int j = 0; j < 4; ++j)   // row n = 16 j + lr, so n & 15 == lr
        wf[j] = *reinterpret_cast<const v8_t<T>*>(wb + (j * 16 + lr) * 256 + (((tx * 4 + lq) ^ lr) << 4));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pr = 2 * (2 * wid + i) + ky;
        const int slot = (pr * 2 + (tx & 1)) * PJ + lr + (tx >> 1);
        pf[i] = *reinterpret_cast<const v8_t<T>*>(s_p + slot * 64 + ((lq ^ ((slot >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32<T>(wf[j], pf[i], acc[i][j]);
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave is done with this step's weight buffer (and, at ky = K-1, the patch)
    if (ky == K - 1 && more) issue_patch(s / K + 1);
  }

  // epilogue: lane holds channels n0 + 16 j + 4 lq + r of pixel (oy0 + 2 wid + i, ox0 + lr)
  const T* __restrict__ res = reinterpret_cast<const T*>(a.res);
  T* __restrict__ y2 = reinterpret_cast<T*>(a.y2);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oy = oy0 + 2 * wid + i, ox = ox0 + lr;
    if (K == 3 && (oy >= a.Ho || ox >= a.Wo)) continue;   // tiles overhanging the image (K = 4: exact tiles)
    const long pix = ((long)b * a.Ho + oy) * a.Wo + ox;
    T* yp = reinterpret_cast<T*>(a.y) + pix * a.ldy + n0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = j * 16 + lq * 4;
      float4 sc = a.scale ? *reinterpret_cast<const float4*>(a.scale + n0 + n) : float4{1.f, 1.f, 1.f, 1.f};
      float4 sh = a.shift ? *reinterpret_cast<const float4*>(a.shift + n0 + n) : float4{0.f, 0.f, 0.f, 0.f};
      float v[4] = {fmaf(acc[i][j][0], sc.x, sh.x), fmaf(acc[i][j][1], sc.y, sh.y), fmaf(acc[i][j][2], sc.z, sh.z),
                    fmaf(acc[i][j][3], sc.w, sh.w)};
      float rv[4] = {0.f, 0.f, 0.f, 0.f};
      float sl[4] = {a.slope, a.slope, a.slope, a.slope};
      if constexpr (K == 3) {
        if (res) {
          const uint2 rr = *reinterpret_cast<const uint2*>(res + pix * a.ldres + n0 + n);
          const T* e = reinterpret_cast<const T*>(&rr);
#pragma unroll
          for (int r = 0; r < 4; ++r) rv[r] = (float)e[r];
        }
        if (a.prelu) {
          const float4 pr = *reinterpret_cast<const float4*>(a.prelu + n0 + n);
          sl[0] = pr.x; sl[1] = pr.y; sl[2] = pr.z; sl[3] = pr.w;
        }
      }
      unsigned short o[4], o2[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // conv_igemm.hip epi_std's order: BN, (residual first), activation, residual
        float u = v[r];
        if (K == 3 && a.res_first) u += rv[r];
        u = u > 0.f ? u : u * sl[r];
        if (K == 3 && !a.res_first) u += rv[r];
        o[r] = __builtin_bit_cast(unsigned short, (T)u);
        if (K == 3 && y2) {
          const float s2 = a.scale2[n0 + n + r], t2 = a.shift2[n0 + n + r];
          o2[r] = __builtin_bit_cast(unsigned short, (T)(u * s2 + t2));
        }
      }
      uint2 pk = {(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
      *reinterpret_cast<uint2*>(yp + n) = pk;
      if (K == 3 && y2) {
        uint2 pk2 = {(unsigned)o2[0] | ((unsigned)o2[1] << 16), (unsigned)o2[2] | ((unsigned)o2[3] << 16)};
        *reinterpret_cast<uint2*>(y2 + pix * a.ldy2 + n0 + n) = pk2;
      }
    }
  }
}

}  // namespace

bool conv4x4s2_patch_supported(const ConvDesc& d) {
  if (d.kind != CONV_FWD || d.kh != 4 || d.kw != 4 || d.stride != 2 || d.pad != 1) return false;
  if (!is16(d.ti) || d.to != d.ti || d.epi != EPI_STD) return false;
  if (d.res || d.prelu || d.y2 || d.tanh_out || d.u8 || d.in_part || d.force_split) return false;
  if (d.Cin % 32 || d.ldx % 8 || (uintptr_t)d.x % 16 || d.N % BN || d.Npad < d.N || d.Kpad < 16 * d.Cin) return false;
  if (d.Hi % 2 || d.Wi % 2) return false;
  const int Ho = d.Hi / 2, Wo = d.Wi / 2;
  if (Ho % TH || Wo % TW || d.ldy % 4 || (uintptr_t)d.y % 8) return false;
  if ((uintptr_t)d.scale % 16 || (uintptr_t)d.shift % 16) return false;
  // one workgroup per output tile and 64 channels, the whole reduction each: under 32 of them (B = 1: the 16 x 16 and
  // 32 x 32 outputs, 8 and 16 workgroups, 27 and 15 us) the implicit GEMM's split K spreads the conv wider
  if ((long)d.B * (Ho / TH) * (Wo / TW) * (d.N / BN) < 32) return false;
  return (long)d.Hi * d.Wi * d.ldx < (1L << 31);
}

// 3x3/s2/p1 (IResNet): the output is Hi/2 x Wi/2; tiles may overhang it, but only where at least 3/4 of the
// tile pixels are real (56 / 28 / 14: 77-88 %; the 7 x 7 output of a 14 x 14 input stays on the implicit GEMM)
bool conv3x3s2_patch_supported(const ConvDesc& d) {
  if (d.kind != CONV_FWD || d.kh != 3 || d.kw != 3 || d.stride != 2 || d.pad != 1) return false;
  if (!is16(d.ti) || d.to != d.ti || d.epi != EPI_STD) return false;
  if (d.tanh_out || d.u8 || d.in_part || d.force_split) return false;
  if (d.Cin % 32 || d.ldx % 8 || (uintptr_t)d.x % 16 || d.N % BN || d.Npad < d.N || d.Kpad < 9 * d.Cin) return false;
  if (d.Hi % 2 || d.Wi % 2) return false;
  const long Ho = d.Hi / 2, Wo = d.Wi / 2;
  const long tiles = ((Ho + TH - 1) / TH) * ((Wo + TW - 1) / TW);
  if (4 * Ho * Wo < 3 * tiles * TH * TW) return false;
  if (d.ldy % 4 || (uintptr_t)d.y % 8) return false;
  if ((uintptr_t)d.scale % 16 || (uintptr_t)d.shift % 16 || (uintptr_t)d.prelu % 16) return false;
  if (d.res && (d.ldres % 4 || (uintptr_t)d.res % 8)) return false;
  if (d.y2 && (d.ldy2 % 4 || (uintptr_t)d.y2 % 8 || !d.scale2 || !d.shift2)) return false;
  return (long)d.Hi * d.Wi * d.ldx < (1L << 31) && (long)d.B * Ho * Wo * d.ldy < (1L << 31);
}

int conv_s2_patch(const ConvDesc& d, hipStream_t s) {
  const int K = d.kh;
  if (K == 4 ? !conv4x4s2_patch_supported(d) : !conv3x3s2_patch_supported(d)) return -1;
  S2Args a{};
  a.x = d.x; a.w = d.w; a.y = d.y;
  a.scale = d.scale; a.shift = d.shift;
  a.Hi = d.Hi; a.Wi = d.Wi; a.ldx = d.ldx; a.Ho = d.Hi / 2; a.Wo = d.Wi / 2; a.ldy = d.ldy; a.Kpad = d.Kpad;
  a.ncb = d.Cin / 32;
  a.tiles_x = (a.Wo + TW - 1) / TW;
  a.tiles_per_img = ((a.Ho + TH - 1) / TH) * a.tiles_x;
  a.slope = d.slope;
  a.prelu = d.prelu; a.res = d.res; a.ldres = d.ldres; a.res_first = d.res_first;
  a.y2 = d.y2; a.ldy2 = d.ldy2; a.scale2 = d.scale2; a.shift2 = d.shift2;
  dim3 grid((unsigned)(d.B * a.tiles_per_img), (unsigned)(d.N / BN));
  const bool h16 = d.ti == GHOST_F16;
  if (K == 4) {
    if (h16) hipLaunchKernelGGL((conv_s2_patch_kernel<_Float16, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_s2_patch_kernel<bf16, 4>), grid, dim3(256), 0, s, a);
  } else {
    if (h16) hipLaunchKernelGGL((conv_s2_patch_kernel<_Float16, 3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_s2_patch_kernel<bf16, 3>), grid, dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}

}  // namespace ghost
