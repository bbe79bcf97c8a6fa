// ghost_amd — 3x3/s1/p1 convolution with the input staged once per channel block as a halo
// tile (AAD_ResBlk's conv3x3, AADLayer.py:64,71; bf16).
//
// The implicit GEMM (conv_igemm.hip) gathers an A tile per K step: for a 3x3 conv every input
// pixel is fetched nine times (once per tap), which makes the narrow-N convs of the 128x128 and
// 256x256 stages (N = 64 / 128) bound by the vector-memory path, not the matrix cores.  Here a
// workgroup owns a 16 x 32 output tile of one sample and 64 output channels; per block of 32
// input channels it DMAs the 18 x 34 halo (1.2x the tile) and the block's 9 x 64 weight rows
// into LDS (global_load_lds, source-side XOR swizzle), then runs all nine taps from LDS:
//   tap (ty, tx): D[n][p] += W_t[n][c] . X[p + (ty, tx)][c]      (v_mfma_f32_16x16x32_bf16)
// The weights are the MFMA A operand, so a lane's accumulators are 4 consecutive output
// channels of one pixel and the epilogue stores 8 bytes per lane.
// 8 waves, each 2 output rows (64 pixels) x 64 channels; 75 KB LDS -> two workgroups per CU,
// which overlap one workgroup's DMA with the other's MFMAs.
// The same plan serves ArcFace's IResNet (arc_runtime.hip) with 16 x 16 tiles (4 waves of 4 rows)
// that may overhang 112/56/28/14-pixel images: the halo DMA zero-fills outside the image and the
// epilogue drops those pixels; it also applies the IBasicBlock epilogue (PReLU, residual, the next
// block's BatchNorm as a second output).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "conv_halo.h"
#include "ghost_common.h"

namespace ghost {

// tile configurations: TH x TW output pixels, WM x WN waves of 64 pixels x 64 channels each.
// IMG > 1: the tile is IMG whole TH x TW images (64 pixels, one per wave) of consecutive samples,
// each with its own zero-padded halo — the generator's 8x8 stage (AADBlk3), where a 16 x 16 tile
// would be three quarters padding and the implicit GEMM re-reads every pixel nine times.
// IMG > 1 with TH * TW > 64: the tile is the same TH x TW window of IMG consecutive samples, WPI waves
// per image (ArcFace's 14 x 14 / 28 x 28 stages: two samples share every weight stage).
template <int TH_, int TW_, int WM_, int WN_, int IMG_ = 1>
struct HaloCfg {
  static constexpr int TH = TH_, TW = TW_, WM = WM_, WN = WN_, IMG = IMG_;
  static constexpr int BN = 64 * WN, NW = WM * WN, WPI = WM / IMG;
  static constexpr int HWW = TW + 2, HHH = TH + 2;
  static constexpr int HIMG = HHH * HWW;                    // halo pixels of one image
  static constexpr int HP = IMG * HIMG;                     // halo pixels
  static constexpr int HPIECES = (HP + 15) / 16;            // DMA pieces of 16 pixels x 64 B
  static constexpr int WPIECES = 9 * BN / 16;               // pieces of 16 weight rows x 64 B
  static constexpr int HALO_B = HPIECES * 1024;
  static constexpr int LDS_B = HALO_B + 9 * BN * 64;
  static constexpr int HPW = (HPIECES + NW - 1) / NW;       // halo pieces per wave
  static constexpr int WPW = (WPIECES + NW - 1) / NW;       // weight pieces per wave
  static_assert(IMG * TH * TW == 64 * WM, "each wave owns 64 output pixels");
  static_assert(IMG == 1 || (WN == 1 && WM % IMG == 0), "multi-image tiles: whole waves per image");
  // wave w: its image within the tile, the first tile row of its 64 pixels, its image's halo base
  GHOST_DEV static int img(int w) { return IMG > 1 ? w / WPI : 0; }
  GHOST_DEV static int hrow0(int w) { return (IMG > 1 ? w % WPI : w) * (64 / TW); }
  GHOST_DEV static int himg(int w) { return img(w) * HIMG; }
};
using HaloWide = HaloCfg<16, 32, 8, 1>;    // W % 32 == 0: 16 x 32 tile, 8 waves, 75 KB LDS
using HaloSmall = HaloCfg<16, 16, 4, 1>;   // W == 16: 16 x 16 tile, 4 waves, 57 KB LDS
using HaloImg8 = HaloCfg<8, 8, 4, 1, 4>;   // 8 x 8 images, four per tile, 4 waves, 61 KB per stage
using HaloPair = HaloCfg<16, 16, 8, 1, 2>; // a 16 x 16 window of two samples, 8 waves, 77 KB per stage

struct HaloArgs {
  const void* x;   // 16-bit storage (bf16 or fp16: the kernels' T)
  const void* w;
  void* y;
  const float* scale;
  const float* shift;
  const void* res;
  int H, W, Cin, ldx, N, Kpad, ldy, ldres, tanh_out;
  float slope;
  int tiles_x, tiles_y, nNt, ntiles;
  int dbg;   // experiment mask (GHOST_HALO_DBG): 2 no halo DMA, 4 no weight DMA, 8 no MFMA
  float* in_part;   // pp kernel: InstanceNorm partials [B][tiles/sample][8 waves][N][2] or null
  // epilogue variants of the non-persistent kernel (IBasicBlock convs, arc_runtime.hip): per-channel
  // PReLU slope, residual before the activation, second output y2 = v*scale2 + shift2 (next BN)
  const float* prelu;
  void* y2;
  const float* scale2;
  const float* shift2;
  int ldy2, res_first;
};

__device__ __attribute__((aligned(16))) unsigned int g_halo_zero[64] = {0};

GHOST_DEV int hswz(int r) { return (r >> 1) & 3; }   // conflict-free for 16 consecutive rows at any offset

GHOST_DEV int xcd_tile(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <typename T, class G>
__global__ void __launch_bounds__(G::NW * 64) __attribute__((amdgpu_waves_per_eu(4, 8))) conv3x3_halo_kernel(const HaloArgs a) {
  T* __restrict__ ay2_ = reinterpret_cast<T*>(a.y2);
  const T* __restrict__ ax_ = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ aw_ = reinterpret_cast<const T*>(a.w);
  T* __restrict__ ay_ = reinterpret_cast<T*>(a.y);
  const T* __restrict__ ares_ = reinterpret_cast<const T*>(a.res);
  constexpr int TH = G::TH, TW = G::TW, BN = G::BN, HWW = G::HWW, HP = G::HP, HPIECES = G::HPIECES;
  constexpr int WPIECES = G::WPIECES, HALO_B = G::HALO_B, NWAVES = G::NW, HPW = G::HPW, WPW = G::WPW;
  constexpr int RPW = 64 / TW;                       // output rows per wave
  __shared__ __attribute__((aligned(1024))) unsigned char lds[G::LDS_B];
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int wid = tid >> 6, wm = wid % G::WM, wn = wid / G::WM;
  // tile order: channel tile fastest, then x, y, sample; XCD-contiguous so neighbouring tiles
  // (shared halo rows, same input pixels for every channel tile) meet in one L2
  int t = xcd_tile(blockIdx.x, gridDim.x);
  const int nt = t % a.nNt;
  t /= a.nNt;
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  const int b = t / a.tiles_y;
  const int y0 = ty * TH, x0 = tx * TW, n0 = nt * BN;
  const long img = (long)b * a.H * a.W;
  const T* __restrict__ xs = ax_ + img * a.ldx;            // this sample
  const T* __restrict__ ws = aw_ + (long)n0 * a.Kpad;      // this channel tile

  // this lane's DMA sources (32-bit element offsets within the sample / tile; + channel block)
  const int prow = lane >> 2, slot = lane & 3;
  int h_off[HPW];
  unsigned h_ok = 0u;
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int piece = wid + j * NWAVES;
    const int P = piece * 16 + prow;
    const int hy = P / HWW, hx = P - hy * HWW;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    const bool ok = piece < HPIECES && P < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    h_off[j] = ok ? (iy * a.W + ix) * a.ldx + ((slot ^ hswz(P)) * 8) : 0;
    h_ok |= (ok ? 1u : 0u) << j;
  }
  int w_off[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int piece = wid + j * NWAVES;           // = tap * BN/16 + 16-row group
    const int tap = piece / (BN / 16), n = (piece % (BN / 16)) * 16 + prow;
    w_off[j] = n * a.Kpad + tap * 32 + ((slot ^ hswz(n)) * 8);
  }

  f32x4 acc[4][4];   // [channel frag j][pixel frag i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ncb = a.Cin / 32;
  for (int cb = 0; cb < ncb; ++cb) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int piece = wid + j * NWAVES;
      if (piece < HPIECES) {
        const void* src = ((h_ok >> j) & 1u) ? (const void*)(xs + h_off[j] + cb * 32) : (const void*)g_halo_zero;
        __builtin_amdgcn_global_load_lds(src, lds + piece * 1024, 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int piece = wid + j * NWAVES;
      if (piece < WPIECES)
        __builtin_amdgcn_global_load_lds(ws + w_off[j] + cb * 288, lds + HALO_B + piece * 1024, 16, 0, 0);
    }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      // keep each tap's fragment reads after the previous tap's MFMAs are issued: hoisting all
      // nine taps' reads needs ~300 VGPRs; the other waves of the SIMD hide the LDS latency
      asm volatile("" ::: "memory");
      const int dy = tap / 3, dx = tap - dy * 3;
      v8_t<T> wf[4], pf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = wn * 64 + j * 16 + lr;
        wf[j] = *reinterpret_cast<const v8_t<T>*>(lds + HALO_B + (tap * BN + n) * 64 + ((lq ^ hswz(n)) * 16));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int P = (wm * RPW + (i * 16) / TW + dy) * HWW + (i * 16) % TW + lr + dx;
        pf[i] = *reinterpret_cast<const v8_t<T>*>(lds + P * 64 + ((lq ^ hswz(P)) * 16));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma16x16x32<T>(wf[j], pf[i], acc[j][i]);
    }
    __syncthreads();   // every wave is done with this block's LDS before the next DMA
  }

  // epilogue: lane holds channels n0 + 64wn + 16j + 4lq + r of pixel (row RPW*wm + 16i/TW,
  // column 16i % TW + lr).  Tiles may overhang the image (H or W not a multiple of the tile: the
  // halo DMA zero-fills outside it); those pixels are computed and dropped here.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oy = y0 + wm * RPW + (i * 16) / TW, ox = x0 + (i * 16) % TW + lr;
    if (oy >= a.H || ox >= a.W) continue;
    const long pix = img + (long)oy * a.W + ox;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + lq * 4;
      if (n >= a.N) continue;
      float v[4];
      float rv[4] = {0.f, 0.f, 0.f, 0.f};
      if (ares_) {
        const uint2 raw = *reinterpret_cast<const uint2*>(ares_ + pix * a.ldres + n);
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int r = 0; r < 4; ++r) rv[r] = (float)e[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // same order as conv_igemm.hip epi_std
        float s = acc[j][i][r];
        if (a.scale) s *= a.scale[n + r];
        if (a.shift) s += a.shift[n + r];
        if (a.res_first) s += rv[r];
        const float sl = a.prelu ? a.prelu[n + r] : a.slope;
        s = s > 0.f ? s : s * sl;
        if (!a.res_first) s += rv[r];
        if (a.tanh_out) s = tanhf(s);
        v[r] = s;
      }
      uint2 o;
      T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
      for (int r = 0; r < 4; ++r) oe[r] = (T)v[r];
      *reinterpret_cast<uint2*>(ay_ + pix * a.ldy + n) = o;
      if (ay2_) {
#pragma unroll
        for (int r = 0; r < 4; ++r) oe[r] = (T)(v[r] * a.scale2[n + r] + a.shift2[n + r]);
        *reinterpret_cast<uint2*>(ay2_ + pix * a.ldy2 + n) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Persistent, double-buffered form of the 16 x 32 halo conv (the 32x32 .. 256x256 stages).
//
// The kernel above stages one channel block, waits for it and computes it: with two workgroups
// per CU each one's DMA latency is exposed about half the time (measured 0.54-0.92 PF on the
// generator stages against a 124 us MFMA floor per 309 GFLOP).  Here ONE workgroup per CU walks
// a strided list of (tile, channel block) stages and keeps the DMA of stage s+1 in flight while it
// computes stage s: two 75 KB LDS stages (halo + the block's 9 x 64 weight rows) = 150 KB.
//   top of stage s:  s_waitcnt vmcnt(0)        (or vmcnt(16) when the previous stage ended a tile:
//                                               its 16 epilogue stores are the wave's youngest ops)
//                    raw s_barrier             (every wave's DMA(s) landed; stage s-1 buffer free)
//                    issue DMA(s+1) -> buffer (s+1)&1
//                    9 taps x 16 MFMA from buffer s&1;  last block of a tile -> epilogue stores
// Barriers are raw __builtin_amdgcn_s_barrier: __syncthreads() would drain the in-flight DMA
// (cdna_hip_programming.md, glds notes).  Scale/shift live in LDS so the epilogue issues no
// ordinary global load while a DMA is outstanding (hipcc would wait vmcnt(0) for its result).
// ---------------------------------------------------------------------------
// f(integral_constant<int, P>) for P in the sequence, in order (compile-time unrolling)
template <int... P, class F>
GHOST_DEV void pp_unroll(std::integer_sequence<int, P...>, F&& f) {
  (f(std::integral_constant<int, P>{}), ...);
}

// InstanceNorm partials of a wave's 64 pixels (4 pixel fragments x 64 channels in acc, the stored
// T-rounded values): per channel the mean and the centred sum of squares, two passes over registers
// (AADLayer.py:16,24 normalises this tensor next; in_stats_from_tiles merges the records in fp64, Chan).
// The 16 channel sums of a lane are reduced over the 16 lanes of its row by a transpose-reduce (8+4+2+1
// DPP exchanges: row_mirror i ^ 15, row_half_mirror i ^ 7, quad_perm [2,3,0,1] i ^ 2, [1,0,3,2] i ^ 1;
// round m keeps the half selected by lane bit m) that leaves channel k = lr in lane lr; the mean goes
// back by the reverse butterfly.  Lane (lr, lq) ends with channel 16 (lr >> 2) + 4 lq + (lr & 3).
// acc is zeroed.
template <int M, int CTL>
GHOST_DEV void stats_round(float (&v)[16], int lr) {
  const bool hi = (lr & M) != 0;
#pragma unroll
  for (int q = 0; q < M; ++q) {
    const float keep = hi ? v[q + M] : v[q], send = hi ? v[q] : v[q + M];
    const int got = __builtin_amdgcn_update_dpp(0, __float_as_int(send), CTL, 0xF, 0xF, false);
    v[q] = keep + __int_as_float(got);
  }
}
template <int M, int CTL>
GHOST_DEV void stats_bround(float (&w)[16], int lr) {
  const int own = lr & M;
#pragma unroll
  for (int q = 0; q < M; ++q) {
    const int got = __builtin_amdgcn_update_dpp(0, __float_as_int(w[q]), CTL, 0xF, 0xF, false);
    const float mine = w[q];
    w[q] = own ? __int_as_float(got) : mine;
    w[q + M] = own ? mine : __int_as_float(got);
  }
}
GHOST_DEV float stats_reduce16(float (&v)[16], int lr) {
  stats_round<8, 0x140>(v, lr);
  stats_round<4, 0x141>(v, lr);
  stats_round<2, 0x4E>(v, lr);
  stats_round<1, 0xB1>(v, lr);
  return v[0];
}
GHOST_DEV void tile_stats64(f32x4 (&acc)[4][4], int lr, float& S1, float& S2) {
  float v1[16];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) v1[j * 4 + r] = acc[j][0][r] + acc[j][1][r] + acc[j][2][r] + acc[j][3][r];
  const float mean = stats_reduce16(v1, lr) * (1.f / 64.f);
  v1[0] = mean;
  stats_bround<1, 0xB1>(v1, lr);
  stats_bround<2, 0x4E>(v1, lr);
  stats_bround<4, 0x141>(v1, lr);
  stats_bround<8, 0x140>(v1, lr);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s2 = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = acc[j][i][r] - v1[j * 4 + r];
        s2 = fmaf(d, d, s2);
        acc[j][i][r] = 0.f;
      }
      v1[j * 4 + r] = s2;
    }
  S1 = mean;
  S2 = stats_reduce16(v1, lr);
}

// the same in one pass (round 4): per channel the sum and the sum of squares over the 64 pixels, each reduced by
// the transpose-reduce, then mean = S1 / 64 and M2 = S2 - S1 mean (one rounding, fma).  The record is the same
// (mean, M2) pair; the cancellation costs ~2^-24 (1 + mean^2 / var) relative in M2 for a tile of 64 pixels,
// far below the 16-bit storage of the tensor it describes.  ~110 instead of ~280 VALU per tile and wave.
GHOST_DEV void tile_stats64_1p(f32x4 (&acc)[4][4], int lr, float& S1, float& S2) {
  float v1[16], v2[16];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      f32x2 s = {0.f, 0.f}, q = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 x = {acc[j][i][r], acc[j][i][r + 1]};
        s = s + x;
        q = fma2(x, x, q);
        acc[j][i][r] = 0.f;
        acc[j][i][r + 1] = 0.f;
      }
      v1[j * 4 + r] = s.x;
      v1[j * 4 + r + 1] = s.y;
      v2[j * 4 + r] = q.x;
      v2[j * 4 + r + 1] = q.y;
    }
  const float s1 = stats_reduce16(v1, lr);
  const float s2 = stats_reduce16(v2, lr);
  S1 = s1 * (1.f / 64.f);
  S2 = fmaxf(fmaf(-s1, S1, s2), 0.f);
}

// G = HaloWide (exact 16 x 32 tiles, the generator) or HaloSmall: 16 x 16 tiles that may overhang
// the image (ArcFace 112 .. 14), 4 waves, with the IBasicBlock epilogue (per-channel PReLU, residual
// before or after it, second output y2 = v*scale2 + shift2 = the next block's BatchNorm).
template <typename T, class G, bool RESW, bool STATS, int NCB, int DBG = 0>
__global__ void __launch_bounds__(G::NW * 64) conv3x3_halo_pp_kernel(const HaloArgs a) {
  T* __restrict__ ay2_ = reinterpret_cast<T*>(a.y2);
  const T* __restrict__ ax_ = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ aw_ = reinterpret_cast<const T*>(a.w);
  T* __restrict__ ay_ = reinterpret_cast<T*>(a.y);
  const T* __restrict__ ares_ = reinterpret_cast<const T*>(a.res);
  static_assert(NCB % 2 == 0 && NCB <= 32 && (!RESW || NCB == 2), "channel blocks per tile");
  constexpr bool EPX = G::TW == 16;   // small tiles: overhang masking + the extended epilogue
  static_assert(!(EPX && STATS), "IN partials only from exact tiles");
  // DBG (experiments only, GHOST_HALO_DBG): 2 no halo DMA, 4 no weight DMA, 8 no LDS reads/MFMA,
  // 16 no output stores, 32 no epilogue, 64 no fragment reads after tap 1 (MFMAs on stale fragments)
  // RESW: Cin <= 64 and N == 64 — the whole weight tensor (<= 2 blocks x 36 KB) stays resident in
  // LDS for the kernel and only the halo (39 KB) streams per stage; otherwise every stage carries
  // its channel block's 9 x 64 weight rows too (75 KB).
  constexpr int TW = G::TW, HWW = G::HWW, HP = G::HP, HPIECES = G::HPIECES, WPIECES = G::WPIECES;
  constexpr int HALO_B = G::HALO_B, NW = G::NW, HPW = G::HPW, WPW = G::WPW, IMG = G::IMG;
  // channel tables (N <= NMAX): the two-sample window fills LDS with its stages (2 x 77 KB) and takes N <= 256
  constexpr int NMAX = IMG > 1 ? (EPX ? 256 : 1024) : 512;
  constexpr int WBLK_B = 9 * 64 * 64;                           // one channel block of weights
  constexpr int STAGE_B = RESW ? HALO_B : HALO_B + WBLK_B;
  // two stage buffers as DISTINCT objects, read/written in an unrolled ping-pong: hipcc then proves
  // that the LDS reads of stage s do not alias the DMA into stage s+1 and does not drain it with a
  // vmcnt(0) before the first read (one object indexed by s & 1 gets that drain)
  __shared__ __attribute__((aligned(1024))) unsigned char lds0[STAGE_B];
  __shared__ __attribute__((aligned(1024))) unsigned char lds1[STAGE_B];
  __shared__ __attribute__((aligned(1024))) unsigned char ldsw[RESW ? 2 * WBLK_B : 16];
  __shared__ __attribute__((aligned(16))) float s_sc[NMAX], s_sh[NMAX];   // N <= NMAX (conv3x3_pp_takes / conv3x3_halo)
  __shared__ __attribute__((aligned(16))) float s_ex[EPX ? 3 * NMAX : 4];   // PReLU slope, scale2, shift2 (EPX)
  // wid through readfirstlane: the DMA pieces' conditions and LDS destinations are then wave-uniform (scalar branches,
  // m0 from SGPRs) instead of exec-masked per-lane code at every stage top
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lq = lane >> 4,
            wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int prow = lane >> 2, slot = lane & 3;

  for (int n = tid; n < a.N; n += NW * 64) {
    s_sc[n] = a.scale ? a.scale[n] : 1.f;
    s_sh[n] = a.shift ? a.shift[n] : 0.f;
    if constexpr (EPX) {
      s_ex[n] = a.prelu ? a.prelu[n] : a.slope;
      s_ex[NMAX + n] = ay2_ ? a.scale2[n] : 0.f;
      s_ex[2 * NMAX + n] = ay2_ ? a.shift2[n] : 0.f;
    }
  }
  constexpr int ncb = NCB;
  // per-lane weight source offsets within a channel block (tap, row) — independent of the tile
  int w_off[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int piece = wid + j * NW;
    const int tap = piece / 4, n = (piece % 4) * 16 + prow;
    w_off[j] = n * a.Kpad + tap * 32 + ((slot ^ hswz(n)) * 8);
  }
  unsigned char* wres = ldsw;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (RESW) {
    for (int cb = 0; cb < ncb; ++cb)
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        const int piece = wid + j * NW;
        if (piece < WPIECES)
          __builtin_amdgcn_global_load_lds(aw_ + w_off[j] + cb * 288, wres + cb * WBLK_B + piece * 1024, 16, 0, 0);
      }
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int G_ = gridDim.x;
  const int xt = xcd_tile(blockIdx.x, G_);
  const int nmine = a.ntiles > xt ? (a.ntiles - xt + G_ - 1) / G_ : 0;

  // tile of this WG's k-th item, and this lane's halo DMA sources for it (element offsets from the
  // sample base; bit j of ok = piece j inside the image)
  struct Tile { long base; int y0, x0, n0; };
  auto tile_of = [&](int k) {
    int t = k * G_ + xt;
    Tile r;
    const int nt = t % a.nNt;
    t /= a.nNt;
    const int tx = t % a.tiles_x;
    t /= a.tiles_x;
    const int ty = t % a.tiles_y;
    r.base = (long)(t / a.tiles_y) * IMG * a.H * a.W;   // IMG > 1: t = group of IMG samples
    r.y0 = ty * G::TH;
    r.x0 = tx * TW;
    r.n0 = nt * 64;
    return r;
  };
  int h_off[HPW];
  unsigned h_ok = 0u;
  long dma_base = 0;
  int dma_n0 = 0;
  auto set_dma_tile = [&](const Tile& t) {
    dma_base = t.base * a.ldx;
    dma_n0 = t.n0;
    h_ok = 0u;
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int piece = wid + j * NW;
      const int P = piece * 16 + prow;
      const int im = IMG > 1 ? P / G::HIMG : 0, hp = P - im * G::HIMG;
      const int hy = hp / HWW, hx = hp - hy * HWW;
      const int iy = t.y0 - 1 + hy, ix = t.x0 - 1 + hx;
      const bool ok = piece < HPIECES && P < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      h_off[j] = ok ? ((im * a.H + iy) * a.W + ix) * a.ldx + ((slot ^ hswz(P)) * 8) : 0;
      h_ok |= (ok ? 1u : 0u) << j;
    }
  };
  // one DMA piece of this lane's wave: jj < HPW a halo piece, else weight piece jj - HPW (jj compile-time)
  auto issue_piece = [&](unsigned char* buf, int cb, auto jt) {
    constexpr int jj = decltype(jt)::value;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (jj < HPW) {
      const int piece = wid + jj * NW;
      if (piece < HPIECES && !(DBG & 2)) {
        const T* __restrict__ xs = ax_ + dma_base + cb * 32;
        const void* src = ((h_ok >> jj) & 1u) ? (const void*)(xs + h_off[jj]) : (const void*)g_halo_zero;
        __builtin_amdgcn_global_load_lds(src, buf + piece * 1024, 16, 0, 0);
      }
    } else if constexpr (!RESW && !(DBG & 4)) {
      constexpr int j = jj - HPW;
      const int piece = wid + j * NW;
      if (piece < WPIECES) {
        const T* __restrict__ ws = aw_ + (long)dma_n0 * a.Kpad + cb * 288;
        __builtin_amdgcn_global_load_lds(ws + w_off[j], buf + HALO_B + piece * 1024, 16, 0, 0);
      }
    }
#endif
  };
  auto issue = [&](unsigned char* buf, int cb) {
#if defined(__HIP_DEVICE_COMPILE__)
    const T* __restrict__ xs = ax_ + dma_base + cb * 32;
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int piece = wid + j * NW;
      if (piece < HPIECES && !(DBG & 2)) {
        const void* src = ((h_ok >> j) & 1u) ? (const void*)(xs + h_off[j]) : (const void*)g_halo_zero;
        __builtin_amdgcn_global_load_lds(src, buf + piece * 1024, 16, 0, 0);
      }
    }
    if constexpr (!RESW && !(DBG & 4)) {
      const T* __restrict__ ws = aw_ + (long)dma_n0 * a.Kpad + cb * 288;
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        const int piece = wid + j * NW;
        if (piece < WPIECES)
          __builtin_amdgcn_global_load_lds(ws + w_off[j], buf + HALO_B + piece * 1024, 16, 0, 0);
      }
    }
#endif
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Stage order: tile k = 0..nmine-1, channel blocks cb = 0..NCB-1 (NCB even, unrolled), so a tile's
  // even stages read lds0 and prefetch into lds1 and its odd stages the reverse, with every wait
  // static.  The first stage of a tile waits vmcnt(NST): the previous tile's NST epilogue stores are
  // the wave's youngest VM ops (VM ops retire in issue order), so the wait covers this stage's DMA
  // without waiting for the stores to reach memory; the later stages wait vmcnt(0).
  // (EPX: overhang-masked stores may be skipped by a whole wave, so the count is not static: wait for 0)
  // W16: the epilogue writes 16-byte pieces (8 stores per wave; see there) — the two-block (Cin = 64) tiles of
  // the 256 x 256 stage only: with more blocks per tile the exchange's registers push the kernel into spills
  constexpr bool W16 = !EPX && NCB == 2 && IMG == 1 && !(DBG & 16);
  // LDSW (round 5): the other exact-tile convs (NCB >= 4: the 128 x 128 .. 32 x 32 stages) stage the epilogue through
  // the LDS of the tile's finished last stage — each wave writes its 64 pixels x 64 channels (8-byte pieces as the
  // accumulators hold them; pixel rows of 128 bytes at a 136-byte pitch) and reads them back as whole 128-byte pixel
  // rows, so its 8 global stores each write 8 whole rows (1 KB) instead of 16 stores of 8-byte quarter pieces.  The
  // register exchange of W16 does the same at NCB = 2 but spills the NCB >= 4 kernels; the LDS path needs no
  // extra live registers, only one barrier per tile (every wave past its last read of the stage).
  constexpr int LPITCH = 136, LWAVE = 64 * LPITCH;
  constexpr bool LDSW = !EPX && !W16 && IMG == 1 && !RESW && !(DBG & 16) && STAGE_B >= NW * LWAVE;
  const bool plain = !a.scale && !a.shift && a.slope == 1.f && !a.tanh_out;
  constexpr int NST = ((DBG & 48) || EPX) ? 0 : ((W16 || LDSW) ? 8 : 16) + (STATS ? 1 : 0);
  if (nmine == 0) return;
  // Round 6: the next stage's DMA pieces (about ten per wave: its halo and weight pieces) go out two per tap, each
  // pair after a tap's 16 MFMAs are issued, instead of all at the top of the stage.  At the top both waves of a SIMD
  // issued theirs back to back after the barrier (60-185 cycles per piece, MI355X_MICROARCH.md) while the matrix
  // pipe idled; spread, each piece issues in the shadow of MFMAs already in flight, and the top of a stage holds
  // only the wait, the barrier and tap 0's fragment reads.  Same-box per-op A/B (B = 64, tools/ab_pp.sh,
  // profiles/r06_ab_kernels.txt): 128x128 331 -> 315 us, 64x64 262 -> 250, 32x32 246 -> 233, 256x256 401 ->
  // 389; one piece per tap or three measured no better.  (DBG & 4096: the old all-at-the-top issue, A/B only.)
  constexpr bool SPREAD = (DBG & 4096) == 0;
  constexpr int NPIECE = HPW + (RESW ? 0 : WPW);
  constexpr int PPT = 2;   // pieces per tap
  Tile cur = tile_of(0);
  set_dma_tile(cur);
  issue(lds0, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0): tile 0 has no stores in front of its DMA
  int k = 0;
  auto step = [&](const unsigned char* buf, unsigned char* nbuf, auto cbt) {
    constexpr int cb = decltype(cbt)::value;
    // gfx9 simm16: vm[3:0] exp[6:4] lgkm[11:8] vm[5:4]@[15:14]
    if constexpr (cb == 0)
      __builtin_amdgcn_s_waitcnt(((NST >> 4) << 14) | 0x0F70 | (NST & 15));
    else
      __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    const bool more = cb + 1 < NCB || k + 1 < nmine;   // a next stage to prefetch
    if constexpr (cb + 1 < NCB) {
      if constexpr (!SPREAD) issue(nbuf, cb + 1);
    } else if (k + 1 < nmine) {
      set_dma_tile(tile_of(k + 1));
      if constexpr (!SPREAD) issue(nbuf, 0);
    }
    constexpr int ncb_next = cb + 1 < NCB ? cb + 1 : 0;
    const unsigned char* wb = RESW ? wres + cb * WBLK_B : buf + HALO_B;
    // fragments of tap t + 1 are read while tap t's 16 MFMAs run (two register sets): the wave never
    // waits for its own LDS reads except at the first tap of a stage
    v8_t<T> wf[2][4], pf[2][4];
    auto load_frags = [&](int tap, v8_t<T> (&w)[4], v8_t<T> (&p)[4]) {
      const int dy = tap / 3, dx = tap - dy * 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = j * 16 + lr;
        w[j] = *reinterpret_cast<const v8_t<T>*>(wb + (tap * 64 + n) * 64 + ((lq ^ hswz(n)) * 16));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = i * 16 + lr;   // the wave's pixel (row q / TW, column q % TW of its 64)
        const int P = G::himg(wid) + (G::hrow0(wid) + q / TW + dy) * HWW + q % TW + dx;
        p[i] = *reinterpret_cast<const v8_t<T>*>(buf + P * 64 + ((lq ^ hswz(P)) * 16));
      }
    };
    // (measured: the same time as one register set read then used, and with s_setprio around the MFMAs)
    if constexpr ((DBG & 8) == 0) {
      load_frags(0, wf[0], pf[0]);
      if constexpr ((DBG & 64) != 0) load_frags(1, wf[1], pf[1]);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        // this tap's fragments (issued during the previous tap's MFMAs) have landed: wait for them BEFORE issuing
        // the next tap's 8 reads — after those the wave has 16 LDS reads outstanding, more than the 4-bit lgkmcnt
        // can distinguish, and the compiler's own wait (placed at the first MFMA) would be lgkmcnt(0)
        if constexpr ((DBG & 128) == 0) __builtin_amdgcn_s_waitcnt(0xC07F);
        if (tap + 1 < 9 && (DBG & 64) == 0) load_frags(tap + 1, wf[(tap + 1) & 1], pf[(tap + 1) & 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = mfma16x16x32<T>(wf[tap & 1][j], pf[tap & 1][i], acc[j][i]);
        if constexpr (SPREAD) {
          if (more) {
            // tap t issues pieces [t PPT, (t + 1) PPT), the last tap also whatever is left
            pp_unroll(std::make_integer_sequence<int, 16>{}, [&](auto qt) {
              constexpr int q = decltype(qt)::value;
              const int pc = tap * PPT + q;
              if ((q < PPT || (tap == 8 && pc < NPIECE)) && pc < NPIECE) {
                // (tap is unrolled: the piece index folds to a constant)
                switch (pc) {
#define GHOST_SPREAD_CASE(N) case N: if constexpr (N < NPIECE) issue_piece(nbuf, ncb_next, std::integral_constant<int, N>{}); break;
                  GHOST_SPREAD_CASE(0) GHOST_SPREAD_CASE(1) GHOST_SPREAD_CASE(2) GHOST_SPREAD_CASE(3)
                  GHOST_SPREAD_CASE(4) GHOST_SPREAD_CASE(5) GHOST_SPREAD_CASE(6) GHOST_SPREAD_CASE(7)
                  GHOST_SPREAD_CASE(8) GHOST_SPREAD_CASE(9) GHOST_SPREAD_CASE(10) GHOST_SPREAD_CASE(11)
                  GHOST_SPREAD_CASE(12) GHOST_SPREAD_CASE(13) GHOST_SPREAD_CASE(14) GHOST_SPREAD_CASE(15)
#undef GHOST_SPREAD_CASE
                  default: break;
                }
              }
            });
          }
        }
        // the software pipeline pinned (round 5): tap + 1's 8 fragment reads go out one per MFMA over the first half
        // of this tap's 16 MFMAs, which then run while they land.  Left to itself the scheduler sank the reads to
        // their first use, and every tap waited two or three times on LDS reads it had just issued.
        if constexpr ((DBG & 128) == 0) {
          if (tap + 1 < 9 && (DBG & 64) == 0) {
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);   // the 8 DS reads
            __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);  // then the 16 MFMAs
          } else {
            __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        } else {
          asm volatile("" ::: "memory");
        }
      }
    }
    if constexpr (cb + 1 < NCB) return;
    if constexpr ((DBG & 32) != 0) {   // (experiments) no epilogue: the accumulators only kept alive
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          t += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      if (__float_as_uint(t) == 0x7fc00123u) ay_[lane] = (T)t;
      return;
    }
    // epilogue: exactly 16 vector stores per wave (N % 64 == 0, full tiles; 8 with W16 / LDSW) + 1 with STATS,
    // the youngest VM ops when the next tile's first stage waits.  The residual tile is loaded as one
    // batch first: a load between two stores would wait for the older store (in-order vmcnt)
    unsigned char* stg = const_cast<unsigned char*>(buf) + wid * LWAVE;   // LDSW: this wave's part of the stage
    if constexpr (LDSW) {
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();         // every wave has read its last fragments of this stage
    }
    // The epilogue in three compile-time forms, chosen once per tile (round 6): MODE 2 = plain (AAD_ResBlk's
    // convs: no scale / shift / activation) without a residual, 1 = plain with the residual, 0 = the general
    // epilogue (and every EPX tile).  Left as runtime tests inside the 16 (pixel, channel) fragment loop, the plain
    // path still ran the residual unpacking, the scale / shift table reads and a scalar branch per fragment: at
    // 256 x 256 (an epilogue every two stages) the epilogue was ~100 of the kernel's ~400 us (GHOST_HALO_DBG=32).
    auto epi_body = [&](auto mt) {
    constexpr int MODE = decltype(mt)::value;
    const bool has_res = MODE == 1 || (MODE == 0 && ares_ != nullptr);
    uint2 rraw[4][4];
    if (has_res) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = i * 16 + lr;
        const int oy = cur.y0 + G::hrow0(wid) + q / TW, ox = cur.x0 + q % TW;
        const long pix = cur.base + (long)G::img(wid) * a.H * a.W + (long)oy * a.W + ox;
        const bool in = !EPX || (oy < a.H && ox < a.W);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rraw[i][j] = in ? *reinterpret_cast<const uint2*>(ares_ + pix * a.ldres + cur.n0 + j * 16 + lq * 4)
                          : make_uint2(0u, 0u);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i * 16 + lr;
      const int oy = cur.y0 + G::hrow0(wid) + q / TW, ox = cur.x0 + q % TW;
      const long pix = cur.base + (long)G::img(wid) * a.H * a.W + (long)oy * a.W + ox;
      uint2 ov[4];   // W16: the 4 channel fragments' T outputs, stored 16 bytes at a time below
      if constexpr (EPX) {
        if (oy >= a.H || ox >= a.W) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = cur.n0 + j * 16 + lq * 4;
        float rv[4] = {0.f, 0.f, 0.f, 0.f};
        if (has_res) {
          const T* e = reinterpret_cast<const T*>(&rraw[i][j]);
#pragma unroll
          for (int r = 0; r < 4; ++r) rv[r] = (float)e[r];
        }
        uint2 o;
        T* oe = reinterpret_cast<T*>(&o);
        if constexpr (EPX) {
          // the lane's 4 channels' tables as one 16-byte LDS read each (n % 4 == 0), not 4 scalar reads
          const f32x4 tsc = *reinterpret_cast<const f32x4*>(s_sc + n);
          const f32x4 tsh = *reinterpret_cast<const f32x4*>(s_sh + n);
          // same order as conv_igemm.hip epi_std
          const f32x4 tpr = *reinterpret_cast<const f32x4*>(s_ex + n);
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = fmaf(acc[j][i][r], tsc[r], tsh[r]);
            if (a.res_first) t += rv[r];
            t = t > 0.f ? t : t * tpr[r];
            if (!a.res_first) t += rv[r];
            if (a.tanh_out) t = tanhf(t);
            v[r] = t;
            oe[r] = (T)t;
            acc[j][i][r] = 0.f;
          }
          *reinterpret_cast<uint2*>(ay_ + pix * a.ldy + n) = o;
          if (ay2_) {
            const f32x4 tsc2 = *reinterpret_cast<const f32x4*>(s_ex + NMAX + n);
            const f32x4 tsh2 = *reinterpret_cast<const f32x4*>(s_ex + 2 * NMAX + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) oe[r] = (T)(v[r] * tsc2[r] + tsh2[r]);
            *reinterpret_cast<uint2*>(ay2_ + pix * a.ldy2 + n) = o;
          }
        } else {
        float v[4];
        if constexpr (MODE != 0) {   // AAD_ResBlk's convs: no scale / shift / activation, at most the residual
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = MODE == 1 ? acc[j][i][r] + rv[r] : acc[j][i][r];
        } else {
          const f32x4 tsc = *reinterpret_cast<const f32x4*>(s_sc + n);
          const f32x4 tsh = *reinterpret_cast<const f32x4*>(s_sh + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = fmaf(acc[j][i][r], tsc[r], tsh[r]);
            t = t > 0.f ? t : t * a.slope;
            t += rv[r];
            if (a.tanh_out) t = tanhf(t);
            v[r] = t;
          }
        }
        // two packed conversions (v_cvt_pk_*) per 4 channels; the statistics read the stored (rounded) values back
        o.x = pack2<T>(v[0], v[1]);
        o.y = pack2<T>(v[2], v[3]);
        if constexpr (STATS) {
          const f32x2 a01 = unpack2<T>(o.x), a23 = unpack2<T>(o.y);
          acc[j][i] = f32x4{a01.x, a01.y, a23.x, a23.y};
        } else {
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if constexpr (W16) ov[j] = o;
        else if constexpr (LDSW) {
          // pixel q's row of 64 channels: this lane's 8 bytes are channels 16 j + 4 lq .. +3
          *reinterpret_cast<uint2*>(stg + q * LPITCH + 32 * j + 8 * lq) = o;
        }
        else if constexpr (!(DBG & 16)) *reinterpret_cast<uint2*>(ay_ + pix * a.ldy + n) = o;
        else if ((o.x ^ o.y) == 0x7fc00001u) *reinterpret_cast<uint2*>(ay_ + pix * a.ldy + n) = o;
        }
      }
      if constexpr (W16) {
        // lanes lq and lq ^ 1 (lane ^ 16) hold channels 16 j + 4 lq .. +3 and the next four: each sends the
        // fragment its partner completes (even lanes keep j = 0, 2, odd lanes j = 1, 3), so every lane writes
        // two 16-byte pieces of 8 channels (8 stores per wave per tile instead of 16 of 8 bytes)
        // (round 6) one v_permlane16_swap per word pair does the exchange: it swaps the odd 16-lane rows of its first
        // operand with the even rows of its second, which leaves (a0, a1) = (own ov[0], partner's ov[0]) in even rows
        // and (partner's ov[1], own ov[1]) in odd rows — what the ds_bpermute + select form computed
        uint2 a0, a1, b0, b1;
        {
          const auto x0 = __builtin_amdgcn_permlane16_swap(ov[0].x, ov[1].x, false, false);
          const auto y0 = __builtin_amdgcn_permlane16_swap(ov[0].y, ov[1].y, false, false);
          const auto x1 = __builtin_amdgcn_permlane16_swap(ov[2].x, ov[3].x, false, false);
          const auto y1 = __builtin_amdgcn_permlane16_swap(ov[2].y, ov[3].y, false, false);
          a0 = make_uint2(x0[0], y0[0]);
          a1 = make_uint2(x0[1], y0[1]);
          b0 = make_uint2(x1[0], y1[0]);
          b1 = make_uint2(x1[1], y1[1]);
        }
        // lane lq now holds chunk m = (lq >> 1) + 2 (lq & 1) of pixel q (a) and chunk 4 + m (b): the tile row's
        // 16 pixels q - lr .. +15 are consecutive, so store_rows16 writes them as 8 whole rows per store
        static_assert(G::TW % 16 == 0, "a pixel fragment lies in one tile row");
        const long p0 = pix - lr + (lr & 7);
        store_rows16<T>(ay_ + cur.n0, p0 * a.ldy, (p0 + 8) * a.ldy, lr, (lq >> 1) + 2 * (lq & 1),
                        u32x4{a0.x, a0.y, a1.x, a1.y}, u32x4{b0.x, b0.y, b1.x, b1.y});
      }
    }
    };
    if constexpr (EPX) {
      epi_body(std::integral_constant<int, 0>{});
    } else {
      if (plain) {
        if (ares_) epi_body(std::integral_constant<int, 1>{});
        else epi_body(std::integral_constant<int, 2>{});
      } else {
        epi_body(std::integral_constant<int, 0>{});
      }
    }
    if constexpr (LDSW) {
      // the wave's tile back as whole rows: store s writes pixels 8 s .. 8 s + 7 (consecutive columns of one tile
      // row), lane L chunk L & 7 of pixel 8 s + L / 8 (LDS ops of a wave complete in order: no wait between the
      // writes above and these reads)
      asm volatile("" ::: "memory");
      const int c = lane & 7, q0 = lane >> 3;
      // the wave's first pixel and this lane's pixel / chunk within a store (element offsets)
      T* __restrict__ yw = ay_ + (cur.base + (long)(cur.y0 + G::hrow0(wid)) * a.W + cur.x0) * a.ldy + cur.n0;
      const int lo = q0 * a.ldy + c * 8;
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int q = 8 * st + q0;   // tile row st / 4, columns 8 (st % 4) .. +7
        const u32x4 v = *reinterpret_cast<const u32x4*>(stg + q * LPITCH + c * 16);
        *reinterpret_cast<u32x4*>(yw + ((st >> 2) * a.W + 8 * (st & 3)) * a.ldy + lo) = v;
      }
    }
    if constexpr (STATS) {
      // InstanceNorm partials of this wave's 64 pixels (tile_stats64)
      float S1, S2;
      tile_stats64_1p(acc, lr, S1, S2);
      // lane (lr, lq) holds channel n0 + 16 (lr >> 2) + 4 lq + (lr & 3)
      const int c = cur.n0 + (lr >> 2) * 16 + lq * 4 + (lr & 3);
      float* dst;
      if constexpr (IMG > 1) {   // the wave's 64 pixels are its whole image: one record per sample
        const long b = cur.base / ((long)a.H * a.W) + G::img(wid);
        dst = a.in_part + (b * (long)a.N + c) * 2;
      } else {
        const int tile = (cur.y0 / G::TH) * a.tiles_x + cur.x0 / TW;
        const long b = cur.base / ((long)a.H * a.W);
        dst = a.in_part + ((((b * a.tiles_x * a.tiles_y) + tile) * 8 + wid) * (long)a.N + c) * 2;
      }
      *reinterpret_cast<float2*>(dst) = make_float2(S1, S2);
    }
  };
  for (; k < nmine; ++k) {
    // the tile's NCB stages unrolled: even ones read lds0, odd ones lds1
    pp_unroll(std::make_integer_sequence<int, NCB / 2>{}, [&](auto pt) {
      constexpr int P = decltype(pt)::value;
      step(lds0, lds1, std::integral_constant<int, 2 * P>{});
      step(lds1, lds0, std::integral_constant<int, 2 * P + 1>{});
    });
    if (k + 1 < nmine) cur = tile_of(k + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// ConvTranspose2d 4x4/s2/p1 (AEI_Net.py:27-41, the encoder's deconv layers) on the same plan:
// a workgroup owns an 8 x 16 tile of INPUT pixels (= a 16 x 32 output tile: four sub-pixel
// phases) and BN output channels.  Per block of 32 input channels it DMAs the 10 x 18 input
// halo and the block's 16 (phase, tap) x BN weight rows; wave w computes phase w/2 for input
// rows 4(w%2) .. +3 with its four 2x2 taps:
//   out(2qy+py, 2qx+px)[n] += W[ky(py,ty)][kx(px,tx)][n][c] . x(qy+py-ty, qx+px-tx)[c]
// ---------------------------------------------------------------------------
template <int BN>
struct HaloTCfg {
  static constexpr int TIH = 8, TIW = 16;                   // input tile
  static constexpr int HWW = TIW + 2, HP = (TIH + 2) * HWW; // 180 halo pixels
  static constexpr int HPIECES = (HP + 15) / 16;            // 12
  static constexpr int WPIECES = 16 * BN / 16;              // (phase, tap) x BN/16
  static constexpr int HALO_B = HPIECES * 1024;
  static constexpr int LDS_B = HALO_B + 16 * BN * 64;
  static constexpr int NW = 8;
  static constexpr int HPW = (HPIECES + NW - 1) / NW;
  static constexpr int WPW = (WPIECES + NW - 1) / NW;
  static constexpr int TN = BN / 16;                        // channel fragments per wave
};

struct HaloTArgs {
  const void* x;
  const void* w;      // [4][Npad][Kpad], K = (cb*4 + ty*2 + tx)*32 + c
  void* y;
  const float* scale;
  const float* shift;
  const void* res;
  long wpar;          // Npad * Kpad
  int H, W, Cin, ldx, N, Kpad, ldy, ldres;
  float slope;
  int tiles_x, tiles_y, nNt;
};

template <typename T, int BN>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8))) convT_halo_kernel(const HaloTArgs a) {
  const T* __restrict__ ax_ = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ aw_ = reinterpret_cast<const T*>(a.w);
  T* __restrict__ ay_ = reinterpret_cast<T*>(a.y);
  const T* __restrict__ ares_ = reinterpret_cast<const T*>(a.res);
  using G = HaloTCfg<BN>;
  constexpr int HWW = G::HWW, HP = G::HP, HPIECES = G::HPIECES, WPIECES = G::WPIECES, HALO_B = G::HALO_B;
  constexpr int NWAVES = G::NW, HPW = G::HPW, WPW = G::WPW, TN = G::TN;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[G::LDS_B];
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lq = lane >> 4, wid = tid >> 6;
  const int ph = wid >> 1, py = ph >> 1, px = ph & 1, hf = wid & 1;
  int t = xcd_tile(blockIdx.x, gridDim.x);
  const int nt = t % a.nNt;
  t /= a.nNt;
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  const int b = t / a.tiles_y;
  const int y0 = ty * G::TIH, x0 = tx * G::TIW, n0 = nt * BN;
  const T* __restrict__ xs = ax_ + (long)b * a.H * a.W * a.ldx;

  const int prow = lane >> 2, slot = lane & 3;
  int h_off[HPW];
  unsigned h_ok = 0u;
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int piece = wid + j * NWAVES;
    const int P = piece * 16 + prow;
    const int hy = P / HWW, hx = P - hy * HWW;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    const bool ok = piece < HPIECES && P < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    h_off[j] = ok ? (iy * a.W + ix) * a.ldx + ((slot ^ hswz(P)) * 8) : 0;
    h_ok |= (ok ? 1u : 0u) << j;
  }
  const T* wsrc[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int piece = wid + j * NWAVES;               // = (phase*4 + tap) * BN/16 + row group
    const int pt = piece / (BN / 16), n = (piece % (BN / 16)) * 16 + prow;
    wsrc[j] = aw_ + (pt >> 2) * a.wpar + (long)(n0 + n) * a.Kpad + (pt & 3) * 32 + ((slot ^ hswz(n)) * 8);
  }

  f32x4 acc[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ncb = a.Cin / 32;
  for (int cb = 0; cb < ncb; ++cb) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int piece = wid + j * NWAVES;
      if (piece < HPIECES) {
        const void* src = ((h_ok >> j) & 1u) ? (const void*)(xs + h_off[j] + cb * 32) : (const void*)g_halo_zero;
        __builtin_amdgcn_global_load_lds(src, lds + piece * 1024, 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int piece = wid + j * NWAVES;
      if (piece < WPIECES) __builtin_amdgcn_global_load_lds(wsrc[j] + cb * 128, lds + HALO_B + piece * 1024, 16, 0, 0);
    }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int tp = 0; tp < 4; ++tp) {
      asm volatile("" ::: "memory");
      const int dy = py - (tp >> 1), dx = px - (tp & 1);     // input offset of this tap
      v8_t<T> wf[TN], pf[4];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = j * 16 + lr;
        wf[j] = *reinterpret_cast<const v8_t<T>*>(lds + HALO_B + ((ph * 4 + tp) * BN + n) * 64 + ((lq ^ hswz(n)) * 16));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int P = (hf * 4 + i + 1 + dy) * HWW + lr + 1 + dx;
        pf[i] = *reinterpret_cast<const v8_t<T>*>(lds + P * 64 + ((lq ^ hswz(P)) * 16));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma16x16x32<T>(wf[j], pf[i], acc[j][i]);
    }
    __syncthreads();
  }

  const int Wo = 2 * a.W, Ho = 2 * a.H;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oy = 2 * (y0 + hf * 4 + i) + py, ox = 2 * (x0 + lr) + px;
    const long pix = ((long)b * Ho + oy) * Wo + ox;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + j * 16 + lq * 4;
      if (n >= a.N) continue;
      float rv[4] = {0.f, 0.f, 0.f, 0.f};
      if (ares_) {
        const uint2 raw = *reinterpret_cast<const uint2*>(ares_ + pix * a.ldres + n);
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int r = 0; r < 4; ++r) rv[r] = (float)e[r];
      }
      uint2 o;
      T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[j][i][r];
        if (a.scale) v *= a.scale[n + r];
        if (a.shift) v += a.shift[n + r];
        v = v > 0.f ? v : v * a.slope;
        oe[r] = (T)(v + rv[r]);
      }
      *reinterpret_cast<uint2*>(ay_ + pix * a.ldy + n) = o;
    }
  }
}

bool convT_halo_supported(const ConvDesc& d) {
  static const int enabled = GHOST_KNOB("GHOST_CONVT_HALO", 1);
  if (!enabled || d.kind != CONV_T4S2 || !is16(d.ti) || d.to != d.ti || d.epi != EPI_STD) return false;
  if (d.u8 || d.tanh_out || d.force_split || d.Cin % 32 || d.ldx % 8 || d.ldy % 4 || (d.res && d.ldres % 4)) return false;
  if (d.res_first || d.prelu || d.y2) return false;   // epilogue variants only the implicit GEMM has
  if (d.Hi % HaloTCfg<64>::TIH || d.Wi % HaloTCfg<64>::TIW || d.Kpad < 4 * d.Cin) return false;
  if (!(d.N % 64 == 0 || d.N == 32) || d.Npad < d.N) return false;
  if ((uintptr_t)d.x % 16 || (uintptr_t)d.w % 16 || (uintptr_t)d.y % 8 || (d.res && (uintptr_t)d.res % 8)) return false;
  // one workgroup per (input tile, 64-channel block) with the whole reduction: a small batch (B = 1: 16-32
  // workgroups, 53 us per deconv) leaves the GPU idle; there the implicit GEMM splits K over >= 256 workgroups
  {
    const int bn = d.N == 32 ? 32 : 64;
    const long nt = (long)d.B * (d.Hi / HaloTCfg<64>::TIH) * (d.Wi / HaloTCfg<64>::TIW) * ((d.N + bn - 1) / bn);
    if (nt < 128) return false;
  }
  return (long)d.Hi * d.Wi * d.ldx < (1L << 31);
}

template <typename T, int BN>
static int haloT_launch(const ConvDesc& d, hipStream_t s) {
  HaloTArgs a{};
  a.x = d.x; a.w = d.w; a.y = d.y;
  a.scale = d.scale; a.shift = d.shift; a.res = d.res;
  a.wpar = (long)d.Npad * d.Kpad;
  a.H = d.Hi; a.W = d.Wi; a.Cin = d.Cin; a.ldx = d.ldx; a.N = d.N; a.Kpad = d.Kpad;
  a.ldy = d.ldy; a.ldres = d.ldres; a.slope = d.slope;
  a.tiles_x = d.Wi / HaloTCfg<BN>::TIW; a.tiles_y = d.Hi / HaloTCfg<BN>::TIH; a.nNt = (d.N + BN - 1) / BN;
  const long ntiles = (long)d.B * a.tiles_x * a.tiles_y * a.nNt;
  hipLaunchKernelGGL((convT_halo_kernel<T, BN>), dim3((unsigned)ntiles), dim3(512), 0, s, a);
  return (int)hipGetLastError();
}

int convT_halo(const ConvDesc& d, hipStream_t s) {
  if (!convT_halo_supported(d)) return -1;
  if (d.ti == GHOST_F16) return d.N == 32 ? haloT_launch<_Float16, 32>(d, s) : haloT_launch<_Float16, 64>(d, s);
  return d.N == 32 ? haloT_launch<bf16, 32>(d, s) : haloT_launch<bf16, 64>(d, s);
}

// which tile the non-persistent kernel uses: 16 x 32 when the image is a multiple of it (every
// generator stage from 32x32 up), else 16 x 16 tiles allowed to overhang the image by up to a
// quarter of the work (ArcFace 112 / 56 / 28 / 14: 100 / 77 / 77 / 77 % of the tile pixels used;
// 7x7 and the generator's 8x8 and below stay on the implicit GEMM)
static bool halo_exact_wide(const ConvDesc& d) { return d.Wi % HaloWide::TW == 0 && d.Hi % HaloWide::TH == 0; }
// the 8 x 8 stage: four whole images per tile (HaloImg8)
static bool halo_img8(const ConvDesc& d) {
  static const int on = GHOST_KNOB("GHOST_HALO_IMG8", 1);
  const int ncb = d.Cin / 32;
  // (only shapes the persistent IMG8 kernel is instantiated for, with its 16-byte stores: anything else
  // falls through to the implicit GEMM instead of failing in conv3x3_halo)
  return on && d.Hi == HaloImg8::TH && d.Wi == HaloImg8::TW && d.B % HaloImg8::IMG == 0 && d.N <= 1024 &&
         !d.prelu && !d.y2 && !d.res_first && !d.tanh_out && d.Cin % 64 == 0 && d.Cin <= 1024 &&
         (ncb == 2 || ncb == 4 || ncb == 8 || ncb == 16 || ncb == 32) && d.ldy % 8 == 0 && (uintptr_t)d.y % 16 == 0;
}
static bool halo_small_ok(const ConvDesc& d) {
  const long tx = (d.Wi + HaloSmall::TW - 1) / HaloSmall::TW, ty = (d.Hi + HaloSmall::TH - 1) / HaloSmall::TH;
  return 4L * d.Hi * d.Wi >= 3L * tx * ty * HaloSmall::TW * HaloSmall::TH;
}

bool conv3x3_halo_supported(const ConvDesc& d) {
  static const int enabled = GHOST_KNOB("GHOST_CONV_HALO", 1);
  if (!enabled || d.kind != CONV_FWD || d.kh != 3 || d.kw != 3 || d.stride != 1 || d.pad != 1) return false;
  if (!is16(d.ti) || d.to != d.ti || d.epi != EPI_STD || d.u8 || d.force_split) return false;
  if (d.Cin % 32 || d.ldx % 8 || d.N % 64 || d.ldy % 4 || (d.res && d.ldres % 4)) return false;
  if (d.y2 && (d.ldy2 % 4 || (uintptr_t)d.y2 % 8 || !d.scale2 || !d.shift2)) return false;
  if ((!halo_exact_wide(d) && !halo_small_ok(d) && !halo_img8(d)) || d.Kpad < 9 * d.Cin || d.Npad < d.N) return false;
  if ((uintptr_t)d.x % 16 || (uintptr_t)d.w % 16 || (uintptr_t)d.y % 8 || (d.res && (uintptr_t)d.res % 8)) return false;
  if ((long)d.Hi * d.Wi * d.ldx >= (1L << 31) || (long)d.Npad * d.Kpad >= (1L << 31)) return false;   // 32-bit offsets
  // a work item is one (tile, 64-channel block) with the whole 9 x Cin reduction: under 64 of them (B = 1 at 32 x 32,
  // 512 -> 512: 16 workgroups, 105 us) most CUs idle, and the implicit GEMM's split K spreads the same conv wider
  if (!halo_img8(d)) {
    const bool wide = halo_exact_wide(d);
    const int th = wide ? HaloWide::TH : HaloSmall::TH, tw = wide ? HaloWide::TW : HaloSmall::TW;
    const long items = (long)d.B * ((d.Hi + th - 1) / th) * ((d.Wi + tw - 1) / tw) * (d.N / 64);
    static const int min_items = GHOST_KNOB("GHOST_HALO_MIN_ITEMS", 64);
    if (items < min_items) return false;
  }
  // measured (tools/bench_ops.py, B = 64): faster than the implicit GEMM at every generator stage
  // from 32x32 up (N = 64 .. 512); GHOST_CONV_HALO_MAXN caps N for A/B runs
  static const int max_n = GHOST_KNOB("GHOST_CONV_HALO_MAXN", 1 << 30);
  return d.N <= max_n;
}

template <typename T, class G>
static int halo_launch(const ConvDesc& d, hipStream_t s) {
  HaloArgs a{};
  a.x = d.x; a.w = d.w; a.y = d.y;
  a.scale = d.scale; a.shift = d.shift; a.res = d.res;
  a.H = d.Hi; a.W = d.Wi; a.Cin = d.Cin; a.ldx = d.ldx; a.N = d.N; a.Kpad = d.Kpad;
  a.ldy = d.ldy; a.ldres = d.ldres; a.tanh_out = d.tanh_out; a.slope = d.slope;
  a.prelu = d.prelu; a.y2 = d.y2; a.scale2 = d.scale2; a.shift2 = d.shift2; a.ldy2 = d.ldy2;
  a.res_first = d.res_first;
  a.tiles_x = (d.Wi + G::TW - 1) / G::TW; a.tiles_y = (d.Hi + G::TH - 1) / G::TH;
  a.nNt = (d.N + G::BN - 1) / G::BN;
  a.ntiles = d.B * a.tiles_x * a.tiles_y * a.nNt;
  hipLaunchKernelGGL((conv3x3_halo_kernel<T, G>), dim3((unsigned)a.ntiles), dim3(G::NW * 64), 0, s, a);
  return (int)hipGetLastError();
}

static int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

// the persistent kernel takes 16 x 16 tiles (HaloSmall) for images that are not a multiple of 16 x 32
// (ArcFace 112 .. 14, overhanging tiles) — or, with GHOST_HALO_PP_SMALL=1, also the generator's 16 x 16 stage (A/B knob;
// its 1024 -> 1024 and cat 2048 -> 512 convs are outside the persistent kernel's N <= 512 / NCB <= 32 anyway)
static bool pp_small(const ConvDesc& d) {
  static const int force = GHOST_KNOB("GHOST_HALO_PP_SMALL", 0);
  return !halo_exact_wide(d) && halo_small_ok(d) &&
         (force || d.Wi % HaloSmall::TW || d.Hi % HaloSmall::TH || d.prelu || d.y2 || d.res_first);
}

template <typename T, class G>
static int halo_pp_launch(const ConvDesc& d, hipStream_t s) {
  HaloArgs a{};
  a.x = d.x; a.w = d.w; a.y = d.y;
  a.scale = d.scale; a.shift = d.shift; a.res = d.res;
  a.H = d.Hi; a.W = d.Wi; a.Cin = d.Cin; a.ldx = d.ldx; a.N = d.N; a.Kpad = d.Kpad;
  a.ldy = d.ldy; a.ldres = d.ldres; a.tanh_out = d.tanh_out; a.slope = d.slope;
  a.prelu = d.prelu; a.y2 = d.y2; a.scale2 = d.scale2; a.shift2 = d.shift2; a.ldy2 = d.ldy2;
  a.res_first = d.res_first;
  a.tiles_x = (d.Wi + G::TW - 1) / G::TW; a.tiles_y = (d.Hi + G::TH - 1) / G::TH; a.nNt = d.N / 64;
  a.ntiles = d.B / G::IMG * a.tiles_x * a.tiles_y * a.nNt;
  static const int dbg = GHOST_KNOB("GHOST_HALO_DBG", 0);
  a.dbg = dbg;
  // (A/B knob, tuning build) the persistent grid as a share of the CUs: with two batches in flight the other
  // batch's kernels can only use the CUs this kernel's 150 KB-LDS workgroups leave free
  static const int pct = GHOST_KNOB("GHOST_PP_GRID_PCT", 100);
  const int ncu = pct >= 100 ? num_cus() : (num_cus() * pct / 100 + 7) / 8 * 8;
  const int g = a.ntiles < ncu ? a.ntiles : ncu;
  a.in_part = d.in_part;
  const bool resw = d.Cin <= 64 && d.N == 64;
  const int ncb = d.Cin / 32;
  constexpr int NT = G::NW * 64;
#ifdef GHOST_TUNING
  if constexpr (G::TW == 32) {
    if (dbg) {   // experiment variants, with or without the InstanceNorm partials (tuning builds only)
#define GHOST_PP_DBX(R, NB, V)                                                                                    \
  if (resw == R && ncb == NB && dbg == V) {                                                                      \
    if (a.in_part)                                                                                               \
      hipLaunchKernelGGL((conv3x3_halo_pp_kernel<T, G, R, true, NB, V>), dim3((unsigned)g), dim3(NT), 0, s, a);  \
    else                                                                                                         \
      hipLaunchKernelGGL((conv3x3_halo_pp_kernel<T, G, R, false, NB, V>), dim3((unsigned)g), dim3(NT), 0, s, a); \
    return (int)hipGetLastError();                                                                               \
  }
      GHOST_PP_DBX(true, 2, 4096) GHOST_PP_DBX(false, 4, 4096) GHOST_PP_DBX(false, 8, 4096)
      // where the 256 x 256 conv's time goes: 2 no halo DMA, 16 no output stores, 32 no epilogue, 34 neither
      GHOST_PP_DBX(true, 2, 2) GHOST_PP_DBX(true, 2, 16) GHOST_PP_DBX(true, 2, 32) GHOST_PP_DBX(true, 2, 34)
      GHOST_PP_DBX(true, 2, 8)
      GHOST_PP_DBX(false, 16, 4096) GHOST_PP_DBX(false, 32, 4096)
#undef GHOST_PP_DBX
    }
  }
#endif
  constexpr bool CAN_ST = G::TW != 16;   // the partials come from exact 16 x 32 tiles or whole 8 x 8 images
#define GHOST_PP(R, ST, NB) \
  hipLaunchKernelGGL((conv3x3_halo_pp_kernel<T, G, R, ST, NB>), dim3((unsigned)g), dim3(NT), 0, s, a)
#define GHOST_PP2(R, NB)                                  \
  if constexpr (CAN_ST) {                                  \
    if (a.in_part) GHOST_PP(R, CAN_ST, NB); else GHOST_PP(R, false, NB); \
  } else {                                                 \
    if (a.in_part) return -1;                              \
    GHOST_PP(R, false, NB);                                \
  }
  if (resw) {
    GHOST_PP2(true, 2)
  } else {
    switch (ncb) {
      case 2: GHOST_PP2(false, 2) break;
      case 4: GHOST_PP2(false, 4) break;
      case 6: GHOST_PP2(false, 6) break;
      case 8: GHOST_PP2(false, 8) break;
      case 16: GHOST_PP2(false, 16) break;
      case 32: GHOST_PP2(false, 32) break;
      default: return -1;
    }
  }
#undef GHOST_PP2
#undef GHOST_PP
  return (int)hipGetLastError();
}

bool conv3x3_pp_takes(const ConvDesc& d, int* nrec) {
  static const int pp = GHOST_KNOB("GHOST_HALO_PP", 1);
  if (!conv3x3_halo_supported(d)) return false;
  if (d.prelu || d.y2 || d.res_first) return false;   // epilogue variants of the non-persistent kernel only
  if (d.ldy % 8 || (uintptr_t)d.y % 16) return false;   // the 16-byte epilogue stores (W16)
  if (halo_img8(d)) {
    const int ncb = d.Cin / 32;
    const bool ok8 = ncb == 2 || ncb == 4 || ncb == 8 || ncb == 16 || ncb == 32;
    if (ok8 && nrec) *nrec = 1;   // a wave's 64 pixels are one whole image
    return ok8;
  }
  const bool wide = halo_exact_wide(d);
  static const int max_cin = GHOST_KNOB("GHOST_HALO_PP_MAXCIN", 1024);
  // measured A/B (B = 64): the persistent form wins at every generator shape with W % 32 == 0 (256x256:
  // -23 %, 128x128: -7 %, 64x64 256->256: -9 %; with the counted first-stage wait also 64x64 512->128
  // -11 %, 32x32 512->512 -6 %, 32x32 1024->256 -8 %: +3 % frames/s end to end)
  const bool cin_ok = d.Cin == 64 || d.Cin == 128 || d.Cin == 192 || d.Cin == 256 || d.Cin == 512 || d.Cin == 1024;
  const bool ok = wide && pp && d.N <= 512 && d.N % 64 == 0 && cin_ok && d.Cin <= max_cin && !d.tanh_out;
  // records per sample: one per wave and tile = 64 pixels each (16 x 32 tiles x 8 waves)
  if (ok && nrec) *nrec = (d.Hi / HaloWide::TH) * (d.Wi / HaloWide::TW) * 8;
  return ok;
}

template <typename T>
static int conv3x3_halo_t(const ConvDesc& d, hipStream_t s) {
  if (halo_img8(d)) return conv3x3_pp_takes(d, nullptr) ? halo_pp_launch<T, HaloImg8>(d, s) : -1;
  if (conv3x3_pp_takes(d, nullptr)) return halo_pp_launch<T, HaloWide>(d, s);
  if (d.in_part) return -1;   // only the persistent 16 x 32 kernel writes InstanceNorm partials
  static const int pp = GHOST_KNOB("GHOST_HALO_PP", 1);
  const int ncb = d.Cin / 32;
  if (pp && pp_small(d) && d.N <= 512 && d.Cin % 64 == 0 &&
      (ncb == 2 || ncb == 4 || ncb == 6 || ncb == 8 || ncb == 16 || ncb == 32)) {
    // two samples per tile (HaloPair) when the batch pairs up: every weight stage serves both.  Measured
    // (ArcFace iresnet100 bf16, per conv): it wins wherever the paired grid still has a work item per CU —
    // B = 128: 14x14 51.2 -> 40.8 us, 28x28 63.9 -> 51.2, 56x56 107.7 -> 83.8; B = 64: 28x28 35.3 -> 29.2,
    // 56x56 59.4 -> 46.6 — and loses below that (B = 64 at 14x14, 128 items: 28.8 -> 36.2 us)
    static const int pair = GHOST_KNOB("GHOST_HALO_PAIR", 1);
    const long pair_items = (long)(d.B / 2) * ((d.Wi + 15) / 16) * ((d.Hi + 15) / 16) * (d.N / 64);
    if (pair && d.B % 2 == 0 && d.N <= 256 && pair_items >= num_cus()) return halo_pp_launch<T, HaloPair>(d, s);
    return halo_pp_launch<T, HaloSmall>(d, s);
  }
  if (halo_exact_wide(d)) return halo_launch<T, HaloWide>(d, s);
  return halo_launch<T, HaloSmall>(d, s);
}

int conv3x3_halo(const ConvDesc& d, hipStream_t s) {
  if (!conv3x3_halo_supported(d)) return -1;
  return d.ti == GHOST_F16 ? conv3x3_halo_t<_Float16>(d, s) : conv3x3_halo_t<bf16>(d, s);
}

}  // namespace ghost
