// ghost_amd — AADLayer kernel for the wide stages (C >= 256: 16x16 .. 64x64, bf16).
//
// AADLayer.py:20-38 (+ the ReLU that follows it) as in aad_v3.hip (transposed MFMA whose
// accumulators are gamma/beta of 16 channels of one pixel, register epilogue), but a
// workgroup owns ONE 64-channel tile of a block of pixels: the tile's 128 permuted weight
// rows (pack.py pack_aad_v3) fit LDS for any Ca <= 512, where all C/64 tiles would not.
// The mask needs every channel of the pixel: it comes from one aad_mask pass over h_in
// (ops.hip), so a 16-pixel tile here is one round trip: z_attr row, the tile's 64 channels of
// h_in and the mask.  The C/64 workgroups of one pixel block are adjacent in launch order (and
// on one XCD), so their shared z_attr reads are L2 hits.
#include <cstdlib>

#include "aad_wide.h"
#include "ghost_common.h"

namespace ghost {

struct AadWideArgs {
  const void* za;
  const void* hin;
  const float* stat;
  const void* w3;
  const float* b3;
  const float* wh;
  const float* bh;
  const float* idgb;
  const float* mask;
  void* out;
  int lda, ldh, ldo, id_ld, HW, PPW, nblk;
  float slope;
};

static constexpr int kWideWaves = 8;

GHOST_DEV int wide_xcd_tile(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <typename T, int C, int CA>
GHOST_DEV void aad_wide_body(const AadWideArgs& a) {
  const T* __restrict__ za = reinterpret_cast<const T*>(a.za);
  const T* __restrict__ hin = reinterpret_cast<const T*>(a.hin);
  const T* __restrict__ w3 = reinterpret_cast<const T*>(a.w3);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  constexpr int CT = C / 64;
  constexpr int KS = CA / 32;
  constexpr int WLD = CA + 8;
  __shared__ __attribute__((aligned(16))) T s_w[128 * WLD];
  __shared__ __attribute__((aligned(16))) float s_b[128];
  __shared__ __attribute__((aligned(16))) float s_rs[64];
  __shared__ __attribute__((aligned(16))) float s_nm[64];
  __shared__ __attribute__((aligned(16))) float s_gi[64];
  __shared__ __attribute__((aligned(16))) float s_bi[64];

  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int tile = wide_xcd_tile(blockIdx.x, gridDim.x);
  const int ct = tile % CT, blk = tile / CT;
  const long p_begin = (long)blk * a.PPW;
  const int b = (int)(p_begin / a.HW);

  for (int idx = tid; idx < 128 * (CA / 8); idx += kWideWaves * 64) {
    const int row = idx / (CA / 8), kc = idx - row * (CA / 8);
    *reinterpret_cast<u32x4*>(&s_w[row * WLD + kc * 8]) =
        *reinterpret_cast<const u32x4*>(w3 + (long)(ct * 128 + row) * CA + kc * 8);
  }
  for (int i = tid; i < 128; i += kWideWaves * 64) s_b[i] = a.b3[ct * 128 + i];
  if (tid < 64) {
    const int c = ct * 64 + tid;
    const float mu = a.stat[((long)b * C + c) * 2], rs = a.stat[((long)b * C + c) * 2 + 1];
    s_rs[tid] = rs;
    s_nm[tid] = -mu * rs;
    s_gi[tid] = a.idgb[(long)b * a.id_ld + c];
    s_bi[tid] = a.idgb[(long)b * a.id_ld + C + c];
  }
  __syncthreads();

  const int ntiles = a.PPW / 16;
  for (int t = wid; t < ntiles; t += kWideWaves) {
    asm volatile("" ::: "memory");
    const long p = p_begin + t * 16 + lr;
    const T* hrow = hin + p * a.ldh + ct * 64;
    // one round trip: the z_attr row, this tile's two h_in chunks and the mask
    constexpr bool ZEARLY = true;   // the whole z_attr row is in flight with the h_in chunks
    u32x4 zc[ZEARLY ? KS : 1];
    if constexpr (ZEARLY) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) zc[ks] = *reinterpret_cast<const u32x4*>(za + p * a.lda + ks * 32 + lq * 8);
    }
    u32x4 hc[2];
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) hc[sh] = *reinterpret_cast<const u32x4*>(hrow + sh * 32 + lq * 8);
    const float Mk = a.mask[p];

#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      asm volatile("" ::: "memory");
      const int cl = sh * 32 + lq * 8;     // channel within the tile
      f32x4 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rt = (i & 1) + 2 * sh + 4 * (i >> 1);
        acc[i] = *reinterpret_cast<const f32x4*>(&s_b[rt * 16 + lq * 4]);
      }
#pragma unroll
      for (int k0 = 0; k0 < KS; k0 += 4) {
        u32x4 zg[4];
        if constexpr (ZEARLY) {
#pragma unroll
          for (int u = 0; u < 4; ++u) if (k0 + u < KS) zg[u] = zc[k0 + u];
        } else {
          asm volatile("" ::: "memory");
#pragma unroll
          for (int u = 0; u < 4; ++u)
            zg[u] = *reinterpret_cast<const u32x4*>(za + p * a.lda + (k0 + u) * 32 + lq * 8);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (k0 + u >= KS) break;
          const int ks = k0 + u;
          v8_t<T> bfrag;
          __builtin_memcpy(&bfrag, &zg[u], 16);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rt = (i & 1) + 2 * sh + 4 * (i >> 1);
            const v8_t<T> afrag = *reinterpret_cast<const v8_t<T>*>(&s_w[(rt * 16 + lr) * WLD + ks * 32 + lq * 8]);
            acc[i] = mfma16x16x32<T>(afrag, bfrag, acc[i]);
          }
        }
      }
      const T* hv = reinterpret_cast<const T*>(&hc[sh]);
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float hh = fmaf((float)hv[e], s_rs[cl + e], s_nm[cl + e]);
        const float A = fmaf(acc[e >> 2][e & 3], hh, acc[2 + (e >> 2)][e & 3]);
        const float I = fmaf(s_gi[cl + e], hh, s_bi[cl + e]);
        const float v = fmaf(Mk, I - A, A);
        o[e] = v > 0.f ? v : v * a.slope;
      }
      store16_f(out + p * a.ldo + ct * 64 + cl, o);
    }
  }
}

// Ca <= 256: 4 waves per SIMD (<= 128 VGPRs), two workgroups per CU.  Ca = 512: the 133 KB of
// weight rows allow one workgroup per CU, so the z_attr row (64 VGPRs) may use the registers.
// (Measured alternative, not kept: each wave on four 16-pixel tiles per weight fragment — 4x less
// LDS traffic per MFMA, 300-390 registers, one wave per SIMD — ran 10-17 % slower at 16x16-64x64.)
template <typename T, int C, int CA>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8))) aad_wide_kernel(const AadWideArgs a) {
  aad_wide_body<T, C, CA>(a);
}
template <typename T, int C, int CA>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 8))) aad_wide_deep_kernel(const AadWideArgs a) {
  aad_wide_body<T, C, CA>(a);
}

// ---------------------------------------------------------------------------------------------
// aad_gemm: the same layer as a 256 x 256 MFMA tile GEMM (the 16x16 stage: C % 128 == 0, Ca = 512).
//
// aad_wide re-reads the z_attr row for every 64-channel tile (C / 64 times: 16x at C = 1024) and keeps
// one 16-pixel tile per wave, so it runs on the L2 -> CU path (measured 78-83 us for a 16x16 layer
// whose HBM and MFMA floors are ~14 us each).  Here a workgroup owns 256 weight rows (two 64-channel
// tiles of the permuted pack_aad_v3 layout) x 256 pixels of one sample, K = Ca streamed in 64-deep
// stages by LDS-DMA into two buffers (128 B rows, chunk c of row r at c ^ ((r >> 1) & 7): conflict-
// free 16-row fragment reads).  4 waves, each 128 rows x 128 pixels (64 accumulator tiles): the
// operands of 64 MFMAs cost 16 fragment reads.  The epilogue is aad_v3's register blend (a lane holds
// gamma / beta of 8 channels of one pixel) with the mask of the aad_mask pass.
// ---------------------------------------------------------------------------------------------
GHOST_DEV int gswz(int r) { return (r >> 1) & 7; }

template <typename T, int CA>
__global__ void __launch_bounds__(256) aad_gemm_kernel(const AadWideArgs a, int C) {
  constexpr int NST = CA / 64;                 // K stages
  static_assert(NST % 2 == 0, "stages are ping-ponged in pairs");
  constexpr int STAGE_B = 512 * 128;           // 256 weight rows + 256 pixel rows, 128 B each
  __shared__ __attribute__((aligned(1024))) unsigned char lds0[STAGE_B];
  __shared__ __attribute__((aligned(1024))) unsigned char lds1[STAGE_B];
  __shared__ __attribute__((aligned(16))) float s_b[256];
  __shared__ __attribute__((aligned(16))) float s_rs[128], s_nm[128], s_gi[128], s_bi[128];
  __shared__ __attribute__((aligned(1024))) float s_mask[256];

  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int ncp = C / 128;
  const int tile = wide_xcd_tile(blockIdx.x, gridDim.x);
  const int cp = tile % ncp, pb = tile / ncp;
  const long p0 = (long)pb * 256;
  const int b = (int)(p0 / a.HW);              // HW % 256 == 0: one sample per tile
  const int c0 = cp * 128;                     // first channel; weight rows cp*256 .. +256
  const T* wsrc = reinterpret_cast<const T*>(a.w3) + (long)cp * 256 * CA;
  const T* zsrc = reinterpret_cast<const T*>(a.za) + p0 * a.lda;

  // DMA: 64 pieces of 8 rows x 128 B per stage (32 weight + 32 pixel), 16 per wave
  const int prow = lane >> 3, pch = lane & 7;
  auto issue = [&](unsigned char* buf, int st) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int k0 = st * 64;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int q = wid + 4 * j;               // piece 0..63: < 32 weights, >= 32 pixels
      const int row = (q & 31) * 8 + prow;
      const int lc = pch ^ gswz(row);          // logical chunk this lane's physical slot holds
      const T* src = q < 32 ? wsrc + (long)row * CA + k0 + lc * 8 : zsrc + (long)row * a.lda + k0 + lc * 8;
      __builtin_amdgcn_global_load_lds(src, buf + q * 1024, 16, 0, 0);
    }
#endif
  };
  issue(lds0, 0);

  for (int i = tid; i < 256; i += 256) s_b[i] = a.b3[cp * 256 + i];
  if (tid < 128) {
    const int c = c0 + tid;
    const float mu = a.stat[((long)b * C + c) * 2], rs = a.stat[((long)b * C + c) * 2 + 1];
    s_rs[tid] = rs;
    s_nm[tid] = -mu * rs;
    s_gi[tid] = a.idgb[(long)b * a.id_ld + c];
    s_bi[tid] = a.idgb[(long)b * a.id_ld + C + c];
  }

  const int wr = wid & 1, wp = wid >> 1;       // rows wr*128.. (channel tile), pixels wp*128..
  f32x4 acc[8][8];
#pragma unroll
  for (int rt = 0; rt < 8; ++rt)
#pragma unroll
    for (int pf = 0; pf < 8; ++pf) acc[rt][pf] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const unsigned char* buf) {
    const unsigned char* Wb = buf;
    const unsigned char* Zb = buf + 256 * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8_t<T> af[8], bfr[8];
#pragma unroll
      for (int rt = 0; rt < 8; ++rt) {
        const int row = wr * 128 + rt * 16 + lr;
        af[rt] = *reinterpret_cast<const v8_t<T>*>(Wb + row * 128 + (((ks * 4 + lq) ^ gswz(row)) * 16));
      }
#pragma unroll
      for (int pf = 0; pf < 8; ++pf) {
        const int row = wp * 128 + pf * 16 + lr;
        bfr[pf] = *reinterpret_cast<const v8_t<T>*>(Zb + row * 128 + (((ks * 4 + lq) ^ gswz(row)) * 16));
      }
#pragma unroll
      for (int rt = 0; rt < 8; ++rt)
#pragma unroll
        for (int pf = 0; pf < 8; ++pf)
          acc[rt][pf] = mfma16x16x32<T>(af[rt], bfr[pf], acc[rt][pf]);
    }
  };
  // the epilogue's inputs — the tile's h_in (256 pixels x 128 channels = 64 KB) and its 256 mask values —
  // are DMA'd into the free stage buffer and s_mask while the last K stage computes, instead of 16
  // dependent global loads per lane after it (chunk c of pixel P at 16-byte slot c ^ (P & 15): the 16
  // pixels a lane group reads hit 16 bank groups)
  auto issue_epi = [&]() {
#if defined(__HIP_DEVICE_COMPILE__)
    const int wu = __builtin_amdgcn_readfirstlane(wid);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int q = wu + 4 * j;                  // piece: pixels 4q .. 4q+3
      const int P = q * 4 + (lane >> 4), lc = (lane & 15) ^ (P & 15);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const T*>(a.hin) + (p0 + P) * a.ldh + c0 + lc * 8, lds0 + q * 1024,
                                       16, 0, 0);
    }
    if (wu == 0) __builtin_amdgcn_global_load_lds(a.mask + p0 + lane * 4, (unsigned char*)s_mask, 16, 0, 0);
#endif
  };
  // stage pairs: even stages read lds0 and prefetch into lds1, odd ones the reverse (distinct LDS
  // objects, static waits: the compiler does not drain the in-flight DMA before the fragment reads)
  for (int st = 0; st < NST; st += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    issue(lds1, st + 1);
    compute(lds0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (st + 2 < NST) issue(lds0, st + 2);
    else issue_epi();
    compute(lds1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue (aad_v3's register blend): lane holds, per pixel fragment pf and half sh, gamma / beta of
  // channels wr*64 + 32sh + 8lq + e (e < 8) of pixel wp*128 + 16pf + lr
#pragma unroll
  for (int pf = 0; pf < 8; ++pf) {
    const int P = wp * 128 + pf * 16 + lr;                  // pixel within the tile
    const long p = p0 + P;
    const float Mk = s_mask[P];
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      const int cl = wr * 64 + sh * 32 + lq * 8;           // channel within the 128 of the tile
      float hv[8];
      {
        const u32x4 raw = *reinterpret_cast<const u32x4*>(lds0 + P * 256 + (((cl >> 3) ^ (P & 15)) * 16));
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int i = 0; i < 8; ++i) hv[i] = (float)e[i];
      }
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i0 = e >> 2, r = e & 3;
        const int rg = (i0 & 1) + 2 * sh, rb = rg + 4;       // gamma / beta row tiles
        const float g = acc[rg][pf][r] + s_b[wr * 128 + rg * 16 + lq * 4 + r];
        const float be = acc[rb][pf][r] + s_b[wr * 128 + rb * 16 + lq * 4 + r];
        const float hh = fmaf(hv[e], s_rs[cl + e], s_nm[cl + e]);
        const float A = fmaf(g, hh, be);
        const float I = fmaf(s_gi[cl + e], hh, s_bi[cl + e]);
        const float v = fmaf(Mk, I - A, A);
        o[e] = v > 0.f ? v : v * a.slope;
      }
      store16_f(reinterpret_cast<T*>(a.out) + p * a.ldo + c0 + cl, o);
    }
  }
}

namespace {
int wide_ppw(int B, int HW, int C, int Ca) {
  // as many pixels per workgroup as keep a full round of workgroups (two per CU; one for the
  // 133 KB Ca = 512 rows): the weight rows staged per workgroup are then amortised over as
  // many 16-pixel tiles as possible
  const long minwg = Ca > 256 ? 256 : 512;
  static const int force = GHOST_KNOB("GHOST_AAD_WIDE_PPW", 0);
  if (force > 0 && HW % force == 0 && force % 16 == 0) return force;
  int best = 0;
  for (int ppw = 16; ppw <= HW && ppw <= 4096; ppw *= 2)
    if (HW % ppw == 0 && (best == 0 || (long)B * HW / ppw * (C / 64) >= minwg)) best = ppw;
  return best;
}
}  // namespace

bool aad_wide_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo) {
  if (!is16(dt)) return false;
  const bool shape = (C == 256 || C == 512 || C == 1024) && (Ca == 64 || Ca == 128 || Ca == 256 || Ca == 512);
  if (!shape || lda % 8 || ldh % 8 || ldo % 8) return false;
  const int ppw = wide_ppw(B, HW, C, Ca);
  return ppw > 0 && (long)B * HW / ppw * (C / 64) >= 256;
}

static bool aad_gemm_ok(const AadWideDesc& d) {
  static const int on = GHOST_KNOB("GHOST_AAD_GEMM", 1);
  // Ca = 512 only: at Ca = 256 (the 32x32 stage) four K stages do not amortise the tile's prologue and
  // epilogue at one workgroup per CU (measured 80-86 us against aad_wide's 52-57 us; Ca = 512: 62-66
  // against 78-83 us)
  // and only where the 256 x 256 tiles make half a round of workgroups: at B = 1 the 16 x 16 stage is 8 of them
  // (28-32 us each, profiles/r05_step_trace_b1.txt); aad_wide's 16-pixel workgroups spread the layer over the CUs
  const long wgs = (long)d.B * d.HW / 256 * (d.C / 128);
  return on && d.HW % 256 == 0 && d.C % 128 == 0 && d.Ca == 512 && d.lda % 8 == 0 &&
         d.ldh % 8 == 0 && d.ldo % 8 == 0 && (uintptr_t)d.za % 16 == 0 && (uintptr_t)d.w3 % 16 == 0 && wgs >= 128;
}

template <typename T>
static int aad_wide_t(const AadWideDesc& d, hipStream_t s);

int aad_wide(const AadWideDesc& d, hipStream_t s) {
  if (!aad_wide_supported(d.dt, d.B, d.HW, d.C, d.Ca, d.lda, d.ldh, d.ldo) || !d.mask) return -1;
  return d.dt == GHOST_F16 ? aad_wide_t<_Float16>(d, s) : aad_wide_t<bf16>(d, s);
}

template <typename T>
static int aad_wide_t(const AadWideDesc& d, hipStream_t s) {
  AadWideArgs a{};
  a.za = d.za; a.hin = d.hin; a.stat = d.stat;
  a.w3 = d.w3; a.b3 = d.b3; a.wh = d.wh; a.bh = d.bh; a.idgb = d.idgb; a.mask = d.mask; a.out = d.out;
  a.lda = d.lda; a.ldh = d.ldh; a.ldo = d.ldo; a.id_ld = d.id_ld; a.HW = d.HW; a.slope = d.slope;
  if (aad_gemm_ok(d)) {
    dim3 g((unsigned)((long)d.B * d.HW / 256 * (d.C / 128)));
    hipLaunchKernelGGL((aad_gemm_kernel<T, 512>), g, dim3(256), 0, s, a, d.C);
    return (int)hipGetLastError();
  }
  a.PPW = wide_ppw(d.B, d.HW, d.C, d.Ca);
  a.nblk = (int)((long)d.B * d.HW / a.PPW);
  dim3 grid((unsigned)(a.nblk * (d.C / 64)));
#define GHOST_W(c, ca)                                                                 \
  if (d.C == c && d.Ca == ca) {                                                        \
    hipLaunchKernelGGL((aad_wide_kernel<T, c, ca>), grid, dim3(kWideWaves * 64), 0, s, a); \
    return (int)hipGetLastError();                                                     \
  }
  GHOST_W(256, 64) GHOST_W(256, 128) GHOST_W(256, 256) GHOST_W(512, 64) GHOST_W(512, 128) GHOST_W(512, 256)
  GHOST_W(1024, 64) GHOST_W(1024, 128) GHOST_W(1024, 256)
#undef GHOST_W
#define GHOST_WD(c, ca)                                                                     \
  if (d.C == c && d.Ca == ca) {                                                             \
    hipLaunchKernelGGL((aad_wide_deep_kernel<T, c, ca>), grid, dim3(kWideWaves * 64), 0, s, a); \
    return (int)hipGetLastError();                                                          \
  }
  GHOST_WD(512, 512) GHOST_WD(1024, 512)
#undef GHOST_WD
  return -1;
}

}  // namespace ghost
