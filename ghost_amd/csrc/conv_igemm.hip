// ghost_amd — implicit-GEMM convolution on CDNA4 matrix cores (gfx950).
//
// Tile: BM output pixels x BN output channels x BK=32 reduction, 256 threads = 4 waves
// in a 2x2 arrangement, each wave owning (BM/2)x(BN/2) as 16x16 MFMA tiles.
//   bf16: v_mfma_f32_16x16x32_bf16  (one instruction per 16x16x32 step)
//   fp32: v_mfma_f32_16x16x4_f32    (exact fp32 products, fp32 accumulate — the 1e-3 parity path)
// The A tile (pixels x (tap,cin)) is gathered from NHWC activations with zero padding
// at the borders; when Cin % 32 == 0 a 32-deep K slice lies inside one tap, so every
// row is one contiguous 64 B (bf16) / 128 B (fp32) run loaded as 16 B vectors.
// Staging: global -> registers -> LDS, double-buffered, one barrier per K step.
#include <cstdio>
#include <cstdlib>

#include "conv_igemm.h"
#include "conv_first.h"
#include "conv_halo.h"
#include "conv_s2.h"
#include "ghost_common.h"

namespace ghost {

struct ConvArgs {
  const void* x;
  const void* w;
  void* y;
  const float* scale;
  const float* shift;
  const void* res;
  const float* prelu;
  void* y2;
  const float* scale2;
  const float* shift2;
  const void* hin;
  const float* stat;
  const float* idgb;
  const float* mask;
  float* partial;
  uint8_t* u8;
  long wpar_stride;
  int B, Hi, Wi, Cin, ldx;
  int Ho, Wo, M;        // GEMM pixel grid (the sub-pixel grid for CONV_T4S2)
  int N, Kpad, K, NT;   // NT = padded channel extent covered by tiles
  int nNt;              // number of channel tiles
  int ldy, ldres, ldh, id_ld, C_aad, ldy2, res_first;
  int stride, ntx, ntaps, tbase, tsign;   // input coord = out*stride + tbase + tsign*tap  (per dim)
  int deconv;           // 1: four parity phases in blockIdx.z, output pixel (2qy+py, 2qx+px)
  int nsplit, kt_per_split;
  float slope;
  int tanh_out;
  int nmajor;           // 1: tiles ordered N-major, so each XCD's contiguous run of tiles shares weight rows
  unsigned* sem;        // split-K fix-up counters, one per (phase, tile) (nullptr: splitk_reduce_kernel follows)
  int fuse;             // the fix-up's epilogue: 1 = standard, 2 = AAD
};

// ---------------------------------------------------------------------------
// epilogues (shared by the GEMM kernel and the split-K reduction)
// ---------------------------------------------------------------------------
template <typename TO>
GHOST_DEV float epi_std(const ConvArgs& a, float v, int n, long opix) {
  if (a.scale) v *= a.scale[n];
  if (a.shift) v += a.shift[n];
  const float r = a.res ? to_f(reinterpret_cast<const TO*>(a.res)[opix * a.ldres + n]) : 0.f;
  if (a.res_first) v += r;
  const float sl = a.prelu ? a.prelu[n] : a.slope;
  v = v > 0.f ? v : v * sl;
  if (!a.res_first) v += r;
  if (a.tanh_out) v = tanhf(v);
  return v;
}

template <typename TO>
GHOST_DEV void store_std(const ConvArgs& a, float v, int n, long opix) {
  reinterpret_cast<TO*>(a.y)[opix * a.ldy + n] = from_f<TO>(v);
  if (a.y2) reinterpret_cast<TO*>(a.y2)[opix * a.ldy2 + n] = from_f<TO>(v * a.scale2[n] + a.shift2[n]);
  if (a.u8) {
    // ((Y*0.5+0.5)*255)[..., [2,1,0]].type(uint8)   (faceshifter_run.py:20-21)
    float t = (v * 0.5f + 0.5f) * 255.0f;
    a.u8[opix * 3 + (2 - n)] = (uint8_t)(int)t;
  }
}

// AADLayer.forward (AADLayer.py:20-38) for one (pixel m, channel c), followed by the
// ReLU of AddBlocksSequential when slope == 0:
//   h = (h_in - mu) * rstd;  A = ga*h + ba;  I = gi*h + bi;  out = (1-M)*A + M*I
template <typename TO>
GHOST_DEV float epi_aad(const ConvArgs& a, float ga, float ba, int c, long m) {
  const int HW = a.Ho * a.Wo;
  const int b = (int)(m / HW);
  const float hin = to_f(reinterpret_cast<const TO*>(a.hin)[m * a.ldh + c]);
  const float mu = a.stat[((long)b * a.C_aad + c) * 2 + 0];
  const float rs = a.stat[((long)b * a.C_aad + c) * 2 + 1];
  const float h = (hin - mu) * rs;
  const float gi = a.idgb[(long)b * a.id_ld + c];
  const float bi = a.idgb[(long)b * a.id_ld + a.C_aad + c];
  const float Mk = a.mask[m];
  const float A = ga * h + ba;
  const float I = gi * h + bi;
  float out = (1.0f - Mk) * A + Mk * I;
  return out > 0.f ? out : out * a.slope;
}

GHOST_DEV long out_pixel(const ConvArgs& a, long m, int py, int px) {
  if (!a.deconv) return m;
  const int HW = a.Ho * a.Wo;
  const int b = (int)(m / HW);
  const int r = (int)(m - (long)b * HW);
  const int qy = r / a.Wo, qx = r - qy * a.Wo;
  return ((long)b * (2 * a.Ho) + 2 * qy + py) * (2 * a.Wo) + 2 * qx + px;
}

// Split-K fix-up, run by every workgroup of a KEPI_SPLIT launch after its partial tile is stored (st_dev): the
// last of a tile's nsplit workgroups to arrive (a counter per (phase, tile), zeroed per call and reset by that
// workgroup) sums the tile's nsplit partials in split order from 0 — splitk_reduce_kernel's order, so the output
// bytes are the same — and applies the epilogue.  Saves the reduction's launch (the small-M GEMMs of the
// generator's 2x2..8x8 stages and the encoder's low-resolution convs each had one).  Only for tiles whose
// partials fit `stage` (the kernel's own LDS, free after the K loop): the last arriver first pulls all of them
// into LDS with one batch of independent device-scope loads per thread (a dependent load per split costs a
// fabric round trip each, cdna_hip_programming.md §6 item 2), then sums from LDS.
template <typename TO, int BM, int BN, int NTHR>
GHOST_DEV void split_fixup(const ConvArgs& a, int tid, int tile_id, int m0, int n0, int par, float* stage) {
  if (!last_arrival(a.sem + tile_id, (unsigned)a.nsplit, reinterpret_cast<int*>(stage))) return;
  __syncthreads();   // every thread has read the flag (stage[0]) before the staging below overwrites it
  const int py = par >> 1, px = par & 1;
  const int mrows = min(BM, a.M - m0);
  const long sstride = (long)a.M * a.NT;
  const float* pbase = a.partial + (long)par * a.nsplit * sstride + (long)m0 * a.NT + n0;
  // stage[s][r][q] = partial of split s, tile row r, tile column q (q < BN: the whole tile width, inside NT)
  const int per_split = mrows * BN, total = a.nsplit * per_split;
  constexpr int U = 8;
  for (int f0 = tid; f0 < total; f0 += U * NTHR) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = min(f0 + u * NTHR, total - 1);   // clamped, not skipped: every load issued before any use
      const int sp = f / per_split, e = f - sp * per_split;
      const int r = e / BN, q = e - r * BN;
      v[u] = ld_dev(pbase + sp * sstride + (long)r * a.NT + q);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (f0 + u * NTHR < total) stage[f0 + u * NTHR] = v[u];
  }
  __syncthreads();
  if (a.fuse == 1) {
    const int ncol = min(BN, a.N - n0);
    for (int i = tid; i < mrows * ncol; i += NTHR) {
      const int r = i / ncol, q = i - r * ncol;
      float v = 0.f;
      for (int sp = 0; sp < a.nsplit; ++sp) v += stage[sp * per_split + r * BN + q];
      const long op = out_pixel(a, m0 + r, py, px);
      store_std<TO>(a, epi_std<TO>(a, v, n0 + q, op), n0 + q, op);
    }
  } else {
    constexpr int CH = BN / 2;   // AAD channels per tile row: column pairs (gamma, beta) 16 apart
    for (int i = tid; i < mrows * CH; i += NTHR) {
      const int r = i / CH, cc = i - r * CH;
      const long m = m0 + r;
      const int q = (cc >> 4) * 32 + (cc & 15), ng = n0 + q;
      const int c = (ng >> 5) * 16 + (ng & 15);
      if (c >= a.C_aad) continue;
      float ga = 0.f, ba = 0.f;
      for (int sp = 0; sp < a.nsplit; ++sp) {
        ga += stage[sp * per_split + r * BN + q];
        ba += stage[sp * per_split + r * BN + q + 16];
      }
      ga += a.shift[ng];
      ba += a.shift[ng + 16];
      reinterpret_cast<TO*>(a.y)[m * a.ldy + c] = from_f<TO>(epi_aad<TO>(a, ga, ba, c, m));
    }
  }
}

// ---------------------------------------------------------------------------
// the GEMM kernel
// ---------------------------------------------------------------------------
enum { KEPI_STD = 0, KEPI_AAD = 1, KEPI_SPLIT = 2 };

// wave layout: 4 waves as 2x2 (BM <= 128, BN >= 32) or 4x1 (BM = 256 or a 16-wide N tile)
template <int BM, int BN> struct WaveGrid { static constexpr int WN = (BM <= 128 && BN >= 32) ? 2 : 1, WM = 4 / WN; };

template <typename TI, typename TO, int BM, int BN, int BK, int EPI, bool FAST>
__global__ void __launch_bounds__(256) conv_igemm_kernel(const ConvArgs a) {
  constexpr int VEC = Vec16<TI>::N;
  constexpr int CPR = BK / VEC;   // 16 B chunks per tile row
  constexpr int RPP = 256 / CPR;  // tile rows covered per load pass
  constexpr int AP = BM / RPP;
  constexpr int BP = (BN + RPP - 1) / RPP;   // BN may be smaller than one pass
  constexpr int LDR = BK + VEC;   // padded LDS row, elements
  constexpr int WM = WaveGrid<BM, BN>::WM, WN = WaveGrid<BM, BN>::WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;   // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(TM >= 1 && TN >= 1 && BK % 32 == 0, "tile shape");
  static_assert(BM % RPP == 0 && (BN % RPP == 0 || RPP % BN == 0), "tile/load mismatch");
  static_assert(EPI != KEPI_AAD || (TN % 2 == 0 && WTN % 32 == 0), "AAD epilogue needs gamma/beta tile pairs");

  __shared__ __attribute__((aligned(16))) TI smem[2 * (BM + BN) * LDR];

  const int tid = threadIdx.x;
  // XCD-aware remap: workgroups are dealt round-robin over the 8 XCDs; give each XCD a
  // contiguous run of tiles so the 3x3/4x4 halo rows a tile shares with its neighbours
  // are re-read from that XCD's L2 instead of HBM (cdna_hip_programming.md T1, bijective form)
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = tile % a.nNt;
  const int mt = tile / a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int split = blockIdx.y;
  const int par = blockIdx.z;
  const int py = par >> 1, px = par & 1;
  const TI* __restrict__ x = reinterpret_cast<const TI*>(a.x);
  const TI* __restrict__ w = reinterpret_cast<const TI*>(a.w) + par * a.wpar_stride;

  const int nk = a.Kpad / BK;
  const int kt0 = split * a.kt_per_split;
  const int kt1 = min(nk, kt0 + a.kt_per_split);

  // per-thread rows of the A tile, decoded once per tile: element offset of the tap-origin
  // pixel and a bitmask of the taps that land inside the image (the rest read as the zero
  // padding).  Per K step only a scalar tap offset and one bit test per row remain.
  const int crow = tid / CPR, cch = tid % CPR;
  const int HoWo = a.Ho * a.Wo;
  const int tby = a.deconv ? py : a.tbase;
  const int tbx = a.deconv ? px : a.tbase;
  const int nty = a.K / (a.Cin * a.ntx);
  long a_off[AP];
  uint64_t a_mask[AP];   // one bit per tap: kernels up to 8x8 (7x7 = 49 taps)
#pragma unroll
  for (int p = 0; p < AP; ++p) {
    const int m = m0 + crow + p * RPP;
    a_off[p] = 0;
    a_mask[p] = 0ull;
    if (m < a.M) {
      const int b = m / HoWo;
      const int r = m - b * HoWo;
      const int oy = r / a.Wo, ox = r - oy * a.Wo;
      const int iyb = oy * a.stride + tby, ixb = ox * a.stride + tbx;
      a_off[p] = ((long)(b * a.Hi + iyb) * a.Wi + ixb) * a.ldx;
      uint64_t mk = 0ull;
      for (int ty = 0; ty < nty; ++ty) {
        const int iy = iyb + a.tsign * ty;
        if (iy < 0 || iy >= a.Hi) continue;
        for (int tx = 0; tx < a.ntx; ++tx) {
          const int ix = ixb + a.tsign * tx;
          if (ix >= 0 && ix < a.Wi) mk |= 1ull << (ty * a.ntx + tx);
        }
      }
      a_mask[p] = mk;
    }
  }
  const TI* wrow[BP];
#pragma unroll
  for (int p = 0; p < BP; ++p) {
    // BN < RPP: the surplus threads re-load an in-tile row and do not store it
    const int n = n0 + (BN >= RPP ? crow + p * RPP : crow % BN);
    wrow[p] = w + (long)n * a.Kpad + cch * VEC;
  }

  u32x4 ra[AP], rb[BP];

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if constexpr (FAST) {
      // K is ordered (channel block of 32, tap, channel): a block's nine (or 16 / 4) taps are
      // consecutive K steps, so a tile re-reads the same few input rows from L1/L2 instead of
      // sweeping all channels once per tap (pack.py pack_conv)
      const int chunk = (k0 + cch * VEC) >> 5;
      const int cb = chunk / a.ntaps, tap = chunk - cb * a.ntaps;
      const int ty = tap / a.ntx, tx = tap - ty * a.ntx;
      const long toff = ((long)a.tsign * ty * a.Wi + a.tsign * tx) * a.ldx + cb * 32 + ((cch * VEC) & 31);
#pragma unroll
      for (int p = 0; p < AP; ++p) {
        if ((a_mask[p] >> tap) & 1ull)
          ra[p] = *reinterpret_cast<const u32x4*>(x + a_off[p] + toff);
        else
          ra[p] = u32x4{0u, 0u, 0u, 0u};
      }
    } else {
#pragma unroll
      for (int p = 0; p < AP; ++p) {
        TI* e = reinterpret_cast<TI*>(&ra[p]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int k = k0 + cch * VEC + j;
          float v = 0.f;
          if (k < a.K) {
            const int tap = k / a.Cin;
            const int c = k - tap * a.Cin;
            const int ty = tap / a.ntx, tx = tap - ty * a.ntx;
            if ((a_mask[p] >> tap) & 1ull)
              v = to_f(x[a_off[p] + ((long)a.tsign * ty * a.Wi + a.tsign * tx) * a.ldx + c]);
          }
          e[j] = from_f<TI>(v);
        }
      }
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) rb[p] = *reinterpret_cast<const u32x4*>(wrow[p] + k0);
  };
  auto store_tile = [&](int buf) {
    TI* As = smem + buf * (BM + BN) * LDR;
    TI* Bs = As + BM * LDR;
#pragma unroll
    for (int p = 0; p < AP; ++p) *reinterpret_cast<u32x4*>(As + (crow + p * RPP) * LDR + cch * VEC) = ra[p];
#pragma unroll
    for (int p = 0; p < BP; ++p)
      if (BN >= RPP || crow < BN) *reinterpret_cast<u32x4*>(Bs + (crow + p * RPP) * LDR + cch * VEC) = rb[p];
  };

  const int wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const TI* As = smem + buf * (BM + BN) * LDR;
    const TI* Bs = As + BM * LDR;
    const TI* Ab = As + (wm * WTM + lr) * LDR;
    const TI* Bb = Bs + (wn * WTN + lr) * LDR;
    if constexpr (sizeof(TI) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        v8_t<TI> af[TM], bfv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const v8_t<TI>*>(Ab + i * 16 * LDR + ks * 32 + lq * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const v8_t<TI>*>(Bb + j * 16 * LDR + ks * 32 + lq * 8);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma16x16x32<TI>(af[i], bfv[j], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int h = 0; h < BK / 16; ++h) {
        f32x4 af[TM], bfv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f32x4*>(Ab + i * 16 * LDR + h * 16 + lq * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const f32x4*>(Bb + j * 16 * LDR + h * 16 + lq * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], bfv[j][e], acc[i][j], 0, 0, 0);
      }
    }
  };

  // one load site and one store site keep the staging registers out of scratch
  int cur = 0;
  if (kt0 < kt1) load_tile(kt0);
  for (int kt = kt0; kt < kt1; ++kt) {
    store_tile(cur);
    __syncthreads();   // LDS[cur] visible; every wave is past compute(kt-2) on this buffer
    if (kt + 1 < kt1) load_tile(kt + 1);
    compute(cur);
    cur ^= 1;
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WTM + i * 16 + lq * 4 + r;
      if (m >= a.M) continue;
      if constexpr (EPI == KEPI_SPLIT) {
        float* dst = a.partial + (((long)par * a.nsplit + split) * a.M + m) * a.NT;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (a.sem) st_dev(dst + n0 + wn * WTN + j * 16 + lr, acc[i][j][r]);
          else dst[n0 + wn * WTN + j * 16 + lr] = acc[i][j][r];
        }
      } else if constexpr (EPI == KEPI_STD) {
        const long op = out_pixel(a, m, py, px);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * WTN + j * 16 + lr;
          if (n < a.N) store_std<TO>(a, epi_std<TO>(a, acc[i][j][r], n, op), n, op);
        }
      } else {  // AAD: column tiles (2jp, 2jp+1) = (gamma, beta) of the same 16 channels
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) {
          const int ng = n0 + wn * WTN + (2 * jp) * 16 + lr;
          const int c = (ng >> 5) * 16 + lr;
          if (c < a.C_aad) {
            const float ga = acc[i][2 * jp][r] + a.shift[ng];
            const float ba = acc[i][2 * jp + 1][r] + a.shift[ng + 16];
            const float v = epi_aad<TO>(a, ga, ba, c, m);
            reinterpret_cast<TO*>(a.y)[(long)m * a.ldy + c] = from_f<TO>(v);
          }
        }
      }
    }
  }
  if constexpr (EPI == KEPI_SPLIT)
    if (a.sem) split_fixup<TO, BM, BN, 256>(a, tid, par * gridDim.x + tile, m0, n0, par, reinterpret_cast<float*>(smem));
}

// split-K reduction + epilogue: one thread per (pixel, channel) [STD] or (pixel, AAD channel)
template <typename TO, int EPI>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const ConvArgs a) {
  const int par = blockIdx.z;
  const int py = par >> 1, px = par & 1;
  const int ncols = (EPI == KEPI_AAD) ? a.C_aad : a.N;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)a.M * ncols) return;
  const long m = idx / ncols;
  const int c = (int)(idx - m * ncols);
  const float* base = a.partial + ((long)par * a.nsplit * a.M + m) * a.NT;
  const long sstride = (long)a.M * a.NT;
  if constexpr (EPI == KEPI_STD) {
    // the slab loads unrolled ahead of the (sequential, order-preserving) sum: a deep split no longer waits
    // one memory latency per slab
    float v = 0.f;
#pragma unroll 8
    for (int s = 0; s < a.nsplit; ++s) v += base[s * sstride + c];
    const long op = out_pixel(a, m, py, px);
    store_std<TO>(a, epi_std<TO>(a, v, c, op), c, op);
  } else {
    const int ng = (c >> 4) * 32 + (c & 15);
    float ga = 0.f, ba = 0.f;
#pragma unroll 8
    for (int s = 0; s < a.nsplit; ++s) {
      ga += base[s * sstride + ng];
      ba += base[s * sstride + ng + 16];
    }
    ga += a.shift[ng];
    ba += a.shift[ng + 16];
    reinterpret_cast<TO*>(a.y)[m * a.ldy + c] = from_f<TO>(epi_aad<TO>(a, ga, ba, c, m));
  }
}

// the same reduction, four channels per thread: 16-byte slab loads (the scalar form read 4 B per lane and ran at
// 0.4-1 TB/s on the B = 64 AAD / encoder reductions); per element the same ordered sum and the same epilogue
template <typename TO, int EPI>
__global__ void __launch_bounds__(256) splitk_reduce4_kernel(const ConvArgs a) {
  const int par = blockIdx.z;
  const int py = par >> 1, px = par & 1;
  const int ncols = (EPI == KEPI_AAD) ? a.C_aad : a.N;
  const int nq = ncols >> 2;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)a.M * nq) return;
  const long m = idx / nq;
  const int c = (int)(idx - m * nq) * 4;
  const float* base = a.partial + ((long)par * a.nsplit * a.M + m) * a.NT;
  const long sstride = (long)a.M * a.NT;
  if constexpr (EPI == KEPI_STD) {
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int s = 0; s < a.nsplit; ++s) v += *reinterpret_cast<const f32x4*>(base + s * sstride + c);
    const long op = out_pixel(a, m, py, px);
#pragma unroll
    for (int e = 0; e < 4; ++e) store_std<TO>(a, epi_std<TO>(a, v[e], c + e, op), c + e, op);
  } else {
    const int ng = (c >> 4) * 32 + (c & 15);   // four consecutive channels: four consecutive gamma columns
    f32x4 ga = f32x4{0.f, 0.f, 0.f, 0.f}, ba = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int s = 0; s < a.nsplit; ++s) {
      ga += *reinterpret_cast<const f32x4*>(base + s * sstride + ng);
      ba += *reinterpret_cast<const f32x4*>(base + s * sstride + ng + 16);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      reinterpret_cast<TO*>(a.y)[m * a.ldy + c + e] =
          from_f<TO>(epi_aad<TO>(a, ga[e] + a.shift[ng + e], ba[e] + a.shift[ng + 16 + e], c + e, m));
  }
}

// one reduction launch for a split-K GEMM's partials: the four-channel form when the columns allow it
template <typename TO, int EPI>
void launch_reduce(const ConvArgs& a, int ncols, int npar, hipStream_t s) {
  static const int vec = GHOST_KNOB("GHOST_SPLITK_VEC", 1);
  const long total = (long)a.M * ncols;
  if (vec && ncols % 4 == 0 && a.NT % 4 == 0) {
    dim3 grid((unsigned)((total / 4 + 255) / 256), 1, npar);
    hipLaunchKernelGGL((splitk_reduce4_kernel<TO, EPI>), grid, dim3(256), 0, s, a);
  } else {
    dim3 grid((unsigned)((total + 255) / 256), 1, npar);
    hipLaunchKernelGGL((splitk_reduce_kernel<TO, EPI>), grid, dim3(256), 0, s, a);
  }
}

// ---------------------------------------------------------------------------
// v2: bf16 implicit GEMM staged by LDS-DMA (global_load_lds_dwordx4) through a STAGES-deep
// ring with counted vmcnt waits and raw barriers (cdna_hip_programming.md §5 "Pipelining
// across barriers").  No register staging: the K loop issues one DMA per 16 tile rows and
// the MFMAs; zero padding comes from DMA reads of a zero line.  LDS rows are 64 B (BK = 32)
// with chunk c of row r stored at c ^ ((r >> 1) & 3): conflict-free ds_read_b128 for the
// 16x16x32 fragments, applied on the DMA *source* side (the LDS image is lane-linear).
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) unsigned int g_zero_line[64] = {0};

GHOST_DEV int swz(int r, int c) { return c ^ ((r >> 1) & 3); }

template <int N>
GHOST_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `after` stages of LPS DMA instructions each are still in flight
// (vmcnt counts this wave's outstanding vector-memory instructions, retired in order)
template <int LPS, int K>
GHOST_DEV void wait_stages(int after) {
  if constexpr (K <= 0) {
    wait_vmcnt<0>();
  } else {
    if (after >= K) wait_vmcnt<K * LPS>();
    else wait_stages<LPS, K - 1>(after);
  }
}

// issue the LDS-DMA of K tile `kt` into ring slot `sb` (one 16-row piece per instruction)
template <typename T, int BM, int NA, int NB>
GHOST_DEV void glds_issue(const ConvArgs& a, const T* __restrict__ x, const T* const (&b_src)[NB],
                          const long (&a_off)[NA], const uint64_t (&a_mask)[NA], const int (&a_gc)[NA], int wid,
                          int kt, unsigned char* sb) {
#if defined(__HIP_DEVICE_COMPILE__)   // the amdgcn builtin does not exist in the host pass of this TU
  const int k0 = kt * 32;
  const int cb = kt / a.ntaps, tap = kt - cb * a.ntaps;    // K order (channel block, tap, channel)
  const int ty = tap / a.ntx, tx = tap - ty * a.ntx;
  const long toff = ((long)a.tsign * ty * a.Wi + a.tsign * tx) * a.ldx + cb * 32;
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const void* src = ((a_mask[j] >> tap) & 1ull) ? (const void*)(x + a_off[j] + toff + a_gc[j])
                                                 : (const void*)g_zero_line;
    __builtin_amdgcn_global_load_lds(src, sb + (wid * NA + j) * 1024, 16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
    __builtin_amdgcn_global_load_lds(b_src[j] + k0, sb + BM * 64 + (wid * NB + j) * 1024, 16, 0, 0);
#endif
}

// WSL = 4: warp-specialised form, 512 threads: waves 0-3 run the MFMAs and the epilogue, waves 4-7 only issue
// the ring's LDS-DMA (same ring, same per-K-step barrier), so no compute wave pays the DMA issue cost
template <typename T, int BM, int BN, int STAGES, int EPI, int WSL = 0>
__global__ void __launch_bounds__(WSL ? 512 : 256) conv_glds_kernel(const ConvArgs a) {
  typedef T TI;
  typedef T TO;
  constexpr int WM = WaveGrid<BM, BN>::WM, WN = WaveGrid<BM, BN>::WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int NA = BM / 64, NB = BN / 64;        // DMA instructions per wave per stage (16 rows each)
  constexpr int LPS = NA + NB;
  constexpr int STAGE_B = (BM + BN) * 64;          // bytes per stage
  static_assert(BM % 64 == 0 && BN % 64 == 0, "v2 tile");
  static_assert(EPI != KEPI_AAD || (TN % 2 == 0 && WTN % 32 == 0), "AAD epilogue needs gamma/beta tile pairs");
  static_assert((STAGES - 2) * LPS <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[STAGES * STAGE_B];

  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, lr = lane & 15,
            lq = lane >> 4;
  const bool loads = !WSL || wid >= 4, computes = !WSL || wid < 4;
  const int lw = WSL ? wid - 4 : wid;   // index of this wave among the DMA-issuing waves
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  // N-major order (deep ring): an XCD's run of tiles covers few channel tiles, whose weight rows
  // then stay in that XCD's 4 MB L2 while every M tile streams past them
  const int nMt = gridDim.x / a.nNt;
  const int nt = a.nmajor ? tile / nMt : tile % a.nNt, mt = a.nmajor ? tile % nMt : tile / a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int split = blockIdx.y, par = blockIdx.z, py = par >> 1, px = par & 1;
  const TI* __restrict__ x = reinterpret_cast<const TI*>(a.x);
  const TI* __restrict__ w = reinterpret_cast<const TI*>(a.w) + par * a.wpar_stride;
  const int nk = a.Kpad / 32;
  const int kt0 = split * a.kt_per_split;
  const int kt1 = min(nk, kt0 + a.kt_per_split);

  // this lane's DMA rows: A rows 16*(wid*NA + j) + lane/4, B rows 16*(wid*NB + j) + lane/4
  const int lrow = lane >> 2, pc = lane & 3;
  const int HoWo = a.Ho * a.Wo;
  const int tby = a.deconv ? py : a.tbase, tbx = a.deconv ? px : a.tbase;
  const int nty = a.K / (a.Cin * a.ntx);
  long a_off[NA];
  uint64_t a_mask[NA];
  int a_gc[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int r = 16 * (lw * NA + j) + lrow;
    const int m = m0 + r;
    a_gc[j] = swz(r, pc) * 8;
    a_off[j] = 0;
    a_mask[j] = 0ull;
    if (m < a.M) {
      const int b = m / HoWo;
      const int rr = m - b * HoWo;
      const int oy = rr / a.Wo, ox = rr - oy * a.Wo;
      const int iyb = oy * a.stride + tby, ixb = ox * a.stride + tbx;
      a_off[j] = ((long)(b * a.Hi + iyb) * a.Wi + ixb) * a.ldx;
      uint64_t mk = 0ull;
      for (int ty = 0; ty < nty; ++ty) {
        const int iy = iyb + a.tsign * ty;
        if (iy < 0 || iy >= a.Hi) continue;
        for (int tx = 0; tx < a.ntx; ++tx) {
          const int ix = ixb + a.tsign * tx;
          if (ix >= 0 && ix < a.Wi) mk |= 1ull << (ty * a.ntx + tx);
        }
      }
      a_mask[j] = mk;
    }
  }
  const TI* b_src[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int r = 16 * (lw * NB + j) + lrow;
    b_src[j] = w + (long)(n0 + r) * a.Kpad + swz(r, pc) * 8;
  }

  const int wm = (wid & 3) / WN, wn = (wid & 3) % WN;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int n = kt1 - kt0;
  if (loads) {
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < n) glds_issue<T, BM, NA, NB>(a, x, b_src, a_off, a_mask, a_gc, lw, kt0 + s, lds + s * STAGE_B);
  }
  for (int it = 0; it < n; ++it) {
    // stages issued after `it` that may stay in flight
    if (loads) wait_stages<LPS, STAGES - 2>(min(STAGES - 2, n - 1 - it));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (loads && it + STAGES - 1 < n)
      glds_issue<T, BM, NA, NB>(a, x, b_src, a_off, a_mask, a_gc, lw, kt0 + it + STAGES - 1,
                             lds + ((it + STAGES - 1) % STAGES) * STAGE_B);
    if (!computes) continue;
    const unsigned char* sb = lds + (it % STAGES) * STAGE_B;
    const unsigned char* As = sb;
    const unsigned char* Bs = sb + BM * 64;
    v8_t<T> af[TM], bfv[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WTM + i * 16 + lr;
      af[i] = *reinterpret_cast<const v8_t<T>*>(As + r * 64 + swz(r, lq) * 16);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = wn * WTN + j * 16 + lr;
      bfv[j] = *reinterpret_cast<const v8_t<T>*>(Bs + r * 64 + swz(r, lq) * 16);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32<T>(af[i], bfv[j], acc[i][j]);
  }

  if constexpr (EPI == KEPI_SPLIT) {
    if (computes) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + lq * 4 + r;
          if (m >= a.M) continue;
          float* dst = a.partial + (((long)par * a.nsplit + split) * a.M + m) * a.NT;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (a.sem) st_dev(dst + n0 + wn * WTN + j * 16 + lr, acc[i][j][r]);
            else dst[n0 + wn * WTN + j * 16 + lr] = acc[i][j][r];
          }
        }
      }
    }
    // (the DMA waves stay for the fix-up: its barriers count every wave, and they share its reduction)
    if (a.sem)
      split_fixup<TO, BM, BN, WSL ? 512 : 256>(a, tid, par * gridDim.x + tile, m0, n0, par, reinterpret_cast<float*>(lds));
    return;
  }
  if (!computes) return;
  // ---- epilogue (as v1) ----
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WTM + i * 16 + lq * 4 + r;
      if (m >= a.M) continue;
      if constexpr (EPI == KEPI_STD) {
        const long op = out_pixel(a, m, py, px);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nn = n0 + wn * WTN + j * 16 + lr;
          if (nn < a.N) store_std<TO>(a, epi_std<TO>(a, acc[i][j][r], nn, op), nn, op);
        }
      } else {  // AAD: column tiles (2jp, 2jp+1) = (gamma, beta) of the same 16 channels
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) {
          const int ng = n0 + wn * WTN + (2 * jp) * 16 + lr;
          const int c = (ng >> 5) * 16 + lr;
          if (c < a.C_aad) {
            const float ga = acc[i][2 * jp][r] + a.shift[ng];
            const float ba = acc[i][2 * jp + 1][r] + a.shift[ng + 16];
            reinterpret_cast<TO*>(a.y)[(long)m * a.ldy + c] = from_f<TO>(epi_aad<TO>(a, ga, ba, c, m));
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host side: tile choice, split-K heuristic, dispatch
// ---------------------------------------------------------------------------
namespace {

struct Plan {
  int BM, BN, BK, nNt, nMt, npar, nsplit, kt_per_split, NT, M, Ho, Wo;
  bool fast;
  bool partial;   // GEMM writes fp32 partials, splitk_reduce_kernel applies the epilogue
  int stages;     // > 0: the LDS-DMA ring kernel with this many stages (deep ring, low-resolution GEMMs)
};


Plan make_plan(const ConvDesc& d) {
  static const int force_bk = GHOST_KNOB("GHOST_CONV_BK", 0);   // tuning knob (0 = heuristic)
  Plan p{};
  p.npar = d.kind == CONV_T4S2 ? 4 : 1;
  if (d.kind == CONV_T4S2) {
    p.Ho = d.Hi;
    p.Wo = d.Wi;
  } else {
    p.Ho = (d.Hi + 2 * d.pad - d.kh) / d.stride + 1;
    p.Wo = (d.Wi + 2 * d.pad - d.kw) / d.stride + 1;
  }
  p.M = d.B * p.Ho * p.Wo;
  const bool bf = is16(d.ti);   // 16-bit operands (bf16 or fp16)
  const int vec = bf ? 8 : 4;
  p.fast = (d.Cin % 32 == 0) && (d.ldx % vec == 0) && ((uintptr_t)d.x % 16 == 0);
  // BK = 64 pays only on deep reductions (measured: 256x64 tiles lose 2x at BK 64 from LDS occupancy)
  const bool bk64_ok = bf && p.fast && d.Cin % 64 == 0 && d.Kpad % 64 == 0;
  // (Kpad 4096: the encoder's 16x16 conv and 8x8 deconv, measured -10..-19 % with BK 64)
  p.BK = (bk64_ok && d.Kpad >= 4096) ? 64 : 32;
  if (force_bk == 32 || (force_bk == 64 && bk64_ok)) p.BK = force_bk;
  if (!p.fast) {
    p.BN = d.N <= 32 ? 32 : 64;
    p.BM = d.N <= 32 ? 256 : 64;
  } else if (d.epi == EPI_AAD) {
    p.BN = 128;
    p.BM = ((p.M + 127) / 128) * ((d.N + 127) / 128) * p.npar >= 512 ? 128 : 64;
  } else if (d.N <= 16) {
    p.BN = 16; p.BM = 256;
  } else if (d.N <= 32) {
    p.BN = 32; p.BM = 256;
  } else if (d.N <= 64) {
    // the encoder's 4x4/s2 convs gather 64-byte tap rows: 128-row tiles take the LDS-DMA ring
    // (measured 128x128 32->64: 56 vs 72 us at 256 rows)
    p.BN = 64; p.BM = (bf && d.kh == 4 && d.stride == 2 && d.kind == CONV_FWD) ? 128 : 256;
  } else {
    p.BN = 128;
    p.BM = ((p.M + 127) / 128) * ((d.N + 127) / 128) * p.npar >= 512 ? 128 : 64;
  }
  if (!p.fast || p.BM >= 256) p.BK = force_bk == 64 && bk64_ok ? 64 : 32;
  // Low-resolution GEMMs (the generator's 2x2..8x8 stages and the encoder's 16x16..2x2 convs at
  // B = 64: M <= 8192 pixels, deep K): a register-staged tile keeps one K step in flight and waits
  // out the memory latency on every step (measured 0.19 of MFMA peak on the 8x8 1024->1024 conv).
  // The LDS-DMA ring keeps 6 K steps of 128x128 tiles in flight instead (128 KB of LDS, one
  // workgroup per CU); split-K fills the CUs when the grid is small.
  static const int deep = GHOST_KNOB("GHOST_CONV_DEEP", 8);
  // (only grids that need split-K: with >= 256 tiles of 128 x 128 the two-workgroup register-staged
  // kernel measured faster, e.g. the 8x8 AAD GEMM 55 vs 74 us)
  const long tiles128 = (long)((p.M + 127) / 128) * ((d.N + 127) / 128) * p.npar;
  // very deep K (>= 4096: IResNet's 7 x 7 512 -> 512 convs) keeps the ring up to two rounds of workgroups:
  // at B = 256 (M = 12 544, 392 tiles) 175 -> 167 us per conv against the register-staged 64 x 128 tile (the
  // second, partial round of 136 tiles costs what the ring saves; at B = 128 the ring with split-K: 63 us)
  const bool deep_k = p.M <= 16384 && d.Kpad >= 4096 && tiles128 < 512;
  if (deep > 0 && bf && p.fast && d.to == d.ti && d.N >= 256 && d.Kpad >= 1024 && d.N % 128 == 0 &&
      ((p.M <= 8192 && tiles128 < 256) || deep_k)) {
    p.BM = 128; p.BN = 128; p.BK = 32; p.stages = deep;
  }
#ifdef GHOST_TUNING
  static const char* force_tile = getenv("GHOST_CONV_TILE");   // tuning knob "BMxBN"
  if (force_tile && p.fast && d.epi != EPI_AAD) {
    int bm = 0, bn = 0;
    if (sscanf(force_tile, "%dx%d", &bm, &bn) == 2 && bn >= d.N / 2 && bm > 0) { p.BM = bm; p.BN = bn; }
  }
#endif
  p.nNt = (d.N + p.BN - 1) / p.BN;
  p.nMt = (p.M + p.BM - 1) / p.BM;
  p.NT = p.nNt * p.BN;
  const int nk = d.Kpad / p.BK;
  const int tiles = p.nMt * p.nNt * p.npar;
  int s = 1;
  if (d.force_split > 0) {
    s = d.force_split;
  } else if (p.stages > 0) {
    // deep ring: one resident workgroup per CU; split K until the grid covers the CUs
    // (GHOST_SPLIT_DEEP: the grid target in workgroups, tuning build)
    static const int deep_target = GHOST_KNOB("GHOST_SPLIT_DEEP", 256);
    static const int deep_minks = GHOST_KNOB("GHOST_SPLIT_DEEP_MINK", 8);
    if (tiles < 256 && nk >= 16) {
      s = (deep_target + tiles - 1) / tiles;
      s = s < nk / deep_minks ? s : nk / deep_minks;
      if (s < 1) s = 1;
    }
  } else if ((tiles < (d.min_wgs > 0 ? d.min_wgs : 256) && nk >= 16) ||
             (d.min_wgs <= 0 && tiles == 256 && nk >= 64)) {
    // one round of 256 tiles with a deep reduction splits in two as well (measured: the 4x4 deconv
    // 2048->512 -26 %, the 16x16 4x4/s2 conv 256->512 -19 %)
    static const int split_mul = GHOST_KNOB("GHOST_SPLIT_MUL", 2);   // (tuning build) workgroups per CU aimed at
    const int target = split_mul * (d.min_wgs > 0 ? d.min_wgs : 256);
    s = (target + tiles - 1) / tiles;       // aim for >= 2 workgroups per CU
    s = s < nk / 8 ? s : nk / 8;            // keep >= 8 K steps per split
    if (s < 1) s = 1;
  }
  if (s > nk) s = nk;
  p.kt_per_split = (nk + s - 1) / s;
  p.nsplit = (nk + p.kt_per_split - 1) / p.kt_per_split;
  // bf16 operands with an fp32 output (the ArcFace embedding layer): the GEMM always writes fp32
  // partials and the reduction kernel applies the epilogue in fp32
  p.partial = p.nsplit > 1 || (is16(d.ti) && d.to == GHOST_F32);
  return p;
}

ConvArgs make_args(const ConvDesc& d, const Plan& p, float* partial) {
  ConvArgs a{};
  a.x = d.x; a.w = d.w; a.y = d.y;
  a.scale = d.scale; a.shift = d.shift; a.res = d.res;
  a.prelu = d.prelu; a.y2 = d.y2; a.scale2 = d.scale2; a.shift2 = d.shift2; a.ldy2 = d.ldy2;
  a.res_first = d.res_first;
  a.hin = d.hin; a.stat = d.stat; a.idgb = d.idgb; a.mask = d.mask;
  a.partial = partial; a.u8 = d.u8;
  a.wpar_stride = (long)d.Npad * d.Kpad;
  a.B = d.B; a.Hi = d.Hi; a.Wi = d.Wi; a.Cin = d.Cin; a.ldx = d.ldx;
  a.Ho = p.Ho; a.Wo = p.Wo; a.M = p.M;
  a.N = d.N; a.Kpad = d.Kpad; a.NT = p.NT; a.nNt = p.nNt;
  a.ldy = d.ldy; a.ldres = d.ldres; a.ldh = d.ldh; a.id_ld = d.id_ld; a.C_aad = d.C_aad;
  if (d.kind == CONV_T4S2) {
    a.K = 4 * d.Cin; a.stride = 1; a.ntx = 2; a.ntaps = 4; a.tbase = 0; a.tsign = -1; a.deconv = 1;
  } else {
    a.K = d.kh * d.kw * d.Cin; a.stride = d.stride; a.ntx = d.kw; a.ntaps = d.kh * d.kw; a.tbase = -d.pad;
    a.tsign = 1; a.deconv = 0;
  }
  a.nsplit = p.nsplit; a.kt_per_split = p.kt_per_split;
  a.slope = d.slope; a.tanh_out = d.tanh_out;
  a.nmajor = p.stages > 0 ? GHOST_KNOB("GHOST_CONV_NMAJOR", 1) : 0;
  return a;
}

template <typename TI, typename TO, int BM, int BN, int BK, int EPI, bool FAST>
void launch_gemm(const ConvArgs& a, const Plan& p, hipStream_t s) {
  dim3 grid(p.nMt * p.nNt, p.nsplit, p.npar);
  hipLaunchKernelGGL((conv_igemm_kernel<TI, TO, BM, BN, BK, EPI, FAST>), grid, dim3(256), 0, s, a);
}

// instantiated configurations (BM x BN x BK); anything else is rejected by the plan
template <typename TI, typename TO, int EPI, bool FAST>
int dispatch_tile(const ConvArgs& a, const Plan& p, hipStream_t s) {
  const int key = p.BM * 100000 + p.BN * 100 + p.BK;
#define GHOST_TILE(bm, bn, bk) \
  case bm * 100000 + bn * 100 + bk: launch_gemm<TI, TO, bm, bn, bk, EPI, FAST>(a, p, s); return 0;
  if constexpr (!FAST) {
    if constexpr (EPI != KEPI_AAD) {
      switch (key) { GHOST_TILE(256, 32, 32) GHOST_TILE(64, 64, 32) default: break; }
    }
    return -1;
  } else if constexpr (sizeof(TI) == 2) {
    if constexpr (EPI == KEPI_AAD) {
      switch (key) { GHOST_TILE(128, 128, 32) GHOST_TILE(128, 128, 64) GHOST_TILE(64, 128, 32)
                     GHOST_TILE(64, 128, 64) default: break; }
    } else {
      switch (key) { GHOST_TILE(128, 128, 32) GHOST_TILE(128, 128, 64) GHOST_TILE(64, 128, 32)
                     GHOST_TILE(64, 128, 64) GHOST_TILE(256, 64, 32) GHOST_TILE(256, 64, 64)
                     GHOST_TILE(256, 32, 32) GHOST_TILE(256, 32, 64) GHOST_TILE(256, 16, 32)
                     GHOST_TILE(256, 16, 64) GHOST_TILE(128, 64, 32) GHOST_TILE(128, 64, 64)
                     GHOST_TILE(64, 64, 32) GHOST_TILE(64, 64, 64) GHOST_TILE(128, 32, 32)
                     GHOST_TILE(128, 16, 32) default: break; }
    }
    return -1;
  } else {
    if constexpr (EPI == KEPI_AAD) {
      switch (key) { GHOST_TILE(128, 128, 32) GHOST_TILE(64, 128, 32) default: break; }
    } else {
      switch (key) { GHOST_TILE(128, 128, 32) GHOST_TILE(64, 128, 32) GHOST_TILE(256, 64, 32)
                     GHOST_TILE(256, 32, 32) GHOST_TILE(256, 16, 32) default: break; }
    }
    return -1;
  }
#undef GHOST_TILE
}

template <typename T, int EPI>
bool launch_glds(const ConvArgs& a, const Plan& p, hipStream_t s) {
  static const int stages_knob = GHOST_KNOB("GHOST_CONV_STAGES", 3);
  // warp-specialised DMA waves (B = 64, same box: 4x4 3x3 1024 conv 50 -> 41 us, encoder conv5..7 49 / 47 / 32 ->
  // 40 / 38 / 28, deconv2 82 -> 64; bench +0.4..1.8 %)
  static const int ws = GHOST_KNOB("GHOST_CONV_WS", 1);
  const int stages = p.stages > 0 ? p.stages : stages_knob;
  dim3 grid(p.nMt * p.nNt, p.nsplit, p.npar);
  if constexpr (EPI == KEPI_AAD) {
    if (p.BM == 128 && p.BN == 128 && stages == 8) {
      if (ws)
        hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, 8, EPI, 4>), grid, dim3(512), 0, s, a);
      else
        hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, 8, EPI>), grid, dim3(256), 0, s, a);
      return true;
    }
    if (p.BM == 128 && p.BN == 128 && stages == 3 && ws) {
      hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, 3, EPI, 4>), grid, dim3(512), 0, s, a);
      return true;
    }
    return false;
  }
#define GHOST_G(bm, bn, st)                                                                      \
  if (p.BM == bm && p.BN == bn && stages == st) {                                                \
    if (ws)                                                                                       \
      hipLaunchKernelGGL((conv_glds_kernel<T, bm, bn, st, EPI, 4>), grid, dim3(512), 0, s, a);      \
    else                                                                                          \
      hipLaunchKernelGGL((conv_glds_kernel<T, bm, bn, st, EPI>), grid, dim3(256), 0, s, a);         \
    return true;                                                                                  \
  }
  GHOST_G(128, 128, 8) GHOST_G(128, 128, 6)
  GHOST_G(128, 128, 4) GHOST_G(256, 64, 4) GHOST_G(128, 64, 4) GHOST_G(64, 128, 4)
  GHOST_G(128, 128, 3) GHOST_G(256, 64, 3) GHOST_G(128, 64, 3) GHOST_G(64, 128, 3)
#undef GHOST_G
  return false;
}

template <typename TI, typename TO>
int dispatch_types(const ConvDesc& d, const ConvArgs& a, const Plan& p, hipStream_t s) {
  int rc;
  if constexpr (sizeof(TI) == 2 && sizeof(TO) == 4) {
    // bf16 GEMM, fp32 epilogue: the partial-sum GEMM does not depend on the output type, so it
    // shares the bf16 instantiations; the reduction writes fp32
    if (!p.partial || d.epi != EPI_STD) return -1;
    rc = p.fast ? dispatch_tile<TI, TI, KEPI_SPLIT, true>(a, p, s) : dispatch_tile<TI, TI, KEPI_SPLIT, false>(a, p, s);
    if (rc) return rc;
    const long total = (long)p.M * d.N;
    dim3 grid((unsigned)((total + 255) / 256), 1, p.npar);
    hipLaunchKernelGGL((splitk_reduce_kernel<float, KEPI_STD>), grid, dim3(256), 0, s, a);
    return 0;
  } else {
  static const int use_v2 = GHOST_KNOB("GHOST_CONV_V2", 1);
  if constexpr (sizeof(TI) == 2 && sizeof(TO) == 2) {
    // measured (tools/bench_ops.py): the DMA ring wins on the 128-row tiles, loses on 256x64
    static const int aad_glds = GHOST_KNOB("GHOST_CONV_AAD_GLDS", 0);   // AAD epilogue on the 3-stage ring
    if (use_v2 && p.fast && p.BK == 32 && (d.epi != EPI_AAD || p.stages > 0 || aad_glds) && p.BM <= 128 &&
        p.partial == (p.nsplit > 1)) {
      const bool ok = p.nsplit > 1 ? launch_glds<TI, KEPI_SPLIT>(a, p, s)
                                   : (d.epi == EPI_AAD ? launch_glds<TI, KEPI_AAD>(a, p, s) : launch_glds<TI, KEPI_STD>(a, p, s));
      if (ok) {
        if (p.nsplit > 1 && !a.sem) {
          if (d.epi == EPI_AAD) launch_reduce<TO, KEPI_AAD>(a, d.C_aad, p.npar, s);
          else launch_reduce<TO, KEPI_STD>(a, d.N, p.npar, s);
        }
        return 0;
      }
    }
  }
  if (p.partial) {
    rc = p.fast ? dispatch_tile<TI, TO, KEPI_SPLIT, true>(a, p, s) : dispatch_tile<TI, TO, KEPI_SPLIT, false>(a, p, s);
    if (rc || a.sem) return rc;
    if (d.epi == EPI_AAD) launch_reduce<TO, KEPI_AAD>(a, d.C_aad, p.npar, s);
    else launch_reduce<TO, KEPI_STD>(a, d.N, p.npar, s);
    return 0;
  }
  if (d.epi == EPI_AAD) {
    if (!p.fast) return -1;
    return dispatch_tile<TI, TO, KEPI_AAD, true>(a, p, s);
  }
  return p.fast ? dispatch_tile<TI, TO, KEPI_STD, true>(a, p, s) : dispatch_tile<TI, TO, KEPI_STD, false>(a, p, s);
  }
}

}  // namespace

size_t conv_workspace_bytes(const ConvDesc& d) {
  if (conv3x3_halo_supported(d) || convT_halo_supported(d) || conv_stem3x3_supported(d) ||
      conv4x4s2_patch_supported(d))
    return 0;
  if (conv_first_supported(d)) return conv_first_workspace_bytes();
  Plan p = make_plan(d);
  if (!p.partial) return 0;
  return (size_t)p.npar * p.nsplit * p.M * p.NT * sizeof(float);
}

int conv_launch(const ConvDesc& d, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!d.x || !d.w || !d.y || d.B <= 0 || d.Cin <= 0 || d.N <= 0) return -1;
  if (d.Kpad % 32 != 0 || d.Npad < d.N) return -1;
  if (d.y2 && (!d.scale2 || !d.shift2 || d.epi != EPI_STD)) return -1;
  if (d.kind == CONV_FWD && (d.kh * d.kw > 64 || d.kh < 1 || d.kw < 1 || d.stride < 1)) return -1;   // 64-bit tap masks
  if (d.epi == EPI_AAD && (d.C_aad % 16 != 0 || d.N != 2 * d.C_aad || !d.hin || !d.stat || !d.idgb || !d.mask || !d.shift))
    return -1;
#ifdef GHOST_TUNING
  // plan listing for profiling (tuning builds only): one line per conv launch with its shape
  static const int trace = GHOST_KNOB("GHOST_CONV_TRACE", 0);
  if (trace)
    fprintf(stderr, "[conv] kind=%d B=%d %dx%d Cin=%d N=%d k=%dx%d s=%d halo=%d\n", (int)d.kind, d.B, d.Hi, d.Wi, d.Cin,
            d.N, d.kh, d.kw, d.stride, (int)conv3x3_halo_supported(d));
#endif
  if (conv3x3_halo_supported(d)) return conv3x3_halo(d, stream);
  if (conv_first_supported(d)) return conv_first(d, ws, ws_bytes, stream);
  if (conv_stem3x3_supported(d)) return conv_stem3x3(d, stream);
  if (convT_halo_supported(d)) return convT_halo(d, stream);
  if (conv4x4s2_patch_supported(d) || conv3x3s2_patch_supported(d)) return conv_s2_patch(d, stream);
  Plan p = make_plan(d);
  if (p.NT > d.Npad) return -1;  // weight rows read by the last tile must exist
  const int K = d.kind == CONV_T4S2 ? 4 * d.Cin : d.kh * d.kw * d.Cin;
  if (d.Kpad < K) return -1;
  float* partial = nullptr;
  if (p.partial) {
    size_t need = (size_t)p.npar * p.nsplit * p.M * p.NT * sizeof(float);
    if (!ws || ws_bytes < need) return -1;
    partial = reinterpret_cast<float*>(ws);
  }
  ConvArgs a = make_args(d, p, partial);
  // split-K fix-up in the GEMM (split_fixup) when the caller gave counters and a tile's partials are small enough
  // for one workgroup to sum them (the last one to finish does it while the rest of the grid has drained):
  // B = 1 and the generator's 2x2..8x8 stages; the large splits keep splitk_reduce_kernel over the whole chip
  // (bf16 operands with an fp32 output keep it too: their reduction writes another type than the GEMM's)
  // (the last arriver reads ~1 us per 16 KB of partials, cdna_hip_programming.md §6 item 2: a few tens of KB per
  // tile; they are staged in the kernel's LDS, so never more than that holds.  Measured at B = 1 bf16: 32-40 KB
  // 1.10-1.11 ms as without the fix-up, 128 KB — the deep ring's 4x4 / 8x8 GEMMs fused — 1.17-1.19 ms)
  static const int fuse_knob = GHOST_KNOB("GHOST_SPLIT_FUSE", 1);
  static const long fuse_max = (long)GHOST_KNOB("GHOST_SPLIT_FUSE_KB", 32) << 10;
  if (p.partial && p.nsplit > 1 && d.sem && fuse_knob && !(is16(d.ti) && d.to == GHOST_F32) &&
      (long)p.nMt * p.nNt * p.npar <= d.nsem) {
    const long tile_bytes = (long)p.nsplit * (p.M < p.BM ? p.M : p.BM) * p.BN * 4;
    // LDS of the kernel that runs it: the deep ring (p.stages, always conv_glds_kernel: 16-bit, fast, 128 x 128)
    // has stages x 16 KB; otherwise the smaller of conv_glds_kernel's 3-stage ring and conv_igemm_kernel's buffers
    const int vec = is16(d.ti) ? 8 : 4, esz = is16(d.ti) ? 2 : 4;
    static const int stages_knob = GHOST_KNOB("GHOST_CONV_STAGES", 3);
    const long ring = (long)(p.stages > 0 ? p.stages : stages_knob) * (p.BM + p.BN) * 64;
    const long bufs = 2L * (p.BM + p.BN) * (p.BK + vec) * esz;
    static const int use_v2 = GHOST_KNOB("GHOST_CONV_V2", 1);
    const bool deep_glds = use_v2 && (p.stages == 8 || p.stages == 6 || p.stages == 4);   // launch_glds' instances
    const long lds = deep_glds ? ring : (ring < bufs ? ring : bufs);
    if (tile_bytes <= lds && (fuse_knob == 2 || tile_bytes <= fuse_max)) {
      a.sem = d.sem;
      a.fuse = d.epi == EPI_AAD ? 2 : 1;
    }
  }
  int rc;
  if (d.ti == GHOST_F32 && d.to == GHOST_F32) rc = dispatch_types<float, float>(d, a, p, stream);
  else if (d.ti == GHOST_BF16 && d.to == GHOST_BF16) rc = dispatch_types<bf16, bf16>(d, a, p, stream);
  else if (d.ti == GHOST_F32 && d.to == GHOST_BF16) rc = dispatch_types<float, bf16>(d, a, p, stream);
  else if (d.ti == GHOST_F16 && d.to == GHOST_F16) rc = dispatch_types<_Float16, _Float16>(d, a, p, stream);
  else if (d.ti == GHOST_F32 && d.to == GHOST_F16) rc = dispatch_types<float, _Float16>(d, a, p, stream);
  else if (d.ti == GHOST_BF16 && d.to == GHOST_F32 && !d.res && !d.y2) rc = dispatch_types<bf16, float>(d, a, p, stream);
  else return -1;
  if (rc) return rc;
  return (int)hipGetLastError();
}

}  // namespace ghost
