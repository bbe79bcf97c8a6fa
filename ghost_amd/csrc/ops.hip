// ghost_amd — bandwidth-bound kernels: InstanceNorm statistics, AAD mask, bilinear x2,
// and the layout/precision conversions at the AEI_Net boundary.  All NHWC, 16-byte
// vector accesses along channels, fp32 arithmetic.
#include <algorithm>
#include <cstdlib>

#include "ghost_common.h"
#include "ops.h"
#include "up2x.h"

namespace ghost {

static constexpr float kInEps = 1e-5f;   // nn.InstanceNorm2d default (AADLayer.py:16)

// ---------------------------------------------------------------------------
// InstanceNorm statistics
// grid (nchunk, ceil(C/64), B); a block reduces `chunk` pixels x 64 channels.
// Shift K_c = x[b, pixel 0, c] makes the partial sums robust to |mean| >> std.
// ---------------------------------------------------------------------------
// mean / rstd of (sample b, channel c) from the fp64 sums of its chunks' shifted partials (K = pixel 0 of the
// sample, also of a virtual upsample)
GHOST_DEV void in_stats_store(float* __restrict__ stat, long i, double K, double S1, double S2, int HW) {
  const double n = (double)HW;
  const double md = S1 / n;
  double var = S2 / n - md * md;
  if (var < 0.0) var = 0.0;
  stat[i * 2 + 0] = (float)(K + md);
  stat[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)kInEps));
}

// Fused final pass (sem != nullptr): the partial workgroups store with st_dev, and the last of the `arrivals` chunk
// workgroups of (sample b, 64-channel group cg) to finish merges that group's partials — the sums of
// in_stats_final_kernel in its order, one launch per statistics pass instead of two.  Each thread's chunk partials are
// loaded as one batch of independent device-scope loads before any is summed (a dependent load per chunk is a fabric
// round trip each).  Round 6: one counter per (sample, channel group), sem[b * ncg + cg], instead of one per sample:
// the sample's last arriver merged all C channels alone (C = 1024: 16 channels per thread behind one workgroup, the
// 8 x 8 .. 32 x 32 stages' statistics 28-30 us against 10-12 for the two-kernel form); now each group's last
// arriver merges its own 64.
template <typename T>
GHOST_DEV void in_stats_fixup(const T* __restrict__ x, int ldx, long bstride, int HW, int C, int nchunk,
                              const float* part, float* stat, unsigned* sem, int b, int cg, int ncg, unsigned arrivals,
                              int* flag) {
  if (!last_arrival(sem + (long)b * ncg + cg, arrivals, flag)) return;
  const int cend = min(C, cg * 64 + 64);
  for (int c = cg * 64 + threadIdx.x; c < cend; c += blockDim.x) {
    const double K = (double)to_f(x[(long)b * bstride * ldx + c]);
    const float* o = part + ((long)b * nchunk * C + c) * 2;   // chunk k: o + 2 k C
    double S1 = 0.0, S2 = 0.0;
    for (int k0 = 0; k0 < nchunk; k0 += 16) {
      float v1[16], v2[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const long k = min(k0 + j, nchunk - 1);   // clamped, not skipped: the whole batch in flight at once
        v1[j] = ld_dev(o + k * C * 2);
        v2[j] = ld_dev(o + k * C * 2 + 1);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (k0 + j < nchunk) {
          S1 += (double)v1[j];
          S2 += (double)v2[j];
        }
    }
    in_stats_store(stat, (long)b * C + c, K, S1, S2, HW);
  }
}

// UP: x is the source of a virtual bilinear x2 upsample (u); the statistics are those of the
// upsampled tensor as upsample2x would store it (values rounded to T), HW = 4 * u.H * u.W.
template <typename T, bool UP>
__global__ void __launch_bounds__(256)
in_stats_partial_kernel(const T* __restrict__ x, int ldx, int HW, int C, int chunk, int nchunk, float* __restrict__ part,
                        const Up2xSrc u, float* stat, unsigned* sem) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int TPP = 64 / VEC;   // threads per pixel (64 channels)
  constexpr int PPP = 256 / TPP;  // pixels per pass
  __shared__ float red[2][PPP][65];
  const int b = blockIdx.z, cg = blockIdx.y, ch = blockIdx.x;
  const int t = threadIdx.x, cc = t % TPP, po = t / TPP;
  const int c0 = cg * 64 + cc * VEC;
  const bool cok = c0 < C;
  const T* xb = x + (long)b * (UP ? u.H * u.W : HW) * ldx;
  float K[VEC], s1[VEC], s2[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) { K[e] = 0.f; s1[e] = 0.f; s2[e] = 0.f; }
  if (cok) load16_f(xb + c0, K);
  const int p0 = ch * chunk;
  const int p1 = min(HW, p0 + chunk);
  if (cok) {
    // (round 6) four of the thread's pixels per iteration, every load issued before the first is used: one pixel
    // per iteration waited a full load latency per pixel (the 16 x 16 stage's statistics, 256 pixels per workgroup:
    // 28 us for 34 MB).  The sums run in the same pixel order as before, so the partials are bit for bit the same.
    constexpr int U = 4;
    for (int p = p0 + po; p < p1; p += U * PPP) {
      float v[U][VEC];
#pragma unroll
      for (int uu = 0; uu < U; ++uu) {
        const int pu = min(p + uu * PPP, p1 - 1);   // clamped, not skipped: all loads in flight at once
        if constexpr (UP) {
          const int oy = pu / (2 * u.W), ox = pu - oy * (2 * u.W);
          up2x_load16_f(xb + c0, ldx, up2x_tap(u, oy, ox), v[uu]);
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[uu][e] = to_f(from_f<T>(v[uu][e]));
        } else {
          load16_f(xb + (long)pu * ldx + c0, v[uu]);
        }
      }
#pragma unroll
      for (int uu = 0; uu < U; ++uu) {
        if (p + uu * PPP >= p1) break;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float d = v[uu][e] - K[e];
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    red[0][po][cc * VEC + e] = s1[e];
    red[1][po][cc * VEC + e] = s2[e];
  }
  __syncthreads();
  if (t < 64) {
    const int c = cg * 64 + t;
    float a = 0.f, q = 0.f;
    for (int i = 0; i < PPP; ++i) { a += red[0][i][t]; q += red[1][i][t]; }
    if (c < C) {
      if (nchunk == 1) {
        // (round 6) one chunk: this workgroup saw every pixel of its channels, so it finishes them itself — the sums
        // in_stats_final_kernel would form from its single record, with no partials, counter or second launch
        in_stats_store(stat, (long)b * C + c, (double)to_f(xb[c]), (double)a, (double)q, HW);
      } else {
        float* o = part + (((long)b * nchunk + ch) * C + c) * 2;
        if (sem) {
          st_dev(o, a);
          st_dev(o + 1, q);
        } else {
          o[0] = a;
          o[1] = q;
        }
      }
    }
  }
  if (sem && nchunk > 1)
    in_stats_fixup(x, ldx, UP ? (long)u.H * u.W : (long)HW, HW, C, nchunk, part, stat, sem, b, cg, (int)gridDim.y,
                   gridDim.x, reinterpret_cast<int*>(&red[0][0][0]));
}

// Statistics of upsample2x(x) without visiting the upsampled pixels.  The x2 bilinear upsample is
// linear and separable, u(oy, ox) = sum_{s,t} a(oy, s) a(ox, t) x(s, t), with each output touching two
// adjacent source rows / columns, so with v = x - K (K = x(0, 0) = u(0, 0), the shift in_stats_final
// adds back):
//   sum_o u - K = sum_{s,t} wy(s) wx(t) v(s,t)                                   w(s)  = sum_o a(o,s)
//   sum_o (u - K)^2 = sum_{s,t} [ G0y G0x v^2 + 2 G0y G1x v v(s,t+1)              G0(s) = sum_o a(o,s)^2
//                     + 2 G1y G0x v v(s+1,t) + 2 G1y G1x (v v(s+1,t+1) + v(s,t+1) v(s+1,t)) ]
//                                                                                G1(s) = sum_o a(o,s) a(o,s+1)
// with the tap weights a of the upsample kernel (same fp32 source coordinates).  These are the
// statistics of the fp32 upsample the reference normalises (AEI_Net.py:137 -> AADLayer.py:16); the
// materialised bf16 upsample differs from it by storage rounding only.  One pass over the source,
// ~10 VALU per source pixel and channel instead of ~44 for the four outputs it feeds.
//
// up2x_tap_weights: the three table entries (w, g0, g1) of source index s along one axis of n source points
// (scale sc).  Round 4: computed by in_stats_up_quad_kernel for its own rows and columns into LDS (a separate
// table kernel was one more launch per block input).
GHOST_DEV void up2x_tap_weights(float sc, int n, int s, float& wo, float& g0o, float& g1o) {
  double w = 0.0, g0 = 0.0, g1 = 0.0;
  for (int o = max(0, 2 * s - 4); o <= min(2 * n - 1, 2 * s + 4); ++o) {
    float r = sc * (float)o;
    asm volatile("" : "+v"(r));
    const int i0 = (int)r;
    const float l1 = r - (float)i0, l0 = 1.f - l1;
    // a(o, i0) = l0, a(o, i0 + 1) = l1 (l1 = 0 at the last source index)
    const double as = i0 == s ? (double)l0 : (i0 + 1 == s ? (double)l1 : 0.0);
    const double an = i0 == s ? (double)l1 : 0.0;   // a(o, s + 1) beside a(o, s)
    w += as;
    g0 += as * as;
    g1 += as * an;
  }
  wo = (float)w;
  g0o = (float)g0;
  g1o = (float)g1;
}

// a workgroup: RB source rows x CPB = 512 / RB source columns of one sample (CPB = min(W, 128)),
// 64 channels; lane (cc, q): channel chunk cc, source row r0 + q % RB, columns c0 + 16 (q / RB) ..
// +15 walked left to right, the next NB columns of both rows loaded as one batch
// (held to <= 128 VGPRs: left alone the compiler hoisted every column's loads into 256 VGPRs + 55 AGPRs, one
// wave per SIMD, and the kernel ran at 1.9 TB/s)
template <typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
in_stats_up_quad_kernel(const T* __restrict__ x, int ldx, int C, int nchunk, float* __restrict__ part,
                        const Up2xSrc u, float* stat, unsigned* sem) {
  __shared__ float red[2][32][65];
  __shared__ float swx[3][128], swy[3][32];   // this workgroup's column / row tap-weight tables
  const int b = blockIdx.z, cg = blockIdx.y, ch = blockIdx.x;
  const int t = threadIdx.x, cc = t & 7, q = t >> 3;
  constexpr int VEC = Vec16<T>::N;
  static_assert(VEC == 8, "16-bit source");
  const int CPB = u.W < 128 ? u.W : 128, RB = 512 / CPB, nxb = u.W / CPB;
  const int cx0 = (ch % nxb) * CPB, ry0 = (ch / nxb) * RB;
  if (t < CPB) {
    up2x_tap_weights(u.sw, u.W, cx0 + t, swx[0][t], swx[1][t], swx[2][t]);
  } else if (t >= 128 && t - 128 < RB) {
    up2x_tap_weights(u.sh, u.H, ry0 + t - 128, swy[0][t - 128], swy[1][t - 128], swy[2][t - 128]);
  }
  __syncthreads();
  const int sy = ry0 + q % RB, sx0 = cx0 + (q / RB) * 16;
  const T* xb = x + (long)b * u.H * u.W * ldx + cg * 64 + cc * 8;
  float K[8];
  load16_f(xb, K);
  const float wy = swy[0][q % RB], g0y = swy[1][q % RB], g1y = swy[2][q % RB];
  const int sy1 = sy + 1 < u.H ? sy + 1 : sy;   // g1y = 0 on the last row
  const T* r0 = xb + (long)sy * u.W * ldx;
  const T* r1 = xb + (long)sy1 * u.W * ldx;
  float v[8], vd[8], R1[8], RT0[8], RT1[8];
  load16_f(r0 + (long)sx0 * ldx, v);
  load16_f(r1 + (long)sx0 * ldx, vd);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] -= K[e];
    vd[e] -= K[e];
    R1[e] = 0.f;
    RT0[e] = 0.f;
    RT1[e] = 0.f;
  }
  // NB columns of both rows per batch; the batches unrolled, so the compiler may issue a batch's loads
  // ahead of the previous batch's arithmetic within the 128-VGPR cap (NB = 4 or 8 spill under it)
  constexpr int NB = 2;
  for (int k0 = 0; k0 < 16; k0 += NB) {
    u32x4 nr0[NB], nr1[NB];   // raw columns sx0 + k0 + 1 .. +NB of both rows
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int sxn = min(sx0 + k0 + 1 + j, u.W - 1);   // g1x = 0 on the last column
      nr0[j] = *reinterpret_cast<const u32x4*>(r0 + (long)sxn * ldx);
      nr1[j] = *reinterpret_cast<const u32x4*>(r1 + (long)sxn * ldx);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int sx = sx0 + k0 + j;
      const float wx = swx[0][sx - cx0], g0x = swx[1][sx - cx0], g1x = swx[2][sx - cx0], g1x2 = 2.f * g1x;
      const T* e0 = reinterpret_cast<const T*>(&nr0[j]);
      const T* e1 = reinterpret_cast<const T*>(&nr1[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float vr = (float)e0[e] - K[e], vdr = (float)e1[e] - K[e];
        R1[e] = fmaf(wx, v[e], R1[e]);
        RT0[e] = fmaf(g0x * v[e], v[e], fmaf(g1x2 * v[e], vr, RT0[e]));
        RT1[e] = fmaf(g0x * v[e], vd[e], fmaf(g1x, fmaf(v[e], vdr, vr * vd[e]), RT1[e]));
        v[e] = vr;
        vd[e] = vdr;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][q][cc * 8 + e] = wy * R1[e];
    red[1][q][cc * 8 + e] = fmaf(g0y, RT0[e], 2.f * g1y * RT1[e]);
  }
  __syncthreads();
  if (t < 64) {
    const int c = cg * 64 + t;
    float a = 0.f, s2 = 0.f;
    for (int i = 0; i < 32; ++i) {
      a += red[0][i][t];
      s2 += red[1][i][t];
    }
    if (c < C) {
      float* o = part + (((long)b * nchunk + ch) * C + c) * 2;
      if (sem) {
        st_dev(o, a);
        st_dev(o + 1, s2);
      } else {
        o[0] = a;
        o[1] = s2;
      }
    }
  }
  if (sem)
    in_stats_fixup(x, ldx, (long)u.H * u.W, 4 * u.H * u.W, C, nchunk, part, stat, sem, b, cg, (int)gridDim.y, gridDim.x,
                   reinterpret_cast<int*>(&red[0][0][0]));
}

template <typename T>
__global__ void __launch_bounds__(256)
in_stats_final_kernel(const T* __restrict__ x, int ldx, long bstride, int B, int HW, int C, int nchunk,
                      const float* __restrict__ part, float* __restrict__ stat) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C;
  const double K = (double)to_f(x[(long)b * bstride * ldx + c]);   // pixel 0 (also of an upsample)
  double S1 = 0.0, S2 = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const float* o = part + (((long)b * nchunk + k) * C + c) * 2;
    S1 += (double)o[0];
    S2 += (double)o[1];
  }
  in_stats_store(stat, i, K, S1, S2, HW);
}

// records [B][nrec][C][2] = (mean, centred sum of squares) over 64 pixels each.  Grid (C/16, B),
// 16 channels x RL record lanes; fp64 sums, reduced across the record lanes in LDS.  (RL = 64 for
// the 256x256 stage's 1024 records per channel: 256 threads took 42 us there, latency-bound on
// 64 serial loads per thread.)
template <int RL>
__global__ void __launch_bounds__(16 * RL)
in_stats_tiles_final_kernel(const float* __restrict__ part, int nrec, int C, float* __restrict__ stat) {
  __shared__ double r1[RL][17], r2[RL][17];
  const int b = blockIdx.y, cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  // pass 1: mean of the record means (equal counts); pass 2: Chan's M2 = sum M2_r + 64 (m_r - mean)^2
  const float* base = part + ((long)b * nrec * C + c) * 2;
  double s1 = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int k = rl; k < nrec; k += RL) s1 += (double)base[(long)k * C * 2];
  }
  r1[rl][cl] = s1;
  __syncthreads();
  double mean = 0.0;
#pragma unroll
  for (int k = 0; k < RL; ++k) mean += r1[k][cl];
  mean /= nrec;
  double m2 = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int k = rl; k < nrec; k += RL) {
      const float2 v = *reinterpret_cast<const float2*>(base + (long)k * C * 2);
      const double d = (double)v.x - mean;
      m2 += (double)v.y + 64.0 * d * d;
    }
  }
  r2[rl][cl] = m2;
  __syncthreads();
  if (rl == 0 && c < C) {
    double t2 = 0.0;
#pragma unroll
    for (int k = 0; k < RL; ++k) t2 += r2[k][cl];
    const double var = t2 / (64.0 * nrec);
    stat[((long)b * C + c) * 2 + 0] = (float)mean;
    stat[((long)b * C + c) * 2 + 1] = (float)(1.0 / sqrt(var + (double)kInEps));
  }
}

int in_stats_from_tiles(const float* part, int B, int nrec, int C, float* stat, hipStream_t s) {
  if (!part || !stat || B <= 0 || nrec <= 0 || C <= 0 || B > 65535) return -1;
  if (nrec >= 512)
    hipLaunchKernelGGL(in_stats_tiles_final_kernel<64>, dim3((C + 15) / 16, B), dim3(1024), 0, s, part, nrec, C, stat);
  else
    hipLaunchKernelGGL(in_stats_tiles_final_kernel<16>, dim3((C + 15) / 16, B), dim3(256), 0, s, part, nrec, C, stat);
  return (int)hipGetLastError();
}

// chunk: pixels per workgroup (<= 1024); smaller while the grid (chunks x 64-channel groups x samples) has fewer than
// 256 workgroups, down to 64 pixels and to at most 16 chunks (the final kernel sums a (sample, channel)'s chunks in
// one thread) — B = 1: one 256-pixel chunk per channel group was 16 workgroups, 14 us
static void stats_geometry(int B, int HW, int C, int& chunk, int& nchunk) {
  chunk = HW < 1024 ? HW : 1024;
  const long groups = (long)B * ((C + 63) / 64);
  while (chunk > 64 && groups * ((HW + chunk - 1) / chunk) < 256 && (HW + chunk / 2 - 1) / (chunk / 2) <= 16)
    chunk /= 2;
  nchunk = (HW + chunk - 1) / chunk;
}

size_t in_stats_workspace_bytes(int B, int HW, int C) {
  int chunk, nchunk;
  stats_geometry(B, HW, C, chunk, nchunk);
  const int nrec = nchunk > HW / 512 ? nchunk : HW / 512;   // >= in_stats_up_quad_kernel's records
  // + the upsample weight tables of in_stats_up_quad_kernel (6 x max(H, W) <= 6 x 4096 floats)
  return (size_t)B * nrec * C * 2 * sizeof(float) + 6 * 4096 * sizeof(float) + 256;
}

bool in_stats_up2x_closed_form(int dt, int H, int W, int C, int ldx) {
  if (!is16(dt) || W % 16 || C % 64 || ldx % 8 || H > 4096 || W > 4096) return false;
  const int cpb = W < 128 ? W : 128;   // source columns per workgroup; 512 / cpb rows
  return W % cpb == 0 && H % (512 / cpb) == 0;
}

template <typename T>
static void in_stats_launch(const T* x, int ldx, int B, int HW, int C, float* stat, float* part, const Up2xSrc* up,
                            hipStream_t s, unsigned* sem) {
  int chunk, nchunk;
  stats_geometry(B, HW, C, chunk, nchunk);
  dim3 g1(nchunk, (C + 63) / 64, B);
  dim3 g2((B * C + 255) / 256);
  const Up2xSrc u = up ? *up : Up2xSrc{0, 0, 0.f, 0.f};
  if constexpr (sizeof(T) == 2) {
    if (up && in_stats_up2x_closed_form(gdt<T>(), u.H, u.W, C, ldx)) {
      // closed form over the source: (H / 4) * (W / 128) records <= the HW / 512 reserved
      const int nr = u.H * u.W / 512;   // workgroups of 512 source pixels
      hipLaunchKernelGGL(in_stats_up_quad_kernel<T>, dim3(nr, C / 64, B), dim3(256), 0, s, x, ldx, C, nr, part, u, stat,
                         sem);
      if (!sem)
        hipLaunchKernelGGL(in_stats_final_kernel<T>, g2, dim3(256), 0, s, x, ldx, (long)u.H * u.W, B, HW, C, nr, part,
                           stat);
      return;
    }
  }
  if (up)
    hipLaunchKernelGGL((in_stats_partial_kernel<T, true>), g1, dim3(256), 0, s, x, ldx, HW, C, chunk, nchunk, part, u,
                       stat, sem);
  else
    hipLaunchKernelGGL((in_stats_partial_kernel<T, false>), g1, dim3(256), 0, s, x, ldx, HW, C, chunk, nchunk, part, u,
                       stat, sem);
  if (sem || nchunk == 1) return;   // the statistics are final (fused fix-up, or one chunk per workgroup)
  const long bstride = up ? (long)u.H * u.W : HW;
  hipLaunchKernelGGL(in_stats_final_kernel<T>, g2, dim3(256), 0, s, x, ldx, bstride, B, HW, C, nchunk, part, stat);
}

static int in_stats_any(int dt, const void* x, int ldx, int B, int HW, int C, float* stat, void* ws, size_t ws_bytes,
                        const Up2xSrc* up, hipStream_t s, unsigned* sem, int nsem) {
  if (C % 16 || ldx % 8 || (uintptr_t)x % 16) return -1;
  if (!ws || ws_bytes < in_stats_workspace_bytes(B, HW, C)) return -1;
  float* part = reinterpret_cast<float*>(ws);
  static const int fuse_knob = GHOST_KNOB("GHOST_STATS_FUSE", 1);
  if (!fuse_knob || (long)B * ((C + 63) / 64) > nsem) sem = nullptr;   // one counter per (sample, 64 channels)
  if (dt == GHOST_F32)
    in_stats_launch((const float*)x, ldx, B, HW, C, stat, part, up, s, sem);
  else if (dt == GHOST_BF16)
    in_stats_launch((const bf16*)x, ldx, B, HW, C, stat, part, up, s, sem);
  else if (dt == GHOST_F16)
    in_stats_launch((const _Float16*)x, ldx, B, HW, C, stat, part, up, s, sem);
  else
    return -1;
  return (int)hipGetLastError();
}

int in_stats(int dt, const void* x, int ldx, int B, int HW, int C, float* stat, void* ws, size_t ws_bytes,
             hipStream_t s, unsigned* sem, int nsem) {
  return in_stats_any(dt, x, ldx, B, HW, C, stat, ws, ws_bytes, nullptr, s, sem, nsem);
}

int in_stats_up2x(int dt, const void* x, int ldx, int B, int H, int W, int C, float* stat, void* ws, size_t ws_bytes,
                  hipStream_t s, unsigned* sem, int nsem) {
  const Up2xSrc u = up2x_src(H, W);
  return in_stats_any(dt, x, ldx, B, 4 * H * W, C, stat, ws, ws_bytes, &u, s, sem, nsem);
}

// ---------------------------------------------------------------------------
// AAD mask: M_l[p] = sigmoid(sum_c wh_l[c] * (h[p,c] - mu[b,c]) * rstd[b,c] + bh_l)  (AADLayer.py:35)
// grid (pixel blocks of one sample, B); per-channel tables (wh*rstd, mu) staged in LDS once per
// block; one lane group of G = min(64, C/VEC) lanes per pixel; L <= 2 layers sharing h_in.
// ---------------------------------------------------------------------------
template <typename T, int L>
__global__ void __launch_bounds__(256)
aad_mask_kernel(const T* __restrict__ h, int ldh, int HW, int C, int G, int ppb, const float* __restrict__ stat,
                const float* __restrict__ wh0, const float* __restrict__ bh0, float* __restrict__ mask0,
                const float* __restrict__ wh1, const float* __restrict__ bh1, float* __restrict__ mask1) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ float s_tab[];   // [L][C] wh * rstd, [C] mean
  float* s_mu = s_tab + L * C;
  const int t = threadIdx.x, b = blockIdx.y;
  const float* st = stat + (long)b * C * 2;
  for (int c = t; c < C; c += 256) {
    const float mu = st[2 * c], rs = st[2 * c + 1];
    s_mu[c] = mu;
    s_tab[c] = wh0[c] * rs;
    if (L == 2) s_tab[C + c] = wh1[c] * rs;
  }
  __syncthreads();
  const int per = 256 / G, gl = t % G;
  const long base = (long)b * HW;
  const int pend = min(HW, (blockIdx.x + 1) * ppb);
  // the G lanes of a pixel share q (and the trip count), so the in-group shuffles stay converged;
  // four pixels per lane group are in flight at once (their loads issued before any FMA)
  constexpr int U = 4;
  for (int q0 = blockIdx.x * ppb + t / G; q0 < pend; q0 += U * per) {
    float s0[U], s1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { s0[u] = 0.f; s1[u] = 0.f; }
    for (int ci = gl; ci < C / VEC; ci += G) {
      float v[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * per;
        if (q < pend) load16_f(h + (base + q) * ldh + ci * VEC, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const int c = ci * VEC + e;
          const float d = v[u][e] - s_mu[c];
          s0[u] = fmaf(s_tab[c], d, s0[u]);
          if (L == 2) s1[u] = fmaf(s_tab[C + c], d, s1[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * per;
      const float a0 = group_sum(s0[u], G);
      const float a1 = L == 2 ? group_sum(s1[u], G) : 0.f;
      if (gl == 0 && q < pend) {
        mask0[base + q] = sigmoidf_ref(a0 + bh0[0]);
        if (L == 2) mask1[base + q] = sigmoidf_ref(a1 + bh1[0]);
      }
    }
  }
}

// 16-bit form with the per-channel tables in registers: lane gl of a G-lane pixel group always owns
// channels 8 (gl + G j), j < NCH, so its (wh * rstd) factors stay in VGPRs and the logit is one FMA
// per channel: sum_c (wh_c rstd_c) h_c - K with K = sum_c wh_c rstd_c mu_c per sample (as aad_v3).
// Measured against the LDS-table kernel above: the per-element LDS reads made it VALU/LDS-bound
// at 2-2.6 TB/s of h_in.
template <typename T, int L, int NCH>
__global__ void __launch_bounds__(256)
aad_mask_reg_kernel(const T* __restrict__ h, int ldh, int HW, int C, int G, int ppb, const float* __restrict__ stat,
                    const float* __restrict__ wh0, const float* __restrict__ bh0, float* __restrict__ mask0,
                    const float* __restrict__ wh1, const float* __restrict__ bh1, float* __restrict__ mask1) {
  const int t = threadIdx.x, b = blockIdx.y;
  const int per = 256 / G, gl = t % G;
  const float* st = stat + (long)b * C * 2;
  float tab[L][NCH][8];
  float k[L];
#pragma unroll
  for (int l = 0; l < L; ++l) k[l] = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = (gl + G * j) * 8 + e;
      const float mu = st[2 * c], rs = st[2 * c + 1];
#pragma unroll
      for (int l = 0; l < L; ++l) {
        tab[l][j][e] = (l ? wh1 : wh0)[c] * rs;
        k[l] = fmaf(tab[l][j][e], mu, k[l]);
      }
    }
  float bias[L];
#pragma unroll
  for (int l = 0; l < L; ++l) bias[l] = (l ? bh1 : bh0)[0] - group_sum(k[l], G);
  const long base = (long)b * HW;
  const int pend = min(HW, (blockIdx.x + 1) * ppb);
  constexpr int U = 4;
  for (int q0 = blockIdx.x * ppb + t / G; q0 < pend; q0 += U * per) {
    u32x4 raw[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * per;
#pragma unroll
      for (int j = 0; j < NCH; ++j)
        raw[u][j] = q < pend ? *reinterpret_cast<const u32x4*>(h + (base + q) * ldh + (gl + G * j) * 8)
                             : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float sl[L];
#pragma unroll
      for (int l = 0; l < L; ++l) sl[l] = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const T* e8 = reinterpret_cast<const T*>(&raw[u][j]);
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int l = 0; l < L; ++l) sl[l] = fmaf(tab[l][j][e], (float)e8[e], sl[l]);
      }
      const int q = q0 + u * per;
#pragma unroll
      for (int l = 0; l < L; ++l) sl[l] = group_sum(sl[l], G);
      if (gl == 0 && q < pend) {
        mask0[base + q] = sigmoidf_ref(sl[0] + bias[0]);
        if (L == 2) mask1[base + q] = sigmoidf_ref(sl[L - 1] + bias[L - 1]);
      }
    }
  }
}

int aad_mask2(int dt, const void* h, int ldh, int B, int HW, int C, const float* stat, const float* wh0,
              const float* bh0, float* mask0, const float* wh1, const float* bh1, float* mask1, hipStream_t s) {
  const int vec = dt == GHOST_F32 ? 4 : 8;
  if (C % vec || ldh % vec || (uintptr_t)h % 16) return -1;
  int G = C / vec;
  if (G > 64) G = 64;
  if (G & (G - 1)) return -1;   // power-of-two lane groups
  // >= ~2048 blocks to fill the chip; each block stages the tables once for its ppb pixels
  int ppb = (int)std::min<long>(256, std::max<long>(256 / G, (long)HW * B / 2048));
  if (ppb > HW) ppb = HW;
  dim3 grid((unsigned)((HW + ppb - 1) / ppb), (unsigned)B);
  const int L = wh1 ? 2 : 1;
  static const int use_reg = GHOST_KNOB("GHOST_MASK_REG", 1);
  if (use_reg && is16(dt) && (C == 8 * G || C == 16 * G)) {
    const int nch = C / (8 * G);
#define GHOST_MR(T, l, n)                                                                                        \
  hipLaunchKernelGGL((aad_mask_reg_kernel<T, l, n>), grid, dim3(256), 0, s, (const T*)h, ldh, HW, C, G, ppb, stat, \
                     wh0, bh0, mask0, wh1, bh1, mask1)
    if (dt == GHOST_BF16) {
      if (L == 2) { if (nch == 1) GHOST_MR(bf16, 2, 1); else GHOST_MR(bf16, 2, 2); }
      else { if (nch == 1) GHOST_MR(bf16, 1, 1); else GHOST_MR(bf16, 1, 2); }
    } else {
      if (L == 2) { if (nch == 1) GHOST_MR(_Float16, 2, 1); else GHOST_MR(_Float16, 2, 2); }
      else { if (nch == 1) GHOST_MR(_Float16, 1, 1); else GHOST_MR(_Float16, 1, 2); }
    }
#undef GHOST_MR
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)(L + 1) * C * sizeof(float);
#define GHOST_M(T, l)                                                                                            \
  hipLaunchKernelGGL((aad_mask_kernel<T, l>), grid, dim3(256), lds, s, (const T*)h, ldh, HW, C, G, ppb, stat, wh0, \
                     bh0, mask0, wh1, bh1, mask1)
  if (dt == GHOST_F32) {
    if (L == 2) GHOST_M(float, 2); else GHOST_M(float, 1);
  } else if (dt == GHOST_BF16) {
    if (L == 2) GHOST_M(bf16, 2); else GHOST_M(bf16, 1);
  } else if (dt == GHOST_F16) {
    if (L == 2) GHOST_M(_Float16, 2); else GHOST_M(_Float16, 1);
  } else {
    return -1;
  }
#undef GHOST_M
  return (int)hipGetLastError();
}

int aad_mask(int dt, const void* h, int ldh, int B, int HW, int C, const float* stat, const float* wh, const float* bh,
             float* mask, hipStream_t s) {
  return aad_mask2(dt, h, ldh, B, HW, C, stat, wh, bh, mask, nullptr, nullptr, nullptr, s);
}

// ---------------------------------------------------------------------------
// Small images (HW <= 64: the generator's 2x2 .. 8x8 stages): InstanceNorm statistics AND the AAD
// masks of up to two AADLayers in one launch, one workgroup per sample.  At these sizes the three
// separate launches (partials, final, mask) are launch-latency bound (~4-6 us each for < 1 MB).
// Phase 1: thread t owns 8 channels and walks the <= 64 pixels (shifted sums, fp64 merge of the
// fp32 partial as in_stats_final does).  Phase 2: one wave per pixel, lanes over the channels.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
stats_mask_small_kernel(const T* __restrict__ x, int ldx, int HW, int C, float* __restrict__ stat,
                        const float* __restrict__ wh0, const float* __restrict__ bh0, float* __restrict__ mask0,
                        const float* __restrict__ wh1, const float* __restrict__ bh1, float* __restrict__ mask1) {
  constexpr int VEC = Vec16<T>::N;
  __shared__ float s_cf[2][1024];
  __shared__ float s_k[2][4];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const T* xb = x + (long)b * HW * ldx;
  const int nch = C / VEC;
  const int L = wh1 ? 2 : 1;
  float kp[2] = {0.f, 0.f};
  for (int ci = t; ci < nch; ci += 256) {
    float K[VEC], s1[VEC], s2[VEC];
    load16_f(xb + ci * VEC, K);
#pragma unroll
    for (int e = 0; e < VEC; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
    for (int p = 0; p < HW; ++p) {
      float v[VEC];
      load16_f(xb + (long)p * ldx + ci * VEC, v);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float d = v[e] - K[e];
        s1[e] += d;
        s2[e] = fmaf(d, d, s2[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int c = ci * VEC + e;
      const double m1 = (double)s1[e] / HW;
      const double var = (double)s2[e] / HW - m1 * m1;
      const float mean = (float)((double)K[e] + m1);
      const float rs = (float)(1.0 / sqrt((var > 0.0 ? var : 0.0) + (double)kInEps));
      stat[((long)b * C + c) * 2 + 0] = mean;
      stat[((long)b * C + c) * 2 + 1] = rs;
      // mask logit = sum_c cf_c h_c + k, cf = wh * rstd, k = bh - sum_c cf_c mu_c
      const float cf0 = wh0[c] * rs;
      s_cf[0][c] = cf0;
      kp[0] = fmaf(-cf0, mean, kp[0]);
      if (L > 1) {
        const float cf1 = wh1[c] * rs;
        s_cf[1][c] = cf1;
        kp[1] = fmaf(-cf1, mean, kp[1]);
      }
    }
  }
  for (int l = 0; l < L; ++l) {
    float k = kp[l];
    for (int o = 32; o >= 1; o >>= 1) k += __shfl_xor(k, o, 64);
    if (lane == 0) s_k[l][wid] = k;
  }
  __syncthreads();
  float kk[2];
  for (int l = 0; l < L; ++l) kk[l] = s_k[l][0] + s_k[l][1] + s_k[l][2] + s_k[l][3] + (l ? bh1[0] : bh0[0]);
  for (int p = wid; p < HW; p += 4) {
    float acc[2] = {0.f, 0.f};
    for (int ci = lane; ci < nch; ci += 64) {
      float v[VEC];
      load16_f(xb + (long)p * ldx + ci * VEC, v);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        acc[0] = fmaf(s_cf[0][ci * VEC + e], v[e], acc[0]);
        if (L > 1) acc[1] = fmaf(s_cf[1][ci * VEC + e], v[e], acc[1]);
      }
    }
    for (int l = 0; l < L; ++l) {
      float a = acc[l];
      for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o, 64);
      if (lane == 0) (l ? mask1 : mask0)[(long)b * HW + p] = sigmoidf_ref(a + kk[l]);
    }
  }
}

bool stats_mask_small_ok(int dt, int HW, int C, int ldx) {
  const int vec = dt == GHOST_F32 ? 4 : 8;
  // (8x8 measured slower: 64 workgroups reading 128 KB each twice, 36 us against 21 us for the
  // separate passes at B = 64)
  return HW >= 1 && HW <= 16 && C % vec == 0 && C <= 1024 && ldx % vec == 0;
}

int stats_mask_small(int dt, const void* x, int ldx, int B, int HW, int C, float* stat, const float* wh0,
                     const float* bh0, float* mask0, const float* wh1, const float* bh1, float* mask1, hipStream_t s) {
  if (!stats_mask_small_ok(dt, HW, C, ldx) || !wh0 || !bh0 || !mask0 || (wh1 && (!bh1 || !mask1))) return -1;
  if (dt == GHOST_F32)
    hipLaunchKernelGGL(stats_mask_small_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)x, ldx, HW, C, stat,
                       wh0, bh0, mask0, wh1, bh1, mask1);
  else if (dt == GHOST_BF16)
    hipLaunchKernelGGL(stats_mask_small_kernel<bf16>, dim3(B), dim3(256), 0, s, (const bf16*)x, ldx, HW, C, stat,
                       wh0, bh0, mask0, wh1, bh1, mask1);
  else if (dt == GHOST_F16)
    hipLaunchKernelGGL(stats_mask_small_kernel<_Float16>, dim3(B), dim3(256), 0, s, (const _Float16*)x, ldx, HW, C,
                       stat, wh0, bh0, mask0, wh1, bh1, mask1);
  else
    return -1;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// bilinear x2, align_corners=True: src = dst * (in-1)/(out-1)
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
upsample2x_kernel(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy, const Up2xSrc u, int C, int lg_nch) {
  // grid: x = chunks of one output row (2W * C/VEC work items), y = b * 2H + oy; 32-bit index math only.
  // lg_nch >= 0: C/VEC is a power of two (every generator stage) and the chunk split is a shift
  constexpr int VEC = Vec16<T>::N;
  const int nch = C / VEC;
  const int Wo = 2 * u.W, Ho = 2 * u.H;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Wo * nch) return;
  const int row = blockIdx.y;
  const int b = row / Ho, oy = row - b * Ho;   // (once per thread, uniform)
  const int ox = lg_nch >= 0 ? i >> lg_nch : i / nch;
  const int ci = i - ox * nch;
  const Up2xTap t = up2x_tap(u, oy, ox);
  float o[VEC];
  up2x_load16_f(x + (long)b * u.H * u.W * ldx + ci * VEC, ldx, t, o);
  store16_f(y + ((long)row * Wo + ox) * ldy + ci * VEC, o);
}

// R output rows per workgroup (same sample: 2H % R == 0), each thread's 4R source loads issued
// before any of them is used: a 256 x 256 x 64 output is 16 K workgroups instead of 64 K
template <typename T, int R, bool NT = false>
__global__ void __launch_bounds__(256)
upsample2x_rows_kernel(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy, const Up2xSrc u, int lg_nch) {
  constexpr int VEC = Vec16<T>::N;
  const int Wo = 2 * u.W, Ho = 2 * u.H;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (Wo << lg_nch)) return;
  const int row0 = blockIdx.y * R;
  const int b = row0 / Ho, oy0 = row0 - b * Ho;
  const int ox = i >> lg_nch, ci = i - (ox << lg_nch);
  const T* xs = x + (long)b * u.H * u.W * ldx + ci * VEC;
  u32x4 raw[R][4];
  Up2xTap t[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    t[r] = up2x_tap(u, oy0 + r, ox);
    raw[r][0] = *reinterpret_cast<const u32x4*>(xs + t[r].o00 * ldx);
    raw[r][1] = *reinterpret_cast<const u32x4*>(xs + t[r].o01 * ldx);
    raw[r][2] = *reinterpret_cast<const u32x4*>(xs + t[r].o10 * ldx);
    raw[r][3] = *reinterpret_cast<const u32x4*>(xs + t[r].o11 * ldx);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const T* e00 = reinterpret_cast<const T*>(&raw[r][0]);
    const T* e01 = reinterpret_cast<const T*>(&raw[r][1]);
    const T* e10 = reinterpret_cast<const T*>(&raw[r][2]);
    const T* e11 = reinterpret_cast<const T*>(&raw[r][3]);
    float o[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e)
      o[e] = up2x_mix(t[r].ly0, t[r].ly1, t[r].lx0, t[r].lx1, to_f(e00[e]), to_f(e01[e]), to_f(e10[e]), to_f(e11[e]));
    if constexpr (NT)
      store16_f_nt(y + ((long)(row0 + r) * Wo + ox) * ldy + ci * VEC, o);
    else
      store16_f(y + ((long)(row0 + r) * Wo + ox) * ldy + ci * VEC, o);
  }
}

// Round 6: 2 x 2 output quads.  With align_corners and an exact x2 scale, output rows 2q-1 and 2q (q >= 1) both
// sample source rows (q-1, q), and output columns 2k-1 and 2k both sample source columns (k-1, k) (up2x_pairing_ok
// checks both facts in fp32 on the host, as aad_v3.hip's v5_pairing_ok does for rows).  So a thread that owns the
// quad {2q-1, 2q} x {2k-1, 2k} (one 16-byte chunk of channels) loads the 4 source chunks once and mixes its 4
// outputs from them — up2x_mix on the same operands with each output's own weights, the rows kernel's values bit for
// bit — 4 loads per 4 outputs instead of 4 per output (the rows kernel was bound by its L1 requests: the encoder's
// z_attr8, 0.69 GB of HBM traffic, took 169 us).  The edge quads (q = 0: rows {0, 2H-1}; k = 0: columns
// {0, 2W-1}) take each output's own taps.
template <typename T, bool NT>
__global__ void __launch_bounds__(256)
upsample2x_quad_kernel(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy, const Up2xSrc u, int lg_nch) {
  constexpr int VEC = Vec16<T>::N;
  const int Wo = 2 * u.W, Ho = 2 * u.H;
  const int i = blockIdx.x * 256 + threadIdx.x;   // (column pair k, chunk ci)
  if (i >= (u.W << lg_nch)) return;
  const int k = i >> lg_nch, ci = i - (k << lg_nch);
  const int bq = blockIdx.y, b = bq / u.H, q = bq - b * u.H;
  const int oy[2] = {q == 0 ? 0 : 2 * q - 1, q == 0 ? Ho - 1 : 2 * q};
  const int ox[2] = {k == 0 ? 0 : 2 * k - 1, k == 0 ? Wo - 1 : 2 * k};
  const T* xs = x + (long)b * u.H * u.W * ldx + ci * VEC;
  T* ys = y + (long)b * Ho * Wo * ldy + ci * VEC;
  auto put = [&](int oyy, int oxx, const float* o) {
    T* d = ys + ((long)oyy * Wo + oxx) * ldy;
    if constexpr (NT) store16_f_nt(d, o);
    else store16_f(d, o);
  };
  if (q == 0 || k == 0) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float o[VEC];
        up2x_load16_f(xs, ldx, up2x_tap(u, oy[r], ox[c]), o);
        put(oy[r], ox[c], o);
      }
    return;
  }
  Up2xTap t[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) t[r][c] = up2x_tap(u, oy[r], ox[c]);
  // every output of the quad has the taps (q-1, q) x (k-1, k): the first output's offsets serve all four
  float v00[VEC], v01[VEC], v10[VEC], v11[VEC];
  load16_f(xs + (long)t[0][0].o00 * ldx, v00);
  load16_f(xs + (long)t[0][0].o01 * ldx, v01);
  load16_f(xs + (long)t[0][0].o10 * ldx, v10);
  load16_f(xs + (long)t[0][0].o11 * ldx, v11);
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const Up2xTap& tt = t[r][c];
      float o[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) o[e] = up2x_mix(tt.ly0, tt.ly1, tt.lx0, tt.lx1, v00[e], v01[e], v10[e], v11[e]);
      put(oy[r], ox[c], o);
    }
}

// both grids of a x2 upsample pair up (see upsample2x_quad_kernel), checked in the kernel's fp32 arithmetic
static bool up2x_pairs(int n, float sc) {
  auto f0 = [&](int o, float* fr) {
    volatile float r = sc * (float)o;   // one fp32 multiply, as up2x_tap (no contraction)
    const int v = (int)r;
    if (fr) *fr = r - (float)v;
    return v;
  };
  float a, z;
  if (n < 2 || f0(0, &a) != 0 || a != 0.f || f0(2 * n - 1, &z) != n - 1 || z != 0.f) return false;
  for (int q = 1; q < n; ++q)
    if (f0(2 * q - 1, nullptr) != q - 1 || f0(2 * q, nullptr) != q - 1) return false;
  return true;
}

int upsample2x(int dt, const void* x, int ldx, void* y, int ldy, int B, int H, int W, int C, hipStream_t s) {
  const int vec = dt == GHOST_F32 ? 4 : 8;
  if (C % vec || ldx % vec || ldy % vec || (uintptr_t)x % 16 || (uintptr_t)y % 16) return -1;
  dim3 grid((unsigned)((2 * W * (C / vec) + 255) / 256), (unsigned)(B * 2 * H));
  // source scale (in-1)/(out-1) rounded once on the host, as PyTorch's area_pixel_compute_scale
  const Up2xSrc u = up2x_src(H, W);
  const int nch = C / vec;
  int lg = -1;
  if ((nch & (nch - 1)) == 0) for (lg = 0; (1 << lg) < nch; ++lg) {}
  static const int rows = GHOST_KNOB("GHOST_UP_ROWS", 2);
  if (is16(dt) && lg >= 0 && (rows == 2 || rows == 4) && (2 * H) % rows == 0 &&
      (long)H * W * ldx < (1L << 31)) {
    grid.y = (unsigned)(B * 2 * H / rows);
    // outputs of >= 64 MB (the encoder's z_attr8: 537 MB at B = 64, read again only by AADBlk8, long after it
    // has left L2 and the Infinity Cache) are written with non-temporal stores
    static const int nt_knob = GHOST_KNOB("GHOST_UP_NT", 1);
    const bool nt = nt_knob && (long)B * 4 * H * W * C * 2 >= (64L << 20);
    static const int quad = GHOST_KNOB("GHOST_UP_QUAD", 1);
    if (quad && up2x_pairs(H, u.sh) && up2x_pairs(W, u.sw)) {
      const dim3 gq((unsigned)((W * nch + 255) / 256), (unsigned)(B * H));
#define GHOST_UPQ(T)                                                                                           \
      if (nt)                                                                                                    \
        hipLaunchKernelGGL((upsample2x_quad_kernel<T, true>), gq, dim3(256), 0, s, (const T*)x, ldx, (T*)y, ldy, u, lg); \
      else                                                                                                       \
        hipLaunchKernelGGL((upsample2x_quad_kernel<T, false>), gq, dim3(256), 0, s, (const T*)x, ldx, (T*)y, ldy, u, lg);
      if (dt == GHOST_BF16) { GHOST_UPQ(bf16) } else { GHOST_UPQ(_Float16) }
#undef GHOST_UPQ
      return (int)hipGetLastError();
    }
#define GHOST_UPR(T)                                                                                               \
    if (rows == 4)                                                                                                 \
      hipLaunchKernelGGL((upsample2x_rows_kernel<T, 4>), grid, dim3(256), 0, s, (const T*)x, ldx, (T*)y, ldy, u, lg); \
    else if (nt)                                                                                                   \
      hipLaunchKernelGGL((upsample2x_rows_kernel<T, 2, true>), grid, dim3(256), 0, s, (const T*)x, ldx, (T*)y, ldy, u, \
                         lg);                                                                                      \
    else                                                                                                           \
      hipLaunchKernelGGL((upsample2x_rows_kernel<T, 2>), grid, dim3(256), 0, s, (const T*)x, ldx, (T*)y, ldy, u, lg);
    if (dt == GHOST_BF16) { GHOST_UPR(bf16) } else { GHOST_UPR(_Float16) }
#undef GHOST_UPR
    return (int)hipGetLastError();
  }
  if (dt == GHOST_F32)
    hipLaunchKernelGGL(upsample2x_kernel<float>, grid, dim3(256), 0, s, (const float*)x, ldx, (float*)y, ldy, u, C, lg);
  else if (dt == GHOST_BF16)
    hipLaunchKernelGGL(upsample2x_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, ldx, (bf16*)y, ldy, u, C, lg);
  else if (dt == GHOST_F16)
    hipLaunchKernelGGL(upsample2x_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)x, ldx, (_Float16*)y, ldy, u,
                       C, lg);
  else
    return -1;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// boundary conversions
// ---------------------------------------------------------------------------
template <typename TX, typename T>
__global__ void __launch_bounds__(256)
input_to_nhwc_kernel(const TX* __restrict__ x, long sb, long sc, long sh, long sw, int B, int C, int H, int W, int ldy,
                     T* __restrict__ y) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;   // one output element (channels >= C are zero)
  const long total = (long)B * ldy * H * W;
  if (idx >= total) return;
  const int c = (int)(idx % ldy);
  const long pix = idx / ldy;
  const int w = (int)(pix % W);
  const int h = (int)((pix / W) % H);
  const int b = (int)(pix / ((long)W * H));
  y[idx] = c < C ? from_f<T>(to_f(x[b * sb + c * sc + h * sh + w * sw])) : from_f<T>(0.f);
}

template <typename TX>
static int input_dispatch(const TX* x, const int64_t* st, int B, int C, int H, int W, int dt, void* y, int ldy,
                          hipStream_t s) {
  const long total = (long)B * ldy * H * W;
  dim3 grid((unsigned)((total + 255) / 256));
  if (dt == GHOST_F32)
    hipLaunchKernelGGL((input_to_nhwc_kernel<TX, float>), grid, dim3(256), 0, s, x, (long)st[0], (long)st[1],
                       (long)st[2], (long)st[3], B, C, H, W, ldy, (float*)y);
  else if (dt == GHOST_BF16)
    hipLaunchKernelGGL((input_to_nhwc_kernel<TX, bf16>), grid, dim3(256), 0, s, x, (long)st[0], (long)st[1],
                       (long)st[2], (long)st[3], B, C, H, W, ldy, (bf16*)y);
  else if (dt == GHOST_F16)
    hipLaunchKernelGGL((input_to_nhwc_kernel<TX, _Float16>), grid, dim3(256), 0, s, x, (long)st[0], (long)st[1],
                       (long)st[2], (long)st[3], B, C, H, W, ldy, (_Float16*)y);
  else
    return -1;
  return (int)hipGetLastError();
}

int input_to_nhwc(int xdt, const void* x, const int64_t strides[4], int B, int C, int H, int W, int dt, void* y,
                  hipStream_t s, int ldy) {
  if (ldy < C) return -1;
  switch (xdt) {
    case GHOST_F32: return input_dispatch((const float*)x, strides, B, C, H, W, dt, y, ldy, s);
    case GHOST_BF16: return input_dispatch((const bf16*)x, strides, B, C, H, W, dt, y, ldy, s);
    case GHOST_F16: return input_dispatch((const _Float16*)x, strides, B, C, H, W, dt, y, ldy, s);
    case GHOST_U8: return input_dispatch((const uint8_t*)x, strides, B, C, H, W, dt, y, ldy, s);
  }
  return -1;
}

// ldy = 3: plain RGB; ldy = 4: RGB + a zero fourth channel (8-byte bf16 pixels: the layout the
// encoder's first conv reads as aligned rows, conv_first.hip)
template <typename T>
__global__ void __launch_bounds__(256)
crops_kernel(const uint8_t* __restrict__ crops, long bstride, int B, int H, int W, T* __restrict__ y, int ldy,
             u32x4* __restrict__ zero, int nzero16) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;   // one output pixel
  if (idx < nzero16) zero[idx] = u32x4{0u, 0u, 0u, 0u};     // the call's reduction counters (zero_words' job)
  const long HW = (long)H * W;
  if (idx >= (long)B * HW) return;
  const int b = (int)(idx / HW);
  const long p = idx - b * HW;
  const uint8_t* src = crops + b * bstride + p * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float t = (float)src[2 - c] / 255.0f;   // BGR -> RGB, /255.
    t = (t - 0.5f) / 0.5f;
    y[idx * ldy + c] = from_f<T>(t);
  }
  if (ldy == 4) y[idx * 4 + 3] = from_f<T>(0.f);
}

int crops_u8_to_input(const uint8_t* crops, int64_t batch_stride, int B, int H, int W, int dt, void* y, hipStream_t s,
                      int ldy, unsigned* zero, int nzero) {
  if (ldy != 3 && ldy != 4) return -1;
  if (zero && (nzero % 4 || (uintptr_t)zero % 16)) return -1;
  const long total = (long)B * H * W;
  const int nz16 = zero ? nzero / 4 : 0;
  dim3 grid((unsigned)((std::max<long>(total, nz16) + 255) / 256));
  u32x4* z = reinterpret_cast<u32x4*>(zero);
  if (dt == GHOST_F32)
    hipLaunchKernelGGL(crops_kernel<float>, grid, dim3(256), 0, s, crops, (long)batch_stride, B, H, W, (float*)y, ldy,
                       z, nz16);
  else if (dt == GHOST_BF16)
    hipLaunchKernelGGL(crops_kernel<bf16>, grid, dim3(256), 0, s, crops, (long)batch_stride, B, H, W, (bf16*)y, ldy,
                       z, nz16);
  else if (dt == GHOST_F16)   // transform_target_to_torch(half=True) of the reference: float16
    hipLaunchKernelGGL(crops_kernel<_Float16>, grid, dim3(256), 0, s, crops, (long)batch_stride, B, H, W,
                       (_Float16*)y, ldy, z, nz16);
  else
    return -1;
  return (int)hipGetLastError();
}

template <typename T>
__global__ void __launch_bounds__(256)
y_u8_kernel(const T* __restrict__ y, int ldy, long P, uint8_t* __restrict__ out) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float t = (to_f(y[p * ldy + c]) * 0.5f + 0.5f) * 255.0f;
    out[p * 3 + (2 - c)] = (uint8_t)(int)t;
  }
}

int y_to_u8_bgr(int dt, const void* y, int ldy, int B, int H, int W, uint8_t* out, hipStream_t s) {
  const long P = (long)B * H * W;
  dim3 grid((unsigned)((P + 255) / 256));
  if (dt == GHOST_F32)
    hipLaunchKernelGGL(y_u8_kernel<float>, grid, dim3(256), 0, s, (const float*)y, ldy, P, out);
  else if (dt == GHOST_BF16)
    hipLaunchKernelGGL(y_u8_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)y, ldy, P, out);
  else if (dt == GHOST_F16)
    hipLaunchKernelGGL(y_u8_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)y, ldy, P, out);
  else
    return -1;
  return (int)hipGetLastError();
}

template <typename TX>
__global__ void __launch_bounds__(256) rows_f32_kernel(const TX* __restrict__ x, long rs, int B, int n, float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * n) return;
  const int b = (int)(i / n), k = (int)(i - (long)b * n);
  y[i] = to_f(x[b * rs + k]);
}

int rows_to_f32(int xdt, const void* x, int64_t row_stride, int B, int n, float* y, hipStream_t s) {
  dim3 grid((unsigned)(((long)B * n + 255) / 256));
  if (xdt == GHOST_F32)
    hipLaunchKernelGGL(rows_f32_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (long)row_stride, B, n, y);
  else if (xdt == GHOST_BF16)
    hipLaunchKernelGGL(rows_f32_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, (long)row_stride, B, n, y);
  else if (xdt == GHOST_F16)
    hipLaunchKernelGGL(rows_f32_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)x, (long)row_stride, B, n, y);
  else
    return -1;
  return (int)hipGetLastError();
}

struct GatherSegs {
  const uint4* tab[2];
  uint4* out[2];
  long row16[2];
};

// blockIdx.y = sample, blockIdx.z = segment; 16-byte copies of one table row
__global__ void __launch_bounds__(256) gather_rows_kernel(GatherSegs g, int n_rows, const int32_t* __restrict__ idx) {
  const int b = blockIdx.y, sg = blockIdx.z;
  int r = idx[b];
  r = r < 0 ? 0 : (r >= n_rows ? n_rows - 1 : r);
  const long n = g.row16[sg];
  const uint4* __restrict__ src = g.tab[sg] + (long)r * n;
  uint4* __restrict__ dst = g.out[sg] + (long)b * n;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
}

__global__ void __launch_bounds__(256) zero_words_kernel(u32x4* __restrict__ p, int n16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n16) p[i] = u32x4{0u, 0u, 0u, 0u};
}

int zero_words(unsigned* p, int nwords, hipStream_t s) {
  if (!p || nwords <= 0 || nwords % 4 || (uintptr_t)p % 16) return -1;
  const int n16 = nwords / 4;
  hipLaunchKernelGGL(zero_words_kernel, dim3((n16 + 255) / 256), dim3(256), 0, s, reinterpret_cast<u32x4*>(p), n16);
  return (int)hipGetLastError();
}

int gather_identity_rows(int nseg, const void* const* tab, const int64_t* row_bytes, void* const* out, int n_rows,
                         const int32_t* idx, int B, hipStream_t s) {
  if (nseg < 1 || nseg > 2 || n_rows < 1 || B < 1 || !idx) return -1;
  GatherSegs g{};
  long most = 0;
  for (int i = 0; i < nseg; ++i) {
    if (!tab[i] || !out[i] || row_bytes[i] <= 0 || row_bytes[i] % 16 || ((uintptr_t)tab[i] | (uintptr_t)out[i]) % 16)
      return -1;
    g.tab[i] = (const uint4*)tab[i];
    g.out[i] = (uint4*)out[i];
    g.row16[i] = row_bytes[i] / 16;
    most = most > g.row16[i] ? most : g.row16[i];
  }
  dim3 grid((unsigned)std::min<long>((most + 255) / 256, 32), (unsigned)B, (unsigned)nseg);
  hipLaunchKernelGGL(gather_rows_kernel, grid, dim3(256), 0, s, g, n_rows, idx);
  return (int)hipGetLastError();
}

template <typename T>
__global__ void __launch_bounds__(256)
nhwc_nchw_kernel(const T* __restrict__ x, int ldx, int B, int H, int W, int C, T* __restrict__ y) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;   // NCHW linear index
  const long HW = (long)H * W;
  if (idx >= (long)B * C * HW) return;
  const long p = idx % HW;
  const int c = (int)((idx / HW) % C);
  const int b = (int)(idx / (HW * C));
  y[idx] = x[(b * HW + p) * ldx + c];
}

int nhwc_to_nchw(int dt, const void* x, int ldx, int B, int H, int W, int C, void* y, hipStream_t s) {
  const long total = (long)B * C * H * W;
  dim3 grid((unsigned)((total + 255) / 256));
  if (dt == GHOST_F32)
    hipLaunchKernelGGL(nhwc_nchw_kernel<float>, grid, dim3(256), 0, s, (const float*)x, ldx, B, H, W, C, (float*)y);
  else if (dt == GHOST_BF16)
    hipLaunchKernelGGL(nhwc_nchw_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, ldx, B, H, W, C, (bf16*)y);
  else if (dt == GHOST_F16)
    hipLaunchKernelGGL(nhwc_nchw_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)x, ldx, B, H, W, C,
                       (_Float16*)y);
  else
    return -1;
  return (int)hipGetLastError();
}

}  // namespace ghost
