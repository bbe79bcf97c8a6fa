// ghost_amd — AADBlk8's tail in one kernel (bf16, C = 64): the block's last add_blocks AADLayer, its
// last_add_block AADLayer, both ReLUs, and the output conv of the fused [x-branch ‖ h'-branch] 3x3
// (128 -> 3) with tanh and the BGR uint8 copy (AADLayer.py:20-38,53-80; AEI_Net.py:138-139;
// faceshifter_run.py:20-21).
//
// Unfused, the two AADLayer outputs (2 x 64 channels at 256x256) are written to HBM and read back by
// the output conv: 2.1 GB per B = 64 batch.  Here a workgroup owns a 16 x 32 output tile and
// computes both AADLayers on its 18 x 34 halo (1.2x the pixels), feeding each 16-pixel fragment of
// the (bf16-rounded, as stored unfused) AADLayer outputs straight into the MFMA of the per-tap partial
// sums Z[p][t*3 + o] = sum_c cat[p][c] w[t][o][c] (the narrow-conv formulation of conv_narrow.hip);
// Z stays in LDS and the 3x3 gather, tanh and stores follow.  HBM: the two AADLayer inputs and
// z_attr once (+ halo), 3 output channels + uint8.
//
// AADLayer math per (pixel, channel) as aad_v3.hip: transposed MFMA with the permuted weight rows of
// pack.py pack_aad_v3 (lane accumulators = gamma, beta of 8 channels of one pixel), mask from the
// lane's 16 channels + two xor-shuffles, blend, ReLU.
#include <cstdlib>

#include "aad_tail.h"
#include "ghost_common.h"
#include "up2x.h"

namespace ghost {

namespace {
constexpr int TH = 16, TW = 32;
constexpr int HHT = TH + 2, HWT = TW + 2;   // 18 x 34 halo
constexpr int HP = HHT * HWT;               // 612 halo pixels
constexpr int NRT = (HP + 15) / 16;         // 39 tiles of 16 pixels
constexpr int ZLD = 33;
constexpr int kW = 8;                       // waves
}  // namespace

struct AadTailArgs {
  const bf16* za;  int lda;
  const bf16* hin[2];  int ldh[2];          // layer 0: the x-branch input, layer 1: the block input m
  Up2xSrc up[2];                            // up[l].H > 0: hin[l] is the [B, H, W] source of an x2 upsample
  const float* stat[2];                     // [B][64][2] mean, rstd of each layer's (virtual) input
  const bf16* w3[2];
  const float* b3[2];
  const float* wh[2];
  const float* bh[2];
  const float* idgb[2];
  int id_ld;
  const bf16* wn;                           // [32][128] narrow conv weights (pack_conv3x3_narrow)
  bf16* y;                                  // [B, H, W, 3]
  uint8_t* u8;
  int H, W, tanh_out;
};

template <int CA, bool UP0, bool UP1>
__global__ void __launch_bounds__(512) aad_tail_kernel(const AadTailArgs a) {
  constexpr int C = 64, KS = CA / 32, WLD = CA + 8;
  __shared__ __attribute__((aligned(16))) bf16 s_w[2 * 128 * WLD];
  __shared__ __attribute__((aligned(16))) float s_b[2 * 128];
  __shared__ __attribute__((aligned(16))) float s_rs[2 * C];
  __shared__ __attribute__((aligned(16))) float s_nm[2 * C];
  __shared__ __attribute__((aligned(16))) float s_cf[2 * C];
  __shared__ __attribute__((aligned(16))) float s_gi[2 * C];
  __shared__ __attribute__((aligned(16))) float s_bi[2 * C];
  __shared__ float s_k[2];
  __shared__ float Z[NRT * 16 * ZLD];

  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int tiles_x = a.W / TW, tiles_y = a.H / TH;
  const int b = blockIdx.x / (tiles_x * tiles_y);
  const int rr = blockIdx.x - b * tiles_x * tiles_y;
  const int y0 = (rr / tiles_x) * TH, x0 = (rr % tiles_x) * TW;
  const long img = (long)b * a.H * a.W;

  for (int l = 0; l < 2; ++l) {
    for (int idx = tid; idx < 128 * (CA / 8); idx += kW * 64) {
      const int row = idx / (CA / 8), kc = idx - row * (CA / 8);
      *reinterpret_cast<u32x4*>(&s_w[(l * 128 + row) * WLD + kc * 8]) =
          *reinterpret_cast<const u32x4*>(a.w3[l] + (long)row * CA + kc * 8);
    }
    for (int idx = tid; idx < 128; idx += kW * 64) s_b[l * 128 + idx] = a.b3[l][idx];
    for (int c = tid; c < C; c += kW * 64) {
      const float mu = a.stat[l][((long)b * C + c) * 2], rs = a.stat[l][((long)b * C + c) * 2 + 1];
      s_rs[l * C + c] = rs;
      s_nm[l * C + c] = -mu * rs;
      s_cf[l * C + c] = a.wh[l][c] * rs;
      s_gi[l * C + c] = a.idgb[l][(long)b * a.id_ld + c];
      s_bi[l * C + c] = a.idgb[l][(long)b * a.id_ld + C + c];
    }
  }
  // narrow-conv weight fragments (B operand): rows lr and 16 + lr, four 32-channel k-steps
  bf16x8 wf0[4], wf1[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32x4 b0 = *reinterpret_cast<const u32x4*>(a.wn + lr * 128 + k * 32 + lq * 8);
    const u32x4 b1 = *reinterpret_cast<const u32x4*>(a.wn + (16 + lr) * 128 + k * 32 + lq * 8);
    __builtin_memcpy(&wf0[k], &b0, 16);
    __builtin_memcpy(&wf1[k], &b1, 16);
  }
  __syncthreads();
  if (wid < 2) {
    float k = 0.f;
    for (int c = lane; c < C; c += 64) k = fmaf(a.wh[wid][c], s_nm[wid * C + c], k);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) k += __shfl_xor(k, o, 64);
    if (lane == 0) s_k[wid] = k;
  }
  __syncthreads();
  const float bh0 = a.bh[0][0] + s_k[0], bh1 = a.bh[1][0] + s_k[1];

  // per 16-pixel halo tile: pixel of this lane, clamped to (0, 0) outside the image
  auto pix_of = [&](int rt, bool& ok, int& iyc, int& ixc, long& p) {
    const int hp = rt * 16 + lr;
    const int hy = hp / HWT, hx = hp - hy * HWT;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    // pixels outside the image (or past the halo) run the same code on pixel (0, 0) and contribute
    // zeros: the output conv zero-pads its input, the AADLayer outputs
    ok = hp < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    iyc = ok ? iy : 0;
    ixc = ok ? ix : 0;
    p = img + (long)iyc * a.W + ixc;
  };
  // z_attr and (when direct) layer 0's h_in of the next tile are loaded while the current tile
  // computes; layer 1 (the block input, through the upsample: L2-resident source) runs first so its
  // loads are the only ones a tile waits for
  auto load_direct = [&](long p, u32x4 (&zz)[KS], u32x4 (&xx)[2]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) zz[ks] = *reinterpret_cast<const u32x4*>(a.za + p * a.lda + ks * 32 + lq * 8);
    if constexpr (!UP0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) xx[j] = *reinterpret_cast<const u32x4*>(a.hin[0] + p * a.ldh[0] + j * 32 + lq * 8);
    }
  };
  u32x4 zc[KS], xc[2], zn[KS], xn[2];
  {
    bool ok0; int iy0, ix0; long p0;
    pix_of(wid, ok0, iy0, ix0, p0);
    load_direct(p0, zc, xc);
  }
  for (int rt = wid; rt < NRT; rt += kW) {
    asm volatile("" ::: "memory");
    bool ok; int iyc, ixc; long p;
    pix_of(rt, ok, iyc, ixc, p);
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      const int l = 1 - li;
      asm volatile("" ::: "memory");
      // this layer's h_in chunks (channels 32 sh + 8 lq .. +7 of the pixel)
      u32x4 hc[2];
      const bool up = l == 0 ? UP0 : UP1;
      if (up) {
        const Up2xSrc u = a.up[l];
        const Up2xTap tp = up2x_tap(u, iyc, ixc);
        const bf16* src = a.hin[l] + (long)b * u.H * u.W * a.ldh[l];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v[8];
          up2x_load16_f(src + j * 32 + lq * 8, a.ldh[l], tp, v);
          bf16* hv = reinterpret_cast<bf16*>(&hc[j]);
#pragma unroll
          for (int e = 0; e < 8; ++e) hv[e] = (bf16)v[e];
        }
      } else if (l == 0) {
        hc[0] = xc[0];
        hc[1] = xc[1];
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          hc[j] = *reinterpret_cast<const u32x4*>(a.hin[l] + p * a.ldh[l] + j * 32 + lq * 8);
      }
      if (li == 1) {
        asm volatile("" ::: "memory");
        if (rt + kW < NRT) {
          bool okn; int iyn, ixn; long pn;
          pix_of(rt + kW, okn, iyn, ixn, pn);
          load_direct(pn, zn, xn);
        }
      }
      float ms = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c0 = j * 32 + lq * 8;
        const bf16* hv = reinterpret_cast<const bf16*>(&hc[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) ms = fmaf(s_cf[l * C + c0 + e], (float)hv[e], ms);
      }
      ms += __shfl_xor(ms, 16, 64);
      ms += __shfl_xor(ms, 32, 64);
      const float Mk = sigmoidf_ref(ms + (l == 0 ? bh0 : bh1));
      const bf16* Wl = s_w + l * 128 * WLD;
#pragma unroll
      for (int sh = 0; sh < 2; ++sh) {
        asm volatile("" ::: "memory");
        f32x4 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rt4 = (i & 1) + 2 * sh + 4 * (i >> 1);
          acc[i] = *reinterpret_cast<const f32x4*>(&s_b[l * 128 + rt4 * 16 + lq * 4]);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          bf16x8 bfrag;
          __builtin_memcpy(&bfrag, &zc[ks], 16);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rt4 = (i & 1) + 2 * sh + 4 * (i >> 1);
            const bf16x8 afrag = *reinterpret_cast<const bf16x8*>(&Wl[(rt4 * 16 + lr) * WLD + ks * 32 + lq * 8]);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afrag, bfrag, acc[i], 0, 0, 0);
          }
        }
        const int c0 = sh * 32 + lq * 8;
        const bf16* hv = reinterpret_cast<const bf16*>(&hc[sh]);
        bf16x8 of;   // the AADLayer output chunk, rounded to bf16 as the unfused path stores it
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float hh = fmaf((float)hv[e], s_rs[l * C + c0 + e], s_nm[l * C + c0 + e]);
          const float g = acc[e >> 2][e & 3];
          const float be = acc[2 + (e >> 2)][e & 3];
          const float A = fmaf(g, hh, be);
          const float I = fmaf(s_gi[l * C + c0 + e], hh, s_bi[l * C + c0 + e]);
          const float v = fmaf(Mk, I - A, A);
          of[e] = (bf16)(ok && v > 0.f ? v : 0.f);      // + the ReLU of AddBlocksSequential
        }
        // cat channel 64 l + 32 sh + 8 lq + e: k-step 2l + sh of the output conv's partial sums
        const int kst = 2 * l + sh;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, wf0[kst], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of, wf1[kst], acc1, 0, 0, 0);
      }
    }
    // C layout: pixel (row) lq*4 + i of the tile, column lr
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rt * 16 + lq * 4 + i;
      Z[row * ZLD + lr] = acc0[i];
      Z[row * ZLD + 16 + lr] = acc1[i];
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) zc[ks] = zn[ks];
    xc[0] = xn[0];
    xc[1] = xn[1];
  }
  __syncthreads();

  // gather: one output pixel per thread (512 threads = the 16 x 32 tile)
  const int oy = tid / TW, ox = tid - oy * TW;
  const long q = img + (long)(y0 + oy) * a.W + (x0 + ox);
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    float s = 0.f;
#pragma unroll
    for (int ty = 0; ty < 3; ++ty)
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) s += Z[((oy + ty) * HWT + ox + tx) * ZLD + (ty * 3 + tx) * 3 + o];
    if (a.tanh_out) s = tanhf(s);
    a.y[q * 3 + o] = (bf16)s;
    if (a.u8) {
      const float t = (s * 0.5f + 0.5f) * 255.0f;   // faceshifter_run.py:20-21
      a.u8[q * 3 + (2 - o)] = (uint8_t)(int)t;
    }
  }
}

bool aad_tail_supported(int dt, int H, int W, int Ca, int lda, int ldh0, int ldh1) {
  return dt == GHOST_BF16 && H % TH == 0 && W % TW == 0 && (Ca == 64 || Ca == 32) && lda % 8 == 0 &&
         ldh0 % 8 == 0 && ldh1 % 8 == 0;
}

int aad_tail(const AadTailDesc& d, hipStream_t s) {
  if (!aad_tail_supported(GHOST_BF16, d.H, d.W, d.Ca, d.lda, d.ldh[0], d.ldh[1])) return -1;
  AadTailArgs a{};
  a.za = (const bf16*)d.za; a.lda = d.lda;
  for (int l = 0; l < 2; ++l) {
    a.hin[l] = (const bf16*)d.hin[l]; a.ldh[l] = d.ldh[l];
    a.up[l] = d.up_H[l] > 0 ? up2x_src(d.up_H[l], d.up_W[l]) : Up2xSrc{0, 0, 0.f, 0.f};
    if (d.up_H[l] > 0 && (2 * d.up_H[l] != d.H || 2 * d.up_W[l] != d.W)) return -1;
    a.stat[l] = d.stat[l]; a.w3[l] = (const bf16*)d.w3[l]; a.b3[l] = d.b3[l]; a.wh[l] = d.wh[l];
    a.bh[l] = d.bh[l]; a.idgb[l] = d.idgb[l];
  }
  a.id_ld = d.id_ld; a.wn = (const bf16*)d.wn; a.y = (bf16*)d.y; a.u8 = d.u8;
  a.H = d.H; a.W = d.W; a.tanh_out = d.tanh_out;
  const bool up0 = d.up_H[0] > 0, up1 = d.up_H[1] > 0;
  dim3 grid((unsigned)(d.B * (d.H / TH) * (d.W / TW)));
#define GHOST_TAIL(ca, u0, u1)                                                                    \
  if (d.Ca == ca && up0 == u0 && up1 == u1) {                                                     \
    hipLaunchKernelGGL((aad_tail_kernel<ca, u0, u1>), grid, dim3(kW * 64), 0, s, a);              \
    return (int)hipGetLastError();                                                                \
  }
  GHOST_TAIL(64, false, true) GHOST_TAIL(64, true, true) GHOST_TAIL(64, false, false)
  GHOST_TAIL(32, false, true) GHOST_TAIL(32, true, true) GHOST_TAIL(32, false, false)
#undef GHOST_TAIL
  return -1;
}

}  // namespace ghost
