// ghost_amd — AADLayer kernel for the high-resolution stages (C in {64, 128}, bf16).
//
// AADLayer.py:20-38 (+ the following ReLU) for up to two AADLayers that read the same
// h_in and z_attr (AAD_ResBlk's first add_block layer and its last_add_block layer,
// AADLayer.py:53-79), sharing every byte of input traffic:
//
//   per 16-pixel tile and wave:
//     h  = (h_in - mu) * rstd                                   (16 channels per lane, fp32)
//     M_l = sigmoid(sum_c wh_l[c] h[c] + bh_l)                   (lane partials + 2 xor-shuffles)
//     [gamma|beta]_l^T = W_l . z_attr^T + b_l                    (MFMA 16x16x32, W_l in LDS,
//                                                                 z_attr fragments straight from HBM)
//     out_l = relu((1 - M_l)(gamma h + beta) + M_l (gi h + bi))  (16-byte stores)
//
// The GEMM is computed transposed (rows = weight rows, columns = pixels) with the weight
// rows permuted (pack.py pack_aad_v3) so that the accumulator a lane holds is gamma and
// beta of 16 *contiguous-in-pairs-of-8* channels of ONE pixel: the blend needs no LDS
// round trip and every global access is a 16-byte vector along channels.
// HBM bytes per launch = |h_in| + |z_attr| + L * |out|  (the algorithmic minimum).
#include <cstdlib>
#include <type_traits>

#include "aad_v3.h"
#include "ghost_common.h"
#include "tap_rows.h"
#include "up2x.h"

namespace ghost {

template <typename T>   // T: the 16-bit storage type (bf16, or fp16 for a .half() module)
struct AadV3ArgsT {
  const T* za;
  const T* hin;
  const float* stat;
  const T* w3[2];
  const float* b3[2];
  const float* wh[2];
  const float* bh[2];
  const float* idgb[2];
  T* out[2];
  int ldo[2];
  int lda, ldh, id_ld, HW, PPW;
  const T* zw[2];   // tap-partial projection rows (ZPM layers), row stride zwld
  int zwld;
  float slope;
  Up2xSrc up;   // UP: h_in is the bilinear x2 upsample of hin (a [B, up.H, up.W] source)
  // in-kernel clock (nullptr = off): per workgroup its start stamp tclk[blockIdx.x], per wave its end stamp
  // tclk[grid + blockIdx.x * 8 + wave], wall-clock ticks (hipDeviceAttributeWallClockRate); plain stores to
  // distinct words, so the clock does not perturb the kernel (one contended atomic per wave did: +100 us)
  unsigned long long* tclk;
  int v5_xcd;   // v5: blocks in XCD-contiguous order
  int v5_ipw;   // v5: 1024-pixel work items per workgroup
  int v5_flags; // v5, tuning build only: epilogue A/B (aad_v5_kernel)
};

static constexpr int kWaves = 8;

// tap partials (tap_rows.h): MFMA row tile o, row 4 dy + dx holds the projection of tap (dy, dx) to channel o
// (dy, dx < 3), so a lane (pixel lr, lq = dy) ends with the three dx of each o; the lane then sums its row
// neighbours inside the 8-column segment and stores fp16 row sums plus the segment-end terms.  LDS holds the
// 27 real rows, 9 o + 3 dy + dx; the A rows with dy or dx = 3 re-read a real row of their 8-lane group (the
// same address: a broadcast, no bank conflict) and produce values nothing stores.
constexpr int ZLD = 64;
constexpr int kZpRows = 27;
// element offset of (row, k) in an unpadded image of 64-element (128-byte) rows with the 16-byte chunks XOR-
// swizzled by row & 7: the ds_read_b128 of rows 16 rt + lr, chunk 4 ks + lq is conflict-free in every 16-lane
// group (the +8-element padding it replaces was 2-way in half the groups and cost 1 KB per 64 rows)
GHOST_DEV int sw64(int row, int k) { return row * 64 + ((((k >> 3) ^ (row & 7)) << 3) | (k & 7)); }
// the same for 32-element (64-byte) rows: chunks XOR-swizzled by (row >> 1) & 3
GHOST_DEV int sw32(int row, int k) { return row * 32 + ((((k >> 3) ^ ((row >> 1) & 3)) << 3) | (k & 7)); }
// 128-element (256-byte, one bank row) rows: chunks XOR-swizzled by row & 15
GHOST_DEV int sw128(int row, int k) { return row * 128 + ((((k >> 3) ^ (row & 15)) << 3) | (k & 7)); }
// the weight-row image of the AAD GEMMs (Ca-element rows, unpadded): the A-fragment ds_read_b128 of rows
// 16 rt + lr, chunk 4 ks + lq meets no bank conflict in any 16-lane group (the Ca + 8 padding these replace
// was 2-way on half the groups' slots at Ca = 64)
template <int CA>
GHOST_DEV int swca(int row, int k) {
  if constexpr (CA == 128) return sw128(row, k);
  else if constexpr (CA == 64) return sw64(row, k);
  else return sw32(row, k);
}
// LDS slot of layer l's projection rows: only the layers in ZPM are staged
template <int ZPM>
GHOST_DEV constexpr int zp_slot(int l) { return l == 0 ? 0 : (ZPM & 1); }
template <int ZPM>
constexpr int zp_nlayers() { return (ZPM & 1) + ((ZPM >> 1) & 1); }

// one K half (K step ks = the half sh just computed) into the three row tiles: 12 accumulator registers live
template <typename T>
GHOST_DEV void zp_mfma_half(const T* __restrict__ W, const v8_t<T>& xf, int ks, f32x4 (&acc)[3], int lr, int lq) {
  const int dy = min(lr >> 2, 2), dx = min(lr & 3, 2);
#pragma unroll
  for (int rt = 0; rt < 3; ++rt) {
    asm volatile("" ::: "memory");   // the projection rows are re-read per use, not held across the tile loop
    const int row = rt * 9 + dy * 3 + dx;
    const v8_t<T> wf = *reinterpret_cast<const v8_t<T>*>(&W[sw64(row, ks * 32 + lq * 8)]);
    acc[rt] = mfma16x16x32<T>(wf, xf, acc[rt]);
  }
}
GHOST_DEV float zp_from_left(float v) {    // lane lr - 1's value (row_shr:1 within the 16-lane row)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true));
}
GHOST_DEV float zp_from_right(float v) {   // lane lr + 1's value (row_shl:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xf, 0xf, true));
}
// the lane's pixel p (in the image) at column lr & 7 of its segment; zimg = the image's buffer (tap_rows.h)
GHOST_DEV void zp_store_acc(const f32x4 (&acc)[3], _Float16* __restrict__ zimg, long p, int HW, int lr, int lq) {
  typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
  const int col = lr & 7;
  float R[3];
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    const float l = zp_from_left(acc[o][0]), r = zp_from_right(acc[o][2]);
    R[o] = ((col != 0 ? l : 0.f) + acc[o][1]) + (col != 7 ? r : 0.f);
  }
  if (lq < 3) {
    *reinterpret_cast<f16x4*>(zimg + p * kZrR + lq * 4) = f16x4{(_Float16)R[0], (_Float16)R[1], (_Float16)R[2], 0};
    _Float16* e = zimg + (long)HW * kZrR + (p >> 3) * kZrE + lq * 4;
    if (col == 0)
      *reinterpret_cast<f16x4*>(e) = f16x4{(_Float16)acc[0][2], (_Float16)acc[1][2], (_Float16)acc[2][2], 0};
    if (col == 7)
      *reinterpret_cast<f16x4*>(e + 12) = f16x4{(_Float16)acc[0][0], (_Float16)acc[1][0], (_Float16)acc[2][0], 0};
  }
}
// the same from both K halves' bf16 outputs (xf[sh] = channels 32 sh + 8 lq .. +7 of pixel lr)
template <typename T>
GHOST_DEV void zp_store(const T* __restrict__ W, const v8_t<T> (&xf)[2], _Float16* __restrict__ zimg, long p, int HW,
                        int lr, int lq) {
  f32x4 acc[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) zp_mfma_half(W, xf[ks], ks, acc, lr, lq);
  zp_store_acc(acc, zimg, p, HW, lr, lq);
}

// projection row 9 o + 3 dy + dx <- the packed narrow-conv row (dy * 3 + dx) * 3 + o (pack_conv3x3_narrow)
template <typename T, int L, int ZPM, int NT>
GHOST_DEV void zp_stage_weights(const AadV3ArgsT<T>& a, T* s_wz, int tid) {
  if constexpr (ZPM != 0) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      if (!((ZPM >> l) & 1)) continue;
      for (int idx = tid; idx < kZpRows * 8; idx += NT) {
        const int row = idx >> 3, kc = idx & 7;
        const int o = row / 9, t = row - o * 9;   // row 9 o + t, t = dy * 3 + dx
        const u32x4 v = *reinterpret_cast<const u32x4*>(a.zw[l] + (long)(t * 3 + o) * a.zwld + kc * 8);
        *reinterpret_cast<u32x4*>(&s_wz[zp_slot<ZPM>(l) * kZpRows * ZLD + sw64(row, kc * 8)]) = v;   // as the reads
      }
    }
  }
}

template <typename T, int C, int CA, int L, bool UP, int NWV = kWaves, int ZPM = 0>
GHOST_DEV void aad_v3_body(const AadV3ArgsT<T>& a) {
  static_assert(ZPM == 0 || C == 64, "tap partials: C = 64");
  constexpr int CT = C / 64;          // 64-channel tiles
  constexpr int KS = CA / 32;         // MFMA k-steps
  constexpr int WLD = CA;             // LDS weight row (T elements; chunks swizzled, swca)
  constexpr int NH = CT * 2;          // 16-byte h_in chunks per lane (8 channels each)
  __shared__ __attribute__((aligned(16))) T s_w[L * CT * 128 * WLD];
  __shared__ __attribute__((aligned(16))) float s_b[L * CT * 128];
  __shared__ __attribute__((aligned(16))) float s_rs[C];
  __shared__ __attribute__((aligned(16))) float s_nm[C];
  // mask rows: cf_l = wh_l * rstd split in three 16-bit parts (hi, mid, lo), the logits as MFMAs over the h
  // fragments (see aad_v5_kernel: the split keeps cf to ~2^-26 through the cancellation against s_k)
  __shared__ __attribute__((aligned(16))) T s_mA[L * 3 * C];
  __shared__ float s_k[L];                                        // sum_c wh * (-mu * rstd)
  __shared__ __attribute__((aligned(16))) float s_gi[L * C];
  __shared__ __attribute__((aligned(16))) float s_bi[L * C];
  __shared__ __attribute__((aligned(16))) T s_wz[ZPM ? zp_nlayers<ZPM>() * kZpRows * ZLD : 8];

  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int mrow = (lr & 3) == 3 ? 0 : (lr & 3);   // mask A row: part lr & 3 of the split (row 3 repeats hi)
  const bool relu = a.slope == 0.f;                // the ReLU after every generator AADLayer: one packed max
  const long p_begin = (long)blockIdx.x * a.PPW;
  const int b = (int)(p_begin / a.HW);     // PPW divides HW: one sample per workgroup
  zp_stage_weights<T, L, ZPM, NWV * 64>(a, s_wz, tid);

  // ---- resident weights, biases and per-channel tables ----
  for (int l = 0; l < L; ++l) {
    for (int idx = tid; idx < CT * 128 * (CA / 8); idx += NWV * 64) {
      const int row = idx / (CA / 8), kc = idx - row * (CA / 8);
      *reinterpret_cast<u32x4*>(&s_w[swca<CA>(l * CT * 128 + row, kc * 8)]) =
          *reinterpret_cast<const u32x4*>(a.w3[l] + (long)row * CA + kc * 8);
    }
    // GEMM bias with the identity path folded in: row rho of tile ct (pack_aad_v3) starts from b3 - gi (gamma
    // rows) or b3 - bi (beta rows) of its channel, so out = I + (1 - M) (D_gamma hh + D_beta)
    for (int idx = tid; idx < CT * 128; idx += NWV * 64) {
      const int ct = idx >> 7, rho = idx & 127, i = rho >> 4;
      const int c = ct * 64 + 32 * ((i >> 1) & 1) + 8 * ((rho >> 2) & 3) + 4 * (i & 1) + (rho & 3);
      s_b[l * CT * 128 + idx] = a.b3[l][idx] - a.idgb[l][(long)b * a.id_ld + (i < 4 ? c : C + c)];
    }
    for (int c = tid; c < C; c += NWV * 64) {
      const float cf = a.wh[l][c] * a.stat[((long)b * C + c) * 2 + 1];
      const T hi = (T)cf;
      const float r1 = cf - (float)hi;
      const T mid = (T)r1;
      s_mA[(l * 3) * C + c] = hi;
      s_mA[(l * 3 + 1) * C + c] = mid;
      s_mA[(l * 3 + 2) * C + c] = (T)(r1 - (float)mid);
      s_gi[l * C + c] = a.idgb[l][(long)b * a.id_ld + c];
      s_bi[l * C + c] = a.idgb[l][(long)b * a.id_ld + C + c];
    }
  }
  for (int c = tid; c < C; c += NWV * 64) {
    const float mu = a.stat[((long)b * C + c) * 2], rs = a.stat[((long)b * C + c) * 2 + 1];
    s_rs[c] = rs;
    s_nm[c] = -mu * rs;
  }
  __syncthreads();
  // mask logit = sum_c wh_c * ((h_c - mu_c) * rs_c) + bh = sum_c cf_c * h_c + k + bh: one FMA per channel
  if (wid < L) {
    float k = 0.f;
    for (int c = lane; c < C; c += 64) k = fmaf(a.wh[wid][c], s_nm[c], k);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) k += __shfl_xor(k, o, 64);
    if (lane == 0) s_k[wid] = k;
  }
  __syncthreads();

  float bh[L];
#pragma unroll
  for (int l = 0; l < L; ++l) bh[l] = a.bh[l][0] + s_k[l];

  // one 16-pixel tile per wave iteration; latency is hidden by the 8 waves of the workgroup
  // and the co-resident workgroups (no software prefetch: it would cost the occupancy)
  const int ntiles = a.PPW / 16;
  for (int t = wid; t < ntiles; t += NWV) {
    // compiler memory barrier: keeps the per-channel LDS tables from being hoisted out of the
    // loop into (hundreds of) registers; re-reading them from LDS each tile is cheap
    asm volatile("" ::: "memory");
    const long p = p_begin + t * 16 + lr;
    u32x4 zc[KS], hc[NH];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) zc[ks] = *reinterpret_cast<const u32x4*>(a.za + p * a.lda + ks * 32 + lq * 8);
    if constexpr (UP) {
      // the tile's 16 pixels lie on one output row; each chunk is interpolated from the four
      // source pixels (L1/L2 hits: a source pixel feeds ~4 outputs) and rounded to T
      const int r = (int)(p - (long)b * a.HW);
      const int oy = r / (2 * a.up.W), ox = r - oy * (2 * a.up.W);
      const Up2xTap tp = up2x_tap(a.up, oy, ox);
      const T* src = a.hin + (long)b * a.up.H * a.up.W * a.ldh;
      // up2x_mix's arithmetic, two channels per packed-fp32 instruction (as aad_v5_kernel's hload)
      const f32x2 ly0 = {tp.ly0, tp.ly0}, ly1 = {tp.ly1, tp.ly1}, lx0 = {tp.lx0, tp.lx0}, lx1 = {tp.lx1, tp.lx1};
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const T* xc = src + (j >> 1) * 64 + (j & 1) * 32 + lq * 8;
        const u32x4 r00 = *reinterpret_cast<const u32x4*>(xc + (long)tp.o00 * a.ldh);
        const u32x4 r01 = *reinterpret_cast<const u32x4*>(xc + (long)tp.o01 * a.ldh);
        const u32x4 r10 = *reinterpret_cast<const u32x4*>(xc + (long)tp.o10 * a.ldh);
        const u32x4 r11 = *reinterpret_cast<const u32x4*>(xc + (long)tp.o11 * a.ldh);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 top = fma2(lx0, unpack2<T>(r00[k]), lx1 * unpack2<T>(r01[k]));
          const f32x2 bot = fma2(lx0, unpack2<T>(r10[k]), lx1 * unpack2<T>(r11[k]));
          const f32x2 v = fma2(ly0, top, ly1 * bot);
          hc[j][k] = pack2<T>(v.x, v.y);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NH; ++j)   // chunk j = (ct, s): channels ct*64 + 32s + 8lq .. +7
        hc[j] = *reinterpret_cast<const u32x4*>(a.hin + p * a.ldh + (j >> 1) * 64 + (j & 1) * 32 + lq * 8);
    }

    // mask logits: per layer NH MFMAs over the h fragments (chunk j is the B operand of K step j: lane (lr, lq)
    // holds channels 32 j + 8 lq .. +7 of pixel lr); lane (lr, lq) gets rows 4 lq .. +3 = (hi, mid, lo, hi) . h
    float Mk[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      f32x4 mac = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        v8_t<T> bfr;
        __builtin_memcpy(&bfr, &hc[j], 16);
        const v8_t<T> afr = *reinterpret_cast<const v8_t<T>*>(&s_mA[(l * 3 + mrow) * C + j * 32 + lq * 8]);
        mac = mfma16x16x32<T>(afr, bfr, mac);
      }
      Mk[l] = sigmoidf_ref((mac[0] + mac[1]) + mac[2] + bh[l]);
    }

#pragma unroll
    for (int l = 0; l < L; ++l) {
      asm volatile("" ::: "memory");   // one layer's accumulators live at a time
      v8_t<T> xf[2];
      const float om = 1.f - Mk[l];
      const f32x2 om2 = {om, om};
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const T* W = s_w + (l * CT + ct) * 128 * WLD;
        // half sh: row tiles {2sh, 2sh+1} (gamma) and {4+2sh, 5+2sh} (beta) = channels
        // ct*64 + 32sh + 8lq + e of this lane's pixel; one half's accumulators live at a time
        u32x4 owp[2];
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
          asm volatile("" ::: "memory");
          f32x4 acc[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rt = (i & 1) + 2 * sh + 4 * (i >> 1);
            acc[i] = *reinterpret_cast<const f32x4*>(&s_b[(l * CT + ct) * 128 + rt * 16 + lq * 4]);
          }
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            v8_t<T> bfrag;
            __builtin_memcpy(&bfrag, &zc[ks], 16);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int rt = (i & 1) + 2 * sh + 4 * (i >> 1);
              const v8_t<T> afrag = *reinterpret_cast<const v8_t<T>*>(&W[swca<CA>(rt * 16 + lr, ks * 32 + lq * 8)]);
              acc[i] = mfma16x16x32<T>(afrag, bfrag, acc[i]);
            }
          }
          const int j = ct * 2 + sh;
          const int c0 = ct * 64 + sh * 32 + lq * 8;
          u32x4 ow;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {   // channels c0 + 2kk, c0 + 2kk + 1
            const int c = c0 + 2 * kk;
            const f32x2 h2 = fma2(unpack2<T>(hc[j][kk]), *reinterpret_cast<const f32x2*>(&s_rs[c]),
                                  *reinterpret_cast<const f32x2*>(&s_nm[c]));
            const f32x2 gg = {acc[kk >> 1][(2 * kk) & 3], acc[kk >> 1][(2 * kk + 1) & 3]};
            const f32x2 be = {acc[2 + (kk >> 1)][(2 * kk) & 3], acc[2 + (kk >> 1)][(2 * kk + 1) & 3]};
            const f32x2 D = fma2(gg, h2, be);
            const f32x2 I = fma2(*reinterpret_cast<const f32x2*>(&s_gi[l * C + c]), h2,
                                 *reinterpret_cast<const f32x2*>(&s_bi[l * C + c]));
            const f32x2 v = fma2(om2, D, I);
            ow[kk] = relu ? relu_pack2<T>(v) : pack2<T>(v.x > 0.f ? v.x : v.x * a.slope, v.y > 0.f ? v.y : v.y * a.slope);
          }
          if (ZPM && ((ZPM >> l) & 1)) __builtin_memcpy(&xf[sh], &ow, 16);
          owp[sh] = ow;
        }
        if (!(ZPM && ((ZPM >> l) & 1))) {
          const long p0 = p - lr + (lr & 7);   // the tile's pixel lr & 7 (pixels are consecutive)
          store_rows16<T>(a.out[l] + ct * 64, p0 * a.ldo[l], (p0 + 8) * a.ldo[l], lr, lq, owp[0], owp[1]);
        }
      }
      if (ZPM && ((ZPM >> l) & 1))
        zp_store(s_wz + zp_slot<ZPM>(l) * kZpRows * ZLD, xf, reinterpret_cast<_Float16*>(a.out[l]) + b * zr_image(a.HW),
                 p - (long)b * a.HW, a.HW, lr, lq);
    }
  }
}

// C = 64: held to 4 waves per SIMD (<= 128 VGPRs) so two 512-thread workgroups share a CU;
// C = 128 keeps the compiler's allocation (forcing it spills)
template <typename T, int C, int CA, int L, bool UP, int ZPM = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8))) aad_v3_kernel(const AadV3ArgsT<T> a) {
  aad_v3_body<T, C, CA, L, UP, kWaves, ZPM>(a);
}
// one layer writing tap partials (AADBlk8's h path): held to 6 waves per SIMD (<= 80 VGPRs; the compiler's
// own allocation is 86, 5 waves), three 512-thread workgroups per CU for this streaming pass
template <typename T, int CA>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(6, 8))) aad_v3_zp1_kernel(const AadV3ArgsT<T> a) {
  aad_v3_body<T, 64, CA, 1, false, kWaves, 1>(a);
}
template <typename T, int C, int CA, int L, bool UP>
__global__ void __launch_bounds__(512) aad_v3_wide_kernel(const AadV3ArgsT<T> a) {
  aad_v3_body<T, C, CA, L, UP>(a);
}

// ---------------------------------------------------------------------------------------------
// v4: the C = 64 kernel with the next tile's inputs in flight while the current one computes.
//
// v3 issues a tile's loads and waits for them: PMC shows its waves parked on memory 57-67 % of the
// time (SQ_WAIT_ANY).  Here every wave keeps TWO 16-pixel tiles in flight: at the top of tile t it
// issues tile t+1's z_attr fragments (to registers) and its h_in pixels (LDS-DMA into a wave-private
// slot; for the through-upsample form the <= 10 source pixels of each of the two source rows), then
// computes tile t, so tile t+1's loads overlap tile t's arithmetic.  (They do not overlap tile t's
// stores: with loads and stores both outstanding the vmcnt counter is not in order, and the waitcnt
// pass waits for zero before the next slot read; peeling / unrolling the loop so every wait could be
// a partial count was measured and only added spills.)  The h_in slot is XOR-swizzled on the source side
// (chunk c of pixel p lands at chunk c ^ (p & 7)) so the 16 pixels a lane group reads hit 16 bank
// groups.
// The per-pixel arithmetic (bilinear mix, mask dot product, normalise / blend) runs two channels per
// packed-fp32 instruction (v_pk_fma_f32 etc., same per-element rounding as the scalar form), the
// ReLU that follows every AADLayer is a template flag (one v_max instead of compare + select), and
// the wave index goes through readfirstlane so every per-tile address is scalar arithmetic: measured
// (B = 64, 256x256, L = 2) 474 -> 453 us with VALU instructions per tile 728 -> 492 (PMC: the round-2
// kernel issued 661 VALU per 16-pixel tile, ~60 % of its SIMD cycles).
// ---------------------------------------------------------------------------------------------
template <int CA, int L, bool UP>
struct V4Cfg {
  static constexpr int C = 64, KS = CA / 32, NH = 2;
  static constexpr int SPX = UP ? 10 : 16;        // h pixels per row held in a slot
  static constexpr int ROWS = UP ? 2 : 1;
  static constexpr int SLOT_B = ROWS * SPX * 128;  // bytes per wave per slot
};

template <int CA, int L, bool UP, bool RELU, int ZPM = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8))) aad_v4_kernel(const AadV3ArgsT<bf16> a) {
  typedef bf16 T;   // (bf16 only: v5 replaces it as the block-input kernel, and is the one fp16 runs)
  static_assert(UP, "v4 is the through-upsample form (v3's register loads win without the upsample)");
  using K = V4Cfg<CA, L, UP>;
  constexpr int C = 64, KS = K::KS, SPX = K::SPX, SLOT_B = K::SLOT_B;
  // weight rows: with tap partials unpadded + XOR-swizzled (swca; keeps the kernel within 80 KB of LDS, two
  // workgroups per CU, next to the projection rows), without them padded by 8 elements (the swizzle's address
  // arithmetic spills the ZPM = 0 form at 128 VGPRs)
  constexpr int WLD = ZPM ? CA : CA + 8;
  auto widx = [](int row, int k) { return ZPM ? swca<CA>(row, k) : row * (CA + 8) + k; };
  __shared__ __attribute__((aligned(16))) T s_w[L * 128 * WLD];
  __shared__ __attribute__((aligned(16))) float s_b[L * 128];
  __shared__ __attribute__((aligned(16))) float s_rs[C];
  __shared__ __attribute__((aligned(16))) float s_nm[C];
  __shared__ __attribute__((aligned(16))) float s_cf[L * C];
  __shared__ float s_k[L];
  __shared__ __attribute__((aligned(16))) float s_gi[L * C];
  __shared__ __attribute__((aligned(16))) float s_bi[L * C];
  __shared__ __attribute__((aligned(1024))) unsigned char s_hA[kWaves * SLOT_B];
  __shared__ __attribute__((aligned(1024))) unsigned char s_hB[kWaves * SLOT_B];
  __shared__ __attribute__((aligned(16))) T s_wz[ZPM ? zp_nlayers<ZPM>() * kZpRows * ZLD : 8];

  // wid through readfirstlane: tile indices and everything derived from them are wave-uniform (SGPRs),
  // so the per-tile address arithmetic runs on the scalar unit and the VALU keeps only lane offsets
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, lr = lane & 15,
            lq = lane >> 4;
  if (a.tclk && tid == 0) a.tclk[blockIdx.x] = (unsigned long long)wall_clock64();
  const long p_begin = (long)blockIdx.x * a.PPW;
  const int b = (int)(p_begin / a.HW);
  zp_stage_weights<T, L, ZPM, kWaves * 64>(a, s_wz, tid);

  for (int l = 0; l < L; ++l) {
    for (int idx = tid; idx < 128 * (CA / 8); idx += kWaves * 64) {
      const int row = idx / (CA / 8), kc = idx - row * (CA / 8);
      *reinterpret_cast<u32x4*>(&s_w[widx(l * 128 + row, kc * 8)]) =
          *reinterpret_cast<const u32x4*>(a.w3[l] + (long)row * CA + kc * 8);
    }
    for (int idx = tid; idx < 128; idx += kWaves * 64) s_b[l * 128 + idx] = a.b3[l][idx];
    for (int c = tid; c < C; c += kWaves * 64) {
      const float rs = a.stat[((long)b * C + c) * 2 + 1];
      s_cf[l * C + c] = a.wh[l][c] * rs;
      s_gi[l * C + c] = a.idgb[l][(long)b * a.id_ld + c];
      s_bi[l * C + c] = a.idgb[l][(long)b * a.id_ld + C + c];
    }
  }
  for (int c = tid; c < C; c += kWaves * 64) {
    const float mu = a.stat[((long)b * C + c) * 2], rs = a.stat[((long)b * C + c) * 2 + 1];
    s_rs[c] = rs;
    s_nm[c] = -mu * rs;
  }
  __syncthreads();
  if (wid < L) {
    float k = 0.f;
    for (int c = lane; c < C; c += 64) k = fmaf(a.wh[wid][c], s_nm[c], k);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) k += __shfl_xor(k, o, 64);
    if (lane == 0) s_k[wid] = k;
  }
  __syncthreads();
  float bh[L];
#pragma unroll
  for (int l = 0; l < L; ++l) bh[l] = a.bh[l][0] + s_k[l];

  const T* src = UP ? a.hin + (long)b * a.up.H * a.up.W * a.ldh : nullptr;
  const int ntiles = a.PPW / 16;
  // this wave's tiles: t = wid + 8 i, i = 0 .. nw-1 (nw even: PPW is a multiple of 256)
  const int nw = ntiles / kWaves;

  const int r_begin = (int)(p_begin - (long)b * a.HW);   // first output pixel of the block in its sample
  const int OW = 2 * a.up.W;
  // lane parts of the addresses (the tile parts are scalar)
  const int z_lane = lr * a.lda + lq * 8;

  // z fragments of tile t (registers) + its h_in pixels (DMA into slot `slot` of this wave)
  auto issue = [&](int t, u32x4 (&zc)[KS], unsigned char* slot) {
    const T* zt = a.za + (p_begin + t * 16) * a.lda;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) zc[ks] = *reinterpret_cast<const u32x4*>(zt + z_lane + ks * 32);
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned char* dst = slot + wid * SLOT_B;
    const int r = r_begin + t * 16;                               // first output pixel of the tile
    const int oy = r / OW, ox0 = r - oy * OW;
    float ry = a.up.sh * (float)oy, rx = a.up.sw * (float)ox0;
    asm volatile("" : "+v"(ry), "+v"(rx));
    const int y0 = __builtin_amdgcn_readfirstlane((int)ry), x_lo = __builtin_amdgcn_readfirstlane((int)rx);
    const int y1 = y0 + (y0 < a.up.H - 1 ? 1 : 0);
#pragma unroll
    for (int row = 0; row < 2; ++row) {
      const T* srow = src + (long)(row ? y1 : y0) * a.up.W * a.ldh;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pl = k * 8 + (lane >> 3), cl = lane & 7;     // LDS pixel / chunk this lane fills
        if (k == 1 && lane >= 16) continue;                    // 10 pixels per row
        const int sx = min(x_lo + pl, a.up.W - 1);
        __builtin_amdgcn_global_load_lds(srow + sx * a.ldh + ((cl ^ (pl & 7)) * 8), dst + row * SPX * 128 + k * 1024,
                                         16, 0, 0);
      }
    }
#endif
  };

  // phase 1: tile t's h_in chunks out of its LDS slot (through the bilinear x2 when UP)
  auto hload = [&](int t, const unsigned char* slot, u32x4 (&hc)[2]) {
    const unsigned char* hs = slot + wid * SLOT_B;
    if constexpr (UP) {
      const int r = r_begin + t * 16;                             // the tile's output row and first column
      const int oy = r / OW, ox0 = r - oy * OW;
      float rx0 = a.up.sw * (float)ox0;
      asm volatile("" : "+v"(rx0));
      const int x_lo = __builtin_amdgcn_readfirstlane((int)rx0);
      // up2x_tap's arithmetic for this lane's output pixel (oy, ox0 + lr); the slot holds rows y0, y1
      float ry = a.up.sh * (float)oy, rx = a.up.sw * (float)(ox0 + lr);
      asm volatile("" : "+v"(ry), "+v"(rx));
      const int y0 = (int)ry, x0 = (int)rx;
      const int x1 = x0 + (x0 < a.up.W - 1 ? 1 : 0);
      const float fly1 = ry - (float)y0, flx1 = rx - (float)x0;
      const int c0 = x0 - x_lo, c1 = x1 - x_lo;
      const f32x2 ly0 = {1.f - fly1, 1.f - fly1}, ly1 = {fly1, fly1}, lx0 = {1.f - flx1, 1.f - flx1}, lx1 = {flx1, flx1};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ch = j * 4 + lq;                    // 16-byte chunk of channels 8ch .. 8ch+7
        auto ld = [&](int row, int col) {
          return *reinterpret_cast<const u32x4*>(hs + row * SPX * 128 + col * 128 + ((ch ^ (col & 7)) * 16));
        };
        // up2x_mix's arithmetic, two channels per packed-fp32 instruction
        const u32x4 r00 = ld(0, c0), r01 = ld(0, c1), r10 = ld(1, c0), r11 = ld(1, c1);
        T* hv = reinterpret_cast<T*>(&hc[j]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 top = fma2(lx0, unpack2<T>(r00[k]), lx1 * unpack2<T>(r01[k]));
          const f32x2 bot = fma2(lx0, unpack2<T>(r10[k]), lx1 * unpack2<T>(r11[k]));
          const f32x2 v = fma2(ly0, top, ly1 * bot);
          hv[2 * k] = (T)v.x;
          hv[2 * k + 1] = (T)v.y;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ch = j * 4 + lq;
        hc[j] = *reinterpret_cast<const u32x4*>(hs + lr * 128 + ((ch ^ (lr & 7)) * 16));
      }
    }
  };
  // phase 2: mask, gamma/beta MFMAs, blend and the stores of tile t
  auto compute = [&](int t, const u32x4 (&zc)[KS], const u32x4 (&hc)[2]) {
    const long p0 = p_begin + t * 16;
    f32x2 ms[L];
#pragma unroll
    for (int l = 0; l < L; ++l) ms[l] = f32x2{0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c0 = j * 32 + lq * 8;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 h2 = unpack2<T>(hc[j][k]);
#pragma unroll
        for (int l = 0; l < L; ++l) ms[l] = fma2(*reinterpret_cast<const f32x2*>(&s_cf[l * C + c0 + 2 * k]), h2, ms[l]);
      }
    }
    float Mk[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float sm = ms[l].x + ms[l].y;
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      Mk[l] = sigmoid_fast(sm + bh[l]);
    }
#pragma unroll
    for (int l = 0; l < L; ++l) {
      asm volatile("" ::: "memory");
      const T* W = s_w + l * 128 * WLD;
      f32x4 zacc[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int sh = 0; sh < 2; ++sh) {
        asm volatile("" ::: "memory");
        f32x4 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rt = (i & 1) + 2 * sh + 4 * (i >> 1);
          acc[i] = *reinterpret_cast<const f32x4*>(&s_b[l * 128 + rt * 16 + lq * 4]);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          v8_t<T> bfrag;
          __builtin_memcpy(&bfrag, &zc[ks], 16);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rt = (i & 1) + 2 * sh + 4 * (i >> 1);
            const v8_t<T> afrag = *reinterpret_cast<const v8_t<T>*>(&W[widx(rt * 16 + lr, ks * 32 + lq * 8)]);
            acc[i] = mfma16x16x32<T>(afrag, bfrag, acc[i]);
          }
        }
        const int c0 = sh * 32 + lq * 8;
        const f32x2 M2 = {Mk[l], Mk[l]};
        float o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // channels c0 + 2k, c0 + 2k + 1
          const int c = c0 + 2 * k;
          const f32x2 hh = fma2(unpack2<T>(hc[sh][k]), *reinterpret_cast<const f32x2*>(&s_rs[c]),
                                *reinterpret_cast<const f32x2*>(&s_nm[c]));
          const f32x2 g = {acc[k >> 1][(2 * k) & 3], acc[k >> 1][(2 * k + 1) & 3]};
          const f32x2 be = {acc[2 + (k >> 1)][(2 * k) & 3], acc[2 + (k >> 1)][(2 * k + 1) & 3]};
          const f32x2 A = fma2(g, hh, be);
          const f32x2 I = fma2(*reinterpret_cast<const f32x2*>(&s_gi[l * C + c]), hh,
                               *reinterpret_cast<const f32x2*>(&s_bi[l * C + c]));
          const f32x2 v = fma2(M2, I - A, A);
          if constexpr (RELU) {
            o[2 * k] = fmaxf(v.x, 0.f);
            o[2 * k + 1] = fmaxf(v.y, 0.f);
          } else {
            o[2 * k] = v.x > 0.f ? v.x : v.x * a.slope;
            o[2 * k + 1] = v.y > 0.f ? v.y : v.y * a.slope;
          }
        }
        if (ZPM && ((ZPM >> l) & 1)) {
          v8_t<T> xf;
#pragma unroll
          for (int e = 0; e < 8; ++e) xf[e] = (T)o[e];
          zp_mfma_half(s_wz + zp_slot<ZPM>(l) * kZpRows * ZLD, xf, sh, zacc, lr, lq);
        } else {
          store16_f(a.out[l] + p0 * a.ldo[l] + (lr * a.ldo[l] + c0), o);
        }
      }
      if (ZPM && ((ZPM >> l) & 1))
        zp_store_acc(zacc, reinterpret_cast<_Float16*>(a.out[l]) + b * zr_image(a.HW), p0 + lr - (long)b * a.HW, a.HW,
                     lr, lq);
    }
  };

  // loop: read tile t's h_in out of its slot (the wait the compiler puts before that read covers
  // tile t's DMA and z loads), THEN issue tile t+1 into the other slot, then compute tile t while
  // those loads are in flight
  u32x4 zc[KS], zn[KS];
  issue(wid, zc, s_hA);
  for (int i = 0; i < nw; ++i) {
    const int t = wid + i * kWaves;
    unsigned char* cur = (i & 1) ? s_hB : s_hA;
    unsigned char* nxt = (i & 1) ? s_hA : s_hB;
    asm volatile("" ::: "memory");
    u32x4 hc[2];
    hload(t, cur, hc);
    asm volatile("" ::: "memory");
    if (i + 1 < nw) issue(t + kWaves, zn, nxt);
    asm volatile("" ::: "memory");
    compute(t, zc, hc);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) zc[ks] = zn[ks];
  }
  if (a.tclk && lane == 0) a.tclk[gridDim.x + blockIdx.x * kWaves + wid] = (unsigned long long)wall_clock64();
}

// ---------------------------------------------------------------------------------------------
// v5: v4 with each wave tile = 2 output rows x 8 columns that read the SAME two source rows.
//
// In v4 a tile is 16 pixels of one output row: it DMAs 10 source pixels of each of its 2 source rows,
// and every source row is fetched again for each of the ~4 output rows that sample it (the h_in source
// came from HBM ~3.6x per launch: PMC 1.025 GB read against 0.671 GB minimum).  With align_corners and
// an exact x2 scale, output rows 2k-1 and 2k sample the same source rows (k-1, k) for k = 1 .. H-1, and
// rows 0 and 2H-1 sample source rows 0 and H-1 alone (interpolation weight exactly 0 on the other row;
// the host checks both facts in fp32, v5_pairing_ok).  So the image's output rows form H "row tiles":
// q = 0 -> rows {0, 2H-1}, q >= 1 -> rows {2q-1, 2q}, each reading 2 source rows.  A wave tile is one row
// tile x 8 columns = 16 pixels (lanes lr 0-7 the first row, 8-15 the second: the MFMA's 16-pixel B
// operand): 2 rows x 6 source pixels = 1.5 KB of DMA per 16 pixels instead of 2.5 KB.  A workgroup
// (1024 pixels) covers RT = 64 / (OW / 8) row tiles; its waves walk them side by side (wave w: row tile
// w % RT, columns 8 (w / RT + (8 / RT) i)), so the source row two neighbouring row tiles share is fetched
// by both at nearly the same time (one L2 miss), and blocks go to XCDs in contiguous runs
// (xcd_remap) so the row a block shares with the next is read on the same L2.
// ---------------------------------------------------------------------------------------------
// Memory ops the compiler does not see (v5 with ASMW): the DMA of the next tile's h_in source pixels and
// z_attr fragments into LDS slots, and the reads of those slots.  Then the only vector-memory ops the
// compiler tracks in the loop are the tile's stores, so it inserts no s_waitcnt vmcnt(0) after them (with
// loads and stores both pending it waits for zero, exposing every tile's store latency); the kernel waits
// itself with a counted vmcnt(2 L) before reading tile i's slots: gfx9 retires vector-memory ops in issue
// order, so that leaves only tile i-1's 2 L stores in flight, overlapping tile i's arithmetic.  (An asm load
// into registers is not safe: the compiler treats its result as ready at the asm and may copy it early.)
GHOST_DEV void asm_dma16(const void* gp, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(gp), "s"(lds_base) : "memory", "m0");
}
// the same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset (the saddr form): no
// 64-bit address arithmetic per lane
GHOST_DEV void asm_dma16_s(const void* base, uint32_t voff, uint32_t lds_base) {
  // the base through readfirstlane so that the "s" operand is an SGPR pair (a value the compiler cannot prove
  // uniform would be handed over in VGPRs)
  const uint64_t bp = (uint64_t)(uintptr_t)base;
  const uint64_t sbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(bp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bp);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(voff), "s"(sbase), "s"(lds_base)
               : "memory", "m0");
}
GHOST_DEV u32x4 asm_lds16(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
// LDS byte offset of a __shared__ object (the low 32 bits of its generic address: the shared aperture base
// has zero low bits)
GHOST_DEV uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)p; }

// C = 64 (AADBlk8, the roofline kernel): 8 waves, two workgroups per CU, double-buffered source slots.
// C = 128 (AADBlk7's block-input pair, aad_v5_wide_kernel): 16 waves in ONE workgroup per CU (the 74 KB of
// weight rows staged once per CU instead of twice; 4 waves per SIMD at <= 128 VGPRs), single-buffered slots
// (a wave reads tile i's slot into registers before it DMAs tile i+1 into it), and hh recomputed per layer
// (holding both 64-channel tiles' hh would cost 32 VGPRs)
template <typename T, int CA, int L, bool RELU, int ZPM, bool ASMW, int C>
GHOST_DEV void aad_v5_body(const AadV3ArgsT<T>& a) {
  static_assert(C == 64 || (C == 128 && ZPM == 0 && !ASMW), "");
  constexpr int CT = C / 64, NH = 2 * CT;         // 64-channel tiles; 16-byte h chunks per lane
  constexpr int NW = C == 64 ? kWaves : 16;       // waves per workgroup
  constexpr int NBUF = C == 64 ? 2 : 1;           // source slot buffers per wave
  constexpr int IPWMAX = C == 64 ? 2 : 4;         // work items per workgroup (host: v5_takes)
  constexpr int CPXH = C / 8;                     // 16-byte chunks per source pixel
  constexpr int KS = CA / 32, SPX = 6, SLOT_B = 2 * SPX * C * 2;
  constexpr int WLD = CA;
  auto widx = [](int row, int k) { return swca<CA>(row, k); };
  __shared__ __attribute__((aligned(16))) T s_w[L * CT * 128 * WLD];
  __shared__ __attribute__((aligned(16))) float s_b[L * CT * 128];
  __shared__ __attribute__((aligned(16))) float s_rs[C];
  __shared__ __attribute__((aligned(16))) float s_nm[C];
  // mask rows (round 4): the logits sum_c (wh_c rs_c) h_c of a layer as MFMAs over the tile's h fragments.  Layer
  // l's rows 3l .. 3l+2 hold cf_l = wh_l rs split into three 16-bit parts: hi = T(cf), mid = T(cf - hi), lo =
  // T(cf - hi - mid) (each residual exact in fp32): the sum carries cf to ~2^-26, as the fp32 FMA chain did.  Two
  // parts (~2^-17) were not enough: sum_c cf_c h_c cancels against the mean term k, and the error showed in the
  // uint8 output.  A row lr reads part lr & 3 of its layer (row 3 repeats part 0), so every lane group gets all
  // three sums;
  // every product of two 16-bit values is exact in the fp32 accumulation.
  __shared__ __attribute__((aligned(16))) T s_mA[L * 3 * C];
  __shared__ float s_k[L];
  __shared__ __attribute__((aligned(16))) int s_rt[NW * IPWMAX * 8];  // per wave its <= IPWMAX row tiles (RowT)
  __shared__ __attribute__((aligned(16))) float s_gi[L * C];
  __shared__ __attribute__((aligned(16))) float s_bi[L * C];
  __shared__ __attribute__((aligned(1024))) unsigned char s_hA[NW * SLOT_B];
  __shared__ __attribute__((aligned(1024))) unsigned char s_hB[NBUF == 2 ? NW * SLOT_B : 16];
  __shared__ __attribute__((aligned(16))) T s_wz[ZPM ? zp_nlayers<ZPM>() * kZpRows * ZLD : 8];
  // ASMW: each wave's z_attr tile (16 pixels x CA channels), single-buffered: read at the top of tile i, then
  // refilled with tile i+1's by DMA
  constexpr int ZSLOT_B = 16 * CA * 2;
  __shared__ __attribute__((aligned(1024))) unsigned char s_z[ASMW ? NW * ZSLOT_B : 16];

  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, lr = lane & 15,
            lq = lane >> 4;
  if (C == 64 && a.tclk && tid == 0) a.tclk[blockIdx.x] = (unsigned long long)wall_clock64();
#ifdef GHOST_TUNING
  // A/B of the round-4 epilogue (tuning build only): bit 0 mask logits by MFMA (else the per-lane FMA chain),
  // bit 1 the identity path folded into the GEMM bias (else A + M (I - A))
  const bool mm = (a.v5_flags & 1) != 0, di = (a.v5_flags & 2) != 0;
  __shared__ __attribute__((aligned(16))) float s_cf[L * C];
#else
  constexpr bool mm = true, di = true;
#endif
  const int H = a.up.H, W = a.up.W, OW = 2 * W;
  const int NCT = OW / 8;                      // 8-column tiles per row tile
  const int RT = 64 / NCT;                     // row tiles per work item (host: 1, 2, 4 or 8; NW % RT == 0)
  const int wpi = H / RT;                      // 1024-pixel work items per image
  const int IPW = a.v5_ipw;                    // work items per workgroup (consecutive, one image: wpi % IPW == 0)
  const int wi = a.v5_xcd ? xcd_remap((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int b = wi * IPW / wpi, g0 = wi * IPW - b * wpi;
  zp_stage_weights<T, L, ZPM, NW * 64>(a, s_wz, tid);

  for (int l = 0; l < L; ++l) {
    for (int idx = tid; idx < CT * 128 * (CA / 8); idx += NW * 64) {
      const int row = idx / (CA / 8), kc = idx - row * (CA / 8);
      *reinterpret_cast<u32x4*>(&s_w[widx(l * CT * 128 + row, kc * 8)]) =
          *reinterpret_cast<const u32x4*>(a.w3[l] + (long)row * CA + kc * 8);
    }
    // the GEMM bias with the identity path folded in (round 4): row rho (pack_aad_v3: i = rho >> 4 row tile,
    // gamma for i < 4, channel 32 ((i >> 1) & 1) + 8 ((rho >> 2) & 3) + 4 (i & 1) + (rho & 3)) starts from
    // b3 - gi (gamma) or b3 - bi (beta), so the accumulators are D = (gamma - gi, beta - bi) and
    // out = A + M (I - A) = I + (1 - M) (D_gamma hh + D_beta)
    // (C = 128: tile ct's rows ct * 128 + rho, channels ct * 64 + the same)
    for (int idx = tid; idx < CT * 128; idx += NW * 64) {
      const int ct = idx >> 7, rho = idx & 127, i = rho >> 4;
      const int c = ct * 64 + 32 * ((i >> 1) & 1) + 8 * ((rho >> 2) & 3) + 4 * (i & 1) + (rho & 3);
      s_b[l * CT * 128 + idx] = a.b3[l][idx] - (di ? a.idgb[l][(long)b * a.id_ld + (i < 4 ? c : C + c)] : 0.f);
    }
    for (int c = tid; c < C; c += NW * 64) {
      s_gi[l * C + c] = a.idgb[l][(long)b * a.id_ld + c];
      s_bi[l * C + c] = a.idgb[l][(long)b * a.id_ld + C + c];
#ifdef GHOST_TUNING
      s_cf[l * C + c] = a.wh[l][c] * a.stat[((long)b * C + c) * 2 + 1];
#endif
    }
  }
  for (int idx = tid; idx < L * C; idx += NW * 64) {
    const int l = idx / C, c = idx - l * C;
    const float cf = a.wh[l][c] * a.stat[((long)b * C + c) * 2 + 1];
    const T hi = (T)cf;
    const float r1 = cf - (float)hi;
    const T mid = (T)r1;
    s_mA[(l * 3) * C + c] = hi;
    s_mA[(l * 3 + 1) * C + c] = mid;
    s_mA[(l * 3 + 2) * C + c] = (T)(r1 - (float)mid);
  }
  for (int c = tid; c < C; c += NW * 64) {
    const float mu = a.stat[((long)b * C + c) * 2], rs = a.stat[((long)b * C + c) * 2 + 1];
    s_rs[c] = rs;
    s_nm[c] = -mu * rs;
  }
  __syncthreads();
  if (wid < L) {
    float k = 0.f;
    for (int c = lane; c < C; c += 64) k = fmaf(a.wh[wid][c], s_nm[c], k);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) k += __shfl_xor(k, o, 64);
    if (lane == 0) s_k[wid] = k;
  }
  __syncthreads();
  float bh[L];
#pragma unroll
  for (int l = 0; l < L; ++l) bh[l] = a.bh[l][0] + s_k[l];

  const T* src = a.hin + (long)b * H * W * a.ldh;
  const long pimg = (long)b * a.HW;
  // per-sample bases (wave-uniform, 64-bit once): every per-tile address below is a 32-bit offset inside the
  // sample (HW * ld < 2^31), so the loop issues no 64-bit multiplies
  const T* __restrict__ za_b = a.za + pimg * a.lda;

  const int ri = lr >> 3, col = lr & 7;        // this lane's pixel: row ri of the row tile, column col
  const int mrow = (lr & 3) == 3 ? 0 : (lr & 3);   // mask A row: part lr & 3 of the split (row 3 repeats hi)
  constexpr int TPI = 64 / NW;                 // tiles per wave and work item (8 or 4)
  const int rtl = wid % RT;                    // this wave's row tile inside a work item
  const int nw = TPI * IPW;                    // tiles per wave
  const int ox_w = 8 * (wid / RT), ox_step = 8 * (NW / RT);   // wave's first column, column step between its tiles
  // row tile of the wave's tile i (item i / 8): q = 0 -> output rows {0, 2H-1}, q >= 1 -> {2q-1, 2q}; its
  // source rows (scalar): sA = y0(oyA); sB = y1(oyA) for a pair, y0(oyB) for the edge tile; and this lane's
  // row: output row offset, y taps as slot rows (top / bottom) and weight
  // Every field is wave-uniform (SGPRs); a lane's own row (ri) selects between the A / B forms at use.
  struct RowT {
    int sA, sB;                // the two source rows in the slot (top slot row 0, bottom 1)
    int prowA, prowB;          // the row tile's two output rows (pixel offsets in the sample)
    float flyA, flyB;          // y weight of rows A / B
    int tbA, tbB;              // slot rows of (y0, y1) for rows A / B: bit 0 = top, bit 1 = bottom
  };
  auto row_tile = [&](int g) {   // g: the wave's work item (row tile (g0 + g) * RT + rtl)
    RowT r;
    const int q = (g0 + g) * RT + rtl;
    const int oyA = q == 0 ? 0 : 2 * q - 1, oyB = q == 0 ? 2 * H - 1 : 2 * q;
    float rA = a.up.sh * (float)oyA, rB = a.up.sh * (float)oyB;
    asm volatile("" : "+v"(rA), "+v"(rB));
    const int y0A = __builtin_amdgcn_readfirstlane((int)rA), y0B = __builtin_amdgcn_readfirstlane((int)rB);
    r.sA = y0A;
    r.sB = q == 0 ? y0B : y0A + (y0A < H - 1 ? 1 : 0);
    r.flyA = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rA - (float)y0A)));
    r.flyB = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rB - (float)y0B)));
    auto tb = [&](int y0) {
      const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
      const int top = y0 == r.sA ? 0 : 1;
      const int bot = y1 == r.sA ? 0 : (y1 == r.sB ? 1 : top);
      return top | (bot << 1);
    };
    r.tbA = tb(y0A);
    r.tbB = tb(y0B);
    r.prowA = oyA * OW;
    r.prowB = oyB * OW;
    return r;
  };
  // the wave's (at most IPWMAX, v5_takes) row tiles, computed once into LDS (8 words each) and read back per tile:
  // holding them in registers across the loop spills, recomputing them costs ~20 VALU per use
  // (row_tile's readfirstlane needs a wave-uniform argument: one call per row tile, lane 0 stores it)
  for (int g = 0; g < IPW; ++g) {
    const RowT r = row_tile(g);
    if (lane == 0) {
      int* d = s_rt + (wid * IPWMAX + g) * 8;
      d[0] = r.sA; d[1] = r.sB; d[2] = r.prowA; d[3] = r.prowB;
      d[4] = __float_as_int(r.flyA); d[5] = __float_as_int(r.flyB); d[6] = r.tbA; d[7] = r.tbB;
    }
  }
  // lane 0 wrote the records, every lane of the wave reads them in rt_of: order the LDS stores before those loads
  // explicitly (the wave-synchronous ordering is not a guarantee of the memory model)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  auto rt_of = [&](int i) -> RowT {
    const int* d = s_rt + (wid * IPWMAX + i / TPI) * 8;
    const int4 u0 = *reinterpret_cast<const int4*>(d), u1 = *reinterpret_cast<const int4*>(d + 4);
    RowT r;
    r.sA = __builtin_amdgcn_readfirstlane(u0.x); r.sB = __builtin_amdgcn_readfirstlane(u0.y);
    r.prowA = __builtin_amdgcn_readfirstlane(u0.z); r.prowB = __builtin_amdgcn_readfirstlane(u0.w);
    r.flyA = __int_as_float(__builtin_amdgcn_readfirstlane(u1.x));
    r.flyB = __int_as_float(__builtin_amdgcn_readfirstlane(u1.y));
    r.tbA = __builtin_amdgcn_readfirstlane(u1.z); r.tbB = __builtin_amdgcn_readfirstlane(u1.w);
    return r;
  };

  // z fragments of tile i (registers) + its 2 x 6 source pixels (DMA into slot `slot` of this wave)
  auto issue = [&](int i, u32x4 (&zc)[KS], unsigned char* slot) {
    const RowT rt = rt_of(i);
    const int ox0 = ox_w + ox_step * (i % TPI);
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (ASMW) {
      // z_attr of the tile's 16 pixels into this wave's z slot: piece = lane of instruction k holds pixel
      // px = (k * 64 + lane) / (CA / 8), 16-byte chunk position c, filled with source chunk c ^ (px & (CA/8 - 1))
      constexpr int CPX = CA / 8;                               // chunks per pixel
      const uint32_t zdst = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_off(s_z + wid * ZSLOT_B));
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int piece = k * 64 + lane, px = piece / CPX, c = piece % CPX;
        const int prx = px >> 3, pcx = px & 7;                  // pixel -> (row of the row tile, column)
        const int pp = (prx ? rt.prowB : rt.prowA) + ox0 + pcx;
        asm_dma16_s(za_b, (uint32_t)(pp * a.lda + ((c ^ (px & (CPX - 1))) * 8)) * 2u, zdst + k * 1024);
      }
    } else {
      const T* zt = za_b + (((ri ? rt.prowB : rt.prowA) + ox0 + col) * a.lda + lq * 8);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) zc[ks] = *reinterpret_cast<const u32x4*>(zt + ks * 32);
    }
    unsigned char* dst = slot + wid * SLOT_B;
    float rx = a.up.sw * (float)ox0;
    asm volatile("" : "+v"(rx));
    const int x_lo = __builtin_amdgcn_readfirstlane((int)rx);
    const int rowA = rt.sA * W, rowB = rt.sB * W;          // source row starts (pixels in the sample)
    constexpr int NPC = 2 * SPX * CPXH;                      // slot pieces: 12 pixels x CPXH chunks (96 / 192)
#pragma unroll
    for (int k = 0; k < (NPC + 63) / 64; ++k) {
      if (k * 64 + 64 > NPC && k * 64 + lane >= NPC) continue;
      const int piece = k * 64 + lane;
      const int qs = piece / CPXH, cl = piece % CPXH;       // slot pixel / chunk position this lane fills
      const int sr = qs >= SPX, px = qs - (sr ? SPX : 0);
      const int sx = min(x_lo + px, W - 1);
      const int off = ((sr ? rowB : rowA) + sx) * a.ldh + ((cl ^ (qs & (CPXH - 1))) * 8);
      if constexpr (ASMW)
        asm_dma16_s(src, (uint32_t)off * 2u, (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_off(dst + k * 1024)));
      else
        __builtin_amdgcn_global_load_lds(src + off, dst + k * 1024, 16, 0, 0);
    }
#endif
  };
  // tile i's h_in chunks out of its LDS slot through the bilinear x2
  auto hload = [&](int i, const unsigned char* slot, u32x4 (&hc)[NH], f32x2 (&hh)[8], int& p, int& pa, int& pb) {
    const unsigned char* hs = slot + wid * SLOT_B;
    const RowT rt = rt_of(i);
    const int ox0 = ox_w + ox_step * (i % TPI);
    pa = rt.prowA + ox0 + col;   // the lane's column in the tile's rows A and B
    pb = rt.prowB + ox0 + col;
    p = ri ? pb : pa;
    const int tb = ri ? rt.tbB : rt.tbA, top = tb & 1, bot = tb >> 1;
    const float fly1 = ri ? rt.flyB : rt.flyA;
    const f32x2 ly0 = {1.f - fly1, 1.f - fly1}, ly1 = {fly1, fly1};
    float rx0 = a.up.sw * (float)ox0;
    asm volatile("" : "+v"(rx0));
    const int x_lo = __builtin_amdgcn_readfirstlane((int)rx0);
    float rx = a.up.sw * (float)(ox0 + col);
    asm volatile("" : "+v"(rx));
    const int x0 = (int)rx;
    const int x1 = x0 + (x0 < W - 1 ? 1 : 0);
    const float flx1 = rx - (float)x0;
    const int q00 = top * SPX + x0 - x_lo, q01 = top * SPX + x1 - x_lo;
    const int q10 = bot * SPX + x0 - x_lo, q11 = bot * SPX + x1 - x_lo;
    const f32x2 lx0 = {1.f - flx1, 1.f - flx1}, lx1 = {flx1, flx1};
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      const int ch = j * 4 + lq;
      auto ld = [&](int qq) {
        if constexpr (ASMW) return asm_lds16(lds_off(hs) + qq * 128 + ((ch ^ (qq & 7)) * 16));
        else return *reinterpret_cast<const u32x4*>(hs + qq * (C * 2) + ((ch ^ (qq & (CPXH - 1))) * 16));
      };
      u32x4 r00 = ld(q00), r01 = ld(q01), r10 = ld(q10), r11 = ld(q11);
      if constexpr (ASMW) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r00), "+v"(r01), "+v"(r10), "+v"(r11));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 tp = fma2(lx0, unpack2<T>(r00[k]), lx1 * unpack2<T>(r01[k]));
        const f32x2 bt = fma2(lx0, unpack2<T>(r10[k]), lx1 * unpack2<T>(r11[k]));
        const f32x2 v = fma2(ly0, tp, ly1 * bt);
        hc[j][k] = pack2<T>(v.x, v.y);
      }
      // hh = (h - mu) rs of the stored (T-rounded) h, once per tile for both layers (C = 64)
      if constexpr (CT == 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = j * 32 + lq * 8 + 2 * k;
        hh[j * 4 + k] = fma2(unpack2<T>(hc[j][k]), *reinterpret_cast<const f32x2*>(&s_rs[c]),
                             *reinterpret_cast<const f32x2*>(&s_nm[c]));
      }
    }
  };
  auto compute = [&](const int p, const int pa, const int pb, const u32x4 (&zc)[KS], const u32x4 (&hc)[NH],
                     const f32x2 (&hh)[8]) {
    // mask logits: per layer one MFMA per 32-channel half over the h fragments (B operand: lane (lr, lq) holds
    // channels 32 j + 8 lq .. +7 of pixel lr, the z_attr layout); lane (lr, lq) gets rows 4 lq .. +3 =
    // (hi, mid, lo, hi) . h of pixel lr (row 3 repeats hi and is not used)
    float Mk[L];
    if (mm) {
#pragma unroll
      for (int l = 0; l < L; ++l) {
        f32x4 mac = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NH; ++j) {
          v8_t<T> bfr;
          __builtin_memcpy(&bfr, &hc[j], 16);
          const v8_t<T> afr = *reinterpret_cast<const v8_t<T>*>(&s_mA[(l * 3 + mrow) * C + j * 32 + lq * 8]);
          mac = mfma16x16x32<T>(afr, bfr, mac);
        }
        Mk[l] = sigmoid_fast((mac[0] + mac[1]) + mac[2] + bh[l]);
      }
    } else {
#ifdef GHOST_TUNING
      f32x2 ms[L];
#pragma unroll
      for (int l = 0; l < L; ++l) ms[l] = f32x2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 h2 = unpack2<T>(hc[j][k]);
#pragma unroll
          for (int l = 0; l < L; ++l)
            ms[l] = fma2(*reinterpret_cast<const f32x2*>(&s_cf[l * C + j * 32 + lq * 8 + 2 * k]), h2, ms[l]);
        }
#pragma unroll
      for (int l = 0; l < L; ++l) {
        float sm = ms[l].x + ms[l].y;
        sm += __shfl_xor(sm, 16, 64);
        sm += __shfl_xor(sm, 32, 64);
        Mk[l] = sigmoid_fast(sm + bh[l]);
      }
#endif
    }
    // layer l's 32 channels (ct, sh) = hs2 of the lane's pixel: the GEMM rows, the blend, the store (or the tap
    // partials); h2[k] = hh of channels c0 + 2k, c0 + 2k + 1
    auto layer_half = [&](const int l, const int hs2, const f32x2 (&h2)[4], f32x4 (&zacc)[3]) -> u32x4 {
      const int ct = hs2 >> 1, sh = hs2 & 1;
      const T* Wt = s_w + (l * CT + ct) * 128 * WLD;
      if constexpr (CT == 1) asm volatile("" ::: "memory");
      f32x4 acc[4];
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const int rt = (i4 & 1) + 2 * sh + 4 * (i4 >> 1);
        acc[i4] = *reinterpret_cast<const f32x4*>(&s_b[(l * CT + ct) * 128 + rt * 16 + lq * 4]);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        v8_t<T> bfrag;
        __builtin_memcpy(&bfrag, &zc[ks], 16);
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int rt = (i4 & 1) + 2 * sh + 4 * (i4 >> 1);
          const v8_t<T> afrag = *reinterpret_cast<const v8_t<T>*>(&Wt[widx(rt * 16 + lr, ks * 32 + lq * 8)]);
          acc[i4] = mfma16x16x32<T>(afrag, bfrag, acc[i4]);
        }
      }
      const int c0 = ct * 64 + sh * 32 + lq * 8;
      const float om = 1.f - Mk[l];
      const f32x2 om2 = {om, om};
      u32x4 ow;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + 2 * k;
        const f32x2 gg = {acc[k >> 1][(2 * k) & 3], acc[k >> 1][(2 * k + 1) & 3]};
        const f32x2 be = {acc[2 + (k >> 1)][(2 * k) & 3], acc[2 + (k >> 1)][(2 * k + 1) & 3]};
        const f32x2 D = fma2(gg, h2[k], be);
        const f32x2 I = fma2(*reinterpret_cast<const f32x2*>(&s_gi[l * C + c]), h2[k],
                             *reinterpret_cast<const f32x2*>(&s_bi[l * C + c]));
        f32x2 v;
        if (di) {
          v = fma2(om2, D, I);
        } else {   // (tuning build) the A + M (I - A) form on an unfolded bias: D is A here
          const f32x2 M2 = {Mk[l], Mk[l]};
          v = fma2(M2, I - D, D);
        }
        if constexpr (RELU) {
          ow[k] = relu_pack2<T>(v);
        } else {
          ow[k] = pack2<T>(v.x > 0.f ? v.x : v.x * a.slope, v.y > 0.f ? v.y : v.y * a.slope);
        }
      }
      if (ZPM && ((ZPM >> l) & 1)) {
        v8_t<T> xf;
        __builtin_memcpy(&xf, &ow, 16);
        zp_mfma_half(s_wz + zp_slot<ZPM>(l) * kZpRows * ZLD, xf, sh, zacc, lr, lq);
      }
      return ow;
    };
    // channel tile ct of layer l as whole 128-byte rows (store_rows16): row A's 8 pixels, then row B's
    auto store_rows = [&](const int l, const int ct, const u32x4& ow0, const u32x4& ow1) {
#ifdef GHOST_TUNING
      if (a.v5_flags & 4) return;   // (tuning build, bit 2) no output stores: what the stores cost
#endif
      store_rows16<T>(a.out[l] + pimg * a.ldo[l] + ct * 64, (long)pa * a.ldo[l], (long)pb * a.ldo[l], lr, lq, ow0, ow1);
    };
    if constexpr (CT == 1) {
      // layer-major: the tap partials of a layer accumulate over its two halves
#pragma unroll
      for (int l = 0; l < L; ++l) {
        asm volatile("" ::: "memory");
        f32x4 zacc[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        u32x4 ow[2];
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
          const f32x2 h2[4] = {hh[sh * 4], hh[sh * 4 + 1], hh[sh * 4 + 2], hh[sh * 4 + 3]};
          ow[sh] = layer_half(l, sh, h2, zacc);
        }
        if (ZPM && ((ZPM >> l) & 1)) {
#ifdef GHOST_TUNING
          if (a.v5_flags & 8) continue;   // (tuning build, bit 3) no tap-partial stores: what they cost
#endif
          zp_store_acc(zacc, reinterpret_cast<_Float16*>(a.out[l]) + b * zr_image(a.HW), p, a.HW, lr, lq);
        } else {
          store_rows(l, 0, ow[0], ow[1]);
        }
      }
    } else {
      // C = 128: channel-tile-major, both layers per 64-channel tile, so a tile's hh (16 registers) is computed
      // once for both layers
      f32x4 zacc[3];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        asm volatile("" ::: "memory");
        f32x2 h2[2][4];
#pragma unroll
        for (int sh = 0; sh < 2; ++sh)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = ct * 64 + sh * 32 + lq * 8 + 2 * k;
            h2[sh][k] = fma2(unpack2<T>(hc[2 * ct + sh][k]), *reinterpret_cast<const f32x2*>(&s_rs[c]),
                             *reinterpret_cast<const f32x2*>(&s_nm[c]));
          }
#pragma unroll
        for (int l = 0; l < L; ++l) {
          const u32x4 ow0 = layer_half(l, 2 * ct, h2[0], zacc);
          const u32x4 ow1 = layer_half(l, 2 * ct + 1, h2[1], zacc);
          store_rows(l, ct, ow0, ow1);
        }
      }
    }
  };

  u32x4 zc[KS], zn[KS];
  issue(0, zc, s_hA);
  if constexpr (ASMW) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < nw; ++i) {
      unsigned char* cur = (i & 1) ? s_hB : s_hA;
      unsigned char* nxt = (i & 1) ? s_hA : s_hB;
      // tile i's DMAs done; tile i-1's 2 L stores may still be in flight
      static_assert(L == 1 || L == 2, "");
      if constexpr (L == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      // z fragments of this lane's pixel lr, channels 32 ks + 8 lq .. +7, out of the z slot
      const uint32_t zs = lds_off(s_z + wid * ZSLOT_B);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        constexpr int CPX = CA / 8;
        const int c = ks * 4 + lq;
        zc[ks] = asm_lds16(zs + (lr * CPX + (c ^ (lr & (CPX - 1)))) * 16);
      }
      if constexpr (KS == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(zc[0]), "+v"(zc[1]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(zc[0]));
      u32x4 hc[NH];
      f32x2 hh[8];
      int p, pa, pb;
      hload(i, cur, hc, hh, p, pa, pb);
      asm volatile("" ::: "memory");
      if (i + 1 < nw) issue(i + 1, zn, nxt);
      asm volatile("" ::: "memory");
      compute(p, pa, pb, zc, hc, hh);
    }
  } else {
    for (int i = 0; i < nw; ++i) {
      unsigned char* cur = (NBUF == 2 && (i & 1)) ? s_hB : s_hA;
      unsigned char* nxt = (NBUF == 2 && !(i & 1)) ? s_hB : s_hA;
      asm volatile("" ::: "memory");
      u32x4 hc[NH];
      f32x2 hh[8];
      int p, pa, pb;
      hload(i, cur, hc, hh, p, pa, pb);
      // one slot buffer: this wave's reads of tile i's slot have returned before tile i+1's DMA refills it
      if constexpr (NBUF == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("" ::: "memory");
      if (i + 1 < nw) issue(i + 1, zn, nxt);
      asm volatile("" ::: "memory");
      compute(p, pa, pb, zc, hc, hh);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) zc[ks] = zn[ks];
    }
  }
  if (C == 64 && a.tclk && lane == 0) a.tclk[gridDim.x + blockIdx.x * kWaves + wid] = (unsigned long long)wall_clock64();
}

template <typename T, int CA, int L, bool RELU, int ZPM = 0, bool ASMW = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8))) aad_v5_kernel(const AadV3ArgsT<T> a) {
  aad_v5_body<T, CA, L, RELU, ZPM, ASMW, 64>(a);
}
template <typename T, int CA, int L, bool RELU>
__global__ void __launch_bounds__(1024) aad_v5_wide_kernel(const AadV3ArgsT<T> a) {
  aad_v5_body<T, CA, L, RELU, 0, false, 128>(a);
}

// v5's row pairing holds for this source height in fp32 (PyTorch's index arithmetic, as up2x_tap): output
// rows 2k-1, 2k share y0 = k-1 (k = 1 .. H-1); rows 0 and 2H-1 land exactly on source rows 0 and H-1
static bool v5_pairing_ok(const Up2xSrc& u) {
  auto y0f = [&](int oy, float* fr) {
    volatile float r = u.sh * (float)oy;   // one fp32 multiply, as the kernel (no contraction)
    const int y = (int)r;
    if (fr) *fr = r - (float)y;
    return y;
  };
  float f0, f1;
  if (y0f(0, &f0) != 0 || f0 != 0.f || y0f(2 * u.H - 1, &f1) != u.H - 1 || f1 != 0.f) return false;
  for (int k = 1; k < u.H; ++k)
    if (y0f(2 * k - 1, nullptr) != k - 1 || y0f(2 * k, nullptr) != k - 1) return false;
  return true;
}

// pixels per workgroup: one sample's block; C = 256 stages its weights once per 1024 pixels, and so may the
// C = 128 layers (128 x 128 stage: GHOST_V3_PPW128, A/B knob)
// B > 0: a small batch halves the C = 128 / 256 workgroups (down to 256 pixels, a multiple of the 8 waves' 16-pixel
// tiles in pairs) while the grid has fewer than 128 of them (B = 1, 128 x 128 block-input pair: 32 -> 64 workgroups)
static int v3_ppw(int HW, int C, long B = 0) {
  int ppw = (HW >= 65536 || C == 256) ? 1024 : 512;
  if (C == 128) {
    static const int p128 = GHOST_KNOB("GHOST_V3_PPW128", 512);
    if ((p128 == 1024 || p128 == 2048) && HW % p128 == 0) ppw = p128;
  }
  if (B > 0 && C != 64)
    while (ppw > 256 && B * HW / ppw < 128) ppw /= 2;
  return ppw;
}

// the v5 kernel's work items per workgroup if it takes this launch, else 0
static int v5_takes(const AadV3Desc& d, int zpm) {
  static const int use_v5 = GHOST_KNOB("GHOST_AAD_V5", 1);
  // two 1024-pixel work items per workgroup (one prologue — statistics tables, weight rows — per 2048 pixels):
  // measured B = 64 unet/2, same box: 384.8 -> 377.8 us one batch at a time, 11 084-11 172 -> 11 272 frames/s
  // with two in flight (profiles/r03_ab_v5.txt; XCD-contiguous order neutral, the compiler-opaque DMA 3 % faster)
  static const int ipw = GHOST_KNOB("GHOST_V5_IPW", 2);
  const bool up = d.up_H > 0;
  // OW / 8 column tiles must divide the 64 tiles of a 1024-pixel work item (OW in {64 .. 512}) and the
  // work items of an image must cover its H row tiles, IPW at a time
  const int nct = 2 * d.up_W / 8, rt = nct > 0 && 64 % nct == 0 ? 64 / nct : 0;
  if (!use_v5 || !up || d.ldh % 8 || d.up_W % 4 || rt < 1 || rt > 8 || d.up_H < 2 ||
      !v5_pairing_ok(up2x_src(d.up_H, d.up_W)))
    return 0;
  if (d.C == 128) {
    // aad_v5_wide_kernel (AADBlk7's block-input pair): one 16-wave workgroup per CU; four work items per
    // workgroup by default = one workgroup per CU for B = 64 at 128 x 128 (GHOST_V5W_IPW, A/B knob)
    // Only where the grid fills the GPU: it is one workgroup per CU, so a small batch (B = 1: 16 work items at
    // 128 x 128) would run on a few CUs — there the v3 kernel's 512-pixel workgroups spread wider.
    static const int use_w = GHOST_KNOB("GHOST_AAD_V5W", 1);
    static const int ipw_max = GHOST_KNOB("GHOST_V5W_IPW", 4);
    if (!use_w || zpm || d.Ca != 64 || d.HW % 1024 || d.up_H % rt) return 0;
    const long items = (long)d.B * d.HW / 1024;
    for (int ipw_w = 4; ipw_w >= 1; ipw_w >>= 1)
      if (ipw_w <= ipw_max && (d.up_H / rt) % ipw_w == 0 && items / ipw_w >= 256) return ipw_w;
    return 0;
  }
  if (d.C != 64 || v3_ppw(d.HW, d.C) != 1024 || ipw < 1 || d.up_H % rt || (d.up_H / rt) % ipw) return 0;
  if (!(d.Ca == 64 || d.Ca == 32) || (zpm && d.L != 2) || ipw > 2) return 0;   // the kernel holds <= 2 row tiles
  // one work item per workgroup where two would leave the grid under a round of workgroups (B = 1: 32 -> 64)
  return (long)d.B * d.HW / 1024 / ipw >= 256 ? ipw : 1;
}

int aad_v3_clock_words(const AadV3Desc& d) {
  long grid = (long)d.B * d.HW / v3_ppw(d.HW, d.C, d.B);
  int zpm = 0;
  for (int l = 0; l < d.L; ++l) zpm |= d.zw[l] ? 1 << l : 0;
  if (const int ipw = v5_takes(d, zpm)) grid = (long)d.B * d.HW / 1024 / ipw;
  return (int)(grid * (1 + kWaves));
}

bool aad_v3_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo) {
  if (!is16(dt)) return false;
  // C = 256 (the 64x64 stage): all four channel tiles' weight rows (139 KB at Ca = 128) resident, one
  // workgroup per CU; the mask is computed in-kernel from the pixel's 256 channels, so no separate
  // mask pass reads h_in (measured B = 64: the per-channel-tile aad_wide + mask pass took 92 + 25 us)
  static const int c256 = GHOST_KNOB("GHOST_AAD_V3_C256", 1);
  const bool shape = (C == 64 && (Ca == 64 || Ca == 32)) || (C == 128 && (Ca == 128 || Ca == 64 || Ca == 32)) ||
                     (c256 && C == 256 && (Ca == 128 || Ca == 64));
  if (!shape || lda % 8 || ldh % 8 || ldo % 8) return false;
  const int ppw = v3_ppw(HW, C, B);
  return HW % ppw == 0 && (long)B * HW / ppw >= 32;
}

template <typename T>
static int aad_v3_t(const AadV3Desc& d, hipStream_t s) {
  AadV3ArgsT<T> a{};
  a.za = (const T*)d.za; a.hin = (const T*)d.hin; a.stat = d.stat;
  for (int l = 0; l < d.L; ++l) {
    a.w3[l] = (const T*)d.w3[l]; a.b3[l] = d.b3[l]; a.wh[l] = d.wh[l]; a.bh[l] = d.bh[l];
    a.idgb[l] = d.idgb[l]; a.out[l] = (T*)d.out[l]; a.ldo[l] = d.ldo[l];
  }
  a.lda = d.lda; a.ldh = d.ldh; a.id_ld = d.id_ld; a.HW = d.HW; a.slope = d.slope;
  a.PPW = v3_ppw(d.HW, d.C, d.B);
  int zpm = 0;
  for (int l = 0; l < d.L; ++l)
    if (d.zw[l]) {
      zpm |= 1 << l;
      a.zw[l] = (const T*)d.zw[l];
    }
  a.zwld = d.zwld;
  if (zpm && (d.C != 64 || d.slope != 0.f || d.zwld % 8)) return -1;
  for (int l = 0; l < d.L; ++l)
    if (d.zw[l] && (uintptr_t)d.zw[l] % 16) return -1;
  const bool up = d.up_H > 0;
  if (up) {
    if (4 * d.up_H * d.up_W != d.HW || d.up_W * 2 < 16 || (d.C != 64 && d.C != 128)) return -1;
    a.up = up2x_src(d.up_H, d.up_W);
  }
  dim3 grid((unsigned)((long)d.B * d.HW / a.PPW));
  if (d.version_out) *d.version_out = 3;
  static const int use_v4 = GHOST_KNOB("GHOST_AAD_V4", 1);
  // v4 (prefetching) only for the through-upsample form: measured B = 64, 256x256 L = 2: 724 vs 734 us
  // with the upsample, 604 vs 550 us without it (there v3's register loads win)
  static const unsigned dyn_lds = GHOST_KNOB("GHOST_AAD_DYNLDS", 0u);
  a.tclk = d.tclk;
  a.v5_xcd = GHOST_KNOB("GHOST_V5_XCD", 1);
  a.v5_ipw = v5_takes(d, zpm);
  a.v5_flags = GHOST_KNOB("GHOST_V5_FLAGS", 3);
  static const int v5_asm = GHOST_KNOB("GHOST_V5_ASM", 1);
  if (a.v5_ipw && d.C == 128) {
    a.PPW = 1024;
    grid = dim3((unsigned)((long)d.B * d.HW / 1024 / a.v5_ipw));
#define GHOST_V5W(l)                                                                             \
    if (d.L == l) {                                                                              \
      if (d.slope == 0.f)                                                                        \
        hipLaunchKernelGGL((aad_v5_wide_kernel<T, 64, l, true>), grid, dim3(1024), 0, s, a);      \
      else                                                                                       \
        hipLaunchKernelGGL((aad_v5_wide_kernel<T, 64, l, false>), grid, dim3(1024), 0, s, a);     \
      if (d.version_out) *d.version_out = 5;                                                     \
      return (int)hipGetLastError();                                                             \
    }
    GHOST_V5W(1) GHOST_V5W(2)
#undef GHOST_V5W
    return -1;
  }
  if (a.v5_ipw) {
    grid = dim3(grid.x / a.v5_ipw);
#define GHOST_V5(ca, l)                                                                          \
    if (d.Ca == ca && d.L == l && !zpm) {                                                        \
      if (d.slope == 0.f)                                                                        \
        hipLaunchKernelGGL((aad_v5_kernel<T, ca, l, true, 0, false>), grid, dim3(kWaves * 64), 0, s, a); \
      else                                                                                       \
        hipLaunchKernelGGL((aad_v5_kernel<T, ca, l, false, 0, false>), grid, dim3(kWaves * 64), 0, s, a); \
      if (d.version_out) *d.version_out = 5;                                                     \
      return (int)hipGetLastError();                                                             \
    }
    GHOST_V5(64, 1) GHOST_V5(64, 2) GHOST_V5(32, 1) GHOST_V5(32, 2)
#undef GHOST_V5
#define GHOST_V5Z(ca, zm)                                                                        \
    if (d.Ca == ca && d.L == 2 && zpm == zm) {                                                   \
      if (v5_asm)                                                                                \
        hipLaunchKernelGGL((aad_v5_kernel<T, ca, 2, true, zm, true>), grid, dim3(kWaves * 64), 0, s, a); \
      else                                                                                       \
        hipLaunchKernelGGL((aad_v5_kernel<T, ca, 2, true, zm, false>), grid, dim3(kWaves * 64), 0, s, a); \
      if (d.version_out) *d.version_out = 5;                                                     \
      return (int)hipGetLastError();                                                             \
    }
    GHOST_V5Z(64, 1) GHOST_V5Z(64, 2) GHOST_V5Z(64, 3) GHOST_V5Z(32, 1) GHOST_V5Z(32, 2) GHOST_V5Z(32, 3)
#undef GHOST_V5Z
    grid = dim3(grid.x * a.v5_ipw);   // (not reached: v5_takes admits only the shapes above)
    a.v5_ipw = 0;
  }
  if constexpr (std::is_same<T, bf16>::value) {
  if (use_v4 && up && d.C == 64 && a.PPW % 256 == 0 && d.ldh % 8 == 0) {
#define GHOST_V4(ca, l, u)                                                                       \
    if (d.Ca == ca && d.L == l && up == u && !zpm) {                                             \
      if (d.slope == 0.f)                                                                        \
        hipLaunchKernelGGL((aad_v4_kernel<ca, l, u, true>), grid, dim3(kWaves * 64), dyn_lds, s, a); \
      else                                                                                       \
        hipLaunchKernelGGL((aad_v4_kernel<ca, l, u, false>), grid, dim3(kWaves * 64), dyn_lds, s, a); \
      if (d.version_out) *d.version_out = 4;                                                     \
      return (int)hipGetLastError();                                                             \
    }
    GHOST_V4(64, 1, true) GHOST_V4(64, 2, true) GHOST_V4(32, 1, true) GHOST_V4(32, 2, true)
#undef GHOST_V4
    // AADBlk8's block-input pair with tap partials: layer 1 (last_add_block, nb >= 2) or both (nb = 1)
#define GHOST_V4Z(ca, zm)                                                                        \
    if (d.Ca == ca && d.L == 2 && zpm == zm) {                                                   \
      hipLaunchKernelGGL((aad_v4_kernel<ca, 2, true, true, zm>), grid, dim3(kWaves * 64), 0, s, a); \
      if (d.version_out) *d.version_out = 4;                                                     \
      return (int)hipGetLastError();                                                             \
    }
    GHOST_V4Z(64, 1) GHOST_V4Z(64, 2) GHOST_V4Z(64, 3) GHOST_V4Z(32, 1) GHOST_V4Z(32, 2) GHOST_V4Z(32, 3)
#undef GHOST_V4Z
  }
  }
  if (zpm) {   // the non-upsampled forms with tap partials (AADBlk8's last add_block; fuse_upsample off)
    if (d.C == 64 && d.L == 1 && !up && zpm == 1 && (d.Ca == 64 || d.Ca == 32)) {
      if (d.Ca == 64)
        hipLaunchKernelGGL((aad_v3_zp1_kernel<T, 64>), grid, dim3(kWaves * 64), 0, s, a);
      else
        hipLaunchKernelGGL((aad_v3_zp1_kernel<T, 32>), grid, dim3(kWaves * 64), 0, s, a);
      return (int)hipGetLastError();
    }
#define GHOST_V3Z(ca, l, zm)                                                                     \
    if (d.C == 64 && d.Ca == ca && d.L == l && !up && zpm == zm) {                               \
      hipLaunchKernelGGL((aad_v3_kernel<T, 64, ca, l, false, zm>), grid, dim3(kWaves * 64), 0, s, a); \
      return (int)hipGetLastError();                                                             \
    }
    GHOST_V3Z(64, 2, 1) GHOST_V3Z(32, 2, 1) GHOST_V3Z(64, 2, 2)
    GHOST_V3Z(32, 2, 2) GHOST_V3Z(64, 2, 3) GHOST_V3Z(32, 2, 3)
#undef GHOST_V3Z
    return -1;
  }
#define GHOST_V3(c, ca, l, u)                                                                   \
  if (d.C == c && d.Ca == ca && d.L == l && up == u) {                                          \
    hipLaunchKernelGGL((aad_v3_kernel<T, c, ca, l, u>), grid, dim3(kWaves * 64), 0, s, a);         \
    return (int)hipGetLastError();                                                              \
  }
#define GHOST_V3W(c, ca, l, u)                                                                  \
  if (d.C == c && d.Ca == ca && d.L == l && up == u) {                                          \
    hipLaunchKernelGGL((aad_v3_wide_kernel<T, c, ca, l, u>), grid, dim3(kWaves * 64), 0, s, a);    \
    return (int)hipGetLastError();                                                              \
  }
  GHOST_V3(64, 64, 1, false) GHOST_V3(64, 64, 2, false) GHOST_V3(64, 32, 1, false) GHOST_V3(64, 32, 2, false)
  // through-upsample forms: the block-input AADLayers of AADBlk8 (first add_block + last_add_block)
  GHOST_V3(64, 64, 2, true) GHOST_V3(64, 32, 2, true) GHOST_V3(64, 64, 1, true) GHOST_V3(64, 32, 1, true)
  GHOST_V3W(128, 128, 1, false) GHOST_V3W(128, 64, 1, false) GHOST_V3W(128, 32, 1, false)
  // the AADBlk7 block-input pair (C = 128, Ca = 64): one pass over h_in / z_attr for both layers, h_in
  // materialised or (UP) sampled from the 64x64 AADBlk6 output on the fly
  GHOST_V3W(128, 64, 2, false) GHOST_V3W(128, 64, 2, true)
  // AADBlk7's block-input AADLayers read upsample2x(AADBlk6 output) on the fly (C = 128)
  GHOST_V3W(128, 128, 1, true) GHOST_V3W(128, 64, 1, true) GHOST_V3W(128, 32, 1, true)
  GHOST_V3W(256, 128, 1, false) GHOST_V3W(256, 64, 1, false)
#undef GHOST_V3W
#undef GHOST_V3
  return -1;
}

int aad_v3(const AadV3Desc& d, hipStream_t s) {
  if (!aad_v3_supported(d.dt, d.B, d.HW, d.C, d.Ca, d.lda, d.ldh, d.ldo[0])) return -1;
  if (d.L == 2 && d.ldo[1] % 8) return -1;
  if (d.L < 1 || d.L > 2 || (d.L == 2 && d.C != 64 && !(d.C == 128 && d.Ca == 64))) return -1;
  return d.dt == GHOST_F16 ? aad_v3_t<_Float16>(d, s) : aad_v3_t<bf16>(d, s);
}

// ---------------------------------------------------------------------------------------------
// AADBlk8's output conv from the tap partials (tap_rows.h): output (y, x) is the sum over both producers'
// buffers (zh: the h path, zx: last_add_block's x') of the row sums R_dy of source row y + dy - 1, plus the
// segment-end terms at columns 8j - 1 / 8j; then tanh, and the BGR uint8 copy of faceshifter_run.py:20-21.
// A thread takes four pixels of an 8-row strip (tap_sum3x3_strip_kernel); consecutive blocks share an XCD.
// ---------------------------------------------------------------------------------------------
// four output pixels of one row from their sums: tanh, the 12 values, their BGR uint8 copy
// (faceshifter_run.py:20-21), as whole dwords where the caller's buffers allow them (vec)
template <typename T>
GHOST_DEV void tap_out4(const float (&s)[4][3], long q, T* __restrict__ y, int ldy, uint8_t* __restrict__ u8, int vec) {
  float v[12];
  uint32_t c[3] = {0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      v[k * 3 + o] = tanhf(s[k][o]);
      const float t = (v[k * 3 + o] * 0.5f + 0.5f) * 255.0f;   // faceshifter_run.py:20-21
      const int bi = k * 3 + (2 - o);                            // BGR
      c[bi >> 2] |= (uint32_t)(uint8_t)(int)t << ((bi & 3) * 8);
    }
  if (vec & 1) {   // ldy = 3, y 8-byte aligned: 12 contiguous values in three 8-byte stores
    typedef __attribute__((ext_vector_type(4))) T t4;
    t4* yp = reinterpret_cast<t4*>(y + q * 3);
#pragma unroll
    for (int j = 0; j < 3; ++j) yp[j] = t4{(T)v[4 * j], (T)v[4 * j + 1], (T)v[4 * j + 2], (T)v[4 * j + 3]};
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int o = 0; o < 3; ++o) y[(q + k) * ldy + o] = (T)v[k * 3 + o];
  }
  if (u8 && (vec & 2)) {
    uint32_t* up = reinterpret_cast<uint32_t*>(u8 + q * 3);   // 12 bytes at a multiple of 12 from a dword base
#pragma unroll
    for (int j = 0; j < 3; ++j) up[j] = c[j];
  } else if (u8) {
#pragma unroll
    for (int j = 0; j < 12; ++j) u8[q * 3 + j] = (uint8_t)(c[j >> 2] >> ((j & 3) * 8));
  }
}

// one source row's contribution to the three output rows it feeds, for four pixels of one buffer: slot dy of
// row s lands on output row s - dy + 1, so up[dy] += R_dy (+ the segment-end terms at pixels 0 / 3)
GHOST_DEV void zr_row4(const _Float16* __restrict__ z, int H, int W, int s, int x0, float (&o2)[4][3],
                       float (&o1)[4][3], float (&o0)[4][3]) {
  typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
  typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
  const long ps = (long)s * W + x0;
  f16x8_t r[6];   // the four pixels' R records: 48 fp16, 96 contiguous bytes
#pragma unroll
  for (int j = 0; j < 6; ++j) r[j] = *reinterpret_cast<const f16x8_t*>(z + ps * kZrR + j * 8);
  const _Float16* __restrict__ e = z + (long)H * W * kZrR;
  const bool first = (x0 & 7) == 0 && x0 > 0, last = (x0 & 7) == 4 && x0 + 4 < W;
  f16x8_t ef = {}, el = {};
  f16x4 ef2 = {}, el2 = {};
  if (first) {   // the previous segment's E_right, dy = 0..2
    const _Float16* q = e + ((ps - 1) >> 3) * kZrE + 12;
    ef = *reinterpret_cast<const f16x8_t*>(q);
    ef2 = *reinterpret_cast<const f16x4*>(q + 8);
  }
  if (last) {    // the next segment's E_left
    const _Float16* q = e + ((ps + 4) >> 3) * kZrE;
    el = *reinterpret_cast<const f16x8_t*>(q);
    el2 = *reinterpret_cast<const f16x4*>(q + 8);
  }
  auto rv = [&](int k, int dy, int o) { const int i = k * 12 + dy * 4 + o; return (float)r[i >> 3][i & 7]; };
  auto ev = [&](const f16x8_t& a, const f16x4& a2, int dy, int o) {
    const int i = dy * 4 + o;
    return i < 8 ? (float)a[i] : (float)a2[i - 8];
  };
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    o2[0][o] += rv(0, 2, o) + ev(ef, ef2, 2, o);
    o1[0][o] += rv(0, 1, o) + ev(ef, ef2, 1, o);
    o0[0][o] += rv(0, 0, o) + ev(ef, ef2, 0, o);
#pragma unroll
    for (int k = 1; k < 3; ++k) {
      o2[k][o] += rv(k, 2, o);
      o1[k][o] += rv(k, 1, o);
      o0[k][o] += rv(k, 0, o);
    }
    o2[3][o] += rv(3, 2, o) + ev(el, el2, 2, o);
    o1[3][o] += rv(3, 1, o) + ev(el, el2, 1, o);
    o0[3][o] += rv(3, 0, o) + ev(el, el2, 0, o);
  }
}

// strips of TS_SR output rows per thread (four pixels wide): the thread walks source rows y0 - 1 .. y0 + SR
// once, each feeding the three output rows around it, so a row-sum record is read (SR + 2) / SR times instead
// of the three 8-byte pieces of it being fetched by three output rows' threads (PMC: 1.6x the minimum bytes)
constexpr int TS_SR = 8;
template <typename T>
__global__ void __launch_bounds__(256) tap_sum3x3_strip_kernel(const _Float16* __restrict__ zh,
                                                               const _Float16* __restrict__ zx, int B, int H, int W,
                                                               T* __restrict__ y, int ldy, uint8_t* __restrict__ u8,
                                                               int vec) {
  const int nb = (int)gridDim.x;
  const int bid = (nb & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nb >> 3) + (int)(blockIdx.x >> 3);
  const long g = (long)bid * 256 + threadIdx.x;   // (sample, strip, 4-pixel column group)
  const int gpr = W / 4, strips = H / TS_SR;
  const long sg = g / gpr;
  if (sg >= (long)B * strips) return;
  const int b = (int)(sg / strips), y0 = (int)(sg - (long)b * strips) * TS_SR, ox = (int)(g - sg * gpr) * 4;
  const long zi = (long)b * zr_image(H * W);
  // o2: the output row that source row s completes (s - 1), o1: row s, o0: row s + 1
  float a2[4][3] = {}, a1[4][3] = {}, a0[4][3] = {};
  for (int sr = y0 - 1; sr <= y0 + TS_SR; ++sr) {
    if (sr >= 0 && sr < H) {
      zr_row4(zh + zi, H, W, sr, ox, a2, a1, a0);
      zr_row4(zx + zi, H, W, sr, ox, a2, a1, a0);
    }
    if (sr - 1 >= y0) tap_out4(a2, ((long)b * H + sr - 1) * W + ox, y, ldy, u8, vec);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        a2[k][o] = a1[k][o];
        a1[k][o] = a0[k][o];
        a0[k][o] = 0.f;
      }
  }
}

int tap_sum3x3(int dt, const void* zh, const void* zx, int B, int H, int W, void* y, int ldy, uint8_t* u8,
               hipStream_t s) {
  if (W % 8 || H % TS_SR || ldy < 3 || (uintptr_t)zh % 16 || (uintptr_t)zx % 16 || !is16(dt)) return -1;
  // whole-dword stores where the caller's buffers allow them (an out= view may start anywhere)
  const int vec = (ldy == 3 && (uintptr_t)y % 8 == 0 ? 1 : 0) | ((uintptr_t)u8 % 4 == 0 ? 2 : 0);
  const dim3 gs((unsigned)(((long)B * (H / TS_SR) * (W / 4) + 255) / 256));
  if (dt == GHOST_F16)
    hipLaunchKernelGGL(tap_sum3x3_strip_kernel<_Float16>, gs, dim3(256), 0, s, (const _Float16*)zh, (const _Float16*)zx,
                       B, H, W, (_Float16*)y, ldy, u8, vec);
  else
    hipLaunchKernelGGL(tap_sum3x3_strip_kernel<bf16>, gs, dim3(256), 0, s, (const _Float16*)zh, (const _Float16*)zx, B,
                       H, W, (bf16*)y, ldy, u8, vec);
  return (int)hipGetLastError();
}

}  // namespace ghost
