// ghost_amd — the fused AADLayer kernel (AADLayer.py:20-38 + the ReLU that follows it).
//
// One workgroup owns BM pixels of one sample and ALL C channels of the layer:
//   1. per-channel tables in LDS from the InstanceNorm statistics: mu, rstd, wh*rstd
//   2. mask pre-pass over h_in[BM x C] (16-byte loads along channels):
//        M[p] = sigmoid(sum_c wh_c * (h_pc - mu_c) * rstd_c + bh)       (AADLayer.py:35)
//   3. for every 64-channel tile: gamma/beta_attr = z_attr[BM x Ca] . W^T on MFMA
//      (columns interleaved gamma c..c+15 | beta c..c+15), accumulator staged through LDS,
//      then the blend epilogue with 16-byte loads/stores along channels:
//        h = (h_in - mu)*rstd; A = ga*h + ba; I = gi*h + bi; out = relu((1-M)*A + M*I)
// HBM traffic per layer = |h_in| (+ an L1/L2 re-read) + |z_attr| + |out|: the algorithmic
// minimum of SURVEY.md §8d.  Layers whose pixel count is too small to fill the chip
// (<= 16x16 at batch 64) use the generic GEMM + separate mask path instead.
#include "aad_fused.h"
#include "ghost_common.h"

namespace ghost {

struct AadArgs {
  const void* za;
  const void* w;
  const float* gbb;
  const void* hin;
  const float* stat;
  const float* wh;
  const float* bh;
  const float* idgb;
  void* out;
  int lda, Ca, Kpad, ldh, id_ld, ldo, C, HW, M;
  float slope;
};

template <typename T, int BM>
__global__ void __launch_bounds__(256) aad_fused_kernel(const AadArgs a) {
  constexpr int BN = 128;                 // 64 channels x (gamma, beta)
  constexpr int CT = 64;                  // channels per tile
  constexpr int BK = 32;
  constexpr int VEC = Vec16<T>::N;
  constexpr int CPR = BK / VEC;
  constexpr int RPP = 256 / CPR;
  constexpr int AP = (BM + RPP - 1) / RPP;
  constexpr int BP = BN / RPP;
  constexpr int LDR = BK + VEC;
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int ACC_LD = BN + 4;
  constexpr int STAGE_BYTES = 2 * (BM + BN) * LDR * (int)sizeof(T);
  constexpr int ACC_BYTES = BM * ACC_LD * 4;
  constexpr int UNION_BYTES = STAGE_BYTES > ACC_BYTES ? STAGE_BYTES : ACC_BYTES;
  static_assert(BM % 32 == 0 && (BM % RPP == 0 || RPP % BM == 0), "tile");

  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  float* s_mu = reinterpret_cast<float*>(lds + UNION_BYTES);
  float* s_rs = s_mu + a.C;
  float* s_cf = s_rs + a.C;
  float* s_mask = s_cf + a.C;
  T* smem = reinterpret_cast<T*>(lds);
  float* s_acc = reinterpret_cast<float*>(lds);

  const int tid = threadIdx.x;
  const int m0 = blockIdx.x * BM;
  const int b = m0 / a.HW;                // HW % BM == 0: one sample per workgroup
  const T* __restrict__ za = reinterpret_cast<const T*>(a.za);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);
  const T* __restrict__ hin = reinterpret_cast<const T*>(a.hin);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);

  // ---- 1. channel tables ----
  for (int c = tid; c < a.C; c += 256) {
    const float mu = a.stat[((long)b * a.C + c) * 2];
    const float rs = a.stat[((long)b * a.C + c) * 2 + 1];
    s_mu[c] = mu;
    s_rs[c] = rs;
    s_cf[c] = a.wh[c] * rs;
  }
  __syncthreads();

  // ---- 2. mask pre-pass ----
  {
    const int cpp = a.C / VEC;                     // 16-byte chunks per pixel
    const int G = cpp < 64 ? cpp : 64;             // lanes per pixel (power of two)
    const int ppp = 256 / G;
    const int gl = tid % G;
    const float bh = a.bh[0];
    for (int p0 = 0; p0 < BM; p0 += ppp) {
      const int p = p0 + tid / G;
      float s = 0.f;
      if (p < BM) {
        const T* hp = hin + (long)(m0 + p) * a.ldh;
        for (int ch = gl; ch < cpp; ch += G) {
          float v[VEC];
          load16_f(hp + ch * VEC, v);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            const int c = ch * VEC + e;
            s = fmaf(s_cf[c], v[e] - s_mu[c], s);
          }
        }
      }
      s = group_sum(s, G);
      if (p < BM && gl == 0) s_mask[p] = sigmoidf_ref(s + bh);
    }
  }

  // ---- 3. channel tiles ----
  const int crow = tid / CPR, cch = tid % CPR;
  const int wid = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int wm = wid >> 1, wn = wid & 1;
  const int nk = a.Kpad / BK;
  const int ntile = a.C / CT;
  for (int ct = 0; ct < ntile; ++ct) {
    u32x4 ra[AP], rb[BP];
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto load_tile = [&](int kt) {
      const int k0 = kt * BK + cch * VEC;
#pragma unroll
      for (int p = 0; p < AP; ++p) {
        const int r = (BM >= RPP) ? crow + p * RPP : crow % BM;
        ra[p] = *reinterpret_cast<const u32x4*>(za + (long)(m0 + r) * a.lda + k0);
      }
#pragma unroll
      for (int p = 0; p < BP; ++p)
        rb[p] = *reinterpret_cast<const u32x4*>(w + (long)(ct * BN + crow + p * RPP) * a.Kpad + k0);
    };
    auto store_tile = [&](int buf) {
      T* As = smem + buf * (BM + BN) * LDR;
      T* Bs = As + BM * LDR;
#pragma unroll
      for (int p = 0; p < AP; ++p)
        if (BM >= RPP || crow < BM) *reinterpret_cast<u32x4*>(As + (crow + p * RPP) * LDR + cch * VEC) = ra[p];
#pragma unroll
      for (int p = 0; p < BP; ++p) *reinterpret_cast<u32x4*>(Bs + (crow + p * RPP) * LDR + cch * VEC) = rb[p];
    };
    auto compute = [&](int buf) {
      const T* As = smem + buf * (BM + BN) * LDR;
      const T* Bs = As + BM * LDR;
      const T* Ab = As + (wm * (BM / 2) + lr) * LDR;
      const T* Bb = Bs + (wn * (BN / 2) + lr) * LDR;
      if constexpr (sizeof(T) == 2) {
        v8_t<T> af[TM], bfv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const v8_t<T>*>(Ab + i * 16 * LDR + lq * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const v8_t<T>*>(Bb + j * 16 * LDR + lq * 8);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma16x16x32<T>(af[i], bfv[j], acc[i][j]);
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
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

    __syncthreads();   // previous tile's epilogue is done with the LDS union
    int cur = 0;
    load_tile(0);
    for (int kt = 0; kt < nk; ++kt) {
      store_tile(cur);
      __syncthreads();
      if (kt + 1 < nk) load_tile(kt + 1);
      compute(cur);
      cur ^= 1;
    }
    __syncthreads();   // all waves done reading the staging buffers
    // accumulators -> LDS [BM][ACC_LD]
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          s_acc[(wm * (BM / 2) + i * 16 + lq * 4 + r) * ACC_LD + wn * (BN / 2) + j * 16 + lr] = acc[i][j][r];
    __syncthreads();

    // blend epilogue: thread -> (pixel, VEC-channel chunk) with 16-byte accesses
    constexpr int TPP = CT / VEC;            // threads per pixel
    constexpr int PPP = 256 / TPP;
    const int cc = tid % TPP;
    const int cl = cc * VEC;                 // channel within the tile
    const int c0 = ct * CT + cl;
    const int colg = (cl >> 4) * 32 + (cl & 15);   // gamma column of channel cl; beta at +16
    float gbg[VEC], gbbeta[VEC], gi[VEC], bi[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      gbg[e] = a.gbb[ct * BN + colg + e];
      gbbeta[e] = a.gbb[ct * BN + colg + 16 + e];
      gi[e] = a.idgb[(long)b * a.id_ld + c0 + e];
      bi[e] = a.idgb[(long)b * a.id_ld + a.C + c0 + e];
    }
    for (int p = tid / TPP; p < BM; p += PPP) {
      const long m = m0 + p;
      float hv[VEC], o[VEC];
      load16_f(hin + m * a.ldh + c0, hv);
      const float Mk = s_mask[p];
      const float* arow = s_acc + p * ACC_LD + colg;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float h = (hv[e] - s_mu[c0 + e]) * s_rs[c0 + e];
        const float A = (arow[e] + gbg[e]) * h + (arow[16 + e] + gbbeta[e]);
        const float I = gi[e] * h + bi[e];
        const float v = (1.0f - Mk) * A + Mk * I;
        o[e] = v > 0.f ? v : v * a.slope;
      }
      store16_f(out + m * a.ldo + c0, o);
    }
  }
}

template <typename T, int BM>
static size_t lds_bytes(int C) {
  constexpr int BN = 128, BK = 32, VEC = Vec16<T>::N, LDR = BK + VEC, ACC_LD = BN + 4;
  constexpr int STAGE = 2 * (BM + BN) * LDR * (int)sizeof(T);
  constexpr int ACCB = BM * ACC_LD * 4;
  return (size_t)(STAGE > ACCB ? STAGE : ACCB) + (size_t)(3 * C + BM) * sizeof(float);
}

bool aad_fused_supported(int dt, int B, int HW, int C, int Ca, int lda, int ldh, int ldo) {
  const int vec = dt == GHOST_F32 ? 4 : 8;
  const int BM = 64;
  if (C % 64 || C > 2048 || Ca % 32 || HW % BM) return false;
  if (lda % vec || ldh % vec || ldo % vec) return false;
  const long tiles = (long)B * HW / BM;
  return tiles >= 512;   // enough workgroups to fill 256 CUs; smaller layers take the split path
}

int aad_fused(int dt, const void* za, int lda, int Ca, const void* w, int Kpad, const float* gbb, const void* hin,
              int ldh, const float* stat, const float* wh, const float* bh, const float* idgb, int id_ld, void* out,
              int ldo, int B, int HW, int C, float slope, hipStream_t s) {
  if (!aad_fused_supported(dt, B, HW, C, Ca, lda, ldh, ldo)) return -1;
  if ((uintptr_t)za % 16 || (uintptr_t)hin % 16 || (uintptr_t)out % 16 || (uintptr_t)w % 16) return -1;
  AadArgs a{};
  a.za = za; a.w = w; a.gbb = gbb; a.hin = hin; a.stat = stat; a.wh = wh; a.bh = bh; a.idgb = idgb; a.out = out;
  a.lda = lda; a.Ca = Ca; a.Kpad = Kpad; a.ldh = ldh; a.id_ld = id_ld; a.ldo = ldo; a.C = C; a.HW = HW;
  a.M = B * HW; a.slope = slope;
  constexpr int BM = 64;
  dim3 grid((unsigned)(a.M / BM));
  if (dt == GHOST_BF16) {
    const size_t lds = lds_bytes<bf16, BM>(C);
    hipLaunchKernelGGL((aad_fused_kernel<bf16, BM>), grid, dim3(256), lds, s, a);
  } else if (dt == GHOST_F16) {
    const size_t lds = lds_bytes<_Float16, BM>(C);
    hipLaunchKernelGGL((aad_fused_kernel<_Float16, BM>), grid, dim3(256), lds, s, a);
  } else if (dt == GHOST_F32) {
    const size_t lds = lds_bytes<float, BM>(C);
    hipLaunchKernelGGL((aad_fused_kernel<float, BM>), grid, dim3(256), lds, s, a);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

}  // namespace ghost
