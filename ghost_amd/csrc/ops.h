// ghost_amd — launchers for the bandwidth-bound kernels around the GEMMs.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ghost {

// InstanceNorm2d(affine=False) statistics (AADLayer.py:16,24): per (b, c) mean and
// 1/sqrt(biased var + eps) over H*W, from shifted partial sums (no Sigma x^2 - n mu^2
// cancellation) merged in fp64.  stat = [B][C][2].
size_t in_stats_workspace_bytes(int B, int HW, int C);
// sem (optional, nsem >= B words, zero on entry and left zero): the partial kernel's last workgroup per sample
// merges that sample's partials (one launch instead of two; same sums in the same order)
int in_stats(int dt, const void* x, int ldx, int B, int HW, int C, float* stat, void* ws, size_t ws_bytes,
             hipStream_t s, unsigned* sem = nullptr, int nsem = 0);
// the same statistics of upsample2x(x) ([B, 2H, 2W, C], values rounded to dt) without materialising
// it: x is the [B, H, W, C] source; workspace = in_stats_workspace_bytes(B, 4HW, C)
// true when in_stats_up2x takes the closed form over the source (cheaper than reading the upsample)
bool in_stats_up2x_closed_form(int dt, int H, int W, int C, int ldx);
int in_stats_up2x(int dt, const void* x, int ldx, int B, int H, int W, int C, float* stat, void* ws, size_t ws_bytes,
                  hipStream_t s, unsigned* sem = nullptr, int nsem = 0);

// statistics from the per-(tile, wave) partials a producer kernel wrote (ConvDesc::in_part): nrec
// records of (mean, centred sum of squares) over 64 pixels per (sample, channel), merged in fp64 (Chan)
// -> stat = [B][C][2] mean, rstd
int in_stats_from_tiles(const float* part, int B, int nrec, int C, float* stat, hipStream_t s);

// AAD mask: M[p] = sigmoid(sum_c wh[c] * (h[p,c]-mu[b,c])*rstd[b,c] + bh)   (AADLayer.py:35)
int aad_mask(int dt, const void* h, int ldh, int B, int HW, int C, const float* stat, const float* wh,
             const float* bh, float* mask, hipStream_t s);
// the masks of two AADLayers reading the same h_in in one pass (wh1 == nullptr: one layer)
int aad_mask2(int dt, const void* h, int ldh, int B, int HW, int C, const float* stat, const float* wh0,
              const float* bh0, float* mask0, const float* wh1, const float* bh1, float* mask1, hipStream_t s);

// HW <= 16 (2x2, 4x4): the statistics above AND the masks of one or two AADLayers (wh1 == nullptr:
// one) from one launch, one workgroup per sample
bool stats_mask_small_ok(int dt, int HW, int C, int ldx);
int stats_mask_small(int dt, const void* x, int ldx, int B, int HW, int C, float* stat, const float* wh0,
                     const float* bh0, float* mask0, const float* wh1, const float* bh1, float* mask1, hipStream_t s);

// bilinear x2, align_corners=True, NHWC (AEI_Net.py:94,125-137)
int upsample2x(int dt, const void* x, int ldx, void* y, int ldy, int B, int H, int W, int C, hipStream_t s);

// Xt [B,C,H,W] of dtype xdt with arbitrary element strides -> NHWC (ld = C) of dtype dt
// ldy >= C: channel stride of y; channels C..ldy-1 are written as zero
int input_to_nhwc(int xdt, const void* x, const int64_t strides[4], int B, int C, int H, int W, int dt, void* y,
                  hipStream_t s, int ldy);

// uint8 BGR NHWC crops -> RGB NHWC in [-1,1]: (v/255 - 0.5)/0.5  (core.py:13-26)
// ldy = 3, or 4 with a zero fourth channel
// zero (optional): nzero words (a multiple of 4, 16-byte aligned) set to 0 by the same launch (zero_words' job)
int crops_u8_to_input(const uint8_t* crops, int64_t batch_stride, int B, int H, int W, int dt, void* y,
                      hipStream_t s, int ldy, unsigned* zero = nullptr, int nzero = 0);

// Y NHWC (3 channels, ld) -> uint8 BGR NHWC: ((Y*0.5+0.5)*255)[..., [2,1,0]].uint8  (faceshifter_run.py:20-21)
int y_to_u8_bgr(int dt, const void* y, int ldy, int B, int H, int W, uint8_t* out, hipStream_t s);

// rows of z_id ([B, c_id] with a row stride, any float dtype) -> fp32 [B, c_id]
int rows_to_f32(int xdt, const void* x, int64_t row_stride, int B, int n, float* y, hipStream_t s);

// per-sample rows from a per-identity table (the identity table of ghost_aei_swap_u8_indexed): for each of
// nseg segments, out[g][b] = tab[g][idx[b]] (row_bytes[g] bytes, multiples of 16, 16-byte aligned).  An index
// outside [0, n_rows) is clamped (memory-safe; the host wrapper validates indices)
int gather_identity_rows(int nseg, const void* const* tab, const int64_t* row_bytes, void* const* out, int n_rows,
                         const int32_t* idx, int B, hipStream_t s);

// p[0 .. nwords) = 0 (a kernel, not a memset: the arrival counters of the fused reductions, zeroed at the start of
// every call, also inside a captured graph; nwords % 4 == 0, 16-byte aligned)
int zero_words(unsigned* p, int nwords, hipStream_t s);

// NHWC (ld) -> NCHW contiguous copy in the same dtype (attr export / tests)
int nhwc_to_nchw(int dt, const void* x, int ldx, int B, int H, int W, int C, void* y, hipStream_t s);

}  // namespace ghost
