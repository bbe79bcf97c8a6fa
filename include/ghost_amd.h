/* ghost_amd — C ABI of the MI355X-native GHOST swap forward path.
 *
 * This is the drop-in boundary for the per-frame face-swap hot path of GHOST
 * (postworthy/ghost, a fork of sber-swap): the AEI_Net generator = attribute
 * encoder + AAD ResBlk decoder.  Every entry point takes plain device pointers,
 * sizes and an hipStream_t (passed as void*), returns an int status
 * (0 = success, <0 = invalid argument / state, >0 = hipError_t), never throws,
 * and never allocates device memory on the hot path (the caller supplies the
 * workspace).  ghost_last_error() describes the last failure of the calling thread.
 *
 * Reference interfaces replaced (paths under the reference repository):
 *   network/AEI_Net.py:143-151   AEI_Net(backbone, num_blocks, c_id)        -> ghost_aei_create
 *   inference.py:27-30           G.load_state_dict(...); .cuda(); .half()   -> ghost_aei_bind (prepacked)
 *   network/AEI_Net.py:153-156   AEI_Net.forward(Xt, z_id) -> (Y, attr)     -> ghost_aei_forward
 *   network/AEI_Net.py:158-159   AEI_Net.get_attr(X)                       -> ghost_aei_get_attr
 *   utils/inference/faceshifter_run.py:5-22 + utils/inference/core.py:13-26
 *                                faceshifter_batch(transform_target_to_torch(crops)) -> ghost_aei_swap_u8
 *   network/AADLayer.py:28-29 + utils/inference/faceshifter_run.py:15-16
 *                                fc1/fc2(z_id) per AADLayer, once per source identity -> ghost_aei_identity_table,
 *                                                                          ghost_aei_swap_u8_indexed
 *   network/AADLayer.py:20-38    AADLayer.forward(h_in, z_attr, z_id)       -> ghost_aad_layer_nhwc
 *   network/AEI_Net.py:19-24     conv4x4 (Conv 4x4/s2 + BN + LReLU)         -> ghost_conv2d_nhwc
 *   network/AEI_Net.py:27-41     deconv4x4 (ConvT 4x4/s2 + BN + LReLU + skip) -> ghost_conv_transpose4x4s2_nhwc
 *   network/AADLayer.py:64,71    Conv2d 3x3 of AAD_ResBlk (+ residual)     -> ghost_conv2d_nhwc
 *   network/AADLayer.py:16,24    InstanceNorm2d statistics                 -> ghost_instnorm_stats_nhwc
 *   network/AEI_Net.py:94,125    F.interpolate(x2, bilinear, align_corners) -> ghost_upsample2x_nhwc
 *
 * Activations crossing this ABI are NHWC with an explicit channel stride `ld`
 * (elements between consecutive pixels).  Packed weight layouts are documented
 * in INTEGRATION.md and produced by ghost_amd/network/pack.py.
 */
#ifndef GHOST_AMD_H
#define GHOST_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { GHOST_DTYPE_F32 = 0, GHOST_DTYPE_BF16 = 1, GHOST_DTYPE_F16 = 2, GHOST_DTYPE_U8 = 3 };
enum { GHOST_OK = 0, GHOST_EINVAL = -1, GHOST_ENOTREADY = -2, GHOST_ENOWS = -3 };

typedef struct ghost_aei ghost_aei;

const char* ghost_version(void);
const char* ghost_last_error(void);

/* ---- whole-network handle (one per device) ---------------------------------------- */
/* backbone: "unet" | "linknet" | "resnet" (MLAttrEncoderResnet, network/resnet.py:147-149); dtype: compute/storage dtype of activations and
 * conv weights (GHOST_DTYPE_F32 = parity path, GHOST_DTYPE_BF16 = throughput path). */
int ghost_aei_create(const char* backbone, int num_blocks, int c_id, int dtype, ghost_aei** out);
void ghost_aei_destroy(ghost_aei* h);
/* bind one prepacked weight tensor (device pointer, numel elements) under its slot name */
int ghost_aei_bind(ghost_aei* h, const char* name, const void* dev_ptr, int64_t numel);
/* number of slots still unbound (0 = ready); name of the first missing one in ghost_last_error() */
int ghost_aei_missing(ghost_aei* h);
/* geometry of z_attr_k (k = 1..8): channels, height, width (NHWC contiguous) */
int ghost_aei_attr_geometry(ghost_aei* h, int level, int* C, int* H, int* W);
/* device workspace needed by one forward of batch B (attr buffers supplied by the caller) */
int64_t ghost_aei_workspace_bytes(ghost_aei* h, int B);

/* AEI_Net.forward.  xt: [B,3,256,256] addressed with element strides xt_strides (any
 * layout, e.g. the permuted NHWC view of core.py:24), dtype f32/f16/bf16.  z_id: [B, c_id]
 * rows with row stride zid_row_stride.  y_nhwc: [B,256,256,3] in the handle dtype (tanh
 * output).  y_u8_bgr (optional): [B,256,256,3] uint8 BGR.  attr_nhwc: 8 device buffers
 * with the geometry above in the handle dtype (all required). */
int ghost_aei_forward(ghost_aei* h, const void* xt, int xt_dtype, const int64_t xt_strides[4], int B,
                      const void* z_id, int zid_dtype, int64_t zid_row_stride, void* y_nhwc, uint8_t* y_u8_bgr,
                      void* const attr_nhwc[8], void* ws, int64_t ws_bytes, void* stream);
/* AEI_Net.get_attr: the encoder only */
int ghost_aei_get_attr(ghost_aei* h, const void* xt, int xt_dtype, const int64_t xt_strides[4], int B,
                       void* const attr_nhwc[8], void* ws, int64_t ws_bytes, void* stream);
/* faceshifter_batch on uint8 BGR crops [B,256,256,3] (crop_batch_stride bytes apart):
 * normalise -> AEI_Net -> ((Y*0.5+0.5)*255)[...,BGR].uint8 into out_u8 [B,256,256,3].
 * y_nhwc and attr buffers come from the workspace. */
int64_t ghost_aei_swap_workspace_bytes(ghost_aei* h, int B);
int ghost_aei_swap_u8(ghost_aei* h, const uint8_t* crops, int64_t crop_batch_stride, int B, const void* z_id,
                      int zid_dtype, int64_t zid_row_stride, uint8_t* out_u8, void* ws, int64_t ws_bytes,
                      void* stream);

/* Per-identity projection table (AADLayer.py:28-29 fc1/fc2 of every AADLayer, AEI_Net.py:101 up1; a source
 * embedding's gamma_id / beta_id / m1 rows do not depend on the target frame, faceshifter_run.py:15-16 repeats one
 * z_id over the batch): computed once per (identity, weight version) and gathered per sample by identity_index.
 * ghost_aei_identity_table writes the rows of n_ident z_id rows (any float dtype, row stride zid_row_stride) into
 * table (device, 256-byte aligned, ghost_aei_identity_table_bytes(h, n_ident) bytes; workspace
 * ghost_aei_identity_table_workspace_bytes).  The table holds results of the handle's bound weights: rebuild it after
 * re-binding.  Rows are bit-identical to the projections a ghost_aei_swap_u8 of up to 64 frames computes.
 * ghost_aei_swap_u8_indexed = ghost_aei_swap_u8 with sample b's identity rows taken from table row
 * identity_index[b] (device int32 [B], values in [0, n_ident); an out-of-range value is clamped to that range, not
 * reported: validate on the host).  table_bytes: the table's size, checked against
 * ghost_aei_identity_table_bytes(h, n_ident) (GHOST_EINVAL if smaller), so the clamped gather stays inside the table.
 * Workspace: ghost_aei_swap_workspace_bytes. */
int64_t ghost_aei_identity_table_bytes(ghost_aei* h, int n_ident);
int64_t ghost_aei_identity_table_workspace_bytes(ghost_aei* h, int n_ident);
int ghost_aei_identity_table(ghost_aei* h, const void* z_id, int zid_dtype, int64_t zid_row_stride, int n_ident,
                             void* table, int64_t table_bytes, void* ws, int64_t ws_bytes, void* stream);
int ghost_aei_swap_u8_indexed(ghost_aei* h, const uint8_t* crops, int64_t crop_batch_stride, int B, const void* table,
                              int n_ident, int64_t table_bytes, const int32_t* identity_index, uint8_t* out_u8, void* ws,
                              int64_t ws_bytes, void* stream);

/* Per-handle plan options (defaults are the measured choices; every forward of the handle uses them):
 *   GHOST_AEI_OPT_FUSE_UPSAMPLE (1): AADBlk8's first AADLayer pair samples upsample2x(AADBlk7 output) on the fly
 *                                    instead of reading a materialised upsample (0 materialises it)
 *   GHOST_AEI_OPT_FUSE_STATS (1):    the persistent 3x3 conv emits the InstanceNorm partials of its output
 *                                    (0: a separate statistics pass)
 *   GHOST_AEI_OPT_TWO_STREAMS (1):   forward / swap run the attribute encoder's up path (deconv1..6 and the
 *                                    z_attr8 upsample) on a second, handle-owned HIP stream, overlapped with
 *                                    the generator's AADBlk k, which waits only for z_attr_k; the caller's
 *                                    stream waits for that stream before the call's last launch, so the
 *                                    ordering seen by the caller is unchanged (0: one stream; batches of
 *                                    fewer than 8 frames always run on one stream).  Same results.
 *   GHOST_AEI_OPT_TAP_PARTIALS (2):  bf16, C = 64 output block (AADBlk8): the 3x3 conv to 3 channels is
 *                                    contracted in its producers: each AADLayer that feeds it writes the
 *                                    per-tap partial sums of its channels, pre-summed along 8-pixel row
 *                                    segments (fp16, 15 per pixel) instead of its 64 bf16 channels, and a
 *                                    gather kernel sums three rows of them (+ tanh, uint8).
 *                                    2: both the h path and last_add_block's x'; 1: the h path only (x' is
 *                                    written and the narrow conv contracts it); 0: neither.  The partials
 *                                    are rounded to fp16 once per row sum (the extra rounding the
 *                                    bf16-storage emulation of oracle/aei_ref.py models).
 *   GHOST_AEI_OPT_FUSE_REDUCE (1):   split-K GEMMs with small partial tiles and the InstanceNorm statistics
 *                                    passes reduce their partials in the last workgroup to finish (arrival
 *                                    counters in the workspace, zeroed once per call) instead of a second
 *                                    kernel: the same sums in the same order, the same bytes, fewer launches
 *                                    (0: the separate reduction kernels).
 * value is 0 or 1 (TAP_PARTIALS: 0..2).  A handle is not shared across threads without external
 * synchronisation.  Two-stream calls of ALL handles on one device share one up-path stream (below): while one
 * call is being captured into a HIP graph (stream capture of the caller's stream), no other handle on that device
 * may run a two-stream call from another thread — its up-path work would join the capture — so capture with
 * GHOST_AEI_OPT_TWO_STREAMS = 0 (ghost_amd.inference.GraphedSwap's default) or serialise the calls. */
enum {
  GHOST_AEI_OPT_FUSE_UPSAMPLE = 0,
  GHOST_AEI_OPT_FUSE_STATS = 1,
  GHOST_AEI_OPT_TWO_STREAMS = 2,
  GHOST_AEI_OPT_TAP_PARTIALS = 3,
  GHOST_AEI_OPT_FUSE_REDUCE = 4,
  GHOST_AEI_NOPT = 5
};
int ghost_aei_set_option(ghost_aei* h, int option, int value);
int ghost_aei_get_option(ghost_aei* h, int option, int* value);
/* Diagnostic taps (parity bisection): while set, every forward / swap of the handle copies the stored
 * output of AADBlk k (k = 1..7, NHWC [B, 2^k, 2^k, cout_k] in the handle dtype, before the x2 upsample)
 * into taps[k-1] when that pointer is non-NULL (taps[7] is unused: AADBlk8's output is Y).
 * NULL taps clears them. */
int ghost_aei_set_taps(ghost_aei* h, void* const taps[8]);

/* the up-path stream on `device` as this handle uses it: ONE low-priority stream per device for the whole process,
 * shared by every handle on that device, created by the first two-stream forward / swap there and never destroyed
 * (valid until the process exits; NULL before this handle's first two-stream call there, or when stream creation
 * failed and the handle runs on one stream).  Diagnostics of hardware-queue sharing (tools/leg_probe.py). */
int ghost_aei_up_stream(ghost_aei* h, int device, void** stream);

/* per-kernel-class device timing with HIP events (bench instrumentation).
 * class_mask bit i enables class i; classes: 0 AAD kernels (all stages), 1 the block-input AAD
 * kernel at 256x256 (through-upsample: aad_v5, aad_v3.hip), 2 conv3x3 (all), 3 conv3x3 at 256x256, 4 IN stats + mask,
 * 5 encoder, 6 upsample, 7 identity projections. */
int ghost_aei_profile(ghost_aei* h, int class_mask);
/* after the stream is synchronised: total ms, launches, algorithmic bytes and flops of class i */
int ghost_aei_profile_read(ghost_aei* h, int cls, double* ms, int64_t* launches, double* bytes, double* flops);
/* class 1's in-kernel clock (armed by ghost_aei_profile with bit 1 set, on the current device): the sum over
 * its launches since then of (latest wave end - earliest workgroup start), in microseconds, read from the
 * kernel's own wall-clock stamps (hipDeviceAttributeWallClockRate) — the kernel's execution span, which
 * unlike a HIP-event bracket does not include queueing behind other streams' kernels.  After a sync.
 * kernel_version (may be NULL): generation of the class-1 AAD kernel that ran last (4: aad_v4, 5: aad_v5). */
int ghost_aei_profile_clock(ghost_aei* h, double* us_total, int64_t* launches, int* kernel_version);

/* ---- single operators (NHWC, per-op parity tests and callers of single layers) ------ */
/* Conv2d kh x kw / stride / pad (+ per-channel scale/shift, leaky slope, residual, tanh).
 * w_packed: [Npad][Kpad] with K index (ky*kw + kx)*Cin + c. */
int ghost_conv2d_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx, const void* w_packed, int Cout,
                      int Npad, int Kpad, int kh, int kw, int stride, int pad, const float* scale, const float* shift,
                      float slope, const void* res, int ldres, int tanh_out, void* y, int ldy, void* ws,
                      int64_t ws_bytes, void* stream);
/* Epilogue of ghost_conv2d_ex_nhwc, applied per output (pixel, channel n):
 *   v = acc*scale[n] + shift[n];  if res_first: v += res;  v = v > 0 ? v : v*(prelu ? prelu[n] : slope);
 *   if !res_first: v += res;  if tanh_out: v = tanh(v);  y = v;  if y2: y2 = v*scale2[n] + shift2[n]
 * Covers Conv+BN+LeakyReLU (AEI_Net.py:19-24), the ResNet Bottleneck tail relu(bn3(conv3) + residual)
 * (network/resnet.py:72-78), and the ArcFace IBasicBlock (conv + BN + PReLU; BN of the next block's
 * input written as the second output).  Pointers may be NULL (scale/shift default 1/0). */
typedef struct ghost_conv_epi {
  const float* scale;
  const float* shift;
  float slope;
  const float* prelu;
  const void* res;
  int ldres;
  int res_first;
  int tanh_out;
  void* y2;
  int ldy2;
  const float* scale2;
  const float* shift2;
  int split_k;   /* 0 = the planner's choice; n > 0 forces n K-splits (tests of the split-K reduction) */
} ghost_conv_epi;
int ghost_conv2d_ex_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx, const void* w_packed,
                         int Cout, int Npad, int Kpad, int kh, int kw, int stride, int pad, const ghost_conv_epi* epi,
                         void* y, int ldy, void* ws, int64_t ws_bytes, void* stream);
/* Conv2d 3x3/p1 to Cout <= 3 channels (the generator's RGB output): halo-tiled per-tap partial
 * sums; w_narrow [32][Kpad], row (ky*3+kx)*Cout + o; optional residual, tanh and BGR uint8 copy. */
int ghost_conv3x3_narrow_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx, const void* w_narrow,
                              int Kpad, int Cout, const void* res, int ldres, int tanh_out, void* y, int ldy,
                              uint8_t* u8, void* stream);
/* ConvTranspose2d 4x4/s2/p1 as four 2x2 sub-pixel phases; w_packed: [4][Npad][Kpad],
 * phase = 2*py + px, K index (ty*2 + tx)*Cin + c. */
int ghost_conv_transpose4x4s2_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx,
                                   const void* w_packed, int Cout, int Npad, int Kpad, const float* scale,
                                   const float* shift, float slope, const void* res, int ldres, void* y, int ldy,
                                   void* ws, int64_t ws_bytes, void* stream);
/* fp32 GEMM y[B, N] = x[B, K] * W^T + bias (Linear / ConvT-on-1x1); out dtype f32 or bf16 */
int ghost_linear_f32(const float* x, int B, int K, const float* w_packed, int N, int Npad, int Kpad,
                     const float* bias, int out_dtype, void* y, int ldy, void* ws, int64_t ws_bytes, void* stream);
/* InstanceNorm statistics: stat[b][c] = (mean, 1/sqrt(var+1e-5)) */
int ghost_instnorm_stats_nhwc(int dtype, const void* x, int B, int HW, int C, int ldx, float* stat, void* ws,
                              int64_t ws_bytes, void* stream);
/* the same statistics of upsample2x(x) (bilinear x2, align_corners, values rounded to dtype as the
 * upsample kernel stores them) for an [B, H, W, C] source, without materialising the upsample
 * (AEI_Net.py:137 feeding AADLayer.py:16's InstanceNorm) */
int ghost_instnorm_stats_up2x_nhwc(int dtype, const void* x, int B, int H, int W, int C, int ldx, float* stat,
                                   void* ws, int64_t ws_bytes, void* stream);
/* AADLayer.forward: gbw_packed [Npad][Kpad] rows interleaved per 16 channels
 * (gamma c0..15, beta c0..15, gamma c16..31, ...), gbb the matching biases (fp32);
 * wh [C] / bh [1] the conv_h weights; idgb [B][id_ld] holds gamma_id at c and beta_id
 * at C + c (fp32).  slope = 1: plain AADLayer; slope = 0: fused following ReLU. */
int ghost_aad_layer_nhwc(int dtype, const void* h_in, int ldh, const void* z_attr, int lda, int B, int H, int W, int C,
                         int Ca, const void* gbw_packed, int Npad, int Kpad, const float* gbb, const float* wh,
                         const float* bh, const float* idgb, int id_ld, float slope, void* out, int ldo, void* ws,
                         int64_t ws_bytes, void* stream);
/* One or two AADLayers (bf16, C in {64,128}) that read the same h_in and z_attr, in one pass:
 * w3/b3 per layer in the permuted layout of pack.py pack_aad_v3; InstanceNorm statistics of h_in
 * are computed into the workspace first.  up2x = 1: h_in is upsample2x of the [B, H/2, W/2, C]
 * tensor passed as h_in (F.interpolate of AEI_Net.py:135-137 fused into the AADLayer read; C in {64, 128}).
 * C = 256 (L = 1, Ca in {64, 128}) keeps all channels in one workgroup; C in {256, 512, 1024} otherwise
 * (L = 1, Ca <= 512) runs the per-channel-tile kernel of aad_wide.hip. */
int ghost_aad_layers_v3_nhwc(const void* h_in, int ldh, int up2x, const void* z_attr, int lda, int B, int H, int W,
                             int C, int Ca, int L, const void* const w3[], const float* const b3[],
                             const float* const wh[], const float* const bh[], const float* const idgb[], int id_ld,
                             float slope, void* const out[], const int ldo[], void* ws, int64_t ws_bytes,
                             void* stream);
int ghost_upsample2x_nhwc(int dtype, const void* x, int ldx, void* y, int ldy, int B, int H, int W, int C,
                          void* stream);
int ghost_nhwc_to_nchw(int dtype, const void* x, int ldx, int B, int H, int W, int C, void* y, void* stream);
/* transform_target_to_torch (core.py:13-26): uint8 BGR NHWC crops -> RGB NHWC in [-1,1] (dtype f32/bf16) */
int ghost_crops_to_input_nhwc(const uint8_t* crops, int64_t crop_batch_stride, int B, int H, int W, int dtype, void* y,
                              void* stream);
/* ---- ArcFace identity encoder (IResNet, the netArc GHOST loads) ------------------------
 * Replaces: inference.py:33-36 iresnet100(fp16=False) + load_state_dict + .cuda().eval();
 *   core.py:43-54 / video_processing.py:136-140 netArc(F.interpolate(normalize_and_torch_batch(crops),
 *   scale_factor=0.5, bilinear, align_corners=True)); video_processing.py:126,139-148 face matching.
 * The IResNet definition itself is not in the reference tree (download_models.sh:3): parity unpinned. */
typedef struct ghost_arc ghost_arc;
/* layers: blocks per stage ({3,13,30,3} = iresnet100); num_features: embedding size (512) */
int ghost_arc_create(const int layers[4], int num_features, int dtype, ghost_arc** out);
void ghost_arc_destroy(ghost_arc* h);
int ghost_arc_bind(ghost_arc* h, const char* name, const void* dev_ptr, int64_t numel);
int ghost_arc_missing(ghost_arc* h);
int64_t ghost_arc_workspace_bytes(ghost_arc* h, int N);
/* x: [N,3,112,112] with element strides (f32/f16/bf16/u8) -> emb fp32 [N, num_features] */
int ghost_arc_forward(ghost_arc* h, const void* x, int x_dtype, const int64_t x_strides[4], int N, float* emb,
                      void* ws, int64_t ws_bytes, void* stream);
/* uint8 aligned crops [N,H,W,3] (H = W = 224, channel order as given): normalize_and_torch_batch
 * (divide by 255 only if the batch max > 1) -> bilinear 0.5x align_corners -> IResNet -> emb */
int ghost_arc_embed_u8(ghost_arc* h, const uint8_t* crops, int64_t crop_batch_stride, int N, int H, int W,
                       float* emb, void* ws, int64_t ws_bytes, void* stream);
/* per target j: best_idx[j] = argmax_i cos(face_i, target_j) (first on ties), best_sim[j] = that
 * cosine, accepted[j] = best_sim[j] > similarity_th */
/* Diagnostic taps (parity bisection): while set, every forward copies, for stage i (0 = the stem, i >= 1 =
 * the i-th IBasicBlock in forward order), the stored residual stream X_i into taps[2i] and the next
 * BatchNorm's output BN(X_i) (the producer's second output, what the next block's conv reads) into
 * taps[2i+1], NHWC [N, H_i, W_i, C_i] in the handle dtype, where those pointers are non-NULL.
 * ntaps = 0 clears them. */
int ghost_arc_set_taps(ghost_arc* h, void* const* taps, int ntaps);
int ghost_arc_match(const float* face_emb, int F, const float* target_emb, int T, int dim, float similarity_th,
                    int32_t* best_idx, float* best_sim, int32_t* accepted, void* stream);

/* ---- paste-back blend (get_final_video, utils/inference/video_processing.py:218-227) ----
 * For each frame f with valid[f] != 0 (valid may be NULL): warp the crop-space swap [Hs,Ws,3] u8 and
 * mask [Hs,Ws] f32 back into the frame with kornia.warp_affine semantics (bilinear, zeros,
 * align_corners=True, destination pixel sampled at mats[f] (x, y, 1), mats = the crop <- frame tfm
 * [F][2][3] fp32) and composite in place: frame = uint8(mask_t*swap_t + (1-mask_t)*frame).
 * Several identities on one frame: call once per identity, in the reference's order. */
int ghost_blend_swaps_u8(uint8_t* frames, int64_t frame_stride, int F, int H, int W, const uint8_t* swaps,
                         int64_t swap_stride, int Hs, int Ws, const float* masks, int64_t mask_stride,
                         const float* mats, const int32_t* valid, void* stream);
/* cv2.resize(src, (Wd, Hd)) INTER_LINEAR for F uint8 [Hs,Ws,3] images (OpenCV's fixed point): the
 * resize of the 256x256 swap to the 224x224 crop size that precedes the warp (video_processing.py:212,
 * image_processing.py:63). */
int ghost_resize_u8_linear(const uint8_t* src, int64_t src_stride, int F, int Hs, int Ws, uint8_t* dst,
                           int64_t dst_stride, int Hd, int Wd, void* stream);
/* get_final_image (utils/inference/image_processing.py:51-76) for one full frame [H,W,3] u8, in place: for
 * each identity j in order, swap_t = cv2.warpAffine(swaps[j] (S x S, already resized), invertAffineTransform
 * (tfm_j), BORDER_REPLICATE), mask_t = the same warp of masks[j] with the constant 0 border, final =
 * mask_t*swap_t + (1-mask_t)*final; one uint8 cast at the end.  masks are float64 [J][S][S] (face_mask_static
 * returns mask/255 of a uint8 array, masks.py:83-85: numpy float64), so the mask warp (float table weights, double
 * accumulation, as cv2 does for CV_64F) and the composite run in double as numpy does.  maps[j] = the [2][3] double
 * matrix warpAffine samples with (the inverse of invertAffineTransform(tfm_j), computed on the host as
 * OpenCV does: ghost_amd.inference.blend.cv_warp_map). */
int ghost_blend_image_u8(uint8_t* frame, int H, int W, const uint8_t* swaps, int64_t swap_stride, int J, int S,
                         const double* masks, int64_t mask_stride, const double* maps, void* stream);

/* ---- face masks (face_mask_static, utils/inference/masks.py:38-107) ----
 * Host, CPU only (no device pointers): for F frames of 106 float32 landmarks [F][106][2] and their
 * (erode, sigmaX, sigmaY) params [F][3] (face_mask_static's, masks.py:43-65), expand_eyebrows on the int32
 * landmarks (masks.py:5-20) and the convex hull (masks.py:31): poly [F][128][2] int32 vertices, nv[F] counts. */
int ghost_mask_polygons(const float* landmarks, int F, int npts, const int32_t* params, int32_t* poly, int32_t* nv);
/* Device: poly / nv / params as above (device copies) -> masks [F][H][W] f32 (frame f at f*mask_stride floats):
 * cv2.fillConvexPoly(255), cv2.erode / dilate with the k x k box, the 2*sigmaY border fade, cv2.GaussianBlur
 * (0, 0, sigmaX, sigmaY), / 255.  H*W <= 57344, H <= 256; ws >= ghost_face_masks_workspace_bytes(F, H, W). */
int64_t ghost_face_masks_workspace_bytes(int F, int H, int W);
int ghost_face_masks(const int32_t* poly, const int32_t* nv, const int32_t* params, int F, int H, int W, float* masks,
                     int64_t mask_stride, void* ws, int64_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GHOST_AMD_H */
