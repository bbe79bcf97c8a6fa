// ghost_amd — ArcFace identity encoder (IResNet) on gfx950, C ABI in include/ghost_amd.h.
//
// GHOST calls netArc = iresnet100(fp16=False) on 112x112 crops (inference.py:33-36,
// utils/inference/core.py:43-54, video_processing.py:136-140).  The network definition is the
// public insightface arcface_torch IResNet (downloaded by download_models.sh:3, absent from the
// reference tree: parity against it is unpinned, see oracle/arcface_ref.py).
//
// Execution plan (NHWC, one stream, every contraction on the implicit-GEMM conv of conv_igemm.hip):
//   stem   conv3x3 3->64 + BN + PReLU                          -> X, and XB = bn1 of block 1 (dual output)
//   block  T  = PReLU(bn2(conv3x3(XB)))                        (IBasicBlock conv1, stride 1)
//          R  = bn(conv1x1/s(X))                              (first block of a layer only)
//          X' = bn3(conv3x3/s(T)) + (R | X);  XB' = bn1'(X')   (next block's BN, or the head's bn2)
//   head   emb = features_BN(fc(flatten(bn2(X))))  = a 7x7 "valid" conv over XB with the fc bias and
//          the BatchNorm1d folded into a per-feature scale/shift, fp32 output.
// Every BatchNorm that precedes a zero-padded conv is applied by its producer's second output, never
// folded into the conv weights (folding is wrong on the padded border).
#include <algorithm>
#include <cstdlib>
#include <string>
#include <map>
#include <vector>
#include <cmath>

#include "ghost_amd.h"
#include "ghost_common.h"
#include "conv_igemm.h"
#include "ops.h"

using namespace ghost;

namespace ghost {
int set_last_error(int rc, const std::string& msg);   // aei_runtime.hip (ghost_last_error)
}
static int arc_fail(int rc, const std::string& msg) { return ghost::set_last_error(rc, msg); }

struct ghost_arc {
  int layers[4] = {3, 13, 30, 3};
  int nf = 512;
  int dt = GHOST_F32, esz = 4;
  std::map<std::string, const void*> slots;
  // diagnostic taps (ghost_arc_set_taps): stage i (0 = stem, i = block i) copies its stored residual
  // stream X into taps[2i] and the next BatchNorm's second output XB into taps[2i+1] when non-null
  std::vector<void*> taps;
};

namespace {

const int kWidths[4] = {64, 128, 256, 512};
inline int rup(int v, int m) { return (v + m - 1) / m * m; }

struct ArcCtx {
  ghost_arc* h;
  bool dry;
  char* base = nullptr;
  size_t off = 0;
  size_t scratch_need = 0;
  char* scratch = nullptr;
  size_t scratch_cap = 0;
  hipStream_t s = nullptr;
  int rc = 0;
  std::string where;

  void* alloc(size_t bytes) {
    off = (off + 255) & ~size_t(255);
    void* p = dry ? reinterpret_cast<void*>(uintptr_t(0x10000000) + off) : base + off;
    off += bytes;
    return p;
  }
  bool ok() const { return rc == 0; }
  void check(int r, const std::string& what) {
    if (r != 0 && rc == 0) { rc = r; where = what; }
  }
  const void* W(const std::string& name) {
    auto it = h->slots.find(name);
    if (it == h->slots.end()) {
      if (rc == 0) { rc = GHOST_EINVAL; where = "plan reads undeclared slot " + name; }
      return nullptr;
    }
    if (dry) return reinterpret_cast<const void*>(uintptr_t(0x1000));
    if (!it->second) {
      if (rc == 0) { rc = GHOST_ENOTREADY; where = "unbound weight slot " + name; }
      return nullptr;
    }
    return it->second;
  }
};

static int arc_min_wgs() {
  static const int v = GHOST_KNOB("GHOST_ARC_MINWG", 0);
  return v;
}

void run_conv(ArcCtx& c, ConvDesc& d, const std::string& what) {
  if (!c.ok()) return;
  d.min_wgs = arc_min_wgs();
  if (c.dry) {
    const size_t need = conv_workspace_bytes(d);
    if (need > c.scratch_need) c.scratch_need = need;
    return;
  }
  c.check(conv_launch(d, c.scratch, c.scratch_cap, c.s), what);
}

// conv + folded BN (+PReLU) (+residual) (+second output = next BN)
void conv_bn(ArcCtx& c, const std::string& w, const std::string& bn, const void* x, int ldx, int N, int H, int Cin,
             int Cout, int k, int stride, void* y, const char* prelu, const void* res, void* y2,
             const std::string& bn2name) {
  ghost_arc* h = c.h;
  ConvDesc d;
  d.ti = d.to = h->dt;
  d.x = x; d.B = N; d.Hi = H; d.Wi = H; d.Cin = Cin; d.ldx = ldx;
  d.w = c.W(w);
  d.N = Cout; d.Npad = rup(Cout, 128); d.Kpad = rup(k * k * Cin, 32);
  d.kind = CONV_FWD; d.kh = d.kw = k; d.stride = stride; d.pad = k / 2;
  d.y = y; d.ldy = Cout;
  d.scale = (const float*)c.W(bn + ".scale");
  d.shift = (const float*)c.W(bn + ".shift");
  d.slope = 1.f;
  if (prelu) d.prelu = (const float*)c.W(prelu);
  if (res) { d.res = res; d.ldres = Cout; }
  if (y2) {
    d.y2 = y2; d.ldy2 = Cout;
    d.scale2 = (const float*)c.W(bn2name + ".scale");
    d.shift2 = (const float*)c.W(bn2name + ".shift");
  }
  run_conv(c, d, w);
}

std::string blk_name(int li, int b) { return "l" + std::to_string(li) + ".b" + std::to_string(b); }

// xin: [N,112,112,4] NHWC (channel 3 = 0) in the handle dtype
void arc_plan(ArcCtx& c, const void* xin, int N, float* emb) {
  ghost_arc* h = c.h;
  const int es = h->esz;
  const size_t big = (size_t)N * 112 * 112 * 64 * es;   // largest activation (stem / layer-1 conv1)
  void* X[2] = {c.alloc(big), c.alloc(big)};
  void* XB[2] = {c.alloc(big), c.alloc(big)};
  void* T = c.alloc(big);
  void* R = c.alloc(big / 2);
  // list of blocks in forward order, to know which BN the producer's second output applies
  std::vector<std::pair<int, int>> blks;
  for (int li = 1; li <= 4; ++li)
    for (int b = 0; b < h->layers[li - 1]; ++b) blks.push_back({li, b});
  auto next_bn = [&](size_t i) {   // BN applied to the output of block i-1 (i = index of the consumer)
    return i < blks.size() ? blk_name(blks[i].first, blks[i].second) + ".bn1" : std::string("head.bn2");
  };
  // per-stage tap copies (parity bisection: the oracle recomputes each stage from the GPU's own inputs)
  auto tap = [&](size_t stage, const void* x, const void* xb, size_t bytes) {
    if (c.dry || !c.ok() || 2 * stage + 1 >= h->taps.size()) return;
    if (h->taps[2 * stage])
      c.check((int)hipMemcpyAsync(h->taps[2 * stage], x, bytes, hipMemcpyDeviceToDevice, c.s), "tap copy");
    if (h->taps[2 * stage + 1])
      c.check((int)hipMemcpyAsync(h->taps[2 * stage + 1], xb, bytes, hipMemcpyDeviceToDevice, c.s), "tap copy");
  };
  // stem: conv1 3x3 3->64 + bn1 + prelu  (X), bn1 of the first block (XB)
  conv_bn(c, "stem.w", "stem.bn", xin, 4, N, 112, 3, 64, 3, 1, X[0], "stem.prelu", nullptr, XB[0], next_bn(0));
  tap(0, X[0], XB[0], (size_t)N * 112 * 112 * 64 * es);
  int cur = 0, H = 112, C = 64;
  for (size_t i = 0; i < blks.size(); ++i) {
    const int li = blks[i].first, b = blks[i].second;
    const int planes = kWidths[li - 1], stride = b == 0 ? 2 : 1;
    const int Ho = H / stride;
    const std::string nm = blk_name(li, b);
    conv_bn(c, nm + ".c1.w", nm + ".bn2", XB[cur], C, N, H, C, planes, 3, 1, T, (nm + ".prelu").c_str(), nullptr,
            nullptr, "");
    const void* res = X[cur];
    if (b == 0) {
      conv_bn(c, nm + ".down.w", nm + ".down", X[cur], C, N, H, C, planes, 1, stride, R, nullptr, nullptr, nullptr,
              "");
      res = R;
    }
    conv_bn(c, nm + ".c2.w", nm + ".bn3", T, planes, N, H, planes, planes, 3, stride, X[cur ^ 1], nullptr, res,
            XB[cur ^ 1], next_bn(i + 1));
    cur ^= 1;
    H = Ho;
    C = planes;
    tap(i + 1, X[cur], XB[cur], (size_t)N * H * H * C * es);
  }
  // head: fc over flatten(bn2(X)) as a 7x7 valid conv, features BatchNorm1d folded with the fc bias
  ConvDesc d;
  d.ti = h->dt; d.to = GHOST_F32;
  d.x = XB[cur]; d.B = N; d.Hi = H; d.Wi = H; d.Cin = C; d.ldx = C;
  d.w = c.W("fc.w");
  d.N = h->nf; d.Npad = rup(h->nf, 128); d.Kpad = rup(H * H * C, 32);
  d.kind = CONV_FWD; d.kh = d.kw = H; d.stride = 1; d.pad = 0;
  d.y = emb; d.ldy = h->nf;
  d.scale = (const float*)c.W("fc.scale");
  d.shift = (const float*)c.W("fc.shift");
  d.slope = 1.f;
  run_conv(c, d, "fc");
}

void declare(ghost_arc* h) {
  auto add = [&](const std::string& s) { h->slots[s] = nullptr; };
  auto bn = [&](const std::string& s) { add(s + ".scale"); add(s + ".shift"); };
  add("stem.w"); bn("stem.bn"); add("stem.prelu");
  for (int li = 1; li <= 4; ++li)
    for (int b = 0; b < h->layers[li - 1]; ++b) {
      const std::string nm = blk_name(li, b);
      bn(nm + ".bn1");
      add(nm + ".c1.w"); bn(nm + ".bn2"); add(nm + ".prelu");
      add(nm + ".c2.w"); bn(nm + ".bn3");
      if (b == 0) { add(nm + ".down.w"); bn(nm + ".down"); }
    }
  bn("head.bn2");
  add("fc.w"); add("fc.scale"); add("fc.shift");
}

int64_t arc_bytes(ghost_arc* h, int N, size_t* scratch) {
  ArcCtx c{};
  c.h = h; c.dry = true;
  void* xin = c.alloc((size_t)N * 112 * 112 * 4 * h->esz);
  float* emb = (float*)uintptr_t(0x30000000);
  arc_plan(c, xin, N, emb);
  if (!c.ok()) return c.rc;
  c.alloc(256);   // u8 max flag
  *scratch = c.scratch_need;
  return (int64_t)(((c.off + 255) & ~size_t(255)) + c.scratch_need + 256);
}

// ---------------------------------------------------------------------------------------------
// pre-processing: normalize_and_torch_batch (image_processing.py:37-48) + F.interpolate(0.5,
// bilinear, align_corners=True) (core.py:44; video_processing.py:138) in one pass
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) u8_max_kernel(const uint8_t* __restrict__ p, long bstride, int per,
                                                      int* out) {
  // one flag for the whole batch: the reference divides by 255 only if batch.max() > 1.
  // blockIdx.y = sample; 16-byte loads where the sample base is aligned, bytes otherwise
  const uint8_t* s = p + (long)blockIdx.y * bstride;
  int m = 0;
  const int nvec = ((uintptr_t)s % 16 == 0) ? per / 16 : 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += gridDim.x * 256) {
    const u32x4 v = reinterpret_cast<const u32x4*>(s)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned w = v[k];
      const unsigned b0 = w & 255u, b1 = (w >> 8) & 255u, b2 = (w >> 16) & 255u, b3 = w >> 24;
      const unsigned mm = max(max(b0, b1), max(b2, b3));
      m = (int)mm > m ? (int)mm : m;
    }
  }
  for (int i = nvec * 16 + blockIdx.x * 256 + threadIdx.x; i < per; i += gridDim.x * 256) {
    const int v = s[i];
    m = v > m ? v : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int t = __shfl_xor(m, o, 64);
    m = t > m ? t : m;
  }
  // one atomic per workgroup at most: same-address atomics serialise in one L2 channel (one per wave cost
  // ~50 us at B = 128, 4096 of them), and the reader only asks max > 1, so a workgroup whose max is <= 1, or
  // that already sees the flag above 1, adds nothing
  __shared__ int wmax[4];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (m > 1 && __hip_atomic_load(out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= 1) atomicMax(out, m);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) arc_prep_kernel(const uint8_t* __restrict__ crops, long bstride, int N,
                                                        int Hs, int Ws, int Ho, int Wo, float sh, float sw,
                                                        const int* __restrict__ maxv, T* __restrict__ y) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;   // one output pixel
  if (idx >= (long)N * Ho * Wo) return;
  const int n = (int)(idx / ((long)Ho * Wo));
  const int r = (int)(idx - (long)n * Ho * Wo);
  const int oy = r / Wo, ox = r - oy * Wo;
  const bool div = *maxv > 1;
  float ry = sh * (float)oy, rx = sw * (float)ox;
  asm volatile("" : "+v"(ry), "+v"(rx));
  const int y0 = (int)ry, x0 = (int)rx;
  const int y1 = y0 + (y0 < Hs - 1 ? 1 : 0), x1 = x0 + (x0 < Ws - 1 ? 1 : 0);
  const float ly1 = ry - (float)y0, ly0 = 1.f - ly1, lx1 = rx - (float)x0, lx0 = 1.f - lx1;
  const uint8_t* src = crops + n * bstride;
  float out[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {   // channel order kept (the reference feeds BGR frames as they are)
    float v[4];
    const long o[4] = {((long)y0 * Ws + x0) * 3, ((long)y0 * Ws + x1) * 3, ((long)y1 * Ws + x0) * 3,
                       ((long)y1 * Ws + x1) * 3};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float t = (float)src[o[q] + ch];
      if (div) t = t / 255.0f;
      v[q] = (t - 0.5f) / 0.5f;
    }
    out[ch] = ly0 * (lx0 * v[0] + lx1 * v[1]) + ly1 * (lx0 * v[2] + lx1 * v[3]);
  }
#pragma unroll
  for (int ch = 0; ch < 4; ++ch) y[idx * 4 + ch] = from_f<T>(out[ch]);
}

// video_processing.py:126,139-148: normalise both sides, per target the best face and its score
__global__ void __launch_bounds__(256) arc_match_kernel(const float* __restrict__ f, int F, const float* __restrict__ t,
                                                         int dim, float th, int32_t* best_idx, float* best_sim,
                                                         int32_t* ok) {
  __shared__ float tn[1024];
  __shared__ float red[4];
  __shared__ float sim_s[4];
  __shared__ int idx_s[4];
  const int j = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // target norm: F.normalize(x) = x / max(||x||_2, 1e-12)
  float ss = 0.f;
  for (int k = tid; k < dim; k += 256) { const float v = t[(long)j * dim + k]; ss += v * v; }
  ss = group_sum(ss, 64);
  if (lane == 0) red[wv] = ss;
  __syncthreads();
  const float tnorm = fmaxf(sqrtf(red[0] + red[1] + red[2] + red[3]), 1e-12f);
  for (int k = tid; k < dim; k += 256) tn[k] = t[(long)j * dim + k] / tnorm;
  __syncthreads();
  float bs = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = wv; i < F; i += 4) {   // one wave per face
    float fs = 0.f;
    for (int k = lane; k < dim; k += 64) { const float v = f[(long)i * dim + k]; fs += v * v; }
    fs = group_sum(fs, 64);
    const float fnorm = fmaxf(sqrtf(fs), 1e-12f);
    float d = 0.f;
    for (int k = lane; k < dim; k += 64) d += (f[(long)i * dim + k] / fnorm) * tn[k];
    d = group_sum(d, 64);
    if (d > bs) { bs = d; bi = i; }   // faces visited in increasing order per wave: first max kept
  }
  if (lane == 0) { sim_s[wv] = bs; idx_s[wv] = bi; }
  __syncthreads();
  if (tid == 0) {
    float b = sim_s[0];
    int bidx = idx_s[0];
    for (int w = 1; w < 4; ++w)
      if (sim_s[w] > b || (sim_s[w] == b && idx_s[w] < bidx)) { b = sim_s[w]; bidx = idx_s[w]; }
    best_idx[j] = bidx;
    best_sim[j] = b;
    ok[j] = b > th ? 1 : 0;
  }
}

int run_arc(ghost_arc* h, int N, const void* xt, int xt_dtype, const int64_t* st, const uint8_t* crops,
            int64_t crop_bs, int Hs, int Ws, float* emb, void* ws, int64_t ws_bytes, void* stream) {
  if (!h) return arc_fail(GHOST_EINVAL, "null handle");
  if (N <= 0 || N > 65535) return arc_fail(GHOST_EINVAL, "batch must be in 1..65535");
  for (auto& kv : h->slots)
    if (!kv.second) return arc_fail(GHOST_ENOTREADY, "unbound weight slot " + kv.first);
  size_t scratch = 0;
  const int64_t need = arc_bytes(h, N, &scratch);
  if (need < 0) return arc_fail((int)need, "plan sizing failed");
  if (!ws || ws_bytes < need) return arc_fail(GHOST_ENOWS, "workspace too small: need " + std::to_string(need));
  ArcCtx c{};
  c.h = h; c.dry = false;
  c.base = (char*)(((uintptr_t)ws + 255) & ~uintptr_t(255));
  c.s = (hipStream_t)stream;
  void* xin = c.alloc((size_t)N * 112 * 112 * 4 * h->esz);
  // same allocation order as arc_bytes: the plan's buffers, then the flag, then the scratch
  ArcCtx probe{};
  probe.h = h; probe.dry = true;
  probe.alloc((size_t)N * 112 * 112 * 4 * h->esz);
  arc_plan(probe, probe.base, N, emb);
  const size_t plan_end = (probe.off + 255) & ~size_t(255);
  int* flag = (int*)(c.base + plan_end);
  c.scratch = c.base + plan_end + 256;
  c.scratch_cap = scratch;
  if (crops) {
    if (hipMemsetAsync(flag, 0, sizeof(int), c.s) != hipSuccess) return arc_fail(GHOST_EINVAL, "memset failed");
    const int per = Hs * Ws * 3;
    hipLaunchKernelGGL(u8_max_kernel, dim3(8, (unsigned)N), dim3(256), 0, c.s, crops, (long)crop_bs, per, flag);
    const float sh = (float)(Hs - 1) / (float)(112 - 1), sw = (float)(Ws - 1) / (float)(112 - 1);
    const long P = (long)N * 112 * 112;
    dim3 grid((unsigned)((P + 255) / 256));
    if (h->dt == GHOST_F32)
      hipLaunchKernelGGL(arc_prep_kernel<float>, grid, dim3(256), 0, c.s, crops, (long)crop_bs, N, Hs, Ws, 112, 112,
                         sh, sw, flag, (float*)xin);
    else
      hipLaunchKernelGGL(arc_prep_kernel<bf16>, grid, dim3(256), 0, c.s, crops, (long)crop_bs, N, Hs, Ws, 112, 112,
                         sh, sw, flag, (bf16*)xin);
    c.check((int)hipGetLastError(), "arc_prep");
  } else {
    c.check(input_to_nhwc(xt_dtype, xt, st, N, 3, 112, 112, h->dt, xin, c.s, 4), "input_to_nhwc");
  }
  arc_plan(c, xin, N, emb);
  if (!c.ok())
    return arc_fail(c.rc, "ArcFace forward failed at " + c.where +
                              (c.rc > 0 ? std::string(": ") + hipGetErrorString((hipError_t)c.rc) : std::string()));
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
extern "C" int ghost_arc_create(const int layers[4], int num_features, int dtype, ghost_arc** out) {
  if (!out || !layers) return arc_fail(GHOST_EINVAL, "null argument");
  for (int i = 0; i < 4; ++i)
    if (layers[i] < 1 || layers[i] > 64) return arc_fail(GHOST_EINVAL, "layers[i] out of range");
  if (num_features <= 0 || num_features % 16) return arc_fail(GHOST_EINVAL, "num_features must be a multiple of 16");
  if (dtype != GHOST_F32 && dtype != GHOST_BF16) return arc_fail(GHOST_EINVAL, "dtype must be f32 or bf16");
  ghost_arc* h = new ghost_arc();
  for (int i = 0; i < 4; ++i) h->layers[i] = layers[i];
  h->nf = num_features;
  h->dt = dtype;
  h->esz = dtype == GHOST_F32 ? 4 : 2;
  declare(h);
  *out = h;
  return 0;
}

extern "C" void ghost_arc_destroy(ghost_arc* h) { delete h; }

extern "C" int ghost_arc_bind(ghost_arc* h, const char* name, const void* p, int64_t numel) {
  if (!h || !name) return arc_fail(GHOST_EINVAL, "null argument");
  auto it = h->slots.find(name);
  if (it == h->slots.end()) return arc_fail(GHOST_EINVAL, std::string("unknown weight slot ") + name);
  if (!p || numel <= 0) return arc_fail(GHOST_EINVAL, std::string("empty tensor for ") + name);
  it->second = p;
  return 0;
}

extern "C" int ghost_arc_missing(ghost_arc* h) {
  if (!h) return arc_fail(GHOST_EINVAL, "null handle");
  int n = 0;
  for (auto& kv : h->slots)
    if (!kv.second) {
      if (n == 0) arc_fail(GHOST_ENOTREADY, "unbound weight slot " + kv.first);
      ++n;
    }
  return n;
}

extern "C" int64_t ghost_arc_workspace_bytes(ghost_arc* h, int N) {
  if (!h || N <= 0) return arc_fail(GHOST_EINVAL, "bad argument");
  size_t scratch = 0;
  return arc_bytes(h, N, &scratch);
}

extern "C" int ghost_arc_forward(ghost_arc* h, const void* x, int x_dtype, const int64_t x_strides[4], int N,
                                 float* emb, void* ws, int64_t ws_bytes, void* stream) {
  if (!x || !x_strides || !emb) return arc_fail(GHOST_EINVAL, "null argument");
  return run_arc(h, N, x, x_dtype, x_strides, nullptr, 0, 0, 0, emb, ws, ws_bytes, stream);
}

extern "C" int ghost_arc_embed_u8(ghost_arc* h, const uint8_t* crops, int64_t crop_batch_stride, int N, int H, int W,
                                  float* emb, void* ws, int64_t ws_bytes, void* stream) {
  if (!crops || !emb) return arc_fail(GHOST_EINVAL, "null argument");
  // F.interpolate(scale_factor=0.5) output size floor(H/2) must be the network's 112
  if (H / 2 != 112 || W / 2 != 112) return arc_fail(GHOST_EINVAL, "crops must be 224x224 (or 225) to give 112x112");
  return run_arc(h, N, nullptr, 0, nullptr, crops, crop_batch_stride, H, W, emb, ws, ws_bytes, stream);
}

extern "C" int ghost_arc_set_taps(ghost_arc* h, void* const* taps, int ntaps) {
  if (!h || ntaps < 0 || (ntaps && !taps)) return arc_fail(GHOST_EINVAL, "bad argument");
  h->taps.assign(taps, taps + ntaps);
  return 0;
}

extern "C" int ghost_arc_match(const float* face_emb, int F, const float* target_emb, int T, int dim,
                               float similarity_th, int32_t* best_idx, float* best_sim, int32_t* accepted,
                               void* stream) {
  if (!face_emb || !target_emb || !best_idx || !best_sim || !accepted) return arc_fail(GHOST_EINVAL, "null argument");
  if (F <= 0 || T <= 0 || dim <= 0 || dim > 1024 || T > 65535) return arc_fail(GHOST_EINVAL, "bad sizes");
  hipLaunchKernelGGL(arc_match_kernel, dim3(T), dim3(256), 0, (hipStream_t)stream, face_emb, F, target_emb, dim,
                     similarity_th, best_idx, best_sim, accepted);
  const int rc = (int)hipGetLastError();
  return rc ? arc_fail(rc, "ghost_arc_match launch failed") : 0;
}
