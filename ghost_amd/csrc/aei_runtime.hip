// ghost_amd — native runtime for the AEI_Net forward (C ABI in include/ghost_amd.h).
//
// The handle holds the layer plan of AEI_Net(backbone, num_blocks, c_id)
// (network/AEI_Net.py:143-159, network/AADLayer.py) and pointers to weights that the
// host packed once (ghost_amd/network/pack.py).  A forward is a fixed sequence of
// launches on one stream; all intermediate tensors are carved from the caller's
// workspace by a bump allocator, whose size is found by a dry run of the same plan.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ghost_amd.h"
#include "aad_fused.h"
#include "aad_v3.h"
#include "conv_halo.h"
#include "aad_wide.h"
#include "conv_igemm.h"
#include "conv_narrow.h"
#include "ghost_common.h"
#include "ops.h"
#include "tap_rows.h"

using namespace ghost;

static thread_local std::string g_err;
static int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc == 0 ? GHOST_EINVAL : rc;
}
namespace ghost {
// shared with the other runtimes of the library (arc_runtime.hip): one ghost_last_error() per thread
int set_last_error(int rc, const std::string& msg) { return fail(rc, msg); }
int set_last_error(int rc, const char* msg) { return fail(rc, std::string(msg)); }
}  // namespace ghost

extern "C" const char* ghost_version(void) { return "ghost_amd 0.1 (gfx950)"; }
extern "C" const char* ghost_last_error(void) { return g_err.c_str(); }

namespace {

constexpr float kBnLrelu = 0.1f;  // LeakyReLU(0.1) (AEI_Net.py:23,32)

const int kEncDown[7][2] = {{3, 32}, {32, 64}, {64, 128}, {128, 256}, {256, 512}, {512, 1024}, {1024, 1024}};
const int kEncUpUnet[6][2] = {{1024, 1024}, {2048, 512}, {1024, 256}, {512, 128}, {256, 64}, {128, 32}};
const int kEncUpLink[6][2] = {{1024, 1024}, {1024, 512}, {512, 256}, {256, 128}, {128, 64}, {64, 32}};
// (cin, cout, c_attr) for AADBlk1..8 (AEI_Net.py:102-118)
const int kGenUnet[8][3] = {{1024, 1024, 1024}, {1024, 1024, 2048}, {1024, 1024, 1024}, {1024, 512, 512},
                            {512, 256, 256},    {256, 128, 128},    {128, 64, 64},      {64, 3, 64}};
const int kGenLink[8][3] = {{1024, 1024, 1024}, {1024, 1024, 1024}, {1024, 1024, 512}, {1024, 512, 256},
                            {512, 256, 128},    {256, 128, 64},     {128, 64, 32},     {64, 3, 32}};

inline int rup(int v, int m) { return (v + m - 1) / m * m; }

struct ProfClass {
  double ms = 0, bytes = 0, flops = 0;
  int64_t launches = 0;
};

}  // namespace

struct ghost_aei {
  bool linknet = false;
  bool resnet = false;   // backbone='resnet': MLAttrEncoderResnet (resnet.py:81-149) + the unet generator
  int nb = 2, c_id = 512, dt = GHOST_F32, esz = 4;
  std::map<std::string, const void*> slots;   // name -> device pointer (nullptr = unbound)
  int id_total = 0;                            // sum over AAD layers of 2*c_x
  // per-handle plan options (ghost_aei_set_option); defaults are the measured choices
  int opt[GHOST_AEI_NOPT] = {1, 1, 1, GHOST_KNOB("GHOST_AAD_ZP", 2), 1};
  // GHOST_AEI_OPT_TWO_STREAMS: the encoder up path's stream and its events, one set per device (created
  // on first use on the device of the caller's stream): zev[k] = z_attr_k written (k = 2..8), zev[0] = the
  // down path done, zev[1] = idgb / m1 ready; zend = everything this call queued on the up stream
  struct UpPath {
    hipStream_t s = nullptr;
    hipEvent_t zev[9] = {nullptr};
    hipEvent_t zend = nullptr;
  };

  std::map<int, UpPath> up_path;
  hipEvent_t* zev = nullptr;                   // the events of the device of the running call
  void* taps[8] = {nullptr};                   // ghost_aei_set_taps: AADBlk1..7 outputs copied here
  // profiling
  int prof_mask = 0;
  std::vector<hipEvent_t> ev;
  struct Pending { int cls; int e0, e1; double bytes, flops; };
  std::vector<Pending> pend;
  int ev_used = 0;
  ProfClass prof[8];
  // in-kernel clock of the roofline kernel's launches (profiling class 1): per launch a region of per-workgroup
  // start and per-wave end stamps (aad_v3_clock_words); clk_cap words of device buffer, bump-allocated
  unsigned long long* clk = nullptr;
  size_t clk_cap = 0, clk_used = 0;
  int clk_dev = -1;
  std::vector<std::pair<size_t, int>> clk_launch;   // (offset, words) per clocked launch
  int roof_version = 0;                        // kernel generation of class 1's last launch (aad_v3.h)
  unsigned long long* next_clk(int words) {
    if (!clk || words <= 0 || clk_used + (size_t)words > clk_cap) return nullptr;
    clk_launch.push_back({clk_used, words});
    unsigned long long* p = clk + clk_used;
    clk_used += (size_t)words;
    return p;
  }
  void drop_last_clk() {
    if (clk_launch.empty()) return;
    clk_used = clk_launch.back().first;
    clk_launch.pop_back();
  }

  typedef int Pair[2];
  typedef int Triple[3];
  const Pair* up() const { return linknet ? kEncUpLink : kEncUpUnet; }
  const Triple* gen() const { return linknet ? kGenLink : kGenUnet; }
  void attr_geom(int k, int& C, int& H) const {  // k = 1..8
    static const int hs[8] = {2, 4, 8, 16, 32, 64, 128, 256};
    H = hs[k - 1];
    if (k == 1) C = 1024;
    else if (k == 8) C = linknet ? 32 : 64;
    else C = linknet ? up()[k - 2][1] : up()[k - 2][1] * 2;
  }
};

namespace {

// ---------------------------------------------------------------------------
// execution context: dry run (sizing) or real run (launches)
// ---------------------------------------------------------------------------
constexpr int kSemWords = 4096;                  // arrival counters per stream (16 KB)
constexpr size_t kSemBytes = 2 * kSemWords * sizeof(unsigned);   // the main and the up-path stream's sets

struct Ctx {
  ghost_aei* h;
  bool dry;
  char* base;
  size_t off = 0, cap = 0;
  size_t scratch_need = 0;  // max split-K / IN-stats partial bytes
  char* scratch = nullptr;
  size_t scratch_cap = 0;
  hipStream_t s;
  // two-stream plan: the up path's stream and its own scratch region (the launches of the two streams
  // overlap, so they cannot share the split-K / statistics partials)
  bool dual = false, force_single = false;
  int dev = 0;
  hipStream_t s_up = nullptr;
  char* scratch_up = nullptr;
  // arrival counters of the fused reductions (split-K fix-up, InstanceNorm final pass): one set per stream,
  // zeroed once per call before the first launch and left zero by every launch (GHOST_AEI_OPT_FUSE_REDUCE)
  unsigned* sem_main = nullptr;
  unsigned* sem_up = nullptr;
  unsigned* sem() const { return scratch_up && scratch == scratch_up ? sem_up : sem_main; }
  int rc = 0;
  std::string where;

  void* alloc(size_t bytes) {
    off = (off + 255) & ~size_t(255);
    void* p = dry ? reinterpret_cast<void*>(uintptr_t(0x10000000) + off) : base + off;
    off += bytes;
    return p;
  }
  bool ok() const { return rc == 0; }
  void check(int r, const char* what) {
    if (r != 0 && rc == 0) {
      rc = r;
      where = what;
    }
  }
  const void* W(const std::string& name) {
    auto it = h->slots.find(name);
    if (dry) {  // sizing needs no weights, but every slot the plan reads must be declared
      if (it == h->slots.end() && rc == 0) {
        rc = GHOST_EINVAL;
        where = "plan reads undeclared slot " + name;
      }
      return reinterpret_cast<const void*>(uintptr_t(0x1000));
    }
    if (it == h->slots.end() || !it->second) {
      if (rc == 0) {
        rc = GHOST_ENOTREADY;
        where = "unbound weight slot " + name;
      }
      return nullptr;
    }
    return it->second;
  }
  // profiling brackets
  int prof_begin(int cls) {
    if (dry || !(h->prof_mask & (1 << cls))) return -1;
    if (h->ev_used + 2 > (int)h->ev.size()) {
      for (int i = 0; i < 64; ++i) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return -1;
        h->ev.push_back(e);
      }
    }
    int e0 = h->ev_used;
    h->ev_used += 2;
    (void)hipEventRecord(h->ev[e0], s);
    return e0;
  }
  void prof_end(int cls, int e0, double bytes, double flops) {
    if (e0 < 0) return;
    (void)hipEventRecord(h->ev[e0 + 1], s);
    h->pend.push_back({cls, e0, e0 + 1, bytes, flops});
  }
};

// one conv launch (or its workspace accounting in the dry run)
static const bool g_trace = GHOST_KNOB("GHOST_PLAN_TRACE", 0) != 0;   // one stderr line per launch (tuning builds)

void run_conv(Ctx& c, ConvDesc& d, int cls_all, int cls_big, double flops) {
  if (!c.ok()) return;
  if (c.dry) {
    size_t need = conv_workspace_bytes(d);
    if (need > c.scratch_need) c.scratch_need = need;
    return;
  }
  if (g_trace)
    fprintf(stderr, "[plan] conv%s %dx%d/s%d %dx%d %d->%d epi=%d res=%d %.1f GFLOP\n",
            d.kind == CONV_T4S2 ? "T" : "", d.kh, d.kw, d.stride, d.Hi, d.Wi, d.Cin, d.N, (int)d.epi, d.res != nullptr,
            flops / 1e9);
  const bool big = d.Hi == 256 || d.Hi * (d.kind == CONV_T4S2 ? 2 : 1) == 256;
  int e_all = c.prof_begin(cls_all);
  int e_big = (big && cls_big >= 0) ? c.prof_begin(cls_big) : -1;
  d.sem = c.sem();
  d.nsem = d.sem ? kSemWords : 0;
  c.check(conv_launch(d, c.scratch, c.scratch_cap, c.s), "conv_launch");
  double bytes = 0;
  if (d.epi == EPI_AAD) {
    // algorithmic AAD bytes: |h_in| + |z_attr| + |out|
    const double P = (double)d.B * d.Hi * d.Wi;
    bytes = P * (2.0 * d.C_aad + d.Cin) * (double)c.h->esz;
  }
  if (e_big >= 0) c.prof_end(cls_big, e_big, bytes, flops);
  if (e_all >= 0) c.prof_end(cls_all, e_all, bytes, flops);
}

void run_stats(Ctx& c, const void* x, int ldx, int B, int HW, int C, float* stat) {
  if (!c.ok()) return;
  if (c.dry) {
    size_t need = in_stats_workspace_bytes(B, HW, C);
    if (need > c.scratch_need) c.scratch_need = need;
    return;
  }
  int e = c.prof_begin(4);
  unsigned* sem = c.sem();
  c.check(in_stats(c.h->dt, x, ldx, B, HW, C, stat, c.scratch, c.scratch_cap, c.s, sem, sem ? kSemWords : 0),
          "in_stats");
  c.prof_end(4, e, (double)B * HW * C * c.h->esz, 0);
}

// statistics of upsample2x(x) for an [B, H, W, C] source, without materialising it
void run_stats_up(Ctx& c, const void* x, int ldx, int B, int H, int W, int C, float* stat) {
  if (!c.ok()) return;
  if (c.dry) {
    size_t need = in_stats_workspace_bytes(B, 4 * H * W, C);
    if (need > c.scratch_need) c.scratch_need = need;
    return;
  }
  int e = c.prof_begin(4);
  unsigned* sem = c.sem();
  c.check(in_stats_up2x(c.h->dt, x, ldx, B, H, W, C, stat, c.scratch, c.scratch_cap, c.s, sem, sem ? kSemWords : 0),
          "in_stats_up2x");
  c.prof_end(4, e, (double)B * H * W * C * c.h->esz, 0);
}

void run_mask(Ctx& c, const void* x, int ldx, int B, int HW, int C, const float* stat, const float* wh,
              const float* bh, float* mask) {
  if (!c.ok() || c.dry) return;
  int e = c.prof_begin(4);
  c.check(aad_mask(c.h->dt, x, ldx, B, HW, C, stat, wh, bh, mask, c.s), "aad_mask");
  c.prof_end(4, e, (double)B * HW * C * c.h->esz, 0);
}

// small images (2x2 .. 8x8): statistics + the masks of the AADLayers named in `ls` (<= 2) in one launch
void run_stats_masks(Ctx& c, const void* x, int ldx, int B, int HW, int C, float* stat, const std::string* ls, int L,
                     float* masks[2]) {
  const float* wh[2] = {nullptr, nullptr};
  const float* bh[2] = {nullptr, nullptr};
  for (int l = 0; l < L; ++l) {
    wh[l] = (const float*)c.W(ls[l] + ".wh");
    bh[l] = (const float*)c.W(ls[l] + ".bh");
  }
  if (!c.ok() || c.dry) return;
  int e = c.prof_begin(4);
  c.check(stats_mask_small(c.h->dt, x, ldx, B, HW, C, stat, wh[0], bh[0], masks[0], wh[1], bh[1], masks[1], c.s),
          "stats_mask_small");
  c.prof_end(4, e, (double)B * HW * C * c.h->esz, 0);
}

void run_up(Ctx& c, const void* x, int ldx, void* y, int ldy, int B, int H, int W, int C) {
  if (!c.ok() || c.dry) return;
  int e = c.prof_begin(6);
  c.check(upsample2x(c.h->dt, x, ldx, y, ldy, B, H, W, C, c.s), "upsample2x");
  c.prof_end(6, e, (double)B * H * W * C * 5 * c.h->esz, 0);
}

// ---------------------------------------------------------------------------
// encoder (MLAttrEncoder.forward, AEI_Net.py:72-95)
// ---------------------------------------------------------------------------
struct Buf {
  void* p;
  int ld;
};

// one Conv2d + BatchNorm(eval) (+ ReLU) of the resnet encoder; NHWC in/out with channel strides
void res_conv(Ctx& c, const std::string& name, const void* x, int ldx, int B, int H, int Cin, int Cout, int k,
              int stride, void* y, int ldy, bool relu, const void* res = nullptr, int ldres = 0) {
  ghost_aei* h = c.h;
  ConvDesc d;
  d.ti = d.to = h->dt;
  d.x = x; d.B = B; d.Hi = H; d.Wi = H; d.Cin = Cin; d.ldx = ldx;
  d.w = c.W(name + ".w");
  d.N = Cout; d.Npad = rup(Cout, 128); d.Kpad = rup(k * k * Cin, 32);
  d.kind = CONV_FWD; d.kh = d.kw = k; d.stride = stride; d.pad = k / 2;
  d.y = y; d.ldy = ldy;
  d.scale = (const float*)c.W(name + ".scale");
  d.shift = (const float*)c.W(name + ".shift");
  d.slope = relu ? 0.f : 1.f;
  if (res) { d.res = res; d.ldres = ldres; d.res_first = 1; }
  const double Ho = (H + 2 * (k / 2) - k) / stride + 1;
  run_conv(c, d, 5, -1, 2.0 * B * Ho * Ho * Cout * k * k * Cin);
}

// MLAttrEncoderResnet = ResNet(Bottleneck, [2]*6) (resnet.py:81-149): returns
// (x7, x6, x5, x4, x3, x2, x1, x0) = z_attr1..8, the same geometry as the unet encoder
void encoder_resnet(Ctx& c, const void* xin, int B, void* const attr[8]) {
  ghost_aei* h = c.h;
  const int es = h->esz;
  // x0 = relu(bn0(conv0 7x7/s1/p3)) -> z_attr8;  x1 = relu(bn1(conv1 7x7/s2/p3)) -> z_attr7
  res_conv(c, "enc.r.conv0", xin, 4, B, 256, 3, 64, 7, 1, attr[7], 64, true);
  res_conv(c, "enc.r.conv1", attr[7], 64, B, 256, 64, 64, 7, 2, attr[6], 64, true);
  static const int planes_of[6] = {32, 64, 128, 256, 512, 256};
  const void* x = attr[6];
  int C = 64, H = 128;
  for (int li = 1; li <= 6; ++li) {
    const int pl = planes_of[li - 1], co = 4 * pl;
    for (int blk = 0; blk < 2; ++blk) {
      const int stride = blk == 0 ? 2 : 1;
      const int Ho = H / stride;
      const std::string pre = "enc.r.l" + std::to_string(li) + ".b" + std::to_string(blk);
      void* t1 = c.alloc((size_t)B * Ho * Ho * pl * es);
      void* t2 = c.alloc((size_t)B * Ho * Ho * pl * es);
      // Bottleneck.forward (resnet.py:57-78): conv1 1x1/s carries the stride
      res_conv(c, pre + ".c1", x, C, B, H, C, pl, 1, stride, t1, pl, true);
      res_conv(c, pre + ".c2", t1, pl, B, Ho, pl, pl, 3, 1, t2, pl, true);
      const void* res = x;
      if (blk == 0) {
        void* r = c.alloc((size_t)B * Ho * Ho * co * es);
        res_conv(c, pre + ".down", x, C, B, H, C, co, 1, stride, r, co, false);
        res = r;
      }
      void* out = blk == 1 ? attr[6 - li] : c.alloc((size_t)B * Ho * Ho * co * es);
      // relu(bn3(conv3(t2)) + residual)
      res_conv(c, pre + ".c3", t2, pl, B, Ho, pl, co, 1, 1, out, co, true, res, co);
      x = out;
      C = co;
      H = Ho;
    }
  }
}

void encoder(Ctx& c, const void* xin, int B, void* const attr[8]) {
  ghost_aei* h = c.h;
  if (h->resnet) {
    encoder_resnet(c, xin, B, attr);
    return;
  }
  const int es = h->esz;
  // where feat_1..feat_6 live: unet -> inside z_attr_{8-j} after the deconv channels
  Buf feat[7];
  int Hs = 256;
  for (int j = 1; j <= 6; ++j) {
    const int co = kEncDown[j - 1][1];
    if (!h->linknet) {
      int C, H;
      h->attr_geom(8 - j, C, H);
      const int off = h->up()[6 - j][1];  // deconv_{7-j} output channels come first
      feat[j] = {(char*)attr[8 - j - 1] + (size_t)off * es, C};
    } else {
      const int H = 256 >> j;
      feat[j] = {c.alloc((size_t)B * H * H * co * es), co};
    }
  }
  // down path: conv_i = Conv4x4/s2/p1 -> BN -> LReLU(0.1)
  Buf in{const_cast<void*>(xin), 4};
  for (int i = 1; i <= 7; ++i) {
    const int ci = kEncDown[i - 1][0], co = kEncDown[i - 1][1];
    Buf out = i <= 6 ? feat[i] : Buf{attr[0], 1024};
    ConvDesc d;
    d.ti = d.to = h->dt;
    d.x = in.p; d.B = B; d.Hi = Hs; d.Wi = Hs; d.Cin = ci; d.ldx = in.ld;
    d.w = c.W("enc.conv" + std::to_string(i) + ".w");
    d.N = co; d.Npad = rup(co, 128); d.Kpad = rup(16 * ci, 32);
    d.kind = CONV_FWD; d.kh = d.kw = 4; d.stride = 2; d.pad = 1;
    d.y = out.p; d.ldy = out.ld;
    d.scale = (const float*)c.W("enc.conv" + std::to_string(i) + ".scale");
    d.shift = (const float*)c.W("enc.conv" + std::to_string(i) + ".shift");
    d.slope = kBnLrelu;
    const double Ho = Hs / 2;
    run_conv(c, d, 5, -1, 2.0 * B * Ho * Ho * co * 16.0 * ci);
    in = out;
    Hs /= 2;
  }
  // up path: deconv_i = ConvT4x4/s2/p1 -> BN -> LReLU -> cat((x, skip)) | x + skip.  Two-stream plan: it
  // runs on the handle's second stream after the down path, and z_attr_{i+1} is published by an event
  // the generator's AADBlk(i+1) waits for (AADBlk1 reads z_attr1, the down path's last output)
  hipStream_t s_main = c.s;
  char* scr_main = c.scratch;
  const bool dual = c.dual && !c.dry;
  if (dual && c.ok()) {
    c.check((int)hipEventRecord(h->zev[0], c.s), "event record");
    c.check((int)hipStreamWaitEvent(c.s_up, h->zev[0], 0), "stream wait");
    c.s = c.s_up;
    c.scratch = c.scratch_up;
  }
  for (int i = 1; i <= 6; ++i) {
    int Cin, H, Cout, Ho;
    h->attr_geom(i, Cin, H);
    h->attr_geom(i + 1, Cout, Ho);
    const int co = h->up()[i - 1][1];
    ConvDesc d;
    d.ti = d.to = h->dt;
    d.x = attr[i - 1]; d.B = B; d.Hi = H; d.Wi = H; d.Cin = Cin; d.ldx = Cin;
    d.w = c.W("enc.deconv" + std::to_string(i) + ".w");
    d.N = co; d.Npad = rup(co, 128); d.Kpad = rup(4 * Cin, 32);
    d.kind = CONV_T4S2;
    d.y = attr[i]; d.ldy = Cout;
    d.scale = (const float*)c.W("enc.deconv" + std::to_string(i) + ".scale");
    d.shift = (const float*)c.W("enc.deconv" + std::to_string(i) + ".shift");
    d.slope = kBnLrelu;
    if (h->linknet) { d.res = feat[7 - i].p; d.ldres = feat[7 - i].ld; }
    run_conv(c, d, 5, -1, 2.0 * B * Ho * Ho * co * 4.0 * Cin);
    if (dual && c.ok()) c.check((int)hipEventRecord(h->zev[i + 1], c.s), "event record");
  }
  int C7, H7, C8, H8;
  h->attr_geom(7, C7, H7);
  h->attr_geom(8, C8, H8);
  run_up(c, attr[6], C7, attr[7], C8, B, H7, H7, C7);   // z_attr8 = F.interpolate(z_attr7) (AEI_Net.py:94)
  if (dual) {
    if (c.ok()) c.check((int)hipEventRecord(h->zev[8], c.s), "event record");
    c.s = s_main;
    c.scratch = scr_main;
  }
}

// ---------------------------------------------------------------------------
// generator (AADGenerator.forward, AEI_Net.py:122-139)
// ---------------------------------------------------------------------------
struct GenShared {
  const float* zid32;
  float* idgb;
};

// one AADLayer (+ fused ReLU) -> out
void aad(Ctx& c, const std::string& name, const void* hin, int ldh, const float* stat, const void* za, int lda,
         int Ca, int B, int n, int C, int id_off, const float* idgb, void* out, int ldo,
         const float* pre_mask = nullptr) {
  ghost_aei* h = c.h;
  const double P = (double)B * n * n;
  const double bytes = P * (2.0 * C + Ca) * (double)h->esz;   // |h_in| + |z_attr| + |out|
  const double flops = 2.0 * P * 2.0 * C * Ca;
  const void* gbw = c.W(name + ".gbw");
  const float* gbb = (const float*)c.W(name + ".gbb");
  const float* wh = (const float*)c.W(name + ".wh");
  const float* bh = (const float*)c.W(name + ".bh");
  if (aad_fused_supported(h->dt, B, n * n, C, Ca, lda, ldh, ldo)) {
    if (!c.ok() || c.dry) return;
    int e_all = c.prof_begin(0);
    int e_big = -1;
    c.check(aad_fused(h->dt, za, lda, Ca, gbw, rup(Ca, 32), gbb, hin, ldh, stat, wh, bh, idgb + id_off, h->id_total,
                      out, ldo, B, n * n, C, 0.0f, c.s),
            "aad_fused");
    if (e_big >= 0) c.prof_end(1, e_big, bytes, flops);
    if (e_all >= 0) c.prof_end(0, e_all, bytes, flops);
    return;
  }
  const float* mask = pre_mask;
  if (!mask) {
    float* m = (float*)c.alloc((size_t)B * n * n * sizeof(float));
    run_mask(c, hin, ldh, B, n * n, C, stat, wh, bh, m);
    mask = m;
  }
  ConvDesc d;
  d.ti = d.to = h->dt;
  d.x = za; d.B = B; d.Hi = n; d.Wi = n; d.Cin = Ca; d.ldx = lda;
  d.w = gbw;
  d.N = 2 * C; d.Npad = rup(2 * C, 128); d.Kpad = rup(Ca, 32);
  d.kind = CONV_FWD; d.kh = d.kw = 1; d.stride = 1; d.pad = 0;
  d.y = out; d.ldy = ldo;
  d.shift = gbb;
  d.slope = 0.0f;  // the ReLU that follows every AADLayer in AddBlocksSequential
  d.epi = EPI_AAD;
  d.hin = hin; d.ldh = ldh; d.stat = stat;
  d.idgb = idgb ? idgb + id_off : nullptr; d.id_ld = h->id_total; d.mask = mask; d.C_aad = C;
  run_conv(c, d, 0, -1, flops);
}

struct AadOut {
  std::string name;
  int id_off;
  void* out;
  int ldo;
  const void* zw = nullptr;   // tap partials (aad_v3.h): out is then the row-summed buffer of tap_rows.h
  int zwld = 0;
};

// AADLayers that read the same h_in / z_attr: the register-epilogue kernel takes up to two at
// once (one pass over the inputs); other shapes run one fused / split AAD kernel per layer
// up_src: h_in is upsample2x of the [B, n/2, n/2] tensor hin (the through-upsample AAD kernel)
// pre_masks: the layers' masks when the statistics pass produced them (run_stats_masks)
void aad_group(Ctx& c, const std::vector<AadOut>& ls, const void* hin, int ldh, const float* stat, const void* za,
               int lda, int Ca, int B, int n, int C, const float* idgb, bool up_src = false,
               float* const* pre_masks = nullptr) {
  ghost_aei* h = c.h;
  bool v3 = aad_v3_supported(h->dt, B, n * n, C, Ca, lda, ldh, 8);
  for (auto& l : ls) v3 = v3 && l.ldo % 8 == 0;
  if (up_src && !v3) {
    c.check(GHOST_EINVAL, "aad_group: through-upsample input needs the v3 kernel");
    return;
  }
  if (!v3) {
    bool wide = aad_wide_supported(h->dt, B, n * n, C, Ca, lda, ldh, 8) && ls.size() <= 2;
    for (auto& l : ls) wide = wide && l.ldo % 8 == 0;
    // the masks of every layer of the group from one pass over h_in
    float* masks[2] = {nullptr, nullptr};
    if (wide && pre_masks) {
      masks[0] = pre_masks[0];
      masks[1] = pre_masks[1];
    } else if (wide) {
      for (size_t i = 0; i < ls.size(); ++i) masks[i] = (float*)c.alloc((size_t)B * n * n * sizeof(float));
      const float* wh0 = (const float*)c.W(ls[0].name + ".wh");
      const float* bh0 = (const float*)c.W(ls[0].name + ".bh");
      const float* wh1 = ls.size() > 1 ? (const float*)c.W(ls[1].name + ".wh") : nullptr;
      const float* bh1 = ls.size() > 1 ? (const float*)c.W(ls[1].name + ".bh") : nullptr;
      if (c.ok() && !c.dry) {
        int e = c.prof_begin(4);
        c.check(aad_mask2(h->dt, hin, ldh, B, n * n, C, stat, wh0, bh0, masks[0], wh1, bh1, masks[1], c.s),
                "aad_mask2");
        c.prof_end(4, e, (double)B * n * n * C * h->esz, 0);
      }
    }
    for (size_t li = 0; li < ls.size(); ++li) {
      const AadOut& l = ls[li];
      if (!wide) {
        aad(c, l.name, hin, ldh, stat, za, lda, Ca, B, n, C, l.id_off, idgb, l.out, l.ldo,
            pre_masks ? pre_masks[li] : nullptr);
        continue;
      }
      AadWideDesc d;
      d.dt = h->dt;
      d.za = za; d.lda = lda; d.Ca = Ca; d.hin = hin; d.ldh = ldh; d.stat = stat;
      d.B = B; d.HW = n * n; d.C = C; d.id_ld = h->id_total; d.slope = 0.0f;   // + the ReLU that follows
      d.w3 = c.W(l.name + ".w3");
      d.b3 = (const float*)c.W(l.name + ".b3");
      d.wh = (const float*)c.W(l.name + ".wh");
      d.bh = (const float*)c.W(l.name + ".bh");
      d.idgb = idgb ? idgb + l.id_off : nullptr;
      d.out = l.out; d.ldo = l.ldo;
      d.mask = masks[li];
      if (!c.ok() || c.dry) continue;
      const double Pn = (double)B * n * n;
      int e_all = c.prof_begin(0);
      c.check(aad_wide(d, c.s), "aad_wide");
      if (e_all >= 0) c.prof_end(0, e_all, Pn * (2.0 * C + Ca) * h->esz, 2.0 * Pn * 2.0 * C * Ca);
    }
    return;
  }
  // AADBlk7's block-input pair (C = 128, Ca = 64; h_in materialised or sampled through the upsample) in one
  // kernel: measured B = 64, 258 vs 2 x 141 us materialised (GHOST_AAD_PAIR128=0: one layer per kernel)
  static const int pair128 = GHOST_KNOB("GHOST_AAD_PAIR128", 1);
  const size_t lmax = (C == 64 || (pair128 && C == 128 && Ca == 64)) ? 2 : 1;
  for (size_t i0 = 0; i0 < ls.size(); i0 += lmax) {
    AadV3Desc d;
    d.dt = h->dt;
    d.za = za; d.lda = lda; d.Ca = Ca; d.hin = hin; d.ldh = ldh; d.stat = stat;
    d.B = B; d.HW = n * n; d.C = C; d.id_ld = h->id_total; d.slope = 0.0f;   // + the ReLU that follows
    d.L = (int)std::min(lmax, ls.size() - i0);
    if (up_src) d.up_H = d.up_W = n / 2;
    for (int l = 0; l < d.L; ++l) {
      const AadOut& o = ls[i0 + l];
      d.w3[l] = c.W(o.name + ".w3");
      d.b3[l] = (const float*)c.W(o.name + ".b3");
      d.wh[l] = (const float*)c.W(o.name + ".wh");
      d.bh[l] = (const float*)c.W(o.name + ".bh");
      d.idgb[l] = idgb ? idgb + o.id_off : nullptr;
      d.out[l] = o.out;
      d.ldo[l] = o.ldo;
      d.zw[l] = o.zw;
      if (o.zw) d.zwld = o.zwld;
    }
    if (!c.ok() || c.dry) continue;
    const double Pn = (double)B * n * n;
    // algorithmic bytes by SURVEY.md §8d's formula, fixed regardless of fusion:
    // sum over the L AADLayers of |h_in| + |z_attr| + |out| (PMC traffic shows what fusion saves)
    const double bytes = Pn * (double)d.L * (2.0 * C + Ca) * h->esz;
    const double flops = 2.0 * Pn * 2.0 * C * Ca * d.L;
    if (g_trace)
      fprintf(stderr, "[plan] aad_v3 %dx%d C=%d Ca=%d L=%d up=%d\n", n, n, C, Ca, d.L, (int)up_src);
    int e_all = c.prof_begin(0);
    // class 1: the block-input AAD kernel at 256x256 (reads h_in through the x2 upsample; one or two layers)
    int e_big = (n == 256 && up_src) ? c.prof_begin(1) : -1;
    if (e_big >= 0 && h->clk_dev == c.dev) d.tclk = h->next_clk(aad_v3_clock_words(d));
    if (e_big >= 0) d.version_out = &h->roof_version;
    c.check(aad_v3(d, c.s), "aad_v3");
    // only the v4 / v5 kernels write clock stamps: a launch that fell back to v3 gives its region back, so
    // ghost_aei_profile_clock never reads unwritten words
    if (d.tclk && h->roof_version != 4 && h->roof_version != 5) h->drop_last_clk();
    if (e_big >= 0) c.prof_end(1, e_big, bytes, flops);
    if (e_all >= 0) c.prof_end(0, e_all, bytes, flops);
  }
}

// returns true when `stat` (if given) was produced from partials written by the conv itself
bool conv3x3(Ctx& c, const std::string& wname, const void* x, int ldx, int Cin, int B, int n, int Cout, void* y,
             int ldy, const void* res, int ldres, int tanh_out, uint8_t* u8, float* stat = nullptr) {
  const double flops = 2.0 * B * n * n * Cout * 9.0 * Cin;
  if (Cout <= 3 && conv3x3_narrow_supported(c.h->dt, n, n, Cin, ldx, Cout)) {
    const void* wn = c.W(wname + "n");   // "...conv{i}.w" + "n" = the narrow layout slot
    if (!c.ok() || c.dry) return false;
    int e_all = c.prof_begin(2);
    int e_big = n == 256 ? c.prof_begin(3) : -1;
    c.check(conv3x3_narrow(c.h->dt, x, B, n, n, Cin, ldx, wn, rup(Cin, 32), Cout, res, ldres, tanh_out, y, ldy, u8, c.s),
            "conv3x3_narrow");
    if (e_big >= 0) c.prof_end(3, e_big, 0, flops);
    if (e_all >= 0) c.prof_end(2, e_all, 0, flops);
    return false;
  }
  ConvDesc d;
  d.ti = d.to = c.h->dt;
  d.x = x; d.B = B; d.Hi = n; d.Wi = n; d.Cin = Cin; d.ldx = ldx;
  d.w = c.W(wname);
  d.N = Cout; d.Npad = rup(Cout, 128); d.Kpad = rup(9 * Cin, 32);
  d.kind = CONV_FWD; d.kh = d.kw = 3; d.stride = 1; d.pad = 1;
  d.y = y; d.ldy = ldy;
  d.res = res; d.ldres = ldres;
  d.tanh_out = tanh_out; d.u8 = u8;
  int nrec = 0;
  const bool fused = stat && c.h->opt[GHOST_AEI_OPT_FUSE_STATS] && conv3x3_pp_takes(d, &nrec);
  if (fused) d.in_part = (float*)c.alloc((size_t)B * nrec * Cout * 2 * sizeof(float));
  run_conv(c, d, 2, 3, flops);
  if (fused && c.ok() && !c.dry) {
    int e = c.prof_begin(4);
    c.check(in_stats_from_tiles(d.in_part, B, nrec, Cout, stat, c.s), "in_stats_from_tiles");
    c.prof_end(4, e, 0, 0);
  }
  return fused;
}

// identity projections of every AADLayer at once (idgb) and up1 (m1): they read z_id only, so the
// two-stream plan runs them on the up-path stream while the encoder's down path runs
struct GenIn {
  float* idgb;
  void* m;
};

// idgb_out / m_out: where to write them (the identity table of ghost_aei_identity_table), else the workspace
GenIn generator_prologue(Ctx& c, int B, const float* zid32, float* idgb_out = nullptr, void* m_out = nullptr) {
  ghost_aei* h = c.h;
  const int es = h->esz;
  // identity projections of every AADLayer at once: idgb[b] = [gamma_id | beta_id] per layer (fc1/fc2)
  float* idgb = idgb_out ? idgb_out : (float*)c.alloc((size_t)B * h->id_total * sizeof(float));
  {
    ConvDesc d;
    d.ti = d.to = GHOST_F32;
    d.x = zid32; d.B = B; d.Hi = 1; d.Wi = 1; d.Cin = h->c_id; d.ldx = h->c_id;
    d.w = c.W("gen.id.w");
    d.N = h->id_total; d.Npad = rup(h->id_total, 128); d.Kpad = rup(h->c_id, 32);
    d.y = idgb; d.ldy = h->id_total;
    d.shift = (const float*)c.W("gen.id.shift");
    run_conv(c, d, 7, -1, 2.0 * B * h->id_total * h->c_id);
  }
  // m1 = up1(z_id): ConvT k2 on a 1x1 input == GEMM to [B, 2, 2, 1024] (AEI_Net.py:101,123)
  void* m = m_out ? m_out : c.alloc((size_t)B * 4 * 1024 * es);
  {
    ConvDesc d;
    d.ti = GHOST_F32; d.to = h->dt;
    d.x = zid32; d.B = B; d.Hi = 1; d.Wi = 1; d.Cin = h->c_id; d.ldx = h->c_id;
    d.w = c.W("gen.up1.w");
    d.N = 4096; d.Npad = 4096; d.Kpad = rup(h->c_id, 32);
    d.y = m; d.ldy = 4096;
    d.shift = (const float*)c.W("gen.up1.shift");
    run_conv(c, d, 7, -1, 2.0 * B * 4096 * h->c_id);
  }
  return {idgb, m};
}

void generator(Ctx& c, int B, const void* const attr[8], GenIn gin, void* y_out, uint8_t* u8) {
  ghost_aei* h = c.h;
  const int es = h->esz;
  const int nb = h->nb;
  float* idgb = gin.idgb;
  void* m = gin.m;
  if (c.dual && !c.dry && c.ok())   // idgb and m1 come from the up-path stream
    c.check((int)hipStreamWaitEvent(c.s, h->zev[1], 0), "stream wait");
  int id_off = 0;
  bool m_virtual = false;   // m is not materialised: h_in = upsample2x(m) at n x n (m is n/2 x n/2)
  const void* m_src = nullptr;   // m = upsample2x(m_src) materialised: its statistics come from the source
  for (int k = 1; k <= 8; ++k) {
    const int cin = h->gen()[k - 1][0], cout = h->gen()[k - 1][1];
    int Ca, n;
    h->attr_geom(k, Ca, n);
    const void* za = attr[k - 1];
    if (c.dual && !c.dry && k >= 2 && c.ok())   // z_attr_k comes from the encoder's up-path stream
      c.check((int)hipStreamWaitEvent(c.s, h->zev[k], 0), "stream wait");
    const std::string blk = "gen.blk" + std::to_string(k);
    const size_t P = (size_t)B * n * n;
    const bool last_k = k == 8;
    const bool split = cin != cout;          // AAD_ResBlk has a last_add_block (AADLayer.py:68-72)
    const int base = id_off;                  // idgb offset of this block's first AADLayer
    float* stat_m = (float*)c.alloc((size_t)B * cin * 2 * sizeof(float));
    // 2x2 and 4x4: statistics and the AAD masks of each layer group from one launch per group
    const bool small = !m_virtual && h->opt[GHOST_AEI_OPT_FUSE_STATS] && stats_mask_small_ok(h->dt, n * n, cin, cin);
    float* gmask[2] = {nullptr, nullptr};
    auto small_masks = [&](const void* xin, float* st, int i) {
      std::string ln[2] = {blk + ".aad" + std::to_string(i), blk + ".aadlast"};
      const int L = (i == 0 && split) ? 2 : 1;
      for (int l = 0; l < L; ++l) gmask[l] = (float*)c.alloc((size_t)B * n * n * sizeof(float));
      gmask[1] = L > 1 ? gmask[1] : nullptr;
      run_stats_masks(c, xin, cin, B, n * n, cin, st, ln, L, gmask);
    };
    if (small)
      small_masks(m, stat_m, 0);
    else if (m_virtual)
      run_stats_up(c, m, cin, B, n / 2, n / 2, cin, stat_m);
    else if (m_src && in_stats_up2x_closed_form(h->dt, n / 2, n / 2, cin, cin))
      run_stats_up(c, m_src, cin, B, n / 2, n / 2, cin, stat_m);   // one pass over the 4x smaller source
    else
      run_stats(c, m, cin, B, n * n, cin, stat_m);
    void* y = last_k ? y_out : c.alloc(P * cout * es);
    // x-branch and h'-branch share the output conv: conv(cat(a_x, a_h), [W_x | W_h]) = x + h'
    // AADBlk8 (cout = 3) with tap partials (GHOST_AEI_OPT_TAP_PARTIALS): the AADLayers feeding that conv write
    // its per-tap partial sums instead of their channels (zh: the h path, zx: last_add_block's x')
    const int zp = (last_k && split && cin == 64 && cout == 3 && is16(h->dt))
                       ? h->opt[GHOST_AEI_OPT_TAP_PARTIALS] : 0;
    const char* wn = zp ? (const char*)c.W(blk + ".conv" + std::to_string(nb - 1) + ".wn") : nullptr;
    const int wnld = rup(2 * cin, 32);
    void* zh = zp ? c.alloc(P * kZrPerPixel * 2) : nullptr;   // row-summed partials (tap_rows.h)
    void* zx = zp == 2 ? c.alloc(P * kZrPerPixel * 2) : nullptr;
    void* xq = zp == 1 ? c.alloc(P * cin * es) : nullptr;   // x' alone (the narrow conv contracts it)
    void* cat = (split && !zp) ? c.alloc(P * 2 * cin * es) : nullptr;
    const void* x = m;
    const float* stat_x = stat_m;
    for (int i = 0; i < nb; ++i) {
      const bool last = i == nb - 1;
      const std::string cn = blk + ".conv" + std::to_string(i) + ".w";
      std::vector<AadOut> group;
      if (zp && last) {
        AadOut o{blk + ".aad" + std::to_string(i), base + 2 * cin * i, zh, 32};
        o.zw = wn; o.zwld = wnld;
        group.push_back(o);
      } else {
        void* a = (last && split) ? cat : c.alloc(P * cin * es);
        const int lda_out = (last && split) ? 2 * cin : cin;
        group.push_back({blk + ".aad" + std::to_string(i), base + 2 * cin * i, a, lda_out});
      }
      if (i == 0 && split) {   // last_add_block's AADLayer reads the block input m as well
        if (zp == 2) {
          AadOut o{blk + ".aadlast", base + 2 * cin * nb, zx, 32};
          o.zw = wn + (size_t)cin * h->esz; o.zwld = wnld;   // the x' half of the K range
          group.push_back(o);
        } else if (zp == 1) {
          group.push_back({blk + ".aadlast", base + 2 * cin * nb, xq, cin});
        } else {
          group.push_back({blk + ".aadlast", base + 2 * cin * nb, (char*)cat + (size_t)cin * es, 2 * cin});
        }
      }
      aad_group(c, group, x, cin, stat_x, za, Ca, Ca, B, n, cin, idgb, i == 0 && m_virtual, small ? gmask : nullptr);
      void* a = group[0].out;
      if (!last) {
        void* xn = c.alloc(P * cin * es);
        float* st = (float*)c.alloc((size_t)B * cin * 2 * sizeof(float));
        // the persistent conv writes the InstanceNorm partials of its output in its epilogue
        // (one pass less over xn); other conv kernels: a separate statistics pass
        if (small) {
          conv3x3(c, cn, a, cin, cin, B, n, cin, xn, cin, nullptr, 0, 0, nullptr, nullptr);
          small_masks(xn, st, i + 1);
        } else if (!conv3x3(c, cn, a, cin, cin, B, n, cin, xn, cin, nullptr, 0, 0, nullptr, st)) {
          run_stats(c, xn, cin, B, n * n, cin, st);
        }
        x = xn;
        stat_x = st;
      } else if (!split) {
        conv3x3(c, cn, a, cin, cin, B, n, cout, y, cout, m, cin, last_k, last_k ? u8 : nullptr);
      } else if (zp == 2) {
        if (c.ok() && !c.dry) {
          int e_all = c.prof_begin(2);
          c.check(tap_sum3x3(h->dt, zh, zx, B, n, n, y, cout, u8, c.s), "tap_sum3x3");
          c.prof_end(2, e_all, 0, 0);
        }
      } else if (zp == 1) {
        if (c.ok() && !c.dry) {
          int e_all = c.prof_begin(2);
          c.check(conv3x3_narrow(h->dt, xq, B, n, n, cin, cin, wn + (size_t)cin * h->esz, wnld, cout, nullptr, 0, 1, y, cout, u8, c.s,
                                 zh),
                  "conv3x3_narrow + tap partials");
          c.prof_end(2, e_all, 0, 2.0 * P * cout * 9.0 * cin);
        }
      } else {
        conv3x3(c, cn, cat, 2 * cin, 2 * cin, B, n, cout, y, cout, nullptr, 0, last_k, last_k ? u8 : nullptr);
      }
    }
    id_off = base + 2 * cin * nb + (split ? 2 * cin : 0);
    if (!last_k && h->taps[k - 1] && c.ok() && !c.dry)   // diagnostic copy of the block output (parity bisection)
      c.check((int)hipMemcpyAsync(h->taps[k - 1], y, P * cout * es, hipMemcpyDeviceToDevice, c.s), "tap copy");
    if (!last_k) {
      // AADBlk(k+1) reads its input m only through the first AADLayer pair and the statistics
      // when cin != cout: those sample the upsample on the fly and m is never written
      int Ca_n, n_n;
      h->attr_geom(k + 1, Ca_n, n_n);
      const int cout_n = h->gen()[k][1];
      // C = 64 (AADBlk8), and C = 128 (AADBlk7) where its pair runs as one dual-layer kernel (Ca = 64): two
      // single-layer kernels re-reading the upsample cost more (+110 us) than the materialised upsample they
      // replace (-85 us), measured B = 64
      static const int up128 = GHOST_KNOB("GHOST_FUSE_UP128", 1);
      const bool fuse = h->opt[GHOST_AEI_OPT_FUSE_UPSAMPLE] && cout != cout_n && Ca_n % 32 == 0 &&
                        (cout == 64 || (up128 && cout == 128 && Ca_n == 64)) &&
                        aad_v3_supported(h->dt, B, n_n * n_n, cout, Ca_n, Ca_n, cout, 8);
      if (fuse) {
        m = y;
        m_src = nullptr;
        m_virtual = true;
      } else {
        void* mn = c.alloc((size_t)B * 4 * n * n * cout * es);
        run_up(c, y, cout, mn, cout, B, n, n, cout);
        m = mn;
        m_src = y;
        m_virtual = false;
      }
    }
  }
}

int check_handle(ghost_aei* h) {
  if (!h) return fail(GHOST_EINVAL, "null handle");
  for (auto& kv : h->slots)
    if (!kv.second) return fail(GHOST_ENOTREADY, "unbound weight slot " + kv.first);
  return 0;
}

void declare_slots(ghost_aei* h) {
  auto add = [&](const std::string& s) { h->slots[s] = nullptr; };
  auto add_conv = [&](const std::string& s) { add(s + ".w"); add(s + ".scale"); add(s + ".shift"); };
  if (h->resnet) {
    add_conv("enc.r.conv0");
    add_conv("enc.r.conv1");
    for (int li = 1; li <= 6; ++li)
      for (int blk = 0; blk < 2; ++blk) {
        const std::string pre = "enc.r.l" + std::to_string(li) + ".b" + std::to_string(blk);
        add_conv(pre + ".c1"); add_conv(pre + ".c2"); add_conv(pre + ".c3");
        if (blk == 0) add_conv(pre + ".down");
      }
  }
  for (int i = 1; i <= 7 && !h->resnet; ++i) {
    add("enc.conv" + std::to_string(i) + ".w");
    add("enc.conv" + std::to_string(i) + ".scale");
    add("enc.conv" + std::to_string(i) + ".shift");
  }
  for (int i = 1; i <= 6 && !h->resnet; ++i) {
    add("enc.deconv" + std::to_string(i) + ".w");
    add("enc.deconv" + std::to_string(i) + ".scale");
    add("enc.deconv" + std::to_string(i) + ".shift");
  }
  add("gen.up1.w"); add("gen.up1.shift"); add("gen.id.w"); add("gen.id.shift");
  h->id_total = 0;
  for (int k = 1; k <= 8; ++k) {
    const int cin = h->gen()[k - 1][0], cout = h->gen()[k - 1][1];
    const std::string blk = "gen.blk" + std::to_string(k);
    int Ca_k, n_k;
    h->attr_geom(k, Ca_k, n_k);
    // permuted register-epilogue AAD layouts (pack.py pack_aad_v3): aad_v3 for C in {64, 128},
    // aad_wide for C in {256, 512, 1024} with Ca <= 512
    const bool v3 = is16(h->dt) && (cin == 64 || cin == 128 ||
                                            ((cin == 256 || cin == 512 || cin == 1024) && Ca_k <= 512));
    for (int i = 0; i < h->nb; ++i) {
      const std::string an = blk + ".aad" + std::to_string(i);
      add(an + ".gbw"); add(an + ".gbb"); add(an + ".wh"); add(an + ".bh");
      if (v3) { add(an + ".w3"); add(an + ".b3"); }
      add(blk + ".conv" + std::to_string(i) + ".w");
      if (i == h->nb - 1 && cout <= 3) add(blk + ".conv" + std::to_string(i) + ".wn");
      h->id_total += 2 * cin;
    }
    if (cin != cout) {
      const std::string an = blk + ".aadlast";
      add(an + ".gbw"); add(an + ".gbb"); add(an + ".wh"); add(an + ".bh");
      if (v3) { add(an + ".w3"); add(an + ".b3"); }
      h->id_total += 2 * cin;
    }
  }
}

// shared driver for forward / get_attr / swap / the identity table
enum Mode { M_FORWARD, M_ATTR, M_SWAP, M_IDTABLE };

struct Io {
  const void* xt = nullptr; int xt_dtype = 0; int64_t st[4] = {0, 0, 0, 0};
  const uint8_t* crops = nullptr; int64_t crop_bs = 0;
  const void* zid = nullptr; int zid_dtype = 0; int64_t zid_rs = 0;
  void* y = nullptr; uint8_t* u8 = nullptr;
  void* attr[8] = {nullptr};
  // identity table (M_IDTABLE writes it; a swap with table != nullptr gathers its rows by idx instead of projecting
  // z_id): n_ident rows of idgb (id_total fp32) then n_ident rows of m1 (4096 in the handle dtype)
  void* table = nullptr; int n_ident = 0; const int32_t* idx = nullptr;
};

// the identity table's layout: [n][id_total] fp32 gamma_id/beta_id rows (256-aligned block), then [n][4096] m1 rows
size_t table_idgb_bytes(const ghost_aei* h, int n) { return ((size_t)n * h->id_total * 4 + 255) & ~size_t(255); }
size_t table_bytes(const ghost_aei* h, int n) { return table_idgb_bytes(h, n) + (size_t)n * 4096 * h->esz; }

void plan(Ctx& c, Mode mode, int B, Io io) {
  ghost_aei* h = c.h;
  const int es = h->esz;
  if (mode == M_IDTABLE) {
    // the per-identity table: B = identities; the same fp32 z rows and GEMMs as a swap's prologue, written into the
    // table instead of the workspace (AADLayer.py:28-29 fc1/fc2 and AEI_Net.py:101 up1 on each source embedding once)
    float* z32 = (float*)c.alloc((size_t)B * h->c_id * sizeof(float));
    if (!c.dry && c.ok()) c.check(rows_to_f32(io.zid_dtype, io.zid, io.zid_rs, B, h->c_id, z32, c.s), "rows_to_f32");
    generator_prologue(c, B, z32, (float*)io.table, io.table ? (char*)io.table + table_idgb_bytes(h, B) : nullptr);
    return;
  }
  void* attr[8];
  for (int k = 1; k <= 8; ++k) {
    int C, H;
    h->attr_geom(k, C, H);
    attr[k - 1] = (mode == M_SWAP) ? c.alloc((size_t)B * H * H * C * es) : io.attr[k - 1];
  }
  // network input NHWC with a zero fourth channel: 8-byte (bf16) pixels for the first conv
  void* xin = c.alloc((size_t)B * 256 * 256 * 4 * es);
  if (!c.dry && c.ok()) {
    if (mode == M_SWAP)
      c.check(crops_u8_to_input(io.crops, io.crop_bs, B, 256, 256, h->dt, xin, c.s, 4, c.sem_main,
                                c.sem_main ? 2 * kSemWords : 0), "crops_u8_to_input");
    else
      c.check(input_to_nhwc(io.xt_dtype, io.xt, io.st, B, 3, 256, 256, h->dt, xin, c.s, 4), "input_to_nhwc");
  }
  // the resnet encoder and get_attr run on one stream; the dry run sizes a second scratch region.  Below 8 frames
  // the plan stays on one stream: at B = 1 the up path's kernels are a few microseconds each and the cross-stream
  // event hand-offs cost more than the overlap returns — eager B = 1 bf16 took 2.40-2.48 ms with the second stream
  // on two of three boxes against 1.72-1.80 on one stream on all three (bench config1_latency, round 4)
  c.dual = h->opt[GHOST_AEI_OPT_TWO_STREAMS] && mode != M_ATTR && !h->resnet && !c.force_single && B >= 8;
  GenIn gin{};
  float* zid32 = nullptr;
  auto prologue = [&]() {
    zid32 = (float*)c.alloc((size_t)B * h->c_id * sizeof(float));
    if (io.table) {
      // per-sample rows of the identity table (one gather launch instead of z -> fp32 and the two projection
      // GEMMs); the same allocations as the projecting prologue, so the swap workspace size covers both
      gin.idgb = (float*)c.alloc((size_t)B * h->id_total * sizeof(float));
      gin.m = c.alloc((size_t)B * 4 * 1024 * es);
      if (c.dry || !c.ok()) return;
      const void* tab[2] = {io.table, (const char*)io.table + table_idgb_bytes(h, io.n_ident)};
      const int64_t rb[2] = {(int64_t)h->id_total * 4, (int64_t)4096 * es};
      void* outs[2] = {gin.idgb, gin.m};
      int e = c.prof_begin(7);
      c.check(gather_identity_rows(2, tab, rb, outs, io.n_ident, io.idx, B, c.s), "gather_identity_rows");
      c.prof_end(7, e, (double)B * (rb[0] + rb[1]) * 2, 0);
      return;
    }
    if (!c.dry && c.ok()) c.check(rows_to_f32(io.zid_dtype, io.zid, io.zid_rs, B, h->c_id, zid32, c.s), "rows_to_f32");
    gin = generator_prologue(c, B, zid32);
  };
  // the identity table's gather runs on the caller's stream, first: identity_index may be a temporary the caller
  // frees stream-ordered on that stream right after this call
  if (mode != M_ATTR && io.table) prologue();
  if (mode != M_ATTR && c.dual) {
    // up-path stream: z_id -> idgb, m1 first (overlapping the down path), then the encoder's up path
    hipStream_t s_main = c.s;
    char* scr_main = c.scratch;
    if (!c.dry) {
      if (c.ok()) c.check((int)hipEventRecord(h->zev[1], s_main), "event record");
      if (c.ok()) c.check((int)hipStreamWaitEvent(c.s_up, h->zev[1], 0), "stream wait");
      c.s = c.s_up;
      c.scratch = c.scratch_up;
    }
    if (!io.table) prologue();
    if (!c.dry) {
      if (c.ok()) c.check((int)hipEventRecord(h->zev[1], c.s), "event record");
      c.s = s_main;
      c.scratch = scr_main;
    }
  }
  encoder(c, xin, B, attr);
  if (mode == M_ATTR) return;
  if (!c.dual && !io.table) prologue();
  void* y = (mode == M_SWAP) ? c.alloc((size_t)B * 256 * 256 * 3 * es) : io.y;
  generator(c, B, attr, gin, y, io.u8);
  // the caller's stream waits for everything this call queued on the up-path stream, also when a launch
  // failed midway (a fresh record: zev[8] may still hold the previous call's record then)
  if (c.dual && !c.dry) {
    const bool rec = hipEventRecord(h->up_path[c.dev].zend, c.s_up) == hipSuccess;
    if (rec) (void)hipStreamWaitEvent(c.s, h->up_path[c.dev].zend, 0);
    else (void)hipStreamSynchronize(c.s_up);
  }
}

// the one-stream fallback of a two-stream plan allocates in another order: alignment padding may differ
constexpr size_t kMainSlack = 64 * 256;

int64_t plan_bytes(ghost_aei* h, Mode mode, int B) {
  Ctx c{};
  c.h = h; c.dry = true;
  Io io;
  uintptr_t fake = 0x20000000;
  for (int k = 0; k < 8; ++k) io.attr[k] = (void*)(fake + k * 0x100000);
  io.y = (void*)(fake + 0x1000000);
  // the table the real M_IDTABLE run writes (so the sizing pass allocates exactly what that run allocates)
  if (mode == M_IDTABLE) io.table = (void*)(fake + 0x2000000);
  plan(c, mode, B, io);
  if (!c.ok()) return (int64_t)c.rc;
  const size_t scr = (c.scratch_need + 255) & ~size_t(255);
  return (int64_t)(((c.off + 255) & ~size_t(255)) + kMainSlack + kSemBytes + (c.dual ? 2 : 1) * scr + 256);
}

// The up-path stream of device `dev`: ONE per device for the whole process, shared by every handle and never
// destroyed.  A process gets 4 hardware queues per priority; streams created and destroyed with each handle (a
// bench leg's second model, a GraphedSwap's runtime) churned that pool, and the D2H / video legs that ran after
// such a leg lost the two-batch overlap (-14 %, tools/leg_probe.py).  The handles' up-path
// work serialises on the shared stream, which it already did for the two batches in flight of one handle; every
// call orders itself against it with its own events.  nullptr: creation failed (the calls run on one stream).
hipStream_t shared_up_stream(int dev) {
  static std::mutex mu;
  static std::map<int, hipStream_t> streams;
  std::lock_guard<std::mutex> lock(mu);
  auto it = streams.find(dev);
  if (it != streams.end()) return it->second;
  // the up path fills the CUs the generator's small low-resolution launches leave idle: its stream gets
  // the lowest priority, so the generator's workgroups dispatch first when both streams have work
  static const int low_prio = GHOST_KNOB("GHOST_UP_STREAM_LOWPRIO", 1);
  int least = 0, greatest = 0;
  if (!low_prio || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least) != hipSuccess) s = nullptr;
  streams[dev] = s;
  return s;
}

// the handle's up-path stream and events on device `dev` (the current device; events created once per device);
// false: this call runs on one stream
bool ensure_up_stream(ghost_aei* h, int dev) {
  auto it = h->up_path.find(dev);
  if (it != h->up_path.end()) return it->second.s != nullptr;
  ghost_aei::UpPath& u = h->up_path[dev];   // a failed creation leaves a null stream: one stream from then on
  ghost_aei::UpPath tmp;
  tmp.s = shared_up_stream(dev);
  bool ok = tmp.s != nullptr;
  for (auto& e : tmp.zev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&tmp.zend, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    for (auto e : tmp.zev)
      if (e) (void)hipEventDestroy(e);
    if (tmp.zend) (void)hipEventDestroy(tmp.zend);
    return false;
  }
  u = tmp;
  return true;
}

// makes the device of the caller's stream current for the duration of a call (every launch, the up-path
// stream and its events then live on the stream's device, whatever device the caller had current)
struct DeviceGuard {
  int prev = -1, dev = -1;
  bool ok = false;
  explicit DeviceGuard(hipStream_t s) {
    if (hipGetDevice(&prev) != hipSuccess) return;
    dev = prev;
    if (s) {
      hipDevice_t d;
      if (hipStreamGetDevice(s, &d) != hipSuccess) return;
      dev = (int)d;
    }
    ok = dev == prev || hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (ok && dev != prev) (void)hipSetDevice(prev);
  }
};

int run(ghost_aei* h, Mode mode, int B, const Io& io, void* ws, int64_t ws_bytes, void* stream) {
  if (int rc = check_handle(h)) return rc;
  if (B <= 0) return fail(GHOST_EINVAL, "batch must be positive");
  Ctx dry{};
  dry.h = h; dry.dry = true;
  plan(dry, mode, B, io);
  if (!dry.ok()) return fail(dry.rc, dry.where);
  const size_t main_bytes = ((dry.off + 255) & ~size_t(255)) + kMainSlack;
  const size_t scr = (dry.scratch_need + 255) & ~size_t(255);
  const size_t need = main_bytes + kSemBytes + (dry.dual ? 2 : 1) * scr + 256;
  if (!ws || (size_t)ws_bytes < need)
    return fail(GHOST_ENOWS, "workspace too small: need " + std::to_string(need) + " bytes");
  Ctx c{};
  c.h = h; c.dry = false;
  c.base = (char*)(((uintptr_t)ws + 255) & ~uintptr_t(255));
  c.cap = main_bytes;
  c.scratch = c.base + main_bytes + kSemBytes;
  c.scratch_cap = dry.scratch_need;
  c.s = (hipStream_t)stream;
  DeviceGuard guard(c.s);
  if (!guard.ok) return fail(GHOST_EINVAL, "cannot make the device of the caller's stream current");
  c.dev = guard.dev;
  if (h->opt[GHOST_AEI_OPT_FUSE_REDUCE]) {
    // the counters start at zero (the workspace is the caller's memory); queued before every launch of the call,
    // which the up-path stream's launches follow through its events
    // (a kernel, not hipMemsetAsync: a captured memset node left GraphedSwap's B = 8 one-chain replay with wrong
    // bytes; a swap's crops conversion zeroes them in its own launch, see plan)
    unsigned* sem = (unsigned*)(c.base + main_bytes);
    c.sem_main = sem;
    c.sem_up = sem + kSemWords;
    if (mode != M_SWAP)
      if (int rc = zero_words(sem, 2 * kSemWords, c.s)) return fail(rc, "counter reset failed");
  }
  if (dry.dual && ensure_up_stream(h, c.dev)) {
    c.s_up = h->up_path[c.dev].s;
    h->zev = h->up_path[c.dev].zev;
    c.scratch_up = c.scratch + scr;
  }
  c.force_single = !c.s_up;   // no second stream on this device: the same plan on one stream
  plan(c, mode, B, io);
  if (!c.ok()) return fail(c.rc, "forward failed at " + c.where + ": " + (c.rc > 0 ? hipGetErrorString((hipError_t)c.rc) : ""));
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI: handle
// ---------------------------------------------------------------------------
extern "C" int ghost_aei_create(const char* backbone, int num_blocks, int c_id, int dtype, ghost_aei** out) {
  if (!out || !backbone) return fail(GHOST_EINVAL, "null argument");
  std::string bb(backbone);
  if (bb != "unet" && bb != "linknet" && bb != "resnet")
    return fail(GHOST_EINVAL, "backbone must be 'unet', 'linknet' or 'resnet' (got " + bb + ")");
  if (num_blocks < 1 || num_blocks > 8) return fail(GHOST_EINVAL, "num_blocks out of range");
  if (c_id <= 0 || c_id % 32) return fail(GHOST_EINVAL, "c_id must be a positive multiple of 32");
  if (dtype != GHOST_F32 && dtype != GHOST_BF16 && dtype != GHOST_F16)
    return fail(GHOST_EINVAL, "dtype must be f32, bf16 or f16");
  ghost_aei* h = new ghost_aei();
  h->linknet = bb == "linknet";
  h->resnet = bb == "resnet";
  h->nb = num_blocks;
  h->c_id = c_id;
  h->dt = dtype;
  h->esz = dtype == GHOST_F32 ? 4 : 2;
  declare_slots(h);
  *out = h;
  return 0;
}

extern "C" void ghost_aei_destroy(ghost_aei* h) {
  if (!h) return;
  for (auto e : h->ev) (void)hipEventDestroy(e);
  if (h->clk) (void)hipFree(h->clk);
  for (auto& kv : h->up_path) {
    for (auto e : kv.second.zev)
      if (e) (void)hipEventDestroy(e);
    if (kv.second.zend) (void)hipEventDestroy(kv.second.zend);
    // kv.second.s is the process's shared up-path stream (shared_up_stream): not the handle's to destroy
  }
  delete h;
}

extern "C" int ghost_aei_bind(ghost_aei* h, const char* name, const void* p, int64_t numel) {
  if (!h || !name) return fail(GHOST_EINVAL, "null argument");
  auto it = h->slots.find(name);
  if (it == h->slots.end()) return fail(GHOST_EINVAL, std::string("unknown weight slot ") + name);
  if (!p || numel <= 0) return fail(GHOST_EINVAL, std::string("null/empty tensor for slot ") + name);
  if ((uintptr_t)p % 16) return fail(GHOST_EINVAL, std::string("slot not 16-byte aligned: ") + name);
  it->second = p;
  return 0;
}

extern "C" int ghost_aei_missing(ghost_aei* h) {
  if (!h) return fail(GHOST_EINVAL, "null handle");
  int n = 0;
  std::string first;
  for (auto& kv : h->slots)
    if (!kv.second) {
      if (!n) first = kv.first;
      ++n;
    }
  if (n) g_err = "unbound weight slot " + first;
  return n;
}

extern "C" int ghost_aei_attr_geometry(ghost_aei* h, int level, int* C, int* H, int* W) {
  if (!h || level < 1 || level > 8 || !C || !H || !W) return fail(GHOST_EINVAL, "bad argument");
  int c, hh;
  h->attr_geom(level, c, hh);
  *C = c; *H = hh; *W = hh;
  return 0;
}

extern "C" int64_t ghost_aei_workspace_bytes(ghost_aei* h, int B) {
  if (!h || B <= 0) return fail(GHOST_EINVAL, "bad argument");
  return plan_bytes(h, M_FORWARD, B);
}

extern "C" int64_t ghost_aei_swap_workspace_bytes(ghost_aei* h, int B) {
  if (!h || B <= 0) return fail(GHOST_EINVAL, "bad argument");
  return plan_bytes(h, M_SWAP, B);
}

extern "C" int ghost_aei_forward(ghost_aei* h, const void* xt, int xt_dtype, const int64_t xt_strides[4], int B,
                                 const void* z_id, int zid_dtype, int64_t zid_row_stride, void* y_nhwc,
                                 uint8_t* y_u8_bgr, void* const attr_nhwc[8], void* ws, int64_t ws_bytes,
                                 void* stream) {
  if (!xt || !xt_strides || !z_id || !y_nhwc || !attr_nhwc) return fail(GHOST_EINVAL, "null argument");
  Io io;
  io.xt = xt; io.xt_dtype = xt_dtype;
  for (int i = 0; i < 4; ++i) io.st[i] = xt_strides[i];
  io.zid = z_id; io.zid_dtype = zid_dtype; io.zid_rs = zid_row_stride;
  io.y = y_nhwc; io.u8 = y_u8_bgr;
  for (int k = 0; k < 8; ++k) {
    if (!attr_nhwc[k]) return fail(GHOST_EINVAL, "attr buffer missing");
    io.attr[k] = attr_nhwc[k];
  }
  return run(h, M_FORWARD, B, io, ws, ws_bytes, stream);
}

extern "C" int ghost_aei_get_attr(ghost_aei* h, const void* xt, int xt_dtype, const int64_t xt_strides[4], int B,
                                  void* const attr_nhwc[8], void* ws, int64_t ws_bytes, void* stream) {
  if (!xt || !xt_strides || !attr_nhwc) return fail(GHOST_EINVAL, "null argument");
  Io io;
  io.xt = xt; io.xt_dtype = xt_dtype;
  for (int i = 0; i < 4; ++i) io.st[i] = xt_strides[i];
  for (int k = 0; k < 8; ++k) {
    if (!attr_nhwc[k]) return fail(GHOST_EINVAL, "attr buffer missing");
    io.attr[k] = attr_nhwc[k];
  }
  return run(h, M_ATTR, B, io, ws, ws_bytes, stream);
}

extern "C" int ghost_aei_swap_u8(ghost_aei* h, const uint8_t* crops, int64_t crop_batch_stride, int B,
                                 const void* z_id, int zid_dtype, int64_t zid_row_stride, uint8_t* out_u8, void* ws,
                                 int64_t ws_bytes, void* stream) {
  if (!crops || !z_id || !out_u8) return fail(GHOST_EINVAL, "null argument");
  Io io;
  io.crops = crops; io.crop_bs = crop_batch_stride;
  io.zid = z_id; io.zid_dtype = zid_dtype; io.zid_rs = zid_row_stride;
  io.u8 = out_u8;
  return run(h, M_SWAP, B, io, ws, ws_bytes, stream);
}

extern "C" int64_t ghost_aei_identity_table_bytes(ghost_aei* h, int n_ident) {
  if (!h || n_ident <= 0) return fail(GHOST_EINVAL, "bad argument");
  return (int64_t)table_bytes(h, n_ident);
}

extern "C" int64_t ghost_aei_identity_table_workspace_bytes(ghost_aei* h, int n_ident) {
  if (!h || n_ident <= 0) return fail(GHOST_EINVAL, "bad argument");
  return plan_bytes(h, M_IDTABLE, n_ident);
}

extern "C" int ghost_aei_identity_table(ghost_aei* h, const void* z_id, int zid_dtype, int64_t zid_row_stride,
                                        int n_ident, void* table, int64_t table_bytes_, void* ws, int64_t ws_bytes,
                                        void* stream) {
  if (!z_id || !table) return fail(GHOST_EINVAL, "null argument");
  if (!h || n_ident <= 0) return fail(GHOST_EINVAL, "bad argument");
  if ((uintptr_t)table % 256) return fail(GHOST_EINVAL, "identity table must be 256-byte aligned");
  if (table_bytes_ < (int64_t)table_bytes(h, n_ident)) return fail(GHOST_EINVAL, "identity table too small");
  Io io;
  io.zid = z_id; io.zid_dtype = zid_dtype; io.zid_rs = zid_row_stride;
  io.table = table; io.n_ident = n_ident;
  return run(h, M_IDTABLE, n_ident, io, ws, ws_bytes, stream);
}

extern "C" int ghost_aei_swap_u8_indexed(ghost_aei* h, const uint8_t* crops, int64_t crop_batch_stride, int B,
                                         const void* table, int n_ident, int64_t table_bytes_,
                                         const int32_t* identity_index, uint8_t* out_u8, void* ws, int64_t ws_bytes,
                                         void* stream) {
  if (!crops || !table || !identity_index || !out_u8) return fail(GHOST_EINVAL, "null argument");
  if (!h || n_ident <= 0) return fail(GHOST_EINVAL, "n_ident must be positive");
  if ((uintptr_t)table % 256) return fail(GHOST_EINVAL, "identity table must be 256-byte aligned");
  // the clamped gather reads rows [0, n_ident) only: a table of fewer rows is refused here, not read past its end
  if (table_bytes_ < (int64_t)table_bytes(h, n_ident)) return fail(GHOST_EINVAL, "identity table too small for n_ident");
  Io io;
  io.crops = crops; io.crop_bs = crop_batch_stride;
  io.table = const_cast<void*>(table); io.n_ident = n_ident; io.idx = identity_index;
  io.u8 = out_u8;
  return run(h, M_SWAP, B, io, ws, ws_bytes, stream);
}

extern "C" int ghost_aei_up_stream(ghost_aei* h, int device, void** stream) {
  if (!h || !stream) return fail(GHOST_EINVAL, "null argument");
  auto it = h->up_path.find(device);
  *stream = it == h->up_path.end() ? nullptr : (void*)it->second.s;
  return 0;
}

extern "C" int ghost_aei_profile(ghost_aei* h, int class_mask) {
  if (!h) return fail(GHOST_EINVAL, "null handle");
  h->prof_mask = class_mask;
  h->pend.clear();
  h->ev_used = 0;
  for (auto& p : h->prof) p = ProfClass{};
  h->clk_used = 0;
  h->clk_launch.clear();
  if (class_mask & 2) {   // class 1: arm the in-kernel clock (buffer on the current device)
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return fail(GHOST_EINVAL, "hipGetDevice failed");
    if (h->clk && h->clk_dev != dev) {
      (void)hipFree(h->clk);
      h->clk = nullptr;
    }
    if (!h->clk) {
      h->clk_cap = size_t(8) << 20;   // 64 MB: 227 launches of the B = 64 256x256 kernel
      if (hipMalloc(&h->clk, sizeof(unsigned long long) * h->clk_cap) != hipSuccess) {
        h->clk = nullptr;
        return fail(GHOST_EINVAL, "clock buffer allocation failed");
      }
      h->clk_dev = dev;
    }
  }
  return 0;
}

extern "C" int ghost_aei_profile_clock(ghost_aei* h, double* us_total, int64_t* launches, int* kernel_version) {
  if (!h || !us_total || !launches) return fail(GHOST_EINVAL, "null argument");
  *us_total = 0;
  *launches = 0;
  if (kernel_version) *kernel_version = h->roof_version;
  if (!h->clk || h->clk_launch.empty()) return 0;
  std::vector<unsigned long long> v(h->clk_used);
  if (hipMemcpy(v.data(), h->clk, v.size() * sizeof(v[0]), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(GHOST_EINVAL, "clock buffer read failed");
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, h->clk_dev) != hipSuccess || rate_khz <= 0)
    return fail(GHOST_EINVAL, "wall clock rate unavailable");
  double ticks = 0;
  int64_t n = 0;
  for (auto& L : h->clk_launch) {
    const size_t grid = (size_t)L.second / 9;   // 1 start + 8 wave ends per workgroup
    unsigned long long t0 = ~0ull, t1 = 0;
    for (size_t i = 0; i < grid; ++i) t0 = std::min(t0, v[L.first + i]);
    for (size_t i = grid; i < (size_t)L.second; ++i) t1 = std::max(t1, v[L.first + i]);
    if (t1 <= t0) continue;
    ticks += (double)(t1 - t0);
    ++n;
  }
  *us_total = ticks / (rate_khz * 1e-3);
  *launches = n;
  return 0;
}

extern "C" int ghost_aei_profile_read(ghost_aei* h, int cls, double* ms, int64_t* launches, double* bytes,
                                      double* flops) {
  if (!h || cls < 0 || cls >= 8) return fail(GHOST_EINVAL, "bad argument");
  // fold completed brackets into the class totals (caller synchronised the stream)
  for (auto& p : h->pend) {
    float t = 0.f;
    hipError_t e = hipEventElapsedTime(&t, h->ev[p.e0], h->ev[p.e1]);
    if (e != hipSuccess) return fail((int)e, "hipEventElapsedTime failed (stream not synchronised?)");
    ProfClass& pc = h->prof[p.cls];
    pc.ms += t;
    pc.launches += 1;
    pc.bytes += p.bytes;
    pc.flops += p.flops;
  }
  h->pend.clear();
  h->ev_used = 0;
  if (ms) *ms = h->prof[cls].ms;
  if (launches) *launches = h->prof[cls].launches;
  if (bytes) *bytes = h->prof[cls].bytes;
  if (flops) *flops = h->prof[cls].flops;
  return 0;
}

// ---------------------------------------------------------------------------
// C ABI: single operators
// ---------------------------------------------------------------------------
extern "C" int ghost_aei_set_option(ghost_aei* h, int option, int value) {
  if (!h) return fail(GHOST_EINVAL, "null handle");
  if (option < 0 || option >= GHOST_AEI_NOPT) return fail(GHOST_EINVAL, "unknown option");
  const int vmax = option == GHOST_AEI_OPT_TAP_PARTIALS ? 2 : 1;
  if (value < 0 || value > vmax) return fail(GHOST_EINVAL, "option value out of range");
  h->opt[option] = value;
  return 0;
}

extern "C" int ghost_aei_get_option(ghost_aei* h, int option, int* value) {
  if (!h || !value) return fail(GHOST_EINVAL, "null argument");
  if (option < 0 || option >= GHOST_AEI_NOPT) return fail(GHOST_EINVAL, "unknown option");
  *value = h->opt[option];
  return 0;
}

extern "C" int ghost_aei_set_taps(ghost_aei* h, void* const taps[8]) {
  if (!h) return fail(GHOST_EINVAL, "null handle");
  for (int k = 0; k < 8; ++k) h->taps[k] = taps ? taps[k] : nullptr;
  return 0;
}

static int conv_op(ConvDesc& d, void* ws, int64_t ws_bytes, void* stream, const char* what) {
  const size_t need = conv_workspace_bytes(d);
  if (need > 0 && (!ws || (size_t)ws_bytes < need))
    return fail(GHOST_ENOWS, std::string(what) + ": workspace too small, need " + std::to_string(need));
  int rc = conv_launch(d, ws, (size_t)ws_bytes, (hipStream_t)stream);
  if (rc) return fail(rc, std::string(what) + " failed");
  return 0;
}

extern "C" int ghost_conv2d_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx, const void* w_packed,
                                 int Cout, int Npad, int Kpad, int kh, int kw, int stride, int pad, const float* scale,
                                 const float* shift, float slope, const void* res, int ldres, int tanh_out, void* y,
                                 int ldy, void* ws, int64_t ws_bytes, void* stream) {
  ConvDesc d;
  d.ti = d.to = dtype;
  d.x = x; d.B = B; d.Hi = H; d.Wi = W; d.Cin = Cin; d.ldx = ldx;
  d.w = w_packed; d.N = Cout; d.Npad = Npad; d.Kpad = Kpad;
  d.kind = CONV_FWD; d.kh = kh; d.kw = kw; d.stride = stride; d.pad = pad;
  d.scale = scale; d.shift = shift; d.slope = slope; d.res = res; d.ldres = ldres; d.tanh_out = tanh_out;
  d.y = y; d.ldy = ldy;
  return conv_op(d, ws, ws_bytes, stream, "ghost_conv2d_nhwc");
}

extern "C" int ghost_conv2d_ex_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx,
                                    const void* w_packed, int Cout, int Npad, int Kpad, int kh, int kw, int stride,
                                    int pad, const ghost_conv_epi* epi, void* y, int ldy, void* ws, int64_t ws_bytes,
                                    void* stream) {
  if (!epi) return fail(GHOST_EINVAL, "ghost_conv2d_ex_nhwc: null epilogue");
  ConvDesc d;
  d.ti = d.to = dtype;
  d.x = x; d.B = B; d.Hi = H; d.Wi = W; d.Cin = Cin; d.ldx = ldx;
  d.w = w_packed; d.N = Cout; d.Npad = Npad; d.Kpad = Kpad;
  d.kind = CONV_FWD; d.kh = kh; d.kw = kw; d.stride = stride; d.pad = pad;
  d.scale = epi->scale; d.shift = epi->shift; d.slope = epi->slope; d.prelu = epi->prelu;
  d.res = epi->res; d.ldres = epi->ldres; d.res_first = epi->res_first; d.tanh_out = epi->tanh_out;
  d.y2 = epi->y2; d.ldy2 = epi->ldy2; d.scale2 = epi->scale2; d.shift2 = epi->shift2;
  if (epi->split_k < 0) return fail(GHOST_EINVAL, "ghost_conv2d_ex_nhwc: split_k must be >= 0");
  d.force_split = epi->split_k;
  d.y = y; d.ldy = ldy;
  return conv_op(d, ws, ws_bytes, stream, "ghost_conv2d_ex_nhwc");
}

extern "C" int ghost_conv_transpose4x4s2_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx,
                                              const void* w_packed, int Cout, int Npad, int Kpad, const float* scale,
                                              const float* shift, float slope, const void* res, int ldres, void* y,
                                              int ldy, void* ws, int64_t ws_bytes, void* stream) {
  ConvDesc d;
  d.ti = d.to = dtype;
  d.x = x; d.B = B; d.Hi = H; d.Wi = W; d.Cin = Cin; d.ldx = ldx;
  d.w = w_packed; d.N = Cout; d.Npad = Npad; d.Kpad = Kpad;
  d.kind = CONV_T4S2;
  d.scale = scale; d.shift = shift; d.slope = slope; d.res = res; d.ldres = ldres;
  d.y = y; d.ldy = ldy;
  return conv_op(d, ws, ws_bytes, stream, "ghost_conv_transpose4x4s2_nhwc");
}

extern "C" int ghost_linear_f32(const float* x, int B, int K, const float* w_packed, int N, int Npad, int Kpad,
                                const float* bias, int out_dtype, void* y, int ldy, void* ws, int64_t ws_bytes,
                                void* stream) {
  ConvDesc d;
  d.ti = GHOST_F32; d.to = out_dtype;
  d.x = x; d.B = B; d.Hi = 1; d.Wi = 1; d.Cin = K; d.ldx = K;
  d.w = w_packed; d.N = N; d.Npad = Npad; d.Kpad = Kpad;
  d.shift = bias; d.y = y; d.ldy = ldy;
  return conv_op(d, ws, ws_bytes, stream, "ghost_linear_f32");
}

extern "C" int ghost_instnorm_stats_nhwc(int dtype, const void* x, int B, int HW, int C, int ldx, float* stat, void* ws,
                                         int64_t ws_bytes, void* stream) {
  if ((size_t)ws_bytes < in_stats_workspace_bytes(B, HW, C)) return fail(GHOST_ENOWS, "in_stats: workspace too small");
  int rc = in_stats(dtype, x, ldx, B, HW, C, stat, ws, (size_t)ws_bytes, (hipStream_t)stream);
  return rc ? fail(rc, "in_stats failed") : 0;
}

extern "C" int ghost_instnorm_stats_up2x_nhwc(int dtype, const void* x, int B, int H, int W, int C, int ldx,
                                              float* stat, void* ws, int64_t ws_bytes, void* stream) {
  if ((size_t)ws_bytes < in_stats_workspace_bytes(B, 4 * H * W, C))
    return fail(GHOST_ENOWS, "in_stats_up2x: workspace too small");
  int rc = in_stats_up2x(dtype, x, ldx, B, H, W, C, stat, ws, (size_t)ws_bytes, (hipStream_t)stream);
  return rc ? fail(rc, "in_stats_up2x failed") : 0;
}

extern "C" int ghost_aad_layer_nhwc(int dtype, const void* h_in, int ldh, const void* z_attr, int lda, int B, int H,
                                    int W, int C, int Ca, const void* gbw_packed, int Npad, int Kpad, const float* gbb,
                                    const float* wh, const float* bh, const float* idgb, int id_ld, float slope,
                                    void* out, int ldo, void* ws, int64_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int HW = H * W;
  // workspace: stat [B][C][2] | mask [B*HW] | scratch (max of IN partials and split-K partials)
  const size_t stat_b = ((size_t)B * C * 2 * sizeof(float) + 255) & ~size_t(255);
  const size_t mask_b = ((size_t)B * HW * sizeof(float) + 255) & ~size_t(255);
  ConvDesc d;
  d.ti = d.to = dtype;
  d.x = z_attr; d.B = B; d.Hi = H; d.Wi = W; d.Cin = Ca; d.ldx = lda;
  d.w = gbw_packed; d.N = 2 * C; d.Npad = Npad; d.Kpad = Kpad;
  d.kind = CONV_FWD; d.kh = d.kw = 1;
  d.y = out; d.ldy = ldo; d.shift = gbb; d.slope = slope; d.epi = EPI_AAD;
  d.hin = h_in; d.ldh = ldh; d.idgb = idgb; d.id_ld = id_ld; d.C_aad = C;
  size_t sc = conv_workspace_bytes(d);
  const size_t st = in_stats_workspace_bytes(B, HW, C);
  if (st > sc) sc = st;
  char* base = (char*)(((uintptr_t)ws + 255) & ~uintptr_t(255));
  if (!ws || (size_t)ws_bytes < stat_b + mask_b + sc + 256) return fail(GHOST_ENOWS, "aad_layer: workspace too small");
  float* stat = (float*)base;
  float* mask = (float*)(base + stat_b);
  char* scratch = base + stat_b + mask_b;
  int rc = in_stats(dtype, h_in, ldh, B, HW, C, stat, scratch, sc, s);
  if (rc) return fail(rc, "aad_layer: in_stats failed");
  if (aad_fused_supported(dtype, B, HW, C, Ca, lda, ldh, ldo)) {
    rc = aad_fused(dtype, z_attr, lda, Ca, gbw_packed, Kpad, gbb, h_in, ldh, stat, wh, bh, idgb, id_ld, out, ldo, B, HW, C,
                   slope, s);
    return rc ? fail(rc, "aad_layer: fused kernel failed") : 0;
  }
  rc = aad_mask(dtype, h_in, ldh, B, HW, C, stat, wh, bh, mask, s);
  if (rc) return fail(rc, "aad_layer: mask failed");
  d.stat = stat; d.mask = mask;
  rc = conv_launch(d, scratch, sc, s);
  if (rc) return fail(rc, "aad_layer: gemm failed");
  return 0;
}

extern "C" int ghost_upsample2x_nhwc(int dtype, const void* x, int ldx, void* y, int ldy, int B, int H, int W, int C,
                                     void* stream) {
  int rc = upsample2x(dtype, x, ldx, y, ldy, B, H, W, C, (hipStream_t)stream);
  return rc ? fail(rc, "upsample2x failed") : 0;
}

extern "C" int ghost_nhwc_to_nchw(int dtype, const void* x, int ldx, int B, int H, int W, int C, void* y, void* stream) {
  int rc = nhwc_to_nchw(dtype, x, ldx, B, H, W, C, y, (hipStream_t)stream);
  return rc ? fail(rc, "nhwc_to_nchw failed") : 0;
}

extern "C" int ghost_crops_to_input_nhwc(const uint8_t* crops, int64_t crop_batch_stride, int B, int H, int W, int dtype,
                                         void* y, void* stream) {
  int rc = crops_u8_to_input(crops, crop_batch_stride, B, H, W, dtype, y, (hipStream_t)stream, 3);
  return rc ? fail(rc, "crops_to_input failed") : 0;
}

extern "C" int ghost_conv3x3_narrow_nhwc(int dtype, const void* x, int B, int H, int W, int Cin, int ldx,
                                         const void* w_narrow, int Kpad, int Cout, const void* res, int ldres,
                                         int tanh_out, void* y, int ldy, uint8_t* u8, void* stream) {
  int rc = conv3x3_narrow(dtype, x, B, H, W, Cin, ldx, w_narrow, Kpad, Cout, res, ldres, tanh_out, y, ldy, u8,
                          (hipStream_t)stream);
  return rc ? fail(rc, "conv3x3_narrow failed (H % 8, W % 32, Cin % 32 and Cout <= 3 required)") : 0;
}

extern "C" int ghost_aad_layers_v3_nhwc(const void* h_in, int ldh, int up2x, const void* z_attr, int lda, int B, int H,
                                        int W, int C, int Ca, int L, const void* const w3[], const float* const b3[],
                                        const float* const wh[], const float* const bh[], const float* const idgb[],
                                        int id_ld, float slope, void* const out[], const int ldo[], void* ws,
                                        int64_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int HW = H * W;
  if (L < 1 || L > 2) return fail(GHOST_EINVAL, "aad_v3: L must be 1 or 2");
  if (up2x & ~1) return fail(GHOST_EINVAL, "aad_v3: up2x must be 0 or 1");
  if (up2x && (H % 2 || W % 2 || (C != 64 && C != 128)))
    return fail(GHOST_EINVAL, "aad_v3: up2x needs even H, W and C in {64, 128}");
  // aad_wide: one layer, C in {256, 512, 1024}, Ca <= 512, where the all-channel kernel does not fit
  const bool wide = C >= 256 && !aad_v3_supported(GHOST_BF16, B, HW, C, Ca, lda, ldh, ldo[0]);
  if (wide && (L != 1 || up2x || !aad_wide_supported(GHOST_BF16, B, HW, C, Ca, lda, ldh, ldo[0])))
    return fail(GHOST_EINVAL, "aad_wide: unsupported shape (one layer, C in {256,512,1024}, Ca <= 512)");
  for (int l = 0; l < L && !wide; ++l)
    if (!aad_v3_supported(GHOST_BF16, B, HW, C, Ca, lda, ldh, ldo[l]))
      return fail(GHOST_EINVAL, "aad_v3: unsupported shape (bf16, C in {64,128}, enough pixels)");
  const size_t stat_b = ((size_t)B * C * 2 * sizeof(float) + 255) & ~size_t(255);
  const size_t sc = in_stats_workspace_bytes(B, HW, C);
  char* base = (char*)(((uintptr_t)ws + 255) & ~uintptr_t(255));
  if (!ws || (size_t)ws_bytes < stat_b + sc + 256) return fail(GHOST_ENOWS, "aad_v3: workspace too small");
  float* stat = (float*)base;
  int rc = up2x ? in_stats_up2x(GHOST_BF16, h_in, ldh, B, H / 2, W / 2, C, stat, base + stat_b, sc, s)
                : in_stats(GHOST_BF16, h_in, ldh, B, HW, C, stat, base + stat_b, sc, s);
  if (rc) return fail(rc, "aad_v3: in_stats failed");
  if (wide) {
    const size_t mask_b = ((size_t)B * HW * sizeof(float) + 255) & ~size_t(255);
    if ((size_t)ws_bytes < stat_b + sc + mask_b + 256) return fail(GHOST_ENOWS, "aad_wide: workspace too small");
    float* mask = (float*)(base + stat_b + sc);
    rc = aad_mask(GHOST_BF16, h_in, ldh, B, HW, C, stat, wh[0], bh[0], mask, s);
    if (rc) return fail(rc, "aad_wide: aad_mask failed");
    AadWideDesc w;
    w.mask = mask;
    w.za = z_attr; w.lda = lda; w.Ca = Ca; w.hin = h_in; w.ldh = ldh; w.stat = stat;
    w.B = B; w.HW = HW; w.C = C; w.id_ld = id_ld; w.slope = slope;
    w.w3 = w3[0]; w.b3 = b3[0]; w.wh = wh[0]; w.bh = bh[0]; w.idgb = idgb[0]; w.out = out[0]; w.ldo = ldo[0];
    rc = aad_wide(w, s);
    return rc ? fail(rc, "aad_wide launch failed") : 0;
  }
  AadV3Desc d;
  d.za = z_attr; d.lda = lda; d.Ca = Ca; d.hin = h_in; d.ldh = ldh; d.stat = stat;
  d.B = B; d.HW = HW; d.C = C; d.L = L; d.id_ld = id_ld; d.slope = slope;
  if (up2x) {
    d.up_H = H / 2;
    d.up_W = W / 2;
  }
  for (int l = 0; l < L; ++l) {
    d.w3[l] = w3[l]; d.b3[l] = b3[l]; d.wh[l] = wh[l]; d.bh[l] = bh[l]; d.idgb[l] = idgb[l];
    d.out[l] = out[l]; d.ldo[l] = ldo[l];
  }
  rc = aad_v3(d, s);
  return rc ? fail(rc, "aad_v3 launch failed") : 0;
}
