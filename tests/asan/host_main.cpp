// Host-side sanitizer run of the native library's CPU code (sanitizers on host code only — GPU
// AddressSanitizer is not available on this pool).  Built by tools/asan_host.sh with -fsanitize=address,undefined
// on the host pass of every ghost_amd/csrc/*.hip (-Xarch_host), linked into this executable and run on the CPU:
// no kernel is launched.  It exercises
//   * ghost_aei_create / ghost_aei_destroy for every backbone, num_blocks and dtype,
//   * the native plan's dry run and its bump allocator (ghost_aei_workspace_bytes, _swap_workspace_bytes,
//     identity-table sizing) at batch sizes 1 .. 128, including the two-stream plan's second scratch region,
//   * argument validation paths (ghost_last_error strings),
//   * ghost_mask_polygons (eyebrow expansion + convex hull, masks.hip) on random and degenerate landmark sets.
// Exit status 0 and no sanitizer report = clean.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ghost_amd.h"

static int fails = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                          \
    }                                                                   \
  } while (0)

int main() {
  const char* bbs[3] = {"unet", "linknet", "resnet"};
  const int dts[3] = {GHOST_DTYPE_F32, GHOST_DTYPE_BF16, GHOST_DTYPE_F16};
  int64_t checked = 0;
  for (const char* bb : bbs)
    for (int nb = 1; nb <= 3; ++nb)
      for (int dt : dts) {
        ghost_aei* h = nullptr;
        CHECK(ghost_aei_create(bb, nb, 512, dt, &h) == 0 && h);
        if (!h) continue;
        CHECK(ghost_aei_missing(h) > 0);   // nothing bound
        for (int k = 1; k <= 8; ++k) {
          int C = 0, H = 0, W = 0;
          CHECK(ghost_aei_attr_geometry(h, k, &C, &H, &W) == 0 && C > 0 && H == (1 << k) && W == H);
        }
        for (int B : {1, 2, 3, 7, 8, 9, 16, 33, 64, 128}) {
          for (int two = 0; two <= 1; ++two) {
            CHECK(ghost_aei_set_option(h, GHOST_AEI_OPT_TWO_STREAMS, two) == 0);
            const int64_t f = ghost_aei_workspace_bytes(h, B), s = ghost_aei_swap_workspace_bytes(h, B);
            CHECK(f > 0 && s > 0);
            checked += 2;
          }
          for (int fr = 0; fr <= 1; ++fr) {
            CHECK(ghost_aei_set_option(h, GHOST_AEI_OPT_FUSE_REDUCE, fr) == 0);
            CHECK(ghost_aei_swap_workspace_bytes(h, B) > 0);
          }
          CHECK(ghost_aei_identity_table_bytes(h, B) > 0);
          CHECK(ghost_aei_identity_table_workspace_bytes(h, B) > 0);
          checked += 3;
        }
        int v = -1;
        CHECK(ghost_aei_get_option(h, GHOST_AEI_OPT_TAP_PARTIALS, &v) == 0 && v >= 0);
        CHECK(ghost_aei_set_option(h, 99, 1) != 0 && std::strlen(ghost_last_error()) > 0);
        CHECK(ghost_aei_workspace_bytes(h, 0) < 0);
        CHECK(ghost_aei_bind(h, "no.such.slot", nullptr, 1) != 0);
        ghost_aei_destroy(h);
      }
  ghost_aei* bad = nullptr;
  CHECK(ghost_aei_create("vgg", 2, 512, GHOST_DTYPE_BF16, &bad) != 0 && bad == nullptr);
  CHECK(ghost_aei_create("unet", 0, 512, GHOST_DTYPE_BF16, &bad) != 0);
  CHECK(ghost_aei_create("unet", 2, 500, GHOST_DTYPE_BF16, &bad) != 0);

  // face-mask polygons: random landmark clouds, a collinear set, all points equal
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(0.f, 224.f);
  const int F = 64;
  std::vector<float> lm(F * 106 * 2);
  for (auto& x : lm) x = U(rng);
  for (int i = 0; i < 106; ++i) { lm[(1 * 106 + i) * 2] = 10.f + i; lm[(1 * 106 + i) * 2 + 1] = 20.f + i; }
  for (int i = 0; i < 106 * 2; ++i) lm[2 * 106 * 2 + i] = 100.f;
  std::vector<int32_t> params(F * 3);
  for (int f = 0; f < F; ++f) { params[f * 3] = (f % 3 == 0) ? 15 : (f % 3 == 1 ? -5 : 10); params[f * 3 + 1] = 7; params[f * 3 + 2] = 5; }
  std::vector<int32_t> poly(F * 128 * 2, -1), nv(F, -1);
  CHECK(ghost_mask_polygons(lm.data(), F, 106, params.data(), poly.data(), nv.data()) == 0);
  for (int f = 0; f < F; ++f) CHECK(nv[f] >= 1 && nv[f] <= 128);
  CHECK(ghost_mask_polygons(lm.data(), F, 68, params.data(), poly.data(), nv.data()) != 0);
  CHECK(ghost_face_masks_workspace_bytes(F, 224, 224) > 0);

  std::printf("asan host run: %lld plan sizings, %d failed checks\n", (long long)checked, fails);
  return fails ? 1 : 0;
}
