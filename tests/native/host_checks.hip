// Host-side checks of the libmatdcml C API, built and run under AddressSanitizer + UndefinedBehaviorSanitizer on
// the CPU (sanitizers on host code; GPU ASan / xnack+ is not available on this pool).
//
// Loads a host-sanitized build of the library (libmatdcml_hostsan.so, same sources compiled with
// -Xarch_host -fsanitize=address,undefined) and exercises every entry point whose host path runs without a GPU:
//   * the host Philox4x32-10 against the published Random123 known-answer vectors;
//   * decode tile geometry over NB x L x B: the chosen EPW / RMAX respect the 160 KiB LDS and 16-row limits;
//   * training tile geometry over L: rows and LDS padding invariants;
//   * argument validation of the launch entry points (must reject bad shapes BEFORE touching the GPU).
// Exit status 0 = all checks passed; the sanitizers abort on the first memory / UB error.
#include <dlfcn.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../mat_dcml_amd/csrc/common.h"

static int g_fail = 0;
#define CHECK(c, ...) do { if (!(c)) { std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
  std::fprintf(stderr, __VA_ARGS__); std::fprintf(stderr, "\n"); ++g_fail; } } while (0)

template <class F> static F sym(void* h, const char* name) {
  void* p = dlsym(h, name);
  if (!p) { std::fprintf(stderr, "missing symbol %s\n", name); std::exit(2); }
  return reinterpret_cast<F>(p);
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "mat_dcml_amd/_lib/libmatdcml_hostsan.so";
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) { std::fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); return 2; }

  // Philox4x32-10 known-answer tests (Random123 kat_vectors)
  struct Kat { uint32_t c[4], k[2], r[4]; } kats[] = {
    {{0, 0, 0, 0}, {0, 0}, {0x6627e8d5u, 0xe169c58du, 0xbc57ac4cu, 0x9b00dbd8u}},
    {{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}, {0xffffffffu, 0xffffffffu},
     {0x408f276du, 0x41c83b0eu, 0xa20bc7c6u, 0x6d5451fdu}},
    {{0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u}, {0xa4093822u, 0x299f31d0u},
     {0xd16cfe09u, 0x94fdccebu, 0x5001e420u, 0x24126ea1u}},
  };
  for (const Kat& t : kats) {
    mdl::u4 r = mdl::philox4x32_10(t.c[0], t.c[1], t.c[2], t.c[3], t.k[0], t.k[1]);
    CHECK(r.x == t.r[0] && r.y == t.r[1] && r.z == t.r[2] && r.w == t.r[3], "philox KAT %08x", t.c[0]);
  }
  for (uint32_t u : {0u, 1u, 0x7fffffffu, 0xffffffffu}) {
    double x = mdl::u01_open(u);
    float xf = mdl::u01_open_f(u);
    CHECK(x > 0.0 && x < 1.0, "u01_open(%u) = %g", u, x);
    CHECK(xf > 0.f && xf <= 1.f && (xf < 1.f || (u >> 8) == 0xffffffu), "u01_open_f(%u) = %g", u, xf);
  }

  // decode geometry
  auto dec_geom = sym<int (*)(int, int, int)>(h, "mdl_mat_decode_geometry");
  int n_dec = 0;
  for (int nb = 1; nb <= 3; ++nb)
    for (int L = 1; L <= 256; L += (L < 40 ? 1 : 7))
      for (int B = 1; B <= 300; B = B < 20 ? B + 1 : B * 2) {
        const int g = dec_geom(nb, L, B);
        ++n_dec;
        if (g == 0) continue;
        const int epw = g & 0xff, rmax = g >> 8;
        CHECK(epw >= 1 && epw <= 16 && (epw & (epw - 1)) == 0, "nb %d L %d B %d: epw %d", nb, L, B, epw);
        CHECK(epw <= B || epw == 1, "nb %d L %d B %d: epw %d > B", nb, L, B, epw);
        CHECK(rmax >= 1 && rmax * epw <= 16, "nb %d L %d B %d: rmax %d epw %d", nb, L, B, rmax, epw);
      }

  // training geometry
  auto tr_geom = sym<int (*)(int)>(h, "mdl_mat_train_geometry_ct");
  int n_fit = 0;
  for (int L = 1; L <= 320; ++L) {
    const int g = tr_geom(L);
    if (g == 0) continue;
    ++n_fit;
    const int sq = g & 0xffff, nrp = g >> 16;
    CHECK(sq >= 1 && sq * L <= nrp && nrp % 32 == 0 && nrp >= 64, "L %d: sq %d nrp %d", L, sq, nrp);
  }
  CHECK(tr_geom(33) != 0 && tr_geom(101) != 0 && tr_geom(129) != 0, "BASELINE agent counts must fit");

  // argument validation happens before any HIP call (zeroed parameter blocks are invalid)
  std::vector<unsigned char> zeros(1 << 14, 0);
  auto decode = sym<int (*)(const void*, int, void*)>(h, "mdl_mat_decode");
  CHECK(decode(zeros.data(), 2, nullptr) < 0, "decode accepted epw = 0");
  auto enc_fwd = sym<int (*)(const void*, const float*, int, int, void*)>(h, "mdl_mat_enc_fwd_ct");
  CHECK(enc_fwd(zeros.data(), nullptr, 2, 1, nullptr) < 0, "enc_fwd accepted od = 0");
  auto enc_bwd = sym<int (*)(const void*, const float*, float*, int, void*)>(h, "mdl_mat_enc_bwd_ct");
  CHECK(enc_bwd(zeros.data(), nullptr, nullptr, 2, nullptr) < 0, "enc_bwd accepted od = 0");
  auto dec_bwd = sym<int (*)(const void*, int, void*)>(h, "mdl_mat_dec_bwd_ct");
  CHECK(dec_bwd(zeros.data(), 2, nullptr) < 0, "dec_bwd accepted A = 0");

  std::printf("host checks: %d decode geometries, %d trainable agent counts, %d failures\n", n_dec, n_fit, g_fail);
  dlclose(h);
  return g_fail ? 1 : 0;
}
