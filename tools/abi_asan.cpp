// abi_asan.cpp — argument-validation paths of the C ABI (include/daclip_hip.h) under a host
// AddressSanitizer build (SURVEY.md §5 "Race detection / sanitizers": a debug build with
// -fsanitize=address for host code). Built by `make -C da-clip_amd asan`: capi.cpp and
// engine.cpp compiled with `-Xarch_host -fsanitize=address` (device code is not sanitized),
// linked with the normal kernel objects into this executable, so the ASan runtime comes with
// the binary (no preload). Every call below must return its documented DAC_E* code without a
// heap error or leak; with a GPU present it also walks a handle through the state machine
// (set_weight / finalize / forward errors) before destroying it.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/daclip_hip.h"

static int g_fail = 0;
#define EXPECT(cond)                                                      \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

static dac_config small_unet() {
  dac_config c;
  std::memset(&c, 0, sizeof c);
  c.unet = 1;
  c.in_nc = 3;
  c.out_nc = 3;
  c.nf = 32;
  c.depth = 2;
  c.ch_mult[0] = 1;
  c.ch_mult[1] = 2;
  c.context_dim = 0;
  return c;
}

int main() {
  // Null handles and pointers: every entry point rejects them before touching memory.
  EXPECT(dac_create(0, DAC_F32, nullptr, nullptr) == DAC_E_ARG);
  dac_handle* h = reinterpret_cast<dac_handle*>(0x1);
  dac_config c = small_unet();
  EXPECT(dac_create(0, DAC_F32, &c, nullptr) == DAC_E_ARG);
  EXPECT(dac_set_weight(nullptr, "k", &c, nullptr, 0, DAC_SRC_F32) == DAC_E_ARG);
  EXPECT(dac_finalize_weights(nullptr) == DAC_E_ARG);
  EXPECT(dac_encode_image(nullptr, nullptr, 1, nullptr, nullptr, nullptr) == DAC_E_ARG);
  EXPECT(dac_unet_forward(nullptr, nullptr, nullptr, 1.f, nullptr, nullptr, 1, 8, 8, nullptr, nullptr) == DAC_E_ARG);
  EXPECT(dac_sde_reverse(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 1, 8, 8, 1, nullptr, 0, nullptr) == DAC_E_ARG);
  EXPECT(dac_profile_enable(nullptr, 0) == DAC_E_ARG);
  EXPECT(dac_unet_flops(nullptr, 1, 8, 8) < 0);
  EXPECT(std::strcmp(dac_last_error(nullptr), "null handle") == 0);
  EXPECT(dac_op_attention(nullptr, nullptr, 1, 64, 1, DAC_F32, 0, nullptr) == DAC_E_ARG);
  float dummy[4] = {0, 0, 0, 0};
  EXPECT(dac_op_attention(dummy, dummy, 1, 64, 1, 99, 0, nullptr) == DAC_E_ARG);      // bad dtype
  EXPECT(dac_op_attention(dummy, dummy, 1, 100, 1, DAC_F32, 2, nullptr) == DAC_E_ARG); // variant 2: fp32
  EXPECT(dac_op_attention(dummy, dummy, 1, 2048, 1, DAC_BF16, 3, nullptr) == DAC_E_ARG); // L > 1024
  std::printf("build: %s\n", dac_build_id());

  // Unsupported UNet configurations fail in dac_create, and the half-built handle is freed.
  dac_config bad = small_unet();
  bad.nf = 30;
  h = nullptr;
  EXPECT(dac_create(0, DAC_F32, &bad, &h) == DAC_E_ARG && h == nullptr);
  bad = small_unet();
  bad.depth = 9;
  EXPECT(dac_create(0, DAC_F32, &bad, &h) == DAC_E_ARG && h == nullptr);
  bad = small_unet();
  bad.out_nc = 4;
  EXPECT(dac_create(0, DAC_F32, &bad, &h) == DAC_E_ARG && h == nullptr);

  // A valid configuration: without a GPU the engine's device setup fails (DAC_E_HIP or
  // DAC_E_ARG for a missing device) and nothing leaks; with one, walk the handle's states.
  const int rc = dac_create(0, DAC_F32, &c, &h);
  if (rc != DAC_OK) {
    EXPECT(h == nullptr && rc < 0);
    std::printf("no device: dac_create -> %d (expected without a GPU)\n", rc);
  } else {
    const int64_t shp[4] = {32, 6, 7, 7};
    std::vector<float> w(32 * 6 * 7 * 7, 0.01f);
    EXPECT(dac_set_weight(h, nullptr, w.data(), shp, 4, DAC_SRC_F32) == DAC_E_ARG);
    EXPECT(dac_set_weight(h, "init_conv.weight", nullptr, shp, 4, DAC_SRC_F32) == DAC_E_ARG);
    EXPECT(dac_set_weight(h, "init_conv.weight", w.data(), shp, -1, DAC_SRC_F32) == DAC_E_ARG);
    EXPECT(dac_set_weight(h, "init_conv.weight", w.data(), nullptr, 4, DAC_SRC_F32) == DAC_E_ARG);
    EXPECT(dac_set_weight(h, "init_conv.weight", w.data(), shp, 4, 7) == DAC_E_ARG);   // src dtype
    EXPECT(dac_set_weight(h, "init_conv.weight", w.data(), shp, 4, DAC_SRC_F32) == DAC_OK);
    // Forward before finalize: a state error, not a fault.
    EXPECT(dac_unet_forward(h, dummy, dummy, 1.f, nullptr, nullptr, 1, 8, 8, dummy, nullptr) == DAC_E_STATE);
    EXPECT(dac_sde_schedule(h, 50.f, 0, DAC_COSINE, 0.005f, nullptr, 0.f) == DAC_E_ARG);    // T < 1
    EXPECT(dac_sde_set_time_scale(h, -1.0) == DAC_E_ARG);
    // Strict load: almost every key is missing.
    const int fr = dac_finalize_weights(h);
    EXPECT(fr == DAC_E_MISSING || fr == DAC_E_KEY);
    EXPECT(std::strlen(dac_last_error(h)) > 0);
    std::printf("finalize with missing keys -> %d: %.80s...\n", fr, dac_last_error(h));
    dac_destroy(h);
  }
  if (g_fail) {
    std::fprintf(stderr, "abi_asan: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("abi_asan: all checks passed\n");
  return 0;
}
