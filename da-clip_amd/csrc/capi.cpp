// capi.cpp — extern "C" boundary of libdaclip_hip.so (declared in include/daclip_hip.h).
// Every entry point converts exceptions into a negative DAC_E* code + dac_last_error().
#include <cstdio>
#include <algorithm>
#include <array>
#include <map>
#include <cmath>
#include <set>

#include "engine.h"

struct dac_handle {
  int device = 0;
  int dtype = 0;
  dac_config cfg{};
  std::string err;
  dac::WStore ws;
  std::unique_ptr<dac::Engine> eng;
  bool finalized = false;
};

namespace {

template <class F>
int guard(dac_handle* h, F&& f) {
  if (!h) return DAC_E_ARG;
  try {
    h->err.clear();
    return f();
  } catch (const dac::Error& e) {
    h->err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    h->err = "out of host memory";
    return DAC_E_NOMEM;
  } catch (const std::exception& e) {
    h->err = e.what();
    return DAC_E_ARG;
  }
}

// Keys of a DaCLIP checkpoint that the image path never reads (text tower, logit scales);
// open_clip/model.py:203-213, daclip_model.py:24.
bool ignorable(const dac_handle* h, const std::string& k) {
  if (!h->cfg.vit) return false;
  if (h->cfg.text) return k == "clip.logit_scale" || k == "logit_scale";
  static const char* pre[] = {"clip.transformer.", "clip.token_embedding.", "clip.ln_final.",
                              "clip.positional_embedding", "clip.text_projection",
                              "clip.logit_scale", "logit_scale"};
  for (auto p : pre)
    if (k.rfind(p, 0) == 0) return true;
  return false;
}

float half_to_float(uint16_t x) {
  const uint32_t s = (x >> 15) & 1, e = (x >> 10) & 0x1f, m = x & 0x3ff;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? NAN : INFINITY;
  else v = std::ldexp((float)(m | 0x400), (int)e - 25);
  return s ? -v : v;
}

}  // namespace

extern "C" {

int dac_create(int device, int dtype, const dac_config* cfg, dac_handle** out) {
  if (!cfg || !out) return DAC_E_ARG;
  *out = nullptr;
  auto* h = new dac_handle();
  h->device = device;
  h->dtype = dtype;
  h->cfg = *cfg;
  int rc = guard(h, [&]() -> int {
    // in_nc = out_nc = 3: the sampler consumes the noise prediction as an image-shaped
    // tensor (sde_utils.py:245-247), and the output / step kernels are laid out for 3 channels.
    if (cfg->unet && (cfg->depth < 1 || cfg->depth > 8 || cfg->nf % 32 || cfg->in_nc != 3 ||
                      cfg->out_nc != 3))
      throw dac::Error(DAC_E_ARG, "unsupported UNet config (needs in_nc = out_nc = 3, nf % 32 == 0, "
                                  "1 <= depth <= 8)");
    h->eng = dac::make_engine(device, dtype, *cfg);
    return DAC_OK;
  });
  if (rc != DAC_OK) {
    delete h;
    return rc;
  }
  *out = h;
  return DAC_OK;
}

void dac_destroy(dac_handle* h) { delete h; }

int dac_set_weight(dac_handle* h, const char* key, const void* data, const int64_t* shape,
                   int ndim, int src_dtype) {
  return guard(h, [&]() -> int {
    if (!key || !data || ndim < 0 || ndim > 8 || (ndim > 0 && !shape))
      throw dac::Error(DAC_E_ARG, "bad argument");
    if (h->finalized) throw dac::Error(DAC_E_STATE, "weights already finalized");
    const std::string k(key);
    if (ignorable(h, k)) return 1;
    dac::HostW w;
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) {
      w.shape.push_back(shape[i]);
      n *= (size_t)shape[i];
    }
    const size_t es = src_dtype == DAC_SRC_F32 ? 4 : 2;
    std::vector<char> raw(n * es);
    hipPointerAttribute_t attr{};
    const bool dev = hipPointerGetAttributes(&attr, data) == hipSuccess &&
                     attr.type == hipMemoryTypeDevice;
    (void)hipGetLastError();
    if (dev) HIP_OK(hipMemcpy(raw.data(), data, n * es, hipMemcpyDeviceToHost));
    else std::memcpy(raw.data(), data, n * es);
    w.v.resize(n);
    if (src_dtype == DAC_SRC_F32) {
      std::memcpy(w.v.data(), raw.data(), n * 4);
    } else if (src_dtype == DAC_SRC_BF16) {
      const uint16_t* s = (const uint16_t*)raw.data();
      for (size_t i = 0; i < n; ++i) {
        uint32_t u = (uint32_t)s[i] << 16;
        std::memcpy(&w.v[i], &u, 4);
      }
    } else if (src_dtype == DAC_SRC_F16) {
      const uint16_t* s = (const uint16_t*)raw.data();
      for (size_t i = 0; i < n; ++i) w.v[i] = half_to_float(s[i]);
    } else {
      throw dac::Error(DAC_E_ARG, "unknown src_dtype");
    }
    h->ws.m[k] = std::move(w);
    return DAC_OK;
  });
}

int dac_finalize_weights(dac_handle* h) {
  return guard(h, [&]() -> int {
    if (h->finalized) return DAC_OK;
    h->ws.missing.clear();
    h->eng->finalize(h->ws);
    std::string unexpected;
    for (auto& kv : h->ws.m)
      if (!kv.second.used) unexpected += (unexpected.empty() ? "\"" : ", \"") + kv.first + "\"";
    if (!unexpected.empty())
      throw dac::Error(DAC_E_KEY, "Unexpected key(s) in state_dict: " + unexpected);
    h->ws.m.clear();     // host copies no longer needed
    h->finalized = true;
    return DAC_OK;
  });
}

static void need_ready(dac_handle* h) {
  if (!h->finalized) throw dac::Error(DAC_E_STATE, "dac_finalize_weights not called");
}

int dac_encode_image(dac_handle* h, const float* img, int B, float* image_ctx, float* degra_ctx,
                     void* stream) {
  return guard(h, [&]() -> int {
    need_ready(h);
    if (!img || !image_ctx || B < 1) throw dac::Error(DAC_E_ARG, "bad argument");
    h->eng->encode(img, B, image_ctx, degra_ctx, (hipStream_t)stream);
    return DAC_OK;
  });
}

int dac_encode_text(dac_handle* h, const int64_t* tokens, int N, float* text_features, void* stream) {
  return guard(h, [&]() -> int {
    need_ready(h);
    if (!tokens || !text_features || N < 1) throw dac::Error(DAC_E_ARG, "bad argument");
    h->eng->encode_text(tokens, N, text_features, (hipStream_t)stream);
    return DAC_OK;
  });
}

int dac_degradation_probs(dac_handle* h, const float* degra, const float* text_features, int B, int K,
                          int E, float* probs, int32_t* argmax, void* stream) {
  return guard(h, [&]() -> int {
    if (!degra || !text_features || !probs || !argmax || B < 1 || K < 1 || K > 64 || E < 1)
      throw dac::Error(DAC_E_ARG, "bad argument (1 <= K <= 64)");
    dac::degradation_probs(degra, text_features, B, K, E, probs, argmax, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return DAC_OK;
  });
}

int dac_unet_forward(dac_handle* h, const float* xt, const float* mu, float t,
                     const float* text_ctx, const float* image_ctx, int B, int H, int W,
                     float* eps_out, void* stream) {
  return guard(h, [&]() -> int {
    need_ready(h);
    if (!xt || !mu || !eps_out || B < 1 || H < 2 || W < 2) throw dac::Error(DAC_E_ARG, "bad argument");
    h->eng->unet_forward(xt, mu, t, text_ctx, image_ctx, B, H, W, eps_out, (hipStream_t)stream);
    return DAC_OK;
  });
}

int dac_sde_schedule(dac_handle* h, float max_sigma, int T, int schedule, float eps,
                     const float* tables, float dt) {
  return guard(h, [&]() -> int {
    if (T < 1) throw dac::Error(DAC_E_ARG, "T must be >= 1");
    auto& s = h->eng->sched;
    const dac::SdeSchedule old = s;
    dac::compute_schedule(s, max_sigma, T, schedule, eps);
    if (tables) {
      const int n = T + 1;
      s.thetas.assign(tables, tables + n);
      s.sigmas.assign(tables + n, tables + 2 * n);
      s.tcum.assign(tables + 2 * n, tables + 3 * n);
      s.sbar.assign(tables + 3 * n, tables + 4 * n);
      s.dt = dt;
    }
    if (s.T != old.T || s.dt != old.dt || s.max_sigma != old.max_sigma || s.thetas != old.thetas ||
        s.sigmas != old.sigmas || s.tcum != old.tcum || s.sbar != old.sbar)
      h->eng->invalidate_graphs();
    return DAC_OK;
  });
}

int dac_sde_set_time_scale(dac_handle* h, double scale) {
  return guard(h, [&]() -> int {
    if (!(scale > 0.0) || !std::isfinite(scale)) throw dac::Error(DAC_E_ARG, "time scale must be > 0");
    auto& s = h->eng->sched;
    if (s.time_scale != scale) {
      s.time_scale = scale;
      h->eng->invalidate_graphs();
    }
    return DAC_OK;
  });
}

int dac_sde_reverse(dac_handle* h, int mode, float* x_inout, const float* mu, const float* text_ctx,
                    const float* image_ctx, int B, int H, int W, int T, const float* noise,
                    uint64_t seed, void* stream) {
  return guard(h, [&]() -> int {
    need_ready(h);
    if (!x_inout || !mu || B < 1 || H < 2 || W < 2 || (mode != DAC_POSTERIOR && mode != DAC_SDE))
      throw dac::Error(DAC_E_ARG, "bad argument");
    h->eng->sde_reverse(mode, x_inout, mu, text_ctx, image_ctx, B, H, W, T, noise, seed,
                        (hipStream_t)stream);
    return DAC_OK;
  });
}

int dac_set_noise_offset(dac_handle* h, uint64_t first_image) {
  return guard(h, [&]() -> int {
    h->eng->set_noise_offset(first_image);
    return DAC_OK;
  });
}

int dac_posterior_step(dac_handle* h, int mode, float* x_inout, const float* eps, const float* mu,
                       const float* z, int t, int n, void* stream) {
  return guard(h, [&]() -> int {
    if (!x_inout || !eps || !mu || n < 1) throw dac::Error(DAC_E_ARG, "bad argument");
    h->eng->posterior_step(mode, x_inout, eps, mu, z, t, n, (hipStream_t)stream);
    return DAC_OK;
  });
}

double dac_unet_flops(dac_handle* h, int B, int H, int W) {
  double f = -1;
  guard(h, [&]() -> int {
    if (!h->cfg.unet) throw dac::Error(DAC_E_ARG, "no UNet");
    f = h->eng->unet_flops(B, H, W);
    return DAC_OK;
  });
  return f;
}

double dac_encode_flops(dac_handle* h, int B) {
  double f = -1;
  guard(h, [&]() -> int {
    if (!h->cfg.vit) throw dac::Error(DAC_E_ARG, "no vision tower");
    f = h->eng->encode_flops(B);
    return DAC_OK;
  });
  return f;
}

int dac_op_attention(const void* qkv, void* out, int B, int L, int H, int dtype, int variant,
                     void* stream) {
  const bool pre = (variant & DAC_ATTN_Q_PRESCALED) != 0;
  variant &= ~DAC_ATTN_Q_PRESCALED;
  if (!qkv || !out || B <= 0 || L <= 0 || H <= 0 ||
      (dtype != DAC_F32 && dtype != DAC_BF16 && dtype != DAC_F16) || variant < 0 || variant > 4 ||
      (variant == 2 && (dtype == DAC_F32 || L % 64)) ||
      (variant >= 3 && (dtype == DAC_F32 || L % 256 || L > 1024)))
    return DAC_E_ARG;
  const float scale = pre ? 0.f : 1.f / std::sqrt(32.f);
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == DAC_BF16) dac::flash_attn_d32_v<__bf16>(qkv, out, B, L, H, scale, variant, st);
  else if (dtype == DAC_F16) dac::flash_attn_d32_v<_Float16>(qkv, out, B, L, H, scale, variant, st);
  else dac::flash_attn_d32_v<float>(qkv, out, B, L, H, scale, variant, st);
  return hipGetLastError() == hipSuccess ? DAC_OK : DAC_E_HIP;
}

int dac_profile_enable(dac_handle* h, int kernel_id) {
  return guard(h, [&]() -> int {
    h->eng->prof.kernel_id = kernel_id;
    h->eng->prof.begin_pass();
    return DAC_OK;
  });
}

int dac_profile_read(dac_handle* h, double* mean_ms, double* flops_per_launch,
                     double* bytes_per_launch) {
  int n = 0;
  int rc = guard(h, [&]() -> int {
    auto& p = h->eng->prof;
    if (p.kernel_id < 0 || p.launches == 0) throw dac::Error(DAC_E_STATE, "nothing profiled");
    double tot = 0;
    std::map<std::string, std::array<double, 3>> by;   // label -> count, ms, flops
    if (p.stamps && p.lms.size() != p.launches) throw dac::Error(DAC_E_STATE, "graph profile incomplete");
    if (!p.stamps) p.lms.assign(p.launches, 0.0);
    for (size_t i = 0; i < p.launches; ++i) {
      if (!p.stamps) {
        HIP_OK(hipEventSynchronize(p.ev[2 * i + 1]));
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, p.ev[2 * i], p.ev[2 * i + 1]));
        p.lms[i] = ms;
      }
      const double ms = p.lms[i];
      tot += ms;
      if (p.kernel_id == dac::Profiler::ALL && i < p.labels.size()) {
        auto& v = by[p.labels[i]];
        v[0] += 1; v[1] += ms; v[2] += p.lflops[i];
      }
    }
    if (!by.empty() && getenv("DAC_PROFILE_PRINT")) {   // per-shape report (kernel_id ALL)
      std::vector<std::pair<double, std::string>> rows;
      for (auto& kv : by) {
        char line[320];
        snprintf(line, sizeof line, "%6.0f x %8.1f us = %8.2f ms  %7.1f TF/s  %s", kv.second[0],
                 1e3 * kv.second[1] / kv.second[0], kv.second[1],
                 kv.second[2] / (kv.second[1] * 1e-3) / 1e12, kv.first.c_str());
        rows.push_back({kv.second[1], line});
      }
      std::sort(rows.rbegin(), rows.rend());
      fprintf(stderr, "[dac conv profile] %zu launches, %.2f ms total\n", p.launches, tot);
      for (auto& r : rows) fprintf(stderr, "  %s\n", r.second.c_str());
    }
    n = (int)p.launches;
    if (mean_ms) *mean_ms = tot / n;
    if (flops_per_launch) *flops_per_launch = p.flops / n;
    if (bytes_per_launch) *bytes_per_launch = p.bytes / n;
    return DAC_OK;
  });
  return rc < 0 ? rc : n;
}

int dac_profile_mode(dac_handle* h, int graph_stamps) {
  return guard(h, [&]() -> int {
    h->eng->prof.stamps = graph_stamps != 0;
    return DAC_OK;
  });
}

int dac_profile_launch(dac_handle* h, int i, double* ms, double* flops, double* bytes, int* kernel_class,
                       double* start_ms, int* in_branch, char* label, int label_len, char* symbol,
                       int symbol_len) {
  return guard(h, [&]() -> int {
    auto& p = h->eng->prof;
    if (i < 0 || (size_t)i >= p.launches || (size_t)i >= p.lms.size())
      throw dac::Error(DAC_E_ARG, "dac_profile_launch: index out of range (call dac_profile_read first)");
    if (ms) *ms = p.lms[i];
    if (flops) *flops = p.lflops[i];
    if (bytes) *bytes = p.lbytes[i];
    if (kernel_class) *kernel_class = p.lcls[i];
    if (start_ms) *start_ms = (size_t)i < p.lt0.size() ? p.lt0[i] : -1.0;
    if (in_branch) *in_branch = (size_t)i < p.lbranch.size() ? p.lbranch[i] : 0;
    if (label && label_len > 0) snprintf(label, label_len, "%s", i < (int)p.labels.size() ? p.labels[i].c_str() : "");
    if (symbol && symbol_len > 0) snprintf(symbol, symbol_len, "%s", i < (int)p.lsym.size() ? p.lsym[i].c_str() : "");
    return DAC_OK;
  });
}

int dac_profile_graph_ms(dac_handle* h, double* ms) {
  return guard(h, [&]() -> int {
    if (!ms) throw dac::Error(DAC_E_ARG, "null output");
    *ms = h->eng->prof.graph_ms;
    return DAC_OK;
  });
}

const char* dac_last_error(dac_handle* h) { return h ? h->err.c_str() : "null handle"; }

#ifndef DAC_BUILD_ID
#define DAC_BUILD_ID "unknown"
#endif
const char* dac_build_id(void) { return DAC_BUILD_ID; }

}  // extern "C"
