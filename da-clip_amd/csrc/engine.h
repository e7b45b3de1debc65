// engine.h — host-side runtime of libdaclip_hip: weight store + repacking, workspace arena,
// and the network executors (ConditionalUNet, DaCLIP vision towers, IR-SDE loop).
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/daclip_hip.h"
#include "common.h"
#include "kernels.h"

namespace dac {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_OK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      throw ::dac::Error(DAC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

// ----------------------------------------------------------------------------- weights
struct HostW {
  std::vector<float> v;
  std::vector<int64_t> shape;
  bool used = false;
};

struct WStore {
  std::unordered_map<std::string, HostW> m;
  std::vector<std::string> missing;
  // Fetch a tensor by reference key; records a miss (strict-load semantics) on absence and
  // throws on a shape mismatch (torch load_state_dict's size-mismatch error).
  const HostW* get(const std::string& key, std::vector<int64_t> shape);
};

// Owns device allocations for packed weights.
struct DevPool {
  std::vector<void*> ptrs;
  ~DevPool();
  void* alloc(size_t bytes);
  void* upload(const void* host, size_t bytes);
};

uint16_t f2bf_host(float f);

// Packed conv/linear weight: [cout][kh][kw][cin] in the compute dtype (+ fp32 bias).
struct ConvW {
  const void* w = nullptr;
  const float* b = nullptr;
  int cout = 0, cin = 0, cin_real = 0, kh = 1, kw = 1;
  int kwp = 0;   // > kw: taps of a kernel row padded to kwp with zero weights (K = kh*kwp*cin)
  // 1: split-precision weights [hi | lo] along K (doubles the executed MFMA work of the layer),
  // see ConvArgs::cwrap. Used in bf16 handles for the layers whose weight rounding error is
  // systematic enough to move the restored image.
  int dual = 0;
  // fp8 handles: e4m3 weights [cout][kp8] + E8M0 block exponents [cout][kp8 / 64] (conv8.hip).
  const uint8_t* w8 = nullptr;
  const uint8_t* ws8 = nullptr;
  int kp8 = 0;
  // fp8 handles, the 64 -> 64 ResBlock block2 convs: e4m3 weights [64][9 taps][64] + E8M0
  // exponents [64][9][2] (per output channel, tap, 32-channel half) for conv3q.hip.
  const uint8_t* q8w = nullptr;
  const uint8_t* q8s = nullptr;
  // GEGLU projections, 16-bit handles: the weights / bias again in the swapped-tile order
  // (ConvArgs::w_gs, b_gs).
  const void* w_gs = nullptr;
  const float* b_gs = nullptr;
  // 16-bit handles, 3x3 convs over a 2x nearest-upsampled input: row-phase weights
  // [cout][4][3][cin] = (W0, W1+W2 | W0+W1, W2) (ConvArgs::uph).
  const void* wph = nullptr;
  // ... and the row- and column-phase weights [cout][4 row sets][4 column sets][cin] (uph = 2).
  const void* wpc = nullptr;
};

// ----------------------------------------------------------------------------- run context
struct Arena {
  char* base = nullptr;
  size_t cap = 0, off = 0, peak = 0;
  bool dry = true;
  void reset() { off = 0; }
  void* get(size_t bytes) {
    size_t o = (off + 255) & ~size_t(255);
    off = o + bytes;
    if (off > peak) peak = off;
    if (dry) return reinterpret_cast<void*>(uintptr_t(0x100000) + o);
    if (off > cap) throw Error(DAC_E_NOMEM, "workspace arena overflow");
    return base + o;
  }
};

struct Profiler {
  int kernel_id = -1;            // conv class to time (kh*100 + conv_variant), -1 = off
  std::vector<hipEvent_t> ev;    // start/stop pairs
  size_t used = 0;               // pairs recorded in the current pass
  double flops = 0, bytes = 0;   // algorithmic work of the recorded launches
  size_t launches = 0;
  // kernel_id == ALL: every conv launch is timed and labelled by shape (per-shape report).
  static constexpr int ALL = 999;
  std::vector<std::string> labels;
  std::vector<double> lflops;
  // Per timed launch: conv class, algorithmic bytes, and (graph mode) measured duration and
  // kernel symbol.
  std::vector<int> lcls;
  std::vector<double> lbytes, lms;
  std::vector<double> lt0;       // graph mode: launch start (ms after the replay's first launch)
  std::vector<char> lbranch;     // launched inside a concurrent branch of the UNet's split section
  std::vector<std::string> lsym;
  // Graph mode (dac_profile_mode 1): the next dac_sde_reverse records its loop into a captured
  // graph exactly as the timed loop does (side-stream branches included), every timed launch
  // carrying a [begin, end] wall-clock stamp pair (ConvArgs::stamp) in sbuf; one replay of that
  // graph gives every launch's in-graph duration. graph_ms = the replay's HIP-event time.
  bool stamps = false;
  unsigned long long* sbuf = nullptr;
  size_t scap = 0;
  double graph_ms = 0;
  void begin_pass() {
    used = 0; flops = 0; bytes = 0; launches = 0; labels.clear(); lflops.clear();
    lcls.clear(); lbytes.clear(); lms.clear(); lsym.clear(); lt0.clear(); lbranch.clear(); graph_ms = 0;
  }
  ~Profiler();
};

struct Run {
  hipStream_t st = nullptr;
  bool dry = false;
  Arena* ar = nullptr;
  Profiler* prof = nullptr;
  const void* zero = nullptr;    // 256 zero bytes on the device (conv padding source)
  double flops = 0;              // executed FLOPs (2*MAC) accumulated by the launches
  // Side streams + fork / join events: the UNet's lowest levels run as concurrent branches of a
  // part of the batch each (UNetNet::forward); null: everything on st.
  static constexpr int kSide = 3;
  hipStream_t side[kSide] = {};
  hipEvent_t evf = nullptr, evj[kSide] = {};
  bool in_branch = false;        // recording one branch of a fork (no nested forks)
  template <class X> X* alloc(size_t n) { return reinterpret_cast<X*>(ar->get(n * sizeof(X))); }
};

// Epilogue options for conv_call.
struct Epi {
  const float* ss = nullptr; int ss_ld = 0;
  const void* res1 = nullptr; int ldr1 = 0;
  const void* res2 = nullptr; int ldr2 = 0;
  const float* bbias = nullptr; int bb_ld = 0;
  int act = ACT_NONE;
  int amode = 0;                 // A-loader transform (ConvArgs::amode)
  long long w_bstride = 0;       // per-image weights (ConvArgs::w_bstride)
  const float* ln_g = nullptr;   // row LayerNorm over Cout in the epilogue (ConvArgs::ln_g)
  float ln_eps = 1e-5f;
  // 3x3 convs: a 1x1 conv over the same input written to y2 (the ResBlock res_conv), fused
  // into the conv kernel when the dispatcher can (ConvArgs::w2), else run right after it.
  const ConvW* fuse1x1 = nullptr;
  void* y2 = nullptr;
  int ldy2 = 0;
  // 1x1 GEMMs with the input row LayerNorm folded into the weights (ConvArgs::lnf_cs).
  const float* lnf_cs = nullptr;
  int lnf_n = 0;
  float lnf_eps = 1e-5f;
  // 1x1 GEMMs applying the input GroupNorm in their A path (ConvArgs::gna_stats).
  const float* gna_stats = nullptr;
  const float* gna_g = nullptr;
  const float* gna_b = nullptr;
  int gna_groups = 0;
  int gna_nb = 0;                // > 0: gna_stats holds per-block group sums (ConvArgs::gna_nb)
  float gna_eps = 1e-6f;
  // fp8 ResBlock pair (ConvArgs::ys8 / xs8): ys8 = the output is e4m3 (ldy bytes per pixel) with
  // these exponents; xs8 = the input x1 is e4m3 with these exponents (conv3q, weights cw.q8w).
  uint8_t* ys8 = nullptr;
  const uint8_t* xs8 = nullptr;
  // 1x1 GEMMs that may split K (conv_split_k): the rows of ONE image (tower token count); the
  // split is chosen from it, never from the batch, so results stay batch-invariant. 0 = no split.
  int split_rows = 0;
};

template <typename T>
void conv_call(Run& r, const ConvW& cw, const void* x1, int ld1, int C1, const void* x2, int ld2,
               int B, int Hs, int Ws, int up, int stride, int pad, void* y, int ldy,
               const Epi& e);

// ----------------------------------------------------------------------------- networks
struct SdeSchedule {
  int T = 0;
  std::vector<float> thetas, sigmas, tcum, sbar;
  float dt = 0, max_sigma = 0;
  double time_scale = 1.0;       // IRSDE.sample_scale = T / sample_T (sde_utils.py:88, 302)
  StepCoef coef(int t, int mode) const;
};
void compute_schedule(SdeSchedule& s, float max_sigma, int T, int schedule, float eps);

class Engine {
 public:
  virtual ~Engine() = default;
  virtual void finalize(WStore& w) = 0;
  virtual void encode(const float* img, int B, float* ic, float* dc, hipStream_t st) = 0;
  virtual void encode_text(const int64_t* tokens, int N, float* out, hipStream_t st) = 0;
  virtual void unet_forward(const float* xt, const float* mu, float t, const float* tc,
                            const float* icx, int B, int H, int W, float* eps,
                            hipStream_t st) = 0;
  virtual void sde_reverse(int mode, float* x, const float* mu, const float* tc,
                           const float* icx, int B, int H, int W, int T, const float* noise,
                           uint64_t seed, hipStream_t st) = 0;
  virtual void posterior_step(int mode, float* x, const float* eps, const float* mu,
                              const float* z, int t, int n, hipStream_t st) = 0;
  virtual double unet_flops(int B, int H, int W) = 0;
  virtual void set_noise_offset(uint64_t first_image) = 0;
  virtual void invalidate_graphs() {}     // captured loops bake in the schedule
  virtual double encode_flops(int B) = 0;
  SdeSchedule sched;
  Profiler prof;
};

std::unique_ptr<Engine> make_engine(int device, int dtype, const dac_config& cfg);

}  // namespace dac
