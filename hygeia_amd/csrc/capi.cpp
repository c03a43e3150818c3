// capi.cpp -- the C ABI of include/hygeia_amd.h: model construction (host
// tables, upload), workspace planning, chain descriptors, launches. Compiled by
// hipcc into hygeia_amd/lib/libhygeia_amd.so together with tg_kernels.hip.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hyg_arith.h"
#include "../../include/hygeia_amd.h"
#include "../../include/hyg_sg_model.h"
#include "sg_common.h"
#include "tg_common.h"
#include "dmp_common.h"

namespace hyg {
int bed_launch_labels(const double* probs, int K, int64_t n, int8_t* label, double* score, void* stream);
int pre_launch_collapse(const int64_t* pos0, int64_t T, const int64_t* plus_start, const int64_t* plus_end,
                        const double* plus_cov, const double* plus_pct, int64_t n_plus, const int64_t* minus_start,
                        const double* minus_cov, const double* minus_pct, int64_t n_minus, int single_base,
                        uint8_t* matched, double* out, int stride, int col, int* conflicts, void* stream);
}

using namespace hyg;

namespace {

thread_local std::string g_err;

// the process's device slot (hyg_device_slot_acquire): the descriptor holding the flock
std::mutex g_slot_mu;
int g_slot_fd = -1, g_slot_device = -1, g_slot_index = -1;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

bool have_device() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return n > 0;
}

template <typename T>
hipError_t dmalloc_copy(T** dst, const T* src, size_t count) {
  hipError_t e = hipMalloc((void**)dst, sizeof(T) * (count ? count : 1));
  if (e != hipSuccess) return e;
  if (count) e = hipMemcpy(*dst, src, sizeof(T) * count, hipMemcpyHostToDevice);
  return e;
}

// The current HIP device must be the one a model's tables live on.
bool on_model_device(int device) {
  int cur = -1;
  return hipGetDevice(&cur) == hipSuccess && cur == device;
}

// Host-to-device upload of per-launch descriptors through a pinned buffer owned
// by the model: the async copy reads memory that outlives the call, and the
// buffer is reused only once the previous upload from it has completed.
struct PinnedStage {
  void* p = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;

  hipError_t upload(void* dst, const void* src, size_t n, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (pending) {
      e = hipEventSynchronize(ev);
      if (e != hipSuccess) return e;
      pending = false;
    }
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (n > cap) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
      if ((e = hipHostMalloc(&p, n, hipHostMallocDefault)) != hipSuccess) return e;
      cap = n;
    }
    std::memcpy(p, src, n);
    if ((e = hipMemcpyAsync(dst, p, n, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipEventRecord(ev, s)) != hipSuccess) return e;
    pending = true;
    return hipSuccess;
  }
  void release() {
    if (pending) (void)hipEventSynchronize(ev);
    if (ev) (void)hipEventDestroy(ev);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    ev = nullptr;
    cap = 0;
    pending = false;
  }
};

// One pinned stage per stream, each behind its own mutex: host threads that
// share a model on different streams neither race on a buffer nor wait for
// each other's kernels (an upload waits only for the previous upload of its
// own stream); two threads on one stream take turns.
class PinnedStages {
 public:
  hipError_t upload(void* dst, const void* src, size_t n, hipStream_t s) {
    Slot* slot;
    {
      std::lock_guard<std::mutex> g(mu_);
      std::unique_ptr<Slot>& u = by_stream_[s];
      if (!u) u.reset(new Slot);
      slot = u.get();
    }
    std::lock_guard<std::mutex> g(slot->mu);
    return slot->st.upload(dst, src, n, s);
  }
  void release() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : by_stream_) {
      std::lock_guard<std::mutex> gs(kv.second->mu);
      kv.second->st.release();
    }
    by_stream_.clear();
  }

 private:
  struct Slot {
    std::mutex mu;
    PinnedStage st;
  };
  std::mutex mu_;
  std::map<hipStream_t, std::unique_ptr<Slot>> by_stream_;
};

}  // namespace

struct hyg_tg_model {
  hyg_tg_consts c{};
  int32_t dcap = 0;
  int32_t nmax_reads = 0;
  int32_t max_duration = 0;
  std::vector<double> hz, lf, lg, cst, bbt;
  bool on_device = false;
  int device = -1;
  hyg_tg_consts* d_consts = nullptr;
  double* d_hz = nullptr;
  double* d_lf = nullptr;
  double* d_lg = nullptr;
  double* d_cst = nullptr;
  double* d_bbt = nullptr;
  mutable PinnedStages stage;  // descriptor uploads (thread-safe, one pinned buffer per stream)

  ModelDev dev() const {
    ModelDev m{};
    m.consts = d_consts;
    m.hz = d_hz;
    m.dcap = dcap;
    m.nmax_reads = nmax_reads;
    m.lf = d_lf;
    m.lg = d_lg;
    m.cst = d_cst;
    m.bbt = d_bbt;
    return m;
  }
};

// The emission's per-(n, y) term table is built when it stays L2-sized (the
// pipeline's coverage: max reads ~170, 0.7 MB at K = 6); beyond that the
// emission forms each term from the lgamma rows.
constexpr size_t kBbtMaxBytes = (size_t)16 << 20;

struct hyg_sg_model {
  hyg_sg_consts c{};
  hyg_sg_params params{};  // as given (initial theta, kappa) for the estimation path
  int32_t dcap = 0;
  int32_t nmax_reads = 0;
  int32_t max_duration = 0;
  std::vector<double> hz, lf, lg, cst;
  std::vector<uint8_t> ex;
  bool on_device = false;
  int device = -1;
  mutable PinnedStages stage;  // descriptor uploads (thread-safe, one pinned buffer per stream)
  hyg_sg_consts* d_consts = nullptr;
  double* d_hz = nullptr;
  uint8_t* d_ex = nullptr;
  double* d_lf = nullptr;
  double* d_lg = nullptr;
  double* d_cst = nullptr;

  SgModelDev dev() const {
    SgModelDev m{};
    m.consts = d_consts;
    m.hz = d_hz;
    m.ex = d_ex;
    m.dcap = dcap;
    m.nmax_reads = nmax_reads;
    m.lf = d_lf;
    m.lg = d_lg;
    m.cst = d_cst;
    return m;
  }
};

extern "C" {

const char* hyg_version(void) { return "hygeia_amd 0.1.0 (gfx950)"; }

const char* hyg_last_error(void) { return g_err.c_str(); }

int hyg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int hyg_device_slot_acquire(const char* lock_dir, int32_t n_devices, int32_t max_per_device, int32_t* device,
                            int32_t* slot) {
  if (!lock_dir || !device || !slot) return fail(HYG_EINVAL, "null argument");
  if (n_devices < 1 || max_per_device < 1) return fail(HYG_EINVAL, "n_devices and max_per_device must be >= 1");
  std::lock_guard<std::mutex> g(g_slot_mu);
  if (g_slot_fd >= 0) {  // one slot per process
    *device = g_slot_device;
    *slot = g_slot_index;
    return HYG_OK;
  }
  for (int j = 0; j < max_per_device; ++j) {
    for (int d = 0; d < n_devices; ++d) {
      const std::string path =
          std::string(lock_dir) + "/hygeia_amd.gpu" + std::to_string(d) + ".slot" + std::to_string(j) + ".lock";
      int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
      if (fd < 0 && errno == EACCES) fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);  // another user's file
      if (fd < 0) return fail(HYG_EINVAL, "device slot lock " + path + ": " + std::strerror(errno));
      if (::flock(fd, LOCK_EX | LOCK_NB) == 0) {
        g_slot_fd = fd;
        g_slot_device = d;
        g_slot_index = j;
        *device = d;
        *slot = j;
        return HYG_OK;
      }
      const int err = errno;
      ::close(fd);
      if (err != EWOULDBLOCK) return fail(HYG_EINVAL, "device slot lock " + path + ": " + std::strerror(err));
    }
  }
  return fail(HYG_EINVAL, "every device slot is held");
}

int hyg_device_slot_release(void) {
  std::lock_guard<std::mutex> g(g_slot_mu);
  if (g_slot_fd >= 0) ::close(g_slot_fd);  // closing the only descriptor drops the flock
  g_slot_fd = -1;
  g_slot_device = g_slot_index = -1;
  return HYG_OK;
}

int hyg_set_device(int32_t device) {
  const int n = hyg_device_count();
  if (n < 1) return fail(HYG_EDEVICE, "no HIP device");
  if (device < 0 || device >= n) return fail(HYG_EINVAL, "device out of range");
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail(HYG_EDEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return HYG_OK;
}

int hyg_get_device(void) {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess) {
    (void)hipGetLastError();
    return fail(HYG_EDEVICE, "no HIP device");
  }
  return d;
}

void hyg_tg_params_default(hyg_tg_params* p) {
  std::memset(p, 0, sizeof(*p));
  const double mu[6] = {0.95, 0.05, 0.80, 0.20, 0.50, 0.50};
  const double sg[6] = {0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751};
  p->n_regimes = 6;
  p->minimum_duration = 3;
  p->num_resampled_ancestors = 50;
  p->num_samples_backward = 25;
  p->optimal_resampling = 1;
  p->multinomial = 0;
  for (int i = 0; i < 6; ++i) {
    p->mu[i] = mu[i];
    p->sigma[i] = sg[i];
  }
  // uniform off-diagonal transitions, omega = 0.8
  p->theta_len = 36;
  for (int i = 0; i < 30; ++i) p->theta[i] = 0.0;
  for (int i = 30; i < 36; ++i) p->theta[i] = std::log(0.8 / 0.2);
  p->omega_case = 0.8;
  p->merge_log_prob = std::log(0.1);
  p->split_prob = 0.01;
  p->kappa_control = 2.0;
  p->kappa_case = 2.0;
}

void hyg_tg_model_destroy(hyg_tg_model* m) {
  if (!m) return;
  if (m->on_device) {
    m->stage.release();
    (void)hipFree(m->d_consts);
    (void)hipFree(m->d_hz);
    (void)hipFree(m->d_lf);
    (void)hipFree(m->d_lg);
    (void)hipFree(m->d_cst);
    (void)hipFree(m->d_bbt);
  }
  delete m;
}

int hyg_tg_model_create(const hyg_tg_params* params, int32_t max_total_reads, int32_t max_duration,
                        hyg_tg_model** out) {
  if (!params || !out) return fail(HYG_EINVAL, "null argument");
  *out = nullptr;
  if (max_total_reads < 0 || max_total_reads > 65535) return fail(HYG_EINVAL, "max_total_reads out of [0, 65535]");
  if (max_duration < 1 || max_duration >= HYG_DMAX - 2) return fail(HYG_EINVAL, "max_duration out of range");
  auto* m = new hyg_tg_model();
  int rc = hyg_tg_derive(params, &m->c);
  if (rc != HYG_OK) {
    delete m;
    return fail(rc, "invalid model parameters");
  }
  m->max_duration = max_duration;
  m->nmax_reads = max_total_reads;
  m->dcap = hyg_hazard_len(&m->c, max_duration + 2);
  const int K = m->c.K, L = max_total_reads + 1;
  m->hz.resize((size_t)2 * K * m->dcap * 2);
  hyg_hazard_fill(&m->c, m->dcap, m->hz.data());
  m->lf.resize(L);
  m->lg.resize((size_t)3 * K * L);
  m->cst.resize(K);
  hyg_bb_tables(&m->c, max_total_reads, m->lf.data(), m->lg.data(), m->cst.data());
  if (hyg_bb_term_table_len(K, max_total_reads) * sizeof(double) <= kBbtMaxBytes) {
    m->bbt.resize(hyg_bb_term_table_len(K, max_total_reads));
    hyg_bb_term_table(K, max_total_reads, m->lf.data(), m->lg.data(), m->cst.data(), m->bbt.data());
  }
  if (have_device()) {
    (void)hipGetDevice(&m->device);
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = dmalloc_copy(&m->d_consts, &m->c, 1);
    if (e == hipSuccess) e = dmalloc_copy(&m->d_hz, m->hz.data(), m->hz.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_lf, m->lf.data(), m->lf.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_lg, m->lg.data(), m->lg.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_cst, m->cst.data(), m->cst.size());
    if (e == hipSuccess && !m->bbt.empty()) e = dmalloc_copy(&m->d_bbt, m->bbt.data(), m->bbt.size());
    m->on_device = true;
    if (e != hipSuccess) {
      hyg_tg_model_destroy(m);
      return fail(HYG_EDEVICE, std::string("device upload failed: ") + hipGetErrorString(e));
    }
  }
  *out = m;
  return HYG_OK;
}

int32_t hyg_tg_num_particles(const hyg_tg_model* m) { return m ? m->c.Nmax : 0; }

int32_t hyg_tg_threads_per_chain(const hyg_tg_model* m, int32_t n_chains) {
  return m ? hyg::tg_threads_per_chain(m->c, n_chains) : 0;
}

int32_t hyg_tg_chains_per_cu(const hyg_tg_model* m, int32_t n_chains) {
  if (!m || !m->on_device) return 0;
  return hyg::tg_resident_per_cu(m->c, n_chains);
}

size_t hyg_tg_lds_bytes(const hyg_tg_model* m, int32_t threads, int32_t backward) {
  return m ? hyg::tg_layout_bytes(m->c, threads, backward != 0) : 0;
}

int hyg_tg_force_threads(int32_t forward, int32_t backward) {
  const int rc = hyg::tg_force_threads(forward, backward);
  return rc == HYG_OK ? rc : fail(rc, "unsupported workgroup size");
}

int hyg_tg_set_tail_overlap(int32_t on) {
  hyg::tg_set_tail_overlap(on != 0);
  return HYG_OK;
}

int32_t hyg_tg_device_cus(int32_t device) { return hyg::tg_device_cus(device); }

int hyg_tg_set_device_cus(int32_t device, int32_t cus) {
  const int rc = hyg::tg_set_device_cus(device, cus);
  return rc == HYG_OK ? rc : fail(rc, "device out of [0, 64) or negative CU count");
}

int hyg_sg_force_key_drop(int32_t bits) {
  const int rc = hyg::sg_force_key_drop(bits);
  return rc == HYG_OK ? rc : fail(rc, "key bits out of range [8, 60]");
}

int hyg_tg_emission(const hyg_tg_model* m, const uint16_t* meth_c, const uint16_t* tot_c, int32_t s_c,
                    const uint16_t* meth_k, const uint16_t* tot_k, int32_t s_k, int64_t n_sites, double* E,
                    void* stream) {
  if (!m) return fail(HYG_EINVAL, "null model");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (s_c < 0 || s_k < 0 || n_sites < 0) return fail(HYG_EINVAL, "negative size");
  if (n_sites > 0 && (!E || (s_c && (!meth_c || !tot_c)) || (s_k && (!meth_k || !tot_k))))
    return fail(HYG_EINVAL, "null buffer");
  return launch_emission(m->dev(), m->c, meth_c, tot_c, s_c, meth_k, tot_k, s_k, n_sites, E, stream);
}

static size_t header_bytes(int32_t n_chains) {
  const size_t h = sizeof(ChainDev) * (size_t)n_chains + (sizeof(int32_t) + sizeof(double)) * (size_t)n_chains;
  return (h + 255) / 256 * 256;
}

size_t hyg_tg_workspace_bytes(const hyg_tg_model* m, int32_t n_chains, int64_t total_steps) {
  if (!m || n_chains < 0 || total_steps < 0) return 0;
  return header_bytes(n_chains) + (size_t)total_steps * record_bytes(m->c.M) + 256 +
         (size_t)n_chains * backward_scratch_bytes(m->c);
}

int hyg_tg_run_chains(const hyg_tg_model* m, const hyg_tg_chain* chains, int32_t n_chains, const double* E,
                      void* workspace, size_t workspace_bytes, const hyg_tg_outputs* out, void* stream) {
  if (!m || !chains || !out || !E || !workspace) return fail(HYG_EINVAL, "null argument");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (n_chains <= 0) return HYG_OK;
  if (!out->merged || !out->control || !out->kase || !out->split_probs || !out->regime_probs || !out->log_z)
    return fail(HYG_EINVAL, "null output buffer");
  if (!m->c.optimal) return fail(HYG_EUNSUPPORTED, "optimal_resampling = 0 is not implemented on the GPU path");
  std::vector<ChainDev> cd(n_chains);
  const size_t hb = header_bytes(n_chains);
  size_t off = hb;
  const size_t rb = record_bytes(m->c.M);
  for (int i = 0; i < n_chains; ++i) {
    const hyg_tg_chain& c = chains[i];
    if (c.n_sites < 1) return fail(HYG_EINVAL, "chain with no sites");
    if (c.n_sites > m->max_duration) return fail(HYG_EINVAL, "chain longer than the model's max_duration");
    if (c.site_begin < 0 || c.out_begin < 0) return fail(HYG_EINVAL, "negative chain offset");
    cd[i].site_begin = c.site_begin;
    cd[i].out_begin = c.out_begin;
    cd[i].ws_offset = (int64_t)off;
    cd[i].seed = c.seed;
    cd[i].chain_id = c.chain_id;
    cd[i].T = c.n_sites;
    cd[i].pad = 0;
    off += (size_t)c.n_sites * rb;
  }
  // the backward's full-N weight scratch of each chain (backward_global_w), behind the records
  const size_t sb = backward_scratch_bytes(m->c);
  off = (off + 255) / 256 * 256;
  for (int i = 0; i < n_chains; ++i) {
    cd[i].wg_offset = sb ? (int64_t)off : 0;
    off += sb;
  }
  if (off > workspace_bytes) return fail(HYG_EINVAL, "workspace too small (see hyg_tg_workspace_bytes)");
  uint8_t* ws = (uint8_t*)workspace;
  hipStream_t s = (hipStream_t)stream;
  if (m->stage.upload(ws, cd.data(), sizeof(ChainDev) * n_chains, s) != hipSuccess)
    return fail(HYG_EDEVICE, "descriptor upload failed");
  hyg_tg_outputs o = *out;
  if (!o.status) o.status = (int32_t*)(ws + sizeof(ChainDev) * n_chains);
  int rc = launch_chains(m->dev(), m->c, (const ChainDev*)ws, n_chains, E, ws, o, stream);
  if (rc == HYG_EUNSUPPORTED) return fail(rc, "particle arrays exceed the 160 KiB LDS of a CU (K too large)");
  if (rc != HYG_OK) return fail(rc, std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
  return HYG_OK;
}

int hyg_tg_run_chains_host(const hyg_tg_model* m, const uint16_t* meth_c, const uint16_t* tot_c, int32_t s_c,
                           const uint16_t* meth_k, const uint16_t* tot_k, int32_t s_k, int64_t n_sites,
                           const hyg_tg_chain* chains, int32_t n_chains, int64_t out_rows, int16_t* merged,
                           int16_t* control, int16_t* kase, float* split, float* regime, double* log_z,
                           double* final_w, int32_t* status) {
  if (!m) return fail(HYG_EINVAL, "null model");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (n_sites < 1 || n_chains < 1 || out_rows < 1 || s_c < 0 || s_k < 0) return fail(HYG_EINVAL, "empty or negative size");
  if (!chains || !merged || !control || !kase || !split || !regime || !log_z || !status)
    return fail(HYG_EINVAL, "null argument");
  if ((s_c && (!meth_c || !tot_c)) || (s_k && (!meth_k || !tot_k))) return fail(HYG_EINVAL, "null count buffer");
  int64_t steps = 0;
  for (int i = 0; i < n_chains; ++i) {
    const hyg_tg_chain& c = chains[i];
    if (c.n_sites < 1 || c.site_begin < 0 || c.out_begin < 0 || c.site_begin + c.n_sites > n_sites ||
        c.out_begin + c.n_sites > out_rows)
      return fail(HYG_EINVAL, "chain outside the sites or the output rows");
    steps += c.n_sites;
  }
  for (int64_t i = 0; i < n_sites * s_c; ++i)
    if (meth_c[i] > tot_c[i] || tot_c[i] > m->nmax_reads) return fail(HYG_EINVAL, "invalid control counts");
  for (int64_t i = 0; i < n_sites * s_k; ++i)
    if (meth_k[i] > tot_k[i] || tot_k[i] > m->nmax_reads) return fail(HYG_EINVAL, "invalid case counts");
  const size_t K = m->c.K, B = m->c.B, Nmax = m->c.Nmax, R = (size_t)out_rows, nch = (size_t)n_chains;
  struct Buf {
    void* p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
  } b_mc, b_tc, b_mk, b_tk, b_E, b_ws, b_mg, b_ct, b_ks, b_sp, b_rp, b_lz, b_fw, b_st;
  auto alloc = [](Buf& b, size_t n) { return hipMalloc(&b.p, n ? n : 1) == hipSuccess; };
  const size_t nc = (size_t)n_sites * s_c, nk = (size_t)n_sites * s_k;
  const size_t wsb = hyg_tg_workspace_bytes(m, n_chains, steps);
  bool ok = alloc(b_mc, nc * 2) && alloc(b_tc, nc * 2) && alloc(b_mk, nk * 2) && alloc(b_tk, nk * 2) &&
            alloc(b_E, sizeof(double) * (size_t)n_sites * 2 * K) && alloc(b_ws, wsb) && alloc(b_mg, 2 * R * B) &&
            alloc(b_ct, 4 * R * B) && alloc(b_ks, 4 * R * B) && alloc(b_sp, 4 * R) && alloc(b_rp, 4 * R * 2 * K) &&
            alloc(b_lz, 8 * nch) && (!final_w || alloc(b_fw, 8 * nch * Nmax)) && alloc(b_st, 4 * nch);
  if (!ok) return fail(HYG_ENOMEM, "device allocation failed");
  auto h2d = [](void* d, const void* h, size_t n) { return n == 0 || hipMemcpy(d, h, n, hipMemcpyHostToDevice) == hipSuccess; };
  auto d2h = [](void* h, const void* d, size_t n) { return hipMemcpy(h, d, n, hipMemcpyDeviceToHost) == hipSuccess; };
  if (!h2d(b_mc.p, meth_c, nc * 2) || !h2d(b_tc.p, tot_c, nc * 2) || !h2d(b_mk.p, meth_k, nk * 2) ||
      !h2d(b_tk.p, tot_k, nk * 2))
    return fail(HYG_EDEVICE, "copy failed");
  int rc = hyg_tg_emission(m, (uint16_t*)b_mc.p, (uint16_t*)b_tc.p, s_c, (uint16_t*)b_mk.p, (uint16_t*)b_tk.p, s_k,
                           n_sites, (double*)b_E.p, nullptr);
  if (rc) return rc;
  hyg_tg_outputs o{};
  o.merged = (int16_t*)b_mg.p;
  o.control = (int16_t*)b_ct.p;
  o.kase = (int16_t*)b_ks.p;
  o.split_probs = (float*)b_sp.p;
  o.regime_probs = (float*)b_rp.p;
  o.log_z = (double*)b_lz.p;
  o.final_log_weights = (double*)b_fw.p;
  o.status = (int32_t*)b_st.p;
  rc = hyg_tg_run_chains(m, chains, n_chains, (double*)b_E.p, b_ws.p, wsb, &o, nullptr);
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return fail(HYG_EDEVICE, "kernel execution failed");
  if (!d2h(status, b_st.p, 4 * nch) || !d2h(merged, b_mg.p, 2 * R * B) || !d2h(control, b_ct.p, 4 * R * B) ||
      !d2h(kase, b_ks.p, 4 * R * B) || !d2h(split, b_sp.p, 4 * R) || !d2h(regime, b_rp.p, 4 * R * 2 * K) ||
      !d2h(log_z, b_lz.p, 8 * nch) || (final_w && !d2h(final_w, b_fw.p, 8 * nch * Nmax)))
    return fail(HYG_EDEVICE, "copy failed");
  return HYG_OK;
}

int hyg_tg_run_chain_host(const hyg_tg_model* m, const uint16_t* meth_c, const uint16_t* tot_c, int32_t s_c,
                          const uint16_t* meth_k, const uint16_t* tot_k, int32_t s_k, int32_t T, uint64_t seed,
                          uint64_t chain_id, int16_t* merged, int16_t* control, int16_t* kase, float* split,
                          float* regime, double* log_z, double* final_w) {
  if (T < 1) return fail(HYG_EINVAL, "no sites");
  hyg_tg_chain ch{};
  ch.site_begin = 0;
  ch.n_sites = T;
  ch.seed = seed;
  ch.chain_id = chain_id;
  ch.out_begin = 0;
  int32_t st = HYG_OK;
  const int rc = hyg_tg_run_chains_host(m, meth_c, tot_c, s_c, meth_k, tot_k, s_k, T, &ch, 1, T, merged, control, kase,
                                        split, regime, log_z, final_w, &st);
  if (rc) return rc;
  if (st != HYG_OK) return fail(st, "all particle weights became -inf");
  return HYG_OK;
}

void hyg_set_kernel_timing(int enable) { set_kernel_timing(enable != 0); }

int hyg_tg_last_kernel_ms(float* ms3) {
  if (!ms3) return fail(HYG_EINVAL, "null argument");
  return last_kernel_ms(ms3);
}

// ============================================================ single group

void hyg_sg_params_default(hyg_sg_params* p) {
  std::memset(p, 0, sizeof(*p));
  // regimes_config defaults (bin/simulate_data:147-157), Beta moments as
  // get_known_parameters (model_functions.R:36-59)
  const double mu[6] = {0.95, 0.05, 0.80, 0.20, 0.50, 0.50};
  const double sg[6] = {0.05, 0.05, 0.1, 0.1, 0.1, 0.2886751};
  const double om[6] = {0.995, 0.975, 0.95, 0.925, 0.9, 0.9};
  p->n_regimes = 6;
  p->minimum_duration = 3;
  p->num_particles_max = 250;
  p->resample_type = 2;
  p->is_kappa_fixed = 1;
  p->theta_len = 36;
  for (int i = 0; i < 6; ++i) {
    const double nu = mu[i] * (1.0 - mu[i]) / (sg[i] * sg[i]) - 1.0;
    p->alpha[i] = mu[i] * nu;
    p->beta[i] = (1.0 - mu[i]) * nu;
    p->kappa[i] = 2.0;
  }
  // uniform off-diagonal transitions (equal log-weights), logit(omega)
  for (int i = 0; i < 30; ++i) p->theta[i] = std::log(1.0 / 5.0);
  for (int i = 0; i < 6; ++i) p->theta[30 + i] = std::log(om[i] / (1.0 - om[i]));
  p->epsilon = 0.01;
}

void hyg_sg_model_destroy(hyg_sg_model* m) {
  if (!m) return;
  if (m->on_device) {
    m->stage.release();
    (void)hipFree(m->d_consts);
    (void)hipFree(m->d_hz);
    (void)hipFree(m->d_ex);
    (void)hipFree(m->d_lf);
    (void)hipFree(m->d_lg);
    (void)hipFree(m->d_cst);
  }
  delete m;
}

int hyg_sg_model_create(const hyg_sg_params* params, int32_t max_total_reads, int32_t max_duration,
                        hyg_sg_model** out) {
  if (!params || !out) return fail(HYG_EINVAL, "null argument");
  *out = nullptr;
  if (max_total_reads < 0 || max_total_reads > 65535) return fail(HYG_EINVAL, "max_total_reads out of [0, 65535]");
  if (max_duration < 1 || max_duration >= HYG_DMAX - 2) return fail(HYG_EINVAL, "max_duration out of range");
  auto* m = new hyg_sg_model();
  int rc = hyg_sg_derive(params, &m->c);
  if (rc != HYG_OK) {
    delete m;
    return fail(rc, rc == HYG_EUNSUPPORTED ? "only resample_type 2 (optimal finite state) is implemented"
                                           : "invalid model parameters");
  }
  if (m->c.Nmax > kSgThreads) {
    delete m;
    return fail(HYG_EUNSUPPORTED, "num_particles_max > 256 (one particle per thread of a workgroup)");
  }
  m->params = *params;
  m->max_duration = max_duration;
  m->nmax_reads = max_total_reads;
  m->dcap = hyg_sg_hazard_len(&m->c, max_duration + 1);
  const int K = m->c.K, L = max_total_reads + 1;
  m->hz.resize((size_t)K * m->dcap * 2);
  m->ex.resize((size_t)K * m->dcap);
  hyg_sg_hazard_fill(&m->c, m->dcap, m->hz.data(), m->ex.data());
  m->lf.resize(L);
  m->lg.resize((size_t)3 * K * L);
  m->cst.resize(K);
  hyg_sg_bb_tables(&m->c, max_total_reads, m->lf.data(), m->lg.data(), m->cst.data());
  if (have_device()) {
    (void)hipGetDevice(&m->device);
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = dmalloc_copy(&m->d_consts, &m->c, 1);
    if (e == hipSuccess) e = dmalloc_copy(&m->d_hz, m->hz.data(), m->hz.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_ex, m->ex.data(), m->ex.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_lf, m->lf.data(), m->lf.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_lg, m->lg.data(), m->lg.size());
    if (e == hipSuccess) e = dmalloc_copy(&m->d_cst, m->cst.data(), m->cst.size());
    m->on_device = true;
    if (e != hipSuccess) {
      hyg_sg_model_destroy(m);
      return fail(HYG_EDEVICE, std::string("device upload failed: ") + hipGetErrorString(e));
    }
  }
  *out = m;
  return HYG_OK;
}

int hyg_sg_emission(const hyg_sg_model* m, const uint16_t* meth, const uint16_t* tot, int32_t n_samples,
                    int64_t n_sites, double* E, void* stream) {
  if (!m) return fail(HYG_EINVAL, "null model");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (n_samples < 0 || n_sites < 0) return fail(HYG_EINVAL, "negative size");
  if (n_sites > 0 && (!E || (n_samples && (!meth || !tot)))) return fail(HYG_EINVAL, "null buffer");
  int rc = sg_launch_emission(m->dev(), m->c, meth, tot, n_samples, n_sites, E, stream);
  if (rc != HYG_OK) return fail(rc, "emission launch failed");
  return HYG_OK;
}

// workspace header: chain descriptors + status words, then the ring control
// words of every chain (one contiguous block, zeroed before each launch)
static size_t sg_desc_bytes(int32_t n_chains) {
  const size_t h = (sizeof(SgChainDev) + sizeof(int32_t)) * (size_t)n_chains;
  return (h + 255) / 256 * 256;
}
static size_t sg_header_bytes(int32_t n_chains) {
  return sg_desc_bytes(n_chains) + (kSgCtlBytes * (size_t)n_chains + 255) / 256 * 256;
}
// per-chain offsets of the psi region, the ring and the control words
static void sg_chain_offsets(SgChainDev& d, int i, int32_t n_chains, size_t region, int K, int cap) {
  d.psi_offset = (int64_t)region;
  d.ring_offset = (int64_t)(region + sg_psi_region_bytes(K, cap) + sg_lists_bytes(cap));
  d.ctl_offset = (int64_t)(sg_desc_bytes(n_chains) + kSgCtlBytes * (size_t)i);
}

size_t hyg_sg_workspace_bytes(const hyg_sg_model* m, int32_t n_chains, int32_t psi_capacity) {
  if (!m || n_chains < 0 || psi_capacity < 0) return 0;
  const int cap = psi_capacity ? psi_capacity : kSgPsiCapDefault;
  return sg_header_bytes(n_chains) + (size_t)n_chains * sg_chain_ws_bytes(m->c.K, cap);
}

int hyg_sg_run_chains(const hyg_sg_model* m, const hyg_sg_chain* chains, int32_t n_chains, const double* E,
                      void* workspace, size_t workspace_bytes, int32_t psi_capacity, double* regime_probs,
                      int32_t* status, void* stream) {
  if (!m || !chains || !E || !workspace || !regime_probs) return fail(HYG_EINVAL, "null argument");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (n_chains <= 0) return HYG_OK;
  if (psi_capacity < 0 || psi_capacity > (1 << 24)) return fail(HYG_EINVAL, "psi_capacity out of range");
  const int cap = psi_capacity ? psi_capacity : kSgPsiCapDefault;
  if (workspace_bytes < hyg_sg_workspace_bytes(m, n_chains, psi_capacity))
    return fail(HYG_EINVAL, "workspace too small (see hyg_sg_workspace_bytes)");
  std::vector<SgChainDev> cd(n_chains);
  size_t off = sg_header_bytes(n_chains);
  const size_t per = sg_chain_ws_bytes(m->c.K, cap);
  for (int i = 0; i < n_chains; ++i) {
    const hyg_sg_chain& c = chains[i];
    if (c.n_sites < 1) return fail(HYG_EINVAL, "chain with no sites");
    if (c.n_sites > m->max_duration) return fail(HYG_EINVAL, "chain longer than the model's max_duration");
    if (c.site_begin < 0 || c.out_begin < 0) return fail(HYG_EINVAL, "negative chain offset");
    cd[i].site_begin = c.site_begin;
    cd[i].out_begin = c.out_begin;
    sg_chain_offsets(cd[i], i, n_chains, off, m->c.K, cap);
    cd[i].seed = c.seed;
    cd[i].chain_id = c.chain_id;
    cd[i].T = c.n_sites;
    cd[i].rcap = 0;
    cd[i].pe_offset = 0;
    cd[i].theta_row = 0;
    off += per;
  }
  uint8_t* ws = (uint8_t*)workspace;
  hipStream_t s = (hipStream_t)stream;
  if (m->stage.upload(ws, cd.data(), sizeof(SgChainDev) * n_chains, s) != hipSuccess)
    return fail(HYG_EDEVICE, "descriptor upload failed");
  int32_t* st = status ? status : (int32_t*)(ws + sizeof(SgChainDev) * n_chains);
  int rc = sg_launch_chains(m->dev(), m->c, (const SgChainDev*)ws, n_chains, E, ws, cap, regime_probs, st,
                            ws + sg_desc_bytes(n_chains), stream);
  if (rc == HYG_EUNSUPPORTED) return fail(rc, "particle arrays exceed the LDS of a CU (K too large)");
  if (rc != HYG_OK) return fail(rc, std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
  return HYG_OK;
}

int hyg_sg_run_chain_host(const hyg_sg_model* m, const uint16_t* meth, const uint16_t* tot, int32_t S, int32_t T,
                          uint64_t seed, uint64_t chain_id, double* regime_probs) {
  if (!m || !regime_probs || (S > 0 && (!meth || !tot))) return fail(HYG_EINVAL, "null argument");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (T < 1 || S < 0) return fail(HYG_EINVAL, "no sites");
  for (int64_t i = 0; i < (int64_t)T * S; ++i)
    if (tot[i] > m->nmax_reads) return fail(HYG_EINVAL, "total read count above the model's max_total_reads");
  const int K = m->c.K;
  struct Buf {
    void* p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
  } b_m, b_t, b_E, b_ws, b_p, b_st;
  auto alloc = [](Buf& b, size_t n) { return hipMalloc(&b.p, n ? n : 1) == hipSuccess; };
  const size_t nc = (size_t)T * S;
  const size_t wsb = hyg_sg_workspace_bytes(m, 1, 0);
  bool ok = alloc(b_m, nc * 2) && alloc(b_t, nc * 2) && alloc(b_E, sizeof(double) * T * K) && alloc(b_ws, wsb) &&
            alloc(b_p, sizeof(double) * T * K) && alloc(b_st, 4);
  if (!ok) return fail(HYG_ENOMEM, "device allocation failed");
  if (nc && hipMemcpy(b_m.p, meth, nc * 2, hipMemcpyHostToDevice) != hipSuccess) return fail(HYG_EDEVICE, "copy failed");
  if (nc && hipMemcpy(b_t.p, tot, nc * 2, hipMemcpyHostToDevice) != hipSuccess) return fail(HYG_EDEVICE, "copy failed");
  int rc = hyg_sg_emission(m, (uint16_t*)b_m.p, (uint16_t*)b_t.p, S, T, (double*)b_E.p, nullptr);
  if (rc) return rc;
  hyg_sg_chain ch{};
  ch.site_begin = 0;
  ch.n_sites = T;
  ch.seed = seed;
  ch.chain_id = chain_id;
  ch.out_begin = 0;
  rc = hyg_sg_run_chains(m, &ch, 1, (double*)b_E.p, b_ws.p, wsb, 0, (double*)b_p.p, (int32_t*)b_st.p, nullptr);
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return fail(HYG_EDEVICE, "kernel execution failed");
  int32_t st = 0;
  if (hipMemcpy(&st, b_st.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return fail(HYG_EDEVICE, "copy failed");
  if (hipMemcpy(regime_probs, b_p.p, sizeof(double) * T * K, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(HYG_EDEVICE, "copy failed");
  if (st == HYG_ENOMEM) return fail(st, "pending smoothing times exceeded psi_capacity");
  if (st != HYG_OK) return fail(st, "all particle weights became -inf");
  return HYG_OK;
}

// ---- online parameter estimation

void hyg_sg_pe_params_default(hyg_sg_pe_params* pe) {
  std::memset(pe, 0, sizeof(*pe));
  // bin/estimate_parameters_and_regimes:130-200 flag defaults
  pe->use_adam = 1;
  pe->normalise_gradients = 0;
  pe->n_steps_without_update = 200;
  pe->learning_rate_exponent = 0.1;
  pe->learning_rate_factor = 0.01;
}

static int sg_pe_rcap(int T) { return T + 1 < HYG_SGPE_DCAP ? T + 1 : HYG_SGPE_DCAP; }

int64_t hyg_sg_pe_theta_rows(const hyg_sg_chain* chains, int32_t n_chains, int32_t every) {
  if (!chains || n_chains < 0 || every < 1) return -1;
  int64_t rows = 0;
  for (int i = 0; i < n_chains; ++i) rows += hyg_sgpe_theta_rows(chains[i].n_sites, every);
  return rows;
}

size_t hyg_sg_pe_workspace_bytes(const hyg_sg_model* m, const hyg_sg_chain* chains, int32_t n_chains,
                                 int32_t psi_capacity) {
  if (!m || !chains || n_chains < 0 || psi_capacity < 0) return 0;
  size_t b = hyg_sg_workspace_bytes(m, n_chains, psi_capacity);
  for (int i = 0; i < n_chains; ++i) b += sg_pe_region_bytes(m->c.K, sg_pe_rcap(std::max(chains[i].n_sites, 1)));
  return b;
}

int hyg_sg_run_chains_pe(const hyg_sg_model* m, const hyg_sg_pe_params* pe, const hyg_sg_chain* chains,
                         int32_t n_chains, const double* E, void* workspace, size_t workspace_bytes,
                         int32_t psi_capacity, double* regime_probs, double* theta_out, int32_t* status,
                         void* stream) {
  if (!m || !pe || !chains || !E || !workspace || !regime_probs || !theta_out) return fail(HYG_EINVAL, "null argument");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (n_chains <= 0) return HYG_OK;
  if (psi_capacity < 0 || psi_capacity > (1 << 24)) return fail(HYG_EINVAL, "psi_capacity out of range");
  hyg_sgpe_consts pc{};
  int rc = hyg_sgpe_consts_make(&m->params, pe, &pc);
  if (rc != HYG_OK) return fail(rc, "invalid parameter-estimation settings");
  const int cap = psi_capacity ? psi_capacity : kSgPsiCapDefault;
  if (workspace_bytes < hyg_sg_pe_workspace_bytes(m, chains, n_chains, psi_capacity))
    return fail(HYG_EINVAL, "workspace too small (see hyg_sg_pe_workspace_bytes)");
  const int K = m->c.K, dim = pc.dim;  // theta length: K^2, or K (K + 1) with kappa estimated
  std::vector<SgChainDev> cd(n_chains);
  size_t off = sg_header_bytes(n_chains);
  const size_t per = sg_chain_ws_bytes(K, cap);
  size_t pe_off = off + per * (size_t)n_chains;
  int64_t row = 0, max_rows = 1;
  int max_rcap = 1;
  for (int i = 0; i < n_chains; ++i) {
    const hyg_sg_chain& c = chains[i];
    if (c.n_sites < 1) return fail(HYG_EINVAL, "chain with no sites");
    if (c.n_sites > m->max_duration) return fail(HYG_EINVAL, "chain longer than the model's max_duration");
    if (c.site_begin < 0 || c.out_begin < 0) return fail(HYG_EINVAL, "negative chain offset");
    cd[i].site_begin = c.site_begin;
    cd[i].out_begin = c.out_begin;
    sg_chain_offsets(cd[i], i, n_chains, off, K, cap);
    cd[i].seed = c.seed;
    cd[i].chain_id = c.chain_id;
    cd[i].T = c.n_sites;
    cd[i].rcap = sg_pe_rcap(c.n_sites);
    cd[i].pe_offset = (int64_t)pe_off;
    cd[i].theta_row = row;
    const int64_t nr = hyg_sgpe_theta_rows(c.n_sites, pc.every);
    row += nr;
    max_rows = std::max(max_rows, nr);
    max_rcap = std::max(max_rcap, cd[i].rcap);
    off += per;
    pe_off += sg_pe_region_bytes(K, cd[i].rcap);
  }
  // model-level inputs: theta0 [dim] | steps [max_rows] | lgk [K][max_rcap] | dgk [K][max_rcap] (kappa estimated)
  std::vector<hyg_sgpe_step> steps((size_t)max_rows);
  hyg_sgpe_steps_fill(pe, (int)max_rows, steps.data());
  std::vector<double> lgk((size_t)K * max_rcap), dgk(pc.kest ? (size_t)K * max_rcap : 0);
  hyg_sgpe_lgk_fill(pc.kappa, K, max_rcap, lgk.data());
  if (pc.kest) hyg_sgpe_dgk_fill(pc.kappa, K, max_rcap, dgk.data());
  const size_t b_th = sizeof(double) * dim, b_st = sizeof(hyg_sgpe_step) * steps.size(),
               b_lg = sizeof(double) * lgk.size(), b_dg = sizeof(double) * dgk.size();
  std::vector<unsigned char> host(b_th + b_st + b_lg + b_dg);
  std::memcpy(host.data(), m->params.theta, b_th);
  std::memcpy(host.data() + b_th, steps.data(), b_st);
  std::memcpy(host.data() + b_th + b_st, lgk.data(), b_lg);
  if (b_dg) std::memcpy(host.data() + b_th + b_st + b_lg, dgk.data(), b_dg);
  hipStream_t s = (hipStream_t)stream;
  void* dbuf = nullptr;
  if (hipMallocAsync(&dbuf, host.size(), s) != hipSuccess) return fail(HYG_ENOMEM, "device allocation failed");
  if (hipMemcpyAsync(dbuf, host.data(), host.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFreeAsync(dbuf, s);
    return fail(HYG_EDEVICE, "upload failed");
  }
  uint8_t* ws = (uint8_t*)workspace;
  if (m->stage.upload(ws, cd.data(), sizeof(SgChainDev) * n_chains, s) != hipSuccess) {
    (void)hipFreeAsync(dbuf, s);
    return fail(HYG_EDEVICE, "descriptor upload failed");
  }
  SgPeDev pd{};
  pd.c = pc;
  pd.theta0 = (const double*)dbuf;
  pd.steps = (const hyg_sgpe_step*)((unsigned char*)dbuf + b_th);
  pd.lgk = (const double*)((unsigned char*)dbuf + b_th + b_st);
  pd.dgk = pc.kest ? (const double*)((unsigned char*)dbuf + b_th + b_st + b_lg) : nullptr;
  pd.lgk_stride = max_rcap;
  pd.theta_out = theta_out;
  int32_t* st = status ? status : (int32_t*)(ws + sizeof(SgChainDev) * n_chains);
  rc = sg_launch_chains(m->dev(), m->c, (const SgChainDev*)ws, n_chains, E, ws, cap, regime_probs, st,
                        ws + sg_desc_bytes(n_chains), stream, &pd);
  (void)hipFreeAsync(dbuf, s);
  if (rc == HYG_EUNSUPPORTED) return fail(rc, "particle arrays exceed the LDS of a CU (K too large)");
  if (rc != HYG_OK) return fail(rc, std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
  return HYG_OK;
}

int hyg_sg_run_chain_host_pe(const hyg_sg_model* m, const hyg_sg_pe_params* pe, const uint16_t* meth,
                             const uint16_t* tot, int32_t S, int32_t T, uint64_t seed, uint64_t chain_id,
                             double* regime_probs, double* theta_out) {
  if (!m || !pe || !regime_probs || !theta_out || (S > 0 && (!meth || !tot))) return fail(HYG_EINVAL, "null argument");
  if (!m->on_device) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (!on_model_device(m->device)) return fail(HYG_EINVAL, "the current HIP device is not the model's device");
  if (T < 1 || S < 0) return fail(HYG_EINVAL, "no sites");
  if (pe->n_steps_without_update < 1) return fail(HYG_EINVAL, "n_steps_without_update < 1");
  for (int64_t i = 0; i < (int64_t)T * S; ++i)
    if (tot[i] > m->nmax_reads) return fail(HYG_EINVAL, "total read count above the model's max_total_reads");
  const int K = m->c.K;
  struct Buf {
    void* p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
  } b_m, b_t, b_E, b_ws, b_p, b_st, b_th;
  auto alloc = [](Buf& b, size_t n) { return hipMalloc(&b.p, n ? n : 1) == hipSuccess; };
  hyg_sg_chain ch{};
  ch.site_begin = 0;
  ch.n_sites = T;
  ch.seed = seed;
  ch.chain_id = chain_id;
  ch.out_begin = 0;
  const size_t nc = (size_t)T * S;
  const size_t wsb = hyg_sg_pe_workspace_bytes(m, &ch, 1, 0);
  const int64_t rows = hyg_sgpe_theta_rows(T, pe->n_steps_without_update);
  const int dth = m->params.is_kappa_fixed ? K * K : K * (K + 1);
  const size_t thb = sizeof(double) * (size_t)rows * dth;
  bool ok = alloc(b_m, nc * 2) && alloc(b_t, nc * 2) && alloc(b_E, sizeof(double) * T * K) && alloc(b_ws, wsb) &&
            alloc(b_p, sizeof(double) * T * K) && alloc(b_st, 4) && alloc(b_th, thb);
  if (!ok) return fail(HYG_ENOMEM, "device allocation failed");
  if (nc && hipMemcpy(b_m.p, meth, nc * 2, hipMemcpyHostToDevice) != hipSuccess) return fail(HYG_EDEVICE, "copy failed");
  if (nc && hipMemcpy(b_t.p, tot, nc * 2, hipMemcpyHostToDevice) != hipSuccess) return fail(HYG_EDEVICE, "copy failed");
  int rc = hyg_sg_emission(m, (uint16_t*)b_m.p, (uint16_t*)b_t.p, S, T, (double*)b_E.p, nullptr);
  if (rc) return rc;
  rc = hyg_sg_run_chains_pe(m, pe, &ch, 1, (double*)b_E.p, b_ws.p, wsb, 0, (double*)b_p.p, (double*)b_th.p,
                            (int32_t*)b_st.p, nullptr);
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return fail(HYG_EDEVICE, "kernel execution failed");
  int32_t st = 0;
  if (hipMemcpy(&st, b_st.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return fail(HYG_EDEVICE, "copy failed");
  if (hipMemcpy(regime_probs, b_p.p, sizeof(double) * T * K, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(theta_out, b_th.p, thb, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(HYG_EDEVICE, "copy failed");
  if (st == HYG_ENOMEM) return fail(st, "pending smoothing times exceeded psi_capacity, or a sojourn outgrew the hazard rows");
  if (st != HYG_OK) return fail(st, "all particle weights became -inf");
  return HYG_OK;
}

// ---- regime BED tracks

int hyg_bed_labels(const double* probs, int32_t K, int64_t n, int8_t* label, double* score, void* stream) {
  if (K < 1 || K > HYG_KMAX || n < 0) return fail(HYG_EINVAL, "K out of [1, 16] or negative n_sites");
  if (n > 0 && (!probs || !label || !score)) return fail(HYG_EINVAL, "null buffer");
  if (!have_device()) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  const int rc = bed_launch_labels(probs, K, n, label, score, stream);
  if (rc != HYG_OK) return fail(rc, "label launch failed");
  return HYG_OK;
}

int64_t hyg_bed_format(const char* chrom, const int64_t* pos, const int8_t* label, const double* score, int64_t n,
                       int32_t K, const char* const* names, const char* const* rgb, char* out, int64_t out_bytes) {
  if (!chrom || K < 1 || K > HYG_KMAX || n < 0 || !names || !rgb) return fail(HYG_EINVAL, "invalid argument");
  if (n > 0 && (!pos || !label || !score)) return fail(HYG_EINVAL, "null buffer");
  for (int r = 0; r <= K; ++r)
    if (!names[r] || !rgb[r]) return fail(HYG_EINVAL, "null name or colour");
  int64_t need = 0;
  char line[512];
  for (int64_t i = 0; i < n; ++i) {
    const int lb = label[i];
    if (lb < -1 || lb >= K) return fail(HYG_EINVAL, "label out of range");
    const int k = lb < 0 ? K : lb;
    char sc[64];
    // fwrite(scipen = 999): fixed notation, <= 15 significant digits, no trailing zeros
    int m = std::snprintf(sc, sizeof sc, "%.15g", score[i]);
    if (std::strchr(sc, 'e')) {  // tiny or huge values: positional form of the same digits
      m = std::snprintf(sc, sizeof sc, "%.17f", score[i]);
      while (m > 1 && sc[m - 1] == '0') sc[--m] = 0;
      if (m > 1 && sc[m - 1] == '.') sc[--m] = 0;
    }
    const long long a = (long long)pos[i] - 1, b = (long long)pos[i] + 1;
    const int len = std::snprintf(line, sizeof line, "%s\t%lld\t%lld\t%s\t%s\t.\t%lld\t%lld\t%s\n", chrom, a, b,
                                  names[k], sc, a, b, rgb[k]);
    if (len < 0 || len >= (int)sizeof line) return fail(HYG_EINVAL, "BED line too long");
    if (out && need + len <= out_bytes) std::memcpy(out + need, line, (size_t)len);
    need += len;
  }
  return need;
}

// ---- preprocess

int hyg_pre_collapse(const int64_t* pos0, int64_t T, const int64_t* plus_start, const int64_t* plus_end,
                     const double* plus_cov, const double* plus_pct, int64_t n_plus, const int64_t* minus_start,
                     const double* minus_cov, const double* minus_pct, int64_t n_minus, int32_t plus_single_base,
                     uint8_t* scratch, double* counts, int32_t stride, int32_t column, int32_t* conflicts,
                     void* stream) {
  if (T < 0 || n_plus < 0 || n_minus < 0 || stride < 2 || column < 0 || column + 2 > stride)
    return fail(HYG_EINVAL, "invalid sizes (need 0 <= column, column + 2 <= stride)");
  if ((T > 0 && (!pos0 || !counts || !conflicts)) || (n_plus > 0 && (!plus_start || !plus_end || !plus_cov || !plus_pct)) ||
      (n_minus > 0 && (!minus_start || !minus_cov || !minus_pct || (!scratch && !plus_single_base))))
    return fail(HYG_EINVAL, "null buffer");
  if (!have_device()) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  const int rc = pre_launch_collapse(pos0, T, plus_start, plus_end, plus_cov, plus_pct, n_plus, minus_start, minus_cov,
                                     minus_pct, n_minus, plus_single_base ? 1 : 0, scratch, counts, stride, column,
                                     conflicts, stream);
  if (rc != HYG_OK) return fail(rc, "preprocess launch failed");
  return HYG_OK;
}

}  // extern "C"

// ================================================ aggregation and DMPs
namespace {

struct DevBuf {  // RAII device allocation
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  bool alloc(size_t n) { return hipMalloc(&p, n ? n : 1) == hipSuccess; }
};

// FDR_procedure's statistics in numpy's sorted order (ascending t = 1 - c/P,
// i.e. descending c), as runs of hist[c] equal values.
struct SortedStats {
  const std::vector<uint32_t>& hist;
  int P;
  double value(int c) const { return 1.0 - (double)c / (double)P; }
};

}  // namespace

extern "C" {

int hyg_tg_posterior_counts(const float* split, const float* regime, int32_t K, int32_t B, const int64_t* segments,
                            int32_t n_segments, int64_t max_rows, int32_t exclusive, int32_t* counts,
                            void* stream) {
  if (!split || !regime || !counts || (n_segments > 0 && !segments) || K < 1 || K > HYG_KMAX || B < 1 ||
      n_segments < 0 || max_rows < 0)
    return fail(HYG_EINVAL, "hyg_tg_posterior_counts: invalid arguments");
  if (!have_device()) return fail(HYG_EDEVICE, "no HIP device: hygeia_amd has no CPU fallback");
  if (launch_post_counts(split, regime, 2 * K, B, segments, n_segments, max_rows, exclusive != 0, counts, stream))
    return fail(HYG_EDEVICE, "posterior_counts launch failed");
  return HYG_OK;
}

int hyg_dmp_site_counts(const int16_t* merged, const int16_t* control, const int16_t* kase, int32_t B, int32_t K,
                        const hyg_dmp_group* groups, const int64_t* block_rows, int32_t n_groups, int32_t n_seeds,
                        int64_t n_sites, int32_t* counts, int32_t* pairs, void* stream) {
  if (!merged || !control || !kase || !counts || B < 1 || K < 1 || K > HYG_KMAX || n_groups < 0 || n_seeds < 1 ||
      (n_groups > 0 && (!groups || !block_rows)))
    return fail(HYG_EINVAL, "hyg_dmp_site_counts: invalid arguments");
  if (!have_device()) return fail(HYG_EDEVICE, "no HIP device");
  if (n_groups == 0) return HYG_OK;
  std::vector<int64_t> row0(n_groups + 1), site(n_groups);
  row0[0] = 0;
  for (int g = 0; g < n_groups; ++g) {
    if (groups[g].n_rows < 0 || groups[g].site_begin < 0 || groups[g].site_begin + groups[g].n_rows > n_sites)
      return fail(HYG_EINVAL, "hyg_dmp_site_counts: group outside [0, n_sites)");
    row0[g + 1] = row0[g] + groups[g].n_rows;
    site[g] = groups[g].site_begin;
  }
  DevBuf d_row0, d_site, d_blk;
  const size_t nb = (size_t)n_groups * n_seeds;
  if (!d_row0.alloc(sizeof(int64_t) * (n_groups + 1)) || !d_site.alloc(sizeof(int64_t) * n_groups) ||
      !d_blk.alloc(sizeof(int64_t) * nb))
    return fail(HYG_ENOMEM, "device allocation failed");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(d_row0.p, row0.data(), sizeof(int64_t) * (n_groups + 1), hipMemcpyHostToDevice, s) ||
      hipMemcpyAsync(d_site.p, site.data(), sizeof(int64_t) * n_groups, hipMemcpyHostToDevice, s) ||
      hipMemcpyAsync(d_blk.p, block_rows, sizeof(int64_t) * nb, hipMemcpyHostToDevice, s))
    return fail(HYG_EDEVICE, "copy failed");
  if (launch_dmp_site_counts(merged, control, kase, B, K, (const int64_t*)d_row0.p, (const int64_t*)d_site.p,
                             (const int64_t*)d_blk.p, n_groups, n_seeds, row0[n_groups], counts, pairs, stream))
    return fail(HYG_EDEVICE, "dmp_site_counts launch failed");
  // the descriptors are freed on return: wait for the kernel
  if (hipStreamSynchronize(s) != hipSuccess) return fail(HYG_EDEVICE, "kernel execution failed");
  return HYG_OK;
}

int hyg_dmp_fdr(const int32_t* counts, int32_t stride, int32_t column, int64_t n, int32_t P, double thr, int64_t* k,
                double* q_k, double* threshold, void* stream) {
  if (!counts || !k || !q_k || !threshold || n < 1 || P < 1 || stride < 1 || column < 0 || column >= stride)
    return fail(HYG_EINVAL, "hyg_dmp_fdr: invalid arguments");
  if (!have_device()) return fail(HYG_EDEVICE, "no HIP device");
  hipStream_t s = (hipStream_t)stream;
  DevBuf d_hist, d_bad;
  if (!d_hist.alloc(sizeof(uint32_t) * (P + 1)) || !d_bad.alloc(sizeof(int32_t)))
    return fail(HYG_ENOMEM, "device allocation failed");
  if (hipMemsetAsync(d_hist.p, 0, sizeof(uint32_t) * (P + 1), s) || hipMemsetAsync(d_bad.p, 0, 4, s))
    return fail(HYG_EDEVICE, "memset failed");
  if (launch_dmp_hist(counts, stride, column, n, P, (uint32_t*)d_hist.p, (int32_t*)d_bad.p, stream))
    return fail(HYG_EDEVICE, "dmp_hist launch failed");
  std::vector<uint32_t> hist(P + 1);
  int32_t bad = 0;
  if (hipMemcpyAsync(hist.data(), d_hist.p, sizeof(uint32_t) * (P + 1), hipMemcpyDeviceToHost, s) ||
      hipMemcpyAsync(&bad, d_bad.p, 4, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
    return fail(HYG_EDEVICE, "kernel execution failed");
  if (bad) return fail(HYG_EINVAL, "hyg_dmp_fdr: a count lies outside [0, n_particles]");
  const SortedStats st{hist, P};
  int cmax = P;
  while (cmax >= 0 && hist[cmax] == 0) --cmax;
  // ordered_test_statistics[0] (:4) is the statistic of the largest count
  if (thr < st.value(cmax)) {  // (:8-9)
    *k = 0; *q_k = 0.0; *threshold = 0.0;
    return HYG_OK;
  }
  // Qs = 1./linspace(1, n, n) * cumsum(ordered) (:5-6), numpy's sequential
  // float64 cumsum; s = sum(Qs <= thr) (:7)
  double acc = 0.0, q_last = 0.0, q_s1 = 0.0;
  int64_t i = 0, cnt = 0;
  for (int c = cmax; c >= 0; --c) {
    const double v = st.value(c);
    for (uint32_t r = 0; r < hist[c]; ++r, ++i) {
      acc = (i == 0) ? v : acc + v;
      const double q = (1.0 / (double)(i + 1)) * acc;
      cnt += (q <= thr) ? 1 : 0;
      q_last = q;
    }
  }
  const int64_t sel = cnt;
  if (sel == n) {  // `s == test_statistics.shape` (:10-11)
    *k = n; *q_k = q_last; *threshold = 1.01;
    return HYG_OK;
  }
  // Qs[s-1] and ordered[s] (:12): replay up to position s
  acc = 0.0; i = 0;
  double ord_s = 0.0;
  bool done = false;
  for (int c = cmax; c >= 0 && !done; --c) {
    const double v = st.value(c);
    for (uint32_t r = 0; r < hist[c]; ++r, ++i) {
      if (i == sel) { ord_s = v; done = true; break; }
      acc = (i == 0) ? v : acc + v;
      q_s1 = (1.0 / (double)(i + 1)) * acc;
    }
  }
  *k = sel; *q_k = q_s1; *threshold = ord_s;
  return HYG_OK;
}

int hyg_dmp_weighted_fdr(const int32_t* counts, int32_t stride, int32_t column, int64_t n, int32_t P, double thr,
                         const double* w_fp, const double* w_fn, int64_t* ranked, int64_t* s_out, double* n_sum,
                         void* stream) {
  if (!counts || !w_fp || !w_fn || !ranked || !s_out || !n_sum || n < 1 || n > 0x7fffffffll || P < 1 ||
      stride < 1 || column < 0 || column >= stride)
    return fail(HYG_EINVAL, "hyg_dmp_weighted_fdr: invalid arguments");
  if (!have_device()) return fail(HYG_EDEVICE, "no HIP device");
  hipStream_t s = (hipStream_t)stream;
  DevBuf d_keys, d_vals, d_exc, d_tmp, d_er;
  if (!d_keys.alloc(8 * (size_t)n) || !d_vals.alloc(4 * (size_t)n) || !d_exc.alloc(8 * (size_t)n) ||
      !d_tmp.alloc(radix_temp_bytes(n)) || !d_er.alloc(8 * (size_t)n))
    return fail(HYG_ENOMEM, "device allocation failed");
  if (launch_dmp_rank(counts, stride, column, n, P, thr, w_fp, w_fn, (uint64_t*)d_keys.p, (uint32_t*)d_vals.p,
                      (double*)d_exc.p, stream))
    return fail(HYG_EDEVICE, "dmp_rank launch failed");
  if (radix_sort_pairs((uint64_t*)d_keys.p, (uint32_t*)d_vals.p, n, d_tmp.p, stream))
    return fail(HYG_EDEVICE, "radix sort launch failed");
  if (launch_dmp_gather((const uint32_t*)d_vals.p, (const double*)d_exc.p, n, (double*)d_er.p, ranked, stream))
    return fail(HYG_EDEVICE, "dmp_gather launch failed");
  std::vector<double> e((size_t)n);
  if (hipMemcpyAsync(e.data(), d_er.p, 8 * (size_t)n, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
    return fail(HYG_EDEVICE, "kernel execution failed");
  // Nsums = np.cumsum(ranked excess rates) (:20), s = sum(Nsums <= 0) (:21)
  double acc = 0.0;
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; ++i) {
    acc = (i == 0) ? e[0] : acc + e[i];
    cnt += (acc <= 0.0) ? 1 : 0;
  }
  const int64_t last = (cnt == 0) ? n - 1 : cnt - 1;  // Nsums[s - 1]
  acc = 0.0;
  for (int64_t i = 0; i <= last; ++i) acc = (i == 0) ? e[0] : acc + e[i];
  *s_out = cnt;
  *n_sum = acc;
  return HYG_OK;
}

}  // extern "C"
