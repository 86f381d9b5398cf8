// bmpc_hip.hip -- the C ABI of libbmpc.so (include/bmpc.h) and the small kernels (scene step,
// model / HMM evaluation, band QP, slab gather / scatter).  The solver kernels live in
// bmpc_dev.h / bmpc_k_*.hip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "bmpc_dev.h"

using namespace bmpc;
using namespace bmpc::dev;

#if defined(BMPC_WITH_PHASED)
#ifndef BMPC_IPM_PHASED_DEFAULT
#define BMPC_IPM_PHASED_DEFAULT 0
#endif
#ifndef BMPC_PH_STREAMS_DEFAULT
#define BMPC_PH_STREAMS_DEFAULT 4
#endif
#endif

namespace {

// LDS-rich launch (topology tables and coupling system in LDS) only when it costs no
// resident ego: a workgroup's LDS bounds the egos per CU (160 KB / bytes, at most 16 with 4
// waves per SIMD).  Deep trees (N=30, NB=2: 17 KB of tables, a 20 KB coupling matrix) run
// lean, 16 egos per CU instead of 4, unless the batch is resident either way.  BMPC_LDS_RICH=0/1
// forces either.
static bool choose_lds_rich(const Plan& P, bool transform, int batch, int cus, size_t lds_per_cu) {
  if (const char* e = getenv("BMPC_LDS_RICH")) return atoi(e) != 0;
  auto egos = [&](size_t b) { return std::min<size_t>(16, lds_per_cu / std::max<size_t>(b, 1)); };
  const size_t rich = egos(solver_lds_bytes(P, transform, true));
  // a batch that is resident either way (one CU per `rich` egos) runs rich: residency is not
  // what limits it
  return (size_t)batch <= (size_t)cus * rich || rich >= egos(solver_lds_bytes(P, transform, false));
}

// one thread per ego: the closed-loop scene step (bmpc_env.h) around the solve
__global__ void k_env(bmpc_env_desc E, double dt, int N, int m, int U, int d, int t, int batch, double* scene,
                      bmpc_policy* pol, const double* upred, const double* J, const int32_t* status,
                      const int32_t* iters, int cvar, double* x, double* z, double* xref, double* stats) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= batch) return;
  double* st = scene + (size_t)e * ENV_STRIDE;
  if (t > 0 && stats && J && status && iters)
    env_accumulate(st, J[e], status[e], iters[e], cvar != 0, stats + (size_t)e * ENVS_STRIDE);
  env_step_ego(E, dt, N, m, t, st, pol + (size_t)e * m, upred ? upred + (size_t)e * U * d : nullptr,
               x + (size_t)e * 4, z + (size_t)e * 4, xref + (size_t)e * 4);
}

__global__ void k_gather(const double* __restrict__ ws, size_t stride, size_t off, int count,
                         double* __restrict__ out, int batch) {
  const size_t tot = (size_t)batch * count;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i / count, j = i % count;
    out[i] = ws[e * stride + off + j];
  }
}

__global__ void k_scatter(double* __restrict__ ws, size_t stride, size_t off, int count,
                          const double* __restrict__ in, const uint8_t* __restrict__ mask, int batch) {
  const size_t tot = (size_t)batch * count;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    const size_t e = i / count, j = i % count;
    if (!mask || mask[e]) ws[e * stride + off + j] = in[i];
  }
}

__global__ void k_reset(double* ws, size_t stride, size_t off, const uint8_t* mask, int batch) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < batch && (!mask || mask[e])) ws[e * stride + off + MISC_INIT] = 0.0;
}

template <class M>
__global__ void k_model(bmpc_plan_desc D, const bmpc_policy* pol, int B, const double* x,
                        const double* u, const double* z, double* A, double* Bm, double* C,
                        double* xp, double* p, double* dp, double* zpred, double* h0, double* dh,
                        LaneRef R) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int n = D.n, d = D.d, m = D.m, N = D.N;
#define OFF(ptr, k) (ptr ? ptr + (size_t)b * (k) : nullptr)
  model_eval_point<M>(D, pol + (size_t)b * m, x + b * n, u + b * d, z + b * n, OFF(A, n * n),
                      OFF(Bm, n * d), OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n),
                      OFF(zpred, N * m * n), OFF(h0, 1), OFF(dh, n), R);
#undef OFF
}

bool is_psiref(int kind) {
  return kind == BMPC_POL_MAINTAIN_PSIREF || kind == BMPC_POL_MAINTAIN_TRACKV_PSIREF ||
         kind == BMPC_POL_BRAKE_PSIREF;
}

// a lane reference as bmpc_model_eval_ref / bmpc_set_lane_ref take it; "" when valid
std::string check_lane_ref(int nref, const double* grid, const double* values) {
  if (nref == 0) return "";
  if (nref < 2 || nref > BMPC_MAX_LANE_REF) return "lane reference: need 2 <= nref <= BMPC_MAX_LANE_REF";
  if (!grid || !values) return "lane reference: null grid / values";
  for (int i = 0; i + 1 < nref; ++i)
    if (!(grid[i + 1] > grid[i])) return "lane reference: the grid must be strictly increasing";
  for (int i = 0; i < nref; ++i)
    if (!std::isfinite(grid[i]) || !std::isfinite(values[i])) return "lane reference: non-finite entry";
  return "";
}

__global__ void k_hmm(int M, int m, const double* __restrict__ hc, int B, const double* xb, const double* u,
                      const double* xbackup, double* xbp, double* A, double* Bm, double* C, double* h0,
                      double* Jh) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= B) return;
  const int nb = 4 + M * m;
#define OFF(ptr, k) (ptr ? ptr + (size_t)p * (k) : nullptr)
  hmm_linearize(M, m, hc, xb + (size_t)p * nb, u + (size_t)p * 2, xbackup + (size_t)p * M * m * 4, OFF(xbp, nb),
                OFF(A, nb * nb), OFF(Bm, nb * 2), OFF(C, nb), OFF(h0, M * m), OFF(Jh, M * m * nb));
#undef OFF
}

// one wave per QP of the batch (bmpc_bandqp.h); d's tables are device pointers
__global__ __launch_bounds__(64) void k_bandqp(BandQPDesc d, const double* __restrict__ vals,
                                               const double* __restrict__ cvals, double* __restrict__ ws,
                                               double* x, double* y, int32_t* status, int32_t* iters, int batch) {
  const int b = blockIdx.x;
  if (b >= batch) return;
  extern __shared__ double lds_dyn[];
  const DevExec ex{(int)threadIdx.x, (ldouble*)lds_dyn, nullptr, nullptr};
  const int st = bandqp_solve(ex, d, vals + (size_t)b * d.nvals, cvals + (size_t)b * d.ncvals, ws + d.stride * b,
                              x + (size_t)b * d.n, y + (size_t)b * d.m, iters ? iters + b : nullptr);
  if (threadIdx.x == 0) status[b] = st;
}

// plans whose solves take S / Fx / bx (bmpc_set_transform, bmpc_set_fx)
bool plan_takes_transform(const Plan& P) {
  return P.desc.model == BMPC_MODEL_HIGHWAY_MERGE ||
         (P.desc.model == BMPC_MODEL_HIGHWAY && (P.desc.flags & BMPC_PLAN_TRANSFORM));
}

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHECK(expr)                                                                      \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) return fail(-5, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

// device buffer owned by the scope (every early return of a HIPCHECK frees it)
struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) hipFree(p);
  }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes); }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// host array -> fresh device copy (or null when the host pointer is null)
hipError_t upload(DevBuf& b, const void* host, size_t bytes) {
  if (!host) return hipSuccess;
  hipError_t e = b.alloc(bytes);
  if (e != hipSuccess) return e;
  return hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice);
}

}  // namespace

namespace {
// A grow-only device buffer (reallocated only when a call needs more).
struct GrowBuf {
  void* p = nullptr;
  size_t cap = 0;
  GrowBuf() = default;
  GrowBuf(const GrowBuf&) = delete;
  GrowBuf& operator=(const GrowBuf&) = delete;
  ~GrowBuf() {
    if (p) hipFree(p);
  }
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// bmpc_qp_solve's analyses, keyed by everything bandqp_analyse reads except the bound
// values: the pattern, the row classes, max_iter, eps and the factor-in-LDS choice.  A caller
// such as PredictiveControllers.MPC or Highway_env re-solves one pattern every control step:
// the ordering, the scatter lists and their device copy are made once.
struct QPCacheEntry {
  std::vector<int32_t> key;
  double eps = 0;
  HostBandQP h;
  GrowBuf tab;
  uint64_t used = 0;
};
}  // namespace

struct bmpc_ctx {
  int device;
  int cus;             // compute units (hipDeviceProp_t::multiProcessorCount)
  size_t lds_per_cu;   // LDS bytes per CU (maxSharedMemoryPerMultiProcessor)
  size_t lds_per_block = 0;      // LDS bytes one workgroup may opt in to (sharedMemPerBlockOptin)
  unsigned long long lds_flat0 = 0;   // flat address of LDS offset 0 (k_lds_aperture), 0 = not probed
  // bmpc_qp_solve: its own stream (synchronised alone, never the device), the analysis cache
  // and grow-only buffers reused across calls
  hipStream_t qstream = nullptr;
  static constexpr int kQPCache = 8;
  std::vector<std::unique_ptr<QPCacheEntry>> qcache;
  uint64_t qclock = 0;
  GrowBuf q_in, q_ws, q_out, q_aux;
  std::vector<double> q_host;
  // bmpc_hmm_eval / bmpc_qp_solve / bmpc_model_eval share the staging buffers, the stream and
  // the QP cache above; ctypes releases the GIL during a call, so calls from several host
  // threads on one context are serialised here
  std::mutex q_mu;
  ~bmpc_ctx() {
    if (qstream) hipStreamDestroy(qstream);
  }
};

struct bmpc_plan {
  bmpc_ctx* ctx;
  HostPlan hp;
  int batch;
  Bundle* d_bundle = nullptr;
  int32_t* d_tables = nullptr;
  double* d_ws = nullptr;
  bmpc_policy* d_pol = nullptr;
  std::vector<bmpc_policy> h_pol;
  double* d_in = nullptr;     // x | z | xref staging
  double* d_out = nullptr;    // upred | xpred | bw | J staging
  int32_t* d_iout = nullptr;  // status | iters
  double* d_scratch = nullptr;
  size_t scratch_len = 0;
  hipStream_t stream = nullptr;
  hipStream_t user_stream = nullptr;
  bool timing = false;
  // timing ring: three events per instrumented solve, read back only when the ring is full
  // or bmpc_timing is called, so timed solves run without a host synchronisation
  static constexpr int kTimeSlots = 32;
  hipEvent_t ev[3 * kTimeSlots] = {};
  int t_pending = 0;
  double t_acc[2] = {0, 0};
  int t_cnt = 0;
  bool pol_on_device = false;   // bmpc_env_step re-targeted d_pol: h_pol is stale
  int last_kernel = BMPC_KERNEL_NONE;   // solver kernel of the last launch (BMPC_INFO_SOLVER)
  double* d_lref = nullptr;   // lane reference of the *_PSIREF policies (grid | values)
  // small-batch kernel: per-ego layouts with LDS-resident spans (blk_layouts), built on the first
  // small-batch solve for this plan's LDS base
  Layout* d_blk_lay = nullptr;
  size_t blk_lay_base = 0, blk_hot_off = 0, blk_hot_bytes = 0;
  bool psiref = false;        // some policy in force tracks the lane reference
#if defined(BMPC_WITH_PHASED)
  int32_t* d_count = nullptr;   // phase-per-kernel IPM: egos going on per iteration [kMaxSub][maxit + 1]
  int32_t* h_count = nullptr;   // ... pinned read-back slots [kMaxSub]
  hipStream_t sub[kMaxSub] = {};   // ... its sub-batch streams
  hipEvent_t sub_ev[kMaxSub + 1] = {};
#endif
};

// the plan's constants and layout, with the table and lane-reference pointers at their device
// copies, into the device Bundle the kernels read
static hipError_t upload_bundle(bmpc_plan* pl) {
  Bundle hb;
  hb.P = pl->hp.plan;
  hb.L = pl->hp.lay;
  HostPlan tmp = pl->hp;       // re-point the table pointers at the device copy
  tmp.point_tables(pl->d_tables);
  hb.P.t = tmp.plan.t;
  hb.P.lref = pl->d_lref;
  return hipMemcpy(pl->d_bundle, &hb, sizeof(Bundle), hipMemcpyHostToDevice);
}

extern "C" {

const char* bmpc_last_error(void) { return g_err.c_str(); }
int bmpc_abi_version(void) { return BMPC_ABI_VERSION; }

int bmpc_open(int hip_device, bmpc_ctx** out) {
  if (!out) return fail(-22, "null output pointer");
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  if (hip_device < 0 || hip_device >= ndev) return fail(-19, "no such HIP device");
  HIPCHECK(hipSetDevice(hip_device));
  hipDeviceProp_t prop;
  HIPCHECK(hipGetDeviceProperties(&prop, hip_device));
  const int cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  const size_t lds = prop.maxSharedMemoryPerMultiProcessor > 0 ? prop.maxSharedMemoryPerMultiProcessor : 160 * 1024;
  bmpc_ctx* c = new bmpc_ctx;
  c->device = hip_device;
  c->cus = cus;
  c->lds_per_cu = lds;
  c->lds_per_block = prop.sharedMemPerBlockOptin > 0 ? std::min(prop.sharedMemPerBlockOptin, lds) : lds;
  *out = c;
  return 0;
}

int bmpc_close(bmpc_ctx* ctx) {
  delete ctx;
  return 0;
}

int bmpc_plan_create(bmpc_ctx* ctx, const bmpc_plan_desc* desc, int batch, bmpc_plan** out) {
  if (!ctx || !desc || !out) return fail(-22, "null argument");
  if (batch <= 0) return fail(-22, "batch must be positive");
  HIPCHECK(hipSetDevice(ctx->device));
  bmpc_plan* pl = new bmpc_plan();
  pl->ctx = ctx;
  pl->batch = batch;
  std::string err = build_plan(*desc, pl->hp);
  if (!err.empty()) {
    delete pl;
    return fail(-22, err);
  }
  const Plan& P = pl->hp.plan;
  const Layout& L = pl->hp.lay;
  auto cleanup = [&](int rc) {
    bmpc_plan_destroy(pl);
    return rc;
  };
  if (hipMalloc(&pl->d_tables, pl->hp.blob.size() * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&pl->d_bundle, sizeof(Bundle)) != hipSuccess ||
      hipMalloc(&pl->d_ws, L.stride * (size_t)batch * sizeof(double)) != hipSuccess ||
      hipMalloc(&pl->d_pol, sizeof(bmpc_policy) * (size_t)batch * P.m) != hipSuccess ||
      hipMalloc(&pl->d_in, sizeof(double) * (size_t)batch * P.n * 3) != hipSuccess ||
      hipMalloc(&pl->d_out, sizeof(double) * (size_t)batch * ((size_t)P.U * P.d + (size_t)P.T * P.n + P.nbranch + 1)) != hipSuccess ||
      hipMalloc(&pl->d_iout, sizeof(int32_t) * (size_t)batch * 2) != hipSuccess)
    return cleanup(fail(-12, "hipMalloc failed (out of device memory?)"));
#if defined(BMPC_WITH_PHASED)
  if (hipMalloc(&pl->d_count, sizeof(int32_t) * kMaxSub * (size_t)(P.desc.maxit + 1)) != hipSuccess ||
      hipHostMalloc(&pl->h_count, sizeof(int32_t) * kMaxSub) != hipSuccess)
    return cleanup(fail(-12, "hipMalloc failed (out of device memory?)"));
#endif
  if (hipMemcpy(pl->d_tables, pl->hp.blob.data(), pl->hp.blob.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(-5, "hipMemcpy tables failed"));
  if (upload_bundle(pl) != hipSuccess ||
      hipMemset(pl->d_ws, 0, L.stride * (size_t)batch * sizeof(double)) != hipSuccess)
    return cleanup(fail(-5, "plan upload failed"));
  pl->h_pol.assign((size_t)batch * P.m, bmpc_policy{});
  if (hipMemcpy(pl->d_pol, pl->h_pol.data(), sizeof(bmpc_policy) * pl->h_pol.size(), hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(-5, "policy upload failed"));
  if (hipStreamCreateWithFlags(&pl->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(-5, "hipStreamCreate failed"));
  for (auto& e : pl->ev)
    if (hipEventCreate(&e) != hipSuccess) return cleanup(fail(-5, "hipEventCreate failed"));
#if defined(BMPC_WITH_PHASED)
  for (auto& q : pl->sub)
    if (hipStreamCreateWithFlags(&q, hipStreamNonBlocking) != hipSuccess) return cleanup(fail(-5, "hipStreamCreate failed"));
  for (auto& e : pl->sub_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return cleanup(fail(-5, "hipEventCreate failed"));
#endif
  *out = pl;
  return 0;
}

int bmpc_plan_destroy(bmpc_plan* pl) {
  if (!pl) return 0;
  hipSetDevice(pl->ctx->device);
  if (pl->stream) hipStreamSynchronize(pl->stream);
  hipFree(pl->d_tables);
  hipFree(pl->d_bundle);
  hipFree(pl->d_ws);
  hipFree(pl->d_pol);
  hipFree(pl->d_in);
  hipFree(pl->d_out);
  hipFree(pl->d_iout);
  hipFree(pl->d_scratch);
  hipFree(pl->d_lref);
  hipFree(pl->d_blk_lay);
  for (auto& e : pl->ev)
    if (e) hipEventDestroy(e);
#if defined(BMPC_WITH_PHASED)
  hipFree(pl->d_count);
  if (pl->h_count) hipHostFree(pl->h_count);
  for (auto& q : pl->sub)
    if (q) {
      hipStreamSynchronize(q);
      hipStreamDestroy(q);
    }
  for (auto& e : pl->sub_ev)
    if (e) hipEventDestroy(e);
#endif
  if (pl->stream) hipStreamDestroy(pl->stream);
  delete pl;
  return 0;
}

int bmpc_plan_info(const bmpc_plan* pl, int32_t* info) {
  if (!pl || !info) return fail(-22, "null argument");
  const Plan& P = pl->hp.plan;
  info[BMPC_INFO_T] = P.T;
  info[BMPC_INFO_U] = P.U;
  info[BMPC_INFO_BDIM] = P.bdim;
  info[BMPC_INFO_NBRANCH] = P.nbranch;
  info[BMPC_INFO_NV] = P.nv;
  info[BMPC_INFO_NEQ] = P.neq;
  info[BMPC_INFO_NROWS] = P.nrows;
  info[BMPC_INFO_NCONES] = P.ncones;
  info[BMPC_INFO_LP] = P.nlp;
  info[BMPC_INFO_BATCH] = pl->batch;
  info[BMPC_INFO_WS_DOUBLES] = (int32_t)pl->hp.lay.stride;
  info[BMPC_INFO_SOLVER] = pl->last_kernel;
  return 0;
}

int bmpc_set_policies(bmpc_plan* pl, const bmpc_policy* pol, const uint8_t* mask) {
  if (!pl || !pol) return fail(-22, "null argument");
  const int m = pl->hp.plan.m;
  for (int e = 0; e < pl->batch; ++e)
    for (int i = 0; i < m; ++i)
      if ((!mask || mask[e]) && is_psiref(pol[(size_t)e * m + i].kind) &&
          pl->hp.plan.desc.model != BMPC_MODEL_HIGHWAY_MERGE)
        return fail(-22, "lane-reference (psiref) policies need a HIGHWAY_MERGE plan");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  if (pl->pol_on_device && mask) {   // keep the device-side re-targets of unmasked egos
    HIPCHECK(hipStreamSynchronize(pl->stream));
    if (pl->user_stream) HIPCHECK(hipStreamSynchronize(pl->user_stream));
    HIPCHECK(hipMemcpy(pl->h_pol.data(), pl->d_pol, sizeof(bmpc_policy) * pl->h_pol.size(), hipMemcpyDeviceToHost));
  }
  pl->pol_on_device = false;
  for (int e = 0; e < pl->batch; ++e)
    if (!mask || mask[e])
      memcpy(&pl->h_pol[(size_t)e * m], pol + (size_t)e * m, sizeof(bmpc_policy) * m);
  pl->psiref = false;
  for (const bmpc_policy& q : pl->h_pol) pl->psiref = pl->psiref || is_psiref(q.kind);
  HIPCHECK(hipMemcpyAsync(pl->d_pol, pl->h_pol.data(), sizeof(bmpc_policy) * pl->h_pol.size(),
                          hipMemcpyHostToDevice, pl->stream));
  HIPCHECK(hipStreamSynchronize(pl->stream));
  return 0;
}

int bmpc_get_policies(bmpc_plan* pl, bmpc_policy* pol) {
  if (!pl || !pol) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  HIPCHECK(hipStreamSynchronize(pl->stream));
  if (pl->user_stream) HIPCHECK(hipStreamSynchronize(pl->user_stream));
  HIPCHECK(hipMemcpy(pol, pl->d_pol, sizeof(bmpc_policy) * pl->h_pol.size(), hipMemcpyDeviceToHost));
  return 0;
}

int bmpc_reset(bmpc_plan* pl, const uint8_t* mask) {
  if (!pl) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  DevBuf d_mask;
  HIPCHECK(upload(d_mask, mask, pl->batch));
  hipLaunchKernelGGL(k_reset, dim3((pl->batch + 255) / 256), dim3(256), 0, pl->stream, pl->d_ws,
                     pl->hp.lay.stride, pl->hp.lay.misc, d_mask.as<uint8_t>(), pl->batch);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(pl->stream));
  return 0;
}

// Scatter per-ego host rows [batch][cnt] into the slab at offset off (one staging copy;
// masked egos only).  The stream is drained before the staging buffers go out of scope.
static int scatter_rows(bmpc_plan* pl, const double* src, size_t off, int cnt, const uint8_t* d_mask) {
  if (!src || cnt <= 0) return 0;
  DevBuf buf;
  HIPCHECK(upload(buf, src, sizeof(double) * (size_t)pl->batch * cnt));
  hipLaunchKernelGGL(k_scatter, dim3(512), dim3(256), 0, pl->stream, pl->d_ws, pl->hp.lay.stride, off, cnt,
                     buf.as<double>(), d_mask, pl->batch);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(pl->stream));
  return 0;
}

// Reads back the pending timing events (waits for the last instrumented solve).  The ring is
// emptied on every exit path: a failed read-back drops the pending samples rather than leaving
// t_pending at kTimeSlots (the next launch would index past ev[]).
static int fold_timing(bmpc_plan* pl) {
  const int pending = pl->t_pending;
  pl->t_pending = 0;
  for (int k = 0; k < pending && k < bmpc_plan::kTimeSlots; ++k) {
    hipEvent_t* ev = pl->ev + 3 * k;
    HIPCHECK(hipEventSynchronize(ev[2]));
    float a = 0, b = 0;
    HIPCHECK(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIPCHECK(hipEventElapsedTime(&b, ev[1], ev[2]));
    pl->t_acc[0] += a;
    pl->t_acc[1] += b;
    pl->t_cnt += 1;
  }
  return 0;
}

#if defined(BMPC_WITH_PHASED)
// 0: monolithic k_ipm, 1: one kernel per IPM phase, 2: one kernel calling grouped phases (k_ipm_g)
static int use_phased() {
  const char* e = getenv("BMPC_IPM_PHASED");
  return e ? atoi(e) : BMPC_IPM_PHASED_DEFAULT;
}
#endif

// the flat (generic) address of LDS offset 0: the LDS aperture base every workgroup's LDS is
// addressed through (the same for every kernel of the process)
__global__ void k_lds_aperture(unsigned long long* out) {
  __shared__ double s[2];
  s[threadIdx.x & 1] = 0.0;
  if (threadIdx.x == 0) out[0] = (unsigned long long)(uintptr_t)(double*)s;
}

// LDS-resident spans of the small-batch kernel (bmpc_dev.h, k_solve_blk): ego e's layout with
// spans of the IPM's own arrays offset from the ego's slab (d_ws + e * stride) to the workgroup's
// LDS after the launch's own lds_base bytes.  Spans in priority order, each kept whole (code
// addresses several fields of a span from one base) and skipped when it does not fit: the NT
// scaling (dl .. vnt), the node factors (hx .. kff), the tree solve's l and x right-hand sides
// (lvec, qx0), z / s / lambda, the tree's A / B and dh (copied in by the kernel).  Every span
// holds arrays a solve writes before it reads them (or that the kernel copies in); the scaling's
// span must fit (the kernel's guard checks it).  Returns the extra LDS bytes (0: no layouts).
static int blk_layouts(bmpc_plan* pl, size_t lds_base) {
  bmpc_ctx* c = pl->ctx;
  if (pl->d_blk_lay && pl->blk_lay_base == lds_base) return 0;
  if (!c->lds_flat0) {
    unsigned long long* d = nullptr;
    HIPCHECK(hipMalloc(&d, sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_lds_aperture, dim3(1), dim3(64), 0, pl->stream, d);
    unsigned long long h = 0;
    hipError_t e = hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, pl->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(pl->stream);
    hipFree(d);
    HIPCHECK(e);
    if (!h) return fail(-5, "LDS aperture probe returned 0");
    c->lds_flat0 = h;
  }
  const Layout& L = pl->hp.lay;
  const size_t off0 = ((lds_base + 63) & ~(size_t)63) / sizeof(double);
  const size_t cap = c->lds_per_block / sizeof(double);
  struct Span { size_t Layout::*a; size_t Layout::*b; };
  const Span spans[] = {{&Layout::dl, &Layout::hx},   {&Layout::hx, &Layout::lvec}, {&Layout::lvec, &Layout::qx0},
                        {&Layout::qx0, &Layout::gk},  {&Layout::z, &Layout::z1},    {&Layout::Ad, &Layout::Cd},
                        {&Layout::dh, &Layout::h0}};
  const int nsp = sizeof(spans) / sizeof(spans[0]);
  size_t at[nsp];   // LDS offset (doubles) of each relocated span, 0 = stays in the slab
  size_t cur = off0;
  for (int k = 0; k < nsp; ++k) {
    const size_t a = L.*spans[k].a, b = L.*spans[k].b;
    at[k] = 0;
    if (b <= a) continue;
    const size_t len = (b - a + 7) & ~(size_t)7;
    if (cur + len <= cap) {
      at[k] = cur;
      cur += len;
    }
  }
  if (!at[0]) return 0;   // not even the scaling fits: the plain layout
  const int B = pl->batch;
  std::vector<Layout> lays(B, L);
  const size_t nf = offsetof(Layout, stride) / sizeof(size_t);
  for (int e = 0; e < B; ++e) {
    const int64_t ws_e = (int64_t)(uintptr_t)(pl->d_ws + (size_t)e * L.stride);
    size_t* f = reinterpret_cast<size_t*>(&lays[e]);
    const size_t* f0 = reinterpret_cast<const size_t*>(&L);
    for (int k = 0; k < nsp; ++k) {
      if (!at[k]) continue;
      const size_t a = L.*spans[k].a, b = L.*spans[k].b;
      // ws_e + 8 (off + delta) = LDS(at[k] + off - a) for every field offset off in [a, b)
      const int64_t delta = ((int64_t)c->lds_flat0 + 8 * (int64_t)at[k] - ws_e) / 8 - (int64_t)a;
      for (size_t i = 0; i < nf; ++i)
        if (f0[i] >= a && f0[i] < b) f[i] = (size_t)((int64_t)f0[i] + delta);
    }
  }
  if (!pl->d_blk_lay) {
    HIPCHECK(hipMalloc(&pl->d_blk_lay, sizeof(Layout) * (size_t)B));
  } else {
    // a rebuild (the launch's LDS base changed, e.g. BMPC_BLOCK_WAVES toggled between solves):
    // a small-batch kernel still in flight on the plan's or the caller's stream reads the old
    // layouts -- let those streams drain before the buffer is overwritten
    HIPCHECK(hipStreamSynchronize(pl->stream));
    if (pl->user_stream) HIPCHECK(hipStreamSynchronize(pl->user_stream));
  }
  HIPCHECK(hipMemcpy(pl->d_blk_lay, lays.data(), sizeof(Layout) * (size_t)B, hipMemcpyHostToDevice));
  pl->blk_lay_base = lds_base;
  pl->blk_hot_off = at[0];
  pl->blk_hot_bytes = (cur - off0) * sizeof(double);
  return 0;
}

static int launch_solve(bmpc_plan* pl, const double* d_x, const double* d_z, const double* d_xref,
                        double* d_upred, double* d_xpred, double* d_bw, double* d_J,
                        int32_t* d_status, int32_t* d_iters, hipStream_t s) {
  const Plan& P = pl->hp.plan;
  const int B = pl->batch;
  const bool merge = P.desc.model == BMPC_MODEL_HIGHWAY_MERGE;
  // HIGHWAY plans that take solve's S / Fx / bx run the transform path of the same model
  const bool hwt = P.desc.model == BMPC_MODEL_HIGHWAY && (P.desc.flags & BMPC_PLAN_TRANSFORM);
  const bool xform = merge || hwt;
  const bool tl = choose_lds_rich(P, xform, B, pl->ctx->cus, pl->ctx->lds_per_cu);
  size_t lds_bytes = solver_lds_bytes(P, xform, tl);
  // occupancy experiments: BMPC_IPM_LDS_BYTES reserves at least that much LDS per workgroup
  // (fewer egos resident per CU => a smaller working set in L2 / Infinity Cache)
  if (const char* e = getenv("BMPC_IPM_LDS_BYTES")) {
    const size_t want = (size_t)atol(e);
    if (want > lds_bytes && want <= pl->ctx->lds_per_cu) lds_bytes = want;
  }
  if (pl->psiref && P.nlref == 0)
    return fail(-22, "the plan's policies track a lane reference: set it first (bmpc_set_lane_ref)");
  if (pl->timing && (pl->t_pending < 0 || pl->t_pending >= bmpc_plan::kTimeSlots))
    return fail(-5, "timing ring out of range (t_pending = " + std::to_string(pl->t_pending) + ")");
  const bool qp = P.desc.controller != BMPC_CTRL_CVAR;
  SolveLaunch a{pl->d_bundle, pl->d_ws, pl->d_pol, d_x, d_z, d_xref, d_upred, d_xpred, d_bw, d_J, d_status,
                d_iters, B, lds_bytes, tl, qp, s};
  a.cus = pl->ctx->cus;
  a.hplan = &P;
  int kernel = qp ? (tl ? BMPC_KERNEL_QP_RICH : BMPC_KERNEL_QP_LEAN) : (tl ? BMPC_KERNEL_IPM_RICH : BMPC_KERNEL_IPM_LEAN);
  hipError_t (*tree)(const SolveLaunch&) = launch_tree_quadruped;
  hipError_t (*solver)(const SolveLaunch&) = launch_solver_quadruped;
  if (hwt) tree = launch_tree_highway_t, solver = launch_solver_highway_t;
  else if (P.desc.model == BMPC_MODEL_HIGHWAY) tree = launch_tree_highway, solver = launch_solver_highway;
  else if (merge) tree = launch_tree_merge, solver = launch_solver_merge;
  // Small batches of the CVaR IPM: one ego per multi-wave workgroup (k_solve_blk) when the batch
  // leaves CUs idle -- 4 waves per ego, 8 for trees of BMPC_BLK_WIDE_T state nodes or more.
  // Measured at one ego (profiles/r03/r03x_blk_waves.log): N=8 NB=2 22 ms vs 30 on one wave,
  // N=20 NB=1 12-14 vs 14-16, N=30 NB=2 44-49 vs 61-65.  BMPC_BLOCK_EGOS: the largest batch that
  // takes this path (default: one ego per CU; 0 disables it); BMPC_BLOCK_WAVES: 4 or 8.
  int blk_max = pl->ctx->cus;
  if (const char* e = getenv("BMPC_BLOCK_EGOS")) blk_max = atoi(e);
  const bool blk = B <= blk_max && P.desc.controller == BMPC_CTRL_CVAR;
  if (blk) {
    a.nw = P.T >= BMPC_BLK_WIDE_T ? 8 : 4;
#if defined(BMPC_BLK_ALLOW2)
    if (const char* e = getenv("BMPC_BLOCK_WAVES")) a.nw = atoi(e) == 8 ? 8 : atoi(e) == 2 ? 2 : 4;   // tools-only A/B
#else
    if (const char* e = getenv("BMPC_BLOCK_WAVES")) a.nw = atoi(e) == 8 ? 8 : 4;
#endif
    a.lds_bytes = solver_lds_bytes_blk(P, xform, a.nw);
    a.rich = true;
    // BMPC_BLK_LDS=0: the small-batch kernel keeps every array in the slab
    const char* el = getenv("BMPC_BLK_LDS");
    if (!(el && atoi(el) == 0)) {
      if (const int rc = blk_layouts(pl, a.lds_bytes)) return rc;
      if (pl->d_blk_lay) {
        a.blk_lay = pl->d_blk_lay;
        a.blk_hot_off = pl->blk_hot_off;
        a.lds_bytes = pl->blk_hot_off * sizeof(double) + pl->blk_hot_bytes;
      }
    }
    kernel = a.nw == 8 ? BMPC_KERNEL_IPM_BLK8 : BMPC_KERNEL_IPM_BLK4;
    if (hwt) solver = launch_solver_blk_highway_t;
    else if (P.desc.model == BMPC_MODEL_HIGHWAY) solver = launch_solver_blk_highway;
    else if (merge) solver = launch_solver_blk_merge;
    else solver = launch_solver_blk_quadruped;
  }
#if defined(BMPC_WITH_PHASED)
  // tools-only builds: the phase-per-kernel IPM (experimental/bmpc_dev_ph.h, mode 1: the factored
  // coupling system re-read into LDS by every kernel that solves with it) or one kernel calling
  // grouped phase functions (mode 2/3), selected by BMPC_IPM_PHASED for large LDS-rich CVaR batches
  a.d_count = pl->d_count;
  a.h_count = pl->h_count;
  a.maxit = P.desc.maxit;
  a.ph_mode = use_phased();
  a.sub = pl->sub;
  a.sub_ev = pl->sub_ev;
  {   // sub-batch streams of the phase-per-kernel IPM (BMPC_PH_STREAMS; 1 = all on the solve's stream)
    const char* e = getenv("BMPC_PH_STREAMS");
    a.nsub = e ? atoi(e) : BMPC_PH_STREAMS_DEFAULT;
  }
  if (!blk && !qp && tl && a.ph_mode != 0) {
    if (hwt) solver = launch_ipm_phased_highway_t;
    else if (P.desc.model == BMPC_MODEL_HIGHWAY) solver = launch_ipm_phased_highway;
    else if (merge) solver = launch_ipm_phased_merge;
  }
#endif
  pl->last_kernel = kernel;
  hipEvent_t* ev = pl->ev + 3 * (pl->timing ? pl->t_pending : 0);
  if (pl->timing) HIPCHECK(hipEventRecord(ev[0], s));
  HIPCHECK(tree(a));
  if (pl->timing) HIPCHECK(hipEventRecord(ev[1], s));
  HIPCHECK(solver(a));
  if (pl->timing) {
    HIPCHECK(hipEventRecord(ev[2], s));
    if (++pl->t_pending == bmpc_plan::kTimeSlots) return fold_timing(pl);
  }
  return 0;
}

int bmpc_solve(bmpc_plan* pl, const double* x, const double* z, const double* xref, double* upred,
               double* xpred, double* branch_w, double* J, int32_t* status, int32_t* iters) {
  if (!pl || !x || !z || !xref) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  const size_t B = pl->batch, n = P.n;
  hipStream_t s = pl->stream;
  double* dx = pl->d_in;
  double* dz = dx + B * n;
  double* dr = dz + B * n;
  HIPCHECK(hipMemcpyAsync(dx, x, sizeof(double) * B * n, hipMemcpyHostToDevice, s));
  HIPCHECK(hipMemcpyAsync(dz, z, sizeof(double) * B * n, hipMemcpyHostToDevice, s));
  HIPCHECK(hipMemcpyAsync(dr, xref, sizeof(double) * B * n, hipMemcpyHostToDevice, s));
  double* up = pl->d_out;
  double* xp = up + B * P.U * P.d;
  double* bw = xp + B * P.T * P.n;
  double* jj = bw + B * (P.nbranch - 1);
  int32_t* st = pl->d_iout;
  int32_t* it = st + B;
  int rc = launch_solve(pl, dx, dz, dr, up, xp, bw, jj, st, it, s);
  if (rc) return rc;
  if (upred) HIPCHECK(hipMemcpyAsync(upred, up, sizeof(double) * B * P.U * P.d, hipMemcpyDeviceToHost, s));
  if (xpred) HIPCHECK(hipMemcpyAsync(xpred, xp, sizeof(double) * B * P.T * P.n, hipMemcpyDeviceToHost, s));
  if (branch_w) HIPCHECK(hipMemcpyAsync(branch_w, bw, sizeof(double) * B * (P.nbranch - 1), hipMemcpyDeviceToHost, s));
  if (J) HIPCHECK(hipMemcpyAsync(J, jj, sizeof(double) * B, hipMemcpyDeviceToHost, s));
  if (status) HIPCHECK(hipMemcpyAsync(status, st, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
  if (iters) HIPCHECK(hipMemcpyAsync(iters, it, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  return 0;
}

int bmpc_solve_device(bmpc_plan* pl, const double* d_x, const double* d_z, const double* d_xref,
                      double* d_upred, double* d_xpred, double* d_branch_w, double* d_J,
                      int32_t* d_status, int32_t* d_iters, void* stream) {
  if (!pl || !d_x || !d_z || !d_xref) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->stream;
  if (stream) pl->user_stream = s;   // (synchronised before the plan's device state is rewritten)
  return launch_solve(pl, d_x, d_z, d_xref, d_upred, d_xpred, d_branch_w, d_J, d_status, d_iters, s);
}

int bmpc_env_step(bmpc_plan* pl, const bmpc_env_desc* env, int t, double* d_scene, const double* d_upred,
                  const double* d_J, const int32_t* d_status, const int32_t* d_iters, double* d_x,
                  double* d_z, double* d_xref, double* d_stats, void* stream) {
  if (!pl || !env || !d_scene || !d_x || !d_z || !d_xref) return fail(-22, "null argument");
  const Plan& P = pl->hp.plan;
  if (P.desc.model != BMPC_MODEL_HIGHWAY || P.n != 4 || P.d != 2)
    return fail(-22, "bmpc_env_step: the overtake scene needs a highway plan (n = 4, d = 2)");
  if (t < 0 || (t > 0 && !d_upred)) return fail(-22, "bmpc_env_step: t > 0 needs the last uPred");
  if (env->n_lane < 1) return fail(-22, "bmpc_env_step: n_lane < 1");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->stream;
  if (stream) pl->user_stream = s;
  hipLaunchKernelGGL(k_env, dim3((pl->batch + 63) / 64), dim3(64), 0, s, *env, P.desc.dt, P.N, P.m, P.U, P.d, t,
                     pl->batch, d_scene, pl->d_pol, d_upred, d_J, d_status, d_iters,
                     P.desc.controller == BMPC_CTRL_CVAR ? 1 : 0, d_x, d_z, d_xref, d_stats);
  HIPCHECK(hipGetLastError());
  pl->pol_on_device = true;
  return 0;
}

// nsteps closed-loop steps (include/bmpc.h): one k_loop launch for CVaR batches that take the
// one-wave IPM, otherwise bmpc_env_step + the solve launches per step (same results either way)
int bmpc_loop_device(bmpc_plan* pl, const bmpc_env_desc* env, int t0, int nsteps, double* d_scene, double* d_upred,
                     double* d_x, double* d_z, double* d_xref, double* d_J, int32_t* d_status, int32_t* d_iters,
                     double* d_stats, void* stream) {
  if (!pl || !env || !d_scene || !d_upred || !d_x || !d_z || !d_xref || !d_J || !d_status || !d_iters)
    return fail(-22, "null argument");
  const Plan& P = pl->hp.plan;
  if (P.desc.model != BMPC_MODEL_HIGHWAY || (P.desc.flags & BMPC_PLAN_TRANSFORM) || P.n != 4 || P.d != 2)
    return fail(-22, "bmpc_loop_device: the overtake scene needs a highway plan (n = 4, d = 2) without transform");
  if (P.desc.controller != BMPC_CTRL_CVAR && P.desc.controller != BMPC_CTRL_ROBUST)
    return fail(-22, "bmpc_loop_device: CVaR or robust controllers only");
  if (nsteps < 1 || t0 < 0) return fail(-22, "bmpc_loop_device: nsteps >= 1 and t0 >= 0");
  if (env->n_lane < 1) return fail(-22, "bmpc_loop_device: n_lane < 1");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->stream;
  if (stream) pl->user_stream = s;
  const int B = pl->batch;
  int blk_max = pl->ctx->cus;   // the small-batch path of launch_solve
  if (const char* e = getenv("BMPC_BLOCK_EGOS")) blk_max = atoi(e);
  bool fused = P.desc.controller == BMPC_CTRL_CVAR && B > blk_max && !pl->psiref;
  if (const char* e = getenv("BMPC_LOOP_FUSED")) fused = fused && atoi(e) != 0;   // 0: per-step launches (A/B)
  if (!fused) {
    for (int k = 0; k < nsteps; ++k) {
      if (int rc = bmpc_env_step(pl, env, t0 + k, d_scene, d_upred, d_J, d_status, d_iters, d_x, d_z, d_xref, d_stats,
                                 stream))
        return rc;
      if (int rc = launch_solve(pl, d_x, d_z, d_xref, d_upred, nullptr, nullptr, d_J, d_status, d_iters, s)) return rc;
    }
    return 0;
  }
  if (pl->timing && (pl->t_pending < 0 || pl->t_pending >= bmpc_plan::kTimeSlots))
    return fail(-5, "timing ring out of range (t_pending = " + std::to_string(pl->t_pending) + ")");
  const bool tl = choose_lds_rich(P, false, B, pl->ctx->cus, pl->ctx->lds_per_cu);
  SolveLaunch a{pl->d_bundle, pl->d_ws, pl->d_pol, d_x, d_z, d_xref, d_upred, nullptr, nullptr, d_J, d_status,
                d_iters, B, solver_lds_bytes(P, false, tl), tl, false, s};
  a.cus = pl->ctx->cus;
  a.hplan = &P;
  pl->last_kernel = tl ? BMPC_KERNEL_LOOP_RICH : BMPC_KERNEL_LOOP_LEAN;
  hipEvent_t* ev = pl->ev + 3 * (pl->timing ? pl->t_pending : 0);
  if (pl->timing) {   // (the whole fused launch is booked as the solver's time, none as the tree's)
    HIPCHECK(hipEventRecord(ev[0], s));
    HIPCHECK(hipEventRecord(ev[1], s));
  }
  HIPCHECK(launch_loop_highway(a, *env, t0, nsteps, d_scene, d_stats));
  pl->pol_on_device = true;
  if (pl->timing) {
    HIPCHECK(hipEventRecord(ev[2], s));
    if (++pl->t_pending == bmpc_plan::kTimeSlots) return fold_timing(pl);
  }
  return 0;
}

static int gather(bmpc_plan* pl, size_t off, int count, double* host) {
  if (!host) return 0;
  const size_t need = (size_t)pl->batch * count;
  if (need > pl->scratch_len) {
    hipFree(pl->d_scratch);
    pl->d_scratch = nullptr;
    HIPCHECK(hipMalloc(&pl->d_scratch, need * sizeof(double)));
    pl->scratch_len = need;
  }
  hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, pl->stream, pl->d_ws, pl->hp.lay.stride, off,
                     count, pl->d_scratch, pl->batch);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpyAsync(host, pl->d_scratch, need * sizeof(double), hipMemcpyDeviceToHost, pl->stream));
  HIPCHECK(hipStreamSynchronize(pl->stream));
  return 0;
}

int bmpc_get_counters(bmpc_plan* pl, double* out) {
  if (!pl || !out) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  return gather(pl, pl->hp.lay.prof, PROF_COUNT, out);
}

int bmpc_get_warm_start(bmpc_plan* pl, double* uLin, double* p, double* jcons, double* old_input) {
  if (!pl) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  const Layout& L = pl->hp.lay;
  int rc;
  if ((rc = gather(pl, L.uLin, (P.U + 1) * P.d, uLin))) return rc;
  if (P.bdim * P.m > 0 && (rc = gather(pl, L.pprev, P.bdim * P.m, p))) return rc;
  if ((rc = gather(pl, L.misc + MISC_JCONS, 1, jcons))) return rc;
  if ((rc = gather(pl, L.misc + MISC_OLDU, P.d, old_input))) return rc;
  return 0;
}

int bmpc_set_warm_start(bmpc_plan* pl, const double* uLin, const double* p, const double* jcons,
                        const double* old_input, const uint8_t* mask) {
  if (!pl || !uLin) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  const Layout& L = pl->hp.lay;
  const int B = pl->batch;
  DevBuf dmask;
  HIPCHECK(upload(dmask, mask, B));
  std::vector<double> ones(B, 1.0);
  struct Part { const double* src; size_t off; int cnt; };
  const Part parts[] = {{uLin, L.uLin, (P.U + 1) * P.d},
                        {p, L.pprev, P.bdim * P.m},
                        {jcons, L.misc + MISC_JCONS, 1},
                        {old_input, L.misc + MISC_OLDU, P.d},
                        {ones.data(), L.misc + MISC_INIT, 1}};
  for (const Part& pt : parts)
    if (int rc = scatter_rows(pl, pt.src, pt.off, pt.cnt, dmask.as<uint8_t>())) return rc;
  return 0;
}

int bmpc_get_robust_warm_start(bmpc_plan* pl, double* xLin, double* uLin, double* old_input) {
  if (!pl) return fail(-22, "null argument");
  if (pl->hp.plan.desc.controller != BMPC_CTRL_ROBUST) return fail(-22, "not a robustMPC plan");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  const Layout& L = pl->hp.lay;
  int rc;
  if (xLin && (rc = gather(pl, L.xlin, P.T * P.n, xLin))) return rc;
  if (uLin && (rc = gather(pl, L.uLin, P.U * P.d, uLin))) return rc;
  if (old_input && (rc = gather(pl, L.misc + MISC_OLDU, P.d, old_input))) return rc;
  return 0;
}

int bmpc_set_robust_warm_start(bmpc_plan* pl, const double* xLin, const double* uLin, const double* old_input,
                               const uint8_t* mask) {
  if (!pl) return fail(-22, "null argument");
  if (pl->hp.plan.desc.controller != BMPC_CTRL_ROBUST) return fail(-22, "not a robustMPC plan");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  const Layout& L = pl->hp.lay;
  const int B = pl->batch;
  DevBuf dmask;
  HIPCHECK(upload(dmask, mask, B));
  std::vector<double> ones(B, 1.0);
  struct Part { const double* src; size_t off; int cnt; };
  const Part parts[] = {{xLin, L.xlin, P.T * P.n},
                        {uLin, L.uLin, P.U * P.d},
                        {old_input, L.misc + MISC_OLDU, P.d},
                        {ones.data(), L.misc + MISC_INIT, 1}};
  for (const Part& pt : parts)
    if (int rc = scatter_rows(pl, pt.src, pt.off, pt.cnt, dmask.as<uint8_t>())) return rc;
  return 0;
}

int bmpc_set_transform(bmpc_plan* pl, const double* S, const uint8_t* s_on, const double* bx, const uint8_t* mask) {
  if (!pl) return fail(-22, "null argument");
  const Plan& P = pl->hp.plan;
  if (!plan_takes_transform(P))
    return fail(-22, "bmpc_set_transform: only HIGHWAY_MERGE plans and HIGHWAY CVaR plans created with "
                     "BMPC_PLAN_TRANSFORM take a state transformation");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Layout& L = pl->hp.lay;
  const int B = pl->batch, n = P.n, nF = P.nFx;
  DevBuf dmask;
  HIPCHECK(upload(dmask, mask, B));
  // S (or zeros) and the "S is not None" flag of every masked ego
  std::vector<double> Sv((size_t)B * n * n, 0.0), on(B, 0.0);
  for (int e = 0; e < B; ++e) {
    if (S) {
      std::copy(S + (size_t)e * n * n, S + (size_t)(e + 1) * n * n, Sv.begin() + (size_t)e * n * n);
      on[e] = (!s_on || s_on[e]) ? 1.0 : 0.0;
    }
  }
  // the slab keeps S at row stride n (XF_S holds n*n values)
  if (int rc = scatter_rows(pl, Sv.data(), L.xform + XF_S, n * n, dmask.as<uint8_t>())) return rc;
  if (int rc = scatter_rows(pl, on.data(), L.xform + XF_SON, 1, dmask.as<uint8_t>())) return rc;
  if (bx) {
    std::vector<double> ones(B, 1.0);
    if (int rc = scatter_rows(pl, bx, L.xform + XF_BX, nF, dmask.as<uint8_t>())) return rc;
    if (int rc = scatter_rows(pl, ones.data(), L.xform + XF_BXSET, 1, dmask.as<uint8_t>())) return rc;
  }
  return 0;
}

int bmpc_set_fx(bmpc_plan* pl, const double* Fx, const uint8_t* mask) {
  if (!pl || !Fx) return fail(-22, "null argument");
  const Plan& P = pl->hp.plan;
  if (!plan_takes_transform(P))
    return fail(-22, "bmpc_set_fx: only HIGHWAY_MERGE plans and HIGHWAY CVaR plans created with "
                     "BMPC_PLAN_TRANSFORM take a per-solve Fx");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Layout& L = pl->hp.lay;
  const int B = pl->batch;
  DevBuf dmask;
  HIPCHECK(upload(dmask, mask, B));
  std::vector<double> ones(B, 1.0);
  if (int rc = scatter_rows(pl, Fx, L.xform + XF_FX, P.nFx * P.n, dmask.as<uint8_t>())) return rc;
  return scatter_rows(pl, ones.data(), L.xform + XF_FXSET, 1, dmask.as<uint8_t>());
}

int bmpc_get_branch_dp(bmpc_plan* pl, double* dp) {
  if (!pl || !dp) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  if (P.bdim * P.m * P.n == 0) return 0;
  return gather(pl, pl->hp.lay.dp, P.bdim * P.m * P.n, dp);
}

int bmpc_get_tree(bmpc_plan* pl, double* xbar, double* ubar, double* zbar, double* w, double* p,
                  double* sol) {
  if (!pl) return fail(-22, "null argument");
  HIPCHECK(hipSetDevice(pl->ctx->device));
  const Plan& P = pl->hp.plan;
  const Layout& L = pl->hp.lay;
  int rc;
  if ((rc = gather(pl, L.xbar, P.T * P.n, xbar))) return rc;
  if ((rc = gather(pl, L.ubar, P.U * P.d, ubar))) return rc;
  if ((rc = gather(pl, L.zbar, P.T * P.n, zbar))) return rc;
  if ((rc = gather(pl, L.w, P.nbranch, w))) return rc;
  if (P.bdim * P.m > 0 && (rc = gather(pl, L.p, P.bdim * P.m, p))) return rc;
  if ((rc = gather(pl, L.sol, P.nv, sol))) return rc;
  return 0;
}

int bmpc_enable_timing(bmpc_plan* pl, int on) {
  if (!pl) return fail(-22, "null argument");
  pl->timing = on != 0;
  pl->t_pending = 0;
  pl->t_acc[0] = pl->t_acc[1] = 0;
  pl->t_cnt = 0;
  return 0;
}

int bmpc_timing(bmpc_plan* pl, double* ms, int32_t* count) {
  if (!pl) return fail(-22, "null argument");
  if (int rc = fold_timing(pl)) return rc;
  const int c = pl->t_cnt;
  if (ms) {
    ms[0] = c ? pl->t_acc[0] / c : 0.0;
    ms[1] = c ? pl->t_acc[1] / c : 0.0;
  }
  if (count) *count = c;
  pl->t_acc[0] = pl->t_acc[1] = 0;
  pl->t_cnt = 0;
  return 0;
}

int bmpc_model_eval(bmpc_ctx* ctx, const bmpc_plan_desc* desc, const bmpc_policy* policies, int B,
                    const double* x, const double* u, const double* z, double* A, double* Bm,
                    double* C, double* xp, double* p, double* dp, double* zpred, double* h0,
                    double* dh) {
  return bmpc_model_eval_ref(ctx, desc, policies, 0, nullptr, nullptr, B, x, u, z, A, Bm, C, xp, p, dp, zpred, h0,
                             dh);
}

int bmpc_model_eval_ref(bmpc_ctx* ctx, const bmpc_plan_desc* desc, const bmpc_policy* policies, int nref,
                        const double* grid, const double* values, int B, const double* x, const double* u,
                        const double* z, double* A, double* Bm, double* C, double* xp, double* p, double* dp,
                        double* zpred, double* h0, double* dh) {
  if (!ctx || !desc || !policies || !x || !u || !z || B <= 0) return fail(-22, "null argument");
  {
    const std::string e = check_lane_ref(nref, grid, values);
    if (!e.empty()) return fail(-22, e);
  }
  for (size_t i = 0; i < (size_t)B * (desc->m > 0 ? desc->m : 0); ++i)
    if (is_psiref(policies[i].kind) && (desc->model != BMPC_MODEL_HIGHWAY_MERGE || nref == 0))
      return fail(-22, "lane-reference (psiref) policies need the HIGHWAY_MERGE model and a lane reference");
  const int n = desc->n, d = desc->d, m = desc->m, N = desc->N;
  if (((desc->model == BMPC_MODEL_HIGHWAY || desc->model == BMPC_MODEL_HIGHWAY_MERGE) && (n != 4 || d != 2)) ||
      (desc->model == BMPC_MODEL_QUADRUPED && (n != 3 || d != 3)) ||
      (desc->model != BMPC_MODEL_HIGHWAY && desc->model != BMPC_MODEL_HIGHWAY_MERGE &&
       desc->model != BMPC_MODEL_QUADRUPED) || m < 1 || m > BMPC_MAX_M || N < 1)
    return fail(-22, "bad model dimensions");
  // one packed upload (policies | x | u | z) and one packed read-back of the requested outputs,
  // on the context's stream into its grow-only buffer: the compat environments call this once
  // per control step, so no allocation and no device-wide synchronisation per call
  const size_t sizes[] = {(size_t)n * n, (size_t)n * d, (size_t)n, (size_t)n, (size_t)m,
                          (size_t)m * n, (size_t)N * m * n, 1, (size_t)n};
  double* hosts[] = {A, Bm, C, xp, p, dp, zpred, h0, dh};
  const bool want[] = {A != nullptr, Bm != nullptr, C != nullptr, xp != nullptr, p != nullptr,
                       dp != nullptr && p != nullptr, zpred != nullptr, h0 != nullptr, dh != nullptr && h0 != nullptr};
  const size_t npol = ((size_t)B * m * sizeof(bmpc_policy) + sizeof(double) - 1) / sizeof(double);
  const size_t tin = npol + (size_t)B * (2 * n + d) + 2 * (size_t)nref;
  size_t tout = 0;
  for (int i = 0; i < 9; ++i) tout += want[i] ? (size_t)B * sizes[i] : 0;
  std::lock_guard<std::mutex> lock(ctx->q_mu);
  HIPCHECK(hipSetDevice(ctx->device));
  std::vector<double>& hv = ctx->q_host;
  hv.resize(tin + tout);
  memcpy(hv.data(), policies, (size_t)B * m * sizeof(bmpc_policy));
  memcpy(hv.data() + npol, x, sizeof(double) * (size_t)B * n);
  memcpy(hv.data() + npol + (size_t)B * n, u, sizeof(double) * (size_t)B * d);
  memcpy(hv.data() + npol + (size_t)B * (n + d), z, sizeof(double) * (size_t)B * n);
  if (nref) {
    memcpy(hv.data() + npol + (size_t)B * (2 * n + d), grid, sizeof(double) * nref);
    memcpy(hv.data() + npol + (size_t)B * (2 * n + d) + nref, values, sizeof(double) * nref);
  }
  HIPCHECK(ctx->q_aux.reserve((tin + tout) * sizeof(double)));
  if (!ctx->qstream) HIPCHECK(hipStreamCreateWithFlags(&ctx->qstream, hipStreamNonBlocking));
  hipStream_t st = ctx->qstream;
  double* buf = ctx->q_aux.as<double>();
  HIPCHECK(hipMemcpyAsync(buf, hv.data(), tin * sizeof(double), hipMemcpyHostToDevice, st));
  const bmpc_policy* dpol = reinterpret_cast<const bmpc_policy*>(buf);
  const double* dxp = buf + npol;
  const double* dup = dxp + (size_t)B * n;
  const double* dzp = dup + (size_t)B * d;
  const double* dref = dzp + (size_t)B * n;
  const LaneRef R{nref ? dref : nullptr, nref ? dref + nref : nullptr, nref};
  double* dev[9];
  double* cur = buf + tin;
  for (int i = 0; i < 9; ++i) {
    dev[i] = want[i] ? cur : nullptr;
    if (want[i]) cur += (size_t)B * sizes[i];
  }
  if (desc->model == BMPC_MODEL_HIGHWAY)
    hipLaunchKernelGGL(k_model<Highway>, dim3((B + 63) / 64), dim3(64), 0, st, *desc, dpol, B, dxp, dup,
                       dzp, dev[0], dev[1], dev[2], dev[3], dev[4], dev[5], dev[6], dev[7], dev[8], R);
  else if (desc->model == BMPC_MODEL_HIGHWAY_MERGE)
    hipLaunchKernelGGL(k_model<HighwayMerge>, dim3((B + 63) / 64), dim3(64), 0, st, *desc, dpol, B, dxp, dup,
                       dzp, dev[0], dev[1], dev[2], dev[3], dev[4], dev[5], dev[6], dev[7], dev[8], R);
  else
    hipLaunchKernelGGL(k_model<Quadruped>, dim3((B + 63) / 64), dim3(64), 0, st, *desc, dpol, B, dxp, dup,
                       dzp, dev[0], dev[1], dev[2], dev[3], dev[4], dev[5], dev[6], dev[7], dev[8], R);
  HIPCHECK(hipGetLastError());
  if (tout) HIPCHECK(hipMemcpyAsync(hv.data() + tin, buf + tin, tout * sizeof(double), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  const double* o = hv.data() + tin;
  for (int i = 0; i < 9; ++i)
    if (want[i]) {
      memcpy(hosts[i], o, sizeof(double) * (size_t)B * sizes[i]);
      o += (size_t)B * sizes[i];
    }
  return 0;
}


int bmpc_set_lane_ref(bmpc_plan* pl, int nref, const double* grid, const double* values) {
  if (!pl) return fail(-22, "null argument");
  if (pl->hp.plan.desc.model != BMPC_MODEL_HIGHWAY_MERGE) return fail(-22, "lane references are for HIGHWAY_MERGE plans");
  {
    const std::string e = check_lane_ref(nref, grid, values);
    if (!e.empty()) return fail(-22, e);
  }
  HIPCHECK(hipSetDevice(pl->ctx->device));
  HIPCHECK(hipStreamSynchronize(pl->stream));   // no solve in flight reads the old reference
  if (pl->user_stream) HIPCHECK(hipStreamSynchronize(pl->user_stream));
  // the new copy is built beside the old one and swapped in only once the device bundle points
  // at it: a failure on the way leaves the plan on its old, still allocated reference
  DevBuf fresh;
  if (nref) {
    HIPCHECK(fresh.alloc(sizeof(double) * 2 * (size_t)nref));
    HIPCHECK(hipMemcpy(fresh.as<double>(), grid, sizeof(double) * nref, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(fresh.as<double>() + nref, values, sizeof(double) * nref, hipMemcpyHostToDevice));
  }
  double* const old = pl->d_lref;
  const int old_n = pl->hp.plan.nlref;
  pl->d_lref = fresh.as<double>();
  pl->hp.plan.nlref = nref;
  pl->hp.plan.lref = nullptr;   // host copy unused; upload_bundle points the device copy at d_lref
  const hipError_t e = upload_bundle(pl);
  if (e != hipSuccess) {
    pl->d_lref = old;
    pl->hp.plan.nlref = old_n;
    return fail(-5, std::string("upload_bundle: ") + hipGetErrorString(e));
  }
  fresh.p = nullptr;   // owned by the plan now
  hipFree(old);
  return 0;
}

int bmpc_hmm_eval(bmpc_ctx* ctx, int M, int m, const double* hc, int B, const double* xb, const double* u,
                  const double* xbackup, double* xbp, double* A, double* Bm, double* C, double* h0,
                  double* Jh) {
  if (!ctx || !hc || !xb || !u || !xbackup || B <= 0) return fail(-22, "null argument");
  if (M < 1 || m < 1 || M > HMM_MAX_AGENTS || m > HMM_MAX_BACKUPS) return fail(-22, "M, m must be in 1..4");
  std::lock_guard<std::mutex> lock(ctx->q_mu);
  HIPCHECK(hipSetDevice(ctx->device));
  const size_t nb = 4 + (size_t)M * m;
  const size_t in_sz[] = {8, (size_t)B * nb, (size_t)B * 2, (size_t)B * M * m * 4};
  const double* in_h[] = {hc, xb, u, xbackup};
  const size_t out_sz[] = {nb, nb * nb, nb * 2, nb, (size_t)M * m, (size_t)M * m * nb};
  double* out_h[] = {xbp, A, Bm, C, h0, Jh};
  // one upload of the packed inputs, one read-back of the packed outputs, on the context's
  // stream into its grow-only buffer (the belief MPC calls this once per control step)
  size_t tin = 0, tout = 0;
  for (size_t v : in_sz) tin += v;
  for (int i = 0; i < 6; ++i) tout += out_h[i] ? (size_t)B * out_sz[i] : 0;
  std::vector<double>& hv = ctx->q_host;
  hv.resize(tin + tout);
  {
    double* c = hv.data();
    for (int i = 0; i < 4; ++i) {
      memcpy(c, in_h[i], in_sz[i] * sizeof(double));
      c += in_sz[i];
    }
  }
  HIPCHECK(ctx->q_aux.reserve((tin + tout) * sizeof(double)));
  if (!ctx->qstream) HIPCHECK(hipStreamCreateWithFlags(&ctx->qstream, hipStreamNonBlocking));
  hipStream_t st = ctx->qstream;
  double* buf = ctx->q_aux.as<double>();
  HIPCHECK(hipMemcpyAsync(buf, hv.data(), tin * sizeof(double), hipMemcpyHostToDevice, st));
  double* din[4];
  double* cur = buf;
  for (int i = 0; i < 4; ++i) {
    din[i] = cur;
    cur += in_sz[i];
  }
  double* dout[6];
  for (int i = 0; i < 6; ++i) {
    dout[i] = out_h[i] ? cur : nullptr;
    if (out_h[i]) cur += (size_t)B * out_sz[i];
  }
  hipLaunchKernelGGL(k_hmm, dim3((B + 63) / 64), dim3(64), 0, st, M, m, din[0], B, din[1], din[2], din[3], dout[0],
                     dout[1], dout[2], dout[3], dout[4], dout[5]);
  HIPCHECK(hipGetLastError());
  if (tout) HIPCHECK(hipMemcpyAsync(hv.data() + tin, buf + tin, tout * sizeof(double), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  const double* o = hv.data() + tin;
  for (int i = 0; i < 6; ++i)
    if (out_h[i]) {
      memcpy(out_h[i], o, (size_t)B * out_sz[i] * sizeof(double));
      o += (size_t)B * out_sz[i];
    }
  return 0;
}

int bmpc_qp_solve(bmpc_ctx* ctx, int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                  const int32_t* Ai, int batch, const double* Px, const double* q, const double* Ax, const double* l,
                  const double* u, int max_iter, double eps, double* x, double* y, int32_t* status, int32_t* iters,
                  int32_t* info) {
  if (!ctx || !q || !x || !status) return fail(-22, "null argument");
  if (n < 1 || m < 0 || batch < 1 || !Pp || !Ap) return fail(-22, "need n >= 1, m >= 0, batch >= 1 and a pattern");
  // the column pointers are checked before they size anything (the cache key below)
  if (Pp[0] != 0 || Ap[0] != 0) return fail(-22, "column pointers must start at 0");
  for (int j = 0; j < n; ++j)
    if (Pp[j + 1] < Pp[j] || Ap[j + 1] < Ap[j]) return fail(-22, "column pointers must be non-decreasing");
  if ((Pp[n] > 0 && !Pi) || (Ap[n] > 0 && !Ai)) return fail(-22, "null row-index array");
  std::lock_guard<std::mutex> lock(ctx->q_mu);
  // the bounds of every problem are checked on every call; the analysis is looked up by
  // pattern + row classes (bandqp_analyse validates the pattern on a miss)
  std::vector<int> cls;
  std::string err = bandqp_classify(m, batch, l, u, cls);
  if (!err.empty()) return fail(-22, err);
  const bool lds_ok = batch <= ctx->cus;   // bandqp_analyse's factor-in-LDS rule depends on this only
  std::vector<int32_t> key;
  key.reserve(6 + 2 * (size_t)n + Pp[n] + Ap[n] + m);
  key.insert(key.end(), {n, m, max_iter, lds_ok ? 1 : 0, Pp[n], Ap[n]});
  key.insert(key.end(), Pp, Pp + n + 1);
  key.insert(key.end(), Ap, Ap + n + 1);
  if (Pp[n] > 0) key.insert(key.end(), Pi, Pi + Pp[n]);
  if (Ap[n] > 0) key.insert(key.end(), Ai, Ai + Ap[n]);
  key.insert(key.end(), cls.begin(), cls.end());
  QPCacheEntry* ent = nullptr;
  for (auto& c : ctx->qcache)
    if (c->eps == eps && c->key == key) ent = c.get();
  HIPCHECK(hipSetDevice(ctx->device));
  if (!ent) {
    auto fresh = std::make_unique<QPCacheEntry>();
    err = bandqp_analyse(n, m, Pp, Pi, Ap, Ai, batch, l, u, max_iter, eps, fresh->h, ctx->cus, ctx->lds_per_cu);
    if (!err.empty()) return fail(-22, err);
    fresh->key.swap(key);
    fresh->eps = eps;
    HIPCHECK(fresh->tab.reserve(fresh->h.blob.size() * sizeof(int32_t)));
    HIPCHECK(hipMemcpy(fresh->tab.p, fresh->h.blob.data(), fresh->h.blob.size() * sizeof(int32_t),
                       hipMemcpyHostToDevice));
    if ((int)ctx->qcache.size() >= bmpc_ctx::kQPCache) {   // evict the least recently used
      auto lru = std::min_element(ctx->qcache.begin(), ctx->qcache.end(),
                                  [](const auto& a, const auto& b) { return a->used < b->used; });
      ctx->qcache.erase(lru);
    }
    ent = fresh.get();
    ctx->qcache.push_back(std::move(fresh));
  }
  ent->used = ++ctx->qclock;
  const HostBandQP& h = ent->h;
  const int nnzP = Pp[n], nnzA = Ap[n];
  if ((nnzP && !Px) || (nnzA && !Ax)) return fail(-22, "null value array");
  if (info) {
    info[0] = h.d.nk;
    info[1] = h.d.bw;
    info[2] = h.d.n_in;
    info[3] = h.d.nscat;
  }
  if (!ctx->qstream) HIPCHECK(hipStreamCreateWithFlags(&ctx->qstream, hipStreamNonBlocking));
  hipStream_t st = ctx->qstream;
  const size_t B = (size_t)batch;
  // host values in the kernel's per-problem order: [Px; Ax] then [q; l; u], one upload
  const size_t nv = std::max<size_t>(B * h.d.nvals, 1), nc = B * h.d.ncvals;
  std::vector<double>& hv = ctx->q_host;
  hv.resize(nv + nc);
  for (size_t b = 0; b < B; ++b) {
    double* v = hv.data() + b * h.d.nvals;
    if (nnzP) memcpy(v, Px + b * nnzP, nnzP * sizeof(double));
    if (nnzA) memcpy(v + nnzP, Ax + b * nnzA, nnzA * sizeof(double));
    double* c = hv.data() + nv + b * h.d.ncvals;
    memcpy(c, q + b * n, n * sizeof(double));
    if (m) {
      memcpy(c + n, l + b * m, m * sizeof(double));
      memcpy(c + n + m, u + b * m, m * sizeof(double));
    }
  }
  HIPCHECK(ctx->q_in.reserve(hv.size() * sizeof(double)));
  HIPCHECK(ctx->q_ws.reserve(B * h.d.stride * sizeof(double)));
  const size_t nout = B * (n + m) * sizeof(double) + 2 * B * sizeof(int32_t);
  HIPCHECK(ctx->q_out.reserve(nout));
  HIPCHECK(hipMemcpyAsync(ctx->q_in.p, hv.data(), hv.size() * sizeof(double), hipMemcpyHostToDevice, st));
  double* dx = ctx->q_out.as<double>();
  double* dy = dx + B * n;
  int32_t* dst = reinterpret_cast<int32_t*>(dy + B * m);
  int32_t* dit = dst + B;
  BandQPDesc d = h.d;
  const int32_t* base = ent->tab.as<int32_t>();
  d.kind = base;
  d.scat = d.kind + h.kind.size();
  d.cscat = d.scat + h.scat.size();
  d.xmap = d.cscat + h.cscat.size();
  d.ymap = d.xmap + h.xmap.size();
  const size_t lds = bandqp_lds_doubles(d.nk, d.W, d.lb_lds) * sizeof(double);
  if (lds > 64 * 1024) HIPCHECK(hipFuncSetAttribute((const void*)k_bandqp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_bandqp, dim3(batch), dim3(64), lds, st, d, ctx->q_in.as<double>(), ctx->q_in.as<double>() + nv,
                     ctx->q_ws.as<double>(), dx, dy, dst, dit, batch);
  HIPCHECK(hipGetLastError());
  // one read-back of x | y | status | iters
  std::vector<char> ho(nout);
  HIPCHECK(hipMemcpyAsync(ho.data(), dx, nout, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  memcpy(x, ho.data(), B * n * sizeof(double));
  if (y && m) memcpy(y, ho.data() + B * n * sizeof(double), B * m * sizeof(double));
  memcpy(status, ho.data() + B * (n + m) * sizeof(double), B * sizeof(int32_t));
  if (iters) memcpy(iters, ho.data() + B * (n + m) * sizeof(double) + B * sizeof(int32_t), B * sizeof(int32_t));
  return 0;
}

}  // extern "C"
