// capi.cpp -- extern "C" boundary of libmpcx.so (declared in include/mpcx.h).
//
// Host-pointer entry points stage inputs into a device workspace owned by the
// handle (grown on demand, never freed inside a solve), launch on the handle's
// stream and copy results back; *_dev entry points only enqueue work.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mpcx.h"
#include "solver.h"


struct mpcx_handle {
  mpcx_spec spec;
  int nw, ng, np;
  hipStream_t stream = nullptr;
  double* d_lbw = nullptr;  // spec bounds
  double* d_ubw = nullptr;
  double* d_lbw_call = nullptr;  // per-call bounds
  double* d_ubw_call = nullptr;
  // workspace (grown on demand)
  size_t cap_B = 0;
  double *d_P = nullptr, *d_w0 = nullptr, *d_w = nullptr, *d_f = nullptr, *d_lam = nullptr;
  double *d_lam0 = nullptr, *d_lamx0 = nullptr, *d_lamx = nullptr;
  int32_t *d_status = nullptr, *d_iters = nullptr;
  double *d_u = nullptr, *d_x = nullptr, *d_q = nullptr, *d_g = nullptr;  // plant / constraint outputs
  size_t cap_sweep = 0;
  double* d_sweep = nullptr;
  // linear model tables (MPCX_MODEL_LINEAR)
  double *d_linA = nullptr, *d_linB = nullptr, *d_linc = nullptr, *d_linW = nullptr;
  int32_t* d_lintab = nullptr;
  int lin_ntab = 0, lin_rows = 0;
  unsigned long long lin_dec = 0;  // LinTables::dec_mask
  const int32_t* ext_tab = nullptr;  // caller-owned device schedule (mpcx_set_linear_tab_dev)
  int ext_rows = 0;
  int n_simd = 0;  // SIMDs of the device (CUs x 4): the solve launch widens lane groups to fill them
  // restoration workspace of the models with a restoration phase (grown on demand)
  size_t cap_ws = 0;
  double* d_ws = nullptr;
  // decoupled-suffix value functions across launches (SolveArgs::pcache)
  double* d_pcache = nullptr;
  double pc_epoch = 0, pc_gen = 1;
  double park_epoch = 0;  // solve launches with a restoration workspace (SolveArgs::park_flag)
  int spec_xbnd = 1;      // the spec bounds bound some state (SolveArgs::xbnd)
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hipfail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return MPCX_EHIP;
}
#define HIPCHK(expr)                                   \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hipfail(e_, #expr);   \
  } while (0)

// The handle's device is made current for the duration of a call and the caller's current
// device restored on every return path (a PyTorch process on another device keeps its state).
struct DeviceScope {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) err = hipSetDevice(dev);
    if (prev == dev || err != hipSuccess) prev = -1;  // nothing to restore
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};
#define DEVICE_SCOPE(dev)                                           \
  DeviceScope device_scope_(dev);                                   \
  if (device_scope_.err != hipSuccess) return hipfail(device_scope_.err, "hipSetDevice")

// (nx, nu) fixed by the model; the linear model takes them from the spec
int nx_of(const mpcx_spec& s) {
  switch (s.model) {
    case MPCX_MODEL_UNICYCLE: case MPCX_MODEL_KIN_BICYCLE: return 3;
    case MPCX_MODEL_DYN_BICYCLE: return 6;
    case MPCX_MODEL_CARTPOLE: return 4;
    default: return s.nx;
  }
}
int nu_of(const mpcx_spec& s) {
  switch (s.model) {
    case MPCX_MODEL_UNICYCLE: case MPCX_MODEL_KIN_BICYCLE: case MPCX_MODEL_DYN_BICYCLE: return 2;
    case MPCX_MODEL_CARTPOLE: return 1;
    default: return s.nu;
  }
}
bool is_ode(int model) { return model >= MPCX_MODEL_KIN_BICYCLE && model <= MPCX_MODEL_CARTPOLE; }

mpcx::OdeParams ode_params(const mpcx_spec& s) {
  mpcx::OdeParams op{};
  op.M = s.M;
  op.h = s.T / s.M;
  for (int i = 0; i < 8; ++i) {
    op.Q[i] = s.Q[i];
    op.R[i] = s.R[i];
    op.par[i] = s.par[i];
  }
  return op;
}

mpcx::StageParams stage_params(const mpcx_spec& s) {
  mpcx::StageParams sp;
  sp.T = s.T;
  sp.M = s.M;
  sp.h = s.T / s.M;
  sp.cost = s.cost;
  for (int i = 0; i < 3; ++i) sp.Q[i] = s.Q[i];
  for (int i = 0; i < 2; ++i) sp.R[i] = s.R[i];
  return sp;
}

void spec_bounds(const mpcx_spec& s, std::vector<double>& lb, std::vector<double>& ub) {
  const int N = s.N, nx = nx_of(s), nu = nu_of(s), nz = nx + nu, nw = nx + nz * N;
  lb.assign(nw, -1e20);
  ub.assign(nw, 1e20);
  for (int k = 0; k < N; ++k) {
    for (int i = 0; i < nu; ++i) {
      lb[nx + nz * k + i] = s.lbu[i];
      ub[nx + nz * k + i] = s.ubu[i];
    }
    for (int i = 0; i < nx; ++i) {
      lb[nx + nz * k + nu + i] = s.lbx[i];
      ub[nx + nz * k + nu + i] = s.ubx[i];
    }
  }
}

// 1 if any node k >= 1 has a finite state bound (X_0 is always free)
int state_bounded(const std::vector<double>& lb, const std::vector<double>& ub, int nx, int nu, int N) {
  for (int k = 1; k <= N; ++k)
    for (int i = 0; i < nx; ++i) {
      const int j = nx + (nx + nu) * (k - 1) + nu + i;
      if (lb[j] > -1e19 || ub[j] < 1e19) return 1;
    }
  return 0;
}

// Device buffers are released by the helpers below, which also null the pointers: a failed
// (re)allocation leaves the handle in a clean state (no dangling or half-set buffers).
template <class T>
void dev_free(T*& p) {
  (void)hipFree(p);
  p = nullptr;
}

void free_workspace(mpcx_handle* h) {
  dev_free(h->d_P);
  dev_free(h->d_w0);
  dev_free(h->d_w);
  dev_free(h->d_f);
  dev_free(h->d_lam);
  dev_free(h->d_status);
  dev_free(h->d_iters);
  dev_free(h->d_lam0);
  dev_free(h->d_lamx0);
  dev_free(h->d_lamx);
  dev_free(h->d_u);
  dev_free(h->d_x);
  dev_free(h->d_q);
  dev_free(h->d_g);
  h->cap_B = 0;
}

void free_linear(mpcx_handle* h) {
  dev_free(h->d_linA);
  dev_free(h->d_linB);
  dev_free(h->d_linc);
  dev_free(h->d_linW);
  dev_free(h->d_lintab);
  h->lin_ntab = h->lin_rows = 0;
  h->ext_tab = nullptr;
  h->ext_rows = 0;
}

// per-batch workspace of the host-pointer entry points, grown on demand (never shrunk)
int ensure(mpcx_handle* h, size_t B) {
  if (B <= h->cap_B) return 0;
  const size_t nb = B < 256 ? 256 : B;
  free_workspace(h);
  const int nx = h->spec.nx, nu = h->spec.nu;
  struct Buf {
    void** p;
    size_t bytes;
  } bufs[] = {{(void**)&h->d_P, nb * h->np * sizeof(double)},   {(void**)&h->d_w0, nb * h->nw * sizeof(double)},
              {(void**)&h->d_w, nb * h->nw * sizeof(double)},   {(void**)&h->d_f, nb * sizeof(double)},
              {(void**)&h->d_lam, nb * h->ng * sizeof(double)}, {(void**)&h->d_status, nb * sizeof(int32_t)},
              {(void**)&h->d_iters, nb * sizeof(int32_t)},      {(void**)&h->d_lam0, nb * h->ng * sizeof(double)},
              {(void**)&h->d_lamx0, nb * h->nw * sizeof(double)}, {(void**)&h->d_lamx, nb * h->nw * sizeof(double)},
              {(void**)&h->d_u, nb * nu * sizeof(double)},      {(void**)&h->d_x, nb * nx * sizeof(double)},
              {(void**)&h->d_q, nb * sizeof(double)},           {(void**)&h->d_g, nb * h->ng * sizeof(double)}};
  for (const Buf& b : bufs) {
    const hipError_t e = hipMalloc(b.p, b.bytes);
    if (e != hipSuccess) {
      free_workspace(h);
      return hipfail(e, "workspace allocation");
    }
  }
  h->cap_B = nb;
  return 0;
}

int check_bounds_vec(const mpcx_handle* h, const double* lbw, const double* ubw) {
  if (!lbw && !ubw) return 0;
  for (int i = 0; i < h->nw; ++i) {
    const double l = lbw ? lbw[i] : -1e20, u = ubw ? ubw[i] : 1e20;
    if (std::isnan(l) || std::isnan(u) || l > u) return fail(MPCX_EINVAL, "lbw/ubw: NaN or lb > ub at index " + std::to_string(i));
    // X_0 (i < nx) is pinned by g_0 and its bounds are replaced by +-inf (mpcx_solve_batch), so
    // a caller fixing it through lbx = ubx (CasADi style) is accepted
    if (l == u && l > -1e19 && i >= h->spec.nx)
      return fail(MPCX_EINVAL, "lbw == ubw (fixed variable) is not supported, index " + std::to_string(i));
  }
  return 0;
}
}  // namespace

extern "C" {

const char* mpcx_last_error(void) { return g_err.c_str(); }

// hash of the sources this library was built from (Makefile: MPCX_SRC_HASH); the loader
// (mpcx/_lib.py) refuses a library whose hash differs from the tree's
const char* mpcx_source_hash(void) {
#ifdef MPCX_SRC_HASH
  return MPCX_SRC_HASH;
#else
  return "unknown";
#endif
}

int mpcx_default_spec(mpcx_spec* s, int32_t model, int32_t N) {
  if (!s) return fail(MPCX_EINVAL, "null spec");
  if (model != MPCX_MODEL_UNICYCLE && !is_ode(model)) return fail(MPCX_EINVAL, "unknown model");
  std::memset(s, 0, sizeof *s);
  // Casadi/multiple_shooting_casadi.py:30-45, 78-84, 101, 188-196
  s->model = model;
  s->cost = MPCX_COST_QUADRATURE;
  s->param_layout = MPCX_P_X0_XREF;
  s->N = N;
  s->M = 4;
  s->max_iter = 2000;
  s->device = 0;
  s->T = 0.2;
  s->tol = 1e-8;
  s->Q[0] = 1.0; s->Q[1] = 5.0; s->Q[2] = 0.1;
  s->R[0] = 0.5; s->R[1] = 0.05;
  s->lbu[0] = -1.0; s->ubu[0] = 1.0;
  s->lbu[1] = -M_PI / 4; s->ubu[1] = M_PI / 4;
  for (int i = 0; i < 3; ++i) {
    s->lbx[i] = -1e20;
    s->ubx[i] = 1e20;
  }
  s->nx = 3;
  s->nu = 2;
  s->warm_mu_init = 1e-4;
  s->warm_bound_push = 1e-4;
  s->warm_mult_push = 1e-4;
  // IPOPT termination options: the reference's acceptable_tol / acceptable_obj_change_tol
  // (:192-193), IPOPT's defaults for the rest
  s->dual_inf_tol = 1.0;
  s->constr_viol_tol = 1e-4;
  s->compl_inf_tol = 1e-4;
  s->acceptable_tol = 1e-8;
  s->acceptable_dual_inf_tol = 1e10;
  s->acceptable_constr_viol_tol = 1e-2;
  s->acceptable_compl_inf_tol = 1e-2;
  s->acceptable_obj_change_tol = 1e-6;
  s->acceptable_iter = 15;
  if (is_ode(model)) {  // no reference script: IPOPT's defaults
    s->acceptable_tol = 1e-6;
    s->acceptable_obj_change_tol = 1e20;
  }
  if (is_ode(model)) {  // defaults of the BASELINE config variants (mpcx/ode.py documents them)
    s->cost = MPCX_COST_NODE;
    s->param_layout = MPCX_P_X0_STAGEREF;
    s->M = 1;
    s->nx = nx_of(*s);
    s->nu = nu_of(*s);
    for (int i = 0; i < 8; ++i) {
      s->Q[i] = s->R[i] = 0.0;
      s->lbx[i] = -1e20;
      s->ubx[i] = 1e20;
    }
  }
  if (model == MPCX_MODEL_KIN_BICYCLE) {  // config 3 variant: circular tracking, T = 0.2
    s->Q[0] = 1.0; s->Q[1] = 1.0; s->Q[2] = 0.1;
    s->R[0] = 0.5; s->R[1] = 0.05;
    s->lbu[0] = -1.0; s->ubu[0] = 1.0;
    s->lbu[1] = -M_PI / 4; s->ubu[1] = M_PI / 4;
    s->par[0] = 0.5;  // wheelbase L
  } else if (model == MPCX_MODEL_DYN_BICYCLE) {  // config 4 variant: lane change, T = 0.05
    s->T = 0.05;
    s->M = 4;  // RK4 stability at 4-8 m/s (|A44| h <= 1.6)
    for (int i = 0; i < 6; ++i) s->Q[i] = 1.0;  // Trajectory_tracking_dynamic_model.py:23-31 (Q = I, R = 1)
    s->R[0] = 1.0; s->R[1] = 1.0;
    s->lbu[0] = -0.5; s->ubu[0] = 0.5;  // steering [rad]
    s->lbu[1] = -5.0; s->ubu[1] = 5.0;  // longitudinal acceleration [m/s^2]
    s->lbx[3] = 2.5;                    // vx >= 2.5 m/s: RK4 (M = 4) stays stable, |A44| h <= 2.55
    const double par[5] = {1200.0, 1.5, 2.0, 55000.0, 1350.0};  // :36-40
    for (int i = 0; i < 5; ++i) s->par[i] = par[i];
  } else if (model == MPCX_MODEL_CARTPOLE) {  // config 5 variant: swing-up, T = 0.01
    s->T = 0.01;
    s->param_layout = MPCX_P_X0_XREF;
    s->Q[0] = 1.44; s->Q[2] = 1.0;  // l = (1.2 (p - p_ref))^2 + phi^2 (inverted_pendulum...py:33-36)
    s->R[0] = 1e-4;                 // (0.01 u)^2
    s->lbu[0] = -200.0; s->ubu[0] = 200.0;  // :28
    const double par[5] = {1.0, 1.0, 0.5, 9.81, 10.0};
    for (int i = 0; i < 5; ++i) s->par[i] = par[i];
  }
  return 0;
}

int mpcx_create(const mpcx_spec* s, mpcx_handle** out) {
  if (!s || !out) return fail(MPCX_EINVAL, "null argument");
  if (s->model != MPCX_MODEL_UNICYCLE && s->model != MPCX_MODEL_LINEAR && !is_ode(s->model))
    return fail(MPCX_EINVAL, "unknown model");
  if (is_ode(s->model) && s->cost != MPCX_COST_NODE) return fail(MPCX_EINVAL, "ODE models use MPCX_COST_NODE");
  if (s->model == MPCX_MODEL_LINEAR &&
      !((s->nx == 4 && s->nu == 1) || (s->nx == 5 && s->nu == 1) || (s->nx == 4 && s->nu == 2)))
    return fail(MPCX_EINVAL, "linear model: (nx, nu) must be (4, 1), (5, 1) or (4, 2)");
  if (s->N < 1 || s->N > 255) return fail(MPCX_EINVAL, "N must be in [1, 255]");
  if (s->M < 1 || s->M > 64) return fail(MPCX_EINVAL, "M must be in [1, 64]");
  if ((s->model == MPCX_MODEL_UNICYCLE || is_ode(s->model)) && !(s->T > 0)) return fail(MPCX_EINVAL, "T must be > 0");
  if (s->cost != MPCX_COST_QUADRATURE && s->cost != MPCX_COST_NODE) return fail(MPCX_EINVAL, "unknown cost");
  if (s->param_layout != MPCX_P_X0_XREF && s->param_layout != MPCX_P_X0_STAGEREF)
    return fail(MPCX_EINVAL, "unknown param_layout");
  if (s->max_iter < 0) return fail(MPCX_EINVAL, "max_iter < 0");
  if (s->group_policy != 0 && s->group_policy != 1) return fail(MPCX_EINVAL, "group_policy must be 0 or 1");
  if (!(s->tol > 0)) return fail(MPCX_EINVAL, "tol must be > 0");
  {
    const double o[7] = {s->dual_inf_tol, s->constr_viol_tol, s->compl_inf_tol, s->acceptable_tol,
                         s->acceptable_dual_inf_tol, s->acceptable_constr_viol_tol, s->acceptable_compl_inf_tol};
    for (double v : o)
      if (!(v >= 0)) return fail(MPCX_EINVAL, "IPOPT tolerance options must be >= 0 (0 = IPOPT default)");
    if (std::isnan(s->acceptable_obj_change_tol))
      return fail(MPCX_EINVAL, "acceptable_obj_change_tol is NaN (negative = IPOPT default)");
    if (s->acceptable_iter < -1) return fail(MPCX_EINVAL, "acceptable_iter must be >= -1");
    if (s->no_restoration != 0 && s->no_restoration != 1) return fail(MPCX_EINVAL, "no_restoration must be 0 or 1");
  }
  if (!(s->warm_mu_init > 0) || !(s->warm_bound_push > 0) || !(s->warm_mult_push > 0))
    return fail(MPCX_EINVAL, "warm_mu_init / warm_bound_push / warm_mult_push must be > 0");
  for (int i = 0; i < nu_of(*s); ++i)
    if (!(s->lbu[i] < s->ubu[i])) return fail(MPCX_EINVAL, "lbu must be < ubu");
  for (int i = 0; i < nx_of(*s); ++i)
    if (!(s->lbx[i] < s->ubx[i])) return fail(MPCX_EINVAL, "lbx must be < ubx");
  if (s->model == MPCX_MODEL_LINEAR && s->param_layout != MPCX_P_X0_STAGEREF)
    return fail(MPCX_EINVAL, "linear model uses param_layout MPCX_P_X0_STAGEREF");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(MPCX_EHIP, "no HIP device available");
  if (s->device < 0 || s->device >= ndev) return fail(MPCX_EINVAL, "device ordinal out of range");
  DEVICE_SCOPE(s->device);
  mpcx_handle* h = new mpcx_handle();
  h->spec = *s;
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, s->device) == hipSuccess) h->n_simd = 4 * n_cu;
  h->spec.nx = nx_of(*s);
  h->spec.nu = nu_of(*s);
  const int nx = h->spec.nx, nz = nx + h->spec.nu;
  h->nw = nx + nz * s->N;
  h->ng = nx * (s->N + 1);
  h->np = s->param_layout == MPCX_P_X0_XREF ? 2 * nx : nx + nz * s->N;
  std::vector<double> lb, ub;
  spec_bounds(*s, lb, ub);
  h->spec_xbnd = state_bounded(lb, ub, h->spec.nx, h->spec.nu, s->N);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&h->d_lbw, h->nw * sizeof(double)) != hipSuccess ||
      hipMalloc(&h->d_ubw, h->nw * sizeof(double)) != hipSuccess ||
      hipMalloc(&h->d_lbw_call, h->nw * sizeof(double)) != hipSuccess ||
      hipMalloc(&h->d_ubw_call, h->nw * sizeof(double)) != hipSuccess ||
      hipMemcpy(h->d_lbw, lb.data(), h->nw * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->d_ubw, ub.data(), h->nw * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    mpcx_destroy(h);
    return fail(MPCX_EHIP, "device allocation failed in mpcx_create");
  }
  *out = h;
  return 0;
}

void mpcx_destroy(mpcx_handle* h) {
  if (!h) return;
  DeviceScope device_scope_(h->spec.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  dev_free(h->d_lbw);
  dev_free(h->d_ubw);
  dev_free(h->d_lbw_call);
  dev_free(h->d_ubw_call);
  free_workspace(h);
  dev_free(h->d_sweep);
  dev_free(h->d_ws);
  dev_free(h->d_pcache);
  free_linear(h);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int mpcx_dims(const mpcx_handle* h, int32_t* n_w, int32_t* n_g, int32_t* n_p) {
  if (!h) return fail(MPCX_EINVAL, "null handle");
  if (n_w) *n_w = h->nw;
  if (n_g) *n_g = h->ng;
  if (n_p) *n_p = h->np;
  return 0;
}

int mpcx_set_linear_model(mpcx_handle* h, int32_t n_tab, const double* A, const double* B, const double* c,
                          const double* W, const int32_t* tab, int32_t tab_rows) {
  if (!h || !A || !B || !W || !tab) return fail(MPCX_EINVAL, "null argument");
  if (h->spec.model != MPCX_MODEL_LINEAR) return fail(MPCX_EINVAL, "handle is not a linear model");
  if (n_tab < 1 || tab_rows < 1) return fail(MPCX_EINVAL, "n_tab and tab_rows must be >= 1");
  const int nx = h->spec.nx, nu = h->spec.nu, nz = nx + nu, nh = nz * (nz + 1) / 2, N = h->spec.N;
  for (long i = 0; i < (long)tab_rows * N; ++i)
    if (tab[i] < 0 || tab[i] >= n_tab) return fail(MPCX_EINVAL, "table index out of range at " + std::to_string(i));
  DEVICE_SCOPE(h->spec.device);
  HIPCHK(hipStreamSynchronize(h->stream));  // no launch may still read the old tables
  free_linear(h);
  std::vector<double> cz((size_t)n_tab * nx, 0.0);
  const hipError_t e = [&]() {
    hipError_t r;
    if ((r = hipMalloc(&h->d_linA, (size_t)n_tab * nx * nx * sizeof(double))) != hipSuccess) return r;
    if ((r = hipMalloc(&h->d_linB, (size_t)n_tab * nx * nu * sizeof(double))) != hipSuccess) return r;
    if ((r = hipMalloc(&h->d_linc, (size_t)n_tab * nx * sizeof(double))) != hipSuccess) return r;
    if ((r = hipMalloc(&h->d_linW, (size_t)n_tab * nh * sizeof(double))) != hipSuccess) return r;
    if ((r = hipMalloc(&h->d_lintab, (size_t)tab_rows * N * sizeof(int32_t))) != hipSuccess) return r;
    if ((r = hipMemcpy(h->d_linA, A, (size_t)n_tab * nx * nx * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
      return r;
    if ((r = hipMemcpy(h->d_linB, B, (size_t)n_tab * nx * nu * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
      return r;
    if ((r = hipMemcpy(h->d_linc, c ? c : cz.data(), (size_t)n_tab * nx * sizeof(double), hipMemcpyHostToDevice)) !=
        hipSuccess)
      return r;
    if ((r = hipMemcpy(h->d_linW, W, (size_t)n_tab * nh * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess)
      return r;
    return hipMemcpy(h->d_lintab, tab, (size_t)tab_rows * N * sizeof(int32_t), hipMemcpyHostToDevice);
  }();
  if (e != hipSuccess) {
    free_linear(h);  // never leave a half-set table behind (check_model_ready tests d_linA)
    return hipfail(e, "mpcx_set_linear_model");
  }
  h->lin_ntab = n_tab;
  h->lin_rows = tab_rows;
  h->pc_gen += 1;  // cached suffix value functions belong to the old tables
  h->lin_dec = 0;
  for (int j = 0; j < n_tab && j < 64; ++j) {
    bool d = true;
    for (int i = 0; i < nx * nu; ++i) d = d && B[(size_t)j * nx * nu + i] == 0.0;
    for (int r = 0; r < nx; ++r)
      for (int l = 0; l < nu; ++l) d = d && W[(size_t)j * nh + r * nz - r * (r - 1) / 2 + (nx + l - r)] == 0.0;
    if (d) h->lin_dec |= 1ull << j;
  }
  // diagnostic knob: MPCX_DEC_SUFFIX=0 disables the reuse (tests compare both paths' bits)
  if (const char* e = getenv("MPCX_DEC_SUFFIX"))
    if (atoi(e) == 0) h->lin_dec = 0;
  return 0;
}

int mpcx_set_linear_tab_dev(mpcx_handle* h, const int32_t* d_tab, int32_t tab_rows) {
  if (!h) return fail(MPCX_EINVAL, "null handle");
  if (h->spec.model != MPCX_MODEL_LINEAR) return fail(MPCX_EINVAL, "handle is not a linear model");
  if (!h->d_linA) return fail(MPCX_EINVAL, "linear model tables not set (mpcx_set_linear_model)");
  if (d_tab && tab_rows < 1) return fail(MPCX_EINVAL, "tab_rows must be >= 1");
  h->ext_tab = d_tab;
  h->ext_rows = d_tab ? tab_rows : 0;
  h->pc_gen += 1;  // the schedule (hence the suffix) may have changed
  return 0;
}

static int check_model_ready(const mpcx_handle* h, int B) {
  if (h->spec.model != MPCX_MODEL_LINEAR) return 0;
  if (!h->d_linA) return fail(MPCX_EINVAL, "linear model tables not set (mpcx_set_linear_model)");
  const int rows = h->ext_tab ? h->ext_rows : h->lin_rows;
  if (rows > 1 && B > rows) return fail(MPCX_EINVAL, "batch larger than the per-instance table rows");
  return 0;
}

static mpcx::SolveArgs make_args(const mpcx_handle* h, int B, const double* P, const double* w0, const double* lam0,
                                 const double* lamx0, const double* lbw, const double* ubw, double* w, double* f,
                                 double* lam, double* lamx, int32_t* st, int32_t* it) {
  mpcx::SolveArgs a{};
  a.B = B;
  a.model = h->spec.model;
  a.n_simd = h->n_simd;
  a.group_policy = h->spec.group_policy;
  a.nx = h->spec.nx;
  a.nu = h->spec.nu;
  a.lin.A = h->d_linA;
  a.lin.B = h->d_linB;
  a.lin.c = h->d_linc;
  a.lin.W = h->d_linW;
  a.lin.tab = h->ext_tab ? h->ext_tab : h->d_lintab;
  a.lin.per_instance = (h->ext_tab ? h->ext_rows : h->lin_rows) > 1 ? 1 : 0;
  a.lin.n_tab = h->lin_ntab;
  a.lin.dec_mask = h->lin_dec;
  a.N = h->spec.N;
  a.max_iter = h->spec.max_iter;
  a.p_layout = h->spec.param_layout;
  a.p_stride = h->np;
  a.tol = h->spec.tol;
  {  // IPOPT options, 0 = IPOPT default
    const mpcx_spec& sp = h->spec;
    auto d = [](double v, double def) { return v > 0 ? v : def; };
    a.dual_inf_tol = d(sp.dual_inf_tol, 1.0);
    a.constr_viol_tol = d(sp.constr_viol_tol, 1e-4);
    a.compl_inf_tol = d(sp.compl_inf_tol, 1e-4);
    a.acc_tol = d(sp.acceptable_tol, 1e-6);
    a.acc_dual_inf_tol = d(sp.acceptable_dual_inf_tol, 1e10);
    a.acc_constr_viol_tol = d(sp.acceptable_constr_viol_tol, 1e-2);
    a.acc_compl_inf_tol = d(sp.acceptable_compl_inf_tol, 1e-2);
    // 0 (a zero-filled spec) or negative = IPOPT's default, as for every field above
    a.acc_obj_change_tol = d(sp.acceptable_obj_change_tol, 1e20);
    a.acc_iter = sp.acceptable_iter == 0 ? 15 : (sp.acceptable_iter < 0 ? 0 : sp.acceptable_iter);
    a.restoration = sp.no_restoration ? 0 : 1;
  }
  a.sp = stage_params(h->spec);
  a.op = ode_params(h->spec);
  a.P = P;
  a.w0 = w0;
  a.lam0 = lam0;
  a.lamx0 = lamx0;
  a.warm = (lam0 || lamx0) ? 1 : 0;
  a.mu_init = h->spec.warm_mu_init;
  a.bound_push = h->spec.warm_bound_push;
  a.mult_push = h->spec.warm_mult_push;
  a.lbw = lbw;
  a.ubw = ubw;
  a.xbnd = h->spec_xbnd;
  a.w_out = w;
  a.f_out = f;
  a.lam_out = lam;
  a.lamx_out = lamx;
  a.status = st;
  a.iters = it;
  return a;
}

int mpcx_launch_shape(const mpcx_handle* h, int32_t B, int32_t* lanes, int32_t* replicas, char* kernel,
                      int32_t kernel_len) {
  if (!h) return fail(MPCX_EINVAL, "null handle");
  if (B < 1) return fail(MPCX_EINVAL, "B < 1");
  if (kernel && kernel_len < 1) return fail(MPCX_EINVAL, "kernel_len < 1");
  const mpcx::SolveArgs a = make_args(h, B, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, nullptr, nullptr);
  int G = 0, R = 0;
  const char* model = nullptr;
  if (mpcx::solve_shape(a, &G, &R, &model) != hipSuccess || !model) return fail(MPCX_EINVAL, "no kernel for this model");
  if (lanes) *lanes = G;
  if (replicas) *replicas = R;
  if (kernel) {
    const int n = snprintf(kernel, (size_t)kernel_len, "void mpcx::solve_kernel<%s, %d, false, %d>(mpcx::SolveArgs)",
                           model, G, R);
    if (n < 0 || n >= kernel_len) return fail(MPCX_EINVAL, "kernel name buffer too small");
  }
  return 0;
}

// launch the solve with the restoration workspace of the model (grown on demand; freed only
// after the device is idle, since a queued launch may still use it)
static int solve_launch(mpcx_handle* h, mpcx::SolveArgs& a, hipStream_t stream) {
  const int slots = mpcx::resto_ws_slots(a.model, a.nx, a.nu);
  if (slots > 0) {  // (the 6-state bicycle's chain stash needs it with restoration off too)
    int Gk = 0, R = 0;  // the launch's lanes per instance (the kernel's grid, kernels.h solve_shape)
    const char* kname = nullptr;
    if (mpcx::solve_shape(a, &Gk, &R, &kname) != hipSuccess) return fail(MPCX_EINVAL, "no kernel for this model");
    const int G = Gk * R;
    const long bs = G > 64 ? G : 64;
    const long threads = ((long)a.B * G + bs - 1) / bs * bs;
    const size_t need = (size_t)slots * threads + 1;  // + the park flag
    if (need > h->cap_ws) {
      HIPCHK(hipDeviceSynchronize());  // a queued launch may still use the old buffer
      dev_free(h->d_ws);
      h->cap_ws = 0;
      HIPCHK(hipMalloc(&h->d_ws, need * sizeof(double)));
      // stream-ordered: the caller's stream may be non-blocking w.r.t. the null stream
      HIPCHK(hipMemsetAsync(h->d_ws, 0, need * sizeof(double), stream));  // no instance parked
      h->cap_ws = need;
    }
    a.ws = h->d_ws;
    a.ws_stride = threads;
    a.park_flag = h->d_ws + (size_t)slots * threads;
    a.park_epoch = (h->park_epoch += 1);
  } else {
    a.restoration = 0;
  }
  // decoupled-suffix value functions of earlier launches (kernels.h "decoupled suffix").  Not
  // with a caller-owned device schedule (mpcx_set_linear_tab_dev): the caller may rewrite it on
  // the device between launches without a call the cache's generation could follow.
  if (a.model == MPCX_MODEL_LINEAR && h->lin_dec != 0 && h->ext_tab == nullptr) {
    if (!h->d_pcache) {
      const size_t n = (size_t)(a.N + 2) * (a.nx * (a.nx + 1) / 2);
      HIPCHK(hipMalloc(&h->d_pcache, n * sizeof(double)));
      HIPCHK(hipMemsetAsync(h->d_pcache, 0, n * sizeof(double), stream));  // header epoch 0: nothing cached
    }
    a.pcache = h->d_pcache;
    a.pc_epoch = (h->pc_epoch += 1);
    a.pc_gen = h->pc_gen;
  }
  HIPCHK(mpcx::launch_solve(a, stream));
  // instances parked at a failed line search continue in the resume launch (restoration)
  if (a.restoration) HIPCHK(mpcx::launch_resume(a, stream));
  return 0;
}

int mpcx_solve_batch_dev(mpcx_handle* h, int32_t B, const double* d_P, const double* d_w0, const double* d_lam_g0,
                         const double* d_lam_x0, double* d_w_out, double* d_f_out, double* d_lam_g,
                         double* d_lam_x, int32_t* d_status, int32_t* d_iters, void* stream) {
  if (!h || !d_P || !d_w_out) return fail(MPCX_EINVAL, "null argument");
  if (B < 0) return fail(MPCX_EINVAL, "B < 0");
  if (B == 0) return 0;
  if (int r = check_model_ready(h, B)) return r;
  DEVICE_SCOPE(h->spec.device);
  mpcx::SolveArgs a = make_args(h, B, d_P, d_w0, d_lam_g0, d_lam_x0, h->d_lbw, h->d_ubw, d_w_out, d_f_out, d_lam_g,
                                d_lam_x, d_status, d_iters);
  if (int r = solve_launch(h, a, (hipStream_t)stream)) return r;
  return 0;
}

int mpcx_step_dev(mpcx_handle* h, int32_t B, double* d_P, double* d_w0, double* d_lam_g0, double* d_lam_x0,
                  int32_t flags, double* d_w_out, double* d_f_out, double* d_lam_g, double* d_lam_x,
                  int32_t* d_status, int32_t* d_iters, void* stream) {
  if (!h || !d_P || !d_w0 || !d_w_out) return fail(MPCX_EINVAL, "null argument");
  if (B < 0) return fail(MPCX_EINVAL, "B < 0");
  if (flags & ~(MPCX_STEP_COLD | MPCX_STEP_PRIMAL_ONLY)) return fail(MPCX_EINVAL, "unknown flags");
  if (B == 0) return 0;
  if (int r = check_model_ready(h, B)) return r;
  DEVICE_SCOPE(h->spec.device);
  const bool cold = flags & MPCX_STEP_COLD;
  const bool duals = !cold && !(flags & MPCX_STEP_PRIMAL_ONLY);
  mpcx::SolveArgs a = make_args(h, B, d_P, cold ? nullptr : d_w0, duals ? d_lam_g0 : nullptr,
                                duals ? d_lam_x0 : nullptr, h->d_lbw, h->d_ubw, d_w_out, d_f_out, d_lam_g, d_lam_x,
                                d_status, d_iters);
  a.P_next = d_P;
  a.w0_next = d_w0;
  a.lam0_next = d_lam_g0;
  a.lamx0_next = d_lam_x0;
  if (int r = solve_launch(h, a, (hipStream_t)stream)) return r;
  return 0;
}

int mpcx_run_dev(mpcx_handle* h, int32_t B, int32_t K, double* d_P, double* d_w0, double* d_lam_g0, double* d_lam_x0,
                 int32_t flags, const double* d_Pseq, const int32_t* d_tabseq, double* d_w_out, double* d_f_out,
                 double* d_lam_g, double* d_lam_x, int32_t* d_status, int32_t* d_iters, void* stream) {
  if (!h || !d_P || !d_w0 || !d_w_out) return fail(MPCX_EINVAL, "null argument");
  if (B < 0) return fail(MPCX_EINVAL, "B < 0");
  if (K < 1) return fail(MPCX_EINVAL, "K must be >= 1");
  if (flags & ~(MPCX_STEP_COLD | MPCX_STEP_PRIMAL_ONLY)) return fail(MPCX_EINVAL, "unknown flags");
  if (d_tabseq && h->spec.model != MPCX_MODEL_LINEAR) return fail(MPCX_EINVAL, "d_tabseq needs a linear model");
  if (B == 0) return 0;
  if (int r = check_model_ready(h, B)) return r;
  DEVICE_SCOPE(h->spec.device);
  const bool cold = flags & MPCX_STEP_COLD;
  const bool duals = !(flags & MPCX_STEP_PRIMAL_ONLY) && (d_lam_g0 || d_lam_x0);
  mpcx::SolveArgs a = make_args(h, B, d_P, cold ? nullptr : d_w0, (duals && !cold) ? d_lam_g0 : nullptr,
                                (duals && !cold) ? d_lam_x0 : nullptr, h->d_lbw, h->d_ubw, d_w_out, d_f_out, d_lam_g,
                                d_lam_x, d_status, d_iters);
  a.P_next = d_P;
  a.w0_next = d_w0;
  a.lam0_next = d_lam_g0;
  a.lamx0_next = d_lam_x0;
  a.steps = K;
  a.warm_next = duals ? 1 : 0;
  a.Pseq = d_Pseq;
  a.tabseq = d_tabseq;
  if (int r = solve_launch(h, a, (hipStream_t)stream)) return r;
  return 0;
}

int mpcx_solve_batch(mpcx_handle* h, int32_t B, const double* P, const double* w0, const double* lam_g0,
                     const double* lam_x0, const double* lbw, const double* ubw, double* w_out, double* f_out,
                     double* g_out, double* lam_g, double* lam_x, int32_t* status, int32_t* iters) {
  if (!h || !P || !w_out) return fail(MPCX_EINVAL, "null argument");
  if (B < 0) return fail(MPCX_EINVAL, "B < 0");
  if (B == 0) return 0;
  if (int r = check_bounds_vec(h, lbw, ubw)) return r;
  if (int r = check_model_ready(h, B)) return r;
  DEVICE_SCOPE(h->spec.device);
  if (int r = ensure(h, B)) return r;
  hipStream_t s = h->stream;
  const double* dl = h->d_lbw;
  const double* du = h->d_ubw;
  int call_xbnd = h->spec_xbnd;
  if (lbw || ubw) {
    std::vector<double> lb, ub;
    spec_bounds(h->spec, lb, ub);
    if (lbw) lb.assign(lbw, lbw + h->nw);
    if (ubw) ub.assign(ubw, ubw + h->nw);
    for (int i = 0; i < h->spec.nx; ++i) {  // X_0 stays free: it is pinned by g_0
      lb[i] = -1e20;
      ub[i] = 1e20;
    }
    for (int i = 0; i < h->nw; ++i) {
      if (!(lb[i] > -1e19)) lb[i] = -1e20;
      if (!(ub[i] < 1e19)) ub[i] = 1e20;
    }
    HIPCHK(hipMemcpyAsync(h->d_lbw_call, lb.data(), h->nw * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(h->d_ubw_call, ub.data(), h->nw * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    dl = h->d_lbw_call;
    du = h->d_ubw_call;
    call_xbnd = state_bounded(lb, ub, h->spec.nx, h->spec.nu, h->spec.N);
  }
  HIPCHK(hipMemcpyAsync(h->d_P, P, (size_t)B * h->np * sizeof(double), hipMemcpyHostToDevice, s));
  if (w0) HIPCHK(hipMemcpyAsync(h->d_w0, w0, (size_t)B * h->nw * sizeof(double), hipMemcpyHostToDevice, s));
  if (lam_g0) HIPCHK(hipMemcpyAsync(h->d_lam0, lam_g0, (size_t)B * h->ng * sizeof(double), hipMemcpyHostToDevice, s));
  if (lam_x0) HIPCHK(hipMemcpyAsync(h->d_lamx0, lam_x0, (size_t)B * h->nw * sizeof(double), hipMemcpyHostToDevice, s));
  mpcx::SolveArgs a = make_args(h, B, h->d_P, w0 ? h->d_w0 : nullptr, lam_g0 ? h->d_lam0 : nullptr,
                                lam_x0 ? h->d_lamx0 : nullptr, dl, du, h->d_w, h->d_f, (lam_g ? h->d_lam : nullptr),
                                (lam_x ? h->d_lamx : nullptr), h->d_status, h->d_iters);
  a.xbnd = call_xbnd;
  if (int r = solve_launch(h, a, s)) return r;
  if (lam_x) HIPCHK(hipMemcpyAsync(lam_x, h->d_lamx, (size_t)B * h->nw * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(w_out, h->d_w, (size_t)B * h->nw * sizeof(double), hipMemcpyDeviceToHost, s));
  if (f_out) HIPCHK(hipMemcpyAsync(f_out, h->d_f, (size_t)B * sizeof(double), hipMemcpyDeviceToHost, s));
  if (lam_g) HIPCHK(hipMemcpyAsync(lam_g, h->d_lam, (size_t)B * h->ng * sizeof(double), hipMemcpyDeviceToHost, s));
  if (status) HIPCHK(hipMemcpyAsync(status, h->d_status, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (iters) HIPCHK(hipMemcpyAsync(iters, h->d_iters, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (g_out) {  // constraint values at the solution (constraints kernel on the device)
    HIPCHK(mpcx::launch_constraints(a, h->d_w, h->d_g, s));
    HIPCHK(hipMemcpyAsync(g_out, h->d_g, (size_t)B * h->ng * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  return 0;
}

int mpcx_plant_step(mpcx_handle* h, int32_t B, const double* P, const double* u, double* xf, double* qf) {
  if (!h || !P || !u || !xf) return fail(MPCX_EINVAL, "null argument");
  if (B <= 0) return B == 0 ? 0 : fail(MPCX_EINVAL, "B < 0");
  if (int r = check_model_ready(h, B)) return r;
  DEVICE_SCOPE(h->spec.device);
  hipStream_t s = h->stream;
  const int nx = h->spec.nx, nu = h->spec.nu;
  if (int r = ensure(h, B)) return r;
  double *dP = h->d_P, *dU = h->d_u, *dX = h->d_x, *dQ = h->d_q;
  HIPCHK(hipMemcpyAsync(dP, P, (size_t)B * h->np * sizeof(double), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(dU, u, (size_t)B * nu * sizeof(double), hipMemcpyHostToDevice, s));
  mpcx::SolveArgs a = make_args(h, B, dP, nullptr, nullptr, nullptr, h->d_lbw, h->d_ubw, nullptr, nullptr, nullptr,
                                nullptr, nullptr, nullptr);
  HIPCHK(mpcx::launch_plant(a, dU, dX, dQ, s));
  HIPCHK(hipMemcpyAsync(xf, dX, (size_t)B * nx * sizeof(double), hipMemcpyDeviceToHost, s));
  if (qf) HIPCHK(hipMemcpyAsync(qf, dQ, (size_t)B * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int mpcx_shift_dev(mpcx_handle* h, int32_t B, double* d_P, const double* d_w, double* d_w0_next,
                   const double* d_lam_g, double* d_lam_g0_next, const double* d_lam_x, double* d_lam_x0_next,
                   void* stream) {
  if (!h || !d_P || !d_w || !d_w0_next) return fail(MPCX_EINVAL, "null argument");
  if (B <= 0) return B == 0 ? 0 : fail(MPCX_EINVAL, "B < 0");
  if ((d_lam_g == nullptr) != (d_lam_g0_next == nullptr) || (d_lam_x == nullptr) != (d_lam_x0_next == nullptr))
    return fail(MPCX_EINVAL, "multiplier shift needs both source and destination");
  if (int r = check_model_ready(h, B)) return r;
  DEVICE_SCOPE(h->spec.device);
  mpcx::SolveArgs a = make_args(h, B, d_P, nullptr, nullptr, nullptr, h->d_lbw, h->d_ubw, nullptr, nullptr, nullptr,
                                nullptr, nullptr, nullptr);
  HIPCHK(mpcx::launch_shift(a, d_P, d_w, d_w0_next, d_lam_g, d_lam_g0_next, d_lam_x, d_lam_x0_next,
                            (hipStream_t)stream));
  return 0;
}

int mpcx_rk4_sens_dev(mpcx_handle* h, int32_t B, const double* d_X, const double* d_U, const double* d_xr,
                      double* d_J, void* stream) {
  if (!h || !d_X || !d_U || !d_xr || !d_J) return fail(MPCX_EINVAL, "null argument");
  if (B <= 0) return B == 0 ? 0 : fail(MPCX_EINVAL, "B < 0");
  if (h->spec.model != MPCX_MODEL_UNICYCLE || h->spec.param_layout != MPCX_P_X0_XREF)
    return fail(MPCX_EINVAL, "rk4_sens_dev: unicycle model with param_layout X0_XREF only");
  DEVICE_SCOPE(h->spec.device);
  HIPCHK(mpcx::launch_rk4_sens(B, h->spec.N, stage_params(h->spec), d_X, d_U, d_xr, d_J, (hipStream_t)stream));
  return 0;
}

int mpcx_rk4_sens(mpcx_handle* h, int32_t B, const double* w, const double* P, double* c, double* q, double* A,
                  double* Bm, double* gq) {
  if (!h || !w || !P || !c || !q || !A || !Bm || !gq) return fail(MPCX_EINVAL, "null argument");
  if (B <= 0) return B == 0 ? 0 : fail(MPCX_EINVAL, "B < 0");
  if (h->spec.model != MPCX_MODEL_UNICYCLE || h->spec.param_layout != MPCX_P_X0_XREF)
    return fail(MPCX_EINVAL, "rk4_sens: unicycle model with param_layout X0_XREF only");
  DEVICE_SCOPE(h->spec.device);
  const int N = h->spec.N;
  const long T = ((long)B + 63) / 64, Bp = T * 64;  // 64-instance tiles (mpcx_rk4_sens_dev layout)
  auto tix = [T](int stage, int F, int i, long b) {
    return (((size_t)stage * T + (b >> 6)) * F + i) * 64 + (b & 63);
  };
  // d_J record: field f of (stage, instance) in the 16-B field-pair layout
  auto jix = [T](int stage, int f, long b) {
    return ((((size_t)stage * T + (b >> 6)) * 12 + (f >> 1)) * 64 + (b & 63)) * 2 + (f & 1);
  };
  const size_t nX = (size_t)(N + 1) * 3 * Bp, nU = (size_t)N * 2 * Bp, nR = (size_t)3 * Bp;
  const size_t nJ = (size_t)N * 24 * Bp;
  const size_t total = nX + nU + nR + nJ;
  if (total > h->cap_sweep) {
    (void)hipFree(h->d_sweep);
    h->d_sweep = nullptr;
    h->cap_sweep = 0;
    HIPCHK(hipMalloc(&h->d_sweep, total * sizeof(double)));
    h->cap_sweep = total;
  }
  std::vector<double> hX(nX, 0.0), hU(nU, 0.0), hR(nR, 0.0);
  for (int b = 0; b < B; ++b) {
    const double* wb = w + (size_t)b * h->nw;
    for (int k = 0; k <= N; ++k)
      for (int i = 0; i < 3; ++i) hX[tix(k, 3, i, b)] = k == 0 ? wb[i] : wb[3 + 5 * (k - 1) + 2 + i];
    for (int k = 0; k < N; ++k)
      for (int i = 0; i < 2; ++i) hU[tix(k, 2, i, b)] = wb[3 + 5 * k + i];
    for (int i = 0; i < 3; ++i) hR[tix(0, 3, i, b)] = P[(size_t)b * h->np + 3 + i];
  }
  double* d = h->d_sweep;
  double *dX = d, *dU = dX + nX, *dR = dU + nU, *dJ = dR + nR;
  hipStream_t s = h->stream;
  HIPCHK(hipMemcpyAsync(dX, hX.data(), nX * sizeof(double), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(dU, hU.data(), nU * sizeof(double), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(dR, hR.data(), nR * sizeof(double), hipMemcpyHostToDevice, s));
  HIPCHK(mpcx::launch_rk4_sens(B, N, stage_params(h->spec), dX, dU, dR, dJ, s));
  std::vector<double> hJ(nJ);
  HIPCHK(hipMemcpyAsync(hJ.data(), dJ, nJ * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < N; ++k) {
      const size_t o = (size_t)b * N + k;
      for (int i = 0; i < 3; ++i) c[o * 3 + i] = hJ[jix(k, i, b)];
      q[o] = hJ[jix(k, 3, b)];
      for (int i = 0; i < 9; ++i) A[o * 9 + i] = hJ[jix(k, 4 + i, b)];
      for (int i = 0; i < 6; ++i) Bm[o * 6 + i] = hJ[jix(k, 13 + i, b)];
      for (int i = 0; i < 5; ++i) gq[o * 5 + i] = hJ[jix(k, 19 + i, b)];
    }
  return 0;
}

}  // extern "C"
