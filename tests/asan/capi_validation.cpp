// capi_validation.cpp -- host-only driver of libmpcx's C ABI argument checking, built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host code (tests/asan/Makefile) and run
// by tests/test_asan.py on a machine with or without a GPU.  It walks every path of
// include/mpcx.h that must fail before touching a device: default specs of every model id (valid
// and invalid), mpcx_create on each kind of invalid spec, every entry point with a null handle or
// null/negative arguments, mpcx_destroy(NULL), mpcx_last_error, mpcx_source_hash.  A valid spec
// is created only when a HIP device is present.  Exit status 0 = every check behaved.
#include <cmath>
#include <cstdio>
#include <cstring>

#include "mpcx.h"

static int failures = 0;
#define EXPECT(c)                                                          \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

int main() {
  mpcx_spec s;
  EXPECT(mpcx_default_spec(nullptr, MPCX_MODEL_UNICYCLE, 20) < 0);
  EXPECT(std::strlen(mpcx_last_error()) > 0);
  for (int model : {MPCX_MODEL_UNICYCLE, MPCX_MODEL_KIN_BICYCLE, MPCX_MODEL_DYN_BICYCLE, MPCX_MODEL_CARTPOLE})
    EXPECT(mpcx_default_spec(&s, model, 30) == 0);
  for (int bad : {-1, 0, 2, 6, 99}) EXPECT(mpcx_default_spec(&s, bad, 30) < 0);
  EXPECT(std::strlen(mpcx_source_hash()) > 0);

  // invalid specs are refused before any device call
  mpcx_handle* h = nullptr;
  EXPECT(mpcx_create(nullptr, &h) < 0);
  mpcx_default_spec(&s, MPCX_MODEL_UNICYCLE, 20);
  EXPECT(mpcx_create(&s, nullptr) < 0);
  auto refused = [&](void (*edit)(mpcx_spec&)) {
    mpcx_spec t;
    mpcx_default_spec(&t, MPCX_MODEL_UNICYCLE, 20);
    edit(t);
    mpcx_handle* hh = nullptr;
    const int r = mpcx_create(&t, &hh);
    EXPECT(r < 0 && hh == nullptr);
    EXPECT(std::strlen(mpcx_last_error()) > 0);
  };
  refused([](mpcx_spec& t) { t.model = 42; });
  refused([](mpcx_spec& t) { t.N = 0; });
  refused([](mpcx_spec& t) { t.N = 256; });
  refused([](mpcx_spec& t) { t.M = 0; });
  refused([](mpcx_spec& t) { t.M = 65; });
  refused([](mpcx_spec& t) { t.T = 0.0; });
  refused([](mpcx_spec& t) { t.T = NAN; });
  refused([](mpcx_spec& t) { t.cost = 7; });
  refused([](mpcx_spec& t) { t.param_layout = 7; });
  refused([](mpcx_spec& t) { t.max_iter = -1; });
  refused([](mpcx_spec& t) { t.group_policy = 2; });
  refused([](mpcx_spec& t) { t.tol = 0.0; });
  refused([](mpcx_spec& t) { t.tol = NAN; });
  refused([](mpcx_spec& t) { t.dual_inf_tol = -1.0; });
  refused([](mpcx_spec& t) { t.acceptable_tol = NAN; });
  refused([](mpcx_spec& t) { t.acceptable_obj_change_tol = NAN; });
  refused([](mpcx_spec& t) { t.acceptable_iter = -2; });
  refused([](mpcx_spec& t) { t.no_restoration = 3; });
  refused([](mpcx_spec& t) { t.warm_mu_init = 0.0; });
  refused([](mpcx_spec& t) { t.lbu[0] = t.ubu[0]; });
  refused([](mpcx_spec& t) { t.lbx[1] = 5.0; t.ubx[1] = 4.0; });
  refused([](mpcx_spec& t) { t.device = -1; });
  refused([](mpcx_spec& t) { t.model = MPCX_MODEL_LINEAR; t.nx = 7; t.nu = 3; });
  refused([](mpcx_spec& t) { t.model = MPCX_MODEL_LINEAR; t.nx = 4; t.nu = 1; t.param_layout = MPCX_P_X0_XREF; });
  refused([](mpcx_spec& t) { t.model = MPCX_MODEL_DYN_BICYCLE; t.cost = MPCX_COST_QUADRATURE; });

  // every entry point with a null handle or null arguments fails without a dereference
  double d[64] = {0};
  int32_t i32[16] = {0};
  EXPECT(mpcx_solve_batch(nullptr, 1, d, nullptr, nullptr, nullptr, nullptr, nullptr, d, nullptr, nullptr, nullptr,
                          nullptr, nullptr, nullptr) < 0);
  EXPECT(mpcx_solve_batch_dev(nullptr, 1, d, nullptr, nullptr, nullptr, d, nullptr, nullptr, nullptr, nullptr,
                              nullptr, nullptr) < 0);
  EXPECT(mpcx_step_dev(nullptr, 1, d, d, nullptr, nullptr, 0, d, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr) < 0);
  EXPECT(mpcx_run_dev(nullptr, 1, 2, d, d, nullptr, nullptr, 0, nullptr, nullptr, d, nullptr, nullptr, nullptr, i32,
                      i32, nullptr) < 0);
  EXPECT(mpcx_shift_dev(nullptr, 1, d, d, d, nullptr, nullptr, nullptr, nullptr, nullptr) < 0);
  EXPECT(mpcx_plant_step(nullptr, 1, d, d, d, nullptr) < 0);
  EXPECT(mpcx_rk4_sens(nullptr, 1, d, d, d, d, d, d, d) < 0);
  EXPECT(mpcx_rk4_sens_dev(nullptr, 1, d, d, d, d, nullptr) < 0);
  EXPECT(mpcx_set_linear_model(nullptr, 1, d, d, d, d, i32, 1) < 0);
  EXPECT(mpcx_set_linear_tab_dev(nullptr, i32, 1) < 0);
  int32_t nw, ng, np;
  EXPECT(mpcx_dims(nullptr, &nw, &ng, &np) < 0);
  int32_t lanes, reps;
  char kname[256];
  EXPECT(mpcx_launch_shape(nullptr, 16, &lanes, &reps, kname, (int32_t)sizeof(kname)) < 0);
  mpcx_destroy(nullptr);

  // a valid spec: created where a device exists, refused with a HIP error elsewhere
  mpcx_default_spec(&s, MPCX_MODEL_UNICYCLE, 20);
  const int rc = mpcx_create(&s, &h);
  if (rc == 0) {
    EXPECT(mpcx_dims(h, &nw, &ng, &np) == 0 && nw == 103 && ng == 63 && np == 6);
    EXPECT(mpcx_solve_batch(h, -1, d, nullptr, nullptr, nullptr, nullptr, nullptr, d, nullptr, nullptr, nullptr,
                            nullptr, nullptr, nullptr) < 0);
    EXPECT(mpcx_solve_batch(h, 0, d, nullptr, nullptr, nullptr, nullptr, nullptr, d, nullptr, nullptr, nullptr,
                            nullptr, nullptr, nullptr) == 0);
    EXPECT(mpcx_set_linear_model(h, 1, d, d, d, d, i32, 1) < 0);  // not a linear handle
    EXPECT(mpcx_launch_shape(h, 0, &lanes, &reps, kname, (int32_t)sizeof(kname)) < 0);
    EXPECT(mpcx_launch_shape(h, 16, &lanes, &reps, kname, 8) < 0);  // name buffer too small
    EXPECT(mpcx_launch_shape(h, 16, &lanes, &reps, kname, (int32_t)sizeof(kname)) == 0 && lanes >= 32 &&
           std::strstr(kname, "solve_kernel<mpcx::UnicycleFreeModel") != nullptr);
    mpcx_destroy(h);
    std::printf("device present: handle created and destroyed\n");
  } else {
    EXPECT(h == nullptr);
    std::printf("no device: %s\n", mpcx_last_error());
  }
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "capi validation clean", failures);
  return failures ? 1 : 0;
}
