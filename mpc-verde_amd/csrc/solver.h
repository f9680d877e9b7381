// solver.h -- device-side launch interface shared by solver.hip and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "unicycle.h"

namespace mpcx {

// Tables of the linear model (MPCX_MODEL_LINEAR), device memory owned by the handle.
struct LinTables {
  const double* A;    // n_tab x NX*NX (row-major)
  const double* B;    // n_tab x NX*NU
  const double* c;    // n_tab x NX
  const double* W;    // n_tab x NZ(NZ+1)/2 (packed upper triangle, z = (x, u))
  const int32_t* tab; // N (shared) or rows x N (per instance) table indices
  int per_instance;
  int n_tab;
  // bit j (j < 64): table j is decoupled -- B_j == 0 and no x-u block in W_j (exact zeros) --
  // so a suffix of such stages keeps P_k across iterations (solver.hip, decoupled suffix)
  unsigned long long dec_mask;
};

// Constants of the nonlinear ODE models (ode.h): RK4 substep, node-cost weights, model constants.
struct OdeParams {
  double h;  // T / M
  int M;
  double Q[8], R[8], par[8];
};

struct SolveArgs {
  int B, N, max_iter, p_layout;
  int p_stride;
  int model, nx, nu;
  int n_simd;           // SIMDs of the device (0 = unknown): lane groups widen to fill them
  int group_policy;     // mpcx_spec.group_policy
  double tol;
  // IPOPT termination options (mpcx_spec, defaults resolved by the host)
  double dual_inf_tol, constr_viol_tol, compl_inf_tol;
  double acc_tol, acc_dual_inf_tol, acc_constr_viol_tol, acc_compl_inf_tol, acc_obj_change_tol;
  int acc_iter;         // <= 0: no acceptable-level termination
  int restoration;      // soft restoration + restoration phase on a failed line search (models with kResto)
  int xbnd;             // 1: some node has a finite state bound in lbw/ubw (picks the kernel variant)
  double* ws;           // restoration workspace: slot i of thread t at ws[i * ws_stride + t] (kResto models)
  long ws_stride;
  // park flag (after the workspace): the solve launch stores park_epoch there when it parks an
  // instance; a resume launch that finds another value returns at once (nothing to resume)
  double* park_flag;
  double park_epoch;
  // linear models with a decoupled suffix: P_k of the suffix stages as a launch of this handle
  // computed them at fs = 1, delta = 0 ((N + 1) x NP doubles, then the header {launch epoch,
  // table generation, kb}), or null; pc_epoch = this launch (> every earlier one), pc_gen = the
  // tables' generation (bumped by every table or schedule change)
  double* pcache;
  double pc_epoch, pc_gen;
  StageParams sp;       // unicycle constants
  LinTables lin;        // linear model tables
  OdeParams op;         // nonlinear ODE models
  const double* P;      // B x p_stride (device)
  const double* w0;     // B x nw or null (cold start: X_k = x0, U = 0)
  const double* lam0;   // B x ng initial constraint multipliers or null
  const double* lamx0;  // B x nw initial bound multipliers (zU - zL) or null
  int warm;             // 1: IPOPT warm_start_init_point (multipliers given)
  double mu_init, bound_push, mult_push;
  const double* lbw;    // nw (device)
  const double* ubw;    // nw
  double* w_out;        // B x nw
  double* f_out;        // B or null
  double* lam_out;      // B x ng or null
  double* lamx_out;     // B x nw or null
  int32_t* status;      // B or null
  int32_t* iters;       // B or null
  // fused receding-horizon update (mpcx_step_dev): written after the solve, in place
  // allowed (every slot is read and written by the same lane).  Null = no update.
  double* P_next;       // B x p_stride: x0 <- F(x0, u_0*)
  double* w0_next;      // B x nw: solution shifted one interval
  double* lam0_next;    // B x ng or null
  double* lamx0_next;   // B x nw or null
  // multi-step launches (mpcx_run_dev): `steps` closed-loop steps per instance in one
  // launch, each instance advancing on its own; status/iters are steps x B.
  int steps;             // <= 1: a single solve
  int warm_next;         // steps >= 1 start from shifted multipliers (1) or primal only (0)
  const double* Pseq;    // steps x B x p_stride stage references per step (x0 part unused) or null
  const int32_t* tabseq; // steps x B x N linear-model schedule per step or null
};

// What a stage model reads (a local copy: taking the address of the kernel argument
// struct itself would force it onto the scratch stack).
struct ModelArgs {
  StageParams sp;
  LinTables lin;
  OdeParams op;
  int p_layout, N;
  double* tc = nullptr;  // ODE models: this lane's slot 0 of the solve kernel's LDS value cache
  int tc_stride = 0;     // slot stride (threads per block)
};
__host__ __device__ inline ModelArgs model_args(const SolveArgs& a) { return ModelArgs{a.sp, a.lin, a.op, a.p_layout, a.N}; }

// lane group of the solve launch: the smallest power of two holding nodes 0..N; a batch too
// small to give every SIMD a wave gets wider groups (up to one instance per wave) unless
// group_policy = 1.  G > 64 spans G/64 waves (one workgroup per instance).
inline int solve_group_size(int N, long B, int n_simd, int group_policy) {
  int G = N < 16 ? 16 : N < 32 ? 32 : N < 64 ? 64 : N < 128 ? 128 : 256;
  if (group_policy == 0)
    while (G < 64 && B * G * 2 <= 64L * n_simd) G *= 2;
  return G;
}
// Restoration workspace (models with kResto; resto.h): the solve loop hands its iterate and
// Newton step to the out-of-line recovery through it and reads the result back.  Structure of
// arrays over threads: slot i of thread t at ws[i * ws_stride + t].  Per lane: z, lam, zL, zU,
// dz, dlam, dzL, dzU and x0 (lane 0's initial state).
struct RestoWs {
  static constexpr int XZ = 0;
  __host__ __device__ static constexpr int XL(int nz) { return nz; }
  __host__ __device__ static constexpr int XZL(int nx, int nz) { return nz + nx; }
  __host__ __device__ static constexpr int XZU(int nx, int nz) { return 2 * nz + nx; }
  __host__ __device__ static constexpr int XDZ(int nx, int nz) { return 3 * nz + nx; }
  __host__ __device__ static constexpr int XDL(int nx, int nz) { return 4 * nz + nx; }
  __host__ __device__ static constexpr int XDZL(int nx, int nz) { return 4 * nz + 2 * nx; }
  __host__ __device__ static constexpr int XDZU(int nx, int nz) { return 5 * nz + 2 * nx; }
  __host__ __device__ static constexpr int XX0(int nx, int nz) { return 6 * nz + 2 * nx; }
  // group scalars of the solve loop at the failed line search (the same value on every lane)
  enum Scalar {
    sPEND = 0,  // 1: the fast solve left this instance to the resume launch
    sFS, sMU, sTAU, sTHMAX, sTHMIN, sDWLAST, sFNEXT, sFN, sFREJ, sNFRESET, sACC, sFLAST,
    sSOFT, sSOFTN, sIT, sSTEP, sWARM, sTHK, sPHK, sGD, sAMAX, sAZ, sSWA, sACCNOW,
    sSOFTTRIED,  // 1: the solve loop already took (and failed) this iteration's soft restoration step
    sFTH,                                      // this lane's filter slots (FilterLds<G>::S of kFilterMax)
    sFPH = sFTH + 16, kScalars = sFPH + 16
  };
  static constexpr int kFilterMax = 16;
  __host__ __device__ static constexpr int SC(int nx, int nz) { return 6 * nz + 3 * nx; }
  __host__ __device__ static constexpr int slots(int nx, int nu) { return SC(nx, nx + nu) + kScalars; }
};
// workspace chain stash of the models with kWsStash (the 6-state bicycle, model 4): the stage
// Hessian (packed), Sigma, A and B of every lane, after the restoration slots, then the row chain's
// value function of the lane's node (rowchain6.h: P's columns and p, (nx + 1) nx doubles) and the
// iterate across the chain (z, zL, zU, bounds, lam)
__host__ __device__ constexpr int chain_ws_slots(int nx, int nu) {
  return (nx + nu) * (nx + nu + 1) / 2 + nx + nu + nx * nx + nx * nu + (nx + 1) * nx + 5 * (nx + nu) + nx;
}
// doubles of workspace per thread (restoration + chain stash; 0: the model uses none)
int resto_ws_slots(int model, int nx, int nu);

hipError_t launch_solve(const SolveArgs& a, hipStream_t stream);
// the solve kernel a launch with these arguments runs: G lanes per group, R replicas of the group per
// wave, and the instantiation's model type ("mpcx::UnicycleFreeModel", ...)
hipError_t solve_shape(const SolveArgs& a, int* G, int* R, const char** kname);
// the resume launch of models with a restoration phase: continues the instances the solve
// launch left at a failed line search (no-op for the others)
hipError_t launch_resume(const SolveArgs& a, hipStream_t stream);
hipError_t launch_rk4_sens(int B, int N, const StageParams& sp, const double* X, const double* U, const double* XR,
                           double* J, hipStream_t stream);
// plant: x+ = F(x0, u) for B instances (stage-0 model of each instance)
hipError_t launch_plant(const SolveArgs& a, const double* U, double* XF, double* QF, hipStream_t stream);
// closed-loop shift (plant + shifted warm start of primal and multipliers)
// constraint values g (B x ng) at w
hipError_t launch_constraints(const SolveArgs& a, const double* W, double* Gout, hipStream_t stream);
hipError_t launch_shift(const SolveArgs& a, double* P, const double* W, double* W0, const double* L, double* L0,
                        const double* LX, double* LX0, hipStream_t stream);

}  // namespace mpcx
