/* mpcx.h -- C ABI of the MI355X-native batched multiple-shooting MPC solver.
 *
 * The drop-in boundary for the hot path of gabrielhaj/mpc-verde.  Every entry
 * point replaces one call site of the reference's CasADi boundary (paths
 * relative to the reference repository):
 *
 *   mpcx_create         ca.nlpsol('solver', 'ipopt', prob, opts)
 *                         Casadi/multiple_shooting_casadi.py:181-197
 *                         (problem = the NLP built at :68-178; options :188-196)
 *   mpcx_solve_batch    sol = solver(x0=, lbx=, ubx=, lbg=, ubg=, p=)
 *                         Casadi/multiple_shooting_casadi.py:235-242, batched
 *                         over B independent parameter vectors p
 *   mpcx_plant_step     state_init = F(args['p'], u[:, 0])[0]
 *                         Casadi/multiple_shooting_casadi.py:273 (F built at :98-114)
 *   mpcx_rk4_sens       the function + derivative evaluations IPOPT requests from
 *                         CasADi inside solver() (F and its AD, :157 / :197):
 *                         kernel-level entry of the RK4 + Jacobian sweep
 *   mpcx_destroy        (Python garbage collection of the solver object)
 *   mpcx_last_error     (CasADi raises RuntimeError; here: message of the last
 *                         failing call on this thread)
 *
 * Conventions.  All arithmetic is IEEE fp64.  Pointers named d_* are device
 * pointers (hipMalloc'ed or torch CUDA tensors); everything else is host memory.
 * Functions return 0 on success and a negative mpcx_err code on error.  Host
 * calls are synchronous.  A handle is owned by one host thread at a time.
 *
 * Decision-vector layout = the reference's interleaved w (:128-170):
 *   w = [X_0(nx) | U_0(nu) X_1(nx) | ... | U_{N-1}(nu) X_N(nx)],  n_w = nx + N(nu+nx)
 * Constraint layout (:131,:172-175), all equalities (lbg = ubg = 0):
 *   g = [P[:nx] - X_0 ; F(X_k,U_k).xf - X_{k+1}  (k = 0..N-1)],  n_g = nx (N+1)
 */
#ifndef MPCX_H_
#define MPCX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mpcx_handle mpcx_handle;

enum mpcx_model {
  MPCX_MODEL_UNICYCLE = 1, /* x=(x,y,theta), u=(v,omega): Casadi/multiple_shooting_casadi.py:68-72 */
  /* x+ = A_j x + B_j u + c_j, l = (z - zr_k)^T W_j (z - zr_k), z = (x, u): the mpctools
     LTI/LTV QPs (Inverted_pendulum/inverted_pendulum_single_shooting_mpctools.py:19-64,
     Trajectory Tracking/Trajectory_tracking_dynamic_model.py:117-145); tables set with
     mpcx_set_linear_model.  (nx, nu) in {(4,1), (5,1), (4,2)}; smaller models
     embed with zero pad states (mpcx/lti.py StatePad). */
  MPCX_MODEL_LINEAR = 2,
  /* Nonlinear ODE models (BASELINE config variants; parity against the CPU oracle only),
     RK4 with M substeps, node cost l = sum Q_i (x_i - xr_i)^2 + sum R_j (u_j - ur_j)^2,
     exact derivatives (mpc-verde_amd/csrc/ode.h).  Constants in mpcx_spec.par. */
  MPCX_MODEL_KIN_BICYCLE = 3, /* x=(X,Y,psi), u=(v,delta); par = (L) */
  MPCX_MODEL_DYN_BICYCLE = 4, /* x=(X,Y,psi,vx,vy,r), u=(delta,ax), linear tyres; par = (m,a,b,Ca,Jz):
                                 the nonlinear parent of Trajectory_tracking_dynamic_model.py:119-128 */
  MPCX_MODEL_CARTPOLE = 5     /* x=(p,p',phi,phi'), u=F; par = (M,m,L,g,c): the nonlinear parent of
                                 inverted_pendulum_single_shooting_mpctools.py:19-23 */
};

enum mpcx_cost {
  /* J = sum_k RK4 quadrature of L over [t_k, t_k+T] (Casadi/multiple_shooting_casadi.py:98-113) */
  MPCX_COST_QUADRATURE = 0,
  /* J = sum_k l(x_k, u_k, p_k) at the shooting nodes (mpctools nmpc;
     Trajectory Tracking/Trajectory_tracking.py:57-61) */
  MPCX_COST_NODE = 1
};

enum mpcx_param_layout {
  /* p = [x0 (nx); x_ref (nx)]  (n_p = 2 nx, Casadi/multiple_shooting_casadi.py:74,228-231) */
  MPCX_P_X0_XREF = 0,
  /* p = [x0 (nx); (x_ref_k, u_ref_k) for k = 0..N-1]  (n_p = nx + N (nx+nu);
     Trajectory Tracking/Trajectory_tracking.py:84-97,105-106).  Always used by
     MPCX_MODEL_LINEAR (z_ref_k = (x_ref_k, u_ref_k)). */
  MPCX_P_X0_STAGEREF = 1
};

enum mpcx_status {
  MPCX_CONVERGED = 0,   /* optimality error <= tol and the unscaled tests hold (IPOPT "Solve_Succeeded") */
  MPCX_ACCEPTABLE = 1,  /* acceptable level for acceptable_iter iterations, or an acceptable point at a
                           failed line search ("Solved_To_Acceptable_Level") */
  MPCX_MAX_ITER = 2,    /* iteration limit reached */
  MPCX_FAILED = 3,      /* line search failed and could not be recovered ("Restoration_Failed") */
  MPCX_INFEASIBLE = 4,  /* the restoration phase converged to a point of local infeasibility
                           ("Infeasible_Problem_Detected") */
  MPCX_STEP_FAILED = 5  /* inertia correction failed ("Error_In_Step_Computation") */
};

enum mpcx_err {
  MPCX_OK = 0,
  MPCX_EINVAL = -1,  /* bad argument (message via mpcx_last_error) */
  MPCX_EHIP = -2,    /* HIP runtime error */
  MPCX_ENOMEM = -3
};

typedef struct mpcx_spec {
  int32_t model;        /* mpcx_model */
  int32_t cost;         /* mpcx_cost */
  int32_t param_layout; /* mpcx_param_layout */
  int32_t N;            /* horizon (intervals), 1..255 (N >= 64: one workgroup of 128/256 lanes per instance) */
  int32_t M;            /* RK4 substeps per interval (M at :101; mpctools M at Trajectory_tracking.py:51) */
  int32_t max_iter;     /* IPOPT max_iter (:190) */
  int32_t device;       /* HIP device ordinal */
  int32_t group_policy; /* lanes per instance: 0 = widen (up to 64) while the batch leaves SIMDs idle,
                           1 = the smallest power of two >= N+1 (the same bits either way; see
                           mpcx_launch_shape) */
  double T;             /* sampling time (:31) */
  double tol;           /* IPOPT tol (default 1e-8) */
  double Q[8];          /* diagonal state weights (:78-83) */
  double R[8];          /* diagonal control weights (:81-84) */
  double lbu[8], ubu[8];/* control bounds (:42-45) */
  double lbx[8], ubx[8];/* state bounds (+-1e20 = free; Trajectory_tracking.py:64-67) */
  /* Warm start (IPOPT warm_start_init_point = yes), used when multipliers are
     passed in (lam_g0 / lam_x0 != NULL): initial barrier parameter, primal bound
     push and bound-multiplier push.  Defaults 1e-4. */
  double warm_mu_init, warm_bound_push, warm_mult_push;
  int32_t nx, nu;       /* state / control dimensions (unicycle: 3, 2) */
  double par[8];        /* model constants of the ODE models (see mpcx_model) */
  /* IPOPT termination and recovery options (IPOPT's names and semantics; the reference passes
     max_iter, acceptable_tol = 1e-8 and acceptable_obj_change_tol = 1e-6 at
     Casadi/multiple_shooting_casadi.py:188-196).  A field left 0 takes IPOPT's default:
     dual_inf_tol 1, constr_viol_tol 1e-4, compl_inf_tol 1e-4 (unscaled tests next to tol),
     acceptable_tol 1e-6, acceptable_dual_inf_tol 1e10, acceptable_constr_viol_tol 1e-2,
     acceptable_compl_inf_tol 1e-2, acceptable_obj_change_tol 1e20, acceptable_iter 15 (-1
     disables the acceptable-level termination).  IPOPT's literal acceptable_obj_change_tol = 0
     is expressed as the smallest positive double (4.9e-324, the same test); a negative value
     also selects the default.  mpcx_default_spec fills every field: the unicycle gets
     the reference script's acceptable_tol 1e-8 / acceptable_obj_change_tol 1e-6 (the problem of
     :181-197 as the script builds it), the ODE models IPOPT's defaults.  (mpcx.nlpsol without
     options uses IPOPT's defaults for every model, as ca.nlpsol without options does.)
     ABI change (round 4): acceptable_obj_change_tol = 0 used to be taken literally; it now
     selects the default like every other 0 field (write 4.9e-324 for IPOPT's literal 0). */
  double dual_inf_tol, constr_viol_tol, compl_inf_tol;
  double acceptable_tol, acceptable_dual_inf_tol, acceptable_constr_viol_tol, acceptable_compl_inf_tol;
  double acceptable_obj_change_tol;
  int32_t acceptable_iter;
  /* 0: a failed line search enters IPOPT's soft restoration and then the feasibility
     restoration phase (models that have one: the ODE models); 1: the solve ends there
     (MPCX_FAILED unless the point is acceptable) */
  int32_t no_restoration;
} mpcx_spec;

/* Fill *s with the reference's constants for model/cost at horizon N
   (unicycle point-to-point: T=0.2, M=4, Q=diag(1,5,0.1), R=diag(0.5,0.05),
   |v|<=1, |omega|<=pi/4, max_iter=2000, tol=1e-8).  ODE models: node cost, M=1,
   param_layout MPCX_P_X0_STAGEREF (cart-pole: MPCX_P_X0_XREF), the constants listed
   at mpcx_model and the defaults of mpcx/ode.py. */
int mpcx_default_spec(mpcx_spec* s, int32_t model, int32_t N);

int mpcx_create(const mpcx_spec* s, mpcx_handle** h);
void mpcx_destroy(mpcx_handle* h);
const char* mpcx_last_error(void);
/* Build identity: a hash of the sources the library was compiled from (no reference
   counterpart; mpcx/_lib.py refuses a libmpcx.so whose hash differs from the tree's). */
const char* mpcx_source_hash(void);

/* Tables of an MPCX_MODEL_LINEAR handle (host pointers, copied to the device):
 *   A n_tab x nx x nx, B n_tab x nx x nu, c n_tab x nx (may be NULL = 0),
 *   W n_tab x nz(nz+1)/2 packed upper triangle of the stage weight (nz = nx+nu),
 *   tab tab_rows x N int32 table index of each stage; tab_rows = 1 (shared by all
 *   instances) or >= the batch size (row b = instance b; LTV schedules).
 * Call before solving; may be called again (e.g. per closed-loop step).
 * Reproducibility: with shared tables whose stages end in a decoupled suffix (B = 0, no x-u
 * weight; the move-blocked cart-pole QP), a launch may find the suffix's value functions cached
 * by an earlier launch of this handle; a factorisation that computes them afresh is redone on the
 * path the cached ones take, so results are bit-identical whatever the cache state (fresh handle,
 * cached handle, a later step of a multi-step launch). */
int mpcx_set_linear_model(mpcx_handle* h, int32_t n_tab, const double* A, const double* B, const double* c,
                          const double* W, const int32_t* tab, int32_t tab_rows);

/* Device-resident stage schedule (LTV closed loops: advance the table index of every
 * instance on the device each step without re-uploading tables).  d_tab is a caller-owned
 * device array tab_rows x N int32 with the meaning of `tab` above; it must stay valid while
 * the handle solves.  Indices outside [0, n_tab) are clamped.  d_tab = NULL reverts to the
 * schedule given to mpcx_set_linear_model (which also clears this one). */
int mpcx_set_linear_tab_dev(mpcx_handle* h, const int32_t* d_tab, int32_t tab_rows);

/* n_w, n_g, n_p of the NLP described by the handle. */
int mpcx_dims(const mpcx_handle* h, int32_t* n_w, int32_t* n_g, int32_t* n_p);

/* Diagnostic environment knobs (A/B of two code paths; never needed in production):
 *   MPCX_DEC_SUFFIX=0           read by mpcx_set_linear_model: no decoupled-suffix reuse (the full Riccati
 *                               recursion at every factorisation; with it, config 5 at N >= 64 sums
 *                               the suffix's vector part in chain order: ~1e-12 relative, same
 *                               iteration counts)
 *   MPCX_UNICYCLE_SCAN_MIN_N=n  read once per process: the unicycle horizon from which the Riccati recursion runs as
 *                               the log-depth scan (default 25; 256 = never; ~1e-12 relative)
 *
 * The solve kernel a batch of B instances runs on this handle's device (no device work; no
 * reference counterpart -- it names what the profiler will show):
 *   lanes     lanes per instance group G (16, 32, 64, 128, 256; > 64 = one workgroup per instance)
 *   replicas  1, or 2 when a batch too small to give every SIMD a wave widens a 32-lane group to
 *             a wave and holds it twice, one replica per half-wave (group_policy 0)
 *   kernel    the kernel's demangled name as rocprofv3 prints it (may be NULL), e.g.
 *             "void mpcx::solve_kernel<mpcx::UnicycleFreeModel, 32, false, 2>(mpcx::SolveArgs)";
 *             kernel_len = buffer size (EINVAL if too small)
 * Batch-size dependence of the results: NONE.  Every group variant (narrow, widened, replicated,
 * multi-wave) gives an instance the same bits, whatever batch, group_policy or device (SIMD count)
 * it is solved with, so a global batch sharded over ranks returns what one device returns. */
int mpcx_launch_shape(const mpcx_handle* h, int32_t B, int32_t* lanes, int32_t* replicas, char* kernel,
                      int32_t kernel_len);

/* Batched NLP solve (host pointers, synchronous).
 *   P      B x n_p parameters (layout per spec.param_layout)
 *   w0     B x n_w initial guesses, or NULL = cold start (X_k = x0, U_k = 0: the
 *          feasible guess X0 = repmat(state_init), u0 = zeros that the script builds at
 *          :212-213; its own first solve passes the all-zero w0 of :118-169, which equals
 *          this guess for its state_init = 0, and later solves pass the shifted guess)
 *   lam_g0 B x n_g, lam_x0 B x n_w: initial multipliers (CasADi's lam_g0 /
 *          lam_x0 solver inputs), or NULL.  If either is given the solve starts
 *          as IPOPT's warm_start_init_point (spec.warm_*); otherwise as IPOPT's
 *          default (mu = 0.1, multipliers 0 / 1).
 *   lbw/ubw n_w bound vectors shared by the batch, or NULL = spec bounds
 *          (the reference's lbx/ubx, :199-206; X_0 is always free: it is
 *          pinned by the lifted constraint g_0 = x0 - X_0 and enters nothing else --
 *          interval 0 integrates from the parameter x0, F(x0=[P[:nx]; ...], p=U_0),
 *          as the script does at :125,157, so lam_g[0:nx] is 0 at a solution: exactly
 *          from a start without multipliers, to the dual tolerance from a warm one)
 *   w_out  B x n_w optimal decision vectors (interleaved reference layout)
 *   f_out  B objective values, or NULL
 *   g_out  B x n_g constraint values at w_out, or NULL
 *   lam_g  B x n_g constraint multipliers (CasADi sign convention), or NULL
 *   lam_x  B x n_w bound multipliers (CasADi convention: z_U - z_L), or NULL
 *   status B mpcx_status codes, or NULL
 *   iters  B iteration counts, or NULL                                        */
int mpcx_solve_batch(mpcx_handle* h, int32_t B, const double* P, const double* w0, const double* lam_g0,
                     const double* lam_x0, const double* lbw, const double* ubw, double* w_out, double* f_out,
                     double* g_out, double* lam_g, double* lam_x, int32_t* status, int32_t* iters);

/* Device-pointer variant: all work is enqueued on `stream` (a hipStream_t, NULL = default
   stream).  Any d_* except d_P and d_w_out may be NULL.  The handle owns scratch buffers that
   every launch of the handle uses (restoration workspace, cached suffix value functions), so a
   handle must not be used on two streams concurrently (one handle per stream, as per thread).
   The first call at a batch size larger than any before grows the restoration workspace: that
   call waits for the device to go idle (an earlier launch may still read the old buffer) and is
   therefore not capturable in a graph; later calls never synchronise. */
int mpcx_solve_batch_dev(mpcx_handle* h, int32_t B, const double* d_P, const double* d_w0, const double* d_lam_g0,
                         const double* d_lam_x0, double* d_w_out, double* d_f_out, double* d_lam_g,
                         double* d_lam_x, int32_t* d_status, int32_t* d_iters, void* stream);

/* Plant / integrator F (host): xf = F(x0, u).xf, qf = F(x0, u).qf for B
   instances; P as in mpcx_solve_batch (only x0 and the stage-0 reference are
   read), u B x nu.  qf may be NULL. */
int mpcx_plant_step(mpcx_handle* h, int32_t B, const double* P, const double* u, double* xf, double* qf);

/* Receding-horizon update on the device (one closed-loop step of
   Casadi/multiple_shooting_casadi.py:271-287): x0 <- F(x0, u_0*) in d_P, and
   d_w0_next = the optimal w shifted by one interval (last interval repeated).
   If d_lam_g / d_lam_x are given, the multipliers are shifted the same way into
   d_lam_g0_next / d_lam_x0_next (warm start of the next solve). */
int mpcx_shift_dev(mpcx_handle* h, int32_t B, double* d_P, const double* d_w, double* d_w0_next,
                   const double* d_lam_g, double* d_lam_g0_next, const double* d_lam_x, double* d_lam_x0_next,
                   void* stream);

/* One closed-loop step on the device in ONE kernel launch: the batched solve of
 * mpcx_solve_batch_dev followed, in the same kernel, by the receding-horizon update of
 * mpcx_shift_dev (identical results), written IN PLACE:
 *   d_P[:, 0:nx]  <- F(x0, u_0*)                      (plant, :273)
 *   d_w0          <- solution shifted by one interval  (warm start of the next step)
 *   d_lam_g0/d_lam_x0 <- multipliers shifted alike (may be NULL: not kept)
 * flags: MPCX_STEP_COLD -- ignore d_w0 / multipliers on input (cold start, see w0 above);
 *        MPCX_STEP_PRIMAL_ONLY -- warm primal start, default multiplier initialisation.
 * Otherwise the solve starts from d_w0 and (if given) the shifted multipliers as IPOPT's
 * warm_start_init_point.  Solution outputs as in mpcx_solve_batch_dev (d_w_out required). */
enum mpcx_step_flags { MPCX_STEP_COLD = 1, MPCX_STEP_PRIMAL_ONLY = 2 };
int mpcx_step_dev(mpcx_handle* h, int32_t B, double* d_P, double* d_w0, double* d_lam_g0, double* d_lam_x0,
                  int32_t flags, double* d_w_out, double* d_f_out, double* d_lam_g, double* d_lam_x,
                  int32_t* d_status, int32_t* d_iters, void* stream);

/* K closed-loop steps in ONE launch: every instance runs its own receding-horizon loop
 * (solve, plant, shift, warm restart -- exactly the sequence of K mpcx_step_dev calls, with
 * bit-identical results) without waiting for the other instances between steps; instances
 * are independent, so this changes no result, only how long the slowest solves hold the
 * batch.  Arguments as mpcx_step_dev, plus:
 *   K         number of steps (>= 1)
 *   d_Pseq    K x B x n_p stage references of every step (row s used from step s >= 1,
 *             the x0 columns are ignored; row 0 must match d_P) or NULL = d_P's for all
 *   d_tabseq  K x B x N linear-model schedules per step (row s from step s >= 1) or NULL
 *   d_status, d_iters  K x B (step-major).
 * On return d_P / d_w0 / d_lam_g0 / d_lam_x0 hold the state after step K (as after K
 * mpcx_step_dev calls) and d_w_out / d_f_out / d_lam_g / d_lam_x step K's solution. */
int mpcx_run_dev(mpcx_handle* h, int32_t B, int32_t K, double* d_P, double* d_w0, double* d_lam_g0, double* d_lam_x0,
                 int32_t flags, const double* d_Pseq, const int32_t* d_tabseq, double* d_w_out, double* d_f_out,
                 double* d_lam_g, double* d_lam_x, int32_t* d_status, int32_t* d_iters, void* stream);

/* RK4 + Jacobian sweep over B x N shooting intervals (host pointers).
 *   w      B x n_w decision vectors (interleaved layout)
 *   P      B x n_p parameters
 * Outputs, per instance b and interval k (row-major, k fastest after b):
 *   c      B x N x nx   defects F(X_k,U_k).xf - X_{k+1}
 *   q      B x N        F(X_k,U_k).qf
 *   A      B x N x nx x nx   dF.xf/dX_k
 *   Bm     B x N x nx x nu   dF.xf/dU_k
 *   gq     B x N x (nx+nu)   dF.qf/d(X_k,U_k)                               */
int mpcx_rk4_sens(mpcx_handle* h, int32_t B, const double* w, const double* P, double* c, double* q, double* A,
                  double* Bm, double* gq);

/* Device variant of the sweep on tiled structure-of-arrays buffers (the layout the
   kernel streams from HBM).  Instances are grouped in T = ceil(B/64)
   tiles of 64; an array with S stages and F fields per stage holds element
   (stage s, field i, instance b) at  ((s*T + b/64)*F + i)*64 + b%64  (size S*T*F*64):
 *   d_X  S=N+1, F=nx;  d_U  S=N, F=nu;  d_xr  S=1, F=nx          (inputs)
 *   d_J  S=N, 24 fields per interval: 0-2 c (defect), 3 q, 4-12 A (row-major),
 *        13-18 Bm (row-major), 19-23 gq (output), stored as 12 field PAIRS so that a lane
 *        writes 16 B: field f of (stage s, instance b) at
 *        (((s*T + b/64)*12 + f/2)*64 + b%64)*2 + f%2   (size N*T*24*64) */
int mpcx_rk4_sens_dev(mpcx_handle* h, int32_t B, const double* d_X, const double* d_U, const double* d_xr,
                      double* d_J, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MPCX_H_ */
