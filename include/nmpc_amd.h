/*
 * nmpc_amd.h -- C-ABI of the MI355X-native batched NMPC solve step.
 *
 * Drop-in boundary for the per-timestep NLP of devsonni/MPC-Implementation
 * (Python/NMPC_TT.py).  The reference builds the NLP symbolically and solves
 * one scenario per call:
 *
 *   solver = ca.nlpsol('solver', 'ipopt', nlp_prob, opts)      Python/NMPC_TT.py:267
 *   sol = solver(x0=, lbx=, ubx=, lbg=, ubg=, p=)              Python/NMPC_TT.py:358-365
 *   u = ca.reshape(sol['x'], n_controls, N)                    Python/NMPC_TT.py:367
 *   ff_value = ff(u, args['p'])                                Python/NMPC_TT.py:368
 *
 * This library replaces that pair with a handle created from a structured
 * problem description (nmpc_create <- nlpsol) and a batched call
 * (nmpc_solve_batch <- solver(...)), B independent scenarios per call, all
 * solved on one MI355X by hand-written HIP kernels (one wavefront per
 * scenario).  Plain pointers and sizes only.
 *
 * Layouts (match CasADi's DM column vectors / Function.map horzcat):
 *   x0, lbx, ubx, x_out, lam_x_out : nw x B column-major, nw = 6*N   (w = vec(U), U is 6 x N)
 *   lbg, ubg, g_out, lam_g_out     : ng x B column-major, ng = (5+n_obs)*(N+1)
 *   p                              : np x B column-major, p = [x0(8); xs(3); dynamic obstacle coords]
 *   X_out                          : 8*(N+1) x B column-major  (ff(u, p), Python/NMPC_TT.py:169)
 *   lam_p_out                      : np x B column-major, -grad_p (f + lam_g' g) at x_out
 *                                    (CasADi nlpsol's lam_p; nullable)
 * A leading dimension of 0 broadcasts one column to every scenario (bounds
 * are normally shared: Python/NMPC_TT.py:269-306).  +-inf (|b| >= 1e19)
 * means "no bound", as ca.inf does (Python/NMPC_TT.py:280-282).
 *
 * Errors: functions return 0 on success and a negative NMPC_E* code on
 * invalid arguments or a HIP failure; nmpc_last_error() gives the message.
 * Non-convergence is NOT an error (the reference never checks it):
 * it is reported per scenario in status[] with IPOPT's ApplicationReturnStatus
 * codes (Ipopt::Solve_Succeeded = 0, Solved_To_Acceptable_Level = 1,
 * Infeasible_Problem_Detected = 2, Search_Direction_Becomes_Too_Small = 3,
 * Maximum_Iterations_Exceeded = -1,
 * Restoration_Failed = -2, Error_In_Step_Computation = -3,
 * Invalid_Number_Detected = -13).
 *
 * Threading/ownership: a handle is not thread-safe (one per GPU/stream).  The
 * caller owns every buffer; nothing is retained past a call.  The handle owns
 * its device workspace, grown on demand.
 */
#ifndef NMPC_AMD_H
#define NMPC_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMPC_MAX_OBS 16
#define NMPC_MAX_N 63

enum {
  NMPC_OK = 0,
  NMPC_E_INVALID = -1, /* bad descriptor / argument */
  NMPC_E_HIP = -2,     /* HIP runtime failure */
  NMPC_E_NOMEM = -3    /* device allocation failed */
};

enum {
  NMPC_MODEL_UAV8G = 0, /* 8 states / 6 controls, Python/NMPC_TT.py:94-151; p = [x0(8); xs(3); ...] */
  NMPC_MODEL_UAV5 = 1   /* no gimbal: 5 states / 3 controls, distance cost, rows [z, theta] (+ obstacles),
                           MATLAB/Dynamic Obstacles/NMPC_TT.m:26-35,102-111,129-134; w = vec(U) with U
                           3 x N, p = [x0(5); xs(3); ...], X_out 5 x (N+1); w2 is ignored.
                           All entry points, including nmpc_shift_dev / nmpc_closed_loop_dev */
};

/* IPOPT options honoured by the solver (names and meaning as IPOPT's;
 * nmpc_default_options() fills IPOPT's defaults, the reference overrides
 * max_iter=100, acceptable_tol=1e-8, acceptable_obj_change_tol=1e-6 at
 * Python/NMPC_TT.py:257-265). */
typedef struct nmpc_options {
  int32_t max_iter, acceptable_iter, max_soc, max_soft_resto_iters;
  /* watchdog procedure of the backtracking line search (IPOPT defaults 10 and 3;
   * a trigger of 0 disables it) */
  int32_t watchdog_shortened_iter_trigger, watchdog_trial_iter_max;
  /* not an IPOPT option: 1 = Riccati factorisation and solves in fp32 (the fp32 leg of
   * BASELINE config 5's fp32-vs-fp64 sweep); the iterate, residuals, line search and
   * termination tests stay fp64.  0 (default) = fp64 throughout. */
  int32_t linear_solver_fp32, reserved0;
  double tol, acceptable_tol, acceptable_obj_change_tol, acceptable_dual_inf_tol;
  double acceptable_constr_viol_tol, acceptable_compl_inf_tol;
  double dual_inf_tol, constr_viol_tol, compl_inf_tol;
  double mu_init, kappa_mu, theta_mu, barrier_tol_factor, tau_min;
  double bound_push, bound_frac, slack_bound_push, slack_bound_frac, bound_relax_factor;
  double bound_mult_init_val, constr_mult_init_max;
  double nlp_scaling_max_gradient, nlp_scaling_min_value, kappa_d, kappa_sigma, s_max;
  double theta_max_fact, theta_min_fact, gamma_theta, gamma_phi, delta, s_theta, s_phi, eta_phi;
  double alpha_red_factor, alpha_min_frac, kappa_soc, obj_max_inc;
  double first_hessian_perturbation, min_hessian_perturbation, max_hessian_perturbation;
  double perturb_inc_fact_first, perturb_inc_fact, perturb_dec_fact;
  double tiny_step_tol, soft_resto_pderror_reduction_factor;
  /* feasibility restoration phase */
  double resto_penalty_parameter, resto_proximity_weight, required_infeasibility_reduction;
  double bound_mult_reset_threshold, constr_mult_reset_threshold;
} nmpc_options;

/* Structured replacement for the symbolic nlp_prob of Python/NMPC_TT.py:247-255. */
typedef struct nmpc_desc {
  int32_t model;    /* NMPC_MODEL_UAV8G */
  int32_t N;        /* horizon, 1..NMPC_MAX_N (reference: 15, Python/NMPC_TT.py:58) */
  int32_t np;       /* length of p, >= 11 */
  int32_t n_obs;    /* 0..NMPC_MAX_OBS obstacle rows per stage */
  double T;         /* Euler step (Python/NMPC_TT.py:57; 0.2 in 10_obstacles.py:95) */
  double w1, w2;    /* cost weights (Python/NMPC_TT.py:204-205) */
  double vfov, hfov;/* FOV angles (Python/NMPC_TT.py:201-202) */
  double obs_x[NMPC_MAX_OBS], obs_y[NMPC_MAX_OBS];
  double obs_rsum[NMPC_MAX_OBS];      /* UAV_r + obs_r (Python/NMPC_TT.py:230-231) */
  int32_t obs_x_pidx[NMPC_MAX_OBS];   /* -1 = constant, else index into p (dynamic obstacles) */
  int32_t obs_y_pidx[NMPC_MAX_OBS];
  nmpc_options opts;
  /* cost weights from p (batched weight sweep; the RL replay of
   * MATLAB/Race Track 1/MPC.m:1,127 rebuilds nlpsol per weight pair): index
   * into p, or -1 to use w1 / w2 above */
  int32_t w1_pidx, w2_pidx;
} nmpc_desc;

typedef struct nmpc_handle nmpc_handle;

/* Fill IPOPT's default option values. */
void nmpc_default_options(nmpc_options* opts);

/* Replaces ca.nlpsol('solver', 'ipopt', nlp_prob, opts) (Python/NMPC_TT.py:267).
 * Binds the current HIP device. */
int nmpc_create(const nmpc_desc* desc, nmpc_handle** out);
int nmpc_destroy(nmpc_handle* h);

/* Problem dimensions: nw = nu N, ng = (nb+n_obs)(N+1), np, nX = nx(N+1)
 * (gimbal model: nu = 6, nb = 5, nx = 8; no-gimbal model: nu = 3, nb = 2, nx = 5). */
int nmpc_dims(const nmpc_handle* h, int32_t* nw, int32_t* ng, int32_t* np, int32_t* nX);

/* Replaces sol = solver(x0=, lbx=, ubx=, lbg=, ubg=, p=) (Python/NMPC_TT.py:358-365)
 * for B scenarios at once.  HOST pointers; synchronous.  Output pointers other
 * than x_out may be NULL.
 * Bounds as IPOPT reads them: |b| >= 1e19 is no bound; lbx == ubx fixes a variable
 * (fixed_variable_treatment = make_parameter: held at the bound, no step, lam_x 0);
 * rows with lbg == ubg are IPOPT's equality constraints c(x) = g(x) - lbg = 0 (no slack,
 * no relaxation; augmented-system step with IPOPT's inertia test), up to 128
 * per scenario.  A batch with any equality row runs on the equality class (global rows,
 * any shape, ~850 KB of device workspace per scenario): this host-pointer entry point scans
 * the bounds on the host, allocates that workspace when the batch needs it and launches
 * the one class that applies.
 * lbx > ubx, more than 128 equality rows, or equality rows with the fp32 Riccati leg
 * report status -11 (IPOPT Invalid_Problem_Definition) for that scenario. */
int nmpc_solve_batch(nmpc_handle* h, int32_t B,
                     const double* x0, int64_t ld_x0,
                     const double* lbx, int64_t ld_lbx, const double* ubx, int64_t ld_ubx,
                     const double* lbg, int64_t ld_lbg, const double* ubg, int64_t ld_ubg,
                     const double* p, int64_t ld_p,
                     double* x_out, double* f_out, double* g_out,
                     double* lam_x_out, double* lam_g_out, double* lam_p_out, double* X_out,
                     int32_t* status, int32_t* iters);

/* Same with DEVICE pointers, enqueued on `stream` (hipStream_t; NULL = default
 * stream); returns without synchronising (no host round trip: once the handle's workspace
 * covers B, a call only enqueues kernels).  Outputs other than x_out may be NULL.
 * Equality rows: the bounds are scanned on the device and a device flag lets exactly one
 * of the problem's class and the equality class run.  The equality class needs its
 * workspace reserved for B scenarios beforehand (nmpc_reserve_eq); without it a batch that
 * has equality rows is not solved and every scenario reports NMPC_STATUS_EQ_UNRESERVED
 * (x_out and f NaN).  Batches without equality rows need no reservation. */
int nmpc_solve_batch_dev(nmpc_handle* h, int32_t B,
                         const double* x0, int64_t ld_x0,
                         const double* lbx, int64_t ld_lbx, const double* ubx, int64_t ld_ubx,
                         const double* lbg, int64_t ld_lbg, const double* ubg, int64_t ld_ubg,
                         const double* p, int64_t ld_p,
                         double* x_out, double* f_out, double* g_out,
                         double* lam_x_out, double* lam_g_out, double* lam_p_out, double* X_out,
                         int32_t* status, int32_t* iters, void* stream);

/* Per-scenario status of a device-pointer call (nmpc_solve_batch_dev, nmpc_closed_loop_dev)
 * whose batch has equality rows (lbg == ubg) while the equality class's workspace does not
 * cover B: the batch was not solved (IPOPT's Insufficient_Memory code).  Reserve first. */
#define NMPC_STATUS_EQ_UNRESERVED (-102)
/* Allocate the equality class's device workspace for B scenarios (synchronous, like any
 * allocation; a no-op when it already covers B or for the fp32 leg, whose equality rows
 * report -11).  The _dev entry points never allocate it themselves, so that they never
 * synchronise the host; nmpc_solve_batch allocates it on demand. */
int nmpc_reserve_eq(nmpc_handle* h, int32_t B);

/* Optional per-iteration trace (debugging / parity): when enabled, the next
 * solve records NMPC_TRACE_FIELDS doubles per iteration per scenario into a
 * device buffer readable with nmpc_read_trace (host pointer,
 * B x (max_iter+3) x NMPC_TRACE_FIELDS, row-major; the last two rows of each
 * scenario are reserved for diagnostic phase timers).  Row i (0 <= i <= max_iter) holds
 *   [0..7]  {iter, mu, f_scaled, theta, delta_w, alpha_pr, alpha_du, ls_trials}
 *           after iteration i+1 (ls_trials < 0: a restoration iteration; i < max_iter), and
 *   [8..11] the convergence check at iteration count i:
 *           {scaled NLP error, dual infeasibility / s_d, constraint violation,
 *            complementarity / s_c} (IpoptCalculatedQuantities::curr_nlp_error); a
 *           NEGATIVE (sign bit set) error marks the restoration NLP's own check
 *           (RestoIpoptNLP), which replaces the main check recorded at the same count. */
#define NMPC_TRACE_FIELDS 12
int nmpc_set_trace(nmpc_handle* h, int32_t enable);
int nmpc_read_trace(nmpc_handle* h, int32_t B, double* host_out);

/* Closed-loop shift (the caller side of the solve, Python/NMPC_TT.py:13-30),
 * on DEVICE pointers, enqueued on `stream`: for each scenario, x0 <- x0 + T f(x0,u0),
 * warm start u <- [u(:,2:N), u(:,N)], target xs <- xs + T [v cos, v sin, w].
 * p (np x B, ld_p) is updated in place (x0 = p[0:8], xs = p[8:11]); w_out
 * (nw x B) receives the shifted warm start; v_t, w_t (length B) are the target
 * speeds (Python/NMPC_TT.py:25).  No-gimbal model: x0 = p[0:5], xs = p[5:8],
 * 3 controls per stage (MATLAB/Dynamic Obstacles/shift1.m). */
int nmpc_shift_dev(nmpc_handle* h, int32_t B, double* p, int64_t ld_p,
                   const double* u_sol, double* w_out,
                   const double* v_t, const double* w_t, void* stream);

/* K closed-loop MPC steps for each of B scenarios in ONE device launch: the
 * reference's main loop (Python/NMPC_TT.py:348-402: solve at :358-365, then
 * shift_timestep at :382 / :13-30) with each scenario advancing on its own
 * wavefront, so no step waits for another scenario's slowest solve.  Step k
 * solves with x0 = w (warm start) and p, records x0 = p[0:8] (x_hist), the
 * applied control u0 = x[0:6] (u_hist), f, status and iterations, then applies
 * x0 <- x0 + T f(x0,u0), w <- [u(:,2:N), u(:,N)], xs <- xs + T [v cos, v sin, w]
 * with the target controls (v, w) = (v_t, w_t)[k*ld_tk + b*ld_tb] (the
 * scripts' con_t schedules: ld_tk = 1, ld_tb = 0 for one shared schedule;
 * ld_tk = 0 for constant controls), and records the FOV-centre error
 * |FOV(x0_{k+1}) - xs_k[0:2]| (Python/NMPC_TT.py:397-400,433-437) in fov_hist.
 * p_step (nullable, K x np with leading dimension ld_ps, shared by all
 * scenarios) is added to p[11:np] after step k: moving obstacles, e.g. the
 * +-1 m/step windows of MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230.
 * DEVICE pointers, enqueued on `stream`.
 *   p   : np x B (ld_p >= np), in/out (advanced K steps)
 *   w   : nw x B (ld nw), in: first warm start; out: the last step's shifted solution
 *   No-gimbal model: the same loop on [x0(5); xs(3)] and 3 controls per stage
 *   (MATLAB/Dynamic Obstacles/NMPC_TT.m:150-183, shift1.m); histories keep the
 *   widths below with absent gimbal entries 0, and the FOV centre of a camera
 *   without gimbal angles is the UAV's ground position (x, y).
 *   u_hist K x B x 6, x_hist K x B x 8, f_hist / fov_hist / status_hist /
 *   iters_hist K x B; each nullable.  Bounds as in nmpc_solve_batch_dev.
 *   order: nullable, B int32 (device): a permutation of 0..B-1 giving the order in
 *          which scenarios are dispatched to wavefronts (order[g] runs g-th).  Results
 *          do not depend on it.  Putting the longest expected chains first (e.g.
 *          sorted by the previous launch's iterations, nmpc_amd.schedule) keeps a
 *          long chain from starting after the first wave of slots has drained.
 *          Entries outside [0,B) are skipped; a duplicated or missing scenario leaves
 *          some scenario short of its K steps, which nmpc_closed_loop_info reports. */
int nmpc_closed_loop_dev(nmpc_handle* h, int32_t B, int32_t K,
                         const double* lbx, int64_t ld_lbx, const double* ubx, int64_t ld_ubx,
                         const double* lbg, int64_t ld_lbg, const double* ubg, int64_t ld_ubg,
                         double* p, int64_t ld_p, double* w,
                         const double* v_t, const double* w_t, int64_t ld_tk, int64_t ld_tb,
                         const double* p_step, int64_t ld_ps,
                         double* u_hist, double* x_hist, double* f_hist, double* fov_hist,
                         int32_t* status_hist, int32_t* iters_hist, const int32_t* order, void* stream);

/* Scheduling of the last nmpc_closed_loop_dev launch (any pointer may be NULL).  When
 * sched_err or steps_done is requested it first synchronises the stream that launch
 * was enqueued on (hipStreamSynchronize), so it is valid for non-blocking streams.
 *   policy: 0 = one workgroup per scenario running its K steps back to back (B <=
 *     resident waves, a device without exactly 8 XCDs, or NMPC_CLOSED_LOOP=static);
 *     1 = step queues: persistent waves claim (scenario, step) pairs whose previous step
 *     is done, lowest step first, each scenario pinned to one XCD.
 *   resident: waves the closed-loop kernel keeps resident (occupancy x CUs; 0 before
 *     the first launch).  waves: workgroups the last launch started.
 *   sched_err: bit 0 a wave gave up waiting for a published step, bit 1 a scenario did
 *     not complete its K steps (its unrun steps carry status and iterations
 *     NMPC_STATUS_NOT_RUN and NaN f / fov / u / x in the histories), bit 2 the batch has
 *     equality rows and the equality workspace was not reserved (nmpc_reserve_eq): no step
 *     ran, and they carry NMPC_STATUS_EQ_UNRESERVED instead.  0 on success.
 *   steps_done: closed-loop steps completed, counted per scenario by a check kernel
 *     after either policy's launch (must equal B*K; 64-bit). */
#define NMPC_STATUS_NOT_RUN (-1000)
int nmpc_closed_loop_info(nmpc_handle* h, int32_t* policy, int32_t* resident, int32_t* sched_err,
                          int32_t* waves, int64_t* steps_done);

const char* nmpc_last_error(void);

/* Diagnostics: with NMPC_STEP_TIMES set in the environment, nmpc_closed_loop_dev records
 * for every (step k, scenario b) the s_memrealtime stamps (100 MHz) at the start and end
 * of the step and the running wave with the step's shader-clock cycles (s_memtime):
 * XCC_ID | workgroup << 8 | cycles << 24, K x B x 3 uint64; this
 * copies the last launch's record to host_out (n >= 3 K B). */
int nmpc_closed_loop_times(nmpc_handle* h, uint64_t* host_out, int64_t n);

/* Hash of the source, header and compile flags the library was built from
 * (__graft_entry__.source_hash); tests compare it with the checked-out source. */
const char* nmpc_build_id(void);

/* Launch geometry / workspace of the last solve, for measurement. */
int nmpc_kernel_info(const nmpc_handle* h, int32_t* lds_bytes, int32_t* threads_per_scenario);

/* Device workspace the handle holds (bytes): the problem class's per-scenario
 * workspace, and the equality class's, which is allocated only by
 * nmpc_reserve_eq or by a host-pointer batch with equality rows (lbg == ubg) and is 0 until
 * then; per scenario: the class layouts' sizes (ws_per_scenario, wsE_per_scenario; nullable). */
int nmpc_memory_info(const nmpc_handle* h, int64_t* ws_bytes, int64_t* ws_eq_bytes, int64_t* ws_per_scenario,
                     int64_t* wsE_per_scenario);

#ifdef __cplusplus
}
#endif
#endif /* NMPC_AMD_H */
