// CPU RESTATEMENT -- TEST INFRASTRUCTURE AND CPU BASELINE ONLY, NOT THE PRODUCT.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
// library (oracle/libnmpc_cpu.so, built by oracle/Makefile); the product path
// (mpc-implementation_amd/) never does and has no CPU fallback.
//
// What this is: the compiled CPU solver of SURVEY.md section 7 step 4 / BASELINE.md
// plan (2) -- "CPU restatement, not CasADi".  It restates, in scalar C++ fp64,
//   * the per-timestep NLP of Python/NMPC_TT.py (Euler single-shooting rollout
//     :153-167, FOV cost :192-221, obstacle rows :234-244, plant/target shift
//     :13-30; the no-gimbal model of MATLAB/Dynamic Obstacles/NMPC_TT.m:26-38);
//   * the IPOPT algorithm the reference calls through ca.nlpsol (NMPC_TT.py:250-267)
//     exactly as oracle/nmpc_oracle.py::IpoptDense restates it (same options,
//     same control flow: scaling, bound push, least-squares multipliers, monotone
//     barrier update, inertia correction, filter line search with SOC, watchdog,
//     soft restoration, feasibility restoration, acceptable termination);
// with one difference in the linear algebra: the Newton step comes from a
// stage-wise Riccati recursion on the multiple-shooting structure (the
// algorithm the HIP kernel runs), not from the dense 6N x 6N Cholesky of the
// numpy oracle.  The two are equal in exact arithmetic (the inertia test is
// "every R~_k pivot positive" <=> the condensed matrix is positive definite);
// tests/test_cpu_restatement.py checks this library against the numpy oracle's
// golden closed-loop fixtures (status, iterations, x, f).
//
// Each function cites the oracle function it follows (oracle/nmpc_oracle.py),
// which in turn cites the reference file:line.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include <omp.h>

namespace {

constexpr double INF = 1e19;  // IPOPT nlp_{lower,upper}_bound_inf
constexpr double EPS = 2.220446049250313e-16;
constexpr double PINF = HUGE_VAL;
constexpr int MAXOBS = 16;

// status codes (IPOPT ApplicationReturnStatus; oracle constants)
constexpr int ST_NONE = -1000, ST_OK = 0, ST_ACC = 1, ST_INFEAS = 2, ST_TINY = 3, ST_MAXIT = -1,
              ST_RESTOFAIL = -2, ST_STEPERR = -3, ST_EQ = -11, ST_INVALID = -13;

// option order = oracle IPOPT_DEFAULTS order; the Python side fills by name
#define NMPC_CPU_OPTS(X)                                                                                  \
  X(max_iter) X(tol) X(acceptable_tol) X(acceptable_iter) X(acceptable_obj_change_tol)                   \
  X(acceptable_dual_inf_tol) X(acceptable_constr_viol_tol) X(acceptable_compl_inf_tol) X(dual_inf_tol)    \
  X(constr_viol_tol) X(compl_inf_tol) X(mu_init) X(kappa_mu) X(theta_mu) X(barrier_tol_factor) X(tau_min) \
  X(bound_push) X(bound_frac) X(slack_bound_push) X(slack_bound_frac) X(bound_relax_factor)               \
  X(bound_mult_init_val) X(constr_mult_init_max) X(nlp_scaling_max_gradient) X(nlp_scaling_min_value)     \
  X(kappa_d) X(kappa_sigma) X(s_max) X(theta_max_fact) X(theta_min_fact) X(gamma_theta) X(gamma_phi)      \
  X(delta) X(s_theta) X(s_phi) X(eta_phi) X(alpha_red_factor) X(alpha_min_frac) X(max_soc) X(kappa_soc)   \
  X(obj_max_inc) X(first_hessian_perturbation) X(min_hessian_perturbation) X(max_hessian_perturbation)    \
  X(perturb_inc_fact_first) X(perturb_inc_fact) X(perturb_dec_fact) X(tiny_step_tol)                     \
  X(soft_resto_pderror_reduction_factor) X(max_soft_resto_iters) X(watchdog_shortened_iter_trigger)       \
  X(watchdog_trial_iter_max) X(resto_penalty_parameter) X(resto_proximity_weight)                         \
  X(required_infeasibility_reduction) X(bound_mult_reset_threshold) X(constr_mult_reset_threshold)

struct Opts {
#define NMPC_F(n) double n;
  NMPC_CPU_OPTS(NMPC_F)
#undef NMPC_F
};

}  // namespace

extern "C" {
// Problem description (mirrors oracle Problem; model 0 = uav8g, 1 = uav5)
typedef struct {
  int32_t N, model, n_obs, np, w1_pidx, w2_pidx;
  double T, w1, w2, vfov, hfov;
  double obs_x[MAXOBS], obs_y[MAXOBS], obs_rsum[MAXOBS];
  int32_t obs_x_pidx[MAXOBS], obs_y_pidx[MAXOBS];
} nmpc_cpu_problem;
}

namespace {

using Vec = std::vector<double>;
using Mask = std::vector<char>;

struct Prob {
  int N, nx, nu, nobs, nb, mr, n, m, np, uav5;
  double T, w1, w2, hv, hh;
  double ox[MAXOBS], oy[MAXOBS], rs[MAXOBS];
  int oxp[MAXOBS], oyp[MAXOBS], w1p, w2p;
  int bs[5];
};

Prob make_prob(const nmpc_cpu_problem& c) {
  Prob P{};
  P.N = c.N;
  P.uav5 = c.model == 1;
  P.nx = P.uav5 ? 5 : 8;
  P.nu = P.uav5 ? 3 : 6;
  P.nobs = c.n_obs;
  P.nb = P.uav5 ? 2 : 5;
  const int b8[5] = {2, 3, 5, 6, 7};
  for (int i = 0; i < P.nb; ++i) P.bs[i] = b8[i];
  P.mr = P.nb + P.nobs;
  P.n = P.nu * P.N;
  P.m = P.mr * (P.N + 1);
  P.np = c.np;
  P.T = c.T;
  P.w1 = c.w1;
  P.w2 = c.w2;
  P.hv = c.vfov / 2;
  P.hh = c.hfov / 2;
  for (int j = 0; j < P.nobs; ++j) {
    P.ox[j] = c.obs_x[j];
    P.oy[j] = c.obs_y[j];
    P.rs[j] = c.obs_rsum[j];
    P.oxp[j] = c.obs_x_pidx[j];
    P.oyp[j] = c.obs_y_pidx[j];
  }
  P.w1p = c.w1_pidx;
  P.w2p = c.w2_pidx;
  return P;
}

// per-solve constants taken from p (Problem.weighted / Problem.obstacles)
struct Ctx {
  double w1, w2, xt, yt, ox[MAXOBS], oy[MAXOBS];
  const double* p;
};

// ---------------------------------------------------------------- evaluation
// One point w: rollout, objective, rows and (optionally) the stage derivatives.
// oracle SSEval.__init__ (stage_cost_derivs, stage_rows, obstacle_derivs, dyn_jac)
struct Ev {
  double F = 0.0;
  bool derivs = false;
  Vec X, g, trig, gl, Hl, og, oH;
  void size(const Prob& P) {
    X.assign((P.N + 1) * 8, 0.0);
    g.assign(P.m, 0.0);
    trig.assign(P.N * 5, 0.0);
    gl.assign((P.N + 1) * 8, 0.0);
    Hl.assign((P.N + 1) * 64, 0.0);
    og.assign((P.N + 1) * MAXOBS * 2, 0.0);
    oH.assign((P.N + 1) * MAXOBS * 3, 0.0);
  }
};

// value, gradient (8) and Hessian (8x8) of one stage cost (oracle _stage_cost_derivs8,
// Python/NMPC_TT.py:209-220 in the ellipse form Q = (r1/a)^2 + (r2/b)^2)
double stage_derivs(const Prob& P, const Ctx& C, const double* xk, double* g8, double* H8) {
  const double xt = C.xt, yt = C.yt;
  const double x = xk[0], y = xk[1];
  const double dx = x - xt, dy = y - yt;
  const double d = std::sqrt(dx * dx + dy * dy);
  if (P.uav5) {  // distance cost only (MATLAB/Dynamic Obstacles/NMPC_TT.m:102-105)
    if (g8) {
      const double d3 = std::pow(d, 3);
      std::fill(g8, g8 + 8, 0.0);
      std::fill(H8, H8 + 64, 0.0);
      g8[0] = C.w1 * (dx / d);
      g8[1] = C.w1 * (dy / d);
      H8[0] = C.w1 * (dy * dy / d3);
      H8[1] = H8[8] = C.w1 * (-dx * dy / d3);
      H8[9] = C.w1 * (dx * dx / d3);
    }
    return C.w1 * d;
  }
  const double hv = P.hv, hh = P.hh;
  const double z = xk[2], x5 = xk[5], x6 = xk[6], x7 = xk[7];
  const double t6p = std::tan(x6 + hv), t6m = std::tan(x6 - hv);
  const double t5p = std::tan(x5 + hh), t5m = std::tan(x5 - hh);
  const double al6 = (t6p - t6m) / 2, be6 = (t6p + t6m) / 2;
  const double al5 = (t5p - t5m) / 2, be5 = (t5p + t5m) / 2;
  const double al6d = (t6p * t6p - t6m * t6m) / 2, be6d = (2 + t6p * t6p + t6m * t6m) / 2;
  const double al5d = (t5p * t5p - t5m * t5m) / 2, be5d = (2 + t5p * t5p + t5m * t5m) / 2;
  const double s6p = t6p * (1 + t6p * t6p), s6m = t6m * (1 + t6m * t6m);
  const double s5p = t5p * (1 + t5p * t5p), s5m = t5m * (1 + t5m * t5m);
  const double al6dd = s6p - s6m, be6dd = s6p + s6m;
  const double al5dd = s5p - s5m, be5dd = s5p + s5m;
  const double ex = xt - x - z * be6;
  const double ey = yt - y - z * be5;
  const double a = z * al6, b = z * al5;
  const double c = std::cos(x7), s = std::sin(x7);
  const double r1 = c * ex + s * ey;
  const double r2 = s * ex - c * ey;
  const double e1 = r1 / a, e2 = r2 / b;
  const double Q = e1 * e1 + e2 * e2;
  const double val = C.w1 * d + C.w2 * (Q - 1);
  if (!g8) return val;
  // local variable order v = (x, y, z, x5, x6, x7)
  const double gex[6] = {-1.0, 0.0, -be6, 0.0, -z * be6d, 0.0};
  const double gey[6] = {0.0, -1.0, -be5, -z * be5d, 0.0, 0.0};
  const double ga[6] = {0.0, 0.0, al6, 0.0, z * al6d, 0.0};
  const double gb[6] = {0.0, 0.0, al5, z * al5d, 0.0, 0.0};
  double Hex[36] = {}, Hey[36] = {}, Ha[36] = {}, Hb[36] = {};
  Hex[2 * 6 + 4] = Hex[4 * 6 + 2] = -be6d;
  Hex[4 * 6 + 4] = -z * be6dd;
  Hey[2 * 6 + 3] = Hey[3 * 6 + 2] = -be5d;
  Hey[3 * 6 + 3] = -z * be5dd;
  Ha[2 * 6 + 4] = Ha[4 * 6 + 2] = al6d;
  Ha[4 * 6 + 4] = z * al6dd;
  Hb[2 * 6 + 3] = Hb[3 * 6 + 2] = al5d;
  Hb[3 * 6 + 3] = z * al5dd;
  double u1[6], u2[6], gr1[6], gr2[6], ge1[6], ge2[6];
  for (int q = 0; q < 6; ++q) {
    const double e7 = q == 5 ? 1.0 : 0.0;
    u1[q] = -s * gex[q] + c * gey[q];
    u2[q] = c * gex[q] + s * gey[q];
    gr1[q] = c * gex[q] + s * gey[q] - r2 * e7;
    gr2[q] = s * gex[q] - c * gey[q] + r1 * e7;
  }
  for (int q = 0; q < 6; ++q) {
    ge1[q] = (gr1[q] - e1 * ga[q]) / a;
    ge2[q] = (gr2[q] - e2 * gb[q]) / b;
  }
  const double d3 = std::pow(d, 3);
  double gd[6] = {dx / d, dy / d, 0, 0, 0, 0};
  double Hd[36] = {};
  Hd[0] = dy * dy / d3;
  Hd[1] = Hd[6] = -dx * dy / d3;
  Hd[7] = dx * dx / d3;
  const int V[6] = {0, 1, 2, 5, 6, 7};
  std::fill(g8, g8 + 8, 0.0);
  std::fill(H8, H8 + 64, 0.0);
  for (int q = 0; q < 6; ++q) g8[V[q]] = C.w1 * gd[q] + C.w2 * (2 * (e1 * ge1[q] + e2 * ge2[q]));
  for (int qa = 0; qa < 6; ++qa) {
    for (int qb = 0; qb < 6; ++qb) {
      const double e7a = qa == 5 ? 1.0 : 0.0, e7b = qb == 5 ? 1.0 : 0.0;
      const int t = qa * 6 + qb;
      const double Hr1 = c * Hex[t] + s * Hey[t] + e7a * u1[qb] + u1[qa] * e7b - r1 * (e7a * e7b);
      const double Hr2 = s * Hex[t] - c * Hey[t] + e7a * u2[qb] + u2[qa] * e7b - r2 * (e7a * e7b);
      const double He1 = (Hr1 - ge1[qa] * ga[qb] - ga[qa] * ge1[qb] - e1 * Ha[t]) / a;
      const double He2 = (Hr2 - ge2[qa] * gb[qb] - gb[qa] * ge2[qb] - e2 * Hb[t]) / b;
      const double HQ = 2 * (ge1[qa] * ge1[qb] + ge2[qa] * ge2[qb] + e1 * He1 + e2 * He2);
      H8[V[qa] * 8 + V[qb]] = C.w1 * Hd[t] + C.w2 * HQ;
    }
  }
  return val;
}

// rollout (oracle rollout, NMPC_TT.py:160-167), F, rows; derivatives if asked
void evaluate(const Prob& P, const Ctx& C, const double* w, Ev& ev, bool derivs) {
  const int N = P.N, nx = P.nx, nu = P.nu;
  double* X = ev.X.data();
  for (int i = 0; i < 8; ++i) X[i] = i < nx ? C.p[i] : 0.0;
  for (int k = 0; k < N; ++k) {
    const double* u = w + nu * k;
    const double* xk = X + k * 8;
    double* xn = X + (k + 1) * 8;
    const double th = xk[3], ps = xk[4], v = u[0];
    const double ct = std::cos(th), st = std::sin(th), cp = std::cos(ps), sp = std::sin(ps);
    double* tg = ev.trig.data() + k * 5;
    tg[0] = ct; tg[1] = st; tg[2] = cp; tg[3] = sp; tg[4] = v;
    xn[0] = xk[0] + P.T * (v * cp * ct);
    xn[1] = xk[1] + P.T * (v * sp * ct);
    xn[2] = xk[2] + P.T * (v * st);
    for (int j = 3; j < nx; ++j) xn[j] = xk[j] + P.T * u[j - 2];
  }
  double F = 0.0;
  for (int k = 0; k < N; ++k)
    F += stage_derivs(P, C, X + k * 8, derivs ? ev.gl.data() + k * 8 : nullptr, derivs ? ev.Hl.data() + k * 64 : nullptr);
  ev.F = F;
  if (derivs) {
    std::fill(ev.gl.begin() + N * 8, ev.gl.begin() + (N + 1) * 8, 0.0);
    std::fill(ev.Hl.begin() + N * 64, ev.Hl.begin() + (N + 1) * 64, 0.0);
  }
  for (int k = 0; k <= N; ++k) {
    const double* xk = X + k * 8;
    double* gr = ev.g.data() + k * P.mr;
    for (int i = 0; i < P.nb; ++i) gr[i] = xk[P.bs[i]];
    for (int j = 0; j < P.nobs; ++j) {
      const double dx = xk[0] - C.ox[j], dy = xk[1] - C.oy[j];
      const double d = std::sqrt(dx * dx + dy * dy);
      gr[P.nb + j] = -d + P.rs[j];
      if (derivs) {
        double* o = ev.og.data() + (k * MAXOBS + j) * 2;
        o[0] = -(dx / d);
        o[1] = -(dy / d);
        const double d3 = std::pow(d, 3);
        double* h = ev.oH.data() + (k * MAXOBS + j) * 3;
        h[0] = -dy * dy / d3;
        h[1] = dx * dy / d3;
        h[2] = -dx * dx / d3;
      }
    }
  }
  ev.derivs = derivs;
}

// A_k = I + E, B_k (oracle dyn_jac): E has five entries (rows 0-2, columns 3-4),
// B has b0 in column 0 (rows 0-2) and T on the diagonal block (3+j, 1+j)
struct AB {
  double E03, E04, E13, E14, E23, b0, b1, b2, T;
  int nx, nu;
};
inline AB dyn_ab(const Prob& P, const double* tg) {
  const double T = P.T, ct = tg[0], st = tg[1], cp = tg[2], sp = tg[3], v = tg[4];
  return AB{-T * v * cp * st, -T * v * sp * ct, -T * v * sp * st, T * v * cp * ct, T * v * ct,
            T * cp * ct,      T * sp * ct,      T * st,           T,  P.nx,        P.nu};
}
// y = A x
inline void A_mul(const AB& a, const double* x, double* y) {
  for (int i = 0; i < a.nx; ++i) y[i] = x[i];
  y[0] += a.E03 * x[3] + a.E04 * x[4];
  y[1] += a.E13 * x[3] + a.E14 * x[4];
  y[2] += a.E23 * x[3];
}
// y = A^T x
inline void AT_mul(const AB& a, const double* x, double* y) {
  for (int i = 0; i < a.nx; ++i) y[i] = x[i];
  y[3] += (a.E03 * x[0] + a.E13 * x[1]) + a.E23 * x[2];
  y[4] += a.E04 * x[0] + a.E14 * x[1];
}
// y += B u
inline void B_muladd(const AB& a, const double* u, double* y) {
  y[0] += a.b0 * u[0];
  y[1] += a.b1 * u[0];
  y[2] += a.b2 * u[0];
  for (int j = 1; j < a.nu; ++j) y[2 + j] += a.T * u[j];
}
// u = B^T x
inline void BT_mul(const AB& a, const double* x, double* u) {
  u[0] = (a.b0 * x[0] + a.b1 * x[1]) + a.b2 * x[2];
  for (int j = 1; j < a.nu; ++j) u[j] = a.T * x[2 + j];
}

// G_k^T v (row Jacobian of stage k transposed, rows scaled by sc*v)
inline void add_GT(const Prob& P, const Ev& ev, int k, const double* v, const double* sc, double* out8) {
  const int r0 = k * P.mr;
  for (int i = 0; i < P.nb; ++i) out8[P.bs[i]] += sc[r0 + i] * v[r0 + i];
  for (int j = 0; j < P.nobs; ++j) {
    const double* o = ev.og.data() + (k * MAXOBS + j) * 2;
    const double wv = sc[r0 + P.nb + j] * v[r0 + P.nb + j];
    out8[0] += wv * o[0];
    out8[1] += wv * o[1];
  }
}

// out = of*gradF + J^T v in w-space, J = diag(dc) G Z (oracle SSEval.gradF / J.T @ y);
// stage 0 does not depend on w (Z_0 = 0) and is skipped
void adjoint(const Prob& P, const Ev& ev, double of, const double* v, const double* dc, double* out) {
  const int N = P.N, nx = P.nx, nu = P.nu;
  double lam[8] = {};
  for (int k = N; k >= 1; --k) {
    double a[8];
    for (int i = 0; i < 8; ++i) a[i] = of * ev.gl[k * 8 + i];
    if (v) add_GT(P, ev, k, v, dc, a);
    if (k < N) {
      double t[8];
      AT_mul(dyn_ab(P, ev.trig.data() + k * 5), lam, t);
      for (int i = 0; i < nx; ++i) a[i] += t[i];
    }
    for (int i = 0; i < 8; ++i) lam[i] = a[i];
    BT_mul(dyn_ab(P, ev.trig.data() + (k - 1) * 5), lam, out + nu * (k - 1));
  }
}

// out = J dw (rows, scaled), dX = the state sensitivities of dw
void jmul(const Prob& P, const Ev& ev, const double* dw, const double* dc, double* out, double* dX) {
  const int N = P.N, nx = P.nx, nu = P.nu;
  std::fill(dX, dX + 8, 0.0);
  for (int k = 0; k < N; ++k) {
    const AB ab = dyn_ab(P, ev.trig.data() + k * 5);
    double* xn = dX + (k + 1) * 8;
    for (int i = nx; i < 8; ++i) xn[i] = 0.0;
    A_mul(ab, dX + k * 8, xn);
    B_muladd(ab, dw + nu * k, xn);
  }
  for (int k = 0; k <= N; ++k) {
    const double* xk = dX + k * 8;
    const int r0 = k * P.mr;
    for (int i = 0; i < P.nb; ++i) out[r0 + i] = dc[r0 + i] * xk[P.bs[i]];
    for (int j = 0; j < P.nobs; ++j) {
      const double* o = ev.og.data() + (k * MAXOBS + j) * 2;
      out[r0 + P.nb + j] = dc[r0 + P.nb + j] * (o[0] * xk[0] + o[1] * xk[1]);
    }
  }
}

// Hessian of the Lagrangian (of*F + (dc*y)^T g) on the multiple-shooting
// structure: Q_k (8x8) for k = 1..N and S_k = Hxu_k^T (6x8) for k = 1..N-1
// (oracle SSEval.hessian, dyn_hess)
void hess_blocks(const Prob& P, const Ev& ev, double of, const double* y, const double* dc, double* Q, double* S) {
  const int N = P.N, nx = P.nx;
  double adj[8] = {};
  const double T = P.T;
  for (int k = N; k >= 1; --k) {
    double* Qk = Q + k * 64;
    for (int t = 0; t < 64; ++t) Qk[t] = of * ev.Hl[k * 64 + t];
    const int r0 = k * P.mr;
    for (int j = 0; j < P.nobs; ++j) {
      const double l = dc[r0 + P.nb + j] * y[r0 + P.nb + j];
      const double* h = ev.oH.data() + (k * MAXOBS + j) * 3;
      Qk[0] += l * h[0];
      Qk[1] += l * h[1];
      Qk[8] += l * h[1];
      Qk[9] += l * h[2];
    }
    double* Sk = S + k * 48;
    std::fill(Sk, Sk + 48, 0.0);
    if (k < N) {  // dyn_hess with adj_{k+1}
      const double* tg = ev.trig.data() + k * 5;
      const double ct = tg[0], st = tg[1], cp = tg[2], sp = tg[3], v = tg[4];
      const double l0 = adj[0], l1 = adj[1], l2 = adj[2];
      Qk[3 * 8 + 3] += T * (-l0 * v * cp * ct - l1 * v * sp * ct - l2 * v * st);
      Qk[4 * 8 + 4] += T * (-l0 * v * cp * ct - l1 * v * sp * ct);
      const double h34 = T * (l0 * v * sp * st - l1 * v * cp * st);
      Qk[3 * 8 + 4] += h34;
      Qk[4 * 8 + 3] += h34;
      Sk[0 * 8 + 3] = T * (-l0 * cp * st - l1 * sp * st + l2 * ct);
      Sk[0 * 8 + 4] = T * (-l0 * sp * ct + l1 * cp * ct);
    }
    // adjoint: adj_k = of*gl_k + G_k^T (dc y)_k + A_k^T adj_{k+1}
    double a[8];
    for (int i = 0; i < 8; ++i) a[i] = of * ev.gl[k * 8 + i];
    add_GT(P, ev, k, y, dc, a);
    if (k < N) {
      double t[8];
      AT_mul(dyn_ab(P, ev.trig.data() + k * 5), adj, t);
      for (int i = 0; i < nx; ++i) a[i] += t[i];
    }
    for (int i = 0; i < 8; ++i) adj[i] = a[i];
  }
}

// Q_k += G_k^T diag(dc^2 wr) G_k, k = 1..N  (J^T diag(wr) J)
void add_rows(const Prob& P, const Ev& ev, const double* wr, const double* dc, double* Q) {
  for (int k = 1; k <= P.N; ++k) {
    double* Qk = Q + k * 64;
    const int r0 = k * P.mr;
    for (int i = 0; i < P.nb; ++i) {
      const int s = P.bs[i];
      Qk[s * 8 + s] += dc[r0 + i] * dc[r0 + i] * wr[r0 + i];
    }
    for (int j = 0; j < P.nobs; ++j) {
      const int r = r0 + P.nb + j;
      const double* o = ev.og.data() + (k * MAXOBS + j) * 2;
      const double wgt = dc[r] * dc[r] * wr[r];
      Qk[0] += wgt * o[0] * o[0];
      Qk[1] += wgt * o[0] * o[1];
      Qk[8] += wgt * o[1] * o[0];
      Qk[9] += wgt * o[1] * o[1];
    }
  }
}

// ------------------------------------------------------------- Riccati LQ
// min 1/2 dw^T M dw + g^T dw with M = sum_k [Q_k S_k^T; S_k diag(R_k)] on the
// stage structure dX_{k+1} = A_k dX_k + B_k du_k, dX_0 = 0.  factor() is the
// inertia test (every R~_k = R_k + B^T P B positive definite).
struct Riccati {
  int N = 0, nx = 0, nu = 0;
  Vec K, L, idg, kv, sg;
  const char* fix = nullptr;  // fixed decision variables (make_parameter): decoupled, zero step
  // signed pivots (problems with equality rows): R~_k = L Sigma L^T, Sigma = diag(+-1), and
  // nneg counts the negative ones for the augmented system's inertia test (the kernel's
  // riccati<true>); otherwise every pivot must be positive (IPOPT's inertia test)
  bool sgn = false;
  int nneg = 0;
  void size(const Prob& p) {
    N = p.N; nx = p.nx; nu = p.nu;
    K.assign(N * 48, 0.0);
    L.assign(N * 36, 0.0);
    idg.assign(N * 6, 0.0);
    kv.assign(N * 6, 0.0);
    sg.assign(N * 6, 1.0);
  }
  bool factor(const Prob& Pr, const Ev& ev, const double* Q, const double* S, const double* R) {
    return nx == 8 ? factor_t<8, 6>(Pr, ev, Q, S, R) : factor_t<5, 3>(Pr, ev, Q, S, R);
  }
  void solve(const Prob& Pr, const Ev& ev, const double* q, const double* r, double* du, double* dX) {
    if (nx == 8) solve_t<8, 6>(Pr, ev, q, r, du, dX);
    else solve_t<5, 3>(Pr, ev, q, r, du, dX);
  }
  // rows of B^T M (M has rows of length W, stride 8)
  template <int NU, int W>
  static void BT_rows(const AB& a, const double* M, double* out /*stride 8*/) {
    for (int j = 0; j < W; ++j) out[j] = (a.b0 * M[j] + a.b1 * M[8 + j]) + a.b2 * M[16 + j];
    for (int c = 1; c < NU; ++c)
      for (int j = 0; j < W; ++j) out[c * 8 + j] = a.T * M[(2 + c) * 8 + j];
  }
  // K = -R~^{-1} S~ for all NX columns at once (L L^T = R~, idg = 1 / diag L)
  template <int NX, int NU>
  static void chol_solve_cols(const double* Lo, const double* idg, const double* Sm, double* Km,
                              const double* sgp = nullptr) {
    double V[NU][8];
    for (int i = 0; i < NU; ++i) {
      for (int j = 0; j < NX; ++j) {
        double s = Sm[i * 8 + j];
        for (int t = 0; t < i; ++t) s -= Lo[i * 6 + t] * V[t][j];
        V[i][j] = s * idg[i];
      }
    }
    if (sgp)
      for (int i = 0; i < NU; ++i)
        for (int j = 0; j < NX; ++j) V[i][j] *= sgp[i];
    for (int i = NU - 1; i >= 0; --i) {
      for (int j = 0; j < NX; ++j) {
        double s = V[i][j];
        for (int t = i + 1; t < NU; ++t) s -= Lo[t * 6 + i] * V[t][j];
        V[i][j] = s * idg[i];
      }
    }
    for (int i = 0; i < NU; ++i)
      for (int j = 0; j < NX; ++j) Km[i * 8 + j] = -V[i][j];
  }
  template <int NU>
  static bool chol_t(const double* M, double* Lo, double* idg) {
    for (int i = 0; i < NU; ++i) {
      for (int j = 0; j <= i; ++j) {
        double s = M[i * 6 + j];
        for (int t = 0; t < j; ++t) s -= Lo[i * 6 + t] * Lo[j * 6 + t];
        if (i == j) {
          if (!(s > 0.0)) return false;
          Lo[i * 6 + i] = std::sqrt(s);
          idg[i] = 1.0 / Lo[i * 6 + i];
        } else {
          Lo[i * 6 + j] = s * idg[j];
        }
      }
    }
    return true;
  }
  // L Sigma L^T with signed pivots (a zero pivot: singular)
  template <int NU>
  static bool chol_sg(const double* M, double* Lo, double* idg, double* sgp, int& neg) {
    for (int i = 0; i < NU; ++i) {
      for (int j = 0; j <= i; ++j) {
        double s = M[i * 6 + j];
        for (int t = 0; t < j; ++t) s -= (sgp[t] * Lo[i * 6 + t]) * Lo[j * 6 + t];
        if (i == j) {
          if (!(s != 0.0)) return false;
          sgp[i] = s < 0.0 ? -1.0 : 1.0;
          if (s < 0.0) ++neg;
          Lo[i * 6 + i] = std::sqrt(std::fabs(s));
          idg[i] = 1.0 / Lo[i * 6 + i];
        } else {
          Lo[i * 6 + j] = (s * idg[j]) * sgp[j];
        }
      }
    }
    return true;
  }
  template <int NU>
  void chol_solve_t(const double* Lo, const double* idg, double* v, const double* sgp = nullptr) const {
    for (int i = 0; i < NU; ++i) {
      double s = v[i];
      for (int t = 0; t < i; ++t) s -= Lo[i * 6 + t] * v[t];
      v[i] = s * idg[i];
    }
    if (sgp)
      for (int i = 0; i < NU; ++i) v[i] *= sgp[i];
    for (int i = NU - 1; i >= 0; --i) {
      double s = v[i];
      for (int t = i + 1; t < NU; ++t) s -= Lo[t * 6 + i] * v[t];
      v[i] = s * idg[i];
    }
  }
  template <int NX, int NU>
  bool factor_t(const Prob& Pr, const Ev& ev, const double* Q, const double* S, const double* R) {
    alignas(32) double Pm[64], PA[64], PB[64], Rt[36], St[48], RB[48];
    for (int t = 0; t < 64; ++t) Pm[t] = Q[N * 64 + t];
    nneg = 0;
    for (int k = N - 1; k >= 0; --k) {
      const AB ab = dyn_ab(Pr, ev.trig.data() + k * 5);
      for (int i = 0; i < NX; ++i) {  // row i of P A = A^T P[i,:]; of P B = B^T P[i,:]
        const double* pr = Pm + i * 8;
        double* pa = PA + i * 8;
        for (int j = 0; j < NX; ++j) pa[j] = pr[j];
        pa[3] += (ab.E03 * pr[0] + ab.E13 * pr[1]) + ab.E23 * pr[2];
        pa[4] += ab.E04 * pr[0] + ab.E14 * pr[1];
        double* pb = PB + i * 8;
        pb[0] = (ab.b0 * pr[0] + ab.b1 * pr[1]) + ab.b2 * pr[2];
        for (int c = 1; c < NU; ++c) pb[c] = ab.T * pr[2 + c];
      }
      BT_rows<NU, NU>(ab, PB, RB);  // B^T P B
      for (int a = 0; a < NU; ++a)
        for (int c = 0; c < NU; ++c) Rt[a * 6 + c] = RB[a * 8 + c] + (a == c ? R[k * NU + a] : 0.0);
      BT_rows<NU, NX>(ab, PA, St);  // B^T P A
      if (k > 0)
        for (int a = 0; a < NU; ++a)
          for (int j = 0; j < NX; ++j) St[a * 8 + j] += S[k * 48 + a * 8 + j];
      if (fix)  // a fixed control leaves the problem: unit pivot, no coupling
        for (int a = 0; a < NU; ++a)
          if (fix[k * NU + a]) {
            for (int c = 0; c < NU; ++c) Rt[a * 6 + c] = Rt[c * 6 + a] = 0.0;
            Rt[a * 6 + a] = 1.0;
            for (int j = 0; j < NX; ++j) St[a * 8 + j] = 0.0;
          }
      double* Lk = L.data() + k * 36;
      double* ik = idg.data() + k * 6;
      double* sk = sg.data() + k * 6;
      if (sgn) {
        if (!chol_sg<NU>(Rt, Lk, ik, sk, nneg)) return false;
      } else if (!chol_t<NU>(Rt, Lk, ik)) {
        return false;
      }
      double* Kk = K.data() + k * 48;
      chol_solve_cols<NX, NU>(Lk, ik, St, Kk, sgn ? sk : nullptr);
      if (k > 0) {  // P_k = Q_k + A^T P A + S~^T K
        double APA[64];
        for (int t = 0; t < 64; ++t) APA[t] = PA[t];
        for (int j = 0; j < NX; ++j) {
          APA[3 * 8 + j] += (ab.E03 * PA[j] + ab.E13 * PA[8 + j]) + ab.E23 * PA[16 + j];
          APA[4 * 8 + j] += ab.E04 * PA[j] + ab.E14 * PA[8 + j];
        }
        double SK[64];
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) {
            double sk = 0.0;
            for (int a = 0; a < NU; ++a) sk += St[a * 8 + i] * Kk[a * 8 + j];
            SK[i * 8 + j] = sk;
          }
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j)
            Pm[i * 8 + j] = Q[k * 64 + i * 8 + j] + 0.5 * (APA[i * 8 + j] + APA[j * 8 + i]) +
                            0.5 * (SK[i * 8 + j] + SK[j * 8 + i]);
      }
    }
    return true;
  }
  // q: (N+1)*8 (k >= 1 used), r: n.  du = the step in w, dX its state sensitivities
  template <int NX, int NU>
  void solve_t(const Prob& Pr, const Ev& ev, const double* q, const double* r, double* du, double* dX) {
    double p[8];
    for (int i = 0; i < 8; ++i) p[i] = q[N * 8 + i];
    for (int k = N - 1; k >= 0; --k) {
      const AB ab = dyn_ab(Pr, ev.trig.data() + k * 5);
      double rt[6], v[6];
      BT_mul(ab, p, rt);
      for (int a = 0; a < NU; ++a) {
        rt[a] += r[k * NU + a];
        if (fix && fix[k * NU + a]) rt[a] = 0.0;
        v[a] = rt[a];
      }
      chol_solve_t<NU>(L.data() + k * 36, idg.data() + k * 6, v, sgn ? sg.data() + k * 6 : nullptr);
      for (int a = 0; a < NU; ++a) kv[k * 6 + a] = -v[a];
      if (k > 0) {  // p_k = q_k + A^T p + K^T r~
        const double* Kk = K.data() + k * 48;
        double t[8];
        AT_mul(ab, p, t);
        for (int i = 0; i < NX; ++i) {
          double kr = 0.0;
          for (int a = 0; a < NU; ++a) kr += Kk[a * 8 + i] * rt[a];
          p[i] = q[k * 8 + i] + t[i] + kr;
        }
      }
    }
    std::fill(dX, dX + 8, 0.0);
    for (int k = 0; k < N; ++k) {
      const AB ab = dyn_ab(Pr, ev.trig.data() + k * 5);
      const double* Kk = K.data() + k * 48;
      const double* xk = dX + k * 8;
      double u[6];
      for (int a = 0; a < NU; ++a) {
        double t = kv[k * 6 + a];
        for (int j = 0; j < NX; ++j) t += Kk[a * 8 + j] * xk[j];
        u[a] = t;
        du[k * NU + a] = t;
      }
      double* xn = dX + (k + 1) * 8;
      for (int i = NX; i < 8; ++i) xn[i] = 0.0;
      A_mul(ab, xk, xn);
      B_muladd(ab, u, xn);
    }
  }
};

// ------------------------------------------------------------------ helpers
inline double amax(const Vec& v) {
  double a = 0.0;
  for (double x : v) a = std::max(a, std::fabs(x));
  return a;
}
inline bool compare_le(double lhs, double rhs, double basval) {  // IPOPT Compare_le
  return lhs - rhs <= 10.0 * EPS * std::fabs(basval);
}
inline bool allfinite(const Vec& v) {
  for (double x : v)
    if (!std::isfinite(x)) return false;
  return true;
}
inline double sumabs(const Vec& v) {
  double s = 0.0;
  for (double x : v) s += std::fabs(x);
  return s;
}

struct Step {  // main-problem Newton step (oracle solve_dir)
  Vec dx, ds, dy, dzl, dzu, dvl, dvu;
  void size(int n, int m) {
    dx.assign(n, 0.0); ds.assign(m, 0.0); dy.assign(m, 0.0);
    dzl.assign(n, 0.0); dzu.assign(n, 0.0); dvl.assign(m, 0.0); dvu.assign(m, 0.0);
  }
};
struct Trial {  // trial point (oracle trial)
  Vec x, s, d;
  Ev ev;
  double f = 0, phi = 0, th = 0;
};
struct RStep {  // restoration Newton step (oracle restoration.rdir)
  Vec dx, ds, dy, dp, dzl, dzu, dvl, dvu, dzp, dzn, dn;
  void size(int n, int m) {
    dx.assign(n, 0.0); ds.assign(m, 0.0); dy.assign(m, 0.0); dp.assign(m, 0.0);
    dzl.assign(n, 0.0); dzu.assign(n, 0.0); dvl.assign(m, 0.0); dvu.assign(m, 0.0);
    dzp.assign(m, 0.0); dzn.assign(m, 0.0); dn.assign(m, 0.0);
  }
};
struct RTrial {
  Vec x, s, p, nn, d;
  Ev ev;
  double phi = 0, th = 0;
};

struct Result {
  int status = ST_NONE, iter = 0;
  double F = 0.0;
  Vec x, g, lam_x, lam_g;
};

// ------------------------------------------------------------------ solver
// oracle IpoptDense.solve, control flow restated statement by statement
class Solver {
 public:
  bool dbg_trace_ = std::getenv("NMPC_CPU_TRACE") != nullptr;
  Solver(const Prob& P, const Opts& o) : P_(P), o_(o) {
    n = P.n; m = P.m;
    ric.size(P);
    Qb.assign((P.N + 1) * 64, 0.0);
    Qw.assign((P.N + 1) * 64, 0.0);
    Sb.assign(P.N * 48 + 48, 0.0);
    qv.assign((P.N + 1) * 8, 0.0);
    dXs.assign((P.N + 1) * 8, 0.0);
  }
  void solve(const double* w0, const double* p, const double* lbx, const double* ubx, const double* lbg,
             const double* ubg, Result& R);

 private:
  const Prob& P_;
  const Opts& o_;
  int n, m;
  Ctx C{};
  Riccati ric;
  Vec Qb, Qw, Sb, qv, dXs;
  // bounds
  Mask xlm, xum, slm, sum_, fixd;
  int nf = 0;  // free decision variables (n minus the fixed ones)
  Vec xl, xu, dl, du, gl_, gu_, dampxl, dampxu, dampsl, dampsu, dc;
  double df = 1.0;
  int nzx = 0, nzs = 0;
  // equality rows (lbg == ubg): IPOPT's c(x) = 0 (oracle IpoptDense, the kernel's CapE).
  // The row keeps its slot with the slack pinned at the scaled target and no bounds; the
  // Newton step adds the rows through the Schur complement S = J_c H^-1 J_c^T of the
  // augmented system, from one unit solve per row with the Riccati factors.
  static constexpr int MEQ = 128;  // the kernel's NMPC_MEQ
  Mask eqm;
  int neq = 0;
  std::vector<int> eqi;
  Vec gE;                // targets (unscaled)
  std::vector<Vec> dxe;  // -H^-1 J_e^T per equality row
  Vec eqL, eqSg;         // signed factor of S + delta_c I (row-major neq x neq) and pivot signs

  // S from the unit solves, its signed factor with delta_c = 0, then IPOPT's
  // jacobian_regularization_value * mu^0.25 if S is singular; inertia (Haynsworth): the
  // augmented matrix has n positive and neq negative eigenvalues iff S + delta_c I has as
  // many negative pivots as H had (ric.nneg).  allow_dc false: the least-squares
  // multipliers (no regularisation; a singular S means y = 0)
  bool eq_schur(const Ev& ev, double mu, bool allow_dc) {
    const int mc = neq;
    dxe.assign(mc, Vec(n, 0.0));
    Vec S(mc * mc, 0.0), unit(m, 0.0), jd(m, 0.0), zr(n, 0.0);
    for (int e = 0; e < mc; ++e) {
      unit[eqi[e]] = 1.0;
      for (int k = 0; k <= P_.N; ++k) {
        double a[8] = {};
        add_GT(P_, ev, k, unit.data(), dc.data(), a);
        for (int i = 0; i < 8; ++i) qv[k * 8 + i] = a[i];
      }
      unit[eqi[e]] = 0.0;
      ric.solve(P_, ev, qv.data(), zr.data(), dxe[e].data(), dXs.data());
      jmul(P_, ev, dxe[e].data(), dc.data(), jd.data(), dXs.data());
      for (int l = 0; l < mc; ++l) S[l * mc + e] = -jd[eqi[l]];
    }
    double scale = 0.0;
    for (int c = 0; c < mc; ++c) scale = std::max(scale, std::fabs(S[c * mc + c]));
    for (int att = 0; att < (allow_dc ? 2 : 1); ++att) {
      const double dcv = att == 0 ? 0.0 : 1e-8 * std::pow(mu, 0.25);
      Vec L = S, sgS(mc, 1.0);
      for (int c = 0; c < mc; ++c) L[c * mc + c] += dcv;
      bool sing = false;
      int negS = 0;
      for (int c = 0; c < mc; ++c) {  // right-looking, as the kernel's lane-per-row factor
        const double d = L[c * mc + c];
        if (!(std::fabs(d) > 1e-14 * scale)) sing = true;
        sgS[c] = d < 0.0 ? -1.0 : 1.0;
        negS += d < 0.0 ? 1 : 0;
        const double ig = 1.0 / std::sqrt(std::fabs(d));
        L[c * mc + c] = std::fabs(d) * ig;
        for (int r = c + 1; r < mc; ++r) L[r * mc + c] = (L[r * mc + c] * ig) * sgS[c];
        for (int c2 = c + 1; c2 < mc; ++c2) {
          const double l2 = L[c2 * mc + c];
          for (int r = c + 1; r < mc; ++r) L[r * mc + c2] -= (L[r * mc + c] * sgS[c]) * l2;
        }
      }
      if (dbg_trace_)
        std::fprintf(stderr, "cpu eq_schur dc %.3g nneg %d negS %d sing %d S00 %.6g\n", dcv, ric.nneg, negS, (int)sing,
                     S[0]);
      if (sing) continue;
      if (negS != ric.nneg) return false;
      eqL = L; eqSg = sgS;
      return true;
    }
    return false;
  }
  // (S + delta_c I)^-1 rhs with the stored signed factor
  void eq_solve(const Vec& rhs, Vec& out) const {
    const int mc = neq;
    Vec z(mc, 0.0), part = rhs;
    for (int c = 0; c < mc; ++c) {
      z[c] = part[c] / eqL[c * mc + c];
      for (int r = c + 1; r < mc; ++r) part[r] -= eqL[r * mc + c] * z[c];
    }
    out.assign(mc, 0.0);
    for (int c = mc - 1; c >= 0; --c) {
      double a = eqSg[c] * z[c];
      for (int j = c + 1; j < mc; ++j) a -= eqL[j * mc + c] * out[j];
      out[c] = a / eqL[c * mc + c];
    }
  }

  void eval(const double* w, Ev& ev, bool derivs) { evaluate(P_, C, w, ev, derivs); }
  void slacks(const Vec& x, const Vec& s, Vec& Sxl, Vec& Sxu, Vec& Ssl, Vec& Ssu) const {
    Sxl.resize(n); Sxu.resize(n); Ssl.resize(m); Ssu.resize(m);
    for (int i = 0; i < n; ++i) {
      Sxl[i] = xlm[i] ? x[i] - xl[i] : 1.0;
      Sxu[i] = xum[i] ? xu[i] - x[i] : 1.0;
    }
    for (int r = 0; r < m; ++r) {
      Ssl[r] = slm[r] ? s[r] - dl[r] : 1.0;
      Ssu[r] = sum_[r] ? du[r] - s[r] : 1.0;
    }
  }
  double barrier_obj(double f, const Vec& x, const Vec& s, double mu) const {
    double logs = 0.0, damp = 0.0;
    for (int i = 0; i < n; ++i) {
      const double a = x[i] - xl[i], b = xu[i] - x[i];
      if (xlm[i]) logs += std::log(a);
      if (xum[i]) logs += std::log(b);
      if (xlm[i]) damp += dampxl[i] * a;
      if (xum[i]) damp += dampxu[i] * b;
    }
    double ls = 0.0, ds = 0.0;
    for (int r = 0; r < m; ++r) {
      const double a = s[r] - dl[r], b = du[r] - s[r];
      if (slm[r]) ls += std::log(a);
      if (sum_[r]) ls += std::log(b);
      if (slm[r]) ds += dampsl[r] * a;
      if (sum_[r]) ds += dampsu[r] * b;
    }
    return f - mu * (logs + ls) + o_.kappa_d * mu * (damp + ds);
  }
  double compl_max(const Vec& x, const Vec& s, const Vec& zl, const Vec& zu, const Vec& vl, const Vec& vu,
                   double mu, double* sum = nullptr) const {
    double c = 0.0, sm = 0.0;
    for (int i = 0; i < n; ++i) {
      if (xlm[i]) { const double v = std::fabs((x[i] - xl[i]) * zl[i] - mu); c = std::max(c, v); sm += v; }
      if (xum[i]) { const double v = std::fabs((xu[i] - x[i]) * zu[i] - mu); c = std::max(c, v); sm += v; }
    }
    for (int r = 0; r < m; ++r) {
      if (slm[r]) { const double v = std::fabs((s[r] - dl[r]) * vl[r] - mu); c = std::max(c, v); sm += v; }
      if (sum_[r]) { const double v = std::fabs((du[r] - s[r]) * vu[r] - mu); c = std::max(c, v); sm += v; }
    }
    if (sum) *sum = sm;
    return c;
  }
  void err_scaling(const Vec& y, const Vec& zl, const Vec& zu, const Vec& vl, const Vec& vu, double& sd,
                   double& sc) const {
    const double smax = o_.s_max;
    const int nd = m + nzx + nzs, nc = nzx + nzs;
    const double bz = sumabs(zl) + sumabs(zu) + sumabs(vl) + sumabs(vu);
    sd = nd ? (sumabs(y) + bz) / nd : 0.0;
    sd = std::max(smax, sd) / smax;
    sc = nc ? bz / nc : 0.0;
    sc = std::max(smax, sc) / smax;
  }
  // grad of the Lagrangian: glx = gf + J^T y - zl + zu (w-space), gls = -y - vl + vu
  void grad_lag(const Ev& ev, const Vec& y, const Vec& zl, const Vec& zu, const Vec& vl, const Vec& vu, Vec& glx,
                Vec& gls) const {
    glx.assign(n, 0.0);
    adjoint(P_, ev, df, y.data(), dc.data(), glx.data());
    for (int i = 0; i < n; ++i) glx[i] = fixd[i] ? 0.0 : glx[i] - zl[i] + zu[i];
    gls.resize(m);
    for (int r = 0; r < m; ++r) gls[r] = eqm[r] ? 0.0 : -y[r] - vl[r] + vu[r];  // slack part: inequality rows
  }
  double cviol_scaled(const Vec& d, const Vec& s) const {
    double c = 0.0;
    for (int r = 0; r < m; ++r) {
      if (slm[r]) c = std::max(c, std::max(0.0, dl[r] - d[r]));
      if (sum_[r]) c = std::max(c, std::max(0.0, d[r] - du[r]));
      if (eqm[r]) c = std::max(c, std::fabs(d[r] - s[r]));
    }
    return c;
  }
  double cviol_unscaled(const Vec& d) const {  // oracle cviol_unscaled
    double c = 0.0;
    for (int r = 0; r < m; ++r) {
      const double g = d[r] / dc[r];
      if (slm[r]) c = std::max(c, std::max(0.0, gl_[r] - g));
      if (sum_[r]) c = std::max(c, std::max(0.0, g - gu_[r]));
      if (eqm[r]) c = std::max(c, std::fabs(g - gE[r]));
    }
    return c;
  }
  double frac_to_bound(double tau, const Vec& x, const Vec& s, const Vec& dx, const Vec& ds) const {
    double a = 1.0;
    for (int i = 0; i < n; ++i) {
      if (xlm[i] && dx[i] < 0) a = std::min(a, -tau * (x[i] - xl[i]) / dx[i]);
    }
    for (int i = 0; i < n; ++i) {
      if (xum[i] && -dx[i] < 0) a = std::min(a, -tau * (xu[i] - x[i]) / (-dx[i]));
    }
    for (int r = 0; r < m; ++r) {
      if (slm[r] && ds[r] < 0) a = std::min(a, -tau * (s[r] - dl[r]) / ds[r]);
    }
    for (int r = 0; r < m; ++r) {
      if (sum_[r] && -ds[r] < 0) a = std::min(a, -tau * (du[r] - s[r]) / (-ds[r]));
    }
    return a;
  }
  double dual_frac_to_bound(double tau, const Vec& zl, const Vec& zu, const Vec& vl, const Vec& vu, const Vec& dzl,
                            const Vec& dzu, const Vec& dvl, const Vec& dvu) const {
    double a = 1.0;
    for (int i = 0; i < n; ++i)
      if (xlm[i] && dzl[i] < 0) a = std::min(a, -tau * zl[i] / dzl[i]);
    for (int i = 0; i < n; ++i)
      if (xum[i] && dzu[i] < 0) a = std::min(a, -tau * zu[i] / dzu[i]);
    for (int r = 0; r < m; ++r)
      if (slm[r] && dvl[r] < 0) a = std::min(a, -tau * vl[r] / dvl[r]);
    for (int r = 0; r < m; ++r)
      if (sum_[r] && dvu[r] < 0) a = std::min(a, -tau * vu[r] / dvu[r]);
    return a;
  }
  Vec relax(const double* b, int len, double sign) const {
    Vec out(b, b + len);
    for (int i = 0; i < len; ++i) {
      if (std::fabs(b[i]) < INF) {
        const double r = std::min(o_.constr_viol_tol, o_.bound_relax_factor * std::max(1.0, std::fabs(b[i])));
        out[i] = b[i] + sign * r;
      }
    }
    return out;
  }
  // IPOPT DefaultIterateInitializer::push_variables (oracle _push)
  static void push(Vec& x, const Vec& lo_, const Vec& hi_, const Mask& lm, const Mask& um, double kp, double kf) {
    for (size_t i = 0; i < x.size(); ++i) {
      const double lo = lm[i] ? lo_[i] : 0.0, hi = um[i] ? hi_[i] : 0.0;
      double pl = kp * std::max(1.0, std::fabs(lo)), pu = kp * std::max(1.0, std::fabs(hi));
      const double span = (lm[i] && um[i]) ? hi - lo : PINF;
      pl = std::min(pl, kf * span);
      pu = std::min(pu, kf * span);
      if (lm[i]) x[i] = std::max(x[i], lo + pl);
      if (um[i]) x[i] = std::min(x[i], hi - pu);
    }
  }
  // least-squares multipliers: wx = (I + w_J J^T J)^-1 (bx + J^T bsx), returns J wx
  void ls_solve(const Ev& ev, double rw, const Vec& bx_ctrl, double of, const Vec& bs, Vec& wx, Vec& jwx) {
    ls_solve_w(ev, Vec(m, rw), bx_ctrl, of, bs, wx, jwx, nullptr);
  }
  // ... with per-row weights; yc: the equality rows' multipliers of
  // [I + J_d^T W J_d, -J_c^T; J_c, 0] [wx; yc] = [b; 0] (false: singular S, y = 0)
  bool ls_solve_w(const Ev& ev, const Vec& wr, const Vec& bx_ctrl, double of, const Vec& bs, Vec& wx, Vec& jwx,
                  Vec* yc) {
    ric.sgn = false;
    std::fill(Qw.begin(), Qw.end(), 0.0);
    std::fill(Sb.begin(), Sb.end(), 0.0);
    Vec R(n, 1.0);
    add_rows(P_, ev, wr.data(), dc.data(), Qw.data());
    // q_k = -(of*gl_k + G^T (dc bs)), r = -bx_ctrl
    for (int k = 0; k <= P_.N; ++k) {
      double a[8];
      for (int i = 0; i < 8; ++i) a[i] = of * ev.gl[k * 8 + i];
      add_GT(P_, ev, k, bs.data(), dc.data(), a);
      for (int i = 0; i < 8; ++i) qv[k * 8 + i] = -a[i];
    }
    Vec r(n);
    for (int i = 0; i < n; ++i) r[i] = -bx_ctrl[i];
    ric.factor(P_, ev, Qw.data(), Sb.data(), R.data());
    wx.assign(n, 0.0);
    ric.solve(P_, ev, qv.data(), r.data(), wx.data(), dXs.data());
    jwx.assign(m, 0.0);
    jmul(P_, ev, wx.data(), dc.data(), jwx.data(), dXs.data());
    if (!yc) return true;
    if (!eq_schur(ev, 0.0, false)) return false;
    Vec rhs(neq);
    for (int e = 0; e < neq; ++e) rhs[e] = -jwx[eqi[e]];
    eq_solve(rhs, *yc);
    for (int e = 0; e < neq; ++e)
      for (int i = 0; i < n; ++i) wx[i] -= (*yc)[e] * dxe[e][i];
    jmul(P_, ev, wx.data(), dc.data(), jwx.data(), dXs.data());
    return true;
  }
  // the main problem's least-squares multipliers: y = bs - J wx (inequality rows), yc
  // (equality rows); y = 0 above ymax or when the system is singular
  void main_ls_mults(const Ev& ev, const Vec& zl_, const Vec& zu_, const Vec& vl_, const Vec& vu_, double ymax,
                     Vec& y) {
    Vec bxc(n), bs(m), wx, jwx;
    for (int i = 0; i < n; ++i) bxc[i] = -zl_[i] + zu_[i];
    for (int r = 0; r < m; ++r) bs[r] = vu_[r] - vl_[r];
    double ym = 0.0;
    bool ok = true;
    if (neq == 0) {
      ls_solve(ev, 1.0, bxc, df, bs, wx, jwx);
      for (int r = 0; r < m; ++r) { y[r] = bs[r] - jwx[r]; ym = std::max(ym, std::fabs(y[r])); }
    } else {
      Vec wr(m), yc;
      for (int r = 0; r < m; ++r) { wr[r] = eqm[r] ? 0.0 : 1.0; if (eqm[r]) bs[r] = 0.0; }
      ok = ls_solve_w(ev, wr, bxc, df, bs, wx, jwx, &yc);
      if (ok) {
        for (int r = 0; r < m; ++r) y[r] = eqm[r] ? 0.0 : bs[r] - jwx[r];
        for (int e = 0; e < neq; ++e) y[eqi[e]] = yc[e];
        for (int r = 0; r < m; ++r) ym = std::max(ym, std::fabs(y[r]));
      }
    }
    if (!ok || ym > ymax) std::fill(y.begin(), y.end(), 0.0);
  }

  struct RestoOut {
    int status = ST_NONE, it = 0;
    Vec x, s, y, zl, zu, vl, vu;
    Ev ev;
  };
  void restoration(const Vec& x0, const Vec& s0, const Vec& d0, const Ev& ev0, const Vec& y0, const Vec& zl0,
                   const Vec& zu0, const Vec& vl0, const Vec& vu0, double mu0, double tau0, double theta0,
                   double phi0, const std::vector<std::pair<double, double>>& ofilt, int it_, RestoOut& out);
};

void Solver::solve(const double* w0p, const double* p, const double* lbxp, const double* ubxp, const double* lbgp,
                   const double* ubgp, Result& R) {
  const Opts& o = o_;
  // per-solve constants from p (Problem.weighted, Problem.obstacles, target_index)
  C.p = p;
  C.w1 = P_.w1p >= 0 ? p[P_.w1p] : P_.w1;
  C.w2 = P_.w2p >= 0 ? p[P_.w2p] : P_.w2;
  C.xt = p[P_.nx];
  C.yt = p[P_.nx + 1];
  for (int j = 0; j < P_.nobs; ++j) {
    C.ox[j] = P_.oxp[j] >= 0 ? p[P_.oxp[j]] : P_.ox[j];
    C.oy[j] = P_.oyp[j] >= 0 ? p[P_.oyp[j]] : P_.oy[j];
  }
  const Vec w0in(w0p, w0p + n);
  R.x.assign(n, 0.0); R.g.assign(m, 0.0); R.lam_x.assign(n, 0.0); R.lam_g.assign(m, 0.0);
  eqm.assign(m, 0); eqi.clear(); gE.assign(m, 0.0);
  for (int r = 0; r < m; ++r) {
    if (std::fabs(lbgp[r]) < INF && lbgp[r] == ubgp[r]) { eqm[r] = 1; eqi.push_back(r); gE[r] = lbgp[r]; }
  }
  neq = (int)eqi.size();
  if (neq > MEQ) {  // more equality rows than the kernel's Schur step holds: Invalid_Problem_Definition
    R.status = ST_EQ; R.iter = 0; R.x = w0in;
    return;
  }
  xlm.assign(n, 0); xum.assign(n, 0); slm.assign(m, 0); sum_.assign(m, 0); fixd.assign(n, 0);
  // fixed variables (lbx == ubx): IPOPT's default make_parameter -- held at the bound,
  // no bounds / multipliers / step, out of the scaling maxima and error norms (oracle)
  Vec w0 = w0in;
  nf = n;
  for (int i = 0; i < n; ++i) {
    fixd[i] = std::fabs(lbxp[i]) < INF && lbxp[i] == ubxp[i];
    if (fixd[i]) { w0[i] = lbxp[i]; --nf; }
    xlm[i] = lbxp[i] > -INF && !fixd[i];
    xum[i] = ubxp[i] < INF && !fixd[i];
  }
  ric.fix = fixd.data();
  for (int r = 0; r < m; ++r) { slm[r] = lbgp[r] > -INF && !eqm[r]; sum_[r] = ubgp[r] < INF && !eqm[r]; }
  xl = relax(lbxp, n, -1.0); xu = relax(ubxp, n, +1.0);
  gl_ = relax(lbgp, m, -1.0); gu_ = relax(ubgp, m, +1.0);
  dampxl.assign(n, 0.0); dampxu.assign(n, 0.0); dampsl.assign(m, 0.0); dampsu.assign(m, 0.0);
  for (int i = 0; i < n; ++i) { dampxl[i] = xlm[i] && !xum[i]; dampxu[i] = xum[i] && !xlm[i]; }
  for (int r = 0; r < m; ++r) { dampsl[r] = slm[r] && !sum_[r]; dampsu[r] = sum_[r] && !slm[r]; }

  auto finish = [&](const Vec& x, int it, int status, const Vec& zl, const Vec& zu, const Vec& y) {
    // oracle _result: honor_original_bounds, re-evaluate, unscale the multipliers
    Ev e; e.size(P_);
    for (int i = 0; i < n; ++i) R.x[i] = std::min(std::max(x[i], lbxp[i]), ubxp[i]);
    eval(R.x.data(), e, false);
    R.F = e.F; R.g = e.g; R.status = status; R.iter = it;
    for (int i = 0; i < n; ++i) R.lam_x[i] = (zu[i] - zl[i]) / df;
    for (int r = 0; r < m; ++r) R.lam_g[r] = y[r] * dc[r] / df;
  };

  // gradient-based scaling at the user's starting point
  Ev ev; ev.size(P_);
  eval(w0.data(), ev, true);
  Vec gradF(n, 0.0);
  adjoint(P_, ev, 1.0, nullptr, nullptr, gradF.data());
  // row maxima of J = G_k Z_k (explicit forward sensitivities, oracle SSEval.J)
  Vec rowmax(m, 0.0);
  bool jfin = true;
  {
    const int N = P_.N, nx = P_.nx, nu = P_.nu;
    Vec Z((N + 1) * 8 * n, 0.0);
    for (int k = 0; k < N; ++k) {  // Z_{k+1} = A_k Z_k + B_k E_k
      const AB ab = dyn_ab(P_, ev.trig.data() + k * 5);
      const double* Zk = Z.data() + k * 8 * n;
      double* Zn = Z.data() + (k + 1) * 8 * n;
      for (int i = 0; i < nx; ++i)
        for (int c = 0; c < n; ++c) Zn[i * n + c] = Zk[i * n + c];
      for (int c = 0; c < n; ++c) {
        Zn[0 * n + c] += ab.E03 * Zk[3 * n + c] + ab.E04 * Zk[4 * n + c];
        Zn[1 * n + c] += ab.E13 * Zk[3 * n + c] + ab.E14 * Zk[4 * n + c];
        Zn[2 * n + c] += ab.E23 * Zk[3 * n + c];
      }
      Zn[0 * n + nu * k] += ab.b0;
      Zn[1 * n + nu * k] += ab.b1;
      Zn[2 * n + nu * k] += ab.b2;
      for (int a = 1; a < nu; ++a) Zn[(2 + a) * n + nu * k + a] += ab.T;
    }
    for (int k = 1; k <= N; ++k) {
      const double* Zk = Z.data() + k * 8 * n;
      for (int i = 0; i < P_.mr; ++i) {
        double mx = 0.0;
        for (int c = 0; c < n; ++c) {
          if (fixd[c]) continue;
          double v;
          if (i < P_.nb) {
            v = Zk[P_.bs[i] * n + c];
          } else {
            const double* og = ev.og.data() + (k * MAXOBS + i - P_.nb) * 2;
            v = og[0] * Zk[0 * n + c] + og[1] * Zk[1 * n + c];
          }
          if (!std::isfinite(v)) jfin = false;
          mx = std::max(mx, std::fabs(v));
        }
        rowmax[k * P_.mr + i] = mx;
      }
    }
  }
  dc.assign(m, 1.0);
  df = 1.0;
  bool gfin = true;
  for (int i = 0; i < n; ++i)
    if (!fixd[i] && !std::isfinite(gradF[i])) gfin = false;
  if (!(gfin && jfin)) {
    Vec zz(n, 0.0), zm(m, 0.0);
    finish(w0, 0, ST_INVALID, zz, zz, zm);
    return;
  }
  double gmax = 0.0;
  for (int i = 0; i < n; ++i)
    if (!fixd[i]) gmax = std::max(gmax, std::fabs(gradF[i]));
  if (gmax > o.nlp_scaling_max_gradient) df = o.nlp_scaling_max_gradient / gmax;
  df = std::max(df, o.nlp_scaling_min_value);
  double rmx = 0.0;
  for (double v : rowmax) rmx = std::max(rmx, v);
  if (m && rmx > o.nlp_scaling_max_gradient) {
    for (int r = 0; r < m; ++r) {
      dc[r] = std::min(1.0, rowmax[r] > 0 ? o.nlp_scaling_max_gradient / rowmax[r] : PINF);
      dc[r] = std::max(dc[r], o.nlp_scaling_min_value);
    }
  }
  dl.assign(m, 0.0); du.assign(m, 0.0);
  for (int r = 0; r < m; ++r) {
    dl[r] = slm[r] ? dc[r] * gl_[r] : -PINF;
    du[r] = sum_[r] ? dc[r] * gu_[r] : PINF;
  }

  // initial point
  Vec x = w0;
  push(x, xl, xu, xlm, xum, o.bound_push, o.bound_frac);
  eval(x.data(), ev, true);
  Vec s(m);
  for (int r = 0; r < m; ++r) s[r] = dc[r] * ev.g[r];
  push(s, dl, du, slm, sum_, o.slack_bound_push, o.slack_bound_frac);
  for (int e = 0; e < neq; ++e) s[eqi[e]] = dc[eqi[e]] * gE[eqi[e]];  // pinned at the scaled target
  Vec zl(n), zu(n), vl(m), vu(m), y(m, 0.0);
  for (int i = 0; i < n; ++i) { zl[i] = xlm[i] ? o.bound_mult_init_val : 0.0; zu[i] = xum[i] ? o.bound_mult_init_val : 0.0; }
  for (int r = 0; r < m; ++r) { vl[r] = slm[r] ? o.bound_mult_init_val : 0.0; vu[r] = sum_[r] ? o.bound_mult_init_val : 0.0; }
  if (o.constr_mult_init_max > 0 && m > 0) main_ls_mults(ev, zl, zu, vl, vu, o.constr_mult_init_max, y);
  double mu = o.mu_init;
  double tau = std::max(o.tau_min, 1.0 - mu);
  nzx = nzs = 0;
  for (int i = 0; i < n; ++i) nzx += xlm[i] + xum[i];
  for (int r = 0; r < m; ++r) nzs += slm[r] + sum_[r];

  double f = df * ev.F;
  Vec d(m);
  for (int r = 0; r < m; ++r) d[r] = dc[r] * ev.g[r];
  std::vector<std::pair<double, double>> filt;
  bool have_tmax = false;
  double theta_max = 0, theta_min = 0;
  double delta_last = 0.0, delta_curr = 0.0;
  bool in_soft_resto = false, tiny_step_flag = false;
  int soft_resto_counter = 0, acc_counter = 0;
  double last_obj = -1e50, curr_obj = -1e50;
  int last_obj_iter = -1, it = 0, status = ST_NONE;
  bool have_acc = false;
  Vec acc_x, acc_zl, acc_zu, acc_y;
  // watchdog
  int wd_cnt = 0, wd_trial = 0;
  bool in_wd = false;
  double wd_alpha = 1.0;
  struct WdPoint {
    Vec x, s, y, zl, zu, vl, vu;
    Ev ev;
    Step step;
    double theta_ref, phi_ref, gBD;
  } wdp;
  const int wd_trigger = (int)o.watchdog_shortened_iter_trigger, wd_max = (int)o.watchdog_trial_iter_max;

  Vec glx, gls, Sxl, Sxu, Ssl, Ssu, SigX, SigS, gphi, gphib, rs, rd, D, gf(n);
  Step step, soc;
  step.size(n, m); soc.size(n, m);
  Trial tri, cur, tmp;
  tri.ev.size(P_); cur.ev.size(P_); tmp.ev.size(P_);

  auto nlp_error = [&](double& dinf, double& cviol, double& cmp) {
    double sd, sc;
    err_scaling(y, zl, zu, vl, vu, sd, sc);
    grad_lag(ev, y, zl, zu, vl, vu, glx, gls);
    dinf = std::max(amax(glx), amax(gls));
    cviol = cviol_scaled(d, s);
    cmp = compl_max(x, s, zl, zu, vl, vu, 0.0);
    return std::max(std::max(dinf / sd, cviol), cmp / sc);
  };
  auto barrier_error = [&](double mu_) {
    double sd, sc;
    err_scaling(y, zl, zu, vl, vu, sd, sc);
    grad_lag(ev, y, zl, zu, vl, vu, glx, gls);
    const double dinf = std::max(amax(glx), amax(gls));
    double pr = 0.0;
    for (int r = 0; r < m; ++r) pr = std::max(pr, std::fabs(d[r] - s[r]));
    return std::max(std::max(dinf / sd, pr), compl_max(x, s, zl, zu, vl, vu, mu_) / sc);
  };
  // primal-dual error at an arbitrary point (soft restoration)
  auto pd_error = [&](const Vec& x_, const Vec& s_, const Vec& d_, const Ev& ev_, const Vec& y_, const Vec& zl_,
                      const Vec& zu_, const Vec& vl_, const Vec& vu_, double mu_) {
    Vec gx, gs;
    grad_lag(ev_, y_, zl_, zu_, vl_, vu_, gx, gs);
    const double dual = (sumabs(gx) + sumabs(gs)) / (nf + m - neq);
    double prim = 0.0;
    for (int r = 0; r < m; ++r) prim += std::fabs(d_[r] - s_[r]);
    prim = m ? prim / m : 0.0;
    double cs = 0.0;
    compl_max(x_, s_, zl_, zu_, vl_, vu_, mu_, &cs);
    const int nc = nzx + nzs;
    return dual + prim + (nc ? cs / nc : 0.0);
  };

  while (true) {
    // ---------------- convergence check
    double dinf, cviol, cmp;
    const double err = nlp_error(dinf, cviol, cmp);
    if (!std::isfinite(err)) { status = ST_INVALID; break; }
    const double u_dinf = dinf / df, u_cviol = cviol_unscaled(d), u_cmp = cmp / df;
    if (err <= o.tol && u_dinf <= o.dual_inf_tol && u_cviol <= o.constr_viol_tol && u_cmp <= o.compl_inf_tol) {
      status = ST_OK;
      break;
    }
    if (it != last_obj_iter) { last_obj = curr_obj; curr_obj = f; last_obj_iter = it; }
    const bool acceptable = err <= o.acceptable_tol && u_dinf <= o.acceptable_dual_inf_tol &&
                            u_cviol <= o.acceptable_constr_viol_tol && u_cmp <= o.acceptable_compl_inf_tol &&
                            std::fabs(curr_obj - last_obj) / std::max(1.0, std::fabs(curr_obj)) <=
                                o.acceptable_obj_change_tol;
    if (o.acceptable_iter > 0 && acceptable) {
      if (++acc_counter >= o.acceptable_iter) { status = ST_ACC; break; }
    } else {
      acc_counter = 0;
    }
    if (it >= o.max_iter) { status = ST_MAXIT; break; }
    if (acceptable) { have_acc = true; acc_x = x; acc_zl = zl; acc_zu = zu; acc_y = y; }

    // ---------------- barrier parameter update
    {
      double sub_err = barrier_error(mu);
      bool done = false, tsf = tiny_step_flag;
      while ((sub_err <= o.barrier_tol_factor * mu || tsf) && !done) {
        double new_mu = std::min(o.kappa_mu * mu, std::pow(mu, o.theta_mu));
        new_mu = std::max(new_mu, std::min(o.tol, o.compl_inf_tol) / (o.barrier_tol_factor + 1.0));
        const bool changed = new_mu != mu;
        if (!changed && tsf) { status = ST_TINY; break; }
        mu = new_mu;
        tau = std::max(o.tau_min, 1.0 - mu);
        if (!changed) {
          done = true;
        } else {
          sub_err = barrier_error(mu);
          done = sub_err > o.barrier_tol_factor * mu;
        }
        if (done && changed) { filt.clear(); in_soft_resto = false; }
        tsf = false;
      }
      if (status != ST_NONE) break;
    }
    tiny_step_flag = false;

    // ---------------- search direction
    slacks(x, s, Sxl, Sxu, Ssl, Ssu);
    SigX.assign(n, 0.0); SigS.assign(m, 0.0); gphib.assign(n, 0.0); rs.assign(m, 0.0); rd.assign(m, 0.0);
    const double kdm = o.kappa_d * mu;
    for (int i = 0; i < n; ++i) {
      SigX[i] = (xlm[i] ? zl[i] / Sxl[i] : 0.0) + (xum[i] ? zu[i] / Sxu[i] : 0.0);
      gphib[i] = -(xlm[i] ? mu / Sxl[i] : 0.0) + (xum[i] ? mu / Sxu[i] : 0.0) + kdm * (dampxl[i] - dampxu[i]);
    }
    for (int r = 0; r < m; ++r) {
      SigS[r] = (slm[r] ? vl[r] / Ssl[r] : 0.0) + (sum_[r] ? vu[r] / Ssu[r] : 0.0);
      rs[r] = -y[r] - (slm[r] ? mu / Ssl[r] : 0.0) + (sum_[r] ? mu / Ssu[r] : 0.0) + kdm * (dampsl[r] - dampsu[r]);
      rd[r] = d[r] - s[r];
    }
    std::fill(gf.begin(), gf.end(), 0.0);
    adjoint(P_, ev, df, nullptr, nullptr, gf.data());
    gphi.resize(n);
    for (int i = 0; i < n; ++i) gphi[i] = (gf[i] - (xlm[i] ? mu / Sxl[i] : 0.0) + (xum[i] ? mu / Sxu[i] : 0.0)) + kdm * (dampxl[i] - dampxu[i]);
    hess_blocks(P_, ev, df, y.data(), dc.data(), Qb.data(), Sb.data());
    if (delta_curr > 0) delta_last = delta_curr;
    double delta = 0.0;
    bool fact = false;
    Vec Rd(n);
    D.assign(m, 0.0);
    while (true) {
      for (int r = 0; r < m; ++r) D[r] = eqm[r] ? 0.0 : SigS[r] + delta;  // equality rows: no slack
      for (int i = 0; i < n; ++i) Rd[i] = SigX[i] + delta;
      Qw = Qb;
      add_rows(P_, ev, D.data(), dc.data(), Qw.data());
      ric.sgn = neq > 0;  // with equality rows: signed pivots and the augmented system's inertia
      if (ric.factor(P_, ev, Qw.data(), Sb.data(), Rd.data()) && (neq == 0 || eq_schur(ev, mu, true))) {
        fact = true;
        break;
      }
      if (delta == 0.0) {
        delta = delta_last == 0.0 ? o.first_hessian_perturbation
                                  : std::max(o.min_hessian_perturbation, delta_last * o.perturb_dec_fact);
      } else {
        if (delta_last == 0.0 || 1e5 * delta_last < delta) delta *= o.perturb_inc_fact_first;
        else delta *= o.perturb_inc_fact;
      }
      if (delta > o.max_hessian_perturbation) { fact = false; break; }
    }
    delta_curr = delta;
    if (!fact) { status = ST_STEPERR; break; }
    for (int r = 0; r < m; ++r) D[r] = eqm[r] ? 0.0 : SigS[r] + delta;
    // solve_dir(rd_): uses the current y, ev (J), zl..vu (late binding as in the oracle)
    auto solve_dir = [&](const Vec& rd_, Step& st) {
      Vec v(m);
      for (int r = 0; r < m; ++r) v[r] = eqm[r] ? y[r] : y[r] + D[r] * rd_[r] + rs[r];
      for (int k = 0; k <= P_.N; ++k) {
        double a[8];
        for (int i = 0; i < 8; ++i) a[i] = df * ev.gl[k * 8 + i];
        add_GT(P_, ev, k, v.data(), dc.data(), a);
        for (int i = 0; i < 8; ++i) qv[k * 8 + i] = a[i];
      }
      ric.solve(P_, ev, qv.data(), gphib.data(), st.dx.data(), dXs.data());
      jmul(P_, ev, st.dx.data(), dc.data(), st.ds.data(), dXs.data());
      Vec dyc;
      if (neq) {  // [H J_c^T; J_c -delta_c I] [dx; dy_c] = [rhs; -c]: dy_c = (S + delta_c)^-1 (c + J_c dx0)
        Vec rhs(neq);
        for (int e = 0; e < neq; ++e) rhs[e] = rd_[eqi[e]] + st.ds[eqi[e]];
        eq_solve(rhs, dyc);
        for (int e = 0; e < neq; ++e)
          for (int i = 0; i < n; ++i) st.dx[i] += dyc[e] * dxe[e][i];
        jmul(P_, ev, st.dx.data(), dc.data(), st.ds.data(), dXs.data());
      }
      for (int r = 0; r < m; ++r) {
        st.ds[r] = eqm[r] ? 0.0 : st.ds[r] + rd_[r];
        st.dy[r] = D[r] * st.ds[r] + rs[r];
        st.dvl[r] = slm[r] ? mu / Ssl[r] - vl[r] - vl[r] / Ssl[r] * st.ds[r] : 0.0;
        st.dvu[r] = sum_[r] ? mu / Ssu[r] - vu[r] + vu[r] / Ssu[r] * st.ds[r] : 0.0;
      }
      for (int e = 0; e < neq; ++e) st.dy[eqi[e]] = dyc[e];
      for (int i = 0; i < n; ++i) {
        st.dzl[i] = xlm[i] ? mu / Sxl[i] - zl[i] - zl[i] / Sxl[i] * st.dx[i] : 0.0;
        st.dzu[i] = xum[i] ? mu / Sxu[i] - zu[i] + zu[i] / Sxu[i] * st.dx[i] : 0.0;
      }
    };
    solve_dir(rd, step);

    // ---------------- line search
    double theta_ref = 0.0;
    for (int r = 0; r < m; ++r) theta_ref += std::fabs(rd[r]);
    double phi_ref = barrier_obj(f, x, s, mu);
    Vec gphi_s(m);
    for (int r = 0; r < m; ++r)
      gphi_s[r] = (-(slm[r] ? mu / Ssl[r] : 0.0) + (sum_[r] ? mu / Ssu[r] : 0.0)) + kdm * (dampsl[r] - dampsu[r]);
    double gBD = 0.0;
    {
      double a = 0.0, b = 0.0;
      for (int i = 0; i < n; ++i) a += gphi[i] * step.dx[i];
      for (int r = 0; r < m; ++r) b += gphi_s[r] * step.ds[r];
      gBD = a + b;
    }
    if (!have_tmax) {
      have_tmax = true;
      theta_max = o.theta_max_fact * std::max(1.0, theta_ref);
      theta_min = o.theta_min_fact * std::max(1.0, theta_ref);
    }
    auto is_ftype = [&](double a) {
      return gBD < 0.0 && a * std::pow(-gBD, o.s_phi) > o.delta * std::pow(theta_ref, o.s_theta);
    };
    auto armijo = [&](double a, double phi_t) { return compare_le(phi_t - phi_ref, o.eta_phi * a * gBD, phi_ref); };
    auto acceptable_to_iterate = [&](double phi_t, double th_t) {
      if (phi_t > phi_ref) {
        double basval = 1.0;
        if (std::fabs(phi_ref) > 10.0) basval = std::log10(std::fabs(phi_ref));
        if (std::log10(phi_t - phi_ref) > o.obj_max_inc + basval) return false;
      }
      return compare_le(th_t, (1.0 - o.gamma_theta) * theta_ref, theta_ref) ||
             compare_le(phi_t - phi_ref, -o.gamma_phi * theta_ref, phi_ref);
    };
    auto filter_ok = [&](double phi_t, double th_t) {
      for (auto& e : filt)
        if (!(phi_t <= e.first || th_t <= e.second)) return false;
      return true;
    };
    auto check_accept = [&](double a_test, double phi_t, double th_t) {
      if (th_t > theta_max) return false;
      bool ok;
      if (a_test > 0.0 && is_ftype(a_test) && theta_ref <= theta_min) ok = armijo(a_test, phi_t);
      else ok = acceptable_to_iterate(phi_t, th_t);
      if (!ok) return false;
      return filter_ok(phi_t, th_t);
    };
    // trial point into T; false = evaluation error (oracle returns None)
    auto trial = [&](double a, const Vec& dx_, const Vec& ds_, Trial& T) {
      T.x.resize(n); T.s.resize(m); T.d.resize(m);
      for (int i = 0; i < n; ++i) T.x[i] = x[i] + a * dx_[i];
      for (int r = 0; r < m; ++r) T.s[r] = s[r] + a * ds_[r];
      eval(T.x.data(), T.ev, false);  // derivatives only once a point is taken
      T.f = df * T.ev.F;
      for (int r = 0; r < m; ++r) T.d[r] = dc[r] * T.ev.g[r];
      if (!(std::isfinite(T.f) && allfinite(T.d))) return false;
      T.phi = barrier_obj(T.f, T.x, T.s, mu);
      double th = 0.0;
      for (int r = 0; r < m; ++r) th += std::fabs(T.d[r] - T.s[r]);
      T.th = th;
      return (bool)std::isfinite(T.phi);
    };
    // accepted point bookkeeping
    enum Kind { K_NONE, K_REG, K_SOFT, K_RESTO };
    Kind kind = K_NONE;
    double alpha_p = 0.0, alpha_d = 0.0;
    const Step* acc_step = nullptr;
    Trial* acc_tri = nullptr;
    // soft-restoration result
    Vec s_y, s_zl, s_zu, s_vl, s_vu;
    auto try_soft_resto = [&](const Step& st, bool& orig) {
      const double ap = frac_to_bound(tau, x, s, st.dx, st.ds);
      const double ad = dual_frac_to_bound(tau, zl, zu, vl, vu, st.dzl, st.dzu, st.dvl, st.dvu);
      const double a = std::min(ap, ad);
      if (!trial(a, st.dx, st.ds, tmp)) return false;
      eval(tmp.x.data(), tmp.ev, true);
      s_y.resize(m); s_zl.resize(n); s_zu.resize(n); s_vl.resize(m); s_vu.resize(m);
      for (int r = 0; r < m; ++r) { s_y[r] = y[r] + a * st.dy[r]; s_vl[r] = vl[r] + a * st.dvl[r]; s_vu[r] = vu[r] + a * st.dvu[r]; }
      for (int i = 0; i < n; ++i) { s_zl[i] = zl[i] + a * st.dzl[i]; s_zu[i] = zu[i] + a * st.dzu[i]; }
      const double e_t = pd_error(tmp.x, tmp.s, tmp.d, tmp.ev, s_y, s_zl, s_zu, s_vl, s_vu, mu);
      const double e_c = pd_error(x, s, d, ev, y, zl, zu, vl, vu, mu);
      if (e_t <= o.soft_resto_pderror_reduction_factor * e_c) {
        orig = check_accept(0.0, tmp.phi, tmp.th);
        alpha_p = alpha_d = a;
        return true;
      }
      return false;
    };
    // line_search(skip_first): returns accepted?, and n_steps / trials / soc / a_test / ev_err / wtri
    int n_steps = 0, ls_trials = 0;
    bool soc_taken = false;
    double a_test = 0.0;
    bool ev_err = false, have_wtri = false;
    const Step* cur_step = &step;
    auto line_search = [&](bool skip_first) -> bool {
      const Vec& dx_ = cur_step->dx;
      const Vec& ds_ = cur_step->ds;
      const double amax_p = frac_to_bound(tau, x, s, dx_, ds_);
      n_steps = 0; soc_taken = false; ev_err = false; have_wtri = false;
      if (in_wd) {
        ls_trials += 1;
        const bool okt = trial(amax_p, dx_, ds_, tri);
        a_test = wd_alpha;
        if (okt && check_accept(wd_alpha, tri.phi, tri.th)) {
          alpha_p = amax_p; acc_step = cur_step; acc_tri = &tri;
          return true;
        }
        ev_err = !okt;
        have_wtri = okt;
        return false;
      }
      double amin = o.gamma_theta;
      if (gBD < 0) {
        amin = std::min(o.gamma_theta, o.gamma_phi * theta_ref / (-gBD));
        if (theta_ref <= theta_min) amin = std::min(amin, o.delta * std::pow(theta_ref, o.s_theta) / std::pow(-gBD, o.s_phi));
      }
      amin *= o.alpha_min_frac;
      double a = amax_p * (skip_first ? o.alpha_red_factor : 1.0);
      int nn_ = 0;
      while (a > amin || nn_ == 0) {
        ls_trials += 1;
        const bool okt = trial(a, dx_, ds_, tri);
        if (okt && check_accept(a, tri.phi, tri.th)) {
          n_steps = nn_; a_test = a; alpha_p = a; acc_step = cur_step; acc_tri = &tri;
          return true;
        }
        if (okt && a == amax_p && theta_ref <= tri.th && o.max_soc > 0) {
          // second-order correction (FilterLSAcceptor::TrySecondOrderCorrection)
          double th_tr = tri.th, th_old = 0.0, a_soc = a;
          Vec dms = rd;
          int cnt = 0;
          Trial* cp = &tri;
          while (cnt < o.max_soc && (cnt == 0 || th_tr <= o.kappa_soc * th_old)) {
            th_old = th_tr;
            for (int r = 0; r < m; ++r) dms[r] = a_soc * dms[r] + (cp->d[r] - cp->s[r]);
            solve_dir(dms, soc);
            a_soc = frac_to_bound(tau, x, s, soc.dx, soc.ds);
            Trial* nx_ = (cp == &cur) ? &tri : &cur;
            ls_trials += 1;
            const bool ok2 = trial(a_soc, soc.dx, soc.ds, *nx_);
            cp = nx_;
            if (!ok2) break;
            if (check_accept(a, cp->phi, cp->th)) {
              n_steps = nn_; a_test = a; soc_taken = true; alpha_p = a_soc; acc_step = &soc; acc_tri = cp;
              return true;
            }
            cnt += 1;
            th_tr = cp->th;
          }
        }
        a *= o.alpha_red_factor;
        nn_ += 1;
      }
      n_steps = nn_; a_test = a;
      return false;
    };

    // tiny step detection
    bool tiny;
    {
      double a1 = 0.0, a2 = 0.0, a3 = 0.0;
      for (int i = 0; i < n; ++i) a1 = std::max(a1, std::fabs(step.dx[i] / (1.0 + std::fabs(x[i]))));
      for (int r = 0; r < m; ++r) a2 = std::max(a2, std::fabs(step.ds[r] / (1.0 + std::fabs(s[r]))));
      for (int r = 0; r < m; ++r) a3 = std::max(a3, std::fabs(rd[r]));
      tiny = a1 <= o.tiny_step_tol && a2 <= o.tiny_step_tol && a3 <= 1e-4;
    }
    auto restore_wd = [&]() {  // StopWatchDog: back to the stored point, step and reference values
      x = wdp.x; s = wdp.s; y = wdp.y; zl = wdp.zl; zu = wdp.zu; vl = wdp.vl; vu = wdp.vu;
      ev = wdp.ev; step = wdp.step;
      theta_ref = wdp.theta_ref; phi_ref = wdp.phi_ref; gBD = wdp.gBD;
      f = df * ev.F;
      for (int r = 0; r < m; ++r) d[r] = dc[r] * ev.g[r];
    };
    if (in_wd && tiny) {
      restore_wd();
      in_wd = false; wd_cnt = 0; tiny = false;
    }
    if (wd_trigger > 0 && !in_wd && !tiny && !in_soft_resto && wd_cnt >= wd_trigger) {
      wdp.x = x; wdp.s = s; wdp.y = y; wdp.zl = zl; wdp.zu = zu; wdp.vl = vl; wdp.vu = vu;
      wdp.ev = ev; wdp.step = step; wdp.theta_ref = theta_ref; wdp.phi_ref = phi_ref; wdp.gBD = gBD;
      wd_alpha = frac_to_bound(tau, x, s, step.dx, step.ds);
      wd_trial = 0; in_wd = true;
    }
    if (in_wd) { theta_ref = wdp.theta_ref; phi_ref = wdp.phi_ref; gBD = wdp.gBD; }
    bool wd_forced = false;
    if (in_soft_resto) {
      soft_resto_counter += 1;
      if (soft_resto_counter <= o.max_soft_resto_iters) {
        bool orig = false;
        if (try_soft_resto(step, orig)) {
          kind = K_SOFT;
          if (orig) in_soft_resto = false;
        }
      }
    } else if (tiny) {
      const double a = frac_to_bound(tau, x, s, step.dx, step.ds);
      if (trial(a, step.dx, step.ds, tri)) {
        kind = K_REG; alpha_p = a; acc_step = &step; acc_tri = &tri;
        tiny_step_flag = true;
      }
    } else {
      bool skip_first = false;
      bool acc = false;
      while (true) {
        acc = line_search(skip_first);
        if (!in_wd) break;
        if (acc) { in_wd = false; break; }
        wd_trial += 1;
        if (ev_err || wd_trial > wd_max) {
          restore_wd();
          cur_step = &step;
          in_wd = false; wd_cnt = 0; skip_first = true;
          continue;
        }
        // a watchdog trial iteration: the full step is taken unchecked
        alpha_p = frac_to_bound(tau, x, s, step.dx, step.ds);
        acc_step = &step; acc_tri = &tri;
        acc = true;
        wd_forced = true;
        break;
      }
      if (acc) kind = K_REG;
      if (!acc) {
        bool orig = false;
        if (try_soft_resto(step, orig)) {
          kind = K_SOFT;
          if (!orig) { in_soft_resto = true; soft_resto_counter = 0; }
        }
      } else if (!wd_forced) {
        const double phi_acc = acc_tri->phi;
        if (!(is_ftype(a_test) && armijo(a_test, phi_acc)))
          filt.emplace_back(phi_ref - o.gamma_phi * theta_ref, (1.0 - o.gamma_theta) * theta_ref);
      }
    }
    if (kind == K_REG) wd_cnt = n_steps == 0 ? 0 : wd_cnt + 1;

    if (kind == K_NONE) {
      // feasibility restoration phase
      if (theta_ref <= 1e-2 * o.tol) {
        if (have_acc) { x = acc_x; zl = acc_zl; zu = acc_zu; y = acc_y; status = ST_ACC; }
        else status = ST_RESTOFAIL;
        break;
      }
      filt.emplace_back(phi_ref - o.gamma_phi * theta_ref, (1.0 - o.gamma_theta) * theta_ref);
      RestoOut ro;
      restoration(x, s, d, ev, y, zl, zu, vl, vu, mu, tau, theta_ref, phi_ref, filt, it, ro);
      it = ro.it;
      if (ro.status != ST_NONE) { status = ro.status; x = ro.x; break; }
      x = ro.x; s = ro.s; ev = ro.ev; y = ro.y; zl = ro.zl; zu = ro.zu; vl = ro.vl; vu = ro.vu;
      f = df * ev.F;
      for (int r = 0; r < m; ++r) d[r] = dc[r] * ev.g[r];
      in_soft_resto = false;
      wd_cnt = 0;
      kind = K_RESTO;
    }
    if (kind == K_REG) {
      const Step& st = *acc_step;
      x = acc_tri->x; s = acc_tri->s; std::swap(ev, acc_tri->ev); f = acc_tri->f; d = acc_tri->d;
      if (!ev.derivs) eval(x.data(), ev, true);
      alpha_d = dual_frac_to_bound(tau, zl, zu, vl, vu, st.dzl, st.dzu, st.dvl, st.dvu);
      for (int r = 0; r < m; ++r) y[r] = y[r] + alpha_p * st.dy[r];
      for (int i = 0; i < n; ++i) { zl[i] = zl[i] + alpha_d * st.dzl[i]; zu[i] = zu[i] + alpha_d * st.dzu[i]; }
      for (int r = 0; r < m; ++r) { vl[r] = vl[r] + alpha_d * st.dvl[r]; vu[r] = vu[r] + alpha_d * st.dvu[r]; }
    } else if (kind == K_SOFT) {
      x = tmp.x; s = tmp.s; std::swap(ev, tmp.ev); f = tmp.f; d = tmp.d;
      y = s_y; zl = s_zl; zu = s_zu; vl = s_vl; vu = s_vu;
    }
    // kappa_sigma safeguard (IpoptAlgorithm::correct_bound_multiplier)
    slacks(x, s, Sxl, Sxu, Ssl, Ssu);
    const double ks = o.kappa_sigma;
    for (int i = 0; i < n; ++i) {
      zl[i] = xlm[i] ? std::max(std::min(zl[i], ks * mu / Sxl[i]), mu / (ks * Sxl[i])) : 0.0;
      zu[i] = xum[i] ? std::max(std::min(zu[i], ks * mu / Sxu[i]), mu / (ks * Sxu[i])) : 0.0;
    }
    for (int r = 0; r < m; ++r) {
      vl[r] = slm[r] ? std::max(std::min(vl[r], ks * mu / Ssl[r]), mu / (ks * Ssl[r])) : 0.0;
      vu[r] = sum_[r] ? std::max(std::min(vu[r], ks * mu / Ssu[r]), mu / (ks * Ssu[r])) : 0.0;
    }
    if (kind != K_RESTO) it += 1;
    if (dbg_trace_) {  // NMPC_CPU_TRACE: per-iteration record on stderr (parity diagnostics)
      double ymax = 0.0;
      for (int r = 0; r < m; ++r) ymax = std::max(ymax, std::fabs(y[r]));
      std::fprintf(stderr, "cpu it %d kind %d mu %.17g f %.17g delta %.6g alpha_p %.17g ls %d soc %d in_wd %d ymax %.6g\n",
                   it, (int)kind, mu, f, delta_curr, alpha_p, ls_trials, (int)soc_taken, (int)in_wd, ymax);
    }
    (void)soc_taken; (void)ls_trials; (void)have_wtri;
  }
  finish(x, it, status, zl, zu, y);
}

// IPOPT's feasibility restoration phase (oracle restoration(); RestoMinC_1Nrm,
// RestoIpoptNLP, RestoIterateInitializer, RestoConvergenceCheck)
void Solver::restoration(const Vec& x0, const Vec& s0, const Vec& d0, const Ev& ev0, const Vec& y0, const Vec& zl0,
                         const Vec& zu0, const Vec& vl0, const Vec& vu0, double mu0, double tau0, double theta0,
                         double phi0, const std::vector<std::pair<double, double>>& ofilt, int it_, RestoOut& out) {
  (void)y0;
  const Opts& o = o_;
  const double rho = o.resto_penalty_parameter;
  ric.sgn = false;  // the restoration problem's condensed matrix must be positive definite
  const Vec xR = x0;
  Vec DR2(n);
  for (int i = 0; i < n; ++i) { const double a = 1.0 / std::max(1.0, std::fabs(xR[i])); DR2[i] = a * a; }
  Vec c0(m);
  for (int r = 0; r < m; ++r) c0[r] = d0[r] - s0[r];
  double muR = std::max(mu0, amax(c0));
  double tauR = std::max(o.tau_min, 1.0 - muR);
  Vec pp(m), nn(m);
  for (int r = 0; r < m; ++r) {
    const double qa = muR / (2.0 * rho) - 0.5 * c0[r];
    const double qb = c0[r] * muR / (2.0 * rho);
    nn[r] = qa + std::sqrt(qa * qa + qb);
    pp[r] = c0[r] + nn[r];
  }
  Vec xx = x0, ss = s0;
  Vec zlR(n), zuR(n), vlR(m), vuR(m), zp(m), zn(m);
  for (int i = 0; i < n; ++i) { zlR[i] = xlm[i] ? std::min(rho, zl0[i]) : 0.0; zuR[i] = xum[i] ? std::min(rho, zu0[i]) : 0.0; }
  for (int r = 0; r < m; ++r) {
    vlR[r] = slm[r] ? std::min(rho, vl0[r]) : 0.0;
    vuR[r] = sum_[r] ? std::min(rho, vu0[r]) : 0.0;
    zp[r] = muR / pp[r];
    zn[r] = muR / nn[r];
  }
  Ev evR = ev0;
  Vec dR = d0;
  auto eta = [&](double mu_) { return o.resto_proximity_weight * std::sqrt(mu_); };
  // least-squares multipliers of the restoration NLP; Jfull = [J, -I, I] with the
  // p, n blocks eliminated: (I + J^T J / 3) wx = bx_x + J^T (bs + (bx_p - bs - bx_n - bs) / 3);
  // an equality row has no slack, so two eliminated blocks: weight 1/2, y = comb - J wx / 2
  Vec yR(m, 0.0);
  if (o.constr_mult_init_max > 0 && m > 0) {
    Vec bxx(n), bs(m), comb(m), wx, jwx;
    for (int i = 0; i < n; ++i) bxx[i] = eta(muR) * DR2[i] * (xx[i] - xR[i]) - zlR[i] + zuR[i];
    for (int r = 0; r < m; ++r) {
      bs[r] = vuR[r] - vlR[r];
      const double rp_ = (rho - zp[r]) - bs[r], rn_ = (rho - zn[r]) + bs[r];
      comb[r] = eqm[r] ? ((rho - zp[r]) - (rho - zn[r])) / 2.0 : bs[r] + (rp_ - rn_) / 3.0;
    }
    if (neq == 0) {
      ls_solve(evR, 1.0 / 3.0, bxx, 0.0, comb, wx, jwx);
    } else {
      Vec wr(m);
      for (int r = 0; r < m; ++r) wr[r] = eqm[r] ? 0.5 : 1.0 / 3.0;
      ls_solve_w(evR, wr, bxx, 0.0, comb, wx, jwx, nullptr);
    }
    double ym = 0.0;
    for (int r = 0; r < m; ++r) {
      const double rp_ = (rho - zp[r]) - bs[r], rn_ = (rho - zn[r]) + bs[r];
      const double wp = (2 * rp_ + rn_ + jwx[r]) / 3.0, wn = (rp_ + 2 * rn_ - jwx[r]) / 3.0;
      yR[r] = eqm[r] ? comb[r] - jwx[r] / 2.0 : bs[r] - (jwx[r] - wp + wn);
      ym = std::max(ym, std::fabs(yR[r]));
    }
    if (ym > o.constr_mult_init_max) std::fill(yR.begin(), yR.end(), 0.0);
  }
  const int nzp = 2 * m;
  auto fR = [&](const Vec& x_, const Vec& p_, const Vec& n_, double mu_) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < m; ++r) a += p_[r] + n_[r];
    for (int i = 0; i < n; ++i) { const double dd = x_[i] - xR[i]; b += DR2[i] * dd * dd; }
    return rho * a + 0.5 * eta(mu_) * b;
  };
  auto phiR = [&](const Vec& x_, const Vec& s_, const Vec& p_, const Vec& n_, double mu_) {
    double val = fR(x_, p_, n_, mu_);
    double logs = 0.0, damp = 0.0, lpn = 0.0, spn = 0.0;
    for (int i = 0; i < n; ++i) {
      const double a = x_[i] - xl[i], b = xu[i] - x_[i];
      if (xlm[i]) { logs += std::log(a); damp += dampxl[i] * a; }
      if (xum[i]) { logs += std::log(b); damp += dampxu[i] * b; }
    }
    for (int r = 0; r < m; ++r) {
      const double a = s_[r] - dl[r], b = du[r] - s_[r];
      if (slm[r]) { logs += std::log(a); damp += dampsl[r] * a; }
      if (sum_[r]) { logs += std::log(b); damp += dampsu[r] * b; }
      lpn += std::log(p_[r]) + std::log(n_[r]);
      spn += p_[r] + n_[r];
    }
    val -= mu_ * (logs + lpn);
    val += o.kappa_d * mu_ * (damp + spn);
    return val;
  };
  auto thetaR = [&](const Vec& d_, const Vec& s_, const Vec& p_, const Vec& n_) {
    double t = 0.0;
    for (int r = 0; r < m; ++r) t += std::fabs(d_[r] - s_[r] - p_[r] + n_[r]);
    return t;
  };
  Vec glx(n), tmpn(n);
  // errR: (overall, dinf, cv, cm, sd, sc, pinf) of the restoration NLP
  auto errR = [&](double mu_, double mu_c, double* dinf_o, double* cv_o, double* cm_o, double* pinf_o) {
    std::fill(tmpn.begin(), tmpn.end(), 0.0);
    adjoint(P_, evR, 0.0, yR.data(), dc.data(), tmpn.data());
    const double et = eta(mu_);
    double dinf = 0.0;
    for (int i = 0; i < n; ++i)
      if (!fixd[i]) dinf = std::max(dinf, std::fabs(et * DR2[i] * (xx[i] - xR[i]) + tmpn[i] - zlR[i] + zuR[i]));
    for (int r = 0; r < m; ++r) {
      if (!eqm[r]) dinf = std::max(dinf, std::fabs(-yR[r] - vlR[r] + vuR[r]));
    }
    for (int r = 0; r < m; ++r) dinf = std::max(dinf, std::fabs(rho - yR[r] - zp[r]));
    for (int r = 0; r < m; ++r) dinf = std::max(dinf, std::fabs(rho + yR[r] - zn[r]));
    double cv = 0.0, pinf = 0.0;
    for (int r = 0; r < m; ++r) {
      const double dr = dR[r] - pp[r] + nn[r];
      if (slm[r]) cv = std::max(cv, std::max(0.0, dl[r] - dr));
      if (sum_[r]) cv = std::max(cv, std::max(0.0, dr - du[r]));
      if (eqm[r]) cv = std::max(cv, std::fabs(dr - ss[r]));
      pinf = std::max(pinf, std::fabs(dR[r] - ss[r] - pp[r] + nn[r]));
    }
    double cm = compl_max(xx, ss, zlR, zuR, vlR, vuR, mu_c);
    for (int r = 0; r < m; ++r) cm = std::max(cm, std::fabs(pp[r] * zp[r] - mu_c));
    for (int r = 0; r < m; ++r) cm = std::max(cm, std::fabs(nn[r] * zn[r] - mu_c));
    const double smax = o.s_max;
    const double bz = sumabs(zlR) + sumabs(zuR) + sumabs(vlR) + sumabs(vuR) + sumabs(zp) + sumabs(zn);
    const int nd = m + nzx + nzs + nzp, nc = nzx + nzs + nzp;
    double sd = (sumabs(yR) + bz) / nd;
    sd = std::max(smax, sd) / smax;
    double sc = bz / nc;
    sc = std::max(smax, sc) / smax;
    if (dinf_o) *dinf_o = dinf;
    if (cv_o) *cv_o = cv;
    if (cm_o) *cm_o = cm;
    if (pinf_o) *pinf_o = pinf;
    return std::max(std::max(dinf / sd, cv), cm / sc);
  };
  auto ftb_R = [&](double tau_, const Vec& dx_, const Vec& ds_, const Vec& dp_, const Vec& dn_) {
    double a = frac_to_bound(tau_, xx, ss, dx_, ds_);
    for (int r = 0; r < m; ++r)
      if (dp_[r] < 0) a = std::min(a, -tau_ * pp[r] / dp_[r]);
    for (int r = 0; r < m; ++r)
      if (dn_[r] < 0) a = std::min(a, -tau_ * nn[r] / dn_[r]);
    return a;
  };
  auto dftb_R = [&](double tau_, const RStep& st) {
    double a = dual_frac_to_bound(tau_, zlR, zuR, vlR, vuR, st.dzl, st.dzu, st.dvl, st.dvu);
    for (int r = 0; r < m; ++r)
      if (st.dzp[r] < 0) a = std::min(a, -tau_ * zp[r] / st.dzp[r]);
    for (int r = 0; r < m; ++r)
      if (st.dzn[r] < 0) a = std::min(a, -tau_ * zn[r] / st.dzn[r]);
    return a;
  };

  std::vector<std::pair<double, double>> rfilt;
  bool have_tm = false;
  double th_max = 0, th_min = 0, dlast = 0.0, dcurr = 0.0;
  bool first = true;
  int racc = 0, rlast_it = -1;
  double rlast_obj = -1e50, rcurr_obj = -1e50;
  int rwd_cnt = 0, rwd_trial = 0;
  bool rin_wd = false;
  double rwd_alpha = 1.0;
  struct RWd {
    Vec xx, ss, pp, nn, dR, yR, zlR, zuR, vlR, vuR, zp, zn;
    Ev evR;
    RStep stp;
    double th_ref, ph_ref, gbd;
  } rwd;
  const int wd_trigger = (int)o.watchdog_shortened_iter_trigger, wd_max = (int)o.watchdog_trial_iter_max;
  Vec Sxl, Sxu, Ssl, Ssu, SigX, SigS, Sp(m), Sn(m), gphi(n), rs_(m), rp(m), rn(m), cR(m), Dt(m), den(m), Spd(m), Snd(m);
  RStep stp, st2;
  stp.size(n, m); st2.size(n, m);
  RTrial rt1, rt2;
  rt1.ev.size(P_); rt2.ev.size(P_);
  Vec Rd(n), Dw(m), v(m);

  while (true) {
    // ---- progress w.r.t. the original problem (RestoConvergenceCheck)
    if (!first) {
      double th_o = 0.0;
      for (int r = 0; r < m; ++r) th_o += std::fabs(dR[r] - ss[r]);
      const double f_o = df * evR.F;
      // barrier_obj of the original problem at mu0
      double phi_o;
      {
        double logs = 0.0, damp = 0.0;
        for (int i = 0; i < n; ++i) {
          const double a = xx[i] - xl[i], b = xu[i] - xx[i];
          if (xlm[i]) logs += std::log(a);
          if (xum[i]) logs += std::log(b);
          if (xlm[i]) damp += dampxl[i] * a;
          if (xum[i]) damp += dampxu[i] * b;
        }
        double ls = 0.0, ds = 0.0;
        for (int r = 0; r < m; ++r) {
          const double a = ss[r] - dl[r], b = du[r] - ss[r];
          if (slm[r]) ls += std::log(a);
          if (sum_[r]) ls += std::log(b);
          if (slm[r]) ds += dampsl[r] * a;
          if (sum_[r]) ds += dampsu[r] * b;
        }
        phi_o = f_o - mu0 * (logs + ls) + o.kappa_d * mu0 * (damp + ds);
      }
      if (th_o <= o.required_infeasibility_reduction * theta0 && std::isfinite(phi_o)) {
        const bool ok = compare_le(th_o, (1.0 - o.gamma_theta) * theta0, theta0) ||
                        compare_le(phi_o - phi0, -o.gamma_phi * theta0, phi0);
        bool fok = true;
        for (auto& e : ofilt)
          if (!(phi_o <= e.first || th_o <= e.second)) { fok = false; break; }
        if (ok && fok) break;
      }
    }
    // ---- the restoration NLP's own termination
    double dinf_r, cv_r, cm_r;
    const double err_r = errR(muR, 0.0, &dinf_r, &cv_r, &cm_r, nullptr);
    if (!std::isfinite(err_r)) { out.status = ST_INVALID; out.it = it_; out.x = xx; return; }
    const bool conv = err_r <= o.tol && dinf_r <= o.dual_inf_tol && cv_r <= o.constr_viol_tol && cm_r <= o.compl_inf_tol;
    if (it_ != rlast_it) { rlast_obj = rcurr_obj; rcurr_obj = fR(xx, pp, nn, muR); rlast_it = it_; }
    const bool racc_ok = err_r <= o.acceptable_tol && dinf_r <= o.acceptable_dual_inf_tol &&
                         cv_r <= o.acceptable_constr_viol_tol && cm_r <= o.acceptable_compl_inf_tol &&
                         std::fabs(rcurr_obj - rlast_obj) / std::max(1.0, std::fabs(rcurr_obj)) <= o.acceptable_obj_change_tol;
    if (o.acceptable_iter > 0 && racc_ok) racc += 1;
    else racc = 0;
    if (conv || (o.acceptable_iter > 0 && racc >= o.acceptable_iter)) {
      if (cviol_unscaled(dR) > o.constr_viol_tol) { out.status = ST_INFEAS; out.it = it_; out.x = xx; return; }
      break;
    }
    if (it_ >= o.max_iter) { out.status = ST_MAXIT; out.it = it_; out.x = xx; return; }
    first = false;
    // ---- monotone barrier update of the restoration problem
    auto sub_err = [&](double mu_) {
      double pinf;
      errR(mu_, mu_, nullptr, nullptr, nullptr, &pinf);
      // dinf / cm at mu_ (errR's sd, sc are mu-independent)
      std::fill(tmpn.begin(), tmpn.end(), 0.0);
      adjoint(P_, evR, 0.0, yR.data(), dc.data(), tmpn.data());
      const double et = eta(mu_);
      double dinf = 0.0;
      for (int i = 0; i < n; ++i)
        if (!fixd[i]) dinf = std::max(dinf, std::fabs(et * DR2[i] * (xx[i] - xR[i]) + tmpn[i] - zlR[i] + zuR[i]));
      for (int r = 0; r < m; ++r) dinf = std::max(dinf, std::fabs(-yR[r] - vlR[r] + vuR[r]));
      for (int r = 0; r < m; ++r) dinf = std::max(dinf, std::fabs(rho - yR[r] - zp[r]));
      for (int r = 0; r < m; ++r) dinf = std::max(dinf, std::fabs(rho + yR[r] - zn[r]));
      double cm = compl_max(xx, ss, zlR, zuR, vlR, vuR, mu_);
      for (int r = 0; r < m; ++r) cm = std::max(cm, std::fabs(pp[r] * zp[r] - mu_));
      for (int r = 0; r < m; ++r) cm = std::max(cm, std::fabs(nn[r] * zn[r] - mu_));
      const double smax = o.s_max;
      const double bz = sumabs(zlR) + sumabs(zuR) + sumabs(vlR) + sumabs(vuR) + sumabs(zp) + sumabs(zn);
      const int nd = m + nzx + nzs + nzp, nc = nzx + nzs + nzp;
      double sd = (sumabs(yR) + bz) / nd;
      sd = std::max(smax, sd) / smax;
      double sc = bz / nc;
      sc = std::max(smax, sc) / smax;
      return std::max(std::max(dinf / sd, pinf), cm / sc);
    };
    {
      double se = sub_err(muR);
      bool done = false;
      while (se <= o.barrier_tol_factor * muR && !done) {
        double new_mu = std::min(o.kappa_mu * muR, std::pow(muR, o.theta_mu));
        new_mu = std::max(new_mu, std::min(o.tol, o.compl_inf_tol) / (o.barrier_tol_factor + 1.0));
        const bool changed = new_mu != muR;
        muR = new_mu;
        tauR = std::max(o.tau_min, 1.0 - muR);
        if (!changed) done = true;
        else { se = sub_err(muR); done = se > o.barrier_tol_factor * muR; }
        if (done && changed) rfilt.clear();
      }
    }
    // ---- Newton step (p, n eliminated per row)
    slacks(xx, ss, Sxl, Sxu, Ssl, Ssu);
    SigX.assign(n, 0.0); SigS.assign(m, 0.0);
    const double et = eta(muR), kdm = o.kappa_d * muR;
    for (int i = 0; i < n; ++i) {
      SigX[i] = (xlm[i] ? zlR[i] / Sxl[i] : 0.0) + (xum[i] ? zuR[i] / Sxu[i] : 0.0);
      gphi[i] = ((et * DR2[i] * (xx[i] - xR[i]) - (xlm[i] ? muR / Sxl[i] : 0.0)) + (xum[i] ? muR / Sxu[i] : 0.0)) +
                kdm * (dampxl[i] - dampxu[i]);
    }
    for (int r = 0; r < m; ++r) {
      SigS[r] = (slm[r] ? vlR[r] / Ssl[r] : 0.0) + (sum_[r] ? vuR[r] / Ssu[r] : 0.0);
      Sp[r] = zp[r] / pp[r];
      Sn[r] = zn[r] / nn[r];
      rs_[r] = ((-yR[r] - (slm[r] ? muR / Ssl[r] : 0.0)) + (sum_[r] ? muR / Ssu[r] : 0.0)) + kdm * (dampsl[r] - dampsu[r]);
      rp[r] = rho - yR[r] - muR / pp[r] + kdm;
      rn[r] = rho + yR[r] - muR / nn[r] + kdm;
      cR[r] = dR[r] - ss[r] - pp[r] + nn[r];
    }
    hess_blocks(P_, evR, 0.0, yR.data(), dc.data(), Qb.data(), Sb.data());
    if (dcurr > 0) dlast = dcurr;
    double delta_ = 0.0;
    bool fact = false;
    while (true) {
      for (int r = 0; r < m; ++r) {
        const double D_ = SigS[r] + delta_;
        const double spd = Sp[r] + delta_, snd = Sn[r] + delta_;
        // equality rows (no slack): the D -> infinity limit
        Dw[r] = eqm[r] ? 1.0 / (1.0 / spd + 1.0 / snd) : D_ / (1.0 + D_ * (1.0 / spd + 1.0 / snd));
      }
      for (int i = 0; i < n; ++i) Rd[i] = et * DR2[i] + (SigX[i] + delta_);
      Qw = Qb;
      add_rows(P_, evR, Dw.data(), dc.data(), Qw.data());
      if (ric.factor(P_, evR, Qw.data(), Sb.data(), Rd.data())) { fact = true; break; }
      if (delta_ == 0.0) {
        delta_ = dlast == 0.0 ? o.first_hessian_perturbation : std::max(o.min_hessian_perturbation, dlast * o.perturb_dec_fact);
      } else {
        if (dlast == 0.0 || 1e5 * dlast < delta_) delta_ *= o.perturb_inc_fact_first;
        else delta_ *= o.perturb_inc_fact;
      }
      if (delta_ > o.max_hessian_perturbation) { fact = false; break; }
    }
    dcurr = delta_;
    if (!fact) { out.status = ST_STEPERR; out.it = it_; out.x = xx; return; }
    for (int r = 0; r < m; ++r) {
      const double D_ = SigS[r] + delta_;
      Spd[r] = Sp[r] + delta_;
      Snd[r] = Sn[r] + delta_;
      den[r] = 1.0 / (1.0 + D_ * (1.0 / Spd[r] + 1.0 / Snd[r]));
      Dt[r] = D_ * den[r];
      if (eqm[r]) { den[r] = 0.0; Dt[r] = 1.0 / (1.0 / Spd[r] + 1.0 / Snd[r]); }
    }
    // rdir(c_): late-bound yR, evR, zlR..zn, pp, nn (as the oracle's closure)
    auto rdir = [&](const Vec& c_, RStep& st) {
      Vec Dr(m), jd(m);
      for (int r = 0; r < m; ++r) {
        Dr[r] = Dt[r] * (c_[r] + rp[r] / Spd[r] - rn[r] / Snd[r]) + rs_[r] * den[r];
        v[r] = yR[r] + Dr[r];
      }
      for (int k = 0; k <= P_.N; ++k) {
        double a[8] = {};
        add_GT(P_, evR, k, v.data(), dc.data(), a);
        for (int i = 0; i < 8; ++i) qv[k * 8 + i] = a[i];
      }
      ric.solve(P_, evR, qv.data(), gphi.data(), st.dx.data(), dXs.data());
      jmul(P_, evR, st.dx.data(), dc.data(), jd.data(), dXs.data());
      for (int r = 0; r < m; ++r) {
        st.dy[r] = Dt[r] * jd[r] + Dr[r];
        st.dp[r] = (st.dy[r] - rp[r]) / Spd[r];
        st.dn[r] = (-st.dy[r] - rn[r]) / Snd[r];
        st.ds[r] = eqm[r] ? 0.0 : jd[r] + c_[r] - st.dp[r] + st.dn[r];  // linearised d(x) - s - p + n = 0
        st.dvl[r] = slm[r] ? muR / Ssl[r] - vlR[r] - vlR[r] / Ssl[r] * st.ds[r] : 0.0;
        st.dvu[r] = sum_[r] ? muR / Ssu[r] - vuR[r] + vuR[r] / Ssu[r] * st.ds[r] : 0.0;
        st.dzp[r] = muR / pp[r] - zp[r] - Sp[r] * st.dp[r];
        st.dzn[r] = muR / nn[r] - zn[r] - Sn[r] * st.dn[r];
      }
      for (int i = 0; i < n; ++i) {
        st.dzl[i] = xlm[i] ? muR / Sxl[i] - zlR[i] - zlR[i] / Sxl[i] * st.dx[i] : 0.0;
        st.dzu[i] = xum[i] ? muR / Sxu[i] - zuR[i] + zuR[i] / Sxu[i] * st.dx[i] : 0.0;
      }
    };
    rdir(cR, stp);
    // ---- filter line search on the restoration problem
    double th_ref = thetaR(dR, ss, pp, nn);
    double ph_ref = phiR(xx, ss, pp, nn, muR);
    double gbd;
    {
      double a = 0.0, b = 0.0, c = 0.0, e = 0.0;
      for (int i = 0; i < n; ++i) a += gphi[i] * stp.dx[i];
      for (int r = 0; r < m; ++r) {
        const double gs = (-(slm[r] ? muR / Ssl[r] : 0.0) + (sum_[r] ? muR / Ssu[r] : 0.0)) + kdm * (dampsl[r] - dampsu[r]);
        b += gs * stp.ds[r];
        c += (rho - muR / pp[r] + kdm) * stp.dp[r];
        e += (rho - muR / nn[r] + kdm) * stp.dn[r];
      }
      gbd = ((a + b) + c) + e;
    }
    if (!have_tm) {
      have_tm = true;
      th_max = o.theta_max_fact * std::max(1.0, th_ref);
      th_min = o.theta_min_fact * std::max(1.0, th_ref);
    }
    auto r_ftype = [&](double a) {
      return gbd < 0.0 && a * std::pow(-gbd, o.s_phi) > o.delta * std::pow(th_ref, o.s_theta);
    };
    auto r_armijo = [&](double a, double ph) { return compare_le(ph - ph_ref, o.eta_phi * a * gbd, ph_ref); };
    auto r_acc_iter = [&](double ph, double th) {
      if (ph > ph_ref) {
        double basval = 1.0;
        if (std::fabs(ph_ref) > 10.0) basval = std::log10(std::fabs(ph_ref));
        if (std::log10(ph - ph_ref) > o.obj_max_inc + basval) return false;
      }
      return compare_le(th, (1.0 - o.gamma_theta) * th_ref, th_ref) ||
             compare_le(ph - ph_ref, -o.gamma_phi * th_ref, ph_ref);
    };
    auto r_check = [&](double a_test, double ph, double th) {
      if (th > th_max) return false;
      bool ok;
      if (a_test > 0.0 && r_ftype(a_test) && th_ref <= th_min) ok = r_armijo(a_test, ph);
      else ok = r_acc_iter(ph, th);
      if (!ok) return false;
      for (auto& e : rfilt)
        if (!(ph <= e.first || th <= e.second)) return false;
      return true;
    };
    auto r_trial = [&](double a, const RStep& st, RTrial& T) {
      T.x.resize(n); T.s.resize(m); T.p.resize(m); T.nn.resize(m); T.d.resize(m);
      for (int i = 0; i < n; ++i) T.x[i] = xx[i] + a * st.dx[i];
      for (int r = 0; r < m; ++r) {
        T.s[r] = ss[r] + a * st.ds[r];
        T.p[r] = pp[r] + a * st.dp[r];
        T.nn[r] = nn[r] + a * st.dn[r];
      }
      eval(T.x.data(), T.ev, false);
      for (int r = 0; r < m; ++r) T.d[r] = dc[r] * T.ev.g[r];
      if (!allfinite(T.d)) return false;
      T.phi = phiR(T.x, T.s, T.p, T.nn, muR);
      if (!std::isfinite(T.phi)) return false;
      T.th = thetaR(T.d, T.s, T.p, T.nn);
      return true;
    };
    const RStep* cstp = &stp;
    const RStep* acc_st = nullptr;
    RTrial* acc_tr = nullptr;
    double a_acc = 0.0, a_last = 0.0;
    int nsteps = 0;
    bool ev_err = false, have_wtri = false;
    auto r_line_search = [&](bool skip_first) -> bool {
      const double amax_p = ftb_R(tauR, cstp->dx, cstp->ds, cstp->dp, cstp->dn);
      nsteps = 0; ev_err = false; have_wtri = false;
      if (rin_wd) {
        const bool okt = r_trial(amax_p, *cstp, rt1);
        a_last = rwd_alpha;
        if (okt && r_check(rwd_alpha, rt1.phi, rt1.th)) { a_acc = amax_p; acc_st = cstp; acc_tr = &rt1; return true; }
        ev_err = !okt;
        have_wtri = okt;
        return false;
      }
      double amin = o.gamma_theta;
      if (gbd < 0) {
        amin = std::min(o.gamma_theta, o.gamma_phi * th_ref / (-gbd));
        if (th_ref <= th_min) amin = std::min(amin, o.delta * std::pow(th_ref, o.s_theta) / std::pow(-gbd, o.s_phi));
      }
      amin *= o.alpha_min_frac;
      double a = amax_p * (skip_first ? o.alpha_red_factor : 1.0);
      int nn_ = 0;
      while (a > amin || nn_ == 0) {
        const bool okt = r_trial(a, *cstp, rt1);
        if (okt && r_check(a, rt1.phi, rt1.th)) {
          nsteps = nn_; a_last = a; a_acc = a; acc_st = cstp; acc_tr = &rt1;
          return true;
        }
        if (okt && a == amax_p && th_ref <= rt1.th && o.max_soc > 0) {
          double th_tr = rt1.th, th_old = 0.0, a_soc = a;
          Vec cms = cR;
          int cnt = 0;
          RTrial* cp = &rt1;
          while (cnt < o.max_soc && (cnt == 0 || th_tr <= o.kappa_soc * th_old)) {
            th_old = th_tr;
            for (int r = 0; r < m; ++r) cms[r] = a_soc * cms[r] + (cp->d[r] - cp->s[r] - cp->p[r] + cp->nn[r]);
            rdir(cms, st2);
            a_soc = ftb_R(tauR, st2.dx, st2.ds, st2.dp, st2.dn);
            RTrial* nx_ = (cp == &rt1) ? &rt2 : &rt1;
            const bool ok2 = r_trial(a_soc, st2, *nx_);
            cp = nx_;
            if (!ok2) break;
            if (r_check(a, cp->phi, cp->th)) {
              nsteps = nn_; a_last = a; a_acc = a_soc; acc_st = &st2; acc_tr = cp;
              return true;
            }
            cnt += 1;
            th_tr = cp->th;
          }
        }
        a *= o.alpha_red_factor;
        nn_ += 1;
      }
      nsteps = nn_; a_last = a;
      return false;
    };
    // ---- watchdog procedure of the restoration phase's own line search
    if (wd_trigger > 0 && !rin_wd && rwd_cnt >= wd_trigger) {
      rwd.xx = xx; rwd.ss = ss; rwd.pp = pp; rwd.nn = nn; rwd.evR = evR; rwd.dR = dR; rwd.yR = yR;
      rwd.zlR = zlR; rwd.zuR = zuR; rwd.vlR = vlR; rwd.vuR = vuR; rwd.zp = zp; rwd.zn = zn; rwd.stp = stp;
      rwd.th_ref = th_ref; rwd.ph_ref = ph_ref; rwd.gbd = gbd;
      rwd_alpha = ftb_R(tauR, stp.dx, stp.ds, stp.dp, stp.dn);
      rwd_trial = 0; rin_wd = true;
    }
    if (rin_wd) { th_ref = rwd.th_ref; ph_ref = rwd.ph_ref; gbd = rwd.gbd; }
    bool skip_first = false, forced = false, acc = false;
    while (true) {
      acc = r_line_search(skip_first);
      if (!rin_wd) break;
      if (acc) { rin_wd = false; break; }
      rwd_trial += 1;
      if (ev_err || rwd_trial > wd_max) {
        xx = rwd.xx; ss = rwd.ss; pp = rwd.pp; nn = rwd.nn; evR = rwd.evR; dR = rwd.dR; yR = rwd.yR;
        zlR = rwd.zlR; zuR = rwd.zuR; vlR = rwd.vlR; vuR = rwd.vuR; zp = rwd.zp; zn = rwd.zn; stp = rwd.stp;
        th_ref = rwd.th_ref; ph_ref = rwd.ph_ref; gbd = rwd.gbd;
        cstp = &stp;
        rin_wd = false; rwd_cnt = 0; skip_first = true;
        continue;
      }
      a_acc = ftb_R(tauR, stp.dx, stp.ds, stp.dp, stp.dn);
      acc_st = &stp; acc_tr = &rt1;
      acc = true;
      forced = true;
      break;
    }
    if (!acc) { out.status = ST_RESTOFAIL; out.it = it_; out.x = xx; return; }
    rwd_cnt = nsteps == 0 ? 0 : rwd_cnt + 1;
    if (!forced && !(r_ftype(a_last) && r_armijo(a_last, acc_tr->phi)))
      rfilt.emplace_back(ph_ref - o.gamma_phi * th_ref, (1.0 - o.gamma_theta) * th_ref);
    const RStep& st = *acc_st;
    const double ad = dftb_R(tauR, st);
    xx = acc_tr->x; ss = acc_tr->s; pp = acc_tr->p; nn = acc_tr->nn; std::swap(evR, acc_tr->ev); dR = acc_tr->d;
    if (!evR.derivs) eval(xx.data(), evR, true);
    for (int r = 0; r < m; ++r) yR[r] = yR[r] + a_acc * st.dy[r];
    for (int i = 0; i < n; ++i) { zlR[i] = zlR[i] + ad * st.dzl[i]; zuR[i] = zuR[i] + ad * st.dzu[i]; }
    for (int r = 0; r < m; ++r) {
      vlR[r] = vlR[r] + ad * st.dvl[r];
      vuR[r] = vuR[r] + ad * st.dvu[r];
      zp[r] = zp[r] + ad * st.dzp[r];
      zn[r] = zn[r] + ad * st.dzn[r];
    }
    slacks(xx, ss, Sxl, Sxu, Ssl, Ssu);
    const double ks = o.kappa_sigma;
    for (int i = 0; i < n; ++i) {
      zlR[i] = xlm[i] ? std::max(std::min(zlR[i], ks * muR / Sxl[i]), muR / (ks * Sxl[i])) : 0.0;
      zuR[i] = xum[i] ? std::max(std::min(zuR[i], ks * muR / Sxu[i]), muR / (ks * Sxu[i])) : 0.0;
    }
    for (int r = 0; r < m; ++r) {
      vlR[r] = slm[r] ? std::max(std::min(vlR[r], ks * muR / Ssl[r]), muR / (ks * Ssl[r])) : 0.0;
      vuR[r] = sum_[r] ? std::max(std::min(vuR[r], ks * muR / Ssu[r]), muR / (ks * Ssu[r])) : 0.0;
      zp[r] = std::max(std::min(zp[r], ks * muR / pp[r]), muR / (ks * pp[r]));
      zn[r] = std::max(std::min(zn[r], ks * muR / nn[r]), muR / (ks * nn[r]));
    }
    it_ += 1;
    (void)have_wtri;
  }
  // ---- back to the original problem (RestoMinC_1Nrm::PerformRestoration)
  Vec dzl(n), dzu(n), dvl(m), dvu(m);
  for (int i = 0; i < n; ++i) {
    const double S0l = xlm[i] ? x0[i] - xl[i] : 1.0, S1l = xlm[i] ? xx[i] - xl[i] : 1.0;
    const double S0u = xum[i] ? xu[i] - x0[i] : 1.0, S1u = xum[i] ? xu[i] - xx[i] : 1.0;
    dzl[i] = xlm[i] ? (mu0 - zl0[i] * (S1l - S0l)) / S0l - zl0[i] : 0.0;
    dzu[i] = xum[i] ? (mu0 - zu0[i] * (S1u - S0u)) / S0u - zu0[i] : 0.0;
  }
  for (int r = 0; r < m; ++r) {
    const double S0l = slm[r] ? s0[r] - dl[r] : 1.0, S1l = slm[r] ? ss[r] - dl[r] : 1.0;
    const double S0u = sum_[r] ? du[r] - s0[r] : 1.0, S1u = sum_[r] ? du[r] - ss[r] : 1.0;
    dvl[r] = slm[r] ? (mu0 - vl0[r] * (S1l - S0l)) / S0l - vl0[r] : 0.0;
    dvu[r] = sum_[r] ? (mu0 - vu0[r] * (S1u - S0u)) / S0u - vu0[r] : 0.0;
  }
  const double ad = dual_frac_to_bound(tau0, zl0, zu0, vl0, vu0, dzl, dzu, dvl, dvu);
  out.zl.resize(n); out.zu.resize(n); out.vl.resize(m); out.vu.resize(m);
  double mx = 0.0;
  for (int i = 0; i < n; ++i) {
    out.zl[i] = zl0[i] + ad * dzl[i];
    out.zu[i] = zu0[i] + ad * dzu[i];
    mx = std::max(mx, std::max(std::fabs(out.zl[i]), std::fabs(out.zu[i])));
  }
  for (int r = 0; r < m; ++r) {
    out.vl[r] = vl0[r] + ad * dvl[r];
    out.vu[r] = vu0[r] + ad * dvu[r];
    mx = std::max(mx, std::max(std::fabs(out.vl[r]), std::fabs(out.vu[r])));
  }
  if (mx > o.bound_mult_reset_threshold) {
    for (int i = 0; i < n; ++i) { out.zl[i] = xlm[i] ? 1.0 : 0.0; out.zu[i] = xum[i] ? 1.0 : 0.0; }
    for (int r = 0; r < m; ++r) { out.vl[r] = slm[r] ? 1.0 : 0.0; out.vu[r] = sum_[r] ? 1.0 : 0.0; }
  }
  out.y.assign(m, 0.0);
  if (o.constr_mult_reset_threshold > 0 && m > 0)
    main_ls_mults(evR, out.zl, out.zu, out.vl, out.vu, o.constr_mult_reset_threshold, out.y);
  out.status = ST_NONE;
  out.it = it_;
  out.x = xx;
  out.s = ss;
  out.ev = evR;
}

// plant Euler step with u0, warm-start shift, target unicycle step (oracle shift_timestep)
void shift(const Prob& P, double* x0, double* w, double* xs, double vt, double wt) {
  const int nx = P.nx, nu = P.nu, N = P.N;
  const double th = x0[3], ps = x0[4], v = w[0];
  double fx[8];
  fx[0] = v * std::cos(ps) * std::cos(th);
  fx[1] = v * std::sin(ps) * std::cos(th);
  fx[2] = v * std::sin(th);
  for (int j = 3; j < nx; ++j) fx[j] = w[j - 2];
  for (int j = 0; j < nx; ++j) x0[j] = x0[j] + P.T * fx[j];
  for (int k = 0; k < N - 1; ++k)
    for (int c = 0; c < nu; ++c) w[k * nu + c] = w[(k + 1) * nu + c];
  const double a0 = vt * std::cos(xs[2]), a1 = vt * std::sin(xs[2]);
  xs[0] = xs[0] + P.T * a0;
  xs[1] = xs[1] + P.T * a1;
  xs[2] = xs[2] + P.T * wt;
}

Opts opts_from(const double* v) {
  Opts o;
  double* dst = reinterpret_cast<double*>(&o);
  std::memcpy(dst, v, sizeof(Opts));
  return o;
}

}  // namespace

extern "C" {

// comma-separated option names in the order nmpc_cpu_* expect them in `opts`
const char* nmpc_cpu_option_names() {
  static const std::string s = [] {
    std::string r;
#define NMPC_N(n) r += #n ",";
    NMPC_CPU_OPTS(NMPC_N)
#undef NMPC_N
    r.pop_back();
    return r;
  }();
  return s.c_str();
}

// B independent solves (oracle IpoptDense.solve per scenario): w0 (B x n), p (B x np),
// shared bounds; outputs x (B x n), f, g (B x m, may be null), lam_x / lam_g (may be
// null), status, iterations.  OpenMP over scenarios, nthreads <= 0 = all.
int nmpc_cpu_solve_batch(const nmpc_cpu_problem* prob, const double* opts, int64_t B, const double* w0,
                         const double* p, const double* lbx, const double* ubx, const double* lbg, const double* ubg,
                         double* x_out, double* f_out, double* g_out, double* lam_x_out, double* lam_g_out,
                         int32_t* status_out, int32_t* iter_out, int nthreads, double* solve_s) {
  if (!prob || !opts || B < 0) return 1;
  const Prob P = make_prob(*prob);
  const Opts o = opts_from(opts);
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
  {
    Solver S(P, o);
    Result R;
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
      const auto ts = std::chrono::steady_clock::now();
      S.solve(w0 + b * P.n, p + b * P.np, lbx, ubx, lbg, ubg, R);
      if (solve_s) solve_s[b] = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
      std::memcpy(x_out + b * P.n, R.x.data(), sizeof(double) * P.n);
      f_out[b] = R.F;
      if (g_out) std::memcpy(g_out + b * P.m, R.g.data(), sizeof(double) * P.m);
      if (lam_x_out) std::memcpy(lam_x_out + b * P.n, R.lam_x.data(), sizeof(double) * P.n);
      if (lam_g_out) std::memcpy(lam_g_out + b * P.m, R.lam_g.data(), sizeof(double) * P.m);
      status_out[b] = R.status;
      iter_out[b] = R.iter;
    }
  }
  return 0;
}

// The closed loop of Python/NMPC_TT.py:346-402 for B scenarios: K warm-started MPC
// steps each (solve, then shift with the target controls vt, wt; obstacle parameters
// p[nx+3:] += p_step[k] when p_step (K x np) is given), starting from
// p (B x np: x0, target, obstacle parameters) and w = 0.  Stops taking new steps
// once budget_s seconds have passed (budget_s <= 0: no limit); steps_done[b] says
// how many steps scenario b ran.  Histories: status / iter (B x K), u0 (B x K x nu), f,
// and (nullable) each solve's wall time in seconds (B x K).
// w0 (nullable: zeros) is each scenario's warm start for its first step; p_out / w_out
// (nullable) receive the state after its last step (the next step's p and warm start), so a
// loop can be continued from where another one stopped (bench.py: W untimed warm-up steps,
// then the K timed ones from the same state as the GPU's timed launch)
int nmpc_cpu_closed_loop(const nmpc_cpu_problem* prob, const double* opts, int64_t B, int32_t K, const double* p0,
                         const double* w0, const double* lbx, const double* ubx, const double* lbg, const double* ubg,
                         double vt, double wt, const double* p_step, double budget_s, int nthreads, int32_t* status_out,
                         int32_t* iter_out, double* u0_out, double* f_out, int32_t* steps_done, double* solve_s,
                         double* p_out, double* w_out) {
  if (!prob || !opts || B < 0 || K < 0) return 1;
  const Prob P = make_prob(*prob);
  const Opts o = opts_from(opts);
  if (nthreads <= 0) nthreads = omp_get_max_threads();
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
#pragma omp parallel num_threads(nthreads)
  {
    Solver S(P, o);
    Result R;
    std::vector<double> p(P.np), w(P.n);
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
      std::memcpy(p.data(), p0 + b * P.np, sizeof(double) * P.np);
      if (w0) std::memcpy(w.data(), w0 + b * P.n, sizeof(double) * P.n);
      else std::fill(w.begin(), w.end(), 0.0);
      int k = 0;
      for (; k < K; ++k) {
        if (budget_s > 0 && elapsed() >= budget_s) break;
        const auto ts = std::chrono::steady_clock::now();
        S.solve(w.data(), p.data(), lbx, ubx, lbg, ubg, R);
        if (solve_s) solve_s[b * K + k] = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
        status_out[b * K + k] = R.status;
        iter_out[b * K + k] = R.iter;
        f_out[b * K + k] = R.F;
        std::memcpy(u0_out + (b * K + k) * P.nu, R.x.data(), sizeof(double) * P.nu);
        std::memcpy(w.data(), R.x.data(), sizeof(double) * P.n);
        shift(P, p.data(), w.data(), p.data() + P.nx, vt, wt);
        if (p_step)
          for (int j = P.nx + 3; j < P.np; ++j) p[j] = p[j] + p_step[(int64_t)k * P.np + j];
      }
      steps_done[b] = k;
      if (p_out) std::memcpy(p_out + b * P.np, p.data(), sizeof(double) * P.np);
      if (w_out) std::memcpy(w_out + b * P.n, w.data(), sizeof(double) * P.n);
    }
  }
  return 0;
}

}  // extern "C"
