// nmpc_solve.hip -- MI355X (gfx950) batched NMPC solve step + C-ABI (include/nmpc_amd.h).
//
// Replaces, for B independent scenarios per call, the per-timestep
//   sol = solver(x0=, lbx=, ubx=, lbg=, ubg=, p=)        Python/NMPC_TT.py:358-365
// of the reference, whose solver is ca.nlpsol('solver','ipopt',...) on the
// single-shooting NLP of Python/NMPC_TT.py:139-267.
//
// Execution model: ONE WAVEFRONT (64 lanes) PER SCENARIO, the
// whole interior-point solve inside one kernel launch, all control flow
// wave-uniform (every branch decision comes from a butterfly all-reduce, so
// every lane holds the bit-identical value).  Lanes parallelise:
//   * stages   (lane k = horizon stage k, N <= 63): rollout by per-lane
//     in-order prefix sums, derivatives, constraint rows, adjoint suffix sums;
//   * matrix entries (lane = 8*i + j) in the Riccati backward sweep;
//   * rows / controls (strided) for fraction-to-boundary, barrier terms,
//     multiplier updates and optimality-error reductions.
// The hot row vectors, trajectories and the current Riccati stage operands live in
// LDS; control vectors, the per-stage Riccati factors (K, R~, Q) and the restoration /
// watchdog copies live in a per-scenario global workspace.
//
// Algorithm: the IPOPT restatement of oracle/nmpc_oracle.py::IpoptDense,
// step for step (same options, same decisions), except that the Newton
// system  (W + Sigma_x + delta I + J^T D J) dU = -rhs  of the single-shooting
// NLP is solved with a Riccati recursion on the multiple-shooting structure
// (X re-simulated every step, defect multipliers = adjoint), which yields the
// identical step in exact arithmetic; inertia = all Riccati pivots positive.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>

#include "nmpc_amd.h"

// Named (not anonymous): the library is built as several translation units (one per
// capacity class, compiled in parallel, plus the host side, NMPC_TU_CLASS / NMPC_TU_HOST)
// that exchange kernel pointers whose signatures use these types.
namespace nmpc_impl {

constexpr int WAVE = 64;
#define LDS __attribute__((address_space(3)))
#define CST __attribute__((address_space(4)))
#define GLB __attribute__((address_space(1)))
constexpr double BIGB = 1e19;  // IPOPT nlp_{lower,upper}_bound_inf
constexpr int FCAP = 128;      // filter capacity (>= max_iter of the reference opts)
constexpr int TRACE_F = NMPC_TRACE_FIELDS;
// equality rows (lbg == ubg) per problem the augmented-system (Schur complement) step
// supports (lane l owns rows l and l + 64 of S); more report Invalid_Problem_Definition (-11)
#define NMPC_MEQ 128

// ---- status codes (IPOPT ApplicationReturnStatus) ----
constexpr int ST_SUCCESS = 0, ST_ACCEPTABLE = 1, ST_INFEASIBLE = 2, ST_TINY = 3, ST_MAXITER = -1,
              ST_RESTO_FAIL = -2, ST_STEP_ERR = -3, ST_INVALID_PROBLEM = -11,
              ST_INVALID_NUMBER = -13;

struct Params {
  int N, m, nobs, np, nw, ng, nX;
  double T, w1, w2, hv, hh;
  int w1p, w2p;  // cost weights from p (-1: constant)
  // model embedding: the no-gimbal model (MATLAB/Dynamic Obstacles/NMPC_TT.m) runs on the
  // gimbal layout with its controls 3..5 / states 5..7 absent
  int model, nb, nuE, nwE, nxE, npE;  // box rows per stage, real controls/decision/states, external np
  double ox[NMPC_MAX_OBS], oy[NMPC_MAX_OBS], orr[NMPC_MAX_OBS];
  int oxp[NMPC_MAX_OBS], oyp[NMPC_MAX_OBS];
  nmpc_options o;
  int nospec;  // diagnostics (NMPC_NO_SPEC=1 at nmpc_create): no speculative restoration trial pairs
  double thv, thh;  // tan(hv), tan(hh) (host libm): the FOV tangent pairs from one tangent (NMPC_TAN2)
};

// Per-scenario memory layout (offsets in doubles).  Computed at compile time
// for a capacity class (NMAX, MMAX) so every array address folds into a base
// register plus an immediate: no pointer registers in the kernel.
struct Lay {
  // global workspace (64 B aligned slices)
  int U, Ut, dU, dU2, zl, zu, xl, xu, sigx, ru, rres, dUr;
  int s, y, vl, vu, d, dt, ds, ds2, dc, dl, du, dms, filt;
  int gl, Hl, Qs, K, Rk;        // stage data / Riccati factors (global copies)
  int tc;                       // transcendental values of the latest rollouts / stage costs (2 x 12 x NS)
  // restoration phase: reference/backup iterate, p/n and their multipliers, steps, filter
  int UR, zl0, zu0, s0, vl0, vu0, pR, nR, zpR, znR, dpR, dnR, dyR, dp2R, dn2R, dy2R, cms, filtR;
  int accU, accZl, accZu, accY;  // last acceptable iterate (BacktrackingLineSearch::StoreAcceptablePoint)
  int eqi, eqS, eqy, eqy2, weqy;  // equality rows: indices, Schur factor, dy_c (row-indexed) of the step / SOC,
                                  // and the watchdog's stored dy_c
  // watchdog procedure: the stored iterate and its step (main loop; the restoration phase
  // reuses them, and adds its p, n, their multipliers and steps)
  int wU, wzl, wzu, wdU, ws, wy, wvl, wvu, wds, wpR, wnR, wzpR, wznR, wdpR, wdnR, wdyR;
  // LDS
  int X, Xt, dX;
  int trig, qs, lam;
  int kf, Rc, Rv, P0, P1, pv0, pv1, St;
  int p, ob, inc, red, rvars, rdX;
  int fixm;     // per-stage bit mask of fixed controls (ints)
  int total;    // LDS doubles per scenario
  int wstotal;  // global-workspace doubles per scenario
};
constexpr int al2(int n) { return (n + 1) & ~1; }
constexpr int al8(int n) { return (n + 7) & ~7; }
// lr: the main iteration's hot row vectors (s, y, vl, vu, d, ds, ds2, dc) live in LDS
// (capacity classes with a small row count: the row passes then never wait on L2 /
// Infinity-Cache latency); otherwise in the global workspace
constexpr Lay make_layout(int N, int m, bool lr, bool refine, bool eq) {
  Lay L{};
  const int nw = 6 * N, ng = m * (N + 1), nX = 8 * (N + 1), NS = N + 1;
  int g = 0, o = 0;
  L.U = g; g += al8(nw); L.Ut = g; g += al8(nw); L.dU = g; g += al8(nw); L.dU2 = g; g += al8(nw);
  L.zl = g; g += al8(nw); L.zu = g; g += al8(nw); L.xl = g; g += al8(nw); L.xu = g; g += al8(nw);
  L.sigx = g; g += al8(nw); L.ru = g; g += al8(nw);
  L.rres = g; g += al8(nw); L.dUr = g; g += al8(nw);  // iterative refinement (fp32 classes)
  if (!lr) {
    L.s = g; g += al8(ng); L.y = g; g += al8(ng); L.vl = g; g += al8(ng); L.vu = g; g += al8(ng);
    L.d = g; g += al8(ng); L.ds = g; g += al8(ng); L.ds2 = g; g += al8(ng); L.dc = g; g += al8(ng);
    // the row bounds go with the rows: in the workspace for the global-row classes, whose
    // LDS then holds only per-stage data (config 5's N = 50 class fits 6 scenarios per CU)
    L.dl = g; g += al8(ng); L.du = g; g += al8(ng);
  }
  // trial row values: in LDS with the hot rows (not in the refinement classes, whose
  // LDS budget holds the refinement's step instead)
  const bool ldt = lr && !refine;
  if (!ldt) { L.dt = g; g += al8(ng); }
  L.dms = g; g += al8(ng);
  L.filt = g; g += al8(2 * FCAP + 2);
  L.gl = g; g += al8(8 * NS); L.Hl = g; g += al8(21 * NS); L.Qs = g; g += al8(36 * NS);
  L.K = g; g += al8(48 * N); L.Rk = g; g += al8(21 * N);
  L.UR = g; g += al8(nw); L.zl0 = g; g += al8(nw); L.zu0 = g; g += al8(nw);
  L.s0 = g; g += al8(ng); L.vl0 = g; g += al8(ng); L.vu0 = g; g += al8(ng);
  L.pR = g; g += al8(ng); L.nR = g; g += al8(ng); L.zpR = g; g += al8(ng); L.znR = g; g += al8(ng);
  L.dpR = g; g += al8(ng); L.dnR = g; g += al8(ng); L.dyR = g; g += al8(ng);
  L.dp2R = g; g += al8(ng); L.dn2R = g; g += al8(ng); L.dy2R = g; g += al8(ng); L.cms = g; g += al8(ng);
  L.filtR = g; g += al8(2 * FCAP + 2);
  L.accU = g; g += al8(nw); L.accZl = g; g += al8(nw); L.accZu = g; g += al8(nw); L.accY = g; g += al8(ng);
  L.wU = g; g += al8(nw); L.wzl = g; g += al8(nw); L.wzu = g; g += al8(nw); L.wdU = g; g += al8(nw);
  L.ws = g; g += al8(ng); L.wy = g; g += al8(ng); L.wvl = g; g += al8(ng); L.wvu = g; g += al8(ng);
  L.wds = g; g += al8(ng); L.wpR = g; g += al8(ng); L.wnR = g; g += al8(ng); L.wzpR = g; g += al8(ng);
  L.wznR = g; g += al8(ng); L.wdpR = g; g += al8(ng); L.wdnR = g; g += al8(ng); L.wdyR = g; g += al8(ng);
  if (eq) {  // equality rows (the equality class only)
    // eqS: S (column-major, NMPC_MEQ x NMPC_MEQ), its signed factor (same layout), pivot signs
    L.eqi = g; g += al8(NMPC_MEQ / 2 + 1); L.eqS = g; g += al8(2 * NMPC_MEQ * NMPC_MEQ + NMPC_MEQ);
    L.eqy = g; g += al8(ng); L.eqy2 = g; g += al8(ng); L.weqy = g; g += al8(ng);
  }
  if (!lr) { L.kf = g; g += al8(6 * N); }
  L.tc = g; g += al8(2 * 12 * NS);
  L.wstotal = g;
  L.X = o; o += al2(nX); L.Xt = o; o += al2(nX); L.dX = o; o += al2(nX);
  L.trig = o; o += al2(8 * NS); L.qs = o; o += al2(10 * NS); L.lam = o; o += al2(8 * NS);
  // the Riccati feed-forward terms k_k: in LDS for the LDS-row class, in the workspace
  // otherwise (the global-row classes' LDS then fits 6 scenarios per CU at N = 50)
  if (lr) { L.kf = o; o += al2(6 * N); }
  L.Rc = o; o += 22; L.Rv = o; o += 8;
  // the Riccati sweep's P / p double buffers: inside `inc` (rollout / adjoint scratch,
  // never live during the sweep) whenever it is large enough (N >= 17)
  const bool pin = 8 * NS >= 144;
  if (!pin) { L.P0 = o; o += 64; L.P1 = o; o += 64; L.pv0 = o; o += 8; L.pv1 = o; o += 8; }
  L.St = o; o += 48;
  // inc: stage rows 0..N plus the -0.0 row N + 1 of the unrolled stage sums (Solver::kZeroRow)
  L.p = o; o += 64; L.ob = o; o += al2(2 * NMPC_MAX_OBS); L.inc = o; o += al2(8 * (NS + 1));
  if (pin) { L.P0 = L.inc; L.P1 = L.inc + 64; L.pv0 = L.inc + 128; L.pv1 = L.inc + 136; }
#ifdef NMPC_STAMPS
  L.red = o; o += 24;  // phase timers
#else
  L.red = o;
#endif
  if (lr) { L.dl = o; o += al2(ng); L.du = o; o += al2(ng); }  // row bounds (constant during a solve, read by every row pass)
  L.rvars = o; o += 48;  // line-search / restoration scalars; [32..36] barrier sums; [37..39] line-search powers (restoration: [23] flag, [37..38]); [40..45] watchdog; [46] #fixed
  L.fixm = o; o += al2(N / 2 + 1);  // fixed-control masks, one int per stage
  L.rdX = o; if (refine) o += al2(nX);  // refinement step in X (fp32 classes)
  if (lr) {
    L.s = o; o += al2(ng); L.y = o; o += al2(ng); L.vl = o; o += al2(ng); L.vu = o; o += al2(ng);
    L.d = o; o += al2(ng); L.ds = o; o += al2(ng); L.ds2 = o; o += al2(ng); L.dc = o; o += al2(ng);
  }
  if (ldt) { L.dt = o; o += al2(ng); }
  L.total = o;
  return L;
}
// waves per SIMD the kernels are register-budgeted for (256 VGPRs at 2)
#ifndef NMPC_WAVES_PER_EU
#define NMPC_WAVES_PER_EU 2
#endif

// LDSR: hot row vectors in LDS (make_layout); such a class needs ~39 KB of LDS per
// scenario, so it runs one wave per SIMD (four per CU) with the full 512-VGPR budget
// RT: arithmetic type of the Riccati factorisation and its solves (double: the
// reference's fp64; float: the fp32 leg of BASELINE config 5's fp32-vs-fp64 sweep --
// everything else, the iterate, residuals, line search and termination tests, stays fp64)
// EQ: equality rows (lbg == ubg) are solved; only the equality class has
// them compiled in, so the other classes' hot loops carry none of that code
template <int NMAX, int MMAX, bool LDSR = false, class RTYPE = double, bool EQ = false>
struct Cap {
  static constexpr int nmax = NMAX, mmax = MMAX;
  static constexpr bool lds_rows = LDSR;
  using RT = RTYPE;
  static constexpr int wpe = LDSR ? 1 : NMPC_WAVES_PER_EU;
  using RowT = std::conditional_t<LDSR, LDS double, GLB double>;
  static constexpr bool refine = !std::is_same<RTYPE, double>::value;  // fp64 refinement of fp32 solves
  static constexpr bool eq = EQ;
  static_assert(!(EQ && !std::is_same<RTYPE, double>::value), "equality rows need the fp64 factorisation");
  static constexpr Lay L = make_layout(NMAX, MMAX, LDSR, refine, EQ);
  // row passes: trips of 64 rows processed together (their loads batched), <= 5
  static constexpr int rtrips = (MMAX * (NMAX + 1) + 63) / 64;
  static constexpr int ru = rtrips < 2 ? rtrips : 2;
  // deep: register-hungry latency hiding (control passes two trips at a time, gains
  // fetched three stages ahead in the forward sweep, stored factors one stage ahead in the
  // re-solve) -- for the one-wave-per-SIMD LDS class; the global-row classes, held to half
  // the registers, spill with it and lose (config 5 measured)
#ifndef NMPC_DEEP_GLOBAL
#define NMPC_DEEP_GLOBAL 0
#endif
  static constexpr bool deep = LDSR || NMPC_DEEP_GLOBAL;
  // control passes: trips of 64 decision variables processed together, <= 2
  static constexpr int ctrips = (6 * NMAX + 63) / 64;
  static constexpr int cu = !deep ? 1 : (ctrips < 2 ? ctrips : 2);
};

struct IO {
  const double *x0, *lbx, *ubx, *lbg, *ubg, *p;
  long long ld_x0, ld_lbx, ld_ubx, ld_lbg, ld_ubg, ld_p;
  double *x_out, *f_out, *g_out, *lam_x, *lam_g, *lam_p, *X_out;
  int *status, *iters;
  double* trace;
  double* ws;  // per-scenario global workspace, B x wstotal
  // launch gate (nullable): 1 when the batch has equality rows.  A class kernel whose
  // CAP::eq differs from it returns at once, so the host enqueues the problem's class and
  // the equality class back to back and exactly one of them runs (no host round trip)
  const int* eqflag;
};

// Wave-wide all-reduces without LDS: DPP within 16-lane rows (quad_perm xor1,
// xor2, row_half_mirror, row_mirror), then gfx950 permlane16/32 swaps across
// rows.  Each step combines a lane's value with its partner's in the same
// order on both sides, so every lane ends with a bitwise-identical result
// (the wave-uniform decisions depend on that).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
struct DPair { double a, b; };
__device__ __forceinline__ DPair swap16_d(double v) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  return {__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1])};
}
__device__ __forceinline__ DPair swap32_d(double v) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  return {__hiloint2double(hi[0], lo[0]), __hiloint2double(hi[1], lo[1])};
}
template <class OP>
__device__ __forceinline__ double wreduce(double v, OP op) {
  v = op(v, dpp_d<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_d<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_d<0x141>(v));  // row_half_mirror
  v = op(v, dpp_d<0x140>(v));  // row_mirror
  const DPair p = swap16_d(v); // {row 2r, row 2r+1} in both rows of the pair
  v = op(p.a, p.b);
  const DPair q = swap32_d(v); // {lanes 0-31, lanes 32-63}
  return op(q.a, q.b);
}
__device__ __forceinline__ double wsum(double v) {
  return wreduce(v, [](double a, double b) { return a + b; });
}
// Sum of logarithms as the logarithm of a product (the barrier terms mu * sum log(slack)
// of IPOPT's phi): a lane keeps the product of its arguments as a mantissa in [0.5, 1)
// (v_frexp_mant) and a binary exponent (v_frexp_exp), renormalised after every factor so
// it can neither overflow nor underflow, and takes ONE logarithm at the end:
//   sum log(x_i) = log(m) + e ln 2,  ln 2 split so that e * LN2_HI is exact.
// A factor costs a multiply and two frexp instead of an fp64 log (~90 dependent
// operations, the row passes' largest cost).  The result differs from the sum of the
// logarithms at the rounding level only: the product carries <= n ulp of relative error
// (n factors per lane, <= 24), i.e. <= 3e-15 absolute in the lane's log sum, below the
// rounding of the sum it replaces.  A non-positive argument gives log(<= 0) = NaN / -inf
// as the sum did, so a trial outside the bounds is still rejected as non-finite.
struct LogAcc {
  double m = 1.0;
  int e = 0;
  __device__ __forceinline__ void mul(double x) {
    const double p = m * x;
    m = __builtin_amdgcn_frexp_mant(p);
    e += __builtin_amdgcn_frexp_exp(p);
  }
  // two factors: their product first (|x|, |y| < 2^500: no overflow), one renormalisation
  __device__ __forceinline__ void mul2(double x, double y) {
    const double xy = x * y;
    const double xe = __builtin_amdgcn_frexp_mant(xy);
    const int ee = __builtin_amdgcn_frexp_exp(xy);
    const double p = m * xe;
    m = __builtin_amdgcn_frexp_mant(p);
    e += ee + __builtin_amdgcn_frexp_exp(p);
  }
  __device__ __forceinline__ double log() const {
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double de = (double)e;
    return (::log(m) + de * LN2_LO) + de * LN2_HI;
  }
};
__device__ __forceinline__ double wmax(double v) {
  return wreduce(v, [](double a, double b) { return fmax(a, b); });
}
__device__ __forceinline__ double wmin(double v) {
  return wreduce(v, [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ bool wany(bool b) { return __any((int)b) != 0; }
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
// reciprocal / reciprocal square root: hardware estimate + two Newton steps
// (~1 ulp; the IEEE-exact fp64 division sequence is ~2x longer).  Only used on
// finite non-zero arguments (slacks, distances, pivots).
__device__ __forceinline__ double rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double r = fma(-h * y, y, 0.5);
  y = fma(y, r, y);
  r = fma(-h * y, y, 0.5);
  return fma(y, r, y);
}
__device__ __forceinline__ float rsq(float x) { return __builtin_amdgcn_rsqf(x); }  // v_rsq_f32, ~1 ulp
// fp64 quotient a / b by the compiler's own sequence without its range fix-ups: the same
// v_rcp_f64 estimate, two Newton steps, q = a r and one Markstein correction as LLVM's
// fdiv lowering, minus v_div_scale (x2), v_div_fmas and v_div_fixup, which act only when an
// operand or the quotient is out of range (exponents near the limits, zero, inf, NaN).  So
// bitwise a / b for finite non-zero operands of moderate range -- slacks, multipliers,
// pivots, distances, step components -- which is what every call site divides; where a
// caller's operand can be 0 or inf (a missing bound, a zero step component) its result is
// discarded by the caller's guard, as a / b's was.  Three fewer instructions per division,
// two of them on the dependence chain.  NMPC_FDIV=0: plain a / b.
#ifndef NMPC_FDIV
#define NMPC_FDIV 1
#endif
__device__ __forceinline__ double qd(double a, double b) {
  if constexpr (NMPC_FDIV) {
    double r = __builtin_amdgcn_rcp(b);
    double e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
  } else {
    return a / b;
  }
}
__device__ __forceinline__ float readlane_d(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// Cross-lane hand-off inside the (single-wave) workgroup.  Every kernel here runs
// exactly one wavefront per workgroup, so a wavefront-scope fence is the complete
// synchronisation: it orders the compiler's memory operations (LDS and global)
// and, per the AMDGPU memory model, needs no hardware wait because a wave's memory
// operations are performed in order.  (__syncthreads' workgroup-scope release
// would wait for every outstanding global store, s_waitcnt vmcnt(0), each time.)
__device__ __forceinline__ void sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// packed index of the symmetric 6x6 local (x,y,z,x5,x6,x7) Hessian, a <= b
__device__ __forceinline__ int hp(int a, int b) {
  if (a > b) { int t = a; a = b; b = t; }
  return a * 6 - (a * (a - 1)) / 2 + (b - a);
}
// state index -> local cost-variable index (-1 if the cost does not depend on it)
__device__ __forceinline__ int vloc(int i) {
  return i < 3 ? i : (i >= 5 ? i - 2 : -1);
}
// model embedding: external (caller-layout) index of an internal
// decision / parameter entry; -1 for an absent gimbal control or state
__device__ __forceinline__ int ext_u(const Params* prm, int i) {
  const int k = i / 6, c = i - 6 * k;
  return c < prm->nuE ? k * prm->nuE + c : -1;
}
__device__ __forceinline__ int ext_p(const Params* prm, int i) {
  if (prm->model == 0) return i;
  return i < 5 ? i : (i < 8 ? -1 : i - 3);  // [x0(5); xs(3); ...] -> [x0(8); xs(3); ...]
}
__device__ __forceinline__ int boxidx(int i) {  // g rows 0..4: z, theta, x5, x6, x7 (NMPC_TT.py:236-240)
  return i == 0 ? 2 : (i == 1 ? 3 : 3 + i);
}

enum SumMode { SUM_NEWTON = 0, SUM_LS = 1, SUM_SOC = 2, SUM_RESTO = 3, SUM_RESTO_SOC = 4, SUM_LS_RESTO = 5 };

// Diagnostic phase timers (-DNMPC_STAMPS builds only): shader-clock cycles per
// phase, accumulated by lane 0 in LDS and written to the two spare rows of the
// trace buffer.  Never compiled into the product library.
enum Phase { PH_ROLLOUT, PH_EVAL, PH_DERIVS, PH_ADJ, PH_SUMM, PH_RIC, PH_RESOLVE, PH_FWD, PH_ROWSTEP,
             PH_BARR, PH_FTB, PH_DFTB, PH_CONV, PH_ACCEPT, PH_INIT, PH_TOTAL,
             PH_RA, PH_RB, PH_RC, PH_RD, PH_RE, PH_SIGX, PH_LSSET, PH_FILT, PH_COUNT };
#ifdef NMPC_STAMPS
#define STAMP0() const unsigned long long _ts0 = __builtin_amdgcn_s_memtime()
#define STAMPV0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define STAMPV1(v, ph) do { const unsigned long long _tv1 = __builtin_amdgcn_s_memtime(); \
    if (lanef() == 0) stamps[ph] += (double)(_tv1 - v); } while (0)
#ifndef NMPC_XSTAMPS
#define STAMP1(ph) do { const unsigned long long _ts1 = __builtin_amdgcn_s_memtime(); \
    if (lanef() == 0) stamps[ph] += (double)(_ts1 - _ts0); } while (0)
#else
#define STAMP1(ph) do { (void)_ts0; } while (0)
#endif
#else
#define STAMP0() do {} while (0)
#define STAMP1(ph) do {} while (0)
#endif
// -DNMPC_RESTO_TRIAL_STAMPS (diagnostics, with NMPC_STAMPS): the slots PH_BARR / PH_FTB /
// PH_DFTB record the restoration line search instead -- cycles inside trial_resto, cycles
// of second-order-correction blocks, number of trial_resto calls
#if defined(NMPC_STAMPS) && defined(NMPC_RESTO_TRIAL_STAMPS)
#define STAMP1G(ph) do {} while (0)
#define RSTAMP0(v) STAMPV0(v)
#define RSTAMP1(v, ph) STAMPV1(v, ph)
#define RCOUNT(ph) do { if (lanef() == 0) stamps[ph] += 1.0; } while (0)
#else
#define STAMP1G(ph) STAMP1(ph)
#define RSTAMP0(v) do {} while (0)
#define RSTAMP1(v, ph) do {} while (0)
#define RCOUNT(ph) do {} while (0)
#endif
#ifndef NMPC_STAMPS
#define STAMPV0(v) do {} while (0)
#define STAMPV1(v, ph) do {} while (0)
#endif
// -DNMPC_XSTAMPS (diagnostics, with NMPC_STAMPS): the generic phase timers are off and the
// slots record the parts of a restoration iteration instead (scripts/chain_xphases.py;
// slots 14, 15, 17, 18 keep their generic meaning)
enum XPhase { X_TCTRL = 0, X_TROLL = 1, X_TEVAL = 2, X_TROWS = 3, X_TFIN = 4, X_TCNT = 5, X_SCMS = 6,
              X_SASM = 7, X_SRES = 8, X_SFWD = 9, X_SBLK = 10, X_NASM = 11, X_NRIC = 12, X_NFIN = 13,
              X_CONV = 16, X_ACC = 19, X_DER = 20, X_LS = 21, X_IT = 22, X_ICNT = 23 };
#if defined(NMPC_STAMPS) && defined(NMPC_XSTAMPS)
#define XSTAMP0(v) STAMPV0(v)
#define XSTAMP1(v, ph) STAMPV1(v, ph)
#define XCOUNT(ph) do { if (lanef() == 0) stamps[ph] += 1.0; } while (0)
#else
#define XSTAMP0(v) do {} while (0)
#define XSTAMP1(v, ph) do {} while (0)
#define XCOUNT(ph) do {} while (0)
#endif

template <class CAP>
struct Solver {
  // stage loops with a lane-dependent range run to the class maximum with a guard
  // (fully unrolled, so their loads issue together) for classes up to 32 stages
  static constexpr bool kUnrollStages = CAP::nmax <= 32;
  static constexpr int kStageUnroll = kUnrollStages ? CAP::nmax : 1;
  // row of `inc` past every stage row (make_layout): -0.0 entries, the additive identity
  // that the unrolled prefix / suffix sums read where a lane's guard is off
  static constexpr int kZeroRow = CAP::nmax + 1;
  const CST Params* __restrict__ P;
  LDS double* sm;
  int lane_, b;
  // The lane index is re-materialised behind an empty asm at every use so the
  // compiler cannot hoist per-lane address arithmetic of every array out of
  // the main loop (that LICM kept ~200 extra VGPRs live for the whole kernel).
  __device__ __forceinline__ int lanef() const { int x = lane_; asm volatile("" : "+v"(x)); return x; }
  // Row-parallel pass, latency-batched: rows r = lane + 64 t are visited CAP::ru trips
  // at a time with a clamped index, f(r, on) with on = (r < ng).  Bodies load every
  // operand unconditionally and fold masked rows out with selects, so a group of
  // trips is one basic block whose global loads are all in flight together (a plain
  // `for (r = lane; r < ng; r += 64)` with loads under `if (hasl(..))` waits on
  // memory several times per trip).  Per lane the rows are still visited in
  // increasing order, so reductions are bitwise those of the plain loop.
  template <int RU = CAP::ru, class F>
  __device__ __forceinline__ void rows(F&& f) const {
    for (int base = 0; base < ng; base += RU * WAVE) {
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int r = base + u * WAVE + lanef();
        const bool on = r < ng;
        f(on ? r : ng - 1, on);
      }
    }
  }
  // the restoration phase's row passes read its global row vectors (p, n, their
  // multipliers and steps) besides the LDS rows: in the LDS-row class they take more trips
  // per group (fewer global round trips per pass); per lane the rows are still visited in
  // increasing order, so the sums are bitwise those of rows()
#ifndef NMPC_RESTO_RU
#define NMPC_RESTO_RU 2
#endif
  static constexpr int kRestoRU = CAP::lds_rows ? (NMPC_RESTO_RU < CAP::rtrips ? NMPC_RESTO_RU : CAP::rtrips) : CAP::ru;
  template <class F>
  __device__ __forceinline__ void rows_r(F&& f) const { rows<kRestoRU>(static_cast<F&&>(f)); }
  // the same for the decision variables (index clamped to the last one when off: every
  // load is valid, so a pass's loads over its trips issue together; f guards its sums and
  // stores with `on`)
  template <class F>
  __device__ __forceinline__ void ctrls(F&& f) const {
    for (int base = 0; base < nw; base += CAP::cu * WAVE) {
#pragma unroll
      for (int u = 0; u < CAP::cu; ++u) {
        const int i = base + u * WAVE + lanef();
        const bool on = i < nw;
        f(on ? i : nw - 1, on);
      }
    }
  }
  int N, m, nobs, nw, ng;
  int nb, nuE, nwE;  // box rows per stage; real controls per stage; real decision length
  double T;
  // pointers into LDS
  GLB double* U, *Ut, *dU, *dU2, *zl, *zu, *xl, *xu, *sigx, *ru, *rres, *dUr;
  LDS double* rdX;
  LDS double* X, *Xt, *dX;
  using RV = typename CAP::RowT;  // hot row vectors: LDS or global (Cap::lds_rows)
  RV *s, *y, *vl, *vu, *d, *ds, *ds2, *dc;
  using DTT = std::conditional_t<CAP::lds_rows && !CAP::refine, LDS double, GLB double>;
  DTT* dt;
  GLB double* dms;
  GLB double *UR, *zl0, *zu0, *s0, *vl0, *vu0, *pR, *nR, *zpR, *znR, *dpR, *dnR, *dyR, *dp2R, *dn2R, *dy2R, *cms, *filtR;
  GLB double *accU, *accZl, *accZu, *accY;
  int meq;                       // number of equality rows (0: none, the common case)
  int nneg;                      // negative Riccati pivots of the last factorization (SG sweeps)
  GLB double *wU, *wzl, *wzu, *wdU, *wsl, *wy, *wvl, *wvu, *wds, *wpR, *wnR, *wzpR, *wznR, *wdpR, *wdnR, *wdyR;
  double rho, etaR;  // restoration: penalty, proximity weight * sqrt(mu)
  double* wsbase;    // workspace base of all scenarios (restoration re-binds from it)
  RV *dl, *du;  // row bounds: LDS or global with the rows (Cap::lds_rows)
  LDS double* rvars;
  GLB double* gl, *Hl, *Qs;
  // The transcendental values a trial's rollout and stage costs form at its states (per
  // stage: cos/sin theta, cos/sin psi, the four FOV tangents, cos/sin x7, the target
  // distance), two buffers: trial group 0 (every single rollout / eval_fg) and group 1 (the
  // second trial of a speculative pair).  The derivatives at an accepted trial point read
  // them instead of evaluating them again (Solver::derivs<.., true>): the same functions of
  // the same doubles, so the same values.
  GLB double* tc;
  static constexpr int TCS = 12 * (CAP::nmax + 1);
  LDS double* trig, *qs, *lam;
  GLB double* K, *Rk;
  using KFT = std::conditional_t<CAP::lds_rows, LDS double, GLB double>;
  KFT* kf;  // k_k: LDS for the LDS-row class, workspace otherwise
  LDS double* Rc, *Rv, *Pa, *Pb, *pva, *pvb, *St;
  LDS double* pp, *obx, *oby, *inc, *stamps;
  GLB double* filt;
  LDS int* fixm;  // fixed decision variables (lbx == ubx, make_parameter): bit c of stage k
  // uniform scalars
  double df, mu, tau, delta;
  int nfilt;
  int nzx, nzs;
  int nfix;  // number of fixed decision variables (0: none, the common case)
  __device__ __forceinline__ bool fixed(int i) const {  // decision i = 6k + c (internal layout)
    return nfix > 0 && ((fixm[i / 6] >> (i - 6 * (i / 6))) & 1);
  }

  __device__ __forceinline__ void bind(const Params* prm, double* smem, double* wsp, int lane_, int b_) {
    constexpr Lay L = CAP::L;
    P = (const CST Params*)prm; sm = (LDS double*)smem; this->lane_ = lane_; b = b_;
    N = prm->N; m = prm->m; nobs = prm->nobs; nw = prm->nw; ng = prm->ng; T = prm->T;
    // the step lives in a VGPR pair: every stage sweep multiplies by it, and as a uniform
    // SGPR pair it is one of the values spilled to VGPR lanes and restored at each use
    asm volatile("" : "+v"(T));
    nb = prm->nb; nuE = prm->nuE; nwE = prm->nwE;
    wsbase = wsp;
    GLB double* gw = (GLB double*)(wsp + (long long)b_ * L.wstotal);
    U = gw + L.U; Ut = gw + L.Ut; dU = gw + L.dU; dU2 = gw + L.dU2;
    zl = gw + L.zl; zu = gw + L.zu; xl = gw + L.xl; xu = gw + L.xu;
    sigx = gw + L.sigx; ru = gw + L.ru; rres = gw + L.rres; dUr = gw + L.dUr; rdX = sm + L.rdX;
    X = sm + L.X; Xt = sm + L.Xt; dX = sm + L.dX;
    auto rvp = [&](int off) -> RV* {
      if constexpr (CAP::lds_rows) return (RV*)(sm + off);
      else return (RV*)(gw + off);
    };
    s = rvp(L.s); y = rvp(L.y); vl = rvp(L.vl); vu = rvp(L.vu);
    d = rvp(L.d); ds = rvp(L.ds); ds2 = rvp(L.ds2);
    if constexpr (CAP::lds_rows && !CAP::refine) dt = (DTT*)(sm + L.dt);
    else dt = (DTT*)(gw + L.dt);
    dc = rvp(L.dc); dl = rvp(L.dl); du = rvp(L.du); dms = gw + L.dms; rvars = sm + L.rvars;
    UR = gw + L.UR; zl0 = gw + L.zl0; zu0 = gw + L.zu0; s0 = gw + L.s0; vl0 = gw + L.vl0; vu0 = gw + L.vu0;
    pR = gw + L.pR; nR = gw + L.nR; zpR = gw + L.zpR; znR = gw + L.znR; dpR = gw + L.dpR; dnR = gw + L.dnR;
    dyR = gw + L.dyR; dp2R = gw + L.dp2R; dn2R = gw + L.dn2R; dy2R = gw + L.dy2R; cms = gw + L.cms;
    filtR = gw + L.filtR;
    accU = gw + L.accU; accZl = gw + L.accZl; accZu = gw + L.accZu; accY = gw + L.accY;
    meq = 0; nneg = 0;
    wU = gw + L.wU; wzl = gw + L.wzl; wzu = gw + L.wzu; wdU = gw + L.wdU; wsl = gw + L.ws; wy = gw + L.wy;
    wvl = gw + L.wvl; wvu = gw + L.wvu; wds = gw + L.wds; wpR = gw + L.wpR; wnR = gw + L.wnR;
    wzpR = gw + L.wzpR; wznR = gw + L.wznR; wdpR = gw + L.wdpR; wdnR = gw + L.wdnR; wdyR = gw + L.wdyR;
    gl = gw + L.gl; Hl = gw + L.Hl; tc = gw + L.tc; trig = sm + L.trig; Qs = gw + L.Qs; qs = sm + L.qs;
    lam = sm + L.lam;
    K = gw + L.K; Rk = gw + L.Rk; Rc = sm + L.Rc; Rv = sm + L.Rv;
    if constexpr (CAP::lds_rows) kf = (KFT*)(sm + L.kf);
    else kf = (KFT*)(gw + L.kf);
    Pa = sm + L.P0; Pb = sm + L.P1; pva = sm + L.pv0; pvb = sm + L.pv1;
    St = sm + L.St;
    pp = sm + L.p; obx = sm + L.ob; oby = obx + NMPC_MAX_OBS; inc = sm + L.inc;
    filt = gw + L.filt;
    stamps = sm + L.red;
    fixm = (LDS int*)(sm + L.fixm);
    nfix = 0;
  }

  __device__ __forceinline__ bool hasl(double v) const { return v > -INFINITY; }
  __device__ __forceinline__ bool hasu(double v) const { return v < INFINITY; }

  // ------------------------------------------------------------------ rollout
  // X[:,0] = p[0:8]; X[:,k+1] = X[:,k] + T f(X[:,k],U[:,k])   (NMPC_TT.py:160-167)
  // Each lanef() k sums the increments j<k in order, i.e. bitwise the sequential
  // recursion; the (x,y,z) increments need theta_j, psi_j, so two passes.
  // (dUs non-null: the controls are Us + a dUs, formed here from the two vectors rather
  // than read back from the trial point just stored -- the same doubles; pre non-null: the
  // two vectors' stage entries were loaded ahead by preload_u)
  struct UPre { double u[6], du[6]; };
  // a trial's stage controls loaded ahead, so the trial's rollout does not start by waiting
  // on them (issued before the trial's control pass): lane l holds stage (l & kmask)'s
  // entries of Us and dUs (clamped stage: no lane-dependent branch)
  __device__ __forceinline__ UPre preload_u(const GLB double* Us, const GLB double* dUs, int kmask) const {
    UPre q;
    const int k = lanef() & kmask;
    const int kc = k < N ? k : 0;
#pragma unroll
    for (int c = 0; c < 6; ++c) { q.u[c] = Us[kc * 6 + c]; q.du[c] = dUs[kc * 6 + c]; }
    return q;
  }
  __device__ __forceinline__ void rollout(const GLB double* Us, LDS double* Xd, const GLB double* dUs = nullptr,
                                          double a_ = 0.0, const UPre* pre = nullptr) {
    STAMP0();
    const int k = lanef();
    auto uk = [&](int c) {  // stage k's control c
      const int j = k * 6 + c;
      return pre ? pre->u[c] + a_ * pre->du[c] : (dUs ? Us[j] + a_ * dUs[j] : Us[j]);
    };
    const double v = k < N ? uk(0) : 0.0;
    if (k < N) {
#pragma unroll
      for (int c = 0; c < 5; ++c) inc[k * 8 + c] = T * uk(1 + c);
    }
    if (kUnrollStages && k < 8) inc[kZeroRow * 8 + k] = -0.0;
    sync();
    double a[5];
    if (k <= N) {
#pragma unroll
      for (int c = 0; c < 5; ++c) a[c] = pp[3 + c];
      if constexpr (kUnrollStages) {
        // every lane reads a row per j -- its increment row while j < k, the -0.0 row
        // otherwise (x + -0.0 == x exactly) -- so the reads carry no lane-dependent branch
        // and issue together; the sums are bitwise the guarded in-order recursion
#pragma unroll
        for (int j = 0; j < CAP::nmax; ++j) {
          const LDS double* ij = inc + (j < k ? j : kZeroRow) * 8;
#pragma unroll
          for (int c = 0; c < 5; ++c) a[c] = a[c] + ij[c];
        }
      } else {
        for (int j = 0; j < k; ++j) {
#pragma unroll
          for (int c = 0; c < 5; ++c) a[c] = a[c] + inc[j * 8 + c];
        }
      }
      {  // (stage N too: its trig goes to the cache only)
        const double ct = cos(a[0]), st_ = sin(a[0]), cp = cos(a[1]), sp = sin(a[1]);
        if (k < N) {
          inc[k * 8 + 5] = T * (v * cp * ct);
          inc[k * 8 + 6] = T * (v * sp * ct);
          inc[k * 8 + 7] = T * (v * st_);
        }
        GLB double* tk = tc + k * 12;
        tk[0] = ct; tk[1] = st_; tk[2] = cp; tk[3] = sp;
      }
    }
    sync();
    if (k <= N) {
      double c0 = pp[0], c1 = pp[1], c2 = pp[2];
      if constexpr (kUnrollStages) {
#pragma unroll
        for (int j = 0; j < CAP::nmax; ++j) {
          const LDS double* ij = inc + (j < k ? j : kZeroRow) * 8;
          c0 = c0 + ij[5];
          c1 = c1 + ij[6];
          c2 = c2 + ij[7];
        }
      } else {
        for (int j = 0; j < k; ++j) {
          c0 = c0 + inc[j * 8 + 5];
          c1 = c1 + inc[j * 8 + 6];
          c2 = c2 + inc[j * 8 + 7];
        }
      }
      LDS double* xk = Xd + k * 8;
      xk[0] = c0; xk[1] = c1; xk[2] = c2;
#pragma unroll
      for (int c = 0; c < 5; ++c) xk[3 + c] = a[c];
    }
    STAMP1(PH_ROLLOUT);
    sync();
  }

  // The FOV tangents tan(x +- h) of one angle (NMPC_TT.py:209-214).  NMPC_TAN2: from the
  // one tangent t = tan(x) by the addition formula, tan(x +- h) = (t +- tan h) / (1 -+ t tan h)
  // with tan h formed on the host -- one fp64 tangent (OCML: a Payne-Hanek / Cody-Waite
  // reduction and a rational approximation, ~100 dependent operations) and two reciprocals
  // instead of two tangents; a few ulp apart from the direct forms (no cancellation in
  // 1 -+ t tan h while |x| < pi/2 - h).
#ifndef NMPC_TAN2
#define NMPC_TAN2 0
#endif
  __device__ __forceinline__ static void tan_pm(double x, double h, double th, double& tp, double& tm) {
    if constexpr (NMPC_TAN2) {
      const double t = tan(x);
      const double ct = t * th;
      tp = (t + th) * rcp(1.0 - ct);
      tm = (t - th) * rcp(1.0 + ct);
    } else {
      tp = tan(x + h);
      tm = tan(x - h);
    }
  }

  // ---------------------------------------------------------- stage cost value
  // Literal restatement of NMPC_TT.py:209-220 (same operation order as the
  // oracle's stage_cost).
  // (tw non-null: the tangents, cos/sin x7 and the target distance also go to the cache)
  __device__ __forceinline__ double stage_cost(const LDS double* x, GLB double* tw = nullptr) const {
    const double hv = P->hv, hh = P->hh;
    const double z = x[2];
    double t6p, t6m, t5p, t5m;
    tan_pm(x[6], hv, P->thv, t6p, t6m);
    tan_pm(x[5], hh, P->thh, t5p, t5m);
    const double a = (z * t6p - z * t6m) / 2;
    const double bb = (z * t5p - z * t5m) / 2;
    const double c7 = cos(x[7]), s7 = sin(x[7]);
    const double a2 = a * a, b2 = bb * bb;
    // (the compiler's divisions: with qd() the objective value moved in its last bit at a few
    // points of the round-6 bitwise A/B -- cause not isolated -- so they stay)
    const double A = (c7 * c7) / a2 + (s7 * s7) / b2;
    const double Bq = 2 * c7 * s7 * ((1 / a2) - (1 / b2));
    const double C = (s7 * s7) / a2 + (c7 * c7) / b2;
    const double XE = x[0] + a + z * t6m;
    const double YE = x[1] + bb + z * t5m;
    const double xt = pp[8], yt = pp[9];
    const double ex = xt - XE, ey = yt - YE;
    const double dx = x[0] - xt, dy = x[1] - yt;
    const double dd = sqrt(dx * dx + dy * dy);
    if (tw) {
      tw[4] = t6p; tw[5] = t6m; tw[6] = t5p; tw[7] = t5m; tw[8] = c7; tw[9] = s7; tw[10] = dd;
    }
    return rvars[30] * dd + rvars[31] * ((A * (ex * ex) + Bq * ey * ex + C * (ey * ey)) - 1);
  }

  __device__ __forceinline__ double row_value(const LDS double* x, int i) const {
    if (i < nb) return x[boxidx(i)];
    const int o = i - nb;
    const double ddx = x[0] - obx[o], ddy = x[1] - oby[o];
    return -sqrt(ddx * ddx + ddy * ddy) + P->orr[o];
  }

  // f = sum_k l_k(X) and rows dst[r] = dc[r] * g_r(X) (dc may be null -> unscaled)
  // (obj = false: the rows only, f = 0 -- the restoration line search, whose trials are judged
  // without the original objective; eval_f forms it for the accepted trial alone)
  template <class DP>
  __device__ __forceinline__ double eval_fg(const LDS double* Xs, DP dst, const RV* scale, bool obj = true) {
    STAMP0();
    const int k = lanef();
    double f = 0.0;
    if (k <= N) {
      const LDS double* xk = Xs + k * 8;
      if (obj && k < N) f = stage_cost(xk, tc + k * 12);
      if constexpr (!CAP::deep) {  // register-limited classes: one row at a time (fewer live values)
#pragma unroll
        for (int i = 0; i < CAP::mmax; ++i) {
          if (i < m) {
            const int r = k * m + i;
            const double g = row_value(xk, i);
            dst[r] = scale ? scale[r] * g : g;
          }
        }
      } else {
        // unrolled over the layout's row capacity; every row value is formed unconditionally
        // (clamped obstacle index) before the guarded stores, so the obstacle rows' loads and
        // square roots overlap instead of running one row at a time behind the wave-uniform
        // row-kind branches (same operations as row_value, so the same bits)
        const double x0 = xk[0], x1 = xk[1];
        double gv[CAP::mmax];
#pragma unroll
        for (int i = 0; i < CAP::mmax; ++i) {
          const int oi = i - nb;
          const int o = oi < 0 ? 0 : (oi < NMPC_MAX_OBS ? oi : NMPC_MAX_OBS - 1);
          const double ddx = x0 - obx[o], ddy = x1 - oby[o];
          const double ov = -sqrt(ddx * ddx + ddy * ddy) + P->orr[o];
          gv[i] = i < 5 ? (i < nb ? xk[boxidx(i < 5 ? i : 0)] : ov) : ov;
        }
#pragma unroll
        for (int i = 0; i < CAP::mmax; ++i) {
          if (i < m) {
            const int r = k * m + i;
            dst[r] = scale ? scale[r] * gv[i] : gv[i];
          }
        }
      }
    }
    sync();
    const double fs = wsum(f);
    STAMP1(PH_EVAL);
    return fs;
  }

  // the objective alone, sum_k l_k(X), its transcendental values into the cache buffer tcb:
  // the same stage costs as eval_fg's, summed by the same wave reduction over the same lanes
  // (stage k on lane k, zeros elsewhere), so the same f -- also for a pair's second trial,
  // whose eval_fg2 sum over lanes 32 + k the butterfly forms in the same order
  __device__ __forceinline__ double eval_f(const LDS double* Xs, GLB double* tcb) {
    STAMP0();
    const int k = lanef();
    double f = 0.0;
    if (k < N) f = stage_cost(Xs + k * 8, tcb + k * 12);
    const double fs = wsum(f);
    STAMP1(PH_EVAL);
    return fs;
  }

  // ------------------------------------ two line-search trials' stage work at once
  // The restoration line search's next backtracking trial (a1 = a0 * alpha_red_factor) has
  // its rollout and row values formed together with the current one's (a0): the stage-
  // parallel work uses N + 1 of 64 lanes, so lanes 32 + k carry stage k of the second trial
  // in the same instructions.  Group 0 (lanes 0..31) writes Xt / dt and its increments to
  // `inc` exactly as rollout / eval_fg do; group 1 writes its X to `lam`, its row values to
  // `dms` and its increments to `qs` (all three dead during a line search: lam is re-formed
  // by the next adjoint, qs by the next assembly, dms is the main phase's scratch).  Every
  // stage's arithmetic is that of rollout / eval_fg, and the objective's wave sum of group 1
  // sits in lanes 32..63 -- the butterfly reduces each 32-lane half in the same order, so
  // both objectives are bitwise those of two separate calls.
  static constexpr bool kSpec = CAP::lds_rows && !CAP::refine && !CAP::eq && CAP::nmax <= 31;
  // Scratch of a pair's second trial: its increments in qs (stride 8, rows 0..nmax + 1, so
  // they overwrite the S_k terms qs[k*10 + 8..9]), its X in lam, its rows in dms.  This is
  // sound because (i) every Newton assembly rewrites qs[k*10 + 8..9] before the next
  // factorisation reads them, and nothing else reads them between (the restoration SOC
  // block's assemble(SUM_RESTO_SOC) writes q_k only, resolve / forward read q_k only, and
  // the refinement that reads S_k is compiled out of the kSpec classes); (ii) between the
  // pair's formation and a from_pair acceptance nothing writes lam or dms (the SOC block's
  // re-solve, forward sweep, row step and spec = 0 trial write qs[0..7], dX, ds2, the
  // *2R vectors, Xt and dt).  Bitwise check against Params::nospec:
  // test_speculative_restoration_pairs_are_bitwise_neutral.
  static_assert(!kSpec || 8 * (CAP::nmax + 2) <= 10 * (CAP::nmax + 1), "qs cannot hold a pair's increments");
  __device__ __forceinline__ void rollout2(const GLB double* Us, const GLB double* dUs, double a0, double a1,
                                           const UPre* pre = nullptr) {
    STAMP0();
    const int l = lanef();
    const int grp = l >> 5, k = l & 31;
    const double a_ = grp ? a1 : a0;
    LDS double* ic = grp ? qs : inc;
    LDS double* Xd = grp ? lam : Xt;
    GLB double* tcg = tc + (grp ? TCS : 0);
    auto uk = [&](int c) {  // stage k's control c
      const int j = k * 6 + c;
      return pre ? pre->u[c] + a_ * pre->du[c] : Us[j] + a_ * dUs[j];
    };
    const double v = k < N ? uk(0) : 0.0;
    if (k < N) {
#pragma unroll
      for (int c = 0; c < 5; ++c) ic[k * 8 + c] = T * uk(1 + c);
    }
    if (k < 8) ic[kZeroRow * 8 + k] = -0.0;
    sync();
    double a[5];
    if (k <= N) {
#pragma unroll
      for (int c = 0; c < 5; ++c) a[c] = pp[3 + c];
#pragma unroll
      for (int j = 0; j < CAP::nmax; ++j) {
        const LDS double* ij = ic + (j < k ? j : kZeroRow) * 8;
#pragma unroll
        for (int c = 0; c < 5; ++c) a[c] = a[c] + ij[c];
      }
      {
        const double ct = cos(a[0]), st_ = sin(a[0]), cp = cos(a[1]), sp = sin(a[1]);
        if (k < N) {
          ic[k * 8 + 5] = T * (v * cp * ct);
          ic[k * 8 + 6] = T * (v * sp * ct);
          ic[k * 8 + 7] = T * (v * st_);
        }
        GLB double* tk = tcg + k * 12;
        tk[0] = ct; tk[1] = st_; tk[2] = cp; tk[3] = sp;
      }
    }
    sync();
    if (k <= N) {
      double c0 = pp[0], c1 = pp[1], c2 = pp[2];
#pragma unroll
      for (int j = 0; j < CAP::nmax; ++j) {
        const LDS double* ij = ic + (j < k ? j : kZeroRow) * 8;
        c0 = c0 + ij[5];
        c1 = c1 + ij[6];
        c2 = c2 + ij[7];
      }
      LDS double* xk = Xd + k * 8;
      xk[0] = c0; xk[1] = c1; xk[2] = c2;
#pragma unroll
      for (int c = 0; c < 5; ++c) xk[3 + c] = a[c];
    }
    STAMP1(PH_ROLLOUT);
    sync();
  }
  // f and scaled rows of both trials (eval_fg's deep form): group 0 -> dt, f0; group 1 -> dms, f1
  __device__ __forceinline__ void eval_fg2(double& f0, double& f1, bool obj = true) {
    STAMP0();
    const int l = lanef();
    const int grp = l >> 5, k = l & 31;
    double f = 0.0;
    if (k <= N) {
      const LDS double* xk = (grp ? lam : Xt) + k * 8;
      if (obj && k < N) f = stage_cost(xk, tc + (grp ? TCS : 0) + k * 12);
      const double x0 = xk[0], x1 = xk[1];
      double gv[CAP::mmax];
#pragma unroll
      for (int i = 0; i < CAP::mmax; ++i) {
        const int oi = i - nb;
        const int o = oi < 0 ? 0 : (oi < NMPC_MAX_OBS ? oi : NMPC_MAX_OBS - 1);
        const double ddx = x0 - obx[o], ddy = x1 - oby[o];
        const double ov = -sqrt(ddx * ddx + ddy * ddy) + P->orr[o];
        gv[i] = i < 5 ? (i < nb ? xk[boxidx(i < 5 ? i : 0)] : ov) : ov;
      }
#pragma unroll
      for (int i = 0; i < CAP::mmax; ++i) {
        if (i < m) {
          const int r = k * m + i;
          const double v = dc[r] * gv[i];
          if (grp) dms[r] = v;
          else dt[r] = v;
        }
      }
    }
    sync();
    f0 = wsum(grp ? 0.0 : f);
    f1 = wsum(grp ? f : 0.0);
    STAMP1(PH_EVAL);
  }

  // --------------------------------------------- stage derivatives at X (lanef()=k)
  // gl[k] = grad l_k (8), Hl[k] = hess l_k packed over (x,y,z,x5,x6,x7), trig[k].
  // Derivation: oracle/nmpc_oracle.py::stage_cost_derivs (Q = (r1/a)^2+(r2/b)^2).
  // HESS = false: trig and the gradient only -- the restoration phase weights the original
  // objective by 0 (hfac = 0 in its assembly, so Hl is never read there; its 0 * gl terms
  // keep the gradient's exact values); the full derivatives are formed again when it
  // returns to the original problem
  // TC: the transcendental values come from the cache buffer tcr, written by the rollout and
  // stage costs that formed Xs (the callers pass the buffer of the trial that became Xs)
  template <bool HESS = true, bool TC = false>
  __device__ __forceinline__ void derivs(const LDS double* Xs, const GLB double* Us,
                                         const GLB double* tcr = nullptr) {
    STAMP0();
    const int k = lanef();
    if (k <= N) {
      const LDS double* xk = Xs + k * 8;
      const double th = xk[3], ps = xk[4];
      LDS double* tg = trig + k * 8;
      const GLB double* tk = TC ? tcr + k * 12 : nullptr;
      if constexpr (TC) {
        tg[0] = tk[0]; tg[1] = tk[1]; tg[2] = tk[2]; tg[3] = tk[3];
      } else {
        tg[0] = cos(th); tg[1] = sin(th); tg[2] = cos(ps); tg[3] = sin(ps);
      }
      tg[4] = (k < N) ? Us[k * 6] : 0.0;
      GLB double* g8 = gl + k * 8;
      GLB double* H = Hl + k * 21;
      if (k == N) {
        for (int i = 0; i < 8; ++i) g8[i] = 0.0;
        if (HESS)
          for (int i = 0; i < 21; ++i) H[i] = 0.0;
      } else {
        const double hv = P->hv, hh = P->hh;
        const double x = xk[0], yy = xk[1], z = xk[2], x5 = xk[5], x6 = xk[6], x7 = xk[7];
        const double xt = pp[8], yt = pp[9];
        double t6p, t6m, t5p, t5m;
        if constexpr (TC) {
          t6p = tk[4]; t6m = tk[5]; t5p = tk[6]; t5m = tk[7];
        } else {
          tan_pm(x6, hv, P->thv, t6p, t6m);
          tan_pm(x5, hh, P->thh, t5p, t5m);
        }
        const double al6 = (t6p - t6m) / 2, be6 = (t6p + t6m) / 2;
        const double al5 = (t5p - t5m) / 2, be5 = (t5p + t5m) / 2;
        const double al6d = (t6p * t6p - t6m * t6m) / 2, be6d = (2 + t6p * t6p + t6m * t6m) / 2;
        const double al5d = (t5p * t5p - t5m * t5m) / 2, be5d = (2 + t5p * t5p + t5m * t5m) / 2;
        const double s6p = t6p * (1 + t6p * t6p), s6m = t6m * (1 + t6m * t6m);
        const double s5p = t5p * (1 + t5p * t5p), s5m = t5m * (1 + t5m * t5m);
        const double al6dd = s6p - s6m, be6dd = s6p + s6m;
        const double al5dd = s5p - s5m, be5dd = s5p + s5m;
        const double ex = xt - x - z * be6;
        const double ey = yt - yy - z * be5;
        double gex[6] = {-1.0, 0.0, -be6, 0.0, -z * be6d, 0.0};
        double gey[6] = {0.0, -1.0, -be5, -z * be5d, 0.0, 0.0};
        const double a = z * al6, bb = z * al5;
        double ga[6] = {0.0, 0.0, al6, 0.0, z * al6d, 0.0};
        double gb[6] = {0.0, 0.0, al5, z * al5d, 0.0, 0.0};
        const double c = TC ? tk[8] : cos(x7), sn = TC ? tk[9] : sin(x7);
        const double r1 = c * ex + sn * ey;
        const double r2 = sn * ex - c * ey;
        double u1[6], u2[6], gr1[6], gr2[6], ge1[6], ge2[6];
        const double ia = qd(1.0, a), ib = qd(1.0, bb);
        const double e1 = r1 * ia, e2 = r2 * ib;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          u1[q] = -sn * gex[q] + c * gey[q];
          u2[q] = c * gex[q] + sn * gey[q];
          gr1[q] = c * gex[q] + sn * gey[q] - (q == 5 ? r2 : 0.0);
          gr2[q] = sn * gex[q] - c * gey[q] + (q == 5 ? r1 : 0.0);
          ge1[q] = (gr1[q] - e1 * ga[q]) * ia;
          ge2[q] = (gr2[q] - e2 * gb[q]) * ib;
        }
        const double ddx = x - xt, ddy = yy - yt;
        const double dd = TC ? tk[10] : sqrt(ddx * ddx + ddy * ddy);
        const double idd = qd(1.0, dd);
        const double id3 = idd * idd * idd;
        const double w1 = rvars[30], w2 = rvars[31];  // this scenario's cost weights
        // gradient
        double g6[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) g6[q] = w2 * (2 * (e1 * ge1[q] + e2 * ge2[q]));
        g6[0] += w1 * (ddx * idd);
        g6[1] += w1 * (ddy * idd);
        g8[0] = g6[0]; g8[1] = g6[1]; g8[2] = g6[2]; g8[3] = 0.0; g8[4] = 0.0;
        g8[5] = g6[3]; g8[6] = g6[4]; g8[7] = g6[5];
        // Hessian, 21 packed entries
#pragma unroll
        for (int qa = 0; qa < (HESS ? 6 : 0); ++qa) {
#pragma unroll
          for (int qb = qa; qb < 6; ++qb) {
            // sparse second derivatives of ex, ey, a, b
            double Hex = 0.0, Hey = 0.0, Ha = 0.0, Hb = 0.0;
            if ((qa == 2 && qb == 4)) { Hex = -be6d; Ha = al6d; }
            if (qa == 4 && qb == 4) { Hex = -z * be6dd; Ha = z * al6dd; }
            if ((qa == 2 && qb == 3)) { Hey = -be5d; Hb = al5d; }
            if (qa == 3 && qb == 3) { Hey = -z * be5dd; Hb = z * al5dd; }
            const double e7a = (qa == 5) ? 1.0 : 0.0, e7b = (qb == 5) ? 1.0 : 0.0;
            const double Hr1 = c * Hex + sn * Hey + e7a * u1[qb] + u1[qa] * e7b - r1 * e7a * e7b;
            const double Hr2 = sn * Hex - c * Hey + e7a * u2[qb] + u2[qa] * e7b - r2 * e7a * e7b;
            const double He1 = (Hr1 - ge1[qa] * ga[qb] - ga[qa] * ge1[qb] - e1 * Ha) * ia;
            const double He2 = (Hr2 - ge2[qa] * gb[qb] - gb[qa] * ge2[qb] - e2 * Hb) * ib;
            double h = w2 * (2 * (ge1[qa] * ge1[qb] + ge2[qa] * ge2[qb] + e1 * He1 + e2 * He2));
            if (qa == 0 && qb == 0) h += w1 * (ddy * ddy * id3);
            if (qa == 0 && qb == 1) h += w1 * (-ddx * ddy * id3);
            if (qa == 1 && qb == 1) h += w1 * (ddx * ddx * id3);
            H[hp(qa, qb)] = h;
          }
        }
      }
    }
    STAMP1(PH_DERIVS);
    sync();
  }

  // E entries of A_k = I + E_k and first column b0 of B_k (oracle dyn_jac)
  __device__ __forceinline__ void stage_AB(int k, double& E03, double& E04, double& E13,
                                           double& E14, double& E23, double& b00, double& b10,
                                           double& b20) const {
    stage_AB(k, T, E03, E04, E13, E14, E23, b00, b10, b20);
  }
  // ... with the step T passed in (a VGPR copy inside the sweeps)
  __device__ __forceinline__ void stage_AB(int k, double T, double& E03, double& E04, double& E13,
                                           double& E14, double& E23, double& b00, double& b10,
                                           double& b20) const {
    const LDS double* tg = trig + k * 8;
    const double ct = tg[0], stt = tg[1], cp = tg[2], sp = tg[3], v = tg[4];
    E03 = -T * v * cp * stt; E04 = -T * v * sp * ct;
    E13 = -T * v * sp * stt; E14 = T * v * cp * ct;
    E23 = T * v * ct;
    b00 = T * cp * ct; b10 = T * sp * ct; b20 = T * stt;
  }
  // a stage's A / B entries, formed a stage ahead in the backward sweeps: they depend on
  // trig only, not on the recursion, and formed at the stage itself their LDS reads and
  // three-deep products sat on the stage's critical path behind its barrier
  struct StageAB { double E03, E04, E13, E14, E23, b00, b10, b20; };
  __device__ __forceinline__ StageAB stage_ab(int k, double T) const {
    StageAB a;
    stage_AB(k, T, a.E03, a.E04, a.E13, a.E14, a.E23, a.b00, a.b10, a.b20);
    return a;
  }

  // --------------------------------------------- adjoint lam_k (lanef() = k)
  // lam_N = G_N^T y_N; lam_k = ofac*gl_k + G_k^T y_k + A_k^T lam_{k+1}
  // (oracle SSEval.hessian).  yy may be null (objective only).
  template <class YP>
  __device__ __forceinline__ void adjoint(double ofac, YP yy) {
    STAMP0();
    const int k = lanef();
    LDS double* wv = inc;  // scratch 8*(N+1)
    if (k <= N) {
      double w[8];
      const LDS double* xk = X + k * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = ofac * gl[k * 8 + i];
      if (yy) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {  // nb <= 5 box rows
          if (i < nb) {
            const int r = k * m + i;
            w[boxidx(i)] += dc[r] * yy[r];
          }
        }
        // compile-time bound so every row's loads issue before the first use
        double cyv[CAP::mmax - 5];
#pragma unroll
        for (int o = 0; o < CAP::mmax - 5; ++o) {
          const int r = k * m + nb + o;
          cyv[o] = o < nobs ? dc[r] * yy[r] : 0.0;
        }
        {
          // every obstacle term formed (LDS reads valid for o < NMPC_MAX_OBS) and kept by a
          // select: the rows' reads and square roots overlap (every class: the global-row
          // class of config 5 gained 2-3 % with no added spills, round 6)
          const double x0 = xk[0], x1 = xk[1];
#pragma unroll
          for (int o = 0; o < CAP::mmax - 5; ++o) {
            const double ddx = x0 - obx[o], ddy = x1 - oby[o];
            const double idd = rsq(ddx * ddx + ddy * ddy);
            const double n0 = w[0] + cyv[o] * (-(ddx * idd));
            const double n1 = w[1] + cyv[o] * (-(ddy * idd));
            w[0] = o < nobs ? n0 : w[0];
            w[1] = o < nobs ? n1 : w[1];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) wv[k * 8 + i] = w[i];
    }
    if (kUnrollStages && k < 8) wv[kZeroRow * 8 + k] = -0.0;
    sync();
    if (k <= N) {
      const int cs[6] = {0, 1, 2, 5, 6, 7};
      double acc[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) acc[q] = wv[N * 8 + cs[q]];
      // suffix sums in the oracle's order (j = N-1 down to k), unrolled to the class
      // maximum; a lane whose guard is off reads the -0.0 row (-0.0 + x == x exactly), so
      // the reads carry no lane-dependent branch and pipeline
      if constexpr (kUnrollStages) {
#pragma unroll
        for (int jj = CAP::nmax - 1; jj >= 0; --jj) {
          const LDS double* wj = wv + ((jj < N && jj >= k) ? jj : kZeroRow) * 8;
#pragma unroll
          for (int q = 0; q < 6; ++q) acc[q] = wj[cs[q]] + acc[q];
        }
      } else {
        for (int jj = N - 1; jj >= k; --jj) {
#pragma unroll
          for (int q = 0; q < 6; ++q) acc[q] = wv[jj * 8 + cs[q]] + acc[q];
        }
      }
#pragma unroll
      for (int q = 0; q < 6; ++q) lam[k * 8 + cs[q]] = acc[q];
    }
    sync();
    // stage j's terms of the theta / psi recursion, ((E03 l0 + E13 l1) + E23 l2) and
    // (E04 l0 + E14 l1) with l = lam_{j+1}: formed once, by lane j, into the w slots 5 and 6
    // (dead after the suffix sums), instead of by every lane for every stage -- the same
    // expressions, so the same bits
    if (k < N) {
      double E03, E04, E13, E14, E23, b00, b10, b20;
      stage_AB(k, E03, E04, E13, E14, E23, b00, b10, b20);
      const LDS double* ln = lam + (k + 1) * 8;
      wv[k * 8 + 5] = (E03 * ln[0] + E13 * ln[1]) + E23 * ln[2];
      wv[k * 8 + 6] = E04 * ln[0] + E14 * ln[1];
    }
    sync();
    if (k <= N) {
      double a3 = wv[N * 8 + 3], a4 = wv[N * 8 + 4];
      if constexpr (kUnrollStages) {
        // every lane reads each stage's terms (clamped stage index: valid reads, no
        // lane-dependent branch) and keeps the sum only where its guard holds
#pragma unroll
        for (int j = CAP::nmax - 1; j >= 0; --j) {
          const bool on = j < N && j >= k;
          const int jc = j < N ? j : 0;
          const LDS double* wj = wv + jc * 8;
          const double n3 = wj[3] + (wj[5] + a3);
          const double n4 = wj[4] + (wj[6] + a4);
          a3 = on ? n3 : a3;
          a4 = on ? n4 : a4;
        }
      } else {
        for (int j = N - 1; j >= k; --j) {
          const LDS double* wj = wv + j * 8;
          a3 = wj[3] + (wj[5] + a3);
          a4 = wj[4] + (wj[6] + a4);
        }
      }
      lam[k * 8 + 3] = a3;
      lam[k * 8 + 4] = a4;
    }
    STAMP1(PH_ADJ);
    sync();
  }

  // dL/du_k[c] = (B_k^T lam_{k+1})[c]
  __device__ __forceinline__ double grad_u(int i) const {
    const int k = i / 6, c = i - 6 * (i / 6);
    const LDS double* ln = lam + (k + 1) * 8;
    if constexpr (CAP::deep) {  // both forms from valid reads, then selected
      const LDS double* tg = trig + k * 8;
      const double ct = tg[0], stt = tg[1], cp = tg[2], sp = tg[3];
      const double g0 = (T * cp * ct) * ln[0] + (T * sp * ct) * ln[1] + (T * stt) * ln[2];
      const double gc = T * ln[2 + c];
      return c == 0 ? g0 : gc;
    } else if (c == 0) {
      const LDS double* tg = trig + k * 8;
      const double ct = tg[0], stt = tg[1], cp = tg[2], sp = tg[3];
      return (T * cp * ct) * ln[0] + (T * sp * ct) * ln[1] + (T * stt) * ln[2];
    }
    return T * ln[2 + c];
  }

  // ------------------------------------------------ slacks / barrier helpers
  __device__ __forceinline__ double sl_x(int i, const LDS double* u) const { return u[i] - xl[i]; }
  __device__ __forceinline__ double su_x(int i, const LDS double* u) const { return xu[i] - u[i]; }

  // phi from the wave sums of barrier_obj (the log and damping sums do not depend on mu)
  __device__ __forceinline__ double phi_of(double f, double logs, double damp) const {
    return f - mu * logs + P->o.kappa_d * mu * damp;
  }
  // barrier objective phi (oracle barrier_obj) at (u, s + a*ds) [sv == null -> s];
  // the sums are kept in rvars[32..33], so the accepted trial's sums serve the next
  // iteration's reference value (same slacks bit for bit: U <- Ut, s <- s + a ds)
  // per-lane partial sums: the control terms first, then the rows in rows() order
  // (the log sums as LogAcc products, one logarithm per lane and pass)
  __device__ __forceinline__ void barrier_ctrl(const GLB double* u, LogAcc& logs, double& damp) const {
    ctrls([&](int i, bool on) { barrier_ctrl1(i, on, u[i], logs, damp); });
  }
  // one control's barrier terms at the value ui (a register: the trial point's controls
  // are formed and consumed in the same pass, no store -> load round trip)
  __device__ __forceinline__ void barrier_ctrl1(int i, bool on, double ui, LogAcc& logs, double& damp) const {
    const double xli = xl[i], xui = xu[i];
    const bool lo = hasl(xli), hi = hasu(xui);
    logs.mul2(on && lo ? ui - xli : 1.0, on && hi ? xui - ui : 1.0);
    if (on) {
      if (lo && !hi) damp += ui - xli;
      if (hi && !lo) damp += xui - ui;
    }
  }
  __device__ __forceinline__ void barrier_row(int r, bool on, double sv, LogAcc& logs, double& damp) const {
    const double lo_ = dl[r], hi_ = du[r];
    const bool lo = hasl(lo_), hi = hasu(hi_);
    logs.mul2(on && lo ? sv - lo_ : 1.0, on && hi ? hi_ - sv : 1.0);
    if (on) {
      if (lo && !hi) damp += sv - lo_;
      if (hi && !lo) damp += hi_ - sv;
    }
  }
  __device__ __forceinline__ double barrier_fin(double f, const LogAcc& la, double damp) {
    const double logs = wsum(la.log());
    damp = wsum(damp);
    rvars[32] = logs; rvars[33] = damp;
    return phi_of(f, logs, damp);
  }
  __device__ __forceinline__ double barrier_obj(double f, const GLB double* u, const RV* sb, const RV* dsv,
                                double a) {
    STAMP0();
    LogAcc logs;
    double damp = 0.0;
    barrier_ctrl(u, logs, damp);
    rows([&](int r, bool on) { barrier_row(r, on, dsv ? sb[r] + a * dsv[r] : sb[r], logs, damp); });
    const double rr = barrier_fin(f, logs, damp);
    STAMP1G(PH_BARR);
    return rr;
  }

  // ------------------------------------------------ equality rows (lbg == ubg)
  // IPOPT's c(x) = g(x) - g_l = 0: the row keeps its slot, its bounds are
  // NaN (so every bound test sees no bound: no slack barrier, no bound multipliers, no
  // fraction to the boundary) and its slack s is pinned at the scaled target, so d - s = c
  // enters theta, the residuals and the filter unchanged.  The Newton step adds the
  // equality rows through the Schur complement of the augmented system.
  __device__ __forceinline__ static bool eqrow(double lo) { return lo != lo; }
  // compile-time false outside the equality class; inside it the wave-uniform meq > 0
  // test first, so a batch without equality rows skips the bound load and the select
  __device__ __forceinline__ bool eqlo(double lo) const { return CAP::eq && meq > 0 && eqrow(lo); }
  __device__ __forceinline__ bool eqr(int r) const { return CAP::eq && meq > 0 && eqrow(dl[r]); }
  // equality-row workspace (indices, factored Schur complement + pivot signs, dy_c of the
  // step / SOC), addressed off U through an opaque copy rather than held as four more
  // pointers live across the whole solve
  __device__ __forceinline__ GLB double* eqw(int off) const {
    GLB double* p = U;
    asm volatile("" : "+s"(p));
    return p + (off - CAP::L.U);
  }
  __device__ __forceinline__ GLB int* eqi_() const { return (GLB int*)eqw(CAP::L.eqi); }
  __device__ __forceinline__ GLB double* eqS_() const { return eqw(CAP::L.eqS); }
  __device__ __forceinline__ GLB double* eqy_() const { return eqw(CAP::L.eqy); }
  __device__ __forceinline__ GLB double* eqy2_() const { return eqw(CAP::L.eqy2); }
  __device__ __forceinline__ GLB double* weqy_() const { return eqw(CAP::L.weqy); }
  // J_r dX (scaled row Jacobian times the state step at the row's stage), as in row_step
  __device__ __forceinline__ double row_jd(int r, const LDS double* dXs) const {
    const int k = r / m, i = r - k * m;
    const LDS double* xk = X + k * 8;
    const LDS double* dxk = dXs + k * 8;
    if (i < nb) return dc[r] * dxk[boxidx(i)];
    const int o = i - nb;
    const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
    const double idd = rsq(ddx * ddx + ddy * ddy);
    return dc[r] * ((-(ddx * idd)) * dxk[0] + (-(ddy * idd)) * dxk[1]);
  }
  // the same row's scaled state gradient (8 entries of stage r / m)
  __device__ __forceinline__ void row_grad8(int r, double g8[8]) const {
    const int k = r / m, i = r - k * m;
#pragma unroll
    for (int c = 0; c < 8; ++c) g8[c] = 0.0;
    const double dcr = dc[r];
    if (i < nb) {
      const int bi = boxidx(i);
#pragma unroll
      for (int c = 0; c < 8; ++c) g8[c] = (c == bi) ? dcr : 0.0;
    } else {
      const LDS double* xk = X + k * 8;
      const int o = i - nb;
      const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
      const double idd = rsq(ddx * ddx + ddy * ddy);
      g8[0] = dcr * (-(ddx * idd));
      g8[1] = dcr * (-(ddy * idd));
    }
  }
  // solve with the stored Riccati factors, signed pivots (the factorization may be
  // indefinite when there are equality rows): ke < 0 -> the assembled linear terms (qs,
  // rv); ke >= 0 -> the unit problem q_ke = g8, every other term 0.  Writes kf.
  __device__ __forceinline__ void resolve_eq(const GLB double* rv, int ke, const double* g8) {
    double p8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p8[i] = ke < 0 ? qs[N * 10 + i] : (ke == N ? g8[i] : 0.0);
    for (int k = N - 1; k >= 0; --k) {
      double E03, E04, E13, E14, E23, b00, b10, b20;
      stage_AB(k, E03, E04, E13, E14, E23, b00, b10, b20);
      double Lm[21], idg[6], sg[6], rt[6], v[6];
#pragma unroll
      for (int t = 0; t < 21; ++t) Lm[t] = Rk[k * 21 + t];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double dg = Lm[c * (c + 1) / 2 + c];
#pragma unroll
        for (int t = 0; t < c; ++t) dg -= (sg[t] * Lm[c * (c + 1) / 2 + t]) * Lm[c * (c + 1) / 2 + t];
        sg[c] = dg < 0.0 ? -1.0 : 1.0;
        dg = fabs(dg);
        const double ig = rsq(dg);
        Lm[c * (c + 1) / 2 + c] = dg * ig;
        idg[c] = ig;
#pragma unroll
        for (int r = c + 1; r < 6; ++r) {
          double a = Lm[r * (r + 1) / 2 + c];
#pragma unroll
          for (int t = 0; t < c; ++t) a -= (sg[t] * Lm[r * (r + 1) / 2 + t]) * Lm[c * (c + 1) / 2 + t];
          Lm[r * (r + 1) / 2 + c] = (a * ig) * sg[c];
        }
      }
      const bool ur = ke < 0;
      rt[0] = (ur ? rv[k * 6 + 0] : 0.0) + ((b00 * p8[0] + b10 * p8[1]) + b20 * p8[2]);
#pragma unroll
      for (int r = 1; r < 6; ++r) rt[r] = (ur ? rv[k * 6 + r] : 0.0) + T * p8[2 + r];
      if (nfix > 0) {
        const int fm = fixm[k];
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if ((fm >> r) & 1) rt[r] = 0.0;
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        double a = rt[r];
#pragma unroll
        for (int t = 0; t < r; ++t) a -= Lm[r * (r + 1) / 2 + t] * v[t];
        v[r] = a * idg[r];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) v[r] *= sg[r];
#pragma unroll
      for (int r = 5; r >= 0; --r) {
        double a = v[r];
#pragma unroll
        for (int t = r + 1; t < 6; ++t) a -= Lm[t * (t + 1) / 2 + r] * v[t];
        v[r] = a * idg[r];
      }
      if (lanef() == 0) {
#pragma unroll
        for (int r = 0; r < 6; ++r) kf[k * 6 + r] = -v[r];
      }
      double pn[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        double atp = p8[i];
        if (i == 3) atp = atp + ((E03 * p8[0] + E13 * p8[1]) + E23 * p8[2]);
        else if (i == 4) atp = atp + (E04 * p8[0] + E14 * p8[1]);
        double kr = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) kr += K[k * 48 + r * 8 + i] * rt[r];
        const double qk = ur ? qs[k * 10 + i] : (k == ke ? g8[i] : 0.0);
        pn[i] = (qk + atp) + kr;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) p8[i] = pn[i];
    }
    sync();
  }
  // Schur complement S = J_c H^-1 J_c^T of the equality rows from meq unit solves, and its
  // signed Cholesky factor with delta_c = 0, then IPOPT's jacobian_regularization_value *
  // mu^0.25 if S is singular.  Inertia test (Haynsworth): the augmented system
  // [H J_c^T; J_c -delta_c I] has n positive and meq negative eigenvalues iff S + delta_c I
  // has exactly as many negative pivots as the Riccati sweep had (nneg).
  // Storage (eqS, workspace): S and the factor column-major, MQ = NMPC_MEQ rows per column;
  // lane l owns rows l + 64 q (slots q < EQR) of every column, so every access is a lane's
  // own entry and the pivot column reaches the other lanes by readlane.
  // (allow_dc false: the least-squares multipliers, which IPOPT computes without
  // regularisation -- a singular S there means y = 0)
  static constexpr int EQR = NMPC_MEQ / WAVE;
  // entry `row` (wave-uniform) of a per-lane slot vector v[EQR]
  __device__ __forceinline__ static double eq_bcast(const double* v, int row) {
    double r = 0.0;
#pragma unroll
    for (int q = 0; q < EQR; ++q)
      if ((row >> 6) == q) r = readlane_d(v[q], row & (WAVE - 1));
    return r;
  }
  __device__ __forceinline__ bool eq_schur(double mu_, bool allow_dc = true) {
    constexpr int MQ = NMPC_MEQ;
    const int ln = lanef();
    GLB double* Sm = eqS_();
    GLB double* Fm = Sm + MQ * MQ;
    GLB double* sgm = Fm + MQ * MQ;
    for (int e = 0; e < meq; ++e) {
      const int re = eqi_()[e];
      double g8[8];
      row_grad8(re, g8);
      resolve_eq(ru, re / m, g8);
      forward(dUr, Xt);  // -H^-1 J_e^T (the fp64 classes' refinement buffer; Xt is free here)
#pragma unroll
      for (int q = 0; q < EQR; ++q) {
        const int l = ln + q * WAVE;
        const double se = l < meq ? -row_jd(eqi_()[l < meq ? l : 0], Xt) : 0.0;
        if (l < meq) Sm[e * MQ + l] = se;  // S[l][e]
      }
      sync();
    }
    double dmax = 0.0;
#pragma unroll
    for (int q = 0; q < EQR; ++q) {
      const int l = ln + q * WAVE;
      if (l < meq) dmax = fmax(dmax, fabs(Sm[l * MQ + l]));
    }
    const double scale = wmax(dmax);
    for (int att = 0; att < (allow_dc ? 2 : 1); ++att) {
      const double dcv = att == 0 ? 0.0 : 1e-8 * pow(mu_, 0.25);
      for (int c = 0; c < meq; ++c) {
#pragma unroll
        for (int q = 0; q < EQR; ++q) {
          const int l = ln + q * WAVE;
          if (l < meq) Fm[c * MQ + l] = Sm[c * MQ + l] + ((c == l) ? dcv : 0.0);
        }
      }
      sync();
      bool sing = false;
      int negS = 0;
      double sgl[EQR];  // slot q of lane l: the sign of pivot l + 64 q
#pragma unroll
      for (int q = 0; q < EQR; ++q) sgl[q] = 1.0;
      for (int c = 0; c < meq; ++c) {
        double col[EQR], lc[EQR];
#pragma unroll
        for (int q = 0; q < EQR; ++q) {
          const int l = ln + q * WAVE;
          col[q] = l < meq ? Fm[c * MQ + l] : 0.0;
        }
        const double d = eq_bcast(col, c);
        if (!(fabs(d) > 1e-14 * scale)) sing = true;
        const double sgc = d < 0.0 ? -1.0 : 1.0;
        negS += d < 0.0 ? 1 : 0;
        const double ig = rsq(fabs(d));
        const double Lcc = fabs(d) * ig;
#pragma unroll
        for (int q = 0; q < EQR; ++q) {
          const int l = ln + q * WAVE;
          if (l == c) sgl[q] = sgc;
          lc[q] = (l == c) ? Lcc : ((l > c) ? (col[q] * ig) * sgc : col[q]);
          if (l < meq) Fm[c * MQ + l] = lc[q];
        }
        // right-looking update of the lane's own trailing entries (rows > c), eight
        // columns per batch (their loads issued together)
        for (int c2 = c + 1; c2 < meq; c2 += 8) {
#pragma unroll
          for (int q = 0; q < EQR; ++q) {
            const int l = ln + q * WAVE;
            if ((q + 1) * WAVE <= c + 1) continue;  // wave-uniform: no row of this slot is > c
            const double lcs = lc[q] * sgc;
            double v[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] = (l < meq && c2 + t < meq) ? Fm[(c2 + t) * MQ + l] : 0.0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              if (c2 + t < meq) {
                const double Lc2c = eq_bcast(lc, c2 + t);
                if (l < meq && l > c) Fm[(c2 + t) * MQ + l] = v[t] - lcs * Lc2c;
              }
            }
          }
        }
        sync();
      }
      if (sing) continue;
      if (negS != nneg) return false;
#pragma unroll
      for (int q = 0; q < EQR; ++q) {
        const int l = ln + q * WAVE;
        if (l < meq) sgm[l] = sgl[q];
      }
      sync();
      return true;
    }
    return false;
  }
  // dy = (S + delta_c I)^-1 rhs with the stored factor (rhs[q]: lane l holds entry l + 64 q);
  // the solution comes back in the same slots
  __device__ __forceinline__ void eq_solve(const double* rhs, double* out) const {
    constexpr int MQ = NMPC_MEQ;
    const int ln = lanef();
    const GLB double* Fm = eqS_() + MQ * MQ;
    const GLB double* sgm = Fm + MQ * MQ;
    double sgl[EQR], part[EQR], zl[EQR], yl[EQR];
#pragma unroll
    for (int q = 0; q < EQR; ++q) {
      const int l = ln + q * WAVE;
      sgl[q] = l < meq ? sgm[l] : 1.0;
      part[q] = l < meq ? rhs[q] : 0.0;
      zl[q] = 0.0;
      yl[q] = 0.0;
    }
    // L z = rhs (column-oriented: each row keeps its partial sum; row c ends with z_c)
    for (int c = 0; c < meq; ++c) {
      double col[EQR];
#pragma unroll
      for (int q = 0; q < EQR; ++q) {
        const int l = ln + q * WAVE;
        col[q] = l < meq ? Fm[c * MQ + l] : 0.0;
      }
      const double Lcc = eq_bcast(col, c);
      const double zc = eq_bcast(part, c) / Lcc;
#pragma unroll
      for (int q = 0; q < EQR; ++q) {
        const int l = ln + q * WAVE;
        if (l == c) zl[q] = zc;
        if (l > c) part[q] -= col[q] * zc;
      }
    }
    // L^T dy = Sigma z, back to front (every lane forms each entry; row c keeps y_c)
    for (int c = meq - 1; c >= 0; --c) {
      double col[EQR];
#pragma unroll
      for (int q = 0; q < EQR; ++q) {
        const int l = ln + q * WAVE;
        col[q] = l < meq ? Fm[c * MQ + l] : 0.0;
      }
      double a = eq_bcast(sgl, c) * eq_bcast(zl, c);
      for (int j = c + 1; j < meq; ++j) a -= eq_bcast(col, j) * eq_bcast(yl, j);
      const double yc = a / eq_bcast(col, c);
#pragma unroll
      for (int q = 0; q < EQR; ++q)
        if (ln + q * WAVE == c) yl[q] = yc;
    }
#pragma unroll
    for (int q = 0; q < EQR; ++q) out[q] = yl[q];
  }
  // the step with the equality rows: base solve (dUo, dXo) with the assembled terms, then
  // dy = (S + delta_c)^-1 (c + J_c dX0), q += J_c^T dy, solve again (Newton / SOC step);
  // for the least-squares multipliers y_c = S^-1 (-J_c w0), q -= J_c^T y_c.  dy goes to
  // dyo[row].
  // MODE 0: c = d - s (Newton step); 1: c = dms (second-order correction); 2: the
  // least-squares multipliers
  template <int MODE>
  __device__ __forceinline__ void eq_step(const GLB double* rv, GLB double* dUo, LDS double* dXo, GLB double* dyo) {
    const int ln = lanef();
    const double g0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    resolve_eq(rv, -1, g0);
    forward(dUo, dXo);
    double rhs[EQR], dy[EQR];
#pragma unroll
    for (int q = 0; q < EQR; ++q) {
      const int l = ln + q * WAVE;
      const int re = eqi_()[l < meq ? l : 0];
      const double jd = row_jd(re, dXo);
      if constexpr (MODE == 0) rhs[q] = (d[re] - s[re]) + jd;
      else if constexpr (MODE == 1) rhs[q] = dms[re] + jd;
      else rhs[q] = -jd;
    }
    eq_solve(rhs, dy);
#pragma unroll
    for (int q = 0; q < EQR; ++q) {
      const int l = ln + q * WAVE;
      if (l < meq) dyo[eqi_()[l]] = dy[q];
    }
    // q_k += (+-) dy_e g8_e at each row's stage (serial over the rows: rows may share a stage)
    for (int e = 0; e < meq; ++e) {
      const int r = eqi_()[e];
      double g8[8];
      row_grad8(r, g8);
      const double de = eq_bcast(dy, e) * (MODE == 2 ? -1.0 : 1.0);
      const int k = r / m;
      if (ln < 8) {
        double gv = 0.0;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (c == ln) gv = g8[c];
        qs[k * 10 + ln] += de * gv;
      }
      sync();
    }
    resolve_eq(rv, -1, g0);
    forward(dUo, dXo);
  }

  // -------------------------------------------- Riccati: stage assembly
  // Stage-parallel (lanef() = stage k) assembly of the LQ subproblem:
  //   Qs[k] = Q_k (8x8 symmetric, packed upper, 36), qs[k] = {q_k (8), S_k[0][3], S_k[0][4]}.
  //  NEWTON: Q = hfac*Hl + Gt^T D Gt + sum_obs y dc Hg + dyn(lam_{k+1}) ; q = gfac*gl + Gt^T (y + D rd + rs)
  //  SOC:    q only, with rd := dms (Q, S unchanged)
  //  LS:     Q = Gt^T Gt ; q = gfac*gl - Gt^T (vu - vl)   (least-squares y init, gfac = -df)
  __device__ __forceinline__ static int pk8(int i, int j) { return i * (15 - i) / 2 + j; }  // i <= j
  __device__ __forceinline__ void assemble(int mode, double hfac, double gfac, bool dyn) {
    STAMP0();
    const double kd = P->o.kappa_d;
    const bool soc = (mode == SUM_SOC || mode == SUM_RESTO_SOC);  // right-hand side only
    // (a) row-parallel (64 rows per trip instead of m rows per stage lane): each row's
    //     weight dc^2 A (Q part) and right-hand side dc Bw, into scratch row vectors that
    //     are dead in every caller at this point (ds2: SOC step, written after the
    //     solve; dt: trial constraints, rewritten by the next trial)
    auto Wr = ds2;
    auto Br = dt;
    const bool curv = !(mode == SUM_LS || mode == SUM_LS_RESTO);  // y-weighted row curvature
    auto rowsA = [&](auto&& body) {  // the restoration modes read its global row vectors: rows_r
      if (mode == SUM_RESTO || mode == SUM_RESTO_SOC || mode == SUM_LS_RESTO) rows_r(body);
      else rows(body);
    };
    rowsA([&](int r, bool on) {
      const double dcr = dc[r];
      double A, Bw;
      if (mode == SUM_LS) {
        A = 1.0;
        Bw = -(vu[r] - vl[r]);
      } else if (mode == SUM_LS_RESTO) {
        // (I + J^T J / 3) w = bx + J^T (bs + bp - bn) / 3 : the restoration NLP's
        // least-squares multipliers with p, n eliminated
        A = 1.0 / 3.0;
        Bw = -((vu[r] - vl[r]) + (rho - zpR[r]) - (rho - znR[r])) / 3.0;
      } else if (mode == SUM_RESTO || mode == SUM_RESTO_SOC) {
        double D, rs, Sp, Sn, rp, rn, Dt, Dr;
        row_resto(r, mode == SUM_RESTO_SOC, D, rs, Sp, Sn, rp, rn, Dt, Dr);
        A = Dt;
        Bw = y[r] + Dr;
      } else {
        const double sr = s[r], vlr = vl[r], vur = vu[r], yr = y[r];
        const double rd = (mode == SUM_SOC) ? dms[r] : d[r] - sr;
        const double lo_ = dl[r], hi_ = du[r];
        const bool lo = hasl(lo_), hi = hasu(hi_);
        const double iSl = lo ? rcp(sr - lo_) : 0.0, iSu = hi ? rcp(hi_ - sr) : 0.0;
        const double D = vlr * iSl + vur * iSu + delta;
        const double rs = -yr - mu * iSl + mu * iSu +
                          kd * mu * ((lo && !hi ? 1.0 : 0.0) - (hi && !lo ? 1.0 : 0.0));
        A = D;
        Bw = yr + D * rd + rs;
      }
      if (eqr(r)) {  // equality rows: no slack elimination (the Schur step adds them)
        if (mode == SUM_LS) { A = 0.0; Bw = 0.0; }
        else if (mode == SUM_LS_RESTO) { A = 0.5; Bw = -((rho - zpR[r]) - (rho - znR[r])) / 2.0; }
        else if (mode == SUM_NEWTON || mode == SUM_SOC) { A = 0.0; Bw = y[r]; }
      }
      if (on) {
        if (!soc) Wr[r] = dcr * dcr * A;
        Br[r] = dcr * Bw;
      }
    });
    sync();
    // (b) stage-parallel (lane = stage k): fold the stage's rows into Q_k, q_k
    const int k = lanef();
    if (k <= N) {
      const LDS double* xk = X + k * 8;
      double Qxy0 = 0, Qxy1 = 0, Qxy2 = 0, qx = 0, qy = 0;
      double Qb[5] = {0, 0, 0, 0, 0}, qb[5] = {0, 0, 0, 0, 0};
      if constexpr (CAP::deep) {
        // the deep (LDS) class: unrolled over the class's row maximum with clamped rows, so
        // every row's loads and its obstacle's reciprocal square root issue without waiting
        // for the previous row (a rolled loop with the branch on the row kind left each
        // row's rsq chain exposed); the sums take the active obstacle rows in order, as
        // below -- the same operations in the same order
#pragma unroll
        for (int i = 0; i < CAP::mmax; ++i) {
          const bool act = i < m;
          const int ic = act ? i : m - 1;
          const int r = k * m + ic;
          const double w = soc ? 0.0 : Wr[r], bw = Br[r];
          const bool box = ic < nb;
          if (i < 5) {
            if (act && box) {
              Qb[i] = w;
              qb[i] = bw;
            }
          }
          const double C = curv ? y[r] * dc[r] : 0.0;
          const int o = box ? 0 : ic - nb;
          const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
          const double idd = rsq(ddx * ddx + ddy * ddy);
          const double gx = -(ddx * idd), gy = -(ddy * idd);
          const double id3 = idd * idd * idd;
          if (act && !box) {
            Qxy0 += w * gx * gx + C * (-ddy * ddy * id3);
            Qxy1 += w * gx * gy + C * (ddx * ddy * id3);
            Qxy2 += w * gy * gy + C * (-ddx * ddx * id3);
            qx += bw * gx;
            qy += bw * gy;
          }
        }
      } else
      for (int i = 0; i < m; ++i) {
        const int r = k * m + i;
        const double w = soc ? 0.0 : Wr[r], bw = Br[r];
        if (i < nb) {
          Qb[i] = w;
          qb[i] = bw;
        } else {
          const double C = curv ? y[r] * dc[r] : 0.0;
          const int o = i - nb;
          const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
          const double idd = rsq(ddx * ddx + ddy * ddy);
          const double gx = -(ddx * idd), gy = -(ddy * idd);
          const double id3 = idd * idd * idd;
          Qxy0 += w * gx * gx + C * (-ddy * ddy * id3);
          Qxy1 += w * gx * gy + C * (ddx * ddy * id3);
          Qxy2 += w * gy * gy + C * (-ddx * ddx * id3);
          qx += bw * gx;
          qy += bw * gy;
        }
      }
      LDS double* qo = qs + k * 10;
      qo[0] = gfac * gl[k * 8 + 0] + qx;
      qo[1] = gfac * gl[k * 8 + 1] + qy;
      qo[2] = gfac * gl[k * 8 + 2] + qb[0];
      qo[3] = gfac * gl[k * 8 + 3] + qb[1];
      qo[4] = gfac * gl[k * 8 + 4];
      qo[5] = gfac * gl[k * 8 + 5] + qb[2];
      qo[6] = gfac * gl[k * 8 + 6] + qb[3];
      qo[7] = gfac * gl[k * 8 + 7] + qb[4];
      if (mode != SUM_SOC && mode != SUM_RESTO_SOC) {
        double Q[36];
#pragma unroll
        for (int t = 0; t < 36; ++t) Q[t] = 0.0;
        if (hfac != 0.0) {
          const int sv[6] = {0, 1, 2, 5, 6, 7};
#pragma unroll
          for (int a = 0; a < 6; ++a) {
#pragma unroll
            for (int bq = a; bq < 6; ++bq) Q[pk8(sv[a], sv[bq])] += hfac * Hl[k * 21 + hp(a, bq)];
          }
        }
        Q[pk8(0, 0)] += Qxy0; Q[pk8(0, 1)] += Qxy1; Q[pk8(1, 1)] += Qxy2;
        Q[pk8(2, 2)] += Qb[0]; Q[pk8(3, 3)] += Qb[1]; Q[pk8(5, 5)] += Qb[2];
        Q[pk8(6, 6)] += Qb[3]; Q[pk8(7, 7)] += Qb[4];
        double s03 = 0.0, s04 = 0.0;
        if (dyn && k < N) {
          const LDS double* tg = trig + k * 8;
          const double ct = tg[0], stt = tg[1], cp = tg[2], sp = tg[3], v = tg[4];
          const LDS double* ln = lam + (k + 1) * 8;
          const double l0 = ln[0], l1 = ln[1], l2 = ln[2];
          Q[pk8(3, 3)] += T * (-l0 * v * cp * ct - l1 * v * sp * ct - l2 * v * stt);
          Q[pk8(4, 4)] += T * (-l0 * v * cp * ct - l1 * v * sp * ct);
          Q[pk8(3, 4)] += T * (l0 * v * sp * stt - l1 * v * cp * stt);
          s03 = T * (-l0 * cp * stt - l1 * sp * stt + l2 * ct);
          s04 = T * (-l0 * sp * ct + l1 * cp * ct);
        }
#pragma unroll
        for (int t = 0; t < 36; ++t) Qs[k * 36 + t] = Q[t];
        qo[8] = s03;
        qo[9] = s04;
      }
    }
    sync();
    STAMP1(PH_SUMM);
  }

  // ----------------------------------------- Riccati factorisation + solve
  // Backward sweep over stages, lane (i,j) owning entry (i,j) of the 8x8
  // cost-to-go matrix, two LDS exchanges per stage:
  //   (1) A^T P A (register), S~ = S + B^T P A and R~ = R + B^T P B (21 lanes)
  //       straight from P (A = I + E, B = [b0 | T e_3..7]);
  //   (2) every lane: Cholesky R~ = L L^T (inertia: all pivots > 0) and Y = L^-1 S~
  //       for its columns i, j: P_k = Q_k + A^T P A - Y_i^T Y_j (= ... + S~^T K);
  //       lanes 0..7: column j of K = -L^-T Y_j, p_k = q_k + A^T p + K^T r~;
  //       lane 8: k = -R~^{-1} r~.
  // Stores K_k, k_k and R~_k (for the gradient-only re-solve).
  // SG: signed pivots (R~_k = L Sigma L^T, Sigma = diag(+-1)) for problems with equality
  // rows, whose inertia test counts the negative ones (nneg); otherwise every pivot must be
  // positive (IPOPT's inertia test for the condensed system), as before
  template <bool SG = false>
  __device__ __forceinline__ bool riccati(const GLB double* Rd, const GLB double* rv) {
#ifdef NMPC_STAMPS
    if (lanef() == 0) stamps[PH_RB] += 1.0;  // count factorisations
#endif
    STAMP0();
    const bool r = riccati_<SG>(Rd, rv);
    STAMP1(PH_RIC);
    return r;
  }
  // arithmetic in CAP::RT (the LDS exchange arrays hold RT values)
  template <bool SG>
  __device__ __forceinline__ bool riccati_(const GLB double* Rd, const GLB double* rv) {
    using R = typename CAP::RT;
    int negs = 0;
    // one opaque lane index for the whole sweep (every lanef() call is a fresh register copy)
    const int ln = lanef();
    const int i = ln >> 3, j = ln & 7;
    const int ij = (i <= j) ? pk8(i, j) : pk8(j, i);
    LDS R* Pc = (LDS R*)Pa;
    LDS R* Pn = (LDS R*)Pb;
    LDS R* pc = (LDS R*)pva;
    LDS R* pn = (LDS R*)pvb;
    LDS R* Stc = (LDS R*)St;
    LDS R* Rcc = (LDS R*)Rc;
    LDS R* rts = (LDS R*)Rv;  // r~ = r_k + B_k^T p_{k+1} of the current stage (lanes 0..5 form it)
    // wave-uniform scalars of the loop held in VGPRs: as SGPR pairs they are spilled to
    // VGPR lanes and restored (v_readlane pair + s_nop) at every use inside the sweep
    double Tv = T;
    R dlt = (R)delta;
    asm volatile("" : "+v"(Tv), "+v"(dlt));
    const R Tr = (R)Tv;
    Pc[ln] = (R)Qs[N * 36 + ij];
    if (ln < 8) pc[ln] = (R)qs[N * 10 + ln];
    // lanes 48..63 -> R~ entries t = 0..15, lanes 0..4 -> t = 16..20 (packed lower); the
    // other lanes duplicate entry 0 (same formula, same value), so every lane stores R~
    // without a branch
    const int tR0 = ln >= 48 ? ln - 48 : (ln < 5 ? 16 + ln : -1);
    const int tR = tR0 >= 0 ? tR0 : 0;
    int rR = 0;
    while ((rR + 1) * (rR + 2) / 2 <= tR) ++rR;
    const int cR = tR - rR * (rR + 1) / 2;
    const int rowS = (i >= 1 && i < 6) ? 2 + i : 3;
    // stage operands in global memory (Q_k entry, diag R_k entry, r_k) do not depend on
    // the recursion: fetch stage k-1's while stage k is formed, so the sweep never
    // waits on a global load.  Lanes 0..5 hold r_k and publish it through LDS.  The
    // fetches and the R~ stores are unconditional (clamped / duplicated addresses: the
    // lanes that carry no R~ entry recompute entry 0).  The K stores stay with lanes
    // 0..7: letting the lanes with the same column store duplicates changed the results
    // at the rounding level (measured against the previous kernel).
    const bool diagR = rR == cR;
    const int lr = ln < 6 ? ln : 5;
    double qvn = Qs[(N - 1) * 36 + ij];
    double rdn = Rd[(N - 1) * 6 + rR];
    double rvn = rv[(N - 1) * 6 + lr];
    // P_k is symmetric: lane (i,j) with i <= j forms entry (i,j) and stores it to both
    // halves; lane 8 = (1,0) is then free to carry r~ through the triangular solves
    const bool upper = i <= j;
    const int ji = j * 8 + i;
    // Stage-invariant lane roles as 0/1 multipliers (exact: every product with a 0 is an
    // exact zero added to the one non-zero term), so the stage body has no divergent code:
    //   A = I + E: column j of E is E03/E13/E23 (j = 3) or E04/E14 (j = 4)
    const R mj3 = (j == 3) ? (R)1 : (R)0, mj4 = (j == 4) ? (R)1 : (R)0;
    const R mi3 = (i == 3) ? (R)1 : (R)0, mi4 = (i == 4) ? (R)1 : (R)0;
    //   S~ row 0 adds s03 (j = 3) / s04 (j = 4)
    const R ms3 = (i == 0 && j == 3) ? (R)1 : (R)0, ms4 = (i == 0 && j == 4) ? (R)1 : (R)0;
    const bool absent = diagR && rR >= nuE;  // absent control (model embedding): unit pivot
    // Per-lane store targets fixed for the sweep (no address arithmetic, no divergent
    // branch around the stores inside it): lanes without an S~ / R~ / r~ entry store to
    // slots of the trial rows `dt`, which are dead during a factorisation (rewritten by the
    // next trial before any read), in the classes that keep dt in LDS; K column ln (lanes
    // 0..7) and R~ entry tR are stored through per-lane base pointers
    constexpr bool kDummy = CAP::lds_rows && !CAP::refine;
    // the dead-slot stores reach dt[191] (dmy + 128 + lane): dt must hold 192 doubles
    static_assert(!kDummy || al2(CAP::mmax * (CAP::nmax + 1)) >= 192, "dt too small for the branch-free Riccati stores");
    LDS R* dmy = kDummy ? (LDS R*)dt : Stc;
    LDS R* const st_dst = ln < 48 ? Stc + ln : dmy + ln;
    LDS R* const rc_dst = tR0 >= 0 ? Rcc + tR : dmy + 64 + ln;
    LDS R* const rt_dst = ln < 6 ? rts + ln : dmy + 128 + ln;
    GLB double* const Kl = K + (ln < 8 ? ln : 0);
    GLB double* const Rkl = Rk + tR;
    // lane 8 carries r~ through the triangular solves: its right-hand-side column is rts
    LDS R* const bcol = ln == 8 ? rts : Stc + j;
    const int bstr = ln == 8 ? 1 : 8;
    // per-lane bases of the prefetched stage operands
    const GLB double* const Qsl = Qs + ij;
    const GLB double* const Rdl = Rd + rR;
    const GLB double* const rvl = rv + lr;
    sync();
    bool ok = true;
    // one stage of the backward sweep (false: a pivot is not positive)
    auto stage = [&](int k, double qvd, double rdd, double rvd, const StageAB& ab, StageAB& abn) -> bool {
      const R qv = (R)qvd, rdk = (R)rdd, rvk = (R)rvd;
      // the deep (LDS) class forms the next stage's A / B here, off the critical path; the
      // register-limited global-row classes form each stage's at the stage (they spill)
      const StageAB abk = CAP::deep ? ab : stage_ab(k, Tv);
      if constexpr (CAP::deep) abn = stage_ab(k > 0 ? k - 1 : 0, Tv);
      const R E03 = (R)abk.E03, E04 = (R)abk.E04, E13 = (R)abk.E13, E14 = (R)abk.E14, E23 = (R)abk.E23;
      const R b00 = (R)abk.b00, b10 = (R)abk.b10, b20 = (R)abk.b20;
      const R zr = (R)0;
      // fixed controls (make_parameter) leave the stage problem: unit pivot, no coupling;
      // the mask is wave-uniform, so its handling is a scalar branch skipped when 0
      const int fm = __builtin_amdgcn_readfirstlane(nfix > 0 ? fixm[k] : 0);
      const R aj0 = mj3 * E03 + mj4 * E04, aj1 = mj3 * E13 + mj4 * E14, aj2 = mj3 * E23;
      const R ai0 = mi3 * E03 + mi4 * E04, ai1 = mi3 * E13 + mi4 * E14, ai2 = mi3 * E23;
      R APA;
      // ---- (1)
      { STAMP0();
        const R P00 = Pc[0], P01 = Pc[1], P02 = Pc[2], P11 = Pc[9], P12 = Pc[10], P22 = Pc[18];
        const R P0j = Pc[j], P1j = Pc[8 + j], P2j = Pc[16 + j];
        const R Pi0 = Pc[i * 8], Pi1 = Pc[i * 8 + 1], Pi2 = Pc[i * 8 + 2], Pij = Pc[ln];
        const R PA0j = P0j + ((P00 * aj0 + P01 * aj1) + P02 * aj2);
        const R PA1j = P1j + ((P01 * aj0 + P11 * aj1) + P12 * aj2);
        const R PA2j = P2j + ((P02 * aj0 + P12 * aj1) + P22 * aj2);
        const R PAij = Pij + ((Pi0 * aj0 + Pi1 * aj1) + Pi2 * aj2);
        APA = PAij + ((ai0 * PA0j + ai1 * PA1j) + ai2 * PA2j);
        const R Prj = Pc[rowS * 8 + j], Pr0 = Pc[rowS * 8], Pr1 = Pc[rowS * 8 + 1], Pr2 = Pc[rowS * 8 + 2];
        const R PArj = Prj + ((Pr0 * aj0 + Pr1 * aj1) + Pr2 * aj2);
        R stv = (i == 0) ? ((b00 * PA0j + b10 * PA1j) + b20 * PA2j) : Tr * PArj;
        stv += ms3 * (R)qs[k * 10 + 8] + ms4 * (R)qs[k * 10 + 9];
        // R~ entry (rR, cR) of B^T P B, B = [b0 | T e_3..7] (lanes that carry no entry
        // compute entry 0 again: same value, so their store below needs no branch)
        R v;
        if constexpr (CAP::deep) {  // the three entry kinds formed by every lane (their LDS reads valid for every lane,
           // issued together) and selected by the lane's kind: no lane-dependent branch
          const LDS R* Pr = Pc + (2 + rR) * 8;
          const R pr0 = Pr[0], pr1 = Pr[1], pr2 = Pr[2], pe = Pc[(2 + rR) * 8 + 2 + cR];
          const R va = b00 * ((P00 * b00 + P01 * b10) + P02 * b20) + b10 * ((P01 * b00 + P11 * b10) + P12 * b20) +
                       b20 * ((P02 * b00 + P12 * b10) + P22 * b20);
          const R vb = Tr * ((pr0 * b00 + pr1 * b10) + pr2 * b20);
          const R vc = Tr * (Tr * pe);
          v = rR == 0 ? va : (cR == 0 ? vb : vc);
        } else if (rR == 0) {  // b0^T P[0:3,0:3] b0
          v = b00 * ((P00 * b00 + P01 * b10) + P02 * b20) + b10 * ((P01 * b00 + P11 * b10) + P12 * b20) +
              b20 * ((P02 * b00 + P12 * b10) + P22 * b20);
        } else if (cR == 0) {
          const LDS R* Pr = Pc + (2 + rR) * 8;
          v = Tr * ((Pr[0] * b00 + Pr[1] * b10) + Pr[2] * b20);
        } else {
          v = Tr * (Tr * Pc[(2 + rR) * 8 + 2 + cR]);
        }
        if (diagR) v = absent ? (R)1 : v + (rdk + dlt);
        if (fm != 0) {
          if ((fm >> i) & 1) stv = zr;
          if (((fm >> rR) | (fm >> cR)) & 1) v = (rR == cR) ? (R)1 : zr;
        }
        // r~ entry lr = r_k[lr] + (B_k^T p_{k+1})[lr] (lanes 0..5; both forms, selected).
        // The contractions are spelled out: selecting between the two forms lets the
        // compiler hoist the add of r_k out of the select and leave Tr * p unfused, a
        // different rounding from the single fused form every other solve of r~ uses
        R rtv;
        {
          const R rt0 = rvk + fma(b20, pc[2], fma(b00, pc[0], b10 * pc[1]));
          const R rtc = fma(Tr, pc[2 + lr], rvk);
          rtv = lr == 0 ? rt0 : rtc;
          if (fm != 0) {
            if ((fm >> lr) & 1) rtv = zr;
          }
        }
        if constexpr (kDummy) {
          *st_dst = stv;
          *rc_dst = v;
          *rt_dst = rtv;
        } else {
          if (ln < 48) *st_dst = stv;
          if (tR0 >= 0) *rc_dst = v;
          if (ln < 6) *rt_dst = rtv;
        }
        Rkl[k * 21] = (double)v;
        sync();
        STAMP1(PH_RA); }
      // ---- (2)
      R rt[6];
      { STAMP0();
        R Lm[21], idg[6], sg[6];
#pragma unroll
        for (int t = 0; t < 21; ++t) Lm[t] = Rcc[t];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          R dg = Lm[c * (c + 1) / 2 + c];
          if constexpr (SG) {
#pragma unroll
            for (int t = 0; t < c; ++t) dg -= (sg[t] * Lm[c * (c + 1) / 2 + t]) * Lm[c * (c + 1) / 2 + t];
            if (!(dg != zr)) ok = false;  // a zero pivot: singular
            sg[c] = dg < zr ? (R)-1 : (R)1;
            negs += dg < zr ? 1 : 0;
            dg = fabs(dg);
          } else {
#pragma unroll
            for (int t = 0; t < c; ++t) dg -= Lm[c * (c + 1) / 2 + t] * Lm[c * (c + 1) / 2 + t];
            if (!(dg > zr)) ok = false;
          }
          const R ig = rsq(dg);
          Lm[c * (c + 1) / 2 + c] = dg * ig;
          idg[c] = ig;
#pragma unroll
          for (int r = c + 1; r < 6; ++r) {
            R v = Lm[r * (r + 1) / 2 + c];
            if constexpr (SG) {
#pragma unroll
              for (int t = 0; t < c; ++t) v -= (sg[t] * Lm[r * (r + 1) / 2 + t]) * Lm[c * (c + 1) / 2 + t];
              Lm[r * (r + 1) / 2 + c] = (v * ig) * sg[c];
            } else {
#pragma unroll
              for (int t = 0; t < c; ++t) v -= Lm[r * (r + 1) / 2 + t] * Lm[c * (c + 1) / 2 + t];
              Lm[r * (r + 1) / 2 + c] = v * ig;
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) rt[r] = rts[r];
        R ya[6], yb[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          R a = Stc[r * 8 + i];
          R bb = bcol[r * bstr];

#pragma unroll
          for (int t = 0; t < r; ++t) {
            a -= Lm[r * (r + 1) / 2 + t] * ya[t];
            bb -= Lm[r * (r + 1) / 2 + t] * yb[t];
          }
          ya[r] = a * idg[r];
          yb[r] = bb * idg[r];
        }
        if constexpr (SG) {  // S~^T R~^-1 S~ = Y^T Sigma Y, K = -L^-T Sigma Y
#pragma unroll
          for (int r = 0; r < 6; ++r) ya[r] *= sg[r];
        }
        if (upper) {
          R sy = zr;
#pragma unroll
          for (int r = 0; r < 6; ++r) sy += ya[r] * yb[r];
          const R pv = (qv + APA) - sy;
          Pn[ln] = pv;
          Pn[ji] = pv;
        }
        if constexpr (SG) {
#pragma unroll
          for (int r = 0; r < 6; ++r) yb[r] *= sg[r];
        }
        // back substitution: lanes 0..7 column ln of K, lane 8 k = -R~^-1 r~ (every lane
        // computes it: branch-free, so it overlaps with the next stage's LDS reads), carried
        // negated (mb = -yb: negation commutes with every rounding, so the same values), so
        // K and k_k are stored without a negation
        R mb[6];
#pragma unroll
        for (int r = 5; r >= 0; --r) {
          R a = -yb[r];
#pragma unroll
          for (int t = r + 1; t < 6; ++t) a -= Lm[t * (t + 1) / 2 + r] * mb[t];
          mb[r] = a * idg[r];
        }
        R atp = pc[j];
        atp = atp + mj3 * ((E03 * pc[0] + E13 * pc[1]) + E23 * pc[2]) + mj4 * (E04 * pc[0] + E14 * pc[1]);
        R kr = zr;
#pragma unroll
        for (int r = 0; r < 6; ++r) kr += mb[r] * rt[r];
        const R pnv = ((R)qs[k * 10 + j] + atp) + kr;
        if (ln < 8) {
          GLB double* Kk = Kl + k * 48;
#pragma unroll
          for (int r = 0; r < 6; ++r) Kk[r * 8] = (double)mb[r];
        }
        if (ln < 8) {
          pn[ln] = pnv;
        } else if (ln == 8) {
#pragma unroll
          for (int r = 0; r < 6; ++r) kf[k * 6 + r] = (double)mb[r];
        }
        sync();
        STAMP1(PH_RD); }
      ok = !wany(!ok);  // every lane computed the same pivots; make it explicit
      if (!ok) return false;
      LDS R* t1 = Pc; Pc = Pn; Pn = t1;
      LDS R* t2 = pc; pc = pn; pn = t2;
      return true;
    };
    // two stages per trip, their prefetched operands in alternating registers: no
    // loop-carried register copies (which made the loop latch wait for every store)
    double qB, rB, vB;
    StageAB abA, abB;
    if constexpr (CAP::deep) abA = stage_ab(N - 1, Tv);
    for (int k = N - 1; k >= 0; k -= 2) {
      {
        const int kp = k > 0 ? k - 1 : 0;
        qB = Qsl[kp * 36]; rB = Rdl[kp * 6]; vB = rvl[kp * 6];
      }
      if (!stage(k, qvn, rdn, rvn, abA, abB) || k == 0) break;
      {
        const int kp = k > 1 ? k - 2 : 0;
        qvn = Qsl[kp * 36]; rdn = Rdl[kp * 6]; rvn = rvl[kp * 6];
      }
      if (!stage(k - 1, qB, rB, vB, abB, abA)) break;
    }
    if constexpr (SG) nneg = __builtin_amdgcn_readfirstlane(negs);
    return ok;
  }

  // gradient-only re-solve with the stored factors (second-order correction): the vector
  // recursion p_k = q_k + A_k^T p_{k+1} + K_k^T r~_k, r~_k = r_k + B_k^T p_{k+1}.
  //  - Lane i < 8 forms p_k[i] (row i: its K_k column, prefetched a stage ahead) and
  //    publishes it through LDS; every lane reads p_{k+1} back and forms r~_k.
  //  - k_k = -R~_k^-1 r~_k is not needed by the recursion, so the stages' re-factorisations
  //    of R~_k and their solves leave the serial sweep: lane k keeps its stage's r~_k and,
  //    after the sweep, factorises its own R~_k and solves for k_k, all stages at once.
  // Every value is formed by the same operations in the same order as when every lane ran
  // the whole recursion (row i's expressions are written out per kind, as before): the
  // same bits.
  // ZQ: linear state terms q_k = 0 (the refinement's right-hand side is a control residual)
  template <bool ZQ = false>
  __device__ __forceinline__ void resolve(const GLB double* rv) {
#ifdef NMPC_STAMPS
    if (lanef() == 0) stamps[PH_RC] += 1.0;  // count SOC re-solves
#endif
    STAMP0();
    using R = typename CAP::RT;  // the factorisation's precision
    const int ln = lanef();
    const int li = ln < 8 ? ln : 7;  // the row of p this lane forms (lanes >= 8 duplicate row 7)
    LDS R* pv = (LDS R*)pva;         // p_{k+1}, published by lanes 0..7
    if (ln < 8) pv[ln] = ZQ ? (R)0 : (R)qs[N * 10 + ln];
    R rtk[6];  // r~ of stage ln (CAP::nmax < WAVE: one stage per lane)
#pragma unroll
    for (int r = 0; r < 6; ++r) rtk[r] = (R)0;
    const GLB double* const Kl = K + li;  // this lane's K column: K_k[r][li] = Kl[k*48 + r*8]
    sync();
    // one stage of the backward recursion with its stored r_k (rin) and K column (kc)
    auto stage = [&](int k, const R (&rin)[6], const R (&kc)[6], const StageAB& ab, StageAB& abn) {
      const StageAB abk = CAP::deep ? ab : stage_ab(k, T);  // (as in riccati_)
      if constexpr (CAP::deep) abn = stage_ab(k > 0 ? k - 1 : 0, T);
      const R E03 = (R)abk.E03, E04 = (R)abk.E04, E13 = (R)abk.E13, E14 = (R)abk.E14, E23 = (R)abk.E23;
      const R b00 = (R)abk.b00, b10 = (R)abk.b10, b20 = (R)abk.b20, Tr = (R)T;
      R p8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) p8[i] = pv[i];
      const R pl = pv[li];
      const R ql = ZQ ? (R)0 : (R)qs[k * 10 + li];
      R rt[6];
      rt[0] = rin[0] + ((b00 * p8[0] + b10 * p8[1]) + b20 * p8[2]);
#pragma unroll
      for (int r = 1; r < 6; ++r) rt[r] = rin[r] + Tr * p8[2 + r];
      if (nfix > 0) {
        const int fm = fixm[k];
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if ((fm >> r) & 1) rt[r] = (R)0;
      }
      const bool mine = ln == k;
#pragma unroll
      for (int r = 0; r < 6; ++r) rtk[r] = mine ? rt[r] : rtk[r];
      // (A^T p)[li]: rows 3 and 4 add the E column terms (both formed, selected by row)
      const R at3 = pl + ((E03 * p8[0] + E13 * p8[1]) + E23 * p8[2]);
      const R at4 = pl + (E04 * p8[0] + E14 * p8[1]);
      const R atp = li == 3 ? at3 : (li == 4 ? at4 : pl);
      R kr = (R)0;
#pragma unroll
      for (int r = 0; r < 6; ++r) kr += kc[r] * rt[r];
      const R pnv = (ql + atp) + kr;
      sync();  // every lane has read p_{k+1}
      if (ln < 8) pv[ln] = pnv;
      sync();
    };
    // the stored r_k and K columns do not depend on the recursion: stage k-1's are fetched
    // while stage k is formed (two stages per trip, alternating register sets; clamped
    // fetches)
    R rA[6], rB[6], kA[6], kB[6];
    auto fetch = [&](R (&ro)[6], R (&ko)[6], int ks) {
      const int kc = ks > 0 ? ks : 0;
#pragma unroll
      for (int r = 0; r < 6; ++r) ro[r] = (R)rv[kc * 6 + r];
#pragma unroll
      for (int r = 0; r < 6; ++r) ko[r] = (R)Kl[kc * 48 + r * 8];
    };
    fetch(rA, kA, N - 1);
    StageAB abA, abB;
    if constexpr (CAP::deep) abA = stage_ab(N - 1, T);
    for (int k = N - 1; k >= 0; k -= 2) {
      fetch(rB, kB, k - 1);
      stage(k, rA, kA, abA, abB);
      if (k == 0) break;
      fetch(rA, kA, k - 2);
      stage(k - 1, rB, kB, abB, abA);
    }
    // k_k = -R~_k^-1 r~_k, lane k: R~_k's Cholesky factor and the two triangular solves
    if (ln < N) {
      R Lm[21], idg[6], v[6];
#pragma unroll
      for (int t = 0; t < 21; ++t) Lm[t] = (R)Rk[ln * 21 + t];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        R dg = Lm[c * (c + 1) / 2 + c];
#pragma unroll
        for (int t = 0; t < c; ++t) dg -= Lm[c * (c + 1) / 2 + t] * Lm[c * (c + 1) / 2 + t];
        const R ig = rsq(dg);
        Lm[c * (c + 1) / 2 + c] = dg * ig;
        idg[c] = ig;
#pragma unroll
        for (int r = c + 1; r < 6; ++r) {
          R a = Lm[r * (r + 1) / 2 + c];
#pragma unroll
          for (int t = 0; t < c; ++t) a -= Lm[r * (r + 1) / 2 + t] * Lm[c * (c + 1) / 2 + t];
          Lm[r * (r + 1) / 2 + c] = a * ig;
        }
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        R a = rtk[r];
#pragma unroll
        for (int t = 0; t < r; ++t) a -= Lm[r * (r + 1) / 2 + t] * v[t];
        v[r] = a * idg[r];
      }
#pragma unroll
      for (int r = 5; r >= 0; --r) {
        R a = v[r];
#pragma unroll
        for (int t = r + 1; t < 6; ++t) a -= Lm[t * (t + 1) / 2 + r] * v[t];
        v[r] = a * idg[r];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) kf[ln * 6 + r] = (double)(-v[r]);
    }
    sync();
    STAMP1(PH_RESOLVE);
  }

  // One step of iterative refinement in fp64 of a step (dUo, dXo) solved with the fp32
  // factorisation (CAP::refine): the U-space residual of the LQ subproblem the factors
  // came from, res_k = S_k dx_k + R_k du_k + r_k + B_k^T lam_{k+1} with
  // lam_k = Q_k dx_k + S_k^T du_k + q_k + A_k^T lam_{k+1} (lam_N = Q_N dx_N + q_N), is
  // formed in fp64 (stage-parallel, adjoint-style suffix sums), solved with the same
  // factors (resolve with q = 0, r = res) and the correction added.  No-op for fp64.
  __device__ __forceinline__ void refine(const GLB double* Rd, const GLB double* rv, GLB double* dUo,
                                         LDS double* dXo) {
    if constexpr (CAP::refine) {
      const int k = lanef();
      LDS double* wv = inc;  // w_k
      LDS double* lm = Xt;   // lam_k (Xt is free whenever a step is being computed)
      if (k <= N) {
        double dx[8], w[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) dx[a] = dXo[k * 8 + a];
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          double acc = qs[k * 10 + a];
#pragma unroll
          for (int c = 0; c < 8; ++c) acc += Qs[k * 36 + (a <= c ? pk8(a, c) : pk8(c, a))] * dx[c];
          w[a] = acc;
        }
        if (k < N) {
          const double du0 = dUo[k * 6];
          w[3] += qs[k * 10 + 8] * du0;
          w[4] += qs[k * 10 + 9] * du0;
        }
#pragma unroll
        for (int a = 0; a < 8; ++a) wv[k * 8 + a] = w[a];
      }
      sync();
      if (k <= N) {  // components 0,1,2,5,6,7: suffix sums of w (A = I + E, E^T only feeds 3, 4)
        const int cs[6] = {0, 1, 2, 5, 6, 7};
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          double acc = 0.0;
          for (int jj = N; jj >= k; --jj) acc += wv[jj * 8 + cs[q]];
          lm[k * 8 + cs[q]] = acc;
        }
      }
      sync();
      if (k <= N) {
        double a3 = wv[N * 8 + 3], a4 = wv[N * 8 + 4];
        for (int jj = N - 1; jj >= k; --jj) {
          double E03, E04, E13, E14, E23, b00, b10, b20;
          stage_AB(jj, E03, E04, E13, E14, E23, b00, b10, b20);
          const LDS double* ln = lm + (jj + 1) * 8;
          a3 = wv[jj * 8 + 3] + (((E03 * ln[0] + E13 * ln[1]) + E23 * ln[2]) + a3);
          a4 = wv[jj * 8 + 4] + ((E04 * ln[0] + E14 * ln[1]) + a4);
        }
        lm[k * 8 + 3] = a3;
        lm[k * 8 + 4] = a4;
      }
      sync();
      if (k < N) {
        double E03, E04, E13, E14, E23, b00, b10, b20;
        stage_AB(k, E03, E04, E13, E14, E23, b00, b10, b20);
        const LDS double* ln = lm + (k + 1) * 8;
        const LDS double* dxk = dXo + k * 8;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double r = rv[k * 6 + c] + (Rd[k * 6 + c] + delta) * dUo[k * 6 + c];
          r += (c == 0) ? ((b00 * ln[0] + b10 * ln[1]) + b20 * ln[2]) + (qs[k * 10 + 8] * dxk[3] + qs[k * 10 + 9] * dxk[4])
                        : T * ln[2 + c];
          rres[k * 6 + c] = (c < nuE && !fixed(k * 6 + c)) ? r : 0.0;  // absent / fixed: zero step
        }
      }
      sync();
      resolve<true>(rres);
      forward(dUr, rdX);
      for (int i = lanef(); i < nw; i += WAVE) dUo[i] += dUr[i];
      for (int i = lanef(); i < 8 * (N + 1); i += WAVE) dXo[i] += rdX[i];
      sync();
    }
  }

  // forward sweep: du_k = K_k dx_k + k_k ; dx_{k+1} = A_k dx_k + B_k du_k.
  // Lanes 0..5 form du_k[r] (row r of K); readlane broadcasts it; every lanef()
  // carries dx redundantly.  Lane 0 stores dX.
  __device__ __forceinline__ void forward(GLB double* dUo, LDS double* dXo) {
    STAMP0();
    const int ln = lanef();
    double dx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) dx[i] = 0.0;
    if (ln < 8) dXo[ln] = 0.0;
    const int r = ln < 6 ? ln : 5;
    // K_k rows come from global memory and do not depend on dx: fetch stage k+1's
    // row while stage k is being formed
    // one stage: du_k = K_k dx_k + k_k (lanes 0..5), dx_{k+1} = A_k dx_k + B_k du_k
    auto stage = [&](int k, const double (&Kr)[8], double kk) {
      double E03, E04, E13, E14, E23, b00, b10, b20;
      stage_AB(k, E03, E04, E13, E14, E23, b00, b10, b20);
      double a = kk;
#pragma unroll
      for (int c = 0; c < 8; ++c) a += Kr[c] * dx[c];
      dUo[k * 6 + r] = a;  // lanes >= 5 all hold row 5: same value, same address
      double du_[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) du_[q] = readlane_d(a, q);
      double xn[8];
      xn[0] = dx[0] + (E03 * dx[3] + E04 * dx[4]) + b00 * du_[0];
      xn[1] = dx[1] + (E13 * dx[3] + E14 * dx[4]) + b10 * du_[0];
      xn[2] = dx[2] + E23 * dx[3] + b20 * du_[0];
#pragma unroll
      for (int c = 0; c < 5; ++c) xn[3 + c] = dx[3 + c] + T * du_[1 + c];
      if (ln == 0) {
#pragma unroll
        for (int c = 0; c < 8; ++c) dXo[(k + 1) * 8 + c] = xn[c];
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) dx[c] = xn[c];
    };
    // K_k rows come from global memory and do not depend on dx: they are fetched ahead,
    // into register sets used in turn (no register copies between stages).  A stage's
    // arithmetic is far shorter than a global load's latency, so the deep classes fetch
    // three stages ahead (four sets), the others one (two sets).
    double K0[8], K1[8], K2[8], K3[8], k0, k1, k2, k3;
    // (fetches clamped to the last stage rather than guarded: no branch, see riccati_)
    auto fetch = [&](double (&Kr)[8], double& kk, int ks) {
      const int kc = ks < N ? ks : N - 1;
#pragma unroll
      for (int c = 0; c < 8; ++c) Kr[c] = K[kc * 48 + r * 8 + c];
      kk = kf[kc * 6 + r];
    };
    if constexpr (CAP::deep) {
      fetch(K0, k0, 0);
      fetch(K1, k1, 1);
      fetch(K2, k2, 2);
      for (int k = 0; k < N; k += 4) {
        fetch(K3, k3, k + 3);
        stage(k, K0, k0);
        if (k + 1 >= N) break;
        fetch(K0, k0, k + 4);
        stage(k + 1, K1, k1);
        if (k + 2 >= N) break;
        fetch(K1, k1, k + 5);
        stage(k + 2, K2, k2);
        if (k + 3 >= N) break;
        fetch(K2, k2, k + 6);
        stage(k + 3, K3, k3);
      }
    } else {
      (void)K2; (void)K3; (void)k2; (void)k3;
      fetch(K0, k0, 0);
      for (int k = 0; k < N; k += 2) {
        fetch(K1, k1, k + 1);
        stage(k, K0, k0);
        if (k + 1 >= N) break;
        fetch(K0, k0, k + 2);
        stage(k + 1, K1, k1);
      }
    }
    sync();
    STAMP1(PH_FWD);
  }

  // second-order correction's row step ds_r = Gt_r dX_k + dms_r (J dU = G Z dU = G dX),
  // and the primal fraction to the boundary of the step (dUs, ds) in the same pass
  // (frac_to_bound: the same expressions; min over the rows and controls)
  __device__ __forceinline__ double row_step_soc(const LDS double* dXs, const GLB double* dUs, RV* dso,
                                                 double tau_) {
    STAMP0();
    double a = 1.0;
    rows([&](int r, bool on) {
      const int k = r / m, i = r - k * m;
      const LDS double* xk = X + k * 8;
      const LDS double* dxk = dXs + k * 8;
      double jd;
      if (i < nb) {
        jd = dc[r] * dxk[boxidx(i)];
      } else {
        const int o = i - nb;
        const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
        const double idd = rsq(ddx * ddx + ddy * ddy);
        jd = dc[r] * ((-(ddx * idd)) * dxk[0] + (-(ddy * idd)) * dxk[1]);
      }
      const double lo = dl[r], hi = du[r], sr = s[r];
      const double dd = eqlo(lo) ? 0.0 : jd + dms[r];  // equality rows: the slack stays at the target
      if (on) dso[r] = dd;
      const double al = qd(-tau_ * (sr - lo), dd), au = qd(-tau_ * (hi - sr), -dd);
      if (on && hasl(lo) && dd < 0) a = fmin(a, al);
      if (on && hasu(hi) && -dd < 0) a = fmin(a, au);
    });
    for (int i = lanef(); i < nw; i += WAVE) {
      const double dx = dUs[i];
      if (hasl(xl[i]) && dx < 0) a = fmin(a, qd(-tau_ * (U[i] - xl[i]), dx));
      if (hasu(xu[i]) && -dx < 0) a = fmin(a, qd(-tau_ * (xu[i] - U[i]), -dx));
    }
    a = wmin(a);
    STAMP1(PH_ROWSTEP);
    sync();
    return a;
  }

  // Newton-direction row step fused with the line-search set-up sums over the
  // same rows: theta = sum |d - s|, the slack part of grad(phi)^T d, and the
  // tiny-step ratio max |ds| / (1 + |s|) (per-lane partials; caller reduces)
  // The same pass also forms the row parts of the step's primal and dual fraction-to-the-
  // boundary (frac_to_bound_x / dual_frac_to_bound_x with tau_, mu_: the same expressions,
  // per-lane partial minima ap / ad, caller reduces), which the line search and the accept
  // pass would otherwise each recompute in a pass of their own.
  __device__ __forceinline__ void row_step_ls(const LDS double* dXs, double mu_, double tau_, double& th, double& g,
                                              double& msv, double& ap, double& ad) {
    STAMP0();
    const double kd = P->o.kappa_d;
    th = 0.0; g = 0.0; msv = 0.0; ap = 1.0; ad = 1.0;
    rows([&](int r, bool on) {
      const int k = r / m, i = r - k * m;
      const double dcr = dc[r], sr = s[r], dr = d[r], lo = dl[r], hi = du[r];
      const LDS double* xk = X + k * 8;
      const LDS double* dxk = dXs + k * 8;
      double jd;
      if (i < nb) {
        jd = dcr * dxk[boxidx(i)];
      } else {
        const int o = i - nb;
        const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
        const double idd = rsq(ddx * ddx + ddy * ddy);
        jd = dcr * ((-(ddx * idd)) * dxk[0] + (-(ddy * idd)) * dxk[1]);
      }
      const double dsr = eqlo(lo) ? 0.0 : jd + (dr - sr);
      if (on) ds[r] = dsr;
      const bool hl = hasl(lo), hu = hasu(hi);
      const double gs = -(hl ? qd(mu_, sr - lo) : 0.0) + (hu ? qd(mu_, hi - sr) : 0.0) +
                        kd * mu_ * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0));
      if (on) {
        th += fabs(dr - sr);
        g += gs * dsr;
        msv = fmax(msv, fabs(qd(dsr, 1.0 + fabs(sr))));
      }
      // fraction to the boundary of this step: primal (frac_to_bound_x) ...
      const double al = qd(-tau_ * (sr - lo), dsr), au = qd(-tau_ * (hi - sr), -dsr);
      if (on && hl && dsr < 0) ap = fmin(ap, al);
      if (on && hu && -dsr < 0) ap = fmin(ap, au);
      // ... and dual (dual_frac_to_bound_x: dv_s with mu_)
      const double vlr = vl[r], vur = vu[r];
      double a1 = 0.0, a2 = 0.0;
      if (hl) { const double iS = rcp(sr - lo); a1 = mu_ * iS - vlr - vlr * iS * dsr; }
      if (hu) { const double iS = rcp(hi - sr); a2 = mu_ * iS - vur + vur * iS * dsr; }
      const double b1 = qd(-tau_ * vlr, a1), b2 = qd(-tau_ * vur, a2);
      if (on && hl && a1 < 0) ad = fmin(ad, b1);
      if (on && hu && a2 < 0) ad = fmin(ad, b2);
    });
    STAMP1(PH_ROWSTEP);
    sync();
  }

  // ------------------------------------------------ restoration phase rows
  // p, n (d(x) - s - p + n = 0, p, n >= 0) eliminated per row: weight
  // D~ = (1/D + 1/Sp + 1/Sn)^-1 and right-hand side D~ r~ (oracle restoration()),
  // written without 1/D so rows with no bound (D = 0) stay finite.
  __device__ __forceinline__ void row_resto(int r, bool soc, double& D, double& rs, double& Sp, double& Sn,
                                            double& rp, double& rn, double& Dt, double& Dr) const {
    row_rs(r, D, rs);
    const double kd = P->o.kappa_d;
    const double pr = pR[r], nr = nR[r];
    const double ip = qd(1.0, pr), in_ = qd(1.0, nr);
    Sp = zpR[r] * ip + delta;
    Sn = znR[r] * in_ + delta;
    rp = rho - y[r] - mu * ip + kd * mu;
    rn = rho + y[r] - mu * in_ + kd * mu;
    const double c = soc ? cms[r] : d[r] - s[r] - pr + nr;
    const double iSp = qd(1.0, Sp), iSn = qd(1.0, Sn);
    const double den = qd(1.0, 1.0 + D * (iSp + iSn));
    Dt = D * den;
    Dr = Dt * (c + rp * iSp - rn * iSn) + rs * den;
    if (eqr(r)) {  // equality row: no slack, the D -> infinity limit
      Dt = qd(1.0, iSp + iSn);
      Dr = Dt * (c + rp * iSp - rn * iSn);
    }
  }
  __device__ __forceinline__ double dr2(int i) const {  // D_R^2 = 1/max(1,|x_R|)^2
    const double a = fmax(1.0, fabs(UR[i]));
    return qd(1.0, a * a);
  }
  // restoration step rows: dy, dp, dn, ds (= J dx + c - dp + dn); for the Newton
  // direction also theta_R and the slack/p/n part of grad(phi_R)^T d
  // The pass also forms the row part of the step's primal fraction to the boundary
  // (frac_to_bound_resto with tau_) and, for the Newton direction (!soc), of its dual one
  // (dual_frac_to_bound_resto with the current mu): per-lane partial minima ap / ad, the
  // caller adds the controls and reduces.
  __device__ __forceinline__ void row_step_resto(const LDS double* dXs, bool soc, RV* dso, GLB double* dpo,
                                                 GLB double* dno, GLB double* dyo, double& th, double& gsum,
                                                 double tau_, double& ap, double& ad) {
    const double kd = P->o.kappa_d;
    th = 0.0; gsum = 0.0; ap = 1.0; ad = 1.0;
    rows_r([&](int r, bool on) {
      const int k = r / m, i = r - k * m;
      const LDS double* xk = X + k * 8;
      const LDS double* dxk = dXs + k * 8;
      double jd;
      if (i < nb) {
        jd = dc[r] * dxk[boxidx(i)];
      } else {
        const int o = i - nb;
        const double ddx = xk[0] - obx[o], ddy = xk[1] - oby[o];
        const double idd = rsq(ddx * ddx + ddy * ddy);
        jd = dc[r] * ((-(ddx * idd)) * dxk[0] + (-(ddy * idd)) * dxk[1]);
      }
      double D, rs, Sp, Sn, rp, rn, Dt, Dr;
      row_resto(r, soc, D, rs, Sp, Sn, rp, rn, Dt, Dr);
      const double pr = pR[r], nr = nR[r];
      const double c = soc ? cms[r] : d[r] - s[r] - pr + nr;
      const double dyv = Dt * jd + Dr;
      const double dpv = qd(dyv - rp, Sp), dnv = qd(-dyv - rn, Sn);
      const double dsv = eqr(r) ? 0.0 : jd + c - dpv + dnv;
      if (on) { dso[r] = dsv; dpo[r] = dpv; dno[r] = dnv; dyo[r] = dyv; }
      const double lo = dl[r], hi = du[r], sr = s[r];
      const bool hl = hasl(lo), hu = hasu(hi);
      // primal fraction to the boundary (frac_to_bound_x rows + the p, n bounds)
      {
        const double al = qd(-tau_ * (sr - lo), dsv), au = qd(-tau_ * (hi - sr), -dsv);
        if (on && hl && dsv < 0) ap = fmin(ap, al);
        if (on && hu && -dsv < 0) ap = fmin(ap, au);
        const double bp = qd(-tau_ * pr, dpv), bn = qd(-tau_ * nr, dnv);
        if (on && dpv < 0) ap = fmin(ap, bp);
        if (on && dnv < 0) ap = fmin(ap, bn);
      }
      if (!soc) {
        // (plain divisions here: with qd() these two lines alone change the restoration
        // line search's results -- the one place the bitwise A/B of round 6 found one, cause
        // not isolated -- so they keep the compiler's division)
        const double gs = -(hl ? mu / (sr - lo) : 0.0) + (hu ? mu / (hi - sr) : 0.0) +
                          kd * mu * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0));
        const double gr = gs * dsv + (rho - mu / pr + kd * mu) * dpv + (rho - mu / nr + kd * mu) * dnv;
        if (on) {
          th += fabs(c);
          gsum += gr;
        }
        // dual fraction to the boundary (dual_frac_to_bound_x rows with dv_s, + the p, n
        // multipliers)
        const double vlr = vl[r], vur = vu[r], zp = zpR[r], zn = znR[r];
        double a1 = 0.0, a2 = 0.0;
        if (hl) { const double iS = rcp(sr - lo); a1 = mu * iS - vlr - vlr * iS * dsv; }
        if (hu) { const double iS = rcp(hi - sr); a2 = mu * iS - vur + vur * iS * dsv; }
        const double b1 = qd(-tau_ * vlr, a1), b2 = qd(-tau_ * vur, a2);
        if (on && hl && a1 < 0) ad = fmin(ad, b1);
        if (on && hu && a2 < 0) ad = fmin(ad, b2);
        const double dzp = qd(mu, pr) - zp - qd(zp, pr) * dpv;
        const double dzn = qd(mu, nr) - zn - qd(zn, nr) * dnv;
        const double cp = qd(-tau_ * zp, dzp), cn = qd(-tau_ * zn, dzn);
        if (on && dzp < 0) ad = fmin(ad, cp);
        if (on && dzn < 0) ad = fmin(ad, cn);
      }
    });
    sync();
  }
  // p, n part of phi_R at s + a ds, p + a dp, n + a dn (the x/s part comes from barrier_obj)
  __device__ __forceinline__ double pn_of(double pn, double lg, double prox) const {
    return rho * pn + 0.5 * etaR * prox - mu * lg + P->o.kappa_d * mu * pn;
  }
  __device__ __forceinline__ double resto_pn_terms(const GLB double* Us, double a, const GLB double* dps,
                                                   const GLB double* dns) {
    double pn = 0.0, prox = 0.0;
    LogAcc la;
    rows_r([&](int r, bool on) {
      const double pv = dps ? pR[r] + a * dps[r] : pR[r], nv = dns ? nR[r] + a * dns[r] : nR[r];
      la.mul2(on ? pv : 1.0, on ? nv : 1.0);
      if (on) pn += pv + nv;
    });
    for (int i = lanef(); i < nw; i += WAVE) {
      const double dd = Us[i] - UR[i];
      prox += dr2(i) * dd * dd;
    }
    double lg;
    pn = wsum(pn); lg = wsum(la.log()); prox = wsum(prox);
    rvars[34] = pn; rvars[35] = lg; rvars[36] = prox;
    return pn_of(pn, lg, prox);
  }
  // restoration trial point: theta_R and phi_R (fo, fo2: 0 -- phi_R does not contain the
  // original objective, so the trials are formed without it and the restoration phase
  // forms it for the accepted trial alone, Solver::eval_f)
  // spec (kSpec classes): 0 this trial alone; 1 this trial and the next backtracking one
  // (a2) formed together (rollout2 / eval_fg2); 2 this trial was formed as the second of a
  // pair: its X in `lam`, its rows in `dms`
  __device__ __forceinline__ bool trial_resto(double a, const GLB double* dUs, const RV* dss,
                                              const GLB double* dps, const GLB double* dns, double& fo,
                                              double& phit, double& tht, int spec = 0, double a2 = 0.0,
                                              double* fo2 = nullptr) {
    // the trial controls, their barrier terms and the proximity term in one pass (each
    // accumulator keeps the per-lane order of barrier_obj / resto_pn_terms)
    RSTAMP0(_trs);
    RCOUNT(PH_DFTB);
    XCOUNT(X_TCNT);
    XSTAMP0(_x0);
    UPre up;  // (a pair's second trial forms no rollout)
    if (spec != 2) up = preload_u(U, dUs, (kSpec && spec == 1) ? 31 : WAVE - 1);
    double th = 0.0, damp = 0.0, pn = 0.0, prox = 0.0;
    LogAcc logs, la;  // the barrier terms' and the p / n terms' log sums
    ctrls([&](int i, bool on) {
      const double ui = U[i] + a * dUs[i];
      if (on) Ut[i] = ui;
      barrier_ctrl1(i, on, ui, logs, damp);
      const double dd = ui - UR[i];
      const double pv = dr2(i) * dd * dd;
      if (on) prox += pv;
    });
    sync();
    XSTAMP1(_x0, X_TCTRL);
    bool bad = false;
    // theta_R, the barrier sums and the p/n sums in one pass over the rows
    auto rowpass = [&](auto dtv) {
      rows_r([&](int r, bool on) {
        const double sv = s[r] + a * dss[r], pv = pR[r] + a * dps[r], nv = nR[r] + a * dns[r];
        const double dtr = dtv[r];
        barrier_row(r, on, sv, logs, damp);
        la.mul2(on ? pv : 1.0, on ? nv : 1.0);
        if (on) {
          th += fabs(dtr - sv - pv + nv);
          if (!isfinite(dtr)) bad = true;
          pn += pv + nv;
        }
      });
    };
    bool done = false;
    if constexpr (kSpec) {
      if (spec == 2) {
        fo = 0.0;
        XSTAMP0(_x3);
        rowpass(dms);
        XSTAMP1(_x3, X_TROWS);
        done = true;
      } else if (spec == 1) {
        XSTAMP0(_x1);
        rollout2(U, dUs, a, a2, &up);
        XSTAMP1(_x1, X_TROLL);
        XSTAMP0(_x2);
        double f0, f1;
        eval_fg2(f0, f1, false);
        fo = 0.0;
        *fo2 = 0.0;
        XSTAMP1(_x2, X_TEVAL);
        XSTAMP0(_x3);
        rowpass(dt);
        XSTAMP1(_x3, X_TROWS);
        done = true;
      }
    }
    if (!done) {
      XSTAMP0(_x1);
      rollout(U, Xt, dUs, a, &up);
      XSTAMP1(_x1, X_TROLL);
      XSTAMP0(_x2);
      fo = 0.0;
      eval_fg(Xt, dt, dc, false);
      XSTAMP1(_x2, X_TEVAL);
      XSTAMP0(_x3);
      rowpass(dt);
      XSTAMP1(_x3, X_TROWS);
    }
    XSTAMP0(_x4);
    tht = wsum(th);
    if (wany(bad)) return false;
    const double phb = barrier_fin(0.0, logs, damp);
    double lg;
    pn = wsum(pn); lg = wsum(la.log()); prox = wsum(prox);
    rvars[34] = pn; rvars[35] = lg; rvars[36] = prox;
    phit = phb + pn_of(pn, lg, prox);
    XSTAMP1(_x4, X_TFIN);
    RSTAMP1(_trs, PH_BARR);
    return isfinite(phit);
  }
  __device__ __forceinline__ double frac_to_bound_resto(double tau_, const GLB double* dUs, const RV* dss,
                                                        const GLB double* dps, const GLB double* dns) const {
    double b = 1.0;  // p, n bounds in the same pass (min is order-free)
    const double a = frac_to_bound_x(tau_, dUs, dss, [&](int r, bool on) {
      const double dp = dps[r], dn = dns[r], pr = pR[r], nr = nR[r];
      const double bp = qd(-tau_ * pr, dp), bn = qd(-tau_ * nr, dn);
      if (on && dp < 0) b = fmin(b, bp);
      if (on && dn < 0) b = fmin(b, bn);
    });
    return fmin(a, wmin(b));
  }
  __device__ __forceinline__ double dual_frac_to_bound_resto(double tau_, const GLB double* dUs, const RV* dss,
                                                             const GLB double* dps, const GLB double* dns) const {
    double b = 1.0;
    const double a = dual_frac_to_bound_x(tau_, dUs, dss, [&](int r, bool on) {
      const double pr = pR[r], nr = nR[r], zp = zpR[r], zn = znR[r], dp = dps[r], dn = dns[r];
      const double dzp = qd(mu, pr) - zp - qd(zp, pr) * dp;
      const double dzn = qd(mu, nr) - zn - qd(zn, nr) * dn;
      const double bp = qd(-tau_ * zp, dzp), bn = qd(-tau_ * zn, dzn);
      if (on && dzp < 0) b = fmin(b, bp);
      if (on && dzn < 0) b = fmin(b, bn);
    });
    return fmin(a, wmin(b));
  }

  // primal fraction to the boundary (oracle frac_to_bound)
  __device__ __forceinline__ double frac_to_bound(double tau_, const GLB double* dUs, const RV* dss) const {
    return frac_to_bound_x(tau_, dUs, dss, [](int, bool) {});
  }
  // ... with `extra(r, on)` run inside the same pass over the rows
  template <class F>
  __device__ __forceinline__ double frac_to_bound_x(double tau_, const GLB double* dUs, const RV* dss,
                                                    F&& extra) const {
    STAMP0();
    double a = 1.0;
    ctrls([&](int i, bool on) {  // (a repeated last entry leaves a minimum unchanged)
      const double dx = dUs[i];
      if (hasl(xl[i]) && dx < 0) a = fmin(a, qd(-tau_ * (U[i] - xl[i]), dx));
      if (hasu(xu[i]) && -dx < 0) a = fmin(a, qd(-tau_ * (xu[i] - U[i]), -dx));
    });
    rows([&](int r, bool on) {
      const double dd = dss[r], sr = s[r], lo = dl[r], hi = du[r];
      const double al = qd(-tau_ * (sr - lo), dd), au = qd(-tau_ * (hi - sr), -dd);
      if (on && hasl(lo) && dd < 0) a = fmin(a, al);
      if (on && hasu(hi) && -dd < 0) a = fmin(a, au);
      extra(r, on);
    });
    a = wmin(a);
    STAMP1G(PH_FTB);
    return a;
  }

  // dual step components (oracle solve_dir) -- current slacks
  __device__ __forceinline__ void dz_x(int i, double dx, double& dzl, double& dzu) const {
    if constexpr (CAP::deep) {
      // loads hoisted and both sides formed, then selected (same arithmetic): the control
      // passes' global loads are not issued one bound at a time behind lane-dependent branches
      const double xli = xl[i], xui = xu[i], ui = U[i], zli = zl[i], zui = zu[i];
      const bool hl = hasl(xli), hu = hasu(xui);
      const double iSl = hl ? rcp(ui - xli) : 0.0, iSu = hu ? rcp(xui - ui) : 0.0;
      dzl = hl ? mu * iSl - zli - zli * iSl * dx : 0.0;
      dzu = hu ? mu * iSu - zui + zui * iSu * dx : 0.0;
    } else {
      dzl = 0.0; dzu = 0.0;
      if (hasl(xl[i])) { const double iS = rcp(U[i] - xl[i]); dzl = mu * iS - zl[i] - zl[i] * iS * dx; }
      if (hasu(xu[i])) { const double iS = rcp(xu[i] - U[i]); dzu = mu * iS - zu[i] + zu[i] * iS * dx; }
    }
  }
  __device__ __forceinline__ void dv_s(int r, double dsv, double& dvl, double& dvu) const {
    dvl = 0.0; dvu = 0.0;
    if (hasl(dl[r])) { const double iS = rcp(s[r] - dl[r]); dvl = mu * iS - vl[r] - vl[r] * iS * dsv; }
    if (hasu(du[r])) { const double iS = rcp(du[r] - s[r]); dvu = mu * iS - vu[r] + vu[r] * iS * dsv; }
  }
  __device__ __forceinline__ double dual_frac_to_bound(double tau_, const GLB double* dUs, const RV* dss) const {
    return dual_frac_to_bound_x(tau_, dUs, dss, [](int, bool) {});
  }
  template <class F>
  __device__ __forceinline__ double dual_frac_to_bound_x(double tau_, const GLB double* dUs, const RV* dss,
                                                         F&& extra) const {
    STAMP0();
    double a = 1.0;
    ctrls([&](int i, bool on) {
      double a1, a2;
      dz_x(i, dUs[i], a1, a2);
      if (hasl(xl[i]) && a1 < 0) a = fmin(a, qd(-tau_ * zl[i], a1));
      if (hasu(xu[i]) && a2 < 0) a = fmin(a, qd(-tau_ * zu[i], a2));
    });
    rows([&](int r, bool on) {
      const double sr = s[r], lo = dl[r], hi = du[r], vlr = vl[r], vur = vu[r], dsv = dss[r];
      const bool hl = hasl(lo), hu = hasu(hi);
      double a1 = 0.0, a2 = 0.0;  // dv_s with the loads hoisted
      if (hl) { const double iS = rcp(sr - lo); a1 = mu * iS - vlr - vlr * iS * dsv; }
      if (hu) { const double iS = rcp(hi - sr); a2 = mu * iS - vur + vur * iS * dsv; }
      const double b1 = qd(-tau_ * vlr, a1), b2 = qd(-tau_ * vur, a2);
      if (on && hl && a1 < 0) a = fmin(a, b1);
      if (on && hu && a2 < 0) a = fmin(a, b2);
      extra(r, on);
    });
    a = wmin(a);
    STAMP1G(PH_DFTB);
    return a;
  }

  // rs_r (oracle rs) and D_r
  __device__ __forceinline__ void row_rs(int r, double& D, double& rs) const {
    const bool lo = hasl(dl[r]), hi = hasu(du[r]);
    const double iSl = lo ? rcp(s[r] - dl[r]) : 0.0, iSu = hi ? rcp(du[r] - s[r]) : 0.0;
    D = vl[r] * iSl + vu[r] * iSu + delta;
    rs = -y[r] - mu * iSl + mu * iSu +
         P->o.kappa_d * mu * ((lo && !hi ? 1.0 : 0.0) - (hi && !lo ? 1.0 : 0.0));
  }

  // complementarity max |S z - mu_| over all bounds
  __device__ __forceinline__ double compl_max(double mu_) const {
    double c = 0.0;
    ctrls([&](int i, bool on) {
      if (hasl(xl[i])) c = fmax(c, fabs((U[i] - xl[i]) * zl[i] - mu_));
      if (hasu(xu[i])) c = fmax(c, fabs((xu[i] - U[i]) * zu[i] - mu_));
    });
    rows([&](int r, bool on) {
      const double sr = s[r], lo = dl[r], hi = du[r], vlr = vl[r], vur = vu[r];
      const double cl = fabs((sr - lo) * vlr - mu_), cu = fabs((hi - sr) * vur - mu_);
      if (on && hasl(lo)) c = fmax(c, cl);
      if (on && hasu(hi)) c = fmax(c, cu);
    });
    return wmax(c);
  }

  // filter
  __device__ __forceinline__ bool filter_ok(double phi, double th) const {
    STAMP0();
    bool ok = true;
    for (int e = lanef(); e < nfilt; e += WAVE) {
      if (!(phi <= filt[2 * e] || th <= filt[2 * e + 1])) ok = false;
    }
    const bool r = !wany(!ok);
    STAMP1(PH_FILT);
    return r;
  }
  __device__ __forceinline__ void filter_add(double phi, double th) {
    // drop entries dominated by the new one, then append (IpFilter::AddEntry);
    // lane-parallel: every lane reads its entries, kept ones are compacted with
    // ballot + mbcnt, so the update costs one global round trip, not nfilt
    constexpr int FCH = (FCAP + WAVE - 1) / WAVE;
    double fp[FCH], ft[FCH];
    bool keep[FCH];
#pragma unroll
    for (int c = 0; c < FCH; ++c) {
      const int e = lanef() + c * WAVE;
      const bool valid = e < nfilt;
      fp[c] = valid ? filt[2 * e] : 0.0;
      ft[c] = valid ? filt[2 * e + 1] : 0.0;
      keep[c] = valid && !(fp[c] >= phi && ft[c] >= th);
    }
    sync();
    int w = 0;
#pragma unroll
    for (int c = 0; c < FCH; ++c) {
      const unsigned long long mask = __ballot(keep[c]);
      const int pos = w + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
      if (keep[c]) { filt[2 * pos] = fp[c]; filt[2 * pos + 1] = ft[c]; }
      w += __popcll(mask);
    }
    sync();
    if (w >= FCAP) {  // capacity guard: drop the oldest entry (never reached with max_iter <= FCAP)
      if (lanef() == 0) {
        for (int e = 1; e < w; ++e) { filt[2 * e - 2] = filt[2 * e]; filt[2 * e - 1] = filt[2 * e + 1]; }
      }
      --w;
      sync();
    }
    if (lanef() == 0) { filt[2 * w] = phi; filt[2 * w + 1] = th; }
    sync();
    nfilt = w + 1;
  }

  // trial point u = U + a dUs, s = s + a dss: rollout into Xt, rows into dt.
  // returns false on an evaluation error (NaN/Inf)
  __device__ __forceinline__ bool trial(double a, const GLB double* dUs, const RV* dss, double& ft, double& phit,
                        double& tht) {
    // the trial controls and their barrier terms in one pass
    const UPre up = preload_u(U, dUs, WAVE - 1);
    double th = 0.0, damp = 0.0;
    LogAcc logs;
    ctrls([&](int i, bool on) {
      const double ui = U[i] + a * dUs[i];
      if (on) Ut[i] = ui;
      barrier_ctrl1(i, on, ui, logs, damp);
    });
    sync();
    rollout(U, Xt, dUs, a, &up);
    ft = df * eval_fg(Xt, dt, dc);
    // theta and the barrier sums in one pass over the rows
    bool bad = false;
    rows([&](int r, bool on) {
      const double sv = s[r] + a * dss[r], dtr = dt[r];
      barrier_row(r, on, sv, logs, damp);
      if (on) {
        th += fabs(dtr - sv);
        if (!isfinite(dtr)) bad = true;
      }
    });
    tht = wsum(th);
    bad = wany(bad) || !isfinite(ft);
    if (bad) return false;
    phit = barrier_fin(ft, logs, damp);
    return isfinite(phit);
  }
};

// ------------------------------------------------------------------ kernel
// Feasibility restoration phase (BacktrackingLineSearch -> RestoMinC_1Nrm; oracle
// restoration()).  Runs between passes of the main iteration loop (which breaks
// out to it), so none of the main loop's temporaries are live here.  It rebuilds
// its own view of the scenario's workspace and exchanges only scalars.
struct RestoIO {
  double mu0, tau0, theta0, phi0, f, df;
  int nfilt, nzx, nzs, it, status;
  double* trace;
};

template <class CAP>
__device__ __forceinline__ void resto_phase(const Params* __restrict__ prm, double* ws, int b, RestoIO& io) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  Solver<CAP> S;
  S.bind(prm, smem, ws, threadIdx.x, b);
  S.nfix = (int)S.rvars[46];
  if constexpr (CAP::eq) S.meq = __builtin_amdgcn_readfirstlane((int)S.rvars[47]);
  S.df = io.df; S.nfilt = io.nfilt; S.nzx = io.nzx; S.nzs = io.nzs; S.delta = 0.0;
  S.mu = io.mu0; S.tau = io.tau0;
  const nmpc_options& o = prm->o;
  const int N = S.N, nw = S.nw, ng = S.ng, m = S.m;
  const int max_iter = o.max_iter;
  const double smax = o.s_max;
  double* trace = io.trace;
  int it = io.it;
  const double eps = 2.220446049250313e-16;
  // loop-carried scalars live in LDS (volatile: one LDS access per use) rather than in
  // registers across the Riccati / rollout calls: restoration is rare, registers are not
  volatile LDS double* V = S.rvars;
  auto cmp_le = [&](double lhs, double rhs, double bas) { return lhs - rhs <= 10.0 * eps * fabs(bas); };
  (void)N;
      V[0] = io.mu0; V[1] = io.tau0; V[2] = io.theta0; V[3] = io.phi0;
      const double rho = o.resto_penalty_parameter;
      const double kd = o.kappa_d, ks = o.kappa_sigma;
      S.rho = rho;
      // x_R and the original multipliers; initial mu, p, n and capped multipliers
      double cmax = 0.0;
      for (int i = S.lanef(); i < nw; i += WAVE) {
        S.UR[i] = S.U[i]; S.zl0[i] = S.zl[i]; S.zu0[i] = S.zu[i];
      }
      for (int r = S.lanef(); r < ng; r += WAVE) {
        S.s0[r] = S.s[r]; S.vl0[r] = S.vl[r]; S.vu0[r] = S.vu[r];
        cmax = fmax(cmax, fabs(S.d[r] - S.s[r]));
      }
      V[4] = fmax(V[0], wmax(cmax));
      V[5] = fmax(o.tau_min, 1.0 - V[4]);
      S.mu = V[4];
      S.etaR = o.resto_proximity_weight * sqrt(V[4]);
      for (int r = S.lanef(); r < ng; r += WAVE) {
        const double c = S.d[r] - S.s[r];
        const double qa = V[4] / (2.0 * rho) - 0.5 * c, qb = c * V[4] / (2.0 * rho);
        const double nv = qa + sqrt(qa * qa + qb), pv = c + nv;
        S.pR[r] = pv; S.nR[r] = nv; S.zpR[r] = V[4] / pv; S.znR[r] = V[4] / nv;
        S.vl[r] = S.hasl(S.dl[r]) ? fmin(rho, S.vl[r]) : 0.0;
        S.vu[r] = S.hasu(S.du[r]) ? fmin(rho, S.vu[r]) : 0.0;
      }
      for (int i = S.lanef(); i < nw; i += WAVE) {
        S.zl[i] = S.hasl(S.xl[i]) ? fmin(rho, S.zl[i]) : 0.0;
        S.zu[i] = S.hasu(S.xu[i]) ? fmin(rho, S.zu[i]) : 0.0;
      }
      sync();
      // least-squares multipliers of the restoration NLP
      {
        bool zero = true;
        if (o.constr_mult_init_max > 0 && ng > 0) {
          for (int i = S.lanef(); i < nw; i += WAVE) { S.sigx[i] = 1.0; S.ru[i] = S.zl[i] - S.zu[i]; }
          S.delta = 0.0;
          S.assemble(SUM_LS_RESTO, 0.0, 0.0, false);
          S.riccati(S.sigx, S.ru);
          S.forward(S.dU, S.dX);
          S.refine(S.sigx, S.ru, S.dU, S.dX);
          double ymax = 0.0;
          for (int r = S.lanef(); r < ng; r += WAVE) {
            const int k = r / m, i = r - k * m;
            const LDS double* xk = S.X + k * 8;
            const LDS double* dxk = S.dX + k * 8;
            double jd;
            if (i < S.nb) jd = S.dc[r] * dxk[boxidx(i)];
            else {
              const int q = i - S.nb;
              const double ddx = xk[0] - S.obx[q], ddy = xk[1] - S.oby[q];
              const double dd = sqrt(ddx * ddx + ddy * ddy);
              jd = S.dc[r] * ((-(ddx / dd)) * dxk[0] + (-(ddy / dd)) * dxk[1]);
            }
            const double yv = S.eqr(r) ? ((rho - S.zpR[r]) - (rho - S.znR[r]) - jd) / 2.0
                                               : ((S.vu[r] - S.vl[r]) + (rho - S.zpR[r]) - (rho - S.znR[r]) - jd) / 3.0;
            S.y[r] = yv;
            ymax = fmax(ymax, fabs(yv));
          }
          ymax = wmax(ymax);
          sync();
          zero = !(ymax <= o.constr_mult_init_max);
        }
        if (zero) {
          for (int r = S.lanef(); r < ng; r += WAVE) S.y[r] = 0.0;
          sync();
        }
      }
      // the restoration problem's own filter
      GLB double* ofilt = S.filt;
      const int onf = S.nfilt;
      S.filt = S.filtR;
      S.nfilt = 0;
      V[6] = -1.0; V[7] = -1.0; V[8] = 0.0; V[9] = 0.0;
      bool firstR = true;
      int raccc = 0, rlast_it = -1;
      V[10] = -1e50; V[11] = -1e50;
      V[12] = io.f;            // original (scaled) objective at the restoration iterate
      int rstat = 1;        // 1 running, 0 back to the original problem, else final status
      // the restoration phase's own watchdog procedure (its line search is a
      // BacktrackingLineSearch with the same defaults); it reuses the main loop's watchdog
      // storage, which is idle while restoration runs
      int rwd_cnt = 0, rwd_trial = 0;
      bool rin_wd = false;
      int tcb_last = -1;  // the cache buffer of the current iterate's trial (-1: none, the entry point)
      volatile LDS double* WD = S.rvars + 40;
      auto lanef = [&]() { return S.lanef(); };  // for the STAMP macros
      (void)lanef;
      LDS double* stamps = S.stamps;
      (void)stamps;
      while (true) {
        STAMP0();
        XSTAMP0(_xit);
        XCOUNT(X_ICNT);
        XSTAMP0(_xcv);
        // after the first restoration iteration rvars[32..36] hold the sums of the
        // accepted trial, i.e. of the current iterate (p, n, s, U updated bit for bit)
        const bool cachedR = !firstR;
        // ---- progress w.r.t. the original problem (RestoConvergenceCheck)
        if (!firstR) {
          // sum |d - s| of the current iterate: formed by the accept pass that produced it
          // (the same rows in the same per-lane order, so the same bits)
          const double tho = V[22];
          S.mu = V[0];
          const double pho = S.phi_of(V[12], S.rvars[32], S.rvars[33]);
          S.mu = V[4];
          if (tho <= o.required_infeasibility_reduction * V[2] && isfinite(pho)) {
            const bool ok = cmp_le(tho, (1.0 - o.gamma_theta) * V[2], V[2]) ||
                            cmp_le(pho - V[3], -o.gamma_phi * V[2], V[3]);
            if (ok) {
              GLB double* rf = S.filt;
              const int rn_ = S.nfilt;
              S.filt = ofilt; S.nfilt = onf;
              const bool fok = S.filter_ok(pho, tho);
              S.filt = rf; S.nfilt = rn_;
              if (fok) { rstat = 0; break; }
            }
          }
        }
        // ---- the restoration NLP's own optimality error / termination
        S.adjoint(0.0, S.y);
        double dinf = 0, cv = 0, cmr = 0, ucv = 0, sumy = 0, sumz = 0, sumv = 0, sump = 0, frp = 0, frx = 0;
        // the barrier error at the current mu (first sub_errR of the mu update below)
        // from the same pass: its dual part is dinf (etaR = weight * sqrt(V[4]))
        double cmu = 0, pinfu = 0;
        const double muc = V[4];
        bool bad = false;
        S.ctrls([&](int i, bool on) {  // (maxima and flags ignore the repeated last entry)
          const double dd = S.U[i] - S.UR[i];
          const double g = S.fixed(i) ? 0.0 : S.grad_u(i) + S.etaR * S.dr2(i) * dd - S.zl[i] + S.zu[i];
          if (!isfinite(g)) bad = true;
          dinf = fmax(dinf, fabs(g));
          if (S.hasl(S.xl[i])) cmr = fmax(cmr, fabs((S.U[i] - S.xl[i]) * S.zl[i]));
          if (S.hasu(S.xu[i])) cmr = fmax(cmr, fabs((S.xu[i] - S.U[i]) * S.zu[i]));
          if (S.hasl(S.xl[i])) cmu = fmax(cmu, fabs((S.U[i] - S.xl[i]) * S.zl[i] - muc));
          if (S.hasu(S.xu[i])) cmu = fmax(cmu, fabs((S.xu[i] - S.U[i]) * S.zu[i] - muc));
          const double sz = fabs(S.zl[i]) + fabs(S.zu[i]), fx = S.dr2(i) * dd * dd;
          if (on) { sumz += sz; frx += fx; }
        });
        S.rows_r([&](int r, bool on) {
          const double yr = S.y[r], pr = S.pR[r], nr = S.nR[r], vlr = S.vl[r], vur = S.vu[r];
          const double zp = S.zpR[r], zn = S.znR[r], dr = S.d[r], sr = S.s[r], dcr = S.dc[r];
          const double lo = S.dl[r], hi = S.du[r];
          const bool hl = S.hasl(lo), hu = S.hasu(hi);
          const bool eq = S.eqlo(lo);
          const double di = fmax(eq ? 0.0 : fabs(-yr - vlr + vur), fmax(fabs(rho - yr - zp), fabs(rho + yr - zn)));
          const double drr = dr - pr + nr;
          double c1 = eq ? fabs(drr - sr) : 0.0, c2 = eq ? fabs(dr - sr) : 0.0;
          if (hl) { c1 = fmax(c1, lo - drr); c2 = fmax(c2, lo - dr); }
          if (hu) { c1 = fmax(c1, drr - hi); c2 = fmax(c2, dr - hi); }
          const double cl = fabs((sr - lo) * vlr), cu = fabs((hi - sr) * vur), uc = c2 / dcr;
          const double clm = fabs((sr - lo) * vlr - muc), cum = fabs((hi - sr) * vur - muc);
          const double cpm = fmax(fabs(pr * zp - muc), fabs(nr * zn - muc));
          const double pim = fabs(dr - sr - pr + nr);
          if (on) {  // max reductions are order-free; sums keep the per-lane row order
            if (hl) cmu = fmax(cmu, clm);
            if (hu) cmu = fmax(cmu, cum);
            cmu = fmax(cmu, cpm);
            pinfu = fmax(pinfu, pim);
            dinf = fmax(dinf, di);
            if (hl) cmr = fmax(cmr, cl);
            if (hu) cmr = fmax(cmr, cu);
            cmr = fmax(cmr, fmax(fabs(pr * zp), fabs(nr * zn)));
            cv = fmax(cv, c1);
            ucv = fmax(ucv, uc);
            sumy += fabs(yr);
            sumv += fabs(vlr) + fabs(vur);
            sump += fabs(zp) + fabs(zn);
            frp += pr + nr;
            if (!isfinite(dr)) bad = true;
          }
        });
        dinf = wmax(dinf); cv = wmax(cv); cmr = wmax(cmr); ucv = wmax(ucv);
        sumy = wsum(sumy); sumz = wsum(sumz); sumv = wsum(sumv); sump = wsum(sump);
        frp = wsum(frp); frx = wsum(frx);
        const int ndR = ng + S.nzx + S.nzs + 2 * ng, ncR = S.nzx + S.nzs + 2 * ng;
        V[13] = fmax(smax, (sumy + sumz + sumv + sump) / ndR) / smax;
        V[14] = fmax(smax, (sumz + sumv + sump) / ncR) / smax;
        const double errR = fmax(fmax(dinf / V[13], cv), cmr / V[14]);
        if (trace && S.lanef() == 0) {  // the restoration NLP's convergence check at `it` (parity
          double* t = trace + (long long)it * TRACE_F;  // diagnostics; negative error: a restoration check)
          t[8] = -errR; t[9] = dinf / V[13]; t[10] = cv; t[11] = cmr / V[14];
        }
        if (wany(bad) || !isfinite(errR)) { rstat = ST_INVALID_NUMBER; break; }
        const bool conv = errR <= o.tol && dinf <= o.dual_inf_tol && cv <= o.constr_viol_tol && cmr <= o.compl_inf_tol;
        if (it != rlast_it) { V[10] = V[11]; V[11] = rho * frp + 0.5 * S.etaR * frx; rlast_it = it; }
        const bool racc = errR <= o.acceptable_tol && dinf <= o.acceptable_dual_inf_tol &&
                          cv <= o.acceptable_constr_viol_tol && cmr <= o.acceptable_compl_inf_tol &&
                          fabs(V[11] - V[10]) / fmax(1.0, fabs(V[11])) <= o.acceptable_obj_change_tol;
        if (o.acceptable_iter > 0 && racc) ++raccc; else raccc = 0;
        if (conv || (o.acceptable_iter > 0 && raccc >= o.acceptable_iter)) {
          rstat = (ucv > o.constr_viol_tol) ? ST_INFEASIBLE : 0;
          break;
        }
        if (it >= max_iter) { rstat = ST_MAXITER; break; }
        firstR = false;
        // ---- monotone barrier update of the restoration problem
        {
          // barrier error at a candidate mu (the proximity weight eta depends on mu)
          auto sub_errR = [&](double mu_) {
            const double et = o.resto_proximity_weight * sqrt(mu_);
            double dn = 0.0, cm = 0.0, pinf = 0.0;
            S.ctrls([&](int i, bool) {  // (maxima ignore the repeated last entry)
              const double g =
                  S.fixed(i) ? 0.0 : S.grad_u(i) + et * S.dr2(i) * (S.U[i] - S.UR[i]) - S.zl[i] + S.zu[i];
              dn = fmax(dn, fabs(g));
              if (S.hasl(S.xl[i])) cm = fmax(cm, fabs((S.U[i] - S.xl[i]) * S.zl[i] - mu_));
              if (S.hasu(S.xu[i])) cm = fmax(cm, fabs((S.xu[i] - S.U[i]) * S.zu[i] - mu_));
            });
            S.rows_r([&](int r, bool on) {
              const double yr = S.y[r], vlr = S.vl[r], vur = S.vu[r], zp = S.zpR[r], zn = S.znR[r];
              const double sr = S.s[r], dr = S.d[r], pr = S.pR[r], nr = S.nR[r], lo = S.dl[r], hi = S.du[r];
              const double dv = fmax(S.eqlo(lo) ? 0.0 : fabs(-yr - vlr + vur), fmax(fabs(rho - yr - zp), fabs(rho + yr - zn)));
              const double cl = fabs((sr - lo) * vlr - mu_), cu = fabs((hi - sr) * vur - mu_);
              const double cp = fmax(fabs(pr * zp - mu_), fabs(nr * zn - mu_));
              const double pi = fabs(dr - sr - pr + nr);
              if (on) {
                dn = fmax(dn, dv);
                if (S.hasl(lo)) cm = fmax(cm, cl);
                if (S.hasu(hi)) cm = fmax(cm, cu);
                cm = fmax(cm, cp);
                pinf = fmax(pinf, pi);
              }
            });
            return fmax(fmax(wmax(dn) / V[13], wmax(pinf)), wmax(cm) / V[14]);
          };
          double se = fmax(fmax(dinf / V[13], wmax(pinfu)), wmax(cmu) / V[14]);  // = sub_errR(V[4])
          bool done = false;
          while (se <= o.barrier_tol_factor * V[4] && !done) {
            double nmu = fmin(o.kappa_mu * V[4], pow(V[4], o.theta_mu));
            nmu = fmax(nmu, fmin(o.tol, o.compl_inf_tol) / (o.barrier_tol_factor + 1.0));
            const bool changed = nmu != V[4];
            V[4] = nmu;
            V[5] = fmax(o.tau_min, 1.0 - V[4]);
            if (!changed) done = true;
            else {
              se = sub_errR(V[4]);
              done = se > o.barrier_tol_factor * V[4];
            }
            if (done && changed) S.nfilt = 0;
          }
          S.mu = V[4];
          S.etaR = o.resto_proximity_weight * sqrt(V[4]);
        }
        STAMP1(PH_CONV);
        XSTAMP1(_xcv, X_CONV);
        // ---- Newton step of the restoration problem (p, n eliminated per row)
        { STAMP0();
        const double muR4 = V[4];  // volatile LDS scalar read once
        S.ctrls([&](int i, bool on) {
          const bool hl = S.hasl(S.xl[i]), hu = S.hasu(S.xu[i]);
          const double Sl = hl ? S.U[i] - S.xl[i] : 1.0, Su = hu ? S.xu[i] - S.U[i] : 1.0;
          const double w2 = S.etaR * S.dr2(i);
          const double sg = w2 + ((hl ? qd(S.zl[i], Sl) : 0.0) + (hu ? qd(S.zu[i], Su) : 0.0));
          const double rr = w2 * (S.U[i] - S.UR[i]) + (-(hl ? qd(muR4, Sl) : 0.0) + (hu ? qd(muR4, Su) : 0.0) +
                            kd * muR4 * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0)));
          if (on) { S.sigx[i] = sg; S.ru[i] = rr; }
        });
        sync();
        STAMP1(PH_SIGX); }
        if (V[9] > 0) V[8] = V[9];
        double dR = 0.0;
        bool fok = false;
        while (true) {
          S.delta = dR;
          XSTAMP0(_xa);
          S.assemble(SUM_RESTO, 0.0, 0.0, true);
          XSTAMP1(_xa, X_NASM);
          XSTAMP0(_xr);
          const bool fact = S.riccati(S.sigx, S.ru);
          XSTAMP1(_xr, X_NRIC);
          if (fact) { fok = true; break; }
          sync();
          if (dR == 0.0) dR = (V[8] == 0.0) ? o.first_hessian_perturbation
                                              : fmax(o.min_hessian_perturbation, V[8] * o.perturb_dec_fact);
          else if (V[8] == 0.0 || 1e5 * V[8] < dR) dR *= o.perturb_inc_fact_first;
          else dR *= o.perturb_inc_fact;
          if (dR > o.max_hessian_perturbation) break;
        }
        V[9] = dR;
        S.delta = dR;
        if (!fok) { rstat = ST_STEP_ERR; break; }
        XSTAMP0(_xnf);
        S.forward(S.dU, S.dX);
        S.refine(S.sigx, S.ru, S.dU, S.dX);
        // primal / dual fraction to the boundary of the Newton step, formed with its row pass
        // (valid until the watchdog restores another iterate and step)
        double rftb_p = 1.0, rftb_d = 1.0;
        bool rftb_ok = true;
        {
          STAMP0();
          double th, g, ap, ad;
          const double tauR = V[5];
          S.row_step_resto(S.dX, false, S.ds, S.dpR, S.dnR, S.dyR, th, g, tauR, ap, ad);
          S.ctrls([&](int i, bool on) {
            const double du_ = S.dU[i];
            const double gi = S.ru[i] * du_;
            if (on) g += gi;
            const double ui = S.U[i], xli = S.xl[i], xui = S.xu[i];
            if (S.hasl(xli) && du_ < 0) ap = fmin(ap, qd(-tauR * (ui - xli), du_));
            if (S.hasu(xui) && -du_ < 0) ap = fmin(ap, qd(-tauR * (xui - ui), -du_));
            double a1, a2;
            S.dz_x(i, du_, a1, a2);
            if (S.hasl(xli) && a1 < 0) ad = fmin(ad, qd(-tauR * S.zl[i], a1));
            if (S.hasu(xui) && a2 < 0) ad = fmin(ad, qd(-tauR * S.zu[i], a2));
          });
          V[15] = wsum(th);
          V[16] = wsum(g);
          rftb_p = wmin(ap);
          rftb_d = wmin(ad);
          STAMP1(PH_ROWSTEP);
        }
        XSTAMP1(_xnf, X_NFIN);
        V[17] = cachedR ? S.phi_of(0.0, S.rvars[32], S.rvars[33]) + S.pn_of(S.rvars[34], S.rvars[35], S.rvars[36])
                        : S.barrier_obj(0.0, S.U, S.s, nullptr, 0.0) + S.resto_pn_terms(S.U, 0.0, nullptr, nullptr);
        if (V[6] < 0) {
          V[6] = o.theta_max_fact * fmax(1.0, V[15]);
          V[7] = o.theta_min_fact * fmax(1.0, V[15]);
        }
        // the switching condition's powers of the reference values V[15], V[16], formed once
        // when first needed (V[23]: valid flag, reset wherever V[15] / V[16] change; the main
        // phase's twin, PW, uses the same slots -- the two phases never overlap)
        V[23] = 0.0;
        auto r_pw = [&]() {
          if (V[23] == 0.0) {
            V[37] = V[16] < 0.0 ? pow(-V[16], o.s_phi) : 0.0;
            V[38] = pow(V[15], o.s_theta);
            V[23] = 1.0;
          }
        };
        auto r_ftype = [&](double a) {
          if (!(V[16] < 0.0)) return false;
          r_pw();
          return a * V[37] > o.delta * V[38];
        };
        auto r_armijo = [&](double a, double ph) { return cmp_le(ph - V[17], o.eta_phi * a * V[16], V[17]); };
        auto r_check = [&](double a_test, double ph, double th) {
          if (th > V[6]) return false;
          bool ok;
          if (a_test > 0.0 && r_ftype(a_test) && V[15] <= V[7]) ok = r_armijo(a_test, ph);
          else {
            ok = true;
            if (ph > V[17]) {
              double basval = 1.0;
              if (fabs(V[17]) > 10.0) basval = log10(fabs(V[17]));
              if (log10(ph - V[17]) > o.obj_max_inc + basval) ok = false;
            }
            ok = ok && (cmp_le(th, (1.0 - o.gamma_theta) * V[15], V[15]) ||
                        cmp_le(ph - V[17], -o.gamma_phi * V[15], V[17]));
          }
          return ok && S.filter_ok(ph, th);
        };
        // ---- watchdog (see the main loop): start, or judge against the stored reference
        bool rwd_dir = false;  // the step is the stored one: its dual components use WD[4]
        if (o.watchdog_shortened_iter_trigger > 0 && !rin_wd && rwd_cnt >= o.watchdog_shortened_iter_trigger) {
          for (int i = S.lanef(); i < nw; i += WAVE) {
            S.wU[i] = S.U[i]; S.wzl[i] = S.zl[i]; S.wzu[i] = S.zu[i]; S.wdU[i] = S.dU[i];
          }
          for (int r = S.lanef(); r < ng; r += WAVE) {
            S.wsl[r] = S.s[r]; S.wy[r] = S.y[r]; S.wvl[r] = S.vl[r]; S.wvu[r] = S.vu[r]; S.wds[r] = S.ds[r];
            S.wpR[r] = S.pR[r]; S.wnR[r] = S.nR[r]; S.wzpR[r] = S.zpR[r]; S.wznR[r] = S.znR[r];
            S.wdpR[r] = S.dpR[r]; S.wdnR[r] = S.dnR[r]; S.wdyR[r] = S.dyR[r];
          }
          const double at = rftb_ok ? rftb_p : S.frac_to_bound_resto(V[5], S.dU, S.ds, S.dpR, S.dnR);
          WD[0] = V[15]; WD[1] = V[16]; WD[2] = V[17]; WD[3] = at; WD[4] = V[4]; WD[5] = S.delta;
          sync();
          rin_wd = true;
          rwd_trial = 0;
        }
        if (rin_wd) { V[15] = WD[0]; V[16] = WD[1]; V[17] = WD[2]; V[23] = 0.0; }
        auto rwd_restore = [&]() {  // StopWatchDog
          for (int i = S.lanef(); i < nw; i += WAVE) {
            S.U[i] = S.wU[i]; S.zl[i] = S.wzl[i]; S.zu[i] = S.wzu[i]; S.dU[i] = S.wdU[i];
          }
          for (int r = S.lanef(); r < ng; r += WAVE) {
            S.s[r] = S.wsl[r]; S.y[r] = S.wy[r]; S.vl[r] = S.wvl[r]; S.vu[r] = S.wvu[r]; S.ds[r] = S.wds[r];
            S.pR[r] = S.wpR[r]; S.nR[r] = S.wnR[r]; S.zpR[r] = S.wzpR[r]; S.znR[r] = S.wznR[r];
            S.dpR[r] = S.wdpR[r]; S.dnR[r] = S.wdnR[r]; S.dyR[r] = S.wdyR[r];
          }
          sync();
          S.rollout(S.U, S.X);
          V[12] = S.df * S.eval_fg(S.X, S.d, S.dc);
          S.template derivs<false, true>(S.X, S.U, S.tc);
          V[15] = WD[0]; V[16] = WD[1]; V[17] = WD[2]; V[23] = 0.0;
          S.delta = WD[5];
          rwd_dir = true;
          rftb_ok = false;
          rin_wd = false;
          rwd_cnt = 0;
        };
        STAMPV0(_tls);
        XSTAMP0(_xls);
        V[19] = 0.0; V[20] = 0.0; V[21] = 0.0;
        int acc = 0, nsteps = 0;  // acc: 1 regular step, 2 SOC step
        int tcb_acc = 0;  // the transcendental-cache buffer of the accepted trial (1: a pair's second)
        double a = 0.0, a_test = 0.0;
        bool rskip = false, rforced = false;
       while (true) {
        V[18] = rftb_ok ? rftb_p : S.frac_to_bound_resto(V[5], S.dU, S.ds, S.dpR, S.dnR);
        if (rin_wd) {
          double fo_t, ph, th;
          const bool ok_t = S.trial_resto(V[18], S.dU, S.ds, S.dpR, S.dnR, fo_t, ph, th);
          const double at = WD[3];
          if (ok_t && r_check(at, ph, th)) {
            acc = 1; V[19] = V[18]; V[20] = fo_t; V[21] = ph; a_test = at; rin_wd = false;
            break;
          }
          if (!ok_t || ++rwd_trial > o.watchdog_trial_iter_max) { rwd_restore(); rskip = true; continue; }
          acc = 1; V[19] = V[18]; V[20] = fo_t; V[21] = ph; rforced = true;
          break;
        }
        double amin = o.gamma_theta;
        if (V[16] < 0) {
          amin = fmin(o.gamma_theta, o.gamma_phi * V[15] / (-V[16]));
          if (V[15] <= V[7]) {
            r_pw();
            amin = fmin(amin, o.delta * V[38] / V[37]);
          }
        }
        amin *= o.alpha_min_frac;
        a = rskip ? V[18] * o.alpha_red_factor : V[18];
        nsteps = 0;
        // speculative pairs (Solver::kSpec): each trial not formed yet is formed together
        // with the next backtracking trial (spec_a), whose X / rows wait in lam / dms
        double spec_a = -1.0, spec_f = 0.0;
        // (Params::nospec, a diagnostic: every trial formed alone -- the reference run of the
        // bitwise test of the pairs, test_speculative_restoration_pairs_are_bitwise_neutral)
        const bool spec_on = Solver<CAP>::kSpec && !prm->nospec;
        while (a > amin || nsteps == 0) {
          double fo_t, ph, th;
          bool ok_t;
          const bool from_pair = Solver<CAP>::kSpec && a == spec_a;
          if (from_pair) {
            ok_t = S.trial_resto(a, S.dU, S.ds, S.dpR, S.dnR, fo_t, ph, th, 2, 0.0, &spec_f);
            spec_a = -1.0;
          } else {
            const double an = a * o.alpha_red_factor;
            ok_t = S.trial_resto(a, S.dU, S.ds, S.dpR, S.dnR, fo_t, ph, th, spec_on ? 1 : 0, an, &spec_f);
            spec_a = spec_on ? an : -1.0;
          }
          if (ok_t && r_check(a, ph, th)) {
            acc = 1; V[19] = a; V[20] = fo_t; V[21] = ph; a_test = a;
            tcb_acc = from_pair ? 1 : 0;
            if (from_pair) {  // the accepted trial's X and rows into Xt / dt for the accept
              if (S.lanef() <= N) {
#pragma unroll
                for (int c = 0; c < 8; ++c) S.Xt[S.lanef() * 8 + c] = S.lam[S.lanef() * 8 + c];
              }
              S.rows([&](int r, bool on) {
                const double v = S.dms[r];
                if (on) S.dt[r] = v;
              });
              sync();
            }
            break;
          }
          if (ok_t && a == V[18] && V[15] <= th && o.max_soc > 0) {
            RSTAMP0(_soc);
            XSTAMP0(_xsb);
            double th_tr = th, th_old = 0.0, a_soc = a;
            for (int r = S.lanef(); r < ng; r += WAVE) S.cms[r] = S.d[r] - S.s[r] - S.pR[r] + S.nR[r];
            sync();
            const auto* dsp = S.ds;
            const GLB double *dpp = S.dpR, *dnp = S.dnR;
            int cnt = 0;
            bool soc_ok = false;
            while (cnt < o.max_soc && (cnt == 0 || th_tr <= o.kappa_soc * th_old)) {
              th_old = th_tr;
              XSTAMP0(_xs1);
              for (int r = S.lanef(); r < ng; r += WAVE) {
                const double sv = S.s[r] + a_soc * dsp[r], pv = S.pR[r] + a_soc * dpp[r], nv = S.nR[r] + a_soc * dnp[r];
                S.cms[r] = a_soc * S.cms[r] + (S.dt[r] - sv - pv + nv);
              }
              sync();
              XSTAMP1(_xs1, X_SCMS);
              XSTAMP0(_xs2);
              S.assemble(SUM_RESTO_SOC, 0.0, 0.0, true);
              XSTAMP1(_xs2, X_SASM);
              XSTAMP0(_xs3);
              S.resolve(S.ru);
              XSTAMP1(_xs3, X_SRES);
              XSTAMP0(_xs4);
              S.forward(S.dU2, S.dX);
              S.refine(S.sigx, S.ru, S.dU2, S.dX);
              XSTAMP1(_xs4, X_SFWD);
              double t0, t1;
              double ap, u1;
              const double tauR = V[5];
              S.row_step_resto(S.dX, true, S.ds2, S.dp2R, S.dn2R, S.dy2R, t0, t1, tauR, ap, u1);
              S.ctrls([&](int i, bool) {  // frac_to_bound_resto's control part
                const double du_ = S.dU2[i], ui = S.U[i], xli = S.xl[i], xui = S.xu[i];
                if (S.hasl(xli) && du_ < 0) ap = fmin(ap, qd(-tauR * (ui - xli), du_));
                if (S.hasu(xui) && -du_ < 0) ap = fmin(ap, qd(-tauR * (xui - ui), -du_));
              });
              a_soc = wmin(ap);
              dsp = S.ds2; dpp = S.dp2R; dnp = S.dn2R;
              double fo2, ph2, th2;
              if (!S.trial_resto(a_soc, S.dU2, S.ds2, S.dp2R, S.dn2R, fo2, ph2, th2)) break;
              if (r_check(a, ph2, th2)) {
                acc = 2; V[19] = a_soc; V[20] = fo2; V[21] = ph2; a_test = a; soc_ok = true;
                break;
              }
              ++cnt;
              th_tr = th2;
            }
            RSTAMP1(_soc, PH_FTB);
            XSTAMP1(_xsb, X_SBLK);
            if (soc_ok) break;
          }
          a *= o.alpha_red_factor;
          ++nsteps;
        }
        break;
       }
        STAMPV1(_tls, PH_INIT);
        XSTAMP1(_xls, X_LS);
        if (acc == 0) { rstat = ST_RESTO_FAIL; break; }  // no restoration inside the restoration phase
        // the accepted trial's original objective (the line search judged its trials by phi_R,
        // which does not contain it): its X is in Xt on every path, its transcendental values
        // go to its cache buffer, where the rollout put its cos / sin
        V[20] = S.df * S.eval_f(S.Xt, S.tc + tcb_acc * Solver<CAP>::TCS);
        rwd_cnt = (nsteps == 0) ? 0 : rwd_cnt + 1;
        // filter augmentation (F-type + Armijo steps do not augment)
        {
          STAMP0();
          XSTAMP0(_xac);
          const GLB double* dUa = (acc == 2) ? S.dU2 : S.dU;
          const auto* dsa = (acc == 2) ? S.ds2 : S.ds;
          const GLB double* dpa = (acc == 2) ? S.dp2R : S.dpR;
          const GLB double* dna = (acc == 2) ? S.dn2R : S.dnR;
          const GLB double* dya = (acc == 2) ? S.dy2R : S.dyR;
          if (!rforced && !(r_ftype(a_test) && r_armijo(a_test, V[21])))
            S.filter_add(V[17] - o.gamma_phi * V[15], (1.0 - o.gamma_theta) * V[15]);
          // ---- accept the restoration trial point (the step's dual components with its
          //      own mu, the kappa_sigma safeguard with the current one)
          if (rwd_dir) S.mu = WD[4];
          const double ad = (acc == 1 && rftb_ok && !rwd_dir) ? rftb_d
                                                               : S.dual_frac_to_bound_resto(V[5], dUa, dsa, dpa, dna);
          const double muA = V[4];  // volatile LDS scalar read once
          // (the accepted controls U <- Ut in the same pass: each lane reads its U[i] for the
          // dual step before it writes it)
          S.ctrls([&](int i, bool on) {
            double dzl, dzu;
            S.dz_x(i, dUa[i], dzl, dzu);
            double nzl = S.zl[i] + ad * dzl, nzu = S.zu[i] + ad * dzu;
            const double un = S.Ut[i];
            if (S.hasl(S.xl[i])) { const double Sn = un - S.xl[i]; nzl = fmax(fmin(nzl, qd(ks * muA, Sn)), qd(muA, ks * Sn)); }
            else nzl = 0.0;
            if (S.hasu(S.xu[i])) { const double Sn = S.xu[i] - un; nzu = fmax(fmin(nzu, qd(ks * muA, Sn)), qd(muA, ks * Sn)); }
            else nzu = 0.0;
            if (on) { S.zl[i] = nzl; S.zu[i] = nzu; S.U[i] = un; }
          });
          const double muR = V[4], aP = V[19];  // volatile LDS scalars read once
          const double dmuR = rwd_dir ? (double)WD[4] : muR;
          double tho = 0.0;  // theta of the original problem at the new iterate (next check)
          S.rows_r([&](int r, bool on) {
            const double sr = S.s[r], lo = S.dl[r], hi = S.du[r], vlr = S.vl[r], vur = S.vu[r];
            const double dsr = dsa[r], dpr = dpa[r], dnr = dna[r], dyr = dya[r];
            const double pr = S.pR[r], nr = S.nR[r], zp = S.zpR[r], zn = S.znR[r], yr = S.y[r], dtr = S.dt[r];
            const bool hl = S.hasl(lo), hu = S.hasu(hi);
            double dvl = 0.0, dvu = 0.0;  // dv_s with the loads hoisted
            if (hl) { const double iS = rcp(sr - lo); dvl = S.mu * iS - vlr - vlr * iS * dsr; }
            if (hu) { const double iS = rcp(hi - sr); dvu = S.mu * iS - vur + vur * iS * dsr; }
            const double dzp = qd(dmuR, pr) - zp - qd(zp, pr) * dpr;
            const double dzn = qd(dmuR, nr) - zn - qd(zn, nr) * dnr;
            const double sn = sr + aP * dsr;
            const double pn = pr + aP * dpr, nn = nr + aP * dnr;
            double nvl = vlr + ad * dvl, nvu = vur + ad * dvu;
            if (hl) { const double Sn = sn - lo; nvl = fmax(fmin(nvl, qd(ks * muR, Sn)), qd(muR, ks * Sn)); }
            else nvl = 0.0;
            if (hu) { const double Sn = hi - sn; nvu = fmax(fmin(nvu, qd(ks * muR, Sn)), qd(muR, ks * Sn)); }
            else nvu = 0.0;
            const double nzp = zp + ad * dzp, nzn = zn + ad * dzn;
            const double zpn = fmax(fmin(nzp, qd(ks * muR, pn)), qd(muR, ks * pn));
            const double znn = fmax(fmin(nzn, qd(ks * muR, nn)), qd(muR, ks * nn));
            const double t = fabs(dtr - sn);
            if (on) {
              S.zpR[r] = zpn; S.znR[r] = znn;
              S.y[r] = yr + aP * dyr;
              S.vl[r] = nvl; S.vu[r] = nvu;
              S.s[r] = sn; S.pR[r] = pn; S.nR[r] = nn;
              S.d[r] = dtr;
              tho += t;
            }
          });
          tho = wsum(tho);
          V[22] = tho;
          S.mu = V[4];
          if (S.lanef() <= N) {
#pragma unroll
            for (int c = 0; c < 8; ++c) S.X[S.lanef() * 8 + c] = S.Xt[S.lanef() * 8 + c];
          }
          sync();
          V[12] = V[20];
          STAMP1(PH_ACCEPT);
          XSTAMP1(_xac, X_ACC);
          XSTAMP0(_xde);
          S.template derivs<false, true>(S.X, S.U, S.tc + tcb_acc * Solver<CAP>::TCS);
          tcb_last = tcb_acc;
          XSTAMP1(_xde, X_DER);
          ++it;
          if (trace && S.lanef() == 0) {
            double th = 0.0;
            for (int r = 0; r < ng; ++r) th += fabs(S.d[r] - S.s[r] - S.pR[r] + S.nR[r]);
            double* t = trace + (long long)(it - 1) * TRACE_F;
            t[0] = it; t[1] = V[4]; t[2] = V[20]; t[3] = th; t[4] = V[9]; t[5] = V[19]; t[6] = ad;
            t[7] = -(double)(nsteps + 1);  // negative: a restoration iteration
          }
          sync();
        }
        XSTAMP1(_xit, X_IT);
      }
      S.filt = ofilt;
      S.nfilt = onf;
      S.mu = V[0];
      S.tau = V[1];
      io.status = rstat;
      io.it = it;
      if (rstat != 0) return;
      // back to the original problem: its objective's Hessian at the current iterate (the
      // restoration iterations formed the gradient only)
      if (tcb_last >= 0) S.template derivs<true, true>(S.X, S.U, S.tc + tcb_last * Solver<CAP>::TCS);
      else S.derivs(S.X, S.U);
      // ---- back to the original problem: bound multipliers by a Newton step for
      //      complementarity over the whole restoration (fraction to the boundary,
      //      reset to 1 above bound_mult_reset_threshold); y = 0 (constr_mult_reset_threshold)
      {
        double a = 1.0, zmax = 0.0;
        for (int i = S.lanef(); i < nw; i += WAVE) {
          if (S.hasl(S.xl[i])) {
            const double S0 = S.UR[i] - S.xl[i], S1 = S.U[i] - S.xl[i];
            const double dz = (V[0] - S.zl0[i] * (S1 - S0)) / S0 - S.zl0[i];
            if (dz < 0) a = fmin(a, (-V[1] * S.zl0[i]) / dz);
            S.ru[i] = dz;
          } else S.ru[i] = 0.0;
          if (S.hasu(S.xu[i])) {
            const double S0 = S.xu[i] - S.UR[i], S1 = S.xu[i] - S.U[i];
            const double dz = (V[0] - S.zu0[i] * (S1 - S0)) / S0 - S.zu0[i];
            if (dz < 0) a = fmin(a, (-V[1] * S.zu0[i]) / dz);
            S.sigx[i] = dz;
          } else S.sigx[i] = 0.0;
        }
        for (int r = S.lanef(); r < ng; r += WAVE) {
          if (S.hasl(S.dl[r])) {
            const double S0 = S.s0[r] - S.dl[r], S1 = S.s[r] - S.dl[r];
            const double dz = (V[0] - S.vl0[r] * (S1 - S0)) / S0 - S.vl0[r];
            if (dz < 0) a = fmin(a, (-V[1] * S.vl0[r]) / dz);
            S.dpR[r] = dz;
          } else S.dpR[r] = 0.0;
          if (S.hasu(S.du[r])) {
            const double S0 = S.du[r] - S.s0[r], S1 = S.du[r] - S.s[r];
            const double dz = (V[0] - S.vu0[r] * (S1 - S0)) / S0 - S.vu0[r];
            if (dz < 0) a = fmin(a, (-V[1] * S.vu0[r]) / dz);
            S.dnR[r] = dz;
          } else S.dnR[r] = 0.0;
        }
        a = wmin(a);
        sync();
        for (int i = S.lanef(); i < nw; i += WAVE) {
          S.zl[i] = S.zl0[i] + a * S.ru[i];
          S.zu[i] = S.zu0[i] + a * S.sigx[i];
          zmax = fmax(zmax, fmax(fabs(S.zl[i]), fabs(S.zu[i])));
        }
        for (int r = S.lanef(); r < ng; r += WAVE) {
          S.vl[r] = S.vl0[r] + a * S.dpR[r];
          S.vu[r] = S.vu0[r] + a * S.dnR[r];
          zmax = fmax(zmax, fmax(fabs(S.vl[r]), fabs(S.vu[r])));
          S.y[r] = 0.0;
        }
        zmax = wmax(zmax);
        sync();
        const bool reset = zmax > o.bound_mult_reset_threshold;
        // kappa_sigma safeguard of the accepted point (IpoptAlgorithm::AcceptTrialPoint)
        for (int i = S.lanef(); i < nw; i += WAVE) {
          double nzl = reset ? 1.0 : S.zl[i], nzu = reset ? 1.0 : S.zu[i];
          if (S.hasl(S.xl[i])) { const double Sn = S.U[i] - S.xl[i]; nzl = fmax(fmin(nzl, ks * V[0] / Sn), V[0] / (ks * Sn)); }
          else nzl = 0.0;
          if (S.hasu(S.xu[i])) { const double Sn = S.xu[i] - S.U[i]; nzu = fmax(fmin(nzu, ks * V[0] / Sn), V[0] / (ks * Sn)); }
          else nzu = 0.0;
          S.zl[i] = nzl; S.zu[i] = nzu;
        }
        for (int r = S.lanef(); r < ng; r += WAVE) {
          double nvl = reset ? 1.0 : S.vl[r], nvu = reset ? 1.0 : S.vu[r];
          if (S.hasl(S.dl[r])) { const double Sn = S.s[r] - S.dl[r]; nvl = fmax(fmin(nvl, ks * V[0] / Sn), V[0] / (ks * Sn)); }
          else nvl = 0.0;
          if (S.hasu(S.du[r])) { const double Sn = S.du[r] - S.s[r]; nvu = fmax(fmin(nvu, ks * V[0] / Sn), V[0] / (ks * Sn)); }
          else nvu = 0.0;
          S.vl[r] = nvl; S.vu[r] = nvu;
        }
        sync();
      }
      io.f = V[12];
      io.it = it;
}

// One scenario's solve (the whole IPOPT loop) by the calling wavefront.
template <class CAP>
__device__ __forceinline__ int solve_one(Solver<CAP>& S, const Params* __restrict__ prm, const IO& io, const int b) {
  auto lanef = [&]() { return S.lanef(); };  // for the STAMP macros
  (void)lanef;
  LDS double* stamps = S.stamps;
  if (S.lanef() < PH_COUNT) stamps[S.lanef()] = 0.0;
  const unsigned long long _tk0 = __builtin_amdgcn_s_memtime();
  (void)_tk0;
  const nmpc_options& o = prm->o;
  const int N = S.N, nw = S.nw, ng = S.ng, m = S.m;
  const int max_iter = o.max_iter;
  double* trace = io.trace ? io.trace + (long long)b * (max_iter + 3) * TRACE_F : nullptr;

  // ---------------- load scenario data
  for (int i = S.lanef(); i < prm->np; i += WAVE) {
    const int e = ext_p(prm, i);  // external p index (model embedding), -1: absent state = 0
    S.pp[i] = e >= 0 ? io.p[(long long)b * io.ld_p + e] : 0.0;
  }
  sync();
  if (S.lanef() < S.nobs) {
    S.obx[S.lanef()] = prm->oxp[S.lanef()] >= 0 ? S.pp[prm->oxp[S.lanef()]] : prm->ox[S.lanef()];
    S.oby[S.lanef()] = prm->oyp[S.lanef()] >= 0 ? S.pp[prm->oyp[S.lanef()]] : prm->oy[S.lanef()];
  }
  if (S.lanef() == 0) {  // cost weights (LDS scalar slots 30, 31)
    S.rvars[30] = prm->w1p >= 0 ? S.pp[prm->w1p] : prm->w1;
    S.rvars[31] = prm->w2p >= 0 ? S.pp[prm->w2p] : prm->w2;
  }
  const double brf = o.bound_relax_factor, cvt = o.constr_viol_tol;
  bool invalid = false;
  if (S.lanef() <= N) S.fixm[S.lanef()] = 0;
  sync();
  double nfix_l = 0.0;
  for (int i = S.lanef(); i < nw; i += WAVE) {
    const int e = ext_u(prm, i);  // external decision index, -1: absent control (fixed at 0, unbounded)
    S.U[i] = e >= 0 ? io.x0[(long long)b * io.ld_x0 + e] : 0.0;
    const double lo = e >= 0 ? io.lbx[(long long)b * io.ld_lbx + e] : -INFINITY;
    const double hi = e >= 0 ? io.ubx[(long long)b * io.ld_ubx + e] : INFINITY;
    S.xl[i] = lo > -BIGB ? lo - fmin(cvt, brf * fmax(1.0, fabs(lo))) : -INFINITY;
    S.xu[i] = hi < BIGB ? hi + fmin(cvt, brf * fmax(1.0, fabs(hi))) : INFINITY;
    if (lo > hi) invalid = true;
    if (lo > -BIGB && lo == hi) {  // fixed variable (IPOPT make_parameter): held at the bound, unbounded
      S.U[i] = lo; S.xl[i] = -INFINITY; S.xu[i] = INFINITY;
      atomicOr((int*)&S.fixm[i / 6], 1 << (i - 6 * (i / 6)));
      nfix_l += 1.0;
    }
  }
  S.nfix = (int)wsum(nfix_l);
  if (S.lanef() == 0) S.rvars[46] = (double)S.nfix;
  if constexpr (!CAP::eq) {
    for (int r = S.lanef(); r < ng; r += WAVE) {
      const double lo = io.lbg[(long long)b * io.ld_lbg + r], hi = io.ubg[(long long)b * io.ld_ubg + r];
      S.dl[r] = lo > -BIGB ? lo - fmin(cvt, brf * fmax(1.0, fabs(lo))) : -INFINITY;  // unscaled for now
      S.du[r] = hi < BIGB ? hi + fmin(cvt, brf * fmax(1.0, fabs(hi))) : INFINITY;
      // an equality row reaches a class without them only on the fp32 leg (the host sends
      // fp64 batches with equality rows to the equality class): Invalid_Problem_Definition
      if (lo >= hi && lo > -BIGB) invalid = true;
      S.dc[r] = 1.0;
    }
  } else {
    int meq_l = 0;
    for (int r0 = 0; r0 < ng; r0 += WAVE) {
      const int r = r0 + S.lanef();
      bool eq = false;
      if (r < ng) {
        const double lo = io.lbg[(long long)b * io.ld_lbg + r], hi = io.ubg[(long long)b * io.ld_ubg + r];
        S.dl[r] = lo > -BIGB ? lo - fmin(cvt, brf * fmax(1.0, fabs(lo))) : -INFINITY;  // unscaled for now
        S.du[r] = hi < BIGB ? hi + fmin(cvt, brf * fmax(1.0, fabs(hi))) : INFINITY;
        if (lo > hi) invalid = true;
        // equality row (IPOPT c(x) = 0, no relaxation): NaN bounds, slack pinned at the target
        eq = lo == hi && lo > -BIGB;
        if (eq) { S.dl[r] = NAN; S.du[r] = NAN; S.s[r] = lo; }
        S.dc[r] = 1.0;
      }
      const unsigned long long mk = __ballot(eq);
      const int pos = meq_l + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mk >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mk, 0u));
      if (eq && pos < NMPC_MEQ) S.eqi_()[pos] = r;
      meq_l += __popcll(mk);
    }
    S.meq = meq_l;
    if (meq_l > NMPC_MEQ) invalid = true;  // more equality rows than the Schur step holds
    if (S.lanef() == 0) S.rvars[47] = (double)meq_l;
  }
  if (S.lanef() == 0) S.filt[2 * FCAP] = 0.0;
  sync();
  S.nfilt = 0;
  S.delta = 0.0;
  S.df = 1.0;
  S.mu = o.mu_init;
  int status = 0, it = 0;
  if (wany(invalid)) {
    status = ST_INVALID_PROBLEM;
  }

  // ---------------- scaling at the user's starting point (IPOPT gradient-based)
  if (status == 0) {
    S.rollout(S.U, S.X);
    const double F0 = S.eval_fg(S.X, S.d, nullptr);
    S.template derivs<true, true>(S.X, S.U, S.tc);
    S.adjoint(1.0, (const GLB double*)nullptr);
    double gmax = 0.0;
    bool bad = !isfinite(F0);
    for (int i = S.lanef(); i < nw; i += WAVE) {
      const double g = S.fixed(i) ? 0.0 : S.grad_u(i);  // fixed variables leave the scaling
      if (!isfinite(g)) bad = true;
      gmax = fmax(gmax, fabs(g));
    }
    for (int r = S.lanef(); r < ng; r += WAVE)
      if (!isfinite(S.d[r])) bad = true;
    gmax = wmax(gmax);
    if (wany(bad)) status = ST_INVALID_NUMBER;
    double dfv = 1.0;
    if (gmax > o.nlp_scaling_max_gradient) dfv = o.nlp_scaling_max_gradient / gmax;
    S.df = fmax(dfv, o.nlp_scaling_min_value);
    // Jacobian row maxima: J rows = G_k Z_k, Z_k[:,u_j] = (I + sum_{l=j+1}^{k-1} E_l) B_j
    if (status == 0) {
      // (every array below has a compile-time size and is indexed by unrolled loop counters
      // only -- box rows rb[0..4], obstacle rows ro[q] -- so none of them lives in scratch)
      constexpr int MO = CAP::mmax;  // obstacle rows per stage <= m - nb <= mmax
      const int k = S.lanef();
      const int nb = S.nb, nobs = S.nobs;
      double rb[5], ro[MO];
#pragma unroll
      for (int i = 0; i < 5; ++i) rb[i] = 0.0;
#pragma unroll
      for (int q = 0; q < MO; ++q) ro[q] = 0.0;
      if (k <= N && k >= 1) {
        const LDS double* xk = S.X + k * 8;
        double gxo[MO], gyo[MO];
#pragma unroll
        for (int q = 0; q < MO; ++q) {
          if (q < nobs) {
            const double ddx = xk[0] - S.obx[q], ddy = xk[1] - S.oby[q];
            const double dd = sqrt(ddx * ddx + ddy * ddy);
            gxo[q] = -(ddx / dd); gyo[q] = -(ddy / dd);
          } else {
            gxo[q] = 0.0; gyo[q] = 0.0;
          }
        }
        double e03 = 0, e04 = 0, e13 = 0, e14 = 0, e23 = 0;  // sums over l in (j, k)
        const double T = S.T;
        for (int j = k - 1; j >= 0; --j) {
          double E03, E04, E13, E14, E23, b00, b10, b20;
          S.stage_AB(j, E03, E04, E13, E14, E23, b00, b10, b20);
          // column of control c of stage j (fixed controls are no columns: make_parameter)
          const int fmj = S.nfix > 0 ? S.fixm[j] : 0;
          auto col = [&](int c, double v) { return ((fmj >> c) & 1) ? 0.0 : fabs(v); };
          // rows z, theta, x5, x6, x7
          rb[0] = fmax(rb[0], fmax(col(0, b20), col(1, T * e23)));
          rb[1] = fmax(rb[1], col(1, T));
          if (nb == 5) {  // gimbal rows x5, x6, x7
            rb[2] = fmax(rb[2], col(3, T));
            rb[3] = fmax(rb[3], col(4, T));
            rb[4] = fmax(rb[4], col(5, T));
          }
#pragma unroll
          for (int q = 0; q < MO; ++q) {
            if (q < nobs) {
              const double jv = gxo[q] * b00 + gyo[q] * b10;
              const double jt = T * (gxo[q] * e03 + gyo[q] * e13);
              const double jp = T * (gxo[q] * e04 + gyo[q] * e14);
              ro[q] = fmax(ro[q], fmax(col(0, jv), fmax(col(1, jt), col(2, jp))));
            }
          }
          e03 += E03; e04 += E04; e13 += E13; e14 += E14; e23 += E23;
        }
      }
      double amax = 0.0;  // (the rows in their order i = 0..m-1: box rows, then obstacles)
#pragma unroll
      for (int i = 0; i < 5; ++i)
        if (i < nb) amax = fmax(amax, rb[i]);
#pragma unroll
      for (int q = 0; q < MO; ++q)
        if (q < nobs) amax = fmax(amax, ro[q]);
      amax = wmax(amax);
      if (amax > o.nlp_scaling_max_gradient && k <= N) {
        auto dcv = [&](double rm) {
          const double v = rm > 0 ? fmin(1.0, o.nlp_scaling_max_gradient / rm) : 1.0;
          return fmax(v, o.nlp_scaling_min_value);
        };
#pragma unroll
        for (int i = 0; i < 5; ++i)
          if (i < nb) S.dc[k * m + i] = dcv(rb[i]);
#pragma unroll
        for (int q = 0; q < MO; ++q)
          if (q < nobs) S.dc[k * m + nb + q] = dcv(ro[q]);
      }
      sync();
    }
  }

  // ---------------- initial point
  if (status == 0) {
    for (int r = S.lanef(); r < ng; r += WAVE) {
      S.dl[r] = S.dc[r] * S.dl[r];
      S.du[r] = S.dc[r] * S.du[r];
    }
    int cx = 0, cs = 0;
    const double kp = o.bound_push, kf_ = o.bound_frac;
    for (int i = S.lanef(); i < nw; i += WAVE) {
      const double lo = S.xl[i], hi = S.xu[i];
      const bool hl = S.hasl(lo), hu = S.hasu(hi);
      double x = S.U[i];
      const double span = (hl && hu) ? hi - lo : INFINITY;
      if (hl) x = fmax(x, lo + fmin(kp * fmax(1.0, fabs(lo)), kf_ * span));
      if (hu) x = fmin(x, hi - fmin(kp * fmax(1.0, fabs(hi)), kf_ * span));
      S.U[i] = x;
      S.zl[i] = hl ? o.bound_mult_init_val : 0.0;
      S.zu[i] = hu ? o.bound_mult_init_val : 0.0;
      cx += (int)hl + (int)hu;
    }
    sync();
    S.rollout(S.U, S.X);
    S.eval_fg(S.X, S.d, S.dc);
    S.template derivs<true, true>(S.X, S.U, S.tc);
    const double skp = o.slack_bound_push, skf = o.slack_bound_frac;
    for (int r = S.lanef(); r < ng; r += WAVE) {
      const double lo = S.dl[r], hi = S.du[r];
      const bool hl = S.hasl(lo), hu = S.hasu(hi);
      double x = S.d[r];
      const double span = (hl && hu) ? hi - lo : INFINITY;
      if (hl) x = fmax(x, lo + fmin(skp * fmax(1.0, fabs(lo)), skf * span));
      if (hu) x = fmin(x, hi - fmin(skp * fmax(1.0, fabs(hi)), skf * span));
      if (S.eqlo(lo)) x = S.dc[r] * S.s[r];  // equality row: pinned at the scaled target
      S.s[r] = x;
      S.vl[r] = hl ? o.bound_mult_init_val : 0.0;
      S.vu[r] = hu ? o.bound_mult_init_val : 0.0;
      S.y[r] = 0.0;
      cs += (int)hl + (int)hu;
    }
    S.nzx = (int)wsum((double)cx);
    S.nzs = (int)wsum((double)cs);
    sync();
    // least-squares constraint multipliers: (I + J^T J) wx = bx + J^T bs ; y = bs - J wx
    if (o.constr_mult_init_max > 0 && ng > 0) {
      for (int i = S.lanef(); i < nw; i += WAVE) { S.sigx[i] = 1.0; S.ru[i] = S.zl[i] - S.zu[i]; }
      S.delta = 0.0;
      S.assemble(SUM_LS, 0.0, -S.df, false);
      bool lsok = S.riccati(S.sigx, S.ru);
      bool lsdone = false;
      if constexpr (CAP::eq) {
        if (S.meq > 0) {  // [I + J_d^T J_d, -J_c^T; J_c, 0] [w; y_c] = [b; 0]
          S.nneg = 0;
          lsok = lsok && S.eq_schur(S.mu, false);
          if (lsok) S.template eq_step<2>(S.ru, S.dU, S.dX, S.eqy_());
          lsdone = true;
        }
      }
      if (!lsdone) {
        S.forward(S.dU, S.dX);
        S.refine(S.sigx, S.ru, S.dU, S.dX);
      }
      double ymax = 0.0;
      for (int r = S.lanef(); r < ng; r += WAVE) {
        // y = bs - J wx with J wx = Gt dX
        const int k = r / m, i = r - k * m;
        const LDS double* xk = S.X + k * 8;
        const LDS double* dxk = S.dX + k * 8;
        double jd;
        if (i < S.nb) jd = S.dc[r] * dxk[boxidx(i)];
        else {
          const int q = i - S.nb;
          const double ddx = xk[0] - S.obx[q], ddy = xk[1] - S.oby[q];
          const double dd = sqrt(ddx * ddx + ddy * ddy);
          jd = S.dc[r] * ((-(ddx / dd)) * dxk[0] + (-(ddy / dd)) * dxk[1]);
        }
        const double yv = S.eqr(r) ? S.eqy_()[r] : (S.vu[r] - S.vl[r]) - jd;
        S.y[r] = yv;
        ymax = fmax(ymax, fabs(yv));
      }
      ymax = wmax(ymax);
      sync();
      if (!lsok || !(ymax <= o.constr_mult_init_max)) {
        for (int r = S.lanef(); r < ng; r += WAVE) S.y[r] = 0.0;
      }
      sync();
    }
  }

#ifdef NMPC_STAMPS
  if (S.lanef() == 0) stamps[PH_INIT] += (double)(__builtin_amdgcn_s_memtime() - _tk0);
#endif
  // ---------------- main loop
  double f = 0.0;
  if (status == 0) {
    f = S.df * S.eval_fg(S.X, S.d, S.dc);
  }
  S.mu = o.mu_init;
  S.tau = fmax(o.tau_min, 1.0 - S.mu);
  // loop-carried scalars read a few times per iteration: kept in LDS (slots 24..29 of the
  // scalar block) instead of registers held across every heavy phase
  volatile LDS double* MV = S.rvars + 24;
  MV[0] = -1.0; MV[1] = -1.0;
  MV[2] = 0.0; MV[3] = 0.0;
  bool in_soft = false, tiny_flag = false, have_acc = false;
  bool phic = false;  // rvars[32..33] hold the barrier sums of the current iterate (its accepted trial)
  int soft_cnt = 0, acc_cnt = 0, last_obj_iter = -1;
  MV[4] = -1e50; MV[5] = -1e50;
  const double smax = o.s_max;
  bool running = (status == 0);
  bool need_resto = false;
  RestoIO rio;
  // watchdog procedure (BacktrackingLineSearch): successive shortened steps, active
  // flag, trial iterations; WD = reference values of the stored point and its step
  // [0] theta, [1] phi, [2] grad(phi)^T d, [3] alpha test, [4] mu, [5] delta of the step
  int wd_cnt = 0, wd_trial = 0;
  bool in_wd = false;
  volatile LDS double* WD = S.rvars + 40;

  while (running) {
  while (true) {
    // ===== adjoint with current y (grad of the Lagrangian, Hessian multipliers)
    S.adjoint(S.df, S.y);
    STAMP0();
    // ===== optimality error (IpoptCalculatedQuantities::curr_nlp_error)
    double dinf = 0, cviol = 0, ucviol = 0, cmp = 0, sumy = 0, sumz = 0, sumv = 0, pinf = 0;
    double cmu = 0;  // = compl_max(mu) of the barrier update below, from the same pass
    const double muc = S.mu;
    bool bad = false;
    S.ctrls([&](int i, bool on) {  // (maxima and flags ignore the repeated last entry)
      const double g = S.fixed(i) ? 0.0 : S.grad_u(i) - S.zl[i] + S.zu[i];
      if (!isfinite(g)) bad = true;
      dinf = fmax(dinf, fabs(g));
      if (S.hasl(S.xl[i])) cmp = fmax(cmp, fabs((S.U[i] - S.xl[i]) * S.zl[i]));
      if (S.hasu(S.xu[i])) cmp = fmax(cmp, fabs((S.xu[i] - S.U[i]) * S.zu[i]));
      if (S.hasl(S.xl[i])) cmu = fmax(cmu, fabs((S.U[i] - S.xl[i]) * S.zl[i] - muc));
      if (S.hasu(S.xu[i])) cmu = fmax(cmu, fabs((S.xu[i] - S.U[i]) * S.zu[i] - muc));
      const double sz = fabs(S.zl[i]) + fabs(S.zu[i]);
      if (on) sumz += sz;
    });
    S.rows([&](int r, bool on) {
      const double yr = S.y[r], vlr = S.vl[r], vur = S.vu[r], dr = S.d[r], sr = S.s[r], dcr = S.dc[r];
      const double lo = S.dl[r], hi = S.du[r];
      const bool hl = on && S.hasl(lo), hu = on && S.hasu(hi);
      const bool eq = S.eqlo(lo);
      const double g = -yr - vlr + vur;  // slack component (inequality rows only)
      if (on && !eq) dinf = fmax(dinf, fabs(g));
      double cv = eq ? fabs(dr - sr) : 0.0;
      if (hl) cv = fmax(cv, lo - dr);
      const double cl = fabs((sr - lo) * vlr);
      if (hl) cmp = fmax(cmp, cl);
      if (hu) cv = fmax(cv, dr - hi);
      const double cu = fabs((hi - sr) * vur);
      if (hu) cmp = fmax(cmp, cu);
      const double clm = fabs((sr - lo) * vlr - muc), cum = fabs((hi - sr) * vur - muc);
      if (hl) cmu = fmax(cmu, clm);
      if (hu) cmu = fmax(cmu, cum);
      const double ucv = cv / dcr;
      if (on) {
        cviol = fmax(cviol, cv);
        ucviol = fmax(ucviol, ucv);
        pinf = fmax(pinf, fabs(dr - sr));
        sumy += fabs(yr);
        sumv += fabs(vlr) + fabs(vur);
        if (!isfinite(dr) || !isfinite(g)) bad = true;
      }
    });
    dinf = wmax(dinf); cviol = wmax(cviol); ucviol = wmax(ucviol); cmp = wmax(cmp);
    pinf = wmax(pinf);
    sumy = wsum(sumy); sumz = wsum(sumz); sumv = wsum(sumv);
    bad = wany(bad) || !isfinite(f);
    const int nd = ng + S.nzx + S.nzs, nc = S.nzx + S.nzs;
    double sd = nd ? (sumy + sumz + sumv) / nd : 0.0;
    sd = fmax(smax, sd) / smax;
    double sc = nc ? (sumz + sumv) / nc : 0.0;
    sc = fmax(smax, sc) / smax;
    const double err = fmax(fmax(dinf / sd, cviol), cmp / sc);
    if (trace && S.lanef() == 0) {  // the convergence check of iteration `it` (parity diagnostics)
      double* t = trace + (long long)it * TRACE_F;
      t[8] = err; t[9] = dinf / sd; t[10] = cviol; t[11] = cmp / sc;
    }
    if (bad || !isfinite(err)) { status = ST_INVALID_NUMBER; break; }
    const double u_dinf = dinf / S.df, u_cmp = cmp / S.df;
    if (err <= o.tol && u_dinf <= o.dual_inf_tol && ucviol <= o.constr_viol_tol && u_cmp <= o.compl_inf_tol) {
      status = ST_SUCCESS; break;
    }
    if (it != last_obj_iter) { MV[4] = MV[5]; MV[5] = f; last_obj_iter = it; }
    const bool acceptable = err <= o.acceptable_tol && u_dinf <= o.acceptable_dual_inf_tol &&
                            ucviol <= o.acceptable_constr_viol_tol && u_cmp <= o.acceptable_compl_inf_tol &&
                            fabs(MV[5] - MV[4]) / fmax(1.0, fabs(MV[5])) <= o.acceptable_obj_change_tol;
    if (o.acceptable_iter > 0 && acceptable) {
      if (++acc_cnt >= o.acceptable_iter) { status = ST_ACCEPTABLE; break; }
    } else {
      acc_cnt = 0;
    }
    if (it >= max_iter) { status = ST_MAXITER; break; }
    if (acceptable) {  // BacktrackingLineSearch::StoreAcceptablePoint
      for (int i = S.lanef(); i < nw; i += WAVE) { S.accU[i] = S.U[i]; S.accZl[i] = S.zl[i]; S.accZu[i] = S.zu[i]; }
      for (int r = S.lanef(); r < ng; r += WAVE) S.accY[r] = S.y[r];
      have_acc = true;
    }

    // ===== monotone barrier update (MonotoneMuUpdate::UpdateBarrierParameter)
    {
      const double base = fmax(dinf / sd, pinf);
      double sub = fmax(base, wmax(cmu) / sc);  // compl_max(S.mu)
      bool done = false, tsf = tiny_flag;
      while ((sub <= o.barrier_tol_factor * S.mu || tsf) && !done) {
        double nmu = fmin(o.kappa_mu * S.mu, pow(S.mu, o.theta_mu));
        nmu = fmax(nmu, fmin(o.tol, o.compl_inf_tol) / (o.barrier_tol_factor + 1.0));
        const bool changed = nmu != S.mu;
        if (!changed && tsf) { status = ST_TINY; break; }
        S.mu = nmu;
        S.tau = fmax(o.tau_min, 1.0 - S.mu);
        if (!changed) done = true;
        else {
          sub = fmax(base, S.compl_max(S.mu) / sc);
          done = sub > o.barrier_tol_factor * S.mu;
        }
        if (done && changed) { S.nfilt = 0; in_soft = false; }
        tsf = false;
      }
      if (status != 0) break;
      tiny_flag = false;
    }
    const double mu = S.mu, tau = S.tau;
    STAMP1(PH_CONV);

    // ===== search direction with inertia correction (PDPerturbationHandler)
    { STAMP0();
    S.ctrls([&](int i, bool on) {
      const bool hl = S.hasl(S.xl[i]), hu = S.hasu(S.xu[i]);
      const double Sl = hl ? S.U[i] - S.xl[i] : 1.0, Su = hu ? S.xu[i] - S.U[i] : 1.0;
      const double sg = (hl ? qd(S.zl[i], Sl) : 0.0) + (hu ? qd(S.zu[i], Su) : 0.0);
      const double rr = -(hl ? qd(mu, Sl) : 0.0) + (hu ? qd(mu, Su) : 0.0) +
                        o.kappa_d * mu * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0));
      if (on) { S.sigx[i] = sg; S.ru[i] = rr; }
    });
    sync();
    STAMP1(PH_SIGX); }
    if (MV[3] > 0) MV[2] = MV[3];
    double delta = 0.0;
    bool fact_ok = false;
    while (true) {
      S.delta = delta;
      S.assemble(SUM_NEWTON, S.df, S.df, true);
      bool okf;
      if constexpr (CAP::eq) {  // equality rows: signed pivots, augmented-system inertia
        okf = S.meq > 0 ? S.template riccati<true>(S.sigx, S.ru) && S.eq_schur(S.mu) : S.riccati(S.sigx, S.ru);
      } else {
        okf = S.riccati(S.sigx, S.ru);
      }
      if (okf) { fact_ok = true; break; }
      sync();
      if (delta == 0.0) {
        delta = (MV[2] == 0.0) ? o.first_hessian_perturbation
                                    : fmax(o.min_hessian_perturbation, MV[2] * o.perturb_dec_fact);
      } else {
        if (MV[2] == 0.0 || 1e5 * MV[2] < delta) delta *= o.perturb_inc_fact_first;
        else delta *= o.perturb_inc_fact;
      }
      if (delta > o.max_hessian_perturbation) break;
    }
    MV[3] = delta;
    S.delta = delta;
    if (!fact_ok) { status = ST_STEP_ERR; break; }
    bool eqs = false;
    if constexpr (CAP::eq) {
      if (S.meq > 0) { S.template eq_step<0>(S.ru, S.dU, S.dX, S.eqy_()); eqs = true; }
    }
    if (!eqs) {
      S.forward(S.dU, S.dX);
      S.refine(S.sigx, S.ru, S.dU, S.dX);
    }

    // ===== line search (BacktrackingLineSearch + FilterLSAcceptor)
    double theta_ref = 0.0, gbd = 0.0, tiny_mx = 0.0, tiny_msv = 0.0;
    // the switching condition's powers pow(-gbd, s_phi), pow(theta_ref, s_theta) depend only
    // on the line search's reference values: formed once (when first needed) and reused by
    // every trial's F-type test, the minimum step and the filter decision, the same doubles
    // as one pow per use (PW[0]: valid flag; reset wherever theta_ref / gbd change)
    volatile LDS double* PW = S.rvars + 37;
    PW[0] = 0.0;
    auto pw_get = [&]() {
      if (PW[0] == 0.0) {
        PW[1] = gbd < 0.0 ? pow(-gbd, o.s_phi) : 0.0;
        PW[2] = pow(theta_ref, o.s_theta);
        PW[0] = 1.0;
      }
    };
    // primal / dual fraction to the boundary of the step (dU, ds) at the current iterate,
    // formed with the step's row pass; valid until the watchdog restores another iterate
    double ftb_p = 1.0, ftb_d = 1.0;
    bool ftb_ok = true;
    {
      double th, g, msv, mx = 0.0, ap, ad;
      S.row_step_ls(S.dX, mu, tau, th, g, msv, ap, ad);
      STAMP0();
      S.ctrls([&](int i, bool on) {
        const double du_ = S.dU[i];
        const double gi = S.ru[i] * du_;
        if (on) g += gi;
        mx = fmax(mx, fabs(qd(du_, 1.0 + fabs(S.U[i]))));
        const double ui = S.U[i], xli = S.xl[i], xui = S.xu[i];
        if (S.hasl(xli) && du_ < 0) ap = fmin(ap, qd(-tau * (ui - xli), du_));
        if (S.hasu(xui) && -du_ < 0) ap = fmin(ap, qd(-tau * (xui - ui), -du_));
        double a1, a2;
        S.dz_x(i, du_, a1, a2);
        if (S.hasl(xli) && a1 < 0) ad = fmin(ad, qd(-tau * S.zl[i], a1));
        if (S.hasu(xui) && a2 < 0) ad = fmin(ad, qd(-tau * S.zu[i], a2));
      });
      ftb_p = wmin(ap);
      ftb_d = wmin(ad);
      if (S.lanef() <= N) {
        double gx = 0.0;
#pragma unroll
        for (int c = 0; c < 8; ++c) gx += S.gl[S.lanef() * 8 + c] * S.dX[S.lanef() * 8 + c];
        g += S.df * gx;
      }
      theta_ref = wsum(th);
      gbd = wsum(g);
      PW[0] = 0.0;  // new reference values: the switching-condition powers are formed anew
      tiny_mx = wmax(mx);
      tiny_msv = wmax(msv);
      STAMP1(PH_LSSET);
    }
    STAMPV0(_tls);  // whole line search incl. nested phases (diagnostic slot of the old Riccati step 3)
    double phi_ref = phic ? S.phi_of(f, S.rvars[32], S.rvars[33]) : S.barrier_obj(f, S.U, S.s, nullptr, 0.0);
    if (MV[0] < 0) {
      MV[0] = o.theta_max_fact * fmax(1.0, theta_ref);
      MV[1] = o.theta_min_fact * fmax(1.0, theta_ref);
    }
    const double eps = 2.220446049250313e-16;
    auto cmp_le = [&](double lhs, double rhs, double bas) { return lhs - rhs <= 10.0 * eps * fabs(bas); };
    auto is_ftype = [&](double a) {
      if (!(gbd < 0.0)) return false;
      pw_get();
      return a * PW[1] > o.delta * PW[2];
    };
    auto armijo = [&](double a, double phit) { return cmp_le(phit - phi_ref, o.eta_phi * a * gbd, phi_ref); };
    auto acc_iter = [&](double phit, double tht) {
      if (phit > phi_ref) {
        double basval = 1.0;
        if (fabs(phi_ref) > 10.0) basval = log10(fabs(phi_ref));
        if (log10(phit - phi_ref) > o.obj_max_inc + basval) return false;
      }
      return cmp_le(tht, (1.0 - o.gamma_theta) * theta_ref, theta_ref) ||
             cmp_le(phit - phi_ref, -o.gamma_phi * theta_ref, phi_ref);
    };
    auto check_accept = [&](double a_test, double phit, double tht) {
      if (tht > MV[0]) return false;
      bool ok;
      if (a_test > 0.0 && is_ftype(a_test) && theta_ref <= MV[1]) ok = armijo(a_test, phit);
      else ok = acc_iter(phit, tht);
      if (!ok) return false;
      return S.filter_ok(phit, tht);
    };

    // accepted step bookkeeping: which step vectors, alphas
    int acc_kind = 0;  // 0 none, 1 regular (dU/ds), 2 regular SOC (dU2/ds2), 3 soft
    double alpha_p = 0.0, alpha_d = 0.0, f_acc = 0.0;
    int ls_trials = 0;
    double a_test_acc = 0.0, phi_acc = 0.0;
    int n_acc = 0;          // backtracking steps before the accepted trial
    bool wd_forced = false; // a watchdog trial iteration: full step taken unchecked

    // ===== watchdog procedure (BacktrackingLineSearch::FindAcceptableTrialPoint)
    // tiny step detection (BacktrackingLineSearch::DetectTinyStep; ratios from row_step_ls)
    bool tiny = tiny_mx <= o.tiny_step_tol && tiny_msv <= o.tiny_step_tol && pinf <= 1e-4;
    // the dual step of the step being taken is formed with the mu / delta it was computed
    // with: after StopWatchDog that is the stored step's (WD[4], WD[5])
    bool wd_dir = false;
    auto dir_mu = [&]() { return wd_dir ? (double)WD[4] : mu; };
    // StopWatchDog: back to the stored iterate, its step and its reference values
    auto wd_restore = [&]() {
      for (int i = S.lanef(); i < nw; i += WAVE) {
        S.U[i] = S.wU[i]; S.zl[i] = S.wzl[i]; S.zu[i] = S.wzu[i]; S.dU[i] = S.wdU[i];
      }
      for (int r = S.lanef(); r < ng; r += WAVE) {
        S.s[r] = S.wsl[r]; S.y[r] = S.wy[r]; S.vl[r] = S.wvl[r]; S.vu[r] = S.wvu[r]; S.ds[r] = S.wds[r];
      }
      if constexpr (CAP::eq) {  // the stored step's equality-multiplier step (WdPoint's dy)
        if (S.meq > 0)
          for (int r = S.lanef(); r < ng; r += WAVE) S.eqy_()[r] = S.weqy_()[r];
      }
      sync();
      S.rollout(S.U, S.X);
      f = S.df * S.eval_fg(S.X, S.d, S.dc);
      S.template derivs<true, true>(S.X, S.U, S.tc);
      S.adjoint(S.df, S.y);  // grad of the Lagrangian there (soft restoration's pd error)
      theta_ref = WD[0]; phi_ref = WD[1]; gbd = WD[2];
      PW[0] = 0.0;
      S.delta = WD[5];
      wd_dir = true;
      ftb_ok = false;  // another iterate and step: the fused fractions no longer apply
      phic = false;
      in_wd = false;
      wd_cnt = 0;
    };
    if (in_wd && tiny) {  // a tiny step inside the watchdog stops it
      wd_restore();
      tiny = false;
    }
    if (o.watchdog_shortened_iter_trigger > 0 && !in_wd && !tiny && !in_soft &&
        wd_cnt >= o.watchdog_shortened_iter_trigger) {  // StartWatchDog
      for (int i = S.lanef(); i < nw; i += WAVE) {
        S.wU[i] = S.U[i]; S.wzl[i] = S.zl[i]; S.wzu[i] = S.zu[i]; S.wdU[i] = S.dU[i];
      }
      for (int r = S.lanef(); r < ng; r += WAVE) {
        S.wsl[r] = S.s[r]; S.wy[r] = S.y[r]; S.wvl[r] = S.vl[r]; S.wvu[r] = S.vu[r]; S.wds[r] = S.ds[r];
      }
      if constexpr (CAP::eq) {
        if (S.meq > 0)
          for (int r = S.lanef(); r < ng; r += WAVE) S.weqy_()[r] = S.eqy_()[r];
      }
      const double at = ftb_ok ? ftb_p : S.frac_to_bound(tau, S.dU, S.ds);
      WD[0] = theta_ref; WD[1] = phi_ref; WD[2] = gbd; WD[3] = at; WD[4] = mu; WD[5] = S.delta;
      sync();
      in_wd = true;
      wd_trial = 0;
    }
    if (in_wd) {  // FilterLSAcceptor::InitThisLineSearch(in_watchdog): the stored reference
      theta_ref = WD[0]; phi_ref = WD[1]; gbd = WD[2];
      PW[0] = 0.0;
    }

    // soft restoration step (BacktrackingLineSearch::TrySoftRestoStep); returns
    // 0 rejected, 1 accepted, 2 accepted & satisfies the original criterion
    auto try_soft = [&]() -> int {
      const double ap = ftb_ok ? ftb_p : S.frac_to_bound(tau, S.dU, S.ds);
      S.mu = dir_mu();  // dual components of the step (its own mu); the barrier terms use mu
      const double ad = (ftb_ok && !wd_dir) ? ftb_d : S.dual_frac_to_bound(tau, S.dU, S.ds);
      S.mu = mu;
      const double a = fmin(ap, ad);
      // current pd error (grad_lag from the adjoint computed at loop start)
      double dual = 0, prim = 0, cm = 0;
      for (int i = S.lanef(); i < nw; i += WAVE) {
        dual += S.fixed(i) ? 0.0 : fabs(S.grad_u(i) - S.zl[i] + S.zu[i]);
        if (S.hasl(S.xl[i])) cm += fabs((S.U[i] - S.xl[i]) * S.zl[i] - mu);
        if (S.hasu(S.xu[i])) cm += fabs((S.xu[i] - S.U[i]) * S.zu[i] - mu);
      }
      for (int r = S.lanef(); r < ng; r += WAVE) {
        if (!S.eqr(r)) dual += fabs(-S.y[r] - S.vl[r] + S.vu[r]);
        prim += fabs(S.d[r] - S.s[r]);
        if (S.hasl(S.dl[r])) cm += fabs((S.s[r] - S.dl[r]) * S.vl[r] - mu);
        if (S.hasu(S.du[r])) cm += fabs((S.du[r] - S.s[r]) * S.vu[r] - mu);
      }
      const double nn = (double)(S.nwE - S.nfix + ng - (CAP::eq ? S.meq : 0));
      const double e_c = wsum(dual) / nn + (ng ? wsum(prim) / ng : 0.0) + (nc ? wsum(cm) / nc : 0.0);
      double ft, phit, tht;
      ++ls_trials;
      if (!S.trial(a, S.dU, S.ds, ft, phit, tht)) return 0;
      // trial multipliers into the "2" buffers: dU2 <- (unused) ; stage them in place later
      // evaluate grad_lag at the trial point: derivatives + adjoint with trial y
      // (overwrites the current derivative data; if rejected the solve stops)
      S.mu = dir_mu();
      for (int r = S.lanef(); r < ng; r += WAVE) {
        double D, rs;
        S.row_rs(r, D, rs);
        S.dms[r] = S.y[r] + a * (S.eqr(r) ? S.eqy_()[r] : D * S.ds[r] + rs);  // trial y
      }
      sync();
      S.template derivs<true, true>(S.Xt, S.Ut, S.tc);
      // adjoint at the trial point: swap X temporarily
      LDS double* Xs = S.X; S.X = S.Xt;
      S.adjoint(S.df, S.dms);
      S.X = Xs;
      double dual2 = 0, prim2 = 0, cm2 = 0;
      for (int i = S.lanef(); i < nw; i += WAVE) {
        double dzl, dzu;
        S.dz_x(i, S.dU[i], dzl, dzu);
        const double zlt = S.zl[i] + a * dzl, zut = S.zu[i] + a * dzu;
        dual2 += S.fixed(i) ? 0.0 : fabs(S.grad_u(i) - zlt + zut);
        if (S.hasl(S.xl[i])) cm2 += fabs((S.Ut[i] - S.xl[i]) * zlt - mu);
        if (S.hasu(S.xu[i])) cm2 += fabs((S.xu[i] - S.Ut[i]) * zut - mu);
      }
      for (int r = S.lanef(); r < ng; r += WAVE) {
        double dvl, dvu;
        S.dv_s(r, S.ds[r], dvl, dvu);
        const double vlt = S.vl[r] + a * dvl, vut = S.vu[r] + a * dvu;
        const double sv = S.s[r] + a * S.ds[r];
        if (!S.eqr(r)) dual2 += fabs(-S.dms[r] - vlt + vut);
        prim2 += fabs(S.dt[r] - sv);
        if (S.hasl(S.dl[r])) cm2 += fabs((sv - S.dl[r]) * vlt - mu);
        if (S.hasu(S.du[r])) cm2 += fabs((S.du[r] - sv) * vut - mu);
      }
      S.mu = mu;
      const double e_t = wsum(dual2) / nn + (ng ? wsum(prim2) / ng : 0.0) + (nc ? wsum(cm2) / nc : 0.0);
      if (e_t <= o.soft_resto_pderror_reduction_factor * e_c) {
        alpha_p = a; alpha_d = a; f_acc = ft;
        acc_kind = 3;
        return check_accept(0.0, phit, tht) ? 2 : 1;
      }
      return 0;
    };

    bool derivs_done = false;  // soft-resto path already computed derivatives at the trial
    if (in_soft) {
      ++soft_cnt;
      if (soft_cnt <= o.max_soft_resto_iters) {
        const int r = try_soft();
        if (r > 0) derivs_done = true;
        if (r == 2) in_soft = false;
      }
    } else {
      if (tiny) {
        const double a = ftb_ok ? ftb_p : S.frac_to_bound(tau, S.dU, S.ds);
        double ft, phit, tht;
        ++ls_trials;
        if (S.trial(a, S.dU, S.ds, ft, phit, tht)) {
          acc_kind = 1; alpha_p = a; f_acc = ft;
          tiny_flag = true;
        }
      } else {
       bool skip_first = false;  // after StopWatchDog: the stored step's full step was rejected
       while (true) {
        if (in_wd) {
          // one trial at the full step, judged against the stored reference values with
          // the stored alpha test, no SOC (BacktrackingLineSearch::DoBacktrackingLineSearch)
          const double amax_w = ftb_ok ? ftb_p : S.frac_to_bound(tau, S.dU, S.ds);
          double ft, phit, tht;
          ++ls_trials;
          const bool okev = S.trial(amax_w, S.dU, S.ds, ft, phit, tht);
          const double at = WD[3];
          if (okev && check_accept(at, phit, tht)) {  // watchdog procedure successful
            acc_kind = 1; alpha_p = amax_w; f_acc = ft; a_test_acc = at; phi_acc = phit;
            in_wd = false;
            break;
          }
          if (!okev || ++wd_trial > o.watchdog_trial_iter_max) {
            wd_restore();
            skip_first = true;
            continue;
          }
          acc_kind = 1; alpha_p = amax_w; f_acc = ft;  // watchdog trial iteration
          wd_forced = true;
          break;
        }
        double amin = o.gamma_theta;
        if (gbd < 0) {
          amin = fmin(o.gamma_theta, o.gamma_phi * theta_ref / (-gbd));
          if (theta_ref <= MV[1]) {
            pw_get();
            amin = fmin(amin, o.delta * PW[2] / PW[1]);
          }
        }
        amin *= o.alpha_min_frac;
        const double amax_p = ftb_ok ? ftb_p : S.frac_to_bound(tau, S.dU, S.ds);
        double a = skip_first ? amax_p * o.alpha_red_factor : amax_p;
        int n_steps = 0;
        while (a > amin || n_steps == 0) {
          double ft, phit, tht;
          ++ls_trials;
          const bool okev = S.trial(a, S.dU, S.ds, ft, phit, tht);
          if (okev && check_accept(a, phit, tht)) {
            acc_kind = 1; alpha_p = a; f_acc = ft; a_test_acc = a; phi_acc = phit; n_acc = n_steps;
            break;
          }
          if (okev && a == amax_p && theta_ref <= tht && o.max_soc > 0) {
            // second-order correction (FilterLSAcceptor::TrySecondOrderCorrection)
            double th_tr = tht, th_old = 0.0, a_soc = a;
            for (int r = S.lanef(); r < ng; r += WAVE) S.dms[r] = S.d[r] - S.s[r];
            int cnt = 0;
            bool soc_acc = false;
            const auto* dsp = S.ds;  // step whose trial is in Ut/dt
            while (cnt < o.max_soc && (cnt == 0 || th_tr <= o.kappa_soc * th_old)) {
              th_old = th_tr;
              for (int r = S.lanef(); r < ng; r += WAVE) {
                const double sv = S.s[r] + a_soc * dsp[r];
                S.dms[r] = a_soc * S.dms[r] + (S.dt[r] - sv);
              }
              sync();
              S.assemble(SUM_SOC, S.df, S.df, true);
              bool eqs2 = false;
              if constexpr (CAP::eq) {
                if (S.meq > 0) { S.template eq_step<1>(S.ru, S.dU2, S.dX, S.eqy2_()); eqs2 = true; }
              }
              if (!eqs2) {
                S.resolve(S.ru);
                S.forward(S.dU2, S.dX);   // dX is free once gBD is known
                S.refine(S.sigx, S.ru, S.dU2, S.dX);
              }
              a_soc = S.row_step_soc(S.dX, S.dU2, S.ds2, tau);
              dsp = S.ds2;
              double ft2, phit2, tht2;
              ++ls_trials;
              if (!S.trial(a_soc, S.dU2, S.ds2, ft2, phit2, tht2)) break;
              if (check_accept(a, phit2, tht2)) {
                acc_kind = 2; alpha_p = a_soc; f_acc = ft2; a_test_acc = a; phi_acc = phit2; n_acc = n_steps;
                soc_acc = true;
                break;
              }
              ++cnt;
              th_tr = tht2;
            }
            if (soc_acc) break;
          }
          a *= o.alpha_red_factor;
          ++n_steps;
        }
        break;
       }
        if (acc_kind == 0) {
          const int r = try_soft();
          if (r > 0) derivs_done = true;
          if (r == 1) { in_soft = true; soft_cnt = 0; }
        } else if (!wd_forced) {
          if (!(is_ftype(a_test_acc) && armijo(a_test_acc, phi_acc)))
            S.filter_add(phi_ref - o.gamma_phi * theta_ref, (1.0 - o.gamma_theta) * theta_ref);
        }
      }
    }
    // successive shortened steps (regular, tiny and watchdog steps) trigger the watchdog
    if (acc_kind == 1 || acc_kind == 2) wd_cnt = (n_acc == 0) ? 0 : wd_cnt + 1;
    if (acc_kind == 0) {
      // ===== feasibility restoration phase (BacktrackingLineSearch -> RestoMinC_1Nrm;
      //       oracle restoration())
      if (theta_ref <= 1e-2 * o.tol) {
        // called at an almost feasible point: back to the last acceptable iterate
        if (have_acc) {
          for (int i = S.lanef(); i < nw; i += WAVE) { S.U[i] = S.accU[i]; S.zl[i] = S.accZl[i]; S.zu[i] = S.accZu[i]; }
          for (int r = S.lanef(); r < ng; r += WAVE) S.y[r] = S.accY[r];
          sync();
          status = ST_ACCEPTABLE;
        } else {
          status = ST_RESTO_FAIL;
        }
        break;
      }
      S.filter_add(phi_ref - o.gamma_phi * theta_ref, (1.0 - o.gamma_theta) * theta_ref);
      rio.mu0 = mu; rio.tau0 = tau; rio.theta0 = theta_ref; rio.phi0 = phi_ref; rio.f = f;
      rio.df = S.df; rio.nfilt = S.nfilt; rio.nzx = S.nzx; rio.nzs = S.nzs; rio.it = it; rio.trace = trace;
      need_resto = true;
      break;  // to the restoration phase below the iteration loop
    }

    STAMPV1(_tls, PH_RE);
    // ===== accept the trial point (IpoptAlgorithm::AcceptTrialPoint)
    {
      STAMP0();
      const GLB double* dUa = (acc_kind == 2) ? S.dU2 : S.dU;
      const auto* dsa = (acc_kind == 2) ? S.ds2 : S.ds;
      S.mu = dir_mu();  // the step's dual components (mu below: the kappa_sigma safeguard)
      if (acc_kind == 1 && ftb_ok && !wd_dir) alpha_d = ftb_d;  // the step's row pass formed it
      else if (acc_kind != 3) alpha_d = S.dual_frac_to_bound(tau, dUa, dsa);
      const double ap = alpha_p, ad = alpha_d;
      const double ks = o.kappa_sigma;
      // bound multipliers of U (old slacks for the step, new slacks for kappa_sigma)
      // (the accepted controls U <- Ut in the same pass: each lane reads its U[i] for the
      // dual step before it writes it)
      S.ctrls([&](int i, bool on) {
        double dzl, dzu;
        S.dz_x(i, dUa[i], dzl, dzu);
        double nzl = S.zl[i] + ad * dzl, nzu = S.zu[i] + ad * dzu;
        const double un = S.Ut[i];
        if (S.hasl(S.xl[i])) { const double Sn = un - S.xl[i]; nzl = fmax(fmin(nzl, qd(ks * mu, Sn)), qd(mu, ks * Sn)); }
        else nzl = 0.0;
        if (S.hasu(S.xu[i])) { const double Sn = S.xu[i] - un; nzu = fmax(fmin(nzu, qd(ks * mu, Sn)), qd(mu, ks * Sn)); }
        else nzu = 0.0;
        if (on) { S.zl[i] = nzl; S.zu[i] = nzu; S.U[i] = un; }
      });
      const double kdm = o.kappa_d * S.mu, dlt = S.delta;
      S.rows([&](int r, bool on) {
        const double sr = S.s[r], yr = S.y[r], vlr = S.vl[r], vur = S.vu[r], dsr = dsa[r], dtr = S.dt[r];
        const double lo = S.dl[r], hi = S.du[r];
        const bool hl = S.hasl(lo), hu = S.hasu(hi);
        // row_rs and dv_s (same arithmetic), loads hoisted
        const double iSl = hl ? rcp(sr - lo) : 0.0, iSu = hu ? rcp(hi - sr) : 0.0;
        const double D = vlr * iSl + vur * iSu + dlt;
        const double rs = -yr - S.mu * iSl + S.mu * iSu + kdm * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0));
        const double dvl = hl ? S.mu * iSl - vlr - vlr * iSl * dsr : 0.0;
        const double dvu = hu ? S.mu * iSu - vur + vur * iSu * dsr : 0.0;
        const double dyv = S.eqlo(lo) ? ((acc_kind == 2) ? S.eqy2_()[r] : S.eqy_()[r]) : D * dsr + rs;
        const double sn = sr + ap * dsr;
        double nvl = vlr + ad * dvl, nvu = vur + ad * dvu;
        if (hl) { const double Sn = sn - lo; nvl = fmax(fmin(nvl, qd(ks * mu, Sn)), qd(mu, ks * Sn)); }
        else nvl = 0.0;
        if (hu) { const double Sn = hi - sn; nvu = fmax(fmin(nvu, qd(ks * mu, Sn)), qd(mu, ks * Sn)); }
        else nvu = 0.0;
        if (on) {
          S.y[r] = yr + ap * dyv;
          S.vl[r] = nvl; S.vu[r] = nvu;
          S.s[r] = sn;
          S.d[r] = dtr;
        }
      });
      S.mu = mu;
      if (S.lanef() <= N) {
#pragma unroll
        for (int c = 0; c < 8; ++c) S.X[S.lanef() * 8 + c] = S.Xt[S.lanef() * 8 + c];
      }
      sync();
      f = f_acc;
      phic = true;  // no barrier_obj call between the accepted trial and the next phi_ref
      STAMP1(PH_ACCEPT);
      if (!derivs_done) S.template derivs<true, true>(S.X, S.U, S.tc);  // the accepted trial: the last one formed
      else {
        // soft resto computed derivatives at the trial; trig uses U (same values)
        sync();
      }
    }
    ++it;
    if (trace && S.lanef() == 0) {
      double th = 0.0;
      for (int r = 0; r < ng; ++r) th += fabs(S.d[r] - S.s[r]);
      double* t = trace + (long long)(it - 1) * TRACE_F;
      t[0] = it; t[1] = mu; t[2] = f; t[3] = th; t[4] = MV[3]; t[5] = alpha_p; t[6] = alpha_d;
      t[7] = ls_trials;
    }
    sync();
  }
  if (!need_resto) break;
  // ===== feasibility restoration phase, then back into the iteration loop
  need_resto = false;
  resto_phase<CAP>(prm, S.wsbase, b, rio);
  S.mu = rio.mu0;
  S.tau = rio.tau0;
  it = rio.it;
  if (rio.status != 0) { status = rio.status; break; }
  f = rio.f;
  in_soft = false;
  phic = false;
  wd_cnt = 0;
  }

  // ---------------- outputs (honor_original_bounds)
  for (int i = S.lanef(); i < nw; i += WAVE) {
    const int e = ext_u(prm, i);
    const double lo = e >= 0 ? io.lbx[(long long)b * io.ld_lbx + e] : -INFINITY;
    const double hi = e >= 0 ? io.ubx[(long long)b * io.ld_ubx + e] : INFINITY;
    S.Ut[i] = fmin(fmax(S.U[i], lo), hi);
  }
  sync();
  S.rollout(S.Ut, S.Xt);
  const double fo = S.eval_fg(S.Xt, S.dt, nullptr);
  for (int i = S.lanef(); i < nw; i += WAVE) {
    const int e = ext_u(prm, i);
    if (e < 0) continue;
    io.x_out[(long long)b * S.nwE + e] = S.Ut[i];
    if (io.lam_x) io.lam_x[(long long)b * S.nwE + e] = (S.zu[i] - S.zl[i]) / S.df;
  }
  for (int r = S.lanef(); r < ng; r += WAVE) {
    if (io.g_out) io.g_out[(long long)b * ng + r] = S.dt[r];
    if (io.lam_g) io.lam_g[(long long)b * ng + r] = S.y[r] * S.dc[r] / S.df;
  }
  if (io.lam_p) {
    // lam_p = -grad_p (f + lam_g' g) at the returned point (CasADi nlpsol's lam_p; the
    // reference never reads it): x0 through the Lagrangian adjoint of the rollout, the
    // target through the stage costs, moving obstacles through their rows, cost weights
    // taken from p through the cost terms they scale
    for (int i = S.lanef(); i < prm->nX; i += WAVE) S.X[i] = S.Xt[i];
    sync();
    S.derivs(S.X, S.Ut);
    S.adjoint(S.df, S.y);  // lam_k = df * dL/dx_k  (lam_g = y dc / df)
    const int k = S.lanef();
    const double gxt = -wsum(k < N ? S.gl[k * 8] : 0.0), gyt = -wsum(k < N ? S.gl[k * 8 + 1] : 0.0);
    double g_w1 = 0.0, g_w2 = 0.0;
    if (prm->w1p >= 0 || prm->w2p >= 0) {
      const double w1s = S.rvars[30], w2s = S.rvars[31];
      sync();
      S.rvars[30] = 1.0; S.rvars[31] = 0.0;
      sync();
      const double cd = k < N ? S.stage_cost(S.X + k * 8) : 0.0;
      sync();
      S.rvars[30] = 0.0; S.rvars[31] = 1.0;
      sync();
      const double cq = k < N ? S.stage_cost(S.X + k * 8) : 0.0;
      sync();
      S.rvars[30] = w1s; S.rvars[31] = w2s;
      sync();
      g_w1 = wsum(cd); g_w2 = wsum(cq);
    }
    const int np = prm->np;
    double v = 0.0;
    if (k < 8) v = S.lam[k] / S.df;
    else if (k == 8) v = gxt;
    else if (k == 9) v = gyt;
    if (k == prm->w1p) v += g_w1;
    if (k == prm->w2p) v += g_w2;
    for (int o = 0; o < S.nobs; ++o) {
      if (prm->oxp[o] < 0 && prm->oyp[o] < 0) continue;
      double cx = 0.0, cy = 0.0;
      if (k <= N) {  // row g = r_sum - |(x, y) - (ox, oy)|: dg/dox = (x - ox) / d
        const int r = k * S.m + S.nb + o;
        const double lg = S.y[r] * S.dc[r] / S.df;
        const LDS double* xk = S.X + k * 8;
        const double ddx = xk[0] - S.obx[o], ddy = xk[1] - S.oby[o];
        const double idd = rsq(ddx * ddx + ddy * ddy);
        cx = lg * (ddx * idd);
        cy = lg * (ddy * idd);
      }
      cx = wsum(cx); cy = wsum(cy);
      if (k == prm->oxp[o]) v += cx;
      if (k == prm->oyp[o]) v += cy;
    }
    const int e = k < np ? ext_p(prm, k) : -1;
    if (e >= 0) io.lam_p[(long long)b * prm->npE + e] = -v;
  }
  if (io.X_out) {
    const int nX = prm->nX, nxE = prm->nxE, nXE = nxE * (N + 1);
    for (int i = S.lanef(); i < nX; i += WAVE) {
      const int k = i >> 3, c = i & 7;
      if (c < nxE) io.X_out[(long long)b * nXE + k * nxE + c] = S.Xt[i];
    }
  }
#ifdef NMPC_STAMPS
  if (trace) {
    sync();
    if (S.lanef() == 0) stamps[PH_TOTAL] = (double)(__builtin_amdgcn_s_memtime() - _tk0);
    sync();
    // rows max_iter + 1, max_iter + 2 (row max_iter holds the convergence check at iteration max_iter)
    if (S.lanef() < PH_COUNT) trace[(long long)(max_iter + 1) * TRACE_F + S.lanef()] = stamps[S.lanef()];
  }
#endif
  if (S.lanef() == 0) {
    if (io.f_out) io.f_out[b] = fo;
    if (io.status) io.status[b] = status;
    if (io.iters) io.iters[b] = it;
  }
  return it;
}

template <class CAP>
__global__ __launch_bounds__(WAVE, CAP::wpe) void nmpc_solve_kernel(const Params* __restrict__ prm, int B, IO io) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if (io.eqflag && ((*io.eqflag != 0) != CAP::eq)) return;  // the other class of the pair runs
  const int b = blockIdx.x;
  if (b >= B) return;
  Solver<CAP> S;
  S.bind(prm, smem, io.ws, threadIdx.x, b);
  solve_one<CAP>(S, prm, io, b);
}

// K-step closed loop per scenario in ONE launch (Python/NMPC_TT.py:348-402 main loop):
// solve, record (x0, u0, f, status, iters), then shift_timestep (:13-30) -- each wave
// advances its own scenario, so no step waits for another scenario's slowest solve.
struct Loop {
  int K;
  double* p;          // np x B (ld_p), advanced in place
  long long ld_p;
  double* w;          // nw x B warm start, in/out (holds the shifted last solution on exit)
  const double *vt, *wt;             // target (v, w) for step k, scenario b: [k * ld_tk + b * ld_tb]
  long long ld_tk, ld_tb;
  double *u_hist, *x_hist, *f_hist;  // K x B x 6, K x B x 8, K x B (nullable)
  double* fov_hist;                  // K x B FOV-centre error (Python/NMPC_TT.py:397-400,433-437)
  const double* pstep;               // K x np parameter increments after each step (nullable)
  long long ld_ps;
  int *st_hist, *it_hist;            // K x B (nullable)
  const int* order;                  // dispatch order: workgroup g runs scenario order[g] (nullable)
  int* done;                         // B: steps completed per scenario (completion guard; nullable)
  unsigned long long* times;         // diagnostics (NMPC_STEP_TIMES): K x B x {start, end, XCC_ID|wave<<8}
};

// One closed-loop step k of scenario b (Python/NMPC_TT.py:348-402 main loop body):
// solve with the warm start w and p, record (x0, u0, f, status, iters), then
// shift_timestep (:13-30).  Everything it reads comes from global memory, so any
// wavefront can run any (scenario, step) once step k-1 of that scenario is done.
template <class CAP>
__device__ __forceinline__ int cl_step(const Params* __restrict__ prm, int B, const IO& io, const Loop& lp,
                                       const int b, const int k, double* smem) {
  // caller layout (external): w = nwE = nuE*N decisions, p = [x0(nxE); xs(3); ...]
  const int nw = prm->nwE, nu = prm->nuE, nx = prm->nxE;
  const double T = prm->T;
  double* wb = lp.w + (long long)b * nw;
  double* pb = lp.p + (long long)b * lp.ld_p;
  constexpr int WR = (6 * CAP::nmax + WAVE - 1) / WAVE;
  // a fresh solver per step: no member is live across steps (a solver kept
  // outside the loop costs ~40 VGPRs of spills)
  Solver<CAP> S;
  S.bind(prm, smem, io.ws, threadIdx.x, b);
  IO ik = io;
  ik.x0 = lp.w; ik.ld_x0 = nw; ik.x_out = lp.w;
  ik.p = lp.p; ik.ld_p = lp.ld_p;
  const long long kb = (long long)k * B;
  ik.f_out = lp.f_hist ? lp.f_hist + kb : nullptr;
  ik.status = lp.st_hist ? lp.st_hist + kb : nullptr;
  ik.iters = lp.it_hist ? lp.it_hist + kb : nullptr;
  const int iters = solve_one<CAP>(S, prm, ik, b);
  sync();
  // shift_timestep: read the solution and the state before anything is overwritten
  const int l = S.lanef();
  double wn[WR];
#pragma unroll
  for (int j = 0; j < WR; ++j) {
    const int i = l + j * WAVE;
    wn[j] = i < nw ? wb[i + nu < nw ? i + nu : i] : 0.0;
  }
  const int npar = prm->npE;
  double pv = l < npar ? pb[l] : 0.0;
  const double u0 = l < nu ? wb[l] : 0.0;
  // histories keep the gimbal model's widths (8 states, 6 controls); an absent
  // state / control of the no-gimbal model is recorded as 0
  if (lp.x_hist && l < 8) lp.x_hist[(kb + b) * 8 + l] = l < nx ? pv : 0.0;
  if (lp.u_hist && l < 6) lp.u_hist[(kb + b) * 6 + l] = u0;
  const double th = readlane_d(pv, 3), ps = readlane_d(pv, 4), xs2 = readlane_d(pv, nx + 2);
  const double v = readlane_d(u0, 0);
  // x0 <- x0 + T f(x0, u0): [v c(psi) c(th), v s(psi) c(th), v s(th), u1..u(nx-3)]
  const double ush = __shfl(u0, l >= 3 && l < nx ? l - 2 : 0, WAVE);
  double fx = 0.0;
  if (l == 0) fx = v * cos(ps) * cos(th);
  else if (l == 1) fx = v * sin(ps) * cos(th);
  else if (l == 2) fx = v * sin(th);
  else if (l < nx) fx = ush;
  else if (l == nx) fx = lp.vt[k * lp.ld_tk + b * lp.ld_tb] * cos(xs2);
  else if (l == nx + 1) fx = lp.vt[k * lp.ld_tk + b * lp.ld_tb] * sin(xs2);
  else if (l == nx + 2) fx = lp.wt[k * lp.ld_tk + b * lp.ld_tb];
  sync();
  const double pnew = pv + T * fx;
  if (l < nx + 3) pb[l] = pnew;
  else if (l < npar && lp.pstep) pb[l] = pv + lp.pstep[k * lp.ld_ps + l];  // moving obstacles etc.
  if (lp.fov_hist) {
    // FOV centre of the new state vs the target before its step; without a gimbal
    // (x5 = x6 = 0) it is the UAV's ground position (x, y)
    const double x1 = readlane_d(pnew, 0), y1 = readlane_d(pnew, 1), z1 = readlane_d(pnew, 2);
    const double g5 = nx > 5 ? readlane_d(pnew, 5) : 0.0, g6 = nx > 5 ? readlane_d(pnew, 6) : 0.0;
    const double xt = readlane_d(pv, nx), yt = readlane_d(pv, nx + 1);
    const double hv = prm->hv, hh = prm->hh;
    const double ap = (z1 * tan(g6 + hv) - z1 * tan(g6 - hv)) / 2;
    const double bp = (z1 * tan(g5 + hh) - z1 * tan(g5 - hh)) / 2;
    const double xe = x1 + ap + z1 * tan(g6 - hv), ye = y1 + bp + z1 * tan(g5 - hh);
    if (l == 0) lp.fov_hist[kb + b] = sqrt((xe - xt) * (xe - xt) + (ye - yt) * (ye - yt));
  }
#pragma unroll
  for (int j = 0; j < WR; ++j) {
    const int i = l + j * WAVE;
    if (i < nw) wb[i] = wn[j];
  }
  sync();
  return iters;
}

// K-step closed loop, one workgroup per scenario running its K steps back to back.
template <class CAP>
__global__ __launch_bounds__(WAVE, CAP::wpe) void nmpc_closed_loop_kernel(const Params* __restrict__ prm, int B, IO io,
                                                                    Loop lp) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if (io.eqflag && ((*io.eqflag != 0) != CAP::eq)) return;  // the other class of the pair runs
  // workgroups start roughly in blockIdx order, so a caller-supplied permutation sets
  // the order in which scenarios begin (an out-of-range entry is skipped)
  const int b = lp.order ? lp.order[blockIdx.x] : (int)blockIdx.x;
  if (b < 0 || b >= B) return;
  for (int k = 0; k < lp.K; ++k) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    cl_step<CAP>(prm, B, io, lp, b, k, smem);
    if (lp.times && threadIdx.x == 0) {
      unsigned long long* t = lp.times + ((long long)k * B + b) * 3;
      t[0] = t0; t[1] = __builtin_amdgcn_s_memrealtime();
      t[2] = (unsigned long long)blockIdx.x << 8 | (__builtin_amdgcn_s_memtime() - c0) << 24;  // + shader cycles
    }
    // completion guard (nmpc_sched_check_kernel): a duplicated or missing dispatch
    // entry leaves some scenario short of its K steps, which the check reports
    if (lp.done && threadIdx.x == 0) lp.done[b] = k + 1;
  }
}

// ---- step-queue scheduler for the K-step closed loop (persistent waves)
// A launch is bounded by its longest scenario chain (K steps of up to max_iter
// iterations each).  With more scenarios than resident waves, a long chain that only
// starts after the first wave of slots has drained finishes last, and which chains
// will be long is hard to predict.  Here every resident wave repeatedly claims the next
// (scenario, step) whose previous step is done, lowest step index first: a scenario
// that has fallen behind (a long chain) is served as soon as its previous step ends,
// so the launch approaches its longest chain without knowing it in advance.
//  * Queue (x, j) receives each scenario of XCD set x exactly once, when its step j-1
//    is done; queue (x, 0) is the dispatch order.  Every queue exists twice: a step
//    whose predecessor took >= hot_iters iterations (max_iter / 2 by default) is
//    published to the "hot" family, which is served first (lowest step first), then
//    the normal family (lowest step first).  A scenario that turns locally infeasible
//    late in its K steps (long steps from then on) would otherwise wait behind the
//    short steps of scenarios at lower step indices while every wave is busy
//    (measured: up to 114 ms of a 359 ms launch, scripts/step_times.py).  Scenarios are pinned to an XCD
//    (set x = dispatch position mod NXCD) and served only by waves running on that XCD
//    (hardware register XCC_ID): the per-XCD L2s are not coherent with each other, so
//    a scenario's state (p, w, histories) is only ever handed between waves sharing
//    an L2, through agent-scope release / acquire fences.
//  * Claims and publishes are agent-scope atomics by lane 0.
//  * Exit: a wave leaves as soon as nothing in its set is claimable: every unfinished
//    scenario is then running on some wave, and each publisher claims again right
//    after publishing, so no published step is left without a live wave and no wave
//    spins.  A claimed slot always has a running writer, so waiting for its store is
//    short; a wave that waits longer than kSchedWaitTicks anyway sets err and leaves.
constexpr int NXCD = 8;  // MI355X: 8 XCDs
struct SchedQ {
  int* head;  // 2 x NXCD x K: claimed count of queue (family, x, j); family 0 normal, 1 hot
  int* tail;  // 2 x NXCD x K: published count
  int* resv;  // 2 x NXCD x K: reserved count
  int* ring;  // 2 x NXCD x K x BX scenario ids (-1 = not yet written)
  int* err;   // [0]: 1 a wave gave up waiting, 2 a scenario did not complete its K steps
  unsigned long long* ndone;  // closed-loop steps completed (nmpc_sched_check_kernel; 64-bit: B*K may exceed 2^31)
  int* done;  // B: steps completed per scenario
  int BX;     // ring capacity per queue = ceil(B / NXCD)
  int one_set;  // test hook (NMPC_SCHED_TEST_ONE_SET): only the waves on XCD 0 run, so
                // sets 1..7 are never drained and the check must report it
  int hot_iters;  // a step after one with >= hot_iters iterations goes to the hot family (0: none)
  const int* eqnows;  // the equality gate flag when the equality class was not launched (nullable)
};
constexpr unsigned long long kSchedWaitTicks = 1000000000ull;  // s_memrealtime (100 MHz): 10 s

// polling loads: relaxed (no L1 invalidation per poll); the claim is followed by one
// acquire fence.  A scenario never leaves its XCD, so its state only has to reach the
// XCD's L2: the writer waits for its stores (vmcnt(0), L1 is write-through) before
// publishing, the reader invalidates its L1 after claiming.  No L2 write-back
// (an agent-scope release fence flushes the whole L2: measured 20x slower).
__device__ __forceinline__ int ld_acq(int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ int xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return (int)(x % NXCD);
}

template <class CAP>
__global__ __launch_bounds__(WAVE, CAP::wpe) void nmpc_closed_loop_sched_kernel(const Params* __restrict__ prm, int B,
                                                                          IO io, Loop lp, SchedQ q) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if (io.eqflag && ((*io.eqflag != 0) != CAP::eq)) return;  // the other class of the pair runs
  const int K = lp.K;
  const int x = xcc_id();
  if (q.one_set && x != 0) return;  // test hook: only XCD 0's waves run (sets 1..7 unserved)
  const int nset = (B - x + NXCD - 1) / NXCD;  // scenarios in this XCD's set
  // family f = 0 (normal) / 1 (hot) of queue (x, j): counters at [(f * NXCD + x) * K + j]
  const long long fo = (long long)NXCD * K;
  int* head = q.head + x * K;
  int* tail = q.tail + x * K;
  int* resv = q.resv + x * K;
  int* ring = q.ring + (long long)x * K * q.BX;
  const long long ro = fo * q.BX;  // ring offset of the hot family
  int jmin = 0;
  for (;;) {
    int cb = -1, ck = -1;
    if (threadIdx.x == 0) {
      // Hot queues first, then normal ones, each lowest step first.  Finding nothing to
      // claim means every unfinished scenario of the set is running on some wave, so
      // this wave is surplus from now on (the unfinished count only shrinks, and every
      // publisher claims again right after publishing): it exits instead of spinning.
      bool claimed = false;
      for (int f = 1; f >= 0 && !claimed; --f) {
        int* hd = head + f * fo;
        int* tl = tail + f * fo;
        int* rg = ring + f * ro;
        for (int j = jmin; j < K; ++j) {
          const int h = ld_acq(hd + j);
          if (f == 0 && h + ld_acq(head + fo + j) >= nset) {  // every scenario has passed queue j
            if (j == jmin) ++jmin;
            continue;
          }
          if (h >= ld_acq(tl + j)) continue;  // nothing published in this queue yet
          int e = h;
          if (!__hip_atomic_compare_exchange_strong(hd + j, &e, h + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)) {
            --j;  // lost the race for this queue: look at it again
            continue;
          }
          // published count > h: slot h's writer has reserved it and stores it next
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          int v = ld_acq(rg + (long long)j * q.BX + h);
          while (v < 0 && __builtin_amdgcn_s_memrealtime() - t0 < kSchedWaitTicks) {
            __builtin_amdgcn_s_sleep(2);
            v = ld_acq(rg + (long long)j * q.BX + h);
          }
          if (v < 0) __hip_atomic_store(q.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else { cb = v; ck = j; }
          claimed = true;
          break;
        }
      }
    }
    cb = __builtin_amdgcn_readfirstlane(cb);
    ck = __builtin_amdgcn_readfirstlane(ck);
    if (ck < 0) break;
    int its = 0;
    if (cb >= 0 && cb < B) {  // an out-of-range dispatch entry is claimed and skipped
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the previous step's p, w (L1 invalidated)
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
      its = cl_step<CAP>(prm, B, io, lp, cb, ck, smem);
      if (lp.times && threadIdx.x == 0) {
        unsigned long long* t = lp.times + ((long long)ck * B + cb) * 3;
        t[0] = t0; t[1] = __builtin_amdgcn_s_memrealtime();
        // XCC_ID | workgroup << 8 | shader-clock cycles of the step << 24 (effective clock)
        t[2] = (unsigned long long)(x | (blockIdx.x << 8)) | (__builtin_amdgcn_s_memtime() - c0) << 24;
      }
      if (threadIdx.x == 0) q.done[cb] = ck + 1;
      stores_done();  // this step's p, w, histories are in the XCD's L2
    }
    if (threadIdx.x == 0 && ck + 1 < K) {
      const int j = ck + 1;
      const int f = (q.hot_iters > 0 && its >= q.hot_iters) ? 1 : 0;
      const int pos = __hip_atomic_fetch_add(resv + f * fo + j, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (pos < q.BX) {
        __hip_atomic_store(ring + f * ro + (long long)j * q.BX + pos, cb, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        stores_done();
        __hip_atomic_fetch_add(tail + f * fo + j, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

#ifndef NMPC_TU_CLASS  // host translation unit: the small non-template kernels and the C-ABI
// queue (x, 0) = the set-x entries of the dispatch order (identity or the caller's
// permutation); every other queue empty
__global__ void nmpc_sched_init_kernel(int B, int K, const int* order, SchedQ q) {
  const long long n = (long long)NXCD * K * q.BX;  // one family's ring
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) q.ring[n + i] = -1;  // hot family: empty
  if (i < (long long)NXCD * K) {  // hot family counters
    q.head[NXCD * K + i] = 0; q.tail[NXCD * K + i] = 0; q.resv[NXCD * K + i] = 0;
  }
  if (i < n) {
    const int x = (int)(i / ((long long)K * q.BX));
    const long long r = i - (long long)x * K * q.BX;
    const int j = (int)(r / q.BX), c = (int)(r - (long long)j * q.BX);
    int v = -1;
    const long long pos = (long long)c * NXCD + x;  // dispatch position
    if (j == 0 && pos < B) {
      v = order ? order[pos] : (int)pos;
      if (v < 0 || v >= B) v = B;  // out-of-range entry: claimed, then skipped
    }
    q.ring[i] = v;
  }
  if (i < (long long)NXCD * K) {
    const int x = (int)(i / K), j = (int)(i - (long long)x * K);
    const int nset = (B - x + NXCD - 1) / NXCD;
    q.head[i] = 0;
    q.tail[i] = j == 0 ? nset : 0;
    q.resv[i] = j == 0 ? nset : 0;
  }
  if (i == 0) { q.err[0] = 0; *q.ndone = 0; }
  if (i < B) q.done[i] = 0;
}

// equality-row gate: flag = 1 if any scenario has a row with lbg == ubg (finite), the
// test solve_one's equality class applies; the flag is zeroed before on the same stream
__global__ void nmpc_eq_scan_kernel(long long n, int ng, const double* lbg, long long ld_lbg, const double* ubg,
                                    long long ld_ubg, int* flag) {
  bool eq = false;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / ng, r = i - b * ng;
    const double lo = lbg[b * ld_lbg + r], hi = ubg[b * ld_ubg + r];
    eq = eq || (lo == hi && lo > -BIGB);
  }
  if (eq) *flag = 1;
}

// a device-pointer solve whose batch has equality rows while the equality class's
// workspace is not reserved (nmpc_reserve_eq): neither class of the pair ran, so every
// scenario reports NMPC_STATUS_EQ_UNRESERVED (IPOPT Insufficient_Memory) with a NaN
// objective and solution (no-op when the flag is 0: the problem's class ran)
__global__ void nmpc_eq_unreserved_kernel(int B, const int* flag, int nw, double* x_out, double* f_out,
                                          int* status, int* iters) {
  if (*flag == 0) return;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double nan = __builtin_nan("");
  if (status) status[b] = NMPC_STATUS_EQ_UNRESERVED;
  if (iters) iters[b] = 0;
  if (f_out) f_out[b] = nan;
  for (int i = 0; i < nw; ++i) x_out[(long long)b * nw + i] = nan;
}

// completion-guard state of a one-workgroup-per-scenario launch (no queues)
__global__ void nmpc_guard_init_kernel(int B, SchedQ q) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) { q.err[0] = 0; *q.ndone = 0; }
  if (i < B) q.done[i] = 0;
}

// After a closed-loop launch (same stream, either policy): every scenario must have
// completed its K steps (Python/NMPC_TT.py:348-402 advances every scenario K times).
// A scenario that did not sets err[0] |= 2, and its unrun steps are marked in every
// history (status / iterations NMPC_STATUS_NOT_RUN; f, fov, u, x NaN) so nothing is
// left uninitialised.
// A batch with equality rows whose equality class was not launched (its workspace not
// reserved, nmpc_reserve_eq; q.eqnows = the gate flag) ran no step: err |= 4 as well, and
// the steps carry NMPC_STATUS_EQ_UNRESERVED instead of NMPC_STATUS_NOT_RUN.
__global__ void nmpc_sched_check_kernel(int B, int K, SchedQ q, const Loop lp) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int d = q.done[b];
  atomicAdd(q.ndone, (unsigned long long)(d < 0 ? 0 : d));
  if (d == K) return;
  const bool nows = q.eqnows && *q.eqnows != 0;
  atomicOr(q.err, nows ? 6 : 2);
  const int code = nows ? NMPC_STATUS_EQ_UNRESERVED : NMPC_STATUS_NOT_RUN;
  const double nan = __builtin_nan("");
  for (int k = d < 0 ? 0 : d; k < K; ++k) {
    const long long kb = (long long)k * B + b;
    if (lp.st_hist) lp.st_hist[kb] = code;
    if (lp.it_hist) lp.it_hist[kb] = code;
    if (lp.f_hist) lp.f_hist[kb] = nan;
    if (lp.fov_hist) lp.fov_hist[kb] = nan;
    if (lp.u_hist)
      for (int c = 0; c < 6; ++c) lp.u_hist[kb * 6 + c] = nan;
    if (lp.x_hist)
      for (int c = 0; c < 8; ++c) lp.x_hist[kb * 8 + c] = nan;
  }
}

// closed-loop shift kernel (Python/NMPC_TT.py:13-30): one thread per scenario
// nx / nu: the model's (external) state / control counts, 8 / 6 with gimbal,
// 5 / 3 without (MATLAB/Dynamic Obstacles/shift1.m: the same step on [x0(5); xs(3)])
__global__ void nmpc_shift_kernel(int B, int N, int nx, int nu, double T, double* p, long long ld_p,
                                  const double* u, double* w_out, const double* vt, const double* wt) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double* pb = p + (long long)b * ld_p;
  const double* ub = u + (long long)b * nu * N;
  const double th = pb[3], ps = pb[4], v = ub[0];
  const double f0 = v * cos(ps) * cos(th), f1 = v * sin(ps) * cos(th), f2 = v * sin(th);
  pb[0] = pb[0] + T * f0; pb[1] = pb[1] + T * f1; pb[2] = pb[2] + T * f2;
  for (int c = 3; c < nx; ++c) pb[c] = pb[c] + T * ub[c - 2];
  double* wb = w_out + (long long)b * nu * N;
  for (int k = 0; k < N; ++k) {
    const int src = (k + 1 < N) ? k + 1 : N - 1;
    for (int c = 0; c < nu; ++c) wb[k * nu + c] = ub[src * nu + c];
  }
  const double xs2 = pb[nx + 2];
  const double vv = vt[b], ww = wt[b];
  pb[nx] = pb[nx] + T * (vv * cos(xs2));
  pb[nx + 1] = pb[nx + 1] + T * (vv * sin(xs2));
  pb[nx + 2] = pb[nx + 2] + T * ww;
}

// ------------------------------------------------------------------ host side
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#endif  // !NMPC_TU_CLASS

}  // namespace nmpc_impl
using namespace nmpc_impl;

typedef void (*KernFn)(const Params*, int, IO);
typedef void (*LoopFn)(const Params*, int, IO, Loop);
typedef void (*SchedFn)(const Params*, int, IO, Loop, SchedQ);
// the kernels of one capacity class (defined in that class's translation unit)
struct ClassFns {
  KernFn fn; LoopFn lfn; SchedFn sfn;
  int lds_doubles, ws_doubles;
};
ClassFns nmpc_class_fns_A();
ClassFns nmpc_class_fns_B();
ClassFns nmpc_class_fns_C();
ClassFns nmpc_class_fns_A32();
ClassFns nmpc_class_fns_C32();
ClassFns nmpc_class_fns_D();
ClassFns nmpc_class_fns_E();

using CapA = Cap<20, 15, true>;   // BASELINE configs 2-4 (N=20, <=10 obstacles) and the reference's N=15 scripts
using CapB = Cap<31, 21>;
using CapC = Cap<63, 21>;   // any supported shape
// BASELINE config 5 (N = 50, 10 obstacles): global rows, row bounds and k_k, 25.6 KB of
// LDS per scenario, so 6 scenarios per CU (round 3: 57 KB allowed 2, then 29 KB 5)
using CapD = Cap<50, 15>;
static_assert(CapD::L.total * 8 <= 163840 / 6, "config 5's class no longer fits 6 scenarios per CU");
// fp32 Riccati factorisation (nmpc_options.linear_solver_fp32; BASELINE config 5's fp32 leg)
using CapA32 = Cap<20, 15, true, float>;
// the LDS-row classes run four scenarios per CU (160 KB of LDS): one wave per SIMD
static_assert(CapA::L.total * 8 <= 40960 && CapA32::L.total * 8 <= 40960, "LDS-row class exceeds a quarter CU");
using CapC32 = Cap<63, 21, false, float>;
// equality rows (lbg == ubg): any supported shape, global rows, the Schur-complement step
// compiled in.  Launched paired with the problem's own class behind IO::eqflag.
using CapE = Cap<63, 21, false, double, true>;

#ifdef NMPC_TU_CLASS
template <class CAP>
static ClassFns class_fns() {
  return {nmpc_solve_kernel<CAP>, nmpc_closed_loop_kernel<CAP>, nmpc_closed_loop_sched_kernel<CAP>, CAP::L.total,
          CAP::L.wstotal};
}
#if NMPC_TU_CLASS == 1
ClassFns nmpc_class_fns_A() { return class_fns<CapA>(); }
#elif NMPC_TU_CLASS == 2
ClassFns nmpc_class_fns_B() { return class_fns<CapB>(); }
#elif NMPC_TU_CLASS == 3
ClassFns nmpc_class_fns_C() { return class_fns<CapC>(); }
#elif NMPC_TU_CLASS == 4
ClassFns nmpc_class_fns_A32() { return class_fns<CapA32>(); }
#elif NMPC_TU_CLASS == 5
ClassFns nmpc_class_fns_C32() { return class_fns<CapC32>(); }
#elif NMPC_TU_CLASS == 6
ClassFns nmpc_class_fns_D() { return class_fns<CapD>(); }
#else
ClassFns nmpc_class_fns_E() { return class_fns<CapE>(); }
#endif
#else  // host translation unit

struct nmpc_handle {
  Params hp;
  Params* dprm = nullptr;
  int device = 0;
  int lds_bytes = 0;
  // staging buffers for the host-pointer API
  double* dbuf = nullptr;
  size_t dbuf_bytes = 0;
  int* ibuf = nullptr;
  size_t ibuf_bytes = 0;
  KernFn kern = nullptr;
  LoopFn loop = nullptr;
  SchedFn sched = nullptr;
  // the equality class, launched paired with the class above behind a device flag
  // (fp64 handles; null for the fp32 leg and when NMPC_FORCE_CLASS=E picks it as the class)
  KernFn kernE = nullptr;
  LoopFn loopE = nullptr;
  SchedFn schedE = nullptr;
  int lds_bytesE = 0;
  int residentE = 0;
  int* deq = nullptr;          // the gate flag (nmpc_eq_scan_kernel)
  // the equality class's own workspace (its layout: global rows up to N = 63 and the
  // 128 x 128 Schur storage, ~840 KB per scenario): allocated only once a batch with
  // equality rows is seen, so handles whose batches have none carry only their class's
  int ws_doublesE = 0;
  double* dwsE = nullptr;
  size_t wsE_bytes = 0;
  int resident = 0;            // closed-loop waves resident at once (occupancy x CUs)
  int* dsched = nullptr;       // step-queue scheduler state
  size_t sched_bytes = 0;
  int nxcc = -1;               // XCDs of the device (hipDeviceAttributeNumberOfXccs)
  int last_policy = 0;         // last closed-loop launch: 0 one workgroup per scenario, 1 step queues
  int last_waves = 0;          // workgroups launched by the last closed-loop launch
  long long last_steps = 0;    // B*K of the last closed-loop launch
  int* last_err = nullptr;     // device flags of the last closed-loop launch (SchedQ::err)
  unsigned long long* last_ndone = nullptr;  // its completed-step counter (SchedQ::ndone)
  hipStream_t last_stream = nullptr;         // the stream it was enqueued on
  unsigned long long* dtimes = nullptr;  // diagnostics: step timestamps of the last closed loop
  size_t times_bytes = 0, times_n = 0;
  int ws_doubles = 0;
  bool trace = false;
  double* dtrace = nullptr;
  double* dws = nullptr;       // per-scenario global workspace
  size_t ws_bytes = 0;
  size_t trace_bytes = 0;
  int last_B = 0;
};



// returns true when NMPC_FORCE_CLASS picked the equality class itself (which then needs
// no partner); any other class, forced or not, is paired with the equality class
static bool pick_class(const Params& P, KernFn* fn, LoopFn* lfn, SchedFn* sfn, int* lds_doubles, int* ws_doubles) {
  bool forcedE = false;
  ClassFns c;
  const bool fit_a = P.N <= CapA::nmax && P.m <= CapA::mmax;
  if (P.o.linear_solver_fp32) c = fit_a ? nmpc_class_fns_A32() : nmpc_class_fns_C32();
  else if (fit_a) c = nmpc_class_fns_A();
  else if (P.N <= CapB::nmax && P.m <= CapB::mmax) c = nmpc_class_fns_B();
  else if (P.N <= CapD::nmax && P.m <= CapD::mmax) c = nmpc_class_fns_D();
  else c = nmpc_class_fns_C();
  // diagnostics: run a fitting problem on a larger class (global row vectors)
  if (const char* e = std::getenv("NMPC_FORCE_CLASS")) {
    if (e[0] == 'B' && P.N <= CapB::nmax && P.m <= CapB::mmax && !P.o.linear_solver_fp32) c = nmpc_class_fns_B();
    if (e[0] == 'C' && !P.o.linear_solver_fp32) c = nmpc_class_fns_C();
    if (e[0] == 'D' && P.N <= CapD::nmax && P.m <= CapD::mmax && !P.o.linear_solver_fp32) c = nmpc_class_fns_D();
    if (e[0] == 'E' && !P.o.linear_solver_fp32) { c = nmpc_class_fns_E(); forcedE = true; }
  }
  *fn = c.fn; *lfn = c.lfn; *sfn = c.sfn; *lds_doubles = c.lds_doubles; *ws_doubles = c.ws_doubles;
  return forcedE;
}

// zero the gate flag and scan the batch's row bounds (stream-ordered before the pair)
static int eq_gate(nmpc_handle* h, int B, const IO& io, hipStream_t st) {
  const int ng = h->hp.ng;
  const long long n = (io.ld_lbg == 0 && io.ld_ubg == 0) ? (long long)ng : (long long)B * ng;
  if (hipMemsetAsync(h->deq, 0, sizeof(int), st) != hipSuccess) return fail(NMPC_E_HIP, "hipMemsetAsync gate");
  const int thr = 256;
  const long long blocks = (n + thr - 1) / thr;
  hipLaunchKernelGGL(nmpc_eq_scan_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(thr), 0, st, n, ng,
                     io.lbg, io.ld_lbg, io.ubg, io.ld_ubg, h->deq);
  return NMPC_OK;
}

static int ensure_buf(double** buf, size_t* bytes, size_t need, const char* what) {
  if (need > *bytes) {
    if (*buf) hipFree(*buf);
    *buf = nullptr; *bytes = 0;
    if (hipMalloc(buf, need) != hipSuccess) return fail(NMPC_E_NOMEM, std::string("hipMalloc ") + what);
    *bytes = need;
  }
  return NMPC_OK;
}
static int ensure_ws(nmpc_handle* h, int B) {
  return ensure_buf(&h->dws, &h->ws_bytes, (size_t)B * h->ws_doubles * sizeof(double), "workspace");
}

// Which kernels of the class pair a launch runs.  The equality class's workspace (~850 KB
// per scenario) is allocated only when needed:
//  * host pointers (nmpc_solve_batch, host_eq 0 / 1): the host has scanned the bounds, so
//    exactly the class that applies is launched, and an equality batch allocates the
//    equality workspace first;
//  * device pointers (the _dev entry points, host_eq -1): never a host round trip.  The
//    bounds are scanned on the device and the pair is enqueued behind the device flag.  If
//    the equality workspace does not cover B (nmpc_reserve_eq was not called for this B),
//    the equality class is not launched; a batch that has equality rows then reports
//    NMPC_STATUS_EQ_UNRESERVED per scenario instead of running (run->Enows: the solve's
//    marker kernel / the closed loop's completion check write it).
struct Run { bool A, E, Enows; };
static int eq_prepare(nmpc_handle* h, int B, IO& io, IO& ioE, hipStream_t st, int host_eq, Run* run) {
  ioE = io;
  io.eqflag = nullptr; ioE.eqflag = nullptr;
  run->A = true; run->E = false; run->Enows = false;
  if (!h->kernE) return NMPC_OK;  // fp32 leg, or NMPC_FORCE_CLASS=E: one class, no partner
  const size_t needE = (size_t)B * h->ws_doublesE * sizeof(double);
  if (host_eq >= 0) {  // known: launch the one class that applies
    run->A = host_eq == 0; run->E = host_eq == 1;
  } else {  // the gated pair, decided on the device
    if (int rc = eq_gate(h, B, io, st)) return rc;
    io.eqflag = h->deq; ioE.eqflag = h->deq;
    run->A = true;
    run->E = needE <= h->wsE_bytes;
    run->Enows = !run->E;
  }
  if (run->E) {
    if (int rc = ensure_buf(&h->dwsE, &h->wsE_bytes, needE, "equality-class workspace")) return rc;
    ioE.ws = h->dwsE;
  }
  return NMPC_OK;
}

// host-pointer bounds: does any scenario have a row with lbg == ubg (finite)?  (the test of
// nmpc_eq_scan_kernel, on the caller's arrays before they are uploaded)
static int host_has_eq(int B, int ng, const double* lbg, int64_t ld_lbg, const double* ubg, int64_t ld_ubg) {
  for (int b = 0; b < B; ++b) {
    const double* lo = lbg + (size_t)b * ld_lbg;
    const double* hi = ubg + (size_t)b * ld_ubg;
    for (int r = 0; r < ng; ++r)
      if (lo[r] == hi[r] && lo[r] > -BIGB) return 1;
    if (ld_lbg == 0 && ld_ubg == 0) break;
  }
  return 0;
}

extern "C" {

void nmpc_default_options(nmpc_options* o) {
  std::memset(o, 0, sizeof(*o));
  o->max_iter = 3000; o->acceptable_iter = 15; o->max_soc = 4; o->max_soft_resto_iters = 10;
  o->watchdog_shortened_iter_trigger = 10; o->watchdog_trial_iter_max = 3;
  o->tol = 1e-8; o->acceptable_tol = 1e-6; o->acceptable_obj_change_tol = 1e20;
  o->acceptable_dual_inf_tol = 1e10; o->acceptable_constr_viol_tol = 1e-2; o->acceptable_compl_inf_tol = 1e-2;
  o->dual_inf_tol = 1.0; o->constr_viol_tol = 1e-4; o->compl_inf_tol = 1e-4;
  o->mu_init = 0.1; o->kappa_mu = 0.2; o->theta_mu = 1.5; o->barrier_tol_factor = 10.0; o->tau_min = 0.99;
  o->bound_push = 1e-2; o->bound_frac = 1e-2; o->slack_bound_push = 1e-2; o->slack_bound_frac = 1e-2;
  o->bound_relax_factor = 1e-8; o->bound_mult_init_val = 1.0; o->constr_mult_init_max = 1e3;
  o->nlp_scaling_max_gradient = 100.0; o->nlp_scaling_min_value = 1e-8; o->kappa_d = 1e-5;
  o->kappa_sigma = 1e10; o->s_max = 100.0;
  o->theta_max_fact = 1e4; o->theta_min_fact = 1e-4; o->gamma_theta = 1e-5; o->gamma_phi = 1e-8;
  o->delta = 1.0; o->s_theta = 1.1; o->s_phi = 2.3; o->eta_phi = 1e-8;
  o->alpha_red_factor = 0.5; o->alpha_min_frac = 0.05; o->kappa_soc = 0.99; o->obj_max_inc = 5.0;
  o->first_hessian_perturbation = 1e-4; o->min_hessian_perturbation = 1e-20; o->max_hessian_perturbation = 1e20;
  o->perturb_inc_fact_first = 100.0; o->perturb_inc_fact = 8.0; o->perturb_dec_fact = 1.0 / 3.0;
  o->tiny_step_tol = 10 * 2.220446049250313e-16; o->soft_resto_pderror_reduction_factor = 0.9999;
  o->resto_penalty_parameter = 1000.0; o->resto_proximity_weight = 1.0; o->required_infeasibility_reduction = 0.9;
  o->bound_mult_reset_threshold = 1000.0; o->constr_mult_reset_threshold = 0.0;
}

const char* nmpc_last_error(void) { return g_err.c_str(); }

int nmpc_closed_loop_times(nmpc_handle* h, uint64_t* host_out, int64_t n) {
  if (!h || !host_out) return fail(NMPC_E_INVALID, "null argument");
  if (!h->dtimes || (size_t)n < h->times_n) return fail(NMPC_E_INVALID, "no step times recorded (NMPC_STEP_TIMES)");
  if (hipMemcpy(host_out, h->dtimes, h->times_n * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(NMPC_E_HIP, "reading step times");
  return NMPC_OK;
}

#ifndef NMPC_SRC_HASH
#define NMPC_SRC_HASH "unknown-unknown-unknown-unknown!"
#endif
// the marker lets the build read the hash back from the binary without loading it
__attribute__((used)) static const char kBuildId[] = "NMPC_SRC_HASH=" NMPC_SRC_HASH;
const char* nmpc_build_id(void) { return kBuildId + 14; }

int nmpc_create(const nmpc_desc* desc, nmpc_handle** out) {
  if (!desc || !out) return fail(NMPC_E_INVALID, "null argument");
  if (desc->model != NMPC_MODEL_UAV8G && desc->model != NMPC_MODEL_UAV5)
    return fail(NMPC_E_INVALID, "unsupported model");
  const bool nog = desc->model == NMPC_MODEL_UAV5;
  const int np_min = nog ? 8 : 11;  // [x0; xs]
  if (desc->N < 1 || desc->N > NMPC_MAX_N) return fail(NMPC_E_INVALID, "N out of range [1,63]");
  if (desc->n_obs < 0 || desc->n_obs > NMPC_MAX_OBS) return fail(NMPC_E_INVALID, "n_obs out of range");
  if (desc->np < np_min || desc->np > 61) return fail(NMPC_E_INVALID, "np out of range [8 or 11, 61]");
  if (!(desc->T > 0)) return fail(NMPC_E_INVALID, "T must be positive");
  if (desc->opts.max_iter < 0 || desc->opts.max_iter > FCAP - 1 + 100000)
    return fail(NMPC_E_INVALID, "bad max_iter");
  for (int j = 0; j < desc->n_obs; ++j) {
    if (desc->obs_x_pidx[j] >= desc->np || desc->obs_y_pidx[j] >= desc->np ||
        (desc->obs_x_pidx[j] >= 0 && desc->obs_x_pidx[j] < np_min) ||
        (desc->obs_y_pidx[j] >= 0 && desc->obs_y_pidx[j] < np_min))
      return fail(NMPC_E_INVALID, "obstacle parameter index must be -1 or in [np_min, np)");
  }
  if (desc->w1_pidx >= desc->np || desc->w2_pidx >= desc->np || desc->w1_pidx < -1 || desc->w2_pidx < -1 ||
      (desc->w1_pidx >= 0 && desc->w1_pidx < np_min) || (desc->w2_pidx >= 0 && desc->w2_pidx < np_min))
    return fail(NMPC_E_INVALID, "weight parameter index must be -1 or in [np_min, np)");
  // parameter indices in the internal (gimbal) layout: [x0(8); xs(3); ...]
  auto pin = [&](int e) { return (e < 0 || !nog) ? e : e + 3; };
  nmpc_handle* h = new nmpc_handle();
  Params& P = h->hp;
  std::memset(&P, 0, sizeof(P));
  P.model = desc->model;
  P.nb = nog ? 2 : 5;                       // box rows per stage: [z, theta] or [z, theta, x5, x6, x7]
  P.nuE = nog ? 3 : 6; P.nxE = nog ? 5 : 8;
  P.N = desc->N; P.nobs = desc->n_obs; P.m = P.nb + desc->n_obs;
  P.npE = desc->np; P.np = desc->np + (nog ? 3 : 0);
  P.nw = 6 * P.N; P.nwE = P.nuE * P.N; P.ng = P.m * (P.N + 1); P.nX = 8 * (P.N + 1);
  // the no-gimbal cost is the distance term alone (MATLAB/Dynamic Obstacles/NMPC_TT.m:102-105)
  P.T = desc->T; P.w1 = desc->w1; P.w2 = nog ? 0.0 : desc->w2; P.hv = desc->vfov / 2; P.hh = desc->hfov / 2;
  P.thv = std::tan(P.hv); P.thh = std::tan(P.hh);
  P.w1p = pin(desc->w1_pidx); P.w2p = nog ? -1 : pin(desc->w2_pidx);
  for (int j = 0; j < NMPC_MAX_OBS; ++j) {
    P.oxp[j] = -1; P.oyp[j] = -1;
  }
  for (int j = 0; j < desc->n_obs; ++j) {
    P.ox[j] = desc->obs_x[j]; P.oy[j] = desc->obs_y[j]; P.orr[j] = desc->obs_rsum[j];
    P.oxp[j] = pin(desc->obs_x_pidx[j]); P.oyp[j] = pin(desc->obs_y_pidx[j]);
  }
  P.o = desc->opts;
  if (const char* e = std::getenv("NMPC_NO_SPEC")) P.nospec = std::atoi(e) != 0;
  {
    int ldsd = 0;
    const bool forcedE = pick_class(P, &h->kern, &h->loop, &h->sched, &ldsd, &h->ws_doubles);
    h->lds_bytes = ldsd * 8;
    if (!P.o.linear_solver_fp32 && !forcedE) {
      const ClassFns ce = nmpc_class_fns_E();
      h->kernE = ce.fn; h->loopE = ce.lfn; h->schedE = ce.sfn; h->lds_bytesE = ce.lds_doubles * 8;
      h->ws_doublesE = ce.ws_doubles;
    }
  }
  if (const char* e = std::getenv("NMPC_LDS_BYTES")) {  // diagnostics: pad LDS to cap workgroups per CU
    const int want = std::atoi(e);
    if (want > h->lds_bytes) h->lds_bytes = want;
  }
  if (h->lds_bytes > 160 * 1024) {
    delete h;
    return fail(NMPC_E_INVALID, "problem too large for the LDS-resident kernel (N*(5+n_obs) too big)");
  }
  if (hipGetDevice(&h->device) != hipSuccess) { delete h; return fail(NMPC_E_HIP, "hipGetDevice failed"); }
  if (hipMalloc(&h->dprm, sizeof(Params)) != hipSuccess) { delete h; return fail(NMPC_E_NOMEM, "hipMalloc params"); }
  if (hipMemcpy(h->dprm, &P, sizeof(Params), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(h->dprm); delete h; return fail(NMPC_E_HIP, "hipMemcpy params");
  }
  if (hipFuncSetAttribute((const void*)h->kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                          h->lds_bytes) != hipSuccess ||
      hipFuncSetAttribute((const void*)h->loop, hipFuncAttributeMaxDynamicSharedMemorySize,
                          h->lds_bytes) != hipSuccess ||
      hipFuncSetAttribute((const void*)h->sched, hipFuncAttributeMaxDynamicSharedMemorySize,
                          h->lds_bytes) != hipSuccess) {
    hipFree(h->dprm); delete h; return fail(NMPC_E_HIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  }
  if (h->kernE) {
    if (hipFuncSetAttribute((const void*)h->kernE, hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytesE) != hipSuccess ||
        hipFuncSetAttribute((const void*)h->loopE, hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytesE) != hipSuccess ||
        hipFuncSetAttribute((const void*)h->schedE, hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytesE) != hipSuccess) {
      hipFree(h->dprm); delete h; return fail(NMPC_E_HIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize), equality class");
    }
    if (hipMalloc(&h->deq, sizeof(int)) != hipSuccess) {
      hipFree(h->dprm); delete h; return fail(NMPC_E_NOMEM, "hipMalloc gate flag");
    }
  }
  *out = h;
  return NMPC_OK;
}

int nmpc_closed_loop_info(nmpc_handle* h, int32_t* policy, int32_t* resident, int32_t* sched_err,
                          int32_t* waves, int64_t* steps_done) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (policy) *policy = h->last_policy;
  if (resident) *resident = h->resident;
  if (waves) *waves = h->last_waves;
  if ((sched_err || steps_done) && h->last_err) {
    // the flags are written by kernels on the launch's stream: wait for that stream
    // (a non-blocking stream does not synchronise with the null stream's memcpy)
    if (hipStreamSynchronize(h->last_stream) != hipSuccess)
      return fail(NMPC_E_HIP, "synchronising the closed-loop stream");
    int e = 0;
    unsigned long long nd = 0;
    if (hipMemcpy(&e, h->last_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&nd, h->last_ndone, sizeof(nd), hipMemcpyDeviceToHost) != hipSuccess)
      return fail(NMPC_E_HIP, "reading the scheduler flags");
    if (sched_err) *sched_err = e;
    if (steps_done) *steps_done = (int64_t)nd;
  } else {
    if (sched_err) *sched_err = 0;
    if (steps_done) *steps_done = 0;
  }
  return NMPC_OK;
}

int nmpc_destroy(nmpc_handle* h) {
  if (!h) return NMPC_OK;
  if (h->dprm) hipFree(h->dprm);
  if (h->dbuf) hipFree(h->dbuf);
  if (h->ibuf) hipFree(h->ibuf);
  if (h->dtrace) hipFree(h->dtrace);
  if (h->dws) hipFree(h->dws);
  if (h->dwsE) hipFree(h->dwsE);
  if (h->dsched) hipFree(h->dsched);
  if (h->dtimes) hipFree(h->dtimes);
  if (h->deq) hipFree(h->deq);
  delete h;
  return NMPC_OK;
}

int nmpc_dims(const nmpc_handle* h, int32_t* nw, int32_t* ng, int32_t* np, int32_t* nX) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (nw) *nw = h->hp.nwE;
  if (ng) *ng = h->hp.ng;
  if (np) *np = h->hp.npE;
  if (nX) *nX = h->hp.nxE * (h->hp.N + 1);
  return NMPC_OK;
}

int nmpc_kernel_info(const nmpc_handle* h, int32_t* lds_bytes, int32_t* tps) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (lds_bytes) *lds_bytes = h->lds_bytes;
  if (tps) *tps = WAVE;
  return NMPC_OK;
}

int nmpc_memory_info(const nmpc_handle* h, int64_t* ws_bytes, int64_t* ws_eq_bytes, int64_t* ws_per_scenario,
                     int64_t* wsE_per_scenario) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (ws_bytes) *ws_bytes = (int64_t)h->ws_bytes;
  if (ws_eq_bytes) *ws_eq_bytes = (int64_t)h->wsE_bytes;
  if (ws_per_scenario) *ws_per_scenario = (int64_t)h->ws_doubles * 8;
  if (wsE_per_scenario) *wsE_per_scenario = (int64_t)h->ws_doublesE * 8;
  return NMPC_OK;
}

int nmpc_reserve_eq(nmpc_handle* h, int32_t B) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (B < 0) return fail(NMPC_E_INVALID, "B < 0");
  if (!h->kernE || B == 0) return NMPC_OK;  // fp32 leg: equality rows report -11 anyway
  return ensure_buf(&h->dwsE, &h->wsE_bytes, (size_t)B * h->ws_doublesE * sizeof(double),
                    "equality-class workspace");
}

int nmpc_set_trace(nmpc_handle* h, int32_t enable) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  h->trace = enable != 0;
  return NMPC_OK;
}

int nmpc_read_trace(nmpc_handle* h, int32_t B, double* host_out) {
  if (!h || !host_out) return fail(NMPC_E_INVALID, "null argument");
  if (!h->dtrace || B > h->last_B) return fail(NMPC_E_INVALID, "no trace recorded for that batch");
  const size_t n = (size_t)B * (h->hp.o.max_iter + 3) * TRACE_F;
  if (hipMemcpy(host_out, h->dtrace, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(NMPC_E_HIP, "hipMemcpy trace");
  return NMPC_OK;
}

static int solve_dev(nmpc_handle* h, int32_t B, const double* x0, int64_t ld_x0, const double* lbx,
                     int64_t ld_lbx, const double* ubx, int64_t ld_ubx, const double* lbg, int64_t ld_lbg,
                     const double* ubg, int64_t ld_ubg, const double* p, int64_t ld_p, double* x_out,
                     double* f_out, double* g_out, double* lam_x_out, double* lam_g_out, double* lam_p_out,
                     double* X_out, int32_t* status, int32_t* iters, void* stream, int host_eq) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (B < 0) return fail(NMPC_E_INVALID, "B < 0");
  if (B == 0) return NMPC_OK;
  if (!x0 || !lbx || !ubx || !lbg || !ubg || !p || !x_out)
    return fail(NMPC_E_INVALID, "required pointer is null");
  const Params& P = h->hp;
  if ((ld_x0 != 0 && ld_x0 < P.nwE) || (ld_lbx != 0 && ld_lbx < P.nwE) || (ld_ubx != 0 && ld_ubx < P.nwE) ||
      (ld_lbg != 0 && ld_lbg < P.ng) || (ld_ubg != 0 && ld_ubg < P.ng) || (ld_p != 0 && ld_p < P.npE))
    return fail(NMPC_E_INVALID, "leading dimension smaller than the vector length");
  IO io;
  io.x0 = x0; io.lbx = lbx; io.ubx = ubx; io.lbg = lbg; io.ubg = ubg; io.p = p;
  io.ld_x0 = ld_x0; io.ld_lbx = ld_lbx; io.ld_ubx = ld_ubx; io.ld_lbg = ld_lbg; io.ld_ubg = ld_ubg; io.ld_p = ld_p;
  io.x_out = x_out; io.f_out = f_out; io.g_out = g_out; io.lam_x = lam_x_out; io.lam_g = lam_g_out;
  io.lam_p = lam_p_out;
  io.X_out = X_out; io.status = status; io.iters = iters; io.trace = nullptr;
  if (h->trace) {
    const size_t need = (size_t)B * (P.o.max_iter + 3) * TRACE_F * sizeof(double);
    if (need > h->trace_bytes) {
      if (h->dtrace) hipFree(h->dtrace);
      h->dtrace = nullptr; h->trace_bytes = 0;
      if (hipMalloc(&h->dtrace, need) != hipSuccess) return fail(NMPC_E_NOMEM, "hipMalloc trace");
      h->trace_bytes = need;
    }
    hipMemsetAsync(h->dtrace, 0, need, (hipStream_t)stream);
    io.trace = h->dtrace;
  }
  if (int rc = ensure_ws(h, B)) return rc;
  io.ws = h->dws;
  h->last_B = B;
  IO ioE;
  Run run;
  if (int rc = eq_prepare(h, B, io, ioE, (hipStream_t)stream, host_eq, &run)) return rc;
  if (run.A)
    hipLaunchKernelGGL(h->kern, dim3(B), dim3(WAVE), h->lds_bytes, (hipStream_t)stream,
                       (const Params*)h->dprm, (int)B, io);
  if (run.E)
    hipLaunchKernelGGL(h->kernE, dim3(B), dim3(WAVE), h->lds_bytesE, (hipStream_t)stream,
                       (const Params*)h->dprm, (int)B, ioE);
  if (run.Enows)
    hipLaunchKernelGGL(nmpc_eq_unreserved_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, (int)B,
                       (const int*)h->deq, P.nwE, x_out, f_out, status, iters);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NMPC_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return NMPC_OK;
}

int nmpc_solve_batch_dev(nmpc_handle* h, int32_t B, const double* x0, int64_t ld_x0, const double* lbx,
                         int64_t ld_lbx, const double* ubx, int64_t ld_ubx, const double* lbg, int64_t ld_lbg,
                         const double* ubg, int64_t ld_ubg, const double* p, int64_t ld_p, double* x_out,
                         double* f_out, double* g_out, double* lam_x_out, double* lam_g_out, double* lam_p_out,
                         double* X_out, int32_t* status, int32_t* iters, void* stream) {
  return solve_dev(h, B, x0, ld_x0, lbx, ld_lbx, ubx, ld_ubx, lbg, ld_lbg, ubg, ld_ubg, p, ld_p, x_out, f_out, g_out,
                   lam_x_out, lam_g_out, lam_p_out, X_out, status, iters, stream, -1);
}

int nmpc_solve_batch(nmpc_handle* h, int32_t B, const double* x0, int64_t ld_x0, const double* lbx, int64_t ld_lbx,
                     const double* ubx, int64_t ld_ubx, const double* lbg, int64_t ld_lbg, const double* ubg,
                     int64_t ld_ubg, const double* p, int64_t ld_p, double* x_out, double* f_out, double* g_out,
                     double* lam_x_out, double* lam_g_out, double* lam_p_out, double* X_out, int32_t* status,
                     int32_t* iters) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (B < 0) return fail(NMPC_E_INVALID, "B < 0");
  if (B == 0) return NMPC_OK;
  if (!x0 || !lbx || !ubx || !lbg || !ubg || !p || !x_out)
    return fail(NMPC_E_INVALID, "required pointer is null");
  const Params& P = h->hp;
  const size_t nw = P.nwE, ng = P.ng, np = P.npE, nX = (size_t)P.nxE * (P.N + 1);
  auto cols = [&](int64_t ld) { return ld == 0 ? (size_t)1 : (size_t)B; };
  auto len = [&](int64_t ld, size_t n) { return ld == 0 ? n : (size_t)(B - 1) * (size_t)ld + n; };
  const size_t n_x0 = len(ld_x0, nw), n_lbx = len(ld_lbx, nw), n_ubx = len(ld_ubx, nw);
  const size_t n_lbg = len(ld_lbg, ng), n_ubg = len(ld_ubg, ng), n_p = len(ld_p, np);
  (void)cols;
  const size_t n_out = (size_t)B * (2 * nw + 2 * ng + nX + np + 1);
  const size_t total = n_x0 + n_lbx + n_ubx + n_lbg + n_ubg + n_p + n_out;
  if (total * sizeof(double) > h->dbuf_bytes) {
    if (h->dbuf) hipFree(h->dbuf);
    h->dbuf = nullptr; h->dbuf_bytes = 0;
    if (hipMalloc(&h->dbuf, total * sizeof(double)) != hipSuccess) return fail(NMPC_E_NOMEM, "hipMalloc staging");
    h->dbuf_bytes = total * sizeof(double);
  }
  if ((size_t)B * 2 * sizeof(int) > h->ibuf_bytes) {
    if (h->ibuf) hipFree(h->ibuf);
    h->ibuf = nullptr; h->ibuf_bytes = 0;
    if (hipMalloc(&h->ibuf, (size_t)B * 2 * sizeof(int)) != hipSuccess) return fail(NMPC_E_NOMEM, "hipMalloc staging");
    h->ibuf_bytes = (size_t)B * 2 * sizeof(int);
  }
  double* q = h->dbuf;
  double* d_x0 = q; q += n_x0;
  double* d_lbx = q; q += n_lbx;
  double* d_ubx = q; q += n_ubx;
  double* d_lbg = q; q += n_lbg;
  double* d_ubg = q; q += n_ubg;
  double* d_p = q; q += n_p;
  double* d_x = q; q += (size_t)B * nw;
  double* d_lx = q; q += (size_t)B * nw;
  double* d_g = q; q += (size_t)B * ng;
  double* d_lg = q; q += (size_t)B * ng;
  double* d_X = q; q += (size_t)B * nX;
  double* d_lp = q; q += (size_t)B * np;
  double* d_f = q; q += (size_t)B;
  int* d_st = h->ibuf;
  int* d_it = h->ibuf + B;
  hipError_t e = hipSuccess;
  auto up = [&](double* dst, const double* src, size_t n) {
    if (e == hipSuccess) e = hipMemcpy(dst, src, n * sizeof(double), hipMemcpyHostToDevice);
  };
  up(d_x0, x0, n_x0); up(d_lbx, lbx, n_lbx); up(d_ubx, ubx, n_ubx);
  up(d_lbg, lbg, n_lbg); up(d_ubg, ubg, n_ubg); up(d_p, p, n_p);
  if (e != hipSuccess) return fail(NMPC_E_HIP, std::string("hipMemcpy H2D: ") + hipGetErrorString(e));
  // the bounds are on the host here: the equality-row test costs no device round trip
  const int heq = h->kernE ? host_has_eq(B, (int)ng, lbg, ld_lbg, ubg, ld_ubg) : 0;
  int rc = solve_dev(h, B, d_x0, ld_x0, d_lbx, ld_lbx, d_ubx, ld_ubx, d_lbg, ld_lbg, d_ubg, ld_ubg,
                     d_p, ld_p, d_x, d_f, d_g, d_lx, d_lg, lam_p_out ? d_lp : nullptr, d_X, d_st, d_it,
                     nullptr, heq);
  if (rc != NMPC_OK) return rc;
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return fail(NMPC_E_HIP, std::string("kernel: ") + hipGetErrorString(e));
  auto down = [&](void* dst, const void* src, size_t bytes) {
    if (dst && e == hipSuccess) e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  };
  down(x_out, d_x, (size_t)B * nw * 8); down(lam_x_out, d_lx, (size_t)B * nw * 8);
  down(g_out, d_g, (size_t)B * ng * 8); down(lam_g_out, d_lg, (size_t)B * ng * 8);
  down(X_out, d_X, (size_t)B * nX * 8); down(f_out, d_f, (size_t)B * 8);
  down(lam_p_out, d_lp, (size_t)B * np * 8);
  down(status, d_st, (size_t)B * 4); down(iters, d_it, (size_t)B * 4);
  if (e != hipSuccess) return fail(NMPC_E_HIP, std::string("hipMemcpy D2H: ") + hipGetErrorString(e));
  return NMPC_OK;
}

int nmpc_shift_dev(nmpc_handle* h, int32_t B, double* p, int64_t ld_p, const double* u_sol, double* w_out,
                   const double* v_t, const double* w_t, void* stream) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (B <= 0) return B == 0 ? NMPC_OK : fail(NMPC_E_INVALID, "B < 0");
  if (!p || !u_sol || !w_out || !v_t || !w_t) return fail(NMPC_E_INVALID, "null pointer");
  if (ld_p < h->hp.npE) return fail(NMPC_E_INVALID, "ld_p < np");
  const int thr = 256;
  hipLaunchKernelGGL(nmpc_shift_kernel, dim3((B + thr - 1) / thr), dim3(thr), 0, (hipStream_t)stream, (int)B,
                     h->hp.N, h->hp.nxE, h->hp.nuE, h->hp.T, p, (long long)ld_p, u_sol, w_out, v_t, w_t);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NMPC_E_HIP, std::string("shift launch: ") + hipGetErrorString(e));
  return NMPC_OK;
}

int nmpc_closed_loop_dev(nmpc_handle* h, int32_t B, int32_t K, const double* lbx, int64_t ld_lbx,
                         const double* ubx, int64_t ld_ubx, const double* lbg, int64_t ld_lbg,
                         const double* ubg, int64_t ld_ubg, double* p, int64_t ld_p, double* w,
                         const double* v_t, const double* w_t, int64_t ld_tk, int64_t ld_tb,
                         const double* p_step, int64_t ld_ps,
                         double* u_hist, double* x_hist, double* f_hist, double* fov_hist,
                         int32_t* status_hist, int32_t* iters_hist, const int32_t* order, void* stream) {
  if (!h) return fail(NMPC_E_INVALID, "null handle");
  if (B < 0 || K < 0) return fail(NMPC_E_INVALID, "B < 0 or K < 0");
  if (B == 0 || K == 0) return NMPC_OK;
  if (!lbx || !ubx || !lbg || !ubg || !p || !w || !v_t || !w_t)
    return fail(NMPC_E_INVALID, "required pointer is null");
  if (ld_tk < 0 || ld_tb < 0) return fail(NMPC_E_INVALID, "negative target-schedule stride");
  if (p_step && ld_ps < 0) return fail(NMPC_E_INVALID, "negative p_step stride");
  const Params& P = h->hp;
  if ((ld_lbx != 0 && ld_lbx < P.nwE) || (ld_ubx != 0 && ld_ubx < P.nwE) || (ld_lbg != 0 && ld_lbg < P.ng) ||
      (ld_ubg != 0 && ld_ubg < P.ng) || ld_p < P.npE)
    return fail(NMPC_E_INVALID, "leading dimension smaller than the vector length");
  if ((long long)B * K > (1LL << 40)) return fail(NMPC_E_INVALID, "B*K too large");
  IO io;
  std::memset(&io, 0, sizeof(io));
  io.lbx = lbx; io.ubx = ubx; io.lbg = lbg; io.ubg = ubg;
  io.ld_lbx = ld_lbx; io.ld_ubx = ld_ubx; io.ld_lbg = ld_lbg; io.ld_ubg = ld_ubg;
  if (int rc = ensure_ws(h, B)) return rc;
  io.ws = h->dws;
  IO ioE;
  Run run;
  if (int rc = eq_prepare(h, B, io, ioE, (hipStream_t)stream, -1, &run)) return rc;
  Loop lp;
  lp.K = K; lp.p = p; lp.ld_p = ld_p; lp.w = w; lp.vt = v_t; lp.wt = w_t; lp.ld_tk = ld_tk; lp.ld_tb = ld_tb;
  lp.u_hist = u_hist; lp.x_hist = x_hist; lp.f_hist = f_hist; lp.fov_hist = fov_hist;
  lp.pstep = p_step; lp.ld_ps = ld_ps;
  lp.st_hist = status_hist; lp.it_hist = iters_hist;
  lp.order = order;
  lp.done = nullptr;
  lp.times = nullptr;
  if (std::getenv("NMPC_STEP_TIMES")) {  // diagnostics: per-(step, scenario) realtime stamps (100 MHz)
    const size_t need = (size_t)K * B * 3 * sizeof(unsigned long long);
    if (need > h->times_bytes) {
      if (h->dtimes) hipFree(h->dtimes);
      h->dtimes = nullptr; h->times_bytes = 0;
      if (hipMalloc(&h->dtimes, need) != hipSuccess) return fail(NMPC_E_NOMEM, "hipMalloc step times");
      h->times_bytes = need;
    }
    lp.times = h->dtimes;
  }
  h->times_n = lp.times ? (size_t)K * B * 3 : 0;
  // more scenarios than resident waves: the step-queue scheduler (persistent waves,
  // lowest step first), unless NMPC_CLOSED_LOOP=static (diagnostics: one workgroup per
  // scenario in dispatch order)
  if (h->resident == 0) {
    int per_cu = 0, cus = 0;
    hipDeviceProp_t prop;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)h->sched, WAVE, h->lds_bytes) != hipSuccess ||
        hipGetDeviceProperties(&prop, h->device) != hipSuccess)
      return fail(NMPC_E_HIP, "occupancy query");
    cus = prop.multiProcessorCount;
    h->resident = per_cu * cus;
    if (h->schedE) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)h->schedE, WAVE, h->lds_bytesE) != hipSuccess)
        return fail(NMPC_E_HIP, "occupancy query");
      h->residentE = per_cu * cus;
    }
  }
  if (h->nxcc < 0) {
    int nx = 0;
    if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, h->device) != hipSuccess) nx = 0;
    h->nxcc = nx;
  }
  const char* pol = std::getenv("NMPC_CLOSED_LOOP");
  // the step queues pin scenarios to XCD sets by the XCC_ID of the running wave: only
  // valid when the device has exactly the NXCD XCDs the sets assume (SPX mode of an
  // MI355X); otherwise one workgroup per scenario
  const bool use_q = (B > h->resident) && h->resident >= NXCD && h->nxcc == NXCD &&
                     !(pol && std::strcmp(pol, "static") == 0);
  h->last_steps = (long long)B * K;
  // scheduler / completion-guard state: [ndone (u64)][err, pad][done (B)][queues]
  const int BX = use_q ? (B + NXCD - 1) / NXCD : 0;
  const size_t nint = 4 + (size_t)B + (use_q ? (size_t)6 * NXCD * K + (size_t)2 * NXCD * K * BX : 0);
  if (nint * sizeof(int) > h->sched_bytes) {
    if (h->dsched) hipFree(h->dsched);
    h->dsched = nullptr; h->sched_bytes = 0;
    if (hipMalloc(&h->dsched, nint * sizeof(int)) != hipSuccess) return fail(NMPC_E_NOMEM, "hipMalloc scheduler");
    h->sched_bytes = nint * sizeof(int);
  }
  SchedQ q;
  std::memset(&q, 0, sizeof(q));
  q.ndone = (unsigned long long*)h->dsched;
  q.err = h->dsched + 2;
  q.done = h->dsched + 4;
  q.eqnows = run.Enows ? h->deq : nullptr;
  const int thr = 256;
  h->last_err = q.err;
  h->last_ndone = q.ndone;
  h->last_stream = (hipStream_t)stream;
  if (use_q) {
    q.head = q.done + B; q.tail = q.head + 2 * NXCD * K; q.resv = q.tail + 2 * NXCD * K;
    q.ring = q.resv + 2 * NXCD * K; q.BX = BX;
    // hot family threshold: half of max_iter (NMPC_SCHED_HOT overrides; 0 = one family only)
    q.hot_iters = h->hp.o.max_iter / 2 > 0 ? h->hp.o.max_iter / 2 : 1;
    if (const char* hv = std::getenv("NMPC_SCHED_HOT")) q.hot_iters = std::atoi(hv);
    const char* one = std::getenv("NMPC_SCHED_TEST_ONE_SET");
    q.one_set = (one && std::atoi(one) != 0) ? 1 : 0;
    const long long n = (long long)NXCD * K * BX;
    hipLaunchKernelGGL(nmpc_sched_init_kernel, dim3((unsigned)((n + thr - 1) / thr)), dim3(thr), 0,
                       (hipStream_t)stream, (int)B, (int)K, (const int*)order, q);
    // persistent waves: all resident ones.  NMPC_SCHED_WAVES (a diagnostic) launches
    // fewer; correctness needs at least one wave on every XCD, which the hardware's
    // round-robin placement of workgroups over the XCDs gives for any count >= NXCD,
    // and the check kernel below reports any scenario left unfinished.
    int waves = h->resident;
    if (const char* ev = std::getenv("NMPC_SCHED_WAVES")) {
      const int w = std::atoi(ev);
      if (w >= NXCD && w < waves) waves = w;
    }
    if (run.A)
      hipLaunchKernelGGL(h->sched, dim3(waves), dim3(WAVE), h->lds_bytes, (hipStream_t)stream,
                         (const Params*)h->dprm, (int)B, io, lp, q);
    // the equality class on the same queues (when paired, exactly one of the pair runs);
    // when its own occupancy cannot put a wave on every XCD, one workgroup per scenario
    // instead, on the same completion-guard state (zeroed by nmpc_sched_init_kernel)
    if (run.E && h->residentE >= NXCD) {
      hipLaunchKernelGGL(h->schedE, dim3(h->residentE < waves ? h->residentE : waves), dim3(WAVE), h->lds_bytesE,
                         (hipStream_t)stream, (const Params*)h->dprm, (int)B, ioE, lp, q);
    } else if (run.E) {
      Loop lpE = lp;
      lpE.done = q.done;
      hipLaunchKernelGGL(h->loopE, dim3(B), dim3(WAVE), h->lds_bytesE, (hipStream_t)stream,
                         (const Params*)h->dprm, (int)B, ioE, lpE);
    }
    h->last_policy = 1;
    h->last_waves = waves;
  } else {
    h->last_policy = 0;
    h->last_waves = B;
    lp.done = q.done;
    hipLaunchKernelGGL(nmpc_guard_init_kernel, dim3((B + thr - 1) / thr), dim3(thr), 0, (hipStream_t)stream,
                       (int)B, q);
    if (run.A)
      hipLaunchKernelGGL(h->loop, dim3(B), dim3(WAVE), h->lds_bytes, (hipStream_t)stream,
                         (const Params*)h->dprm, (int)B, io, lp);
    if (run.E)
      hipLaunchKernelGGL(h->loopE, dim3(B), dim3(WAVE), h->lds_bytesE, (hipStream_t)stream,
                         (const Params*)h->dprm, (int)B, ioE, lp);
  }
  // completion guard, both policies: every scenario ran its K steps, else err |= 2 and
  // the unrun steps are marked in the histories
  hipLaunchKernelGGL(nmpc_sched_check_kernel, dim3((B + thr - 1) / thr), dim3(thr), 0, (hipStream_t)stream,
                     (int)B, (int)K, q, lp);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NMPC_E_HIP, std::string("closed-loop launch: ") + hipGetErrorString(e));
  return NMPC_OK;
}

}  // extern "C"
#endif  // NMPC_TU_CLASS
