// TEST INFRASTRUCTURE (not the product): a host AddressSanitizer / UBSan driver of the CPU
// restatement ("optional host ASan/UBSan build").  It links
// oracle/cpu_ipopt.cpp into a standalone executable (`make -C oracle sanitize`) and runs
// nmpc_cpu_solve_batch on a batch written by tests/test_cpu_sanitize.py:
//   input:  int64 B, n, np, m, nopts | nmpc_cpu_problem | opts[nopts] | w0[B*n] | p[B*np] |
//           lbx[n] | ubx[n] | lbg[m] | ubg[m]
//   output: int32 status[B] | int32 iter[B] | double f[B] | double x[B*n]
// Any sanitizer report aborts the run with a non-zero exit status.
#include <cstdint>
#include <cstdio>
#include <vector>

#define MAXOBS 16
extern "C" {
typedef struct {
  int32_t N, model, n_obs, np, w1_pidx, w2_pidx;
  double T, w1, w2, vfov, hfov;
  double obs_x[MAXOBS], obs_y[MAXOBS], obs_rsum[MAXOBS];
  int32_t obs_x_pidx[MAXOBS], obs_y_pidx[MAXOBS];
} nmpc_cpu_problem;
int nmpc_cpu_solve_batch(const nmpc_cpu_problem* prob, const double* opts, int64_t B, const double* w0,
                         const double* p, const double* lbx, const double* ubx, const double* lbg, const double* ubg,
                         double* x_out, double* f_out, double* g_out, double* lam_x_out, double* lam_g_out,
                         int32_t* status_out, int32_t* iter_out, int nthreads, double* solve_s);
}

template <class T>
static bool rd(FILE* f, T* v, size_t n) { return fread(v, sizeof(T), n, f) == n; }

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s <in> <out>\n", argv[0]); return 2; }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int64_t h[5];
  nmpc_cpu_problem prob;
  if (!rd(f, h, 5) || !rd(f, &prob, 1)) return 3;
  const int64_t B = h[0], n = h[1], np = h[2], m = h[3], no = h[4];
  std::vector<double> opts(no), w0(B * n), p(B * np), lbx(n), ubx(n), lbg(m), ubg(m);
  if (!rd(f, opts.data(), no) || !rd(f, w0.data(), B * n) || !rd(f, p.data(), B * np) || !rd(f, lbx.data(), n) ||
      !rd(f, ubx.data(), n) || !rd(f, lbg.data(), m) || !rd(f, ubg.data(), m))
    return 3;
  fclose(f);
  std::vector<double> x(B * n), fo(B), g(B * m), lx(B * n), lg(B * m);
  std::vector<int32_t> st(B), it(B);
  const int rc = nmpc_cpu_solve_batch(&prob, opts.data(), B, w0.data(), p.data(), lbx.data(), ubx.data(), lbg.data(),
                                      ubg.data(), x.data(), fo.data(), g.data(), lx.data(), lg.data(), st.data(),
                                      it.data(), 2, nullptr);
  if (rc != 0) return 4;
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;
  fwrite(st.data(), sizeof(int32_t), B, o);
  fwrite(it.data(), sizeof(int32_t), B, o);
  fwrite(fo.data(), sizeof(double), B, o);
  fwrite(x.data(), sizeof(double), B * n, o);
  fclose(o);
  return 0;
}
