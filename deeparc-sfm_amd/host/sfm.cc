// sfm.cc — solve(), fitHemisphere() and the sfm.cc main() loop over libdab (see sfm.hh).
#include "sfm.hh"

#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <functional>
#include <iostream>

#include "DabScene.hh"

int solveWith(DeepArcManager& m, const dab_options& options, bool freeze_camera, dab_summary* summary) {
  // the manager's resident problem (handle reused across the sfm.cc loop's solves and
  // filters; re-set only when the structure or the constancy changed)
  DabSession& S = m.dabSession();
  int rc = S.ensure(m, freeze_camera ? 1 : 0);
  if (rc) return rc;
  DabHandle& dh = S.handle;
  DabScene& scene = S.scene;
  dab_summary local{};
  dab_summary* s = summary ? summary : &local;
  const double t0 = dab_now_seconds();
  rc = dab_solve(dh.h, &options, s);
  if (rc == DAB_E_UNSUPPORTED && options.linear_solver_type == DAB_LINEAR_SOLVER_EXPLICIT_SCHUR) {
    // The explicit reduced system is refused only when it is both too large for the LDS
    // tiles (more than 160 free cameras) and too large for the pair tables (> 2e8 entry
    // pairs). The step is then the inexact implicit-Schur PCG one: say so, and the summary
    // records it (linear_solver_type_used), so the result is not read as DENSE_SCHUR parity.
    std::fprintf(stderr, "solve: DENSE_SCHUR refused (%s); running ITERATIVE_SCHUR (PCG) instead\n",
                 dab_last_error());
    dab_options o = options;
    o.linear_solver_type = DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG;
    rc = dab_solve(dh.h, &o, s);
  }
  if (rc) {
    S.resident = false;  // a failed solve leaves the device state unspecified
    return rc;
  }
  const double t1 = dab_now_seconds();
  S.t.lm += s->total_time_in_seconds;
  S.t.prep += (t1 - t0) - s->total_time_in_seconds;
  scene.write_back(m);  // dab_solve wrote the optimised values into scene.points / ext
  S.t.writeback += dab_now_seconds() - t1;
  return 0;
}

namespace {
// solve() of sfm.cc:31-75 with the reference's options; verbose: its progress and summary
dab_summary solve_opts(DeepArcManager& m, int max_iteration, int max_second, bool freeze_camera, bool verbose) {
  dab_options o;
  dab_options_init(&o);
  o.linear_solver_type = DAB_LINEAR_SOLVER_EXPLICIT_SCHUR;  // sfm.cc:67 DENSE_SCHUR
  o.minimizer_progress_to_stdout = verbose ? 1 : 0;         // sfm.cc:68
  o.max_num_iterations = max_iteration;                     // sfm.cc:69
  o.num_threads = 16;                                       // sfm.cc:70 (unused on the GPU)
  o.max_solver_time_in_seconds = max_second;                // sfm.cc:71
  dab_summary s{};
  dab_check(solveWith(m, o, freeze_camera, &s));
  if (verbose)
    std::printf("Solver Summary: %s, initial cost %.6e, final cost %.6e, %d iterations (%d successful), %s\n",
                s.linear_solver_type_used == DAB_LINEAR_SOLVER_EXPLICIT_SCHUR ? "DENSE_SCHUR" : "ITERATIVE_SCHUR (PCG)",
                s.initial_cost, s.final_cost, s.num_iterations, s.num_successful_steps, s.message);
  return s;
}
double now_seconds() { return dab_now_seconds(); }
}  // namespace

void solve(DeepArcManager& deeparcManager, int max_iteration, int max_second, bool freeze_camera) {
  (void)solve_opts(deeparcManager, max_iteration, max_second, freeze_camera, true);
}

// ---- small dense trust-region LM with Ceres semantics ---------------------
namespace {

using Eval = std::function<void(const std::vector<double>&, std::vector<double>&, std::vector<double>&)>;

bool chol_solve(std::vector<double> A, std::vector<double>& b, int n) {
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / d;
    }
  }
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= A[i * n + k] * b[k];
    b[i] = s / A[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= A[k * n + i] * b[k];
    b[i] = s / A[i * n + i];
  }
  return true;
}

// Minimises 0.5 |r(x)|^2 from x; m residuals, n parameters; J row-major [m][n].
void tiny_lm(int n, int m, const Eval& eval, std::vector<double>& x, int max_iteration) {
  const double ftol = 1e-6, gtol = 1e-10, ptol = 1e-8, min_rel = 1e-3, max_radius = 1e16, min_radius = 1e-32;
  const double min_diag = 1e-6, max_diag = 1e32;
  std::vector<double> r(m), J((size_t)m * n), rc(m), Jc((size_t)m * n), s(n, 1.0), g(n);
  auto cost_of = [&](const std::vector<double>& rr) {
    double c = 0.0;
    for (int i = 0; i < m; ++i) c += rr[i] * rr[i];
    return std::isfinite(c) ? 0.5 * c : DBL_MAX;
  };
  auto gradient = [&]() {
    double gm = 0.0;
    for (int j = 0; j < n; ++j) {
      double t = 0.0;
      for (int i = 0; i < m; ++i) t += J[(size_t)i * n + j] * r[i];
      g[j] = t;
      gm = std::fmax(gm, std::fabs(x[j] - (x[j] + (-t))));
    }
    return gm;
  };
  auto norm = [](const std::vector<double>& v) {
    double t = 0.0;
    for (double a : v) t += a * a;
    return std::sqrt(t);
  };
  eval(x, r, J);
  double cost = cost_of(r);
  if (cost == DBL_MAX) return;
  for (int j = 0; j < n; ++j) {  // Jacobi scaling, iteration 0
    double c = 0.0;
    for (int i = 0; i < m; ++i) c += J[(size_t)i * n + j] * J[(size_t)i * n + j];
    s[j] = 1.0 / (1.0 + std::sqrt(c));
  }
  double gmax = gradient(), x_norm = norm(x), radius = 1e4, decrease = 2.0, best = cost;
  std::vector<double> xbest = x;
  bool successful = true;
  int invalid = 0;
  for (int it = 0;;) {
    if (successful && cost < best) {
      best = cost;
      xbest = x;
    }
    if (it >= max_iteration || (successful && gmax <= gtol) || radius <= min_radius) break;
    ++it;
    // (Js^T Js + D^2) y = Js^T r, delta = -y * s
    std::vector<double> A((size_t)n * n, 0.0), b(n, 0.0);
    for (int i = 0; i < m; ++i)
      for (int a = 0; a < n; ++a) {
        const double ja = J[(size_t)i * n + a] * s[a];
        b[a] += ja * r[i];
        for (int c = 0; c < n; ++c) A[(size_t)a * n + c] += ja * J[(size_t)i * n + c] * s[c];
      }
    for (int a = 0; a < n; ++a) {
      const double d = std::fmin(std::fmax(A[(size_t)a * n + a], min_diag), max_diag);
      const double D = std::sqrt(d / radius);
      A[(size_t)a * n + a] += D * D;
    }
    bool ok = chol_solve(A, b, n);
    std::vector<double> delta(n), xc(n);
    for (int a = 0; a < n; ++a) delta[a] = -b[a] * s[a];
    double model = 0.0;
    for (int i = 0; ok && i < m; ++i) {
      double mi = 0.0;
      for (int a = 0; a < n; ++a) mi += J[(size_t)i * n + a] * delta[a];
      model += -(mi * (r[i] + mi / 2.0));
    }
    if (!ok || !std::isfinite(model) || !(model > 0.0)) {
      if (++invalid >= 5) break;
      radius /= decrease;
      decrease *= 2.0;
      successful = false;
      continue;
    }
    invalid = 0;
    for (int a = 0; a < n; ++a) xc[a] = x[a] + delta[a];
    eval(xc, rc, Jc);
    const double ccost = cost_of(rc);
    double step_norm = 0.0;
    for (int a = 0; a < n; ++a) step_norm += (x[a] - xc[a]) * (x[a] - xc[a]);
    if (std::sqrt(step_norm) <= ptol * (x_norm + ptol)) break;
    if (std::fabs(cost - ccost) <= ftol * cost) break;
    const double rho = (cost - ccost) / model;
    if (rho > min_rel) {
      x = xc;
      r = rc;
      J = Jc;
      cost = ccost;
      x_norm = norm(x);
      gmax = gradient();
      radius = std::fmin(max_radius, radius / std::fmax(1.0 / 3.0, 1.0 - std::pow(2.0 * rho - 1.0, 3)));
      decrease = 2.0;
      successful = true;
    } else {
      radius /= decrease;
      decrease *= 2.0;
      successful = false;
    }
  }
  x = xbest;
}

}  // namespace

void fitHemisphere(const std::vector<std::vector<double> >& centers, double center[3], double* radius,
                   int max_iteration) {
  const int m = (int)centers.size();
  if (m == 0) return;  // an empty Ceres problem leaves the parameters as they are
  std::vector<double> x{center[0], center[1], center[2], *radius};
  Eval eval = [&](const std::vector<double>& p, std::vector<double>& r, std::vector<double>& J) {
    for (int i = 0; i < m; ++i) {
      double sum = 0.0;  // HemisphereRadius::operator(), hemisphere_radius.hh:20-28
      for (int k = 0; k < 3; ++k) {
        const double d = p[k] - centers[i][k];
        sum += d * d;
        J[(size_t)i * 4 + k] = 2.0 * d;
      }
      r[i] = sum - p[3];
      J[(size_t)i * 4 + 3] = -1.0;
    }
  };
  tiny_lm(4, m, eval, x, max_iteration);
  for (int k = 0; k < 3; ++k) center[k] = x[k];
  *radius = x[3];
}

PipelineReport runPipeline(const std::string& input, const std::string& output, const std::string& ply_prefix,
                           int max_iteration, int max_second, double error_boundary, bool verbose) {
  const double t_start = now_seconds();
  DeepArcManager m;
  m.read(input);
  PipelineReport rep{};
  const double t_read = now_seconds();
  rep.read_seconds = t_read - t_start;
  double center[3] = {0, 0, 0}, radius = 1.0;  // sfm.cc:87-88
  fitHemisphere(m.getCameraCenter(), center, &radius);
  rep.fit_seconds = now_seconds() - t_read;
  double t_w = now_seconds();
  if (!ply_prefix.empty()) m.writePly(ply_prefix + "init.ply");
  rep.write_seconds += now_seconds() - t_w;
  // the manager keeps one libdab handle: each filter runs on the problem its solve left
  // resident, and each solve after a filter re-sets the compacted problem on that handle
  auto do_solve = [&](bool freeze) {
    const double t = now_seconds();
    const dab_summary s = solve_opts(m, max_iteration, max_second, freeze, verbose);
    rep.solve_seconds += now_seconds() - t;
    rep.solves++;
    rep.lm_iterations += s.num_iterations;
    rep.final_cost = s.final_cost;
  };
  auto do_filter = [&]() {
    const double t = now_seconds();
    m.filterPoint3d(error_boundary, center, radius);
    rep.filter_seconds += now_seconds() - t;
  };
  do_solve(true);  // sfm.cc:111: points only
  do_filter();
  int step = 0;
  t_w = now_seconds();
  if (!ply_prefix.empty()) m.writePly(ply_prefix + std::to_string(step) + ".ply");
  rep.write_seconds += now_seconds() - t_w;
  int old_points = 1, cur_points = 10000000;  // sfm.cc:106
  while (cur_points != old_points) {
    ++step;
    old_points = cur_points;
    do_solve(false);
    do_filter();
    cur_points = (int)m.point3ds()->size();
    t_w = now_seconds();
    if (!ply_prefix.empty()) m.writePly(ply_prefix + std::to_string(step) + ".ply");
    rep.write_seconds += now_seconds() - t_w;
  }
  t_w = now_seconds();
  if (!ply_prefix.empty()) m.writePly(ply_prefix + "clear.ply");
  if (!output.empty()) m.write(output);
  rep.write_seconds += now_seconds() - t_w;
  const DabTimers& T = m.dabSession().t;
  rep.marshal_seconds = T.marshal;
  rep.setup_seconds = T.setup;
  rep.update_seconds = T.update;
  rep.prep_seconds = T.prep;
  rep.lm_seconds = T.lm;
  rep.writeback_seconds = T.writeback;
  rep.filter_device_seconds = T.filter_dev;
  rep.filter_host_seconds = T.filter_host;
  for (int k = 0; k < 3; ++k) rep.hemisphere_center[k] = center[k];
  rep.hemisphere_radius = radius;
  rep.rounds = step;
  rep.final_blocks = (int)m.parameters()->size();
  rep.final_points = (int)m.point3ds()->size();
  rep.total_seconds = now_seconds() - t_start;
  return rep;
}
