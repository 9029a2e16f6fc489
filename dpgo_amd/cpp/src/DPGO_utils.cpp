// Host utilities (reference src/DPGO_utils.cpp); the g2o parser is the library's own reader.
#include <DPGO/DPGO_robust.h>
#include <DPGO/DPGO_utils.h>
#include <dpgo_rbcd.h>

#include <algorithm>
#include <cassert>
#include <cmath>
#include <random>
#include <stdexcept>
#include <string>

namespace DPGO {

std::vector<RelativeSEMeasurement> read_g2o_file(const std::string& filename, size_t& num_poses) {
  dpgo_graph g = nullptr;
  if (dpgo_graph_read_g2o(filename.c_str(), &g) != DPGO_HIP_OK)
    throw std::runtime_error(std::string("read_g2o_file: ") + dpgo_hip_last_error());
  int d = 0, n = 0, m = 0, dup = 0;
  dpgo_graph_info(g, &d, &n, &m, &dup);
  std::vector<int> p1(m), p2(m);
  std::vector<double> R(static_cast<size_t>(m) * d * d), t(static_cast<size_t>(m) * d), kappa(m), tau(m);
  dpgo_graph_copy_out(g, p1.data(), p2.data(), R.data(), t.data(), kappa.data(), tau.data());
  dpgo_graph_destroy(g);
  std::vector<RelativeSEMeasurement> out;
  out.reserve(m);
  for (int e = 0; e < m; ++e) {
    Matrix Rm(d, d), tm(d, 1);
    for (int u = 0; u < d; ++u) {
      for (int v = 0; v < d; ++v) Rm(u, v) = R[static_cast<size_t>(e) * d * d + u * d + v];
      tm(u, 0) = t[static_cast<size_t>(e) * d + u];
    }
    out.emplace_back(0, 0, p1[e], p2[e], Rm, tm, kappa[e], tau[e]);
  }
  num_poses = static_cast<size_t>(n);  // App. B1 fix: max index + 1
  return out;
}

SparseMatrix constructConnectionLaplacianSE(const std::vector<RelativeSEMeasurement>& measurements, size_t n) {
  const size_t d = measurements.empty() ? 0 : static_cast<size_t>(measurements[0].t.rows());
  const size_t b = d + 1;
  std::vector<std::pair<std::pair<int, int>, double>> trip;
  trip.reserve(measurements.size() * 4 * b * b);
  for (const auto& m : measurements) {
    Matrix T = Matrix::Zero(b, b), Om = Matrix::Zero(b, b);
    T.setBlock(0, 0, m.R);
    T.setBlock(0, d, m.t);
    T(d, d) = 1.0;
    for (size_t u = 0; u < d; ++u) Om(u, u) = m.weight * m.kappa;
    Om(d, d) = m.weight * m.tau;
    const Matrix Wii = T * Om * T.transpose(), Wij = -(T * Om), Wji = -(Om * T.transpose());
    const int i = static_cast<int>(m.p1), j = static_cast<int>(m.p2);
    for (size_t u = 0; u < b; ++u)
      for (size_t v = 0; v < b; ++v) {
        trip.push_back({{static_cast<int>(i * b + u), static_cast<int>(i * b + v)}, Wii(u, v)});
        trip.push_back({{static_cast<int>(j * b + u), static_cast<int>(j * b + v)}, Om(u, v)});
        trip.push_back({{static_cast<int>(i * b + u), static_cast<int>(j * b + v)}, Wij(u, v)});
        trip.push_back({{static_cast<int>(j * b + u), static_cast<int>(i * b + v)}, Wji(u, v)});
      }
  }
  SparseMatrix Q(static_cast<long>(b * n), static_cast<long>(b * n));
  Q.setFromTriplets(trip);
  return Q;
}

SparseMatrix constructConnectionLaplacianSE(const std::vector<RelativeSEMeasurement>& measurements) {
  size_t n = 0;
  for (const auto& m : measurements) n = std::max(n, std::max(m.p1, m.p2));  // :223-228
  return constructConnectionLaplacianSE(measurements, n + 1);
}

Matrix odometryInitialization(size_t dimension, size_t num_poses, const std::vector<RelativeSEMeasurement>& odometry) {
  const size_t d = dimension, b = d + 1;
  Matrix T(d, num_poses * b);
  T.setBlock(0, 0, Matrix::Identity(d, d));
  for (size_t src = 0; src < odometry.size(); ++src) {
    const auto& m = odometry[src];
    if (m.p1 != src || m.p2 != src + 1) throw std::invalid_argument("odometryInitialization: not a chain");
    const Matrix Rs = T.block(0, src * b, d, d), ts = T.block(0, src * b + d, d, 1);
    T.setBlock(0, (src + 1) * b, Rs * m.R);
    T.setBlock(0, (src + 1) * b + d, ts + Rs * m.t);
  }
  return T;
}

Matrix chordalInitialization(size_t dimension, size_t num_poses, const std::vector<RelativeSEMeasurement>& measurements) {
  // src/DPGO_utils.cpp:377-424 -> dpgo_chordal_initialization (native host block-Cholesky solve)
  const size_t d = dimension, m = measurements.size();
  std::vector<int> p1(m), p2(m);
  std::vector<double> R(m * d * d), t(m * d), kappa(m), tau(m);
  for (size_t e = 0; e < m; ++e) {
    const auto& x = measurements[e];
    p1[e] = static_cast<int>(x.p1);
    p2[e] = static_cast<int>(x.p2);
    for (size_t u = 0; u < d; ++u) {
      for (size_t v = 0; v < d; ++v) R[e * d * d + u * d + v] = x.R(static_cast<long>(u), static_cast<long>(v));
      t[e * d + u] = x.t(static_cast<long>(u), 0);
    }
    kappa[e] = x.kappa;
    tau[e] = x.tau;
  }
  Matrix T(static_cast<long>(d), static_cast<long>(num_poses * (d + 1)));
  if (dpgo_chordal_initialization(static_cast<int>(d), static_cast<int>(num_poses), static_cast<int>(m), p1.data(),
                                  p2.data(), R.data(), t.data(), kappa.data(), tau.data(), T.data()) != DPGO_HIP_OK)
    throw std::runtime_error(std::string("chordalInitialization: ") + dpgo_hip_last_error());
  return T;
}

// one-sided Jacobi SVD of an r x c matrix (r >= c): A V = U Sigma
static void jacobi_svd(const Matrix& M, Matrix& U, Matrix& S, Matrix& V) {
  const long r = M.rows(), c = M.cols();
  U = M;
  V = Matrix::Identity(c, c);
  for (int sweep = 0; sweep < 60; ++sweep) {
    bool rot = false;
    for (long p = 0; p < c - 1; ++p)
      for (long q = p + 1; q < c; ++q) {
        double al = 0, be = 0, ga = 0;
        for (long a = 0; a < r; ++a) {
          al += U(a, p) * U(a, p);
          be += U(a, q) * U(a, q);
          ga += U(a, p) * U(a, q);
        }
        if (ga == 0.0 || std::fabs(ga) <= 1e-17 * std::sqrt(al * be)) continue;
        rot = true;
        const double z = (be - al) / (2 * ga);
        const double t = std::copysign(1.0, z) / (std::fabs(z) + std::sqrt(1 + z * z));
        const double cs = 1 / std::sqrt(1 + t * t), sn = cs * t;
        for (long a = 0; a < r; ++a) {
          const double up = U(a, p), uq = U(a, q);
          U(a, p) = cs * up - sn * uq;
          U(a, q) = sn * up + cs * uq;
        }
        for (long a = 0; a < c; ++a) {
          const double vp = V(a, p), vq = V(a, q);
          V(a, p) = cs * vp - sn * vq;
          V(a, q) = sn * vp + cs * vq;
        }
      }
    if (!rot) break;
  }
  S = Matrix(c, 1);
  for (long q = 0; q < c; ++q) {
    double nn = 0;
    for (long a = 0; a < r; ++a) nn += U(a, q) * U(a, q);
    S(q, 0) = std::sqrt(nn);
    for (long a = 0; a < r; ++a) U(a, q) = S(q, 0) > 0 ? U(a, q) / S(q, 0) : 0.0;
  }
}

Matrix projectToStiefelManifold(const Matrix& M) {
  Matrix U, S, V;
  jacobi_svd(M, U, S, V);
  return U * V.transpose();
}

Matrix projectToRotationGroup(const Matrix& M) {
  Matrix U, S, V;
  jacobi_svd(M, U, S, V);
  if (U.determinant() * V.determinant() < 0) {
    // flip the direction of the smallest singular value (:486-490)
    long k = 0;
    for (long q = 1; q < S.rows(); ++q)
      if (S(q, 0) < S(k, 0)) k = q;
    for (long a = 0; a < U.rows(); ++a) U(a, k) = -U(a, k);
  }
  return U * V.transpose();
}

Matrix fixedStiefelVariable(unsigned d, unsigned r) {
  std::mt19937_64 rng(1);
  std::normal_distribution<double> N(0.0, 1.0);
  Matrix M(r, d);
  for (unsigned j = 0; j < d; ++j)
    for (unsigned i = 0; i < r; ++i) M(i, j) = N(rng);
  return projectToStiefelManifold(M);
}

double computeMeasurementError(const RelativeSEMeasurement& m, const Matrix& R1, const Matrix& t1, const Matrix& R2,
                               const Matrix& t2) {
  const double rot = (R1 * m.R - R2).squaredNorm();
  const double tr = (t2 - t1 - R1 * m.t).squaredNorm();
  return m.kappa * rot + m.tau * tr;
}

}  // namespace DPGO

namespace DPGO {

namespace {

// Regularized lower incomplete gamma P(a, x): series below a + 1, Lentz continued fraction above.
double gamma_p(double a, double x) {
  if (x <= 0) return 0.0;
  const double lg = std::lgamma(a);
  if (x < a + 1) {
    double term = 1.0 / a, sum = term;
    for (int k = 1; k < 10000; ++k) {
      term *= x / (a + k);
      sum += term;
      if (std::fabs(term) < std::fabs(sum) * 1e-17) break;
    }
    return sum * std::exp(-x + a * std::log(x) - lg);
  }
  const double tiny = 1e-300;
  double b = x + 1 - a, c = 1 / tiny, dd = 1 / b, h = dd;
  for (int k = 1; k < 10000; ++k) {
    const double an = -k * (k - a);
    b += 2;
    dd = an * dd + b;
    if (std::fabs(dd) < tiny) dd = tiny;
    c = b + an / c;
    if (std::fabs(c) < tiny) c = tiny;
    dd = 1 / dd;
    const double del = dd * c;
    h *= del;
    if (std::fabs(del - 1) < 1e-17) break;
  }
  return 1.0 - std::exp(-x + a * std::log(x) - lg) * h;
}

Vector ones_or(const Vector& v, size_t n, double fill) {
  if (static_cast<size_t>(v.rows()) == n && n > 0) return v;
  Vector o(static_cast<long>(n), 1);
  for (size_t i = 0; i < n; ++i) o(static_cast<long>(i), 0) = fill;
  return o;
}

}  // namespace

double chi2inv(double quantile, size_t dof) {
  if (!(quantile > 0 && quantile < 1) || dof == 0) throw std::invalid_argument("chi2inv: quantile in (0,1), dof > 0");
  const double a = 0.5 * static_cast<double>(dof);
  double lo = 0, hi = std::max(1.0, 2.0 * a);
  while (gamma_p(a, hi) < quantile) hi *= 2;
  for (int it = 0; it < 200 && hi - lo > 1e-15 * hi; ++it) {
    const double mid = 0.5 * (lo + hi);
    (gamma_p(a, mid) < quantile ? lo : hi) = mid;
  }
  return 2.0 * 0.5 * (lo + hi);  // chi2 quantile = 2 * Gamma(k/2, 1) quantile
}

double angular2ChordalSO3(double rad) { return 2 * std::sqrt(2.0) * std::sin(rad / 2); }

void checkRotationMatrix(const Matrix& R) {  // asserts in the reference (compiled out in Release)
  const long d = R.rows();
  assert(R.cols() == d);
  assert(std::fabs(R.determinant() - 1.0) < 1e-8);
  assert((R.transpose() * R - Matrix::Identity(d, d)).norm() < 1e-8);
  (void)d;
}

void singleTranslationAveraging(Vector& tOpt, const std::vector<Vector>& tVec, const Vector& tau) {
  const size_t n = tVec.size();
  if (n == 0) throw std::invalid_argument("singleTranslationAveraging: empty input");
  const Vector w = ones_or(tau, n, 1.0);
  Vector s = Matrix::Zero(tVec[0].rows(), 1);
  double ws = 0;
  for (size_t i = 0; i < n; ++i) {
    s += w(static_cast<long>(i), 0) * tVec[i];
    ws += w(static_cast<long>(i), 0);
  }
  tOpt = s * (1.0 / ws);
}

void singleRotationAveraging(Matrix& ROpt, const std::vector<Matrix>& RVec, const Vector& kappa) {
  const size_t n = RVec.size();
  if (n == 0) throw std::invalid_argument("singleRotationAveraging: empty input");
  const Vector w = ones_or(kappa, n, 1.0);
  Matrix M = Matrix::Zero(RVec[0].rows(), RVec[0].cols());
  for (size_t i = 0; i < n; ++i) M += w(static_cast<long>(i), 0) * RVec[i];
  ROpt = projectToRotationGroup(M);
}

void singlePoseAveraging(Matrix& ROpt, Vector& tOpt, const std::vector<Matrix>& RVec, const std::vector<Vector>& tVec,
                         const Vector& kappa, const Vector& tau) {
  if (RVec.empty() || RVec.size() != tVec.size()) throw std::invalid_argument("singlePoseAveraging: bad input");
  singleTranslationAveraging(tOpt, tVec, tau);
  singleRotationAveraging(ROpt, RVec, kappa);
}

namespace {

// The GNC-TLS loop shared by both robust averages (src/DPGO_utils.cpp:600-640 and :672-705):
// mu0 = min(cbar^2 / (2 max r^2 - cbar^2), 1e-5); skipped when mu0 <= 0 (all residuals small).
template <typename Solve, typename Residual>
void gnc_tls_average(size_t n, double barc, unsigned maxIters, Vector& weights, Solve solve, Residual rsq) {
  const double w_tol = 1e-8;
  solve(weights);
  double maxr = 0;
  for (size_t i = 0; i < n; ++i) maxr = std::max(maxr, rsq(i));
  const double barcSq = barc * barc;
  const double muInit = std::min(barcSq / (2 * maxr - barcSq), 1e-5);
  if (!(muInit > 0)) return;
  RobustCostParameters params;
  params.GNCBarc = barc;
  params.GNCMaxNumIters = maxIters;
  params.GNCInitMu = muInit;
  RobustCost cost(GNC_TLS, params);
  for (unsigned iter = 0; iter < maxIters; ++iter) {
    solve(weights);
    size_t nc = 0;
    for (size_t i = 0; i < n; ++i) {
      const double wi = cost.weight(std::sqrt(rsq(i)));
      if (wi < w_tol || wi > 1 - w_tol) nc++;
      weights(static_cast<long>(i), 0) = wi;
    }
    if (nc == n) break;
    cost.update();
  }
}

void inliers_of(const Vector& weights, std::vector<size_t>& idx) {
  idx.clear();
  for (long i = 0; i < weights.rows(); ++i)
    if (weights(i, 0) > 1 - 1e-8) idx.push_back(static_cast<size_t>(i));
}

}  // namespace

void robustSingleRotationAveraging(Matrix& ROpt, std::vector<size_t>& inlierIndices, const std::vector<Matrix>& RVec,
                                   const Vector& kappa, double errorThreshold) {
  const size_t n = RVec.size();
  if (n == 0) throw std::invalid_argument("robustSingleRotationAveraging: empty input");
  const Vector k = ones_or(kappa, n, 1.0);
  for (const auto& Ri : RVec) checkRotationMatrix(Ri);
  Vector w = ones_or(Vector(), n, 1.0);
  auto solve = [&](const Vector& wt) {  // kappa .* w (w = 1 for the initial estimate, :600)
    Vector kw = k;
    for (size_t i = 0; i < n; ++i) kw(static_cast<long>(i), 0) *= wt(static_cast<long>(i), 0);
    singleRotationAveraging(ROpt, RVec, kw);
  };
  auto rsq = [&](size_t i) { return k(static_cast<long>(i), 0) * (ROpt - RVec[i]).squaredNorm(); };
  gnc_tls_average(n, errorThreshold, 1000, w, solve, rsq);
  inliers_of(w, inlierIndices);
}

void robustSinglePoseAveraging(Matrix& ROpt, Vector& tOpt, std::vector<size_t>& inlierIndices,
                               const std::vector<Matrix>& RVec, const std::vector<Vector>& tVec, const Vector& kappa,
                               const Vector& tau, double errorThreshold) {
  const size_t n = RVec.size();
  if (n == 0 || tVec.size() != n) throw std::invalid_argument("robustSinglePoseAveraging: bad input");
  const Vector k = ones_or(kappa, n, 10000.0), t = ones_or(tau, n, 100.0);
  for (const auto& Ri : RVec) checkRotationMatrix(Ri);
  Vector w = ones_or(Vector(), n, 1.0);
  auto solve = [&](const Vector& wt) {
    Vector kw = k, tw = t;
    for (size_t i = 0; i < n; ++i) {
      kw(static_cast<long>(i), 0) *= wt(static_cast<long>(i), 0);
      tw(static_cast<long>(i), 0) *= wt(static_cast<long>(i), 0);
    }
    singlePoseAveraging(ROpt, tOpt, RVec, tVec, kw, tw);
  };
  auto rsq = [&](size_t i) {
    return k(static_cast<long>(i), 0) * (ROpt - RVec[i]).squaredNorm() +
           t(static_cast<long>(i), 0) * (tOpt - tVec[i]).squaredNorm();
  };
  gnc_tls_average(n, errorThreshold, 10000, w, solve, rsq);
  inliers_of(w, inlierIndices);
}

}  // namespace DPGO
