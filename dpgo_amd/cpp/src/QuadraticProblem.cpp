// QuadraticProblem -> libdpgo_hip.so (reference src/QuadraticProblem.cpp:16-101).
#include <DPGO/QuadraticProblem.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace DPGO {

static void hip_check(int rc, const char* what) {
  if (rc != DPGO_HIP_OK) throw std::runtime_error(std::string(what) + ": " + dpgo_hip_last_error());
}

QuadraticProblem::QuadraticProblem(size_t nIn, size_t dIn, size_t rIn) : n(nIn), d(dIn), r(rIn) {
  if (r < d) throw std::invalid_argument("QuadraticProblem: r < d");
  hip_check(dpgo_hip_problem_create(static_cast<int>(n), static_cast<int>(d), static_cast<int>(r), &h),
            "dpgo_hip_problem_create");
  // PreConditioner applies the factor of Q + 0.1 I, as the reference's CHOLMOD solver (:37-41, :75-87)
  hip_check(dpgo_hip_set_precon(h, DPGO_PRECON_EXACT), "dpgo_hip_set_precon");
  // ctor sets empty Q and G (:23-24)
  mQ = SparseMatrix(static_cast<long>((d + 1) * n), static_cast<long>((d + 1) * n));
  mG = SparseMatrix(static_cast<long>(r), static_cast<long>((d + 1) * n));
}

QuadraticProblem::~QuadraticProblem() { dpgo_hip_problem_destroy(h); }

void QuadraticProblem::setQ(const SparseMatrix& QIn) {
  if (static_cast<size_t>(QIn.rows()) != (d + 1) * n || static_cast<size_t>(QIn.cols()) != (d + 1) * n)
    throw std::invalid_argument("setQ: Q must be (d+1)n x (d+1)n");
  mQ = QIn;
  hip_check(dpgo_hip_set_Q_csr(h, 0, static_cast<int>(QIn.rows()), QIn.outerIndexPtr(), QIn.innerIndexPtr(),
                               QIn.valuePtr()),
            "setQ");
}

void QuadraticProblem::setG(const SparseMatrix& GIn) {
  if (static_cast<size_t>(GIn.rows()) != r || static_cast<size_t>(GIn.cols()) != (d + 1) * n)
    throw std::invalid_argument("setG: G must be r x (d+1)n");
  mG = GIn;
  const Matrix Gd = GIn.toDense();
  hip_check(dpgo_hip_set_G_dense(h, 0, Gd.data()), "setG");
}

void QuadraticProblem::check(const Matrix& Y) const {
  if (static_cast<size_t>(Y.rows()) != r || static_cast<size_t>(Y.cols()) != (d + 1) * n)
    throw std::invalid_argument("QuadraticProblem: X must be r x (d+1)n");
}

double QuadraticProblem::f(const Matrix& Y) const {
  check(Y);
  double fv = 0.0;
  hip_check(dpgo_hip_f(h, Y.data(), &fv), "f");
  return fv;
}

Matrix QuadraticProblem::EucGrad(const Matrix& Y) const {
  check(Y);
  Matrix out(Y.rows(), Y.cols());
  hip_check(dpgo_hip_egrad(h, Y.data(), out.data()), "EucGrad");
  return out;
}

Matrix QuadraticProblem::EucHessianEta(const Matrix& V) const {
  check(V);
  Matrix out(V.rows(), V.cols());
  hip_check(dpgo_hip_ehvp(h, V.data(), out.data()), "EucHessianEta");
  return out;
}

Matrix QuadraticProblem::RieHessianEta(const Matrix& Y, const Matrix& V) const {
  check(Y);
  check(V);
  Matrix out(V.rows(), V.cols());
  hip_check(dpgo_hip_rhvp(h, Y.data(), V.data(), out.data()), "RieHessianEta");
  return out;
}

Matrix QuadraticProblem::PreConditioner(const Matrix& Y, const Matrix& V) const {
  check(Y);
  check(V);
  Matrix out(V.rows(), V.cols());
  hip_check(dpgo_hip_precondition(h, Y.data(), V.data(), out.data()), "PreConditioner");
  return out;
}

Matrix QuadraticProblem::RieGrad(const Matrix& Y) const {
  check(Y);
  Matrix out(Y.rows(), Y.cols());
  double nrm = 0.0;
  hip_check(dpgo_hip_riegrad(h, Y.data(), out.data(), &nrm, nullptr), "RieGrad");
  return out;
}

double QuadraticProblem::RieGradNorm(const Matrix& Y) const {
  check(Y);
  double nrm = 0.0;
  hip_check(dpgo_hip_riegrad(h, Y.data(), nullptr, &nrm, nullptr), "RieGradNorm");
  return nrm;
}

}  // namespace DPGO
