// LiftedSEManifold -> libdpgo_hip.so (reference src/manifold/LiftedSEManifold.cpp:16-45).
#include <DPGO/manifold/LiftedSEManifold.h>
#include <dpgo_hip.h>

#include <stdexcept>
#include <string>

namespace DPGO {

LiftedSEManifold::LiftedSEManifold(int r, int d, int n) : r_(r), d_(d), n_(n) {}
LiftedSEManifold::~LiftedSEManifold() = default;

static void hip_check(int rc, const char* what) {
  if (rc != DPGO_HIP_OK) throw std::runtime_error(std::string(what) + ": " + dpgo_hip_last_error());
}

Matrix LiftedSEManifold::project(const Matrix& M) const {
  if (static_cast<size_t>(M.rows()) != r_ || static_cast<size_t>(M.cols()) != (d_ + 1) * n_)
    throw std::invalid_argument("LiftedSEManifold::project: dimension mismatch");
  Matrix X(M.rows(), M.cols());
  hip_check(dpgo_hip_project_polar(static_cast<int>(r_), static_cast<int>(d_), static_cast<int>(n_), M.data(), X.data()),
            "project");
  return X;
}

Matrix LiftedSEManifold::projectToTangent(const Matrix& X, const Matrix& V) const {
  Matrix out(V.rows(), V.cols());
  hip_check(dpgo_hip_tangent_project(static_cast<int>(r_), static_cast<int>(d_), static_cast<int>(n_), X.data(),
                                     V.data(), out.data()),
            "projectToTangent");
  return out;
}

Matrix LiftedSEManifold::retract(const Matrix& X, const Matrix& V) const {
  Matrix out(V.rows(), V.cols());
  hip_check(dpgo_hip_retract_qf(static_cast<int>(r_), static_cast<int>(d_), static_cast<int>(n_), X.data(), V.data(),
                                1.0, out.data()),
            "retract");
  return out;
}

}  // namespace DPGO
