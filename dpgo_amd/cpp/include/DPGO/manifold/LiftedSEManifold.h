// LiftedSEManifold = (St(d, r) x R^r)^n  (reference include/DPGO/manifold/LiftedSEManifold.h:21-32).
// getManifold() returned a ROPTLIB object and is dropped; project() runs on the GPU.
#ifndef DPGO_AMD_LIFTEDSEMANIFOLD_H
#define DPGO_AMD_LIFTEDSEMANIFOLD_H

#include <DPGO/DPGO_types.h>

namespace DPGO {

class LiftedSEManifold {
 public:
  LiftedSEManifold(int r, int d, int n);
  ~LiftedSEManifold();
  Matrix project(const Matrix& M) const;  // src/manifold/LiftedSEManifold.cpp:34-45
  Matrix projectToTangent(const Matrix& X, const Matrix& V) const;
  Matrix retract(const Matrix& X, const Matrix& V) const;  // QF retraction

 private:
  size_t r_, d_, n_;
};

}  // namespace DPGO

#endif
