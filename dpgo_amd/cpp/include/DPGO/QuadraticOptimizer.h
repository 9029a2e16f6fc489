// QuadraticOptimizer on MI355X: RTR (truncated CG) or one RGD step, fully on device.
// Mirrors include/DPGO/QuadraticOptimizer.h:22-76 of the reference.
#ifndef DPGO_AMD_QUADRATICOPTIMIZER_H
#define DPGO_AMD_QUADRATICOPTIMIZER_H

#include <DPGO/DPGO_types.h>
#include <DPGO/QuadraticProblem.h>

namespace DPGO {

class QuadraticOptimizer {
 public:
  explicit QuadraticOptimizer(QuadraticProblem* p);
  ~QuadraticOptimizer();

  Matrix optimize(const Matrix& Y);

  void setProblem(QuadraticProblem* p) { problem = p; }
  void setVerbose(bool v) { verbose = v; }
  void setAlgorithm(ROPTALG alg) { algorithm = alg; }
  void setGradientDescentStepsize(double s) { gradientDescentStepsize = s; }
  void setTrustRegionIterations(unsigned iter) { trustRegionIterations = iter; }
  void setTrustRegionTolerance(double tol) { trustRegionTolerance = tol; }
  void setTrustRegionInitialRadius(double radius) { trustRegionInitialRadius = radius; }
  void setTrustRegionMaxInnerIterations(int iter) { trustRegionMaxInnerIterations = iter; }
  // Extension (the reference always uses its CHOLMOD factor): DPGO_PRECON_EXACT (default, the
  // factor of Q + 0.1 I), DPGO_PRECON_BLOCK_JACOBI (per-pose blocks, the throughput setting) or
  // DPGO_PRECON_NONE; see DESIGN.md section 7.
  void setPreconditioner(int mode) { preconditioner = mode; }

  ROPTResult getOptResult() const { return result; }

 private:
  QuadraticProblem* problem;
  ROPTALG algorithm;
  ROPTResult result;
  double gradientDescentStepsize;
  unsigned trustRegionIterations;
  double trustRegionTolerance;
  double trustRegionInitialRadius;
  int trustRegionMaxInnerIterations;
  bool verbose;
  int preconditioner;
};

}  // namespace DPGO

#endif
