// QuadraticOptimizer -> dpgo_hip_optimize (reference src/QuadraticOptimizer.cpp:20-149).
#include <DPGO/QuadraticOptimizer.h>

#include <cstdio>
#include <stdexcept>
#include <string>

namespace DPGO {

QuadraticOptimizer::QuadraticOptimizer(QuadraticProblem* p)
    : problem(p), algorithm(ROPTALG::RTR), gradientDescentStepsize(1e-3), trustRegionIterations(1),
      trustRegionTolerance(1e-2), trustRegionInitialRadius(1e1), trustRegionMaxInnerIterations(50), verbose(false),
      preconditioner(DPGO_PRECON_EXACT) {
  result.success = false;
}

QuadraticOptimizer::~QuadraticOptimizer() = default;

Matrix QuadraticOptimizer::optimize(const Matrix& Y) {
  dpgo_opt_params p;
  dpgo_hip_default_params(&p);
  p.algorithm = algorithm == ROPTALG::RTR ? DPGO_ALG_RTR : DPGO_ALG_RGD;
  p.rgd_stepsize = gradientDescentStepsize;
  p.tr_iterations = static_cast<int>(trustRegionIterations);
  p.tr_tolerance = trustRegionTolerance;
  p.tr_initial_radius = trustRegionInitialRadius;
  p.tr_max_inner = trustRegionMaxInnerIterations;
  p.verbose = verbose ? 1 : 0;
  p.precon = preconditioner;
  Matrix YOpt(Y.rows(), Y.cols());
  dpgo_opt_result res;
  const int rc = dpgo_hip_optimize(problem->handle(), &p, Y.data(), YOpt.data(), &res);
  if (rc != DPGO_HIP_OK) throw std::runtime_error(std::string("optimize: ") + dpgo_hip_last_error());
  result = ROPTResult(res.success != 0, res.fInit, res.gradNormInit, res.fOpt, res.gradNormOpt, res.relativeChange,
                      res.elapsedMs);
  result.tCGStatus = res.tCGStatus;
  if (res.gave_up) std::printf("Too many RTR rejections. Returning initial guess.\n");  // :102-104
  return YOpt;
}

}  // namespace DPGO
