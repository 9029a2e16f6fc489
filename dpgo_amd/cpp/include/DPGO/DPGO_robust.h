// Robust cost weights (reference include/DPGO/DPGO_robust.h:20-68, src/DPGO_robust.cpp:23-103).
#ifndef DPGO_AMD_ROBUST_H
#define DPGO_AMD_ROBUST_H

#include <cstddef>

namespace DPGO {

enum RobustCostType { L2, L1, TLS, Huber, GM, GNC_TLS };

struct RobustCostParameters {
  unsigned GNCMaxNumIters;
  double GNCBarc, GNCMuStep, GNCInitMu, HuberThreshold, TLSThreshold;
  explicit RobustCostParameters(unsigned gncMaxIters = 100, double gncBarc = 10, double gncMuStep = 1.4,
                                double gncInitMu = 1e-4, double huberThresh = 3, double TLSThresh = 10)
      : GNCMaxNumIters(gncMaxIters), GNCBarc(gncBarc), GNCMuStep(gncMuStep), GNCInitMu(gncInitMu),
        HuberThreshold(huberThresh), TLSThreshold(TLSThresh) {}
};

class RobustCost {
 public:
  RobustCost(RobustCostType type, const RobustCostParameters& params);
  double weight(double r) const;
  void reset();
  void update();
  // include/DPGO/DPGO_robust.h:107-113: sqrt(chi2inv(quantile, 6)) for 3D measurements, 1e5 at quantile >= 1
  static double computeErrorThresholdAtQuantile(double quantile, size_t dimension);

 private:
  RobustCostType mCostType;
  RobustCostParameters mParams;
  double mu = 0;
  unsigned mGNCIteration = 0;
};

}  // namespace DPGO

#endif
