// Mirrors include/DPGO/RelativeSEMeasurement.h:21-71 of the reference.
#ifndef DPGO_AMD_RELATIVESEMEASUREMENT_H
#define DPGO_AMD_RELATIVESEMEASUREMENT_H

#include <DPGO/DPGO_types.h>

namespace DPGO {

struct RelativeSEMeasurement {
  size_t r1 = 0, r2 = 0, p1 = 0, p2 = 0;
  Matrix R;  // d x d
  Matrix t;  // d x 1
  double kappa = 0, tau = 0;
  bool isKnownInlier = false;
  double weight = 1.0;

  RelativeSEMeasurement() = default;
  RelativeSEMeasurement(size_t first_robot, size_t second_robot, size_t first_pose, size_t second_pose,
                        const Matrix& relative_rotation, const Matrix& relative_translation,
                        double rotational_precision, double translational_precision)
      : r1(first_robot), r2(second_robot), p1(first_pose), p2(second_pose), R(relative_rotation),
        t(relative_translation), kappa(rotational_precision), tau(translational_precision) {}
};

}  // namespace DPGO

#endif
