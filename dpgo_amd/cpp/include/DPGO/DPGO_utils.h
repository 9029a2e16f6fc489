// Host utilities on the hot path's input side (reference include/DPGO/DPGO_utils.h).
#ifndef DPGO_AMD_UTILS_H
#define DPGO_AMD_UTILS_H

#include <DPGO/DPGO_types.h>
#include <DPGO/RelativeSEMeasurement.h>

#include <string>
#include <vector>

namespace DPGO {

// src/DPGO_utils.cpp:78-212 with SURVEY App. B fixes (num_poses = max index + 1, blank lines skipped)
std::vector<RelativeSEMeasurement> read_g2o_file(const std::string& filename, size_t& num_poses);
// src/DPGO_utils.cpp:280-286: Q = A Omega A^T (row-major CSR, (d+1)n square)
SparseMatrix constructConnectionLaplacianSE(const std::vector<RelativeSEMeasurement>& measurements);
SparseMatrix constructConnectionLaplacianSE(const std::vector<RelativeSEMeasurement>& measurements, size_t n);
// src/DPGO_utils.cpp:426-447
Matrix odometryInitialization(size_t dimension, size_t num_poses, const std::vector<RelativeSEMeasurement>& odometry);
// src/DPGO_utils.cpp:377-424 (SPQR there; native host block Cholesky of the normal equations here)
Matrix chordalInitialization(size_t dimension, size_t num_poses, const std::vector<RelativeSEMeasurement>& measurements);
// src/DPGO_utils.cpp:478-500 (host, Jacobi SVD)
Matrix projectToRotationGroup(const Matrix& M);
Matrix projectToStiefelManifold(const Matrix& M);
// src/DPGO_utils.cpp:502-507: repo-defined seeded point of St(d, r) (ROPTLIB's RNG is not available)
Matrix fixedStiefelVariable(unsigned d, unsigned r);
// src/DPGO_utils.cpp:509-515
double computeMeasurementError(const RelativeSEMeasurement& m, const Matrix& R1, const Matrix& t1, const Matrix& R2,
                               const Matrix& t2);

// src/DPGO_utils.cpp:517-520 (boost::math chi-squared quantile there; regularized incomplete gamma
// inverted by bisection here, to ~1e-14 relative)
double chi2inv(double quantile, size_t dof);
// src/DPGO_utils.cpp:522-531
double angular2ChordalSO3(double rad);
void checkRotationMatrix(const Matrix& R);
// src/DPGO_utils.cpp:533-580: weighted averages (kappa / tau empty = all ones)
void singleTranslationAveraging(Vector& tOpt, const std::vector<Vector>& tVec, const Vector& tau = Vector());
void singleRotationAveraging(Matrix& ROpt, const std::vector<Matrix>& RVec, const Vector& kappa = Vector());
void singlePoseAveraging(Matrix& ROpt, Vector& tOpt, const std::vector<Matrix>& RVec, const std::vector<Vector>& tVec,
                         const Vector& kappa = Vector(), const Vector& tau = Vector());
// src/DPGO_utils.cpp:582-710: GNC-TLS robust averages, inlier indices in ascending order
void robustSingleRotationAveraging(Matrix& ROpt, std::vector<size_t>& inlierIndices, const std::vector<Matrix>& RVec,
                                   const Vector& kappa = Vector(), double errorThreshold = 0.1);
void robustSinglePoseAveraging(Matrix& ROpt, Vector& tOpt, std::vector<size_t>& inlierIndices,
                               const std::vector<Matrix>& RVec, const std::vector<Vector>& tVec,
                               const Vector& kappa = Vector(), const Vector& tau = Vector(),
                               double errorThreshold = 0.1);

}  // namespace DPGO

#endif
