// QuadraticProblem on MI355X: f(X) = 0.5 <Q, X^T X> + <X, G> over (St(d,r) x R^r)^n.
// Public API mirrors include/DPGO/QuadraticProblem.h:33-109 of the reference; the ROPTLIB
// virtuals (f / EucGrad / EucHessianEta / PreConditioner on ROPTLIB::Variable) become
// Matrix-valued methods.  Every evaluation runs on the GPU through libdpgo_hip.so.
#ifndef DPGO_AMD_QUADRATICPROBLEM_H
#define DPGO_AMD_QUADRATICPROBLEM_H

#include <DPGO/DPGO_types.h>
#include <dpgo_hip.h>

namespace DPGO {

class QuadraticProblem {
 public:
  QuadraticProblem(size_t nIn, size_t dIn, size_t rIn);
  ~QuadraticProblem();
  QuadraticProblem(const QuadraticProblem&) = delete;
  QuadraticProblem& operator=(const QuadraticProblem&) = delete;

  unsigned int num_poses() const { return static_cast<unsigned>(n); }
  unsigned int dimension() const { return static_cast<unsigned>(d); }
  unsigned int relaxation_rank() const { return static_cast<unsigned>(r); }

  SparseMatrix getQ() const { return mQ; }
  SparseMatrix getG() const { return mG; }
  void setQ(const SparseMatrix& QIn);  // src/QuadraticProblem.cpp:31-42
  void setG(const SparseMatrix& GIn);  // :44-48

  double f(const Matrix& Y) const;                                // :50-55
  Matrix EucGrad(const Matrix& Y) const;                          // :62-66
  Matrix EucHessianEta(const Matrix& V) const;                    // :68-73
  Matrix RieHessianEta(const Matrix& Y, const Matrix& V) const;   // ROPTLIB HessianEta
  Matrix PreConditioner(const Matrix& Y, const Matrix& V) const;  // :75-87 (exact factor of Q + 0.1 I)
  Matrix RieGrad(const Matrix& Y) const;                          // :89-97
  double RieGradNorm(const Matrix& Y) const;                      // :99-101

  dpgo_hip_problem handle() const { return h; }

 private:
  void check(const Matrix& Y) const;
  const size_t n, d, r;
  SparseMatrix mQ, mG;
  dpgo_hip_problem h = nullptr;
};

}  // namespace DPGO

#endif
