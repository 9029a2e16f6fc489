// DPGO types for the MI355X drop-in (mirrors include/DPGO/DPGO_types.h:20-68 of the reference).
// Eigen is not part of this build, so Matrix / SparseMatrix are small self-contained types with
// the subset of the Eigen API the reference's call sites use on this path.
#ifndef DPGO_AMD_TYPES_H
#define DPGO_AMD_TYPES_H

#include <cmath>
#include <cstddef>
#include <map>
#include <stdexcept>
#include <utility>
#include <vector>

namespace DPGO {

// Dense column-major double matrix (Eigen::MatrixXd subset).
class Matrix {
 public:
  Matrix() = default;
  Matrix(long rows, long cols) : r_(rows), c_(cols), v_(static_cast<size_t>(rows * cols), 0.0) {}
  static Matrix Zero(long rows, long cols) { return Matrix(rows, cols); }
  static Matrix Identity(long rows, long cols) {
    Matrix M(rows, cols);
    for (long i = 0; i < std::min(rows, cols); ++i) M(i, i) = 1.0;
    return M;
  }
  long rows() const { return r_; }
  long cols() const { return c_; }
  long size() const { return r_ * c_; }
  double* data() { return v_.data(); }
  const double* data() const { return v_.data(); }
  double& operator()(long i, long j) { return v_[static_cast<size_t>(j * r_ + i)]; }
  double operator()(long i, long j) const { return v_[static_cast<size_t>(j * r_ + i)]; }
  void resize(long rows, long cols) {
    r_ = rows;
    c_ = cols;
    v_.assign(static_cast<size_t>(rows * cols), 0.0);
  }
  void setZero() { std::fill(v_.begin(), v_.end(), 0.0); }

  Matrix block(long i, long j, long p, long q) const {
    Matrix B(p, q);
    for (long b = 0; b < q; ++b)
      for (long a = 0; a < p; ++a) B(a, b) = (*this)(i + a, j + b);
    return B;
  }
  void setBlock(long i, long j, const Matrix& B) {
    for (long b = 0; b < B.cols(); ++b)
      for (long a = 0; a < B.rows(); ++a) (*this)(i + a, j + b) = B(a, b);
  }
  Matrix transpose() const {
    Matrix T(c_, r_);
    for (long j = 0; j < c_; ++j)
      for (long i = 0; i < r_; ++i) T(j, i) = (*this)(i, j);
    return T;
  }
  double squaredNorm() const {
    double s = 0.0;
    for (double x : v_) s += x * x;
    return s;
  }
  double norm() const { return std::sqrt(squaredNorm()); }
  double sum() const {
    double s = 0.0;
    for (double x : v_) s += x;
    return s;
  }
  double determinant() const;  // d <= 4, LU with partial pivoting
  Matrix inverse() const;      // Gauss-Jordan

  Matrix& operator+=(const Matrix& o) {
    check_same(o);
    for (size_t k = 0; k < v_.size(); ++k) v_[k] += o.v_[k];
    return *this;
  }
  Matrix& operator-=(const Matrix& o) {
    check_same(o);
    for (size_t k = 0; k < v_.size(); ++k) v_[k] -= o.v_[k];
    return *this;
  }
  Matrix& operator*=(double s) {
    for (double& x : v_) x *= s;
    return *this;
  }
  friend Matrix operator+(Matrix a, const Matrix& b) { return a += b; }
  friend Matrix operator-(Matrix a, const Matrix& b) { return a -= b; }
  friend Matrix operator*(Matrix a, double s) { return a *= s; }
  friend Matrix operator*(double s, Matrix a) { return a *= s; }
  friend Matrix operator-(Matrix a) { return a *= -1.0; }
  friend Matrix operator*(const Matrix& a, const Matrix& b) {
    if (a.cols() != b.rows()) throw std::invalid_argument("Matrix product: dimension mismatch");
    Matrix C(a.rows(), b.cols());
    for (long j = 0; j < b.cols(); ++j)
      for (long k = 0; k < a.cols(); ++k) {
        const double bk = b(k, j);
        for (long i = 0; i < a.rows(); ++i) C(i, j) += a(i, k) * bk;
      }
    return C;
  }

 private:
  void check_same(const Matrix& o) const {
    if (o.r_ != r_ || o.c_ != c_) throw std::invalid_argument("Matrix: dimension mismatch");
  }
  long r_ = 0, c_ = 0;
  std::vector<double> v_;
};

typedef Matrix Vector;  // column vector (cols() == 1)

// Row-major CSR with int32 indices (Eigen::SparseMatrix<double, Eigen::RowMajor> subset).
class SparseMatrix {
 public:
  SparseMatrix() = default;
  SparseMatrix(long rows, long cols) : r_(rows), c_(cols), outer_(static_cast<size_t>(rows) + 1, 0) {}
  long rows() const { return r_; }
  long cols() const { return c_; }
  long nonZeros() const { return static_cast<long>(inner_.size()); }
  const int* outerIndexPtr() const { return outer_.data(); }
  const int* innerIndexPtr() const { return inner_.data(); }
  const double* valuePtr() const { return val_.data(); }
  // Build from (row, col, value) triplets; duplicates are summed.
  void setFromTriplets(const std::vector<std::pair<std::pair<int, int>, double>>& t);
  double coeff(long i, long j) const;
  Matrix toDense() const;

 private:
  long r_ = 0, c_ = 0;
  std::vector<int> outer_{0}, inner_;
  std::vector<double> val_;
};

enum ROPTALG { RTR, RGD };

enum tCGstatusSet { TR_NEGCURVTURE = 0, TR_EXCREGION = 1, TR_LCON = 2, TR_SCON = 3, TR_MAXITER = 4 };

struct ROPTResult {
  ROPTResult(bool suc = false, double f0 = 0, double gn0 = 0, double fStar = 0, double gnStar = 0,
             double relchange = 0, double ms = 0)
      : success(suc), fInit(f0), gradNormInit(gn0), fOpt(fStar), gradNormOpt(gnStar),
        relativeChange(relchange), elapsedMs(ms) {}
  bool success;
  double fInit;
  double gradNormInit;
  double fOpt;
  double gradNormOpt;
  double relativeChange;
  double elapsedMs;
  int tCGStatus = -1;  // tCGstatusSet of the last tCG (-1: none ran)
};

typedef std::pair<unsigned, unsigned> PoseID;
typedef std::map<PoseID, Matrix> PoseDict;

}  // namespace DPGO

#endif
