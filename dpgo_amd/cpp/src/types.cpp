// DPGO::Matrix / SparseMatrix helpers (host).
#include <DPGO/DPGO_types.h>

#include <algorithm>

namespace DPGO {

double Matrix::determinant() const {
  if (r_ != c_) throw std::invalid_argument("determinant of a non-square matrix");
  Matrix A = *this;
  double det = 1.0;
  for (long c = 0; c < r_; ++c) {
    long piv = c;
    for (long i = c + 1; i < r_; ++i)
      if (std::fabs(A(i, c)) > std::fabs(A(piv, c))) piv = i;
    if (A(piv, c) == 0.0) return 0.0;
    if (piv != c) {
      for (long j = 0; j < r_; ++j) std::swap(A(c, j), A(piv, j));
      det = -det;
    }
    det *= A(c, c);
    for (long i = c + 1; i < r_; ++i) {
      const double f = A(i, c) / A(c, c);
      for (long j = c; j < r_; ++j) A(i, j) -= f * A(c, j);
    }
  }
  return det;
}

Matrix Matrix::inverse() const {
  if (r_ != c_) throw std::invalid_argument("inverse of a non-square matrix");
  const long n = r_;
  Matrix A = *this, I = Identity(n, n);
  for (long c = 0; c < n; ++c) {
    long piv = c;
    for (long i = c + 1; i < n; ++i)
      if (std::fabs(A(i, c)) > std::fabs(A(piv, c))) piv = i;
    if (A(piv, c) == 0.0) throw std::runtime_error("singular matrix");
    for (long j = 0; j < n; ++j) {
      std::swap(A(c, j), A(piv, j));
      std::swap(I(c, j), I(piv, j));
    }
    const double inv = 1.0 / A(c, c);
    for (long j = 0; j < n; ++j) {
      A(c, j) *= inv;
      I(c, j) *= inv;
    }
    for (long i = 0; i < n; ++i)
      if (i != c) {
        const double f = A(i, c);
        for (long j = 0; j < n; ++j) {
          A(i, j) -= f * A(c, j);
          I(i, j) -= f * I(c, j);
        }
      }
  }
  return I;
}

void SparseMatrix::setFromTriplets(const std::vector<std::pair<std::pair<int, int>, double>>& t) {
  std::vector<std::pair<std::pair<int, int>, double>> s(t);
  std::stable_sort(s.begin(), s.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  outer_.assign(static_cast<size_t>(r_) + 1, 0);
  inner_.clear();
  val_.clear();
  for (size_t k = 0; k < s.size();) {
    size_t e = k;
    double v = 0.0;
    while (e < s.size() && s[e].first == s[k].first) v += s[e++].second;
    inner_.push_back(s[k].first.second);
    val_.push_back(v);
    outer_[s[k].first.first + 1]++;
    k = e;
  }
  for (long i = 0; i < r_; ++i) outer_[i + 1] += outer_[i];
}

double SparseMatrix::coeff(long i, long j) const {
  for (int k = outer_[i]; k < outer_[i + 1]; ++k)
    if (inner_[k] == j) return val_[k];
  return 0.0;
}

Matrix SparseMatrix::toDense() const {
  Matrix M(r_, c_);
  for (long i = 0; i < r_; ++i)
    for (int k = outer_[i]; k < outer_[i + 1]; ++k) M(i, inner_[k]) += val_[k];
  return M;
}

}  // namespace DPGO
