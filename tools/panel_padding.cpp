// Panel padding of the exact preconditioner on one grid agent (measurement tool, host only): the nested-dissection
// symbolic tree of a k^3 lattice pose graph (chol.cpp supernodal_symbolic), per depth the stored 64 x 64 tile doubles
// against the factor entries they hold (lower triangle of L_SS^-1 and L_RS L_SS^-1).
//   g++ -O2 -std=c++17 -include array -include algorithm -o /tmp/panel_padding tools/panel_padding.cpp \
//       dpgo_amd/csrc/chol.cpp && /tmp/panel_padding 25
#include "../dpgo_amd/csrc/chol_internal.h"
#include <cstdio>
#include <map>
using namespace dpgo;
int main(int argc, char** argv) {
  int k = argc > 1 ? atoi(argv[1]) : 25, b = 4;
  int n = k * k * k;
  auto id = [&](int x, int y, int z) { return x + k * (y + k * z); };
  std::vector<int> rowptr(n + 1, 0), col;
  for (int z = 0; z < k; ++z) for (int y = 0; y < k; ++y) for (int x = 0; x < k; ++x) {
    std::vector<int> c{id(x, y, z)};
    if (x > 0) c.push_back(id(x - 1, y, z)); if (x + 1 < k) c.push_back(id(x + 1, y, z));
    if (y > 0) c.push_back(id(x, y - 1, z)); if (y + 1 < k) c.push_back(id(x, y + 1, z));
    if (z > 0) c.push_back(id(x, y, z - 1)); if (z + 1 < k) c.push_back(id(x, y, z + 1));
    std::sort(c.begin(), c.end());
    for (int v : c) col.push_back(v);
    rowptr[id(x, y, z) + 1] = col.size();
  }
  SupernodalFactor F; std::string err;
  if (supernodal_symbolic(n, b, rowptr, col, 1L << 40, F, err)) { printf("%s\n", err.c_str()); return 1; }
  std::map<int, std::array<double, 4>> lv;  // depth: nodes, padded doubles, useful doubles, ns tiles sum
  double P = 0, U = 0;
  for (auto& nd : F.nodes) {
    const int sb = nd.S.size() * b, tb = nd.R.size() * b;
    double pad = sn_panel_tiles(sb, tb) * 4096.0, use = sb * (sb + 1) / 2.0 + (double)tb * sb;
    auto& a = lv[nd.depth]; a[0] += 1; a[1] += pad; a[2] += use; a[3] += sn_pad(sb) / 64;
    P += pad; U += use;
  }
  printf("nodes %zu padded %.1f MB useful %.1f MB ratio %.2f\n", F.nodes.size(), P * 8e-6, U * 8e-6, P / U);
  for (auto& [d, a] : lv) printf("depth %2d nodes %5.0f padded %8.1f MB useful %8.1f MB ratio %.2f avg ns %.2f\n", d, a[0], a[1] * 8e-6, a[2] * 8e-6, a[1] / a[2], a[3] / a[0]);
}
