// (f2) TEASER++ robust registration (GNC-TLS rotation, adaptive-voting TLS translation,
// max-clique inlier selection) as the alternative pose solver of scripts/test_teaser.py:327-331,
// 362-435: RobustRegistrationSolver with cbar2 = 1, noise_bound = 0.05, estimate_scaling = false,
// rotation_estimation_algorithm = GNC_TLS, rotation_gnc_factor = 1.4,
// rotation_max_iterations = 100, rotation_cost_threshold = 1e-12; defaults elsewhere
// (inlier_selection_mode = PMC_EXACT, kcore_heuristic_threshold = 0.5, rotation_tim_graph =
// CHAIN). teaserpp_python is absent from the container and the TEASER-plusplus submodule is
// empty: the algorithm is restated from the published TEASER++ source (parity unpinned).
//
//   1. Translation-invariant measurements of every pair (i, j): |a_j - a_i| vs |b_j - b_i|. With no
//      scale estimation, the pair is consistent iff ||a_j - a_i| - |b_j - b_i|| <= 2 noise
//      sqrt(cbar2) (ScaleInliersSelector). The consistency graph has an edge per consistent pair.
//   2. Max clique of that graph (PMC): if the max k-core number exceeds 0.5 n, the max k-core
//      itself is taken (TEASER's k-core heuristic); otherwise an exact maximum clique. The
//      clique is sorted by correspondence index.
//   3. Chain TIMs over the clique (clique[i] -> clique[i+1], the last back to the first); GNC-TLS
//      rotation with noise bound 2 noise: weighted rotation fit, mu from the largest initial
//      residual, closed-form TLS weights, mu *= 1.4, stop on |dcost| < 1e-12 or 100 iterations;
//      rotation inliers = weights >= 0.5.
//   4. Translation: per axis, adaptive voting (scalar TLS over the 2m interval endpoints of
//      b - R a, ranges = noise sqrt(cbar2)) over the clique.
//
// MI355X split: step 1 is the O(n^2) data-parallel part (n = 5 V2 spatial-filter
// correspondences: 2.6e7 pairs per crop at V2 = 1024) and runs on the device — one workgroup
// per (crop, row), a wave's 64 column tests packed into one 64-bit adjacency word by a ballot,
// the row degree reduced in the block. Steps 2-4 are combinatorial / sequential over the
// clique (k-core peeling, branch and bound, a 3x3 fit per GNC iteration) and run as native host
// code on the downloaded bitset adjacency, crops spread over host threads.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

#include "posekern.h"
#include "common.hpp"
#include "rigid.hpp"

namespace {

constexpr int kGThreads = 256;

// grid (nmax, B): row i of crop b; thread t tests columns t, t + 256, ...; wave ballots form the
// 64-bit words of the row's adjacency bitset; the row degree is the popcount sum.
__global__ __launch_bounds__(kGThreads) void teaser_graph_kernel(const double* __restrict__ src,
                                                                 const double* __restrict__ dst,
                                                                 const int64_t* __restrict__ off, int nmax, int W,
                                                                 double beta, uint64_t* __restrict__ adj,
                                                                 int32_t* __restrict__ deg) {
  __shared__ int wsum[kGThreads / 64];
  const int b = blockIdx.y, i = blockIdx.x;
  const int64_t o = off[b];
  const int n = (int)(off[b + 1] - o);
  uint64_t* row = adj + ((int64_t)b * nmax + i) * W;
  if (i >= n) {  // padding rows: empty (block-uniform)
    for (int w = threadIdx.x; w < W; w += kGThreads) row[w] = 0ull;
    if (threadIdx.x == 0) deg[(int64_t)b * nmax + i] = 0;
    return;
  }
  const double* A = src + 3 * o;
  const double* D = dst + 3 * o;
  const double ax = A[3 * i], ay = A[3 * i + 1], az = A[3 * i + 2];
  const double bx = D[3 * i], by = D[3 * i + 1], bz = D[3 * i + 2];
  int cnt = 0;
  for (int j0 = 0; j0 < W * 64; j0 += kGThreads) {
    const int j = j0 + threadIdx.x;
    bool e = false;
    if (j < n && j != i) {
      const double sx = A[3 * j] - ax, sy = A[3 * j + 1] - ay, sz = A[3 * j + 2] - az;
      const double tx = D[3 * j] - bx, ty = D[3 * j + 1] - by, tz = D[3 * j + 2] - bz;
      const double ns = sqrt((sx * sx + sy * sy) + sz * sz);
      const double nd = sqrt((tx * tx + ty * ty) + tz * tz);
      e = fabs(ns - nd) <= beta;
    }
    const uint64_t word = __ballot(e);
    if (pk::lane_id() == 0 && (j0 >> 6) + pk::wave_id() < W) row[(j0 >> 6) + pk::wave_id()] = word;
    cnt += e ? 1 : 0;
  }
  cnt = pk::wave_sum_i32(cnt);
  if (pk::lane_id() == 0) wsum[pk::wave_id()] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < kGThreads / 64; ++w) s += wsum[w];
    deg[(int64_t)b * nmax + i] = s;
  }
}

// ------------------------------------------------------------------------------ host side

// Batagelj-Zaversnik core numbers (O(E)).
std::vector<int> core_numbers(const uint64_t* adj, int W, int n, const int32_t* deg_in) {
  std::vector<int> deg(deg_in, deg_in + n), core(n), pos(n), vert(n);
  int md = 0;
  for (int v = 0; v < n; ++v) md = std::max(md, deg[v]);
  std::vector<int> bin(md + 1, 0);
  for (int v = 0; v < n; ++v) bin[deg[v]]++;
  for (int d = 0, start = 0; d <= md; ++d) {
    const int c = bin[d];
    bin[d] = start;
    start += c;
  }
  for (int v = 0; v < n; ++v) {
    pos[v] = bin[deg[v]];
    vert[pos[v]] = v;
    bin[deg[v]]++;
  }
  for (int d = md; d >= 1; --d) bin[d] = bin[d - 1];
  if (md >= 0) bin[0] = 0;
  for (int k = 0; k < n; ++k) {
    const int v = vert[k];
    core[v] = deg[v];
    const uint64_t* row = adj + (int64_t)v * W;
    for (int w = 0; w < W; ++w) {
      uint64_t m = row[w];
      while (m) {
        const int u = w * 64 + __builtin_ctzll(m);
        m &= m - 1;
        if (deg[u] > deg[v]) {
          const int du = deg[u], pu = pos[u], pw = bin[du], wv = vert[pw];
          if (u != wv) {
            pos[u] = pw;
            vert[pu] = wv;
            pos[wv] = pu;
            vert[pw] = u;
          }
          bin[du]++;
          deg[u]--;
        }
      }
    }
  }
  return core;
}

// Exact maximum clique: bitset branch and bound with greedy colouring bounds (Tomita / San
// Segundo BBMC) on the graph renumbered by (core desc, degree desc, index asc), seeded with a
// greedy lower bound. `budget` bounds the search nodes; when it runs out the best clique found
// so far is returned and *exact = 0.
struct CliqueSearch {
  int n, W;
  std::vector<uint64_t> g;  // renumbered adjacency [n][W]
  std::vector<int> order;   // new -> old
  std::vector<int> best, cur;
  int64_t nodes = 0, budget;
  bool out_of_budget = false;

  void expand(std::vector<uint64_t>& P) {
    if (++nodes > budget) {
      out_of_budget = true;
      return;
    }
    // greedy colouring of P in index order: vertex list + colour bound
    std::vector<int> vs, col;
    std::vector<uint64_t> U(P), Q(W);
    int k = 0;
    int left = 0;
    for (int w = 0; w < W; ++w) left += __builtin_popcountll(U[w]);
    while (left > 0) {
      ++k;
      Q = U;
      for (int w = 0; w < W; ++w) {
        while (Q[w]) {
          const int v = w * 64 + __builtin_ctzll(Q[w]);
          Q[w] &= Q[w] - 1;
          U[w] &= ~(1ull << (v & 63));
          --left;
          const uint64_t* nv = &g[(int64_t)v * W];
          for (int x = w; x < W; ++x) Q[x] &= ~nv[x];
          vs.push_back(v);
          col.push_back(k);
        }
      }
    }
    for (int idx = (int)vs.size() - 1; idx >= 0; --idx) {
      if ((int)cur.size() + col[idx] <= (int)best.size()) return;
      const int v = vs[idx];
      cur.push_back(v);
      std::vector<uint64_t> NP(W);
      bool any = false;
      const uint64_t* nv = &g[(int64_t)v * W];
      for (int w = 0; w < W; ++w) {
        NP[w] = P[w] & nv[w];
        any |= NP[w] != 0;
      }
      if (!any) {
        if (cur.size() > best.size()) best = cur;
      } else {
        expand(NP);
        if (out_of_budget) return;
      }
      cur.pop_back();
      P[v >> 6] &= ~(1ull << (v & 63));
    }
  }
};

std::vector<int> max_clique(const uint64_t* adj, int W, int n, const int32_t* deg, const std::vector<int>& core,
                            int64_t budget, bool* exact) {
  *exact = true;
  std::vector<int> order(n);
  for (int v = 0; v < n; ++v) order[v] = v;
  std::sort(order.begin(), order.end(), [&](int x, int y) {
    if (core[x] != core[y]) return core[x] > core[y];
    if (deg[x] != deg[y]) return deg[x] > deg[y];
    return x < y;
  });
  std::vector<int> inv(n);
  for (int k = 0; k < n; ++k) inv[order[k]] = k;
  const int Wn = (n + 63) / 64;
  CliqueSearch cs;
  cs.n = n;
  cs.W = Wn;
  cs.budget = budget;
  cs.order = order;
  cs.g.assign((size_t)n * Wn, 0ull);
  for (int k = 0; k < n; ++k) {
    const uint64_t* row = adj + (int64_t)order[k] * W;
    uint64_t* out = &cs.g[(size_t)k * Wn];
    for (int w = 0; w < W; ++w) {
      uint64_t m = row[w];
      while (m) {
        const int u = w * 64 + __builtin_ctzll(m);
        m &= m - 1;
        const int nu = inv[u];
        out[nu >> 6] |= 1ull << (nu & 63);
      }
    }
  }
  // greedy lower bound from the first 64 vertices of the order
  for (int s = 0; s < std::min(n, 64); ++s) {
    std::vector<int> c{s};
    std::vector<uint64_t> P(cs.g.begin() + (size_t)s * Wn, cs.g.begin() + (size_t)(s + 1) * Wn);
    for (;;) {
      int pick = -1;
      for (int w = 0; w < Wn && pick < 0; ++w)
        if (P[w]) pick = w * 64 + __builtin_ctzll(P[w]);
      if (pick < 0) break;
      c.push_back(pick);
      const uint64_t* np = &cs.g[(size_t)pick * Wn];
      for (int w = 0; w < Wn; ++w) P[w] &= np[w];
    }
    if (c.size() > cs.best.size()) cs.best = c;
  }
  std::vector<uint64_t> P(Wn, 0ull);
  for (int v = 0; v < n; ++v) P[v >> 6] |= 1ull << (v & 63);
  if (n > 0 && (int)cs.best.size() <= core[order[0]]) cs.expand(P);  // core + 1 bounds the clique
  *exact = !cs.out_of_budget;
  std::vector<int> out;
  for (int v : cs.best) out.push_back(order[v]);
  std::sort(out.begin(), out.end());
  return out;
}

// Weighted rotation fit d ≈ R s (TEASER svdRot = the det-fixed SVD maximiser, here Horn's
// quaternion of pk_rigid).
void rot_fit(const std::vector<double>& s, const std::vector<double>& d, const std::vector<double>& w, double R[9]) {
  double S[3][3] = {};
  const size_t m = w.size();
  for (size_t k = 0; k < m; ++k)
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) S[r][c] += w[k] * s[3 * k + r] * d[3 * k + c];
  const double z[3] = {0.0, 0.0, 0.0};
  double t[3];
  pk_rigid::rigid_from_cov(S, z, z, R, t);
}

// scalar TLS by adaptive voting (TEASER ScalarTLSEstimator::estimate)
double scalar_tls(const std::vector<double>& X, double range, std::vector<char>* inl) {
  const int N = (int)X.size();
  std::vector<std::pair<double, int>> h;
  h.reserve(2 * N);
  for (int i = 0; i < N; ++i) {
    h.emplace_back(X[i] - range, i + 1);
    h.emplace_back(X[i] + range, -i - 1);
  }
  std::stable_sort(h.begin(), h.end(), [](const std::pair<double, int>& a, const std::pair<double, int>& b) {
    return a.first < b.first;
  });
  const double wgt = 1.0 / (range * range);
  double ranges_sum = range * N, dot_xw = 0.0, dot_w = 0.0, sum_x = 0.0, sum_x2 = 0.0;
  int card = 0;
  double best_cost = std::numeric_limits<double>::infinity(), est = 0.0;
  for (int k = 0; k < 2 * N; ++k) {
    const int idx = std::abs(h[k].second) - 1;
    const int eps = h[k].second > 0 ? 1 : -1;
    card += eps;
    dot_w += eps * wgt;
    dot_xw += eps * wgt * X[idx];
    ranges_sum -= eps * range;
    sum_x += eps * X[idx];
    sum_x2 += eps * X[idx] * X[idx];
    const double xh = dot_xw / dot_w;
    const double cost = (card * xh * xh + sum_x2 - 2 * sum_x * xh) + ranges_sum;
    if (cost < best_cost) {  // first minimum (Eigen minCoeff)
      best_cost = cost;
      est = xh;
    }
  }
  inl->assign(N, 0);
  for (int i = 0; i < N; ++i) (*inl)[i] = std::fabs(X[i] - est) <= range;
  return est;
}

void solve_one(const double* a, const double* b, int n, const uint64_t* adj, int W, const int32_t* deg,
               const pk_teaser_params& p, double* T, int32_t* clique, int32_t* csize, int32_t* info) {
  for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  info[0] = info[1] = info[2] = info[3] = 0;
  *csize = 0;
  if (n < 2) return;
  const std::vector<int> core = core_numbers(adj, W, n, deg);
  int max_core = 0;
  for (int v = 0; v < n; ++v) max_core = std::max(max_core, core[v]);
  std::vector<int> C;
  bool exact = true;
  if (p.kcore_heuristic_threshold != 1.0 && max_core > (int)(p.kcore_heuristic_threshold * (double)n)) {
    for (int v = 0; v < n; ++v)
      if (core[v] >= max_core) C.push_back(v);
    info[1] = 2;  // k-core heuristic
  } else {
    C = max_clique(adj, W, n, deg, core, p.max_clique_nodes, &exact);
    info[1] = exact ? 1 : 0;
  }
  *csize = (int32_t)C.size();
  for (size_t k = 0; k < C.size(); ++k) clique[k] = C[k];
  if (C.size() <= 1) return;  // TEASER: solution invalid
  const int m = (int)C.size();
  // chain TIMs
  std::vector<double> s(3 * m), d(3 * m), w(m, 1.0), r2(m);
  for (int k = 0; k < m; ++k) {
    const int root = C[k], leaf = C[(k + 1) % m];
    for (int c = 0; c < 3; ++c) {
      s[3 * k + c] = a[3 * leaf + c] - a[3 * root + c];
      d[3 * k + c] = b[3 * leaf + c] - b[3 * root + c];
    }
  }
  // GNC-TLS (noise bound 2 noise / scale, scale = 1)
  double nb2 = std::pow(2.0 * p.noise_bound, 2);
  if (nb2 < 1e-16) nb2 = 1e-2;
  double R[9], mu = 1.0, prev_cost = std::numeric_limits<double>::infinity();
  for (int it = 0; it < p.rotation_max_iterations; ++it) {
    rot_fit(s, d, w, R);
    double maxr = 0.0;
    for (int k = 0; k < m; ++k) {
      double e = 0.0;
      for (int r = 0; r < 3; ++r) {
        const double q = d[3 * k + r] - ((R[3 * r] * s[3 * k] + R[3 * r + 1] * s[3 * k + 1]) + R[3 * r + 2] * s[3 * k + 2]);
        e += q * q;
      }
      r2[k] = e;
      maxr = std::max(maxr, e);
    }
    if (it == 0) {
      mu = 1.0 / (2.0 * maxr / nb2 - 1.0);
      if (mu <= 0) break;
    }
    const double th1 = (mu + 1.0) / mu * nb2, th2 = mu / (mu + 1.0) * nb2;
    double cost = 0.0;
    for (int k = 0; k < m; ++k) {
      cost += w[k] * r2[k];
      if (r2[k] >= th1) w[k] = 0.0;
      else if (r2[k] <= th2) w[k] = 1.0;
      else w[k] = std::sqrt(nb2 * mu * (mu + 1.0) / r2[k]) - mu;
    }
    const double diff = std::fabs(cost - prev_cost);
    mu *= p.rotation_gnc_factor;
    prev_cost = cost;
    if (diff < p.rotation_cost_threshold) break;
  }
  int rin = 0;
  for (int k = 0; k < m; ++k) rin += w[k] >= 0.5;
  info[2] = rin;
  // translation: adaptive voting per axis over the clique
  const double range = p.noise_bound * std::sqrt(p.cbar2);
  std::vector<char> all(m, 1), tmp;
  double t[3];
  for (int r = 0; r < 3; ++r) {
    std::vector<double> X(m);
    for (int k = 0; k < m; ++k) {
      const double* ak = a + 3 * C[k];
      X[k] = b[3 * C[k] + r] - ((R[3 * r] * ak[0] + R[3 * r + 1] * ak[1]) + R[3 * r + 2] * ak[2]);
    }
    t[r] = scalar_tls(X, range, &tmp);
    for (int k = 0; k < m; ++k) all[k] &= tmp[k];
  }
  int tin = 0;
  for (int k = 0; k < m; ++k) tin += all[k];
  info[3] = tin;
  info[0] = 1;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T[4 * r + c] = R[3 * r + c];
    T[4 * r + 3] = t[r];
  }
}

}  // namespace

extern "C" int pk_teaser_graph(const double* src, const double* dst, const int64_t* off, int B, int nmax,
                               double beta, uint64_t* adj, int32_t* deg, void* stream) {
  PK_REQUIRE(B >= 0 && nmax >= 0 && beta >= 0.0);
  if (B == 0 || nmax == 0) return PK_OK;
  PK_REQUIRE(src && dst && off && adj && deg);
  const int W = (nmax + 63) / 64;
  hipLaunchKernelGGL(teaser_graph_kernel, dim3(nmax, B), dim3(kGThreads), 0, pk::as_stream(stream), src, dst, off,
                     nmax, W, beta, adj, deg);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_teaser_solve(const double* src, const double* dst, const int64_t* off, int B, int nmax,
                               const uint64_t* adj, const int32_t* deg, const pk_teaser_params* params, int threads,
                               double* T, int32_t* clique, int32_t* clique_size, int32_t* info) {
  PK_REQUIRE(B >= 0 && nmax >= 0 && params);
  if (B == 0) return PK_OK;
  PK_REQUIRE(src && dst && off && adj && deg && T && clique && clique_size && info);
  const int W = (nmax + 63) / 64;
  for (int b = 0; b < B; ++b) PK_REQUIRE(off[b + 1] - off[b] >= 0 && off[b + 1] - off[b] <= nmax);
  auto work = [&](int b) {
    const int64_t o = off[b];
    solve_one(src + 3 * o, dst + 3 * o, (int)(off[b + 1] - o), adj + (int64_t)b * nmax * W, W,
              deg + (int64_t)b * nmax, *params, T + 16 * b, clique + (int64_t)b * nmax, clique_size + b, info + 4 * b);
  };
  const int nt = std::max(1, std::min(threads, B));
  if (nt == 1) {
    for (int b = 0; b < B; ++b) work(b);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
      pool.emplace_back([&, t] {
        for (int b = t; b < B; b += nt) work(b);
      });
    for (auto& th : pool) th.join();
  }
  return PK_OK;
}
