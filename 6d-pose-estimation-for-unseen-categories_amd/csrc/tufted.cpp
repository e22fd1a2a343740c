// f1 — the intrinsic stage of robust_laplacian.point_cloud_laplacian (host code, C++17).
//
// Reference: dataset/object.py:246 geometry.get_operators(verts=pcd_depth, faces=[]) ->
// diffusion-net compute_operators -> robust_laplacian.point_cloud_laplacian(verts,
// mollify_factor=1e-5, n_neighbors=30) (third-party, absent from /root/reference; restated from
// Sharp & Crane, "A Laplacian for Nonmanifold Triangle Meshes", SGP 2020, and the published
// robust-laplacians-py / geometry-central algorithm):
//   1. the union of every point's local Delaunay fan (pk_pc_local_tri, on the device) is a
//      nonmanifold triangle soup in which a triangle appears up to three times;
//   2. intrinsic mollification: with eps = mollify_factor * (mean length of the distinct soup
//      edges), delta = max(0, max over every triangle corner of l_c - l_a - l_b + eps) is added
//      to every edge length, so every triangle is strictly non-degenerate;
//   3. the tufted cover: each soup face becomes two oppositely oriented copies; around each soup
//      edge the incident faces are sorted by their angle about the edge and the copy of face i
//      facing the next face is glued to that face's copy facing back (a face alone on an edge is
//      glued to its own back); the cover is a closed, oriented, manifold Delta-complex with the
//      soup's edge lengths;
//   4. intrinsic Delaunay flips on the cover until every edge's cotan weight
//      (cot alpha + cot beta) / 2 >= -1e-12 (lengths of flipped edges from the quad's planar layout);
//   5. the cotan Laplacian and the lumped mass (area / 3 per corner) of the flipped cover, times
//      1/2 (the cover counts every soup face twice) times 1/3 (the soup counts a triangle up to
//      three times).
// Without flips and mollification this is exactly pk_cotan_dense's soup Laplacian at scale 1/3.
// The flip loop is a sequential graph algorithm over ~10^5 edges per crop: it runs on the host
// next to the device stages (the reference runs the whole operator build on the CPU), one call
// per cloud; the device takes the result back as dense L (dpfm_amd/geometry.py).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <deque>
#include <unordered_map>
#include <vector>

#include "posekern.h"

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr int kOk = 0, kErrArg = 1000;  // csrc/common.hpp PK_OK / PK_ERR_ARG (this TU is plain C++)

struct Cover {
  // halfedge h lives in face h / 3 at corner h % 3: tail vertex vtx[h], twin[h], edge id eid[h];
  // next(h) = 3 (h / 3) + (h % 3 + 1) % 3
  std::vector<int32_t> vtx, twin, eid;
  std::vector<double> len;  // per cover edge
  static int nxt(int h) { return 3 * (h / 3) + (h % 3 + 1) % 3; }
  static int prv(int h) { return 3 * (h / 3) + (h % 3 + 2) % 3; }
};

double face_area(double a, double b, double c) {  // Heron, clamped at 0
  const double s = 0.5 * (a + b + c);
  const double arg = s * (s - a) * (s - b) * (s - c);
  return arg > 0.0 ? std::sqrt(arg) : 0.0;
}

// cot of the angle opposite halfedge h in its face, from the three edge lengths
double cot_opp(const Cover& C, int h) {
  const double lc = C.len[C.eid[h]], la = C.len[C.eid[Cover::nxt(h)]], lb = C.len[C.eid[Cover::prv(h)]];
  const double A = face_area(la, lb, lc);
  return (la * la + lb * lb - lc * lc) / (4.0 * A);
}

double edge_weight(const Cover& C, int h) { return 0.5 * (cot_opp(C, h) + cot_opp(C, C.twin[h])); }

// Flip the edge of halfedge h (faces (i, j, k) and (j, i, l)) to (k, l); returns the flipped
// edge's halfedge k -> l (corner 0 of h's face), or -1 when both sides lie in one face (not a
// flippable diamond).
int flip(Cover& C, int h) {
  const int t = C.twin[h];
  const int f1 = h / 3, f2 = t / 3;
  if (f1 == f2) return -1;
  const int a = Cover::nxt(h), b = Cover::prv(h);  // j -> k, k -> i
  const int c = Cover::nxt(t), d = Cover::prv(t);  // i -> l, l -> j
  const int vi = C.vtx[h], vj = C.vtx[t], vk = C.vtx[b], vl = C.vtx[d];
  // planar layout: i = (0, 0), j = (L, 0), k above, l below
  const double L = C.len[C.eid[h]];
  const double lik = C.len[C.eid[b]], ljk = C.len[C.eid[a]], lil = C.len[C.eid[c]], ljl = C.len[C.eid[d]];
  const double kx = (L * L + lik * lik - ljk * ljk) / (2.0 * L), ky = std::sqrt(std::max(0.0, lik * lik - kx * kx));
  const double lx = (L * L + lil * lil - ljl * ljl) / (2.0 * L), ly = -std::sqrt(std::max(0.0, lil * lil - lx * lx));
  const double nl = std::hypot(kx - lx, ky - ly);
  // new faces: f1 = (k -> l, l -> j, j -> k), f2 = (l -> k, k -> i, i -> l)
  const int s0 = 3 * f1, s1 = s0 + 1, s2 = s0 + 2, u0 = 3 * f2, u1 = u0 + 1, u2 = u0 + 2;
  const int outer[4] = {a, b, c, d}, dest[4] = {s2, u1, u2, s1};
  int otw[4], oe[4];
  for (int q = 0; q < 4; ++q) {
    otw[q] = C.twin[outer[q]];
    oe[q] = C.eid[outer[q]];
  }
  auto remap = [&](int x) {
    for (int q = 0; q < 4; ++q)
      if (x == outer[q]) return dest[q];
    return -1;
  };
  const int e = C.eid[h];
  const int nv[6] = {vk, vl, vj, vl, vk, vi};
  const int slot[6] = {s0, s1, s2, u0, u1, u2};
  for (int q = 0; q < 6; ++q) C.vtx[slot[q]] = nv[q];
  C.eid[s0] = e;
  C.eid[u0] = e;
  C.twin[s0] = u0;
  C.twin[u0] = s0;
  for (int q = 0; q < 4; ++q) {
    const int nd = dest[q];
    C.eid[nd] = oe[q];
    const int r = remap(otw[q]);
    if (r >= 0) {
      C.twin[nd] = r;
    } else {
      C.twin[nd] = otw[q];
      C.twin[otw[q]] = nd;
    }
  }
  C.len[e] = nl;
  return s0;
}

}  // namespace

extern "C" int pk_tufted_laplacian(const double* pts, int64_t n, const int32_t* tri, int64_t ntri,
                                   double mollify_factor, int64_t cap, int32_t* ii, int32_t* jj, double* ww,
                                   int64_t* nnz, double* mass, int64_t* nflips) {
  if (n < 0 || ntri < 0 || cap < 0 || !nnz || !mass || (ntri > 0 && (!pts || !tri))) return kErrArg;
  for (int64_t v = 0; v < n; ++v) mass[v] = 0.0;
  *nnz = 0;
  if (nflips) *nflips = 0;
  if (ntri == 0) return kOk;
  for (int64_t f = 0; f < ntri; ++f)
    for (int r = 0; r < 3; ++r) {
      const int32_t v = tri[3 * f + r];
      if (v < 0 || v >= n || v == tri[3 * f + (r + 1) % 3]) return kErrArg;
    }
  const int64_t F = ntri;
  auto P = [&](int v, int d) { return pts[3 * (int64_t)v + d]; };
  auto dist = [&](int u, int v) {
    const double dx = P(u, 0) - P(v, 0), dy = P(u, 1) - P(v, 1), dz = P(u, 2) - P(v, 2);
    return std::sqrt(dx * dx + dy * dy + dz * dz);
  };
  // distinct soup edges (u < v) and the faces around each
  std::unordered_map<uint64_t, int32_t> emap;
  emap.reserve((size_t)F * 2);
  std::vector<std::vector<int32_t>> around;  // per soup edge: corner halfedges 3 f + r (front copy)
  std::vector<double> slen;
  std::vector<int32_t> sedge((size_t)F * 3);
  for (int64_t f = 0; f < F; ++f)
    for (int r = 0; r < 3; ++r) {
      const int u = tri[3 * f + r], v = tri[3 * f + (r + 1) % 3];
      const uint64_t key = ((uint64_t)(uint32_t)std::min(u, v) << 32) | (uint32_t)std::max(u, v);
      auto it = emap.find(key);
      int32_t e;
      if (it == emap.end()) {
        e = (int32_t)slen.size();
        emap.emplace(key, e);
        slen.push_back(dist(u, v));
        around.emplace_back();
      } else {
        e = it->second;
      }
      sedge[3 * f + r] = e;
      around[e].push_back((int32_t)(3 * f + r));
    }
  // mollification
  double mean = 0.0;
  for (double l : slen) mean += l;
  mean /= (double)slen.size();
  const double eps = mollify_factor * mean;
  double delta = 0.0;
  for (int64_t f = 0; f < F; ++f)
    for (int r = 0; r < 3; ++r) {
      const double la = slen[sedge[3 * f + r]], lb = slen[sedge[3 * f + (r + 1) % 3]];
      const double lc = slen[sedge[3 * f + (r + 2) % 3]];
      delta = std::max(delta, lc - la - lb + eps);
    }
  if (mollify_factor > 0.0)
    for (double& l : slen) l += delta;
  // tufted cover: face f -> copies 2 f (a, b, c) and 2 f + 1 (a, c, b)
  Cover C;
  C.vtx.resize((size_t)F * 6);
  C.twin.assign((size_t)F * 6, -1);
  C.eid.resize((size_t)F * 6);
  for (int64_t f = 0; f < F; ++f) {
    const int a = tri[3 * f], b = tri[3 * f + 1], c = tri[3 * f + 2];
    const int64_t fr = 6 * f, bk = 6 * f + 3;
    C.vtx[fr] = a; C.vtx[fr + 1] = b; C.vtx[fr + 2] = c;
    C.vtx[bk] = a; C.vtx[bk + 1] = c; C.vtx[bk + 2] = b;
  }
  // the back copy's halfedge along front corner r (edge r -> r + 1 reversed): corner (3 - r) % 3
  // of (a, c, b): r = 0 (a -> b) <-> b -> a = corner 2; r = 1 (b -> c) <-> c -> b = corner 1;
  // r = 2 (c -> a) <-> a -> c = corner 0
  auto back_of = [](int64_t f, int r) { return (int32_t)(6 * f + 3 + (r == 0 ? 2 : r == 1 ? 1 : 0)); };
  std::vector<std::pair<double, int32_t>> fins;
  for (size_t e = 0; e < around.size(); ++e) {
    const auto& hs = around[e];
    // the soup edge u -> v with u < v; fin angle of each face about the axis v - u
    const int h0 = hs[0];
    const int64_t f0 = h0 / 3;
    const int r0 = h0 % 3;
    int u = tri[3 * f0 + r0], v = tri[3 * f0 + (r0 + 1) % 3];
    if (u > v) std::swap(u, v);
    double ax[3] = {P(v, 0) - P(u, 0), P(v, 1) - P(u, 1), P(v, 2) - P(u, 2)};
    const double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    for (double& x : ax) x /= an > 0.0 ? an : 1.0;
    double e1[3] = {0, 0, 0}, e2[3];
    fins.clear();
    bool have_ref = false;
    for (int32_t h : hs) {
      const int64_t f = h / 3;
      const int r = h % 3;
      const int w = tri[3 * f + (r + 2) % 3];
      double p[3] = {P(w, 0) - P(u, 0), P(w, 1) - P(u, 1), P(w, 2) - P(u, 2)};
      const double pa = p[0] * ax[0] + p[1] * ax[1] + p[2] * ax[2];
      for (int d = 0; d < 3; ++d) p[d] -= pa * ax[d];
      if (!have_ref) {  // the first fin's direction is angle 0
        const double pn = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
        if (pn > 0.0) {
          for (int d = 0; d < 3; ++d) e1[d] = p[d] / pn;
          e2[0] = ax[1] * e1[2] - ax[2] * e1[1];
          e2[1] = ax[2] * e1[0] - ax[0] * e1[2];
          e2[2] = ax[0] * e1[1] - ax[1] * e1[0];
          have_ref = true;
        }
      }
      const double x = have_ref ? p[0] * e1[0] + p[1] * e1[1] + p[2] * e1[2] : 0.0;
      const double y = have_ref ? p[0] * e2[0] + p[1] * e2[1] + p[2] * e2[2] : 0.0;
      double th = std::atan2(y, x);
      if (th < 0.0) th += 2.0 * kPi;
      fins.emplace_back(th, h);
    }
    std::stable_sort(fins.begin(), fins.end(),
                     [](const std::pair<double, int32_t>& p, const std::pair<double, int32_t>& q) {
                       return p.first < q.first;
                     });
    // copy of fin i with halfedge u -> v (faces the next fin) glued to the next fin's copy with
    // v -> u; the front copy of face f runs its corner r from tri[r] to tri[r + 1]
    const size_t m = fins.size();
    for (size_t i = 0; i < m; ++i) {
      const int32_t h = fins[i].second, hn = fins[(i + 1) % m].second;
      const int64_t f = h / 3, fn = hn / 3;
      const int r = h % 3, rn = hn % 3;
      const bool fwd = tri[3 * f + r] == u;     // front corner runs u -> v
      const bool fwdn = tri[3 * fn + rn] == u;
      const int32_t A = fwd ? (int32_t)(6 * f + r) : back_of(f, r);      // u -> v side of fin i
      const int32_t B = fwdn ? back_of(fn, rn) : (int32_t)(6 * fn + rn);  // v -> u side of fin i + 1
      C.twin[A] = B;
      C.twin[B] = A;
    }
  }
  // cover edges: one per twin pair, with the soup edge's (mollified) length
  for (int64_t f = 0; f < F; ++f)
    for (int r = 0; r < 3; ++r) {
      const int32_t hf = (int32_t)(6 * f + r), hb = back_of(f, r);
      C.eid[hf] = -1;
      C.eid[hb] = -1;
    }
  for (size_t h = 0; h < C.vtx.size(); ++h) {
    if (C.twin[h] < 0) return kErrArg;  // not reached: every corner is glued
    if (C.eid[h] >= 0) continue;
    const int64_t f = (int64_t)h / 6;
    const int cr = (int)(h % 6);
    const int r = cr < 3 ? cr : (cr == 3 ? 2 : cr == 4 ? 1 : 0);  // soup corner of this halfedge
    const int32_t e = (int32_t)C.len.size();
    C.len.push_back(slen[sedge[3 * f + r]]);
    C.eid[h] = e;
    C.eid[C.twin[h]] = e;
  }
  // intrinsic Delaunay flips (queue of cover edges, each by one of its halfedges)
  const int64_t E = (int64_t)C.len.size();
  std::vector<int32_t> rep(E, -1);
  for (size_t h = 0; h < C.vtx.size(); ++h)
    if (rep[C.eid[h]] < 0) rep[C.eid[h]] = (int32_t)h;
  std::deque<int32_t> q;
  std::vector<char> queued(E, 1);
  for (int64_t e = 0; e < E; ++e) q.push_back((int32_t)e);
  const double tol = 1e-12;
  int64_t flips = 0;
  const int64_t max_flips = 1000 * E + 1000;
  while (!q.empty()) {
    const int32_t e = q.front();
    q.pop_front();
    queued[e] = 0;
    const int32_t h = rep[e];
    if (edge_weight(C, h) >= -tol) continue;
    const int32_t hk = flip(C, h);
    if (hk < 0) continue;
    if (++flips > max_flips) return kErrArg;  // not reached for a valid metric
    rep[e] = hk;
    const int32_t t = C.twin[hk];
    // the diamond's four sides moved slots: re-point their edges and re-check them
    const int32_t nb[4] = {Cover::nxt(hk), Cover::prv(hk), Cover::nxt(t), Cover::prv(t)};
    for (int32_t x : nb) {
      const int32_t ex = C.eid[x];
      rep[ex] = x;
      if (!queued[ex]) {
        queued[ex] = 1;
        q.push_back(ex);
      }
    }
  }
  if (nflips) *nflips = flips;
  // cotan weights per cover edge -> vertex pairs (i < j), summed in edge order; lumped mass
  const double s = 1.0 / 6.0;  // 1/2 (cover) x 1/3 (soup)
  std::unordered_map<uint64_t, int64_t> pmap;
  pmap.reserve((size_t)E);
  std::vector<std::pair<uint64_t, double>> pairs;
  for (int64_t e = 0; e < E; ++e) {
    const int32_t h = rep[e];
    const int i = C.vtx[h], j = C.vtx[C.twin[h]];
    if (i == j) continue;  // a loop edge adds w (e_i - e_i)(...)^T = 0
    const double w = s * edge_weight(C, h);
    const uint64_t key = ((uint64_t)(uint32_t)std::min(i, j) << 32) | (uint32_t)std::max(i, j);
    auto it = pmap.find(key);
    if (it == pmap.end()) {
      pmap.emplace(key, (int64_t)pairs.size());
      pairs.emplace_back(key, w);
    } else {
      pairs[it->second].second += w;
    }
  }
  const int64_t nf = (int64_t)C.vtx.size() / 3;
  for (int64_t f = 0; f < nf; ++f) {
    const double A = face_area(C.len[C.eid[3 * f]], C.len[C.eid[3 * f + 1]], C.len[C.eid[3 * f + 2]]);
    for (int r = 0; r < 3; ++r) mass[C.vtx[3 * f + r]] += s * A / 3.0;
  }
  *nnz = (int64_t)pairs.size();
  if ((int64_t)pairs.size() > cap) return kOk;  // the caller retries with cap >= nnz
  if (pairs.size() && (!ii || !jj || !ww)) return kErrArg;
  std::sort(pairs.begin(), pairs.end(),
            [](const std::pair<uint64_t, double>& p, const std::pair<uint64_t, double>& q) { return p.first < q.first; });
  for (size_t p = 0; p < pairs.size(); ++p) {
    ii[p] = (int32_t)(pairs[p].first >> 32);
    jj[p] = (int32_t)(pairs[p].first & 0xffffffffu);
    ww[p] = pairs[p].second;
  }
  return kOk;
}
