// bmpc_qpplan.cpp -- symbolic analysis of a batched QP (see bmpc_qpplan.h, bmpc_bandqp.h).
#include "bmpc_qpplan.h"

#include <algorithm>
#include <cmath>
#include <cstdio>

namespace bmpc {

namespace {

enum { ROW_FREE = 0, ROW_UP = 1, ROW_LO = 2, ROW_EQ = 4 };

int classify(double lo, double hi) {
  const bool fl = lo > -kQPInfinity, fu = hi < kQPInfinity;
  if (fl && fu && lo == hi) return ROW_EQ;
  return (fu ? ROW_UP : 0) | (fl ? ROW_LO : 0);
}

std::string fmt(const char* f, long a, long b = 0, long c = 0) {
  char buf[256];
  std::snprintf(buf, sizeof buf, f, a, b, c);
  return buf;
}

// breadth-first levels from s over the nodes with mark == 0; returns the last level
std::vector<int> bfs_last_level(const std::vector<std::vector<int>>& adj, const std::vector<char>& done, int s,
                                std::vector<int>& lvl, int& ecc) {
  std::vector<int> cur{s}, seen{s};
  lvl[s] = 0;
  ecc = 0;
  for (;;) {
    std::vector<int> nxt;
    for (int v : cur)
      for (int w : adj[v])
        if (!done[w] && lvl[w] < 0) {
          lvl[w] = lvl[v] + 1;
          nxt.push_back(w);
          seen.push_back(w);
        }
    if (nxt.empty()) break;
    cur.swap(nxt);
    ++ecc;
  }
  for (int v : seen) lvl[v] = -1;
  return cur;
}

// reverse Cuthill-McKee: order[k] = old index of new position k
std::vector<int> rcm(const std::vector<std::vector<int>>& adj) {
  const int nk = (int)adj.size();
  std::vector<char> done(nk, 0);
  std::vector<int> lvl(nk, -1), order;
  order.reserve(nk);
  auto deg = [&](int v) { return (int)adj[v].size(); };
  while ((int)order.size() < nk) {
    int s = -1;
    for (int v = 0; v < nk; ++v)
      if (!done[v] && (s < 0 || deg(v) < deg(s))) s = v;
    // pseudo-peripheral start (George & Liu): move to a min-degree node of the last level
    // while that raises the eccentricity
    int ecc = 0;
    std::vector<int> last = bfs_last_level(adj, done, s, lvl, ecc);
    for (int rep = 0; rep < 8; ++rep) {
      int c = last[0];
      for (int v : last)
        if (deg(v) < deg(c)) c = v;
      int ecc2 = 0;
      std::vector<int> last2 = bfs_last_level(adj, done, c, lvl, ecc2);
      if (ecc2 <= ecc) break;
      s = c;
      ecc = ecc2;
      last.swap(last2);
    }
    size_t head = order.size();
    order.push_back(s);
    done[s] = 1;
    while (head < order.size()) {
      const int v = order[head++];
      std::vector<int> nb;
      for (int w : adj[v])
        if (!done[w]) {
          done[w] = 1;
          nb.push_back(w);
        }
      std::sort(nb.begin(), nb.end(), [&](int a, int b) { return deg(a) != deg(b) ? deg(a) < deg(b) : a < b; });
      order.insert(order.end(), nb.begin(), nb.end());
    }
  }
  std::reverse(order.begin(), order.end());
  return order;
}

}  // namespace

std::string bandqp_classify(int m, int batch, const double* l, const double* u, std::vector<int>& cls) {
  cls.assign(m > 0 ? m : 0, 0);
  if (m > 0 && (!l || !u)) return "null pattern or bounds";
  for (int b = 0; b < batch; ++b) {
    const double* lb = l + (size_t)b * m;
    const double* ub = u + (size_t)b * m;
    for (int r = 0; r < m; ++r) {
      const double lo = lb[r], hi = ub[r];
      if (std::isnan(lo) || std::isnan(hi)) return fmt("NaN bound in row %ld (problem %ld)", r, b);
      if (lo > hi) return fmt("l > u in row %ld (problem %ld)", r, b);
      const int c = classify(lo, hi);
      if (b == 0) cls[r] = c;
      else if (c != cls[r]) return fmt("row %ld is classified differently in problem %ld (eq / one-sided / free)", r, b);
    }
  }
  return "";
}

void HostBandQP::point_tables(const int32_t* base) {
  const int32_t* p = base;
  d.kind = p;
  p += kind.size();
  d.scat = p;
  p += scat.size();
  d.cscat = p;
  p += cscat.size();
  d.xmap = p;
  p += xmap.size();
  d.ymap = p;
}

std::string bandqp_analyse(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap, const int32_t* Ai,
                           int batch, const double* l, const double* u, int max_iter, double eps, HostBandQP& out,
                           int cus, size_t lds_per_cu) {
  if (n < 1 || m < 0 || batch < 1) return "need n >= 1, m >= 0, batch >= 1";
  if (!Pp || !Ap || (m > 0 && (!l || !u))) return "null pattern or bounds";
  if (max_iter < 1 || !(eps > 0)) return "need max_iter >= 1 and eps > 0";
  if (Pp[0] != 0 || Ap[0] != 0) return "CSC column pointers must start at 0";
  for (int c = 0; c < n; ++c) {
    if (Pp[c + 1] < Pp[c] || Ap[c + 1] < Ap[c]) return "CSC column pointers must be non-decreasing";
    for (int t = Pp[c]; t < Pp[c + 1]; ++t) {
      if (Pi[t] < 0 || Pi[t] > c) return fmt("P must be upper triangular CSC (entry row %ld in column %ld)", Pi[t], c);
      if (t > Pp[c] && Pi[t] <= Pi[t - 1]) return fmt("P column %ld: row indices must increase", c);
    }
    for (int t = Ap[c]; t < Ap[c + 1]; ++t) {
      if (Ai[t] < 0 || Ai[t] >= m) return fmt("A row index %ld out of range in column %ld", Ai[t], c);
      if (t > Ap[c] && Ai[t] <= Ai[t - 1]) return fmt("A column %ld: row indices must increase", c);
    }
  }
  const int nnzP = Pp[n], nnzA = Ap[n];
  // ---- rows: one class for the whole batch
  std::vector<int> cls;
  std::string err = bandqp_classify(m, batch, l, u, cls);
  if (!err.empty()) return err;
  // ---- KKT indices before ordering: x, then per row its eq or upper / lower copies
  std::vector<int> k_up(m, -1), k_lo(m, -1), kindv(n, QPK_X);
  int nk = n, n_in = 0;
  for (int r = 0; r < m; ++r) {
    if (cls[r] == ROW_EQ) {
      k_up[r] = nk++;
      kindv.push_back(QPK_EQ);
      continue;
    }
    if (cls[r] & ROW_UP) {
      k_up[r] = nk++;
      kindv.push_back(QPK_IN);
      ++n_in;
    }
    if (cls[r] & ROW_LO) {
      k_lo[r] = nk++;
      kindv.push_back(QPK_IN);
      ++n_in;
    }
  }
  std::vector<std::vector<int>> adj(nk);
  for (int c = 0; c < n; ++c) {
    for (int t = Pp[c]; t < Pp[c + 1]; ++t)
      if (Pi[t] != c) {
        adj[Pi[t]].push_back(c);
        adj[c].push_back(Pi[t]);
      }
    for (int t = Ap[c]; t < Ap[c + 1]; ++t)
      for (int k : {k_up[Ai[t]], k_lo[Ai[t]]})
        if (k >= 0) {
          adj[k].push_back(c);
          adj[c].push_back(k);
        }
  }
  for (auto& a : adj) {
    std::sort(a.begin(), a.end());
    a.erase(std::unique(a.begin(), a.end()), a.end());
  }
  const std::vector<int> order = rcm(adj);
  std::vector<int> pos(nk);
  for (int k = 0; k < nk; ++k) pos[order[k]] = k;
  int bw = 0;
  for (int v = 0; v < nk; ++v)
    for (int w : adj[v]) bw = std::max(bw, std::abs(pos[v] - pos[w]));
  const int W = bw + 1;
  const size_t lds_bytes = bandqp_lds_doubles(nk, W, false) * sizeof(double);
  if (lds_bytes > lds_per_cu)
    return fmt("KKT bandwidth %ld after reverse Cuthill-McKee ordering (dimension %ld) needs more than the %ld KB "
               "LDS of a CU for the factorisation window",
               bw, nk, (long)(lds_per_cu / 1024));

  HostBandQP& h = out;
  h = HostBandQP();
  h.kind.resize(nk);
  for (int k = 0; k < nk; ++k) h.kind[pos[k]] = kindv[k];
  auto band = [&](int a, int b) {   // band index of KKT entry (a, b), new indices
    if (a < b) std::swap(a, b);
    return (int32_t)((size_t)a * W + (a - b));
  };
  for (int c = 0; c < n; ++c) {
    for (int t = Pp[c]; t < Pp[c + 1]; ++t) h.scat.insert(h.scat.end(), {t, band(pos[Pi[t]], pos[c]), 1});
    for (int t = Ap[c]; t < Ap[c + 1]; ++t) {
      const int r = Ai[t];
      if (k_up[r] >= 0) h.scat.insert(h.scat.end(), {nnzP + t, band(pos[k_up[r]], pos[c]), 1});
      if (k_lo[r] >= 0) h.scat.insert(h.scat.end(), {nnzP + t, band(pos[k_lo[r]], pos[c]), -1});
    }
  }
  if ((size_t)nk * W > (size_t)INT32_MAX) return "KKT band too large";
  for (int j = 0; j < n; ++j) h.cscat.insert(h.cscat.end(), {j, pos[j], 1});
  h.xmap.resize(n);
  for (int j = 0; j < n; ++j) h.xmap[j] = pos[j];
  h.ymap.assign((size_t)4 * m, -1);
  for (int r = 0; r < m; ++r) {
    if (cls[r] == ROW_EQ) {
      h.cscat.insert(h.cscat.end(), {n + r, pos[k_up[r]], 1});
    } else {
      if (k_up[r] >= 0) h.cscat.insert(h.cscat.end(), {n + m + r, pos[k_up[r]], 1});
      if (k_lo[r] >= 0) h.cscat.insert(h.cscat.end(), {n + r, pos[k_lo[r]], -1});
    }
    if (k_up[r] >= 0) {
      h.ymap[4 * r] = pos[k_up[r]];
      h.ymap[4 * r + 1] = 1;
    }
    if (k_lo[r] >= 0) {
      h.ymap[4 * r + 2] = pos[k_lo[r]];
      h.ymap[4 * r + 3] = -1;
    }
  }
  BandQPDesc& d = h.d;
  d.n = n;
  d.m = m;
  d.nk = nk;
  d.bw = bw;
  d.W = W;
  d.n_in = n_in;
  d.nvals = nnzP + nnzA;
  d.ncvals = n + 2 * m;
  d.nscat = (int32_t)(h.scat.size() / 3);
  d.ncscat = (int32_t)(h.cscat.size() / 3);
  d.max_iter = max_iter;
  // the factor in LDS when it fits and the batch is small enough to have a CU per problem
  // anyway (a 100 KB workgroup leaves one problem per CU: 2.7x fewer solves/s at 4096)
  d.lb_lds = batch <= cus && bandqp_lds_doubles(nk, W, true) * sizeof(double) <= lds_per_cu ? 1 : 0;
  d.eps = eps;
  d.stride = bandqp_stride(nk, W);
  for (auto* v : {&h.kind, &h.scat, &h.cscat, &h.xmap, &h.ymap}) h.blob.insert(h.blob.end(), v->begin(), v->end());
  h.point_tables(h.blob.data());
  return "";
}

}  // namespace bmpc
