// host_model.cpp -- native host pieces of the emitted Stan model that sit
// around the likelihood: the tree-height transform, its log-Jacobian, the
// branch-span chain rule and the constant-population coalescent, each with
// its reverse pass, batched over n draws (row-major [n][...] arrays).
//
// These are the per-leapfrog-step host costs of a clock model (NUTS calls
// them once per gradient round): the numpy restatements in posterior.py /
// priors.py are the specification and the tests compare the two.  Plain C
// ABI, loaded by phylostan_amd/hostlib.py.
//
//   heights      generate_script.py:711-736  (props -> heights, pre-order)
//   log-Jacobian generate_script.py:739-752
//   blens        generate_script.py:660-679  (heights[parent] - heights[node])
//   coalescent   generate_script.py:285-349  (constant_coalescent_log)
#include <algorithm>
#include <cmath>
#include <numeric>
#include <vector>

extern "C" {

// Heights of the internal nodes h[n][H] (H = S-1, index = node - S).  The m
// non-root internal nodes are listed parents-first: node[i] (h index),
// par[i] (the parent's h index), prop[i] (its proportion), low[i] (its
// lower bound): h = low + (h[par] - low) * props[prop].
void phh_heights(int n, int H, int m, const int* node, const int* par, const int* prop, const double* low,
                 int root, int np, const double* props, const double* height, double* h) {
  for (int d = 0; d < n; ++d) {
    double* hd = h + (size_t)d * H;
    const double* pd = props + (size_t)d * np;
    hd[root] = height[d];
    for (int i = 0; i < m; ++i) hd[node[i]] = low[i] + (hd[par[i]] - low[i]) * pd[prop[i]];
  }
}

// Reverse of phh_heights: consumes gh (d logp / d h, modified in place),
// accumulates d/d props into gprops[n][np] and d/d height into gheight[n].
void phh_heights_back(int n, int H, int m, const int* node, const int* par, const int* prop, const double* low,
                      int root, int np, const double* props, const double* h, double* gh, double* gprops,
                      double* gheight) {
  for (int d = 0; d < n; ++d) {
    double* g = gh + (size_t)d * H;
    const double* hd = h + (size_t)d * H;
    const double* pd = props + (size_t)d * np;
    double* gp = gprops + (size_t)d * np;
    for (int i = m - 1; i >= 0; --i) {
      const double gn = g[node[i]];
      gp[prop[i]] += gn * (hd[par[i]] - low[i]);
      g[par[i]] += gn * pd[prop[i]];
    }
    gheight[d] += g[root];
  }
}

// log-Jacobian of the height transform: lp += sum log(h[par] - low) over
// the non-root internal nodes, gh[par] += 1 / (h[par] - low).
void phh_height_jacobian(int n, int H, int m, const int* par, const double* low, const double* h, double* lp,
                         double* gh) {
  for (int d = 0; d < n; ++d) {
    const double* hd = h + (size_t)d * H;
    double* g = gh + (size_t)d * H;
    double s = 0.0;
    for (int i = 0; i < m; ++i) {
      const double gap = hd[par[i]] - low[i];
      s += std::log(gap);
      g[par[i]] += 1.0 / gap;
    }
    lp[d] += s;
  }
}

// Branch spans [n][B]: h[bpar[b]] - (bh[b] >= 0 ? h[bh[b]] : blow[b]).
void phh_span(int n, int H, int B, const int* bpar, const int* bh, const double* blow, const double* h,
              double* span) {
  for (int d = 0; d < n; ++d) {
    const double* hd = h + (size_t)d * H;
    double* sp = span + (size_t)d * B;
    for (int b = 0; b < B; ++b) sp[b] = hd[bpar[b]] - (bh[b] >= 0 ? hd[bh[b]] : blow[b]);
  }
}

// Reverse of phh_span: gh[bpar[b]] += gspan[b], gh[bh[b]] -= gspan[b].
void phh_span_back(int n, int H, int B, const int* bpar, const int* bh, const double* gspan, double* gh) {
  for (int d = 0; d < n; ++d) {
    double* g = gh + (size_t)d * H;
    const double* gs = gspan + (size_t)d * B;
    for (int b = 0; b < B; ++b) {
      g[bpar[b]] += gs[b];
      if (bh[b] >= 0) g[bh[b]] -= gs[b];
    }
  }
}

// constant_coalescent_log (generate_script.py:285-349) over node times
// [n][N] (tips: sampling ages, internal: heights), internal[N] in {0,1}:
// events in stable ascending time order, lineage count k before each event,
// interval coefficient k(k-1)/2 (zero-length intervals contribute nothing).
// lp[n] = -sum dt * c / theta - (#internal) log theta; dtimes[n][N]; dtheta[n].
void phh_constant_coalescent(int n, int N, const double* times, const unsigned char* internal, const double* theta,
                             double* lp, double* dtimes, double* dtheta) {
  std::vector<int> order(N);
  std::vector<double> a(N);
  int nint = 0;
  for (int i = 0; i < N; ++i) nint += internal[i] ? 1 : 0;
  for (int d = 0; d < n; ++d) {
    const double* t = times + (size_t)d * N;
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return t[x] < t[y]; });
    double k = 0.0, sdt = 0.0, prev = t[order[0]];
    for (int i = 0; i < N; ++i) {
      const int o = order[i];
      const double step = internal[o] ? -1.0 : 1.0;
      const double dt = t[o] - prev;  // 0 for the first event
      prev = t[o];
      const double c = k * (k - 1.0) * 0.5;
      a[i] = dt != 0.0 ? c : 0.0;
      sdt += dt * a[i];
      k += step;
    }
    const double inv = 1.0 / theta[d];
    lp[d] = -sdt * inv - nint * std::log(theta[d]);
    double* g = dtimes + (size_t)d * N;
    for (int i = 0; i < N; ++i) g[order[i]] = ((i + 1 < N ? a[i + 1] : 0.0) - a[i]) * inv;
    dtheta[d] = sdt * inv * inv - nint * inv;
  }
}

}  // extern "C"
