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
//
// phh_strict_*: the whole log density + gradient around the likelihood for
// the strict-clock family (phylostan's default build: Weibull or no site
// rates, JC69 / HKY / GTR, estimated or fixed rate, constant coalescent or
// none) -- posterior.py's _lpg_gen restated in one native pass per phase.
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

// ---------------------------------------------------------------------------
// Strict-clock posterior (posterior.py: _declare, constrain, _lpg_gen; the
// transforms of transforms.py).  Two phases around the likelihood:
//   pre   U [n][dim] -> the branch lengths and model vectors of the draws
//         that reach the likelihood, packed first-come (sel[d] = their row,
//         -1: rejected -- out of support or non-finite, lp = -inf)
//   post  U and the likelihood's rows -> lp [n], G [n][dim]
// post recomputes the transforms (cheaper than keeping them).
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

// The constrained values of one draw and what the reverse pass needs.
struct Draw {
  double logj = 0.0;
  double w = 0.0, ew = 0.0, rate = 0.0, erate = 0.0, height = 0.0, eheight = 0.0, theta = 0.0, etheta = 0.0;
  double kappa = 0.0, ekappa = 0.0;
  double freqs[4], fst[3], fz[3];    // simplex value, sticks, z
  double rates[6], rst[5], rz[5];
  std::vector<double> props, h, span, g;  // props, heights, spans, Weibull g
};

struct Strict {
  int S, H, B, C, N, np, dim;
  int model;      // 0 JC69, 1 HKY, 2 GTR
  int weibull;    // categories > 1 (wshape)
  int est_rate;   // rate is a parameter (exponential(1000)), else fixed_rate
  double fixed_rate;
  int coal;       // constant coalescent (theta ~ oneOnX)
  double lower_root;
  int o_w, o_props, o_rate, o_height, o_theta, o_kappa, o_rates, o_freqs;
  int root;
  std::vector<int> node, par, prop, bpar, bh, jpar;
  std::vector<double> low, blow, jlow, tip_times, wx;
  std::vector<unsigned char> internal;
  // pre's transformed draws, reused by post when it gets the same U
  std::vector<Draw> cache;
  std::vector<double> cache_u;
  std::vector<int> order;  // the coalescent's event order, kept across calls (nearly sorted next time)
};

inline double log1p_exp(double x) { return std::max(x, 0.0) + std::log1p(std::exp(-std::fabs(x))); }
// transforms.py's _inv_logit (Stan Math's form)
inline double inv_logit(double u) {
  const double e = std::exp(-std::fabs(u));
  return (u >= 0.0 ? 1.0 : e) / (1.0 + e);
}

// Lower: x = L + e^u (support x > L); Unit: x = inv_logit(u) (0 < x < 1);
// Simplex: Stan's stick-breaking with offsets log(K-1-k) (support x > 0).
bool lower(double u, double L, double& x, double& e, double& logj) {
  e = std::exp(u);
  x = L + e;
  logj += u;
  return std::isfinite(x) && x > L;
}
bool simplex(const double* u, int K, double* x, double* st, double* zs, double& logj) {
  double stick = 1.0;
  bool ok = true;
  for (int k = 0; k < K - 1; ++k) {
    const double a = u[k] - std::log((double)(K - 1 - k));
    const double z = inv_logit(a);
    st[k] = stick;
    zs[k] = z;
    x[k] = stick * z;
    logj += std::log(stick) - log1p_exp(-a) - log1p_exp(a);
    stick = stick - x[k];
  }
  x[K - 1] = stick;
  for (int k = 0; k < K; ++k) ok = ok && std::isfinite(x[k]) && x[k] > 0.0;
  return ok;
}
void simplex_back(const double* gx, int K, const double* st, const double* zs, double* gu) {
  double g_stick = gx[K - 1];
  for (int k = K - 2; k >= 0; --k) {
    const double s = st[k], z = zs[k];
    const double g_xk = gx[k] - g_stick;
    const double g_s = g_stick + g_xk * z + 1.0 / s;
    const double g_z = g_xk * s;
    gu[k] = g_z * z * (1.0 - z) + (1.0 - 2.0 * z);
    g_stick = g_s;
  }
}

// constrain + support + heights + spans: false = rejected
bool forward(const Strict& m, const double* u, Draw& d) {
  for (int k = 0; k < m.dim; ++k)
    if (!std::isfinite(u[k])) return false;
  bool ok = true;
  d.logj = 0.0;
  if (m.weibull) ok &= lower(u[m.o_w], 0.1, d.w, d.ew, d.logj);
  d.props.resize(m.np);
  {
    // x = inv_logit(u), log|J| = -(log1p_exp(u) + log1p_exp(-u)) = -(|u| + 2 log(1 + e)),
    // e = exp(-|u|): one exp per proportion, and the logs summed as the log of
    // a product (each factor in (1, 2], renormalised every 512 factors)
    double su = 0.0, prod = 1.0;
    int pexp = 0;
    for (int k = 0; k < m.np; ++k) {
      const double uu = u[m.o_props + k];
      const double e = std::exp(-std::fabs(uu));
      const double x = (uu >= 0.0 ? 1.0 : e) / (1.0 + e);
      d.props[k] = x;
      su += std::fabs(uu);
      prod *= 1.0 + e;
      if ((k & 511) == 511) {
        int ex;
        prod = std::frexp(prod, &ex);
        pexp += ex;
      }
      ok &= std::isfinite(x) && x > 0.0 && x < 1.0;
    }
    d.logj -= su + 2.0 * (std::log(prod) + pexp * 0.69314718055994530942);
  }
  if (m.est_rate) ok &= lower(u[m.o_rate], 0.0, d.rate, d.erate, d.logj);
  ok &= lower(u[m.o_height], m.lower_root, d.height, d.eheight, d.logj);
  if (m.coal) ok &= lower(u[m.o_theta], 0.0, d.theta, d.etheta, d.logj);
  if (m.model == 1) ok &= lower(u[m.o_kappa], 0.0, d.kappa, d.ekappa, d.logj);
  if (m.model == 2) ok &= simplex(u + m.o_rates, 6, d.rates, d.rst, d.rz, d.logj);
  if (m.model >= 1) ok &= simplex(u + m.o_freqs, 4, d.freqs, d.fst, d.fz, d.logj);
  if (!ok || !std::isfinite(d.logj)) return false;
  d.h.resize(m.H);
  d.h[m.root] = d.height;
  for (size_t i = 0; i < m.node.size(); ++i) d.h[m.node[i]] = m.low[i] + (d.h[m.par[i]] - m.low[i]) * d.props[m.prop[i]];
  d.span.resize(m.B);
  for (int b = 0; b < m.B; ++b) d.span[b] = d.h[m.bpar[b]] - (m.bh[b] >= 0 ? d.h[m.bh[b]] : m.blow[b]);
  return true;
}

// model vector [freqs 4, exchangeabilities 6, rs C, ps C]
void model_vec(const Strict& m, Draw& d, double* mv) {
  const int C = m.C;
  for (int k = 0; k < 4; ++k) mv[k] = m.model >= 1 ? d.freqs[k] : 0.25;
  for (int k = 0; k < 6; ++k) mv[4 + k] = m.model == 2 ? d.rates[k] : 1.0;
  if (m.model == 1) mv[4 + 1] = mv[4 + 4] = d.kappa;
  if (m.weibull) {
    d.g.resize(C);
    double sg = 0.0;
    for (int c = 0; c < C; ++c) sg += (d.g[c] = std::pow(m.wx[c], 1.0 / d.w));
    for (int c = 0; c < C; ++c) mv[10 + c] = d.g[c] / (sg / C);
    for (int c = 0; c < C; ++c) mv[10 + C + c] = 1.0 / C;
  } else {
    for (int c = 0; c < C; ++c) mv[10 + c] = mv[10 + C + c] = 1.0;
  }
}

// constant_coalescent_log of one draw (phh_constant_coalescent's algebra) with
// the event order carried over from the previous draw / call: node times
// move little between leapfrog steps, so an insertion sort of the old order
// is nearly linear.  Stable (ties keep index order, as std::stable_sort of
// the index sequence does): a strict comparison on (time, index).
void coalescent_ordered(std::vector<int>& order, int N, const double* t, const unsigned char* internal, double theta,
                        double& lp, double* dtimes, double& dtheta, std::vector<double>& a) {
  if ((int)order.size() != N) {
    order.resize(N);
    std::iota(order.begin(), order.end(), 0);
  }
  auto before = [&](int x, int y) { return t[x] < t[y] || (t[x] == t[y] && x < y); };
  for (int i = 1; i < N; ++i) {
    const int v = order[i];
    int j = i - 1;
    while (j >= 0 && before(v, order[j])) {
      order[j + 1] = order[j];
      --j;
    }
    order[j + 1] = v;
  }
  a.resize(N);
  int nint = 0;
  for (int i = 0; i < N; ++i) nint += internal[i] ? 1 : 0;
  double k = 0.0, sdt = 0.0, prev = t[order[0]];
  for (int i = 0; i < N; ++i) {
    const int o = order[i];
    const double dt = t[o] - prev;
    prev = t[o];
    const double c = k * (k - 1.0) * 0.5;
    a[i] = dt != 0.0 ? c : 0.0;
    sdt += dt * a[i];
    k += internal[o] ? -1.0 : 1.0;
  }
  const double inv = 1.0 / theta;
  lp = -sdt * inv - nint * std::log(theta);
  for (int i = 0; i < N; ++i) dtimes[order[i]] = ((i + 1 < N ? a[i + 1] : 0.0) - a[i]) * inv;
  dtheta = sdt * inv * inv - nint * inv;
}

}  // namespace

extern "C" {

// tree arrays as ClockTreeNative holds them (hostlib.py); offs = parameter
// offsets [wshape, props, rate, height, theta, kappa, rates, freqs] (-1: absent)
void* phh_strict_create(int S, int B, int C, int model, int weibull, int est_rate, double fixed_rate, int coal,
                        int heterochronous, double lower_root, int dim, const int* offs, int m, const int* node,
                        const int* par, const int* prop, const double* low, int root, const int* bpar, const int* bh,
                        const double* blow, int jm, const int* jpar, const double* jlow, const double* lowers) {
  Strict* t = new Strict();
  t->S = S;
  t->H = S - 1;
  t->B = B;
  t->C = C;
  t->N = 2 * S - 1;
  t->np = S - 2;
  t->dim = dim;
  t->model = model;
  t->weibull = weibull;
  t->est_rate = est_rate;
  t->fixed_rate = fixed_rate;
  t->coal = coal;
  t->lower_root = lower_root;
  t->o_w = offs[0];
  t->o_props = offs[1];
  t->o_rate = offs[2];
  t->o_height = offs[3];
  t->o_theta = offs[4];
  t->o_kappa = offs[5];
  t->o_rates = offs[6];
  t->o_freqs = offs[7];
  t->root = root;
  t->node.assign(node, node + m);
  t->par.assign(par, par + m);
  t->prop.assign(prop, prop + m);
  t->low.assign(low, low + m);
  t->bpar.assign(bpar, bpar + B);
  t->bh.assign(bh, bh + B);
  t->blow.assign(blow, blow + B);
  t->jpar.assign(jpar, jpar + jm);
  t->jlow.assign(jlow, jlow + jm);
  t->tip_times.assign(S, 0.0);
  if (heterochronous)
    for (int i = 0; i < S; ++i) t->tip_times[i] = lowers[i];
  t->internal.assign(t->N, 0);
  for (int i = S; i < t->N; ++i) t->internal[i] = 1;
  for (int c = 0; c < C; ++c) t->wx.push_back(-std::log(1.0 - (2.0 * c + 1.0) / (2.0 * C)));
  return t;
}

void phh_strict_free(void* h) { delete static_cast<Strict*>(h); }

int phh_strict_pre(void* hnd, int n, const double* U, double* blens, double* mv, int* sel) {
  Strict& m = *static_cast<Strict*>(hnd);
  const int ml = 10 + 2 * m.C;
  if ((int)m.cache.size() < n) m.cache.resize(n);
  m.cache_u.assign(U, U + (size_t)n * m.dim);
  int cnt = 0;
  for (int k = 0; k < n; ++k) {
    sel[k] = -1;
    Draw& d = m.cache[k];
    if (!forward(m, U + (size_t)k * m.dim, d)) continue;
    double* bl = blens + (size_t)cnt * m.B;
    double* v = mv + (size_t)cnt * ml;
    const double mult = m.est_rate ? d.rate : m.fixed_rate;
    bool ok = true;
    for (int b = 0; b < m.B; ++b) ok &= std::isfinite(bl[b] = d.span[b] * mult);
    model_vec(m, d, v);
    for (int q = 0; q < ml; ++q) ok &= std::isfinite(v[q]);
    for (int q = 0; q < 4; ++q) ok &= v[q] > 0.0;
    if (ok) sel[k] = cnt++;
  }
  return cnt;
}

// rows [cnt][rowlen]: log L, d/dblens [B], d/drs [C], d/dps [C], the root
// frequency term [4], d/d exchangeabilities [6], d/dfreqs [4], ...
void phh_strict_post(void* hnd, int n, const double* U, const double* rows, int rowlen, const int* sel,
                     int need_grad, double* lp, double* G) {
  Strict& m = *static_cast<Strict*>(hnd);
  const int S = m.S, B = m.B, C = m.C, H = m.H;
  const int o = 1 + B + 2 * C;
  // pre's draws when U is the one pre saw (the begin / end pair), else anew
  const bool cached = (int)m.cache.size() >= n && m.cache_u.size() == (size_t)n * m.dim &&
                      std::equal(m.cache_u.begin(), m.cache_u.end(), U);
  Draw fresh;
  std::vector<double> gh(H), times(m.N), gt(m.N), gprops(m.np), ml(10 + 2 * C), ca;
  for (int k = 0; k < n; ++k) {
    double* Gk = need_grad ? G + (size_t)k * m.dim : nullptr;
    if (Gk) std::fill(Gk, Gk + m.dim, 0.0);
    lp[k] = -INFINITY;
    if (sel[k] < 0) continue;
    Draw& d = cached ? m.cache[k] : fresh;
    if (!cached && !forward(m, U + (size_t)k * m.dim, d)) continue;
    const double* row = rows + (size_t)sel[k] * rowlen;
    double l = d.logj + row[0];
    double gw = 0.0, grate = 0.0, gheight = 0.0, gtheta = 0.0, gkappa = 0.0, gfreqs[4] = {0, 0, 0, 0};
    double grates[6] = {0, 0, 0, 0, 0, 0};
    // priors (posterior.py _lpg_gen, constants dropped)
    if (m.weibull) {
      l -= d.w;  // wshape ~ exponential(1)
      gw -= 1.0;
    }
    if (m.model == 1) {  // kappa ~ lognormal(1, 1.25)
      const double lk = std::log(d.kappa);
      l -= lk + (lk - 1.0) * (lk - 1.0) / (2.0 * 1.25 * 1.25);
      gkappa += -1.0 / d.kappa - (lk - 1.0) / (1.25 * 1.25 * d.kappa);
    }
    std::fill(gh.begin(), gh.end(), 0.0);
    if (m.est_rate) {  // rate ~ exponential(1000)
      l -= 1000.0 * d.rate;
      grate -= 1000.0;
    }
    {  // log-Jacobian of the height transform: sum log(gap) as the log of a
       // product renormalised after every factor (mantissa in [0.5, 1), so no
       // under- or overflow and no subnormal precision loss for any normal
       // gap); a gap that is not a positive normal number -- <= 0, NaN,
       // subnormal -- takes the sum of logs, so -inf / NaN come out exactly
       // as the reference's sum of logs gives them
      double prod = 1.0;
      int pexp = 0;
      bool plain = true;
      for (size_t i = 0; i < m.jpar.size(); ++i) {
        const double gap = d.h[m.jpar[i]] - m.jlow[i];
        plain &= std::isnormal(gap) && gap > 0.0;
        int ex;
        prod = std::frexp(prod * gap, &ex);
        pexp += ex;
        gh[m.jpar[i]] += 1.0 / gap;
      }
      if (plain) {
        l += std::log(prod) + pexp * 0.69314718055994530942;
      } else {
        double s = 0.0;
        for (size_t i = 0; i < m.jpar.size(); ++i) s += std::log(d.h[m.jpar[i]] - m.jlow[i]);
        l += s;
      }
    }
    if (m.coal) {  // constant coalescent, theta ~ oneOnX
      for (int i = 0; i < S; ++i) times[i] = m.tip_times[i];
      for (int i = 0; i < H; ++i) times[S + i] = d.h[i];
      double clp, gth;
      coalescent_ordered(m.order, m.N, times.data(), m.internal.data(), d.theta, clp, gt.data(), gth, ca);
      l += clp - std::log(d.theta);
      gtheta += gth - 1.0 / d.theta;
      for (int i = 0; i < H; ++i) gh[i] += gt[S + i];
    }
    if (!std::isfinite(l)) continue;
    lp[k] = l;
    if (!Gk) continue;
    // the likelihood's gradients -> constrained parameters
    const double* g_bl = row + 1;
    const double* g_rs = row + 1 + B;
    if (m.model >= 1) {
      for (int q = 0; q < 4; ++q) gfreqs[q] += row[o + 10 + q];
      if (m.model == 2)
        for (int q = 0; q < 6; ++q) grates[q] += row[o + 4 + q];
      else
        gkappa += row[o + 4 + 1] + row[o + 4 + 4];  // kappa enters AG and CT
    }
    if (m.weibull) {  // rs = g / mean(g), g = wx^(1/w)
      model_vec(m, d, ml.data());
      double sg = 0.0, sdg = 0.0;
      std::vector<double>& g = d.g;
      double dgv[64];
      for (int c = 0; c < C; ++c) {
        dgv[c] = g[c] * std::log(m.wx[c]) * (-1.0 / (d.w * d.w));
        sg += g[c];
        sdg += dgv[c];
      }
      const double mg = sg / C, mdg = sdg / C;
      double acc = 0.0;
      for (int c = 0; c < C; ++c) acc += g_rs[c] * (dgv[c] / mg - g[c] * mdg / (mg * mg));
      gw += acc;
    }
    const double mult = m.est_rate ? d.rate : m.fixed_rate;
    double gmult = 0.0;
    for (int b = 0; b < B; ++b) {
      const double gs = g_bl[b] * mult;
      gmult += g_bl[b] * d.span[b];
      gh[m.bpar[b]] += gs;
      if (m.bh[b] >= 0) gh[m.bh[b]] -= gs;
    }
    if (m.est_rate) grate += gmult;
    std::fill(gprops.begin(), gprops.end(), 0.0);
    for (int i = (int)m.node.size() - 1; i >= 0; --i) {
      const double gn = gh[m.node[i]];
      gprops[m.prop[i]] += gn * (d.h[m.par[i]] - m.low[i]);
      gh[m.par[i]] += gn * d.props[m.prop[i]];
    }
    gheight += gh[m.root];
    // constrained -> unconstrained (+ log-Jacobian terms)
    if (m.weibull) Gk[m.o_w] = gw * d.ew + 1.0;
    for (int q = 0; q < m.np; ++q) {
      const double x = d.props[q];
      Gk[m.o_props + q] = gprops[q] * x * (1.0 - x) + (1.0 - 2.0 * x);
    }
    if (m.est_rate) Gk[m.o_rate] = grate * d.erate + 1.0;
    Gk[m.o_height] = gheight * d.eheight + 1.0;
    if (m.coal) Gk[m.o_theta] = gtheta * d.etheta + 1.0;
    if (m.model == 1) Gk[m.o_kappa] = gkappa * d.ekappa + 1.0;
    if (m.model == 2) simplex_back(grates, 6, d.rst, d.rz, Gk + m.o_rates);
    if (m.model >= 1) simplex_back(gfreqs, 4, d.fst, d.fz, Gk + m.o_freqs);
    for (int q = 0; q < m.dim; ++q)
      if (!std::isfinite(Gk[q])) Gk[q] = 0.0;
  }
}

}  // extern "C"
