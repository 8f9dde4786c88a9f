// nuts_host.cpp -- native NUTS chains: nuts.py's Chain (Stan's
// adapt_diag_e_nuts: multinomial trajectory sampling, across-subtree U-turn
// checks, expl_leapfrog, dual-averaging step size, windowed diagonal metric,
// init_stepsize) restated as a resumable state machine per chain.
//
// Why native: with every gradient on the GPU, a sampler round of config 5
// (4 chains of fluA) costs ~105 us of GPU call and, with the chains in
// Python generators, ~235 us of host work, more than half of it the
// interpreter's tree building.  Stan's own sampler is C++
// (the reference runs it through pystan, phylostan.py:318-321).
//
// nuts.py stays the specification; tests/test_nuts_native.py runs both on
// the same seeds.  The random streams are the chains' numpy Generators:
// momenta through numpy's own random_standard_normal (libnpyrandom.a, the
// function Generator.standard_normal calls per element) and uniforms through
// the bit generator's next_double (Generator.uniform() of [0, 1) is exactly
// that value), so both implementations draw the same numbers in the same
// order.  Dot products are one sequential sum of rounded products (dot
// below; nuts.py's _sdot is numpy's strictly sequential cumsum of the same
// products, and this file is built with -ffp-contract=off), so the chains
// are bitwise equal to nuts.py's in every dimension, on any CPU and BLAS.
//
// Protocol (phn_*): phn_step takes the (lp, grad) of the positions asked
// for last time and returns the next positions to evaluate, one per chain
// that is not finished -- run_chains batches them into one likelihood call.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "numpy/random/bitgen.h"

extern "C" double random_standard_normal(bitgen_t* bitgen_state);

namespace {

typedef std::vector<double> Vec;

struct Point {
  Vec q, p, g;
  double lp;
};

// a valid subtree: build_tree's returned tuple (nuts.py:196-230)
struct Sub {
  int level;
  Point zp;
  Vec ps_beg, ps_end, rho, p_beg, p_end;
  double lsw;
};

enum { ERR_NONE = 0, ERR_INIT = 1, ERR_IMPROPER = 2, ERR_SMALL = 3 };

double log_sum_exp(double a, double b) {  // nuts.py:26
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  double m = (b > a) ? b : a;  // Python's max(a, b)
  return m + std::log(std::exp(a - m) + std::exp(b - m));
}

// nuts.py _sdot: ((a0 b0 + a1 b1) + a2 b2) + ..., every product rounded
double dot(const Vec& a, const Vec& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
  return s;
}

Vec add(const Vec& a, const Vec& b) {
  Vec r(a.size());
  for (size_t i = 0; i < a.size(); ++i) r[i] = a[i] + b[i];
  return r;
}

bool criterion(const Vec& ps_minus, const Vec& ps_plus, const Vec& rho) {  // nuts.py:193
  return dot(ps_plus, rho) > 0 && dot(ps_minus, rho) > 0;
}

struct Chain {
  // waits: the chain has asked for (lp, grad) at q_eval
  enum State { W_INIT, W_ISS_FIRST, W_ISS_LOOP, W_LEAF, W_HMC, DONE, FAILED };
  enum Cont { AFTER_INIT, AFTER_WINDOW };

  int dim;
  bitgen_t* rng;
  int num_warmup, total, thin, max_depth;
  double delta, gamma, kappa, t0, max_delta_h;
  double eps;
  Vec im;  // inverse metric
  // windowed variance adaptation (nuts.py:71-126)
  bool windows;
  int adapt_init, adapt_term, adapt_base, win_counter, win_size, next_window, w_n;
  Vec w_mean, w_m2;
  // dual averaging
  int da_counter;
  double s_bar, x_bar, mu;
  // program
  State state;
  int err;
  int it;
  bool warm;
  double eps_used;
  Point z;
  Vec q0;
  // init_stepsize
  Point zt;
  double iH0;
  int idir;
  Cont cont;
  // transition
  double H0, lsw, smp;
  int depth, n_lf;
  bool divergent, forward;
  Point z_fwd, z_bck, z_sample;
  Vec p_ff, p_fb, p_bf, p_bb, ps_ff, ps_fb, ps_bf, ps_bb, rho, rho_fwd, rho_bck;
  std::vector<Sub> stack;
  double t_accept, t_energy;
  int t_depth, t_nlf;
  bool t_div;
  // static HMC (nuts.py StaticHMCChain: Stan's adapt_diag_e_static_hmc)
  bool hmc = false;
  double T = 0.0;  // integration time
  long L = 1;      // leapfrog steps
  long hk = 0;     // steps taken in this transition
  Point z_init;
  // the pending evaluation
  Point* ev;
  double ev_eps;
  // output
  Vec dq;
  std::vector<double> dstat;  // lp, accept, eps, depth, n_leapfrog, divergent, energy, warmup
  long n_grad;

  double uniform() { return rng->next_double(rng->state); }

  Vec sample_p() {  // nuts.py:145
    Vec r(dim);
    for (int i = 0; i < dim; ++i) r[i] = random_standard_normal(rng);
    for (int i = 0; i < dim; ++i) r[i] = r[i] / std::sqrt(im[i]);
    return r;
  }

  Vec scaled(const Vec& p) const {
    Vec r(dim);
    for (int i = 0; i < dim; ++i) r[i] = im[i] * p[i];
    return r;
  }

  double H(const Point& a) const {  // nuts.py:148
    if (!std::isfinite(a.lp)) return INFINITY;
    double s = 0.0;
    for (int i = 0; i < dim; ++i) s += (im[i] * a.p[i]) * a.p[i];
    return -a.lp + 0.5 * s;
  }

  // expl_leapfrog (nuts.py:153): the half-kick and drift, then the wait
  void evolve_begin(Point& a, double e) {
    double he = 0.5 * e;
    for (int i = 0; i < dim; ++i) a.p[i] = a.p[i] + he * a.g[i];
    for (int i = 0; i < dim; ++i) a.q[i] = a.q[i] + (e * im[i]) * a.p[i];
    ev = &a;
    ev_eps = e;
  }

  void evolve_end(double lp, const double* g) {
    Point& a = *ev;
    ++n_grad;
    a.lp = lp;
    bool fin = true;
    for (int i = 0; i < dim; ++i) fin = fin && std::isfinite(g[i]);
    for (int i = 0; i < dim; ++i) a.g[i] = fin ? g[i] : 0.0;
    if (!std::isfinite(lp)) a.lp = -INFINITY;
    double he = 0.5 * ev_eps;
    for (int i = 0; i < dim; ++i) a.p[i] = a.p[i] + he * a.g[i];
  }

  // ------------------------------------------------------------ adaptation
  void setup_windows(int init_buffer, int term_buffer, int base_window) {
    int W = num_warmup;
    if (W < 20) {
      adapt_init = W, adapt_term = 0, adapt_base = 0;
      windows = false;
      return;
    }
    windows = true;
    if (init_buffer + base_window + term_buffer > W) {
      init_buffer = (int)(0.15 * W);
      term_buffer = (int)(0.1 * W);
      base_window = W - (init_buffer + term_buffer);
    }
    adapt_init = init_buffer, adapt_term = term_buffer, adapt_base = base_window;
    win_counter = 0;
    win_size = base_window;
    next_window = init_buffer + base_window - 1;
    w_n = 0;
    w_mean.assign(dim, 0.0);
    w_m2.assign(dim, 0.0);
  }

  void compute_next_window() {
    int W = num_warmup, term = adapt_term;
    if (next_window == W - term - 1) return;
    win_size *= 2;
    next_window = win_counter + win_size;
    if (next_window != W - term - 1 && next_window + 2 * win_size >= W - term) next_window = W - term - 1;
  }

  bool learn_variance(const Vec& q) {
    if (!windows) return false;
    int W = num_warmup;
    if (adapt_init <= win_counter && win_counter < W - adapt_term && win_counter != W) {
      ++w_n;
      for (int i = 0; i < dim; ++i) {
        double d = q[i] - w_mean[i];
        w_mean[i] += d / w_n;
        w_m2[i] += d * (q[i] - w_mean[i]);
      }
    }
    if (win_counter == next_window && win_counter != W) {
      compute_next_window();
      double n = (double)w_n;
      double a = n / (n + 5.0), b = 1e-3 * (5.0 / (n + 5.0));
      for (int i = 0; i < dim; ++i) im[i] = a * (n > 1 ? w_m2[i] / (n - 1.0) : 1.0) + b;
      w_n = 0;
      w_mean.assign(dim, 0.0);
      w_m2.assign(dim, 0.0);
      ++win_counter;
      return true;
    }
    ++win_counter;
    return false;
  }

  void da_restart() {
    da_counter = 0;
    s_bar = 0.0;
    x_bar = 0.0;
    mu = std::log(10.0 * eps);
  }

  void learn_stepsize(double stat) {  // nuts.py:134
    ++da_counter;
    stat = (stat < 1.0) ? stat : 1.0;  // Python's min(1.0, stat)
    double eta = 1.0 / (da_counter + t0);
    s_bar = (1.0 - eta) * s_bar + eta * (delta - stat);
    double x = mu - s_bar * std::sqrt((double)da_counter) / gamma;
    double x_eta = std::pow((double)da_counter, -kappa);
    x_bar = (1.0 - x_eta) * x_bar + x_eta * x;
    eps = std::exp(x);
  }

  // ------------------------------------------------------- init_stepsize
  // nuts.py:165; returns true when it asked for an evaluation
  bool iss_start(Cont c) {
    cont = c;
    if (eps == 0 || eps > 1e7 || std::isnan(eps)) return false;
    zt = z;
    zt.p = sample_p();
    iH0 = H(zt);
    evolve_begin(zt, eps);
    state = W_ISS_FIRST;
    return true;
  }

  void iss_loop() {
    zt = z;
    zt.p = sample_p();
    iH0 = H(zt);
    evolve_begin(zt, eps);
    state = W_ISS_LOOP;
  }

  double iss_dH() {
    double h = H(zt);
    return iH0 - (std::isnan(h) ? INFINITY : h);
  }

  // --------------------------------------------------------- transition
  void tr_start() {  // nuts.py:232
    Point a = z;
    a.p = sample_p();
    H0 = H(a);
    z_fwd = a, z_bck = a, z_sample = a;
    Vec ps0 = scaled(a.p);
    p_ff = p_fb = p_bf = p_bb = rho = a.p;
    ps_ff = ps_fb = ps_bf = ps_bb = ps0;
    lsw = 0.0;
    n_lf = 0, smp = 0.0, divergent = false;
    depth = 0;
  }

  // one depth of the doubling loop; false: the transition is over
  bool tr_depth() {
    if (depth >= max_depth) return false;
    forward = uniform() > 0.5;
    if (forward) {
      rho_bck = rho;
      p_bf = p_fb, ps_bf = ps_fb;
    } else {
      rho_fwd = rho;
      p_fb = p_bf, ps_fb = ps_bf;
    }
    stack.clear();
    leaf_begin();
    return true;
  }

  void leaf_begin() {
    evolve_begin(forward ? z_fwd : z_bck, (forward ? 1.0 : -1.0) * eps);
    state = W_LEAF;
  }

  // a leaf's evaluation is back: merge it into the subtree stack (the
  // recursion's post-order); 0 = next leaf, 1 = this depth's tree is built
  // and valid, -1 = invalid (the transition stops)
  int leaf_end() {
    Point& a = forward ? z_fwd : z_bck;
    ++n_lf;
    double h = H(a);
    if (std::isnan(h)) h = INFINITY;
    if (h - H0 > max_delta_h) divergent = true;
    double leaf_lsw = (h != INFINITY) ? H0 - h : -INFINITY;
    smp += (H0 - h > 0) ? 1.0 : std::exp(H0 - h);
    if (divergent) return -1;
    Sub s;
    s.level = 0;
    s.zp = a;
    s.ps_beg = scaled(a.p);
    s.ps_end = s.ps_beg;
    s.rho = a.p, s.p_beg = a.p, s.p_end = a.p;
    s.lsw = leaf_lsw;
    stack.push_back(std::move(s));
    while (stack.size() >= 2 && stack[stack.size() - 1].level == stack[stack.size() - 2].level) {
      Sub fin = std::move(stack.back());
      stack.pop_back();
      Sub& ini = stack.back();
      double lsw_sub = log_sum_exp(ini.lsw, fin.lsw);
      bool take = fin.lsw > lsw_sub;
      if (!take) take = uniform() < std::exp(fin.lsw - lsw_sub);
      Vec rho_sub = add(ini.rho, fin.rho);
      bool ok = criterion(ini.ps_beg, fin.ps_end, rho_sub);
      ok = criterion(ini.ps_beg, fin.ps_beg, add(ini.rho, fin.p_beg)) && ok;
      ok = criterion(ini.ps_end, fin.ps_end, add(fin.rho, ini.p_end)) && ok;
      if (!ok) return -1;
      if (take) ini.zp = std::move(fin.zp);
      ini.ps_end = std::move(fin.ps_end);
      ini.rho = std::move(rho_sub);
      ini.p_end = std::move(fin.p_end);
      ini.lsw = lsw_sub;
      ini.level += 1;
    }
    return (stack.size() == 1 && stack[0].level == depth) ? 1 : 0;
  }

  // the depth's tree is built: extend the trajectory; false = U-turn
  bool tr_extend() {
    Sub& r = stack[0];
    if (forward) {
      ps_fb = r.ps_beg, ps_ff = r.ps_end, rho_fwd = r.rho, p_fb = r.p_beg, p_ff = r.p_end;
    } else {
      ps_bf = r.ps_beg, ps_bb = r.ps_end, rho_bck = r.rho, p_bf = r.p_beg, p_bb = r.p_end;
    }
    ++depth;
    if (r.lsw > lsw)
      z_sample = r.zp;
    else if (uniform() < std::exp(r.lsw - lsw))
      z_sample = r.zp;
    lsw = log_sum_exp(lsw, r.lsw);
    rho = add(rho_bck, rho_fwd);
    bool ok = criterion(ps_bb, ps_ff, rho);
    ok = criterion(ps_bb, ps_fb, add(rho_bck, p_fb)) && ok;
    ok = criterion(ps_bf, ps_ff, add(rho_fwd, p_bf)) && ok;
    return ok;
  }

  void tr_finish() {
    t_nlf = n_lf;
    t_accept = smp / (n_lf > 1 ? n_lf : 1);
    t_depth = depth;
    t_div = divergent;
    t_energy = H(z_sample);
  }

  // ---------------------------------------------------- static HMC
  void update_L() {  // nuts.py StaticHMCChain._update_L: L = max(1, int(T / eps))
    const double r = T / eps;
    L = r >= 1.0 ? (r < 2147483647.0 ? (long)r : 2147483647L) : 1;
  }

  void hmc_start() {  // StaticHMCChain._transition up to its first leapfrog
    z_sample = z;
    z_sample.p = sample_p();
    z_init = z_sample;
    H0 = H(z_sample);
    n_lf = (int)L;
    hk = 0;
    evolve_begin(z_sample, eps);
    state = W_HMC;
  }

  void hmc_finish() {
    double h = H(z_sample);
    if (std::isnan(h)) h = INFINITY;
    const double acc = h == INFINITY ? 0.0 : (H0 - h > 0 ? 1.0 : std::exp(H0 - h));
    if (acc < 1.0 && uniform() > acc) z_sample = z_init;
    t_accept = (acc < 1.0) ? acc : 1.0;  // Python's min(1.0, accept)
    t_nlf = n_lf;
    t_div = false;
    t_energy = H(z_sample);
  }

  // ------------------------------------------------------------ program
  void iter_finish() {
    if (warm && it == num_warmup - 1) eps = std::exp(x_bar);  // complete_adaptation
    if (it % thin == 0) {
      dq.insert(dq.end(), z.q.begin(), z.q.end());
      double st[8] = {z.lp, t_accept, eps_used, hmc ? T : (double)t_depth, (double)t_nlf, t_div ? 1.0 : 0.0,
                      t_energy, warm ? 1.0 : 0.0};
      dstat.insert(dstat.end(), st, st + 8);
    }
    ++it;
  }

  // run until the chain needs an evaluation (true; its position is *ev's q)
  // or is finished / failed (false)
  bool run_iterations() {
    while (it < total) {
      warm = it < num_warmup;
      eps_used = eps;
      if (hmc) {
        hmc_start();
        return true;
      }
      tr_start();
      if (tr_depth()) return true;
      tr_finish();
      if (after_transition()) return true;
    }
    state = DONE;
    return false;
  }

  // the transition is over: adaptation, then the draw; true = init_stepsize
  // asked for an evaluation
  bool after_transition() {
    Point a;
    a.q = z_sample.q, a.p.assign(dim, 0.0), a.g = z_sample.g, a.lp = z_sample.lp;
    z = std::move(a);
    if (warm) {
      learn_stepsize(t_accept);
      if (hmc) update_L();
      if (learn_variance(z.q)) {
        if (iss_start(AFTER_WINDOW)) return true;
        if (hmc) update_L();
        da_restart();
      }
    }
    iter_finish();
    return false;
  }

  bool fail(int code) {
    err = code;
    state = FAILED;
    return false;
  }

  // the (lp, grad) of the pending position; returns true when the chain
  // asks for another one
  bool feed(double lp, const double* g) {
    switch (state) {
      case W_INIT: {
        z.q = q0, z.p.assign(dim, 0.0), z.g.assign(g, g + dim), z.lp = lp;
        if (!std::isfinite(lp)) return fail(ERR_INIT);
        if (iss_start(AFTER_INIT)) return true;
        da_restart();
        it = 0;
        return run_iterations();
      }
      case W_ISS_FIRST:
      case W_ISS_LOOP: {
        evolve_end(lp, g);
        double dH = iss_dH();
        const double l08 = std::log(0.8);
        if (state == W_ISS_FIRST) {
          idir = dH > l08 ? 1 : -1;
        } else {
          bool stop = (idir == 1 && !(dH > l08)) || (idir == -1 && !(dH < l08));
          if (stop) {
            if (cont == AFTER_WINDOW && hmc) update_L();  // (not after the initial one: nuts.py's order)
            da_restart();
            if (cont == AFTER_INIT) {
              it = 0;
              return run_iterations();
            }
            iter_finish();
            return run_iterations();
          }
          eps = idir == 1 ? eps * 2.0 : eps * 0.5;
          if (eps > 1e7) return fail(ERR_IMPROPER);
          if (eps == 0) return fail(ERR_SMALL);
        }
        iss_loop();
        return true;
      }
      case W_HMC: {
        evolve_end(lp, g);
        if (++hk < n_lf) {
          evolve_begin(z_sample, eps);
          return true;
        }
        hmc_finish();
        if (after_transition()) return true;
        return run_iterations();
      }
      case W_LEAF: {
        evolve_end(lp, g);
        int r = leaf_end();
        if (r == 0) {
          leaf_begin();
          return true;
        }
        if (r == 1 && tr_extend() && tr_depth()) return true;
        tr_finish();
        if (after_transition()) return true;
        return run_iterations();
      }
      default:
        return false;
    }
  }
};

struct Sampler {
  int n, dim;
  std::vector<Chain> chains;
  // phn_run's round state: the pending positions and their chains, and the
  // round's work arrays
  bool started = false;
  int m = 0;
  Vec Q, Q2, bl, mv, rows, lp, G;
  std::vector<int> idx, idx2, sel;
};

}  // namespace

extern "C" {

// nchains chains of dimension dim from q0 [nchains][dim]; bitgens[c] is
// chain c's numpy bit generator (Generator.bit_generator.ctypes.bit_generator).
// The remaining arguments are nuts.py Chain's (same defaults there).
void* phn_create(int nchains, int dim, const double* q0, void* const* bitgens, int num_warmup, int num_samples,
                 int thin, int max_depth, double delta, double gamma, double kappa, double t0, double stepsize,
                 int init_buffer, int term_buffer, int base_window, double max_delta_h) {
  Sampler* s = new Sampler;
  s->n = nchains, s->dim = dim;
  s->chains.resize(nchains);
  for (int c = 0; c < nchains; ++c) {
    Chain& ch = s->chains[c];
    ch.dim = dim;
    ch.rng = (bitgen_t*)bitgens[c];
    ch.num_warmup = num_warmup;
    ch.total = num_warmup + num_samples;
    ch.thin = thin > 1 ? thin : 1;
    ch.max_depth = max_depth;
    ch.delta = delta, ch.gamma = gamma, ch.kappa = kappa, ch.t0 = t0;
    ch.eps = stepsize;
    ch.max_delta_h = max_delta_h;
    ch.im.assign(dim, 1.0);
    ch.setup_windows(init_buffer, term_buffer, base_window);
    ch.da_counter = 0, ch.s_bar = 0, ch.x_bar = 0, ch.mu = 0;
    ch.q0.assign(q0 + (size_t)c * dim, q0 + (size_t)(c + 1) * dim);
    ch.state = Chain::W_INIT;
    ch.err = ERR_NONE;
    ch.it = 0;
    ch.ev = nullptr;
    ch.n_grad = 0;
  }
  return s;
}

void phn_free(void* h) { delete (Sampler*)h; }

// Every chain a static HMC chain instead (nuts.py StaticHMCChain: a fixed
// integration time T over L = max(1, int(T / eps)) leapfrog steps, one
// Metropolis accept of the end point; the draw record carries T in the
// tree-depth slot); call before the first phn_step.
void phn_set_static_hmc(void* h, double int_time) {
  for (Chain& ch : ((Sampler*)h)->chains) {
    ch.hmc = true;
    ch.T = int_time;
    ch.update_L();
  }
}

// One gradient round.  n_in chains (idx_in) hand back (lp_in[k], G_in[k]) for
// the positions the previous call asked for (n_in = 0 on the first call:
// every chain asks for its initial point).  Writes the next positions to
// Q_out [n_out][dim] with their chains in idx_out and returns n_out (0: all
// chains finished), or -(1 + chain) when a chain failed (phn_error).
int phn_step(void* h, int n_in, const int* idx_in, const double* lp_in, const double* G_in, double* Q_out,
             int* idx_out) {
  Sampler* s = (Sampler*)h;
  int dim = s->dim, m = 0;
  if (n_in == 0) {
    for (int c = 0; c < s->n; ++c) {
      Chain& ch = s->chains[c];
      if (ch.state != Chain::W_INIT) continue;
      std::memcpy(Q_out + (size_t)m * dim, ch.q0.data(), sizeof(double) * dim);
      idx_out[m++] = c;
    }
    return m;
  }
  for (int k = 0; k < n_in; ++k) {
    Chain& ch = s->chains[idx_in[k]];
    if (ch.feed(lp_in[k], G_in + (size_t)k * dim)) {
      std::memcpy(Q_out + (size_t)m * dim, ch.ev->q.data(), sizeof(double) * dim);
      idx_out[m++] = idx_in[k];
    } else if (ch.state == Chain::FAILED) {
      return -(1 + idx_in[k]);
    }
  }
  return m;
}

// The whole sampling loop natively: each gradient round maps the pending
// positions through the strict-clock posterior's native pre phase
// (host_model.cpp phh_strict_pre), evaluates the draws that reach the
// likelihood through `submit` / `wait` (the HIP library's phy_eval_submit /
// phy_eval_wait on its context `lik`, or any functions of that shape), maps
// the rows back through phh_strict_post and advances the chains -- what
// nuts.py's run_chains does through Posterior.log_prob_grad, without a
// Python round trip per round.  Runs at most max_rounds rounds per call
// (the caller reports progress between calls).  Returns 1 while chains
// remain, 0 when all are finished, -(1 + chain) when a chain failed
// (phn_error), -(1000000 + rc) when submit / wait returned rc != 0.
typedef int (*phn_submit_t)(void* ctx, int n, const double* blens, const double* model);
typedef int (*phn_wait_t)(void* ctx, double* out);
}  // extern "C"
extern "C" int phh_strict_pre(void* hnd, int n, const double* U, double* blens, double* mv, int* sel);
extern "C" void phh_strict_post(void* hnd, int n, const double* U, const double* rows, int rowlen, const int* sel,
                                int need_grad, double* lp, double* G);
extern "C" {

int phn_run(void* h, void* post, void* lik, phn_submit_t submit, phn_wait_t wait, int B, int ml, int rowlen,
            int max_rounds, long* rounds) {
  Sampler* s = (Sampler*)h;
  const int n = s->n, dim = s->dim;
  if (!s->started) {
    s->Q.assign((size_t)n * dim, 0.0), s->Q2 = s->Q, s->G = s->Q;
    s->bl.assign((size_t)n * B, 0.0), s->mv.assign((size_t)n * ml, 0.0), s->rows.assign((size_t)n * rowlen, 0.0);
    s->lp.assign(n, 0.0), s->idx.assign(n, 0), s->idx2.assign(n, 0), s->sel.assign(n, 0);
    s->m = phn_step(h, 0, nullptr, nullptr, nullptr, s->Q.data(), s->idx.data());
    s->started = true;
  }
  for (int r = 0; r < max_rounds && s->m > 0; ++r) {
    const int m = s->m;
    const int cnt = phh_strict_pre(post, m, s->Q.data(), s->bl.data(), s->mv.data(), s->sel.data());
    if (cnt > 0) {
      int rc = submit(lik, cnt, s->bl.data(), s->mv.data());
      if (!rc) rc = wait(lik, s->rows.data());
      if (rc) return -(1000000 + rc);
    }
    phh_strict_post(post, m, s->Q.data(), s->rows.data(), rowlen, s->sel.data(), 1, s->lp.data(), s->G.data());
    const int m2 = phn_step(h, m, s->idx.data(), s->lp.data(), s->G.data(), s->Q2.data(), s->idx2.data());
    if (m2 < 0) return m2;
    std::swap(s->Q, s->Q2);
    std::swap(s->idx, s->idx2);
    s->m = m2;
    if (rounds) ++*rounds;
  }
  return s->m > 0 ? 1 : 0;
}

// chain c's failure: 1 non-finite initial log density, 2 step size > 1e7,
// 3 no acceptable small step size
int phn_error(void* h, int c) { return ((Sampler*)h)->chains[c].err; }

// chain c's results: the number of draws, gradient evaluations, final step
// size; inv_metric [dim] when non-null
int phn_info(void* h, int c, long* n_grad, double* eps, double* inv_metric) {
  Chain& ch = ((Sampler*)h)->chains[c];
  if (n_grad) *n_grad = ch.n_grad;
  if (eps) *eps = ch.eps;
  if (inv_metric) std::memcpy(inv_metric, ch.im.data(), sizeof(double) * ch.dim);
  return (int)(ch.dstat.size() / 8);
}

// chain c's draws: q [nd][dim] and stats [nd][8] (lp, accept, step size,
// depth, n_leapfrog, divergent, energy, warmup) -- nuts.py's draw tuples
void phn_draws(void* h, int c, double* q, double* stats) {
  Chain& ch = ((Sampler*)h)->chains[c];
  std::memcpy(q, ch.dq.data(), sizeof(double) * ch.dq.size());
  std::memcpy(stats, ch.dstat.data(), sizeof(double) * ch.dstat.size());
}

}  // extern "C"
