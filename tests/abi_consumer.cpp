// abi_consumer.cpp -- a C++ consumer of include/phylo_hip.h, compiled with
// g++ against libphylo_hip.so exactly as a Stan model would link the
// drop-in prune_stan.hpp of INTEGRATION.md section 1.
//
// The reference's plugin boundary (eigen/prune_stan.hpp:9-17) is a pair of
// overloads of `pruning_loglik`: the double one returns log P
// (eigen/eigen.j2:171-177); the autodiff one returns
// stan::math::precomputed_gradients(log_P, blens, grad) (prune_stan.hpp:16,
// struct value_grad eigen/value_grad.hpp:5-8).  Stan Math is absent here,
// so `standin::var` / `standin::precomputed_gradients` below keep only the
// part of its contract the boundary relies on: a value plus the partials
// with respect to each operand.  The pruning_loglik bodies are INTEGRATION.md
// section 1's, unchanged apart from the namespace.
//
// Test infrastructure: tests/test_gpu_abi_consumer.py writes the input
// file, runs this program on the GPU box and compares its output with the
// oracle.  Usage:
//   abi_consumer INPUT [single|multi2]
// INPUT (whitespace-separated text):
//   S P C rooted model n_draws
//   tipcodes[S*P] weights[P] peel[(S-1)*3]
//   then n_draws x (blens[B] model[10+2C])
// Output, one line per draw and overload:
//   <overload> <draw> loglik grad[0] .. grad[B-1]   (%.17g)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "phylo_hip.h"

namespace standin {
// stan::math::var reduced to what precomputed_gradients exposes: the value
// and the partial derivatives with respect to the operands it was built from
struct var {
  double val = 0.0;
  std::vector<const var*> operands;
  std::vector<double> partials;
  var() = default;
  explicit var(double v) : val(v) {}
};
inline double value_of(const var& v) { return v.val; }
inline var precomputed_gradients(double value, const std::vector<var>& operands, const std::vector<double>& grads) {
  if (operands.size() != grads.size()) throw std::invalid_argument("precomputed_gradients: size mismatch");
  var r(value);
  for (const var& o : operands) r.operands.push_back(&o);
  r.partials = grads;
  return r;
}
}  // namespace standin

// --- INTEGRATION.md section 1 (drop-in prune_stan.hpp), Eigen vectors as std::vector
phy_ctx* g_phy = nullptr;
std::vector<double> g_model;  // [pi(4), exch(6), rs(C), ps(C)] of this draw

inline double pruning_loglik(const std::vector<double>& blens, std::ostream*) {
  return phy_pruning_loglik(g_phy, blens.data(), g_model.data(), nullptr);
}

inline standin::var pruning_loglik(const std::vector<standin::var>& blens, std::ostream*) {
  std::vector<double> b(blens.size()), grad(blens.size());
  for (size_t i = 0; i < blens.size(); ++i) b[i] = standin::value_of(blens[i]);
  double lp = phy_pruning_loglik(g_phy, b.data(), g_model.data(), grad.data());
  if (lp != lp) throw std::domain_error(phy_last_error());  // misuse -> rejected draw
  return standin::precomputed_gradients(lp, blens, grad);  // as prune_stan.hpp:16
}
// ---

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s INPUT [single|multi2]\n", argv[0]);
    return 2;
  }
  const std::string mode = argc > 2 ? argv[2] : "single";
  std::ifstream in(argv[1]);
  int S, P, C, rooted, model, n;
  if (!(in >> S >> P >> C >> rooted >> model >> n)) {
    std::fprintf(stderr, "bad input header\n");
    return 2;
  }
  std::vector<uint8_t> tips((size_t)S * P);
  for (auto& t : tips) {
    int v;
    in >> v;
    t = (uint8_t)v;
  }
  std::vector<double> w(P);
  for (auto& x : w) in >> x;
  std::vector<int32_t> peel((size_t)(S - 1) * 3);
  for (auto& x : peel) in >> x;
  const int B = rooted ? 2 * S - 2 : 2 * S - 3;
  const int ml = PHY_MODEL_LEN(C);
  std::vector<std::vector<double>> bl(n, std::vector<double>(B)), md(n, std::vector<double>(ml));
  for (int d = 0; d < n; ++d) {
    for (auto& x : bl[d]) in >> x;
    for (auto& x : md[d]) in >> x;
  }
  if (!in) {
    std::fprintf(stderr, "truncated input\n");
    return 2;
  }
  int rc;
  if (mode == "multi2") {  // two pattern shards behind one handle (same device on a one-GPU box)
    const int devs[2] = {0, 0};
    rc = phy_create_multi(S, P, C, rooted, model, tips.data(), w.data(), peel.data(), 1, 2, devs, &g_phy);
  } else {
    rc = phy_create(S, P, C, rooted, model, tips.data(), w.data(), peel.data(), 1, 0, &g_phy);
  }
  if (rc) {
    std::fprintf(stderr, "phy_create failed (%d): %s\n", rc, phy_last_error());
    return 1;
  }
  if (phy_num_branches(g_phy) != B) {
    std::fprintf(stderr, "branch count mismatch\n");
    return 1;
  }
  for (int d = 0; d < n; ++d) {
    g_model = md[d];
    const double lp = pruning_loglik(bl[d], nullptr);
    std::printf("double %d %.17g\n", d, lp);
    std::vector<standin::var> bv(B);
    for (int b = 0; b < B; ++b) bv[b] = standin::var(bl[d][b]);
    const standin::var r = pruning_loglik(bv, nullptr);
    std::printf("var %d %.17g", d, r.val);
    for (int b = 0; b < B; ++b) std::printf(" %.17g", r.partials[b]);
    std::printf("\n");
    if (r.operands.size() != (size_t)B || r.operands[0] != &bv[0]) {
      std::fprintf(stderr, "precomputed_gradients lost its operands\n");
      return 1;
    }
  }
  // misuse is a NaN plus a message, never an abort (prune_stan.hpp's throw path)
  const double bad = phy_pruning_loglik(g_phy, nullptr, g_model.data(), nullptr);
  std::printf("misuse %s %s\n", std::isnan(bad) ? "nan" : "value", std::strlen(phy_last_error()) ? "msg" : "nomsg");
  phy_destroy(g_phy);
  return 0;
}
