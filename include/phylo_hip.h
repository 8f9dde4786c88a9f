/*
 * phylo_hip.h -- C-ABI of the MI355X Felsenstein-pruning likelihood engine.
 *
 * This is the drop-in boundary that replaces phylostan's likelihood hot path
 * (SURVEY.md 8b).  In the reference the same role is played by
 *
 *   - the Stan external function declared without a body
 *       real pruning_loglik(vector blens);            eigen/example.stan:3
 *     with its double overload (eigen/eigen.j2:171-177) and its autodiff
 *     overload returning precomputed_gradients(log_P, blens, grad)
 *       (eigen/prune_stan.hpp:9-17), backed by
 *       value_grad vbsky_loglik(const vector<double>& times)
 *       (eigen/eigen.j2:56-168; struct value_grad eigen/value_grad.hpp:5-8),
 *   - and, for the generated models, the Stan code emitted by
 *       phylostan/generate_script.py:961-1055 (likelihood loop),
 *       :755-892 (JC69 / HKY / GTR P-matrices) and
 *       :249-282 (Weibull site rates -> rs, ps),
 *     differentiated by Stan's reverse-mode autodiff.
 *
 * This header is the consumer boundary: what a Stan external function or a
 * sampler host binds.  Planning, tuning and introspection calls (tests,
 * bench.py, diagnostics) are in phylo_hip_diag.h.
 *
 * Plain C types only: pointers + sizes, no torch / HIP types in signatures.
 * Every function returns 0 on success and a nonzero PHY_E* code on misuse or
 * a HIP failure; phy_last_error() then returns a message (thread-local).
 * A non-finite log-likelihood is NOT an error: it is returned as -inf with
 * status 0 so a sampler rejects the draw, as Stan does.
 *
 * Conventions (identical to the reference's, minus one for 0-based ids):
 *   S taxa, P site patterns, C rate categories.
 *   Node ids: tips 0..S-1 in taxon-namespace order, internal S..2S-2 in
 *     post-order, root 2S-2   (phylostan/utils.py:59-72).
 *   peel[(S-1)*3]: rows (child1, child2, parent), post-order
 *     (phylostan/utils.py:75-81).  Unrooted (no clock) trees: the last row's
 *     child2 must be node 2S-3, whose branch is merged into child1's
 *     (phylostan/phylostan.py:264-267, generate_script.py:1019).
 *   B = 2S-2 branches (rooted) or 2S-3 (unrooted); branch b is the edge
 *     above node b, so blens[b] == Stan blens[b+1]
 *     (generate_script.py:1193-1196, :663-671).
 *   tipcodes[S*P]: 4-bit state masks, A=1 C=2 G=4 T=8; any other symbol 15
 *     (the reference's [1,1,1,1], phylostan/utils.py:180-187).
 *   Per-draw model vector, length PHY_MODEL_LEN(C) = 10 + 2C:
 *     [0..3]  freqs (pi_A, pi_C, pi_G, pi_T)
 *     [4..9]  exchangeabilities AC, AG, AT, CG, CT, GT (GTR; HKY passes
 *             (1,kappa,1,1,kappa,1), generate_script.py:799-802; JC69 ignores)
 *     [10..10+C)     rs  (category rates)
 *     [10+C..10+2C)  ps  (category weights)
 *   Per-draw output vector, length phy_output_len() = 1 + B + 2C + 14 + 16*C*B
 *   (1 + B + 2C + 14 when compact, phy_set_output):
 *     [0]                 log-likelihood  sum_i w_i log L_i
 *     [1 .. 1+B)          dlogL/dblens
 *     [1+B .. 1+B+C)      dlogL/drs
 *     [1+B+C .. 1+B+2C)   dlogL/dps
 *     [1+B+2C .. +4)      dlogL/dfreqs, explicit root term only
 *     [1+B+2C+4 .. +6)    dlogL/d exchangeabilities AC AG AT CG CT GT through
 *                         the normalised Q and its eigendecomposition
 *                         (generate_script.py:839-892; HKY: dlogL/dkappa is
 *                         the AG + CT entries; zeros for JC69)
 *     [1+B+2C+10 .. +4)   dlogL/dfreqs, total (through Q plus the root term)
 *     [PHY_OUT_G(B,C) ..) dlogL/dP[c][b][4][4] (row-major P[j][k]); index
 *                         c*B + b is Stan's pmats[b + c*bcount]
 */
#ifndef PHYLO_HIP_H
#define PHYLO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct phy_ctx phy_ctx;

enum { PHY_JC69 = 0, PHY_HKY = 1, PHY_GTR = 2 };

enum {
  PHY_OK = 0,
  PHY_EINVAL = 1,   /* bad argument / inconsistent topology */
  PHY_EHIP = 2,     /* HIP runtime failure */
  PHY_ENOMEM = 3,   /* device allocation failed */
  PHY_ERANGE = 4    /* n_draws > max_draws etc. */
};

#define PHY_MODEL_LEN(C) (10 + 2 * (C))
#define PHY_OUT_G(B, C) (1 + (B) + 2 * (C) + 14)

/* Build a context: copies the static data (tips, weights, topology) to the
 * device, derives the kernel traversal program and allocates every work
 * buffer.  Replaces the compile-time baking of topology / tips / Q into the
 * generated header (eigen/util.py:103-109, eigen/eigen.j2:19-38) and the
 * Stan data block (generate_script.py:1186-1197).
 *   rooted: 1 = clock variants (:984-1012), 0 = unrooted (:1013-1040).
 *   max_draws: most independent parameter points one phy_eval may batch.
 *   device: HIP device ordinal (one process per GPU). */
int phy_create(int S, int P, int C, int rooted, int model,
               const uint8_t* tipcodes, const double* weights, const int32_t* peel,
               int max_draws, int device, phy_ctx** out);

/* One context over several devices (phy_create's n_dev; 8e:
 * single-process multi-device with RCCL inside the context).  The P
 * patterns are split into n_shards contiguous ranges of whole 128-pattern
 * blocks (counts differ by <= 1), shard k a full context on devices[k].  An
 * evaluation runs every shard on its own stream, then reduces the fp64
 * output rows once: ncclAllReduce(sum) over the shards' communicators
 * (ncclCommInitAll; RCCL is loaded on first use) when the devices are all
 * distinct, a device-side sum in shard order when they are all the same
 * (any other mix is PHY_EINVAL).  Rows equal the single-context rows to
 * rounding (every entry is a sum over patterns); site log-likelihoods are
 * gathered into [n][P] by phy_eval.  phy_eval, phy_eval_submit / wait,
 * phy_pruning_loglik, phy_eval_device (buffers on devices[0], no site_ll),
 * phy_set_output / engine / tuning (applied to every shard) and the info
 * queries (shard 0) accept the returned handle; phy_destroy frees it all.
 * The reference's boundary is one synchronous call per log_prob
 * (eigen/prune_stan.hpp:9-17): this is how that single handle reaches a
 * whole node. */
int phy_create_multi(int S, int P, int C, int rooted, int model, const uint8_t* tipcodes, const double* weights,
                     const int32_t* peel, int max_draws, int n_shards, const int* devices, phy_ctx** out);

int phy_destroy(phy_ctx* ctx);

/* Message of the last failure on this thread ("" if none). */
const char* phy_last_error(void);

int phy_num_branches(const phy_ctx* ctx);
int phy_output_len(const phy_ctx* ctx);
/* Log-likelihood + full gradient of n_draws parameter points, host buffers,
 * synchronous.  blens[n_draws*B], model[n_draws*PHY_MODEL_LEN(C)],
 * out[n_draws*phy_output_len()], site_ll[n_draws*P] (per-site log L_i, may
 * be NULL).  The batched analogue of vbsky_loglik (eigen/eigen.j2:56). */
int phy_eval(phy_ctx* ctx, int n_draws, const double* blens, const double* model,
             double* out, double* site_ll);

/* Same, device buffers, asynchronous on `stream` (a hipStream_t).  Nothing is
 * copied to or from the host.  The work is ordered after everything queued
 * on `stream` before the call, and everything queued on `stream` after the
 * call is ordered after it -- for stream = NULL that is HIP's legacy null
 * stream (the default stream of a HIP / torch caller), so a producer and a
 * consumer on the null stream need no synchronisation of their own.  (On the
 * null stream the engine runs on the context's own stream fenced both ways
 * with events; phy_sync also waits for it.) */
int phy_eval_device(phy_ctx* ctx, int n_draws, const double* d_blens, const double* d_model,
                    double* d_out, double* d_site_ll, void* stream);

/* Asynchronous small batches (host buffers, 1 <= n_draws <= min(max_draws,
 * 128)): phy_eval_submit copies the inputs into the context's pinned staging
 * and queues the upload, the evaluation and the download of the output rows
 * on the context's stream, then returns; phy_eval_wait blocks until they are
 * done and copies the n_draws rows (phy_output_len doubles each) into `out`.
 * One submission in flight per context (phy_eval refuses while one is);
 * contexts on one device run concurrently.  phy_eval takes the same path for
 * n_draws <= 128 (ADVI's elbo_samples = 100 fits), plus site
 * log-likelihoods.  No reference counterpart: the reference's log_prob is
 * synchronous (eigen/prune_stan.hpp:9-17). */
int phy_eval_submit(phy_ctx* ctx, int n_draws, const double* blens, const double* model);
int phy_eval_wait(phy_ctx* ctx, double* out);

/* Mirror of the reference's external Stan function: the double overload
 * returns log P (eigen/eigen.j2:171-177); with grad != NULL it also fills
 * dlogL/dblens[B] -- the `grads` that prune_stan.hpp:16 hands to
 * precomputed_gradients.  Returns NaN (and sets phy_last_error) on misuse. */
double phy_pruning_loglik(phy_ctx* ctx, const double* blens, const double* model, double* grad);

/* Wait for all work of the context (its stream, and phy_eval_device work
 * queued on the null stream). */
int phy_sync(phy_ctx* ctx);

/* Output rows: compact = 1 drops the dL/dP block (rows end after the
 * model-parameter gradients: what a sampler consumes, 1 + B + 2C + 14
 * doubles per draw instead of + 16CB more); 0 = full rows (default).
 * phy_output_len follows. */
int phy_set_output(phy_ctx* ctx, int compact);

#ifdef __cplusplus
}
#endif
#endif /* PHYLO_HIP_H */
