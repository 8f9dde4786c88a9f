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
/* Traversal-program facts: steps (= S-1), partial slots, deep-stack entries
 * (operands that wait while a sibling subtree runs), pattern blocks of the
 * current column plan. */
int phy_program_info(const phy_ctx* ctx, int* nsteps, int* nslots, int* depth, int* nblocks);

/* Log-likelihood + full gradient of n_draws parameter points, host buffers,
 * synchronous.  blens[n_draws*B], model[n_draws*PHY_MODEL_LEN(C)],
 * out[n_draws*phy_output_len()], site_ll[n_draws*P] (per-site log L_i, may
 * be NULL).  The batched analogue of vbsky_loglik (eigen/eigen.j2:56). */
int phy_eval(phy_ctx* ctx, int n_draws, const double* blens, const double* model,
             double* out, double* site_ll);

/* Same, device buffers, asynchronous on `stream` (a hipStream_t; NULL =
 * the context's own stream).  Nothing is copied to or from the host. */
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

/* Wait for all work of the context's stream. */
int phy_sync(phy_ctx* ctx);

/* Measurement hooks (bench.py): while enabled, every phy_eval* records HIP
 * events around the sweep kernel on the stream it runs on;
 * phy_timing_read synchronises and returns the summed sweep-kernel time in
 * ms and the number of launches since phy_timing_start. */
int phy_timing_start(phy_ctx* ctx);
int phy_timing_read(phy_ctx* ctx, double* total_ms, int* launches);

/* Tuning: persistent workgroup budget per launch (0 = keep), columns per
 * lane `cols` (0 = automatic: 2 for C <= 8, else 1) and the LDS bytes one
 * workgroup may use (0 = keep; smaller budgets stage the P-matrix records
 * in more chunks).  The automatic LDS plan (no PHY_LDS_BUDGET, nothing set
 * here) takes the most workgroups per CU the kernel's register budget
 * allows whose LDS share still holds chunks of >= 24 matrices (or the whole
 * program).  The environment variables PHY_WG_BUDGET, PHY_COLS and
 * PHY_LDS_BUDGET set the defaults at phy_create. */
int phy_set_tuning(phy_ctx* ctx, int wg_budget, int cols, int lds_budget);

/* The LDS plan the next launch will use: chunks per pass, matrices per
 * chunk, LDS bytes per workgroup. */
int phy_lds_plan(const phy_ctx* ctx, int* n_chunks, int* matrices_per_chunk, int* lds_bytes);

/* Pattern columns each lane carries in the current plan (1 or 2). */
int phy_columns_per_lane(const phy_ctx* ctx);

/* Where the sweep keeps its deep stack (operands that wait while a sibling
 * subtree runs; phy_program_info's `depth` entries): 0 = automatic (all of
 * it in LDS when that leaves matrix chunks of >= 24 at the plan's
 * occupancy, else its outermost entries in LDS and the rest in the global
 * per-workgroup region), 1 = LDS, 2 = global.  Replans; PHY_DEEP sets the
 * default at phy_create.  phy_deep_stack_in_lds returns how many entries
 * the current plan holds in LDS. */
int phy_set_deep_stack(phy_ctx* ctx, int mode);
int phy_deep_stack_in_lds(const phy_ctx* ctx);

/* Recomputed cherries (default on; PHY_RECOMPUTE=0 at phy_create turns it
 * off): a node whose two children are tips, computed by the step just before
 * its parent's and in the same LDS chunk, is not written to scratch in the
 * forward half; the parent's reverse step rebuilds it from LDS.  Results are
 * identical either way (same operations in the same order).
 * phy_recomputed_partials: moved partials per column the current plan does
 * not store. */
int phy_set_recompute(phy_ctx* ctx, int on);

/* HIP graphs (default off; PHY_GRAPH=1 at phy_create turns them on): an
 * evaluation whose operands (draw count, buffers, stream) repeat is
 * captured once -- its copies and every kernel launch, up to ~50 for the
 * class sweep -- and replayed as one graph launch.  The first run of an
 * operand set is direct, the second captures; any replan, output-layout or
 * engine change rebuilds.  Evaluations under phy_timing_start run direct.
 * Results are identical either way.  Measured on MI355X: no gain (a 4-draw
 * call 167 -> 174 us; the class sweep's ~50 launches are bound by GPU-side
 * gaps between dependent kernels, which a graph keeps).  No reference
 * counterpart (a launch mechanism). */
int phy_set_graphs(phy_ctx* ctx, int on);
int phy_recomputed_partials(const phy_ctx* ctx);

/* Output rows: compact = 1 drops the dL/dP block (rows end after the
 * model-parameter gradients: what a sampler consumes, 1 + B + 2C + 14
 * doubles per draw instead of + 16CB more); 0 = full rows (default).
 * phy_output_len follows. */
int phy_set_output(phy_ctx* ctx, int compact);

/* Engine: 1 = pattern sweep (one lane per pattern column; a call of at most
 * 16 draws takes its quad form -- a quad of lanes per column, matrix records
 * built in the sweep when the eigensystems are host-formed, an epilogue split
 * over workgroups; PHY_QUAD=0 at phy_create keeps the column sweep), 2 = class sweep
 * (site repeats: the forward pass once per distinct tip-state tuple of each
 * subtree, the reverse on upper partials aggregated per tuple -- the exact,
 * total form of the reference's column-reuse cache, pruner/tree.cpp:140-174),
 * 0 = automatic (class sweep for alignments of >= 16384 patterns whose
 * subtree classes are at most a quarter of the pattern sweep's node-pattern
 * work).  Results agree to rounding either way.  PHY_ENGINE sets the default
 * at phy_create.  Mode 3 (round 3's resident class sweep) is retired and
 * refused with PHY_EINVAL: the quad sweep is faster for a sampler's calls on
 * every workload.  phy_engine returns the engine the next launch uses (0
 * pattern, 1 class). */
int phy_set_engine(phy_ctx* ctx, int mode);
int phy_engine(const phy_ctx* ctx);

/* The class sweep's launch form: 1 = ONE dataflow launch for the whole sweep
 * -- forward chunks, root, the reverse's tile reductions, span fix-ups and
 * chunks as work items that wait only for the items they read (per-node
 * completion counters, no grid-wide barrier); 0 (default; PHY_FLOW=1 at
 * phy_create sets 1) = one launch per tree level and phase, measured faster
 * on MI355X.  Results are bitwise the same.  Shards of a same-device phy_create_multi context always use the
 * level launches (their launches run concurrently).  phy_flow returns 1 when
 * the next class-sweep launch is the dataflow one.  No reference counterpart
 * (a launch mechanism for the column-reuse idea of pruner/tree.cpp:140-174). */
int phy_set_flow(phy_ctx* ctx, int on);
int phy_flow(const phy_ctx* ctx);

/* Class-plan facts (zeros when no plan is built): non-root subtree classes
 * (the class sweep's forward work per category), levels (the root's level),
 * root classes (distinct site patterns by tip state), contributions (sum over
 * internal nodes of classes x internal children: the reverse's aggregation
 * inputs), the part of them staged through HBM (secondary children; a
 * primary child's are reduced in registers), reduction tiles and
 * tile-crossing segments. */
int phy_class_info(const phy_ctx* ctx, long long* classes, int* levels, int* root_classes, long long* stage,
                   long long* staged, int* tiles, int* spans);

/* Bottom clades of the class plan: the levels 1..fused_levels run as one
 * workgroup per clade (a maximal subtree of nodes at those levels) instead
 * of one launch per level and phase; clades, and the classes of the largest.
 * Chosen automatically (the deepest level whose largest clade has at most
 * 1024 classes); PHY_CLADE=k at phy_create fixes k levels (0: off).
 * Results are bitwise the same either way. */
int phy_class_clades(const phy_ctx* ctx, int* fused_levels, int* clades, long long* largest);

/* Top chain of the class plan: the run of single-node levels below the root
 * (caterpillar-like trees), fused into one forward and one reverse launch
 * (one lane per class of the top node, the classes below it from host
 * tables); chain levels (0: none), the lowest chained level and the top
 * node's classes.  Chosen when at least two such levels lie above the clade
 * levels (at most 8); PHY_CHAIN=0 at phy_create turns it off.  The forward
 * values are bitwise the level launches'; the dL/dP sums of the chained
 * branches run over the top classes, so they agree to rounding, not bits.
 * A plan with a chain has no dataflow launch (phy_set_flow has no effect). */
int phy_class_chain(const phy_ctx* ctx, int* levels, int* lowest, int* top_classes);

/* Launch fusions of the class sweep's level launches, both bitwise the
 * unfused values (read at phy_create):
 *   level_pairs   forward level pairs -- adjacent levels (above the fused
 *                 clade levels, below the top chain) in one launch, the upper
 *                 level recomputing its children of the level below from
 *                 theirs.  PHY_PAIR=0: none; PHY_PAIR_MAX=n: only upper
 *                 levels of at most n classes (default: no cap).
 *   chunk_spans   long tile-crossing segments summed by the reverse chunk
 *                 of their class (the whole wave), so those levels have no
 *                 FIX launch.  PHY_REVFIX=0: none. */
int phy_class_fused(const phy_ctx* ctx, int* level_pairs, int* chunk_spans);

/* The sampler's small-call sweep (calls of <= 16 draws, the quad sweep):
 * waves per category (0: the quad sweep does not apply to this context, 1:
 * the one-wave quad sweep, 2-4: the multi-wave form, whose host list-schedule
 * splits the post-order program over that many waves with LDS hand-offs),
 * the schedule's length in program steps (the one-wave sweep: every step),
 * and its LDS hand-off slots.  PHY_QMW=0 at phy_create keeps the one-wave
 * form; the rows are bitwise the same either way. */
int phy_quad_plan(const phy_ctx* ctx, int* waves, int* span, int* slots);

#ifdef __cplusplus
}
#endif
#endif /* PHYLO_HIP_H */
