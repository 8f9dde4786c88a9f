/*
 * phylo_hip_diag.h -- planning, tuning and introspection calls of the
 * MI355X pruning engine (libphylo_hip.so), beside the consumer boundary in
 * phylo_hip.h.  None of these has a reference counterpart: they expose the
 * launch plans (LDS chunks, column plans, class-sweep fusions, the sampler's
 * quad schedule), switch between engines and between bitwise-equal fused and
 * unfused forms (the tests' reference paths), and time the dominant kernel
 * (bench.py).  A Stan external function needs none of them.
 */
#ifndef PHYLO_HIP_DIAG_H
#define PHYLO_HIP_DIAG_H

#include "phylo_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Traversal-program facts: steps (= S-1), partial slots, deep-stack entries
 * (operands that wait while a sibling subtree runs), pattern blocks of the
 * current column plan. */
int phy_program_info(const phy_ctx* ctx, int* nsteps, int* nslots, int* depth, int* nblocks);

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
int phy_recomputed_partials(const phy_ctx* ctx);

/* Engine: 1 = pattern sweep (one lane per pattern column; a call of at most
 * 32 draws takes its quad form -- a quad of lanes per column, matrix records
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
 */
int phy_class_chain(const phy_ctx* ctx, int* levels, int* lowest, int* top_classes);

/* Launch fusions and layouts of the class sweep's level launches, all
 * bitwise the unfused / default values (read at phy_create):
 *   level_pairs   forward level pairs -- adjacent levels (above the fused
 *                 clade levels, below the top chain) in one launch, the upper
 *                 level recomputing its children of the level below from
 *                 theirs.  PHY_PAIR=0: none; PHY_PAIR_MAX=n: only upper
 *                 levels of at most n classes (default: no cap).
 *   chunk_spans   long tile-crossing segments summed by the reverse chunk
 *                 of their class (the whole wave), so those levels have no
 *                 FIX launch.  PHY_REVFIX=0: none.
 *   parent_order_levels  levels whose secondary children's staging is
 *                 written in the parent's class order and gathered by the
 *                 RED tiles through a permutation (levels staging at least
 *                 100,000 classes; PHY_STAGE_ORDER=n sets that threshold,
 *                 0: every level above the clades). */
int phy_class_fused(const phy_ctx* ctx, int* level_pairs, int* chunk_spans, int* parent_order_levels);

/* The sampler's small-call sweep (calls of <= 32 draws, the quad sweep):
 * waves per category (0: the quad sweep does not apply to this context, 1:
 * the one-wave quad sweep, 2 up to 16 / C: the multi-wave form, whose host
 * list-schedule splits the post-order program over that many waves with LDS
 * hand-offs -- the most waves whose hand-off slots still fit LDS),
 * the schedule's length in program steps (the one-wave sweep: every step),
 * and its LDS hand-off slots.  PHY_QMW=0 at phy_create keeps the one-wave
 * form; the rows are bitwise the same either way. */
int phy_quad_plan(const phy_ctx* ctx, int* waves, int* span, int* slots);

#ifdef __cplusplus
}
#endif
#endif /* PHYLO_HIP_DIAG_H */
