/*
 * pf_lower.h — host-side C ABI of libpflower.so: register allocation and emission of one
 * constraint DAG into the bytecode of include/pf_bytecode.h (the native form of
 * mythril_amd/lower.py:lower, which stays as the reference the tests compare against).
 *
 * Reference interface it replaces: nothing in the reference lowers anything — every query
 * goes to libz3 through z3py (mythril/support/model.py:37-59).  This is the host half of
 * the engine's replacement for that call; it runs once per new independence bucket, so its
 * cost is the live analysis's per-query host latency.
 *
 * Host only (no HIP): the lowering worker processes load it without a GPU runtime.
 */
#ifndef PF_LOWER_H
#define PF_LOWER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* leaf kinds of DAG nodes (interior nodes carry a pf_opcode) */
#define PFL_K_VAR 200    /* aux = variable index (W variable)           */
#define PFL_K_CONST 201  /* aux = index into const_pool (8 x u32 each)  */
#define PFL_K_BCONST 202 /* aux = 0 / 1                                 */
#define PFL_K_BVAR 203   /* aux = variable index (Bool variable)        */

/* One node = 8 x u32: kind, width, nargs, arg0, arg1, arg2, aux, is_bool.  Nodes are in
 * topological order (operands first).  roots: the asserted Bool nodes, in order.
 * forced: constants pinned at pool indices 0.. (schema hints refer to them).
 * n_wregs: W registers the allocation may use (3..PF_NW; 0 = PF_NW).  PF_NW_NARROW makes a
 * program the 8-register search kernels run (3 waves/SIMD, pf_eval.hip).
 * Outputs: code_out (cap_ins x 4 u32; aux1 left 0), consts_out (cap_const x 8 u32).
 * Returns 0; -2 when the set needs more live values than the register file and spill
 * slots hold (LoweringError: the query goes to z3); -3 when an output is too small;
 * -1 on malformed input.  The message is in pfl_last_error().                          */
int pfl_lower(const uint32_t* nodes, size_t n_nodes, const uint32_t* const_pool, size_t n_pool,
              const uint32_t* roots, size_t n_roots, const uint32_t* forced, size_t n_forced,
              uint32_t n_wregs, uint32_t* code_out, size_t cap_ins, size_t* n_ins_out,
              uint32_t* consts_out, size_t cap_const, size_t* n_const_out);
const char* pfl_last_error(void);

/* Hint model of one DAG (the native form of mythril_amd/seed.py:Seeder.run, identical
 * values): nodes / const_pool / roots as for pfl_lower; var_widths[n_vars]; soft = the
 * caller's parent values (n_vars x 8 u32, the bits no constraint fixes).  hints_out gets
 * n_vars x 8 u32; n_sat_out the number of distinct roots the hint model satisfies.
 * Returns 0, or -1 on malformed input.                                                  */
int pfl_hints(const uint32_t* nodes, size_t n_nodes, const uint32_t* const_pool, size_t n_pool,
              const uint32_t* roots, size_t n_roots, const uint32_t* var_widths, size_t n_vars,
              const uint32_t* soft, uint32_t* hints_out, int* n_sat_out);
int pfl_version(void);

/* ---- term store: constraint terms -> DAG -> program, natively (csrc/pf_terms.cpp) -------
 * The native form of mythril_amd/smt/to_dag.py:TermLowering + lower.py:Dag, node for node,
 * followed by pfl_hints and pfl_lower (tests/test_native_terms.py).  Reference interface it
 * serves: the objective-free query path of mythril/support/model.py:63-125 (one bucket per
 * call; the fork-prune call site svm.py:351-358 poses two queries per fork).
 *
 * Terms (mythril_amd/smt/terms.py) enter the store once, children first; pflt_add returns
 * the term's id (or -1).  op = PFLT_* below; sortk 0 Bool / 1 bit-vector (w1 = width) /
 * 2 array (w1 = domain, w2 = range); i0/i1 = extract hi/lo or zero_extend's count; limbs =
 * a constant's value (little-endian u32); name = symbol, array or function name (for an
 * operator the store does not lower: its SMT-LIB name, quoted in the error). */
#define PFLT_BV 1
#define PFLT_TRUE 2
#define PFLT_FALSE 3
#define PFLT_VAR 4
#define PFLT_BVAR 5
#define PFLT_ARRAY 6
#define PFLT_K 7
#define PFLT_SELECT 8
#define PFLT_STORE 9
#define PFLT_APPLY 10
#define PFLT_EXTRACT 11
#define PFLT_CONCAT 12
#define PFLT_ZERO_EXTEND 13
#define PFLT_ITE 14
#define PFLT_EQ 15
#define PFLT_IFF 16
#define PFLT_AND 17
#define PFLT_OR 18
#define PFLT_NOT 19
#define PFLT_XOR 20
#define PFLT_BVNOT 21
#define PFLT_BVNEG 22
#define PFLT_BVADD 30
#define PFLT_BVSUB 31
#define PFLT_BVMUL 32
#define PFLT_BVUDIV 33
#define PFLT_BVUREM 34
#define PFLT_BVSDIV 35
#define PFLT_BVSREM 36
#define PFLT_BVSMOD 37
#define PFLT_BVAND 38
#define PFLT_BVOR 39
#define PFLT_BVXOR 40
#define PFLT_BVSHL 41
#define PFLT_BVLSHR 42
#define PFLT_BVASHR 43
#define PFLT_BVEXP 44
#define PFLT_BVULT 50
#define PFLT_BVULE 51
#define PFLT_BVSLT 52
#define PFLT_BVSLE 53
#define PFLT_BVUADD_NOOVF 54
#define PFLT_BVUMUL_NOOVF 55
#define PFLT_OTHER 99
/* var_terms descriptor types: the variable's term / select(array a, index b) /
 * extract(hi c, lo b) of term a */
#define PFLT_VT_TERM 0
#define PFLT_VT_SELECT 1
#define PFLT_VT_EXTRACT 2
/* pflt_lower flags */
#define PFLT_HINTS 1u    /* derive the hint model (seed.apply_hints) */
#define PFLT_PROGRAM 2u  /* allocate registers and emit (lower.lower) */
#define PFLT_EXPLICIT 4u /* explicit-model lowering (to_dag.ExplicitLowering): every base-array
                            read and UF application is a leaf variable (GPU-resident ModelCache) */
/* pflt_result_get selectors */
#define PFLT_GET_VARS 0
#define PFLT_GET_VAR_TERMS 1
#define PFLT_GET_UF_APPS 2
#define PFLT_GET_READS 3
#define PFLT_GET_CODE 4
#define PFLT_GET_CONSTS 5
#define PFLT_GET_NODES 6
#define PFLT_GET_POOL 7
#define PFLT_GET_ROOTS 8
#define PFLT_GET_FORCED 9
#define PFLT_GET_IN_ROOTS 10  /* the bucket's conjuncts as given */

/* A new term store.  Also throws and catches one C++ exception, so the process's one-time
 * unwinder set-up (~80 ms with PyTorch's libraries loaded) happens here, not inside the first
 * lowering whose hint solver meets a conflict. */
void* pflt_store_new(void);
/* optional pflt_lower modes this build has (PFLT_FEAT_*) */
#define PFLT_FEAT_EXPLICIT 1u
#define PFLT_FEAT_SYNTH 2u
uint32_t pflt_features(void);
/* BASELINE config 3's synthetic DAGs natively: results[i] = the lowered program of
 * mythril_amd.synth.random_dag_set(first_id + i, plant) bit for bit (numpy's Philox4x64
 * Generator stream restated), for pflt_pack_batch; cdf = the op mix's 8 normalised cumulative
 * probabilities; witness_limbs (optional, 8 x 8 u32 per DAG) and n_vars_out (optional) get
 * the planted witness.  0, or -1 with pflt_last_error(); free each result with
 * pflt_result_free.  Not the reference's: the benchmark's input generator. */
int pflt_synth(uint32_t first_id, size_t n, uint32_t plant, const double* cdf, void** results,
               uint32_t* witness_limbs, uint32_t* n_vars_out);
void pflt_store_free(void* store);
size_t pflt_store_size(void* store);
int64_t pflt_add(void* store, uint32_t op, uint32_t sortk, uint32_t w1, uint32_t w2, const uint32_t* args,
                 uint32_t nargs, int64_t i0, int64_t i1, const uint32_t* limbs, uint32_t nlimbs,
                 const char* name);
/* Lower one bucket (roots = its conjuncts' term ids).  registry = n_actors, actors x 8 u32,
 * n_specs, then per keccak width: n, has_lo, base x 8, n_concrete, per concrete hash: the
 * input value (ceil(n / 32) u32) and the digest (8 u32).  Parent models: symbol names
 * ('\0'-separated) with values (per name: its limb count, then the limbs — any width), and
 * array reads (array id, index id) with values (8 u32 each).  Returns a result handle (0 and *rc_out = -2 when the set leaves the lowering's
 * vocabulary or register file: LoweringError -> z3; -1 on malformed input); the message is
 * in pflt_last_error().  flags: PFLT_HINTS | PFLT_PROGRAM. */
void* pflt_lower(void* store, const uint32_t* roots, size_t n_roots, const uint32_t* registry,
                 size_t n_registry, const char* par_names, const uint32_t* par_name_vals, size_t n_par_names,
                 const uint32_t* par_reads, const uint32_t* par_read_vals, size_t n_par_reads,
                 uint32_t flags, uint32_t seed, int* rc_out);
const char* pflt_last_error(void);
void pflt_result_free(void* result);
void pflt_result_info(void* result, uint64_t* info);  /* 17 sizes, see pf_terms.cpp */
/* n results at once (pflt_lower_many's): out = n rows of 18 u64, the result's status
 * (pflt_result_status) then its 17 pflt_result_info sizes (zeros for a failed result). */
void pflt_result_info_many(void* const* results, size_t n, uint64_t* out);
void pflt_result_get(void* result, uint32_t which, uint32_t* out, char* names_out);
/* Candidate 0 of the result's program when every variable carries a parent value: the
 * parents masked to their widths, 8 u32 per variable, into out (the generator keeps every
 * parented variable's parent at candidate 0, pf_bytecode.h).  Returns 1, or 0 (out untouched)
 * when some variable has no parent.  Replaces a pf_materialize launch for such witnesses. */
int pflt_result_candidate0(const void* result, uint32_t* out);

/* A stored term, read-only (pointers valid until the next pflt_add). */
typedef struct pflt_term_view {
    uint32_t op, sortk, w1, w2, nargs;
    const uint32_t* args;
    int64_t i0, i1;
    const uint32_t* limbs;
    uint32_t nlimbs;
    const char* name;
} pflt_term_view;
int pflt_view(void* store, uint32_t id, pflt_term_view* out);

/* Independence buckets of one query (mythril_amd/smt/independence.py:buckets — the same
 * partition, bucket order and conjunct order; reference: independence_solver.py:38-83):
 * roots = the query's constraints; out_ids gets the flattened conjuncts bucket by bucket
 * (capacity >= their number), out_sizes each bucket's size.  Returns the number of buckets,
 * -1 when a capacity is too small, -2 on an unknown id.  Keys are memoised per term. */
int64_t pflt_buckets(void* store, const uint32_t* roots, size_t n_roots, uint32_t* out_ids, size_t cap_ids,
                     uint32_t* out_sizes, size_t cap_sizes);
/* pflt_buckets over n_queries queries at once (check_sets' batch): query q's constraints are
 * roots[offsets[q] .. offsets[q + 1]); its buckets follow the previous queries' in out_ids /
 * out_sizes and out_counts[q] gets their number.  Returns the total number of buckets, or
 * pflt_buckets' -1 (a capacity too small: retry larger) / -2. */
int64_t pflt_buckets_many(void* store, const uint32_t* roots, const uint64_t* offsets, size_t n_queries,
                          uint32_t* out_ids, size_t cap_ids, uint32_t* out_sizes, size_t cap_sizes,
                          int64_t* out_counts);

/* Host re-check of a bucket witness (csrc/pf_recheck.cpp; mythril_amd/smt/interp.py
 * Witness.ev, bit for bit): var_desc = n_vars x 4 u32 (the result's var_terms descriptors:
 * type, a, b, c) with values n_vars x 8 u32; uf_apps = application term ids in registration
 * order; reads = (array id, index id) pairs, grouped per array in lookup order; registry as
 * for pflt_lower.  out[i] = value of roots[i] (0/1).  Returns 0, or -1 when a term is not
 * evaluable here (the caller re-checks in Python). */
int pflt_recheck(void* store, const uint32_t* var_desc, size_t n_vars, const uint32_t* values,
                 const uint32_t* uf_apps, size_t n_uf, const uint32_t* reads, size_t n_reads,
                 const uint32_t* registry, size_t n_registry, const uint32_t* roots, size_t n_roots,
                 uint8_t* out);

/* ---- batches (the live path's per-call pipeline, mythril_amd/smt/gpu_check.check_sets) ----
 * Parent models: a handle holding values by symbol name and by base-array read, built from
 * explicit values (pflt_parent_new: the par_* layout of pflt_lower) or from the store's
 * recent-value tables (pflt_recent_parent: the newest value of each symbol / read the
 * bucket's dependence keys name — gpu_check._recent_parent; NULL when none is known).  The
 * tables are filled by pflt_note_vars (z3 model values) and pflt_note_result (an accepted
 * bucket witness: gpu_check._note_witness), least-recently-updated first out (recent_size
 * symbols; 1024 arrays of 256 reads). */
void* pflt_parent_new(const char* names, const uint32_t* name_vals, size_t n_names, const uint32_t* reads,
                      const uint32_t* read_vals, size_t n_reads);
void pflt_parent_free(void* parents);
void pflt_parent_info(const void* parents, uint64_t* info); /* n_names, name bytes, value words, n_reads */
void pflt_parent_get(const void* parents, char* names, uint32_t* name_vals, uint32_t* reads, uint32_t* read_vals);
void pflt_recent_clear(void* store);
void pflt_note_vars(void* store, const char* names, const uint32_t* vals, size_t n, size_t recent_size);
void pflt_note_result(void* store, const void* result, const uint32_t* values, size_t recent_size);
void* pflt_recent_parent(void* store, const uint32_t* roots, size_t n_roots);

/* One bucket of a pflt_lower_many call. */
typedef struct pflt_job {
    const uint32_t* roots;  /* the bucket's conjuncts */
    size_t n_roots;
    const void* parents;    /* a parent-model handle or NULL */
    uint32_t flags;         /* PFLT_HINTS | PFLT_PROGRAM */
    uint32_t seed;
} pflt_job;
/* Lower n buckets on n_threads host threads (the store is only read: no pflt_add may run
 * meanwhile).  results[j] is always a handle: pflt_result_status 0, or pflt_lower's rc with
 * the message in pflt_result_error. */
void pflt_lower_many(void* store, const pflt_job* jobs, size_t n, const uint32_t* registry, size_t n_registry,
                     uint32_t n_threads, void** results);
int pflt_result_status(const void* result);
const char* pflt_result_error(const void* result);
int pflt_result_parented(const void* result);
/* Free the program and DAG tables of a result (kept: variables, witness metadata, roots). */
void pflt_result_shrink(void* result);
/* The flat arrays of a pf_batch_create batch (mythril_amd/ir.py Batch) from n results:
 * sizes = total instructions, constants, variables, parent values; then code (x4 u32, word 3
 * = reach_lut[op * lut_w + width]), consts (x8), schema (x4), parents (x8), descs (x8). */
void pflt_pack_sizes(void* const* results, size_t n, uint64_t* sizes);
void pflt_pack_batch(void* const* results, size_t n, const uint32_t* seeds, const uint32_t* reach_lut,
                     uint32_t lut_w, uint32_t* code, uint32_t* consts, uint32_t* schema, uint32_t* parents,
                     uint32_t* descs);
/* pflt_recheck of n results at once on n_threads threads: values = each result's variables
 * x 8 u32, results back to back; status[j] = 1 (every conjunct true), 0 (some false), -1
 * (not evaluable here: re-check in Python). */
void pflt_recheck_many(void* store, void* const* results, size_t n, const uint32_t* values,
                       const uint32_t* registry, size_t n_registry, uint32_t n_threads, int8_t* status);
/* A GPU witness kept for the quick-sat cache (mythril_amd/model_cache.py; replaces the Python
 * interp.Witness.leaf_value walk behind reference mythril/support/model.py:52-58 model.eval):
 * the interpretation of n_parts lowering results (the variable-disjoint buckets of one found
 * set, values back to back as for pflt_recheck_many), with its evaluation memo kept between
 * calls.  reg_serial names the registry blob's state.  NULL on a malformed registry blob. */
void* pflt_witness_new(void* store, void* const* results, size_t n_parts, const uint32_t* values,
                       const uint32_t* registry, size_t n_registry, uint64_t reg_serial);
void pflt_witness_free(void* witness);
/* terms[0..n_terms) under each of n_models witnesses (the store locked by the caller), with
 * the registry's current state (re-parsed by a witness whose reg_serial differs).  slots
 * (optional): the caller's dense number of each term, under which a witness keeps the value
 * (forgotten when slot_epoch changes) so that a term read again is a copy:
 * out_limbs[(m * n_terms + i) * 8 + k] = limb k of the value (masked to the term's width,
 * at most 256 bits; a Bool is 0 / 1), ok[m * n_terms + i] = 1
 * where it evaluated (0: not evaluable natively); the witnesses on n_threads threads. */
void pflt_witness_values(void* const* witnesses, size_t n_models, const uint32_t* terms, size_t n_terms,
                         const uint32_t* slots, uint64_t slot_epoch,
                         const uint32_t* registry, size_t n_registry, uint64_t reg_serial,
                         uint32_t n_threads, uint32_t* out_limbs, uint8_t* ok);

#ifdef __cplusplus
}
#endif
#endif /* PF_LOWER_H */
