/*
 * pathfeas.h — C ABI of the MI355X batched path-feasibility engine (libpathfeas.so).
 *
 * Plain pointers and sizes, caller-owned buffers, int status (0 ok, < 0 error, message in
 * pf_last_error()), no C++ exceptions across the boundary.  Every entry point takes an
 * internal mutex and calls hipSetDevice, because Mythril's query funnel enters from a fresh
 * ThreadPool(1) worker thread on every query (mythril/support/model.py:99-117).
 *
 * Reference interfaces each entry point replaces (the reference binds libz3 through z3py's
 * ctypes, so these are the calls a ctypes binding in mythril would make instead):
 *   pf_check_batch        z3 Optimize.check() for objective-free queries
 *                         (mythril/support/model.py:37-59 solver_worker, :99-117) and the
 *                         quick-sat model scan (mythril/support/support_utils.py:57-71)
 *   pf_materialize        z3 Optimize.model() (mythril/laser/smt/solver/solver.py:99-108) —
 *                         turns a witness index into concrete variable values
 *   pf_eval_assignments   z3 ModelRef.eval(expr, model_completion=True) over a batch of
 *                         explicit models (mythril/support/support_utils.py:63-67)
 *   pf_keccak256_batch    eth_hash keccak via support_utils.sha3 (support_utils.py:93-101) as
 *                         called by KeccakFunctionManager.find_concrete_keccak
 *                         (keccak_function_manager.py:57-69) and get_code_hash (:74-90)
 *   pf_check_batches      the same over several devices of one process (one batch each):
 *                         the tx-boundary batch of svm.py:266-286 split across a node
 * The *_dev variants take device pointers (HBM-resident inputs, e.g. torch tensors) and an
 * optional hipStream_t (NULL = the library stream of the batch's device).
 */
#ifndef PATHFEAS_H
#define PATHFEAS_H

#include <stddef.h>
#include <stdint.h>

#include "pf_bytecode.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pf_stats {
    uint64_t evals_full;     /* candidate lanes that evaluated the whole program            */
    uint64_t cands_decided;  /* candidate lanes whose verdict was decided (incl. short-circuit) */
    uint64_t ops;            /* algorithmic int32 ops executed (PF_FLAG_COUNT_OPS only)      */
    uint64_t n_sat;          /* sets with a witness                                          */
    float kernel_ms;         /* device time of the check kernel (HIP events, its stream)     */
    uint32_t timed_out;      /* 1 if the timeout_ms deadline cut any wave's search: the
                                NOT_FOUND verdicts are then incomplete                      */
} pf_stats;

/* ---- lifetime ---------------------------------------------------------------------- */
/* Initialise the devices of device_mask (bit d = HIP device d; all must be gfx950): one
 * library stream per device.  Callable again to add devices.  The lowest initialised device
 * is the default one (pf_batch_create, Keccak).  One process can drive every GPU of a node
 * this way (Mythril's analysis is one process); one process per GPU passes one bit.      */
int pf_init(uint64_t device_mask);
/* Add one execution context per entry of devices[]: its own library stream, device-block pool
 * and events on that HIP device — the same device may appear several times.  ctx_out[i]
 * receives the context's id (>= PF_CONTEXT_BASE), usable wherever an entry point takes a
 * device (pf_batch_create_on; batches remember it).  A node's split
 * (pf_check_batches over one batch per context) can so run with two contexts on one GPU:
 * the same code path as two GPUs, each context's launches on its own stream.           */
#define PF_CONTEXT_BASE 64
int pf_init_contexts(const int32_t* devices, size_t n, int32_t* ctx_out);
int pf_shutdown(void);
const char* pf_last_error(void);
int pf_version(void);               /* ABI version                                         */
int pf_device_count(void);

/* ---- constraint-set batches (uploaded once, resident in HBM) --------------------------- */
/* code: n_ins x 4 u32; consts: n_const x 8 u32; schema: n_vars x 4 u32;
 * parents: n_parents x 8 u32; descs: n_sets x pf_set_desc.  Instruction aux1 carries the
 * algorithmic op cost used by PF_FLAG_COUNT_OPS.                                           */
int pf_batch_create(const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                    const uint32_t* schema, size_t n_vars, const uint32_t* parents,
                    size_t n_parents, const pf_set_desc* descs, size_t n_sets,
                    uint64_t* handle_out);
/* same, on a given initialised device (-1 = the default device)                            */
int pf_batch_create_on(int device, const uint32_t* code, size_t n_ins, const uint32_t* consts,
                       size_t n_const, const uint32_t* schema, size_t n_vars,
                       const uint32_t* parents, size_t n_parents, const pf_set_desc* descs,
                       size_t n_sets, uint64_t* handle_out);

/* Host only (no device call; for tests): the program pf_batch_create puts on the device for
 * this batch — traffic/unit bits recomputed, then its peepholes (an ASSERT folded into the
 * compare before it, PF_I_ASSERT; a W_CONST folded into its readers, PF_I_KA / PF_I_KB, only
 * when its constant fits the W_CONST's width — consts may be NULL: all taken to fit).
 * code_out: room for n_ins instructions; descs_out: n_sets entries (code ranges shifted). */
int pf_device_program(const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                      const pf_set_desc* descs, size_t n_sets, uint32_t* code_out, size_t* n_ins_out,
                      pf_set_desc* descs_out);
int pf_batch_free(uint64_t handle);

/* Generate candidates [0, budget) on device for every set and search for a witness.
 * found_out[s]  = smallest satisfying candidate index found, or 0xFFFFFFFF
 *                 (with PF_FLAG_EARLY_EXIT the smallest one is still guaranteed: a wave
 *                  stops only once a witness below its own candidates exists)
 * sat_bitmap_out (optional) = bit s set iff found_out[s] != 0xFFFFFFFF
 * timeout_ms = 0: no device-side deadline.                                                 */
int pf_check_batch(uint64_t handle, uint64_t global_seed, uint32_t budget, uint32_t flags,
                   uint32_t timeout_ms, uint32_t* found_out, uint8_t* sat_bitmap_out,
                   pf_stats* stats);
/* Search n batches (typically one per device) at once: every launch is enqueued on its
 * device's stream before any result is read, so the devices run concurrently; found_out
 * receives the verdicts concatenated in handle order; stats (optional) has n entries.    */
int pf_check_batches(const uint64_t* handles, size_t n, uint64_t global_seed, uint32_t budget,
                     uint32_t flags, uint32_t timeout_ms, uint32_t* found_out, pf_stats* stats);
/* same, result left in a device buffer of n_sets u32 (d_found), no host copy of results   */
int pf_check_batch_dev(uint64_t handle, uint64_t global_seed, uint32_t budget, uint32_t flags,
                       uint32_t timeout_ms, uint32_t* d_found, pf_stats* stats, void* stream);

/* Regenerate the full assignment of candidate cand_ids[i] of set set_ids[i]: writes
 * n_vars(set) x 8 u32 per request, concatenated in request order.                        */
int pf_materialize(uint64_t handle, uint64_t global_seed, const uint32_t* set_ids,
                   const uint32_t* cand_ids, size_t n, uint32_t* values_out);

/* Evaluate set `set` on n_cand explicit assignments, SoA limbs [var][limb][cand].          */
int pf_eval_assignments(uint64_t handle, uint32_t set, const uint32_t* soa, uint32_t n_cand,
                        uint8_t* sat_out);
/* One program evaluated over explicit assignments in one call (no batch object): validated
 * and transformed exactly as pf_batch_create does, uploaded with its assignments
 * ([var][limb][cand] u32, like pf_eval_assignments) through pinned staging, one launch,
 * verdicts copied back.  Replaces z3 ModelRef.eval(C, model_completion=True) over the <= 100
 * cached models of check_quick_sat (mythril/support/support_utils.py:57-71), one lane per
 * model (the GPU-resident ModelCache, mythril_amd/model_cache.py). */
int pf_eval_program(int device, const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                    const uint32_t* schema, size_t n_vars, const uint32_t* soa, uint32_t n_cand,
                    uint8_t* sat_out);
/* Several programs (n_sets descriptors over code / consts / schema, as for pf_batch_create)
 * over one call's explicit assignments: set s reads its variables from SoA rows
 * descs[s].var_off .. + n_vars(s) ([var][limb][cand] u32 over all sets' variables); one wave
 * per (set, 64 candidates), all in one launch; sat_out[s * n_cand + cand].  The quick-sat of
 * the GPU-resident ModelCache with the query's conjuncts split into groups (the same
 * reference loop as pf_eval_program: support_utils.py:57-71), the groups side by side. */
int pf_eval_programs(int device, const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                     const uint32_t* schema, size_t n_vars, const pf_set_desc* descs, size_t n_sets,
                     const uint32_t* soa, uint32_t n_cand, uint8_t* sat_out);
int pf_eval_assignments_dev(uint64_t handle, uint32_t set, const uint32_t* d_soa,
                            uint32_t n_cand, uint8_t* d_sat_out, void* stream);

/* Keccak-256 (original padding) of n messages data[offsets[i] .. offsets[i+1]).           */
int pf_keccak256_batch(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32);
/* device variant for fixed-length messages: msg i = d_data[i*len .. (i+1)*len)              */
int pf_keccak256_fixed_dev(const uint8_t* d_data, uint32_t len, size_t n, uint8_t* d_out32,
                           float* kernel_ms, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PATHFEAS_H */
