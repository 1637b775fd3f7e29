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

#ifdef __cplusplus
}
#endif
#endif /* PF_LOWER_H */
