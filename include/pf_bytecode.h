/*
 * pf_bytecode.h — the flat register bytecode that carries one Mythril path-constraint
 * set (a conjunction of 256-bit BitVec/Bool DAGs) across the C ABI into the gfx950
 * evaluator.  This header is the single source of truth for opcode numbers, the
 * instruction layout, the variable schema and the candidate-generator contract; the
 * Python host (mythril_amd/ir.py) mirrors it and tests/test_abi.py checks the mirror.
 *
 * Semantics of every opcode are SMT-LIB2 FixedSizeBitVectors (z3's total-division
 * conventions), i.e. what z3's model.eval(expr, model_completion=True) computes for the
 * term shapes built by mythril/laser/smt/{bitvec,bitvec_helper,bool}.py.  The CPU
 * restatement that pins them is oracle/pyoracle.py.
 *
 * Instruction = 4 x uint32:
 *   w0 = op | (width << 8) | (traffic << 18)    width = result width (W ops) or the
 *           | (unit << 21)                      operand width (compare ops), 1..256;
 *                                               traffic = PF_TR_* bits and unit =
 *                                               PF_U_* datapath, both recomputed from
 *                                               the opcode by pf_batch_create
 *   w1 = dst | (a << 8) | (b << 16) | (c << 24) register indices
 *   w2 = aux0, w3 = aux1                        op specific
 *
 * Register classes
 *   W : 256-bit values, PF_NW registers.  A value of width w < 256 is kept
 *       zero-extended (bits >= w are 0) — every op re-masks its result.
 *   B : booleans, PF_NB registers (0/1 per candidate).
 * The conjunction root is an accumulator: PF_ASSERT ands a B register into it.
 */
#ifndef PF_BYTECODE_H
#define PF_BYTECODE_H

#include <stdint.h>

#ifndef PF_NW
#define PF_NW 15          /* usable wide registers (limb-sliced VGPR banks on gfx950) */
#endif
#define PF_W_SINK 15      /* 16th bank slot: write sink of ops without a W result     */
#ifndef PF_NW_NARROW
#define PF_NW_NARROW 7    /* a batch whose programs write only W registers < 7 runs the
                             8-register search kernels (3 waves/SIMD); sink = register 7 */
#endif
/* waves per workgroup of the search kernels (each wave owns its LDS slice, so the
 * workgroup size only sets how finely the CU's LDS and wave slots are handed out) */
#ifndef PF_SEARCH_WG_WAVES
#define PF_SEARCH_WG_WAVES 1
#endif
/* search work queues: PF_EARLY_QUEUES heads per launch (probe / search phase x narrow / wide
 * part: 4 launches), PF_EARLY_QUEUE_STRIDE u32 (128 B, one L2 line) apart, in the batch scratch
 * from byte PF_EARLY_QUEUE_OFF on */
#define PF_EARLY_QUEUES 16
#define PF_EARLY_QUEUE_STRIDE 32
#define PF_EARLY_QUEUE_OFF 512
/* per-launch counters (evals_full, cands_decided, ops, timed-out items): PF_COUNTER_STRIPES
 * lines of 4 u64, 128 B apart, after the queue heads; a wave adds its non-zero totals
 * into line wave % PF_COUNTER_STRIPES and the host sums the lines (one line took every wave's
 * atomics in series: ~60 us at the end of a 4,096-wave grid) */
#define PF_COUNTER_STRIPES 16
#define PF_COUNTER_OFF (PF_EARLY_QUEUE_OFF + 4 * PF_EARLY_QUEUES * PF_EARLY_QUEUE_STRIDE * 4)
#define PF_SCRATCH_BYTES (PF_COUNTER_OFF + PF_COUNTER_STRIPES * 128)
#define PF_NB 32          /* bool registers                                          */
#define PF_LIMBS 8        /* 8 x 32-bit limbs = 256 bits, little-endian limb order   */
#define PF_MAX_WIDTH 256
#define PF_MAX_SPILL 64   /* spill slots per lane (8 x u32 each, private scratch)       */

/* ---- opcodes ------------------------------------------------------------------ */
enum pf_opcode {
    PF_END = 0,
    /* W results */
    PF_W_CONST = 1,   /* dst <- const[aux0]                                            */
    PF_W_VAR = 2,     /* dst <- candidate value of variable aux0                       */
    PF_W_MOV = 3,     /* dst <- a masked to width (zero_extend / no-op copy)           */
    PF_W_ADD = 4,     /* bvadd                                                         */
    PF_W_SUB = 5,     /* bvsub                                                         */
    PF_W_MUL = 6,     /* bvmul                                                         */
    PF_W_UDIV = 7,    /* bvudiv   (x / 0 = 2^w - 1)                                    */
    PF_W_UREM = 8,    /* bvurem   (x % 0 = x)                                          */
    PF_W_SDIV = 9,    /* bvsdiv   (x / 0 = x <s 0 ? 1 : 2^w - 1)                       */
    PF_W_SREM = 10,   /* bvsrem   (sign of dividend; x % 0 = x)                        */
    PF_W_SMOD = 11,   /* bvsmod   (sign of divisor;  x mod 0 = x)                      */
    PF_W_AND = 12,
    PF_W_OR = 13,
    PF_W_XOR = 14,
    PF_W_NOT = 15,    /* bvnot a                                                       */
    PF_W_NEG = 16,    /* bvneg a                                                       */
    PF_W_SHL = 17,    /* bvshl  (b >= w -> 0)                                          */
    PF_W_LSHR = 18,   /* bvlshr (b >= w -> 0)                                          */
    PF_W_ASHR = 19,   /* bvashr (b >= w -> sign fill)                                  */
    PF_W_EXP = 20,    /* a ** b mod 2^w (EVM EXP; 256-step square-and-multiply)        */
    PF_W_EXTRACT = 21,/* dst <- (a >> aux0) masked to width  ((_ extract hi lo), width = hi-lo+1) */
    PF_W_CONCAT = 22, /* dst <- (a << aux0) | b   where aux0 = width(b)               */
    PF_W_SEXT = 23,   /* dst <- sign_extend(a) from aux0 bits to width                 */
    PF_W_ITE = 24,    /* dst <- B[c] ? a : b                                           */
    PF_W_HASH = 25,   /* dst <- H_aux0(a): keyed 256-bit mix of a (two Philox4x32-10
                         blocks, see below) — the by-construction interpretation of
                         uninterpreted functions (keccak256_<n>, unknown UFs)          */
    PF_W_SPILL = 26,  /* spill slot aux0 <- W a      (register pressure; no W result)       */
    PF_W_FILL = 27,   /* dst <- spill slot aux0                                          */
    /* B results */
    PF_B_CONST = 40,  /* dst <- aux0 & 1                                               */
    PF_B_VAR = 41,    /* dst <- candidate value of Bool variable aux0                  */
    PF_B_EQ = 42,     /* W a == W b                                                    */
    PF_B_ULT = 43,
    PF_B_ULE = 44,
    PF_B_SLT = 45,    /* signed at width w                                             */
    PF_B_SLE = 46,
    PF_B_AND = 47,    /* B a & B b                                                     */
    PF_B_OR = 48,
    PF_B_XOR = 49,
    PF_B_NOT = 50,
    PF_B_ITE = 51,    /* B[c] ? B a : B b                                              */
    PF_B_UADD_NOOVF = 52, /* a + b < 2^w   (z3 BVAddNoOverflow(a, b, False))          */
    PF_B_UMUL_NOOVF = 53, /* a * b < 2^w   (z3 BVMulNoOverflow(a, b, False), bvumul_noovfl) */
    PF_B_FILL = 54,   /* dst <- limb 0 of spill slot aux0 (a spilled B value)              */
    PF_B_SPILL = 55,  /* limb 0 of spill slot aux0 <- B a                                  */
    PF_ASSERT = 60,   /* root &= B a; with PF_FLAG_SHORTCIRCUIT a wave whose lanes are all
                         false stops evaluating the set here                           */
    PF_NUM_OPCODES = 64
};

/* w0 bit 24 on a compare or bool op: also PF_ASSERT its B result.  Set only by
 * pf_batch_create's peephole (an ASSERT of the B register the previous instruction wrote),
 * never by the host lowering, whose programs the oracles evaluate as written. */
#define PF_I_ASSERT (1u << 24)

/* w0 bits 25 / 26: operand a / b is the set's constant const[a] / const[b] (the 8-bit
 * register field holds the constant index) instead of a W register.  Set only by
 * pf_batch_create's constant-operand peephole, which deletes a W_CONST whose every reader
 * (up to the next write of its register) can take the constant this way — one dispatched
 * instruction and one register write-back less per constant; the kernel reads the
 * constant with a scalar load where it would have copied the register.  Never set by the
 * host lowering (the oracles evaluate the program as lowered). */
#define PF_I_KA (1u << 25)
#define PF_I_KB (1u << 26)

/* w0 bits 27 / 28: operand a / b is the W result of the instruction right before (its
 * traffic bit cleared: no register read).  Set only by pf_batch_create's forwarding
 * peephole, which also clears the previous instruction's PF_TR_WW when nothing else reads
 * that result before its register's next write (no write-back).  Never set by the host
 * lowering. */
#define PF_I_FA (1u << 27)
#define PF_I_FB (1u << 28)

/* aux of a W/B SPILL or FILL: PF_SPILL_LDS | e keeps the value in LDS entry e (1..3) of the
 * lane's EXP window table instead of private scratch slot aux.  Set only by pf_batch_create's
 * spill peephole, for a spill whose fills all come before the next W_EXP (which rewrites
 * entries 1..3) and, for entry 1, the next B_UMUL_NOOVF (which parks an operand there):
 * scratch traffic is dirty L2 lines of every resident wave. */
#define PF_SPILL_LDS 0x100u

/* operand traffic bits (w0 >> 18): reads W[a], reads W[b], writes W[d] */
#define PF_TR_RA 1u
#define PF_TR_RB 2u
#define PF_TR_WW 4u

/* datapath unit of each opcode (w0 >> 21): the kernel dispatches on it first */
enum pf_unit {
    PF_U_ALU = 0,   /* W add/sub/logic/const/mov/not/neg/sext/ite/hash */
    PF_U_MUL = 1,   /* MUL, EXP                                        */
    PF_U_DIV = 2,   /* UDIV..SMOD, UMUL_NOOVF                          */
    PF_U_SHIFT = 3, /* SHL/LSHR/ASHR/EXTRACT/CONCAT                    */
    PF_U_GEN = 4,   /* W_VAR, B_VAR (candidate generator)             */
    PF_U_CMP = 5,   /* B_EQ..B_SLE, UADD_NOOVF                         */
    PF_U_BOOL = 6,  /* B_CONST, B_AND..B_ITE, ASSERT                   */
    PF_U_END = 7
};

#ifdef __cplusplus
static inline uint32_t pf_op_unit(uint32_t op) {
    if (op == PF_W_MUL || op == PF_W_EXP) return PF_U_MUL;
    if ((op >= PF_W_UDIV && op <= PF_W_SMOD) || op == PF_B_UMUL_NOOVF) return PF_U_DIV;
    if ((op >= PF_W_SHL && op <= PF_W_ASHR) || op == PF_W_EXTRACT || op == PF_W_CONCAT) return PF_U_SHIFT;
    if (op == PF_W_VAR || op == PF_B_VAR) return PF_U_GEN;
    if ((op >= PF_B_EQ && op <= PF_B_SLE) || op == PF_B_UADD_NOOVF) return PF_U_CMP;
    if (op == PF_B_CONST || (op >= PF_B_AND && op <= PF_B_ITE) || op == PF_ASSERT || op == PF_B_FILL ||
        op == PF_B_SPILL)
        return PF_U_BOOL;
    if (op == PF_END || op >= PF_NUM_OPCODES) return PF_U_END;
    return PF_U_ALU;
}

/* traffic of each opcode (host side; the kernel reads the bits from the instruction) */
static inline uint32_t pf_op_traffic(uint32_t op) {
    const uint32_t rab_w = PF_TR_RA | PF_TR_RB | PF_TR_WW, ra_w = PF_TR_RA | PF_TR_WW;
    if (op == PF_W_CONST || op == PF_W_VAR || op == PF_W_FILL) return PF_TR_WW;
    if (op == PF_W_SPILL) return PF_TR_RA;
    if (op == PF_W_MOV || op == PF_W_NOT || op == PF_W_NEG || op == PF_W_EXTRACT ||
        op == PF_W_SEXT || op == PF_W_HASH)
        return ra_w;
    if ((op >= PF_W_ADD && op <= PF_W_SMOD) || (op >= PF_W_AND && op <= PF_W_XOR) ||
        (op >= PF_W_SHL && op <= PF_W_EXP) || op == PF_W_CONCAT || op == PF_W_ITE)
        return rab_w;
    if ((op >= PF_B_EQ && op <= PF_B_SLE) || op == PF_B_UADD_NOOVF || op == PF_B_UMUL_NOOVF)
        return PF_TR_RA | PF_TR_RB;
    return 0u;
}
#endif

/* B results are the opcodes PF_B_CONST..PF_B_FILL (a B destination register is written) */
#define PF_OP_WRITES_B(op) ((op) >= PF_B_CONST && (op) <= PF_B_FILL)

/* ---- variable schema (4 x uint32 per variable) -------------------------------- */
/* s0 = kind | (width << 8); s1 = hint0; s2 = hint1; s3 = parent slot (or PF_NO_PARENT) */
enum pf_var_kind {
    PF_VK_GENERIC = 0, /* plain BitVec symbol                                          */
    PF_VK_ACTOR = 1,   /* sender_*: const[hint0 .. hint0+hint1) are the actor addresses */
    PF_VK_KECCAK = 2,  /* keccak UF output slot: const[hint0] + 64*k, k < 2^117         */
    PF_VK_SMALL = 3,   /* sizes: uniform in [0, hint0], or ABI-aligned (4 + 32 k)       */
    PF_VK_BOOL = 4,    /* free Bool symbol                                              */
    PF_VK_CDBYTE = 5,  /* calldata byte at a constant offset: hint0 = its bit position in
                          its big-endian ABI word (selector or 32-byte argument, bits
                          0..7) | K << 8 | start << 20 (the set's word constants are
                          const[start .. start+K), 12 bits each; K = 0: the whole pool),
                          hint1 = the word's id (bytes of one word share it)            */
    PF_VK_VALUE = 6    /* call values (call_value<tx>): 0 in half the candidates (every
                          non-payable function requires it), else PF_VK_GENERIC        */
};
#define PF_NO_PARENT 0xffffffffu

/* ---- per-set descriptor (8 x uint32) ------------------------------------------- */
typedef struct pf_set_desc {
    uint32_t code_off;   /* first instruction (in 16-byte instructions)               */
    uint32_t n_ins;      /* instructions including the final PF_END                   */
    uint32_t const_off;  /* first constant (in 32-byte constants)                     */
    uint32_t n_const;
    uint32_t var_off;    /* first schema entry                                        */
    uint32_t n_vars;
    uint32_t seed;       /* per-set candidate seed (independent of batch position)    */
    uint32_t parent_off; /* first parent value (32-byte each) or PF_NO_PARENT          */
} pf_set_desc;

/* ---- candidate generator contract ---------------------------------------------- */
/* Candidate c of a set with seed S and global seed G assigns variable v the value
 * produced from three Philox4x32-10 blocks with key (G_lo ^ S, G_hi) and counters
 * (c, v, 0, 0), (c, v, 1, 0), (c, v, 2, 0): r[0..7] (value bits) and m[0..3]
 * (strategy bits).  Strategies (m[0] & 15) for PF_VK_GENERIC, width w:
 *    0..4  uniform r masked to w
 *    5..8  boundary table[m[1] % 12] with k = m[2] % w:
 *          {0, 1, 2, 3, 2^w-1, 2^w-2, 2^(w-1), 2^(w-1)-1, 2^k, 2^k-1, 2^k+1, 2^160-1}
 *    9..11 harvested constant const[m[1] % n_const] + {0,+1,-1}[m[2] % 3]  (uniform if n_const == 0)
 *    12,13 parent value (bit m[2] % w flipped when (m[1] & 3) == 0), else r[0] & 0xff
 *    14,15 small: r[0] & (2^(1 + m[1] % 16) - 1)
 * Candidate 0 is the exact parent value for every variable that has one.
 * Neighbourhood candidates: for an odd candidate c, a variable with a parent value keeps
 * it exactly when (m[3] & ((4 << ((c >> 1) & 3)) - 1)) != 0 — probability 3/4, 7/8, 15/16
 * or 31/32 by (c >> 1) & 3 — and is generated by its kind's rule below otherwise, so half
 * of the candidates are few-variable mutations of the parent (hint) model.
 * PF_VK_ACTOR: m[1] % 4 < hint1 -> const[hint0 + m[1] % 4], else generic.
 * PF_VK_KECCAK: const[hint0] + ((r[0..3] & (2^117 - 1)) << 6).
 * PF_VK_SMALL: if (m[0] & 16) and 4 <= hint0 < 2^32 - 1, the ABI-aligned size
 *   4 + 32 (r[1] % ((hint0 - 4) / 32 + 1)) (selector + whole argument words, what the ABI
 *   size checks compare against), else r[0] % (hint0 + 1).   PF_VK_BOOL: r[0] & 1.
 * PF_VK_VALUE: 0 if (m[0] & 16), else the PF_VK_GENERIC rules.
 * PF_VK_CDBYTE (LASER's calldata bytes, state/calldata.py:233-246): one hash per
 *   (candidate, ABI word) u = mix32(cand ^ key0 ^ hint1 * 0x9E3779B9) — so every byte of
 *   one word takes the same decision; with s = hint0 & 0xff, K = (hint0 >> 8) & 0xfff and
 *   start = hint0 >> 20 (K = 0: start = 0, K = n_const), if (u & 1) and K > 0 the byte is
 *   ((const[start + (u >> 1) % K] + {0, +1, -1, 0}[u >> 30]) mod 2^256 >> s) & 0xff: a
 *   whole selector or argument word spelled from one harvested constant or its neighbour
 *   (a dispatcher's `selector == 0xa9059cbb` needs all four bytes at once, an argument
 *   bound `x < c` the word c - 1); else the PF_VK_GENERIC rules at width 8.
 *   mix32(x): x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16.
 * All results are masked to the variable's width.                                  */
#define PF_MIX_M1 0x7feb352du
#define PF_MIX_M2 0x846ca68bu
#define PF_CDWORD_MUL 0x9E3779B9u
/* PF_W_HASH with salt s of value x (limbs x0..x7):
 *   h = Philox(ctr=(x0,x1,x2,x3), key=(s, 0x5BD1E995)),
 *   g = Philox(ctr=(x4^h0, x5^h1, x6^h2, x7^h3), key=(s, 0x27D4EB2F)),
 *   H = limbs (h0,h1,h2,h3,g0,g1,g2,g3) masked to width.                              */
#define PF_HASH_K1A 0x5BD1E995u
#define PF_HASH_K1B 0x27D4EB2Fu
#define PF_PHILOX_M0 0xD2511F53u
#define PF_PHILOX_M1 0xCD9E8D57u
#define PF_PHILOX_W0 0x9E3779B9u
#define PF_PHILOX_W1 0xBB67AE85u

/* flags for pf_check_batch */
#define PF_FLAG_SHORTCIRCUIT 1u  /* stop a wave's set evaluation once all its lanes are false */
#define PF_FLAG_EARLY_EXIT 2u    /* stop a set once any candidate satisfies it             */
#define PF_FLAG_COUNT_OPS 4u     /* accumulate algorithmic int32-op counts                  */
#define PF_FLAG_NO_PROBE 8u      /* no candidate-0 probe launch before an early-exit search:  \
                                    the caller knows some set's candidate 0 misses (its host \
                                    hint model leaves a root false); answers are unchanged    */

#endif /* PF_BYTECODE_H */
