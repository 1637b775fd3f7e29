"""Test tooling: straight-line EVM programs (the reference's VMTests fixtures) -> constraint DAGs.

Maps each arithmetic opcode onto the bit-vector terms Mythril's LASER builds for it
(mythril/laser/ethereum/instructions.py: ADD/MUL/SUB :436-480, DIV/SDIV/MOD/SMOD with the
concrete ==0 guard :506-552, SHL/SHR/SAR :554-579, EXP :625-639 (concrete operands),
SIGNEXTEND :641-660, LT/GT/SLT/SGT/EQ/ISZERO :700-790, AND/OR/XOR/NOT/BYTE :330-430),
then asserts ``storage[key] == expected`` for every post-state slot.  Evaluated under the
(empty) assignment, the conjunction must be true on the oracle and on the GPU.
Programs using ADDMOD/MULMOD (257/512-bit intermediates) are skipped.
"""

from __future__ import annotations

from mythril_amd import ir
from mythril_amd.lower import Dag

W = 256


class Unsupported(Exception):
    pass


def _bool_to_word(dag, b):
    return dag.op(ir.W_ITE, W, b, dag.const(1, W), dag.const(0, W))


def build(code_hex: str, storage: dict) -> Dag:
    code = bytes.fromhex(code_hex[2:])
    dag = Dag()
    st = []
    sto = {}
    i = 0
    zero = dag.const(0, W)

    def const_of(n):
        nd = dag.nodes[n]
        if nd.kind != "const":
            raise Unsupported("non-constant operand where a constant is required")
        return nd.aux

    while i < len(code):
        o = code[i]
        if 0x60 <= o <= 0x7F:
            n = o - 0x5F
            st.append(dag.const(int.from_bytes(code[i + 1:i + 1 + n].ljust(n, b"\0"), "big"), W))
            i += n + 1
            continue
        i += 1
        if o == 0x00:
            break
        if 0x80 <= o <= 0x8F:
            st.append(st[-(o - 0x7F)])
            continue
        if 0x90 <= o <= 0x9F:
            k = o - 0x8F
            st[-1], st[-1 - k] = st[-1 - k], st[-1]
            continue
        if o == 0x50:
            st.pop()
            continue
        if o == 0x55:
            key, val = st.pop(), st.pop()
            sto[const_of(key)] = val
            continue
        if o in (0x08, 0x09):
            raise Unsupported("ADDMOD/MULMOD")
        if o in (0x15, 0x19):  # ISZERO, NOT
            a = st.pop()
            if o == 0x15:
                st.append(_bool_to_word(dag, dag.op(ir.B_EQ, W, a, zero)))
            else:
                st.append(dag.op(ir.W_NOT, W, a))
            continue
        a, b = st.pop(), st.pop()
        if o == 0x01:
            r = dag.op(ir.W_ADD, W, a, b)
        elif o == 0x02:
            r = dag.op(ir.W_MUL, W, a, b)
        elif o == 0x03:
            r = dag.op(ir.W_SUB, W, a, b)
        elif o in (0x04, 0x05, 0x06, 0x07):
            opc = {0x04: ir.W_UDIV, 0x05: ir.W_SDIV, 0x06: ir.W_UREM, 0x07: ir.W_SREM}[o]
            r = dag.op(ir.W_ITE, W, dag.op(ir.B_EQ, W, b, zero), zero, dag.op(opc, W, a, b))
        elif o == 0x0A:
            r = dag.op(ir.W_EXP, W, a, b)
        elif o == 0x0B:  # SIGNEXTEND(b=a(byte index), x=b)
            k = const_of(a)
            if k >= 31:
                r = b
            else:
                nb = 8 * (k + 1)
                r = dag.op(ir.W_SEXT, W, dag.op(ir.W_EXTRACT, nb, b, aux=0), aux=nb)
        elif o in (0x10, 0x11, 0x12, 0x13, 0x14):
            if o == 0x10:
                c = dag.op(ir.B_ULT, W, a, b)
            elif o == 0x11:
                c = dag.op(ir.B_ULT, W, b, a)
            elif o == 0x12:
                c = dag.op(ir.B_SLT, W, a, b)
            elif o == 0x13:
                c = dag.op(ir.B_SLT, W, b, a)
            else:
                c = dag.op(ir.B_EQ, W, a, b)
            r = _bool_to_word(dag, c)
        elif o == 0x16:
            r = dag.op(ir.W_AND, W, a, b)
        elif o == 0x17:
            r = dag.op(ir.W_OR, W, a, b)
        elif o == 0x18:
            r = dag.op(ir.W_XOR, W, a, b)
        elif o == 0x1A:  # BYTE(i=a, x=b)
            k = const_of(a)
            if k >= 32:
                r = zero
            else:
                r = dag.op(ir.W_MOV, W, dag.op(ir.W_EXTRACT, 8, b, aux=248 - 8 * k))
        elif o == 0x1B:  # SHL(shift=a, value=b)
            r = dag.op(ir.W_SHL, W, b, a)
        elif o == 0x1C:
            r = dag.op(ir.W_LSHR, W, b, a)
        elif o == 0x1D:
            r = dag.op(ir.W_ASHR, W, b, a)
        else:
            raise Unsupported(hex(o))
        st.append(r)
    for k, v in storage.items():
        k = int(k, 16)
        expected = int(v, 16)
        got = sto.get(k, zero)
        dag.assert_(dag.op(ir.B_EQ, W, got, dag.const(expected, W)))
    present = {int(k, 16) for k in storage}
    for k, node in sto.items():
        if k not in present:
            dag.assert_(dag.op(ir.B_EQ, W, node, zero))  # slot written with 0 is absent from post
    return dag
