"""CPU restatement of the reference GKR driver around the sum-check hot path
(SURVEY.md 8(f2)): gkr/src/gkr_circuit.rs and gkr/src/gkr_protocol.rs.

TEST INFRASTRUCTURE ONLY (the oracle for tests/ and smoke()). It follows the
reference literally — dense add_i / mul_i tables of 2^n_bits entries
(gkr_circuit.rs:39-104), multi-partial evaluation, scale and add
(gkr_protocol.rs:243-292) — so it only runs small circuits. The library builds
the same folded tables sparsely on the GPU.

The reference's input-layer step commits to the input MLE with KZG and random
taus (gkr_protocol.rs:92-118, row f3); here the input layer's two claimed
evaluations (which KZG::open returns: input_poly.evaluate(r_b / r_c)) are
output directly and the verifier recomputes them from the inputs.
"""
from __future__ import annotations

from pyoracle import (MODULI, Transcript, evaluate, fq_vec_to_bytes, gkr_prove, gkr_verify, partial_evaluate,
                      tensor_add_mul)

ADD, MUL = "add", "mul"


def op_apply(p: int, op: str, a: int, b: int) -> int:  # multilinear_polynomial_evaluation.rs:11-17
    return (a + b) % p if op == ADD else (a * b) % p


def circuit_evaluate(p: int, structure: list[list[str]], inputs: list[int]) -> list[list[int]]:  # gkr_circuit.rs:127-143
    """Layers input -> output; gate i of a layer takes (in[2i], in[2i+1]) (chunks_exact(2)
    zipped with the gates: gates without a pair keep their initial output op(0, 0))."""
    result, cur = [], list(inputs)
    for ops in structure:
        outs = [op_apply(p, op, 0, 0) for op in ops]  # Gate::new(0, 0, op) :119
        for i, op in enumerate(ops):
            if 2 * i + 1 < len(cur):
                outs[i] = op_apply(p, op, cur[2 * i], cur[2 * i + 1])
        result.append(outs)
        cur = outs
    return result


def bits_for_gates(n_gates: int) -> int:  # gkr_circuit.rs:54-65
    if n_gates <= 0:
        raise ValueError("There must be at least one gate in the layer.")
    if n_gates == 1:
        return 3
    lg = n_gates.bit_length() - 1
    return lg + 2 * (lg + 1)


def gate_to_bits(n_gates: int) -> list[int]:  # gkr_circuit.rs:67-104
    lg = n_gates.bit_length() - 1
    out = []
    for idx in range(n_gates):
        segs = [(idx, 1), (2 * idx, 1), (2 * idx + 1, 1)] if n_gates == 1 else \
            [(idx, lg), (2 * idx, lg + 1), (2 * idx + 1, lg + 1)]
        v = 0
        for value, width in segs:
            v = (v << width) | value
        out.append(v)
    return out


def get_add_mul_i(ops: list[str], op: str) -> list[int]:  # gkr_circuit.rs:39-52
    table = [0] * (1 << bits_for_gates(len(ops)))
    for v, g in zip(gate_to_bits(len(ops)), ops):
        if g == op:
            table[v] = 1
    return table


def multi_partial_evaluate(p: int, evals: list[int], values: list[int]) -> list[int]:  # :65-77
    if len(values) > len(evals).bit_length() - 1:
        raise ValueError("Invalid number of values")
    cur = list(evals)
    for v in values:
        cur = partial_evaluate(p, cur, 0, v)
    return cur


def get_fbc_poly(p: int, r0: int, ops: list[str], w_b: list[int], w_c: list[int]):  # gkr_protocol.rs:243-263
    add_i = partial_evaluate(p, get_add_mul_i(ops, ADD), 0, r0)
    mul_i = partial_evaluate(p, get_add_mul_i(ops, MUL), 0, r0)
    return [add_i, tensor_add_mul(p, w_b, w_c, "add"), mul_i, tensor_add_mul(p, w_b, w_c, "mul")]


def get_folded_fbc_poly(p: int, ops: list[str], w_b, w_c, r_b, r_c, alpha: int, beta: int):  # :265-292
    tabs = []
    for op in (ADD, MUL):
        t = get_add_mul_i(ops, op)
        a = multi_partial_evaluate(p, t, r_b)
        c = multi_partial_evaluate(p, t, r_c)
        tabs.append([(alpha * x + beta * y) % p for x, y in zip(a, c)])
    return [tabs[0], tensor_add_mul(p, w_b, w_c, "add"), tabs[1], tensor_add_mul(p, w_b, w_c, "mul")]


def initiate_protocol(p: int, t: Transcript, output_poly: list[int]):  # gkr_protocol.rs:229-241
    t.append(fq_vec_to_bytes(output_poly))
    r = t.get_random_challenge()
    m0 = evaluate(p, output_poly, [r])
    t.append(fq_vec_to_bytes([m0]))
    return m0, r


def prove(field: int, structure: list[list[str]], inputs: list[int]) -> dict:  # gkr_protocol.rs:31-126
    p = MODULI[field]
    t = Transcript(field)
    evals = circuit_evaluate(p, structure, inputs)
    w0 = list(evals[-1])
    if len(w0) == 1:
        w0.append(0)
    claimed, r0 = initiate_protocol(p, t, w0)
    layers = list(reversed(structure))
    evals = list(reversed(evals))
    n = len(layers)
    polys, claims = [], []
    rb = rc = []
    alpha = beta = 0
    for idx, ops in enumerate(layers):
        w = list(inputs) if idx == n - 1 else list(evals[idx + 1])
        tabs = get_fbc_poly(p, r0, ops, w, w) if idx == 0 else get_folded_fbc_poly(p, ops, w, w, rb, rc, alpha, beta)
        rp, _, chal = gkr_prove(field, claimed, tabs, t)
        polys.append(rp)
        mid = len(chal) // 2
        rb, rc = chal[:mid], chal[mid:]
        o1, o2 = evaluate(p, w, rb), evaluate(p, w, rc)
        if idx < n - 1:
            t.append(fq_vec_to_bytes([o1]))
            alpha = t.get_random_challenge()
            t.append(fq_vec_to_bytes([o2]))
            beta = t.get_random_challenge()
            claimed = (alpha * o1 + beta * o2) % p
            claims.append((o1, o2))
        else:
            input_evals = (o1, o2)  # what KZG::open returns for r_b / r_c (:106-111)
    return {"output_poly": w0, "proof_polynomials": polys, "claimed_evaluations": claims,
            "input_evaluations": input_evals, "final_rb": rb, "final_rc": rc}


def verify(field: int, proof: dict, structure: list[list[str]], inputs: list[int] | None = None) -> bool:  # :128-227
    p = MODULI[field]
    t = Transcript(field)
    claim, r0 = initiate_protocol(p, t, proof["output_poly"])
    layers = list(reversed(structure))
    n = len(layers)
    alpha = beta = 0
    prev = []
    for i, ops in enumerate(layers):
        ok, final, chal = gkr_verify(field, proof["proof_polynomials"][i], claim, t)
        if not ok:
            return False
        if i == n - 1:
            o1, o2 = proof["input_evaluations"]
            if inputs is not None:  # stands in for the two KZG::verify calls (:162-180)
                mid = len(chal) // 2
                if (o1, o2) != (evaluate(p, list(inputs), chal[:mid]), evaluate(p, list(inputs), chal[mid:])):
                    return False
        else:
            o1, o2 = proof["claimed_evaluations"][i]
        if i == 0:  # get_verifier_claim :294-314
            pt = [r0] + list(chal)
            a_r = evaluate(p, get_add_mul_i(ops, ADD), pt)
            m_r = evaluate(p, get_add_mul_i(ops, MUL), pt)
        else:  # get_folded_verifier_claim :316-341
            mid = len(prev) // 2
            fb = get_folded_fbc_poly(p, ops, [0, 0], [0, 0], prev[:mid], prev[mid:], alpha, beta)
            a_r = evaluate(p, fb[0], list(chal))
            m_r = evaluate(p, fb[2], list(chal))
        if (a_r * (o1 + o2) + m_r * (o1 * o2)) % p != final:
            return False
        prev = chal
        t.append(fq_vec_to_bytes([o1]))
        alpha = t.get_random_challenge()
        t.append(fq_vec_to_bytes([o2]))
        beta = t.get_random_challenge()
        claim = (alpha * o1 + beta * o2) % p
    return True
