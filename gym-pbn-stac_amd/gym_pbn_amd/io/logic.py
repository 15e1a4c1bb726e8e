"""Logic-function networks -> probability truth tables.

Mirrors ``logic_funcs_to_PBN_data`` (``gym_PBN/utils/converters.py:9-40``) and the
expression language of ``LogicExpressionEvaluator`` (``gym_PBN/utils/logic/eval.py:47-167``):
``and`` / ``or`` / ``not`` / parentheses / ``True`` / ``False`` over node-name symbols
(``[a-zA-Z]+\\d*`` prefix match, ``eval.py:105``).

An expression is compiled once to a postfix program with the reference's own
tokenisation and operator-stack rules -- including its corner cases, so that
an expression the reference accepts gives the same function here and one it
rejects is rejected here too:

* a whitespace-separated piece carrying both ``(`` and ``)`` keeps only the
  opening parentheses (``eval.py:80-92``), so ``"(a)"`` is a missing-parenthesis
  error while ``"(a and b)"`` is fine;
* ``True`` / ``False`` go to the operator stack (``eval.py:124-125``) and an
  ``and`` / ``or`` arriving on top of one is an error (the reference raises
  ``KeyError`` from its precedence table);
* juxtaposed symbols (``"a b"``) evaluate to the last one (``eval.py:164``).

The program is then run once over all ``2**k`` input assignments at a time
(numpy boolean vectors) instead of once per assignment. Probabilities accumulate
in function order per table entry, the same floating-point sums as
``truth_table[state] += prob`` (``converters.py:30-34``).
"""

from __future__ import annotations

import re
from typing import Dict, List, Sequence, Tuple

import numpy as np

__all__ = ["LogicSyntaxError", "LogicExpressionEvaluator", "compile_expression", "logic_funcs_to_pbn_data"]

_SYMBOL = re.compile(r"[a-zA-Z]+\d*")
# token kinds
SYM, AND, OR, NOT, LP, RP, HIGH, LOW = range(8)
_KEYWORDS = {"and": AND, "or": OR, "not": NOT, "(": LP, ")": RP, "True": HIGH, "False": LOW}
_PREC = {NOT: 20, AND: 11, OR: 10, SYM: 0, LP: 0, RP: 0}  # HIGH/LOW deliberately absent (see module doc)


class LogicSyntaxError(Exception):
    """An expression the reference evaluator rejects."""


def _split(expr: str) -> List[str]:
    """Whitespace split, then peel parentheses off the ends of each piece (eval.py:74-92)."""
    pieces = expr.split()
    out: List[str] = []
    for piece in pieces:
        n_open, n_close = piece.count("("), piece.count(")")
        core = piece.strip("()")
        if (n_open or n_close) and core:
            if n_open:
                out.extend(["("] * n_open)
                out.append(core)
            else:
                out.append(core)
                out.extend([")"] * n_close)
        else:
            out.append(piece)
    # bare "(" / ")" / "((" pieces stay as they are: one keyword token only if exactly "(" or ")"
    return out


def tokenize(expr: str) -> List[Tuple[int, str]]:
    words = _split(expr)
    toks: List[Tuple[int, str]] = []
    for pos, w in enumerate(words):
        if w in _KEYWORDS:
            kind = _KEYWORDS[w]
            prev = toks[-1][0] if toks else None
            if kind in (NOT, LP) and prev in (SYM, RP):
                raise LogicSyntaxError(f"Invalid syntax at {w} ({pos})")
            if kind == RP:
                if not toks:  # the reference fails on toks[-1] here
                    raise LogicSyntaxError(f"Invalid syntax at {w} ({pos})")
                if prev == LP:
                    raise LogicSyntaxError(f"Invalid syntax at {w} ({pos})")
            if kind in (AND, OR) and pos == len(words) - 1:
                raise LogicSyntaxError(f"Invalid syntax at {w} ({pos})")
            toks.append((kind, ""))
        elif _SYMBOL.match(w):
            toks.append((SYM, w))
        else:
            raise LogicSyntaxError(f"Illegal token {w}")
    return toks


def _postfix(toks: List[Tuple[int, str]]) -> List[Tuple[int, str]]:
    ops: List[Tuple[int, str]] = []
    out: List[Tuple[int, str]] = []
    for t in toks:
        k = t[0]
        if k in (AND, OR):
            while ops:
                top = ops[-1][0]
                if top not in _PREC:
                    raise LogicSyntaxError("constant operand before a binary operator")
                if _PREC[top] < _PREC[k]:
                    break
                out.append(ops.pop())
            ops.append(t)
        elif k == SYM:
            out.append(t)
        elif k in (NOT, LP, HIGH, LOW):
            ops.append(t)
        else:  # RP
            if not ops:
                raise LogicSyntaxError("Missing parenthesis")
            while ops[-1][0] != LP:
                out.append(ops.pop())
                if not ops:
                    raise LogicSyntaxError("Missing parenthesis")
            ops.pop()
    if ops and ops[-1][0] == LP:
        raise LogicSyntaxError("Missing parenthesis")
    out.extend(reversed(ops))  # deeper "(" tokens are emitted and ignored by the evaluator
    return out


def compile_expression(expr: str):
    """Return ``(symbols, program)``; symbols in order of appearance (duplicates kept, as get_symbols)."""
    if not expr:
        raise LogicSyntaxError("Empty expression string")
    toks = tokenize(expr)
    return [v for k, v in toks if k == SYM], _postfix(toks)


def run_program(program, values: Dict[str, np.ndarray], shape) -> np.ndarray:
    """Evaluate a postfix program over boolean vectors (one entry per input assignment)."""
    stack: List[np.ndarray] = []
    for k, v in program:
        if k == SYM:
            if v not in values:
                raise LogicSyntaxError(f"Symbol {v} doesn't exist.")
            stack.append(np.asarray(values[v], dtype=bool))
        elif k == HIGH:
            stack.append(np.ones(shape, dtype=bool))
        elif k == LOW:
            stack.append(np.zeros(shape, dtype=bool))
        elif k == NOT:
            if not stack:
                raise LogicSyntaxError("operand missing")
            stack.append(~stack.pop())
        elif k in (AND, OR):
            if len(stack) < 2:
                raise LogicSyntaxError("operand missing")
            r, l_ = stack.pop(), stack.pop()
            stack.append(l_ & r if k == AND else l_ | r)
    if not stack:
        raise LogicSyntaxError("empty program")
    return np.broadcast_to(stack[-1], shape)


class LogicExpressionEvaluator:
    """Same surface as the reference class: ``dictionary``, ``evaluate``, ``get_symbols``."""

    def __init__(self, role_dict: dict):
        self.dictionary = role_dict

    @classmethod
    def get_symbols(cls, in_str: str) -> List[str]:
        return [v for k, v in tokenize(in_str) if k == SYM]

    def evaluate(self, in_str: str) -> bool:
        _, prog = compile_expression(in_str)
        vals = {s: np.array(bool(v)) for s, v in self.dictionary.items()}
        return bool(run_program(prog, vals, ()))


def logic_funcs_to_pbn_data(nodes: Sequence[str], node_functions: Sequence[Sequence[Tuple[str, float]]]):
    """``PBN_DATA`` from logic functions: ``[(input_mask, truth_table, name, is_control), ...]``.

    Node i's inputs are every symbol of its functions (ascending node order, the
    first input is the most significant truth-table axis); its table entry for an
    input assignment is the summed probability of the functions true there.
    ``is_control`` is "no inputs" (``converters.py:36``) -- also for a node whose
    only function is a constant.
    """
    nodes = list(nodes)
    N = len(nodes)
    data = []
    for i, name in enumerate(nodes):
        mask = np.zeros(N, dtype=bool)
        progs = []
        for func, prob in node_functions[i]:
            syms, prog = compile_expression(func)
            for s in syms:
                if s in ("True", "False"):
                    continue
                if s not in nodes:
                    raise ValueError(f"{s!r} is not in list")  # nodes.index(symbol), converters.py:19
                mask[nodes.index(s)] = True
            progs.append((prog, prob))
        idx = np.nonzero(mask)[0]
        k = idx.size
        codes = np.arange(1 << k, dtype=np.int64)
        vals = {nodes[j]: ((codes >> (k - 1 - a)) & 1).astype(bool) for a, j in enumerate(idx)}
        flat = np.zeros(1 << k, dtype=np.float64)
        for prog, prob in progs:
            on = run_program(prog, vals, (1 << k,))
            flat[on] = flat[on] + prob
        data.append((mask, flat.reshape((2,) * k), name, k == 0))
    return data
