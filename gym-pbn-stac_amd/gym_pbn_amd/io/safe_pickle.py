"""No-execution decoder for the predictor-set pickles gym-PBN ships.

The reference caches its inferred networks as pickles
(``gym_PBN/envs/bittner/gen/predictor_sets.py:22-24,37-38``): a list with one
numpy object array of shape ``(3, n_pred)`` per node holding
``(COD, A, inputIDs)`` columns (``predictor_sets.py:45,80-102``).

Unpickling such a file would let it call any importable function. This module
never does: it walks the opcode stream with :func:`pickletools.genops` (a
parser, not an unpickler), builds an inert symbolic tree, and then materialises
only a whitelist of shapes -- numpy ``_reconstruct``/``ndarray``/``dtype``
triples, tuples, lists, dicts, ints, floats, bytes, str, None and bools. Any
other global, or any call outside the whitelist, raises
:class:`UnsafePickleError`. No name in the file is ever imported or called.
"""

from __future__ import annotations

import pickletools
from typing import Any

import numpy as np

__all__ = ["UnsafePickleError", "load_pickle_safely", "decode_pickle_bytes"]


class UnsafePickleError(ValueError):
    """Raised when a pickle needs anything outside the data-only whitelist."""


_NDARRAY_RECON = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")}
_NDARRAY_TYPE = {("numpy", "ndarray")}
_DTYPE = {("numpy", "dtype")}
_SCALAR = {("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar")}


class _Global:
    __slots__ = ("module", "name")

    def __init__(self, module: str, name: str):
        self.module, self.name = module, name

    @property
    def key(self):
        return (self.module, self.name)


class _Call:
    """A REDUCE node: ``func(*args)`` recorded, never executed."""

    __slots__ = ("func", "args", "state")

    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None


class _Mark:
    pass


_MARK = _Mark()


def _pop_mark(stack):
    items = []
    while True:
        x = stack.pop()
        if x is _MARK:
            break
        items.append(x)
    items.reverse()
    return items


def _parse(data: bytes):
    stack: list = []
    memo: dict = {}
    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("PUT", "BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n in ("GET", "BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG"):
            stack.append(int(arg))
        elif n in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE"):
            stack.append(str(arg))
        elif n in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif n == "SHORT_BINSTRING" or n == "BINSTRING":
            stack.append(arg.encode("latin-1") if isinstance(arg, str) else bytes(arg))
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "TUPLE1":
            stack[-1:] = [(stack[-1],)]
        elif n == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif n == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        elif n == "TUPLE":
            stack.append(tuple(_pop_mark(stack)))
        elif n == "LIST":
            stack.append(list(_pop_mark(stack)))
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = _pop_mark(stack)
            stack[-1].extend(items)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][_hashable(k)] = v
        elif n == "SETITEMS":
            items = _pop_mark(stack)
            d = stack[-1]
            for k, v in zip(items[0::2], items[1::2]):
                d[_hashable(k)] = v
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            module = stack.pop()
            stack.append(_Global(module, name))
        elif n == "GLOBAL":
            module, name = arg.split(" ", 1)
            stack.append(_Global(module, name))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            if not isinstance(func, _Global):
                raise UnsafePickleError("REDUCE on a non-global callable")
            stack.append(_Call(func, args))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, _Call):
                raise UnsafePickleError("BUILD on a non-reconstructed object")
            obj.state = state
        else:
            raise UnsafePickleError(f"pickle opcode {n} is outside the data-only whitelist")
    if len(stack) != 1:
        raise UnsafePickleError("malformed pickle stream")
    return stack[0]


def _hashable(k):
    if isinstance(k, (int, float, str, bytes, tuple, bool)) or k is None:
        return k
    raise UnsafePickleError("unhashable dict key in pickle")


def _make_dtype(node) -> np.dtype:
    if not (isinstance(node, _Call) and node.func.key in _DTYPE):
        raise UnsafePickleError("expected a numpy dtype record")
    code = node.args[0]
    if not isinstance(code, str):
        raise UnsafePickleError("dtype code must be a string")
    dt = np.dtype(code)
    st = node.state
    if st is not None and isinstance(st, tuple) and len(st) >= 2 and st[1] in ("<", ">"):
        dt = dt.newbyteorder(st[1])
    return dt


def _materialise(node, cache: dict) -> Any:
    key = id(node)
    if key in cache:
        return cache[key]
    if isinstance(node, (int, float, str, bytes, bool)) or node is None:
        return node
    if isinstance(node, tuple):
        out = tuple(_materialise(x, cache) for x in node)
        cache[key] = out
        return out
    if isinstance(node, list):
        out = []
        cache[key] = out
        out.extend(_materialise(x, cache) for x in node)
        return out
    if isinstance(node, dict):
        out = {}
        cache[key] = out
        for k, v in node.items():
            out[k] = _materialise(v, cache)
        return out
    if isinstance(node, _Call):
        fk = node.func.key
        if fk in _NDARRAY_RECON:
            if not (isinstance(node.args[0], _Global) and node.args[0].key in _NDARRAY_TYPE):
                raise UnsafePickleError("_reconstruct of a non-ndarray type")
            st = node.state
            if not (isinstance(st, tuple) and len(st) == 5):
                raise UnsafePickleError("unexpected ndarray state")
            _ver, shape, dtnode, fortran, raw = st
            dt = _make_dtype(dtnode)
            shape = tuple(int(s) for s in shape)
            if dt.kind == "O":
                items = [_materialise(x, cache) for x in raw]
                arr = np.empty(len(items), dtype=object)
                for i, it in enumerate(items):
                    arr[i] = it
                arr = arr.reshape(shape, order="F" if fortran else "C")
            else:
                if not isinstance(raw, (bytes, bytearray)):
                    raise UnsafePickleError("numeric ndarray payload must be bytes")
                arr = np.frombuffer(raw, dtype=dt).copy()
                arr = arr.reshape(shape, order="F" if fortran else "C")
            cache[key] = arr
            return arr
        if fk in _SCALAR:
            dt = _make_dtype(node.args[0])
            raw = node.args[1]
            if not isinstance(raw, (bytes, bytearray)):
                raise UnsafePickleError("numpy scalar payload must be bytes")
            val = np.frombuffer(raw, dtype=dt)[0]
            cache[key] = val
            return val
        raise UnsafePickleError(f"global {fk[0]}.{fk[1]} is not whitelisted")
    if isinstance(node, _Global):
        raise UnsafePickleError(f"bare global {node.module}.{node.name} is not data")
    raise UnsafePickleError(f"unsupported node {type(node).__name__}")


def decode_pickle_bytes(data: bytes) -> Any:
    """Decode a data-only pickle without importing or calling anything."""
    return _materialise(_parse(data), {})


def load_pickle_safely(path) -> Any:
    with open(path, "rb") as f:
        return decode_pickle_bytes(f.read())
