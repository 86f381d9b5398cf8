"""A minimal CasADi stand-in for running the reference's model code HERE (test infrastructure).

CasADi is not installed in this image.  The reference's model modules
(``highway_branch_dyn.py``, ``quadruped_branch_dyn.py``, ``HMM_backup_dyn.py``) build
CasADi ``SX``/``MX`` expression graphs with ``from casadi import *`` and then call the
compiled ``Function`` objects.  This module implements the subset of that API those three
files use -- enumerated from their text (SURVEY §8(c) route 2) -- so the reference's own
Python code can build its graphs unchanged and be evaluated numerically:

* ``SX``/``MX`` matrices of expression nodes: ``.sym``, ``SX(r, c)`` (structural zeros),
  ``SX(k)`` (a k x 1 column), ``SX(ndarray)``, ``SX.ones/zeros``, CasADi indexing
  (``x[k]`` linear and column-major, ``x[i, j]``, slices, ``x[i, :] = column`` by element
  count), ``.T``, ``.shape``, element-wise ``+ - * / **``, ``@`` (mtimes), NumPy ufuncs on
  symbols (``np.exp(dx)``);
* ``vertcat``, ``horzcat``, ``sum1``, ``sum2``, ``dot``, ``sumsqr``, ``norm_1``, ``kron``,
  ``reshape`` (column-major), ``diag``, ``transpose``, ``exp``, ``log``, ``cos``, ``sin``,
  ``fabs``, ``sqrt``, ``tanh``, ``fmax``, ``fmin``;
* ``jacobian(f, x)`` (entries are derivative nodes evaluated by forward-mode AD over the
  graph when the Function is called), ``Function(name, inputs, outputs)`` returning ``DM``;
* ``DM`` numeric matrices with CasADi's conversion of 1-D NumPy arrays to columns;
* ``interpolant(name, 'linear', [grid], values)`` (1-D, linear; the merge scene).

Arithmetic follows the graph the reference builds, operation by operation, in fp64; sums
(``sum1``, ``mtimes``, ``dot``) accumulate left to right as CasADi's SX does after its
``1*x``/``0+x`` simplifications.  Derivatives are exact forward-mode AD (CasADi builds
its derivative graphs symbolically; the two agree to rounding).

Used only by ``tools/gen_golden_model.py`` / ``tools/gen_golden.py`` (this container); it
never travels into the product path.
"""
from __future__ import annotations

import math
import sys

import numpy
import numpy as np

casadi = sys.modules[__name__]      # the reference tests ``isinstance(x, casadi.SX)``

# ---------------------------------------------------------------------------------------
# expression nodes
# ---------------------------------------------------------------------------------------
_ids = [0]


class _Node:
    __slots__ = ("op", "args", "val", "id")

    def __init__(self, op, args=(), val=None):
        self.op, self.args, self.val = op, args, val
        _ids[0] += 1
        self.id = _ids[0]


_ZERO = _Node("const", (), 0.0)
_ONE = _Node("const", (), 1.0)


def _const(v):
    v = float(v)
    if v == 0.0 and math.copysign(1.0, v) > 0:
        return _ZERO
    if v == 1.0:
        return _ONE
    return _Node("const", (), v)


def _is_const(a, v=None):
    return a.op == "const" and (v is None or a.val == v)


_UN = {"neg": lambda a: -a, "exp": math.exp, "log": math.log, "cos": math.cos, "sin": math.sin,
       "fabs": math.fabs, "sqrt": math.sqrt, "tanh": math.tanh,
       "sign": lambda a: (a > 0) - (a < 0)}
_BIN = {"add": lambda a, b: a + b, "sub": lambda a, b: a - b, "mul": lambda a, b: a * b,
        "div": lambda a, b: a / b, "pow": lambda a, b: a ** b, "fmax": max, "fmin": min}


def _un(op, a):
    if _is_const(a):
        return _const(_UN[op](a.val))
    if op == "neg" and a.op == "neg":
        return a.args[0]
    return _Node(op, (a,))


def _bin(op, a, b):
    # CasADi SXElem simplifications that do not change values: 0+x, x+0, x-0, 1*x, x*1, x/1
    if _is_const(a) and _is_const(b):
        return _const(_BIN[op](a.val, b.val))
    if op == "add":
        if _is_const(a, 0.0):
            return b
        if _is_const(b, 0.0):
            return a
    elif op == "sub":
        if _is_const(b, 0.0):
            return a
        if _is_const(a, 0.0):
            return _un("neg", b)
    elif op == "mul":
        if _is_const(a, 1.0):
            return b
        if _is_const(b, 1.0):
            return a
        if _is_const(a, 0.0) or _is_const(b, 0.0):
            return _ZERO
    elif op == "div":
        if _is_const(b, 1.0):
            return a
        if _is_const(a, 0.0):
            return _ZERO
    return _Node(op, (a, b))


# ---------------------------------------------------------------------------------------
# matrices of nodes
# ---------------------------------------------------------------------------------------
def _to_nodes(v):
    """Anything -> 2-D object array of nodes (1-D NumPy arrays become columns)."""
    if isinstance(v, _Mat):
        return v.a
    if isinstance(v, DM):
        return np.vectorize(_const, otypes=[object])(v.v) if v.v.size else np.empty(v.v.shape, object)
    if isinstance(v, _Node):
        return np.array([[v]], dtype=object)
    arr = np.asarray(v, dtype=float)
    if arr.ndim == 0:
        arr = arr.reshape(1, 1)
    elif arr.ndim == 1:
        arr = arr.reshape(-1, 1)
    out = np.empty(arr.shape, dtype=object)
    for idx, x in np.ndenumerate(arr):
        out[idx] = _const(x)
    return out


def _result_type(*xs):
    return MX if any(isinstance(x, MX) for x in xs) else SX


def _bcast(a, b):
    if a.shape == b.shape:
        return a, b
    if a.shape == (1, 1):
        return np.full(b.shape, a[0, 0], dtype=object), b
    if b.shape == (1, 1):
        return a, np.full(a.shape, b[0, 0], dtype=object)
    if a.size == b.size and 1 in a.shape and 1 in b.shape:     # row vs column vector
        return a, b.reshape(a.shape, order="F")
    raise ValueError(f"dimension mismatch {a.shape} vs {b.shape}")


def _elementwise(op, x, y):
    a, b = _bcast(_to_nodes(x), _to_nodes(y))
    out = np.empty(a.shape, dtype=object)
    for idx in np.ndindex(a.shape):
        out[idx] = _bin(op, a[idx], b[idx])
    return _result_type(x, y)(out)


def _map(op, x):
    if not isinstance(x, _Mat):
        return _numeric_un(op, x)
    out = np.empty(x.a.shape, dtype=object)
    for idx in np.ndindex(x.a.shape):
        out[idx] = _un(op, x.a[idx])
    return type(x)(out)


def _numeric_un(op, x):
    f = {"exp": np.exp, "log": np.log, "cos": np.cos, "sin": np.sin, "fabs": np.abs, "sqrt": np.sqrt,
         "tanh": np.tanh, "neg": np.negative, "sign": np.sign}[op]
    if isinstance(x, DM):
        return DM(f(x.v))
    r = f(x)
    return float(r) if np.ndim(r) == 0 else r


def _norm_index(k, n):
    if isinstance(k, slice):
        return list(range(n))[k]
    if isinstance(k, (list, tuple, np.ndarray)):
        return [int(i) + (n if int(i) < 0 else 0) for i in k]
    k = int(k)
    if k < 0:
        k += n
    if not 0 <= k < n:
        raise IndexError(f"index {k} out of range for {n}")
    return k


class _Mat:
    __array_priority__ = 1000

    def __init__(self, *args):
        if len(args) == 0:
            self.a = np.empty((1, 1), dtype=object)
            self.a[0, 0] = _ZERO
        elif len(args) == 1 and isinstance(args[0], np.ndarray) and args[0].dtype == object:
            a = args[0]
            self.a = a.reshape(-1, 1) if a.ndim == 1 else a
        elif len(args) == 1 and isinstance(args[0], (int, np.integer)) and not isinstance(args[0], bool):
            self.a = np.full((int(args[0]), 1), _ZERO, dtype=object)
        elif len(args) == 2:
            self.a = np.full((int(args[0]), int(args[1])), _ZERO, dtype=object)
        else:
            self.a = _to_nodes(args[0]).copy()

    # ---- construction ----
    @classmethod
    def sym(cls, name, r=1, c=1):
        a = np.empty((r, c), dtype=object)
        for j in range(c):
            for i in range(r):
                a[i, j] = _Node("sym", (), f"{name}_{i}_{j}")
        return cls(a)

    @classmethod
    def zeros(cls, r, c=1):
        return cls(r, c)

    @classmethod
    def ones(cls, r, c=1):
        return cls(np.full((r, c), _ONE, dtype=object))

    @classmethod
    def eye(cls, n):
        return cls(np.eye(n))

    # ---- shape ----
    @property
    def shape(self):
        return self.a.shape

    def size1(self):
        return self.a.shape[0]

    def size2(self):
        return self.a.shape[1]

    def numel(self):
        return self.a.size

    def is_scalar(self):
        return self.a.size == 1

    @property
    def T(self):
        return type(self)(self.a.T.copy())

    def __len__(self):
        return self.a.size

    # ---- indexing (CasADi semantics: one index = linear, column-major) ----
    def _lin(self):
        return self.a.reshape(-1, order="F")

    def __getitem__(self, k):
        if isinstance(k, tuple):
            i, j = k
            ii, jj = _norm_index(i, self.a.shape[0]), _norm_index(j, self.a.shape[1])
            sub = self.a[np.ix_(np.atleast_1d(ii), np.atleast_1d(jj))]
            return type(self)(sub.copy())
        lin = self._lin()
        idx = _norm_index(k, lin.size)
        if isinstance(idx, int):
            return type(self)(np.array([[lin[idx]]], dtype=object))
        sel = np.array([lin[i] for i in idx], dtype=object)
        return type(self)(sel.reshape(1, -1) if self.a.shape[0] == 1 and self.a.shape[1] > 1 else sel.reshape(-1, 1))

    def __setitem__(self, k, v):
        vals = _to_nodes(v)
        if isinstance(k, tuple):
            i, j = k
            ii = np.atleast_1d(_norm_index(i, self.a.shape[0]))
            jj = np.atleast_1d(_norm_index(j, self.a.shape[1]))
            tgt = [(r, c) for c in jj for r in ii]          # column-major order of the target block
        else:
            lin = _norm_index(k, self.a.size)
            lin = np.atleast_1d(lin)
            r0 = self.a.shape[0]
            tgt = [(int(q) % r0, int(q) // r0) for q in lin]
        flat = vals.reshape(-1, order="F")
        if flat.size == 1:
            flat = np.full(len(tgt), flat[0], dtype=object)
        if flat.size != len(tgt):
            raise ValueError(f"assignment of {vals.shape} to {len(tgt)} entries")
        for (r, c), node in zip(tgt, flat):
            self.a[r, c] = node

    # ---- arithmetic ----
    def __add__(self, o):
        return _elementwise("add", self, o)

    def __radd__(self, o):
        return _elementwise("add", o, self)

    def __sub__(self, o):
        return _elementwise("sub", self, o)

    def __rsub__(self, o):
        return _elementwise("sub", o, self)

    def __mul__(self, o):
        return _elementwise("mul", self, o)

    def __rmul__(self, o):
        return _elementwise("mul", o, self)

    def __truediv__(self, o):
        return _elementwise("div", self, o)

    def __rtruediv__(self, o):
        return _elementwise("div", o, self)

    def __pow__(self, o):
        return _elementwise("pow", self, o)

    def __neg__(self):
        return _map("neg", self)

    def __matmul__(self, o):
        return mtimes(self, o)

    def __rmatmul__(self, o):
        return mtimes(o, self)

    def __array_ufunc__(self, ufunc, method, *inputs, **kw):
        if method != "__call__":
            return NotImplemented
        un = {np.exp: "exp", np.log: "log", np.cos: "cos", np.sin: "sin", np.sqrt: "sqrt",
              np.abs: "fabs", np.fabs: "fabs", np.tanh: "tanh", np.negative: "neg", np.sign: "sign"}
        bi = {np.add: "add", np.subtract: "sub", np.multiply: "mul", np.true_divide: "div", np.power: "pow",
              np.matmul: "matmul"}
        if ufunc in un:
            return _map(un[ufunc], inputs[0])
        if ufunc in bi:
            if bi[ufunc] == "matmul":
                return mtimes(*inputs)
            return _elementwise(bi[ufunc], *inputs)
        return NotImplemented

    def __repr__(self):
        return f"{type(self).__name__}{self.a.shape}"


class SX(_Mat):
    pass


class MX(_Mat):
    pass


# ---------------------------------------------------------------------------------------
# numeric matrices
# ---------------------------------------------------------------------------------------
class DM:
    """Numeric matrix; 1-D NumPy operands are columns (CasADi's conversion)."""

    __array_priority__ = 1000

    def __init__(self, v=0.0, c=None):
        if c is not None:
            self.v = np.zeros((int(v), int(c)))
            return
        if isinstance(v, DM):
            v = v.v
        a = np.array(v, dtype=float)
        self.v = a.reshape(1, 1) if a.ndim == 0 else (a.reshape(-1, 1) if a.ndim == 1 else a)

    @staticmethod
    def _col(o):
        if isinstance(o, DM):
            return o.v
        a = np.asarray(o, dtype=float)
        return a.reshape(1, 1) if a.ndim == 0 else (a.reshape(-1, 1) if a.ndim == 1 else a)

    @property
    def shape(self):
        return self.v.shape

    def full(self):
        return self.v.copy()

    def __array__(self, dtype=None, copy=None):
        return self.v.astype(dtype) if dtype is not None else self.v.copy()

    def __float__(self):
        return float(self.v.reshape(-1)[0])

    def __getitem__(self, k):
        if isinstance(k, tuple):
            return DM(self.v[k])
        return DM(self.v.reshape(-1, order="F")[k])

    def _bin(self, o, f, rev=False):
        if isinstance(o, _Mat):
            return NotImplemented
        a, b = self.v, self._col(o)
        return DM(f(b, a) if rev else f(a, b))

    def __add__(self, o):
        return self._bin(o, np.add)

    def __radd__(self, o):
        return self._bin(o, np.add, True)

    def __sub__(self, o):
        return self._bin(o, np.subtract)

    def __rsub__(self, o):
        return self._bin(o, np.subtract, True)

    def __mul__(self, o):
        return self._bin(o, np.multiply)

    def __rmul__(self, o):
        return self._bin(o, np.multiply, True)

    def __truediv__(self, o):
        return self._bin(o, np.true_divide)

    def __matmul__(self, o):
        if isinstance(o, _Mat):
            return mtimes(self, o)
        return DM(self.v @ self._col(o))

    def __rmatmul__(self, o):
        return DM(self._col(o) @ self.v)

    def __neg__(self):
        return DM(-self.v)

    def __array_ufunc__(self, ufunc, method, *inputs, **kw):
        args = [i.v if isinstance(i, DM) else i for i in inputs]
        if method != "__call__":          # reductions (np.sum ...) give plain NumPy results
            return getattr(ufunc, method)(*args, **kw)
        if ufunc is np.matmul:
            return DM(self._col(inputs[0]) @ self._col(inputs[1]))
        return DM(getattr(ufunc, method)(*args, **kw))

    @property
    def T(self):
        return DM(self.v.T)

    def __repr__(self):
        return f"DM({self.v!r})"


# ---------------------------------------------------------------------------------------
# free functions of the CasADi API used by the reference
# ---------------------------------------------------------------------------------------
def _sym_any(*xs):
    return any(isinstance(x, _Mat) for x in xs)


def _as_mat(x):
    return x if isinstance(x, _Mat) else SX(_to_nodes(x))


def mtimes(a, b):
    if not _sym_any(a, b):
        return DM(DM._col(a) @ DM._col(b))
    A, Bm = _to_nodes(a), _to_nodes(b)
    if A.shape == (1, 1) or Bm.shape == (1, 1):
        return _elementwise("mul", a, b)
    if A.shape[1] != Bm.shape[0]:
        raise ValueError(f"mtimes dimension mismatch {A.shape} @ {Bm.shape}")
    out = np.empty((A.shape[0], Bm.shape[1]), dtype=object)
    for i in range(A.shape[0]):
        for j in range(Bm.shape[1]):
            acc = _ZERO
            for k in range(A.shape[1]):
                acc = _bin("add", acc, _bin("mul", A[i, k], Bm[k, j]))
            out[i, j] = acc
    return _result_type(a, b)(out)


def vertcat(*xs):
    if not _sym_any(*xs):
        return DM(np.vstack([DM._col(x) for x in xs]))
    return _result_type(*xs)(np.vstack([_to_nodes(x) for x in xs]))


def horzcat(*xs):
    if not _sym_any(*xs):
        return DM(np.hstack([DM._col(x) for x in xs]))
    return _result_type(*xs)(np.hstack([_to_nodes(x) for x in xs]))


def sum1(x):
    if not isinstance(x, _Mat):
        return DM(np.sum(DM._col(x), axis=0, keepdims=True))
    out = np.empty((1, x.a.shape[1]), dtype=object)
    for j in range(x.a.shape[1]):
        acc = _ZERO
        for i in range(x.a.shape[0]):
            acc = _bin("add", acc, x.a[i, j])
        out[0, j] = acc
    return type(x)(out)


def sum2(x):
    return sum1(x.T).T


def dot(a, b):
    if not _sym_any(a, b):
        return float(np.sum(DM._col(a) * DM._col(b)))
    A, Bm = _bcast(_to_nodes(a), _to_nodes(b))
    acc = _ZERO
    for p, q in zip(A.reshape(-1, order="F"), Bm.reshape(-1, order="F")):
        acc = _bin("add", acc, _bin("mul", p, q))
    return _result_type(a, b)(np.array([[acc]], dtype=object))


def sumsqr(x):
    return dot(x, x)


def norm_1(x):
    if not isinstance(x, _Mat):
        return float(np.sum(np.abs(DM._col(x))))
    acc = _ZERO
    for p in x.a.reshape(-1, order="F"):
        acc = _bin("add", acc, _un("fabs", p))
    return type(x)(np.array([[acc]], dtype=object))


def kron(a, b):
    if not _sym_any(a, b):
        return DM(np.kron(DM._col(a), DM._col(b)))
    A, Bm = _to_nodes(a), _to_nodes(b)
    r1, c1 = A.shape
    r2, c2 = Bm.shape
    out = np.empty((r1 * r2, c1 * c2), dtype=object)
    for i in range(r1):
        for j in range(c1):
            for k in range(r2):
                for l in range(c2):
                    out[i * r2 + k, j * c2 + l] = _bin("mul", A[i, j], Bm[k, l])
    return _result_type(a, b)(out)


def reshape(x, r, c=None):
    if isinstance(r, tuple):
        r, c = r
    if not isinstance(x, _Mat):
        v = DM._col(x)
        r = v.size // c if r == -1 else r
        c = v.size // r if c == -1 else c
        return DM(v.reshape((r, c), order="F"))
    n = x.a.size
    r = n // c if r == -1 else r
    c = n // r if c == -1 else c
    return type(x)(x.a.reshape((r, c), order="F").copy())


def transpose(x):
    return x.T


def diag(x):
    if not isinstance(x, _Mat):
        v = DM._col(x)
        return DM(np.diag(v.reshape(-1)) if 1 in v.shape else np.diag(v).reshape(-1, 1))
    if 1 in x.a.shape:
        v = x.a.reshape(-1, order="F")
        out = np.full((v.size, v.size), _ZERO, dtype=object)
        for i, p in enumerate(v):
            out[i, i] = p
        return type(x)(out)
    return type(x)(np.array([[x.a[i, i]] for i in range(min(x.a.shape))], dtype=object))


def exp(x):
    return _map("exp", x)


def log(x):
    return _map("log", x)


def cos(x):
    return _map("cos", x)


def sin(x):
    return _map("sin", x)


def fabs(x):
    return _map("fabs", x)


def sqrt(x):
    return _map("sqrt", x)


def tanh(x):
    return _map("tanh", x)


def sign(x):
    return _map("sign", x)


def fmax(a, b):
    if not _sym_any(a, b):
        return np.maximum(a, b)
    return _elementwise("fmax", a, b)


def fmin(a, b):
    if not _sym_any(a, b):
        return np.minimum(a, b)
    return _elementwise("fmin", a, b)


# ---------------------------------------------------------------------------------------
# differentiation and compiled functions
# ---------------------------------------------------------------------------------------
def jacobian(f, x):
    """d vec(f) / d vec(x): F x n matrix of derivative nodes (x: purely symbolic)."""
    F = _to_nodes(f).reshape(-1, order="F")
    X = _to_nodes(x).reshape(-1, order="F")
    for s in X:
        if s.op != "sym":
            raise ValueError("jacobian w.r.t. a non-symbolic expression")
    out = np.empty((F.size, X.size), dtype=object)
    for i, fn in enumerate(F):
        for j, s in enumerate(X):
            out[i, j] = _ZERO if _is_const(fn) else _Node("d", (fn, s))
    return _result_type(f, x)(out)


class _Interp:
    """1-D linear ``interpolant``: CasADi's 'linear' plugin (linear on each grid cell, the
    end cells extended beyond the grid)."""

    def __init__(self, name, grid, values):
        self.name = name
        self.g = np.asarray(grid, float).reshape(-1)
        self.v = np.asarray(values, float).reshape(-1)

    def cell(self, t):
        i = int(np.searchsorted(self.g, t, side="right") - 1)
        return min(max(i, 0), self.g.size - 2)

    def value(self, t):
        i = self.cell(t)
        g0, g1, v0, v1 = self.g[i], self.g[i + 1], self.v[i], self.v[i + 1]
        return v0 + (t - g0) / (g1 - g0) * (v1 - v0)

    def slope(self, t):
        i = self.cell(t)
        return (self.v[i + 1] - self.v[i]) / (self.g[i + 1] - self.g[i])

    def __call__(self, t):
        if isinstance(t, _Mat):
            out = np.empty(t.a.shape, dtype=object)
            for idx in np.ndindex(t.a.shape):
                out[idx] = _Node("interp", (t.a[idx],), self)
            return type(t)(out)
        if isinstance(t, DM):
            return DM(np.vectorize(self.value)(t.v))
        # a scalar in gives a float out here (CasADi gives a 1x1 DM): the reference's NumPy
        # branch np.array([0.5*(v0 - v), psiref(X) - Kpsi*psi]) (highway_branch_dyn.py:96) is a
        # ragged list under NumPy >= 1.24 with a DM in it; its value is the same
        return float(self.value(float(t)))


def interpolant(name, solver, grid, values, *opts):
    if solver != "linear" or len(grid) != 1:
        raise NotImplementedError("shim: only 1-D linear interpolants")
    return _Interp(name, grid[0], values)


def _topo(roots):
    """Nodes reachable from roots (derivative nodes pull in their function node), in an
    order where arguments come first."""
    order, seen = [], set()
    stack = [(r, False) for r in roots]
    while stack:
        node, done = stack.pop()
        if done:
            order.append(node)
            continue
        if node.id in seen:
            continue
        seen.add(node.id)
        stack.append((node, True))
        kids = node.args if node.op != "d" else (node.args[0],)
        for k in kids:
            if k.id not in seen:
                stack.append((k, False))
    return order


class Function:
    """Compiled evaluation of the output matrices at numeric inputs (returns DM)."""

    def __init__(self, name, inputs, outputs, *opts):
        self.name = name
        self.ins = [_to_nodes(i).reshape(-1, order="F") for i in inputs]
        self.in_shapes = [_to_nodes(i).shape for i in inputs]
        for vec in self.ins:
            for s in vec:
                if s.op != "sym":
                    raise ValueError(f"Function {name}: inputs must be purely symbolic")
        self.outs = [_to_nodes(o) for o in outputs]
        roots = [n for o in self.outs for n in o.reshape(-1)]
        self.order = _topo(roots)
        dsyms = []
        for n in self.order:
            if n.op == "d":
                if any(a.op == "d" for a in _topo([n.args[0]])):
                    raise NotImplementedError("shim: nested derivatives")
                if n.args[1].id not in {s.id for s in dsyms}:
                    dsyms.append(n.args[1])
        self.dpos = {s.id: k for k, s in enumerate(dsyms)}
        self.nd = len(dsyms)

    def __call__(self, *args):
        if len(args) != len(self.ins):
            raise TypeError(f"Function {self.name}: {len(self.ins)} inputs expected")
        val, tan = {}, {}
        nd = self.nd
        for vec, shp, arg in zip(self.ins, self.in_shapes, args):
            a = np.asarray(arg.v if isinstance(arg, DM) else arg, dtype=float)
            if a.size != vec.size:
                raise ValueError(f"Function {self.name}: input of {a.size} entries for {shp}")
            flat = a.reshape(shp, order="C").reshape(-1, order="F") if a.ndim == 2 else a.reshape(-1)
            for s, v in zip(vec, flat):
                val[s.id] = float(v)
        for n in self.order:
            op = n.op
            if op == "sym":
                if n.id not in val:
                    raise ValueError(f"Function {self.name}: free symbol {n.val}")
                t = np.zeros(nd)
                if n.id in self.dpos:
                    t[self.dpos[n.id]] = 1.0
                tan[n.id] = t
                continue
            if op == "const":
                val[n.id], tan[n.id] = n.val, np.zeros(nd)
                continue
            if op == "d":
                val[n.id] = float(tan[n.args[0].id][self.dpos[n.args[1].id]])
                tan[n.id] = np.zeros(nd)
                continue
            if op == "interp":
                a = val[n.args[0].id]
                val[n.id] = n.val.value(a)
                tan[n.id] = n.val.slope(a) * tan[n.args[0].id]
                continue
            if len(n.args) == 1:
                a, ta = val[n.args[0].id], tan[n.args[0].id]
                v = _UN[op](a)
                if op == "neg":
                    t = -ta
                elif op == "exp":
                    t = v * ta
                elif op == "log":
                    t = ta / a
                elif op == "cos":
                    t = -math.sin(a) * ta
                elif op == "sin":
                    t = math.cos(a) * ta
                elif op == "fabs":
                    t = float((a > 0) - (a < 0)) * ta
                elif op == "sqrt":
                    t = ta / (2.0 * v)
                elif op == "tanh":
                    t = (1.0 - v * v) * ta
                elif op == "sign":
                    t = np.zeros(nd)
                else:
                    raise NotImplementedError(op)
            else:
                a, b = val[n.args[0].id], val[n.args[1].id]
                ta, tb = tan[n.args[0].id], tan[n.args[1].id]
                v = _BIN[op](a, b)
                if op == "add":
                    t = ta + tb
                elif op == "sub":
                    t = ta - tb
                elif op == "mul":
                    t = ta * b + a * tb
                elif op == "div":
                    t = (ta - v * tb) / b
                elif op == "pow":
                    t = b * a ** (b - 1) * ta + (v * math.log(a) * tb if a > 0 else 0.0 * tb)
                elif op == "fmax":
                    t = ta if a >= b else tb
                elif op == "fmin":
                    t = ta if a <= b else tb
                else:
                    raise NotImplementedError(op)
            val[n.id], tan[n.id] = v, t
        res = []
        for o in self.outs:
            out = np.empty(o.shape)
            for idx in np.ndindex(o.shape):
                out[idx] = val[o[idx].id]
            res.append(DM(out))
        return res[0] if len(res) == 1 else tuple(res)


inf = float("inf")
pi = math.pi
