"""Probe-only stand-in for OR-Tools' `pywraplp` (OR-Tools 9.6.2534 is absent offline).

It RECORDS the model the reference's own builders emit through the subset of the
pywraplp API they use (`core/solvers/solver.py:1-45`, `core/solvers/neptune/utils/*.py`):
NumVar/BoolVar/IntVar/infinity/Sum/Add/Objective/SetCoefficient/SetMinimization/
SetMaximization/Value/Solve/solution_value/EnableOutput/OPTIMAL.

`Solve()` turns the recorded model into a CSR matrix and solves it with HiGHS through
`scipy.optimize.milp` (MIP, or the LP relaxation when `Solver.RELAX` is set).  Every
solved model is appended to `Solver.RECORD` so tools/gen_golden.py can dump it as a
fixture.  This file contains no reference code and is never shipped or run on the GPU
box: it lives under tools/ and is only put on sys.path by tools/gen_golden.py.
"""
import math

import numpy as np
import scipy.sparse as sp
from scipy.optimize import Bounds, LinearConstraint, milp


class LinExpr:
    __array_ufunc__ = None  # make numpy scalars defer to our reflected operators
    __slots__ = ("terms", "const")

    def __init__(self, terms=None, const=0.0):
        self.terms = terms if terms is not None else {}
        self.const = float(const)

    @staticmethod
    def _lift(o):
        if isinstance(o, LinExpr):
            return o
        return LinExpr({}, float(o))

    def _combine(self, other, sign):
        o = LinExpr._lift(other)
        t = dict(self.terms)
        for k, v in o.terms.items():
            t[k] = t.get(k, 0.0) + sign * v
        return LinExpr(t, self.const + sign * o.const)

    def __add__(self, o):
        return self._combine(o, 1.0)

    __radd__ = __add__

    def __sub__(self, o):
        return self._combine(o, -1.0)

    def __rsub__(self, o):
        return LinExpr._lift(o)._combine(self, -1.0)

    def __mul__(self, s):
        if isinstance(s, LinExpr):
            raise TypeError("non-linear product")
        s = float(s)
        return LinExpr({k: v * s for k, v in self.terms.items()}, self.const * s)

    __rmul__ = __mul__

    def __neg__(self):
        return self * -1.0

    def __le__(self, o):
        e = self - o
        return Constraint(e, -math.inf, 0.0)

    def __ge__(self, o):
        e = self - o
        return Constraint(e, 0.0, math.inf)

    def __eq__(self, o):
        e = self - o
        return Constraint(e, 0.0, 0.0)

    __hash__ = object.__hash__


class Variable(LinExpr):
    __slots__ = ("index", "lb", "ub", "integer", "name", "_solver")

    def __init__(self, solver, index, lb, ub, integer, name):
        super().__init__({index: 1.0}, 0.0)
        self._solver = solver
        self.index = index
        self.lb, self.ub, self.integer, self.name = float(lb), float(ub), integer, name

    def solution_value(self):
        sol = self._solver._solution
        return 0.0 if sol is None else float(sol[self.index])

    def name_(self):
        return self.name

    __hash__ = object.__hash__


class Constraint:
    __slots__ = ("expr", "lo", "hi")

    def __init__(self, expr, lo, hi):
        self.expr, self.lo, self.hi = expr, lo, hi


class Objective:
    def __init__(self, solver):
        self._solver = solver
        self.coefs = {}
        self.offset = 0.0
        self.maximize = False

    def SetCoefficient(self, var, coef):
        self.coefs[var.index] = float(coef)

    def SetMinimization(self):
        self.maximize = False

    def SetMaximization(self):
        self.maximize = True

    def SetOffset(self, v):
        self.offset = float(v)

    def Value(self):
        sol = self._solver._solution
        if sol is None:
            return 0.0
        return self.offset + sum(c * sol[k] for k, c in self.coefs.items())


class Solver:
    OPTIMAL, FEASIBLE, INFEASIBLE, UNBOUNDED, ABNORMAL, NOT_SOLVED = 0, 1, 2, 3, 4, 6
    RELAX = False          # solve the LP relaxation instead of the MIP
    TIME_LIMIT = None      # seconds, optional
    RECORD = None          # list to append every solved model to (or None)

    def __init__(self, name="SCIP"):
        self._vars = []
        self._cons = []
        self._obj = Objective(self)
        self._solution = None

    @staticmethod
    def CreateSolver(name):
        return Solver(name)

    def EnableOutput(self):
        pass

    def infinity(self):
        return math.inf

    def NumVar(self, lb, ub, name=""):
        v = Variable(self, len(self._vars), lb, ub, False, name)
        self._vars.append(v)
        return v

    def IntVar(self, lb, ub, name=""):
        v = Variable(self, len(self._vars), lb, ub, True, name)
        self._vars.append(v)
        return v

    def BoolVar(self, name=""):
        return self.IntVar(0, 1, name)

    def Sum(self, items):
        t = {}
        const = 0.0
        for it in items:
            if isinstance(it, LinExpr):
                for k, v in it.terms.items():
                    t[k] = t.get(k, 0.0) + v
                const += it.const
            else:
                const += float(it)
        return LinExpr(t, const)

    def Add(self, con):
        if isinstance(con, (bool, np.bool_)):
            # trivially true/false comparisons between constants
            con = Constraint(LinExpr({}, 0.0 if con else 1.0), 0.0, 0.0)
        self._cons.append(con)
        return con

    def Objective(self):
        return self._obj

    def model_arrays(self):
        nv = len(self._vars)
        rows, cols, vals, lo, hi = [], [], [], [], []
        for r, con in enumerate(self._cons):
            for k, v in con.expr.terms.items():
                rows.append(r)
                cols.append(k)
                vals.append(v)
            lo.append(con.lo - con.expr.const)
            hi.append(con.hi - con.expr.const)
        A = sp.csr_matrix((np.asarray(vals, float), (np.asarray(rows, np.int64), np.asarray(cols, np.int64))),
                          shape=(len(self._cons), nv))
        A.sum_duplicates()
        c = np.zeros(nv)
        for k, v in self._obj.coefs.items():
            c[k] = v
        lb = np.array([v.lb for v in self._vars])
        ub = np.array([v.ub for v in self._vars])
        integ = np.array([1 if v.integer else 0 for v in self._vars], np.int8)
        names = [v.name for v in self._vars]
        return dict(A=A, lo=np.asarray(lo, float), hi=np.asarray(hi, float), c=c, lb=lb, ub=ub,
                    integrality=integ, names=names, maximize=self._obj.maximize, offset=self._obj.offset)

    def Solve(self):
        m = self.model_arrays()
        c = -m["c"] if m["maximize"] else m["c"]
        integ = np.zeros_like(m["integrality"]) if Solver.RELAX else m["integrality"]
        opts = {"mip_rel_gap": 0.0, "presolve": True}
        if Solver.TIME_LIMIT:
            opts["time_limit"] = Solver.TIME_LIMIT
        cons = [LinearConstraint(m["A"], m["lo"], m["hi"])] if m["A"].shape[0] else []
        res = milp(c, constraints=cons, integrality=integ, bounds=Bounds(m["lb"], m["ub"]), options=opts)
        if res.status == 0:
            status = Solver.OPTIMAL
        elif res.status == 2:
            status = Solver.INFEASIBLE
        elif res.status == 3:
            status = Solver.UNBOUNDED
        elif res.x is not None:
            status = Solver.FEASIBLE
        else:
            status = Solver.NOT_SOLVED
        self._solution = None if res.x is None else np.asarray(res.x, float)
        m["status"] = status
        m["relaxed"] = bool(Solver.RELAX)
        m["x"] = self._solution
        m["objective"] = self._obj.Value() if self._solution is not None else None
        if Solver.RECORD is not None:
            Solver.RECORD.append(m)
        return status
