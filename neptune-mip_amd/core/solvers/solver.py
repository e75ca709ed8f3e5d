"""Solver base class — the reference lifecycle (`core/solvers/solver.py:5-46`) over the MI355X engine.

Reference: `__init__` creates a pywraplp SCIP solver (:6-13), `load_data` runs init_vars and
init_constraints (:15-20), `solve` sets the objective, calls `Solve()` and returns
`status == OPTIMAL` (:35-40), `score` returns the objective value (:45-46).

Here the model is structured, not enumerated: `load_data` binds the data (init_vars /
init_constraints have nothing to create), and `solve` runs the batched GPU branch-and-bound
(core/engine/bnb.py) whose every LP relaxation is solved by the gfx950 engine.  The engine is
created inside `solve`, i.e. after any fork of the serving process.  Unknown
keyword arguments are kept in `self.args`, as in the reference (:13).
"""
import datetime


class Solver:
    def __init__(self, verbose: bool = True, **kwargs):
        self.verbose = verbose
        self.data = None
        self.args = kwargs
        self._value = 0.0

    def load_data(self, data):
        self.data = data
        self.log("Initializing variables...")
        self.init_vars()
        self.log("Initializing constraints...")
        self.init_constraints()

    def init_vars(self):
        raise NotImplementedError("Solvers must implement init_vars()")

    def init_constraints(self):
        raise NotImplementedError("Solvers must implement init_constraints()")

    def init_objective(self):
        raise NotImplementedError("Solvers must implement init_objective()")

    def log(self, msg: str):
        if self.verbose:
            print(f"{datetime.datetime.now()}: {msg}")

    def solve(self):
        raise NotImplementedError("Solvers must implement solve()")

    def results(self):
        raise NotImplementedError("Solvers must implement results()")

    def score(self) -> float:
        return self._value
