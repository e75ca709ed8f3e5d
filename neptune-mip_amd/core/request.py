"""The reference's request handling, without the web server: one REST payload in, the response body out.

Mirrors `main.py:31-62` of the reference (the body of its Flask route `serve()`): resolve
`solver.type` (default NeptuneMinDelayAndUtilization) with its `args`, build the solver input from
the payload (`with_db`, default True; `workload_coeff`, default 1), time load_data + solve, and
return the JSON body `{"cpu_routing_rules", "cpu_allocations", "gpu_routing_rules": {},
"gpu_allocations": {}, "score", "processing_time"}`.  The reference resolves the type with `eval`;
here it goes through the `core.solvers.SOLVERS` whitelist (an unknown type raises KeyError, which
the reference's server turns into HTTP 500 like any exception).

The reference serves every request in a forked Werkzeug child (`main.py:69`, processes=10); the
engine creates its HIP context on first use, so a child forked from a parent that never touched
the GPU solves normally (tests/test_gpu_request.py)."""
import time

from .solvers import SOLVERS
from .utils import check_input, data_to_solver_input


def solve_request(payload, solver_out=None):
    """Response body of the reference's `serve()` for one payload (dict).  A malformed payload fails
    the reference's input assertions (`check_input`, main.py:35) before any engine call.  solver_out: a list
    that receives the solver object (bench.py reads each step's B&B status from it)."""
    check_input(payload)
    solver = payload.get("solver", {"type": "NeptuneMinDelayAndUtilization"})
    solver_type = solver.get("type")
    solver_args = solver.get("args", {})
    with_db = payload.get("with_db", True)
    s = SOLVERS[solver_type](**solver_args)
    if solver_out is not None:
        solver_out.append(s)
    start = time.time()
    s.load_data(data_to_solver_input(payload, with_db=with_db, workload_coeff=payload.get("workload_coeff", 1)))
    s.solve()
    processing_time = time.time() - start
    x, c = s.results()
    score = s.score()
    return {
        "cpu_routing_rules": x,
        "cpu_allocations": c,
        "gpu_routing_rules": {},
        "gpu_allocations": {},
        "score": score,
        "processing_time": processing_time,
    }
