"""NEPTUNE placement MIP on MI355X — drop-in for the reference's `core` package.

Same import surface as the reference (`from core import data_to_solver_input, check_input`;
`from core.solvers import *`), with the MIP's LP relaxations solved by the gfx950 engine.
"""
from .utils import *  # noqa: F401,F403
