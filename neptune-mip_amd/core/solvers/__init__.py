"""Solver classes importable as in the reference (`core/solvers/__init__.py`): `from core.solvers
import *` exposes the NEPTUNE variants that `main.py` dispatches by name.

SOLVERS is the whitelist the REST entry point resolves `solver.type` through (the reference uses
`eval`, `main.py:44`).
"""
from .neptune import *  # noqa: F401,F403
from .efttc import *  # noqa: F401,F403
from .efttc import EfttcMinDelay, EfttcMinDelayAndUtilization, EfttcMinUtilization
from .neptune import (NeptuneMinDelay, NeptuneMinDelayAndUtilization, NeptuneMinUtilization,
                      NeptuneWithEFTTCMinDelay, NeptuneWithEFTTCMinDelayAndUtilization,
                      NeptuneWithEFTTCMinUtilization)
from .solver import Solver  # noqa: F401

SOLVERS = {
    "NeptuneMinDelayAndUtilization": NeptuneMinDelayAndUtilization,
    "NeptuneMinDelay": NeptuneMinDelay,
    "NeptuneMinUtilization": NeptuneMinUtilization,
    "NeptuneWithEFTTCMinDelay": NeptuneWithEFTTCMinDelay,
    "NeptuneWithEFTTCMinUtilization": NeptuneWithEFTTCMinUtilization,
    "NeptuneWithEFTTCMinDelayAndUtilization": NeptuneWithEFTTCMinDelayAndUtilization,
    "EfttcMinDelay": EfttcMinDelay,
    "EfttcMinUtilization": EfttcMinUtilization,
    "EfttcMinDelayAndUtilization": EfttcMinDelayAndUtilization,
}
