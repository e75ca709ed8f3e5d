"""EF-TTC heuristic solvers (reference `core/solvers/efttc`): host-side, not on the GPU LP path."""
from .efttc import EfttcBase, EfttcMinDelay, EfttcMinDelayAndUtilization, EfttcMinUtilization  # noqa: F401
from .efttc_step1 import (EfttcStep1CPUMinDelay, EfttcStep1CPUMinDelayAndUtilization,  # noqa: F401
                          EfttcStep1CPUMinUtilization)
