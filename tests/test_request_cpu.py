"""The request boundary's input validation (reference main.py:35 `check_input(input)` runs before the
solver is built): malformed payloads raise the reference's AssertionError before any engine call, so
these run without a GPU."""
import copy

import pytest

from golden_util import payload


def _no_engine(monkeypatch):
    import core.request as rq

    class Boom(dict):
        def __getitem__(self, k):
            raise RuntimeError("engine reached before check_input")
    monkeypatch.setattr(rq, "SOLVERS", Boom())
    return rq


@pytest.mark.parametrize("mutate", [
    lambda p: p.pop("node_names"),
    lambda p: p["function_memories"].append(1),
    lambda p: p["node_memories"].pop(),
])
def test_malformed_payload_rejected_before_engine(monkeypatch, mutate):
    rq = _no_engine(monkeypatch)
    p = copy.deepcopy(payload("payload"))
    mutate(p)
    with pytest.raises(AssertionError):
        rq.solve_request(p)


def test_valid_payload_passes_check(monkeypatch):
    rq = _no_engine(monkeypatch)
    with pytest.raises(RuntimeError, match="engine reached"):
        rq.solve_request(copy.deepcopy(payload("payload")))
