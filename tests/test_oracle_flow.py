"""The oracle's two-step flow reproduces (a) the reference's committed SCIP output for test.py
(`output-mip.json`) and (b) the responses the reference code produced on every golden payload."""
import json
import os

import numpy as np
import pytest

from golden_util import golden, payload
from oracle.solve import run_flow

G = golden()
FLOW_CASES = [k for k, v in G.items() if "response" in v]


def _close_routing(a, b):
    assert set(a) == set(b)
    for s in a:
        assert set(a[s]) == set(b[s])
        for f in a[s]:
            assert set(a[s][f]) == set(b[s][f])
            for d in a[s][f]:
                assert abs(a[s][f][d] - b[s][f][d]) <= 1e-3


def test_testpy_matches_scip_output():
    got = run_flow(payload("testpy"))
    scip = G["testpy"]["scip_response"]
    assert abs(got["score"]["step1"] - scip["score"]["step1"]) <= 1e-6
    assert abs(got["score"]["step2"] - scip["score"]["step2"]) <= 1e-6
    assert got["cpu_allocations"] == scip["cpu_allocations"]
    _close_routing(got["cpu_routing_rules"], scip["cpu_routing_rules"])


@pytest.mark.parametrize("name", FLOW_CASES)
def test_flow_matches_reference_code(name):
    ref = G[name]["response"]
    got = run_flow(payload(name))
    for k in ("step1", "step2"):
        assert abs(got["score"][k] - ref["score"][k]) <= 1e-6 * max(1.0, abs(ref["score"][k])), k
    models = G[name]["models"]
    final_unique = False
    last = [m for m in models if m["status"] == 0]
    if last:
        final_unique = last[-1].get("mip_tied") is False
    if final_unique:
        assert got["cpu_allocations"] == ref["cpu_allocations"]
