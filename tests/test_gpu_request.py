"""The reference's request boundary end to end on the MI355X engine (main.py:31-62, 69):
core.request.solve_request builds the response body the reference's Flask route returns, and it
works in a child forked — as the reference's Werkzeug server forks one per request — from a parent
that never touched the GPU."""
import json
import os
import subprocess
import sys

import pytest

from golden_util import golden, payload

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"cpu_routing_rules", "cpu_allocations", "gpu_routing_rules", "gpu_allocations", "score", "processing_time"}


def _check_payload_response(resp):
    ref = golden()["payload"]["response"]
    assert set(resp) == KEYS
    assert resp["gpu_routing_rules"] == {} and resp["gpu_allocations"] == {}
    assert isinstance(resp["processing_time"], float) and resp["processing_time"] >= 0.0
    for k in ("step1", "step2"):
        assert abs(resp["score"][k] - ref["score"][k]) <= 1e-6 * max(1.0, abs(ref["score"][k])), (resp["score"], ref["score"])
    # payload.json's step-2 optimum is unique: the whole wire format
    assert resp["cpu_allocations"] == ref["cpu_allocations"]
    assert set(resp["cpu_routing_rules"]) == set(ref["cpu_routing_rules"])
    for src, fns in ref["cpu_routing_rules"].items():
        for fn, dsts in fns.items():
            got = resp["cpu_routing_rules"][src][fn]
            assert set(got) == set(dsts), (src, fn, got, dsts)
            for dst, val in dsts.items():
                assert abs(got[dst] - val) <= 1e-3, (src, fn, dst, got[dst], val)
    json.dumps(resp)   # the body is JSON-serialisable as the reference's json.dumps requires


def test_request_response_matches_reference():
    from core.request import solve_request
    _check_payload_response(solve_request(payload("payload")))


_CHILD = r"""
import json, multiprocessing as mp, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
from golden_util import payload
from core.request import solve_request      # the engine library loads; no HIP call before the fork

def run(q):
    q.put(solve_request(payload("payload")))

ctx = mp.get_context("fork")
q = ctx.Queue()
p = ctx.Process(target=run, args=(q,))
p.start()
resp = q.get(timeout=300)
p.join(60)
print(json.dumps({"exitcode": p.exitcode, "resp": resp}))
"""


def test_request_in_forked_child():
    out = subprocess.run([sys.executable, "-c", _CHILD, os.path.join(REPO, "neptune-mip_amd"),
                          os.path.join(REPO, "tests")], capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["exitcode"] == 0
    _check_payload_response(r["resp"])
