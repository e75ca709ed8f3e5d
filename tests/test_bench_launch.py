"""bench.py --gpus N starts N ranks itself (--gpus was never read, so a driver run of
`bench.py --gpus 8` measured one rank).  CPU-only: NEP_BENCH_PROBE_RANKS makes every rank join a gloo group,
report its replay entries and exit before any GPU work."""
import gzip
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks_one_instance_each():
    r = _run(["--gpus", "2"], {"NEP_BENCH_PROBE_RANKS": "6"})
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2
    ranks = sorted(out["ranks"], key=lambda d: d["rank"])
    assert [d["rank"] for d in ranks] == [0, 1] and all(d["world"] == 2 for d in ranks)
    for d in ranks:        # rank r replays the whole recorded trace of instance seed r (one B&B per GPU)
        assert d["seed"] == d["rank"]
        with gzip.open(os.path.join(REPO, "tests", "golden", f"bnb_trace_512x256_s{d['seed']}.json.gz"), "rt") as fh:
            lps = [e for e in json.load(fh)["lps"] if e["parent"] is not None]
        assert d["entries"] == len(lps)
        assert d["ids"] == [lps[q]["id"] for q in range(6)]


def test_launcher_world_must_match_gpus():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "NEP_BENCH_PROBE_RANKS": "1"})
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 1 rank" in r.stderr
