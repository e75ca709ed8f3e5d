#!/usr/bin/env python3
"""One entry point for the dev probes (tools/probes/*.py): measurement and diagnosis scripts of the DESIGN.md
sections that cite them, run on the GPU box through tools/gpu/run.sh (`py:<probe>,<args>`) or here.

  python3 tools/probe.py list                 every probe with the first line of its docstring
  python3 tools/probe.py <name> [args...]     run tools/probes/<name>.py with those arguments
"""
import ast
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PROBES = os.path.join(HERE, "probes")


def probes():
    out = {}
    for fn in sorted(os.listdir(PROBES)):
        if fn.endswith(".py"):
            with open(os.path.join(PROBES, fn)) as fh:
                doc = ast.get_docstring(ast.parse(fh.read())) or ""
            out[fn[:-3]] = doc.strip().splitlines()[0] if doc.strip() else ""
    return out


def main():
    if len(sys.argv) < 2 or sys.argv[1] in ("list", "-h", "--help"):
        for name, line in probes().items():
            print(f"{name:22s} {line}")
        return
    name = sys.argv[1][:-3] if sys.argv[1].endswith(".py") else sys.argv[1]
    path = os.path.join(PROBES, name + ".py")
    if not os.path.exists(path):
        raise SystemExit(f"no probe {name!r} (python3 tools/probe.py list)")
    sys.argv = [path] + sys.argv[2:]
    runpy.run_path(path, run_name="__main__")


if __name__ == "__main__":
    main()
