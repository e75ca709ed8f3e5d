"""Helpers to read the committed golden fixtures (tests/golden, made by tools/gen_golden.py)."""
import json
import os

import numpy as np
import scipy.sparse as sp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def payload(name):
    with open(os.path.join(GOLDEN, "inputs", f"{name}.json")) as f:
        return json.load(f)


def model(name, k):
    z = np.load(os.path.join(GOLDEN, "models", f"{name}__{k}.npz"))
    A = sp.csr_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=tuple(z["A_shape"]))
    out = {k2: z[k2] for k2 in z.files if not k2.startswith("A_")}
    out["A"] = A
    return out


def model_names():
    out = []
    for fn in sorted(os.listdir(os.path.join(GOLDEN, "models"))):
        name, k = fn[:-4].rsplit("__", 1)
        out.append((name, int(k)))
    return out
