"""Wire format of the placement (reference `core/solvers/neptune/utils/output.py:23-39`).

routing[source][function][destination] = round(x, 3) for every x > 0.001 (all sources, including
zero-workload ones, `output-mip.json`); allocations[function][destination] = True for c > 0.001.
Vectorised: only the entries above the threshold are visited.
"""
import numpy as np


def convert_x_matrix(matrix, nodes, functions):
    if hasattr(matrix, "wire_entries"):
        # core.engine.routing.SparseRouting: the device-compacted entries, in the dense path's (i, f, j)
        # order and with its threshold / rounding, so the dict is the same byte for byte
        assert tuple(matrix.shape) == (len(nodes), len(functions), len(nodes))
        out = {}
        ii, ff, jj, vals = matrix.wire_entries(0.001)
        for i, f, j, v in zip(ii.tolist(), ff.tolist(), jj.tolist(), vals.tolist()):
            out.setdefault(nodes[i], {}).setdefault(functions[f], {})[nodes[j]] = float(v)
        return out
    matrix = np.asarray(matrix)
    assert matrix.shape == (len(nodes), len(functions), len(nodes)), (
        f"X matrix shape malformed. matrix shape is {matrix.shape} but it should be "
        f"{(len(nodes), len(functions), len(nodes))}")
    out = {}
    ii, ff, jj = np.nonzero(matrix > 0.001)
    vals = np.round(matrix[ii, ff, jj], 3)
    for i, f, j, v in zip(ii.tolist(), ff.tolist(), jj.tolist(), vals.tolist()):
        out.setdefault(nodes[i], {}).setdefault(functions[f], {})[nodes[j]] = float(v)
    return out


def convert_c_matrix(matrix, functions, nodes):
    matrix = np.asarray(matrix)
    assert matrix.shape == (len(functions), len(nodes)), (
        f"X matrix shape malformed. matrix shape is {matrix.shape} but it should be "
        f"{(len(functions), len(nodes))}")
    out = {}
    ff, jj = np.nonzero(matrix > 0.001)
    for f, j in zip(ff.tolist(), jj.tolist()):
        out.setdefault(functions[f], {})[nodes[j]] = True
    return out
