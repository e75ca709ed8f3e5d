import sys; sys.path[:0]=["/root/repo/neptune-mip_amd","/root/repo","/root/repo/tests"]
import ctypes, numpy as np
from gpu_cases import build_args
import ref_pdhg as R
from core.engine.lp import LPModel, _ptr
np.set_printoptions(precision=6, linewidth=200)
for case in sys.argv[1:]:
    name, k = case.rsplit("__", 1); k = int(k)
    data, variant, step, kw = build_args(name, k)
    m = LPModel(data, variant, step=step, max_batch=1, **kw)
    ref = R.RefModel(data, variant, step=step, **kw)
    print("==", case, "n_int", m.n_int, "R", m.info.n_rows, "eta", m.info.step_size, ref.eta)
    for it in [1, 2, 3, 64, 128]:
        res = m.solve([0], max_iters=it, check_every=1)
        d = m.diag(0)
        y = np.zeros(ref.n_dual); kz = np.zeros(ref.n_dual); lb = np.zeros(m.n_int); ub = np.zeros(m.n_int)
        m._lib.nep_debug_state(m._h, 0, _ptr(y), _ptr(kz), None, _ptr(lb), _ptr(ub))
        z, x = m.solution(0)
        print(f"it={it} res={ {k2: res[k2][0] for k2 in res} }")
        print("  diag", {k2: round(v, 6) if isinstance(v, float) else v for k2, v in d.items()})
        print("  z", z, "lb", lb, "ub", ub)
        print("  y", y)
        print("  kz", kz)
        print("  x", x.reshape(-1)[:16])
