"""Communicators for the sharded branch-and-bound.

The only exchanges of the multi-GPU search are latency-bound scalars and one placement:
  * `agree(inc, stop, open)` — once per B&B loop, ONE collective (an all-gather of 3 numbers per rank):
    the incumbent bound (MIN), whether any rank hit its limit (OR) and the open + in-flight node count
    (SUM);
  * `gather(values)` — the end-of-search summary (bounds, flags, counters) in one collective;
  * `bcast` — the winning placement from its owner (the integer vector and the compacted routing
    entries, never the dense x).
`TorchComm` carries them over `torch.distributed` — RCCL over xGMI with the "nccl" backend on MI355X
(device tensors), gloo on CPU for the multi-process tests.  `LocalComm` is the single-process identity.
"""
import numpy as np


class LocalComm:
    rank, world = 0, 1

    def min(self, v):
        return float(v)

    def max(self, v):
        return float(v)

    def sum(self, v):
        return int(v)

    def agree(self, inc, stop, open_n):
        return float(inc), bool(stop), int(open_n)

    def gather(self, values):
        return np.asarray(values, np.float64).reshape(1, -1)

    def bcast(self, arr, src):
        return arr


class TorchComm:
    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self._t, self._d, self._g = torch, dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None:
            device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        self.device = device

    def _reduce(self, v, op, dtype):
        t = self._t.tensor([v], dtype=dtype, device=self.device)
        self._d.all_reduce(t, op=op, group=self._g)
        return t.item()

    def min(self, v):
        return float(self._reduce(float(v), self._d.ReduceOp.MIN, self._t.float64))

    def max(self, v):
        return float(self._reduce(float(v), self._d.ReduceOp.MAX, self._t.float64))

    def sum(self, v):
        return int(self._reduce(int(v), self._d.ReduceOp.SUM, self._t.int64))

    def gather(self, values):
        """[world, k] float64: every rank's `values` (one all-gather, one host sync)."""
        t = self._t.tensor(np.asarray(values, np.float64).ravel(), dtype=self._t.float64, device=self.device)
        out = [self._t.empty_like(t) for _ in range(self.world)]
        self._d.all_gather(out, t, group=self._g)
        return self._t.stack(out).cpu().numpy()

    def agree(self, inc, stop, open_n):
        g = self.gather([inc, 1.0 if stop else 0.0, float(open_n)])
        return float(g[:, 0].min()), bool(g[:, 1].max() > 0), int(round(g[:, 2].sum()))

    def bcast(self, arr, src):
        """Broadcast from the member of rank `src` WITHIN this communicator's group (torch's
        broadcast takes a global rank: mapped with get_global_rank for non-default groups)."""
        a = np.ascontiguousarray(arr)
        t = self._t.from_numpy(a.copy()).to(self.device)
        gsrc = src if self._g is None else self._d.get_global_rank(self._g, src)
        self._d.broadcast(t, src=gsrc, group=self._g)
        return t.cpu().numpy().reshape(a.shape)
