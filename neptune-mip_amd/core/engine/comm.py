"""Communicators for the sharded branch-and-bound.

The only exchanges of the multi-GPU search are latency-bound scalars: all-reduce(MIN) of the
incumbent bound, all-reduce(SUM) of open-node counts for termination, and one broadcast of the
winning placement.  `TorchComm` carries them over `torch.distributed` — RCCL over xGMI with the
"nccl" backend on MI355X (device tensors), gloo on CPU for the multi-process tests.  `LocalComm`
is the single-process identity.
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

    def bcast(self, arr, src):
        """Broadcast from the member of rank `src` WITHIN this communicator's group (torch's
        broadcast takes a global rank: mapped with get_global_rank for non-default groups)."""
        a = np.ascontiguousarray(arr)
        t = self._t.from_numpy(a.copy()).to(self.device)
        gsrc = src if self._g is None else self._d.get_global_rank(self._g, src)
        self._d.broadcast(t, src=gsrc, group=self._g)
        return t.cpu().numpy().reshape(a.shape)
