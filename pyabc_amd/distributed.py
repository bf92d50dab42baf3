"""One process per GPU: rank/world plumbing over torch.distributed.

Backend "nccl" (RCCL on ROCm, over xGMI) on the GPU box; "gloo" for the CPU
tests.  The generation path uses exactly three collectives per generation
(engine.py): all-gather of the accepted rows (theta, distance, weight),
all-reduce of the evaluation count, and an all-gather of per-rank row counts
that sizes the first one.  Everything after the gather (weight
normalisation, fit, epsilon) is computed redundantly and deterministically
on every rank from identical inputs, so no further exchange is needed.
"""
import os

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank=0, world=1, group=None):
        self.rank = rank
        self.world = world
        self.group = group

    @staticmethod
    def single():
        return Comm(0, 1, None)

    @staticmethod
    def from_env(backend=None, device=None):
        """Initialise from torchrun's RANK / WORLD_SIZE / LOCAL_RANK.

        ``device`` overrides the GPU of this rank (default LOCAL_RANK); a
        rehearsal of the multi-rank path on a one-GPU box puts every rank on
        device 0 with the "gloo" backend."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world == 1:
            return Comm.single()
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl" or device is not None:
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0"))
                                      if device is None else device)
            dist.init_process_group(backend=backend)
        return Comm(dist.get_rank(), dist.get_world_size(), None)

    @property
    def _host_staged(self):
        # gloo's all_gather takes host tensors only
        return dist.get_backend() == "gloo"

    @property
    def active(self):
        return self.world > 1

    def barrier(self):
        if self.active:
            dist.barrier()

    def all_gather_rows(self, t):
        """Concatenate each rank's rows (possibly different counts) in rank
        order."""
        if not self.active:
            return t
        if self._host_staged and t.is_cuda:
            return self.all_gather_rows(t.cpu()).to(t.device)
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        mx = max(sizes)
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        pad[:t.shape[0]] = t
        bufs = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(bufs, pad.contiguous())
        return torch.cat([b[:s] for b, s in zip(bufs, sizes)])

    def all_reduce_int(self, v):
        if not self.active:
            return int(v)
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() and \
            dist.get_backend() == "nccl" else torch.device("cpu")
        x = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        dist.all_reduce(x)
        return int(x.item())

    def all_reduce_max_float(self, v):
        if not self.active:
            return float(v)
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() and \
            dist.get_backend() == "nccl" else torch.device("cpu")
        x = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return float(x.item())
