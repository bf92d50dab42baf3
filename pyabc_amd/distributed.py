"""One process per GPU: rank/world plumbing over torch.distributed.

Backend "nccl" (RCCL on ROCm, over xGMI) on the GPU box; "gloo" for the CPU
tests.  The generation path (engine.py) exchanges, per sampling round, the per-rank
in-support and accepted counts (two R-int all-gathers: they assign global
evaluation ids and find the n-th acceptance), and once per generation the
accepted rows (theta, distance; all-gather), the evaluation count
(all-reduce) and the KDE log-densities of each rank's row slice
(all-gather).  Everything after that (weight normalisation, fit, epsilon) is
computed redundantly and deterministically on every rank from identical
inputs, so no further exchange is needed.
"""
import math
import os

import torch
import torch.distributed as dist


def _copy_rows(dst, src):
    """dst[:] = src, rows of 8-byte words: the library's strided word copy on
    the device (no torch kernel); a plain copy for host tensors."""
    if src.shape[0] == 0:
        return dst
    if dst.is_cuda and src.element_size() == 8:
        from . import kernels as K
        K.gather_words(src.reshape(src.shape[0], -1), None, src.shape[0],
                       dst.view(dst.shape[0], -1))
    else:
        dst.copy_(src)
    return dst


def _cat_rows(pieces, like):
    """Row pieces back to back in one new tensor (torch.cat through
    :func:`_copy_rows`)."""
    n = sum(int(p.shape[0]) for p in pieces)
    out = like.new_empty((n,) + tuple(like.shape[1:]))
    r = 0
    for p in pieces:
        _copy_rows(out[r:r + p.shape[0]], p)
        r += p.shape[0]
    return out


class Comm:
    def __init__(self, rank=0, world=1, group=None, force=False):
        self.rank = rank
        self.world = world
        self.group = group
        # a one-rank process group whose collectives still run (the RCCL
        # self-test on a one-GPU box: ABC_COMM_FORCE=1 under torchrun)
        self.force = force

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
        force = os.environ.get("ABC_COMM_FORCE") == "1"
        if world == 1 and not force:
            return Comm.single()
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl" or device is not None:
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0"))
                                      if device is None else device)
            dist.init_process_group(backend=backend)
        return Comm(dist.get_rank(), dist.get_world_size(), None, force)

    @staticmethod
    def current():
        """The already-initialised process group (or a single rank)."""
        force = os.environ.get("ABC_COMM_FORCE") == "1"
        if dist.is_available() and dist.is_initialized() and \
                (dist.get_world_size() > 1 or force):
            return Comm(dist.get_rank(), dist.get_world_size(), None, force)
        return Comm.single()

    def broadcast_int(self, v, src=0):
        """Rank ``src``'s int on every rank."""
        if not self.active:
            return int(v)
        x = torch.tensor([int(v)], dtype=torch.int64, device=self._int_dev())
        dist.broadcast(x, src)
        return int(x.item())

    @property
    def _host_staged(self):
        # gloo's all_gather takes host tensors only
        return dist.get_backend() == "gloo"

    @property
    def active(self):
        return self.world > 1 or self.force

    def barrier(self):
        if self.active:
            dist.barrier()

    def all_gather_rows(self, t, sizes=None):
        """Concatenate each rank's rows (possibly different counts) in rank
        order.  ``sizes`` (every rank's row count, when the caller knows
        them) saves the count exchange."""
        if not self.active:
            return t
        if self._host_staged and t.is_cuda:
            return self.all_gather_rows(t.cpu(), sizes).to(t.device)
        if sizes is None:
            sizes = self.all_gather_ints(t.shape[0])
        assert sizes[self.rank] == t.shape[0], "all_gather_rows: bad sizes"
        mx = max(sizes)
        # every rank's (padded) block into ONE tensor, then the valid
        # prefixes back to back through the library's copy on the device
        # (the padding rows are never read: no fill); the gloo rehearsals
        # run the same path on host tensors
        pad = t
        if t.shape[0] != mx or not t.is_contiguous():
            pad = t.new_empty((mx,) + tuple(t.shape[1:]))
            _copy_rows(pad[:t.shape[0]], t)
        out = t.new_empty((self.world * mx,) + tuple(t.shape[1:]))
        dist.all_gather_into_tensor(out, pad)
        if all(c == mx for c in sizes):
            return out
        return _cat_rows([out[r * mx:r * mx + c]
                          for r, c in enumerate(sizes)], t)

    def _int_dev(self):
        return torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() and \
            dist.get_backend() == "nccl" else torch.device("cpu")

    def all_gather_ints(self, v):
        """[v_0, ..., v_{R-1}] from every rank's int (or 1-element tensor)."""
        if not self.active:
            return [int(v.item()) if torch.is_tensor(v) else int(v)]
        dev = self._int_dev()
        x = v.reshape(1).to(device=dev, dtype=torch.int64) if torch.is_tensor(v) \
            else torch.tensor([int(v)], dtype=torch.int64, device=dev)
        out = torch.empty(self.world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, x)   # one tensor: no concatenation
        return [int(a) for a in out.cpu().tolist()]              # one sync

    def all_gather_int_lists(self, vals):
        """Every rank's equal-length int list, indexed [rank][k]."""
        if not self.active:
            return [list(vals)]
        dev = self._int_dev()
        x = torch.tensor(list(vals), dtype=torch.int64, device=dev)
        out = torch.empty(self.world * x.numel(), dtype=torch.int64,
                          device=dev)
        dist.all_gather_into_tensor(out, x)   # one tensor: no stacking
        return out.cpu().view(self.world, -1).tolist()           # one sync

    def all_reduce_ints(self, vals):
        """Element-wise sum over ranks of an int list (one collective)."""
        if not self.active:
            return [int(v) for v in vals]
        x = torch.tensor([int(v) for v in vals], dtype=torch.int64,
                         device=self._int_dev())
        dist.all_reduce(x)
        return [int(a) for a in x.cpu().tolist()]

    def all_reduce_int(self, v):
        if not self.active:
            return int(v)
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() and \
            dist.get_backend() == "nccl" else torch.device("cpu")
        x = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        dist.all_reduce(x)
        return int(x.item())

    def all_reduce_words(self, x, op):
        """In-place all-reduce of an int64 device view (op 1 sum, 2 max,
        3 min, 4 max of x[0] and min of x[1]); gloo stages through host."""
        if not self.active:
            return
        ops = {1: dist.ReduceOp.SUM, 2: dist.ReduceOp.MAX,
               3: dist.ReduceOp.MIN}
        staged = self._host_staged and x.is_cuda
        y = x.cpu() if staged else x   # RCCL reduces the view in place
        if op == 4:
            dist.all_reduce(y[0:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(y[1:2], op=dist.ReduceOp.MIN)
        else:
            dist.all_reduce(y, op=ops[op])
        if staged:
            x.copy_(y)

    def all_reduce_max_float(self, v):
        if not self.active:
            return float(v)
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() and \
            dist.get_backend() == "nccl" else torch.device("cpu")
        x = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return float(x.item())


def env_rank():
    """This process's rank from the torchrun environment (before or without
    an initialised process group)."""
    return int(os.environ.get("RANK", "0"))


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1"))


def agree_int(v):
    """Rank 0's value of a host decision on every rank (seeds, adapted
    population sizes: anything the ranks' collectives depend on).  A single
    process returns ``v``; under torchrun the process group is initialised
    on first use."""
    if env_world() == 1:
        return int(v)
    return Comm.from_env().broadcast_int(v)


class RankSliceComm(Comm):
    """Rank 0 of an R-rank job, emulated in ONE process on one GPU
    (``bench.py --rank-slice R``): the engine runs exactly rank 0's share of
    a generation -- its B/R proposals per sampling round, its M/R rows of
    the KDE pass against the full population, and every full-population
    stage each rank repeats -- while the other R-1 ranks are taken to be
    statistically identical to this one:

    * count all-gathers return R copies of this rank's count, sums are R
      times this rank's value, maxima / minima are this rank's own;
    * a row all-gather returns this rank's rows in every other rank's slot
      (shape and byte count of the real exchange, the contents of a
      replicated population);
    * the weighted-quantile histogram all-reduces (SUM) multiply by R.

    Nothing crosses a link, so every collective is counted instead
    (``log``: kind, payload bytes this rank sends, bytes it receives), for
    the xGMI model in DESIGN.md section 5.  Measurement infrastructure: the
    generation it produces is a valid population but not the R-rank one."""

    def __init__(self, world):
        super().__init__(0, int(world), None, force=True)
        self.log = []

    def _note(self, kind, sent, recv):
        self.log.append((kind, int(sent), int(recv)))

    @property
    def _host_staged(self):
        return False

    def barrier(self):
        self._note("barrier", 0, 0)

    def broadcast_int(self, v, src=0):
        self._note("broadcast", 8, 8)
        return int(v)

    def all_gather_rows(self, t, sizes=None):
        R = self.world
        if sizes is None:
            sizes = self.all_gather_ints(t.shape[0])
        assert sizes[0] == t.shape[0], "all_gather_rows: bad sizes"
        row = math.prod(t.shape[1:]) * t.element_size()
        pieces = []
        for s in range(R):
            c = sizes[s]
            if c <= t.shape[0]:
                pieces.append(t[:c])
            elif t.shape[0] == 0:   # nothing to repeat: zero rows, same shape
                pieces.append(t.new_zeros((c,) + tuple(t.shape[1:])))
            else:   # more rows than this rank holds: repeat them
                reps = -(-c // t.shape[0])
                pieces.append(t.repeat((reps,) + (1,) * (t.dim() - 1))[:c])
        self._note("all_gather_rows", sizes[0] * row,
                   (sum(sizes) - sizes[0]) * row)
        return _cat_rows(pieces, t)

    def all_gather_ints(self, v):
        x = int(v.item()) if torch.is_tensor(v) else int(v)
        self._note("all_gather_ints", 8, 8 * (self.world - 1))
        return [x] * self.world

    def all_gather_int_lists(self, vals):
        n = len(vals)
        self._note("all_gather_int_lists", 8 * n, 8 * n * (self.world - 1))
        return [list(vals) for _ in range(self.world)]

    def all_reduce_ints(self, vals):
        self._note("all_reduce_ints", 8 * len(vals), 8 * len(vals))
        return [int(v) * self.world for v in vals]

    def all_reduce_int(self, v):
        self._note("all_reduce_int", 8, 8)
        return int(v) * self.world

    def all_reduce_words(self, x, op):
        self._note(f"all_reduce_words_op{op}", 8 * x.numel(), 8 * x.numel())
        if op == 1:
            x.mul_(self.world)

    def all_reduce_max_float(self, v):
        self._note("all_reduce_max_float", 8, 8)
        return float(v)

    def summary(self, since=0):
        """{kind: [calls, bytes sent, bytes received]} over log[since:]."""
        out = {}
        for kind, s, r in self.log[since:]:
            e = out.setdefault(kind, [0, 0, 0])
            e[0] += 1
            e[1] += s
            e[2] += r
        return out
