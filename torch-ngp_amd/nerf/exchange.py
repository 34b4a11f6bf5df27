"""Touched-entry gradient exchange of the replicated data-parallel step
(FusedTrainer options sparse_exchange=True; DESIGN.md §7 option B).

The reference trains data parallel through DDP (nerf/utils.py:325-327): every
rank all-reduces every gradient and runs the full Adam. The fused engine's
backward leaves the hash-table gradient a few percent dense (live rows x 16
levels x 8 corners), so each rank instead

  1. lists its nonzero fp16 channel pairs (`ngp_grad_exchange_list`): one
     fixed-size int64 buffer of a header (count, flags), a table of where
     each 4096-pair bin's items start, and up to `cap` items
     (half2 bits << 32 | pair index);
  2. all-gathers the buffers (one collective of a fixed size: no host round
     trip, so the exchange is captured in the step's graph);
  3. sums every rank's items of a bin in LDS in int64 2^-24 fixed point
     (`ngp_grad_exchange_reduce`; exact, so the order does not matter) and
     writes the bin of its flat gradient densely as fp16(sum / world).

Every rank then holds the same averaged gradient bit for bit and runs the
world-1 step's full Adam on it (inside the next march launch), so the
parameters stay identical with no parameter collective at all. A rank's
GradScaler flag (a non-finite gradient) travels in its header and is raised on
every rank, so every rank skips the same steps. The lists hold every pair by
default, so none can overflow; `fit` (FusedTrainer.fit_exchange) sizes them
to a margin over the longest list of the steps since the last fit, once
training is in its steady regime. A list longer than that is seen by every
rank in the gathered headers: every rank then skips the update (without a
scale back-off) and counts it in `overflows`, which the bench requires to be
0 over its timed region. `check` (run by FusedTrainer.flush, i.e. at every
density update, checkpoint and read-out) reads that count: after a new
overflow it warns and grows the lists to twice the longest list seen (and at
least twice their capacity), and the trainer captures its graphs again.

Per step a rank sends its list buffer (8 bytes per item of capacity) and
receives the other ranks'; the dense ZeRO-1 step (nerf/zero1.py) moves
2 x (world - 1) / world of the flat fp16 buffer instead (byte counts in
DESIGN.md §7).
"""
import warnings

import torch
import torch.distributed as dist

import _ngp_native as nat


class SparseExchange:
    def __init__(self, flat_grad, inf_flag, world, nccl, cap=None):
        """flat_grad: this rank's flat fp16 gradient (n % 8 == 0); inf_flag:
        device address of the GradScaler flag the optimizer reads (the rank's
        backward kernels raise it; the exchange raises it on every rank when
        any rank's is raised); nccl: collectives on device tensors (gloo:
        staged through the host); cap: items per list (default: every pair,
        so no list can overflow; `fit` resizes it to what the steps list)."""
        assert flat_grad.dtype == torch.float16 and flat_grad.numel() % 8 == 0
        self.grad, self.n = flat_grad, flat_grad.numel()
        self.inf_flag, self.world, self.nccl = inf_flag, int(world), bool(nccl)
        self.pairs = self.n // 2
        self.n_bins = int(nat.lib().ngp_grad_exchange_bins(self.n))
        # device: [overflowed exchanges, the largest list seen]
        self.stats = torch.zeros(2, dtype=torch.int32, device=flat_grad.device)
        self.seen_overflows = 0  # overflows `check` has already answered
        self.grown = 0           # resizes `check` made
        self.resize(cap if cap is not None else self.pairs)

    def resize(self, cap):
        """Items per list (the fixed size every step all-gathers): a step
        whose list on some rank is longer skips its update on every rank (see
        csrc/exchange.hip). Graphs captured before hold the old buffers:
        capture again after a resize."""
        self.cap = int(min(max(cap, 1), self.pairs))
        self.words = int(nat.lib().ngp_grad_exchange_words(self.n, self.cap))
        dev = self.grad.device
        self.send = torch.zeros(self.words, dtype=torch.int64, device=dev)
        self.recv = torch.zeros(self.world * self.words, dtype=torch.int64, device=dev)

    def fit(self, margin=2.0):
        """Resize the lists to margin x the longest list any rank has sent
        since the last fit (a host read of the device statistics, the same on
        every rank: they are the gathered headers'), and restart the
        statistics; returns the new cap."""
        peak = int(self.stats[1])
        if peak > 0:
            self.resize(int(peak * margin) + 1024)
        self.stats.zero_()
        self.seen_overflows = 0
        return self.cap

    def reset_stats(self):
        """Restart the statistics (the longest list, the overflow count), so a
        later `fit` sizes the lists on the steps after this call only."""
        self.stats.zero_()
        self.seen_overflows = 0

    def check(self):
        """After an overflow since the last check (a host read of the device
        statistics, the same on every rank: they come from the gathered
        headers), warn and grow the lists to 2 x the longest list seen and at
        least 2 x the old capacity. Returns True when it resized (graphs that
        hold the old buffers must be captured again)."""
        over, peak = (int(v) for v in self.stats.tolist())
        if over <= self.seen_overflows:
            return False
        self.seen_overflows = over
        if self.cap >= self.pairs:
            return False
        old = self.cap
        self.resize(max(2 * peak + 1024, 2 * old))
        self.grown += 1
        warnings.warn(f"SparseExchange: {over} update(s) skipped since the lists overflowed (longest list {peak} > "
                      f"capacity {old}); lists grown to {self.cap} items", RuntimeWarning, stacklevel=3)
        return True

    @property
    def overflows(self):
        """Exchanges (steps) whose update was skipped because a list overflowed."""
        return int(self.stats[0])

    def bytes_per_step(self):
        """Bytes one rank sends (its whole list buffer) and receives."""
        return 8 * self.words, 8 * self.words * (self.world - 1)

    def __call__(self):
        """Exchange this step's gradient (after the backward wrote it, before
        the optimizer reads it). No host round trip: capturable (RCCL)."""
        self.list()
        if self.nccl:
            dist.all_gather_into_tensor(self.recv, self.send)
        else:
            host = torch.empty(self.recv.shape, dtype=self.recv.dtype)
            dist.all_gather_into_tensor(host, self.send.cpu())
            self.recv.copy_(host)
        self.reduce()

    # ---- the kernels (csrc/exchange.hip; the CPU tests restate them) -------
    def list(self):
        lib, P = nat.lib(), nat.ptr
        nat.check(lib.ngp_grad_exchange_list(P(self.grad), self.n, self.inf_flag, P(self.send), self.cap,
                                             nat.stream_of(self.grad)), "grad_exchange_list")

    def reduce(self):
        lib, P = nat.lib(), nat.ptr
        nat.check(lib.ngp_grad_exchange_reduce(P(self.recv), self.world, self.cap, P(self.grad), self.n,
                                               self.inf_flag, P(self.stats), P(self.send), nat.stream_of(self.grad)),
                  "grad_exchange_reduce")
