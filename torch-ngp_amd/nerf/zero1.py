"""ZeRO-1 layout of the fused engine's data-parallel step (nerf/fused.py).

The reference trains data parallel through DDP (nerf/utils.py:325-327): every
rank all-reduces every gradient and runs the full Adam. Here the parameters,
their fp16 gradients and fp16 forward copies are each ONE flat buffer with the
same layout (tensor k at an 8-aligned start), padded to `world` equal chunks
of a multiple of 64 values; rank r owns chunk [r c, (r + 1) c). A step
reduce-scatters (average) the flat gradient into the owner's shard, the owner
runs Adam on its shard only, and the fp16 forward copy is all-gathered: per
rank the bytes of one all-reduce and 1/world of the optimizer sweep.

This module holds the layout arithmetic (host-only, no GPU): the fused
trainer builds its buffers and optimizer sections from it, and the CPU gloo
tests run the same plan through real collectives (tests/test_dp_gloo.py).
"""
import numpy as np


class ShardPlan:
    def __init__(self, sizes, world=1, rank=0, align=8, shard_align=64):
        assert world >= 1 and 0 <= rank < world
        self.sizes = [int(n) for n in sizes]
        self.world, self.rank = int(world), int(rank)
        starts = np.cumsum([0] + [(n + align - 1) // align * align for n in self.sizes])
        self.starts = [int(a) for a in starts[:-1]]
        self.used = int(starts[-1])
        # shard: a shard_align-aligned chunk per rank (world * chunk >= the layout)
        self.chunk = int(-(-self.used // (shard_align * self.world)) * shard_align)
        self.total = self.chunk * self.world
        self.lo, self.hi = self.rank * self.chunk, (self.rank + 1) * self.chunk

    def views(self, flat):
        """Views of tensor k's values in a flat buffer of this layout."""
        return [flat[a:a + n] for a, n in zip(self.starts, self.sizes)]

    def sections(self, split_first):
        """Optimizer sections of this rank's shard, (offset in the shard,
        length, has an fp16 forward copy). split_first (world 1, fp32 table
        read by the forward): the first tensor gets no fp16 copy, the rest do;
        otherwise one section with a copy."""
        if split_first:
            nt = self.starts[1]
            return [(0, nt, False), (nt, self.chunk - nt, True)]
        return [(0, self.chunk, True)]

    def owned(self, k):
        """[lo, hi) of tensor k's values that this rank owns (lo == hi: none),
        as offsets into the tensor."""
        a, n = self.starts[k], self.sizes[k]
        lo, hi = max(a, self.lo), min(a + n, self.hi)
        return (lo - a, hi - a) if lo < hi else (0, 0)
