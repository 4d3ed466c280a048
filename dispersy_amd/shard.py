"""One process per GPU for the sync path's data-parallel jobs.

- cfg2, the responder (`_get_packets_for_bloomfilters`, community.py:1000-1062): the claims of a batch are split in
  contiguous blocks over the ranks, the store is replicated; no collective touches the data path, the job's totals
  are one all-reduce (max of the ranks' times, sum of their pairs).
- cfg4, large filters (`BloomFilter.add_keys`, bloomfilter.py:176-183): the keys are split over the ranks, every rank
  ORs its shard into a partial filter, the partials are all-gathered and OR-ed on the GPU (dsy_filter_or_reduce) into
  the filter of all keys, identical on every rank.
- cfg3, the gossip simulator (sim.EpidemicSim): block-sharded peers, two all-to-all(v) exchanges per round.

`Collectives` runs these on the tensors' own device over RCCL (backend "nccl").  With a gloo group -- the CPU tests,
and the GPU tests' two ranks sharing one GPU -- device tensors are staged through host memory for the exchange
itself; the OR, the hashing and the tests stay on the GPU either way."""
from . import _native


def shard_range(n, rank, world):
    """[lo, hi) of rank's contiguous block of n units; the first n % world ranks hold one unit more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d outside a world of %d" % (rank, world))
    base, extra = divmod(int(n), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class Collectives(object):
    """The few collectives the sharded jobs use, over torch.distributed's default group (or `group`)."""

    def __init__(self, dist, group=None):
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host_staged = dist.get_backend(group) == "gloo"

    def _stage(self, t):
        return t.cpu() if self.host_staged and t.is_cuda else t

    def barrier(self):
        self.dist.barrier(group=self.group)

    def all_reduce(self, t, op="sum"):
        """In place; op "sum" or "max"."""
        reduce_op = self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MAX
        s = self._stage(t)
        self.dist.all_reduce(s, op=reduce_op, group=self.group)
        if s is not t:
            t.copy_(s)
        return t

    def scalar(self, value, op="sum", dtype=None, device=None):
        import torch
        dtype = dtype or (torch.float64 if isinstance(value, float) else torch.int64)
        t = torch.tensor([value], dtype=dtype, device=device)
        return self.all_reduce(t, op).item()

    def all_gather_into(self, out, t):
        """out (world * t.numel() elements, same dtype) = every rank's t, rank order."""
        so, st = self._stage(out), self._stage(t)
        if self.host_staged:
            parts = list(so.view(self.world, -1).unbind(0))
            self.dist.all_gather(parts, st.reshape(-1), group=self.group)
        else:
            self.dist.all_gather_into_tensor(so, st, group=self.group)
        if so is not out:
            out.copy_(so)
        return out

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        so, si = self._stage(out), self._stage(inp)
        self.dist.all_to_all_single(so, si, output_split_sizes=out_splits, input_split_sizes=in_splits,
                                    group=self.group)
        if so is not out:
            out.copy_(so)
        return out

    def all_gather_object(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out


def union_filter(ctx, coll, partial):
    """The OR of every rank's partial filter (int32 words on the device), on every rank: all-gather of the partials,
    then dsy_filter_or_reduce on the GPU.  The ctx stream and torch's stream (which the collective is ordered on)
    are chained by device events, both ways: the result is ready for torch work queued after the call."""
    import torch
    words = partial.numel()
    if coll is None or coll.world == 1:
        ctx.signal_torch(partial.device)  # the ctx kernels that built `partial` come first
        return partial.clone()
    ctx.signal_torch(partial.device)
    parts = torch.empty(coll.world * words, dtype=torch.int32, device=partial.device)
    coll.all_gather_into(parts, partial)
    union = torch.empty_like(partial)
    ctx.wait_torch(partial.device)
    _native.check(ctx.lib.dsy_filter_or_reduce(ctx.handle, parts.data_ptr(), coll.world, words, union.data_ptr()))
    ctx.signal_torch(partial.device)
    return union


def add_sharded(ctx, params, blob, offsets, n, coll, filt):
    """cfg4's build as a job: rank r adds keys shard_range(n, r, world) of the packed keys (blob, offsets: device
    uint8 / int64 tensors, key i = blob[offsets[i]:offsets[i + 1]]) into its partial filter `filt` (device int32
    words, zeroed by the caller or holding earlier adds), and returns the union of all ranks' partials."""
    import ctypes
    rank, world = (coll.rank, coll.world) if coll is not None else (0, 1)
    lo, hi = shard_range(n, rank, world)
    ctx.wait_torch(filt.device)  # torch work that filled or zeroed blob / offsets / filt comes first
    if hi > lo:
        _native.check(ctx.lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(params), blob.data_ptr(),
                                                offsets[lo:].data_ptr(), hi - lo, filt.data_ptr()))
    return union_filter(ctx, coll, filt)
