"""Multi-GPU epidemic-sync simulator (BASELINE config 3): many peers run Dispersy's Bloom-filter sync against each
other, round after round, sharded over the GPUs of one node.

Every round each peer
  1. claims: builds its MTU bloom filter over the packets it holds (community.py:808-821) with a fresh 1-byte
     prefix and sends it to a partner chosen by a counter-based RNG (the walker's role, community.py:1209-1221);
  2. responds: for every claim it receives, returns its packets the filter lacks, in global-time order, until
     the 5 KiB budget is spent (community.py:2555-2567);
  3. stores what it received (Dispersy._store, dispersy.py:1475-1532).

Peers are block-sharded over ranks (one process per GPU).  The two exchanges of a round -- claims to the
responders' ranks, responses back -- are all-to-all(v) collectives over RCCL (torch.distributed "nccl"); the
record counts travel first in a small all-to-all.  Pairing, prefixes and initial stores come from splitmix64 of
(seed, round, peer), so the outcome is identical at 1, 2, 4 or 8 GPUs.

The per-rank work runs in an *engine*: `GpuEngine` calls the HIP kernels through the C-ABI (dsy_sim_* in
include/dsybloom.h).  Tests can pass the CPU engine of oracle/sim_ref.py to exercise the distributed logic with
the gloo backend.
"""
import ctypes
import math

import numpy as np

from . import _native
from .bloomfilter import BloomFilter
from .shard import Collectives


class SimConfig(ctypes.Structure):
    _fields_ = [("n_peers", ctypes.c_uint64), ("peer_begin", ctypes.c_uint64), ("peer_end", ctypes.c_uint64),
                ("peers_per_rank", ctypes.c_uint64), ("universe", ctypes.c_uint32), ("words", ctypes.c_uint32),
                ("m_bits", ctypes.c_uint64), ("k", ctypes.c_uint32), ("hash_kind", ctypes.c_int32),
                ("chunk_bytes", ctypes.c_uint32), ("capacity", ctypes.c_uint32), ("byte_limit", ctypes.c_int64),
                ("seed", ctypes.c_uint64), ("claim_bytes", ctypes.c_uint32), ("resp_bytes", ctypes.c_uint32)]


def make_config(n_peers, universe, rank, world, bits=10160, error_rate=0.01, byte_limit=5120, seed=11, chunks=1):
    """The claim filter is the community's MTU filter (community.py:637-666, f = 0.01 -> MD5, k = 7).  chunks: the
    rank's peers split into that many equal chunks for the overlapped round (EpidemicSim.chunks), so the block size
    is rounded up to a multiple of it (the outcome does not depend on the split)."""
    probe = BloomFilter(bits, error_rate)
    ppr = int(math.ceil(n_peers / float(world)))
    ppr = (ppr + chunks - 1) // chunks * chunks
    c = SimConfig()
    c.n_peers, c.peers_per_rank = n_peers, ppr
    c.peer_begin, c.peer_end = min(n_peers, rank * ppr), min(n_peers, (rank + 1) * ppr)
    c.universe = universe
    c.words = (universe + 31) // 32
    c.m_bits, c.k = probe.size, probe.functions
    c.hash_kind, c.chunk_bytes = _native.HASH_KINDS[probe.hash_name], probe.chunk_bytes
    c.capacity = probe.get_capacity(error_rate)
    c.byte_limit = byte_limit
    c.seed = seed
    c.claim_bytes = (32 + ((c.m_bits + 31) // 32) * 4 + 15) // 16 * 16
    c.resp_bytes = (16 + 2 * 64 + 15) // 16 * 16
    return c


def make_universe(universe, seed=11, lo=100, hi=1500):
    """The packet universe (identical on every rank): lengths ~ U[lo, hi], random bytes, global_time = id + 1."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = rng.integers(lo, hi + 1, size=universe, dtype=np.int64)
    offsets = np.zeros(universe + 1, dtype=np.uint64)
    np.cumsum(lengths, out=offsets[1:])
    return rng.bytes(int(offsets[-1])), offsets


class GpuEngine(object):
    """Per-rank simulator state in HBM + the dsy_sim_* kernels.  A round's calls only enqueue on the ctx stream (no
    host wait); the claim / response buffers are the engine's own, grow-only, reused every round, so no buffer a
    queued kernel still reads is ever handed back to torch's allocator."""

    MATRIX_ROUNDS = 16  # claim matrices computed per dsy_sim_claim_matrix call

    def __init__(self, cfg, blob, offsets, device, ctx=None):
        import torch
        self.torch = torch
        self.cfg = cfg
        self.dev = device
        self.ctx = ctx or _native.Context(device.index if device.index is not None else 0)
        self.lib = self.ctx.lib
        _native.check(self.lib.dsy_sim_setup(ctypes.byref(cfg)))
        # a response holds at most DSY_SIM_RESP_MAX packets: every packet but the budget-crossing last one costs at
        # least the universe's shortest packet, so refuse a configuration that could overflow it (the merge's sticky
        # overflow flag, reported by dsy_sim_stats, stays as the backstop)
        lens = np.diff(np.asarray(offsets, dtype=np.int64))
        if len(lens) and cfg.byte_limit > 0:
            most = cfg.byte_limit // max(int(lens.min()), 1) + 1
            if most > _native.SIM_RESP_MAX:
                raise ValueError("byte_limit %d over packets of >= %d bytes allows %d packets per response; the "
                                 "simulator's responses hold %d" % (cfg.byte_limit, int(lens.min()), most,
                                                                     _native.SIM_RESP_MAX))
        G = _native.BLOB_GUARD
        full = bytearray(G) + bytearray(blob) + bytearray(G)
        self.ublob_t = torch.frombuffer(full, dtype=torch.uint8).to(device)
        self.ublob = self.ublob_t.data_ptr() + G
        self.uoff_t = torch.from_numpy(offsets.astype(np.int64)).to(device)
        local = cfg.peer_end - cfg.peer_begin
        self.bits = torch.zeros(max(local, 1) * cfg.words, dtype=torch.int32, device=device)
        torch.cuda.current_stream(device).synchronize()  # the uploads above ran on torch's stream
        self._bufs = {}
        self._matrix = {}
        self._tested_base = self._tested_ctx()

    def buffer(self, name, nbytes):
        """The engine's grow-only device buffer `name`, at least nbytes long (a view of exactly nbytes)."""
        b = self._bufs.get(name)
        if b is None or b.numel() < nbytes:
            if b is not None:
                # queued kernels -- and an overlapped round's collectives on their own stream -- may still use the
                # old one
                self.ctx.synchronize()
                self.torch.cuda.synchronize(self.dev)
            b = self._bufs[name] = self.torch.empty(max(int(nbytes * 1.25), 1), dtype=self.torch.uint8, device=self.dev)
        return b[:max(nbytes, 1)]

    def seed(self, initial):
        _native.check(self.lib.dsy_sim_seed(self.ctx.handle, ctypes.byref(self.cfg), self.bits.data_ptr(), initial))
        self.ctx.synchronize()

    def claim_counts(self, rnd, world):
        out = (ctypes.c_uint32 * world)()
        _native.check(self.lib.dsy_sim_claim_counts(self.ctx.handle, ctypes.byref(self.cfg), rnd, out, world))
        return np.array(out, dtype=np.int64)

    def claim_matrix(self, rnd, world):
        """[src, dst] claims of round rnd, every rank (dsy_sim_claim_matrix: one call per MATRIX_ROUNDS rounds, on a
        second stream, so it does not wait for the queued rounds)."""
        key = (rnd, world)
        if key not in self._matrix:
            n = self.MATRIX_ROUNDS
            out = np.zeros(n * world * world, dtype=np.uint32)
            _native.check(self.lib.dsy_sim_claim_matrix(self.ctx.handle, ctypes.byref(self.cfg), rnd, n,
                                                        out.ctypes.data, world))
            self._matrix = {(rnd + i, world): out[i * world * world:(i + 1) * world * world].reshape(world, world)
                            .astype(np.int64) for i in range(n)}
        return self._matrix[key]

    def chunk_cfg(self, j, cs):
        """The config of chunk j (cs peers) of this rank's peers, as a rank of its own: its peers, and cs as the block
        size, so the kernels group its claims by destination CHUNK (a virtual rank)."""
        c = SimConfig.from_buffer_copy(self.cfg)
        c.peer_begin = min(self.cfg.peer_end, self.cfg.peer_begin + j * cs)
        c.peer_end = min(self.cfg.peer_end, c.peer_begin + cs)
        c.peers_per_rank = cs
        return c

    def claim_matrix_v(self, rnd, nv, cs):
        """[src, dst] claims of round rnd over virtual ranks of cs peers (nv of them), identical on every rank."""
        key = (rnd, nv, cs)
        if key not in self._matrix:
            n = self.MATRIX_ROUNDS
            c = SimConfig.from_buffer_copy(self.cfg)
            c.peers_per_rank = cs
            out = np.zeros(n * nv * nv, dtype=np.uint32)
            _native.check(self.lib.dsy_sim_claim_matrix(self.ctx.handle, ctypes.byref(c), rnd, n, out.ctypes.data, nv))
            self._matrix = {(rnd + i, nv, cs): out[i * nv * nv:(i + 1) * nv * nv].reshape(nv, nv).astype(np.int64)
                            for i in range(n)}
        return self._matrix[key]

    def build_claims_chunk(self, rnd, j, cs, offsets, total, buf):
        """Claims of chunk j's peers, grouped by destination chunk (offsets: one start per virtual rank)."""
        c = self.chunk_cfg(j, cs)
        if c.peer_end > c.peer_begin:
            offs = (ctypes.c_uint32 * len(offsets))(*[int(x) for x in offsets])
            bits = self.bits.data_ptr() + (c.peer_begin - self.cfg.peer_begin) * self.cfg.words * 4
            _native.check(self.lib.dsy_sim_build_claims(self.ctx.handle, ctypes.byref(c), rnd, self.ublob,
                                                        self.uoff_t.data_ptr(), bits, buf.data_ptr(), offs,
                                                        len(offsets)))
        return buf

    def build_claims(self, rnd, offsets, total, buf=None):
        buf = self.buffer("claims", total * self.cfg.claim_bytes) if buf is None else buf
        offs = (ctypes.c_uint32 * len(offsets))(*[int(x) for x in offsets])
        _native.check(self.lib.dsy_sim_build_claims(self.ctx.handle, ctypes.byref(self.cfg), rnd, self.ublob,
                                                    self.uoff_t.data_ptr(), self.bits.data_ptr(), buf.data_ptr(),
                                                    offs, len(offsets)))
        return buf

    def resp_counts(self, claims, n, world):
        out = (ctypes.c_uint32 * world)()
        _native.check(self.lib.dsy_sim_resp_counts(self.ctx.handle, ctypes.byref(self.cfg), claims.data_ptr(), n,
                                                   out, world))
        return np.array(out, dtype=np.int64)

    def respond(self, claims, n, offsets, total, buf=None):
        """(response buffer, None): the pairs tested stay on the device (tested_total)."""
        buf = self.buffer("resps", total * self.cfg.resp_bytes) if buf is None else buf
        offs = (ctypes.c_uint32 * len(offsets))(*[int(x) for x in offsets])
        _native.check(self.lib.dsy_sim_respond(self.ctx.handle, ctypes.byref(self.cfg), self.ublob,
                                               self.uoff_t.data_ptr(), self.bits.data_ptr(), claims.data_ptr(), n,
                                               buf.data_ptr(), offs, len(offsets), None))
        return buf, None

    def _tested_ctx(self):
        return int(self.ctx.work(_native.TIME_SIM_RESPOND)["useful_pairs"])

    def tested_total(self):
        """(claim, packet) pairs tested since this engine was built -- or since the ctx's counters were last reset
        (dsy_ctx_reset_timing), whichever is later.  The counter is the ctx's: give each engine its own ctx when
        several run at once."""
        now = self._tested_ctx()
        if now < self._tested_base:  # the ctx's counters were reset since
            self._tested_base = 0
        return now - self._tested_base

    def merge(self, resps, n):
        _native.check(self.lib.dsy_sim_merge(self.ctx.handle, ctypes.byref(self.cfg), self.bits.data_ptr(),
                                             resps.data_ptr(), n))

    def stats(self):
        out = (ctypes.c_uint64 * 2)()
        _native.check(self.lib.dsy_sim_stats(self.ctx.handle, ctypes.byref(self.cfg), self.bits.data_ptr(), out))
        return int(out[0]), int(out[1])

    def to_torch(self):
        """torch's current stream (RCCL's collectives are ordered on it) waits for the queued kernels."""
        self.ctx.signal_torch(self.dev)

    def from_torch(self):
        """The ctx stream waits for torch's current stream (a collective's output)."""
        self.ctx.wait_torch(self.dev)

    def wait_event(self, ev):
        """The ctx stream waits for a recorded torch.cuda.Event (one collective on the communication stream)."""
        self.ctx.wait_event(ev)

    def sync(self):
        self.ctx.synchronize()


class EpidemicSim(object):
    """Drives the rounds on one rank; `dist` is torch.distributed (or None for a single process).

    A round on rank q: the claim matrix M (computed identically on every rank, no count exchange) gives the send
    counts M[q] and receive counts M[:, q]; build -> all-to-all(v) of the claims -> respond -> all-to-all(v) of the
    responses (one per claim, so the counts reverse) -> merge.  The host never waits inside a round: the engine's
    kernels and the collectives are ordered on the device (to_torch / from_torch events around each exchange).

    chunks = C > 1 (cfg from make_config(..., chunks=C)): the round overlaps the exchanges with the kernels.  Each
    rank's peers are C chunks of cs = peers_per_rank / C peers, treated as virtual ranks in the claim matrix (world x C
    of them), so the counts per (source chunk, destination rank) come from the same kernel.  Chunk j's claims are built
    and sent while chunk j - 1's received claims are answered; the exchanges run on one communication stream (in the
    same order on every rank), the kernels on the engine's stream, each side waiting only for the one event it needs.
    Every merge runs after the round's last respond, so every response still reads the responders' stores before any
    merge of the round (the outcome is the unchunked round's, at any C and world)."""

    def __init__(self, engine, cfg, rank=0, world=1, dist=None, device=None, chunks=1, exchange_always=False):
        self.e, self.cfg, self.rank, self.world, self.dist = engine, cfg, rank, world, dist
        # exchange_always: run the collectives even at world 1 (a one-rank RCCL job exercises the exchange path)
        self.coll = Collectives(dist) if dist is not None and (world > 1 or exchange_always) else None
        self.device = device
        self._tested = 0
        self.exchanged_bytes = 0      # bytes this rank sent, itself included
        self.exchanged_remote = 0     # ... to other ranks
        if chunks > 1 and cfg.peers_per_rank % chunks:
            raise ValueError("peers_per_rank %d is not a multiple of chunks=%d (make_config(..., chunks=%d))"
                             % (cfg.peers_per_rank, chunks, chunks))
        self.chunks = chunks
        self._comm = None  # the communication stream of an overlapped round (RCCL on device buffers)

    @property
    def tested(self):
        if hasattr(self.e, "tested_total"):
            return self.e.tested_total()
        return self._tested

    def _exchange(self, name, buf, send_counts, recv_counts, rec_bytes):
        if self.coll is None:
            return buf
        in_splits = [int(c) * rec_bytes for c in send_counts]
        out_splits = [int(c) * rec_bytes for c in recv_counts]
        total_in = sum(out_splits)
        if hasattr(self.e, "buffer"):
            out = self.e.buffer(name, total_in)
        else:
            import torch
            out = torch.empty(max(total_in, 1), dtype=torch.uint8, device=self.device)
        to_torch, from_torch = getattr(self.e, "to_torch", None), getattr(self.e, "from_torch", None)
        if to_torch:
            to_torch()
        self.coll.all_to_all_single(out[:total_in], buf[:sum(in_splits)], out_splits, in_splits)
        if from_torch:
            from_torch()
        self._account(in_splits)
        return out

    def _round_chunked(self, rnd):
        c, e, W, C, me = self.cfg, self.e, self.world, self.chunks, self.rank
        cs = c.peers_per_rank // C
        nv = W * C
        Mv = e.claim_matrix_v(rnd, nv, cs)  # [source chunk, destination chunk]
        M4 = Mv.reshape(W, C, W, C)
        send = M4[me].sum(axis=2)           # send[j][d]: chunk j's claims to rank d
        recv = M4[:, :, me, :].sum(axis=2)  # recv[q][j]: claims from rank q's chunk j
        overlap = self._overlapped()
        if overlap:
            import torch
            if self._comm is None:
                self._comm = torch.cuda.Stream(device=self.device)
            comm = self._comm
        got = [None] * C   # (claims received from every rank's chunk j, how many)
        ev = [None] * C

        def exchange(name, buf, s_counts, r_counts, rec):
            in_splits = [int(x) * rec for x in s_counts]
            out_splits = [int(x) * rec for x in r_counts]
            self._account(in_splits)
            if self.coll is None:
                return buf
            total_in = sum(out_splits)
            out = e.buffer(name, total_in) if hasattr(e, "buffer") else self._host_buffer(total_in)
            if not overlap:
                if hasattr(e, "to_torch"):
                    e.to_torch()
                self.coll.all_to_all_single(out[:total_in], buf[:sum(in_splits)], out_splits, in_splits)
                if hasattr(e, "from_torch"):
                    e.from_torch()
                return out
            import torch
            e.ctx.signal_stream(comm)  # comm waits for what the engine has queued (this buffer's producer)
            with torch.cuda.stream(comm):
                self.coll.all_to_all_single(out[:total_in], buf[:sum(in_splits)], out_splits, in_splits)
            return out

        def record():
            import torch
            x = torch.cuda.Event()
            x.record(comm)
            return x

        def answer(j):
            if overlap:
                e.wait_event(ev[j])  # chunk j's claims have arrived (and nothing queued on comm after them)
            claims_in, n_in = got[j]
            rc = recv[:, j]
            poffs = np.concatenate([[0], np.cumsum(rc)[:-1]])
            resps, tested = e.respond(claims_in, n_in, poffs, n_in, **self._bufkw("resps%d" % j, n_in * c.resp_bytes))
            if tested is not None:
                self._tested += tested
            return exchange("resps_in%d" % j, resps, rc, send[j], c.resp_bytes)

        back = []
        for j in range(C):
            counts_v = Mv[me * C + j]
            offs = np.concatenate([[0], np.cumsum(counts_v)[:-1]])
            n_out = int(counts_v.sum())
            buf = e.build_claims_chunk(rnd, j, cs, offs, n_out, self._buf("claims%d" % j, n_out * c.claim_bytes))
            got[j] = (exchange("claims_in%d" % j, buf, send[j], recv[:, j], c.claim_bytes), int(recv[:, j].sum()))
            if overlap:
                ev[j] = record()
            if j:
                back.append(answer(j - 1))
        back.append(answer(C - 1))
        if overlap:
            e.wait_event(record())  # every response has arrived
        for j in range(C):
            e.merge(back[j], int(send[j].sum()))

    def _buf(self, name, nbytes):
        return self.e.buffer(name, nbytes) if hasattr(self.e, "buffer") else None

    def _bufkw(self, name, nbytes):
        return {"buf": self.e.buffer(name, nbytes)} if hasattr(self.e, "buffer") else {}

    def _host_buffer(self, n):
        import torch
        return torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)

    def _account(self, in_splits):
        self.exchanged_bytes += sum(in_splits)
        self.exchanged_remote += sum(in_splits) - in_splits[self.rank]

    def _overlapped(self):
        """Exchanges on a stream of their own (device collectives over RCCL, a GPU engine); gloo / CPU exchanges are
        synchronous anyway."""
        if self.coll is None or not hasattr(self.e, "wait_event"):
            return False
        return self.dist.get_backend() == "nccl"

    def round(self, rnd):
        if self.chunks > 1:
            return self._round_chunked(rnd)
        c = self.cfg
        M = self.e.claim_matrix(rnd, self.world)
        counts = M[self.rank]
        rcounts = M[:, self.rank]
        offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
        claims = self.e.build_claims(rnd, offs, int(counts.sum()))
        claims_in = self._exchange("claims_in", claims, counts, rcounts, c.claim_bytes)
        n_in = int(rcounts.sum())
        # every received claim gets exactly one response record, grouped by the requester's rank: what goes back to
        # rank d is what came from d, so the response counts are the claim counts reversed
        poffs = np.concatenate([[0], np.cumsum(rcounts)[:-1]])
        resps, tested = self.e.respond(claims_in, n_in, poffs, n_in)
        if tested is not None:
            self._tested += tested
        resps_in = self._exchange("resps_in", resps, rcounts, counts, c.resp_bytes)
        self.e.merge(resps_in, int(counts.sum()))

    def global_stats(self):
        held, chk = self.e.stats()
        chk &= 0x7fffffffffffffff
        if self.coll is None:
            return held, chk
        import torch
        held = self.coll.scalar(held, "sum", device=self.device)
        parts = torch.zeros(self.world, dtype=torch.int64, device=self.device)
        self.coll.all_gather_into(parts, torch.tensor([chk], dtype=torch.int64, device=self.device))
        x = 0
        for p in parts.tolist():
            x ^= int(p)
        return int(held), x
