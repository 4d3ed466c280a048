"""ORACLE -- test infrastructure only.

CPU engine for dispersy_amd.sim.EpidemicSim: the same per-rank operations as the HIP kernels of
dispersy_amd/csrc/dsy_sim_kernels.hip, written with OracleBloom (hashlib) and Python loops, exchanging the same
record layouts.  Used by tests to (1) check the GPU simulator peer by peer at small sizes and (2) exercise the
multi-rank exchange logic with the gloo backend on CPU.

Protocol steps restated: claim = _dispersy_claim_sync_bloom_filter_largest's below-capacity branch
(community.py:808-821); response = _get_packets_for_bloomfilters + byte-limited not_filter loop
(community.py:2746-2811, :2555-2567); the requester stores what it receives.
"""
import struct

import numpy as np

from oracle.bloom_ref import OracleBloom

M64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9e3779b97f4a7c15) & M64
    x = ((x ^ (x >> 30)) * 0xbf58476d1ce4e5b9) & M64
    x = ((x ^ (x >> 27)) * 0x94d049bb133111eb) & M64
    return x ^ (x >> 31)


def partner(c, rnd, p):
    h = splitmix64(c.seed ^ ((rnd << 40) & M64) ^ ((p * 0x2545f4914f6cdd1d) & M64))
    return (p + 1 + h % (c.n_peers - 1)) % c.n_peers


def prefix(c, rnd, p):
    return (splitmix64((c.seed * 3 + 0x51ed27 + rnd * c.n_peers + p) & M64) >> 32) & 0xFF


def owner(c, p):
    return p // c.peers_per_rank


CLAIM_HDR = struct.Struct("<QQQII")
RESP_HDR = struct.Struct("<QII")


class _NumpyBuffers(object):
    """The two torch calls the engine makes, over numpy (bench.py's forked CPU workers stay out of torch)."""

    @staticmethod
    def frombuffer(buf, dtype=None):
        return np.frombuffer(buf, dtype=np.uint8)

    uint8 = None


class OracleEngine(object):
    def __init__(self, cfg, blob, offsets, arrays="torch"):
        if arrays == "torch":
            import torch
            self.torch = torch
        else:
            self.torch = _NumpyBuffers
        self.c = cfg
        self.packets = [blob[int(offsets[i]):int(offsets[i + 1])] for i in range(cfg.universe)]
        self.local = cfg.peer_end - cfg.peer_begin
        self.stores = [set() for _ in range(self.local)]

    def seed(self, initial):
        c = self.c
        for lp in range(self.local):
            p = c.peer_begin + lp
            s, j = self.stores[lp], 0
            while len(s) < min(initial, c.universe):
                s.add(splitmix64((c.seed * 7 + 0xabcdef + p * 1000003 + j) & M64) % c.universe)
                j += 1

    def claim_counts(self, rnd, world):
        out = np.zeros(world, dtype=np.int64)
        for lp in range(self.local):
            out[owner(self.c, partner(self.c, rnd, self.c.peer_begin + lp))] += 1
        return out

    def claim_matrix(self, rnd, world):
        """[src, dst] claims of round rnd over every peer (dsy_sim_claim_matrix)."""
        out = np.zeros((world, world), dtype=np.int64)
        for p in range(self.c.n_peers):
            out[owner(self.c, p), owner(self.c, partner(self.c, rnd, p))] += 1
        return out

    def claim_matrix_v(self, rnd, nv, cs):
        """[src, dst] claims over virtual ranks of cs peers (dsy_sim_claim_matrix with peers_per_rank = cs)."""
        out = np.zeros((nv, nv), dtype=np.int64)
        for p in range(self.c.n_peers):
            out[p // cs, partner(self.c, rnd, p) // cs] += 1
        return out

    def build_claims_chunk(self, rnd, j, cs, offsets, total, buf=None):
        """Claims of this rank's peers [j cs, (j + 1) cs), grouped by destination chunk (the GPU engine's chunk_cfg)."""
        return self.build_claims(rnd, offsets, total, lps=range(min(self.local, j * cs), min(self.local, (j + 1) * cs)),
                                 owner_div=cs)

    def build_claims(self, rnd, offsets, total, lps=None, owner_div=None):
        c = self.c
        buf = bytearray(max(total, 1) * c.claim_bytes)
        cursor = [int(x) for x in offsets]
        for lp in (range(self.local) if lps is None else lps):
            p = c.peer_begin + lp
            ids = sorted(self.stores[lp])
            time_high = 0x7fffffffffffffff
            if len(ids) > c.capacity:  # _select_and_fix over-full: keep the first `capacity` (distinct gts)
                ids = ids[:c.capacity]
                time_high = ids[-1] + 1
            pre = prefix(c, rnd, p)
            bf = OracleBloom(c.m_bits, c.k, bytes([pre]))
            bf.add_keys(self.packets[i] for i in ids)
            q = partner(c, rnd, p)
            d = owner(c, q) if owner_div is None else q // owner_div
            at = cursor[d] * c.claim_bytes
            cursor[d] += 1
            CLAIM_HDR.pack_into(buf, at, p, q, time_high, pre, len(ids))
            raw = bf.to_bytes()
            buf[at + 32:at + 32 + len(raw)] = raw
        return self._out(buf)

    def _out(self, buf):
        t = self.torch.frombuffer(buf, dtype=self.torch.uint8)
        return t.copy() if isinstance(t, np.ndarray) else t.clone()

    @staticmethod
    def _raw(t):
        return (t if isinstance(t, np.ndarray) else t.numpy()).tobytes()

    def _claims(self, claims, n):
        raw = self._raw(claims)
        for i in range(n):
            at = i * self.c.claim_bytes
            yield CLAIM_HDR.unpack_from(raw, at), raw[at + 32:at + 32 + self.c.m_bits // 8]

    def resp_counts(self, claims, n, world):
        out = np.zeros(world, dtype=np.int64)
        for (req, _, _, _, _), _ in self._claims(claims, n):
            out[owner(self.c, req)] += 1
        return out

    def respond(self, claims, n, offsets, total):
        c = self.c
        buf = bytearray(max(total, 1) * c.resp_bytes)
        cursor = [int(x) for x in offsets]
        tested = [0]
        for (req, resp, time_high, pre, _), fraw in self._claims(claims, n):
            bf = OracleBloom.from_bytes(fraw, c.k, bytes([pre]))
            ids = [i for i in sorted(self.stores[resp - c.peer_begin]) if i + 1 <= time_high]

            def gen():
                for i in ids:
                    tested[0] += 1
                    yield (self.packets[i], i)
            sent, budget = [], c.byte_limit
            for packet, i in bf.not_filter(gen()):
                sent.append(i)
                budget -= len(packet)
                if budget <= 0:
                    break
            d = owner(c, req)
            at = cursor[d] * c.resp_bytes
            cursor[d] += 1
            RESP_HDR.pack_into(buf, at, req, min(len(sent), 64), int(len(sent) > 64))
            struct.pack_into("<%dH" % min(len(sent), 64), buf, at + 16, *sent[:64])
        return self._out(buf), tested[0]

    def merge(self, resps, n):
        raw = self._raw(resps)
        for i in range(n):
            at = i * self.c.resp_bytes
            req, cnt, ovf = RESP_HDR.unpack_from(raw, at)
            assert not ovf
            self.stores[req - self.c.peer_begin].update(struct.unpack_from("<%dH" % cnt, raw, at + 16))

    def stats(self):
        c = self.c
        held, h = 0, 0
        for lp, s in enumerate(self.stores):
            held += len(s)
            words = [0] * c.words
            for i in s:
                words[i >> 5] |= 1 << (i & 31)
            for w, val in enumerate(words):
                h ^= splitmix64((((c.peer_begin + lp) << 20) ^ (w << 32) ^ val) & M64)
        return held, h

    def bitsets(self):
        c = self.c
        out = np.zeros((self.local, c.words), dtype=np.uint32)
        for lp, s in enumerate(self.stores):
            for i in s:
                out[lp, i >> 5] |= np.uint32(1 << (i & 31))
        return out

    def sync(self):
        pass
