"""dispersy_amd -- MI355X-native Bloom-filter synchronisation hot path of Dispersy.

The public surface mirrors the reference: `BloomFilter` (bloomfilter.py), and the sync claim / responder
surface of `Community` (community.py:599-941, :2746-2811) on top of a packed HBM `SyncStore`.
"""
from .bloomfilter import BloomFilter  # noqa: F401

__version__ = "0.1.0"
