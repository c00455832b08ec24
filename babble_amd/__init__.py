"""babble_amd -- MI355X-native engine for Babble's Hashgraph consensus hot path.

The product is libhgx.so (C ABI: include/hgx.h; HIP kernels for gfx950 in
babble_amd/csrc). `babble_amd.hashgraph` mirrors the reference Go API
(hashgraph.Hashgraph: InsertEvent / DivideRounds / DecideFame / FindOrder and the
Store views) over that C ABI.
"""
__all__ = ["hashgraph", "trace"]
