"""ctypes binding of libhgx.so (the C ABI declared in include/hgx.h).

The library is built in-tree by __graft_entry__.build() (babble_amd/build.py).
Loading fails loudly if it is missing: there is no Python or CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, os.environ.get("HGX_LIB", "libhgx.so"))  # HGX_LIB: in-tree variant (profiling builds)

_L = None


class HgxError(RuntimeError):
    """A Go-equivalent error returned through the C ABI (code + verbatim message)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.msg = msg


class hgx_error(C.Structure):
    _fields_ = [("code", C.c_int32), ("msg", C.c_char * 252)]


class hgx_events(C.Structure):
    _fields_ = [(nm, C.c_void_p) for nm in
                ("creator", "index", "self_parent", "other_parent", "timestamp_ns", "hash", "sig_s",
                 "ntx", "tx_nil")]


class hgx_events32(C.Structure):
    _fields_ = [(nm, C.c_void_p) for nm in
                ("creator", "index", "self_parent", "other_parent", "timestamp_ns", "coin", "sig_s", "ntx")]


class hgx_events_packed(C.Structure):
    _fields_ = [(nm, C.c_void_p) for nm in ("creator", "index", "self_parent_back", "other_parent_back")] + \
               [("n_exc", C.c_int64)] + \
               [(nm, C.c_void_p) for nm in ("exc_pos", "exc_self_parent", "exc_other_parent", "timestamp_ns", "coin",
                                            "sig_s", "ntx")]


class hgx_wire_events(C.Structure):
    _fields_ = [(nm, C.c_void_p) for nm in
                ("creator_id", "index", "self_parent_index", "other_parent_creator", "other_parent_index",
                 "timestamp_ns", "hash", "sig_s", "ntx", "tx_nil")]


def ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


# void (*)(void* user, int32 graph, int64 b, int32 rr, int64 first, int32 n_events, int64 n_tx)
COMMIT_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_int32, C.c_int64)


def _sig(L, name, res, args):
    f = getattr(L, name, None)
    if f is None:
        return
    f.restype = res
    f.argtypes = args


def _one_hip_runtime():
    """One HIP runtime per process. PyTorch-ROCm bundles its own libamdhip64 + libhsa-runtime64;
    its libraries name the runtime "libamdhip64.so", libhgx names "libamdhip64.so.7" (the SONAME
    both copies carry). If libhgx is loaded first and torch after, the process maps TWO HIP and
    HSA runtimes, and libhgx's stops working once torch's initialises (measured: occupancy
    queries fail, HIP events become invalid handles). If torch is loaded first, libhgx's NEEDED
    entry resolves to torch's copy by SONAME and there is one runtime. So torch, when it is
    installed, is imported before libhgx is opened (HGX_NO_TORCH=1 skips this, for processes
    that never import torch). Loading libhgx by other means and torch later is unsupported."""
    if os.environ.get("HGX_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401  (loads torch's HIP runtime; no device is touched)
    except ImportError:
        pass
    except Exception as e:  # installed but broken (e.g. an OSError from its ROCm libraries)
        import warnings
        warnings.warn(f"libhgx: importing torch failed ({type(e).__name__}: {e}); libhgx is loaded with its own "
                      "HIP runtime, so a later torch import in this process is unsupported", RuntimeWarning)


def lib():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    _one_hip_runtime()
    L = C.CDLL(LIB_PATH)
    i32, i64, u64, p, d = C.c_int32, C.c_int64, C.c_uint64, C.c_void_p, C.c_double
    E = C.POINTER(hgx_error)
    _sig(L, "hgx_trace_gossip", i32, [i32, i32, i64, u64, d, i32] + [p] * 10)
    _sig(L, "hgx_trace_tx_payload", i32, [i32, i64, p, i32])
    _sig(L, "hgx_abi_version", i32, [])
    _sig(L, "hgx_create", p, [i32, i64, i32, E])
    _sig(L, "hgx_create_batch", p, [i32, i32, i64, i32, E])
    _sig(L, "hgx_create_sharded", p, [i32, i64, i32, p, E])
    _sig(L, "hgx_destroy", None, [p])
    _sig(L, "hgx_insert_events", i32, [p, C.POINTER(hgx_events), i64, C.POINTER(C.c_int64), E])
    _sig(L, "hgx_insert_events_device", i32, [p, C.POINTER(hgx_events), i64, C.POINTER(C.c_int64), E])
    _sig(L, "hgx_insert_and_run", i32, [p, C.POINTER(hgx_events), i64, C.POINTER(C.c_int64), E])
    for nm in ("hgx_insert_events32", "hgx_insert_and_run32"):
        _sig(L, nm, i32, [p, C.POINTER(hgx_events32), i64, C.POINTER(C.c_int64), E])
    for nm in ("hgx_insert_events_packed", "hgx_insert_and_run_packed"):
        _sig(L, nm, i32, [p, C.POINTER(hgx_events_packed), i64, C.POINTER(C.c_int64), E])
    _sig(L, "hgx_pack_events32", i32, [C.POINTER(hgx_events32), i64, i64, p, p, p, p, p, p, i64,
                                       C.POINTER(C.c_int64), E])
    _sig(L, "hgx_host_alloc", p, [i64])
    _sig(L, "hgx_host_free", None, [p])
    _sig(L, "hgx_set_participant_keys", i32, [p, p, E])
    for nm in ("hgx_insert_events_verified", "hgx_insert_events_verified_device"):
        _sig(L, nm, i32, [p, C.POINTER(hgx_events), p, p, i64, C.POINTER(C.c_int64), E])
    _sig(L, "hgx_reset_consensus", i32, [p])
    _sig(L, "hgx_save", i32, [p, C.c_char_p, E])
    _sig(L, "hgx_save_ex", i32, [p, C.c_char_p, p, p, E])
    _sig(L, "hgx_get_event_id", i32, [p, i64, p, E])
    _sig(L, "hgx_get_event_payload", i32, [p, i64, p, i64, C.POINTER(C.c_int64), E])
    _sig(L, "hgx_checksum", u64, [p, i64])
    _sig(L, "hgx_bootstrap", i32, [p, C.c_char_p, E])
    _sig(L, "hgx_clear", i32, [p])
    for nm in ("hgx_divide_rounds", "hgx_decide_fame", "hgx_find_order", "hgx_run_consensus"):
        _sig(L, nm, i32, [p, E])
    _sig(L, "hgx_num_events", i64, [p])
    _sig(L, "hgx_super_majority", i32, [p])
    _sig(L, "hgx_num_undetermined", i64, [p, i32])
    _sig(L, "hgx_undecided_rounds", i32, [p, i32, p, i32])
    _sig(L, "hgx_last_consensus_round", i32, [p, i32, C.POINTER(C.c_int32)])
    _sig(L, "hgx_last_commited_round_events", i32, [p, i32])
    _sig(L, "hgx_consensus_transactions", i64, [p, i32])
    _sig(L, "hgx_pending_loaded_events", i64, [p, i32])
    _sig(L, "hgx_last_round", i32, [p, i32])
    _sig(L, "hgx_round_event_count", i32, [p, i32, i32])
    _sig(L, "hgx_round_witnesses", i32, [p, i32, i32, p, i32])
    _sig(L, "hgx_known", i32, [p, i32, p])
    _sig(L, "hgx_consensus_events_count", i64, [p, i32])
    _sig(L, "hgx_consensus_events", i32, [p, i32, i64, i64, p])
    _sig(L, "hgx_num_blocks", i64, [p, i32])
    _sig(L, "hgx_block_info", i32, [p, i32, i64, p, p, p, p, p, p])
    _sig(L, "hgx_get_block", i32, [p, i32, i32, p, E])
    _sig(L, "hgx_consensus_received", i32, [p, i32, i64, i64, p, p, p])
    _sig(L, "hgx_last_from", i32, [p, i32, p, p, E])
    _sig(L, "hgx_participant_events", i32, [p, i32, i64, p, i64, p, E])
    _sig(L, "hgx_participant_event", i32, [p, i32, i64, p, E])
    _sig(L, "hgx_get_root", i32, [p, i32, p, p, p, p, E])
    _sig(L, "hgx_get_event", i32, [p, i64, p, p, p, p, p, p, p, E])
    _sig(L, "hgx_wire_info", i32, [p, i64, i64, p, p, p])
    _sig(L, "hgx_read_wire_info", i32, [p, i32, i64, i32, i64, p, p, E])
    _sig(L, "hgx_get_rounds", i32, [p, i64, i64, p, p, p])
    _sig(L, "hgx_get_received", i32, [p, i64, i64, p, p])
    _sig(L, "hgx_get_coords", i32, [p, i64, p, p])
    for nm in ("hgx_ancestor", "hgx_self_ancestor", "hgx_see", "hgx_strongly_see", "hgx_round", "hgx_witness"):
        _sig(L, nm, i32, [p, i64, i64] if nm not in ("hgx_round", "hgx_witness") else [p, i64])
    _sig(L, "hgx_oldest_self_ancestor_to_see", i64, [p, i64, i64])
    _sig(L, "hgx_block_hash", i32, [i64, i32, p, p, i32, p])
    _sig(L, "hgx_sha256_batch", i32, [i32, p, p, i64, p, p])
    _sig(L, "hgx_sha256_batch_device", i32, [p, p, i64, p, p])
    _sig(L, "hgx_p256_verify_batch", i32, [i32, p, i32, p, p, p, p, i64, p, p])
    _sig(L, "hgx_p256_verify_bench", i32, [i32, p, i32, p, p, p, p, i64, i32, i32, p, C.POINTER(C.c_double)])
    _sig(L, "hgx_sha256_bench", i32, [i32, i64, i32, i32, C.c_uint64, i32, i32, C.POINTER(C.c_double),
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int64), i64, p])
    _sig(L, "hgx_phase_times", i32, [p, p, i32])
    _sig(L, "hgx_kernel_stats", i32, [p, i32, C.c_char_p, i32, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                      C.POINTER(C.c_double)])
    _sig(L, "hgx_reset_stats", i32, [p])
    _sig(L, "hgx_set_kernel_timing", i32, [p, i32])
    _sig(L, "hgx_set_coord_storage", i32, [p, i32])
    _sig(L, "hgx_set_fame_tally", i32, [p, i32])
    _sig(L, "hgx_set_round_kernel", i32, [p, i32])
    _sig(L, "hgx_set_sort_kernel", i32, [p, i32])
    _sig(L, "hgx_set_round_shards", i32, [p, i32])
    _sig(L, "hgx_set_shard_remote", i32, [p, i32])
    _sig(L, "hgx_exchange_floor_bench", i32, [i32, i32, i32, i32, C.POINTER(C.c_double)])
    _sig(L, "hgx_set_cts_kernel", i32, [p, i32])
    _sig(L, "hgx_set_root_others", i32, [p, p, i64, p])
    _sig(L, "hgx_set_la_kernel", i32, [p, i32])
    _sig(L, "hgx_set_incremental", i32, [p, i32])
    _sig(L, "hgx_find_order_begin", i32, [p, p])
    _sig(L, "hgx_find_order_end", i32, [p, p])
    _sig(L, "hgx_set_shard", i32, [p, i32, i32])
    _sig(L, "hgx_reset", i32, [p, p, p, p, p])
    _sig(L, "hgx_insert_wire_events", i32, [p, p, i64, p, p])
    _sig(L, "hgx_set_commit_callback", i32, [p, C.c_void_p, p])
    _sig(L, "hgx_get_frame", i32, [p, p, i64, p, p, p, p, p, p, p, i64, p, p])
    _sig(L, "hgx_shard_values", i64, [p, i32])
    _sig(L, "hgx_shard_export", i32, [p, p, i32])
    _sig(L, "hgx_shard_import", i32, [p, i32, p, i32])
    _sig(L, "hgx_reserve_rounds", i32, [p, i32])
    _sig(L, "hgx_device_alloc", i32, [i32, i64, C.POINTER(C.c_void_p)])
    _sig(L, "hgx_device_free", i32, [i32, p])
    _sig(L, "hgx_device_copy", i32, [i32, p, p, i64, i32])
    _L = L
    return L


def check(rc: int, err: hgx_error):
    if rc != 0:
        raise HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
