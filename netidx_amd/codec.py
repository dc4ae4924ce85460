"""ctypes binding of the C ABI in include/nxg_codec.h (netidx_amd/lib/libnxg_codec.so).

The Python surface mirrors the two seams that the codec replaces in the reference:

* ``Codec.decode_batch(frame)`` replaces the ``decode_task`` -> ``receive_batch_fn`` loop
  (netidx/src/subscriber/connection.rs:209-242, netidx/src/channel.rs:504-521). A malformed
  frame raises ``PackError`` with the reference's kind and the offset of the first failing
  message, and the whole frame is rejected, as in connection.rs:228-231.
* ``Codec.encode_batch(cols)`` replaces the ``handle_updates`` -> ``queue_send`` loop
  (netidx/src/publisher/server.rs:610-612, netidx/src/channel.rs:177-202).

The product path is the HIP library. There is no CPU fallback: if the shared library or a GPU
is missing, the calls raise.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NXG_LIB: another build of the same library (A/B experiments, scripts/ab_variants.sh)
LIB_PATH = os.environ.get("NXG_LIB") or os.path.join(HERE, "lib", "libnxg_codec.so")

# NxgErrKind (include/nxg_codec.h) = PackError (netidx-core/src/pack.rs:89-95) + codec kinds
OK, UNKNOWN_TAG, TOO_BIG, INVALID_FORMAT, BUFFER_SHORT = 0, 1, 2, 3, 4
DEPTH, CAPACITY, NOT_F64, TIMEOUT = 6, 7, 8, 9
ERR_NAMES = {1: "UnknownTag", 2: "TooBig", 3: "InvalidFormat", 4: "BufferShort", 6: "Depth",
             7: "Capacity", 8: "NotF64", 9: "Timeout"}
LAYOUT_F64, LAYOUT_MIXED = 1, 2
MEM_DEVICE, MEM_HOST = 0, 1
HINT_MIXED = 1


class PackError(Exception):
    """A frame the reference would reject (netidx-core/src/pack.rs:89-95)."""

    def __init__(self, kind, offset):
        self.kind = kind
        self.offset = offset
        super().__init__(f"{ERR_NAMES.get(kind, kind)} at message offset {offset}")


class CodecError(RuntimeError):
    """API misuse or a HIP failure (NetidxError)."""


class NetidxError(C.Structure):
    _fields_ = [("msg", C.c_char_p)]


U64P, U32P, U8P = C.c_void_p, C.c_void_p, C.c_void_p


class NxgColumns(C.Structure):
    _fields_ = [
        ("layout", C.c_uint32), ("mem", C.c_uint32),
        ("cap_rows", C.c_uint64), ("cap_children", C.c_uint64), ("cap_ctl", C.c_uint64),
        ("n_rows", C.c_uint64), ("n_children", C.c_uint64), ("n_ctl", C.c_uint64),
        ("n_heartbeat", C.c_uint64),
        ("id", C.c_void_p), ("tag", C.c_void_p), ("fixed", C.c_void_p), ("aux", C.c_void_p),
        ("ctag", C.c_void_p), ("cfixed", C.c_void_p), ("caux", C.c_void_p),
        ("ctl_row", C.c_void_p), ("ctl_off", C.c_void_p), ("ctl_len", C.c_void_p),
        ("ctl_variant", C.c_void_p),
    ]


class NxgRange(C.Structure):
    _fields_ = [("begin", C.c_uint64), ("end", C.c_uint64), ("entry", C.c_uint64),
                ("exit", C.c_uint64), ("n_rows", C.c_uint64), ("ok", C.c_uint32),
                ("err_kind", C.c_uint32), ("err_offset", C.c_uint64)]

    def tuple(self):
        return (self.begin, self.end, self.entry, self.exit, self.n_rows, self.ok, self.err_kind,
                self.err_offset)

    @classmethod
    def of(cls, t):
        return cls(*t)


class NxgSubTable(C.Structure):
    _fields_ = [("n_ids", C.c_uint64), ("slot_of_id", C.c_void_p), ("n_slots", C.c_uint64),
                ("slot_sub_id", C.c_void_p), ("slot_stream_off", C.c_void_p),
                ("stream_chan", C.c_void_p), ("slot_has_last", C.c_void_p),
                ("n_chans", C.c_uint32)]


class NxgDispatch(C.Structure):
    _fields_ = [("cap_entries", C.c_uint64), ("chan_off", C.c_void_p), ("ent_sub", C.c_void_p),
                ("ent_row", C.c_void_p), ("last_row", C.c_void_p), ("n_entries", C.c_uint64),
                ("n_unmatched", C.c_uint64)]


TAG_BINS = 256


class NxgTagView(C.Structure):
    _fields_ = [("cap_rows", C.c_uint64), ("rank", C.c_void_p), ("row_of", C.c_void_p),
                ("fixed", C.c_void_p), ("aux", C.c_void_p), ("n_rows", C.c_uint64),
                ("count", C.c_uint64 * TAG_BINS), ("off", C.c_uint64 * (TAG_BINS + 1))]


class NxgPubTable(C.Structure):
    _fields_ = [("n_ids", C.c_uint64), ("slot_of_id", C.c_void_p), ("n_slots", C.c_uint64),
                ("slot_client_off", C.c_void_p), ("client", C.c_void_p), ("n_clients", C.c_uint32),
                ("cur_tag", C.c_void_p), ("cur_fixed", C.c_void_p), ("cur_aux", C.c_void_p),
                ("cur_heap", C.c_void_p), ("cur_ctag", C.c_void_p), ("cur_cfixed", C.c_void_p),
                ("cur_caux", C.c_void_p)]


class NxgCtlMsg(C.Structure):
    _fields_ = [("msg_len", C.c_uint64), ("variant", C.c_uint32), ("permissions", C.c_uint32),
                ("id", C.c_uint64), ("path_off", C.c_uint64), ("path_len", C.c_uint64),
                ("timestamp", C.c_uint64), ("token_off", C.c_uint64), ("token_len", C.c_uint64),
                ("value_off", C.c_uint64), ("value_len", C.c_uint64), ("value_fixed", C.c_uint64),
                ("value_tag", C.c_uint32), ("value_aux", C.c_uint32)]


class NxgResolved(C.Structure):
    _fields_ = [("n_publishers", C.c_uint32), ("publisher_ipv4", C.c_uint32),
                ("publisher_id", C.c_uint64), ("publisher_port", C.c_uint16),
                ("resolver_port", C.c_uint16), ("resolver_ipv4", C.c_uint32),
                ("timestamp", C.c_uint64), ("flags", C.c_uint32), ("permissions", C.c_uint32)]


class NxgArchiveRecord(C.Structure):
    _fields_ = [("off", C.c_uint64), ("len", C.c_uint64), ("out_off", C.c_uint64),
                ("out_len", C.c_uint64), ("err", C.c_uint32), ("pad", C.c_uint32)]


class NxgStatus(C.Structure):
    _fields_ = [
        ("n_rows", C.c_uint64), ("n_children", C.c_uint64), ("n_ctl", C.c_uint64),
        ("n_heartbeat", C.c_uint64), ("err_kind", C.c_int32), ("path", C.c_uint32),
        ("err_offset", C.c_uint64),
    ]


# every symbol include/nxg_codec.h declares, with its ctypes signature
SIGNATURES = {
    "nxg_ctx_new": (C.c_void_p, [C.c_int, C.POINTER(NetidxError)]),
    "nxg_ctx_destroy": (None, [C.c_void_p]),
    "nxg_ctx_set_stream": (C.c_bool, [C.c_void_p, C.c_void_p, C.POINTER(NetidxError)]),
    "nxg_ctx_stream": (C.c_void_p, [C.c_void_p]),
    "nxg_error_free": (None, [C.POINTER(NetidxError)]),
    "nxg_version": (C.c_char_p, []),
    "nxg_columns_alloc": (C.c_bool, [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                     C.c_uint32, C.POINTER(NxgColumns), C.POINTER(NetidxError)]),
    "nxg_columns_free": (None, [C.c_void_p, C.POINTER(NxgColumns)]),
    "nxg_decode_updates": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(NxgColumns),
                                      C.c_uint32, C.POINTER(NxgStatus), C.POINTER(NetidxError)]),
    "nxg_decode_updates_async": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64,
                                            C.POINTER(NxgColumns), C.c_uint32,
                                            C.POINTER(NetidxError)]),
    "nxg_ctx_sync": (C.c_bool, [C.c_void_p, C.POINTER(NxgStatus), C.POINTER(NetidxError)]),
    "nxg_decode_frames_async": (C.c_bool, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_uint32, C.POINTER(NetidxError)]),
    "nxg_encoded_len": (C.c_bool, [C.c_void_p, C.POINTER(NxgColumns), C.c_void_p,
                                   C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_encode_updates": (C.c_bool, [C.c_void_p, C.POINTER(NxgColumns), C.c_void_p, C.c_void_p,
                                      C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_encode_updates_async": (C.c_bool, [C.c_void_p, C.POINTER(NxgColumns), C.c_void_p,
                                            C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                            C.POINTER(NetidxError)]),
    "nxg_encode_frames": (C.c_bool, [C.c_void_p, C.POINTER(NxgColumns), C.c_void_p, C.c_void_p,
                                     C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p, C.c_uint64,
                                     C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_decode_range": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                    C.POINTER(NxgColumns), C.POINTER(NxgRange),
                                    C.POINTER(NetidxError)]),
    "nxg_decode_share": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                    C.POINTER(NxgColumns), C.POINTER(C.c_uint64),
                                    C.POINTER(NxgStatus), C.POINTER(NetidxError)]),
    "nxg_range_link": (C.c_bool, [C.POINTER(NxgRange), C.c_uint32, C.c_uint64, C.c_void_p,
                                  C.POINTER(C.c_uint32), C.POINTER(NetidxError)]),
    "nxg_comm_unique_id": (C.c_bool, [C.c_void_p, C.POINTER(NetidxError)]),
    "nxg_comm_init": (C.c_void_p, [C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                   C.POINTER(NetidxError)]),
    "nxg_comm_init_ops": (C.c_void_p, [C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                       C.POINTER(NetidxError)]),
    "nxg_comm_destroy": (None, [C.c_void_p]),
    "nxg_encode_allgather": (C.c_bool, [C.c_void_p, C.c_void_p, C.POINTER(NxgColumns),
                                        C.c_void_p, C.c_void_p, C.c_uint64,
                                        C.POINTER(C.c_uint64), C.c_void_p,
                                        C.POINTER(NetidxError)]),
    "nxg_decode_sharded": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                      C.POINTER(NxgColumns), C.POINTER(C.c_uint64),
                                      C.POINTER(NxgRange), C.POINTER(NetidxError)]),
    "nxg_partition_by_tag": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.POINTER(NetidxError)]),
    "nxg_dispatch_updates": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                        C.c_void_p, C.POINTER(NetidxError)]),
    "nxg_publish_commit": (C.c_bool, [C.c_void_p, C.c_void_p, C.POINTER(NxgColumns), C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.POINTER(NetidxError)]),
    "nxg_publish_unsubscribes": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                            C.c_uint32, C.c_void_p, C.POINTER(NetidxError)]),
    "nxg_zstd_dict_new": (C.c_void_p, [C.c_void_p, C.c_void_p, C.c_uint64,
                                       C.POINTER(NetidxError)]),
    "nxg_zstd_dict_free": (None, [C.c_void_p]),
    "nxg_archive_decompress": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                          C.POINTER(NxgArchiveRecord), C.c_uint32, C.c_bool,
                                          C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                          C.POINTER(NetidxError)]),
    "nxg_decode_archive_batch": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64,
                                            C.POINTER(NxgColumns), C.POINTER(NxgStatus),
                                            C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_encode_archive_batch": (C.c_bool, [C.c_void_p, C.POINTER(NxgColumns), C.c_void_p,
                                            C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                            C.POINTER(NetidxError)]),
    "nxg_session_connect": (C.c_void_p, [C.c_char_p, C.c_uint16, C.POINTER(NetidxError)]),
    "nxg_session_listen": (C.c_void_p, [C.c_char_p, C.c_uint16, C.POINTER(C.c_uint16),
                                        C.POINTER(NetidxError)]),
    "nxg_session_accept": (C.c_void_p, [C.c_void_p, C.POINTER(NetidxError)]),
    "nxg_session_close": (None, [C.c_void_p]),
    "nxg_session_stats": (None, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "nxg_session_send": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(NetidxError)]),
    "nxg_session_recv_frame": (C.c_bool, [C.c_void_p, C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_session_recv_decode": (C.c_bool, [C.c_void_p, C.c_void_p, C.POINTER(NxgColumns),
                                           C.c_uint32, C.POINTER(NxgStatus),
                                           C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_session_publish": (C.c_bool, [C.c_void_p, C.c_void_p, C.POINTER(NxgColumns), C.c_void_p,
                                       C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_msg_subscribe": (C.c_int64, [C.c_char_p, C.c_uint64, C.c_uint32, C.c_uint16, C.c_uint64,
                                      C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p,
                                      C.c_uint64]),
    "nxg_msg_subscribed": (C.c_int64, [C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint8, C.c_uint64,
                                       C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64]),
    "nxg_msg_heartbeat": (C.c_int64, [C.c_void_p, C.c_uint64]),
    "nxg_msg_update": (C.c_int64, [C.c_uint64, C.c_uint8, C.c_uint64, C.c_uint32, C.c_void_p,
                                   C.c_void_p, C.c_uint64]),
    "nxg_resolver_start": (C.c_void_p, [C.c_char_p, C.c_uint16, C.POINTER(C.c_uint16),
                                        C.c_uint64, C.POINTER(NetidxError)]),
    "nxg_resolver_stop": (None, [C.c_void_p]),
    "nxg_resolver_n_published": (C.c_uint64, [C.c_void_p]),
    "nxg_resolver_connect_write": (C.c_void_p, [C.c_char_p, C.c_uint16, C.c_uint32, C.c_uint16,
                                                C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_resolver_connect_read": (C.c_void_p, [C.c_char_p, C.c_uint16, C.POINTER(NetidxError)]),
    "nxg_resolver_client_close": (None, [C.c_void_p]),
    "nxg_resolver_publish": (C.c_bool, [C.c_void_p, C.c_char_p, C.c_uint64,
                                        C.POINTER(NetidxError)]),
    "nxg_resolver_resolve": (C.c_bool, [C.c_void_p, C.c_char_p, C.c_uint64,
                                        C.POINTER(NxgResolved), C.POINTER(NetidxError)]),
    "nxg_msg_parse": (C.c_bool, [C.c_void_p, C.c_uint64, C.c_int, C.POINTER(NxgCtlMsg),
                                 C.POINTER(NetidxError)]),
    "nxg_frame_reader_new": (C.c_void_p, [C.POINTER(NetidxError)]),
    "nxg_frame_reader_free": (None, [C.c_void_p]),
    "nxg_frame_reader_push": (C.c_bool, [C.c_void_p, C.c_void_p, C.c_uint64,
                                         C.POINTER(NetidxError)]),
    "nxg_frame_reader_next": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_uint64), C.POINTER(NetidxError)]),
    "nxg_frame_reader_buffered": (C.c_uint64, [C.c_void_p]),
    "nxg_frame_split": (C.c_int64, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]),
    "nxg_frame_header": (None, [C.c_uint32, C.c_bool, C.c_void_p]),
    "nxg_frame_parse_header": (C.c_uint32, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32),
                                            C.POINTER(C.c_bool)]),
}

_lib = None


def lib():
    """Load libnxg_codec.so (loud failure if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CodecError(f"{LIB_PATH} missing: build it (python -c 'import __graft_entry__ as g; g.build()')")
        # One HIP runtime per process: torch carries its own libamdhip64 and must load it before
        # this library's NEEDED libamdhip64.so.7 is resolved (the loader then reuses torch's); if
        # /opt/rocm's were loaded first, torch would find no GPU ("No HIP GPUs are available").
        try:
            import torch
            torch.cuda.is_available()
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("NXG_LIB") and not hasattr(L, name):
                continue  # an A/B build of an older source may lack newer entry points
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(ok, err):
    if not ok:
        msg = err.msg.decode() if err.msg else "unknown error"
        lib().nxg_error_free(C.byref(err))
        raise CodecError(msg)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


class ZstdDict:
    """A device-resident zstd dictionary (nxg_zstd_dict_new / _free)."""

    def __init__(self, h):
        self.h = h

    def close(self):
        if self.h:
            lib().nxg_zstd_dict_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Columns:
    """Columnar batch (include/nxg_codec.h). Arrays are torch tensors on `device` (or pinned
    host numpy-backed tensors when device is 'cpu')."""

    FIELDS = [("id", "torch.int64", "rows"), ("fixed", "torch.int64", "rows"),
              ("tag", "torch.uint8", "rows"), ("aux", "torch.int32", "rows"),
              ("ctag", "torch.uint8", "children"), ("cfixed", "torch.int64", "children"),
              ("caux", "torch.int32", "children"), ("ctl_row", "torch.int64", "ctl"),
              ("ctl_off", "torch.int64", "ctl"), ("ctl_len", "torch.int32", "ctl"),
              ("ctl_variant", "torch.uint8", "ctl")]

    def __init__(self, cap_rows, cap_children=0, cap_ctl=0, layout=LAYOUT_MIXED, device="cuda"):
        import torch
        self.device = torch.device(device)
        self.layout = layout
        self.caps = {"rows": max(cap_rows, 1), "children": max(cap_children, 1),
                     "ctl": max(cap_ctl, 1)}
        self.t = {}
        dt = {"torch.int64": torch.int64, "torch.int32": torch.int32, "torch.uint8": torch.uint8}
        for name, d, kind in self.FIELDS:
            if layout == LAYOUT_F64 and name not in ("id", "fixed"):
                self.t[name] = None
                continue
            x = torch.zeros(self.caps[kind], dtype=dt[d], device=self.device)
            if self.device.type == "cpu":
                x = x.pin_memory()
            self.t[name] = x
        self.s = NxgColumns()
        self.s.layout = layout
        self.s.mem = MEM_DEVICE if self.device.type == "cuda" else MEM_HOST
        self.s.cap_rows, self.s.cap_children, self.s.cap_ctl = (
            self.caps["rows"], self.caps["children"], self.caps["ctl"])
        for name, _, _ in self.FIELDS:
            setattr(self.s, name, _ptr(self.t[name]).value)
        if self.device.type == "cuda":
            # the zero fill ran on torch's current stream; a codec on another stream (set_stream)
            # must not start writing before it is done
            torch.cuda.synchronize(self.device)

    @classmethod
    def for_frame(cls, nbytes, layout=LAYOUT_MIXED, device="cuda"):
        """Capacity bounds of include/nxg_codec.h for a frame of `nbytes`."""
        return cls(nbytes // 4 + 1, nbytes + 1, nbytes // 2 + 1, layout, device)

    def __getattr__(self, k):
        t = self.__dict__.get("t", {})
        if k in t:
            return t[k]
        raise AttributeError(k)

    @property
    def n_rows(self):
        return self.s.n_rows

    def numpy(self):
        """Trimmed host copy: {field: ndarray} (unsigned views)."""
        n = {"rows": self.s.n_rows, "children": self.s.n_children, "ctl": self.s.n_ctl}
        out = {}
        u = {"torch.int64": np.uint64, "torch.int32": np.uint32, "torch.uint8": np.uint8}
        for name, d, kind in self.FIELDS:
            x = self.t[name]
            if x is None:
                continue
            out[name] = x[: n[kind]].cpu().numpy().view(u[d])
        if self.s.layout == LAYOUT_F64:  # homogeneous result: tag 9 implied, aux unused
            out["tag"] = np.full(n["rows"], 9, np.uint8)
            if "aux" in out:
                out["aux"] = np.zeros(n["rows"], np.uint32)
        out["n_heartbeat"] = self.s.n_heartbeat
        out["layout"] = self.s.layout
        return out


class Codec:
    """One codec context per connection/thread (NxgCtx)."""

    def __init__(self, device=0):
        err = NetidxError()
        self.ctx = lib().nxg_ctx_new(device, C.byref(err))
        _check(self.ctx is not None, err)
        self.device = device

    def close(self):
        if self.ctx:
            lib().nxg_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        err = NetidxError()
        _check(lib().nxg_ctx_set_stream(self.ctx, C.c_void_p(stream_ptr), C.byref(err)), err)

    def decode_into(self, frame, nbytes, cols, flags=0, check=True):
        """frame: device pointer (int), torch tensor or bytes. Returns NxgStatus."""
        keep = None
        if isinstance(frame, (bytes, bytearray, memoryview)):
            keep = np.frombuffer(bytes(frame), np.uint8)
            ptr = keep.ctypes.data
        elif isinstance(frame, np.ndarray):
            keep = np.ascontiguousarray(frame)
            ptr = keep.ctypes.data
        elif hasattr(frame, "data_ptr"):
            ptr = frame.data_ptr()
        else:
            ptr = int(frame)
        st, err = NxgStatus(), NetidxError()
        ok = lib().nxg_decode_updates(self.ctx, C.c_void_p(ptr), nbytes, C.byref(cols.s), flags,
                                      C.byref(st), C.byref(err))
        _check(ok, err)
        if check and st.err_kind:
            raise PackError(st.err_kind, st.err_offset)
        return st

    def decode_archive(self, buf, nbytes, cols, check=True):
        """An archive batch (Vec<BatchItem>, netidx-archive logfile/mod.rs:150-205) in device
        memory into MIXED device columns. Returns (NxgStatus, bytes consumed)."""
        ptr = buf.data_ptr() if hasattr(buf, "data_ptr") else int(buf)
        st, err, used = NxgStatus(), NetidxError(), C.c_uint64(0)
        _check(lib().nxg_decode_archive_batch(self.ctx, C.c_void_p(ptr), nbytes, C.byref(cols.s),
                                              C.byref(st), C.byref(used), C.byref(err)), err)
        if check and st.err_kind:
            raise PackError(st.err_kind, st.err_offset)
        return st, used.value

    def encode_archive(self, cols, heap=None, out=None):
        """Device MIXED columns -> an archive batch (Vec<BatchItem>). Returns a uint8 tensor on
        the device (out=None), or the length written into `out` (a device tensor)."""
        import torch
        err, n = NetidxError(), C.c_uint64(0)
        if out is None:
            _check(lib().nxg_encode_archive_batch(self.ctx, C.byref(cols.s), _heap_ptr(heap),
                                                  None, 0, C.byref(n), C.byref(err)), err)
            out = torch.empty(max(n.value, 1), dtype=torch.uint8, device=cols.id.device)
            _check(lib().nxg_encode_archive_batch(self.ctx, C.byref(cols.s), _heap_ptr(heap),
                                                  C.c_void_p(out.data_ptr()), out.numel(),
                                                  C.byref(n), C.byref(err)), err)
            return out[: n.value]
        _check(lib().nxg_encode_archive_batch(self.ctx, C.byref(cols.s), _heap_ptr(heap),
                                              C.c_void_p(out.data_ptr()), out.numel(), C.byref(n),
                                              C.byref(err)), err)
        return n.value

    def zstd_dict(self, data):
        """A compressed archive's zstd dictionary on the device (nxg_zstd_dict_new)."""
        b = bytes(data)
        a = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b + b"\0")
        err = NetidxError()
        h = lib().nxg_zstd_dict_new(self.ctx, a, len(b), C.byref(err))
        _check(bool(h), err)
        return ZstdDict(h)

    def archive_decompress(self, src, records, indexed=False, zdict=None, out=None):
        """Compressed archive records (host bytes `src`, [(off, len)] after each RecordHeader)
        decompressed on the device (nxg_archive_decompress). Returns (device uint8 tensor,
        [(out_off, out_len, err)])."""
        import torch
        b = src if isinstance(src, np.ndarray) else np.frombuffer(bytes(src), np.uint8)
        b = np.ascontiguousarray(b)
        n = len(records)
        recs = (NxgArchiveRecord * max(n, 1))()
        for i, (o, ln) in enumerate(records):
            recs[i].off, recs[i].len = o, ln
        need, err = C.c_uint64(0), NetidxError()
        dh = zdict.h if zdict else None
        _check(lib().nxg_archive_decompress(self.ctx, dh, C.c_void_p(b.ctypes.data), len(b), recs,
                                            n, indexed, None, 0, C.byref(need), C.byref(err)), err)
        if out is None:
            out = torch.empty(max(need.value, 1), dtype=torch.uint8, device="cuda")
        _check(lib().nxg_archive_decompress(self.ctx, dh, C.c_void_p(b.ctypes.data), len(b), recs,
                                            n, indexed, C.c_void_p(out.data_ptr()), out.numel(),
                                            C.byref(need), C.byref(err)), err)
        return out, [(recs[i].out_off, recs[i].out_len, recs[i].err) for i in range(n)]

    def decode_batch(self, frame, layout=LAYOUT_MIXED, flags=0, device="cuda"):
        """Decode one frame payload; returns (Columns, NxgStatus)."""
        n = len(frame) if not hasattr(frame, "numel") else frame.numel()
        cols = Columns.for_frame(n, layout, device)
        st = self.decode_into(frame, n, cols, flags)
        return cols, st

    def last_status(self):
        """(fast_fail, irregular, path, n_rows, err_kind, timeout) of the last completed decode's
        device status (diagnostics, not ABI)."""
        a = (C.c_ulonglong * 6)()
        lib().nxg_debug_status(C.c_void_p(self.ctx), a)
        return list(a)

    def last_diag(self):
        """DevStatus.diag of the last completed decode (diagnostics, not ABI): for an f64 frame,
        diag[1] == 1 when the sequential-id decoder (nxg_decode_f64_seq.hip) produced it."""
        a = (C.c_ulonglong * 8)()
        lib().nxg_debug_diag(C.c_void_p(self.ctx), a)
        return list(a)

    def last_encode_kernel(self):
        """Which f64 encoder wrote the last f64 encode (diagnostics, not ABI): "seq" for the
        sequential-id kernel (nxg_encode_f64_seq.hip), "tile" for the tiled look-back kernel."""
        f = lib().nxg_debug_enc_kernel
        f.restype = C.c_uint
        return {1: "seq", 2: "tile"}.get(f(C.c_void_p(self.ctx)), None)

    def decode_async(self, dframe_ptr, nbytes, cols, flags=0):
        err = NetidxError()
        _check(lib().nxg_decode_updates_async(self.ctx, C.c_void_p(dframe_ptr), nbytes,
                                              C.byref(cols.s), flags, C.byref(err)), err)

    def decode_frames_async(self, dframe_ptrs, lens, cols_list, flags=0):
        """A backlog of device frames (nxg_decode_frames_async), decoded in order; frame j into
        cols_list[j] (one Columns object may repeat). Complete with sync()."""
        n = len(dframe_ptrs)
        fp = (C.c_void_p * n)(*[int(p) for p in dframe_ptrs])
        ln = (C.c_uint64 * n)(*[int(x) for x in lens])
        cp = (C.c_void_p * n)(*[C.addressof(c.s) for c in cols_list])
        err = NetidxError()
        _check(lib().nxg_decode_frames_async(self.ctx, n, fp, ln, cp, flags, C.byref(err)), err)

    def sync(self, check=True):
        st, err = NxgStatus(), NetidxError()
        ok = lib().nxg_ctx_sync(self.ctx, C.byref(st), C.byref(err))
        self.__dict__["_pending_len"] = []
        _check(ok, err)
        if check and st.err_kind:
            raise PackError(st.err_kind, st.err_offset)
        return st

    def dispatch_updates(self, table, ids, n_rows=None, cap=None):
        """process_updates_batch (connection.rs:546-567) for decoded rows: `ids` is the device id
        column (int64/uint64 tensor). Returns a Dispatch."""
        import torch
        n = ids.numel() if n_rows is None else int(n_rows)
        dev = ids.device
        streams = table.stream_chan.numel()
        if cap is None:  # each row reaches at most the largest fan-out of any subscription
            offs = table.slot_stream_off.cpu().numpy().view(np.uint32).astype(np.int64)
            cap = n * int((offs[1:] - offs[:-1]).max()) if streams else 0
        chan_off = torch.zeros(table.n_chans + 1, dtype=torch.int64, device=dev)
        ent_sub = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        ent_row = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        last_row = torch.empty(max(table.slot_sub_id.numel(), 1), dtype=torch.int64, device=dev)
        tb = table.c_struct()
        out = NxgDispatch(cap, chan_off.data_ptr(), ent_sub.data_ptr(), ent_row.data_ptr(),
                          last_row.data_ptr(), 0, 0)
        err = NetidxError()
        _check(lib().nxg_dispatch_updates(self.ctx, C.byref(tb), C.c_void_p(ids.data_ptr()), n,
                                          C.byref(out), C.byref(err)), err)
        return Dispatch(chan_off, ent_sub, ent_row, last_row[: table.slot_sub_id.numel()],
                        out.n_entries, out.n_unmatched)

    def partition_by_tag(self, cols, view=None):
        """nxg_partition_by_tag: the type-partitioned view of decoded mixed device columns
        (per-tag dense runs of fixed / aux, the dense index -> row map, the row -> rank map).
        Returns a TagView (its device tensors are reused when `view` is passed)."""
        n = int(cols.s.n_rows)
        if view is None or view.cap < n:
            view = TagView(max(n, 1), cols.device)
        v = NxgTagView()
        v.cap_rows = view.cap
        v.rank, v.row_of = view.rank.data_ptr(), view.row_of.data_ptr()
        v.fixed, v.aux = view.fixed.data_ptr(), view.aux.data_ptr()
        err = NetidxError()
        _check(lib().nxg_partition_by_tag(self.ctx, C.byref(cols.s), C.byref(v), C.byref(err)),
               err)
        view.n_rows = int(v.n_rows)
        view.count = np.frombuffer(bytes(v.count), np.uint64).copy()
        view.off = np.frombuffer(bytes(v.off), np.uint64).copy()
        return view

    def publish_commit(self, table, batch, kind, to_client=None, heap=None, cap=None):
        """UpdateBatch::commit on device columns: `batch` (Columns: id, tag, fixed, aux and the
        children of its Array/Map/Error(Value) values), per-row
        `kind` (PUB_UPDATE / PUB_UPDATE_CHANGED / PUB_UPDATE_CLIENT, uint8 tensor) and
        `to_client` (int32 tensor, for PUB_UPDATE_CLIENT rows). Returns a Dispatch whose
        channels are the clients and whose entries are (Id, row); last_row[slot] = 1 + the row
        that became current."""
        import torch
        n = batch.s.n_rows
        dev = batch.id.device
        if to_client is None:
            to_client = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        if cap is None:
            offs = table.slot_client_off.cpu().numpy().view(np.uint32).astype(np.int64)
            cap = n * max(1, int((offs[1:] - offs[:-1]).max()) if len(offs) > 1 else 1)
        chan_off = torch.zeros(table.n_clients + 1, dtype=torch.int64, device=dev)
        ent_id = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        ent_row = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        n_slots = table.slot_client_off.numel() - 1
        last_row = torch.empty(max(n_slots, 1), dtype=torch.int64, device=dev)
        out = NxgDispatch(cap, chan_off.data_ptr(), ent_id.data_ptr(), ent_row.data_ptr(),
                          last_row.data_ptr(), 0, 0)
        tb = table.c_struct()
        err = NetidxError()
        _check(lib().nxg_publish_commit(self.ctx, C.byref(tb), C.byref(batch.s), _heap_ptr(heap),
                                        C.c_void_p(kind.data_ptr()),
                                        C.c_void_p(to_client.data_ptr()), C.byref(out),
                                        C.byref(err)), err)
        return Dispatch(chan_off, ent_id, ent_row, last_row[:n_slots], out.n_entries,
                        out.n_unmatched)

    def publish_unsubscribes(self, ids, clients, n_clients):
        """The commit's unsubscribes (publisher/mod.rs:820-832): device tensors of Ids (int64)
        and clients (int32), in queue order. Returns a Dispatch whose channels are the clients
        and whose entries are (Id, index in the queue)."""
        import torch
        n = ids.numel()
        dev = ids.device
        chan_off = torch.zeros(n_clients + 1, dtype=torch.int64, device=dev)
        ent_id = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        ent_row = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        out = NxgDispatch(n, chan_off.data_ptr(), ent_id.data_ptr(), ent_row.data_ptr(), None,
                          0, 0)
        err = NetidxError()
        _check(lib().nxg_publish_unsubscribes(self.ctx, C.c_void_p(ids.data_ptr()),
                                              C.c_void_p(clients.data_ptr()), n, n_clients,
                                              C.byref(out), C.byref(err)), err)
        return Dispatch(chan_off, ent_id, ent_row, chan_off[:0], out.n_entries, 0)

    def encoded_len(self, cols, heap=None):
        n, err = C.c_uint64(0), NetidxError()
        _check(lib().nxg_encoded_len(self.ctx, C.byref(cols.s), _heap_ptr(heap), C.byref(n),
                                     C.byref(err)), err)
        return n.value

    def encode_into(self, cols, heap, out_ptr, cap):
        n, err = C.c_uint64(0), NetidxError()
        _check(lib().nxg_encode_updates(self.ctx, C.byref(cols.s), _heap_ptr(heap),
                                        C.c_void_p(out_ptr), cap, C.byref(n), C.byref(err)), err)
        return n.value

    def encode_batch(self, cols, heap=None):
        """Encode columns to one frame payload (torch uint8 tensor on the columns' device)."""
        import torch
        n = self.encoded_len(cols, heap)
        out = torch.empty(max(n, 16), dtype=torch.uint8, device=cols.device)
        m = self.encode_into(cols, heap, out.data_ptr(), n)
        assert m == n
        return out[:n]

    def decode_range(self, dframe, frame_len, begin, end, cols):
        """Decode the messages that start in [begin, end) of a device frame (rows at cols[0:]);
        returns the NxgRange summary (entry / exit / n_rows / ok)."""
        ptr = dframe.data_ptr() if hasattr(dframe, "data_ptr") else int(dframe)
        rng, err = NxgRange(), NetidxError()
        _check(lib().nxg_decode_range(self.ctx, C.c_void_p(ptr), frame_len, begin, end,
                                      C.byref(cols.s), C.byref(rng), C.byref(err)), err)
        return rng

    def decode_share(self, dframe, frame_len, share, shares, cols):
        """nxg_decode_share: the frame decoded whole, row share `share` of `shares` into cols;
        returns (first row of the share, NxgStatus)."""
        ptr = dframe.data_ptr() if hasattr(dframe, "data_ptr") else int(dframe)
        off, st, err = C.c_uint64(0), NxgStatus(), NetidxError()
        _check(lib().nxg_decode_share(self.ctx, C.c_void_p(ptr), frame_len, share, shares,
                                      C.byref(cols.s), C.byref(off), C.byref(st), C.byref(err)),
               err)
        return off.value, st

    def encode_frames(self, cols, heap, out_ptr, cap, max_frames=16):
        """Encode into out_ptr and return (total length, [frame payload lengths]) as
        WriteChannel::queue_send / try_flush would cut them (MAX_BATCH, channel.rs:177-257)."""
        n, k, err = C.c_uint64(0), C.c_uint64(0), NetidxError()
        chunks = np.zeros(max_frames, np.uint64)
        _check(lib().nxg_encode_frames(self.ctx, C.byref(cols.s), _heap_ptr(heap),
                                       C.c_void_p(out_ptr), cap, C.byref(n),
                                       C.c_void_p(chunks.ctypes.data), max_frames, C.byref(k),
                                       C.byref(err)), err)
        return n.value, [int(x) for x in chunks[: k.value]]

    def encode_async(self, cols, heap, out_ptr, cap):
        """Enqueue an encode; the returned c_uint64 holds the length after sync()."""
        n, err = C.c_uint64(0), NetidxError()
        self.__dict__.setdefault("_pending_len", []).append(n)  # written by the C side at sync
        _check(lib().nxg_encode_updates_async(self.ctx, C.byref(cols.s), _heap_ptr(heap),
                                              C.c_void_p(out_ptr), cap, C.byref(n),
                                              C.byref(err)), err)
        return n


NO_SLOT = 0xFFFFFFFF


class SubTable:
    """Device-resident Id -> subscription table: ConnectionCtx.subscriptions and each Sub's
    sub_id / streams / last (netidx/src/subscriber/connection.rs:54-60), as the CSR arrays of
    include/nxg_codec.h's NxgSubTable. Publisher Ids are dense (netidx-core/src/utils.rs:130-134),
    so the map is a table indexed by Id."""

    def __init__(self, slot_of_id, slot_sub_id, slot_stream_off, stream_chan, slot_has_last,
                 n_chans, device="cuda"):
        import torch

        def t(a, dt):
            return torch.as_tensor(np.array(a, dtype=dt, copy=True)).to(device)

        self.slot_of_id = t(slot_of_id, np.uint32).view(torch.int32)
        self.slot_sub_id = t(slot_sub_id, np.uint64).view(torch.int64)
        self.slot_stream_off = t(slot_stream_off, np.uint32).view(torch.int32)
        self.stream_chan = t(stream_chan, np.uint32).view(torch.int32)
        self.slot_has_last = t(slot_has_last, np.uint8)
        self.n_chans = int(n_chans)
        assert self.slot_stream_off.numel() == self.slot_sub_id.numel() + 1
        assert self.slot_has_last.numel() == self.slot_sub_id.numel()

    @classmethod
    def from_subscriptions(cls, subs, n_chans, n_ids=None, device="cuda"):
        """subs: {id: (sub_id, [chan, ...], keeps_last)} -- one subscription per Id, its streams
        in registration order (handle_connect_stream, connection.rs:320-359)."""
        n_ids = (max(subs) + 1 if subs else 0) if n_ids is None else n_ids
        slot_of_id = np.full(n_ids, NO_SLOT, np.uint32)
        sub_ids, offs, chans, last = [], [0], [], []
        for slot, (i, (sid, streams, keep)) in enumerate(sorted(subs.items())):
            if i < n_ids:
                slot_of_id[i] = slot
            sub_ids.append(sid)
            chans.extend(streams)
            offs.append(len(chans))
            last.append(1 if keep else 0)
        return cls(slot_of_id, np.array(sub_ids, np.uint64), np.array(offs, np.uint32),
                   np.array(chans, np.uint32), np.array(last, np.uint8), n_chans, device)

    def c_struct(self):
        return NxgSubTable(self.slot_of_id.numel(), self.slot_of_id.data_ptr(),
                           self.slot_sub_id.numel(), self.slot_sub_id.data_ptr(),
                           self.slot_stream_off.data_ptr(), self.stream_chan.data_ptr(),
                           self.slot_has_last.data_ptr(), self.n_chans)


class TagView:
    """Device tensors of the type-partitioned view (include/nxg_codec.h NxgTagView): tag t's rows
    are the dense indices [off[t], off[t+1]): row_of (int32 holding u32), fixed (int64), aux
    (int32); rank[i] is row i's index among its tag's rows."""

    def __init__(self, cap, device="cuda"):
        import torch
        self.cap = cap
        self.rank = torch.empty(cap, dtype=torch.int32, device=device)
        self.row_of = torch.empty(cap, dtype=torch.int32, device=device)
        self.fixed = torch.empty(cap, dtype=torch.int64, device=device)
        self.aux = torch.empty(cap, dtype=torch.int32, device=device)
        self.n_rows, self.count, self.off = 0, None, None

    def numpy(self):
        n = self.n_rows
        return {"rank": self.rank[:n].cpu().numpy().view(np.uint32),
                "row_of": self.row_of[:n].cpu().numpy().view(np.uint32),
                "fixed": self.fixed[:n].cpu().numpy().view(np.uint64),
                "aux": self.aux[:n].cpu().numpy().view(np.uint32),
                "count": self.count, "off": self.off}


class Dispatch:
    """Per-channel update batches (by_chan, connection.rs:62-65): channel c's batch is
    (ent_sub, ent_row)[chan_off[c]:chan_off[c+1]], in batch order; last_row[slot] = 1 + the last
    row of the slot's subscription (0: none)."""

    def __init__(self, chan_off, ent_sub, ent_row, last_row, n_entries, n_unmatched):
        self.chan_off, self.ent_sub, self.ent_row, self.last_row = chan_off, ent_sub, ent_row, last_row
        self.n_entries, self.n_unmatched = n_entries, n_unmatched

    def batches(self):
        """{chan: [(sub_id, row), ...]} on the host (non-empty channels only)."""
        off = self.chan_off.cpu().numpy().view(np.uint64)
        sub = self.ent_sub[: self.n_entries].cpu().numpy().view(np.uint64)
        row = self.ent_row[: self.n_entries].cpu().numpy().view(np.uint64)
        return {c: list(zip(sub[off[c]:off[c + 1]].tolist(), row[off[c]:off[c + 1]].tolist()))
                for c in range(len(off) - 1) if off[c + 1] > off[c]}


PUB_UPDATE, PUB_UPDATE_CHANGED, PUB_UPDATE_CLIENT = 0, 1, 2
TAG_UNSUBSCRIBED = 0x40  # archive rows: Event::Unsubscribed


class PubTable:
    """Device-resident publisher state for UpdateBatch::commit (netidx/src/publisher/mod.rs:
    776-845): pb.by_id as a dense slot table (Id -> slot), each slot's subscribed clients (CSR)
    and current value (tag/fixed/aux columns; text, Decimal and Abstract bytes in cur_heap; the
    elements of container values in cur_ctag/cur_cfixed/cur_caux)."""

    def __init__(self, slot_of_id, slot_client_off, client, n_clients, cur_tag, cur_fixed,
                 cur_aux=None, cur_heap=None, device="cuda", cur_ctag=None, cur_cfixed=None,
                 cur_caux=None):
        import torch

        def t(a, dt):
            return torch.as_tensor(np.array(a, dtype=dt, copy=True)).to(device)

        self.slot_of_id = t(slot_of_id, np.uint32).view(torch.int32)
        self.slot_client_off = t(slot_client_off, np.uint32).view(torch.int32)
        self.client = t(client, np.uint32).view(torch.int32)
        self.n_clients = int(n_clients)
        self.cur_tag = None if cur_tag is None else t(cur_tag, np.uint8)
        self.cur_fixed = t(cur_fixed, np.uint64).view(torch.int64)
        self.cur_aux = None if cur_aux is None else t(cur_aux, np.uint32).view(torch.int32)
        self.cur_heap = None if cur_heap is None else t(cur_heap, np.uint8)
        self.cur_ctag = None if cur_ctag is None else t(cur_ctag, np.uint8)
        self.cur_cfixed = None if cur_cfixed is None else t(cur_cfixed, np.uint64).view(torch.int64)
        self.cur_caux = None if cur_caux is None else t(cur_caux, np.uint32).view(torch.int32)

    def c_struct(self):
        def p(x):
            return x.data_ptr() if x is not None and x.numel() else None
        return NxgPubTable(self.slot_of_id.numel(), p(self.slot_of_id),
                           self.slot_client_off.numel() - 1, p(self.slot_client_off),
                           p(self.client), self.n_clients, p(self.cur_tag), p(self.cur_fixed),
                           p(self.cur_aux), p(self.cur_heap), p(self.cur_ctag),
                           p(self.cur_cfixed), p(self.cur_caux))


def _heap_ptr(heap):
    if heap is None:
        return C.c_void_p(0)
    if hasattr(heap, "data_ptr"):
        return C.c_void_p(heap.data_ptr())
    if isinstance(heap, np.ndarray):
        return C.c_void_p(heap.ctypes.data)
    return C.c_void_p(int(heap))


# ---- host framing (netidx/src/channel.rs) ----------------------------------------------------
class FrameReader:
    """read_task's frame assembly (channel.rs:379-443): feed() the bytes read from a socket in
    any pieces; frames() yields each complete frame payload in order (a copy, as bytes, or
    written into `into`). An encrypted frame raises CodecError("encryption is not supported")."""

    def __init__(self):
        err = NetidxError()
        r = lib().nxg_frame_reader_new(C.byref(err))
        if not r:
            _check(False, err)
        self.r = r

    def close(self):
        if getattr(self, "r", None):
            lib().nxg_frame_reader_free(self.r)
            self.r = None

    def __del__(self):
        self.close()

    def feed(self, data, n=None):
        """Append bytes (bytes, bytearray, memoryview or numpy uint8); `n`: only the first n."""
        if isinstance(data, np.ndarray):
            ptr, size = data.ctypes.data, data.nbytes
        elif isinstance(data, bytes):
            ptr, size = C.cast(C.c_char_p(data), C.c_void_p).value, len(data)
        else:
            mv = memoryview(data).cast("B")
            size = mv.nbytes
            ptr = C.addressof((C.c_uint8 * size).from_buffer(mv)) if size else 0
        size = size if n is None else min(size, int(n))
        err = NetidxError()
        _check(lib().nxg_frame_reader_push(self.r, C.c_void_p(ptr), size, C.byref(err)), err)

    def next_view(self):
        """(address, length) of the next complete payload, valid until the next feed(); None
        if it is not complete yet."""
        p, n, err = C.c_void_p(), C.c_uint64(), NetidxError()
        rc = lib().nxg_frame_reader_next(self.r, C.byref(p), C.byref(n), C.byref(err))
        if rc < 0:
            _check(False, err)
        return (p.value or 0, n.value) if rc == 1 else None

    def frames(self):
        while True:
            v = self.next_view()
            if v is None:
                return
            yield C.string_at(v[0], v[1]) if v[1] else b""

    def buffered(self):
        return lib().nxg_frame_reader_buffered(self.r)


def _msg(fn, *args):
    n = fn(*args, None, 0)
    if n < 0:
        raise CodecError(f"message builder failed ({-n})")
    out = (C.c_uint8 * max(n, 1))()
    m = fn(*args, out, n)
    assert m == n
    return bytes(out[:n])


def msg_subscribe(path, timestamp=0, permissions=0, token=b"", resolver=(0, 0)):
    """To::Subscribe (netproto publisher.rs:57-63) as one len-wrapped message."""
    p = path.encode() if isinstance(path, str) else path
    tok = (C.c_uint8 * max(len(token), 1)).from_buffer_copy(token + b"\0")
    return _msg(lib().nxg_msg_subscribe, p, len(p), resolver[0], resolver[1], timestamp,
                permissions, tok, len(token))


def msg_subscribed(path, id, tag, fixed=0, aux=0, text=b""):
    """From::Subscribed(path, id, scalar value)."""
    p = path.encode() if isinstance(path, str) else path
    t = (C.c_uint8 * max(len(text), 1)).from_buffer_copy(text + b"\0")
    return _msg(lib().nxg_msg_subscribed, p, len(p), id, tag, fixed, aux, t)


def msg_heartbeat():
    return _msg(lib().nxg_msg_heartbeat)


def msg_update(id, tag, fixed=0, aux=0, text=b""):
    """From::Update(id, scalar value) as one len-wrapped message (nxg_msg_update)."""
    t = (C.c_uint8 * max(len(text), 1)).from_buffer_copy(text + b"\0")
    return _msg(lib().nxg_msg_update, id, tag, fixed, aux, t)


def _ip4(ip):
    a = [int(x) for x in ip.split(".")]
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


class Resolver:
    """A machine-local anonymous resolver server (nxg_resolver_start): threads in the library."""

    def __init__(self, ip="127.0.0.1", port=0, writer_ttl=120):
        err, bp = NetidxError(), C.c_uint16(0)
        self.h = lib().nxg_resolver_start(ip.encode(), port, C.byref(bp), writer_ttl,
                                          C.byref(err))
        _check(bool(self.h), err)
        self.ip, self.port = ip, bp.value

    def n_published(self):
        return lib().nxg_resolver_n_published(self.h)

    def stop(self):
        if self.h:
            lib().nxg_resolver_stop(self.h)
            self.h = None

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass


class ResolverClient:
    """A publisher's (write) or subscriber's (read) connection to a resolver."""

    def __init__(self, h, ttl=None):
        self.h, self.ttl = h, ttl

    @classmethod
    def write(cls, ip, port, write_addr):
        err, ttl = NetidxError(), C.c_uint64(0)
        h = lib().nxg_resolver_connect_write(ip.encode(), port, _ip4(write_addr[0]),
                                             write_addr[1], C.byref(ttl), C.byref(err))
        _check(bool(h), err)
        return cls(h, ttl.value)

    @classmethod
    def read(cls, ip, port):
        err = NetidxError()
        h = lib().nxg_resolver_connect_read(ip.encode(), port, C.byref(err))
        _check(bool(h), err)
        return cls(h)

    def publish(self, path):
        p = path.encode() if isinstance(path, str) else path
        err = NetidxError()
        _check(lib().nxg_resolver_publish(self.h, p, len(p), C.byref(err)), err)

    def resolve(self, path):
        """NxgResolved; publisher address as ("a.b.c.d", port) in .addr"""
        p = path.encode() if isinstance(path, str) else path
        r, err = NxgResolved(), NetidxError()
        _check(lib().nxg_resolver_resolve(self.h, p, len(p), C.byref(r), C.byref(err)), err)
        ip = r.publisher_ipv4
        r.addr = (f"{ip >> 24}.{(ip >> 16) & 255}.{(ip >> 8) & 255}.{ip & 255}", r.publisher_port)
        return r

    def close(self):
        if self.h:
            lib().nxg_resolver_client_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def msg_parse(buf, to=False):
    """Parse one control message (publisher::From, or To with to=True); returns NxgCtlMsg."""
    b = bytes(buf)
    a = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b + b"\0")
    m, err = NxgCtlMsg(), NetidxError()
    _check(lib().nxg_msg_parse(a, len(b), 1 if to else 0, C.byref(m), C.byref(err)), err)
    return m


class Session:
    """One publisher<->subscriber connection (nxg_session_*, include/nxg_codec.h): the handshake,
    frames, the device data path. Blocking; use one thread per session."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def connect(cls, ip, port):
        err = NetidxError()
        h = lib().nxg_session_connect(ip.encode(), port, C.byref(err))
        _check(bool(h), err)
        return cls(h)

    @classmethod
    def listen(cls, ip="127.0.0.1", port=0):
        err, bp = NetidxError(), C.c_uint16(0)
        h = lib().nxg_session_listen(ip.encode(), port, C.byref(bp), C.byref(err))
        _check(bool(h), err)
        s = cls(h)
        s.port = bp.value
        return s

    def accept(self):
        err = NetidxError()
        h = lib().nxg_session_accept(self.h, C.byref(err))
        _check(bool(h), err)
        return Session(h)

    def close(self):
        if self.h:
            lib().nxg_session_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        a = (C.c_uint64 * 4)()
        lib().nxg_session_stats(self.h, a)
        return dict(zip(("frames_in", "bytes_in", "frames_out", "bytes_out"), list(a)))

    def send(self, payload):
        b = bytes(payload)
        a = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b + b"\0")
        err = NetidxError()
        _check(lib().nxg_session_send(self.h, a, len(b), C.byref(err)), err)

    def recv_frame(self):
        """The next frame's payload (a copy)."""
        p, n, err = C.c_void_p(), C.c_uint64(), NetidxError()
        _check(lib().nxg_session_recv_frame(self.h, C.byref(p), C.byref(n), C.byref(err)), err)
        return C.string_at(p.value, n.value) if n.value else b""

    def recv_decode(self, codec, cols, flags=0):
        """The next frame decoded on the device; returns (NxgStatus, frame length)."""
        st, n, err = NxgStatus(), C.c_uint64(), NetidxError()
        _check(lib().nxg_session_recv_decode(self.h, codec.ctx, C.byref(cols.s), flags,
                                             C.byref(st), C.byref(n), C.byref(err)), err)
        return st, n.value

    def publish(self, codec, cols, heap=None):
        """Device columns encoded on the GPU and written as frames; returns the bytes sent."""
        n, err = C.c_uint64(), NetidxError()
        _check(lib().nxg_session_publish(self.h, codec.ctx, C.byref(cols.s), _heap_ptr(heap),
                                         C.byref(n), C.byref(err)), err)
        return n.value


def range_link(ranges, frame_len):
    """nxg_range_link: row offsets of consecutive byte-range summaries, or (None, bad_index)
    when range `bad_index` does not enter the chain where its predecessor leaves it."""
    n = len(ranges)
    arr = (NxgRange * max(n, 1))(*[r if isinstance(r, NxgRange) else NxgRange.of(r)
                                   for r in ranges])
    offs = np.zeros(max(n, 1), np.uint64)
    bad, err = C.c_uint32(0), NetidxError()
    ok = lib().nxg_range_link(arr, n, frame_len, C.c_void_p(offs.ctypes.data), C.byref(bad),
                              C.byref(err))
    if err.msg:
        lib().nxg_error_free(C.byref(err))
    return (offs[:n], None) if ok else (None, int(bad.value))


_AG = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)
_AGV = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32,
                   C.c_uint32)
_ELEN = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.POINTER(NxgColumns), C.c_void_p,
                    C.POINTER(C.c_uint64))
_ENC = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.POINTER(NxgColumns), C.c_void_p, C.c_void_p,
                   C.c_uint64, C.POINTER(C.c_uint64))
_DRNG = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                    C.POINTER(NxgColumns), C.POINTER(NxgRange))
_DSHR = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                    C.POINTER(NxgColumns), C.POINTER(C.c_uint64), C.POINTER(NxgStatus))


class NxgCommOps(C.Structure):
    _fields_ = [("user", C.c_void_p), ("allgather", _AG), ("allgatherv", _AGV),
                ("encoded_len", _ELEN), ("encode", _ENC), ("decode_range", _DRNG),
                ("decode_share", _DSHR)]


def _guard(fn):
    """A Python callback behind a C function pointer: an exception becomes `false` (the library
    then agrees the failure with the other ranks) after it is printed."""
    def call(*a):
        try:
            r = fn(*a)
            return True if r is None else bool(r)
        except Exception:  # noqa: BLE001 -- reported, then turned into the C failure code
            import traceback
            traceback.print_exc()
            return False
    return call


class Comm:
    """Communicator of the sharded calls (one process per GPU): RCCL (nxg_comm_init), or a
    caller-provided transport and optional local codec (nxg_comm_init_ops, Comm.with_ops)."""

    @staticmethod
    def unique_id():
        buf, err = (C.c_uint8 * 128)(), NetidxError()
        _check(lib().nxg_comm_unique_id(C.byref(buf), C.byref(err)), err)
        return bytes(buf)

    def __init__(self, codec, nranks, rank, uid):
        err = NetidxError()
        b = (C.c_uint8 * 128).from_buffer_copy(uid)
        self.h = lib().nxg_comm_init(codec.ctx, nranks, rank, C.byref(b), C.byref(err))
        _check(self.h is not None, err)
        self.codec, self.nranks, self.rank = codec, nranks, rank

    @classmethod
    def with_ops(cls, codec, nranks, rank, allgather, allgatherv, encoded_len=None, encode=None,
                 decode_range=None, decode_share=None):
        """nxg_comm_init_ops. allgather(mine: bytes) -> bytes of every rank's, in rank order;
        allgatherv(buf_ptr, offsets, nranks, rank) fills every shard of the buffer at its
        offset. The optional local codec: encoded_len(NxgColumns) -> int; encode(NxgColumns,
        out_ptr, cap) -> int; decode_range(frame_ptr, frame_len, begin, end, NxgColumns) ->
        (begin, end, entry, exit, n_rows, ok, err_kind); and, optionally with it,
        decode_share(frame_ptr, frame_len, share, shares, NxgColumns) -> (row_off, n_rows,
        err_kind, err_offset). codec may be None with the codec."""
        self = cls.__new__(cls)

        def ag(user, mine, all_, nbytes):
            got = allgather(C.string_at(mine, nbytes))
            assert len(got) == nbytes * nranks
            C.memmove(all_, got, len(got))

        def agv(user, buf, off, n, r):
            allgatherv(int(buf or 0), [int(off[i]) for i in range(n + 1)], int(n), int(r))

        fns = [_AG(_guard(ag)), _AGV(_guard(agv))]
        if decode_range is not None:
            def elen(user, cols, heap, out):
                out[0] = int(encoded_len(cols.contents))

            def enc(user, cols, heap, out, cap, n):
                n[0] = int(encode(cols.contents, int(out or 0), int(cap)))

            def drng(user, frame, flen, b, e, cols, rng):
                t = decode_range(int(frame or 0), int(flen), int(b), int(e), cols.contents)
                rng[0] = t if isinstance(t, NxgRange) else NxgRange.of(t)

            fns += [_ELEN(_guard(elen)), _ENC(_guard(enc)), _DRNG(_guard(drng))]
        else:
            fns += [_ELEN(), _ENC(), _DRNG()]
        if decode_share is not None:
            def dshr(user, frame, flen, share, shares, cols, off, st):
                o, nr, ek, eo = decode_share(int(frame or 0), int(flen), int(share), int(shares),
                                             cols.contents)
                off[0] = int(o)
                st[0] = NxgStatus(n_rows=int(nr), err_kind=int(ek), err_offset=int(eo))

            fns.append(_DSHR(_guard(dshr)))
        else:
            fns.append(_DSHR())
        self._fns = fns  # the C function pointers live as long as the communicator
        self.ops = NxgCommOps(None, *fns)
        err = NetidxError()
        self.h = lib().nxg_comm_init_ops(codec.ctx if codec else None, nranks, rank,
                                         C.byref(self.ops), C.byref(err))
        _check(self.h is not None, err)
        self.codec, self.nranks, self.rank = codec, nranks, rank
        return self

    def _ctx(self):
        return self.codec.ctx if self.codec else None

    def close(self):
        if getattr(self, "h", None):
            lib().nxg_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode_allgather(self, cols, heap, out_ptr, cap):
        """Every rank's shard into one frame on every rank; returns (length, shard offsets)."""
        n, err = C.c_uint64(0), NetidxError()
        offs = np.zeros(self.nranks, np.uint64)
        cs = cols.s if hasattr(cols, "s") else cols
        _check(lib().nxg_encode_allgather(self._ctx(), self.h, C.byref(cs),
                                          _heap_ptr(heap), C.c_void_p(out_ptr), cap, C.byref(n),
                                          C.c_void_p(offs.ctypes.data), C.byref(err)), err)
        return n.value, [int(x) for x in offs]

    def decode_sharded(self, dframe, frame_len, cols):
        """This rank's byte range of one frame (or, for a frame the byte-range decoders decline,
        its row share: rng.ok == 2); returns (first global row, NxgRange)."""
        ptr = dframe.data_ptr() if hasattr(dframe, "data_ptr") else int(dframe)
        off, rng, err = C.c_uint64(0), NxgRange(), NetidxError()
        cs = cols.s if hasattr(cols, "s") else cols
        _check(lib().nxg_decode_sharded(self._ctx(), self.h, C.c_void_p(ptr), frame_len,
                                        C.byref(cs), C.byref(off), C.byref(rng),
                                        C.byref(err)), err)
        return off.value, rng


def frame_split(msg_lens):
    """Frame payload lengths for a queue of encoded messages (WriteChannel::queue_send)."""
    a = np.ascontiguousarray(msg_lens, np.uint64)
    out = np.zeros(len(a) + 1, np.uint64)
    n = lib().nxg_frame_split(a.ctypes.data, len(a), out.ctypes.data, len(out))
    if n < 0:
        raise CodecError("message exceeds MAX_BATCH")
    return out[:n]


def frame_header(payload_len, encrypted=False):
    b = (C.c_uint8 * 4)()
    lib().nxg_frame_header(payload_len, encrypted, b)
    return bytes(b)


def frame_parse_header(buf):
    ln, enc = C.c_uint32(0), C.c_bool(False)
    a = np.frombuffer(bytes(buf), np.uint8)
    n = lib().nxg_frame_parse_header(a.ctypes.data, len(a), C.byref(ln), C.byref(enc))
    return (None if n == 0 else (ln.value, bool(enc.value)))


def columns_from_arrays(id, fixed, tag=None, aux=None, ctag=None, cfixed=None, caux=None,
                        ctl_row=None, ctl_off=None, ctl_len=None, ctl_variant=None,
                        device="cuda"):
    """Build encode-input Columns from host numpy arrays (uploaded to `device`)."""
    import torch
    n = len(id)
    nc = 0 if ctag is None else len(ctag)
    nk = 0 if ctl_row is None else len(ctl_row)
    layout = LAYOUT_F64 if tag is None else LAYOUT_MIXED
    cols = Columns(n, nc, nk, layout, device)

    def put(name, arr, dt):
        if arr is None or len(arr) == 0:
            return
        src = torch.from_numpy(np.ascontiguousarray(arr).view(dt))
        cols.t[name][: len(arr)].copy_(src)

    put("id", id, np.int64)
    put("fixed", fixed, np.int64)
    put("tag", tag, np.uint8)
    put("aux", aux, np.int32)
    put("ctag", ctag, np.uint8)
    put("cfixed", cfixed, np.int64)
    put("caux", caux, np.int32)
    put("ctl_row", ctl_row, np.int64)
    put("ctl_off", ctl_off, np.int64)
    put("ctl_len", ctl_len, np.int32)
    put("ctl_variant", ctl_variant, np.uint8)
    cols.s.n_rows, cols.s.n_children, cols.s.n_ctl = n, nc, nk
    return cols
