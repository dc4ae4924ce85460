"""netidx_amd: MI355X-native batch-update codec for netidx's publisher->subscriber stream.

The hot path (decode/encode of length-wrapped From::Update(Id, Value) batches) and the
subscriber's update dispatch run in hand-written gfx950 HIP kernels behind the C ABI in
include/nxg_codec.h. This package is the
Python binding used by the tests and bench.py.
"""
from .codec import (BUFFER_SHORT, CAPACITY, DEPTH, HINT_MIXED, INVALID_FORMAT, LAYOUT_F64,
                    LAYOUT_MIXED, NO_SLOT, NOT_F64, TOO_BIG, UNKNOWN_TAG, Codec, CodecError,
                    Columns, Dispatch, FrameReader, PackError, PubTable, PUB_UPDATE, PUB_UPDATE_CHANGED,
                    PUB_UPDATE_CLIENT, SubTable, columns_from_arrays, frame_header,
                    frame_parse_header, frame_split, lib, Comm, NxgRange, range_link, Session,
                    msg_subscribe, msg_subscribed, msg_heartbeat, msg_parse, msg_update,
                    TAG_UNSUBSCRIBED, Resolver, ResolverClient, TagView, TAG_BINS)

__all__ = ["Codec", "Columns", "PackError", "CodecError", "columns_from_arrays", "lib",
           "frame_split", "frame_header", "frame_parse_header", "LAYOUT_F64", "LAYOUT_MIXED",
           "HINT_MIXED", "UNKNOWN_TAG", "TOO_BIG", "INVALID_FORMAT", "BUFFER_SHORT", "DEPTH",
           "CAPACITY", "NOT_F64", "SubTable", "Dispatch", "NO_SLOT",
           "PubTable", "FrameReader", "PUB_UPDATE", "PUB_UPDATE_CHANGED", "PUB_UPDATE_CLIENT",
           "Comm", "NxgRange", "range_link", "Session", "msg_subscribe", "msg_subscribed",
           "msg_heartbeat", "msg_parse", "msg_update", "TAG_UNSUBSCRIBED", "Resolver",
           "ResolverClient", "TagView", "TAG_BINS"]
