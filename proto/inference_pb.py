"""Runtime-built protobuf classes for ``proto/inference.proto`` (no protoc needed).

``grpc_tools`` is not part of the image, so instead of generated
``*_pb2.py`` files the message descriptors are assembled here from a compact
field table that mirrors ``inference.proto`` field-for-field (names, numbers,
types, ``repeated`` and the ``metadata`` map).  The wire format is therefore
identical to what protoc-generated stubs produce.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "distributed_inference"
T = descriptor_pb2.FieldDescriptorProto
_TYPES = {"string": T.TYPE_STRING, "bytes": T.TYPE_BYTES, "int32": T.TYPE_INT32, "int64": T.TYPE_INT64,
          "bool": T.TYPE_BOOL, "float": T.TYPE_FLOAT}

# message -> [(name, number, type, repeated)] ; type may be a message name
MESSAGES = {
    "InferenceRequest": [("session_id", 1, "string", 0), ("step_id", 2, "string", 0), ("hidden_states", 3, "bytes", 0),
                         ("shape", 4, "int64", 1), ("dtype", 5, "string", 0), ("position", 6, "int32", 0),
                         ("kv_cache_keys", 7, "string", 1), ("next_worker_address", 8, "string", 0),
                         ("next_session_id", 9, "string", 0), ("metadata", 10, "map<string,string>", 1)],
    "InferenceResponse": [("session_id", 1, "string", 0), ("step_id", 2, "string", 0), ("hidden_states", 3, "bytes", 0),
                          ("shape", 4, "int64", 1), ("dtype", 5, "string", 0), ("updated_kv_keys", 6, "string", 1),
                          ("latency_ms", 7, "int64", 0), ("tokens_processed", 8, "int32", 0), ("success", 9, "bool", 0),
                          ("error_message", 10, "string", 0)],
    "ForwardRequest": [("session_id", 1, "string", 0), ("input", 2, "bytes", 0), ("shape", 3, "int64", 1),
                       ("dtype", 4, "string", 0), ("start_layer", 5, "int32", 0), ("end_layer", 6, "int32", 0),
                       ("position", 7, "int32", 0), ("kv_cache_keys", 8, "string", 1), ("use_cache", 9, "bool", 0)],
    "ForwardResponse": [("output", 1, "bytes", 0), ("shape", 2, "int64", 1), ("dtype", 3, "string", 0),
                        ("updated_kv_keys", 4, "string", 1), ("success", 5, "bool", 0), ("error_message", 6, "string", 0),
                        ("latency_ms", 7, "int64", 0)],
    "KVCacheRequest": [("prefix_key", 1, "string", 0), ("start_layer", 2, "int32", 0), ("end_layer", 3, "int32", 0),
                       ("layers", 4, "KVCacheLayer", 1)],
    "KVCacheLayer": [("layer_idx", 1, "int32", 0), ("keys", 2, "bytes", 0), ("values", 3, "bytes", 0),
                     ("shape", 4, "int64", 1), ("dtype", 5, "string", 0)],
    "KVCacheResponse": [("success", 1, "bool", 0), ("error_message", 2, "string", 0),
                        ("bytes_transferred", 3, "int64", 0), ("latency_ms", 4, "int64", 0)],
    "CreateSessionRequest": [("model_name", 1, "string", 0), ("max_length", 2, "int32", 0),
                             ("start_layer", 3, "int32", 0), ("end_layer", 4, "int32", 0),
                             ("temperature", 5, "float", 0), ("top_p", 6, "float", 0),
                             ("max_new_tokens", 7, "int32", 0)],
    "CreateSessionResponse": [("session_id", 1, "string", 0), ("success", 2, "bool", 0),
                              ("error_message", 3, "string", 0), ("cache_tokens_available", 4, "int32", 0)],
    "CloseSessionRequest": [("session_id", 1, "string", 0)],
    "CloseSessionResponse": [("success", 1, "bool", 0), ("error_message", 2, "string", 0)],
    "HealthCheckRequest": [("include_stats", 1, "bool", 0)],
    "HealthCheckResponse": [("healthy", 1, "bool", 0), ("worker_id", 2, "string", 0), ("status", 3, "string", 0),
                            ("gpu_memory_used_gb", 4, "float", 0), ("gpu_memory_total_gb", 5, "float", 0),
                            ("active_sessions", 6, "int32", 0), ("cache_tokens_used", 7, "int32", 0),
                            ("cache_tokens_available", 8, "int32", 0), ("throughput_tokens_per_sec", 9, "float", 0),
                            ("avg_latency_ms", 10, "float", 0)],
}

# rpc name -> (request, response, client_streaming, server_streaming)
SERVICE = "DistributedInference"
METHODS = {
    "StreamInference": ("InferenceRequest", "InferenceResponse", True, True),
    "Forward": ("ForwardRequest", "ForwardResponse", False, False),
    "TransferKVCache": ("KVCacheRequest", "KVCacheResponse", False, False),
    "CreateSession": ("CreateSessionRequest", "CreateSessionResponse", False, False),
    "CloseSession": ("CloseSessionRequest", "CloseSessionResponse", False, False),
    "HealthCheck": ("HealthCheckRequest", "HealthCheckResponse", False, False),
}


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="inference.proto", package=PACKAGE, syntax="proto3")
    for mname, fields in MESSAGES.items():
        m = fd.message_type.add(name=mname)
        for fname, num, ftype, rep in fields:
            f = m.field.add(name=fname, number=num)
            f.label = T.LABEL_REPEATED if rep else T.LABEL_OPTIONAL
            if ftype.startswith("map<"):
                entry = m.nested_type.add(name="MetadataEntry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=T.TYPE_STRING, label=T.LABEL_OPTIONAL)
                entry.field.add(name="value", number=2, type=T.TYPE_STRING, label=T.LABEL_OPTIONAL)
                f.type = T.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{mname}.MetadataEntry"
            elif ftype in _TYPES:
                f.type = _TYPES[ftype]
            else:
                f.type = T.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{ftype}"
    svc = fd.service.add(name=SERVICE)
    for name, (req, resp, cs, ss) in METHODS.items():
        svc.method.add(name=name, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}",
                       client_streaming=cs, server_streaming=ss)
    pool = descriptor_pool.DescriptorPool()
    fdesc = pool.Add(fd)
    classes = {}
    for mname in MESSAGES:
        desc = pool.FindMessageTypeByName(f"{PACKAGE}.{mname}")
        classes[mname] = message_factory.GetMessageClass(desc)
    return pool, classes


POOL, CLASSES = _build()
globals().update(CLASSES)
FULL_SERVICE = f"{PACKAGE}.{SERVICE}"
