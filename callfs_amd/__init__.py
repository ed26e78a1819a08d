"""callfs_amd — MI355X-native Reed-Solomon erasure-coding path for CallFS.

Drop-in for the GF(2^8) hot path behind erasure/codec.go (Encode / Decode) of
ebogdum/callfs: hand-written HIP kernels for gfx950 behind the C ABI in
include/callfs_rs.h (libcallfs_rs.so), with this package as the host-side mirror of
the Go `erasure` codec API. See DESIGN.md.
"""
from .erasure import (  # noqa: F401
    Codec,
    ErasureError,
    ErasureProfile,
    ErrInsufficientShards,
    ErrInvalidProfile,
    ErrShardCorrupted,
    ErrShardNoData,
    ErrShardNotFound,
    ErrShardSize,
    ErrShortData,
    ErrSingular,
    ErrTooFewShards,
    ErrUnsupportedProfile,
    decode_rows,
    encode_matrix,
    encode_shards,
    reconstruct,
    shard_checksum,
    shard_layout,
    verify,
)

__all__ = [
    "Codec", "ErasureProfile", "ErasureError", "ErrInsufficientShards", "ErrInvalidProfile",
    "ErrShardCorrupted", "ErrShardNotFound", "ErrShortData", "ErrTooFewShards",
    "ErrShardNoData", "ErrShardSize", "ErrSingular", "ErrUnsupportedProfile",
    "decode_rows", "encode_matrix", "encode_shards", "reconstruct", "verify",
    "shard_checksum", "shard_layout",
]
