"""GPU SHA-256 (ShardChecksum, erasure/codec.go:81-84) vs hashlib — bit-exact hex."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LENGTHS = [0, 1, 3, 55, 56, 57, 63, 64, 65, 100, 119, 120, 121, 127, 128, 129, 191, 192,
           1000, 4095, 4096, 65537, 1 << 20, 6_710_887]


@pytest.mark.parametrize("misalign", [0, 1, 3, 16])
def test_sha256_lengths_vs_hashlib(native_lib, misalign):
    import torch
    from callfs_amd.device import HashPlan
    rng = np.random.default_rng(misalign)
    blobs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in LENGTHS]
    offs, pos = [], 0
    for b in blobs:
        pos = (pos + 255) // 256 * 256 + misalign
        offs.append(pos)
        pos += len(b)
    buf = np.zeros(pos + 16, np.uint8)
    for o, b in zip(offs, blobs):
        buf[o:o + len(b)] = np.frombuffer(b, np.uint8)
    d = torch.from_numpy(buf).to("cuda:0")
    hp = HashPlan([d.data_ptr() + o for o in offs], [len(b) for b in blobs])
    got = hp.hexdigests()
    assert got == [hashlib.sha256(b).hexdigest() for b in blobs]


def test_shard_checksums_of_encoded_batch(native_lib):
    import torch
    from callfs_amd import shard_checksum
    from callfs_amd.device import Plan, StripeBatch, shard_checksums
    sb = StripeBatch(10, 4, 1 << 20, 6, torch.device("cuda:0"))
    sb.fill_random(31)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    got = shard_checksums(sb)
    host = sb.buf[:, :, :sb.S].cpu().numpy()
    for b in range(sb.batch):
        for i in range(sb.n):
            assert got[b][i] == shard_checksum(host[b, i].tobytes())


def test_codec_test_shard_checksum_vectors(native_lib):
    """codec_test.go:90-107 TestShardChecksum on the device path."""
    import torch
    from callfs_amd.device import HashPlan
    msgs = [b"hello world", b"hello world", b"hello world!"]
    buf = torch.zeros(3 * 256, dtype=torch.uint8, device="cuda:0")
    for i, m in enumerate(msgs):
        buf[256 * i:256 * i + len(m)] = torch.tensor(list(m), dtype=torch.uint8)
    got = HashPlan([buf.data_ptr() + 256 * i for i in range(3)], [len(m) for m in msgs]).hexdigests()
    assert all(len(h) == 64 for h in got)
    assert got[0] == got[1] != got[2]
    assert got[0] == hashlib.sha256(b"hello world").hexdigest()
