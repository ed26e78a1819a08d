"""The bit-sliced kernels (csrc/bitslice_gen.hpp): an XOR network over bit
planes generated for each launch group's coefficient block and compiled by hiprtc. Every
case is bit-exact against the C oracle (oracle/rs_oracle.c via oracle.cref): encodes of
wide profiles, 9..16-erasure decodes, Verify rows that pass on clean stripes and flag a
flipped byte, ragged shard sizes (partial waves, a lane's second vector past the shard, the
S % 16 byte tail), misaligned layouts, two launch groups, and every tile order pinned."""
import os

import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

BS_ORDERS = ["bs", "bs-g8", "bs-g2", "bs-q8", "bs-q16", "bs-x8", "bs-x32"]


@pytest.fixture(autouse=True)
def _no_tuned_forms(native_lib):
    """The forms asserted below are the rule's: forget what other tests' tuners recorded."""
    native_lib.lib.rs_tune_table_reset(None)
    yield
    native_lib.lib.rs_tune_table_reset(None)


def _consistent(k, m, S, batch, seed, layout="planar"):
    """A resident batch whose parity the oracle computed (so every stripe is consistent),
    and its host copy [batch][n][S]."""
    import torch
    from callfs_amd.device import StripeBatch
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"), layout=layout)
    sb.fill_random(seed)
    host = sb.gather().cpu().numpy()
    for b in range(batch):
        want = cref.encode([host[b, i] for i in range(k)], k, m)
        for j in range(m):
            host[b, k + j] = want[j]
            sb.shard(b, k + j).copy_(torch.from_numpy(want[j]))
    return sb, host


def _pin(plan, name):
    from callfs_amd import _native as N
    plan.set_orders([name] * int(N.lib.rs_plan_groups(plan.handle)))


@pytest.mark.parametrize("k", [20, 32])
@pytest.mark.parametrize("m", [9, 12, 16])
def test_wide_encode_and_decode_vs_oracle(native_lib, k, m):
    """Verdict r05 item 1: k in {20, 32}, m in {9, 12, 16}; encode and an m-erasure decode
    (data and parity shards lost) through the rule (which takes the bit-sliced kernel for
    every wide group) and each pinned order; S = 3 full tiles + a partial wave + 9 tail bytes."""
    from callfs_amd.device import Plan
    S = 3 * 8192 + 1024 + 16 * 37 + 9
    batch = 3
    n = k + m
    sb, host = _consistent(k, m, S, batch, seed=k * 131 + m)
    enc = Plan.for_batch(sb)
    assert enc.forms() == ["bs-g8"], enc.forms()
    data_lost = list(range(0, k, max(1, k // (m // 2))))[: m // 2]
    erase = data_lost + list(range(k, k + m - len(data_lost)))
    assert len(erase) == m
    dec = Plan.for_batch(sb, present=[i not in erase for i in range(n)])
    for name in ["rule"] + BS_ORDERS:
        for p, lost in ((enc, range(k, n)), (dec, erase)):
            if name != "rule":
                _pin(p, name)
            for i in lost:
                sb.zero_shard(i)
            p.launch()
            assert not p.corrupt(), (name, lost)
            assert np.array_equal(sb.gather().cpu().numpy(), host), (name, list(lost))


@pytest.mark.parametrize("k,m", [(1, 16), (2, 12), (3, 9), (4, 13), (6, 9)])
def test_few_inputs_many_rows_vs_oracle(native_lib, k, m):
    """Groups of 9..16 rows over 1..6 inputs (any m >= 1 per request,
    post_file_enhanced.go:36-44): the rule's bit-sliced kernel for the encode and for a decode
    that loses every data shard it can, and two pinned orders; k <= 3 is where the nibble path
    would be the v_perm kernel (rs_apply_vec)."""
    from callfs_amd.device import Plan
    S = 2 * 8192 + 16 * 5 + 3
    batch = 3
    n = k + m
    sb, host = _consistent(k, m, S, batch, seed=k * 17 + m)
    enc = Plan.for_batch(sb)
    assert enc.forms() == ["bs-g8"], enc.forms()
    erase = list(range(k)) + list(range(k, k + m - k))  # all data, then parity up to m lost
    assert len(erase) == m
    dec = Plan.for_batch(sb, present=[i not in erase for i in range(n)])
    assert all(f.startswith("bs") for f in dec.forms()), dec.forms()
    for name in ("rule", "bs-x32", "bs"):
        for p, lost in ((enc, range(k, n)), (dec, erase)):
            if name != "rule":
                _pin(p, name)
            for i in lost:
                sb.zero_shard(i)
            p.launch()
            assert not p.corrupt(), (name, lost)
            assert np.array_equal(sb.gather().cpu().numpy(), host), (name, list(lost))


@pytest.mark.parametrize("k,m,erase", [(20, 16, 12), (32, 12, 9), (10, 16, 14)])
def test_wide_decode_verify_rows_flag_corruption(native_lib, k, m, erase):
    """Fewer erasures than m: the present parity beyond the first k are Verify rows compared
    inside the kernel (codec.go:59); a flipped byte in one flags exactly its stripe."""
    from callfs_amd.device import Plan
    S = 65_536 + 45
    batch = 4
    n = k + m
    sb, host = _consistent(k, m, S, batch, seed=erase * 7 + k)
    lost = list(range(1, 1 + erase))
    dec = Plan.for_batch(sb, present=[i not in lost for i in range(n)])
    assert dec.forms()[0].startswith("bs"), dec.forms()
    for name in ("rule", "bs-x32", "bs"):
        if name != "rule":
            _pin(dec, name)
        for i in lost:
            sb.zero_shard(i)
        dec.launch()
        assert not dec.corrupt(), name
        assert np.array_equal(sb.gather().cpu().numpy(), host), name
        vrow = n - 1
        sb.shard(2, vrow)[S - 3] ^= 0x21  # the ragged tail's byte kernel compares too
        dec.launch()
        assert dec.corrupt_stripes() == [2], name
        sb.shard(2, vrow)[S - 3] ^= 0x21
        sb.shard(1, vrow)[100] ^= 0x80
        dec.launch()
        assert dec.corrupt_stripes() == [1], name
        sb.shard(1, vrow)[100] ^= 0x80


@pytest.mark.parametrize("k,m,S,batch", [
    (10, 8, 553_574, 3),      # verdict r05 item 2: the worst readall one-shard decode cells
    (10, 8, 122_190, 4),
    (8, 8, 312_855, 3),
    (16, 8, 100_003, 3),
])
def test_readall_one_shard_decode_into_fresh_buffers(native_lib, k, m, S, batch):
    """R 5..8 decodes of CallFS's io.ReadAll layout (survivors at odd offsets, the lost
    shard rebuilt into a buffer of its own, m - 1 compared rows): the rule's bit-sliced X32
    form and the pinned orders rebuild every byte, and a flipped compared byte is flagged."""
    import torch
    from callfs_amd.device import Plan, StripeBatch, _aligned_empty
    n = k + m
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"), layout="readall")
    sb.fill_random(S + k)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    host = sb.gather().cpu().numpy()
    for b in range(batch):
        want = cref.encode([host[b, i] for i in range(k)], k, m)
        assert all(np.array_equal(host[b, k + j], want[j]) for j in range(m)), b
    fp = -(-S // 64) * 64
    for erase in ([1], [0, k]):
        fresh = _aligned_empty((batch, len(erase), fp), 256, torch.device("cuda:0"))
        ptrs = list(sb.pointers())
        for b in range(batch):
            for j, i in enumerate(erase):
                ptrs[b * n + i] = fresh[b, j].data_ptr()
        dec = Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)])
        assert dec.forms() == ["bs-x32"], dec.forms()
        for name in ("rule", "bs-g8", "bs"):
            if name != "rule":
                _pin(dec, name)
            fresh.fill_(0xA5)
            dec.launch()
            assert not dec.corrupt(), (erase, name)
            got = fresh.cpu().numpy()
            for b in range(batch):
                for j, i in enumerate(erase):
                    assert np.array_equal(got[b, j, :S], host[b, i]), (erase, name, b, i)
        sb.shard(batch - 1, n - 1)[S // 3] ^= 1
        dec.launch()
        assert dec.corrupt_stripes() == [batch - 1], erase
        sb.shard(batch - 1, n - 1)[S // 3] ^= 1
        del dec, fresh


@pytest.mark.parametrize("k,m,S,off", [(20, 10, 300_001, 1), (12, 9, 65_536 + 3, 5),
                                       (32, 8, 1 << 16, 8)])
def test_split_layout_misaligned_inputs_and_outputs(native_lib, k, m, S, off):
    """Upstream Split of a contiguous object (every shard at its own byte offset): the
    bit-sliced kernel's unaligned 16-B loads and stores, pinned in every order."""
    import torch
    from callfs_amd.device import Plan
    n = k + m
    batch = 2
    total = batch * n * S
    buf = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device="cuda:0")
    base = buf.data_ptr() + off
    ptrs = [base + (b * n + i) * S for b in range(batch) for i in range(n)]
    host = buf.cpu().numpy()[off:off + total].copy()
    for b in range(batch):
        st = host[b * n * S:(b + 1) * n * S]
        want = cref.encode([st[i * S:(i + 1) * S] for i in range(k)], k, m)
        for j in range(m):
            st[(k + j) * S:(k + j + 1) * S] = want[j]
    good = torch.from_numpy(host).to("cuda:0")
    plan = Plan(k, m, S, batch, ptrs)
    for name in ["rule"] + BS_ORDERS:
        if name != "rule":
            _pin(plan, name)
        buf[off:off + total].copy_(good)
        for b in range(batch):
            for i in range(k, n):
                s0 = off + (b * n + i) * S
                buf[s0:s0 + S].zero_()
        plan.launch()
        assert torch.equal(buf[off:off + total], good), name


@pytest.mark.parametrize("k,m", [(10, 20), (6, 17)])
def test_two_launch_groups(native_lib, k, m):
    """More than 16 rows: launch groups of 16 + the rest, each with its own kernel."""
    from callfs_amd.device import Plan
    S = 40_000 + 13
    sb, host = _consistent(k, m, S, 2, seed=k + m)
    enc = Plan.for_batch(sb)
    forms = enc.forms()
    assert len(forms) == 2 and forms[0].startswith("bs"), forms
    for name in ("rule", "bs", "bs-x32"):
        if name != "rule":
            _pin(enc, name)
        for i in range(k, k + m):
            sb.zero_shard(i)
        enc.launch()
        assert np.array_equal(sb.gather().cpu().numpy(), host), name


@pytest.mark.parametrize("k,m,S", [(9, 9, 16), (9, 9, 17), (16, 10, 40), (20, 16, 1023),
                                   (5, 12, 2049), (24, 4, 8192 * 5 + 16)])
def test_tiny_and_ragged_shards(native_lib, k, m, S):
    """One vector per shard, one lane's second vector missing, tails of 1..15 bytes, and
    R <= 4 pinned to the bit-sliced form (the tuner's candidate there)."""
    from callfs_amd.device import Plan
    sb, host = _consistent(k, m, S, 3, seed=S + k)
    enc = Plan.for_batch(sb)
    for name in ("rule", "bs", "bs-g2"):
        if name != "rule":
            _pin(enc, name)
        for i in range(k, k + m):
            sb.zero_shard(i)
        enc.launch()
        assert np.array_equal(sb.gather().cpu().numpy(), host), (name, S)


def test_read_only_verify_pinned(native_lib):
    """Nothing lost (a download's Verify): every row compared; the rule runs read-only
    launches on the bit-sliced kernel (G8), the nibble kernel pinned compares the same bytes,
    and a flipped byte is flagged in either."""
    from callfs_amd.device import Plan
    k, m, S = 20, 8, 65_536 + 17
    sb, host = _consistent(k, m, S, 3, seed=99)
    ver = Plan.for_batch(sb, present=[True] * (k + m))
    assert ver.forms() == ["bs-g8"], ver.forms()
    for name in ("rule", "bs", "x32", "consecutive"):
        if name != "rule":
            _pin(ver, name)
        ver.launch()
        assert not ver.corrupt(), name
        sb.shard(0, k + 5)[S - 1] ^= 0xFF
        ver.launch()
        assert ver.corrupt_stripes() == [0], name
        sb.shard(0, k + 5)[S - 1] ^= 0xFF
    assert np.array_equal(sb.gather().cpu().numpy(), host)


def test_tune_offers_bitslice_and_stays_exact(native_lib):
    """rs_plan_tune times the bit-sliced orders beside the nibble kernels; whatever it keeps
    reproduces the oracle's bytes."""
    from callfs_amd.device import Plan
    k, m, S = 32, 8, 262_144
    sb, host = _consistent(k, m, S, 8, seed=5)
    enc = Plan.for_batch(sb)
    chosen = enc.tune(reps=2)
    assert enc.forms() == chosen
    for i in range(k, k + m):
        sb.zero_shard(i)
    enc.launch()
    assert np.array_equal(sb.gather().cpu().numpy(), host), chosen


def test_host_codec_wide_profile_roundtrip(native_lib):
    """The host-memory entry points (rs_codec_encode / rs_codec_decode) on a wide profile:
    the rule's bit-sliced launch runs once compiled (compiled in the background), and the
    bytes match the oracle either way."""
    from callfs_amd import Codec, ErasureProfile
    c = Codec()
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 3 * (1 << 20) + 11, dtype=np.uint8).tobytes()
    k, m = 20, 12
    shards = c.encode(data, ErasureProfile(k, m))
    S = len(shards[0])
    want = cref.encode([np.frombuffer(bytes(shards[i]), dtype=np.uint8) for i in range(k)], k, m)
    for j in range(m):
        assert np.array_equal(np.frombuffer(bytes(shards[k + j]), dtype=np.uint8), want[j]), j
    lost = list(shards)
    for i in range(0, 24, 2):
        lost[i] = None
    assert c.decode(lost, ErasureProfile(k, m), len(data)) == data
    assert S == -(-len(data) // k)


def test_tune_table_serves_untuned_plans_and_persists(native_lib, tmp_path):
    """Verdict r05 item 5: rs_plan_tune's choices land in a per-device table keyed by shape;
    an untuned plan of the same shape (another size in the same tiles-per-stripe bucket) runs
    the recorded form, bit-exact; CALLFS_RS_TUNE_TABLE's file keeps it for later processes;
    a reset returns launches to the rule."""
    from callfs_amd.device import Plan
    L = native_lib.lib
    path = str(tmp_path / "tune.txt")
    assert L.rs_tune_table_reset(path.encode()) == 0
    k, m, S = 32, 8, 262_144
    sb, host = _consistent(k, m, S, 8, seed=11)
    rule = Plan.for_batch(sb).forms()
    # another shard size in the same key: 32..63 tiles of 8 KiB, shard pitch a multiple of
    # 128 KiB (the planar layout's pitch is S here)
    S2 = 3 * 131_072
    sb2, host2 = _consistent(k, m, S2, 4, seed=12)
    rule2 = Plan.for_batch(sb2).forms()
    tuned = Plan.for_batch(sb)
    chosen = tuned.tune(reps=2)
    assert L.rs_tune_table_entries() >= 1
    other = Plan.for_batch(sb2)
    assert other.forms() == chosen, (rule, chosen)
    for i in range(k, k + m):
        sb2.zero_shard(i)
    other.launch()
    assert np.array_equal(sb2.gather().cpu().numpy(), host2), chosen
    lines = open(path).read().split("\n")
    assert any(ln.split()[1:3] == [str(k), str(m)] for ln in lines if ln.strip()), lines
    # a fresh binding reads the file back; a reset to memory only forgets it
    assert L.rs_tune_table_reset(path.encode()) == 0
    assert L.rs_tune_table_entries() >= 1
    assert Plan.for_batch(sb2).forms() == chosen
    assert L.rs_tune_table_reset(None) == 0
    assert L.rs_tune_table_entries() == 0
    assert Plan.for_batch(sb2).forms() == rule2


def test_bitslice_off_runs_the_nibble_kernels(native_lib, tmp_path):
    """CALLFS_RS_BITSLICE=0 (or a box where hiprtc cannot compile): every launch group runs
    the ahead-of-time nibble-table kernels, bit-exact, and no bit-sliced order is offered."""
    import subprocess
    import sys
    prog = tmp_path / "off.py"
    prog.write_text(
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})\n"
        "import torch\n"
        "from oracle import cref\n"
        "from callfs_amd import _native as N\n"
        "from callfs_amd.device import Plan, StripeBatch\n"
        "k, m, S = 20, 16, 40_000 + 9\n"
        "sb = StripeBatch(k, m, S, 2, torch.device('cuda:0'), layout='planar')\n"
        "sb.fill_random(3)\n"
        "p = Plan.for_batch(sb)\n"
        "assert not p.forms()[0].startswith('bs'), p.forms()\n"
        "try:\n"
        "    p.set_orders(['bs'])\n"
        "    raise SystemExit('bs offered')\n"
        "except N.NativeError as e:\n"
        "    assert e.code == N.RS_E_ARG\n"
        "p.launch(); torch.cuda.synchronize()\n"
        "h = sb.gather().cpu().numpy()\n"
        "for b in range(2):\n"
        "    want = cref.encode([h[b, i] for i in range(k)], k, m)\n"
        "    assert all(np.array_equal(h[b, k + j], want[j]) for j in range(m))\n"
        "print('off ok')\n")
    env = dict(os.environ, CALLFS_RS_BITSLICE="0")
    r = subprocess.run([sys.executable, str(prog)], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0 and "off ok" in r.stdout, r.stdout + r.stderr[-2000:]


def test_host_memory_paths_with_bitslice_sync(native_lib, tmp_path):
    """The host-memory entry points on wide profiles with CALLFS_RS_BITSLICE=sync (the first
    call compiles and waits, so every launch group the rule gives the bit-sliced kernel runs
    it): rs_codec_encode / rs_codec_decode through the staged pipeline (pageable buffers,
    several chunks), rs_encode / rs_reconstruct on rs_host_alloc buffers (zero-copy: the
    kernel reads host memory over PCIe), and rs_encode_batch / rs_reconstruct_batch; every
    byte against the C oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = tmp_path / "sync.py"
    prog.write_text(
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {root!r})\n"
        "import torch\n"
        "from oracle import cref\n"
        "from callfs_amd import Codec, ErasureProfile, erasure as E, _native as N\n"
        "rng = np.random.default_rng(21)\n"
        "c = Codec()\n"
        "for k, m, L in ((20, 12, 40 * (1 << 20) + 13), (32, 16, 3 * (1 << 20) + 5), (24, 9, 777_777)):\n"
        "    data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()\n"
        "    sh = c.encode(data, ErasureProfile(k, m))\n"
        "    want = cref.encode([np.frombuffer(bytes(sh[i]), dtype=np.uint8) for i in range(k)], k, m)\n"
        "    assert all(np.array_equal(np.frombuffer(bytes(sh[k + j]), dtype=np.uint8), want[j]) for j in range(m)), (k, m)\n"
        "    lost = list(sh)\n"
        "    for i in list(range(0, k, 3))[: m // 2] + list(range(k, k + m - m // 2)):\n"
        "        lost[i] = None\n"
        "    assert c.decode(lost, ErasureProfile(k, m), L) == data, (k, m)\n"
        "# zero-copy: every buffer from rs_host_alloc\n"
        "ctx = N.default_context()\n"
        "k, m, S = 20, 16, 2 * (1 << 20) + 48\n"
        "bufs = [N.PinnedBuffer(S, ctx) for _ in range(k + m)]\n"
        "for i in range(k):\n"
        "    bufs[i].array[:] = rng.integers(0, 256, S, dtype=np.uint8)\n"
        "E.encode_shards([b.array for b in bufs], k, m, ctx)\n"
        "want = cref.encode([bufs[i].array.copy() for i in range(k)], k, m)\n"
        "assert all(np.array_equal(bufs[k + j].array, want[j]) for j in range(m))\n"
        "keep = [b.array.copy() for b in bufs]\n"
        "gone = [0, 1, 2, 3, 4, 5, 6, 7, 20, 21, 22, 23, 24, 25, 26, 27]\n"
        "arrs = [b.array for b in bufs]\n"
        "for i in gone:\n"
        "    arrs[i][:] = 0\n"
        "lens_shards = [None if i in gone else arrs[i] for i in range(k + m)]\n"
        "E.reconstruct(lens_shards, k, m, ctx)\n"
        "assert all(np.array_equal(np.frombuffer(bytes(lens_shards[i]), dtype=np.uint8), keep[i]) for i in gone)\n"
        "# batch\n"
        "st = [[rng.integers(0, 256, 65_536 + 7 * b, dtype=np.uint8).tobytes() for _ in range(20)] for b in range(5)]\n"
        "par, status = E.encode_batch(st, 20, 12)\n"
        "assert status == [0] * 5\n"
        "for b in range(5):\n"
        "    w = cref.encode([np.frombuffer(s, dtype=np.uint8) for s in st[b]], 20, 12)\n"
        "    assert all(np.array_equal(np.frombuffer(bytes(par[b][j]), dtype=np.uint8), w[j]) for j in range(12)), b\n"
        "full = [list(st[b]) + [bytes(p) for p in par[b]] for b in range(5)]\n"
        "dmg = [[None if i in (0, 5, 9, 20, 21, 22, 23, 24, 25, 26) else s for i, s in enumerate(f)] for f in full]\n"
        "assert E.reconstruct_batch(dmg, 20, 12) == [0] * 5\n"
        "assert all(bytes(dmg[b][i]) == full[b][i] for b in range(5) for i in range(32))\n"
        "# the download path of every profile: Decode with nothing lost is a read-only Verify\n"
        "# launch (the bit-sliced kernel at every R); a flipped parity byte must be reported\n"
        "from callfs_amd import ErrShardCorrupted\n"
        "for k, m, L in ((1, 1, 5000), (2, 1, 70_001), (4, 2, 1 << 20), (10, 4, 3 * (1 << 20) + 1), (16, 4, 999_999), (10, 8, 2 * (1 << 20))):\n"
        "    data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()\n"
        "    sh = [bytearray(s) for s in c.encode(data, ErasureProfile(k, m))]\n"
        "    assert c.decode(list(sh), ErasureProfile(k, m), L) == data, (k, m)\n"
        "    sh[k + m - 1][len(sh[0]) // 2] ^= 0x40\n"
        "    try:\n"
        "        c.decode(list(sh), ErasureProfile(k, m), L)\n"
        "        raise SystemExit(f'corruption not flagged {k},{m}')\n"
        "    except ErrShardCorrupted:\n"
        "        pass\n"
        "print('sync ok')\n")
    env = dict(os.environ, CALLFS_RS_BITSLICE="sync", CALLFS_RS_JIT_CACHE="0")
    r = subprocess.run([sys.executable, str(prog)], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0 and "sync ok" in r.stdout, r.stdout + r.stderr[-3000:]


@pytest.mark.parametrize("k,m", [(33, 9), (64, 16), (120, 12)])
def test_more_than_32_inputs(native_lib, k, m):
    """K > 32 (round 6's first generator named shard 32's buffer after its load helper, and
    those kernels did not compile): encode and an m-erasure decode, rule and pinned, against
    the oracle."""
    from callfs_amd.device import Plan
    S = 8192 * 2 + 16 * 9 + 3
    n = k + m
    sb, host = _consistent(k, m, S, 2, seed=k)
    enc = Plan.for_batch(sb)
    assert enc.forms()[0].startswith("bs"), enc.forms()
    erase = list(range(1, k, k // (m // 2)))[: m // 2]
    erase += list(range(k, k + m - len(erase)))
    dec = Plan.for_batch(sb, present=[i not in erase for i in range(n)])
    for name in ("rule", "bs-x32"):
        for p, lost in ((enc, range(k, n)), (dec, erase)):
            if name != "rule":
                _pin(p, name)
            for i in lost:
                sb.zero_shard(i)
            p.launch()
            assert not p.corrupt(), (name, k)
            assert np.array_equal(sb.gather().cpu().numpy(), host), (name, k, list(lost))


@pytest.mark.parametrize("k,m,S,layout", [(10, 4, (1 << 20) + 1, "readall"), (4, 2, 65_536 + 7, "readall"),
                                          (10, 4, 1 << 20, "planar"), (6, 6, 300_003, "planar")])
def test_read_only_verify_rule_and_flags(native_lib, k, m, S, layout):
    """Read-only launches of every row count take the bit-sliced kernel (X32 on misaligned
    io.ReadAll bodies, G8 else): clean stripes pass, a flipped byte in a data shard or a
    parity shard (vector part or byte tail) flags exactly its stripe."""
    import torch
    from callfs_amd.device import Plan, StripeBatch
    n = k + m
    sb = StripeBatch(k, m, S, 3, torch.device("cuda:0"), layout=layout)
    sb.fill_random(S % 1000 + k)
    Plan.for_batch(sb).launch()
    ver = Plan.for_batch(sb, present=[True] * n)
    assert ver.forms() == ["bs-x32" if (layout == "readall" and S % 16) else "bs-g8"], ver.forms()
    ver.launch()
    assert not ver.corrupt()
    for b, i, pos in ((0, 0, 5), (2, n - 1, S - 1), (1, k, S // 2)):
        sb.shard(b, i)[pos] ^= 0x10
        ver.launch()
        assert ver.corrupt_stripes() == [b], (b, i, pos)
        sb.shard(b, i)[pos] ^= 0x10
    ver.launch()
    assert not ver.corrupt()


def test_process_exits_cleanly_during_background_compiles(native_lib, tmp_path):
    """A short-lived process (one host-memory call, then exit) leaves bit-sliced compiles
    queued or running on the worker: it must exit 0 with no crash in comgr's teardown
    (bitslice.cpp Worker: drained by an atexit handler registered after comgr initialised)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = tmp_path / "short.py"
    prog.write_text(
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {root!r})\n"
        "import torch\n"
        "from callfs_amd import Codec, ErasureProfile\n"
        "rng = np.random.default_rng(5)\n"
        "c = Codec()\n"
        "for k, m in ((20, 16), (10, 4), (32, 9)):\n"
        "    data = rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()\n"
        "    sh = c.encode(data, ErasureProfile(k, m))\n"
        "    assert c.decode(list(sh), ErasureProfile(k, m), len(data)) == data\n"
        "print('short ok', flush=True)\n")
    env = dict(os.environ, CALLFS_RS_JIT_CACHE="0")
    for _ in range(2):
        r = subprocess.run([sys.executable, str(prog)], capture_output=True, text=True, env=env,
                           timeout=300)
        assert r.returncode == 0 and "short ok" in r.stdout, (r.returncode, r.stderr[-3000:])


def test_large_block_compiles_in_background(native_lib):
    """A plan waits for at most 2,048 coefficients' worth of compiles; a larger block
    (RS(180,16): 2,880) compiles in the background: the plan runs whichever kernel is ready
    and every launch is bit-exact; pinning the bit-sliced order waits for the compile."""
    from callfs_amd.device import Plan
    k, m, S, batch = 180, 16, 16_384 + 48, 2
    sb, host = _consistent(k, m, S, batch, seed=180)
    enc = Plan.for_batch(sb)
    assert enc.forms()[0] in ("bs-g8", "consecutive", "g8", "g2", "x32", "q8"), enc.forms()
    for name in ("rule", "bs-g8"):
        if name != "rule":
            _pin(enc, name)
        for i in range(k, k + m):
            sb.zero_shard(i)
        enc.launch()
        assert np.array_equal(sb.gather().cpu().numpy(), host), name
    assert enc.forms() == ["bs-g8"], enc.forms()


def test_compile_failure_falls_back_to_nibble_tables(native_lib, tmp_path):
    """A box where hiprtc cannot build the bit-sliced kernels (here: gfx942 forced through
    CALLFS_OFFLOAD_ARCH, a target without v_bitop3, so every compile fails) keeps every path
    on the nibble-table kernels: the
    plan's rule, rs_plan_tune (which drops the bit-sliced candidates instead of failing, so
    bench.py still runs) and the host-memory calls, all bit-exact."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = tmp_path / "nocompile.py"
    prog.write_text(
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {root!r})\n"
        "import torch\n"
        "from oracle import cref\n"
        "from callfs_amd import Codec, ErasureProfile\n"
        "from callfs_amd.device import Plan, StripeBatch\n"
        "k, m, S = 20, 16, 65_536 + 5\n"
        "sb = StripeBatch(k, m, S, 2, torch.device('cuda:0'))\n"
        "sb.fill_random(9)\n"
        "p = Plan.for_batch(sb)\n"
        "assert not p.forms()[0].startswith('bs'), p.forms()\n"
        "orders = p.tune()\n"
        "assert not any(o.startswith('bs') for o in orders), orders\n"
        "p.launch(); torch.cuda.synchronize()\n"
        "h = sb.buf[1, :, :S].cpu().numpy()\n"
        "want = cref.encode([h[i] for i in range(k)], k, m)\n"
        "assert all(np.array_equal(h[k + j], want[j]) for j in range(m))\n"
        "rng = np.random.default_rng(3)\n"
        "data = rng.integers(0, 256, 2 << 20, dtype=np.uint8).tobytes()\n"
        "c = Codec()\n"
        "sh = c.encode(data, ErasureProfile(k, m))\n"
        "lost = list(sh); lost[0] = lost[3] = lost[k] = None\n"
        "assert c.decode(lost, ErasureProfile(k, m), len(data)) == data\n"
        "print('nocompile ok', flush=True)\n")
    env = dict(os.environ, CALLFS_RS_JIT_CACHE="0", CALLFS_OFFLOAD_ARCH="gfx942")
    r = subprocess.run([sys.executable, str(prog)], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0 and "nocompile ok" in r.stdout, r.stdout + r.stderr[-3000:]


def test_concurrent_decodes_with_background_compiles(native_lib):
    """A repair server's traffic: eight request threads decoding wide objects with a different
    erasure set each call (a new coefficient block, so a background compile, then a module
    load once it is ready) while the others launch; every object comes back bit-exact."""
    import threading
    from callfs_amd import Codec, ErasureProfile
    k, m = 20, 12
    prof = ErasureProfile(k, m)
    rng = np.random.default_rng(77)
    objs = [rng.integers(0, 256, (1 << 20) + 37 * i, dtype=np.uint8).tobytes() for i in range(4)]
    c = Codec()
    shards = [c.encode(o, prof) for o in objs]
    errors = []

    # ten erasure sets shared by the threads: the first calls of each run the nibble tables
    # while its kernel compiles, later ones the bit-sliced kernel (loaded by whichever thread
    # launches first); 5 s of traffic covers both
    pr = np.random.default_rng(99)
    pool = [pr.choice(k + m, size=int(pr.integers(1, m + 1)), replace=False) for _ in range(10)]
    import time
    t_end = time.time() + 5.0
    calls = [0] * 8

    def worker(t):
        r = np.random.default_rng(1000 + t)
        try:
            it = 0
            while time.time() < t_end:
                i = (t + it) % len(objs)
                lost = pool[int(r.integers(0, len(pool)))]
                sh = [None if j in lost else s for j, s in enumerate(shards[i])]
                if c.decode(sh, prof, len(objs[i])) != objs[i]:
                    errors.append((t, it, sorted(lost.tolist())))
                it += 1
            calls[t] = it
        except Exception as e:  # pragma: no cover - reported below
            errors.append((t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    assert min(calls) > 10, calls


@pytest.mark.parametrize("k,m", [(255, 1), (128, 128)])
def test_largest_profiles_pinned(native_lib, k, m):
    """k + m = 256, the largest GF(2^8) profiles: one row over 255 inputs (encode and a
    one-shard decode), and a decode that loses 128 of RS(128,128)'s shards, data and parity (8
    launch groups of 16 rows over 128 inputs); every group pinned to its bit-sliced kernel,
    against the oracle. (Sixteen 2,048-coefficient compiles would take a minute: the
    RS(128,128) encode is left to the rule's paths.)"""
    from callfs_amd.device import Plan
    S, batch = 4096 + 16 * 3 + 5, 2
    n = k + m
    sb, host = _consistent(k, m, S, batch, seed=k)
    lost = list(range(0, n, 2))[:m]
    todo = [(None, lost)] if k == 128 else [("enc", range(k, n)), (None, lost)]
    for what, gone in todo:  # plans made here: creating one compiles its rule's kernels
        p = (Plan.for_batch(sb) if what == "enc"
             else Plan.for_batch(sb, present=[i not in lost for i in range(n)]))
        _pin(p, "bs-g2")
        for i in gone:
            sb.zero_shard(i)
        p.launch()
        assert not p.corrupt(), list(gone)[:4]
        assert np.array_equal(sb.gather().cpu().numpy(), host), list(gone)[:4]
