"""FormatV1 files through every device reading surface, against the oracle.

The reference's V1 branch: magic 0x77846676 (/root/reference/src/metadata.rs:29-33), u32 LE
content length of the index block (src/reader.rs:54-56) and of every data block (:146-148)
instead of varint64.  The product's V1 code: the host footer / index framing (csrc/host.cpp),
the device directory (csrc/reader.hip k_block_dir), the batched get and the index seek
(k_get, k_index_seek), all given Metadata::file_version.  Files: the hand-derived golden
one_key_v1.mtbl and corpus.to_v1 copies of Writer output (tests/test_v1.py pins those on the CPU),
plus corrupted u32 lengths (past the end of the file: the reference's slice panics).
"""
import os
import subprocess

import numpy as np
import pytest

import corpus
import test_reader_gpu as trg
import test_seek_gpu as tsg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _write(recs, bs, iv, comp=0):
    from mtblx.writer import Writer
    w = Writer(bs, iv, comp)
    for k, v in recs:
        w.insert(k, v)
    return w.into_inner()


def _v1_files(rng):
    out = []
    for bs, iv, n, comp in ((1024, 1, 300, 0), (4096, 16, 1500, 0), (512, 3, 400, 1), (2048, 7, 600, 2),
                            (8192, 16, 2000, 5), (65536, 16, 3000, 0)):
        recs = corpus.random_records(rng, n, 0, 60, 0, 150)
        out.append((corpus.to_v1(_write(recs, bs, iv, comp)), recs, comp))
    out.append((corpus.to_v1(_write([], 4096, 16)), [], 0))
    return out


def test_v1_golden_reader(oracle):
    rd = trg._reader()
    b = open(os.path.join(GOLD, "one_key_v1.mtbl"), "rb").read()
    r = rd.ReaderBuilder().read(b)
    assert r.version == 0 and r.meta == [35, 8192, 0, 1, 1, 35, 25, 5, 11]
    assert r.iter().records() == [(b"hello", b"I'm the one")]
    assert r.get(b"hello") == b"I'm the one" and r.get(b"hell") is None
    trg._check(oracle, open(os.path.join(GOLD, "empty_v1.mtbl"), "rb").read())


@pytest.mark.parametrize("verify", [True, False])
def test_v1_iter(oracle, verify):
    rng = np.random.default_rng(121)
    for data, recs, _ in _v1_files(rng):
        exp = trg._check(oracle, data, verify=verify)
        assert exp["records"] == recs


def test_v1_get_batch(oracle):
    rng = np.random.default_rng(122)
    for data, recs, comp in _v1_files(rng):
        if not recs:
            continue
        keys = [k for k, _ in recs]
        qs = [keys[int(i)] for i in rng.integers(0, len(keys), 60)]
        qs += [k + b"\x00" for k in qs[:20]] + [b"", b"\xff" * 40, keys[-1] + b"\x01"]
        trg._check_get(oracle, data, qs)
        trg._check_get(oracle, data, qs[:30], verify=False)


def test_v1_seek_bulk_and_scripts(oracle):
    rng = np.random.default_rng(123)
    for data, recs, comp in _v1_files(rng):
        if not recs:
            continue
        assert tsg._bulk_check(oracle, data, True, rng, recs) > 0
        for t in range(4):
            keys = tsg._probe_keys(rng, recs, 6)
            ops = [int(rng.choice([1, 3, 40])), ("seek", keys[1]), 5, ("seek", keys[0]), 2, ("seek", keys[-1]), 30]
            mode = str(rng.choice(["iter", "from", "prefix", "range"]))
            k = keys[int(rng.integers(0, len(keys)))]
            tsg._script_check(oracle, data, bool(t & 1), mode, k if mode != "prefix" else k[:2], k + b"\x80", ops)


def test_v1_pipe(oracle):
    """end-to-end pipe over the V1 reader's block directory == the oracle's decode of the same
    block bytes"""
    trg._reader()
    from mtblx import pipe, reader
    rng = np.random.default_rng(124)
    recs = corpus.random_records(rng, 4000, 4, 40, 16, 100)
    data = corpus.to_v1(_write(recs, 4096, 16))
    r = reader.ReaderBuilder().read(data)
    off, ln, st, _ = r.directory()
    assert (st.cpu().numpy() == 0).all()
    o = off.cpu().numpy().view(np.uint64).copy()
    n = ln.cpu().numpy().view(np.uint32).copy()
    host = np.frombuffer(data, np.uint8).copy()
    exp = oracle.decode_blocks(host, o, n)
    p = pipe.HostPipe(chunk_bytes=256 << 10, max_blocks=64, threads=8)
    out = pipe.HostOutputs(o.size, int(exp.nrec.sum()), exp.keys.size, exp.vals.size)
    p.decode(host, o, n, out, compression=0)
    assert np.array_equal(out.status[: o.size], exp.status) and np.array_equal(out.nrec[: o.size], exp.nrec)
    nr = int(exp.nrec.sum())
    assert np.array_equal(out.key_end[:nr], exp.key_end) and np.array_equal(out.val_end[:nr], exp.val_end)
    assert np.array_equal(out.keys[: exp.keys.size], exp.keys) and np.array_equal(out.vals[: exp.vals.size], exp.vals)
    assert nr == len(recs)


@pytest.mark.parametrize("verify", [True, False])
def test_v1_corrupt_lengths(oracle, verify):
    """u32 content lengths past the end of the file, shorter and longer than the content, the
    index block's length, and the V1 magic on a V2-framed file"""
    rng = np.random.default_rng(125)
    recs = corpus.random_records(rng, 1200, 4, 30, 10, 80)
    v2 = _write(recs, 2048, 8)
    v1 = corpus.to_v1(v2)
    frames = corpus.v1_frames(v1)
    cases = []
    for b in (0, 3, len(frames) - 2):
        off, n = frames[b]
        for new in (len(v1) + 100, 0xFFFFFFFF, n - 9, n + 3, 0, 4, 7):
            d = bytearray(v1)
            d[off: off + 4] = int(new).to_bytes(4, "little")
            cases.append(bytes(d))
    io, ni = frames[-1]
    for new in (1 << 31, ni + 1, ni - 4, 3):
        d = bytearray(v1)
        d[io: io + 4] = int(new).to_bytes(4, "little")
        cases.append(bytes(d))
    mix = bytearray(v2)                                 # V1 magic on varint framing
    mix[-4:] = corpus.MAGIC_V1.to_bytes(4, "little")
    cases.append(bytes(mix))
    ends = set()
    for d in cases:
        exp = trg._check(oracle, d, verify=verify)
        ends.add(exp["end"])
        if exp["end"] not in (1, 3):   # opened: the batched get on a few keys too
            trg._check_get(oracle, d, [recs[0][0], recs[600][0], recs[-1][0]], verify=verify)
    assert 3 in ends   # the reference panics on some of them (slice past the end)


def test_v1_cpp_examples(tmp_path, oracle):
    """examples/info.rs and examples/dump.rs on V1 files (include/mtbl.hpp over the C ABI)"""
    trg._reader()
    bin_ = os.path.join(ROOT, "oxidized-mtbl_amd", "build")
    if not os.path.exists(os.path.join(bin_, "info")):
        pytest.skip("C++ examples not built")
    r = subprocess.run([os.path.join(bin_, "info"), os.path.join(GOLD, "one_key_v1.mtbl")], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout == ("Metadata {\n    file_version: FormatV1,\n    index_block_offset: 35,\n"
                        "    data_block_size: 8192,\n    compression_algorithm: None,\n    count_entries: 1,\n"
                        "    count_data_blocks: 1,\n    bytes_data_blocks: 35,\n    bytes_index_block: 25,\n"
                        "    bytes_keys: 5,\n    bytes_values: 11,\n}\n")
    from mtblx import synth
    data = corpus.to_v1(_write(list(synth.cfg1_records()), 4096, 16))
    path = tmp_path / "cfg1_v1.mtbl"
    path.write_bytes(data)
    exp = oracle.file_scan(data, "iter")["records"]
    assert len(exp) == 10000
    r = subprocess.run([os.path.join(bin_, "dump"), str(path)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout == b"".join(b'"' + k + b'" "' + v + b'"\n' for k, v in exp)
    k, v = exp[777]
    r = subprocess.run([os.path.join(bin_, "get_key"), str(path), k.decode()], capture_output=True, timeout=60)
    assert r.returncode == 0 and r.stdout == b'"' + k + b'" "' + v + b'"\n', r
