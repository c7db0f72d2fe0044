"""Chunk and object digests, host side, no GPU.

SHA-256 is store.DataV's sha256.Sum256 (internal/store/store.go:104-110),
checked against the FIPS 180-2 example vectors and Python's hashlib (an
independent SHA-256); the chunk-file header is storedir's FNV-1a-64 over
SHA-256 ‖ data (storedir/directory.go:548-553), checked against Go hash/fnv's
published vectors through the C oracle (oracle_fnv1a64).  The device pipeline
that feeds write_chunks_digest is covered in tests/test_gpu_digest.py.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from oracle import oracle_c as OC
from slime_amd import _native as N
from slime_amd import objects as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NIST = [  # FIPS 180-2 appendix B
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
]

FNV64A = [(b"", 0xcbf29ce484222325), (b"a", 0xaf63dc4c8601ec8c), (b"ab", 0x089c4407b545986a),
          (b"abc", 0xe71fa2190541574b)]  # Go src/hash/fnv/fnv_test.go golden64a


def test_sha256_nist_vectors():
    for msg, want in NIST:
        assert O.sha256(msg).hex() == want


def test_sha256_matches_hashlib_at_every_block_boundary():
    rng = np.random.default_rng(7)
    for n in list(range(0, 200)) + [1000, 4095, 4096, 4097, 65536 + 55, 1 << 20, 3 * (1 << 20) + 13]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.sha256(b) == hashlib.sha256(b).digest(), n


def test_portable_sha256_path_matches():
    """The loop for CPUs without the SHA extensions (SLIME_RS_SHA_NI=0 forces it)."""
    code = ("import hashlib, numpy as np\n"
            "from slime_amd import objects as O, _native as N\n"
            "assert not N.digest_info()[0]\n"
            "rng = np.random.default_rng(3)\n"
            "for n in list(range(0, 140)) + [1000, 65599]:\n"
            "    b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()\n"
            "    assert O.sha256(b) == hashlib.sha256(b).digest(), n\n"
            "assert O.sha256(b'abc').hex().startswith('ba7816bf')\n")
    env = dict(os.environ, SLIME_RS_SHA_NI="0", PYTHONPATH=ROOT)
    subprocess.run([sys.executable, "-c", code], check=True, env=env, cwd=ROOT, timeout=120)


def test_fnv_oracle_pinned_by_go_vectors():
    for msg, want in FNV64A:
        assert OC.fnv1a64(msg) == want


@pytest.mark.parametrize("sizes", [[0], [1, 2, 3], [0, 5, 64, 4096, 70001], [4096] * 50])
def test_chunk_digests_vs_oracle(sizes):
    rng = np.random.default_rng(len(sizes))
    chunks = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    shas, hdrs = O.chunk_digests(chunks, headers=True)
    for c, s, h in zip(chunks, shas, hdrs):
        assert (s, h) == OC.chunk_digests(c)
    shas2, none = O.chunk_digests(chunks)
    assert shas2 == shas and none is None


def test_chunk_digests_from_concurrent_callers():
    rng = np.random.default_rng(11)
    sets = [[rng.integers(0, 256, 100000 + 17 * i + j, dtype=np.uint8) for j in range(12)] for i in range(6)]
    want = [[hashlib.sha256(c.tobytes()).digest() for c in s] for s in sets]
    got = [None] * len(sets)

    def work(i):
        for _ in range(5):
            got[i] = O.chunk_digests(sets[i])[0]
            assert got[i] == want[i]

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(sets))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == want


def test_digest_argument_checks():
    with pytest.raises(N.NativeError):
        N.check(N.lib.slime_rs_sha256(None, 5, None))
    lens = (N.ctypes.c_uint64 * 1)(3)
    ptrs = (N.ctypes.c_void_p * 1)(None)
    out = np.zeros(32, dtype=np.uint8)
    with pytest.raises(N.NativeError):
        N.check(N.lib.slime_rs_chunk_digests(ptrs, lens, 1, out.ctypes.data, None))
    assert N.lib.slime_rs_chunk_digests(None, None, 0, None, None) == 0


def test_bad_hash_status_maps_to_reference_error():
    assert N.lib.slime_rs_status_string(N.ERR_BAD_HASH).decode() == "bad checksum after reconstruction"
    assert issubclass(N.BadHash, N.NativeError)


def test_write_chunks_refuses_overlap_other_than_whole_data_chunks():
    """Zero-copy data chunks (chunk j = data + j*chunk_size, wholly inside the
    object) are admitted; any other overlap with the object is refused before
    any device work (so this runs without a GPU)."""
    import ctypes
    size, need, total = 1000, 4, 6
    cb = O.chunk_size(size, need)
    data = np.zeros(size, dtype=np.uint8)
    own = [np.zeros(cb, dtype=np.uint8) for _ in range(total)]
    m = ctypes.c_uint32()

    def call(ptrs):
        arr = (ctypes.c_void_p * total)(*ptrs)
        return N.lib.slime_rs_write_chunks(data.ctypes.data, size, need, total, arr, ctypes.byref(m))

    base = data.ctypes.data
    good = [o.ctypes.data for o in own]
    assert (size + 3) // 4 > 3 * (cb // 4)  # the last data chunk is partly padding
    for bad in ([base + 1] + good[1:],                                 # misaligned alias
                good[:3] + [base + 3 * cb] + good[4:],                 # chunk 3 runs past the object
                good[:4] + [base] + good[5:],                          # a parity chunk inside the object
                [base + cb] + good[1:]):                               # chunk 0 at chunk 1's bytes
        assert call(bad) == N.ERR_INVALID_ARG
    assert "overlaps the object" in N.lib.slime_rs_last_error().decode()
    rc = call([base, base + cb, base + 2 * cb] + good[3:])
    assert rc in (N.OK, N.ERR_NO_DEVICE)
