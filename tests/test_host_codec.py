"""The host codec (slime_amd/csrc/host_codec.cpp) on CPU, against the oracle.

gf.MapToGF / MapToGFWith / MapFromGF on host memory run on the host cores
(slime_gf_codec_placement 0, the default), so they are testable here without
a GPU.  Checked bit-exact against oracle/rs_oracle.c (map.go:15-113):

- every length 0..67 (every partial last word, the AVX2 body and its
  scalar tail) and lengths around the library's piece boundaries;
- MapToGF's flag scan at both mapping edges: words p-1 / p (mapping 0 fits
  or not) and 0x7FFFFFFA / 0x7FFFFFFB (1<<31 fits or not), each placed in
  the vector body, in the scalar tail, in the partial last word and in a
  later piece of a multi-piece call;
- the random fallback (map.go:64-66): a fitting mapping and the oracle's
  MapToGFWith under it;
- RecoverData with every data shard present: unit inverse rows, done on the
  host (non-canonical symbols x >= p come back as x mod p, vector.go:97).

The same checks run again with SLIME_RS_CODEC_ISA=scalar (the portable form).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle_c as OC
from slime_amd import _native as N
from slime_amd import gf, rs

P = gf.MaxVal
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Words at the mapping edges (map.go:37, :51): p-1 fits mapping 0, p does not;
# 0x7FFFFFFA ^ 1<<31 = p-1 fits 1<<31, 0x7FFFFFFB ^ 1<<31 = p does not.
FITS_0, BREAKS_0 = P - 1, P
FITS_HI, BREAKS_HI = 0x7FFFFFFA, 0x7FFFFFFB


@pytest.fixture(autouse=True)
def host_placement():
    prev = N.lib.slime_gf_codec_placement(-1)
    N.check(N.lib.slime_gf_codec_placement(0))
    yield
    N.check(N.lib.slime_gf_codec_placement(prev))


def _with_word(data: bytearray, pos: int, w: int) -> bytearray:
    data[4 * pos:4 * pos + 4] = int(w).to_bytes(4, "big")
    return data


def _check_map(data: bytes):
    n, v = gf.MapToGF(data)
    rc, n2, v2 = OC.map_to_gf(data)
    if rc == 0:  # mapping 0 or 1<<31: fully determined
        assert n == n2 and np.array_equal(v, v2), (len(data), n, n2)
    else:  # random fallback: any fitting value, and the words are MapToGFWith under it
        assert n not in (0, 1 << 31)
        assert np.array_equal(v, OC.map_to_gf_with(data, n))
    assert int(v.max(initial=0)) < P
    assert bytes(gf.MapFromGF(n, v)) == OC.map_from_gf(n, v)
    assert bytes(gf.MapFromGF(n, v))[:len(data)] == bytes(data)
    return n


def test_every_partial_word_length():
    rng = np.random.default_rng(1)
    for length in range(0, 68):
        data = rng.integers(0, 256, size=length, dtype=np.uint8).tobytes()
        _check_map(data)
        for m in (0, 1 << 31, 0x12345678, 0xFFFFFFFF):
            assert np.array_equal(gf.MapToGFWith(data, m), OC.map_to_gf_with(data, m))
            w = OC.map_to_gf_with(data, m)
            assert bytes(gf.MapFromGF(m, w)) == OC.map_from_gf(m, w)


@pytest.mark.parametrize("nwords", [16, 17, 31, 300_000])
def test_flag_scan_at_both_mapping_edges(nwords):
    """nwords = 300000 spans two pieces of the library's split (256 Ki words
    run serially, larger calls in 128 Ki-word pieces)."""
    rng = np.random.default_rng(nwords)
    base = bytearray(rng.integers(0, 0x7FFFFFF0, size=nwords, dtype=np.uint32).astype(">u4").tobytes())
    positions = sorted({0, 5, nwords - 1, nwords // 2, min(nwords - 1, 131_072 + 3)})
    for pos in positions:
        for word, want in ((FITS_0, 0), (BREAKS_0, 1 << 31), (FITS_HI, 0)):
            assert _check_map(bytes(_with_word(bytearray(base), pos, word))) == want, (pos, hex(word))
        # 1<<31 is refuted by a word that maps to p under it: random fallback
        d = _with_word(_with_word(bytearray(base), pos, BREAKS_0), (pos + 1) % nwords, BREAKS_HI)
        assert _check_map(bytes(d)) not in (0, 1 << 31)
        d = _with_word(_with_word(bytearray(base), pos, BREAKS_0), (pos + 1) % nwords, FITS_HI)
        assert _check_map(bytes(d)) == 1 << 31
    # the partial last word (1..3 bytes, zero low bytes) can never reach p
    for extra in (1, 2, 3):
        assert _check_map(bytes(base) + b"\xff" * extra) == 0


def test_reference_kats_and_golden(kats, golden):
    for case in kats["map_trivial"]:
        data = bytes(case["in"])
        n, v = gf.MapToGF(data)
        assert n == case["n"] and v.tolist() == case["v"]
        assert gf.MapFromGF(n, v)[: len(data)] == data
    gf.Seed(99)
    for case in kats["map_tricky"]:
        _check_map(bytes(case))
    for case in golden["map"]:
        n, v = gf.MapToGF(bytes(case["bytes"]))
        assert n == case["n"] and v.tolist() == case["words"]
        assert list(gf.MapFromGF(n, v)) == case["back"]


def test_large_random_bodies_and_unaligned_buffers():
    rng = np.random.default_rng(7)
    for length in [(1 << 20) + 3, (3 << 20) + 1, 5 << 20]:
        raw = rng.integers(0, 256, size=length + 1, dtype=np.uint8)
        data = raw[1:]  # odd address: unaligned loads
        _check_map(data.tobytes())
        n, v = gf.MapToGF(data)
        w = np.zeros(v.size + 1, dtype=np.uint32)[1:]
        w[:] = v
        assert bytes(gf.MapFromGF(n, w)) == OC.map_from_gf(n, v)


def test_recover_data_all_data_present_is_host_mod_p():
    """Every data shard present: RecoverData's inverse is the identity (unit
    rows), so the outputs are the chunks mod p -- no device involved."""
    rng = np.random.default_rng(3)
    for need, L in [(1, 5), (4, 1001), (8, 300_001)]:
        chunks = [rng.integers(0, 2**32, size=L, dtype=np.uint64).astype(np.uint32) for _ in range(need)]
        for c in chunks:
            c[: 6] = np.array([P - 1, P, P + 1, 0xFFFFFFFF, 0, 1], dtype=np.uint32)[: min(L, 6)]
        have = list(range(need))[::-1]  # any order
        got = rs.RecoverData(chunks[::-1], have)
        rc, want = OC.recover_data(chunks[::-1], have)
        assert rc == 0
        for g, w in zip(got, want):
            assert np.array_equal(g, w)


def test_concurrent_callers_share_the_pool():
    """Several threads in the codec at once (a proxy serves many requests,
    main.go:107-109): their multi-piece jobs interleave on one copy pool; every
    result must equal the oracle's for its own input."""
    from concurrent.futures import ThreadPoolExecutor

    rng = np.random.default_rng(11)
    cases = []
    for t in range(12):
        nwords = (3 << 18) + 17 * t  # 3 MiB and a little: several pieces per call
        words = rng.integers(0, 0x7FFFFFF0, size=nwords, dtype=np.uint32)
        if t % 3 == 1:
            words[nwords // 3] = BREAKS_0  # 1<<31 objects in the mix
        data = words.astype(">u4").tobytes() + bytes([t + 1])
        rc, n, v = OC.map_to_gf(data)
        assert rc == 0
        cases.append((data, n, v, OC.map_from_gf(n, v)))

    def one(i):
        data, n, v, back = cases[i % len(cases)]
        for _ in range(3):
            n2, v2 = gf.MapToGF(data)
            if n2 != n or not np.array_equal(v2, v):
                return f"MapToGF case {i}"
            if not np.array_equal(gf.MapToGFWith(data, n), v):
                return f"MapToGFWith case {i}"
            if bytes(gf.MapFromGF(n, v)) != back:
                return f"MapFromGF case {i}"
        return None

    with ThreadPoolExecutor(max_workers=6) as ex:
        errors = [e for e in ex.map(one, range(24)) if e]
    assert not errors, errors


def test_codec_placement_knob():
    assert N.lib.slime_gf_codec_placement(-1) == 0
    with pytest.raises(N.NativeError):
        N.check(N.lib.slime_gf_codec_placement(2))
    assert N.lib.slime_gf_codec_placement(-1) == 0


@pytest.mark.skipif(os.environ.get("SLIME_RS_CODEC_ISA") == "scalar", reason="already the scalar run")
def test_scalar_form_in_a_subprocess():
    env = dict(os.environ, SLIME_RS_CODEC_ISA="scalar")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", __file__],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
