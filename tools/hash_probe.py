#!/usr/bin/env python3
"""§8(f3) probe: can chunk hashes (SHA-256 per chunk/object, FNV-1a-64 per
chunk file) ride on the GPU?  Both are sequential chains inside a message, so
the GPU gets one lane per message.  Times tools/hash_probe.hip over 1 GiB
split into M messages for several M, checks digests against hashlib / a
Python FNV-1a-64, and times hashlib SHA-256 on the host cores for comparison.

    make hashprobe && python tools/hash_probe.py
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libhashprobe.so"))
for fn in (lib.hp_sha256, lib.hp_fnv1a64):
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_float


def fnv1a64(b: bytes) -> int:
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def main():
    total = 1 << 30
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
    dig = torch.empty(8 * 65536, dtype=torch.int32, device="cuda")
    fout = torch.empty(65536, dtype=torch.int64, device="cuda")
    # correctness on 4 messages of 4 KiB
    n, M = 4096, 4
    assert lib.hp_sha256(buf.data_ptr(), n, M, dig.data_ptr(), 1) > 0
    assert lib.hp_fnv1a64(buf.data_ptr(), n, M, fout.data_ptr(), 1) > 0
    torch.cuda.synchronize()
    host = buf[: n * M].cpu().numpy().tobytes()
    d = dig[: 8 * M].cpu().numpy().astype(np.uint32).reshape(M, 8)
    f = fout[:M].cpu().numpy().view(np.uint64)
    for m in range(M):
        msg = host[m * n:(m + 1) * n]
        assert b"".join(int(x).to_bytes(4, "big") for x in d[m]) == hashlib.sha256(msg).digest(), m
        assert int(f[m]) == fnv1a64(msg), m
    res = {"checked": "sha256 vs hashlib, fnv1a64 vs python, 4 x 4 KiB", "gpu": []}
    for M in (64, 300, 1536, 16384, 65536):
        nb = (total // M) // 64 * 64
        ms_s = lib.hp_sha256(buf.data_ptr(), nb, M, dig.data_ptr(), 2)
        ms_f = lib.hp_fnv1a64(buf.data_ptr(), nb, M, fout.data_ptr(), 2)
        res["gpu"].append({"messages": M, "msg_bytes": nb, "sha256_GBps": round(M * nb / ms_s / 1e6, 1),
                           "fnv1a64_GBps": round(M * nb / ms_f / 1e6, 1)})
        print(json.dumps(res["gpu"][-1]), flush=True)
    # host SHA-256 (OpenSSL via hashlib releases the GIL) on 16 threads, 1536 messages
    M = 1536
    nb = (total // M) // 64 * 64
    hb = buf[: M * nb].cpu().numpy()
    mv = memoryview(hb)
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(16) as ex:
        list(ex.map(lambda i: hashlib.sha256(mv[i * nb:(i + 1) * nb]).digest(), range(M)))
    dt = time.perf_counter() - t0
    res["cpu_sha256_16thr_GBps"] = round(M * nb / dt / 1e9, 1)
    t0 = time.perf_counter()
    hashlib.sha256(mv[:nb * 64]).digest()
    res["cpu_sha256_1thr_GBps"] = round(nb * 64 / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
