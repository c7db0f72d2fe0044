#!/usr/bin/env python3
"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM): counters are in KiB; FETCH_SIZE
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read,
so it is doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <session> [<existing json>] > profiles/r05/pmc_traffic.json
        # symbol path: one entry per config; with an existing file (one entry or a list) the
        # entries of other configs are kept and the result is a list
    python tools/pmc_traffic.py --all <fetch_dir> <write_dir>    # every kernel: HBM bytes per dispatch
    python tools/pmc_traffic.py --bytes <fetch_dir> <write_dir> <config> <session> [<existing json>]
        # the fused byte path's kernels (bench.py object_bytes_path), appended to a list

`kernel_code` (slime_amd/codeobj.py: a hash of the measured kernel's gfx950
machine code in the built library) ties the summary to the build it was
measured on: bench.py replays `hbm_bytes_per_launch` only into lines whose
build runs the same machine code.  Run it against the library that ran the
passes (the tree the GPU session was sent).
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_source_id() -> str:
    h = hashlib.sha256()
    for f in ("rs_apply_kernel.hpp", "rs_apply.hip", "gfp.hpp"):
        h.update(open(os.path.join(ROOT, "slime_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:16]


KERNELS = ("rs_apply_queue_kernel", "rs_apply_pipe_kernel", "rs_apply_kernel")  # product apply kernels (rs_apply.hip)


def per_dispatch(d, counter, need, only=None):
    """Dispatches of the apply kernels instantiated for k = need (a bench run
    also launches other k, e.g. its C5 leg's 10/14); `only`: one kernel name."""
    vals, seen = {}, set()
    for path in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(path)):
            name = next((k for k in KERNELS if f"{k}<{need}," in r["Kernel_Name"]), None)
            if name and (only is None or name == only) and r["Counter_Name"] == counter:
                vals[int(r["Dispatch_Id"])] = float(r["Counter_Value"])
                seen.add(name)
    return vals, seen


def batch_kernel(fetch_dir, need):
    """The apply kernel of the bench's batch launches: of the kernels seen at
    k = need, the one with the largest dispatch (host calls of the same k take
    the static kernel on one-object windows, far smaller)."""
    best, size = None, -1.0
    for k in KERNELS:
        v, _ = per_dispatch(fetch_dir, "FETCH_SIZE", need, k)
        if v and max(v.values()) > size:
            best, size = k, max(v.values())
    return best


def dominant(vals):
    """The dispatches of the most common size (within 1%), and how many others."""
    groups = []
    for k, v in sorted(vals.items(), key=lambda kv: kv[1]):
        if groups and v <= groups[-1][0] * 1.01:
            groups[-1][1][k] = v
        else:
            groups.append((v, {k: v}))
    best = max(groups, key=lambda g: len(g[1]))[1]
    return best, len(vals) - len(best)


def all_kernels(fetch_dir, write_dir):
    """Per kernel (template name up to '<'): dispatches and mean read / write
    bytes per dispatch, with the same gfx950 corrections."""
    acc = {}
    for d, counter in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        for path in glob.glob(f"{d}/*counter_collection.csv"):
            for r in csv.DictReader(open(path)):
                if r["Counter_Name"] != counter:
                    continue
                name = r["Kernel_Name"].split("(")[0]
                e = acc.setdefault(name, {"FETCH_SIZE": [], "WRITE_SIZE": []})
                e[counter].append(float(r["Counter_Value"]))
    out = {}
    for name, e in sorted(acc.items()):
        f, w = e["FETCH_SIZE"], e["WRITE_SIZE"]
        rd = 2 * 1024 * sum(f) / len(f) if f else None
        wr = 1024 * sum(w) / len(w) if w else None
        out[name] = {"dispatches": [len(f), len(w)], "read_bytes": int(rd) if rd is not None else None,
                     "write_bytes": int(wr) if wr is not None else None,
                     "hbm_bytes": int(rd + wr) if rd is not None and wr is not None else None}
    print(json.dumps(out, indent=1))


def kernel_code(kernel: str, need: int) -> str | None:
    sys.path.insert(0, ROOT)
    from slime_amd.codeobj import kernel_code_id
    return kernel_code_id(os.path.join(ROOT, "slime_amd", "lib", "libslime_rs.so"), (f"{kernel}ILi{need}E",))


BYTE_KERNELS = ("encode_bytes_queue_kernel", "encode_bytes_queue_bits_kernel", "encode_bytes_fix_kernel",
                "encode_bytes_redo_kernel", "decode_bytes_queue_kernel")


def byte_kernels(fetch_dir, write_dir, config, session, existing=None):
    """HBM bytes per dispatch of the byte path's product kernels at `config`
    ("need/total S=<bytes> nobj=<n>"), with each kernel's machine code."""
    need = int(config.split("/")[0])
    sums = {}
    for d, counter in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        for path in glob.glob(f"{d}/*counter_collection.csv"):
            for r in csv.DictReader(open(path)):
                name = next((k for k in BYTE_KERNELS if k + "<" in r["Kernel_Name"]), None)
                if name and r["Counter_Name"] == counter:
                    sums.setdefault(name, {}).setdefault(counter, []).append(float(r["Counter_Value"]))
    entry = {"config": config, "session": session, "kernels": {}}
    for name, c in sums.items():
        f, w = c.get("FETCH_SIZE", []), c.get("WRITE_SIZE", [])
        if not f or not w:
            continue
        entry["kernels"][name] = {"kernel_code": kernel_code(name, need), "dispatches": [len(f), len(w)],
                                  "read_bytes": int(2 * 1024 * sum(f) / len(f)),
                                  "write_bytes": int(1024 * sum(w) / len(w)),
                                  "hbm_bytes": int(2 * 1024 * sum(f) / len(f) + 1024 * sum(w) / len(w))}
    entries = json.load(open(existing)) if existing and os.path.exists(existing) else []
    entries = [e for e in entries if e.get("config") != config] + [entry]
    print(json.dumps(entries, indent=1))


def main():
    if sys.argv[1] == "--all":
        return all_kernels(sys.argv[2], sys.argv[3])
    if sys.argv[1] == "--bytes":
        return byte_kernels(*sys.argv[2:7])
    fetch_dir, write_dir, config = sys.argv[1:4]
    session = sys.argv[4] if len(sys.argv) > 4 else "?"
    need = int(config.split("/")[0])
    only = batch_kernel(fetch_dir, need)
    f, fk = per_dispatch(fetch_dir, "FETCH_SIZE", need, only)
    w, wk = per_dispatch(write_dir, "WRITE_SIZE", need, only)
    assert len(fk | wk) == 1, f"expected one apply kernel, saw {fk | wk}"
    # The bench's launches all move the same bytes; the allocator's placement
    # probe over a larger buffer (another leg's) runs the same kernel over
    # more.  Keep the dominant launch size (values within 1% of each other).
    f, f_other = dominant(f)
    w, w_other = dominant(w)
    fetch_kib = sum(f.values()) / len(f)
    write_kib = sum(w.values()) / len(w)
    read_bytes = 2 * fetch_kib * 1024
    write_bytes = write_kib * 1024
    entry = {
        "config": config,
        "session": session,
        "kernel_source": kernel_source_id(),
        "kernel_code": kernel_code(next(iter(fk | wk)), int(config.split("/")[0])),
        "kernel": (fk | wk).pop(),
        "dispatches": {"fetch_pass": len(f), "write_pass": len(w),
                       "other_sizes_left_out": {"fetch_pass": f_other, "write_pass": w_other}},
        "fetch_size_kib_avg": fetch_kib,
        "write_size_kib_avg": write_kib,
        "read_bytes_per_launch": int(read_bytes),
        "write_bytes_per_launch": int(write_bytes),
        "hbm_bytes_per_launch": int(read_bytes + write_bytes),
        "correction": "read = 2 x FETCH_SIZE (gfx950 wide-stream undercount), x1024 (KiB)",
    }
    existing = sys.argv[5] if len(sys.argv) > 5 else None
    if not existing:
        print(json.dumps(entry, indent=1))
        return
    old = json.load(open(existing)) if os.path.exists(existing) else []
    old = old if isinstance(old, list) else [old]
    print(json.dumps([e for e in old if e.get("config") != config] + [entry], indent=1))


if __name__ == "__main__":
    main()
