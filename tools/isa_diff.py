#!/usr/bin/env python3
"""Is the device code of the apply kernels identical between a past commit
and the working tree?  Compiles rs_apply.hip of both to gfx950 assembly and
compares the named kernels' bodies (comments and debug lines dropped).

    python tools/isa_diff.py <commit> [K:U ...]      (default 8:3 4:1 10:3 16:1)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = ("rs_apply.hip", "rs_apply_kernel.hpp", "gfp.hpp", "gfp_host.hpp", "kernels.hpp")


def asm(src_dir: str, out: str) -> str:
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{ROOT}/include",
                    f"-I{src_dir}", "--cuda-device-only", "-S", os.path.join(src_dir, "rs_apply.hip"), "-o", out],
                   check=True, capture_output=True)
    return open(out).read()


def body(text: str, name: str) -> list:
    m = re.search("^" + re.escape(name) + r":.*$", text, re.M)
    j = text.index(".Lfunc_end", m.start())
    return [ln for ln in text[m.start():j].splitlines()[1:] if not ln.strip().startswith((";", ".loc"))]


def main():
    commit = sys.argv[1]
    shapes = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]] or [(8, 3), (4, 1), (10, 3), (16, 1)]
    with tempfile.TemporaryDirectory() as d:
        old_dir = os.path.join(d, "old")
        os.makedirs(old_dir)
        for f in SRC:
            with open(os.path.join(old_dir, f), "w") as fh:
                fh.write(subprocess.run(["git", "-C", ROOT, "show", f"{commit}:slime_amd/csrc/{f}"], check=True,
                                        capture_output=True, text=True).stdout)
        old = asm(old_dir, os.path.join(d, "old.s"))
        new = asm(os.path.join(ROOT, "slime_amd", "csrc"), os.path.join(d, "new.s"))
    same = True
    for k, u in shapes:
        n = f"_ZN5slime5apply20rs_apply_pipe_kernelILi{k}ELi{u}ELb1ELb1ELi0EEEvPKjPjmmmmS3_S3_S3_mjjjj"
        a, b = body(old, n), body(new, n)
        print(f"rs_apply_pipe_kernel<{k},{u}>: {len(a)} vs {len(b)} lines, {'identical' if a == b else 'DIFFERENT'}")
        same &= a == b
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
