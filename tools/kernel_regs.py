#!/usr/bin/env python3
"""Register table of a HIP source's kernels for gfx950 (hipcc's
kernel-resource-usage remarks): VGPRs, AGPRs, spills, LDS, waves per SIMD.

    python tools/kernel_regs.py slime_amd/csrc/rs_bytes_mfma.hip [--filter ILi5] [-D NAME=V ...]

Compiles to a scratch object under /tmp; build-time tool only."""
import argparse
import re
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--filter", default="")
    ap.add_argument("-D", dest="defs", action="append", default=[])
    a = ap.parse_args()
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Iinclude",
           "-Islime_amd/csrc", "-c", a.source, "-o", "/tmp/kernel_regs.o", "-Rpass-analysis=kernel-resource-usage"]
    cmd += ["-D" + d for d in a.defs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        sys.exit(r.returncode)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|"
                      r"Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for row in rows:
        if a.filter and a.filter not in row["name"]:
            continue
        dem = subprocess.run(["c++filt", row["name"]], capture_output=True, text=True)
        name = dem.stdout.strip().split("(")[0]
        print(f"{row.get('VGPRs','?'):>4} v {row.get('AGPRs','?'):>3} a  spill v {row.get('VGPRs Spill','?'):>3} "
              f"s {row.get('SGPRs Spill','?'):>3}  waves {row.get('Occupancy [waves/SIMD]','?'):>2}  {name}")


if __name__ == "__main__":
    main()
