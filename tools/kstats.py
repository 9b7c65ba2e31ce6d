"""Register / LDS / spill summary of the gfx950 kernels (compiler resource-usage remarks).

    python tools/kstats.py [name-filter] [-DFOO ...]
"""
import os
import re
import subprocess
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "recoup_amd", "csrc", "rcp_kernels.hip")


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    defs = sys.argv[2:]
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                        "-c", SRC, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + defs,
                       capture_output=True, text=True)
    name, acc = None, {}
    for ln in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            if name and flt in name:
                print(acc)
            name, acc = m.group(1), {"fn": m.group(1)[:90]}
            continue
        m = re.search(r"remark: ([^:]+): (\d+)", ln)
        if m and name:
            k = m.group(1).strip()
            if k in ("VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"):
                acc[k.split()[0]] = int(m.group(2))
    if name and flt in name:
        print(acc)


if __name__ == "__main__":
    main()
