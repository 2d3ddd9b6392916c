"""Per-kernel register / occupancy table from the build's resource-usage remarks
(build/obj/*.remarks, written by latentsync_amd/build.py).
usage: python scripts/kernel_regs.py [name-substring ...]"""
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "VGPRs Spill": "spill", "Occupancy [waves/SIMD]": "occ",
          "LDS Size [bytes/block]": "lds", "ScratchSize [bytes/lane]": "scratch"}


def main():
    rows, cur = {}, None
    for path in sorted(glob.glob(os.path.join(REPO, "build", "obj*", "*.remarks"))):
        for line in open(path):
            m = re.search(r"remark: +Function Name: (\S+)", line)
            if m:
                cur = m.group(1)
                rows[cur] = {}
                continue
            m = re.search(r"remark: +([A-Za-z][^:]*?): (\d+)\b", line)
            if m and cur and m.group(1).strip() in FIELDS:
                rows[cur][FIELDS[m.group(1).strip()]] = int(m.group(2))
    want = sys.argv[1:]
    for f, r in rows.items():
        n = subprocess.run(["c++filt", f], capture_output=True, text=True).stdout.strip()
        if want and not any(w in n for w in want):
            continue
        print(f"{n[:100]:100s} " + " ".join(f"{k}={r.get(k, '-')}" for k in ("vgpr", "agpr", "spill", "occ", "lds")))


if __name__ == "__main__":
    main()
