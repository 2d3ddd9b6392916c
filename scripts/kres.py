"""Per-kernel register / spill / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.  usage: python scripts/kres.py file.hip"""
import re, subprocess, sys
src = sys.argv[1]
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from latentsync_amd.build import FLAGS  # noqa: E402
r = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + ["-c", src,
                    "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = []
for l in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", l)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
dm = subprocess.run(["c++filt"], input="\n".join(x["name"] for x in rows), capture_output=True, text=True).stdout.split("\n")
for x, n in zip(rows, dm):
    n = re.sub(r"\(.*\)$", "", n)
    print(f"{n[:80]:80s} V{x.get('VGPRs','?'):>4} A{x.get('AGPRs','?'):>4} spillV {x.get('VGPRs Spill','?'):>4} "
          f"occ {x.get('Occupancy [waves/SIMD]','?')} lds {x.get('LDS Size [bytes/block]','?')}")
