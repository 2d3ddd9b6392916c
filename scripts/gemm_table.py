"""Tabulate scripts/gemm_bench.py logs: TF/s per shape per mode."""
import collections, re, sys
rows = collections.OrderedDict()
modes = []
for l in open(sys.argv[1]):
    m = re.match(r"(\S+)\s+(.+?)\s+M=\s*(\d+).*?(\d+\.\d) us\s+(\d+\.\d) TF/s", l)
    if m:
        rows.setdefault(m.group(2), {})[m.group(1)] = float(m.group(5))
        if m.group(1) not in modes:
            modes.append(m.group(1))
    m = re.match(r"(\S+)\s+TOTAL (\S+) ms\s+(\S+) TF/s", l)
    if m:
        rows.setdefault("TOTAL", {})[m.group(1)] = float(m.group(3))
print(f"{'shape':26s}" + "".join(f"{m:>9s}" for m in modes))
for k, v in rows.items():
    print(f"{k:26s}" + "".join(f"{v.get(m, 0):9.0f}" for m in modes))
