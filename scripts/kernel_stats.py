"""rocprofv3 kernel summary (name, calls, total/avg/min/max ns, %) from a
kernel-trace CSV or the rocpd .db -- the `--stats` table in a stable form."""
import collections, sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from step_breakdown import load  # noqa: E402

rows = load(sys.argv[1])
agg = collections.defaultdict(list)
for r in rows:
    agg[r['Kernel_Name']].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in agg.values())
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f'"{n}",{len(v)},{sum(v)},{sum(v)/len(v):.1f},{100*sum(v)/tot:.2f},{min(v)},{max(v)}')
