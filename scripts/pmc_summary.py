"""Per-kernel average of rocprofv3 --pmc counter CSVs (every dir given; counters of
several passes of the same run merged by kernel name).  usage: python scripts/pmc_summary.py DIR..."""
import collections
import csv
import glob
import os
import re
import sys


def main():
    groups = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        if not os.path.isdir(d):
            continue
        key = re.sub(r"_p\d+$", "", os.path.basename(d))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                per[(did, r["Counter_Name"])] += float(r["Counter_Value"])
                names[did] = r["Kernel_Name"].split("(")[0][:70]
            for (did, cn), v in per.items():
                if any(k in names[did] for k in ("conv_gemm", "halo", "rowblock", "attn", "ff_fused", "tattn")):
                    groups[(key, names[did])][cn].append(v)
    for (key, kn), cs in sorted(groups.items()):
        print(f"== {key}  {kn}")
        for cn in sorted(cs):
            vals = cs[cn][1:] if len(cs[cn]) > 2 else cs[cn]  # drop the first (cold) dispatch
            print(f"   {cn:32s} {sum(vals) / len(vals):16.1f}")


if __name__ == "__main__":
    main()
