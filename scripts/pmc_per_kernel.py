"""Per-kernel HBM traffic of one UNet step from the two rocprofv3 --pmc passes of
scripts/pmc_pass.sh (FETCH_SIZE, WRITE_SIZE): dispatches of the middle step grouped
by (kernel, grid), with the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md (x2 for
16-B-per-lane streaming reads, which every GEMM / attention / norm kernel here uses).

usage: python scripts/pmc_per_kernel.py FETCH_DIR WRITE_DIR [top]
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    per = collections.OrderedDict()
    for r in csv.DictReader(open(files[0])):
        did = int(r.get("Dispatch_Id") or r.get("Dispatch_ID") or r["Correlation_Id"])
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        if did not in per:
            per[did] = [r["Kernel_Name"], grid, 0.0]
        per[did][2] += float(r["Counter_Value"])
    return [v for _, v in sorted(per.items())]


def one_step(disp):
    idx = [i for i, (n, _, _) in enumerate(disp) if "ddim_cfg_kernel" in n]
    k = len(idx) // 2
    return disp[idx[k] + 1: idx[k + 1] + 1]


def short(n):
    n = n.split("(")[0].replace("void ", "")
    return n[:70]


def main():
    fetch, write = one_step(load(sys.argv[1])), one_step(load(sys.argv[2]))
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    assert len(fetch) == len(write), (len(fetch), len(write))
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for (n, g, f), (n2, _, w) in zip(fetch, write):
        assert n == n2
        a = agg[(short(n), g)]
        a[0] += 1
        a[1] += 2.0 * f * 1024
        a[2] += w * 1024
    tot_f = sum(v[1] for v in agg.values())
    tot_w = sum(v[2] for v in agg.values())
    print(f"one UNet step: {len(fetch)} dispatches, fetch {tot_f / 1e9:.2f} GB (x2 corrected), write {tot_w / 1e9:.2f} GB")
    print(f"{'kernel':70s} {'grid':>9s} {'n':>4s} {'fetch MB/call':>14s} {'write MB/call':>14s} {'total GB':>9s}")
    for (n, g), (c, f, w) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:top]:
        print(f"{n:70s} {g:>9s} {c:4d} {f / c / 1e6:14.1f} {w / c / 1e6:14.1f} {(f + w) / 1e9:9.2f}")


if __name__ == "__main__":
    main()
